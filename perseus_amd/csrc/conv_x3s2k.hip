// fp16x3 (parity mode) layer3 BasicBlock entry (conv 3x3 s2 + bn1 + relu, and the 1x1 s2
// downsample + bn; torchvision resnet18 layer3 block 0 behind perseus/detector/models.py:20,
// SURVEY.md 8a7) with the hi / lo weight planes resident in VGPRs and the K sum split over the
// waves by 64-channel input block (conv_x3s2v.hip's design at Cin = 128).
//
// A wave holds the hi and lo weights of 16 output channels for ONE 64-channel input block (the
// conv's 9 taps and the downsample: 2 planes x 20 fragments = 160 VGPRs); a workgroup of 8 waves
// is 4 channel tiles (64 channels, its "quarter" h of Cout = 256) x 2 input blocks and walks
// 1 x 16 output tiles (one output row) persistently.  The whole patch of a tile (3 input rows x
// 33 columns x [hi 128 | lo 128] of both blocks, 272-byte positions per block) is double-
// buffered.  Per (tap, 32-channel half) group a wave reads the x_hi and x_lo fragments of its
// block (2 ds_read_b128) for 3 MFMAs, read two groups ahead (one 16-pixel fragment per wave:
// 48 MFMA cycles per group would not cover the LDS latency at one group ahead, as conv_s2k.hip's
// layer4 form showed); the three products go to three accumulators (x_hi w_hi, x_hi w_lo,
// x_lo w_hi: no back-to-back dependent MFMAs).  At the end of a tile the block-1 waves hand their
// conv partial and the block-0 waves their downsample partial over through LDS, and each
// finalizes one: (block 0 + block 1), each block's (hh + lh) + hl.
//
// Sum order: another order than conv_s2w.h's X3 form (one accumulator over all taps and blocks,
// plane by plane): within f32 rounding of it, far inside the parity mode's 1e-3 px.
#include "conv_gx.h"

namespace pa {

__host__ __device__ constexpr int x3k_tap(int g) {  // group g: tap [3 4 5 0 1 2 6 7 8][g / 2], half g & 1
  return (g >> 1) < 3 ? 3 + (g >> 1) : ((g >> 1) < 6 ? (g >> 1) - 3 : (g >> 1));
}

struct X3s2k {
  static constexpr int NB = 2, WC = 4, TW = 16, PW = 2 * TW + 1, NP = 3 * PW;  // 99 positions per block
  static constexpr int PXB = 272;                          // [hi 128 B | lo 128 B | pad 16 B]
  static constexpr int NRC = NP * 17;                      // chunks per block region
  static constexpr int PJ = (NB * NRC + 63) / 64;          // patch wave-DMAs per tile (53)
  static constexpr int PDW = (PJ + 7) / 8;                 // per wave (7, the last round partial)
  static constexpr int PATCHB = PJ * 1024;
  static constexpr int XB = 8 * 1024;                      // partials handed over per tile
  static constexpr int SMEM = 2 * PATCHB + 2 * XB;
  static_assert(SMEM + 4 * 64 * 4 <= 160 * 1024, "LDS");
  static_assert(PDW <= 18 - 2, "patch DMAs within the K loop");
};

__device__ __forceinline__ void x3k_store8(void* base, unsigned off, half4 v) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, (int)off, 0, 16);
}

// DBG = 4: s_memrealtime stamps into a.trace (0 start, 1 first patch landed; tile t < 20: 2 + 3 t
// start, 3 + 3 t K loop done, 4 + 3 t hand-over barrier passed; 63 end)
// DS: a tile's two output half4 per lane (its finalized group's hi and lo) are stored during the next
// tile's K loop (the two groups after the patch DMAs) instead of at the tile's end
template <int DBG = 0, bool DS = false>
__global__ __launch_bounds__(512, 1) void conv3x3s2_k3(ConvS2Args a, int ntiles, int nh, int xo) {
  using G = X3s2k;
  constexpr int NB = G::NB, WC = G::WC, TW = G::TW, PW = G::PW, NP = G::NP, PXB = G::PXB, NRC = G::NRC;
  constexpr int PJ = G::PJ, PDW = G::PDW, PATCHB = G::PATCHB, XB = G::XB;
  constexpr int CIN = 128, XS = 2, RA = 3;  // RA: fragment sets in flight (reads two groups ahead)
  __shared__ __attribute__((aligned(1024))) char smem[G::SMEM];
  __shared__ __attribute__((aligned(16))) float epi_l[4 * 64];  // [bias | scale | bias2 | scale2] of the quarter
  char* patch = smem;
  char* xch = smem + 2 * PATCHB;

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, r16 = lane & 15;
  const int wc = wid % WC, wb = wid / WC;  // channel tile, input block
  if constexpr (DBG == 4) trace_stamp(a.trace, 0);
  const int H = a.Hout, W = a.Wout, Hin = a.Hin, Win = a.Win, Cout = a.Cout;
  // workgroup -> (quarter h, slot); xo: blocks b, b + 8, .. (one XCD) take the quarters of the
  // same tiles (the patch is an L2 hit after the first)
  const int b = blockIdx.x;
  int h, slot;
  if (xo) {
    h = (b >> 3) % nh;
    slot = (b & 7) + ((b >> 3) / nh) * 8;
  } else {
    h = b % nh;
    slot = b / nh;
  }
  const int nslots = (int)gridDim.x / nh;
  const int c0 = 64 * h;
  const int tpi = H;  // one output row per tile (W == TW)
  const bool xm = xo && nslots % 8 == 0 && ntiles % (8 * tpi) == 0;
  auto tmap = [&](int j) __attribute__((always_inline)) {
    if (!xm) return j;
    const int c = j / (8 * tpi), r = j - c * 8 * tpi;
    return c * 8 * tpi + (r & 7) * tpi + (r >> 3);
  };
  const unsigned abytes = (unsigned)((size_t)a.B * Hin * Win * XS * CIN * 2 < 0x7fffffffu
                                         ? (size_t)a.B * Hin * Win * XS * CIN * 2
                                         : 0x7fffffffu);
  const s2w_u4 rsrc = s2w_rsrc(a.in, abytes);
  struct Org {
    int img, h0;
    bool on;
  };
  auto origin = [&](int t, bool on) __attribute__((always_inline)) {
    const int img = t / tpi;
    return Org{img, 2 * (t - img * tpi) - 1, on};
  };
  // patch DMA i of this wave: chunk c = (i * 8 + wid) * 64 + lane = block c / NRC, position
  // p = (c % NRC) / 17 (input row p / PW, position p % PW: odd run, then even run), slot c % 17:
  // plane (s >> 3), chunk position s & 7, 16 = pad.  Packed: bits 0-17 byte offset from the patch
  // origin (column -1 of input row 2 y - 1), 18-21 row, 22-27 column, 28 pad / past the patch.
  unsigned pk[PDW];
#pragma unroll
  for (int i = 0; i < PDW; ++i) {
    const int c = (i * 8 + wid) * 64 + lane;
    const int blk = c / NRC, rc = c - blk * NRC, p = rc / 17, sl = rc - p * 17;
    const bool bad = c >= NB * NRC || sl >= 16;
    const int pr = bad ? 0 : p / PW, pc = bad ? 0 : p - (p / PW) * PW;
    const int co = pc <= TW ? 2 * pc : 2 * (pc - TW - 1) + 1;
    const int chan = (sl >> 3) * CIN + 64 * blk + ((sl & 1) * 4 + ((sl & 7) >> 1)) * 8;
    const unsigned rel = bad ? 0u : (unsigned)(((pr * Win + co) * XS * CIN + chan) * 2);
    pk[i] = (rel & 0x3ffffu) | ((unsigned)pr << 18) | ((unsigned)co << 22) | ((bad ? 1u : 0u) << 28);
  }
  auto dma_one = [&](int i, const Org& o, int buf) __attribute__((always_inline)) {
    if (PJ == PDW * 8 || i < PDW - 1 || wid < PJ - (PDW - 1) * 8) {  // wave-uniform
      const unsigned v = pk[i];
      const int pr = (int)((v >> 18) & 15u), co = (int)((v >> 22) & 63u);
      const unsigned tb = (unsigned)(((o.img * Hin + o.h0) * Win - 1) * XS * CIN * 2);  // wave-uniform (may wrap)
      const bool ok = o.on && !(v >> 28) && (unsigned)(o.h0 + pr) < (unsigned)Hin && (unsigned)(co - 1) < (unsigned)Win;
      s2w_dma16(rsrc, ok ? tb + (v & 0x3ffffu) : S2W_OOB, patch + buf * PATCHB + (i * 8 + wid) * 1024);
    }
  };

  const int o = xfrag(r16);
  // this lane's patch-read base: its block's region, position o of patch row 0, chunk position 2 q
  const unsigned rbase = (unsigned)(size_t)(__attribute__((address_space(3))) char*)patch +
                         (unsigned)(wb * NRC * 16 + o * PXB + q * 32);
  if (tid < 64) {
    epi_l[tid] = a.bias[c0 + tid];
    epi_l[64 + tid] = a.scale[c0 + tid];
    epi_l[128 + tid] = a.bias2[c0 + tid];
    epi_l[192 + tid] = a.scale2[c0 + tid];
  }
  __builtin_amdgcn_sched_barrier(0);

  // prologue: the first tile's patch, then this wave's hi / lo fragments straight into its VGPRs
  // (wfrag: [h][wb][wc][fragment 20][plane 2][lane 64][8 fp16])
  int j = slot;
  {
    const Org o0 = origin(tmap(j < ntiles ? j : 0), j < ntiles);
#pragma unroll
    for (int i = 0; i < PDW; ++i) dma_one(i, o0, 0);
  }
  xu4 wh[18], wl[18], dh[2], dl[2];
  {
    const xu4* __restrict__ wf =
        reinterpret_cast<const xu4*>(a.wfrag) + (size_t)((h * NB + wb) * WC + wc) * 20 * 2 * 64 + lane;
    gx_for<0, 18>([&](auto gc) __attribute__((always_inline)) {
      constexpr int Gi = decltype(gc)::value, TAP = x3k_tap(Gi), K = 2 * TAP + (Gi & 1);
      wh[K] = wf[(K * 2 + 0) * 64];
      wl[K] = wf[(K * 2 + 1) * 64];
      if constexpr (TAP == 4) {
        dh[Gi & 1] = wf[((18 + (Gi & 1)) * 2 + 0) * 64];
        dl[Gi & 1] = wf[((18 + (Gi & 1)) * 2 + 1) * 64];
      }
    });
  }
  xwait_vm<40>();  // the first patch landed (this wave's DMAs, issued before the 40 weight loads)
  lds_barrier();   // ... and every wave's
  if constexpr (DBG == 4) trace_stamp(a.trace, 1);

  _Float16* __restrict__ out = (_Float16*)a.out;
  _Float16* __restrict__ out2 = (_Float16*)a.out2;
  int jn = j + nslots;
  half4 phi, plo;        // DS: the previous tile's outputs
  unsigned pob = 0;      // DS: their byte offset (per lane)
  _Float16* const dsto = wb ? out2 : out;
  auto run_tile = [&](auto firstc, int t) __attribute__((always_inline)) {
    const int buf = t & 1;
    const int tile = tmap(j);
    const bool has_next = jn < ntiles;
    const Org onext = origin(has_next ? tmap(jn) : tile, has_next);
    const int img = tile / tpi, y = tile - img * tpi;
    if constexpr (DBG == 4) {
      if (t < 20) trace_stamp(a.trace, 2 + 3 * t);
    }
    f32x4 ahh = {0.f, 0.f, 0.f, 0.f}, alh = ahh, ahl = ahh, dhh = ahh, dlh = ahh, dhl = ahh;
    const __attribute__((address_space(3))) char* pb =
        (const __attribute__((address_space(3))) char*)(size_t)(rbase + buf * PATCHB);
    xu4 xh[RA], xl[RA];
    auto rd = [&](auto gc) __attribute__((always_inline)) {
      constexpr int Gi = decltype(gc)::value, TAP = x3k_tap(Gi), HG = Gi & 1, S = Gi % RA;
      constexpr int KH = TAP / 3, KW = TAP % 3;
      constexpr int POFF = KW == 0 ? 0 : (KW == 1 ? TW + 1 : 1);
      const auto* p = reinterpret_cast<const __attribute__((address_space(3))) xu4*>(pb + (KH * PW + POFF) * PXB + HG * 16);
      xh[S] = p[0];
      xl[S] = p[8];  // + 128 bytes: the lo plane
    };
    auto mm = [&](auto gc) __attribute__((always_inline)) {
      constexpr int Gi = decltype(gc)::value, TAP = x3k_tap(Gi), HG = Gi & 1, S = Gi % RA;
      constexpr int K = 2 * TAP + HG;
      const half8 h = __builtin_bit_cast(half8, xh[S]), l = __builtin_bit_cast(half8, xl[S]);
      ahh = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, wh[K]), h, ahh, 0, 0, 0);
      alh = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, wl[K]), h, alh, 0, 0, 0);
      ahl = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, wh[K]), l, ahl, 0, 0, 0);
      if constexpr (TAP == 4) {  // the downsample reads tap 4's pixels
        dhh = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, dh[HG]), h, dhh, 0, 0, 0);
        dlh = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, dl[HG]), h, dlh, 0, 0, 0);
        dhl = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, dh[HG]), l, dhl, 0, 0, 0);
      }
    };
    rd(xic<0>{});
    rd(xic<1>{});
    gx_for<0, 18>([&](auto gc) __attribute__((always_inline)) {
      constexpr int Gi = decltype(gc)::value;
      if constexpr (Gi + 2 < 18) rd(xic<Gi + 2>{});
      __builtin_amdgcn_sched_barrier(0);  // reads two groups ahead of this group's MFMAs
      if constexpr (Gi < PDW) {           // next tile's patch, one DMA per group
        __builtin_amdgcn_sched_barrier(0);
        dma_one(Gi, onext, buf ^ 1);
        __builtin_amdgcn_sched_barrier(0);
      } else if constexpr (DS && Gi < PDW + 2) {  // the previous tile's outputs
        __builtin_amdgcn_sched_barrier(0);
        if (t > 0) x3k_store8(dsto, Gi == PDW ? pob : pob + Cout * 2, Gi == PDW ? phi : plo);
        __builtin_amdgcn_sched_barrier(0);
      }
      mm(gc);
    });
    if constexpr (DBG == 4) {
      if (t < 20) trace_stamp(a.trace, 3 + 3 * t);
    }
    // this block's partials: conv (hh + lh) + hl, downsample the same; the block-1 waves hand the
    // conv over, the block-0 waves the downsample
    const f32x4 pc = (ahh + alh) + ahl, pd = (dhh + dlh) + dhl;
    char* xb = xch + buf * XB;
    *reinterpret_cast<f32x4*>(xb + ((wb * WC + wc) * 64 + lane) * 16) = wb ? pc : pd;
    // next patch landed (this wave's DMAs; DS: the previous tile's two stores, issued after them, may
    // stay in flight)
    if constexpr (DS) {
      if (t > 0)
        xwait_vm<2>();
      else
        xwait_vm<0>();
    } else {
      xwait_vm<0>();
    }
    lds_barrier();  // every wave's, the partials written, every read of buf retired
    if constexpr (DBG == 4) {
      if (t < 20) trace_stamp(a.trace, 4 + 3 * t);
    }
    const f32x4 other = *reinterpret_cast<const f32x4*>(xb + (((wb ^ 1) * WC + wc) * 64 + lane) * 16);
    // block 0's partial + block 1's
    const f32x4 v = wb ? other + pd : pc + other;
    const int ch = 16 * wc + 4 * q;  // within the quarter
    const f32x4 bb = *reinterpret_cast<const f32x4*>(epi_l + 128 * wb + ch);
    const f32x4 ss = *reinterpret_cast<const f32x4*>(epi_l + 128 * wb + 64 + ch);
    half4 hi, lo;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float z = v[e] * ss[e] + bb[e];
      const HiLo s = split_x3(wb ? z : fmaxf(z, 0.f));
      hi[e] = s.hi;
      lo[e] = s.lo;
    }
    const unsigned ob = (unsigned)((((img * H + y) * W + o) * XS * Cout + c0 + ch) * 2);
    if constexpr (DS) {
      phi = hi;
      plo = lo;
      pob = ob;
    } else {
      x3k_store8(dsto, ob, hi);
      x3k_store8(dsto, ob + Cout * 2, lo);
    }
    j = jn;
    jn = j + nslots;
  };
  const bool any = j < ntiles;
  if (any) run_tile(std::true_type{}, 0);
  for (int t = 1; j < ntiles; ++t) run_tile(std::false_type{}, t);  // (run_tile advances j)
  if constexpr (DS) {  // the last tile's outputs
    if (any) {
      x3k_store8(dsto, pob, phi);
      x3k_store8(dsto, pob + Cout * 2, plo);
    }
  }
  if constexpr (DBG == 4) {
    __builtin_amdgcn_s_waitcnt(0);
    trace_stamp(a.trace, 63);
  }
}

// variant 0: shipped form; 1: s_memrealtime stamps into a.trace; 2: deferred stores (DS)
int launch_conv3x3s2_k3(const ConvS2Args& a, int variant, hipStream_t s, const char** kname) {
  PA_CHECK(a.wfrag, "x3 s2k conv: no VGPR-order weights (ConvS2Args::wfrag)");
  PA_CHECK(a.scale && a.scale2, "x3 s2k conv: scales required");
  PA_CHECK(a.Cin == 128 && a.Cout % 64 == 0 && a.Wout == 16 && a.Hin == 2 * a.Hout && a.Win == 2 * a.Wout,
           "x3 s2k conv: Cin 128, Wout 16 only, got %d -> %d, %dx%d", a.Cin, a.Cout, a.Hout, a.Wout);
  PA_CHECK((size_t)a.B * a.Hin * a.Win * 512 < 0x7fffffffu && (size_t)a.B * a.Hout * a.Wout * a.Cout * 4 < 0x7fffffffu,
           "x3 s2k conv: activations over 2 GB");
  if (a.B <= 0) return PA_OK;
  if (kname) *kname = "conv3x3s2k3_l3";
  const int nh = a.Cout / 64;
  const int tiles = a.B * a.Hout;
  const int cus = conv_stream_cus(s);
  int grid = (cus / (8 * nh)) * 8 * nh, xo = 1;
  if (grid == 0) {
    grid = cus >= nh ? (cus / nh) * nh : nh;
    xo = 0;
  }
  if (grid / nh > tiles) grid = (xo ? ((tiles + 7) / 8) * 8 : tiles) * nh;
  if (variant == 1 && a.trace)
    hipLaunchKernelGGL((conv3x3s2_k3<4>), dim3(grid), dim3(512), 0, s, a, tiles, nh, xo);
  else if (variant == 2)
    hipLaunchKernelGGL((conv3x3s2_k3<0, true>), dim3(grid), dim3(512), 0, s, a, tiles, nh, xo);
  else
    hipLaunchKernelGGL((conv3x3s2_k3<0>), dim3(grid), dim3(512), 0, s, a, tiles, nh, xo);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

}  // namespace pa
