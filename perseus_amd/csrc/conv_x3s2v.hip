// fp16x3 (parity mode) layer2 BasicBlock entry (conv 3x3 s2 + bn1 + relu, and the 1x1 s2
// downsample + bn, one pass over the input; torchvision resnet18 layer2 block 0 behind
// perseus/detector/models.py:20) with the hi / lo weight planes resident in VGPRs:
// conv_s2v.hip's design on the fp16x3 planes.
//
// conv_s2w.h's X3 form streams a 16 KB weight tile per step through an LDS ring, three virtual
// 64-channel blocks per input block (x_hi w_hi, x_hi w_lo, x_lo w_hi), on 64-channel tiles (the
// 128-channel X3 tile spills): 0.23 of the MFMA peak counting the three products.  Here each of
// the 8 waves owns 16 output channels and holds their hi and lo weights for all 640 K of the conv
// and the downsample (2 planes x 20 fragments x 16 B per lane = 160 VGPRs) for the whole launch;
// one workgroup per CU walks 2 x 16 output tiles persistently, the whole patch of a tile (5 input
// rows x 33 columns x [hi 64 | lo 64], 272-byte positions) double-buffered.  Per (tap, 32-channel
// half) group a wave reads the x_hi and x_lo fragments of its 2 pixel rows (4 ds_read_b128) for 6
// MFMAs (w_hi x_hi, w_lo x_hi, w_hi x_lo per row): 0.67 reads per MFMA and no weight traffic
// through LDS (conv_x3v.hip, the layer1 form, reads at the same rate).
//
// Patch positions: conv_s2v.hip's column order (the 17 odd input columns, then the 16 even ones:
// a fragment's 16 consecutive output pixels read 16 consecutive positions for every tap), 272
// bytes each = 17 chunks: hi chunks at chunk position 2 q + h (input channels 32 h + 8 q .. + 7),
// lo chunks the same 128 bytes later, one pad chunk.  A 16-lane group reads 16 positions 272 B
// apart = bank quads 4 o mod 64: conflict-free.
//
// Sum order: each accumulator adds, group by group in conv_s2w.h's tap order (3 4 5 0 1 2 6 7 8,
// halves in order; the downsample with tap 4), x_hi w_hi, x_hi w_lo, x_lo w_hi.  Another order
// than conv_s2w.h's X3 form (all taps of x_hi w_hi, then of x_hi w_lo, then of x_lo w_hi), so
// not bit-identical to it (both well inside the parity mode's 1e-3 px).  Epilogue: conv_s2w.h
// X3's (exact unscale by 2^-e, bias, ReLU, (hi, lo) split), 8-byte stores per plane.
#include "conv_gx.h"

namespace pa {

__host__ __device__ constexpr int x3v_tap(int g) {  // group g: tap [3 4 5 0 1 2 6 7 8][g / 2], half g & 1
  return (g >> 1) < 3 ? 3 + (g >> 1) : ((g >> 1) < 6 ? (g >> 1) - 3 : (g >> 1));
}

struct X3s2v {
  static constexpr int TH = 2, TW = 16, PW = 2 * TW + 1, NP = (2 * TH + 1) * PW;  // 165 positions
  static constexpr int NWAVE = 8;
  static constexpr int PXB = 272;                       // [hi 128 B | lo 128 B | pad 16 B]
  static constexpr int PJ = (NP * 17 + 63) / 64;        // patch wave-DMAs per tile (44)
  static constexpr int PDW = (PJ + NWAVE - 1) / NWAVE;  // per wave (6, the last round partial)
  static constexpr int PATCHB = PJ * 1024;
  static constexpr int STG = 8 * 8 * 64 * 8;           // DS: a tile's outputs, 8 half4 per lane and wave
  static constexpr int SMEM = 2 * PATCHB + STG;
  static_assert(SMEM + 512 * 4 <= 160 * 1024, "LDS");
};

__device__ __forceinline__ void x3_store8(void* base, unsigned off, half4 v) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, (int)off, 0, 16);
}

// DBG = 4: s_memrealtime stamps into a.trace (0 start, 1 first patch landed; tile t < 15: 2 + 4 t
// start, 3 + 4 t K loop done and next patch landed, 4 + 4 t stores issued; 63 end)
// DS (deferred stores): a tile's 8 output half4 per lane are staged in this wave's own 4 KB of LDS
// and stored during the next tile's K loop (groups 6 .. 13, after the patch DMAs), instead of at
// the tile's end, where every CU stores at the same moment (traced: ~1.5 us of store issue and
// ~2.6 us of barrier per tile, profiles/r06g)
template <int DBG = 0, bool DS = false>
__global__ __launch_bounds__(512, 1) void conv3x3s2_v3(ConvS2Args a, int ntiles) {
  using G = X3s2v;
  constexpr int TW = G::TW, PW = G::PW, NP = G::NP, PXB = G::PXB, PJ = G::PJ, PDW = G::PDW, PATCHB = G::PATCHB;
  constexpr int TM = 2, CIN = 64, XS = 2;  // XS: fp16 planes per element
  __shared__ __attribute__((aligned(1024))) char smem[G::SMEM];
  __shared__ __attribute__((aligned(16))) float epi_l[512];  // [bias | scale | bias2 | scale2] (128 each)
  char* patch = smem;

  const int tid = threadIdx.x, lane = tid & 63, wn = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, r16 = lane & 15;
  if constexpr (DBG == 4) trace_stamp(a.trace, 0);
  const int H = a.Hout, W = a.Wout, Hin = a.Hin, Win = a.Win, Cout = a.Cout;
  const int tw_n = W / TW, tpi = (H / 2) * tw_n;
  // XCD-grouped tile order (conv_s2v.hip): an image's tiles on one XCD in one round
  const bool xm = ntiles % (8 * tpi) == 0 && gridDim.x % 8 == 0;
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
    int img, h0, x0;
    bool on;
  };
  auto origin = [&](int t, bool on) __attribute__((always_inline)) {
    const int img = t / tpi, rem = t - img * tpi;
    return Org{img, 4 * (rem / tw_n) - 1, 2 * (rem - (rem / tw_n) * tw_n) * TW - 1, on};
  };
  // patch DMA i of this wave: chunk c = (i * 8 + wn) * 64 + lane = position p = c / 17 (input row
  // p / PW, position p % PW: odd run, then even run), slot s = c % 17: plane s >> 3, chunk position
  // s & 7 (channels 8 (((s & 1) * 4 + ((s & 7) >> 1))), 16: pad.  Packed as conv_s2v.hip: bits 0-17
  // byte offset from the patch origin, 18-21 row, 22-27 column offset, 28 pad / past the patch.
  unsigned pk[PDW];
#pragma unroll
  for (int i = 0; i < PDW; ++i) {
    const int c = (i * 8 + wn) * 64 + lane;
    const int p = c / 17, sl = c - p * 17;
    const bool bad = sl >= 16 || p >= NP;
    const int pr = bad ? 0 : p / PW, pc = bad ? 0 : p - (p / PW) * PW;
    const int co = pc <= TW ? 2 * pc : 2 * (pc - TW - 1) + 1;
    const int chan = (sl >> 3) * CIN + ((sl & 1) * 4 + ((sl & 7) >> 1)) * 8;
    const unsigned rel = bad ? 0u : (unsigned)(((pr * Win + co) * XS * CIN + chan) * 2);
    pk[i] = (rel & 0x3ffffu) | ((unsigned)pr << 18) | ((unsigned)co << 22) | ((bad ? 1u : 0u) << 28);
  }
  auto dma_one = [&](int i, const Org& o, int buf) __attribute__((always_inline)) {
    if (PJ == PDW * 8 || i < PDW - 1 || wn < PJ - (PDW - 1) * 8) {  // wave-uniform
      const unsigned v = pk[i];
      const int pr = (int)((v >> 18) & 15u), co = (int)((v >> 22) & 63u);
      const unsigned tb = (unsigned)(((o.img * Hin + o.h0) * Win + o.x0) * XS * CIN * 2);  // wave-uniform (may wrap)
      const bool ok = o.on && !(v >> 28) && (unsigned)(o.h0 + pr) < (unsigned)Hin && (unsigned)(o.x0 + co) < (unsigned)Win;
      s2w_dma16(rsrc, ok ? tb + (v & 0x3ffffu) : S2W_OOB, patch + buf * PATCHB + (i * 8 + wn) * 1024);
    }
  };

  const int o = xfrag(r16);
  // this lane's patch-read base: position o of patch row 0, chunk position 2 q (hi plane)
  const unsigned rbase = (unsigned)(size_t)(__attribute__((address_space(3))) char*)patch + (unsigned)(o * PXB + q * 32);
  if (tid < 128) {
    epi_l[tid] = a.bias[tid];
    epi_l[128 + tid] = a.scale[tid];
    epi_l[256 + tid] = a.bias2[tid];
    epi_l[384 + tid] = a.scale2[tid];
  }
  __builtin_amdgcn_sched_barrier(0);

  // prologue: the first tile's patch, then this wave's hi / lo weight fragments straight into its
  // VGPRs in the order the K loop uses them (wfrag: [wave 8][fragment 20][plane 2][lane 64][8 fp16],
  // fragment k < 18: tap k / 2, half k & 1; 18, 19: the downsample's halves)
  int j = blockIdx.x;
  {
    const Org o0 = origin(tmap(j < ntiles ? j : 0), j < ntiles);
#pragma unroll
    for (int i = 0; i < PDW; ++i) dma_one(i, o0, 0);
  }
  xu4 wh[18], wl[18], dh[2], dl[2];
  {
    const xu4* __restrict__ wf = reinterpret_cast<const xu4*>(a.wfrag) + (size_t)wn * 20 * 2 * 64 + lane;
    gx_for<0, 18>([&](auto gc) __attribute__((always_inline)) {
      constexpr int Gi = decltype(gc)::value, TAP = x3v_tap(Gi), K = 2 * TAP + (Gi & 1);
      wh[K] = wf[(K * 2 + 0) * 64];
      wl[K] = wf[(K * 2 + 1) * 64];
      if constexpr (TAP == 4) {
        dh[Gi & 1] = wf[((18 + (Gi & 1)) * 2 + 0) * 64];
        dl[Gi & 1] = wf[((18 + (Gi & 1)) * 2 + 1) * 64];
      }
    });
  }
  xwait_vm<40>();  // the first patch landed (this wave's DMAs: issued before the 40 weight loads)
  lds_barrier();   // ... and every wave's
  if constexpr (DBG == 4) trace_stamp(a.trace, 1);

  _Float16* __restrict__ out = (_Float16*)a.out;
  _Float16* __restrict__ out2 = (_Float16*)a.out2;
  int jn = j + (int)gridDim.x;
  // DS: this wave's staging slots (index s = tm * 4 + kind * 2 + plane), the lane's output offset
  // within a tile (row tm adds tm * W * 512 bytes, lo plane + 256, out2 the same), the staged tile's base
  char* stg = smem + 2 * PATCHB + wn * 8 * 512 + lane * 8;
  const unsigned olane = (unsigned)((o * XS * Cout + 16 * wn + 4 * q) * 2);
  unsigned pend_base = 0;
  auto store_staged = [&](int sidx) __attribute__((always_inline)) {
    const int tm = sidx >> 2, kind = (sidx >> 1) & 1, pl = sidx & 1;
    const half4 v = *reinterpret_cast<const half4*>(stg + sidx * 512);
    x3_store8(kind ? out2 : out, pend_base + olane + (unsigned)(tm * W * XS * Cout * 2 + pl * Cout * 2), v);
  };
  // one tile; the first is its own copy of the body (FIRST): there the compiler's vmcnt waits hold
  // each group's MFMAs until that group's weight fragments have landed
  auto run_tile = [&](auto firstc, int t) __attribute__((always_inline)) {
    const int buf = t & 1;
    const int tile = tmap(j);
    const bool has_next = jn < ntiles;
    const Org onext = origin(has_next ? tmap(jn) : tile, has_next);
    const int img = tile / tpi, rem = tile - img * tpi;
    const int th0 = (rem / tw_n) * 2, tw0 = (rem - (rem / tw_n) * tw_n) * TW;
    if constexpr (DBG == 4) {
      if (t < 15) trace_stamp(a.trace, 2 + 4 * t);
    }

    f32x4 acc[TM], accd[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      accd[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const __attribute__((address_space(3))) char* pb =
        (const __attribute__((address_space(3))) char*)(size_t)(rbase + buf * PATCHB);
    xu4 xh[2][TM], xl[2][TM];
    auto rd = [&](auto gc) __attribute__((always_inline)) {
      constexpr int Gi = decltype(gc)::value, TAP = x3v_tap(Gi), HG = Gi & 1, S = Gi & 1;
      constexpr int KH = TAP / 3, KW = TAP % 3;
      constexpr int POFF = KW == 0 ? 0 : (KW == 1 ? TW + 1 : 1);
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const auto* p = reinterpret_cast<const __attribute__((address_space(3))) xu4*>(
            pb + ((2 * tm + KH) * PW + POFF) * PXB + HG * 16);
        xh[S][tm] = p[0];
        xl[S][tm] = p[8];  // + 128 bytes: the lo plane
      }
    };
    auto mm = [&](auto gc) __attribute__((always_inline)) {
      constexpr int Gi = decltype(gc)::value, TAP = x3v_tap(Gi), HG = Gi & 1, S = Gi & 1;
      constexpr int K = 2 * TAP + HG;
      auto m3 = [&](f32x4(&ac)[TM], const xu4& h, const xu4& l) __attribute__((always_inline)) {
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
          ac[tm] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, h), __builtin_bit_cast(half8, xh[S][tm]),
                                                          ac[tm], 0, 0, 0);
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
          ac[tm] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, l), __builtin_bit_cast(half8, xh[S][tm]),
                                                          ac[tm], 0, 0, 0);
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
          ac[tm] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, h), __builtin_bit_cast(half8, xl[S][tm]),
                                                          ac[tm], 0, 0, 0);
      };
      m3(acc, wh[K], wl[K]);
      if constexpr (TAP == 4) m3(accd, dh[HG], dl[HG]);  // the downsample reads tap 4's pixels
    };
    rd(xic<0>{});
    gx_for<0, 18>([&](auto gc) __attribute__((always_inline)) {
      constexpr int Gi = decltype(gc)::value;
      if constexpr (Gi + 1 < 18) rd(xic<Gi + 1>{});
      __builtin_amdgcn_sched_barrier(0);  // next group's reads ahead of this group's MFMAs
      if constexpr (Gi < PDW) {           // next tile's patch, one DMA per group
        __builtin_amdgcn_sched_barrier(0);
        dma_one(Gi, onext, buf ^ 1);  // (no next tile: onext.on = false, zeros into buf ^ 1)
        __builtin_amdgcn_sched_barrier(0);
      } else if constexpr (DS && Gi < PDW + 8) {  // the previous tile's outputs
        __builtin_amdgcn_sched_barrier(0);
        if (t > 0) store_staged(Gi - PDW);
        __builtin_amdgcn_sched_barrier(0);
      }
      mm(gc);
    });
    // next patch landed (this wave's DMAs; DS: the previous tile's stores, issued after them, may
    // stay in flight)
    if constexpr (DS) {
      if (t > 0)
        xwait_vm<8>();
      else
        xwait_vm<0>();
    } else {
      xwait_vm<0>();
    }
    if constexpr (DBG == 4) {
      if (t < 15) trace_stamp(a.trace, 3 + 4 * t);
    }

    // epilogue (conv_s2w.h X3's): lane (q, r16) holds channels 16 wn + 4 q .. + 3 of pixel o of
    // output row th0 + tm
    const int ch = 16 * wn + 4 * q;
    const f32x4 b1 = *reinterpret_cast<const f32x4*>(epi_l + ch), s1 = *reinterpret_cast<const f32x4*>(epi_l + 128 + ch);
    const f32x4 b2 = *reinterpret_cast<const f32x4*>(epi_l + 256 + ch),
                s2 = *reinterpret_cast<const f32x4*>(epi_l + 384 + ch);
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
      half4 h1, l1, h2, l2;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const HiLo v1 = split_x3(fmaxf(acc[tm][e] * s1[e] + b1[e], 0.f));
        const HiLo v2 = split_x3(accd[tm][e] * s2[e] + b2[e]);
        h1[e] = v1.hi;
        l1[e] = v1.lo;
        h2[e] = v2.hi;
        l2[e] = v2.lo;
      }
      if constexpr (DS) {
        *reinterpret_cast<half4*>(stg + (tm * 4 + 0) * 512) = h1;
        *reinterpret_cast<half4*>(stg + (tm * 4 + 1) * 512) = l1;
        *reinterpret_cast<half4*>(stg + (tm * 4 + 2) * 512) = h2;
        *reinterpret_cast<half4*>(stg + (tm * 4 + 3) * 512) = l2;
      } else {
        const unsigned ob = (unsigned)((((img * H + th0 + tm) * W + tw0 + o) * XS * Cout + ch) * 2);
        x3_store8(out, ob, h1);
        x3_store8(out, ob + Cout * 2, l1);
        x3_store8(out2, ob, h2);
        x3_store8(out2, ob + Cout * 2, l2);
      }
    }
    if constexpr (DS) pend_base = (unsigned)((((img * H + th0) * W + tw0) * XS * Cout) * 2);
    if constexpr (DBG == 4) {
      if (t < 15) trace_stamp(a.trace, 4 + 4 * t);
    }
    // every wave's DMAs into buf ^ 1 landed (its wait above) and its reads of buf retired
    lds_barrier();
    j = jn;
    jn = j + (int)gridDim.x;
  };
  const bool any = j < ntiles;
  if (any) run_tile(std::true_type{}, 0);
  for (int t = 1; j < ntiles; ++t) run_tile(std::false_type{}, t);  // (run_tile advances j)
  if constexpr (DS) {  // the last tile's outputs (this wave's own staged writes)
    if (any) {
#pragma unroll
      for (int i = 0; i < 8; ++i) store_staged(i);
    }
  }
  if constexpr (DBG == 4) {
    __builtin_amdgcn_s_waitcnt(0);
    trace_stamp(a.trace, 63);
  }
}

// variant 0: stores at the tile end; 1: with s_memrealtime stamps into a.trace; 2 / 3: 0 / 1 with
// deferred stores (DS)
int launch_conv3x3s2_v3(const ConvS2Args& a, int variant, hipStream_t s, const char** kname) {
  PA_CHECK(a.wfrag, "x3 s2v conv: no VGPR-order weights (ConvS2Args::wfrag)");
  PA_CHECK(a.scale && a.scale2, "x3 s2v conv: scales required");
  PA_CHECK(a.Cin == 64 && a.Cout == 128, "x3 s2v conv: Cin 64 -> Cout 128 only, got %d -> %d", a.Cin, a.Cout);
  PA_CHECK(a.Hin == 2 * a.Hout && a.Win == 2 * a.Wout && a.Hout % 2 == 0 && a.Wout % 16 == 0,
           "x3 s2v conv: %dx%d -> %dx%d", a.Hin, a.Win, a.Hout, a.Wout);
  PA_CHECK(a.Win <= 64, "x3 s2v conv: input width %d (packed patch offsets)", a.Win);
  PA_CHECK((size_t)a.B * a.Hin * a.Win * 256 < 0x7fffffffu && (size_t)a.B * a.Hout * a.Wout * 512 < 0x7fffffffu,
           "x3 s2v conv: activations over 2 GB");
  if (a.B <= 0) return PA_OK;
  if (kname) *kname = "conv3x3s2v3_l2";
  const int tiles = a.B * (a.Hout / 2) * (a.Wout / 16);
  const int slots = conv_stream_cus(s);  // one 8-wave workgroup per CU
  const int grid = tiles < slots ? tiles : slots;
  if (variant == 1 && a.trace)
    hipLaunchKernelGGL((conv3x3s2_v3<4>), dim3(grid), dim3(512), 0, s, a, tiles);
  else if (variant == 2)
    hipLaunchKernelGGL((conv3x3s2_v3<0, true>), dim3(grid), dim3(512), 0, s, a, tiles);
  else if (variant == 3 && a.trace)
    hipLaunchKernelGGL((conv3x3s2_v3<4, true>), dim3(grid), dim3(512), 0, s, a, tiles);
  else
    hipLaunchKernelGGL((conv3x3s2_v3<0>), dim3(grid), dim3(512), 0, s, a, tiles);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

}  // namespace pa
