// Layer3 / layer4 BasicBlock entries (conv 3x3 s2 + bn1 + relu, and the 1x1 s2 downsample + bn,
// one pass over the input; torchvision resnet18 layer3 / layer4 block 0 behind
// perseus/detector/models.py:20), fp16, with the weights resident in VGPRs and
// the K sum split over the waves by 64-channel input block.
//
// conv_s2v.hip holds the whole K of 32 output channels in a wave's VGPRs (K = 576 + 64 at Cin = 64:
// 160 VGPRs).  At Cin = 128 / 256 that is 2 / 4 times too many, so here a wave holds the weights
// of 32 output channels for ONE 64-channel input block (the same 160 VGPRs: 9 taps x 64 + the
// downsample's 64) and a workgroup of 8 waves is WN = 8 / NB channel quarters x NB input blocks.
// Every wave runs s2v's K loop over its block's patch region (0.45 ds_read_b128 per MFMA, no
// weight traffic through LDS at all), and at the end of a tile the NB partial sums of every
// output are exchanged through LDS and added in block order (block 0 + block 1 [+ 2 + 3]), each
// wave finalizing NU / NB of the tile's accumulator groups (NB = 2: the conv outputs on block 0's
// waves, the downsample's on block 1's).  Conv_s2w.h / conv_s2x.h instead stream a 16 KB weight
// tile per step through an LDS ring (0.75 fragment reads per MFMA + the ring's DMA writes, LDS
// bound: 0.28 / 0.24 of the MFMA peak).
//
// A workgroup owns 32 WN output channels (its "half" h of Cout) for the whole launch and walks
// 2 x TW output tiles persistently; the whole patch of a tile (5 input rows x (2 TW + 1) columns
// x Cin, 144-byte positions as conv_s2v.hip) is double-buffered, the next tile's DMA'd during
// this one.  One barrier per tile: the partials are written, the next patch has landed, the
// patch just read is free.
//   NB = 2, TW = 16 (layer3, 128 -> 256): 4 quarters x 2 blocks, 128 channels per workgroup
//   NB = 4, TW = 8  (layer4, 256 -> 512): 2 quarters x 4 blocks, 64 channels per workgroup;
//     a 16-pixel fragment is 2 output rows x 8, so a patch row pair is padded to 2 x 156 chunks
//     (row pitch = 64 mod 128 bytes): the fragment's two rows then fall on disjoint banks.
//
// Sum order: within a block, taps 3 4 5 0 1 2 6 7 8 (conv_s2w.h's order; the downsample with tap
// 4), then the blocks' partials added in block order.  Another order than conv_s2w.h / conv_s2x.h
// (which run the blocks in one accumulator), so not bit-identical to them; variants of this kernel
// agree bit for bit.
#include "conv_gx.h"

namespace pa {

__host__ __device__ constexpr int s2k_tap(int g) {  // group g: tap [3 4 5 0 1 2 6 7 8][g / 2], half g & 1
  return (g >> 1) < 3 ? 3 + (g >> 1) : ((g >> 1) < 6 ? (g >> 1) - 3 : (g >> 1));
}

template <int NB, int TW>
struct S2k {
  static constexpr int NWAVE = 8, WN = 8 / NB;
  static constexpr int TM = 2 * TW / 16;                  // 16-pixel fragments per wave (the tile's 2 rows)
  static constexpr int PW = 2 * TW + 1;                   // positions per input row: odd run, then even run
  static constexpr int RPC = TW == 16 ? PW * 9 : 156;     // 16-byte chunks per input row (TW = 8: padded)
  static constexpr int NRC = 5 * RPC;                     // chunks per block region (5 input rows)
  static constexpr int NCH = NB * NRC;
  static constexpr int PJ = (NCH + 63) / 64;              // patch wave-DMAs per tile
  static constexpr int PDW = (PJ + NWAVE - 1) / NWAVE;    // per wave
  static constexpr int PATCHB = PJ * 1024;
  static constexpr int NU = 4 * TM;                       // f32x4 accumulator groups per lane: (kind, tm, tn)
  static constexpr int UPW = NU / NB;                     // groups each wave finalizes
  static constexpr int XB = WN * NB * (NB - 1) * UPW * 1024;  // partials exchanged per tile
  static constexpr int SMEM = 2 * PATCHB + 2 * XB;
  static_assert(SMEM + 64 * WN * 4 <= 160 * 1024, "LDS");
  static_assert(UPW == 1 || UPW % 2 == 0, "finalize units");
};

__device__ __forceinline__ void store8(void* base, unsigned off, half4 v) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, (int)off, 0, 16);
}

// DBG = 4: s_memrealtime stamps into a.trace (0 start, 1 first patch landed; tile t: 2 + 3 t
// start, 3 + 3 t K loop done, 4 + 3 t barrier passed; 63 end)
template <int NB, int TW, int DBG = 0>
__global__ __launch_bounds__(512, 1) void conv3x3s2_k(ConvS2Args a, int ntiles, int nh, int xo) {
  using G = S2k<NB, TW>;
  constexpr int WN = G::WN, TM = G::TM, RPC = G::RPC, NRC = G::NRC, NCH = G::NCH, PJ = G::PJ, PDW = G::PDW;
  constexpr int PATCHB = G::PATCHB, NU = G::NU, UPW = G::UPW, XB = G::XB;
  constexpr int TN = 2, PXB = 144;
  __shared__ __attribute__((aligned(1024))) char smem[G::SMEM];
  __shared__ __attribute__((aligned(16))) float bias_l[64 * WN];  // [bias (32 WN) | bias2 (32 WN)]
  char* patch = smem;
  char* xch = smem + 2 * PATCHB;

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, r16 = lane & 15;
  const int wn = wid % WN, wb = wid / WN;  // channel quarter, input block
  if constexpr (DBG == 4) trace_stamp(a.trace, 0);
  const int H = a.Hout, W = a.Wout, Hin = a.Hin, Win = a.Win, Cin = a.Cin, Cout = a.Cout;
  // workgroup -> (channel half h, slot): xo = 1: blocks b and b + 8 (same XCD) take the halves of
  // the same tiles (the patch is an L2 hit for the second)
  const int b = blockIdx.x;
  int h, slot, nslots;
  if (xo) {
    h = (b >> 3) % nh;
    slot = (b & 7) + ((b >> 3) / nh) * 8;
    nslots = (int)gridDim.x / nh;
  } else {
    h = b % nh;
    slot = b / nh;
    nslots = (int)gridDim.x / nh;
  }
  const int c0 = h * 32 * WN;  // this workgroup's first output channel
  const int tw_n = W / TW, tpi = (H / 2) * tw_n;
  // XCD-grouped tile order (conv_s2v.hip): an image's tiles on one XCD in one round
  const bool xm = xo && nslots % 8 == 0 && ntiles % (8 * tpi) == 0;
  auto tmap = [&](int j) __attribute__((always_inline)) {
    if (!xm) return j;
    const int c = j / (8 * tpi), r = j - c * 8 * tpi;
    return c * 8 * tpi + (r & 7) * tpi + (r >> 3);
  };

  const unsigned abytes =
      (unsigned)((size_t)a.B * Hin * Win * Cin * 2 < 0x7fffffffu ? (size_t)a.B * Hin * Win * Cin * 2 : 0x7fffffffu);
  const s2w_u4 rsrc = s2w_rsrc(a.in, abytes);
  struct Org {
    int img, h0, x0;
    bool on;
  };
  auto origin = [&](int t, bool on) __attribute__((always_inline)) {
    const int img = t / tpi, rem = t - img * tpi;
    return Org{img, 2 * 2 * (rem / tw_n) - 1, 2 * (rem - (rem / tw_n) * tw_n) * TW - 1, on};
  };
  // patch DMA i of this wave: chunk c = (i * 8 + wid) * 64 + lane of the tile's patch = block
  // c / NRC, input row (c % NRC) / RPC, position p = (c % RPC) / 9 (run: odd columns 0 .. TW, even
  // columns TW + 1 ..), chunk position c % 9 (8: pad) = input channels 8 ((pos & 1) * 4 + (pos >> 1))
  // of the block.  Packed: bits 0-17 byte offset from the patch origin, 18-21 row, 22-27 column
  // offset, 28 pad / past the patch.
  unsigned pk[PDW];
#pragma unroll
  for (int i = 0; i < PDW; ++i) {
    const int c = (i * 8 + wid) * 64 + lane;
    const int blk = c / NRC, rc = c - blk * NRC, pr = rc / RPC, rem = rc - pr * RPC;
    const int p = rem / 9, pos = rem - p * 9;
    const bool bad = c >= NCH || pos >= 8 || p >= G::PW;
    const int co = bad ? 0 : (p <= TW ? 2 * p : 2 * (p - TW - 1) + 1);
    const int row = bad ? 0 : pr;
    const unsigned rel = bad ? 0u : (unsigned)(((row * Win + co) * Cin + 64 * blk + ((pos & 1) * 4 + (pos >> 1)) * 8) * 2);
    pk[i] = (rel & 0x3ffffu) | ((unsigned)row << 18) | ((unsigned)co << 22) | ((bad ? 1u : 0u) << 28);
  }
  auto dma_one = [&](int i, const Org& o, int buf) __attribute__((always_inline)) {
    if (PJ == PDW * 8 || i < PDW - 1 || wid < PJ - (PDW - 1) * 8) {  // wave-uniform
      const unsigned v = pk[i];
      const int pr = (int)((v >> 18) & 15u), co = (int)((v >> 22) & 63u);
      const unsigned tb = (unsigned)(((o.img * Hin + o.h0) * Win + o.x0) * Cin * 2);  // wave-uniform (may wrap)
      const bool ok = o.on && !(v >> 28) && (unsigned)(o.h0 + pr) < (unsigned)Hin && (unsigned)(o.x0 + co) < (unsigned)Win;
      s2w_dma16(rsrc, ok ? tb + (v & 0x3ffffu) : S2W_OOB, patch + buf * PATCHB + (i * 8 + wid) * 1024);
    }
  };

  const int o = xfrag(r16);
  // this lane's patch-read base per fragment: pixel m = 16 tm + o of the 2 x TW tile (row y, column
  // x) reads patch row 2 y (+ tap row), position x (+ tap offset), chunk position 2 q (+ half)
  // (TW = 16: fragment tm is output row tm, a compile-time offset of 2 tm patch rows)
  constexpr int NRB = TW == 16 ? 1 : TM;
  unsigned rbase[NRB];
#pragma unroll
  for (int tm = 0; tm < NRB; ++tm) {
    const int m = 16 * tm + o, y = m / TW, x = m - (m / TW) * TW;
    rbase[tm] = (unsigned)(size_t)(__attribute__((address_space(3))) char*)patch +
                (unsigned)(wb * NRC * 16 + 2 * y * RPC * 16 + x * PXB + q * 32);
  }
  if (tid < 32 * WN) {
    bias_l[tid] = a.bias[c0 + tid];
    bias_l[32 * WN + tid] = a.bias2[c0 + tid];
  }
  __builtin_amdgcn_sched_barrier(0);

  // prologue: the first tile's patch, then this wave's weight fragments straight into its VGPRs
  // in the order the K loop uses them (wfrag: [h][wb][wn][fragment 20][tn 2][lane 64][8 fp16])
  int j = slot;
  {
    const Org o0 = origin(tmap(j < ntiles ? j : 0), j < ntiles);
#pragma unroll
    for (int i = 0; i < PDW; ++i) dma_one(i, o0, 0);
  }
  xu4 wr[18][TN], wd[2][TN];
  {
    const xu4* __restrict__ wf =
        reinterpret_cast<const xu4*>(a.wfrag) + (size_t)((h * NB + wb) * WN + wn) * 20 * TN * 64 + lane;
    gx_for<0, 18>([&](auto gc) __attribute__((always_inline)) {
      constexpr int Gi = decltype(gc)::value, TAP = s2k_tap(Gi), K = 2 * TAP + (Gi & 1);
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) wr[K][tn] = wf[(K * TN + tn) * 64];
      if constexpr (TAP == 4) {
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) wd[Gi & 1][tn] = wf[((18 + (Gi & 1)) * TN + tn) * 64];
      }
    });
  }
  // the first patch landed (this wave's DMAs, issued before the weight loads) and every wave's
  xwait_vm<18 * TN + 2 * TN>();
  lds_barrier();
  if constexpr (DBG == 4) trace_stamp(a.trace, 1);

  _Float16* __restrict__ out = (_Float16*)a.out;
  _Float16* __restrict__ out2 = (_Float16*)a.out2;
  int jn = j + nslots;
  // one tile; the first is its own copy of the body (FIRST): there the compiler's vmcnt waits
  // hold each group's MFMAs until that group's weight fragments have landed
  auto run_tile = [&](auto firstc, int t) __attribute__((always_inline)) {
    constexpr bool FIRST = decltype(firstc)::value;
    const int buf = t & 1;
    const int tile = tmap(j);
    const bool has_next = jn < ntiles;
    const Org onext = origin(has_next ? tmap(jn) : tile, has_next);
    const int img = tile / tpi, rem = tile - img * tpi;
    const int th0 = (rem / tw_n) * 2, tw0 = (rem - (rem / tw_n) * tw_n) * TW;
    if constexpr (DBG == 4) trace_stamp(a.trace, 2 + 3 * t);

    f32x4 acc[TM][TN], accd[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int k = 0; k < TN; ++k) {
        acc[i][k] = f32x4{0.f, 0.f, 0.f, 0.f};
        accd[i][k] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    xu4 fb[2][TM];
    auto rd = [&](auto gc) __attribute__((always_inline)) {
      constexpr int Gi = decltype(gc)::value, TAP = s2k_tap(Gi), HG = Gi & 1, S = Gi & 1;
      constexpr int KH = TAP / 3, KW = TAP % 3;
      constexpr int OFF = KH * RPC * 16 + (KW == 0 ? 0 : (KW == 1 ? TW + 1 : 1)) * PXB + HG * 16;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
        fb[S][tm] = *reinterpret_cast<const __attribute__((address_space(3))) xu4*>(
            (const __attribute__((address_space(3))) char*)(size_t)(rbase[TW == 16 ? 0 : tm] + buf * PATCHB) + OFF +
            (TW == 16 ? 2 * tm * RPC * 16 : 0));
    };
    auto mm = [&](auto gc) __attribute__((always_inline)) {
      constexpr int Gi = decltype(gc)::value, TAP = s2k_tap(Gi), HG = Gi & 1, S = Gi & 1;
      constexpr int K = 2 * TAP + HG;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, wr[K][tn]),
                                                               __builtin_bit_cast(half8, fb[S][tm]), acc[tm][tn], 0, 0, 0);
      if constexpr (TAP == 4) {  // the downsample reads tap 4's pixels: (2 y, 2 x), same fragments
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
          for (int tn = 0; tn < TN; ++tn)
            accd[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, wd[HG][tn]),
                                                                  __builtin_bit_cast(half8, fb[S][tm]), accd[tm][tn], 0, 0, 0);
      }
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
      }
      mm(gc);
    });
    if constexpr (DBG == 4) trace_stamp(a.trace, 3 + 3 * t);

    // partial sums: group u = kind * 2 TM + tm * 2 + tn (kind 0 conv, 1 downsample); wave (wn, wb)
    // finalizes groups wb * UPW .. + UPW - 1 and sends the others to their owners
    auto grp = [&](auto uc) __attribute__((always_inline)) -> f32x4& {
      constexpr int u = decltype(uc)::value, kind = u / (2 * TM), tm = (u / 2) % TM, tn = u & 1;
      if constexpr (kind) return accd[tm][tn];
      else return acc[tm][tn];
    };
    char* xb = xch + buf * XB;
    // slot of (owner ow, source sb, unit k) in this quarter's exchange area
    auto xoff = [&](int ow, int sb, int k) __attribute__((always_inline)) {
      const int s = sb < ow ? sb : sb - 1;
      return ((((wn * NB + ow) * (NB - 1) + s) * UPW + k) * 64 + lane) * 16;
    };
    // (wb is wave-uniform: one compile-time copy per block, the accumulators indexed statically)
    gx_for<0, NB>([&](auto wc) __attribute__((always_inline)) {
      constexpr int WB = decltype(wc)::value;
      if (wb == WB) {
        gx_for<0, NU>([&](auto uc) __attribute__((always_inline)) {
          constexpr int u = decltype(uc)::value, ow = u / UPW;
          if constexpr (ow != WB) *reinterpret_cast<f32x4*>(xb + xoff(ow, WB, u - ow * UPW)) = grp(uc);
        });
      }
    });
    xwait_vm<0>();  // next patch landed (this wave's DMAs; the previous tile's stores)
    lds_barrier();  // ... every wave's, the partials written, every read of buf retired
    if constexpr (DBG == 4) trace_stamp(a.trace, 4 + 3 * t);

    // finalize this wave's groups: blocks added in order 0, 1, ..; + bias (+ relu) -> fp16
    gx_for<0, NB>([&](auto wc) __attribute__((always_inline)) {
      constexpr int WB = decltype(wc)::value;
      if (wb != WB) return;
      f32x4 fin[UPW];
      gx_for<0, UPW>([&](auto kc) __attribute__((always_inline)) {
        constexpr int k = decltype(kc)::value;
        f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
        gx_for<0, NB>([&](auto sc) __attribute__((always_inline)) {
          constexpr int SB = decltype(sc)::value;
          f32x4 v;
          if constexpr (SB == WB)
            v = grp(xic<WB * UPW + k>{});
          else
            v = *reinterpret_cast<const f32x4*>(xb + xoff(WB, SB, k));
          if constexpr (SB == 0)
            s = v;
          else
            s = s + v;
        });
        fin[k] = s;
      });
#pragma unroll
      for (int k = 0; k < UPW; k += (UPW > 1 ? 2 : 1)) {
        const int u = WB * UPW + k;
        const int kind = u / (2 * TM), tm = (u / 2) % TM, tn = u & 1;
        const int m = 16 * tm + o, y = m / TW, x = m - (m / TW) * TW;
        const int ch = 32 * wn + 8 * q + 4 * tn;  // (tn = 0 when UPW > 1: the pair's first)
        const f32x4* b4 = reinterpret_cast<const f32x4*>(bias_l + kind * 32 * WN + ch);
        const unsigned ob = (unsigned)((((img * H + th0 + y) * W + tw0 + x) * Cout + c0 + ch) * 2);
        _Float16* dst = kind ? out2 : out;
        if constexpr (UPW > 1) {
          const f32x4 b0 = b4[0], b1 = b4[1];
          half8 hv;
#pragma unroll
          for (int e8 = 0; e8 < 8; ++e8) {
            const float v = fin[k + (e8 >> 2)][e8 & 3] + (e8 < 4 ? b0 : b1)[e8 & 3];
            hv[e8] = (_Float16)(kind ? v : fmaxf(v, 0.f));
          }
          store16<true>(dst, ob, hv);
        } else {
          const f32x4 b0 = b4[0];
          half4 hv;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float v = fin[k][e] + b0[e];
            hv[e] = (_Float16)(kind ? v : fmaxf(v, 0.f));
          }
          store8(dst, ob, hv);
        }
      }
    });
    j = jn;
    jn = j + nslots;
  };
  const bool any = j < ntiles;
  if (any) run_tile(std::true_type{}, 0);
  for (int t = 1; j < ntiles; ++t) run_tile(std::false_type{}, t);  // (run_tile advances j)
  if constexpr (DBG == 4) {
    __builtin_amdgcn_s_waitcnt(0);
    trace_stamp(a.trace, 63);
  }
}

template <int NB, int TW, int DBG = 0>
static int run_s2k(const ConvS2Args& a, hipStream_t s) {
  using G = S2k<NB, TW>;
  const int nh = a.Cout / (32 * G::WN);
  const int tiles = a.B * (a.Hout / 2) * (a.Wout / TW);
  const int cus = conv_stream_cus(s);
  // one 8-wave workgroup per CU; per channel half a slot count that keeps b and b + 8 on one XCD
  int grid = (cus / (8 * nh)) * 8 * nh;
  int xo = 1;
  if (grid == 0) {  // a few CUs (CU-masked stream): plain order
    grid = cus >= nh ? (cus / nh) * nh : nh;
    xo = 0;
  }
  const int per_half = grid / nh;
  if (per_half > tiles) grid = (xo ? ((tiles + 7) / 8) * 8 : tiles) * nh;
  hipLaunchKernelGGL((conv3x3s2_k<NB, TW, DBG>), dim3(grid), dim3(512), 0, s, a, tiles, nh, xo);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

// variant 0: shipped; 1: s_memrealtime stamps into a.trace
int launch_conv3x3s2_k(const ConvS2Args& a, int variant, hipStream_t s, const char** kname) {
  PA_CHECK(a.wfrag, "s2k conv: no VGPR-order weights (ConvS2Args::wfrag)");
  PA_CHECK(a.Hin == 2 * a.Hout && a.Win == 2 * a.Wout && a.Hout % 2 == 0, "s2k conv: %dx%d -> %dx%d", a.Hin, a.Win,
           a.Hout, a.Wout);
  PA_CHECK((size_t)a.B * a.Hin * a.Win * a.Cin * 2 < 0x7fffffffu && (size_t)a.B * a.Hout * a.Wout * a.Cout * 2 < 0x7fffffffu,
           "s2k conv: activations over 2 GB");
  if (a.B <= 0) return PA_OK;
  if (a.Cin == 128 && a.Cout == 256 && a.Wout == 16) {
    PA_CHECK(a.Win <= 32, "s2k conv: input width %d", a.Win);
    if (kname) *kname = "conv3x3s2k_l3";
    if (variant == 1 && a.trace) return run_s2k<2, 16, 4>(a, s);
    return run_s2k<2, 16>(a, s);
  }
  if (a.Cin == 256 && a.Cout == 512 && a.Wout == 8) {
    if (kname) *kname = "conv3x3s2k_l4";
    if (variant == 1 && a.trace) return run_s2k<4, 8, 4>(a, s);
    return run_s2k<4, 8>(a, s);
  }
  set_error("s2k conv: no configuration for %d -> %d, %dx%d", a.Cin, a.Cout, a.Hout, a.Wout);
  return PA_EINVAL;
}

}  // namespace pa
