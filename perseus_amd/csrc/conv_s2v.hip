// Layer2 BasicBlock entry (conv 3x3 s2 + bn1 + relu, and the 1x1 s2 downsample + bn, one pass
// over the input; torchvision resnet18 layer2 block 0 behind perseus/detector/models.py:20,
// SURVEY.md 8a6), fp16, with the weights resident in VGPRs: conv_c64v.hip's design on the
// stride-2 entry (Cin = 64, so K = 576 like layer1).
//
// conv_s2w.h streams a 16 KB weight tile per step through an LDS ring behind one barrier per step
// and runs 8 waves of 32 px x 64 ch (0.75 ds_read_b128 per MFMA): 0.22 of the MFMA peak.  Here
// each wave owns 32 output pixels (two output rows of a TH x 16 tile) x 32 output channels and
// holds those channels' weights for all 576 K of the conv (144 VGPRs) and the 64 K of the
// downsample (16 VGPRs) for the whole launch.  The K loop reads only pixel fragments: 2 per
// (tap, 32-channel) group for 4 MFMAs (0.5 per MFMA), and the downsample reads none of its own
// (its input pixel is tap 4's, so its MFMAs reuse tap 4's fragments).  A workgroup of 2 TH waves
// (4 channel quarters x TH / 2 row pairs) walks TH x 16 x 128 tiles persistently; the whole patch
// of a tile (2 TH + 1 input rows x 33 input columns x 64 channels) is double-buffered, the next
// tile's DMA'd during this one, so a tile needs one barrier (the hand-over).  TH = 2 (shipped):
// 4 waves, two workgroups per CU (a SIMD's two waves in different workgroups, so neither waits for
// the other at a tile boundary, as conv_c64v.hip's residual form); TH = 4: 8 waves, one per CU.
//
// The weights come straight from HBM / L2 into the VGPRs: pa_detector_create packs them in
// register order (ConvS2Args::wfrag: [wave][fragment][tile][lane][8 fp16]), so each load is one
// contiguous KB per wave-instruction, issued in the order the K loop uses them; the compiler's
// own vmcnt waits hold each MFMA of the first tile until its fragment has landed, so the first
// tile computes while the rest of the weights arrive.  (Staging them through LDS in two rounds
// of 80 KB, one 8-wave workgroup per CU, took 5.5 us before the first tile could start:
// profiles/r06b.)
//
// Patch layout: 33 positions per input row, the 17 odd input columns 2 tw0 - 1 + 2 j first
// (kw = 0 reads position x, kw = 2 position x + 1), then the 16 even ones 2 tw0 + 2 j (kw = 1 and
// the downsample: position 17 + x), so a fragment's 16 consecutive output pixels read 16
// consecutive positions; 144 bytes per position (conv_c64v.hip's 8 data chunks + 1 pad chunk,
// the chunk of input channels 32 h + 8 q .. + 7 at 2 q + h): one VGPR plus ds_read immediates
// addresses every fragment of the loop, and the ds_read_b128 lane groups are conflict-free
// (conv_c64v.hip: with the xfrag pixel order a group's q = 0 lanes hit the even 16-byte bank
// quads, its q = 1 lanes the odd ones).
//
// Sum order (bit-identity): each conv accumulator adds its MFMAs tap by tap in conv_s2w.h's
// order (taps 3 4 5, 0 1 2, 6 7 8; the two 32-channel halves of each tap in order), the
// downsample's its two halves, and the epilogue is conv_s2w.h's, so the outputs are bit for
// bit those of the round-5 kernel (variant 6:40).
#include "conv_gx.h"

namespace pa {

// group g of a tile's K loop: conv_s2w.h's tap order [3 4 5 0 1 2 6 7 8][g / 2], half g & 1
__host__ __device__ constexpr int s2v_tap(int g) {
  return (g >> 1) < 3 ? 3 + (g >> 1) : ((g >> 1) < 6 ? (g >> 1) - 3 : (g >> 1));
}

template <int TH>
struct S2v {
  static constexpr int TW = 16;
  static constexpr int PH = 2 * TH + 1, PW = 2 * TW + 1, NP = PH * PW;  // input rows / positions per row
  static constexpr int NWAVE = 2 * TH;                  // wave = 2 output rows x one channel quarter
  static constexpr int PXB = 144;                       // bytes per patch position (8 chunks + 1 pad)
  static constexpr int PJ = (NP * 9 + 63) / 64;         // patch wave-DMAs (TH = 4: 42)
  static constexpr int PATCHB = PJ * 1024;
  static constexpr int PDW = (PJ + NWAVE - 1) / NWAVE;  // per wave (TH = 2: 6, 4: 6), the last round partial
  static constexpr int SMEM = 2 * PATCHB;
  static constexpr int WGCU = TH == 2 ? 2 : 1;          // workgroups per CU
  static_assert((SMEM + 1024) * WGCU <= 160 * 1024, "LDS");
};

// DBG = 4: s_memrealtime stamps into a.trace (0 start, 1 first patch landed; tile t: 2 + 4 t start,
// 3 + 4 t K loop done and next patch landed, 4 + 4 t stores issued; 63 end)
// DS (deferred stores): a tile's outputs stay in 16 VGPRs and go out during the next tile's K
// loop, one 16-byte store per group after the patch DMAs (every CU ends its tiles at about the
// same time, so stores issued at the tile end queue behind the whole chip's: ~0.8 us per tile,
// profiles/r06c trace)
template <int TH, int DBG = 0, bool DS = false>
__global__ __launch_bounds__(TH * 128, 2) void conv3x3s2_v(ConvS2Args a, int ntiles) {
  using G = S2v<TH>;
  constexpr int TW = G::TW, PW = G::PW, NP = G::NP, NWAVE = G::NWAVE, PXB = G::PXB, PJ = G::PJ;
  constexpr int PATCHB = G::PATCHB, PDW = G::PDW;
  constexpr int TM = 2, TN = 2;  // wave tile: 32 pixels (2 rows of 16) x 32 channels
  __shared__ __attribute__((aligned(1024))) char smem[G::SMEM];
  __shared__ __attribute__((aligned(16))) float bias_l[256];  // [bias (128) | bias2 (128)]
  char* patch = smem;

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, r16 = lane & 15;
  const int wn = wid & 3, wm = wid >> 2;  // channel quarter, output rows 2 wm, 2 wm + 1 of the tile
  if constexpr (DBG == 4) trace_stamp(a.trace, 0);
  const int H = a.Hout, W = a.Wout, Hin = a.Hin, Win = a.Win;
  const _Float16* __restrict__ in = (const _Float16*)a.in;
  const _Float16* __restrict__ w = (const _Float16*)a.w;
  const _Float16* __restrict__ wds = (const _Float16*)a.wds;
  const int tw_n = W / TW, tpi = (H / TH) * tw_n;
  // XCD-grouped tile order (conv_c64d.hip XM): an image's tiles on one XCD in one round
  const bool xm = ntiles % (8 * tpi) == 0;
  auto tmap = [&](int j) __attribute__((always_inline)) {
    if (!xm) return j;
    const int c = j / (8 * tpi), r = j - c * 8 * tpi;
    return c * 8 * tpi + (r & 7) * tpi + (r >> 3);
  };

  const unsigned abytes =
      (unsigned)((size_t)a.B * Hin * Win * 128 < 0x7fffffffu ? (size_t)a.B * Hin * Win * 128 : 0x7fffffffu);
  const s2w_u4 rsrc = s2w_rsrc(in, abytes);
  struct Org {
    int img, h0, x0;  // input row / column of patch position (0, 0): 2 th0 - 1, 2 tw0 - 1
    bool on;
  };
  auto origin = [&](int t, bool on) __attribute__((always_inline)) {
    const int img = t / tpi, rem = t - img * tpi;
    return Org{img, 2 * (rem / tw_n) * TH - 1, 2 * (rem - (rem / tw_n) * tw_n) * TW - 1, on};
  };
  // patch DMA i of this wave: LDS slot c = (i * NWAVE + wid) * 64 + lane (16-byte units) holds
  // position p = c / 9 (input row pr = p / PW, position pc = p % PW), chunk position c % 9 (8: pad)
  // = input channels 8 ((pos & 1) * 4 + (pos >> 1)) .. + 7.  One packed word per lane and DMA:
  // bits 0-17 the byte offset from the patch origin, 18-21 the row, 22-27 the column offset
  // (position -> column: odd run 2 pc, even run 2 (pc - 17) + 1), 28 pad / past the patch.
  unsigned pk[PDW];
#pragma unroll
  for (int i = 0; i < PDW; ++i) {
    const int c = (i * NWAVE + wid) * 64 + lane;
    const int p = c / 9, pos = c - p * 9;
    const int pr = p < NP ? p / PW : 0, pc = p < NP ? p - (p / PW) * PW : 0;
    const int co = pc <= TW ? 2 * pc : 2 * (pc - TW - 1) + 1;
    const unsigned bad = (pos >= 8 || p >= NP) ? 1u : 0u;
    const unsigned rel = (unsigned)(((pr * Win + co) * 64 + ((pos & 1) * 4 + (pos >> 1)) * 8) * 2);
    pk[i] = (rel & 0x3ffffu) | ((unsigned)pr << 18) | ((unsigned)co << 22) | (bad << 28);
  }
  auto dma_patch = [&](int i, const Org& o, int buf) __attribute__((always_inline)) {
    const unsigned v = pk[i];
    const int pr = (int)((v >> 18) & 15u), co = (int)((v >> 22) & 63u);
    const unsigned tb = (unsigned)(((o.img * Hin + o.h0) * Win + o.x0) * 128);  // wave-uniform (may wrap)
    const bool ok = o.on && !(v >> 28) && (unsigned)(o.h0 + pr) < (unsigned)Hin && (unsigned)(o.x0 + co) < (unsigned)Win;
    s2w_dma16(rsrc, ok ? tb + (v & 0x3ffffu) : S2W_OOB, patch + buf * PATCHB + (i * NWAVE + wid) * 1024);
  };
  auto dma_one = [&](int i, const Org& o, int buf) __attribute__((always_inline)) {
    if constexpr (PJ == PDW * NWAVE)
      dma_patch(i, o, buf);
    else if (i < PDW - 1 || wid < PJ - (PDW - 1) * NWAVE)
      dma_patch(i, o, buf);  // wave-uniform
  };

  const int o = xfrag(r16);
  // this lane's patch-read base: input row 4 wm (of the patch), position o, chunk position 2 q
  const unsigned rbase =
      (unsigned)(size_t)(__attribute__((address_space(3))) char*)patch + (unsigned)((4 * wm * PW + o) * PXB + q * 32);
  if (tid < 128) {
    bias_l[tid] = a.bias[tid];
    bias_l[128 + tid] = a.bias2[tid];
  }
  __builtin_amdgcn_sched_barrier(0);

  // prologue: the first tile's patch, then every weight fragment of this wave straight into its
  // VGPRs, in the order the K loop uses them (k: tap k / 2, half k & 1; the downsample with tap 4)
  int j = blockIdx.x;
  {
    const Org o0 = origin(tmap(j), true);
#pragma unroll
    for (int i = 0; i < PDW; ++i) dma_one(i, o0, 0);
  }
  xu4 wr[18][TN], wd[2][TN];
  {
    const xu4* __restrict__ wf = reinterpret_cast<const xu4*>(a.wfrag) + (size_t)wn * 20 * TN * 64 + lane;
    gx_for<0, 18>([&](auto gc) __attribute__((always_inline)) {
      constexpr int Gi = decltype(gc)::value, TAP = s2v_tap(Gi), K = 2 * TAP + (Gi & 1);
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) wr[K][tn] = wf[(K * TN + tn) * 64];
      if constexpr (TAP == 4) {
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) wd[Gi & 1][tn] = wf[((18 + (Gi & 1)) * TN + tn) * 64];
      }
    });
  }
  // the first patch landed (this wave's DMAs: issued before the weight loads) and every wave's
  xwait_vm<18 * TN + 2 * TN>();
  lds_barrier();
  if constexpr (DBG == 4) trace_stamp(a.trace, 1);

  _Float16* __restrict__ out = (_Float16*)a.out;
  _Float16* __restrict__ out2 = (_Float16*)a.out2;
  int jn = j + (int)gridDim.x;
  half8 pend[2 * TM];       // DS: the previous tile's outputs (out rows tm, then out2 rows tm)
  unsigned pend_base = 0;   // DS: their tile's byte offset (wave-uniform)
  unsigned olane[TM];       // this lane's byte offset in a tile: row 2 wm + tm, pixel o, channels 32 wn + 8 q
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) olane[tm] = (unsigned)((((2 * wm + tm) * W + o) * 128 + wn * 32 + q * 8) * 2);
  // one tile; the first is its own copy of the body (FIRST): there the compiler's vmcnt waits
  // hold each group's MFMAs until that group's weight fragments have landed (in a loop the waits
  // would cover every weight load at the first group)
  auto run_tile = [&](auto firstc, int t) __attribute__((always_inline)) {
    constexpr bool FIRST = decltype(firstc)::value;
    const int buf = t & 1;
    const int tile = tmap(j);
    const bool has_next = jn < ntiles;
    const Org onext = origin(has_next ? tmap(jn) : tile, has_next);
    const int img = tile / tpi, rem = tile - img * tpi;
    const int th0 = (rem / tw_n) * TH, tw0 = (rem - (rem / tw_n) * tw_n) * TW;
    if constexpr (DBG == 4) trace_stamp(a.trace, 2 + 4 * t);

    f32x4 acc[TM][TN], accd[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int k = 0; k < TN; ++k) {
        acc[i][k] = f32x4{0.f, 0.f, 0.f, 0.f};
        accd[i][k] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    const __attribute__((address_space(3))) char* pb =
        (const __attribute__((address_space(3))) char*)(size_t)(rbase + buf * PATCHB);
    xu4 fb[2][TM];
    auto rd = [&](auto gc) __attribute__((always_inline)) {
      constexpr int Gi = decltype(gc)::value, TAP = s2v_tap(Gi), HG = Gi & 1, S = Gi & 1;
      constexpr int KH = TAP / 3, KW = TAP % 3;
      constexpr int POFF = KW == 0 ? 0 : (KW == 1 ? TW + 1 : 1);
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
        fb[S][tm] = *reinterpret_cast<const __attribute__((address_space(3))) xu4*>(
            pb + ((2 * tm + KH) * PW + POFF) * PXB + HG * 16);
    };
    auto mm = [&](auto gc) __attribute__((always_inline)) {
      constexpr int Gi = decltype(gc)::value, TAP = s2v_tap(Gi), HG = Gi & 1, S = Gi & 1;
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
      if constexpr (Gi < PDW) {  // next tile's patch, one DMA per group
        __builtin_amdgcn_sched_barrier(0);
        dma_one(Gi, onext, buf ^ 1);  // (no next tile: onext.on = false, zeros into buf ^ 1)
        __builtin_amdgcn_sched_barrier(0);
      } else if constexpr (DS && !FIRST && Gi < PDW + 2 * TM) {  // the previous tile's outputs
        constexpr int I = Gi - PDW;
        __builtin_amdgcn_sched_barrier(0);
        store16<true>(I < TM ? out : out2, pend_base + olane[I % TM], pend[I]);
        __builtin_amdgcn_sched_barrier(0);
      }
      mm(gc);
    });
    // next patch landed (this wave's DMAs; DS: the previous tile's stores, issued after them,
    // may still be in flight)
    if constexpr (DS && !FIRST)
      xwait_vm<2 * TM>();
    else
      xwait_vm<0>();
    if constexpr (DBG == 4) trace_stamp(a.trace, 3 + 4 * t);

    // epilogue (conv_s2w.h's): lane (q, r16) holds channels 32 wn + 8 q .. + 7 of pixel o of rows
    // 2 wm + tm (conv_gx.h xperm): relu(conv + bias) -> out, downsample + bias2 -> out2
    const f32x4* b4 = reinterpret_cast<const f32x4*>(bias_l + wn * 32 + q * 8);
    const f32x4 b0 = b4[0], b1 = b4[1], d0 = b4[32], d1 = b4[33];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
      half8 h1, h2;
#pragma unroll
      for (int e8 = 0; e8 < 8; ++e8) {
        const int tn = e8 >> 2, e = e8 & 3;
        h1[e8] = (_Float16)fmaxf(acc[tm][tn][e] + (e8 < 4 ? b0 : b1)[e], 0.f);
        h2[e8] = (_Float16)(accd[tm][tn][e] + (e8 < 4 ? d0 : d1)[e]);
      }
      if constexpr (DS) {
        pend[tm] = h1;
        pend[TM + tm] = h2;
      } else {
        const unsigned ob = (unsigned)((((img * H + th0 + 2 * wm + tm) * W + tw0 + o) * 128 + wn * 32 + q * 8) * 2);
        store16<true>(out, ob, h1);
        store16<true>(out2, ob, h2);
      }
    }
    if constexpr (DS) pend_base = (unsigned)(((img * H + th0) * W + tw0) * 256);
    if constexpr (DBG == 4) trace_stamp(a.trace, 4 + 4 * t);
    // every wave's DMAs into buf ^ 1 landed (its wait above) and its reads of buf retired
    lds_barrier();
    j = jn;
    jn = j + (int)gridDim.x;
  };
  const bool any = j < ntiles;
  if (any) run_tile(std::true_type{}, 0);
  for (int t = 1; j < ntiles; ++t) run_tile(std::false_type{}, t);
  if constexpr (DS) {  // the last tile's outputs
    if (any) {
#pragma unroll
      for (int i = 0; i < 2 * TM; ++i) store16<true>(i < TM ? out : out2, pend_base + olane[i % TM], pend[i]);
    }
  }
  if constexpr (DBG == 4) {
    __builtin_amdgcn_s_waitcnt(0);
    trace_stamp(a.trace, 63);
  }
}

template <int TH, int DBG = 0, bool DS = false>
static int run_s2v(const ConvS2Args& a, hipStream_t s) {
  const int tiles = a.B * (a.Hout / TH) * (a.Wout / 16);
  const int slots = conv_stream_cus(s) * S2v<TH>::WGCU;  // resident workgroups
  const int grid = tiles < slots ? tiles : slots;
  hipLaunchKernelGGL((conv3x3s2_v<TH, DBG, DS>), dim3(grid), dim3(TH * 128), 0, s, a, tiles);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

// variant 0: shipped (2 x 16 tiles, 4 waves, two workgroups per CU); 1: 4 x 16 tiles, 8 waves, one
// workgroup per CU; 2 / 3: 0 / 1 with deferred stores (DS); 4 / 5 / 6: s_memrealtime stamps into
// a.trace (0 / 1 / 2)
int launch_conv3x3s2_v(const ConvS2Args& a, int variant, hipStream_t s, const char** kname) {
  PA_CHECK(a.wfrag, "s2v conv: no VGPR-order weights (ConvS2Args::wfrag)");
  PA_CHECK(a.Cin == 64 && a.Cout == 128, "s2v conv: Cin 64 -> Cout 128 only (weights in VGPRs), got %d -> %d", a.Cin,
           a.Cout);
  PA_CHECK(a.Hin == 2 * a.Hout && a.Win == 2 * a.Wout, "s2v conv: %dx%d -> %dx%d", a.Hin, a.Win, a.Hout, a.Wout);
  PA_CHECK(a.Hout % 4 == 0 && a.Wout % 16 == 0, "s2v conv: %dx%d not tiled by 4x16", a.Hout, a.Wout);
  PA_CHECK(a.Cin * 9 == 576, "s2v conv: weights in VGPRs for K = 576 only");
  PA_CHECK(a.Win <= 200, "s2v conv: input width %d (packed patch offsets: 18 bits)", a.Win);
  PA_CHECK((size_t)a.B * a.Hin * a.Win * 128 < 0x7fffffffu && (size_t)a.B * a.Hout * a.Wout * 256 < 0x7fffffffu,
           "s2v conv: activations over 2 GB");
  if (a.B <= 0) return PA_OK;
  if (kname) *kname = "conv3x3s2v_l2";
  if (variant == 4 && a.trace) return run_s2v<2, 4>(a, s);
  if (variant == 5 && a.trace) return run_s2v<4, 4>(a, s);
  if (variant == 1) return run_s2v<4>(a, s);
  if (variant == 2) return run_s2v<2, 0, true>(a, s);
  if (variant == 3) return run_s2v<4, 0, true>(a, s);
  if (variant == 6 && a.trace) return run_s2v<2, 4, true>(a, s);
  return run_s2v<2>(a, s);
}

}  // namespace pa
