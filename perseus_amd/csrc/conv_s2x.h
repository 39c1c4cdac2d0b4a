// Stride-2 BasicBlock entry on conv_gx.h's machinery, fp16: conv 3x3 s2 (+ bn1,
// relu) and the 1x1 s2 downsample (+ bn) in one pass over the input
// (torchvision resnet18 layer2/3/4 block 0; replaces the
// one-tile kernel of conv_s2.hip on the fp16 path).
//
// The downsample reads input pixel (2y, 2x), the centre tap of the 3x3 window of
// output (y, x): per 64-channel input block the K loop has 10 steps, the 9 taps
// into `acc` and the downsample slice (its 1x1 weights against the centre tap's
// patch pixels) into `accd`.  Every step is a conv_gx step: weight tile DMA'd
// PD steps ahead into a ring, fragments read half a step ahead, compile-time
// vmcnt plan (GxPlan with 10 steps per block), a bare s_barrier every G steps.
//
// Patch: (2TH + 1) input rows x (2TW + 1) columns, stored de-interleaved (the TW + 1
// even input columns, then the TW odd ones) so that for every tap 16 consecutive
// output columns read 16 consecutive LDS positions; out-of-image pixels read a
// zero line.  Output pixels are row-major over the TH x TW tile (16-pixel MFMA
// fragment = one row at TW = 16, two rows at TW = 8; for TW = 8 the row pitch is
// padded to 20 positions so the two rows of a fragment fall on disjoint banks).
//
// X3 (fp16x3 parity mode): activation / weight hi-lo planes and 3 virtual blocks per
// 64-channel block, as conv_gx.h's X3; the downsample's weights carry their own
// per-channel power-of-2 scale (scale2).
//
// TPW > 1: one workgroup runs TPW spatial tiles (same output channels, same image) as
// ONE step stream: the weight ring runs on across the tile boundary, the next tile's
// first patch is DMA'd during the current tile's K loop like any next block's patch, and
// a tile's output stores open the next tile's first step (counted in the vmcnt plan:
// loads, stores and LDS-DMA retire in issue order).  At B = 64 the layer2 / layer3
// entries have two workgroups' worth of tiles per CU; as two rounds of workgroups each
// round paid the patch + weight prologue and the store drain (3.7 + 1.8 us of 10 on
// layer2).  Bias / scales are loaded in the prologue (one set for all tiles).
#pragma once
#include "conv_gx.h"

namespace pa {

// DBG = 4: s_memrealtime stamps into a.trace (conv.h trace_stamp: 0 start, 1 prologue landed,
// 2 K loop done, 3 epilogue stores issued, 63 stores retired; TPW > 1: 4 + j tile j + 1's
// first step)
// PART = NS > 0 (split-K for small batches, conv_splitk.hip): as conv_gx.h's PART, the
// workgroup runs input channels CIN * blockIdx.y .. of an a.Cin = NS * CIN channel conv and
// writes its f32 accumulators (conv -> a.part[split], downsample -> a.part[NS + split]),
// no epilogue
template <int TH, int TW, int BN, int WM, int WN, int CIN, int PD, int G, bool WT = true, bool X3 = false, int DBG = 0,
          int TPW = 1, int PART = 0>
__global__ __launch_bounds__(WM * WN * 64) void conv3x3s2_x(ConvS2Args a, int xg) {
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int NCB = CIN / 64;
  using VB = GxBlocks<X3, NCB>;
  constexpr int XS = X3 ? 2 : 1;
  constexpr int SPB = 10;  // 9 taps + downsample per 64-channel block
  constexpr int SPT = VB::NVB * SPB;  // steps per tile
  constexpr int NBLK = TPW * VB::NVB;  // patch blocks in the stream
  constexpr int NSTEPS = TPW * SPT;
  constexpr int PH = 2 * TH + 1;
  constexpr int PW = TW == 8 ? 20 : 2 * TW + 1;  // LDS positions per patch row
  constexpr int NP = PH * PW;
  constexpr int NPC = (NP * 8 + 63) / 64 * 64;
  constexpr int PDMA = NPC / 64 / NW + (NPC / 64 % NW ? 1 : 0);
  constexpr int PATCHB = (PDMA * NW * 64) * 16;
  constexpr int NPB = NBLK > 1 ? 2 : 1;  // patch buffers
  constexpr int WB = BN * 128;
  constexpr int WDMA = BN * 8 / NT;
  constexpr int BM = TH * TW;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  static_assert(TW == 8 || TW == 16, "tile width");
  static_assert(BN * 8 % NT == 0 && WDMA >= 1, "weight tile / threads");
  static_assert(WTM % 16 == 0 && WTN % 32 == 0, "wave tile");
  static_assert(G >= 1 && G <= 3 && PD >= G + 1 && PD <= 8, "prefetch distance / steps per barrier");
  constexpr int NSLOT = PD + G;
  static_assert(!PART || TPW == 1, "split-K partials: one tile per workgroup");
  constexpr int RL = (TPW > 1 || PART) ? 0 : 2 * XS * TN;  // epilogue loads in the stream: bias, bias2 (+ scale, scale2)
  constexpr int RSD = 4;
  constexpr int NST = TM * (TN / 2) * 2 * XS;  // output stores per tile (out, out2; hi, lo)
  constexpr GxPlan plan{NSTEPS, NBLK, PD, WDMA, PDMA, RL, NSTEPS > RSD ? NSTEPS - RSD : 0, G, SPB,
                        TPW > 1 ? SPT : 0, NST};
  static_assert(NPB * PATCHB + NSLOT * WB <= 163840, "LDS");
  __shared__ __attribute__((aligned(1024))) char smem[NPB * PATCHB + NSLOT * WB];
  char* patch = smem;
  char* wring = smem + NPB * PATCHB;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int q = lane >> 4, r16 = lane & 15;
  const int H = a.Hout, W = a.Wout, Hin = a.Hin, Win = a.Win, Cout = a.Cout;
  // PART: pixel and tap strides are the full conv's a.Cin; split blockIdx.y starts at input
  // channel CIN * blockIdx.y
  // as conv_gx.h: CF = the full conv's channels per plane, kin = pixel / tap stride,
  // gx_boff = a 64-channel block's offset in the [hi (CF) | lo (CF)] planes
  constexpr int CF = PART ? PART * CIN : CIN;
  constexpr int kin = XS * CF;
  const int kc0 = PART ? CIN * (int)blockIdx.y : 0;
  const _Float16* __restrict__ in = (const _Float16*)a.in + kc0;
  const _Float16* __restrict__ w = (const _Float16*)a.w + kc0;
  const _Float16* __restrict__ wds = (const _Float16*)a.wds + kc0;

  const int ntn = Cout / BN;
  int tn_idx, sp;  // sp: the workgroup's group of TPW consecutive spatial tiles
  if (xg == 2) {  // 2 x 4 XCD split: XCD residue x8 takes channel half x8 & 1 of image group x8 >> 1
    // (each XCD's L2 then holds half the weights and a quarter of the images: weight + input
    // fetch 10.5 + 16.8 MB at layer4 / B = 64 instead of 21 + 8.4)
    const int b = blockIdx.x, x8 = b & 7, i = b >> 3, nh = ntn >> 1;
    tn_idx = (x8 & 1) * nh + i % nh;
    sp = (i / nh) * 4 + (x8 >> 1);
  } else if (xg) {  // blocks b and b + 8 share an XCD: the N-tiles of one spatial tile there
    const int b = blockIdx.x, x8 = b & 7, i = b >> 3;
    tn_idx = i % ntn;
    sp = (i / ntn) * 8 + x8;
  } else {
    tn_idx = blockIdx.x % ntn;
    sp = blockIdx.x / ntn;
  }
  if constexpr (DBG == 4) trace_stamp(a.trace, 0);
  const int tw_n = W / TW, tpi = (H / TH) * tw_n;
  const int img = (sp * TPW) / tpi;  // one image per group (tpi % TPW == 0)
  if (img >= a.B) return;
  const int n0 = tn_idx * BN;
  auto tile_origin = [&](int j, int& th0, int& tw0) __attribute__((always_inline)) {
    const int rem = sp * TPW + j - img * tpi;
    th0 = (rem / tw_n) * TH;
    tw0 = (rem - (rem / tw_n) * tw_n) * TW;
  };

  // patch DMA: LDS slot c = (i * NW + wid) * 64 + lane holds position p = c >> 3,
  // logical chunk (c & 7) ^ swizzle(p); block blk = tile j's virtual block vb.  Through a
  // buffer resource over this image (conv_gx.h s2w_dma16): the per-lane byte offset of a tile
  // is computed once (tile_off), a block adds a constant, and halo / padding lanes carry an
  // out-of-range offset (S2W_OOB + block offset stays out of range) and read zeros.  (The
  // pointer form recomputed the tile, selected a 64-bit pointer against a zero line whose
  // address came through the GOT behind s_waitcnt lgkmcnt(0) -- draining the fragment reads --
  // at every DMA of the K loop.)
  const s2w_u4 prs = s2w_rsrc((const _Float16*)a.in + (size_t)img * Hin * Win * kin,
                              (unsigned)((size_t)Hin * Win * kin * 2));
  auto tile_off = [&](int j, unsigned (&po)[PDMA]) __attribute__((always_inline)) {
    int th0, tw0;
    tile_origin(j, th0, tw0);
#pragma unroll
    for (int i = 0; i < PDMA; ++i) {
      const int c = (i * NW + wid) * 64 + lane;
      const int p = c >> 3, pc = c & 7;
      const int lc = pc ^ ((p >> 1) & 7);
      const int pr = p / PW, pos = p - (p / PW) * PW;
      const int col = pos <= TW ? 2 * pos : 2 * (pos - TW - 1) + 1;
      const int h = 2 * th0 - 1 + pr, x = 2 * tw0 - 1 + col;
      const bool ok = p < NP && pos < 2 * TW + 1 && (unsigned)h < (unsigned)Hin && (unsigned)x < (unsigned)Win;
      po[i] = ok ? (unsigned)(((h * Win + x) * kin + kc0 + lc * 8) * 2) : S2W_OOB;
    }
  };
  unsigned poff[PDMA];
  int poff_tile = -1;
  auto dma_patch = [&](int blk, int buf) __attribute__((always_inline)) {
    const int j = blk / VB::NVB, vb = blk - (blk / VB::NVB) * VB::NVB;
    if (j != poff_tile) {  // compile-time after unrolling (blk is a step constant)
      tile_off(j, poff);
      poff_tile = j;
    }
    const unsigned bo = (unsigned)(gx_boff<NCB, CF>(VB::pblk(vb)) * 2);
#pragma unroll
    for (int i = 0; i < PDMA; ++i) s2w_dma16(prs, poff[i] + bo, patch + buf * PATCHB + (i * NW + wid) * 1024);
  };
  // weights: ring row co holds output channel n0 + xperm(co) (16-byte epilogue)
  const _Float16* wsrc[WDMA];
  const _Float16* dsrc[WDMA];
#pragma unroll
  for (int i = 0; i < WDMA; ++i) {
    const int c = (i * NW + wid) * 64 + lane;
    const int co = c >> 3, lc = (c & 7) ^ ((co >> 1) & 7);
    wsrc[i] = w + (size_t)(n0 + xperm(co)) * (9 * kin) + lc * 8;
    dsrc[i] = wds + (size_t)(n0 + xperm(co)) * kin + lc * 8;
  }
  auto dma_w = [&](int s) __attribute__((always_inline)) {
    const int vb = (s % SPT) / SPB, t = s % SPB;
    const int wb = gx_boff<NCB, CF>(VB::wblk(vb));
#pragma unroll
    for (int i = 0; i < WDMA; ++i) {
      const _Float16* src = t < 9 ? wsrc[i] + t * kin + wb : dsrc[i] + wb;
      xdma16(src, wring + (s % NSLOT) * WB + (i * NW + wid) * 1024);
    }
  };

  const int o = xfrag(r16);
  int ppix[TM];  // LDS position of tap (0, 0) for this lane's pixel of fragment tm
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int m = wm * WTM + tm * 16 + o;
    const int y = m / TW, x = m - (m / TW) * TW;
    ppix[tm] = 2 * y * PW + x;
  }
  f32x4 bias[TN], bias2[TN];
  f32x4 scl[X3 ? TN : 1], scl2[X3 ? TN : 1];
  auto load_epi = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int c = n0 + wn * WTN + (tn >> 1) * 32 + q * 8 + (tn & 1) * 4;
      bias[tn] = *reinterpret_cast<const f32x4*>(a.bias + c);
      bias2[tn] = *reinterpret_cast<const f32x4*>(a.bias2 + c);
      if constexpr (X3) {
        scl[tn] = *reinterpret_cast<const f32x4*>(a.scale + c);
        scl2[tn] = *reinterpret_cast<const f32x4*>(a.scale2 + c);
      }
    }
  };

  f32x4 acc[TM][TN], accd[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      accd[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

  dma_patch(0, 0);
#pragma unroll
  for (int t = 0; t < PD; ++t)
    if (t < NSTEPS) dma_w(t);
  if constexpr (TPW > 1) load_epi();
  xwait_vm<0>();
  __builtin_amdgcn_s_barrier();
  if constexpr (DBG == 4) trace_stamp(a.trace, 1);

  _Float16* __restrict__ out = (_Float16*)a.out;
  _Float16* __restrict__ out2 = (_Float16*)a.out2;
  auto epilogue = [&](int j) __attribute__((always_inline)) {
    int th0, tw0;
    tile_origin(j, th0, tw0);
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
      const int m = wm * WTM + tm * 16 + o;
      const int y = m / TW, x = m - (m / TW) * TW;
      const size_t pixo = (((size_t)img * H + th0 + y) * W + tw0 + x) * (XS * Cout) + n0 + wn * WTN + q * 8;
#pragma unroll
      for (int p = 0; p < TN / 2; ++p) {
        half8 h1, h2, l1, l2;
#pragma unroll
        for (int e8 = 0; e8 < 8; ++e8) {
          const int tn = 2 * p + (e8 >> 2), e = e8 & 3;
          if constexpr (X3) {
            const HiLo a1 = split_x3(fmaxf(acc[tm][tn][e] * scl[tn][e] + bias[tn][e], 0.f));
            const HiLo a2 = split_x3(accd[tm][tn][e] * scl2[tn][e] + bias2[tn][e]);
            h1[e8] = a1.hi;
            l1[e8] = a1.lo;
            h2[e8] = a2.hi;
            l2[e8] = a2.lo;
          } else {
            h1[e8] = (_Float16)fmaxf(acc[tm][tn][e] + bias[tn][e], 0.f);
            h2[e8] = (_Float16)(accd[tm][tn][e] + bias2[tn][e]);
          }
        }
        store16<WT>(out, (unsigned)((pixo + p * 32) * 2), h1);
        store16<WT>(out2, (unsigned)((pixo + p * 32) * 2), h2);
        if constexpr (X3) {
          store16<WT>(out, (unsigned)((pixo + Cout + p * 32) * 2), l1);
          store16<WT>(out2, (unsigned)((pixo + Cout + p * 32) * 2), l2);
        }
      }
    }
  };

  xu4 fa[2][TN], fb[2][TM];
  auto read_frags = [&](auto kc) __attribute__((always_inline)) {
    constexpr int K = decltype(kc)::value;
    constexpr int S = K >> 1, HG = K & 1, CB = S / SPB, T = S % SPB;
    constexpr int TT = T < 9 ? T : 4;  // the downsample reads the centre tap's pixels
    constexpr int KX = TT % 3;
    constexpr int TOFF = (TT / 3) * PW + (KX == 0 ? 0 : (KX == 1 ? TW + 1 : 1));
    const char* pb = patch + (NPB == 2 ? (CB & 1) : 0) * PATCHB;
    const char* wb = wring + (S % NSLOT) * WB;
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
      fa[HG][tn] = *reinterpret_cast<const xu4*>(wb + xswz(wn * WTN + tn * 16 + r16, HG * 4 + q));
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) fb[HG][tm] = *reinterpret_cast<const xu4*>(pb + xswz(ppix[tm] + TOFF, HG * 4 + q));
  };
  auto mfma = [&](auto hc, auto dsc) __attribute__((always_inline)) {
    constexpr int HG = decltype(hc)::value;
    constexpr bool DS = decltype(dsc)::value;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        f32x4& d = DS ? accd[tm][tn] : acc[tm][tn];
        d = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, fa[HG][tn]),
                                                   __builtin_bit_cast(half8, fb[HG][tm]), d, 0, 0, 0);
      }
  };
  read_frags(xic<0>{});
  gx_for<0, NSTEPS>([&](auto sc) __attribute__((always_inline)) {
    constexpr int S = decltype(sc)::value;
    constexpr int CB = S / SPB;
    using DS = std::integral_constant<bool, S % SPB == 9>;
    if constexpr (S > 0 && S % SPT == 0) {  // previous tile done: its stores (plan.ns), fresh accumulators
      if constexpr (DBG == 4) trace_stamp(a.trace, 3 + S / SPT);
      epilogue(S / SPT - 1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
          accd[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      __builtin_amdgcn_sched_barrier(0);
    }
    read_frags(xic<2 * S + 1>{});
    __builtin_amdgcn_s_setprio(1);
    mfma(xic<0>{}, DS{});
    __builtin_amdgcn_s_setprio(0);
    if constexpr (S + 1 < NSTEPS) read_frags(xic<2 * S + 2>{});
    // DMAs after this step's LDS reads (see xdma16); order = GxPlan's
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (S + PD < NSTEPS) dma_w(S + PD);
    if constexpr (CB + 1 < NBLK && S == plan.ps(CB + 1)) dma_patch(CB + 1, (CB + 1) & 1);
    if constexpr (TPW == 1 && S == plan.rs && !PART) {
      __builtin_amdgcn_sched_barrier(0);
      load_epi();
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    mfma(xic<1>{}, DS{});
    __builtin_amdgcn_s_setprio(0);
    if constexpr ((S + 1) % G == 0 && S + 2 < NSTEPS) {
      constexpr int V = S + G + 1 < NSTEPS ? S + G + 1 : NSTEPS - 1;
      xwait_vm<plan.vm_after(S, V)>();
      __builtin_amdgcn_s_barrier();
    }
  });
  if constexpr (DBG == 4) trace_stamp(a.trace, 2);
  xwait_vm<0>();
  if constexpr (PART > 0) {  // f32 partials of both: acc / accd[tm][tn] = 4 consecutive channels of one pixel
    const size_t plane = (size_t)a.B * H * W * Cout;
    float* __restrict__ pt = a.part + blockIdx.y * plane;
    float* __restrict__ pd = a.part + (PART + blockIdx.y) * plane;
    int th0, tw0;
    tile_origin(0, th0, tw0);
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
      const int m = wm * WTM + tm * 16 + o;
      const int y = m / TW, x = m - (m / TW) * TW;
      const size_t pixo = (((size_t)img * H + th0 + y) * W + tw0 + x) * Cout + n0 + wn * WTN + q * 8;
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const size_t e = pixo + (tn >> 1) * 32 + (tn & 1) * 4;
        *reinterpret_cast<f32x4*>(pt + e) = acc[tm][tn];
        *reinterpret_cast<f32x4*>(pd + e) = accd[tm][tn];
      }
    }
    return;
  }
  epilogue(TPW - 1);
  if constexpr (DBG == 4) {
    trace_stamp(a.trace, 3);
    __builtin_amdgcn_s_waitcnt(0);
    trace_stamp(a.trace, 63);
  }
}

template <int TH, int TW, int BN, int WM, int WN, int CIN, int PD, int G = 1, bool WT = true, bool X3 = false,
          int DBG = 0, int TPW = 1>
static int run_s2x(const ConvS2Args& a, int xg, hipStream_t s) {
  PA_CHECK(!WT || (size_t)a.B * a.Hout * a.Wout * a.Cout * 2 * (X3 ? 2 : 1) < 0x7fffffffu, "s2x conv: output over 2 GB");
  PA_CHECK(!X3 || (a.scale && a.scale2), "s2x conv (fp16x3): scales required");
  PA_CHECK(a.Cin == CIN, "s2x conv: Cin %d != %d", a.Cin, CIN);
  PA_CHECK(a.Hin == 2 * a.Hout && a.Win == 2 * a.Wout, "s2x conv: %dx%d -> %dx%d", a.Hin, a.Win, a.Hout, a.Wout);
  PA_CHECK(a.Hout % TH == 0 && a.Wout % TW == 0, "s2x conv: %dx%d not tiled by %dx%d", a.Hout, a.Wout, TH, TW);
  PA_CHECK(a.Cout % BN == 0, "s2x conv: Cout %d %% BN %d", a.Cout, BN);
  PA_CHECK((a.Hout / TH) * (a.Wout / TW) % TPW == 0, "s2x conv: %d tiles per image not grouped by %d",
           (a.Hout / TH) * (a.Wout / TW), TPW);
  const int ntn = a.Cout / BN;
  const int nsp = a.B * (a.Hout / TH) * (a.Wout / TW) / TPW;  // groups of TPW tiles
  // xg 2 (the 2 x 4 split) needs an even channel-tile count and image groups of 4; else the 1-D order
  const int x = (xg == 2 && ntn % 2 == 0 && nsp % 4 == 0) ? 2 : (xg && nsp % 8 == 0) ? 1 : 0;
  hipLaunchKernelGGL((conv3x3s2_x<TH, TW, BN, WM, WN, CIN, PD, G, WT, X3, DBG, TPW>), dim3(nsp * ntn),
                     dim3(WM * WN * 64), 0, s, a, x);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

// split-K partial launch (PART = NS): grid.y = NS splits of CIN channels, f32 partials to a.part
template <int TH, int TW, int BN, int WM, int WN, int CIN, int PD, int NS, bool X3 = false>
static int run_s2x_part(const ConvS2Args& a, hipStream_t s) {
  PA_CHECK(a.part && a.Cin == NS * CIN && a.Hin == 2 * a.Hout && a.Win == 2 * a.Wout && a.Hout % TH == 0 &&
               a.Wout % TW == 0 && a.Cout % BN == 0,
           "s2x split-K: Cin %d Cout %d %dx%d", a.Cin, a.Cout, a.Hout, a.Wout);
  const int ntn = a.Cout / BN;
  const int nsp = a.B * (a.Hout / TH) * (a.Wout / TW);
  hipLaunchKernelGGL((conv3x3s2_x<TH, TW, BN, WM, WN, CIN, PD, 1, true, X3, 0, 1, NS>), dim3(nsp * ntn, NS),
                     dim3(WM * WN * 64), 0, s, a, 0);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

}  // namespace pa
