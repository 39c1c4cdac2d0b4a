// Stride-2 BasicBlock entry (conv 3x3 s2 + bn1 + relu, and the 1x1 s2 downsample + bn, in
// one pass over the input; torchvision resnet18 layer2 / layer3 block 0 behind
// perseus/detector/models.py:20) on 8 x 16-pixel x BN-channel tiles
// with a row-split patch.
//
// Why ("stride-2 entries"): conv_s2x.h's 4 x 16 x 128 tiles stream a 16 KB
// weight tile per step for 64 output pixels, i.e. 2 / 64 bytes per MAC, and the patch of a
// stride-2 tile is ~4.6 input pixels per output pixel; per CU that is ~20 KB of LDS-DMA per
// 64 x 128 x 64-MAC step, 0.31 DMA pieces (1 KB wave-instructions) per MFMA, and the entries
// ran at 0.19-0.23 of the MFMA peak against 0.40 for the stride-1 convs (0.19 pieces per
// MFMA).  Twice the pixels per tile halves the weight bytes per MAC, but the 8 x 16 tile's
// 64-channel patch is 17 x 33 input pixels = 72 KB, and the classic double buffer (next
// block's patch in flight while this block computes) does not fit beside a weight ring.
//
// Row-split patch: output row y reads input rows 2y - 1 (tap row kh = 0), 2y (kh = 1) and
// 2y + 1 (kh = 2), so the patch splits by input-row parity into an "even" region (the 8
// rows 2y: tap row 1, and the downsample's centre pixel) and an "odd" region (the 9 rows
// 2y - 1 / 2y + 1: tap rows 0 and 2).  Each unit (one tile's 64-channel block) runs its 10
// steps in the order
//     kh = 1 (kw = 0, 1, 2), downsample, kh = 0 (kw = 0, 1, 2), kh = 2 (kw = 0, 1, 2)
// so the even region is free after step 3: the next unit's even rows are DMA'd at step 4
// (landing in steps 4-9), its odd rows at its own step 0 (needed from its step 4 on).  ONE
// 80 KB patch buffer + a 4-slot ring of 16 KB weight tiles = 144 KB of LDS.
//
// The rest is conv_s2x.h's machinery: weight tile of step s + PD DMA'd into the ring at step
// s, fragments half a step ahead, one bare s_barrier per step behind a compile-time vmcnt
// (S2wPlan below simulates the per-wave issue order: output stores of the previous tile,
// weight tile, odd rows, even rows, epilogue loads), XCD-aware block order, TPW tiles per
// workgroup as one step stream, register epilogue with write-through 16-byte stores.  The
// conv's K sum runs in the step order above (taps 3-5, 0-2, 6-8 of each block), so the
// outputs are not bit-identical to conv_s2x.h's (taps 0-8); the downsample's are.
#pragma once
#include "conv_gx.h"

namespace pa {

// issue schedule per wave (compile time): U units of 10 steps.  x3: units are fp16x3 virtual
// blocks (x_hi w_hi, x_hi w_lo, x_lo w_hi per 64 channels): the second one reads the patch
// the first one loaded, so it loads nothing (ld)
struct S2wPlan {
  int nsteps, nunits, pd, wdma, po, pe, rl, rs, ut, nstore, x3;  // ut = units per tile, rs = epilogue-load lead
  constexpr bool ld(int u) const { return !x3 || (u % ut) % 3 != 1; }  // unit u loads its own patch
  constexpr int src(int u) const { return ld(u) ? u : u - 1; }          // the unit whose patch u reads
  constexpr int ns(int t) const { return (t > 0 && t % (10 * ut) == 0) ? nstore : 0; }  // previous tile's stores
  constexpr int nw(int t) const { return t + pd < nsteps ? wdma : 0; }
  constexpr int npo(int t) const { return (t % 10 == 0 && t / 10 >= 1 && ld(t / 10)) ? po : 0; }  // odd rows, this unit
  constexpr int npe(int t) const {  // even rows, next unit
    return (t % 10 == 4 && t / 10 + 1 < nunits && ld(t / 10 + 1)) ? pe : 0;
  }
  constexpr int nr(int t) const { return (t + rs) % (10 * ut) == 0 ? rl : 0; }  // rs steps before each tile's end
  constexpr int cum(int t) const {
    int c = 0;
    for (int u = 0; u <= t; ++u) c += ns(u) + nw(u) + npo(u) + npe(u) + nr(u);
    return c;
  }
  constexpr int before(int t) const { return t > 0 ? cum(t - 1) : 0; }
  // ops issued after the newest op the fragments of step v need (its weight tile, and the
  // region of its unit its taps read), counted at the end of step s
  // The prologue issues unit 0's even rows, W(0 .. pd - 1), then unit 0's odd rows (po ops) and
  // waits for all but those: the odd rows land during steps 0-3, which read only the even rows.
  // Positions of prologue ops are <= 0: the even rows and prologue weights -po, the odd rows 0.
  constexpr int vm_after(int s, int v) const {
    int need = -po;  // prologue weights / even rows: the odd rows' po DMAs were issued after them
    if (v >= pd) {
      const int t = v - pd;
      need = before(t) + ns(t) + nw(t);
    }
    const int u = src(v / 10), tv = v % 10;
    if (tv < 4 && u >= 1) {  // even rows of unit u, DMA'd at unit u - 1's step 4
      const int t = (u - 1) * 10 + 4;
      const int e = before(t) + ns(t) + nw(t) + npo(t) + npe(t);
      need = e > need ? e : need;
    } else if (tv >= 4 && u >= 1) {  // odd rows of unit u, DMA'd at its step 0
      const int t = u * 10;
      const int e = before(t) + ns(t) + nw(t) + npo(t);
      need = e > need ? e : need;
    } else if (tv >= 4) {  // unit 0's odd rows: the newest prologue ops
      need = 0 > need ? 0 : need;
    }
    const int n = cum(s) - need;
    return n < 0 ? 0 : (n > 63 ? 63 : n);
  }
};

// step t of a unit: patch region / row offset (in LDS positions) and tap
//   t 0-2: kh = 1, kw = t (even rows);  t 3: downsample (even rows, centre column);
//   t 4-6: kh = 0, kw = t - 4 (odd rows, row y);  t 7-9: kh = 2, kw = t - 7 (odd rows, row y + 1)
__host__ __device__ constexpr int s2w_tap(int t) { return t < 3 ? 3 + t : (t == 3 ? -1 : (t < 7 ? t - 4 : t - 1)); }
__host__ __device__ constexpr int s2w_kw(int t) { return t < 3 ? t : (t == 3 ? 1 : (t < 7 ? t - 4 : t - 7)); }

// X3 (fp16x3 parity mode, conv_gx.h X3): activation planes [hi (CIN) | lo (CIN)] per pixel,
// weights hi / lo planes of w * 2^e; a unit is one of the 3 virtual blocks per 64 channels
// (GxBlocks), the epilogue unscales exactly and writes (hi, lo) plane pairs.
template <int BN, int WM, int WN, int CIN, int PD, int TPW, bool WT = true, bool X3 = false>
__global__ __launch_bounds__(WM * WN * 64) void conv3x3s2_w(ConvS2Args a, int xg) {
  constexpr int TH = 8, TW = 16;
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int NCB = CIN / 64;
  using VB = GxBlocks<X3, NCB>;
  constexpr int XS = X3 ? 2 : 1;     // fp16 planes per element
  constexpr int NVB = VB::NVB;       // units per tile
  constexpr int NU = TPW * NVB;      // units (tile, virtual 64-channel block) in the stream
  constexpr int NSTEPS = NU * 10;
  constexpr int PW = 2 * TW + 1;     // LDS positions per patch row: 17 even-local + 16 odd-local columns
  constexpr int RO = TH + 1, RE = TH;  // odd / even region rows
  constexpr int PO = (RO * PW * 8 + NT - 1) / NT;  // DMA pieces per wave: odd region
  constexpr int PE = (RE * PW * 8 + NT - 1) / NT;  // even region
  constexpr int POS_E = PO * NT / 8;  // first LDS position (128-byte row) of the even region
  constexpr int PATCHB = (PO + PE) * NT * 16;
  constexpr int WB = BN * 128;
  constexpr int WDMA = BN * 8 / NT;
  constexpr int BM = TH * TW;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  static_assert(BN * 8 % NT == 0 && WDMA >= 1, "weight tile / threads");
  static_assert(WTM % 16 == 0 && WTN % 32 == 0, "wave tile");
  static_assert(PD >= 2 && PD <= 6, "prefetch distance");
  constexpr int NSLOT = PD + 1;  // one barrier per step
  constexpr int RL = 0;  // bias / bias2 are staged in LDS by the prologue (32 VGPRs not held across the stream)
  constexpr int RSD = 4;
  constexpr int NST = TM * (TN / 2) * 2 * XS;  // output stores per tile (out, out2; hi, lo)
  constexpr S2wPlan plan{NSTEPS, NU, PD, WDMA, PO, PE, RL, RSD, NVB, NST, X3 ? 1 : 0};
  constexpr int EB = 2 * XS * BN * 4;  // epilogue constants: bias, bias2 (X3: scale, scale2)
  static_assert(PATCHB + NSLOT * WB + EB <= 163840, "LDS");
  __shared__ __attribute__((aligned(1024))) char smem[PATCHB + NSLOT * WB + EB];
  char* patch = smem;
  char* wring = smem + PATCHB;
  float* bl = reinterpret_cast<float*>(smem + PATCHB + NSLOT * WB);  // [bias | bias2 | scale | scale2] (BN each)

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int q = lane >> 4, r16 = lane & 15;
  const int H = a.Hout, W = a.Wout, Hin = a.Hin, Win = a.Win, Cout = a.Cout;
  const _Float16* __restrict__ in = (const _Float16*)a.in;
  const _Float16* __restrict__ w = (const _Float16*)a.w;
  const _Float16* __restrict__ wds = (const _Float16*)a.wds;

  const int ntn = Cout / BN;
  int tn_idx, sp;  // sp: the workgroup's group of TPW consecutive spatial tiles
  if (xg) {  // blocks b and b + 8 share an XCD: the N-tiles of one spatial tile there
    const int b = blockIdx.x, x8 = b & 7, i = b >> 3;
    tn_idx = i % ntn;
    sp = (i / ntn) * 8 + x8;
  } else {
    tn_idx = blockIdx.x % ntn;
    sp = blockIdx.x / ntn;
  }
  const int tw_n = W / TW, tpi = (H / TH) * tw_n;
  const int img = (sp * TPW) / tpi;  // one image per group (tpi % TPW == 0)
  if (img >= a.B) return;
  const int n0 = tn_idx * BN;
  auto tile_origin = [&](int j, int& th0, int& tw0) __attribute__((always_inline)) {
    const int rem = sp * TPW + j - img * tpi;
    th0 = (rem / tw_n) * TH;
    tw0 = (rem - (rem / tw_n) * tw_n) * TW;
  };

  // patch DMA of one region of unit u (tile u / NCB, block u % NCB): LDS chunk slot
  // c = (i * NW + wid) * 64 + lane of the region holds region position p = c >> 3 (global
  // LDS row base + p), logical chunk (c & 7) ^ swizzle(row); odd region row r -> input row
  // 2 th0 - 1 + 2 r, even region row r -> 2 th0 + 2 r; position -> column as conv_s2x.h
  auto dma_region = [&](int u, auto ev) __attribute__((always_inline)) {
    constexpr bool even = decltype(ev)::value;
    constexpr int rows = even ? RE : RO, base = even ? POS_E : 0, npc = even ? PE : PO;
    const int j = u / NVB, vb = u - (u / NVB) * NVB;
    const int boff = gx_boff<NCB, CIN>(VB::pblk(vb));  // element offset of the unit's plane block
    int th0, tw0;
    tile_origin(j, th0, tw0);
    // the per-lane index made opaque per call: the address arithmetic is redone at every
    // region DMA instead of being shared across all units' DMAs and held live through the
    // K loop
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const s2w_u4 rs = s2w_rsrc(in + (size_t)img * Hin * Win * XS * CIN, (unsigned)(Hin * Win * XS * CIN * 2));
#pragma unroll
    for (int i = 0; i < npc; ++i) {
      const int c = (i * NW + wid) * 64 + ln;
      const int p = c >> 3, pc = c & 7;
      const int row = base + p;
      const int lc = pc ^ ((row >> 1) & 7);
      const int pr = p / PW, pos = p - (p / PW) * PW;
      const int col = pos <= TW ? 2 * pos : 2 * (pos - TW - 1) + 1;
      const int h = 2 * th0 + (even ? 2 * pr : 2 * pr - 1), x = 2 * tw0 - 1 + col;
      const bool ok = pr < rows && (unsigned)h < (unsigned)Hin && (unsigned)x < (unsigned)Win;
      const unsigned vo = ok ? (unsigned)(((h * Win + x) * XS * CIN + boff + lc * 8) * 2) : S2W_OOB;
      s2w_dma16(rs, vo, patch + base * 128 + (i * NW + wid) * 1024);
    }
  };
  // weights: ring row co holds output channel n0 + xperm(co) (16-byte epilogue)
  const _Float16* wsrc[WDMA];
  const _Float16* dsrc[WDMA];
#pragma unroll
  for (int i = 0; i < WDMA; ++i) {
    const int c = (i * NW + wid) * 64 + lane;
    const int co = c >> 3, lc = (c & 7) ^ ((co >> 1) & 7);
    wsrc[i] = w + (size_t)(n0 + xperm(co)) * (9 * XS * CIN) + lc * 8;
    dsrc[i] = wds + (size_t)(n0 + xperm(co)) * XS * CIN + lc * 8;
  }
  auto dma_w = [&](int s) __attribute__((always_inline)) {
    const int t = s % 10, vb = (s / 10) % NVB, tap = s2w_tap(t);
    const int wo = gx_boff<NCB, CIN>(VB::wblk(vb));
#pragma unroll
    for (int i = 0; i < WDMA; ++i) {
      const _Float16* src = tap >= 0 ? wsrc[i] + tap * XS * CIN + wo : dsrc[i] + wo;
      xdma16(src, wring + (s % NSLOT) * WB + (i * NW + wid) * 1024);
    }
  };

  const int o = xfrag(r16);
  int ppix[TM];  // LDS position of (row y of its region, column position of kw = 0) for this lane's pixel
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int m = wm * WTM + tm * 16 + o;
    const int y = m / TW, x = m - (m / TW) * TW;
    ppix[tm] = y * PW + x;
  }

  f32x4 acc[TM][TN], accd[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      accd[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

  // prologue: bias / bias2 of this workgroup's channels to LDS, unit 0's even rows, W(0 .. PD-1), unit 0's
  // odd rows; everything but the odd rows waited for
  if (tid < BN) {
    bl[tid] = a.bias[n0 + tid];
    bl[BN + tid] = a.bias2[n0 + tid];
    if constexpr (X3) {
      bl[2 * BN + tid] = a.scale[n0 + tid];
      bl[3 * BN + tid] = a.scale2[n0 + tid];
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  dma_region(0, std::true_type{});
#pragma unroll
  for (int t = 0; t < PD; ++t)
    if (t < NSTEPS) dma_w(t);
  dma_region(0, std::false_type{});  // odd rows last: needed from step 4 on (S2wPlan::vm_after)
  xwait_vm<PO>();
  __builtin_amdgcn_s_barrier();

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
        // this lane's 8 channels wn * WTN + p * 32 + q * 8 .. + 7 (tiles 2p, 2p + 1)
        const f32x4* b4 = reinterpret_cast<const f32x4*>(bl + wn * WTN + p * 32 + q * 8);
        const f32x4 b0 = b4[0], b1 = b4[1], d0 = b4[BN / 4], d1 = b4[BN / 4 + 1];
        half8 h1, h2, l1, l2;
        if constexpr (X3) {
          const f32x4 s0 = b4[BN / 2], s1 = b4[BN / 2 + 1], t0 = b4[3 * BN / 4], t1 = b4[3 * BN / 4 + 1];
#pragma unroll
          for (int e8 = 0; e8 < 8; ++e8) {
            const int tn = 2 * p + (e8 >> 2), e = e8 & 3;
            const HiLo a1 = split_x3(fmaxf(acc[tm][tn][e] * (e8 < 4 ? s0 : s1)[e] + (e8 < 4 ? b0 : b1)[e], 0.f));
            const HiLo a2 = split_x3(accd[tm][tn][e] * (e8 < 4 ? t0 : t1)[e] + (e8 < 4 ? d0 : d1)[e]);
            h1[e8] = a1.hi;
            l1[e8] = a1.lo;
            h2[e8] = a2.hi;
            l2[e8] = a2.lo;
          }
        } else {
#pragma unroll
          for (int e8 = 0; e8 < 8; ++e8) {
            const int tn = 2 * p + (e8 >> 2), e = e8 & 3;
            h1[e8] = (_Float16)fmaxf(acc[tm][tn][e] + (e8 < 4 ? b0 : b1)[e], 0.f);
            h2[e8] = (_Float16)(accd[tm][tn][e] + (e8 < 4 ? d0 : d1)[e]);
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

  const int abase[2] = {xswz(r16, q), xswz(r16, 4 + q)};
  xu4 fa[2][TN], fb[2][TM];
  auto read_frags = [&](auto kc) __attribute__((always_inline)) {
    constexpr int K = decltype(kc)::value;
    constexpr int S = K >> 1, HG = K & 1, T = S % 10;
    constexpr int KW = s2w_kw(T);
    constexpr int ROFF = T < 4 ? POS_E : (T < 7 ? 0 : PW);
    constexpr int TOFF = ROFF + (KW == 0 ? 0 : (KW == 1 ? TW + 1 : 1));
    // weight rows wn * WTN + tn * 16 + r16: the swizzle (row >> 1) & 7 is (r16 >> 1) & 7 for every
    // tn / wn (multiples of 16 rows), so every read is one per-lane base + an immediate offset
    const char* wb = wring + (S % NSLOT) * WB + wn * WTN * 128 + abase[HG];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) fa[HG][tn] = *reinterpret_cast<const xu4*>(wb + tn * 16 * 128);
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) fb[HG][tm] = *reinterpret_cast<const xu4*>(patch + xswz(ppix[tm] + TOFF, HG * 4 + q));
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
    constexpr int U = S / 10, T = S % 10;
    using DS = std::integral_constant<bool, T == 3>;
    if constexpr (S > 0 && S % (10 * NVB) == 0) {  // previous tile done: its stores (plan.ns), fresh accumulators
      __builtin_amdgcn_sched_barrier(0);
      epilogue(S / (10 * NVB) - 1);
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
    // DMAs after this step's LDS reads (see xdma16); order = S2wPlan's
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (S + PD < NSTEPS) dma_w(S + PD);
    if constexpr (T == 0 && U >= 1 && plan.ld(U)) dma_region(U, std::false_type{});  // this unit's odd rows (read from its step 4)
    if constexpr (T == 4 && U + 1 < NU && plan.ld(U + 1))
      dma_region(U + 1, std::true_type{});  // the next unit's even rows (this unit's are done)
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    mfma(xic<1>{}, DS{});
    __builtin_amdgcn_s_setprio(0);
    if constexpr (S + 2 < NSTEPS) {
      // the next step reads the fragments of step S + 2's first half at its end
      xwait_vm<plan.vm_after(S, S + 2)>();
      __builtin_amdgcn_s_barrier();
    }
  });
  xwait_vm<0>();
  epilogue(TPW - 1);
}

template <int BN, int WM, int WN, int CIN, int PD, int TPW, bool WT = true, bool X3 = false>
static int run_s2w(const ConvS2Args& a, bool xg, hipStream_t s) {
  PA_CHECK(!WT || (size_t)a.B * a.Hout * a.Wout * a.Cout * 2 * (X3 ? 2 : 1) < 0x7fffffffu, "s2w conv: output over 2 GB");
  PA_CHECK(!X3 || (a.scale && a.scale2), "s2w conv (fp16x3): scales required");
  PA_CHECK(a.Cin == CIN, "s2w conv: Cin %d != %d", a.Cin, CIN);
  PA_CHECK(a.Hin == 2 * a.Hout && a.Win == 2 * a.Wout, "s2w conv: %dx%d -> %dx%d", a.Hin, a.Win, a.Hout, a.Wout);
  PA_CHECK(a.Hout % 8 == 0 && a.Wout % 16 == 0, "s2w conv: %dx%d not tiled by 8x16", a.Hout, a.Wout);
  PA_CHECK(a.Cout % BN == 0, "s2w conv: Cout %d %% BN %d", a.Cout, BN);
  PA_CHECK((a.Hout / 8) * (a.Wout / 16) % TPW == 0, "s2w conv: %d tiles per image not grouped by %d",
           (a.Hout / 8) * (a.Wout / 16), TPW);
  const int ntn = a.Cout / BN;
  const int nsp = a.B * (a.Hout / 8) * (a.Wout / 16) / TPW;
  const int x = xg && nsp % 8 == 0;
  hipLaunchKernelGGL((conv3x3s2_w<BN, WM, WN, CIN, PD, TPW, WT, X3>), dim3(nsp * ntn), dim3(WM * WN * 64), 0, s, a, x);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

}  // namespace pa
