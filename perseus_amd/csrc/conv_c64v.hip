// Layer1 3x3 stride-1 conv (Cin = Cout = 64), fp16, with the weights resident in VGPRs.
//
// conv_c64d.hip keeps the 72 KB of folded weights in LDS and reads both MFMA operands from it:
// per (tap, 32-channel) group a wave of 32 pixels x 64 channels reads 2 pixel and 4 weight
// fragments for 8 MFMAs (0.75 ds_read_b128 per 16-cycle MFMA), and its K loop runs at the
// LDS-fed rate of that shape.  Here each wave owns 64 pixels x 32 output channels and holds
// its 32 channels' weights for all 576 K (18 groups x 2 fragments x 16 B per lane = 144 VGPRs)
// for the whole launch: the K loop reads only the 4 pixel fragments of a group for its 8 MFMAs
// (0.5 reads per MFMA, nothing for the weights).  tools/ubench/mfma_shapes.hip, 8 waves,
// 16x16x32 (profiles/r05o_mfma_shapes_regs.txt): 0.60 of 2.5 PF against 0.49 for c64d's shape;
// in the kernel a tile's K loop takes 2.3-2.5 us against c64d's 3.1 (r05r trace).
//
// Two workgroup shapes (TH = tile rows, 16 columns):
//  * TH = 16: 8 waves, one workgroup per CU (conv_c64d's tile).  The trace shows where the K-loop
//    gain goes: the younger wave of each SIMD loses arbitration to its partner, finishes the
//    tile ~1.1 us later and runs alone meanwhile, and the hand-over barrier holds the older one
//    (4.1 us per tile against 2.4 us of MFMA work per SIMD).
//  * TH = 8: 4 waves (one per SIMD), TWO workgroups per CU.  A SIMD's two waves now belong to
//    different workgroups with their own barriers and patch buffers, so neither waits for the
//    other at a tile boundary and one's epilogue overlaps the other's MFMAs.  Costs: a 10 x 18
//    patch per 128 pixels (1.41x halo reads against 1.27x), and the weights staged in two halves
//    (each workgroup has ~68 KB of LDS).
//
// Patch layout: 144 bytes per pixel (8 data chunks of 16 B + 1 pad chunk), the chunk holding
// input channels 32 h + 8 q .. + 7 at position 2 q + h.  A lane's fragment address is then
// (its pixel) * 144 + 32 q + a compile-time offset for (row, tap, half): one VGPR addresses every
// patch read of the K loop (ds_read_b128 immediates).  The XOR swizzle of conv_c64d's 128-byte
// rows needs a VGPR per (row, tap, half) address -- 72 here, which with the weights does not fit
// in 256.  Conflict-free for ds_read_b128's lane groups (MI355X_MICROARCH.md LDS table): with
// the xfrag pixel order, a group's q = 0 lanes hit 16-byte bank quads 9 P mod 16 = the even (odd)
// quads and its q = 1 lanes 9 P + 2 mod 16 = the odd (even) ones.  The LDS-DMA writes 64 x 16 B
// contiguous per wave-instruction, so the pad chunks are DMA'd too (out-of-range offset: zeros).
//
// Double-buffered patch (next tile's in the first third of the K loop), the residual tile by
// LDS-DMA (not 16 VGPRs through the K loop), XCD-grouped tile order, lane -> pixel map and
// channel permutation as conv_c64d.hip; each accumulator sums its MFMAs in the same order (tap
// 0..8, 32-channel halves) and the epilogue is the same (bias, residual, ReLU in f32), so the
// output is bit-identical to conv_c64d's.
#include "conv_gx.h"

namespace pa {

template <int TH>
struct C64v {
  static constexpr int TW = 16, PH = TH + 2, PW = TW + 2, NP = PH * PW;
  static constexpr int NWAVE = TH / 2;                   // wave = 4 pixel rows x one channel half
  static constexpr int PXB = 144;                        // bytes per patch pixel (8 chunks + 1 pad)
  static constexpr int PJ = (NP * 9 + 63) / 64;          // patch wave-DMAs (46 / 26)
  static constexpr int PATCHB = PJ * 1024;
  static constexpr int PDW = (PJ + NWAVE - 1) / NWAVE;   // per wave (6 / 7), the last round partial
  static constexpr int RESB = TH * TW * 128;             // residual tile
  static constexpr int RDW = RESB / 1024 / NWAVE;        // residual DMAs per wave (4)
  static constexpr int WROUND = TH == 16 ? 9 : 5;        // weight taps staged per round
  // RP (one workgroup per CU only: LDS): the residual tile double-buffered and DMA'd one tile
  // ahead with the patch, so the epilogue needs no barrier of its own.  LDS = [patch 0 | res 0 |
  // patch 1 | res 1] (RP) or [patch 0 | patch 1 | res]; the weights are staged in the second half
  static constexpr bool RP = TH == 16;
  static constexpr int BSTR = RP ? PATCHB + RESB : PATCHB;  // buffer stride
  static constexpr int SMEM = 2 * PATCHB + (RP ? 2 : 1) * RESB;
  static_assert(RESB / 1024 % NWAVE == 0, "residual DMA split");
  static_assert(SMEM - BSTR >= WROUND * 64 * 128, "weight staging in patch buffer 1 + residual tile(s)");
  static_assert((SMEM + 256) * (TH == 16 ? 1 : 2) <= 160 * 1024, "LDS per CU");
};

// DBG = 4 (timing only): s_memrealtime stamps into a.trace (0 start, 1 prologue landed; tile t:
// 2 + 4 t start, 3 + 4 t K loop done and DMAs landed, 4 + 4 t stores issued, 5 + 4 t hand-over
// barrier passed; 20 + 8 t + wave: that wave's K loop done, t < 5)
// DYN: tiles after the first are taken from a per-XCD counter (a.cnt[x], x = blockIdx.x % 8;
// a.cnt[8] counts finished workgroups, and the last one zeroes all nine, so the counters are zero
// between launches and across graph replays).  With two workgroups per CU the one that wins
// arbitration on every SIMD runs ~30 % faster than its partner; with a static 4 tiles each the
// launch ended ~3 us after the median workgroup (r05u trace), with stolen tiles it takes more.
// The next tile's index is fetched one tile ahead (its patch is DMA'd during the current one).
// Measured and not shipped: bit-identical but ~13 us slower per launch (2,048 device-scope
// atomics on eight counters serialise, profiles/r05_c64v/r05ze_dyn_ab.log).
// DS (deferred stores, conv_s2v.hip's): a tile's outputs go out during the next tile's K loop, one
// 16-byte store per group after its DMAs, instead of at the tile's end, where every CU issues its
// stores at about the same moment and they queue behind the whole chip's (0.84 us per tile from K
// loop done to stores issued on the 16-row form, profiles/r06e trace).  Plain convs (RP): the
// outputs are staged in the idle residual buffer of the tile (the residual tile's layout: 4 VGPRs
// per store, read back just before it); residual convs: held in 16 VGPRs (pend).
// ND (VGPR form): only the tile's last ND of its TM rows are deferred, the others stored at the tile end
template <int EPI, int TH, int DBG = 0, bool DYN = false, bool DS = false, int ND = 4>
__global__ __launch_bounds__(TH * 32, 2) void conv3x3_c64v(ConvArgs a, int ntiles) {
  using G = C64v<TH>;
  constexpr int TW = G::TW, PW = G::PW, NP = G::NP, NWAVE = G::NWAVE, PXB = G::PXB, PJ = G::PJ;
  constexpr int PATCHB = G::PATCHB, PDW = G::PDW, RDW = G::RDW, BSTR = G::BSTR;
  constexpr bool RP = G::RP;
  constexpr int TM = 4, TN = 2;  // wave tile: 64 pixels (4 rows of 16) x 32 channels
  // LDS layout: C64v::RP (the weights pass through the second half in the prologue, before it is
  // first written)
  __shared__ __attribute__((aligned(1024))) char smem[G::SMEM];
  char* patch = smem;
  auto resb = [&](int b) __attribute__((always_inline)) { return RP ? smem + b * BSTR + PATCHB : smem + 2 * PATCHB; };
  char* wst = smem + BSTR;
  __shared__ __attribute__((aligned(16))) float bias_l[64];

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, r16 = lane & 15;
  const int wn = wid & 1, wm = wid >> 1;  // channel half, pixel rows 4 wm .. 4 wm + 3
  if constexpr (DBG == 4) trace_stamp(a.trace, 0);
  const int H = a.Hout, W = a.Wout;
  const _Float16* __restrict__ in = (const _Float16*)a.in;
  const _Float16* __restrict__ w = (const _Float16*)a.w;
  const int tw_n = W / TW, tpi = (H / TH) * tw_n;
  // XCD-grouped tile order (conv_c64d.hip XM)
  const bool xm = ntiles % (8 * tpi) == 0;
  auto tmap = [&](int j) __attribute__((always_inline)) {
    if (!xm) return j;
    const int c = j / (8 * tpi), r = j - c * 8 * tpi;
    return c * 8 * tpi + (r & 7) * tpi + (r >> 3);
  };

  const unsigned abytes = (unsigned)((size_t)a.B * H * W * 128 < 0x7fffffffu ? (size_t)a.B * H * W * 128 : 0x7fffffffu);
  const s2w_u4 rsrc = s2w_rsrc(in, abytes);
  struct Org {
    int img, h0, x0;
    bool on;
  };
  auto origin = [&](int t, bool on) __attribute__((always_inline)) {
    const int img = t / tpi, rem = t - img * tpi;
    return Org{img, (rem / tw_n) * TH - 1, (rem - (rem / tw_n) * tw_n) * TW - 1, on};
  };
  // patch DMA i of this wave: LDS slot c = (i * NWAVE + wid) * 64 + lane (16-byte units) holds
  // pixel p = c / 9 (row pr, column pc of the patch), position c % 9 (8: pad), i.e. input
  // channels 8 ((pos & 1) * 4 + (pos >> 1)) .. + 7.  Per lane and DMA one packed word, computed
  // once: bits 0-17 the byte offset from the patch origin, 18-22 pr, 23-27 pc, 28 pad / past the
  // patch; a DMA is then two bit-field extracts, the halo test and one add on a wave-uniform
  // tile base.  (Decoding c at every DMA cost ~25 VALU each, six per tile in the K loop: the
  // timing-only variant without that arithmetic ran 3-4 us faster per launch, r05v.)
  // (DYN, short of VGPRs for the tile fetch: two DMAs per word, 16 bits each = pr | pc << 5 |
  // pos << 10 | pad << 14, the offset recomputed at the DMA)
  constexpr int NPK = DYN ? (PDW + 1) / 2 : PDW;
  unsigned pk[NPK];
#pragma unroll
  for (int i = 0; i < NPK; ++i) pk[i] = 0;
#pragma unroll
  for (int i = 0; i < PDW; ++i) {
    const int c = (i * NWAVE + wid) * 64 + lane;
    const int p = c / 9, pos = c - p * 9;
    const int pr = p < NP ? p / PW : 0, pc = p < NP ? p - (p / PW) * PW : 0;
    const unsigned bad = (pos >= 8 || p >= NP) ? 1u : 0u;
    if constexpr (DYN) {
      pk[i >> 1] |= ((unsigned)pr | ((unsigned)pc << 5) | ((unsigned)(pos & 15) << 10) | (bad << 14)) << (16 * (i & 1));
    } else {
      const unsigned rel = (unsigned)(((pr * W + pc) * 64 + ((pos & 1) * 4 + (pos >> 1)) * 8) * 2);
      pk[i] = (rel & 0x3ffffu) | ((unsigned)pr << 18) | ((unsigned)pc << 23) | (bad << 28);
    }
  }
  auto dma_patch = [&](int i, const Org& o, int buf) __attribute__((always_inline)) {
    if constexpr (DBG == 7) {  // timing only: no offset arithmetic (wrong data)
      s2w_dma16(rsrc, (unsigned)(lane * 16 + i * 1024), patch + buf * BSTR + (i * NWAVE + wid) * 1024);
      return;
    }
    if constexpr (DYN) {
      const unsigned f = (pk[i >> 1] >> (16 * (i & 1))) & 0xffffu;
      const int pr = (int)(f & 31u), pc = (int)((f >> 5) & 31u), pos = (int)((f >> 10) & 15u);
      const unsigned tb = (unsigned)(((o.img * H + o.h0) * W + o.x0) * 128);
      const unsigned rel = (unsigned)(((pr * W + pc) * 64 + ((pos & 1) * 4 + (pos >> 1)) * 8) * 2);
      const bool ok = o.on && !(f >> 14) && (unsigned)(o.h0 + pr) < (unsigned)H && (unsigned)(o.x0 + pc) < (unsigned)W;
      s2w_dma16(rsrc, ok ? tb + rel : S2W_OOB, patch + buf * BSTR + (i * NWAVE + wid) * 1024);
      return;
    }
    const unsigned v = pk[i];
    const int pr = (int)((v >> 18) & 31u), pc = (int)((v >> 23) & 31u);
    if constexpr (DBG == 8) {  // timing only: the real arithmetic on every tile's origin = tile 1's (L2-hot data)
      const Org o1{0, -1, 15, true};
      const unsigned tb = (unsigned)(((o1.img * H + o1.h0) * W + o1.x0) * 128) + (unsigned)(o.img & 0);
      const bool ok = o1.on && !(v >> 28) && (unsigned)(o1.h0 + pr) < (unsigned)H && (unsigned)(o1.x0 + pc) < (unsigned)W;
      s2w_dma16(rsrc, ok ? tb + (v & 0x3ffffu) : S2W_OOB, patch + buf * BSTR + (i * NWAVE + wid) * 1024);
      return;
    }
    const unsigned tb = (unsigned)(((o.img * H + o.h0) * W + o.x0) * 128);  // wave-uniform (may wrap)
    const bool ok = o.on && !(v >> 28) && (unsigned)(o.h0 + pr) < (unsigned)H && (unsigned)(o.x0 + pc) < (unsigned)W;
    s2w_dma16(rsrc, ok ? tb + (v & 0x3ffffu) : S2W_OOB, patch + buf * BSTR + (i * NWAVE + wid) * 1024);
  };
  auto dma_one = [&](int i, const Org& o, int buf) __attribute__((always_inline)) {
    if (i < PDW - 1 || wid < PJ - (PDW - 1) * NWAVE) dma_patch(i, o, buf);  // wave-uniform
  };
  // residual tile (EPI_RES) by DMA i of each wave: slot c -> tile pixel c >> 3 = i * 8 NWAVE + m
  // (m = 8 wid + lane / 8), slot chunk c & 7 = logical chunk (c & 7) ^ (pixel & 7) (the epilogue's
  // reads are then conflict-free); DMA i adds i * NWAVE / 2 rows to DMA 0's per-lane offset
  const s2w_u4 rres = s2w_rsrc(a.res ? a.res : a.in, abytes);
  const int mres = 8 * wid + (lane >> 3);
  const unsigned rrel = (unsigned)((((mres >> 4) * W + (mres & 15)) * 64 + (((lane & 7) ^ (mres & 7)) * 8)) * 2);
  auto dma_res = [&](int i, int img, int th0, int tw0, int rb) __attribute__((always_inline)) {
    if constexpr (DBG == 7) {
      s2w_dma16(rres, (unsigned)(lane * 16 + i * 1024), resb(rb) + (i * NWAVE + wid) * 1024);
      return;
    }
    const unsigned tb = (unsigned)((((img * H + th0 + i * (NWAVE / 2)) * W + tw0) * 128));
    s2w_dma16(rres, tb + rrel, resb(rb) + (i * NWAVE + wid) * 1024);
  };

  const int o = xfrag(r16);
  // this lane's patch-read base: pixel (row 4 wm, column o), chunk position 2 q
  const unsigned rbase = (unsigned)(size_t)(__attribute__((address_space(3))) char*)patch + (unsigned)((wm * 4 * PW + o) * PXB + q * 32);
  if (tid < 64) bias_l[tid] = a.bias[tid];  // read back in the epilogue (8 VGPRs not held through the K loop)
  __builtin_amdgcn_sched_barrier(0);

  // prologue: the first tile's patch; the weights by LDS-DMA (conv_c64d.hip's layout: row
  // tap * 64 + rho holds channel xperm(rho), 16-byte chunks XOR-swizzled), once per workgroup, in
  // rounds of WROUND taps; every wave reads its 36 fragments: (K, tn) = channel
  // xperm(32 wn + 16 tn + r16), tap K / 2, input channels 32 (K & 1) + 8 q .. + 7.  (Loading them
  // straight into VGPRs had the waves of a channel half fetch the same bytes from L2: 295 KB per
  // workgroup, a 10 us prologue, r05q trace.)
  int j = blockIdx.x;
  // double-buffered by tile parity: tid 0 writes slot (t + 1) & 1 during tile t + 1 while a slow
  // wave may still read slot t & 1 after tile t's hand-over barrier
  __shared__ int jnext_l[2];
  const int x8 = blockIdx.x & 7;
  auto jof = [&](unsigned k) __attribute__((always_inline)) { return (int)gridDim.x + 8 * (int)k + x8; };
  if constexpr (DYN) {
    if (tid == 0) jnext_l[1] = jof(atomicAdd(a.cnt + x8, 1u));  // read after the prologue's barriers
  }
  {
    const Org o0 = origin(tmap(j), true);
#pragma unroll
    for (int i = 0; i < PDW; ++i) dma_one(i, o0, 0);
    if constexpr (RP && (EPI & EPI_RES)) {
#pragma unroll
      for (int i = 0; i < RDW; ++i) dma_res(i, o0.img, o0.h0 + 1, o0.x0 + 1, 0);
    }
  }
  xu4 wr[18][TN];
  {
    constexpr int DPT = 8 / NWAVE;  // DMAs (8 rows of 128 B each) per wave per tap
    static_assert(DPT * NWAVE * 1024 == 64 * 128, "weight DMA split");
    auto stage = [&](auto t0c, auto t1c) __attribute__((always_inline)) {
      constexpr int T0 = decltype(t0c)::value, T1 = decltype(t1c)::value;
#pragma unroll
      for (int tap = T0; tap < T1; ++tap)
#pragma unroll
        for (int d = 0; d < DPT; ++d) {
          const int row0 = (d * NWAVE + wid) * 8 + (lane >> 3);  // row within the tap
          const int lc = (lane & 7) ^ ((row0 >> 1) & 7);
          xdma16(w + (size_t)xperm(row0) * 576 + tap * 64 + lc * 8, wst + ((tap - T0) * 8 + d * NWAVE + wid) * 1024);
        }
      xwait_vm<0>();
      lds_barrier();
#pragma unroll
      for (int k = 2 * T0; k < 2 * T1; ++k)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          wr[k][tn] = *reinterpret_cast<const xu4*>(wst + xswz(((k >> 1) - T0) * 64 + wn * 32 + tn * 16 + r16, (k & 1) * 4 + q));
      lds_barrier();  // reads retired before the staging area is rewritten
    };
    if constexpr (G::WROUND >= 9) {
      stage(xic<0>{}, xic<9>{});
    } else {
      stage(xic<0>{}, xic<G::WROUND>{});
      stage(xic<G::WROUND>{}, xic<9>{});
    }
  }
  if constexpr (DBG == 4) trace_stamp(a.trace, 1);

  int jn = DYN ? 0 : j + (int)gridDim.x;
  if constexpr (DYN) jn = __builtin_amdgcn_readfirstlane(jnext_l[1]);
  unsigned kdyn = 0;
  static_assert(!(DS && DYN), "deferred stores with static tiles");
  _Float16* __restrict__ out = (_Float16*)a.out;
  constexpr bool DSL = DS && RP && !(EPI & EPI_RES) && ND >= TM;  // DS through LDS (the residual buffers are idle)
  constexpr int NDR = DSL ? TM : (ND < TM ? ND : TM);  // rows deferred: TM - NDR .. TM - 1
  half8 pend[DSL ? 1 : NDR];  // DS in VGPRs: the previous tile's outputs, rows 4 wm + TM - NDR + i
  unsigned pend_base = 0;  // DS: their tile's byte offset (wave-uniform)
  // this lane's byte offset in a tile: row 4 wm (+ tm rows), column o, channels 32 wn + 8 q
  const unsigned olane = (unsigned)(((wm * 4 * W + o) * 64 + wn * 32 + q * 8) * 2);
  const unsigned orow = (unsigned)(W * 128);
  for (int t = 0; j < ntiles; ++t) {
    const int buf = t & 1;
    const int tile = tmap(j);
    const int next = jn;
    const bool has_next = next < ntiles;
    const Org onext = origin(has_next ? tmap(next) : tile, has_next);
    const int img = tile / tpi, rem = tile - img * tpi;
    const int th0 = (rem / tw_n) * TH, tw0 = (rem - (rem / tw_n) * tw_n) * TW;
    if constexpr (DBG == 4) trace_stamp(a.trace, 2 + 4 * t);

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int k = 0; k < TN; ++k) acc[i][k] = f32x4{0.f, 0.f, 0.f, 0.f};
    const __attribute__((address_space(3))) char* pb =
        (const __attribute__((address_space(3))) char*)(size_t)(rbase + buf * BSTR);
    xu4 fb[2][TM];
    auto rd = [&](auto kc) __attribute__((always_inline)) {
      constexpr int K = decltype(kc)::value, TAP = K >> 1, HG = K & 1, S = K & 1;
      constexpr int TOFF = (TAP / 3) * PW + (TAP % 3);
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
        fb[S][tm] = *reinterpret_cast<const __attribute__((address_space(3))) xu4*>(pb + (tm * PW + TOFF) * PXB + HG * 16);
    };
    auto mm = [&](auto kc) __attribute__((always_inline)) {
      constexpr int K = decltype(kc)::value, S = K & 1;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, wr[K][tn]),
                                                               __builtin_bit_cast(half8, fb[S][tm]), acc[tm][tn], 0, 0, 0);
    };
    if constexpr (DYN) {  // the tile after next (its return is first used after the K loop's wait)
      if (tid == 0 && has_next) kdyn = atomicAdd(a.cnt + x8, 1u);
    }
    rd(xic<0>{});
    gx_for<0, 18>([&](auto kc) __attribute__((always_inline)) {
      constexpr int K = decltype(kc)::value;
      if constexpr (K + 1 < 18) rd(xic<K + 1>{});
      __builtin_amdgcn_sched_barrier(0);  // next group's reads ahead of this group's MFMAs
      if constexpr (K < PDW) {  // next tile's patch, one DMA per group
        __builtin_amdgcn_sched_barrier(0);
        dma_one(K, onext, buf ^ 1);
        __builtin_amdgcn_sched_barrier(0);
      } else if constexpr ((EPI & EPI_RES) && K < PDW + RDW) {  // this (RP: the next) tile's residual
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (RP) {
          if (has_next) dma_res(K - PDW, onext.img, onext.h0 + 1, onext.x0 + 1, buf ^ 1);
        } else {
          dma_res(K - PDW, img, th0, tw0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      } else if constexpr (DS && K >= PDW + ((EPI & EPI_RES) ? RDW : 0) && K < PDW + ((EPI & EPI_RES) ? RDW : 0) + NDR) {
        constexpr int I = K - PDW - ((EPI & EPI_RES) ? RDW : 0);  // the previous tile's row TM - NDR + I (issued last)
        __builtin_amdgcn_sched_barrier(0);
        if (t > 0) {
          if constexpr (DSL) {
            const int px = (wm * 4 + I) * TW + o;  // staged in the previous tile's buffer
            const half8 v = *reinterpret_cast<const half8*>(resb(buf ^ 1) + px * 128 + (((wn * 4 + q) ^ (px & 7)) << 4));
            store16<true>(out, pend_base + olane + I * orow, v);
          } else {
            store16<true>(out, pend_base + olane + (TM - NDR + I) * orow, pend[I]);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      mm(kc);
    });
    // next patch (+ residual, + the dynamic fetch); DS: the previous tile's stores, issued after
    // them, may stay in flight
    if constexpr (DS) {
      if (t > 0)
        xwait_vm<NDR>();
      else
        xwait_vm<0>();
    } else {
      xwait_vm<0>();
    }
    if constexpr (DYN) {
      if (tid == 0) jnext_l[t & 1] = has_next ? jof(kdyn) : ntiles;  // read after the hand-over barrier
    }
    if constexpr (DBG == 4) {  // (after the wait: a stamp's store would otherwise be waited for)
      trace_stamp(a.trace, 3 + 4 * t);
      if (lane == 0 && t < 5) a.trace[blockIdx.x * TRACE_SLOTS + 20 + 8 * t + wid] = __builtin_amdgcn_s_memrealtime();
    }
    if constexpr (!RP && (EPI & EPI_RES)) lds_barrier();  // every wave's residual DMAs landed

    f32x4 bias[TN];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) bias[tn] = *reinterpret_cast<const f32x4*>(bias_l + wn * 32 + q * 8 + tn * 4);
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
      const int px = (wm * 4 + tm) * TW + o;  // tile pixel
      half8 rv;
      if constexpr (EPI & EPI_RES) rv = *reinterpret_cast<const half8*>(resb(buf) + px * 128 + (((wn * 4 + q) ^ (px & 7)) << 4));
      half8 hv;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float v = acc[tm][e >> 2][e & 3] + bias[e >> 2][e & 3];
        if constexpr (EPI & EPI_RES) v += (float)rv[e];
        hv[e] = (_Float16)fmaxf(v, 0.f);
      }
      if constexpr (DSL) {
        *reinterpret_cast<half8*>(resb(buf) + px * 128 + (((wn * 4 + q) ^ (px & 7)) << 4)) = hv;
      } else if constexpr (DS) {
        if (tm >= TM - NDR) {
          pend[tm - (TM - NDR)] = hv;
        } else {
          const unsigned ob = (unsigned)((((img * H + th0 + wm * 4 + tm) * W + tw0 + o) * 64 + wn * 32 + q * 8) * 2);
          store16<true>(out, ob, hv);
        }
      } else {
        const unsigned ob = (unsigned)((((img * H + th0 + wm * 4 + tm) * W + tw0 + o) * 64 + wn * 32 + q * 8) * 2);
        store16<true>(out, ob, hv);
      }
    }
    if constexpr (DS) pend_base = (unsigned)(((img * H + th0) * W + tw0) * 128);
    if constexpr (DBG == 4) trace_stamp(a.trace, 4 + 4 * t);
    // every wave's DMAs into buf ^ 1 landed (its wait above) and its reads of buf (and of the
    // residual tile) retired
    lds_barrier();
    if constexpr (DBG == 4) trace_stamp(a.trace, 5 + 4 * t);
    j = jn;
    if constexpr (DYN) {
      jn = __builtin_amdgcn_readfirstlane(jnext_l[t & 1]);
    } else {
      jn = j + (int)gridDim.x;
    }
  }
  if constexpr (DS) {  // the last tile's outputs
    if ((int)blockIdx.x < ntiles) {
      if constexpr (DSL) {  // (this wave's own staged writes: no barrier needed)
        const int lb = (int)((((ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x) & 1));  // the last tile's buffer
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
          const int px = (wm * 4 + tm) * TW + o;
          const half8 v = *reinterpret_cast<const half8*>(resb(lb) + px * 128 + (((wn * 4 + q) ^ (px & 7)) << 4));
          store16<true>(out, pend_base + olane + tm * orow, v);
        }
      } else {
#pragma unroll
        for (int i = 0; i < NDR; ++i) store16<true>(out, pend_base + olane + (TM - NDR + i) * orow, pend[i]);
      }
    }
  }
  if constexpr (DYN) {  // the last workgroup out zeroes the counters (vector atomics)
    if (tid == 0 && atomicAdd(a.cnt + 8, 1u) == gridDim.x - 1) {
#pragma unroll
      for (int i = 0; i < 9; ++i) atomicExch(a.cnt + i, 0u);
    }
  }
  if constexpr (DBG == 4) {
    __builtin_amdgcn_s_waitcnt(0);
    trace_stamp(a.trace, 63);
  }
}

template <int TH, int DBG, bool DYN = false, bool DS = false, int ND = 4>
static int run_c64v(const ConvArgs& a, hipStream_t s) {
  PA_CHECK(!DYN || a.cnt, "c64v conv: dynamic tiles need the handle's counters");
  PA_CHECK(a.Hout % TH == 0 && a.Wout % 16 == 0, "c64v conv: %dx%d not tiled by %dx16", a.Hout, a.Wout, TH);
  const int tiles = a.B * (a.Hout / TH) * (a.Wout / 16);
  const int slots = conv_stream_cus(s) * (TH == 16 ? 1 : 2);  // resident workgroups
  const int grid = tiles < slots ? tiles : slots;
  // dynamic tiles: workgroup b claims gridDim.x + 8 k + b % 8, which covers every tile only when
  // all eight residues have a workgroup (a CU-masked stream of 1-3 CUs has fewer): static tiles
  if constexpr (DYN) {
    if (grid < 8) return run_c64v<TH, DBG, false>(a, s);
  }
  if (a.epi & EPI_RES)
    hipLaunchKernelGGL((conv3x3_c64v<EPI_RELU | EPI_RES, TH, DBG, DYN, DS, ND>), dim3(grid), dim3(TH * 32), 0, s, a, tiles);
  else
    hipLaunchKernelGGL((conv3x3_c64v<EPI_RELU, TH, DBG, DYN, DS, ND>), dim3(grid), dim3(TH * 32), 0, s, a, tiles);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

// variant: 0 = 16-row tiles, one 8-wave workgroup per CU; 1 = 8-row tiles, two 4-wave
// workgroups per CU; 2 (shipped, conv_patch.hip) = 16-row tiles on the plain convs, 8-row on the
// residual ones; 3 / 5 = 1 / 2 with dynamic tiles (DYN); 4 / 6 = s_memrealtime traces; timing only
// (wrong data): 7 / 8 = the DMAs without their offset arithmetic, 9 = every patch DMA on one tile
int launch_conv3x3_c64v(const ConvArgs& a, int variant, hipStream_t s) {
  PA_CHECK(a.Cin == 64 && a.Cout == 64 && a.stride == 1 && a.pad == 1 && a.Hin == a.Hout && a.Win == a.Wout,
           "c64v conv: Cin=Cout=64 stride-1 only");
  PA_CHECK(a.epi == EPI_RELU || a.epi == (EPI_RELU | EPI_RES), "c64v conv: epilogue %d", a.epi);
  PA_CHECK((size_t)a.B * a.Hout * a.Wout * 64 * 2 < 0x7fffffffu, "c64v conv: output over 2 GB");
  PA_CHECK(a.Wout <= 96, "c64v conv: width %d (packed patch offsets: 18 bits)", a.Wout);
  if (a.B <= 0) return PA_OK;
  if (variant == 4 && a.trace) return run_c64v<16, 4>(a, s);
  if (variant == 6 && a.trace) return run_c64v<8, 4>(a, s);
  if (variant == 1) return run_c64v<8, 0>(a, s);
  if (variant == 2) return (a.epi & EPI_RES) ? run_c64v<8, 0>(a, s) : run_c64v<16, 0>(a, s);
  if (variant == 3) return run_c64v<8, 0, true>(a, s);
  if (variant == 5) return (a.epi & EPI_RES) ? run_c64v<8, 0, true>(a, s) : run_c64v<16, 0>(a, s);
  // 10: variant 2 with deferred stores (DS); 11 / 12: 16-row / 8-row DS with s_memrealtime stamps
  if (variant == 10) return (a.epi & EPI_RES) ? run_c64v<8, 0, false, true>(a, s) : run_c64v<16, 0, false, true>(a, s);
  if (variant == 13) return (a.epi & EPI_RES) ? run_c64v<8, 0>(a, s) : run_c64v<16, 0, false, true>(a, s);
  // 15: the plain convs with their last row of 4 deferred in VGPRs (254; two rows spill), residual as shipped
  if (variant == 15) return (a.epi & EPI_RES) ? run_c64v<8, 0>(a, s) : run_c64v<16, 0, false, true, 1>(a, s);
  if (variant == 11 && a.trace) return run_c64v<16, 4, false, true>(a, s);
  if (variant == 12 && a.trace) return run_c64v<8, 4, false, true>(a, s);
#if PA_TIMING_VARIANTS
  if (variant == 7) return run_c64v<16, 7>(a, s);  // timing only: DMA offsets without arithmetic
  if (variant == 8) return run_c64v<8, 7>(a, s);
  if (variant == 9) return run_c64v<16, 8>(a, s);  // timing only: every patch DMA reads tile 1's patch
#endif
  return run_c64v<16, 0>(a, s);
}

}  // namespace pa
