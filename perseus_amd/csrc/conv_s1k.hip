// Layer2's 3x3 stride-1 convs (Cin = Cout = 128, 32 x 32; torchvision resnet18 layer2 BasicBlock
// conv2 of block 0 and both convs of block 1, behind perseus/detector/models.py:20),
// fp16, with the weights resident in VGPRs and the K sum split over the waves by 64-channel input
// block: conv_s2k.hip's scheme on a stride-1 patch, with half the output channels per workgroup.
//
// conv_gx.h runs these convs one 16 x 16 x 128 tile per workgroup (one round of 256 workgroups),
// streaming 16 KB weight tiles through an LDS ring: 0.75 fragment reads per MFMA plus the ring's DMA
// writes, and a prologue / epilogue that no other tile overlaps.  Here a workgroup owns 64 output
// channels (half h) for the whole launch and walks 2 x 32-pixel tiles (two output rows of an image)
// persistently.  Its 8 waves are 2 channel quarters (32 channels) x 2 input blocks (64 channels)
// x 2 output rows; a wave holds its quarter's weights for its block (18 fragments x 2 tiles = 144
// VGPRs) and reads only pixel fragments in the K loop (0.5 ds_read_b128 per MFMA).  The weights
// (147 KB per workgroup) pass through LDS once, a block per round, so that the two waves of a
// (quarter, block) pair do not both pull them from L2 (conv_c64v.hip's r05q finding).
//
// Per tile a wave accumulates 32 channels x 32 pixels (fragments tm = 0, 1: columns 16 tm + o) over
// its block's 576 K; the partner wave (other block, same quarter and row) holds the other half of
// the K sum.  Block 0's wave finalizes fragment 0, block 1's fragment 1, each receiving the
// partner's partial through LDS (2 KB per wave, double-buffered by tile parity): the sum is block
// 0's partial + block 1's (f32 addition commutes, so either wave forms the same bits).
//
// Patch: 4 input rows x 34 positions x 2 blocks, 144-byte positions (8 chunks + a pad chunk, the
// chunk of channels 32 h + 8 q at position 2 q + h: conv_c64v.hip's conflict-free layout, one
// address VGPR and ds_read immediates), double-buffered; the next tile's DMA'd during this one's
// first groups.  Epilogue: bias (+ residual, read into VGPRs during the K loop) + ReLU in f32,
// 16-byte write-through stores.  One barrier per tile.
//
// Sum order: within a block taps 0..8, 32-channel halves inner; then block 0 + block 1.  Another
// order than conv_gx.h's single accumulator, so not bit-identical to it (within the 0.05 px the
// ring kernels' orders share); its variants agree bit for bit.
//
// Measured, not shipped (variants 2:80 - 2:82, profiles/r06n/): 22.4 - 23.2 us per launch against
// conv_gx.h's 19.1 - 20.6.  The trace: the weight prologue takes 4.3 - 4.9 us (147 KB per CU, every
// CU at once: ~33 GB/s per CU), and a tile's 144 MFMAs per SIMD take ~2.0 us (26 cycles each, not
// 16): at 0.5 ds_read_b128 per MFMA the K loop is LDS-bound at ~0.6 of the MFMA rate (DESIGN.md
// 5.1), so the loop gains ~20 % on conv_gx's 0.75 reads per MFMA and the prologue takes it back.
// Triple-buffering the patch (the DMAs two tiles ahead, 2:80) did not shorten the tile: the wait
// before the hand-over barrier is the younger wave of each SIMD finishing its K loop, not the DMAs.
#include "conv_gx.h"

namespace pa {

template <int NBUF>
struct S1k {
  static constexpr int NWAVE = 8, TW = 32, PWP = TW + 2;  // positions per patch row
  static constexpr int RPC = PWP * 9;                      // 16-byte chunks per patch row (306)
  static constexpr int NRC = 4 * RPC;                      // per block region (4 input rows)
  static constexpr int NCH = 2 * NRC;                      // 2,448
  static constexpr int PJ = (NCH + 63) / 64;               // patch wave-DMAs per tile (39)
  static constexpr int PDW = (PJ + NWAVE - 1) / NWAVE;     // per wave (5, the last round partial)
  static constexpr int PATCHB = PJ * 1024;
  static constexpr int XB = NWAVE * 2 * 1024;              // partials handed over per tile
  static constexpr int WSB = 2 * 18 * 2 * 1024;            // one block's weights of the workgroup (72 KB)
  static constexpr int SMEM_RUN = NBUF * PATCHB + 2 * XB;
  // prologue: the weights are staged in [patch 1 | ..], before it is first written
  static constexpr int SMEM = PATCHB + WSB > SMEM_RUN ? PATCHB + WSB : SMEM_RUN;
  static_assert(SMEM + 256 <= 160 * 1024, "LDS");
};

// NBUF = 3: the patch triple-buffered, DMA'd two tiles ahead (a tile's K loop, ~1.2 us, is shorter
// than the DMAs' latency); NBUF = 2: one tile ahead.
// DBG = 4: s_memrealtime stamps into a.trace (0 start, 1 weights in VGPRs; tile t: 2 + 3 t start,
// 3 + 3 t K loop done, 4 + 3 t hand-over barrier passed; 63 end)
template <int EPI, int NBUF, int DBG = 0>
__global__ __launch_bounds__(512, 1) void conv3x3_s1k(ConvArgs a, const _Float16* __restrict__ wk, int ntiles,
                                                      int xo) {
  using G = S1k<NBUF>;
  constexpr int TW = G::TW, RPC = G::RPC, NRC = G::NRC, NCH = G::NCH, PJ = G::PJ, PDW = G::PDW;
  constexpr int PATCHB = G::PATCHB, XB = G::XB, WSB = G::WSB;
  constexpr int TM = 2, TN = 2, PXB = 144, NG = 18, RA = 2;  // RA: groups read ahead
  __shared__ __attribute__((aligned(1024))) char smem[G::SMEM];
  __shared__ __attribute__((aligned(16))) float bias_l[64];
  char* patch = smem;
  char* xch = smem + NBUF * PATCHB;
  char* wst = smem + PATCHB;

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, r16 = lane & 15;
  const int wn = wid & 1, wb = (wid >> 1) & 1, ph = wid >> 2;  // channel quarter, input block, output row
  if constexpr (DBG == 4) trace_stamp(a.trace, 0);
  const int H = a.Hout, W = a.Wout;
  // workgroup -> (channel half h, slot): xo = 1: blocks b and b + 8 (same XCD) take the halves of
  // the same tiles (the second reads the patch from L2)
  const int b = blockIdx.x;
  int h, slot;
  if (xo) {
    h = (b >> 3) & 1;
    slot = (b & 7) + (b >> 4) * 8;
  } else {
    h = b & 1;
    slot = b >> 1;
  }
  const int nslots = (int)gridDim.x / 2;
  const int c0 = 64 * h;
  const int tpi = H / 2;
  // XCD-grouped tile order (conv_s2v.hip): an image's tiles on one XCD in one round
  const bool xm = xo && nslots % 8 == 0 && ntiles % (8 * tpi) == 0;
  auto tmap = [&](int j) __attribute__((always_inline)) {
    if (!xm) return j;
    const int c = j / (8 * tpi), r = j - c * 8 * tpi;
    return c * 8 * tpi + (r & 7) * tpi + (r >> 3);
  };

  const unsigned abytes = (unsigned)((size_t)a.B * H * W * 256 < 0x7fffffffu ? (size_t)a.B * H * W * 256 : 0x7fffffffu);
  const s2w_u4 rsrc = s2w_rsrc(a.in, abytes);
  struct Org {
    int img, h0;
    bool on;
  };
  auto origin = [&](int t, bool on) __attribute__((always_inline)) {
    const int img = t / tpi;
    return Org{img, 2 * (t - img * tpi) - 1, on};
  };
  // patch DMA i of this wave: chunk c = (i * 8 + wid) * 64 + lane = block c / NRC, input row
  // (c % NRC) / RPC, position p = (c % RPC) / 9 (input column p - 1), chunk position c % 9 (8: pad)
  // = input channels 8 ((pos & 1) * 4 + (pos >> 1)) of the block.  Packed: bits 0-17 byte offset
  // from the patch origin (row h0, column -1), 18-21 row, 22-27 position, 28 pad / past the patch.
  unsigned pk[PDW];
#pragma unroll
  for (int i = 0; i < PDW; ++i) {
    const int c = (i * 8 + wid) * 64 + lane;
    const int blk = c / NRC, rc = c - blk * NRC, pr = rc / RPC, rem = rc - pr * RPC;
    const int p = rem / 9, pos = rem - p * 9;
    const bool bad = c >= NCH || pos >= 8;
    const unsigned rel = bad ? 0u : (unsigned)(((pr * W + p) * 128 + 64 * blk + ((pos & 1) * 4 + (pos >> 1)) * 8) * 2);
    pk[i] = (rel & 0x3ffffu) | ((unsigned)(bad ? 0 : pr) << 18) | ((unsigned)(bad ? 0 : p) << 22) | ((bad ? 1u : 0u) << 28);
  }
  auto dma_one = [&](int i, const Org& o, int buf) __attribute__((always_inline)) {
    if (PJ == PDW * 8 || i < PDW - 1 || wid < PJ - (PDW - 1) * 8) {  // wave-uniform
      const unsigned v = pk[i];
      const int pr = (int)((v >> 18) & 15u), p = (int)((v >> 22) & 63u);
      const unsigned tb = (unsigned)(((o.img * H + o.h0) * W - 1) * 256);  // wave-uniform (may wrap)
      const bool ok = o.on && !(v >> 28) && (unsigned)(o.h0 + pr) < (unsigned)H && (unsigned)(p - 1) < (unsigned)W;
      s2w_dma16(rsrc, ok ? tb + (v & 0x3ffffu) : S2W_OOB, patch + buf * PATCHB + (i * 8 + wid) * 1024);
    }
  };

  const int o = xfrag(r16);
  // this lane's patch-read base: block wb's region, patch row ph (+ tap row), position o (+ tap
  // column, + 16 tm), chunk position 2 q (+ half)
  const unsigned rbase = (unsigned)(size_t)(__attribute__((address_space(3))) char*)patch +
                         (unsigned)(wb * NRC * 16 + ph * RPC * 16 + o * PXB + q * 32);
  if (tid < 64) bias_l[tid] = a.bias[c0 + tid];
  __builtin_amdgcn_sched_barrier(0);

  // prologue: the first tile's patch; the weights ([h][wb][wn][fragment 18][tn 2][lane 64][8 fp16],
  // pa_detector_create) staged through LDS one block per round, each wave reading its 36 fragments
  int j = slot;
  {
    const Org o0 = origin(tmap(j < ntiles ? j : 0), j < ntiles);
#pragma unroll
    for (int i = 0; i < PDW; ++i) dma_one(i, o0, 0);
  }
  xu4 wr[NG][TN];
  {
    const char* wsrc = reinterpret_cast<const char*>(wk) + (size_t)h * 2 * WSB;
    gx_for<0, 2>([&](auto rc) __attribute__((always_inline)) {
      constexpr int R = decltype(rc)::value;
#pragma unroll
      for (int i = 0; i < WSB / 1024 / 8; ++i) {
        const int d = i * 8 + wid;
        xdma16(wsrc + (size_t)R * WSB + d * 1024 + lane * 16, wst + d * 1024);
      }
      xwait_vm<0>();
      lds_barrier();
      if (wb == R) {
#pragma unroll
        for (int k = 0; k < NG; ++k)
#pragma unroll
          for (int tn = 0; tn < TN; ++tn)
            wr[k][tn] = *reinterpret_cast<const xu4*>(wst + ((wn * NG + k) * TN + tn) * 1024 + lane * 16);
      }
      lds_barrier();  // reads retired before the area is rewritten
    });
  }
  if constexpr (NBUF == 3) {  // the second tile's patch (into the staging area, now free)
    const int j1 = j + nslots;
    const Org o1 = origin(tmap(j1 < ntiles ? j1 : 0), j1 < ntiles);
#pragma unroll
    for (int i = 0; i < PDW; ++i) dma_one(i, o1, 1);
  }
  if constexpr (DBG == 4) trace_stamp(a.trace, 1);

  _Float16* out = (_Float16*)a.out;
  const char* resp = (const char*)a.res;
  // this lane's output in a tile: row ph, column 16 wb + o, channels c0 + 32 wn + 8 q .. + 7
  const int ch = 32 * wn + 8 * q;
  int jn = j + (NBUF - 1) * nslots;  // the tile whose patch this one DMAs
  int buf = 0;                        // this tile's patch buffer
  for (int t = 0; j < ntiles; ++t) {
    const int dbuf = buf + NBUF - 1 >= NBUF ? buf - 1 : buf + NBUF - 1;  // (buf + NBUF - 1) % NBUF
    const int tile = tmap(j);
    const bool has_next = jn < ntiles;
    const Org onext = origin(has_next ? tmap(jn) : tile, has_next);
    const int img = tile / tpi, th0 = 2 * (tile - img * tpi);
    const unsigned ob = (unsigned)((((img * H + th0 + ph) * W + 16 * wb + o) * 128 + c0 + ch) * 2);
    if constexpr (DBG == 4) trace_stamp(a.trace, 2 + 3 * t);

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int k = 0; k < TN; ++k) acc[i][k] = f32x4{0.f, 0.f, 0.f, 0.f};
    xu4 fb[RA + 1][TM];
    half8 rv{};
    const unsigned rb = rbase + buf * PATCHB;
    auto rd = [&](auto gc) __attribute__((always_inline)) {
      constexpr int Gi = decltype(gc)::value, TAP = Gi >> 1, HG = Gi & 1, S = Gi % (RA + 1);
      constexpr int OFF = (TAP / 3) * RPC * 16 + (TAP % 3) * PXB + HG * 16;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
        fb[S][tm] = *reinterpret_cast<const __attribute__((address_space(3))) xu4*>(
            (const __attribute__((address_space(3))) char*)(size_t)rb + OFF + tm * 16 * PXB);
    };
    auto mm = [&](auto gc) __attribute__((always_inline)) {
      constexpr int Gi = decltype(gc)::value, S = Gi % (RA + 1);
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, wr[Gi][tn]),
                                                               __builtin_bit_cast(half8, fb[S][tm]), acc[tm][tn], 0, 0, 0);
    };
    gx_for<0, RA>([&](auto gc) __attribute__((always_inline)) { rd(gc); });
    gx_for<0, NG>([&](auto gc) __attribute__((always_inline)) {
      constexpr int Gi = decltype(gc)::value;
      if constexpr (Gi + RA < NG) rd(xic<Gi + RA>{});
      __builtin_amdgcn_sched_barrier(0);  // reads ahead of this group's MFMAs
      if constexpr ((EPI & EPI_RES) && Gi == 0) {  // the residual (before the DMAs: in-order vmcnt)
        rv = *reinterpret_cast<const half8*>(resp + ob);
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (Gi < PDW) {       // patch of tile jn, one DMA per group
        dma_one(Gi, onext, dbuf);     // (no such tile: onext.on = false, zeros)
        __builtin_amdgcn_sched_barrier(0);
      }
      mm(gc);
    });
    if constexpr (DBG == 4) trace_stamp(a.trace, 3 + 3 * t);

    // hand-over: block 0's wave finalizes fragment 0 and sends fragment 1 to its partner (wid ^ 2),
    // block 1's the reverse
    char* xb = xch + (t & 1) * XB;
    // (wb is wave-uniform: one compile-time copy per block, the accumulators indexed statically)
    const int pw = wid ^ 2;
    gx_for<0, 2>([&](auto wc) __attribute__((always_inline)) {
      constexpr int WB = decltype(wc)::value;
      if (wb == WB) {
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          *reinterpret_cast<f32x4*>(xb + (pw * TN + tn) * 1024 + lane * 16) = acc[1 - WB][tn];
      }
    });
    // next tile's patch landed (this wave's DMAs), residual loaded; NBUF = 3: this tile's DMAs (the
    // newest VMEM ops, 5 or 4 of them per wave) stay in flight
    if constexpr (NBUF == 2) {
      xwait_vm<0>();
    } else {
      static_assert(PJ > (PDW - 1) * 8, "DMAs per wave");
      if (PJ == PDW * 8 || wid < PJ - (PDW - 1) * 8)
        xwait_vm<PDW>();
      else
        xwait_vm<PDW - 1>();
    }
    lds_barrier();  // ... every wave's, the partials written, every read of buf retired
    if constexpr (DBG == 4) trace_stamp(a.trace, 4 + 3 * t);

    f32x4 fin[TN];
    gx_for<0, 2>([&](auto wc) __attribute__((always_inline)) {
      constexpr int WB = decltype(wc)::value;
      if (wb == WB) {
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)  // block 0 + block 1 (the same bits either way round)
          fin[tn] = acc[WB][tn] + *reinterpret_cast<const f32x4*>(xb + (wid * TN + tn) * 1024 + lane * 16);
      }
    });
    const f32x4 b0 = *reinterpret_cast<const f32x4*>(bias_l + ch);
    const f32x4 b1 = *reinterpret_cast<const f32x4*>(bias_l + ch + 4);
    half8 hv;
#pragma unroll
    for (int e8 = 0; e8 < 8; ++e8) {
      float v = fin[e8 >> 2][e8 & 3] + (e8 < 4 ? b0 : b1)[e8 & 3];
      if constexpr (EPI & EPI_RES) v += (float)rv[e8];
      hv[e8] = (_Float16)fmaxf(v, 0.f);
    }
    store16<true>(out, ob, hv);
    j += nslots;
    jn += nslots;
    buf = buf + 1 == NBUF ? 0 : buf + 1;
  }
  if constexpr (DBG == 4) {
    __builtin_amdgcn_s_waitcnt(0);
    trace_stamp(a.trace, 63);
  }
}

// variant 0: the triple-buffered patch; 1: its s_memrealtime stamps into a.trace; 2: the
// double-buffered patch
int launch_conv3x3_s1k(const ConvArgs& a, const _Float16* wk, int variant, hipStream_t s, const char** kname) {
  PA_CHECK(wk, "s1k conv: no VGPR-order weights");
  PA_CHECK(a.Cin == 128 && a.Cout == 128 && a.stride == 1 && a.pad == 1 && a.Hin == a.Hout && a.Win == a.Wout &&
               a.Wout == 32 && a.Hout % 2 == 0,
           "s1k conv: 128 -> 128 stride-1 on 32-wide maps only (%d -> %d, %dx%d)", a.Cin, a.Cout, a.Hout, a.Wout);
  PA_CHECK(a.epi == EPI_RELU || (a.epi == (EPI_RELU | EPI_RES) && a.res), "s1k conv: epilogue %d", a.epi);
  PA_CHECK((size_t)a.B * a.Hout * a.Wout * 256 < 0x7fffffffu, "s1k conv: activations over 2 GB");
  if (kname) *kname = "conv3x3k_l2";
  if (a.B <= 0) return PA_OK;
  const int tiles = a.B * (a.Hout / 2);
  const int cus = conv_stream_cus(s);
  // one 8-wave workgroup per CU; slots in groups of 8 per channel half (b and b + 8 on one XCD)
  int grid = (cus / 16) * 16;
  int xo = 1;
  if (grid == 0) {  // a few CUs (CU-masked stream): plain order
    grid = cus >= 2 ? (cus / 2) * 2 : 2;
    xo = 0;
  }
  if (grid / 2 > tiles) grid = xo ? ((tiles + 7) / 8) * 16 : 2 * tiles;
  const bool tr = variant == 1 && a.trace;
  if (a.epi & EPI_RES) {
    if (tr)
      hipLaunchKernelGGL((conv3x3_s1k<EPI_RELU | EPI_RES, 3, 4>), dim3(grid), dim3(512), 0, s, a, wk, tiles, xo);
    else if (variant == 2)
      hipLaunchKernelGGL((conv3x3_s1k<EPI_RELU | EPI_RES, 2>), dim3(grid), dim3(512), 0, s, a, wk, tiles, xo);
    else
      hipLaunchKernelGGL((conv3x3_s1k<EPI_RELU | EPI_RES, 3>), dim3(grid), dim3(512), 0, s, a, wk, tiles, xo);
  } else {
    if (tr)
      hipLaunchKernelGGL((conv3x3_s1k<EPI_RELU, 3, 4>), dim3(grid), dim3(512), 0, s, a, wk, tiles, xo);
    else if (variant == 2)
      hipLaunchKernelGGL((conv3x3_s1k<EPI_RELU, 2>), dim3(grid), dim3(512), 0, s, a, wk, tiles, xo);
    else
      hipLaunchKernelGGL((conv3x3_s1k<EPI_RELU, 3>), dim3(grid), dim3(512), 0, s, a, wk, tiles, xo);
  }
  PA_LAUNCH_CHECK();
  return PA_OK;
}

}  // namespace pa
