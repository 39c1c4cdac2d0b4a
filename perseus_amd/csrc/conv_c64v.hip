// Layer1 3x3 stride-1 conv (Cin = Cout = 64), fp16, with the weights resident in VGPRs.
//
// conv_c64d.hip keeps the 72 KB of folded weights in LDS and reads both MFMA operands from it:
// per (tap, 32-channel) group a wave of 32 pixels x 64 channels reads 2 pixel and 4 weight
// fragments for 8 MFMAs (0.75 ds_read_b128 per 16-cycle MFMA), and its K loop runs at the
// LDS-fed rate of that shape.  Here each wave owns 64 pixels x 32 output channels and holds
// its 32 channels' weights for all 576 K (18 groups x 2 fragments x 16 B per lane = 144 VGPRs)
// for the whole launch: the K loop reads only the 4 pixel fragments of a group for its 8 MFMAs
// (0.5 reads per MFMA, nothing for the weights).  tools/ubench/mfma_shapes.hip, 8 waves,
// 16x16x32 (profiles/r05o_mfma_shapes_regs.txt): 0.60 of 2.5 PF against 0.49 for c64d's shape.
//
// Patch layout: 144 bytes per pixel (8 data chunks of 16 B + 1 pad chunk), the chunk holding
// input channels 32 h + 8 q .. + 7 at position 2 q + h.  A lane's fragment address is then
// (its pixel) * 144 + 32 q + a compile-time offset for (row, tap, half): one VGPR addresses every
// patch read of the K loop (ds_read_b128 immediates).  The XOR swizzle of conv_c64d's 128-byte
// rows needs a VGPR per (row, tap, half) address -- 72 here, which with the weights does not fit
// in 256.  Conflict-free for ds_read_b128's lane groups (MI355X_MICROARCH.md LDS table): with
// the xfrag pixel order, a group's q = 0 lanes hit 16-byte bank quads 9 P mod 16 = the even (odd)
// quads and its q = 1 lanes 9 P + 2 mod 16 = the odd (even) ones.  The LDS-DMA writes 64 x 16 B
// contiguous per wave-instruction, so the pad chunks are DMA'd too (out-of-range offset: zeros):
// 46 wave-DMAs per patch instead of 41.
//
// Same tile (16 x 16 pixels), double-buffered patch (next tile's in the first third of the K
// loop), XCD-grouped tile order, lane -> pixel map and channel permutation as conv_c64d.hip;
// each accumulator sums its MFMAs in the same order (tap 0..8, 32-channel halves) and the
// epilogue is the same (bias, residual, ReLU in f32), so the output is bit-identical to
// conv_c64d's.
#include "conv_gx.h"

namespace pa {

namespace c64v {
constexpr int TH = 16, TW = 16, PH = TH + 2, PW = TW + 2, NP = PH * PW;  // 324 patch pixels
constexpr int NWAVE = 8;
constexpr int PXB = 144;                // bytes per patch pixel (8 chunks + 1 pad)
constexpr int PJ = (NP * 9 + 63) / 64;  // 46 patch wave-DMAs
constexpr int PATCHB = PJ * 1024;
constexpr int PDW = (PJ + NWAVE - 1) / NWAVE;  // 6 per wave (waves 6, 7: 5)
static_assert(PJ == 46 && PDW == 6, "patch DMA split");
constexpr int RESB = TH * TW * 128;  // residual tile (LDS-DMA, 4 per wave)
static_assert(2 * PATCHB + RESB + 256 <= 160 * 1024, "LDS");
}  // namespace c64v

template <int EPI>
__global__ __launch_bounds__(512) void conv3x3_c64v(ConvArgs a, int ntiles) {
  using namespace c64v;
  constexpr int TM = 4, TN = 2;  // wave tile: 64 pixels (4 rows of 16) x 32 channels
  __shared__ __attribute__((aligned(1024))) char patch[2 * PATCHB];
  __shared__ __attribute__((aligned(1024))) char resl[RESB];
  __shared__ __attribute__((aligned(16))) float bias_l[64];

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, r16 = lane & 15;
  const int wn = wid & 1, wm = wid >> 1;  // channel half, pixel quarter (rows 4 wm .. 4 wm + 3)
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
  // patch DMA i of this wave: LDS slot c = (i * 8 + wid) * 64 + lane (16-byte units) holds
  // pixel c / 9, position c % 9 (8: pad), i.e. input channels 8 ((pos & 1) * 4 + (pos >> 1)) .. + 7
  // (offsets computed at the DMA: six per tile, outside the MFMA-dense part of the loop)
  // (lane laundered through an empty asm at each use: otherwise the loop-invariant per-DMA
  // offsets are hoisted out of the tile loop and held in ~30 VGPRs next to the weights)
  auto fresh_lane = [&]() __attribute__((always_inline)) {
    int l = lane;
    asm volatile("" : "+v"(l));
    return l;
  };
  auto dma_patch = [&](int i, const Org& o, int buf) __attribute__((always_inline)) {
    const int c = (i * NWAVE + wid) * 64 + fresh_lane();
    const int p = c / 9, pos = c - p * 9;
    const int pr = p / PW, pc = p - pr * PW;
    const int h = o.h0 + pr, x = o.x0 + pc;
    const bool ok = o.on && pos < 8 && p < NP && (unsigned)h < (unsigned)H && (unsigned)x < (unsigned)W;
    const unsigned vo = ok ? (unsigned)((((o.img * H + h) * W + x) * 64 + ((pos & 1) * 4 + (pos >> 1)) * 8) * 2) : S2W_OOB;
    s2w_dma16(rsrc, vo, patch + buf * PATCHB + (i * NWAVE + wid) * 1024);
  };
  auto dma_one = [&](int i, const Org& o, int buf) __attribute__((always_inline)) {
    if (i < PDW - 1 || wid < PJ - (PDW - 1) * NWAVE) dma_patch(i, o, buf);  // wave-uniform
  };
  // residual tile (EPI_RES) into LDS by DMA i = 0..3 of each wave: slot c -> tile pixel c >> 3,
  // slot chunk c & 7 = logical chunk (c & 7) ^ (pixel & 7) (the epilogue's reads are then
  // conflict-free); held in LDS, not in 16 VGPRs through the K loop
  const s2w_u4 rres = s2w_rsrc(a.res ? a.res : a.in, abytes);
  auto dma_res = [&](int i, int img, int th0, int tw0) __attribute__((always_inline)) {
    const int c = (i * NWAVE + wid) * 64 + fresh_lane();
    const int px = c >> 3, lc = (c & 7) ^ (px & 7);
    const unsigned vo = (unsigned)((((img * H + th0 + (px >> 4)) * W + tw0 + (px & 15)) * 64 + lc * 8) * 2);
    s2w_dma16(rres, vo, resl + (i * NWAVE + wid) * 1024);
  };

  const int o = xfrag(r16);
  // this lane's patch-read base: pixel (row 4 wm, column o), chunk position 2 q
  const unsigned rbase = (unsigned)(size_t)(__attribute__((address_space(3))) char*)patch + (unsigned)((wm * 4 * PW + o) * PXB + q * 32);
  if (tid < 64) bias_l[tid] = a.bias[tid];  // read back in the epilogue (8 VGPRs not held through the K loop)
  __builtin_amdgcn_sched_barrier(0);

  // prologue: the first tile's patch, then this wave's weights into registers: fragment (K, tn) =
  // channel xperm(32 wn + 16 tn + r16), tap K / 2, input channels 32 (K & 1) + 8 q .. + 7
  int j = blockIdx.x;
  {
    const Org o0 = origin(tmap(j), true);
#pragma unroll
    for (int i = 0; i < PDW; ++i) dma_one(i, o0, 0);
  }
  __builtin_amdgcn_sched_barrier(0);
  xu4 wr[18][TN];
  {
    const _Float16* ws0 = w + (size_t)xperm(wn * 32 + r16) * 576 + q * 8;
    const _Float16* ws1 = w + (size_t)xperm(wn * 32 + 16 + r16) * 576 + q * 8;
#pragma unroll
    for (int k = 0; k < 18; ++k) {
      wr[k][0] = *reinterpret_cast<const xu4*>(ws0 + (k >> 1) * 64 + (k & 1) * 32);
      wr[k][1] = *reinterpret_cast<const xu4*>(ws1 + (k >> 1) * 64 + (k & 1) * 32);
    }
  }
  xwait_vm<0>();  // patch + weights (the compiler's waitcnt pass sees this wait: no weight waits in the loop)
  lds_barrier();

  for (int t = 0; j < ntiles; ++t, j += gridDim.x) {
    const int buf = t & 1;
    const int tile = tmap(j);
    const int next = j + gridDim.x;
    const bool has_next = next < ntiles;
    const Org onext = origin(has_next ? tmap(next) : tile, has_next);
    const int img = tile / tpi, rem = tile - img * tpi;
    const int th0 = (rem / tw_n) * TH, tw0 = (rem - (rem / tw_n) * tw_n) * TW;

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int k = 0; k < TN; ++k) acc[i][k] = f32x4{0.f, 0.f, 0.f, 0.f};
    const __attribute__((address_space(3))) char* pb =
        (const __attribute__((address_space(3))) char*)(size_t)(rbase + buf * PATCHB);
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
    rd(xic<0>{});
    gx_for<0, 18>([&](auto kc) __attribute__((always_inline)) {
      constexpr int K = decltype(kc)::value;
      if constexpr (K + 1 < 18) rd(xic<K + 1>{});
      if constexpr (K < PDW) {  // next tile's patch, one DMA per group
        __builtin_amdgcn_sched_barrier(0);
        dma_one(K, onext, buf ^ 1);
        __builtin_amdgcn_sched_barrier(0);
      } else if constexpr ((EPI & EPI_RES) && K < PDW + 4) {  // this tile's residual
        __builtin_amdgcn_sched_barrier(0);
        dma_res(K - PDW, img, th0, tw0);
        __builtin_amdgcn_sched_barrier(0);
      }
      mm(kc);
    });
    xwait_vm<0>();  // next patch (+ residual)
    if constexpr (EPI & EPI_RES) lds_barrier();  // every wave's residual DMAs landed

    _Float16* __restrict__ out = (_Float16*)a.out;
    f32x4 bias[TN];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) bias[tn] = *reinterpret_cast<const f32x4*>(bias_l + wn * 32 + q * 8 + tn * 4);
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
      const int px = (wm * 4 + tm) * TW + o;  // tile pixel
      half8 rv;
      if constexpr (EPI & EPI_RES) rv = *reinterpret_cast<const half8*>(resl + px * 128 + (((wn * 4 + q) ^ (px & 7)) << 4));
      half8 hv;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float v = acc[tm][e >> 2][e & 3] + bias[e >> 2][e & 3];
        if constexpr (EPI & EPI_RES) v += (float)rv[e];
        hv[e] = (_Float16)fmaxf(v, 0.f);
      }
      const unsigned ob = (unsigned)((((img * H + th0 + wm * 4 + tm) * W + tw0 + o) * 64 + wn * 32 + q * 8) * 2);
      store16<true>(out, ob, hv);
    }
    // every wave's DMAs into buf ^ 1 landed (its wait above) and its reads of buf retired
    lds_barrier();
  }
}

int launch_conv3x3_c64v(const ConvArgs& a, int variant, hipStream_t s) {
  PA_CHECK(a.Cin == 64 && a.Cout == 64 && a.stride == 1 && a.pad == 1 && a.Hin == a.Hout && a.Win == a.Wout,
           "c64v conv: Cin=Cout=64 stride-1 only");
  PA_CHECK(a.Hout % c64v::TH == 0 && a.Wout % c64v::TW == 0, "c64v conv: %dx%d not tiled by 16x16", a.Hout, a.Wout);
  PA_CHECK(a.epi == EPI_RELU || a.epi == (EPI_RELU | EPI_RES), "c64v conv: epilogue %d", a.epi);
  PA_CHECK((size_t)a.B * a.Hout * a.Wout * 64 * 2 < 0x7fffffffu, "c64v conv: output over 2 GB");
  (void)variant;
  if (a.B <= 0) return PA_OK;
  const int tiles = a.B * (a.Hout / c64v::TH) * (a.Wout / c64v::TW);
  const int cus = conv_stream_cus(s);
  const int grid = tiles < cus ? tiles : cus;
  if (a.epi & EPI_RES)
    hipLaunchKernelGGL((conv3x3_c64v<EPI_RELU | EPI_RES>), dim3(grid), dim3(512), 0, s, a, tiles);
  else
    hipLaunchKernelGGL((conv3x3_c64v<EPI_RELU>), dim3(grid), dim3(512), 0, s, a, tiles);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

}  // namespace pa
