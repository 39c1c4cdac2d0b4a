// Layer1 3x3 stride-1 conv (Cin = Cout = 64), fp16, wide tiles: conv_c64d.hip's
// weight-resident persistent kernel with a 16 x 32-pixel tile, so that each of the
// 8 waves holds a 64-pixel x 64-channel accumulator (TM = TN = 4): 8 ds_read_b128
// per 16 MFMAs (0.5) instead of c64d's 6 per 8 (0.75).  tools/ubench/mfma_clock.hip
// puts an LDS-fed 16x16x32 loop at 0.57-0.59 of the nominal peak at 0.5 reads per
// MFMA against 0.49-0.54 at 0.75.
//
// LDS: the 72 KB of weights stay resident (c64d's 128-byte rows, tap * 64 + permuted
// output channel), and the 18 x 34 halo patch (612 pixels) is held as two CHANNEL
// halves of 64-byte rows (channels 0-31 | 32-63, 40 KB each).  The K loop runs
// half-major: groups 0-8 are the 9 taps of channels 0-31, groups 9-17 those of
// channels 32-63.  So one patch image is double-buffered by halves: once every wave
// is past group 8, half 0 takes the NEXT tile's channels 0-31 (DMA'd during groups
// 9-13), and once the tile is done, half 1 takes the next tile's channels 32-63
// (DMA'd during its groups 0-4).  2 x 40 KB + 72 KB + the bias = 152 KB.
//
// 64-byte rows: patch pixel p = (row, col)'s 16-byte chunk q (channels 8q .. 8q + 7 of
// the half) sits at p * 64 + ((q ^ ((col >> 2) & 3)) << 4).  A fragment's 16 pixels are
// consecutive columns of one row, and with conv_gx.h's lane -> pixel map (xfrag) every
// ds_read_b128 lane group then hits 16 distinct 16-byte bank slots for any start column
// (checked exhaustively on the host; tests/test_host.py).  Because the swizzle depends on
// the column only, a tap's row offset kh is a compile-time immediate on a per-(fragment,
// kw) lane address: 12 address registers for the B fragments, 8 for the A fragments
// (the weight rows' swizzle does not depend on the tap), instead of one per (fragment,
// tap), which the compiler hoisted out of the tile loop and spilled.  The DMA applies the
// swizzle through the per-lane source address, as conv_gx.h does.  The residual and the
// bias is read from LDS in the epilogue, not held across the K loop.
//
// The accumulation order differs from c64d's (half-major instead of tap-major), so
// the results are not bit-identical to it; they are deterministic and batch-invariant.
#include "conv_gx.h"

namespace pa {

namespace c64w {
constexpr int TH = 16, TW = 32, PH = TH + 2, PW = TW + 2, NP = PH * PW;  // 612 patch pixels
constexpr int NWAVE = 8, NT = NWAVE * 64;
constexpr int PJ = 40;  // wave-DMAs per half: 612 pixels x 4 chunks = 38.25 KB, padded to 5 per wave
constexpr int HALFB = PJ * 1024;
constexpr int WBYTES = 9 * 64 * 128;  // 73,728
static_assert(NP * 4 <= PJ * 64 && PJ == 5 * NWAVE, "patch DMA split: 5 per wave");
static_assert(WBYTES + 2 * HALFB <= 160 * 1024, "LDS");
}  // namespace c64w


template <int EPI, bool WT = true>
__global__ __launch_bounds__(512) void conv3x3_c64w(ConvArgs a, int ntiles) {
  using namespace c64w;
  constexpr int TM = 4, TN = 4;
  __shared__ __attribute__((aligned(1024))) char smem[WBYTES + 2 * HALFB + 64 * 4];
  char* wl = smem;
  char* patch = smem + WBYTES;  // half h at patch + h * HALFB
  float* bl = reinterpret_cast<float*>(smem + WBYTES + 2 * HALFB);  // bias, read in the epilogue

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int q = lane >> 4, r16 = lane & 15;
  const int H = a.Hout, W = a.Wout;
  const _Float16* __restrict__ in = (const _Float16*)a.in;
  const _Float16* __restrict__ w = (const _Float16*)a.w;
  const int tw_n = W / TW, tpi = (H / TH) * tw_n;

  // this lane's patch chunk of DMA i of wave wid: chunk (i * 8 + wid) * 64 + lane of a
  // half; pixel p = chunk >> 2, logical chunk = physical ^ swizzle.  Recomputed at each
  // DMA from `ln` (the lane id behind an opaque move per tile): held across the K loop,
  // the 15 values pushed the residual kernel into spills
  auto dma_half = [&](int i, int ln, int tile, int hf) __attribute__((always_inline)) {
    const int c = (i * NWAVE + wid) * 64 + ln;
    const int p = c >> 2;
    const int prow = p < NP ? p / PW : 1 << 20;  // padding chunks: always out of range (zero line)
    const int pcol = p - (p / PW) * PW;
    const int pch = ((c & 3) ^ ((pcol >> 2) & 3)) * 8;
    const int img = tile / tpi, rem = tile - img * tpi;
    const int h = (rem / tw_n) * TH + prow - 1, x = (rem - (rem / tw_n) * tw_n) * TW + pcol - 1;
    const void* src = ((unsigned)h < (unsigned)H && (unsigned)x < (unsigned)W)
                          ? (const void*)(in + (((size_t)img * H + h) * W + x) * 64 + hf * 32 + pch)
                          : (const void*)gx_zero_line;
    xdma16(src, patch + hf * HALFB + (i * NWAVE + wid) * 1024);
  };

  const int o = xfrag(r16);
  // fragment addresses: B (pixels) per (tm, kw), the tap row kh and the channel half as
  // immediates; A (weights) per (tn, half), the tap as an immediate.  Wave wid holds tile
  // rows 2 wid, 2 wid + 1; fragment tm = (row 2 wid + tm / 2, columns 16 (tm & 1) + 0..15)
  const char* bfr[TM][3];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm)
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int col = (tm & 1) * 16 + o + kw;
      bfr[tm][kw] = patch + ((2 * wid + (tm >> 1)) * PW + col) * 64 + ((q ^ ((col >> 2) & 3)) << 4);
    }
  const char* afr[TN][2];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) afr[tn][hf] = wl + xswz(tn * 16 + r16, hf * 4 + q);

  // prologue: half 0 of the first tile, then the 9 weight taps (tap i = DMA i of every
  // wave); the first tile waits for each tap just before it reads it
  int tile = blockIdx.x;
#pragma unroll
  for (int i = 0; i < 5; ++i) dma_half(i, lane, tile, 0);
  {
    const int row0 = wid * 8 + (lane >> 3);  // row within the tap
    const int lc = (lane & 7) ^ ((row0 >> 1) & 7);
    const _Float16* src = w + (size_t)xperm(row0) * 576 + lc * 8;
#pragma unroll
    for (int i = 0; i < 9; ++i) xdma16(src + i * 64, wl + (i * NWAVE + wid) * 1024);
  }
  if (tid < 64) bl[tid] = a.bias[tid];
  xwait_vm<8>();  // half 0 + tap 0
  lds_barrier();

  for (int t = 0; tile < ntiles; ++t, tile += gridDim.x) {
    const int next = tile + gridDim.x;
    const bool has_next = next < ntiles;
    const int img = tile / tpi, rem = tile - img * tpi;
    const int th0 = (rem / tw_n) * TH, tw0 = (rem - (rem / tw_n) * tw_n) * TW;
    int ln;  // the lane id, opaque to the compiler: per-lane address arithmetic stays in the tile
    asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
    auto pixo = [&](int tm) __attribute__((always_inline)) {
      return (((size_t)img * H + th0 + 2 * wid + (tm >> 1)) * W + tw0 + (tm & 1) * 16 + xfrag(ln & 15)) * 64 + (ln >> 4) * 8;
    };
    half8 rv[TM][TN / 2];
    auto load_epi = [&]() __attribute__((always_inline)) {
      if constexpr (EPI & EPI_RES) {
        const _Float16* __restrict__ res = (const _Float16*)a.res;
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
          for (int p = 0; p < TN / 2; ++p) rv[tm][p] = *reinterpret_cast<const half8*>(res + pixo(tm) + p * 32);
      }
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    xu4 fa[2][TN], fb[2][TM];
    // group K: channel half HF = K / 9, tap K % 9
    auto rd = [&](auto kc) __attribute__((always_inline)) {
      constexpr int K = decltype(kc)::value, HF = K / 9, TAP = K % 9, S = K & 1;
      constexpr int KH = TAP / 3, KW = TAP % 3;
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) fa[S][tn] = *reinterpret_cast<const xu4*>(afr[tn][HF] + TAP * 64 * 128);
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
        fb[S][tm] = *reinterpret_cast<const xu4*>(bfr[tm][KW] + HF * HALFB + KH * PW * 64);
    };
    auto mm = [&](auto kc) __attribute__((always_inline)) {
      constexpr int S = decltype(kc)::value & 1;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, fa[S][tn]),
                                                               __builtin_bit_cast(half8, fb[S][tm]), acc[tm][tn], 0, 0, 0);
    };
    rd(xic<0>{});
    gx_for<0, 18>([&](auto kc) __attribute__((always_inline)) {
      constexpr int K = decltype(kc)::value;
      if constexpr (K + 1 < 9) {
        // first tile: tap K + 1's weights.  VMEM ops issued after that DMA: the later
        // taps and this tile's half-1 DMAs so far (groups 0 .. K - 1)
        if (t == 0) {
          constexpr int J = K < 5 ? K : 5;
          xwait_vm<7 - K + J>();
          lds_barrier();
        }
      }
      if constexpr (K == 8) {
        // half 1 (DMA'd in groups 0-4) has landed everywhere, and every wave's reads of
        // half 0 have returned: half 0 is free for the next tile
        xwait_vm<0>();
        lds_barrier();
      }
      if constexpr (K + 1 < 18) rd(xic<K + 1>{});
      // this tile's half 1 in groups 0-4, the next tile's half 0 in groups 9-13
      if constexpr (K < 5 || (K >= 9 && K < 14)) {
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (K < 5)
          dma_half(K, ln, tile, 1);
        else if (has_next)
          dma_half(K - 9, ln, next, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (K == 9) {
        // the residual, 9 groups ahead of the epilogue (in group 14 it did not land in time;
        // at the tile start the compiler spilled)
        load_epi();
        __builtin_amdgcn_sched_barrier(0);
      }
      mm(kc);
    });
    xwait_vm<0>();  // next tile's half 0, residual
    f32x4 bias[TN];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) bias[tn] = *reinterpret_cast<const f32x4*>(bl + (tn >> 1) * 32 + q * 8 + (tn & 1) * 4);

    _Float16* __restrict__ out = (_Float16*)a.out;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
      for (int p = 0; p < TN / 2; ++p) {
        half8 hv;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float v = acc[tm][2 * p + (j >> 2)][j & 3] + bias[2 * p + (j >> 2)][j & 3];
          if constexpr (EPI & EPI_RES) v += (float)rv[tm][p][j];
          hv[j] = (_Float16)fmaxf(v, 0.f);
        }
        store16<WT>(out, (unsigned)((pixo(tm) + p * 32) * 2), hv);
      }
    // every wave's DMAs into half 0 landed (its wait above) and its reads of half 1
    // returned: one barrier hands both halves to the next tile
    lds_barrier();
  }
}

static int num_cus_w() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

int launch_conv3x3_c64w(const ConvArgs& a, hipStream_t s) {
  PA_CHECK(a.Cin == 64 && a.Cout == 64 && a.stride == 1 && a.pad == 1 && a.Hin == a.Hout && a.Win == a.Wout,
           "c64w conv: Cin=Cout=64 stride-1 only");
  PA_CHECK(a.Hout % c64w::TH == 0 && a.Wout % c64w::TW == 0, "c64w conv: %dx%d not tiled by 16x32", a.Hout, a.Wout);
  PA_CHECK(a.epi == EPI_RELU || a.epi == (EPI_RELU | EPI_RES), "c64w conv: epilogue %d", a.epi);
  PA_CHECK((size_t)a.B * a.Hout * a.Wout * 64 * 2 < 0x7fffffffu, "c64w conv: output over 2 GB");
  if (a.B <= 0) return PA_OK;
  const int tiles = a.B * (a.Hout / c64w::TH) * (a.Wout / c64w::TW);
  const int grid = tiles < num_cus_w() ? tiles : num_cus_w();
  if (a.epi & EPI_RES)
    hipLaunchKernelGGL((conv3x3_c64w<EPI_RELU | EPI_RES>), dim3(grid), dim3(512), 0, s, a, tiles);
  else
    hipLaunchKernelGGL((conv3x3_c64w<EPI_RELU>), dim3(grid), dim3(512), 0, s, a, tiles);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

}  // namespace pa
