// Layer1 3x3 stride-1 conv (Cin = Cout = 64, 64 x 64 maps; torchvision resnet18
// layer1), fp16: weight-resident persistent kernel, version 2.
//
// conv_c64.hip ran 8 waves of 32 pixels x 64 channels: 6 LDS fragment reads per 8
// MFMAs, 75 % of the LDS read rate at full MFMA rate, with the fragments of a
// group read only one group ahead.  Here a workgroup is 4 waves (one per SIMD),
// each owning 64 pixels x 64 channels of the 16 x 16 tile: 8 reads per 16 MFMAs
// (50 %), fragments read two groups ahead (three register sets).  The next tile's
// halo patch is DMA'd into the other buffer at the start of a tile (inline-asm
// LDS-DMA, conv_gx.h) instead of being staged through registers, and waited for
// with a counted vmcnt at the tile's end: one barrier per tile.
//
// LDS: 9 x 64 x 64 folded weights (72 KB, DMA'd once) + 2 patch buffers
// (18 x 18 x 64 fp16, padded to whole wave-instructions) = 160 KB.
// Same image conventions as conv_gx.h: 128-byte rows, XOR-swizzled 16-B chunks,
// lane -> pixel map xfrag, MFMA A = weights / B = pixels, channel-pair weight row
// permutation for 16-byte epilogue accesses.
#include "conv_gx.h"

namespace pa {

namespace l1x {
constexpr int TH = 16, TW = 16, PH = TH + 2, PW = TW + 2, NP = PH * PW;  // 324 patch pixels
constexpr int NW = 4;
constexpr int PDMA = ((NP * 8 + 63) / 64 + NW - 1) / NW;  // patch DMA instructions per wave (11)
constexpr int PATCHB = PDMA * NW * 1024;                  // 45,056 B
constexpr int WROWS = 9 * 64, WBYTES = WROWS * 128;       // tap-major weight rows, 73,728 B
constexpr int WDMA = WROWS * 8 / 64 / NW;                 // 18
constexpr int TM = 4, TN = 4;                             // wave tile 64 px x 64 ch
static_assert(WBYTES + 2 * PATCHB <= 163840, "LDS");
}  // namespace l1x

template <int EPI>
__global__ __launch_bounds__(256) void conv3x3_l1x(ConvArgs a, int ntiles) {
  using namespace l1x;
  __shared__ __attribute__((aligned(1024))) char smem[WBYTES + 2 * PATCHB];
  char* wl = smem;
  char* patch = smem + WBYTES;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int q = lane >> 4, r16 = lane & 15;
  constexpr int H = 64, W = 64, C = 64;
  const _Float16* __restrict__ in = (const _Float16*)a.in;
  const _Float16* __restrict__ w = (const _Float16*)a.w;
  constexpr int TPI = (H / TH) * (W / TW);

  // weights once: LDS row tap * 64 + co <- w[xperm(co)][tap][.] (chunk swizzled at the source)
#pragma unroll
  for (int i = 0; i < WDMA; ++i) {
    const int c = (i * NW + wid) * 64 + lane;
    const int row = c >> 3, lc = (c & 7) ^ ((row >> 1) & 7);
    const int tap = row >> 6, co = row & 63;
    xdma16(w + (size_t)xperm(co) * 576 + tap * 64 + lc * 8, wl + (i * NW + wid) * 1024);
  }
  auto dma_patch = [&](int tile, int buf) __attribute__((always_inline)) {
    const int img = tile / TPI, rem = tile - (tile / TPI) * TPI;
    const int th0 = (rem / (W / TW)) * TH, tw0 = (rem % (W / TW)) * TW;
#pragma unroll
    for (int i = 0; i < PDMA; ++i) {
      const int c = (i * NW + wid) * 64 + lane;
      const int p = c >> 3, pc = c & 7;
      const int lc = pc ^ ((p >> 1) & 7);
      const int pr = p / PW, pcl = p - (p / PW) * PW;
      const int h = th0 + pr - 1, x = tw0 + pcl - 1;
      const bool ok = p < NP && tile < ntiles && (unsigned)h < (unsigned)H && (unsigned)x < (unsigned)W;
      const void* src = ok ? (const void*)(in + (((size_t)img * H + h) * W + x) * C + lc * 8) : (const void*)gx_zero_line;
      xdma16(src, patch + buf * PATCHB + (i * NW + wid) * 1024);
    }
  };

  const int o = xfrag(r16);
  int ppix[TM];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) ppix[tm] = (4 * wid + tm) * PW + o;  // wave wid: tile rows 4 wid .. 4 wid + 3
  f32x4 bias[TN];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) bias[tn] = *reinterpret_cast<const f32x4*>(a.bias + (tn >> 1) * 32 + q * 8 + (tn & 1) * 4);

  int tile = blockIdx.x;
  dma_patch(tile, 0);
  xwait_vm<0>();
  __builtin_amdgcn_s_barrier();

  const _Float16* __restrict__ res = (const _Float16*)a.res;
  _Float16* __restrict__ out = (_Float16*)a.out;
  for (int t = 0; tile < ntiles; ++t, tile += gridDim.x) {
    const int buf = t & 1;
    dma_patch(tile + gridDim.x, buf ^ 1);  // zero lines past the last tile (never read)

    const int img = tile / TPI, rem = tile - (tile / TPI) * TPI;
    const int th0 = (rem / (W / TW)) * TH, tw0 = (rem % (W / TW)) * TW;
    size_t pixo[TM];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) pixo[tm] = (((size_t)img * H + th0 + 4 * wid + tm) * W + tw0 + o) * C + q * 8;
    half8 rv[TM][TN / 2];
    if constexpr (EPI & EPI_RES) {
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int p = 0; p < TN / 2; ++p) rv[tm][p] = *reinterpret_cast<const half8*>(res + pixo[tm] + p * 32);
      __builtin_amdgcn_sched_barrier(0);  // keep them here, not next to their use
    }

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* pb = patch + buf * PATCHB;
    // 18 groups (tap, 32-channel half); fragments two groups ahead, three sets
    xu4 fa[3][TN], fb[3][TM];
    auto rd = [&](auto kc) __attribute__((always_inline)) {
      constexpr int K = decltype(kc)::value, TAP = K >> 1, HG = K & 1, SET = K % 3;
      constexpr int TOFF = (TAP / 3) * PW + (TAP % 3);
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        fa[SET][tn] = *reinterpret_cast<const xu4*>(wl + xswz(TAP * 64 + tn * 16 + r16, HG * 4 + q));
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
        fb[SET][tm] = *reinterpret_cast<const xu4*>(pb + xswz(ppix[tm] + TOFF, HG * 4 + q));
    };
    rd(xic<0>{});
    rd(xic<1>{});
    gx_for<0, 18>([&](auto kc) __attribute__((always_inline)) {
      constexpr int K = decltype(kc)::value, SET = K % 3;
      if constexpr (K + 2 < 18) rd(xic<K + 2>{});
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, fa[SET][tn]),
                                                               __builtin_bit_cast(half8, fb[SET][tm]), acc[tm][tn], 0,
                                                               0, 0);
    });

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
        *reinterpret_cast<half8*>(out + pixo[tm] + p * 32) = hv;
      }
    // the next patch (DMA'd before the residual loads and these 8 stores) must have
    // landed in every wave before the next tile's reads; the stores may stay in flight
    xwait_vm<TM * TN / 2>();
    __builtin_amdgcn_s_barrier();
  }
}

static int l1x_num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

int launch_conv3x3_l1x(const ConvArgs& a, hipStream_t s) {
  PA_CHECK(a.Cin == 64 && a.Cout == 64 && a.stride == 1 && a.pad == 1 && a.Hin == 64 && a.Win == 64 && a.Hout == 64 &&
               a.Wout == 64,
           "l1x conv: layer1 shape only");
  PA_CHECK(a.epi == EPI_RELU || a.epi == (EPI_RELU | EPI_RES), "l1x conv: epilogue %d", a.epi);
  if (a.B <= 0) return PA_OK;
  const int tiles = a.B * (64 / l1x::TH) * (64 / l1x::TW);
  const int grid = tiles < l1x_num_cus() ? tiles : l1x_num_cus();
  if (a.epi & EPI_RES)
    hipLaunchKernelGGL((conv3x3_l1x<EPI_RELU | EPI_RES>), dim3(grid), dim3(256), 0, s, a, tiles);
  else
    hipLaunchKernelGGL((conv3x3_l1x<EPI_RELU>), dim3(grid), dim3(256), 0, s, a, tiles);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

}  // namespace pa
