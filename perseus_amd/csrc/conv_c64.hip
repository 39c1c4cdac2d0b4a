// Weight-resident persistent 3x3 stride-1 conv for Cin = Cout = 64 (the four
// layer1 convs of torchvision resnet18), fp16.
//
// All 9 x 64 x 64 folded weights (72 KB) are staged into LDS once per workgroup;
// the grid is one workgroup per CU and each walks tiles blockIdx.x + t*gridDim.x
// (16 x 16 output pixels x 64 channels).  The input halo patch (18 x 18 x 64,
// 41.5 KB) is double-buffered: the next tile's patch is loaded into registers at
// the start of a tile and stored after its MFMAs, so there is ONE barrier per
// tile and none inside the 9-tap x 64-channel reduction -- the waves stream LDS
// fragment reads against back-to-back MFMAs (the per-tap barrier of
// conv_patch.hip is what held layer1 at ~0.25 of peak).
//
// Same LDS image conventions as conv_patch.hip: 128-byte rows (a pixel's or an
// output channel's 64 fp16), 16-byte chunks XOR-swizzled by (row >> 1) & 7,
// lane -> pixel map frag_off, MFMA A = weights / B = pixels so each lane holds 4
// consecutive output channels of one pixel for the register epilogue.
#include <type_traits>

#include "conv.h"

namespace pa {

typedef unsigned c64u4 __attribute__((ext_vector_type(4)));

template <int V>
using c64ic = std::integral_constant<int, V>;

// compile-time loop: f(integral_constant<int, I>) for I in [B, E)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(c64ic<B>{});
    static_for<B + 1, E>(f);
  }
}

namespace c64 {
constexpr int TH = 16, TW = 16;
constexpr int PH = TH + 2, PW = TW + 2, NP = PH * PW;  // 324 patch pixels
constexpr int PATCHB = NP * 128;                        // 41,472 B
constexpr int WROWS = 9 * 64;                           // tap-major weight rows
constexpr int WBYTES = WROWS * 128;                     // 73,728 B
}  // namespace c64

__device__ __forceinline__ int c64swz(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }
__device__ __forceinline__ int c64frag(int r) { return r < 4 ? 2 * r : (r < 12 ? 2 * (r - 4) + 1 : 2 * (r - 8)); }
// Output-channel order of the weight rows inside each group of 32: LDS row
// rho = 16 t + 4 q + v (MFMA tile t of a pair, lane quad q, accumulator slot v)
// holds channel 8 q + 4 t + v, so a lane's two tiles of a pair cover 8
// consecutive channels of its pixel -> 16-byte residual loads and output stores.
__device__ __forceinline__ int c64perm(int rho) {
  return (rho & ~31) | (((rho >> 2) & 3) << 3) | (((rho >> 4) & 1) << 2) | (rho & 3);
}

// DBG (timing-only variants, wrong results): 1 = no MFMA loop, 2 = no next-patch
// loads (every tile reuses the first patch), 3 = no weight staging; 4 = the
// shipped kernel plus s_memrealtime stamps into a.trace (conv.h trace_stamp)
template <int WM, int EPI, int DBG = 0, bool WT = false>
__global__ __launch_bounds__(WM * 64) void conv3x3_c64(ConvArgs a, int ntiles) {
  using namespace c64;
  constexpr int NT = WM * 64;
  constexpr int WTM = TH * TW / WM;  // pixels per wave
  constexpr int TM = WTM / 16, TN = 4;
  constexpr int PCH = (NP * 8 + NT - 1) / NT;
  constexpr int WCH = WROWS * 8 / NT;
  static_assert(WROWS * 8 % NT == 0, "weight chunks / threads");
  __shared__ __attribute__((aligned(16))) char smem[WBYTES + 2 * PATCHB];
  char* wl = smem;
  char* patch = smem + WBYTES;

  const int tid = threadIdx.x, lane = tid & 63, wm = tid >> 6;
  const int q = lane >> 4, r16 = lane & 15;
  const int H = a.Hout, W = a.Wout;
  const _Float16* __restrict__ in = (const _Float16*)a.in;
  const _Float16* __restrict__ w = (const _Float16*)a.w;
  const int tw_n = W / TW, tpi = (H / TH) * tw_n;
  if constexpr (DBG == 4) trace_stamp(a.trace, 0);

  // ---- weights -> LDS once: row = tap * 64 + co, source [co][tap][64 ch]
  if constexpr (DBG != 3) {
    constexpr int HALF = (WCH + 1) / 2;  // two batches to bound live registers
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      c64u4 v[HALF];
#pragma unroll
      for (int i = 0; i < HALF; ++i) {
        const int c = tid + (h * HALF + i) * NT;
        if (h * HALF + i < WCH) {
          const int row = c >> 3, ch = c & 7;
          const int tap = row >> 6, co = row & 63;
          v[i] = *reinterpret_cast<const c64u4*>(w + (size_t)c64perm(co) * 576 + tap * 64 + ch * 8);
        }
      }
#pragma unroll
      for (int i = 0; i < HALF; ++i) {
        const int c = tid + (h * HALF + i) * NT;
        if (h * HALF + i < WCH) *reinterpret_cast<c64u4*>(wl + c64swz(c >> 3, c & 7)) = v[i];
      }
    }
  }

  c64u4 rp[PCH];
  auto load_patch = [&](int tile) __attribute__((always_inline)) {
    const int img = tile / tpi, rem = tile - (tile / tpi) * tpi;
    const int th0 = (rem / tw_n) * TH, tw0 = (rem - (rem / tw_n) * tw_n) * TW;
#pragma unroll
    for (int i = 0; i < PCH; ++i) {
      const int c = tid + i * NT;
      c64u4 v = c64u4{0u, 0u, 0u, 0u};
      const int p = c >> 3, ch = c & 7;
      const int pr = p / PW, pc = p - (p / PW) * PW;
      const int h = th0 + pr - 1, x = tw0 + pc - 1;
      if (c < NP * 8 && tile < ntiles && (unsigned)h < (unsigned)H && (unsigned)x < (unsigned)W)
        v = *reinterpret_cast<const c64u4*>(in + (((size_t)img * H + h) * W + x) * 64 + ch * 8);
      rp[i] = v;
    }
  };
  auto store_patch = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < PCH; ++i) {
      const int c = tid + i * NT;
      if (c < NP * 8) *reinterpret_cast<c64u4*>(patch + buf * PATCHB + c64swz(c >> 3, c & 7)) = rp[i];
    }
  };

  const int o = c64frag(r16);
  int ppix[TM];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int mb = wm * WTM + tm * 16;
    ppix[tm] = (mb / TW) * PW + mb % TW + o;
  }
  // lane's channels for tile pair p: 32 p + 8 q + [0, 8)
  f32x4 bias[TN];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) bias[tn] = *reinterpret_cast<const f32x4*>(a.bias + (tn >> 1) * 32 + q * 8 + (tn & 1) * 4);

  int tile = blockIdx.x;
  load_patch(tile);
  store_patch(0);
  __syncthreads();
  if constexpr (DBG == 4) trace_stamp(a.trace, 1);

  for (int t = 0; tile < ntiles; ++t, tile += gridDim.x) {
    const int buf = t & 1;
    const int next = tile + gridDim.x;
    if constexpr (DBG != 2) load_patch(next);  // zeros past the last tile (never read)
    if constexpr (DBG == 4) trace_stamp(a.trace, 2 + 4 * t);

    const int img = tile / tpi, rem = tile - (tile / tpi) * tpi;
    const int th0 = (rem / tw_n) * TH, tw0 = (rem - (rem / tw_n) * tw_n) * TW;
    size_t pixo[TM];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
      const int mb = wm * WTM + tm * 16;
      pixo[tm] = (((size_t)img * H + th0 + mb / TW) * W + tw0 + mb % TW + o) * 64;
    }
    // residual issued now, kept raw: converting here would make the MFMAs below
    // wait for it (and, vmcnt being in order, for the next patch's loads)
    half8 rv[TM][TN / 2];
    if constexpr (EPI & EPI_RES) {
      const _Float16* __restrict__ res = (const _Float16*)a.res;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int p = 0; p < TN / 2; ++p) rv[tm][p] = *reinterpret_cast<const half8*>(res + pixo[tm] + p * 32 + q * 8);
      // keep them here: the scheduler would otherwise sink them next to their use
      __builtin_amdgcn_sched_barrier(0);
    }

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* pb = patch + buf * PATCHB;
    // 18 (tap, 32-channel half) groups; the fragments of group k+1 are read into
    // the other register set before group k's MFMAs issue (software pipeline).
    c64u4 fa[2][TN], fb[2][TM];
    auto rd = [&](auto kc) __attribute__((always_inline)) {
      constexpr int K = decltype(kc)::value, TAP = K >> 1, G = K & 1, S = K & 1;
      constexpr int TOFF = (TAP / 3) * PW + (TAP % 3);
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        fa[S][tn] = *reinterpret_cast<const c64u4*>(wl + c64swz(TAP * 64 + tn * 16 + r16, G * 4 + q));
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
        fb[S][tm] = *reinterpret_cast<const c64u4*>(pb + c64swz(ppix[tm] + TOFF, G * 4 + q));
    };
    auto mm = [&](auto kc) __attribute__((always_inline)) {
      constexpr int S = decltype(kc)::value & 1;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, fa[S][tn]),
                                                               __builtin_bit_cast(half8, fb[S][tm]), acc[tm][tn], 0,
                                                               0, 0);
    };
    if constexpr (DBG != 1) {
    rd(c64ic<0>{});
    static_for<0, 18>([&](auto kc) __attribute__((always_inline)) {
      constexpr int K = decltype(kc)::value;
      if constexpr (K + 1 < 18) rd(c64ic<K + 1>{});
      mm(kc);
    });
    }

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
          v = fmaxf(v, 0.f);
          hv[j] = (_Float16)v;
        }
        store16<WT>(out, (unsigned)((pixo[tm] + p * 32 + q * 8) * 2), hv);
      }
    if constexpr (DBG == 4) trace_stamp(a.trace, 3 + 4 * t);

    // next tile's patch into the other buffer (last read during tile t-1, before
    // the previous barrier), then one barrier
    if constexpr (DBG != 2) store_patch(buf ^ 1);
    if constexpr (DBG == 4) trace_stamp(a.trace, 4 + 4 * t);
    __syncthreads();
    if constexpr (DBG == 4) trace_stamp(a.trace, 5 + 4 * t);
  }
  if constexpr (DBG == 4) {
    __builtin_amdgcn_s_waitcnt(0);
    trace_stamp(a.trace, 63);
  }
}

static int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

template <int WM, int DBG = 0, bool WT = false>
static int run_c64(const ConvArgs& a, hipStream_t s) {
  PA_CHECK(!WT || (size_t)a.B * a.Hout * a.Wout * 64 * 2 < 0x7fffffffu, "c64 conv: output over 2 GB");
  const int tiles = a.B * (a.Hout / c64::TH) * (a.Wout / c64::TW);
  const int grid = tiles < num_cus() ? tiles : num_cus();
  if (a.epi & EPI_RES)
    hipLaunchKernelGGL((conv3x3_c64<WM, EPI_RELU | EPI_RES, DBG, WT>), dim3(grid), dim3(WM * 64), 0, s, a, tiles);
  else
    hipLaunchKernelGGL((conv3x3_c64<WM, EPI_RELU, DBG, WT>), dim3(grid), dim3(WM * 64), 0, s, a, tiles);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

int launch_conv3x3_c64(const ConvArgs& a, int variant, hipStream_t s) {
  PA_CHECK(a.Cin == 64 && a.Cout == 64 && a.stride == 1 && a.pad == 1 && a.Hin == a.Hout && a.Win == a.Wout,
           "c64 conv: Cin=Cout=64 stride-1 only");
  PA_CHECK(a.Hout % c64::TH == 0 && a.Wout % c64::TW == 0, "c64 conv: %dx%d not tiled by 16x16", a.Hout, a.Wout);
  PA_CHECK(a.epi == EPI_RELU || a.epi == (EPI_RELU | EPI_RES), "c64 conv: epilogue %d", a.epi);
  if (a.B <= 0) return PA_OK;
  switch (variant) {
    case 1: return run_c64<4>(a, s);
    case 5: return run_c64<8, 0, false>(a, s);  // plain (write-back) stores
#if PA_TIMING_VARIANTS
    case 7: return run_c64<8, 1>(a, s);  // timing only (wrong results)
    case 8: return run_c64<8, 2>(a, s);
    case 9: return run_c64<8, 3>(a, s);
#endif
    case 6: return a.trace ? run_c64<8, 4>(a, s) : run_c64<8>(a, s);
    default: return run_c64<8, 0, true>(a, s);
  }
}

}  // namespace pa
