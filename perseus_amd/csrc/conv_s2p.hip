// Persistent stride-2 BasicBlock entry conv (3x3 s2 + bn1 + relu) with the 1x1 s2
// downsample (+ bn) fused, fp16 (torchvision resnet18 layer2/3/4 block 0,
// SURVEY.md 8a6-a8).  Replaces conv_s2.hip's one-tile-per-workgroup kernel,
// whose 72 KB input patch per 128 output pixels made every workgroup wait on
// HBM before a short K loop (0.11-0.15 of MFMA peak).
//
// Work unit = (output tile, 64-channel input block cb).  A workgroup owns one
// N-tile of BN output channels and walks its tiles blockIdx.x + k*gridDim.x; for
// every unit the input patch (2TH+1 rows x 2TW+1 de-interleaved columns), the 9
// tap weight slices and the downsample slice of block cb sit in LDS, and the
// NEXT unit's are loaded into registers while this one computes (one unit of
// prefetch = the whole HBM latency hidden behind 9 taps of MFMAs).  The 9-tap
// reduction has no barrier; fragment reads of tap k+1 are issued before the
// MFMAs of tap k.  Two barriers per unit (LDS free -> refill -> visible).  With
// one input block (layer2) the weights are loaded once per workgroup.
//
// LDS images as conv_s2.hip: 128-byte rows, XOR-swizzled 16-B chunks, the
// centre tap's B fragments feed the downsample MFMAs too.
#include <type_traits>

#include "conv.h"

namespace pa {

typedef unsigned s2pu4 __attribute__((ext_vector_type(4)));

template <int V>
using s2pic = std::integral_constant<int, V>;

template <int B, int E, typename F>
__device__ __forceinline__ void s2p_for(F&& f) {
  if constexpr (B < E) {
    f(s2pic<B>{});
    s2p_for<B + 1, E>(f);
  }
}

__device__ __forceinline__ int s2pswz(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }
__device__ __forceinline__ int s2pfrag(int r) { return r < 4 ? 2 * r : (r < 12 ? 2 * (r - 4) + 1 : 2 * (r - 8)); }

template <int TH, int TW, int BN, int WM, int WN, int CIN>
__global__ __launch_bounds__(WM * WN * 64) void conv3x3s2_ds_p(ConvS2Args a, int ntiles) {
  constexpr int NT = WM * WN * 64;
  constexpr int NCB = CIN / 64;
  constexpr int PH = 2 * TH + 1, PW = 2 * TW + 1, NP = PH * PW;
  constexpr int BM = TH * TW;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int PATCHB = NP * 128;
  constexpr int WROWS = 9 * BN;
  constexpr int WBYTES = WROWS * 128, DBYTES = BN * 128;
  constexpr int PCH = (NP * 8 + NT - 1) / NT;
  constexpr int WCH = WROWS * 8 / NT, DCH = BN * 8 / NT;
  static_assert(TW == 16 && BM % WM == 0 && WTM % 16 == 0 && WTN % 16 == 0, "tile geometry");
  static_assert(WROWS * 8 % NT == 0 && BN * 8 % NT == 0, "staging / threads");
  __shared__ __attribute__((aligned(16))) char smem[PATCHB + WBYTES + DBYTES];
  char* patch = smem;
  char* wl = smem + PATCHB;
  char* dl = wl + WBYTES;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int q = lane >> 4, r16 = lane & 15;
  const int H = a.Hout, W = a.Wout, Hin = a.Hin, Win = a.Win, Cout = a.Cout;
  const _Float16* __restrict__ in = (const _Float16*)a.in;
  const _Float16* __restrict__ w = (const _Float16*)a.w;
  const _Float16* __restrict__ wds = (const _Float16*)a.wds;
  const int ntn = Cout / BN;
  const int n0 = (blockIdx.x % ntn) * BN;
  const int tw_n = W / TW, tpi = (H / TH) * tw_n;

  s2pu4 rp[PCH], rw[NCB > 1 ? WCH : 1], rd[NCB > 1 ? DCH : 1];
  auto load_patch = [&](int tile, int cb) __attribute__((always_inline)) {
    const int sp = tile / ntn;
    const int img = sp / tpi, rem = sp - (sp / tpi) * tpi;
    const int th0 = (rem / tw_n) * TH, tw0 = (rem - (rem / tw_n) * tw_n) * TW;
#pragma unroll
    for (int i = 0; i < PCH; ++i) {
      const int c = tid + i * NT;
      const int p = c >> 3, ch = c & 7;
      const int pr = p / PW, pos = p - (p / PW) * PW;
      const int col = pos <= TW ? 2 * pos : 2 * (pos - TW - 1) + 1;  // de-interleaved columns
      const int h = 2 * th0 - 1 + pr, x = 2 * tw0 - 1 + col;
      s2pu4 v = s2pu4{0u, 0u, 0u, 0u};
      if (c < NP * 8 && tile < ntiles && (unsigned)h < (unsigned)Hin && (unsigned)x < (unsigned)Win)
        v = *reinterpret_cast<const s2pu4*>(in + (((size_t)img * Hin + h) * Win + x) * CIN + cb * 64 + ch * 8);
      rp[i] = v;
    }
  };
  auto store_patch = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < PCH; ++i) {
      const int c = tid + i * NT;
      if (c < NP * 8) *reinterpret_cast<s2pu4*>(patch + s2pswz(c >> 3, c & 7)) = rp[i];
    }
  };
  // weights of block cb: LDS row tap * BN + co  <-  w[n0 + co][tap][cb*64 + ch*8]
  auto load_w = [&](int cb, s2pu4* v) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < WCH; ++i) {
      const int c = tid + i * NT;
      const int row = c >> 3, ch = c & 7;
      const int tap = row / BN, co = row - (row / BN) * BN;
      v[i] = *reinterpret_cast<const s2pu4*>(w + (size_t)(n0 + co) * (9 * CIN) + tap * CIN + cb * 64 + ch * 8);
    }
  };
  auto store_w = [&](const s2pu4* v) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < WCH; ++i) {
      const int c = tid + i * NT;
      *reinterpret_cast<s2pu4*>(wl + s2pswz(c >> 3, c & 7)) = v[i];
    }
  };
  auto load_d = [&](int cb, s2pu4* v) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < DCH; ++i) {
      const int c = tid + i * NT;
      v[i] = *reinterpret_cast<const s2pu4*>(wds + (size_t)(n0 + (c >> 3)) * CIN + cb * 64 + (c & 7) * 8);
    }
  };
  auto store_d = [&](const s2pu4* v) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < DCH; ++i) {
      const int c = tid + i * NT;
      *reinterpret_cast<s2pu4*>(dl + s2pswz(c >> 3, c & 7)) = v[i];
    }
  };

  const int o = s2pfrag(r16);
  int ppix[TM];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int mb = wm * WTM + tm * 16;
    ppix[tm] = (2 * (mb / TW)) * PW + mb % TW + o;
  }
  f32x4 b1[TN], b2[TN];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) {
    b1[tn] = *reinterpret_cast<const f32x4*>(a.bias + n0 + wn * WTN + tn * 16 + q * 4);
    b2[tn] = *reinterpret_cast<const f32x4*>(a.bias2 + n0 + wn * WTN + tn * 16 + q * 4);
  }

  // ---- prologue: unit (first tile, block 0)
  int tile = blockIdx.x;
  {
    s2pu4 v[WCH], vd[DCH];
    load_patch(tile, 0);
    load_w(0, v);
    load_d(0, vd);
    store_patch();
    store_w(v);
    store_d(vd);
  }
  __syncthreads();

  f32x4 acc[TM][TN], accd[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      accd[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

  int cb = 0;
  while (tile < ntiles) {
    // next unit: (tile, cb + 1) or (tile + grid, 0); prefetched into registers
    const int ncb = cb + 1 < NCB ? cb + 1 : 0;
    const int ntile = cb + 1 < NCB ? tile : tile + (int)gridDim.x;
    load_patch(ntile, ncb);
    if constexpr (NCB > 1) {
      load_w(ncb, rw);
      load_d(ncb, rd);
    }

    // 18 (tap, channel-half) groups, fragments of group k+1 read before group k's MFMAs
    s2pu4 fa[2][TN], fb[2][TM], fd[TN];
    auto rd_frag = [&](auto kc) __attribute__((always_inline)) {
      constexpr int K = decltype(kc)::value, TAP = K >> 1, G = K & 1, S = K & 1;
      constexpr int KR = TAP / 3, KC = TAP % 3;
      constexpr int COL = KC == 0 ? 0 : (KC == 1 ? TW + 1 : 1);
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        fa[S][tn] = *reinterpret_cast<const s2pu4*>(wl + s2pswz(TAP * BN + wn * WTN + tn * 16 + r16, G * 4 + q));
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
        fb[S][tm] = *reinterpret_cast<const s2pu4*>(patch + s2pswz(ppix[tm] + KR * PW + COL, G * 4 + q));
    };
    auto mm = [&](auto kc) __attribute__((always_inline)) {
      constexpr int K = decltype(kc)::value, TAP = K >> 1, G = K & 1, S = K & 1;
      if constexpr (TAP == 4) {
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          fd[tn] = *reinterpret_cast<const s2pu4*>(dl + s2pswz(wn * WTN + tn * 16 + r16, G * 4 + q));
      }
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, fa[S][tn]),
                                                               __builtin_bit_cast(half8, fb[S][tm]), acc[tm][tn], 0, 0,
                                                               0);
          if constexpr (TAP == 4)  // centre tap = the 1x1 stride-2 downsample's input
            accd[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, fd[tn]),
                                                                  __builtin_bit_cast(half8, fb[S][tm]), accd[tm][tn],
                                                                  0, 0, 0);
        }
    };
    rd_frag(s2pic<0>{});
    s2p_for<0, 18>([&](auto kc) __attribute__((always_inline)) {
      constexpr int K = decltype(kc)::value;
      if constexpr (K + 1 < 18) rd_frag(s2pic<K + 1>{});
      mm(kc);
    });

    if (cb == NCB - 1) {
      // epilogue: conv1 -> relu -> out; downsample -> out2 (no relu)
      const int sp = tile / ntn;
      const int img = sp / tpi, rem = sp - (sp / tpi) * tpi;
      const int th0 = (rem / tw_n) * TH, tw0 = (rem - (rem / tw_n) * tw_n) * TW;
      _Float16* __restrict__ out = (_Float16*)a.out;
      _Float16* __restrict__ out2 = (_Float16*)a.out2;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const int mb = wm * WTM + tm * 16;
        const size_t pix = (((size_t)img * H + th0 + mb / TW) * W + tw0 + mb % TW + o) * Cout;
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
          const int co = n0 + wn * WTN + tn * 16 + q * 4;
          half4 v1, v2;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v1[j] = (_Float16)fmaxf(acc[tm][tn][j] + b1[tn][j], 0.f);
            v2[j] = (_Float16)(accd[tm][tn][j] + b2[tn][j]);
          }
          *reinterpret_cast<half4*>(out + pix + co) = v1;
          *reinterpret_cast<half4*>(out2 + pix + co) = v2;
          acc[tm][tn] = f32x4{0.f, 0.f, 0.f, 0.f};
          accd[tm][tn] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    }

    __syncthreads();  // every wave is done with this unit's LDS
    store_patch();
    if constexpr (NCB > 1) {
      store_w(rw);
      store_d(rd);
    }
    __syncthreads();
    cb = ncb;
    tile = ntile;
  }
}

static int s2p_num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

template <int TH, int TW, int BN, int WM, int WN, int CIN>
static int run_s2p(const ConvS2Args& a, hipStream_t s) {
  PA_CHECK(a.Cin == CIN, "s2p conv: Cin %d != %d", a.Cin, CIN);
  PA_CHECK(a.Hin == 2 * a.Hout && a.Win == 2 * a.Wout, "s2p conv: %dx%d -> %dx%d", a.Hin, a.Win, a.Hout, a.Wout);
  PA_CHECK(a.Hout % TH == 0 && a.Wout % TW == 0, "s2p conv: %dx%d not tiled by %dx%d", a.Hout, a.Wout, TH, TW);
  PA_CHECK(a.Cout % BN == 0, "s2p conv: Cout %d %% BN %d", a.Cout, BN);
  const int ntn = a.Cout / BN;
  const int tiles = a.B * (a.Hout / TH) * (a.Wout / TW) * ntn;
  int grid = s2p_num_cus() / ntn * ntn;  // a multiple of the N-tile count: fixed channels per workgroup
  if (grid > tiles) grid = tiles;
  hipLaunchKernelGGL((conv3x3s2_ds_p<TH, TW, BN, WM, WN, CIN>), dim3(grid), dim3(WM * WN * 64), 0, s, a, tiles);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

int launch_conv3x3s2_ds_p(const ConvS2Args& a, int variant, hipStream_t s) {
  if (a.B <= 0) return PA_OK;
  if (a.Hout == 32) {
    switch (variant) {
      case 1: return run_s2p<8, 16, 64, 2, 2, 64>(a, s);
      default: return run_s2p<8, 16, 64, 4, 1, 64>(a, s);
    }
  }
  if (a.Hout == 16) {
    switch (variant) {
      case 1: return run_s2p<8, 16, 64, 2, 2, 128>(a, s);
      default: return run_s2p<8, 16, 64, 4, 1, 128>(a, s);
    }
  }
  set_error("s2p conv: no configuration for %dx%d", a.Hout, a.Wout);
  return PA_EINVAL;
}

}  // namespace pa
