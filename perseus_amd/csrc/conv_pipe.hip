// Software-pipelined halo-patch 3x3 stride-1 conv (fp16 / f32), 1 wave per SIMD.
//
// Same data layout and GEMM mapping as conv_patch.hip (LDS input patch reused by
// the 9 taps, weights streamed per (channel block, tap), A = weights, B = pixels,
// register epilogue), restructured so that the MFMA pipe never waits on LDS:
//   * each wave owns a 64 x 64 (pixels x channels) tile = 16 MFMA tiles, so a
//     fragment read feeds 4 MFMAs;
//   * the fragments of step s+1 are read (into a second register set) while the
//     MFMAs of step s run; hence W(s+1) and the patch of step s+1 must already be
//     in LDS when step s starts: W(s+2) is written during step s (2 LDS buffers),
//     the next channel block's patch during tap 7 (2 patch buffers);
//   * weight tiles are register-staged two steps ahead, the next patch for a
//     whole channel block, the residual for the whole last channel block.
// One barrier per step.  Parity-dependent register sets are static because the
// step sequence is unrolled by whole channel-block pairs.
#include <type_traits>

#include "conv.h"

namespace pa {

typedef unsigned p4 __attribute__((ext_vector_type(4)));

template <int V>
using pc = std::integral_constant<int, V>;

template <typename T>
struct QElem;
template <>
struct QElem<_Float16> {
  static constexpr int KB = 64;
};
template <>
struct QElem<float> {
  static constexpr int KB = 32;
};

__device__ __forceinline__ int qswz(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }
__device__ __forceinline__ int qfrag_off(int r) { return r < 4 ? 2 * r : (r < 12 ? 2 * (r - 4) + 1 : 2 * (r - 8)); }

template <typename T>
__device__ __forceinline__ void qmma(f32x4& acc, const p4& a, const p4& b);
template <>
__device__ __forceinline__ void qmma<_Float16>(f32x4& acc, const p4& a, const p4& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, a), __builtin_bit_cast(half8, b), acc, 0, 0,
                                               0);
}
template <>
__device__ __forceinline__ void qmma<float>(f32x4& acc, const p4& a, const p4& b) {
  f32x4 fa = __builtin_bit_cast(f32x4, a), fb = __builtin_bit_cast(f32x4, b);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[0], fb[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[1], fb[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[2], fb[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[3], fb[3], acc, 0, 0, 0);
}

template <typename T>
struct Res4;
template <>
struct Res4<_Float16> {
  typedef half4 type;
};
template <>
struct Res4<float> {
  typedef f32x4 type;
};

// TH x TW x NI output pixels per workgroup, BN channels; WM x WN waves each with a
// (BM/WM) x (BN/WN) tile.
template <typename T, int TH, int TW, int NI, int BN, int WM, int WN, int CIN, int EPI>
__global__ __launch_bounds__(WM* WN * 64) void conv3x3_pipe(ConvArgs a) {
  constexpr int NT = WM * WN * 64;
  constexpr int KB = QElem<T>::KB;
  constexpr int CPR = 16 / sizeof(T);
  constexpr int NCB = CIN / KB;
  constexpr int NSTEPS = NCB * 9;
  constexpr int KTOT = 9 * CIN;
  constexpr int PH = TH + 2, PW = TW + 2;
  constexpr int IMS = (TW == 8) ? ((PH * PW + 7) / 16 * 16 + 8) : PH * PW;
  constexpr int NP = NI * IMS;
  constexpr int BM = NI * TH * TW;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int PCH = (NP * 8 + NT - 1) / NT;
  constexpr int BCH = BN * 8 / NT;
  constexpr int PBUF = NCB > 1 ? 2 : 1;
  constexpr int PATCHB = NP * 128;
  constexpr int WB = BN * 128;
  static_assert(BN * 8 % NT == 0, "weight tile / threads");
  static_assert(TW >= 16 || (TW == 8 && NI == 2), "fragment geometry");
  static_assert(NCB == 1 || NCB % 2 == 0, "channel blocks are processed in pairs");
  __shared__ __attribute__((aligned(16))) char smem[PBUF * PATCHB + 2 * WB];
  char* patch = smem;
  char* wbuf = smem + PBUF * PATCHB;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int q = lane >> 4, r16 = lane & 15;
  const int H = a.Hout, W = a.Wout;
  const int Cout = a.Cout;
  const T* __restrict__ in = (const T*)a.in;
  const T* __restrict__ w = (const T*)a.w;

  const int ntn = Cout / BN;
  const int tn_idx = blockIdx.x % ntn;
  const int sp = blockIdx.x / ntn;
  const int tw_n = W / TW, tpi = (H / TH) * tw_n;
  const int img0 = (sp / tpi) * NI;
  const int rem = sp - (sp / tpi) * tpi;
  const int th0 = (rem / tw_n) * TH, tw0 = (rem - (rem / tw_n) * tw_n) * TW;
  const int n0 = tn_idx * BN;

  // ------------------------------------------------------------ staging
  p4 rp[PCH];
  p4 rb[2][BCH];
  auto load_patch = [&](int cb) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < PCH; ++i) {
      const int c = tid + i * NT;
      p4 v = p4{0u, 0u, 0u, 0u};
      if (c < NP * 8) {
        const int p = c >> 3, ch = c & 7;
        const int img = p / IMS, pp = p - (p / IMS) * IMS;
        const int pr = pp / PW, pcol = pp - (pp / PW) * PW;
        const int n = img0 + img, h = th0 + pr - 1, x = tw0 + pcol - 1;
        if (pr < PH && n < a.B && (unsigned)h < (unsigned)H && (unsigned)x < (unsigned)W)
          v = *reinterpret_cast<const p4*>(in + (((size_t)n * H + h) * W + x) * CIN + cb * KB + ch * CPR);
      }
      rp[i] = v;
    }
  };
  auto store_patch = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < PCH; ++i) {
      const int c = tid + i * NT;
      if (c < NP * 8) *reinterpret_cast<p4*>(patch + buf * PATCHB + qswz(c >> 3, c & 7)) = rp[i];
    }
  };
  auto load_w = [&](int s, auto setc) __attribute__((always_inline)) {
    constexpr int SET = decltype(setc)::value;
    s = s < NSTEPS ? s : NSTEPS - 1;
    const int cb = s / 9, tap = s - (s / 9) * 9;
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int c = tid + i * NT;
      rb[SET][i] = *reinterpret_cast<const p4*>(w + (size_t)(n0 + (c >> 3)) * KTOT + tap * CIN + cb * KB + (c & 7) * CPR);
    }
  };
  auto store_w = [&](int buf, auto setc) __attribute__((always_inline)) {
    constexpr int SET = decltype(setc)::value;
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int c = tid + i * NT;
      *reinterpret_cast<p4*>(wbuf + buf * WB + qswz(c >> 3, c & 7)) = rb[SET][i];
    }
  };

  const int o = qfrag_off(r16);
  int ppix[TM];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int mb = wm * WTM + tm * 16;
    if constexpr (TW == 8) {
      ppix[tm] = (o >> 3) * IMS + (mb / 16) * PW + (o & 7);
    } else {
      ppix[tm] = (mb / (TH * TW)) * IMS + ((mb / TW) % TH) * PW + mb % TW + o;
    }
  }

  // fragment register sets (parity) and accumulators
  p4 fa[2][2][TN], fb[2][2][TM];
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto read_frags = [&](int s, auto parc) __attribute__((always_inline)) {
    constexpr int P = decltype(parc)::value;
    const int cb = s / 9, tap = s - (s / 9) * 9;
    const char* pb = patch + (PBUF == 2 ? (cb & 1) * PATCHB : 0);
    const char* wb = wbuf + (s & 1) * WB;
    const int toff = (tap / 3) * PW + (tap - (tap / 3) * 3);
#pragma unroll
    for (int g = 0; g < 2; ++g) {
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        fa[P][g][tn] = *reinterpret_cast<const p4*>(wb + qswz(wn * WTN + tn * 16 + r16, g * 4 + q));
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
        fb[P][g][tm] = *reinterpret_cast<const p4*>(pb + qswz(ppix[tm] + toff, g * 4 + q));
    }
  };
  auto mfmas = [&](auto parc) __attribute__((always_inline)) {
    constexpr int P = decltype(parc)::value;
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) qmma<T>(acc[tm][tn], fa[P][g][tn], fb[P][g][tm]);
  };

  // residual prefetch (whole last channel block ahead of the epilogue)
  typedef typename Res4<T>::type R4;
  R4 rres[TM][TN];
  const T* __restrict__ res = (const T*)a.res;
  size_t pixo[TM];
  bool ok[TM];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int mb = wm * WTM + tm * 16;
    int img, y, x;
    if constexpr (TW == 8) {
      y = mb / 16;
      img = o >> 3;
      x = o & 7;
    } else {
      img = mb / (TH * TW);
      y = (mb / TW) % TH;
      x = mb % TW + o;
    }
    const int n = img0 + img;
    ok[tm] = n < a.B;
    pixo[tm] = ((((size_t)(ok[tm] ? n : 0)) * H + th0 + y) * W + tw0 + x) * Cout;
  }
  auto load_res = [&]() __attribute__((always_inline)) {
    if constexpr (EPI & EPI_RES) {
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          rres[tm][tn] = *reinterpret_cast<const R4*>(res + pixo[tm] + n0 + wn * WTN + tn * 16 + q * 4);
    }
  };

  // ------------------------------------------------------------ prologue
  load_patch(0);
  load_w(0, pc<0>{});
  load_w(1, pc<1>{});
  store_patch(0);
  store_w(0, pc<0>{});
  store_w(1, pc<1>{});
  load_w(2, pc<0>{});
  load_w(3, pc<1>{});
  __syncthreads();
  read_frags(0, pc<0>{});
  __syncthreads();  // step 0 overwrites LDS W buffer 0 (= W(0)) after every wave has read it

  // ------------------------------------------------------------ main loop
  // step s (parity P): write W(s+2) (set P) -> LDS buf s&1, refill set P with
  // W(s+4); read frags of s+1 into set 1-P while the MFMAs of s run; barrier.
  auto step = [&](int cb, auto tapc, auto parc) __attribute__((always_inline)) {
    constexpr int TAP = decltype(tapc)::value;
    constexpr int P = decltype(parc)::value;
    const int s = cb * 9 + TAP;
    store_w(s & 1, pc<P>{});  // buffer of W(s): its frags were read during step s-1
    load_w(s + 4, pc<P>{});
    if constexpr (TAP == 0 && NCB > 1) load_patch(cb + 1 < NCB ? cb + 1 : NCB - 1);
    if constexpr (TAP == 0) {
      if (cb == NCB - 1) load_res();
    }
    if (s + 1 < NSTEPS) read_frags(s + 1, pc<1 - P>{});
    mfmas(pc<P>{});
    if constexpr (TAP == 7 && NCB > 1) {
      if (cb + 1 < NCB) store_patch((cb + 1) & 1);
    }
    __syncthreads();
  };
  auto cblock = [&](int cb, auto p0c) __attribute__((always_inline)) {
    constexpr int P0 = decltype(p0c)::value;  // parity of step cb*9
    step(cb, pc<0>{}, pc<P0>{});
    step(cb, pc<1>{}, pc<1 - P0>{});
    step(cb, pc<2>{}, pc<P0>{});
    step(cb, pc<3>{}, pc<1 - P0>{});
    step(cb, pc<4>{}, pc<P0>{});
    step(cb, pc<5>{}, pc<1 - P0>{});
    step(cb, pc<6>{}, pc<P0>{});
    step(cb, pc<7>{}, pc<1 - P0>{});
    step(cb, pc<8>{}, pc<P0>{});
  };
  if constexpr (NCB == 1) {
    cblock(0, pc<0>{});
  } else {
    for (int cb = 0; cb < NCB; cb += 2) {
      cblock(cb, pc<0>{});
      cblock(cb + 1, pc<1>{});
    }
  }

  // ------------------------------------------------------------ epilogue
  T* __restrict__ out = (T*)a.out;
  f32x4 bias[TN];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) bias[tn] = *reinterpret_cast<const f32x4*>(a.bias + n0 + wn * WTN + tn * 16 + q * 4);
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    if (!ok[tm]) continue;
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      R4 ov;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v = acc[tm][tn][j] + bias[tn][j];
        if constexpr (EPI & EPI_RES) v += (float)rres[tm][tn][j];
        if constexpr (EPI & EPI_RELU) v = fmaxf(v, 0.f);
        ov[j] = (T)v;
      }
      *reinterpret_cast<R4*>(out + pixo[tm] + n0 + wn * WTN + tn * 16 + q * 4) = ov;
    }
  }
}

template <typename T, int TH, int TW, int NI, int BN, int WM, int WN, int CIN>
static int run_pipe(const ConvArgs& a, hipStream_t s) {
  PA_CHECK(a.Cin == CIN, "pipe conv: Cin %d != %d", a.Cin, CIN);
  PA_CHECK(a.Hout % TH == 0 && a.Wout % TW == 0, "pipe conv: %dx%d not tiled by %dx%d", a.Hout, a.Wout, TH, TW);
  PA_CHECK(a.Cout % BN == 0, "pipe conv: Cout %d %% BN %d", a.Cout, BN);
  PA_CHECK(a.epi == EPI_RELU || a.epi == (EPI_RELU | EPI_RES), "pipe conv: epilogue %d", a.epi);
  const int tiles = ((a.B + NI - 1) / NI) * (a.Hout / TH) * (a.Wout / TW) * (a.Cout / BN);
  if (a.epi & EPI_RES)
    hipLaunchKernelGGL((conv3x3_pipe<T, TH, TW, NI, BN, WM, WN, CIN, EPI_RELU | EPI_RES>), dim3(tiles),
                       dim3(WM * WN * 64), 0, s, a);
  else
    hipLaunchKernelGGL((conv3x3_pipe<T, TH, TW, NI, BN, WM, WN, CIN, EPI_RELU>), dim3(tiles), dim3(WM * WN * 64), 0,
                       s, a);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

// variant dispatch for the pipelined kernel (layer = feature-map stage 1..4)
template <typename T>
int launch_conv3x3_pipe(const ConvArgs& a, int variant, hipStream_t s) {
  if (a.Hout == 64) {
    switch (variant) {
      case 1: return run_pipe<T, 16, 16, 1, 64, 4, 1, 64>(a, s);   // 256 px x 64 ch, 1024 WGs
      default: return run_pipe<T, 8, 16, 1, 64, 2, 1, 64>(a, s);   // 128 px x 64 ch, 2048 WGs
    }
  }
  if (a.Hout == 32) {
    switch (variant) {
      case 1: return run_pipe<T, 8, 16, 1, 128, 2, 2, 128>(a, s);  // 128 px x 128 ch, 512 WGs
      default: return run_pipe<T, 16, 16, 1, 64, 4, 1, 128>(a, s); // 256 px x 64 ch, 512 WGs
    }
  }
  if (a.Hout == 16) {
    switch (variant) {
      case 1: return run_pipe<T, 8, 16, 1, 128, 2, 2, 256>(a, s);  // 512 WGs
      default: return run_pipe<T, 16, 16, 1, 64, 4, 1, 256>(a, s); // 256 WGs
    }
  }
  if (a.Hout == 8) {
    switch (variant) {
      case 1: return run_pipe<T, 8, 8, 2, 32, 2, 1, 512>(a, s);    // 128 px x 32 ch, 512 WGs
      default: return run_pipe<T, 8, 8, 2, 64, 2, 1, 512>(a, s);   // 128 px x 64 ch, 256 WGs
    }
  }
  set_error("pipe conv: no configuration for %dx%d", a.Hout, a.Wout);
  return PA_EINVAL;
}

template int launch_conv3x3_pipe<_Float16>(const ConvArgs&, int, hipStream_t);
template int launch_conv3x3_pipe<float>(const ConvArgs&, int, hipStream_t);

}  // namespace pa
