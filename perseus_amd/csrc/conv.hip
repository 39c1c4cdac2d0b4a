// Detector kernels for gfx950 (MI355X): implicit-GEMM convolutions on MFMA with
// LDS-staged NHWC tiles, the RGBD stem, max-pool, and the avgpool+fc head.
//
// Replaces the ATen/cuDNN/MIOpen kernels behind torchvision resnet18 as used by
// KeypointCNN (perseus/detector/models.py:20-40).  GEMM view of a convolution:
//   M = B*Hout*Wout output pixels, N = Cout, K = KS*KS*Cin,
//   A[m][k] = in[n][ho*S-P+kr][wo*S-P+ks][c]  (zero outside the image),
//   B[k][co] = W'[co][kr][ks][c]  (BatchNorm folded on the host),
// k ordered (kr, ks, c) so that one K-step = one filter tap x 128 bytes of
// channels = one contiguous 128-byte NHWC segment per output pixel.
#include <type_traits>

#include "conv.h"

namespace pa {

// ---------------------------------------------------------------- helpers
// LDS image of a tile: rows of 128 B (one K-step), 8 chunks of 16 B; chunk c
// of row r lives at chunk slot c ^ ((r >> 1) & 7).  A 16x16x32 (f16) or
// 16x16x4 (f32) fragment read has 16 consecutive rows x one chunk per 16-lane
// group, which this XOR spreads over all 16 bank slots of a 256-B bank row for
// every ds_read_b128 lane group.
__device__ __forceinline__ int swz(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }

template <typename T>
struct Elem;
template <>
struct Elem<_Float16> {
  static constexpr int KB = 64;  // elements per 128-B K-step
};
template <>
struct Elem<float> {
  static constexpr int KB = 32;
};

// One 16-byte K-chunk per lane: lane l holds A[row l&15][chunk l>>4] and
// B[k][col l&15] for the same k range.
template <typename T>
__device__ __forceinline__ void mma16(f32x4& acc, const uint4& a, const uint4& b);

template <>
__device__ __forceinline__ void mma16<_Float16>(f32x4& acc, const uint4& a, const uint4& b) {
  half8 ha = __builtin_bit_cast(half8, a);
  half8 hb = __builtin_bit_cast(half8, b);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ha, hb, acc, 0, 0, 0);
}

template <>
__device__ __forceinline__ void mma16<float>(f32x4& acc, const uint4& a, const uint4& b) {
  // The 16 B per lane hold k = 4q..4q+3 (q = lane>>4); MFMA step j consumes
  // element j of every lane, i.e. k = 4q + j.  A and B use the same permutation
  // of k, so the sum over k is unchanged.
  f32x4 fa = __builtin_bit_cast(f32x4, a);
  f32x4 fb = __builtin_bit_cast(f32x4, b);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[0], fb[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[1], fb[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[2], fb[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[3], fb[3], acc, 0, 0, 0);
}

// 8 consecutive elements <-> f32
__device__ __forceinline__ void load8(const _Float16* p, float* v) {
  half8 h = *reinterpret_cast<const half8*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (float)h[i];
}
__device__ __forceinline__ void load8(const float* p, float* v) {
  f32x4 a = *reinterpret_cast<const f32x4*>(p);
  f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] = a[i];
    v[4 + i] = b[i];
  }
}
__device__ __forceinline__ void store8(_Float16* p, const float* v) {
  half8 h;
#pragma unroll
  for (int i = 0; i < 8; ++i) h[i] = (_Float16)v[i];
  *reinterpret_cast<half8*>(p) = h;
}
__device__ __forceinline__ void store8(float* p, const float* v) {
  f32x4 a, b;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a[i] = v[i];
    b[i] = v[4 + i];
  }
  *reinterpret_cast<f32x4*>(p) = a;
  *reinterpret_cast<f32x4*>(p + 4) = b;
}

// ----------------------------------------------------- implicit-GEMM conv
// 256 threads = 4 waves in a 2x2 grid; wave tile (BM/2) x (BN/2) of 16x16
// MFMA tiles.  Register-staged double buffer: the global loads of K-step t+1
// are issued before the MFMAs of step t and written to the other LDS buffer
// after them; one barrier per K-step.  Epilogue through LDS (f32) so that the
// NHWC stores, the residual loads and the bias are 16-B coalesced.
template <typename T, int BM, int BN, int KS>
__global__ __launch_bounds__(256) void conv_igemm(ConvArgs a) {
  constexpr int KB = Elem<T>::KB;
  constexpr int CPR = 16 / sizeof(T);
  constexpr int TM = BM / 32, TN = BN / 32;
  constexpr int AR = BM / 32, BR = BN / 32;
  constexpr int LDS_AB = 2 * (BM + BN) * 128;
  constexpr int CST = BN + 4;
  constexpr int LDS_C = BM * CST * 4;
  constexpr int LDS = LDS_AB > LDS_C ? LDS_AB : LDS_C;
  __shared__ __attribute__((aligned(16))) char smem[LDS];
  char* As = smem;
  char* Bs = smem + 2 * BM * 128;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const T* __restrict__ in = (const T*)a.in;
  const T* __restrict__ w = (const T*)a.w;
  const int Cin = a.Cin, Hin = a.Hin, Win = a.Win;
  const int Ktot = KS * KS * Cin;
  const int cblocks = Cin / KB;
  const int nk = KS * KS * cblocks;
  const int HWo = a.Hout * a.Wout;

  const int srow = tid >> 3, schunk = tid & 7;
  int a_base[AR], a_hi[AR], a_wi[AR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    int m = m0 + srow + 32 * i;
    if (m < a.M) {
      int n = m / HWo;
      int r = m - n * HWo;
      int ho = r / a.Wout;
      int wo = r - ho * a.Wout;
      a_base[i] = n * Hin * Win;
      a_hi[i] = ho * a.stride - a.pad;
      a_wi[i] = wo * a.stride - a.pad;
    } else {
      a_base[i] = 0;
      a_hi[i] = -(1 << 28);
      a_wi[i] = 0;
    }
  }

  uint4 ra[AR], rb[BR];
  auto gload = [&](int kt) {
    int tap = kt / cblocks;
    int cb = kt - tap * cblocks;
    int kr = tap / KS, kc = tap - kr * KS;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      int hi = a_hi[i] + kr, wi = a_wi[i] + kc;
      if ((unsigned)hi < (unsigned)Hin && (unsigned)wi < (unsigned)Win) {
        const T* p = in + (size_t)(a_base[i] + hi * Win + wi) * Cin + cb * KB + schunk * CPR;
        ra[i] = *reinterpret_cast<const uint4*>(p);
      } else {
        ra[i] = make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const T* p = w + (size_t)(n0 + srow + 32 * i) * Ktot + kt * KB + schunk * CPR;
      rb[i] = *reinterpret_cast<const uint4*>(p);
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < AR; ++i) *reinterpret_cast<uint4*>(As + buf * BM * 128 + swz(srow + 32 * i, schunk)) = ra[i];
#pragma unroll
    for (int i = 0; i < BR; ++i) *reinterpret_cast<uint4*>(Bs + buf * BN * 128 + swz(srow + 32 * i, schunk)) = rb[i];
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int q = lane >> 4, r16 = lane & 15;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    const char* Ab = As + buf * BM * 128;
    const char* Bb = Bs + buf * BN * 128;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      uint4 fa[TM], fb[TN];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
        fa[tm] = *reinterpret_cast<const uint4*>(Ab + swz(wr * (BM / 2) + tm * 16 + r16, g * 4 + q));
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        fb[tn] = *reinterpret_cast<const uint4*>(Bb + swz(wc * (BN / 2) + tn * 16 + r16, g * 4 + q));
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) mma16<T>(acc[tm][tn], fa[tm], fb[tn]);
    }
    if (kt + 1 < nk) lstore(buf ^ 1);
    __syncthreads();
  }

  // epilogue: acc + bias -> LDS (f32) -> (+ residual, ReLU) -> 16-B NHWC stores
  float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) {
    const int col = wc * (BN / 2) + tn * 16 + r16;
    const float bv = a.bias[n0 + col];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
      for (int j = 0; j < 4; ++j) Cs[(wr * (BM / 2) + tm * 16 + q * 4 + j) * CST + col] = acc[tm][tn][j] + bv;
  }
  __syncthreads();
  constexpr int C8 = BN / 8;
  const T* __restrict__ res = (const T*)a.res;
  T* __restrict__ out = (T*)a.out;
  for (int idx = tid; idx < BM * C8; idx += 256) {
    const int row = idx / C8, c8 = idx - (idx / C8) * C8;
    const int m = m0 + row;
    if (m >= a.M) continue;
    float v[8];
    const float* cp = Cs + row * CST + c8 * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = cp[i];
    const size_t o = (size_t)m * a.Cout + n0 + c8 * 8;
    if (a.epi & EPI_RES) {
      float r[8];
      load8(res + o, r);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] += r[i];
    }
    if (a.epi & EPI_RELU) {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = fmaxf(v[i], 0.f);
    }
    store8(out + o, v);
  }
}

template <typename T, int BM, int BN, int KS>
static int run_conv(const ConvArgs& a, hipStream_t s) {
  dim3 grid((a.M + BM - 1) / BM, a.Cout / BN);
  hipLaunchKernelGGL((conv_igemm<T, BM, BN, KS>), grid, dim3(256), 0, s, a);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

template <typename T>
int launch_conv(const ConvArgs& a, int ks, hipStream_t s, const char** kname) {
  constexpr int KB = Elem<T>::KB;
  PA_CHECK(a.Cin % KB == 0, "conv: Cin %d not a multiple of %d", a.Cin, KB);
  PA_CHECK(a.Cout % 64 == 0, "conv: Cout %d not a multiple of 64", a.Cout);
  PA_CHECK(ks == 1 || ks == 3, "conv: kernel size %d", ks);
  if (a.M <= 0) return PA_OK;
  // Tile choice: keep >= ~512 workgroups where the layer allows it.
  int bm, bn;
  if (a.Cout == 64) {
    bm = 128;
    bn = 64;
  } else if (a.M >= 65536) {
    bm = 128;
    bn = 128;
  } else if (a.M >= 16384) {
    bm = 64;
    bn = 128;
  } else {
    bm = 64;
    bn = 64;
  }
  if (a.Cout % bn) bn = 64;
  if (kname) {
    *kname =ks == 3 ? (bm == 128 ? (bn == 128 ? "conv3x3_128x128" : "conv3x3_128x64")
                                  : (bn == 128 ? "conv3x3_64x128" : "conv3x3_64x64"))
                     : (bm == 128 ? (bn == 128 ? "conv1x1_128x128" : "conv1x1_128x64")
                                  : (bn == 128 ? "conv1x1_64x128" : "conv1x1_64x64"));
  }
#define PA_DISPATCH(BM_, BN_)                                           \
  if (bm == BM_ && bn == BN_) {                                         \
    return ks == 3 ? run_conv<T, BM_, BN_, 3>(a, s) : run_conv<T, BM_, BN_, 1>(a, s); \
  }
  PA_DISPATCH(128, 64)
  PA_DISPATCH(128, 128)
  PA_DISPATCH(64, 128)
  PA_DISPATCH(64, 64)
#undef PA_DISPATCH
  set_error("conv: no tile for M=%d N=%d", a.M, a.Cout);
  return PA_EINVAL;
}

// --------------------------------------------------------------- RGBD stem
// conv 7x7 s2 p3 (Cin <= 4 -> 64) + folded BN + ReLU, reading the caller's f32
// NCHW frames directly (the NCHW->NHWC + precision conversion is fused into the
// LDS patch load).  One workgroup = one image x 2 output rows x 128 columns
// (M = 256) x 64 channels.  K per filter row kh = 7 taps x 4 channels = 28,
// padded to 32 with zero weights, so K = 7 x 32 = 224 and the A operand of
// (pixel, kh) is the 32 contiguous elements patch[2r+kh][2wo .. 2wo+7][0..3].
constexpr int STEM_PW = 262;  // patch columns: wi = c - 3, c in [0, 262)
constexpr int STEM_PR = 9;    // patch rows:    hi = 2*ho0 - 3 + r
constexpr int STEM_K = 224;

template <typename T>
__global__ __launch_bounds__(256) void stem_kernel(const float* __restrict__ x, int Cin, const T* __restrict__ w,
                                                   const float* __restrict__ bias, T* __restrict__ out) {
  constexpr int WROW = STEM_K * sizeof(T) + 16;  // padded weight row (bytes)
  constexpr int PATCH = STEM_PR * STEM_PW * 4 * sizeof(T);
  constexpr int WB = 64 * WROW;
  constexpr int OST = 64 + 16 / sizeof(T);  // output staging row (elements)
  constexpr int OUTB = 256 * OST * sizeof(T);
  constexpr int LDS = (PATCH + WB) > OUTB ? (PATCH + WB) : OUTB;
  __shared__ __attribute__((aligned(16))) char smem[LDS];
  T* patch = reinterpret_cast<T*>(smem);
  char* wl = smem + PATCH;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int n = blockIdx.y, ho0 = blockIdx.x * 2;
  const int hi0 = 2 * ho0 - 3;
  const float* xn = x + (size_t)n * Cin * 256 * 256;

  // patch load: one thread per (row, col) pixel, 4 channels
  for (int p = tid; p < STEM_PR * STEM_PW; p += 256) {
    const int r = p / STEM_PW, c = p - r * STEM_PW;
    const int hi = hi0 + r, wi = c - 3;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if ((unsigned)hi < 256u && (unsigned)wi < 256u) {
      for (int ch = 0; ch < Cin; ++ch) v[ch] = xn[((size_t)ch * 256 + hi) * 256 + wi];
    }
    T* d = patch + p * 4;
    d[0] = (T)v[0];
    d[1] = (T)v[1];
    d[2] = (T)v[2];
    d[3] = (T)v[3];
  }
  // weights [64][224] -> LDS rows of WROW bytes
  constexpr int WCH = STEM_K * sizeof(T) / 16;  // 16-B chunks per row
  for (int i = tid; i < 64 * WCH; i += 256) {
    const int row = i / WCH, ch = i - row * WCH;
    *reinterpret_cast<uint4*>(wl + row * WROW + ch * 16) =
        *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(w) + (size_t)row * STEM_K * sizeof(T) + ch * 16);
  }
  __syncthreads();

  // wave w: pixels [64w, 64w+64) of the 256 (conv row w>>1, cols (w&1)*64 ..)
  const int q = lane >> 4, r16 = lane & 15;
  const int hr = wid >> 1, wo_base = (wid & 1) * 64;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr int NG = 32 * sizeof(T) / 64;  // 16-B-per-lane groups per kh
#pragma unroll 1
  for (int kh = 0; kh < 7; ++kh) {
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      uint4 fa[4], fb[4];
#pragma unroll
      for (int tm = 0; tm < 4; ++tm) {
        const int wo = wo_base + tm * 16 + r16;
        const char* p = reinterpret_cast<const char*>(patch + ((2 * hr + kh) * STEM_PW + 2 * wo) * 4);
        fa[tm] = *reinterpret_cast<const uint4*>(p + g * 64 + q * 16);
      }
#pragma unroll
      for (int tn = 0; tn < 4; ++tn) {
        const int co = tn * 16 + r16;
        fb[tn] = *reinterpret_cast<const uint4*>(wl + co * WROW + kh * 32 * sizeof(T) + g * 64 + q * 16);
      }
#pragma unroll
      for (int tm = 0; tm < 4; ++tm)
#pragma unroll
        for (int tn = 0; tn < 4; ++tn) mma16<T>(acc[tm][tn], fa[tm], fb[tn]);
    }
  }
  __syncthreads();
  // epilogue: bias + ReLU, stage [256 pixels][64 ch] in LDS, contiguous copy out
  T* ost = reinterpret_cast<T*>(smem);
#pragma unroll
  for (int tn = 0; tn < 4; ++tn) {
    const int co = tn * 16 + r16;
    const float bv = bias[co];
#pragma unroll
    for (int tm = 0; tm < 4; ++tm)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int pix = wid * 64 + tm * 16 + q * 4 + j;
        ost[pix * OST + co] = (T)fmaxf(acc[tm][tn][j] + bv, 0.f);
      }
  }
  __syncthreads();
  // rows ho0, ho0+1 of image n are one contiguous 256*64-element NHWC block
  T* ob = out + ((size_t)n * 128 + ho0) * 128 * 64;
  constexpr int EPC = 16 / sizeof(T);
  for (int i = tid; i < 256 * 64 / EPC; i += 256) {
    const int pix = i / (64 / EPC), c = (i - pix * (64 / EPC)) * EPC;
    *reinterpret_cast<uint4*>(ob + pix * 64 + c) = *reinterpret_cast<const uint4*>(ost + pix * OST + c);
  }
}

template <typename T>
int launch_stem(const float* x, int B, int Cin, const T* w, const float* bias, T* out, hipStream_t s) {
  PA_CHECK(Cin >= 1 && Cin <= 4, "stem: Cin %d", Cin);
  if (B <= 0) return PA_OK;
  hipLaunchKernelGGL(stem_kernel<T>, dim3(64, B), dim3(256), 0, s, x, Cin, w, bias, out);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

// ------------------------------------------------------------ max-pool 3x3 s2 p1
// torchvision stem maxpool (padding = -inf: only in-image taps take part; the
// centre tap is always in the image).  One thread = one output pixel x 8 channels.
template <typename T>
__global__ __launch_bounds__(256) void maxpool_kernel(const T* __restrict__ in, int B, int H, int W, int C,
                                                      T* __restrict__ out) {
  const int Ho = H / 2, Wo = W / 2, C8 = C / 8;
  const long total = (long)B * Ho * Wo * C8;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c8 = (int)(i % C8);
    long p = i / C8;
    const int wo = (int)(p % Wo);
    p /= Wo;
    const int ho = (int)(p % Ho);
    const int n = (int)(p / Ho);
    float m[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) m[k] = -INFINITY;
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy) {
      const int hi = 2 * ho + dy;
      if ((unsigned)hi >= (unsigned)H) continue;
#pragma unroll
      for (int dx = -1; dx <= 1; ++dx) {
        const int wi = 2 * wo + dx;
        if ((unsigned)wi >= (unsigned)W) continue;
        float v[8];
        load8(in + (((size_t)n * H + hi) * W + wi) * C + c8 * 8, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) m[k] = fmaxf(m[k], v[k]);
      }
    }
    store8(out + (((size_t)n * Ho + ho) * Wo + wo) * C + c8 * 8, m);
  }
}

template <typename T>
int launch_maxpool(const T* in, int B, int H, int W, int C, T* out, hipStream_t s) {
  PA_CHECK(C % 8 == 0 && H % 2 == 0 && W % 2 == 0, "maxpool: shape");
  if (B <= 0) return PA_OK;
  const long total = (long)B * (H / 2) * (W / 2) * (C / 8);
  long blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(maxpool_kernel<T>, dim3((unsigned)blocks), dim3(256), 0, s, in, B, H, W, C, out);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

// -------------------------------------------------------- avgpool + fc head
// AdaptiveAvgPool2d((1,1)) + flatten + Linear(512, 2K) (models.py:31-32).
// One workgroup per frame.  Thread t reads 8-channel chunks of pixel group t/64
// (a wave-instruction reads one contiguous pixel row, every thread has HW/4
// independent loads); the 4 group sums are combined in a fixed order through LDS
// (bit-reproducible), then the fc dot products are reduced across the workgroup.
template <typename T>
__global__ __launch_bounds__(256) void head_kernel(const T* __restrict__ in, int HW, int C,
                                                   const float* __restrict__ fcw, const float* __restrict__ fcb,
                                                   int nout, float* __restrict__ y) {
  __shared__ float csum[4][512];
  __shared__ float part[4][32];
  const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const T* p = in + (size_t)n * HW * C;
  const int C8 = C / 8;  // 16-B chunks per pixel (fp16) / 32-B (f32)
  // thread -> (pixel group g = tid / C8, chunk c8 = tid % C8); 256 / C8 pixel groups
  const int groups = 256 / C8;
  const int g = tid / C8, c8 = tid - (tid / C8) * C8;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (g < groups) {
    // HW = 64 for 256x256 inputs: 16 pixels per thread, all loads issued before the adds
    int px = g;
    for (; px + 7 * groups < HW; px += 8 * groups) {
      float v[8][8];
#pragma unroll
      for (int u = 0; u < 8; ++u) load8(p + (size_t)(px + u * groups) * C + c8 * 8, v[u]);
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int e = 0; e < 8; ++e) s[e] += v[u][e];
    }
    for (; px < HW; px += groups) {
      float v[8];
      load8(p + (size_t)px * C + c8 * 8, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += v[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) csum[g][c8 * 8 + e] = s[e];  // fixed order: deterministic
  }
  __syncthreads();
  const float inv = 1.0f / (float)HW;
  const int c = 2 * tid;
  float m0 = 0.f, m1 = 0.f;
  if (c < C) {
    m0 = (csum[0][c] + csum[1][c] + csum[2][c] + csum[3][c]) * inv;
    m1 = (csum[0][c + 1] + csum[1][c + 1] + csum[2][c + 1] + csum[3][c + 1]) * inv;
  }
  for (int j = 0; j < nout; ++j) {
    float v = 0.f;
    if (c < C) v = fmaf(fcw[(size_t)j * C + c + 1], m1, fcw[(size_t)j * C + c] * m0);  // explicit: head_fp16 matches
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (lane == 0) part[wid][j] = v;
  }
  __syncthreads();
  if (tid < nout) y[(size_t)n * nout + tid] = part[0][tid] + part[1][tid] + part[2][tid] + part[3][tid] + fcb[tid];
}

// fp16, HW = 64, C = 512 (the 256x256 forward): head_kernel's arithmetic in the same
// order, with every load (16 pixels per thread, the thread's fc weights) issued
// before the first add.  head_kernel's runtime-length fc loop waits for each
// output's weights in turn (~10 us per batch-64 launch).
// px (optional): the keypoints also denormalized to pixels (postprocess_kernel's
// arithmetic, the streaming tick's output) by the threads that write y
template <int NOUT>
__global__ __launch_bounds__(256) void head_fp16(const _Float16* __restrict__ in, const float* __restrict__ fcw,
                                                 const float* __restrict__ fcb, float* __restrict__ y,
                                                 float* __restrict__ px, int H, int W) {
  constexpr int HW = 64, C = 512;
  __shared__ float csum[4][C];
  __shared__ float part[4][NOUT];
  const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = tid >> 6, c8 = tid & 63;  // pixel group, 16-B channel chunk
  const _Float16* p = in + (size_t)n * HW * C + c8 * 8;
  half8 h[HW / 4];
#pragma unroll
  for (int u = 0; u < HW / 4; ++u) h[u] = *reinterpret_cast<const half8*>(p + (size_t)(g + 4 * u) * C);
  const int c = 2 * tid;
  float fw[NOUT][2];
#pragma unroll
  for (int j = 0; j < NOUT; ++j) {
    const float2 v = *reinterpret_cast<const float2*>(fcw + (size_t)j * C + c);
    fw[j][0] = v.x;
    fw[j][1] = v.y;
  }
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < HW / 4; ++u)
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] += (float)h[u][e];
#pragma unroll
  for (int e = 0; e < 8; ++e) csum[g][c8 * 8 + e] = s[e];
  __syncthreads();
  const float inv = 1.0f / (float)HW;
  const float m0 = (csum[0][c] + csum[1][c] + csum[2][c] + csum[3][c]) * inv;
  const float m1 = (csum[0][c + 1] + csum[1][c + 1] + csum[2][c + 1] + csum[3][c + 1]) * inv;
#pragma unroll
  for (int j = 0; j < NOUT; ++j) {
    float v = fmaf(fw[j][1], m1, fw[j][0] * m0);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (lane == 0) part[wid][j] = v;
  }
  __syncthreads();
  if (tid < NOUT) {
    const float v = part[0][tid] + part[1][tid] + part[2][tid] + part[3][tid] + fcb[tid];
    y[(size_t)n * NOUT + tid] = v;
    if (px) px[(size_t)n * NOUT + tid] = kornia_denorm(v, (tid & 1) ? H : W);
  }
}

// fp16x3 parity mode: head_fp16's arithmetic on the f32 values hi + lo of the layer4
// output's plane pair ([hi (512) | lo (512)] per pixel; hi + lo is exact in f32).
// px (optional): the keypoints also denormalized (postprocess_kernel's arithmetic), as head_fp16
template <int NOUT>
__global__ __launch_bounds__(256) void head_x3(const _Float16* __restrict__ in, const float* __restrict__ fcw,
                                               const float* __restrict__ fcb, float* __restrict__ y,
                                               float* __restrict__ px, int H, int W) {
  constexpr int HW = 64, C = 512;
  __shared__ float csum[4][C];
  __shared__ float part[4][NOUT];
  const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = tid >> 6, c8 = tid & 63;
  const _Float16* p = in + (size_t)n * HW * 2 * C + c8 * 8;
  half8 h[HW / 4], l[HW / 4];
#pragma unroll
  for (int u = 0; u < HW / 4; ++u) {
    h[u] = *reinterpret_cast<const half8*>(p + (size_t)(g + 4 * u) * 2 * C);
    l[u] = *reinterpret_cast<const half8*>(p + (size_t)(g + 4 * u) * 2 * C + C);
  }
  const int c = 2 * tid;
  float fw[NOUT][2];
#pragma unroll
  for (int j = 0; j < NOUT; ++j) {
    const float2 v = *reinterpret_cast<const float2*>(fcw + (size_t)j * C + c);
    fw[j][0] = v.x;
    fw[j][1] = v.y;
  }
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < HW / 4; ++u)
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] += (float)h[u][e] + (float)l[u][e];
#pragma unroll
  for (int e = 0; e < 8; ++e) csum[g][c8 * 8 + e] = s[e];
  __syncthreads();
  const float inv = 1.0f / (float)HW;
  const float m0 = (csum[0][c] + csum[1][c] + csum[2][c] + csum[3][c]) * inv;
  const float m1 = (csum[0][c + 1] + csum[1][c + 1] + csum[2][c + 1] + csum[3][c + 1]) * inv;
#pragma unroll
  for (int j = 0; j < NOUT; ++j) {
    float v = fmaf(fw[j][1], m1, fw[j][0] * m0);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (lane == 0) part[wid][j] = v;
  }
  __syncthreads();
  if (tid < NOUT) {
    const float v = part[0][tid] + part[1][tid] + part[2][tid] + part[3][tid] + fcb[tid];
    y[(size_t)n * NOUT + tid] = v;
    if (px) px[(size_t)n * NOUT + tid] = kornia_denorm(v, (tid & 1) ? H : W);
  }
}

int launch_head_x3(const _Float16* in, int B, int HW, int C, const float* fcw, const float* fcb, int nout, float* y,
                   hipStream_t s, float* px, int H, int W) {
  PA_CHECK(HW == 64 && C == 512 && nout >= 1 && nout <= 32, "head x3: HW=%d C=%d nout=%d", HW, C, nout);
  if (B <= 0) return PA_OK;
  switch (nout) {
#define PA_HX3(N) \
  case N: hipLaunchKernelGGL(head_x3<N>, dim3(B), dim3(256), 0, s, in, fcw, fcb, y, px, H, W); break;
    PA_HX3(2) PA_HX3(4) PA_HX3(6) PA_HX3(8) PA_HX3(10) PA_HX3(12) PA_HX3(14) PA_HX3(16) PA_HX3(18) PA_HX3(20)
    PA_HX3(22) PA_HX3(24) PA_HX3(26) PA_HX3(28) PA_HX3(30) PA_HX3(32)
#undef PA_HX3
    default: PA_CHECK(false, "head x3: nout %d (2 * n_keypoints)", nout);
  }
  PA_LAUNCH_CHECK();
  return PA_OK;
}

template <typename T>
int launch_head(const T* in, int B, int HW, int C, const float* fcw, const float* fcb, int nout, float* y,
                hipStream_t s, float* px, int H, int W) {
  PA_CHECK(C == 512 && nout <= 32, "head: C=%d nout=%d", C, nout);  // 4 pixel groups x 64 chunks
  if (B <= 0) return PA_OK;
  if constexpr (std::is_same<T, _Float16>::value) {
    if (HW == 64 && nout == 16 && g_variant[7] != 1) {  // 1: the generic head_kernel
      hipLaunchKernelGGL(head_fp16<16>, dim3(B), dim3(256), 0, s, in, fcw, fcb, y, px, H, W);
      PA_LAUNCH_CHECK();
      return PA_OK;
    }
  }
  hipLaunchKernelGGL(head_kernel<T>, dim3(B), dim3(256), 0, s, in, HW, C, fcw, fcb, nout, y);
  PA_LAUNCH_CHECK();
  return px ? launch_postprocess(y, nullptr, B, nout / 2, H, W, px, nullptr, s) : PA_OK;
}

// ------------------------------------------------------ pre/post-processing
// scripts/streaming.py:59-82 (ZED frame -> model input) with the val-mode
// near/far clip of augmentations.py:128-169 made deterministic.
__global__ void preprocess_kernel(const uint8_t* __restrict__ rgb, const float* __restrict__ depth, int B, int Hs,
                                  int Ws, int bgr, float near_m, float far_m, int H, int W, float* __restrict__ x) {
  const long total = (long)B * H * W;
  const int r0 = Hs / 2 - H / 2, c0 = Ws / 2 - W / 2;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int wc = (int)(i % W);
    const int hr = (int)((i / W) % H);
    const int n = (int)(i / ((long)H * W));
    const size_t src = ((size_t)n * Hs + (hr + r0)) * Ws + (wc + c0);
    const uint8_t* px = rgb + src * 3;
    float* xo = x + (size_t)n * 4 * H * W + (size_t)hr * W + wc;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int sc = bgr ? 2 - c : c;
      xo[(size_t)c * H * W] = (float)((double)px[sc] / 255.0);  // numpy f64 /255 then .float()
    }
    float d = depth[src];
    if (isnan(d) || isinf(d)) d = 0.f;
    d = d / 0.035f;  // streaming.py:76 (f32 array /= python float)
    if (near_m >= 0.f || far_m >= 0.f) {
      float sd = 0.035f * d;  // DepthPlaneAugmentation: scale, clip, unscale
      if (near_m >= 0.f && sd < near_m) sd = 0.f;
      if (far_m >= 0.f && sd > far_m) sd = 0.f;
      d = sd / 0.035f;
    }
    xo[(size_t)3 * H * W] = d;
  }
}

int launch_preprocess(const uint8_t* rgb, const float* depth, int B, int Hs, int Ws, int bgr, float near_m,
                      float far_m, int H, int W, float* x, hipStream_t s) {
  PA_CHECK(Hs >= H && Ws >= W, "preprocess: source %dx%d smaller than %dx%d", Hs, Ws, H, W);
  if (B <= 0) return PA_OK;
  long total = (long)B * H * W;
  long blocks = (total + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(preprocess_kernel, dim3((unsigned)blocks), dim3(256), 0, s, rgb, depth, B, Hs, Ws, bgr, near_m,
                     far_m, H, W, x);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

// kornia denormalize_pixel_coordinates (validate.py:144-153; kornia_denorm in
// common.h) + SmoothL1(beta=1,
// reduction='none') against normalized targets (validate.py:130-133).
__global__ void postprocess_kernel(const float* __restrict__ y, const float* __restrict__ target, int total, int H,
                                   int W, float* __restrict__ px, float* __restrict__ loss) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const float v = y[i];
  px[i] = kornia_denorm(v, (i & 1) ? H : W);
  if (target) {
    const float d = fabsf(target[i] - v);
    loss[i] = d < 1.0f ? 0.5f * d * d : d - 0.5f;
  }
}

int launch_postprocess(const float* y, const float* target, int B, int n_kp, int H, int W, float* px, float* loss,
                       hipStream_t s) {
  const int total = B * n_kp * 2;
  if (total <= 0) return PA_OK;
  PA_CHECK(!target || loss, "postprocess: loss buffer required with target");
  hipLaunchKernelGGL(postprocess_kernel, dim3((total + 255) / 256), dim3(256), 0, s, y, target, total, H, W, px, loss);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

// explicit instantiations
template int launch_conv<_Float16>(const ConvArgs&, int, hipStream_t, const char**);
template int launch_conv<float>(const ConvArgs&, int, hipStream_t, const char**);
template int launch_stem<_Float16>(const float*, int, int, const _Float16*, const float*, _Float16*, hipStream_t);
template int launch_stem<float>(const float*, int, int, const float*, const float*, float*, hipStream_t);
template int launch_maxpool<_Float16>(const _Float16*, int, int, int, int, _Float16*, hipStream_t);
template int launch_maxpool<float>(const float*, int, int, int, int, float*, hipStream_t);
template int launch_head<_Float16>(const _Float16*, int, int, int, const float*, const float*, int, float*, hipStream_t, float*, int, int);
template int launch_head<float>(const float*, int, int, int, const float*, const float*, int, float*, hipStream_t, float*, int, int);

}  // namespace pa
