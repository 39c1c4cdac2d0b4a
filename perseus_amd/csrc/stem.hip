// Fused RGBD stem for the fp16 path: conv 7x7 s2 p3 (Cin <= 4 -> 64) + folded BN
// + ReLU + max-pool 3x3 s2 p1, reading the caller's f32 NCHW frames directly and
// writing only the pooled fp16 NHWC map (torchvision resnet18 stem behind
// perseus/detector/models.py:27-28,34-40).  The 128x128x64 conv map never
// touches HBM.
//
// Workgroup = one image x PB pooled rows (all 64 columns, 64 channels).  Conv
// rows are produced in pairs from a 16-row ring of input rows in LDS (f32->fp16
// converted on the way in, 4 channels interleaved per pixel); each pair needs 9
// input rows and brings in 4 new ones, prefetched into registers while the
// MFMAs of the current pair run.  Conv rows (post-ReLU) go to a 3-row LDS ring;
// pooled row p needs conv rows 2p-1, 2p, 2p+1, i.e. the previous pair's second
// row and the current pair.  The band recomputes one halo conv row.
//
// GEMM per pair: M = 256 pixels, N = 64 channels, K = 7 kh x 32 (28 real: 7 kw
// x 4 ch, 4 zero-weight pad) with MFMA A = weights, B = input patch.
#include <type_traits>

#include "conv.h"

namespace pa {

typedef unsigned su32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));

namespace stem {
constexpr int NT = 512;       // 8 waves
constexpr int RING = 16;      // input-row ring
constexpr int PW = 262;       // ring row width in pixels (wi = c - 3)
constexpr int ROWB = PW * 8;  // bytes per ring row (4 x fp16 per pixel)
constexpr int WBYTES = 7 * 64 * 64;       // weights [kh][co][32 halves]
constexpr int CROWB = 128 * 128;          // one conv row: 128 px x 64 ch fp16
constexpr int LDS = RING * ROWB + WBYTES + 3 * CROWB;
constexpr int F[4] = {0, 2, 3, 1};        // 64-B-row chunk swizzle (conflict-free A reads)
}  // namespace stem

__device__ __forceinline__ int stem_wswz(int kh, int co, int chunk) {
  constexpr int F[4] = {0, 2, 3, 1};
  return (kh * 64 + co) * 64 + ((chunk ^ F[(co >> 2) & 3]) << 4);
}
__device__ __forceinline__ int crow_swz(int px, int chunk) { return px * 128 + ((chunk ^ ((px >> 1) & 7)) << 4); }

template <int V>
using stc = std::integral_constant<int, V>;

template <int B, int E, typename F>
__device__ __forceinline__ void stem_for(F&& f) {
  if constexpr (B < E) {
    f(stc<B>{});
    stem_for<B + 1, E>(f);
  }
}

// PBT pooled rows per workgroup; D = input-row prefetch depth in conv-row pairs
// (rows for pair j + D are loaded into registers at pair j and reach the LDS ring
// at the end of pair j + D - 1), so D x 16 KB of input is in flight per CU.
template <int PBT, int D>
__global__ __launch_bounds__(512) void stem_pool_fp16(const float* __restrict__ x, int B, int Cin,
                                                      const _Float16* __restrict__ w, const float* __restrict__ bias,
                                                      _Float16* __restrict__ out) {
  using namespace stem;
  static_assert(RING >= 9 + 4 && D >= 1 && D <= 3, "ring / prefetch depth");
  __shared__ __attribute__((aligned(16))) char smem[LDS];
  char* ring = smem;
  char* wl = smem + RING * ROWB;
  char* crow = wl + WBYTES;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int q = lane >> 4, r16 = lane & 15;
  const int n = blockIdx.y;
  const int p0 = blockIdx.x * PBT;
  const float* xn = x + (size_t)n * Cin * 256 * 256;

  // ---- weights [64][7][32] fp16 (global) -> LDS [kh][co][4 swizzled chunks]
  for (int i = tid; i < 64 * 7 * 4; i += NT) {
    const int co = i / 28, r = i - (i / 28) * 28, kh = r >> 2, ch = r & 3;
    *reinterpret_cast<su32x4*>(wl + stem_wswz(kh, co, ch)) =
        *reinterpret_cast<const su32x4*>(w + (size_t)co * 224 + kh * 32 + ch * 8);
  }

  // ---- 4 input rows per pair: thread t -> row (t >> 7), pixels 4*((t >> 1) & 63)..+3,
  // channels 2*(t & 1), 2*(t & 1) + 1 (two float4 loads, 4 x 4-byte LDS stores)
  const int lr = tid >> 7, lcg = (tid >> 1) & 63, lcp = tid & 1;
  auto load_rows = [&](int hi0, float4* v) __attribute__((always_inline)) {
    const int hi = hi0 + lr;
    const bool ok = (unsigned)hi < 256u;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int ch = 2 * lcp + c;
      v[c] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (ok && ch < Cin) v[c] = *reinterpret_cast<const float4*>(xn + ((size_t)ch * 256 + hi) * 256 + lcg * 4);
    }
  };
  auto store_rows = [&](int hi0, const float4* v) __attribute__((always_inline)) {
    const int slot = (hi0 + lr + 64) & (RING - 1);
    char* row = ring + slot * ROWB + (lcg * 4 + 3) * 8 + lcp * 4;
    const float a0[4] = {v[0].x, v[0].y, v[0].z, v[0].w};
    const float a1[4] = {v[1].x, v[1].y, v[1].z, v[1].w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      half2_t h;
      h.x = (_Float16)a0[k];
      h.y = (_Float16)a1[k];
      *reinterpret_cast<half2_t*>(row + k * 8) = h;
    }
  };
  // zero the 3 left / 3 right pad pixels of every ring row once (never rewritten)
  for (int i = tid; i < RING * 6; i += NT) {
    const int slot = i / 6, k = i - (i / 6) * 6;
    const int px = k < 3 ? k : 256 + k;  // 0,1,2 and 259,260,261
    *reinterpret_cast<uint2*>(ring + slot * ROWB + px * 8) = make_uint2(0, 0);
  }
  // prologue: the 9 input rows of pair 0 (hi = 4*p0 - 7 .. 4*p0 + 1) straight to the ring
  const int hbase = 4 * p0 - 7;
  {
    float4 v[2];
#pragma unroll
    for (int k = 0; k < 9; k += 4) {
      if (lr + k < 9) {
        load_rows(hbase + k, v);
        store_rows(hbase + k, v);
      }
    }
  }
  // register prefetch sets: set (j % D) holds the 4 rows of pair j + D... loaded at pair j
  float4 pf[D][2];
#pragma unroll
  for (int k = 1; k < D; ++k) load_rows(hbase + 9 + 4 * (k - 1), pf[k]);  // pairs 1..D-1: rows needed by pair k
  __syncthreads();

  // wave w: pixels [32w, 32w+32) of the pair (conv row w>>2, cols (w&3)*32..), all 64 channels
  constexpr int TM = 2, TN = 4;
  const int hr = wid >> 2, wo0 = (wid & 3) * 32;
  f32x4 bv[TN];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) bv[tn] = *reinterpret_cast<const f32x4*>(bias + tn * 16 + q * 4);

  stem_for<0, PBT + 1>([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    const int r0 = 2 * p0 - 2 + 2 * j;  // conv rows r0, r0+1
    const int hs = 4 * p0 - 7 + 4 * j;  // first input row of this pair
    // rows of pair j + D (first row hs + 9 + 4 (D - 1)) -> set j % D
    if constexpr (j + D <= PBT) load_rows(hs + 9 + 4 * (D - 1), pf[j % D]);
    f32x4 acc[TM][TN];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kh = 0; kh < 7; ++kh) {
      const int slot = (hs + 2 * hr + kh + 64) & (RING - 1);
      const char* row = ring + slot * ROWB;
      su32x4 fa[TN], fb[TM];
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        fa[tn] = *reinterpret_cast<const su32x4*>(wl + stem_wswz(kh, tn * 16 + r16, q));
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const int wo = wo0 + tm * 16 + r16;
        fb[tm] = *reinterpret_cast<const su32x4*>(row + (2 * wo) * 8 + q * 16);
      }
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, fa[tn]),
                                                               __builtin_bit_cast(half8, fb[tm]), acc[tm][tn], 0, 0, 0);
    }
    __syncthreads();  // (A) pooling of the previous pair has finished reading the conv ring
    // conv rows -> conv ring (fp16, bias + ReLU; rows above the image are 0, which
    // equals max-pool's -inf padding because every window keeps >= 1 real value >= 0)
    {
      const int r = r0 + hr;
      char* cr = crow + ((r + 6) % 3) * CROWB;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const int wo = wo0 + tm * 16 + r16;
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
          half4 h;
#pragma unroll
          for (int e = 0; e < 4; ++e) h[e] = r >= 0 ? (_Float16)fmaxf(acc[tm][tn][e] + bv[tn][e], 0.f) : (_Float16)0.f;
          const int c = tn * 16 + q * 4;
          *reinterpret_cast<half4*>(cr + crow_swz(wo, c >> 3) + (c & 7) * 2) = h;
        }
      }
    }
    // rows of pair j + 1 (loaded at pair j + 1 - D into set (j + 1) % D) -> ring
    if constexpr (j < PBT) store_rows(hs + 9, pf[(j + 1) % D]);
    __syncthreads();  // (B) conv rows + next input rows visible
    if constexpr (j >= 1) {
      // pooled row p = p0 + j - 1 from conv rows 2p-1, 2p, 2p+1 (= r0-1, r0, r0+1)
      const int p = p0 + j - 1;
      const int qc = tid >> 3, c8 = tid & 7;
      float m[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) m[e] = 0.f;
#pragma unroll
      for (int dr = -1; dr <= 1; ++dr) {
        const char* cr = crow + ((2 * p + dr + 6) % 3) * CROWB;
#pragma unroll
        for (int dc = -1; dc <= 1; ++dc) {
          const int wc = 2 * qc + dc;
          if (wc < 0) continue;
          half8 h = *reinterpret_cast<const half8*>(cr + crow_swz(wc, c8));
#pragma unroll
          for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], (float)h[e]);
        }
      }
      half8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (_Float16)m[e];
      *reinterpret_cast<half8*>(out + (((size_t)n * 64 + p) * 64 + qc) * 64 + c8 * 8) = o;
    }
  });
}

// Version 2: one LDS barrier per conv-row pair.  Pooling is delayed by one pair
// (pooled row p0 + j - 2 at pair j, from a 5-row conv ring), so a pair's MFMAs,
// the pooling of an older row, the conv-row writes and the input-row stores all
// fall between the same two barriers; waves 0-3 run MFMAs first and pooling
// second, waves 4-7 (their SIMD partners) the other way round, so one wave's
// MFMAs overlap its partner's VALU/LDS work.  The barrier orders LDS only
// (lds_barrier), so the D-deep global prefetch stays in flight across it.
// Pooling takes packed fp16 maxima (exact: max of fp16 values is an fp16 value).
namespace stem2 {
constexpr int NCR = 5;  // conv-row ring
constexpr int LDS = stem::RING * stem::ROWB + stem::WBYTES + NCR * stem::CROWB;
}  // namespace stem2

template <int PBT, int D>
__global__ __launch_bounds__(512) void stem_pool2_fp16(const float* __restrict__ x, int B, int Cin,
                                                       const _Float16* __restrict__ w, const float* __restrict__ bias,
                                                       _Float16* __restrict__ out) {
  using namespace stem;
  static_assert(RING >= 9 + 4 && D >= 2 && D <= 3, "ring / prefetch depth");
  __shared__ __attribute__((aligned(16))) char smem[stem2::LDS];
  char* ring = smem;
  char* wl = smem + RING * ROWB;
  char* crow = wl + WBYTES;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int q = lane >> 4, r16 = lane & 15;
  const int n = blockIdx.y;
  const int p0 = blockIdx.x * PBT;
  const float* xn = x + (size_t)n * Cin * 256 * 256;

  for (int i = tid; i < 64 * 7 * 4; i += NT) {
    const int co = i / 28, r = i - (i / 28) * 28, kh = r >> 2, ch = r & 3;
    *reinterpret_cast<su32x4*>(wl + stem_wswz(kh, co, ch)) =
        *reinterpret_cast<const su32x4*>(w + (size_t)co * 224 + kh * 32 + ch * 8);
  }
  const int lr = tid >> 7, lcg = (tid >> 1) & 63, lcp = tid & 1;
  // unconditional loads from clamped addresses (no branch, no early register write
  // that would make the compiler wait on the prefetch); out-of-image rows and absent
  // channels are zeroed when the rows are stored to the ring
  auto load_rows = [&](int hi0, float4* v) __attribute__((always_inline)) {
    const int hi = min(max(hi0 + lr, 0), 255);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int ch = min(2 * lcp + c, Cin - 1);
      v[c] = *reinterpret_cast<const float4*>(xn + ((size_t)ch * 256 + hi) * 256 + lcg * 4);
    }
  };
  auto store_rows = [&](int hi0, const float4* v) __attribute__((always_inline)) {
    const int slot = (hi0 + lr + 64) & (RING - 1);
    char* row = ring + slot * ROWB + (lcg * 4 + 3) * 8 + lcp * 4;
    const bool rok = (unsigned)(hi0 + lr) < 256u;
    const float m0 = (rok && 2 * lcp < Cin) ? 1.f : 0.f, m1 = (rok && 2 * lcp + 1 < Cin) ? 1.f : 0.f;
    const float a0[4] = {v[0].x * m0, v[0].y * m0, v[0].z * m0, v[0].w * m0};
    const float a1[4] = {v[1].x * m1, v[1].y * m1, v[1].z * m1, v[1].w * m1};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      half2_t h;
      h.x = (_Float16)a0[k];
      h.y = (_Float16)a1[k];
      *reinterpret_cast<half2_t*>(row + k * 8) = h;
    }
  };
  for (int i = tid; i < RING * 6; i += NT) {
    const int slot = i / 6, k = i - (i / 6) * 6;
    const int px = k < 3 ? k : 256 + k;
    *reinterpret_cast<uint2*>(ring + slot * ROWB + px * 8) = make_uint2(0, 0);
  }
  const int hbase = 4 * p0 - 7;
  {
    float4 v[2];
#pragma unroll
    for (int k = 0; k < 9; k += 4) {
      if (lr + k < 9) {
        load_rows(hbase + k, v);
        store_rows(hbase + k, v);
      }
    }
  }
  float4 pf[D][2];
#pragma unroll
  for (int k = 1; k < D; ++k) load_rows(hbase + 9 + 4 * (k - 1), pf[k]);
  __syncthreads();

  constexpr int TM = 2, TN = 4;
  const int hr = wid >> 2, wo0 = (wid & 3) * 32;
  f32x4 bv[TN];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) bv[tn] = *reinterpret_cast<const f32x4*>(bias + tn * 16 + q * 4);
  const bool mfma_first = wid < 4;
  const int qc = tid >> 3, c8 = tid & 7;

  stem_for<0, PBT + 2>([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    const int r0 = 2 * p0 - 2 + 2 * j;  // conv rows r0, r0 + 1 (pair j)
    const int hs = 4 * p0 - 7 + 4 * j;  // first input row of pair j
    if constexpr (j + D <= PBT) load_rows(hs + 9 + 4 * (D - 1), pf[j % D]);
    f32x4 acc[TM][TN];
    auto conv = [&]() __attribute__((always_inline)) {
      if constexpr (j <= PBT) {
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kh = 0; kh < 7; ++kh) {
          const int slot = (hs + 2 * hr + kh + 64) & (RING - 1);
          const char* row = ring + slot * ROWB;
          su32x4 fa[TN], fb[TM];
#pragma unroll
          for (int tn = 0; tn < TN; ++tn) fa[tn] = *reinterpret_cast<const su32x4*>(wl + stem_wswz(kh, tn * 16 + r16, q));
#pragma unroll
          for (int tm = 0; tm < TM; ++tm)
            fb[tm] = *reinterpret_cast<const su32x4*>(row + (2 * (wo0 + tm * 16 + r16)) * 8 + q * 16);
#pragma unroll
          for (int tm = 0; tm < TM; ++tm)
#pragma unroll
            for (int tn = 0; tn < TN; ++tn)
              acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, fa[tn]),
                                                                   __builtin_bit_cast(half8, fb[tm]), acc[tm][tn], 0, 0,
                                                                   0);
        }
      }
    };
    auto pool = [&]() __attribute__((always_inline)) {
      if constexpr (j >= 2) {
        // pooled row p = p0 + j - 2 from conv rows 2p-1, 2p, 2p+1 (= r0-3, r0-2, r0-1)
        const int p = p0 + j - 2;
        half8 m = half8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int dr = -1; dr <= 1; ++dr) {
          const char* cr = crow + ((2 * p + dr + 10) % stem2::NCR) * CROWB;
#pragma unroll
          for (int dc = -1; dc <= 1; ++dc) {
            const int wc = 2 * qc + dc;
            if (dc < 0 && qc == 0) continue;
            m = __builtin_elementwise_max(m, *reinterpret_cast<const half8*>(cr + crow_swz(wc, c8)));
          }
        }
        *reinterpret_cast<half8*>(out + (((size_t)n * 64 + p) * 64 + qc) * 64 + c8 * 8) = m;
      }
    };
    if (mfma_first) {
      conv();
      pool();
    } else {
      pool();
      conv();
    }
    if constexpr (j <= PBT) {
      // conv row -> ring (fp16, bias + ReLU; rows above the image are 0, which equals
      // max-pool's -inf padding since every window keeps >= 1 real value >= 0)
      const int r = r0 + hr;
      char* cr = crow + ((r + 10) % stem2::NCR) * CROWB;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const int wo = wo0 + tm * 16 + r16;
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
          half4 h;
#pragma unroll
          for (int e = 0; e < 4; ++e) h[e] = r >= 0 ? (_Float16)fmaxf(acc[tm][tn][e] + bv[tn][e], 0.f) : (_Float16)0.f;
          const int c = tn * 16 + q * 4;
          *reinterpret_cast<half4*>(cr + crow_swz(wo, c >> 3) + (c & 7) * 2) = h;
        }
      }
    }
    if constexpr (j < PBT) store_rows(hs + 9, pf[(j + 1) % D]);
    if constexpr (j <= PBT) lds_barrier();
  });
}

// Version 3: weights in VGPRs, vertical pooling in registers.  Wave w owns conv
// columns [16w, 16w + 16) of BOTH rows of every pair (2p, 2p + 1), so it forms the
// vertical max V_p = max(row 2p-1, row 2p, row 2p+1) in registers, keeping row
// 2p + 1 for the next pair.  Only V_p (one 128 x 64 row) goes to LDS (2-slot
// ring) and the pooled row is the horizontal max of 3 V pixels.  The A operand
// (all 7 kh x 64 channels, 112 VGPRs per lane) is loaded once, so the MFMA phase
// reads only the input fragments from LDS.  One LDS-only barrier per pair; waves
// 0-3 do MFMAs then pooling, waves 4-7 the other order (SIMD partners overlap).
template <int PBT, int D, bool WT = false>
__global__ __launch_bounds__(512) void stem_pool3_fp16(const float* __restrict__ x, int B, int Cin,
                                                       const _Float16* __restrict__ w, const float* __restrict__ bias,
                                                       _Float16* __restrict__ out) {
  using namespace stem;
  static_assert(RING >= 9 + 4 && D >= 2 && D <= 3, "ring / prefetch depth");
  __shared__ __attribute__((aligned(16))) char smem[RING * ROWB + 2 * CROWB + 64 * 4];
  char* ring = smem;
  char* vring = smem + RING * ROWB;
  float* bl = reinterpret_cast<float*>(vring + 2 * CROWB);  // bias (re-read per pair: VGPRs are full)

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int q = lane >> 4, r16 = lane & 15;
  const int n = blockIdx.y;
  const int p0 = blockIdx.x * PBT;
  const float* xn = x + (size_t)n * Cin * 256 * 256;

  const int lr = tid >> 7, lcg = (tid >> 1) & 63, lcp = tid & 1;
  auto load_rows = [&](int hi0, float4* v) __attribute__((always_inline)) {
    const int hi = min(max(hi0 + lr, 0), 255);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int ch = min(2 * lcp + c, Cin - 1);
      v[c] = *reinterpret_cast<const float4*>(xn + ((size_t)ch * 256 + hi) * 256 + lcg * 4);
    }
  };
  auto store_rows = [&](int hi0, const float4* v) __attribute__((always_inline)) {
    const int slot = (hi0 + lr + 64) & (RING - 1);
    char* row = ring + slot * ROWB + (lcg * 4 + 3) * 8 + lcp * 4;
    const bool rok = (unsigned)(hi0 + lr) < 256u;
    const float m0 = (rok && 2 * lcp < Cin) ? 1.f : 0.f, m1 = (rok && 2 * lcp + 1 < Cin) ? 1.f : 0.f;
    const float a0[4] = {v[0].x * m0, v[0].y * m0, v[0].z * m0, v[0].w * m0};
    const float a1[4] = {v[1].x * m1, v[1].y * m1, v[1].z * m1, v[1].w * m1};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      half2_t h;
      h.x = (_Float16)a0[k];
      h.y = (_Float16)a1[k];
      *reinterpret_cast<half2_t*>(row + k * 8) = h;
    }
  };
  for (int i = tid; i < RING * 6; i += NT) {
    const int slot = i / 6, k = i - (i / 6) * 6;
    const int px = k < 3 ? k : 256 + k;
    *reinterpret_cast<uint2*>(ring + slot * ROWB + px * 8) = make_uint2(0, 0);
  }
  constexpr int TN = 4;
  // A fragments: output channel tn * 16 + r16, k = kh * 32 + 8 q .. + 7
  su32x4 wf[7][TN];
#pragma unroll
  for (int kh = 0; kh < 7; ++kh)
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
      wf[kh][tn] = *reinterpret_cast<const su32x4*>(w + (size_t)(tn * 16 + r16) * 224 + kh * 32 + q * 8);
  if (tid < 64) bl[tid] = bias[tid];

  const int hbase = 4 * p0 - 7;
  {
    float4 v[2];
#pragma unroll
    for (int k = 0; k < 9; k += 4) {
      if (lr + k < 9) {
        load_rows(hbase + k, v);
        store_rows(hbase + k, v);
      }
    }
  }
  float4 pf[D][2];
#pragma unroll
  for (int k = 1; k < D; ++k) load_rows(hbase + 9 + 4 * (k - 1), pf[k]);
  __syncthreads();

  const int wo = wid * 16 + r16;  // this lane's conv column
  const bool mfma_first = wid < 4;
  const int qc = tid >> 3, c8 = tid & 7;
  half4 prev[TN];  // post-ReLU conv row 2p - 1 (this lane's column, 4 channels per tile)

  stem_for<0, PBT + 2>([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    const int r0 = 2 * p0 - 2 + 2 * j;  // pair j: conv rows r0 = 2p, r0 + 1 (p = p0 - 1 + j)
    const int hs = 4 * p0 - 7 + 4 * j;
    if constexpr (j + D <= PBT) load_rows(hs + 9 + 4 * (D - 1), pf[j % D]);
    f32x4 acc[2][TN];
    auto conv = [&]() __attribute__((always_inline)) {
      if constexpr (j <= PBT) {
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b) acc[a][b] = *reinterpret_cast<const f32x4*>(bl + b * 16 + q * 4);
#pragma unroll
        for (int kh = 0; kh < 7; ++kh) {
          su32x4 fb[2];
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            const int slot = (hs + 2 * t + kh + 64) & (RING - 1);
            fb[t] = *reinterpret_cast<const su32x4*>(ring + slot * ROWB + (2 * wo) * 8 + q * 16);
          }
#pragma unroll
          for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int tn = 0; tn < TN; ++tn)
              acc[t][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, wf[kh][tn]),
                                                                  __builtin_bit_cast(half8, fb[t]), acc[t][tn], 0, 0, 0);
        }
      }
    };
    auto pool = [&]() __attribute__((always_inline)) {
      if constexpr (j >= 2) {
        const int p = p0 + j - 2;
        const char* vr = vring + ((j - 1) & 1) * CROWB;
        half8 m = *reinterpret_cast<const half8*>(vr + crow_swz(2 * qc, c8));
        m = __builtin_elementwise_max(m, *reinterpret_cast<const half8*>(vr + crow_swz(2 * qc + 1, c8)));
        if (qc > 0) m = __builtin_elementwise_max(m, *reinterpret_cast<const half8*>(vr + crow_swz(2 * qc - 1, c8)));
        store16<WT>(out, (unsigned)(((((size_t)n * 64 + p) * 64 + qc) * 64 + c8 * 8) * 2), m);
      }
    };
    if (mfma_first) {
      conv();
      pool();
    } else {
      pool();
      conv();
    }
    if constexpr (j <= PBT) {
      // rows above the image (only the whole pair r0 = -2, -1) are 0 = max-pool's
      // -inf padding, since every window keeps >= 1 real post-ReLU value
      const half4 z4 = half4{0, 0, 0, 0};
      half4 v0[TN], v1[TN];
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v0[tn][e] = (_Float16)acc[0][tn][e];
          v1[tn][e] = (_Float16)acc[1][tn][e];
        }
        v0[tn] = __builtin_elementwise_max(v0[tn], z4);
        v1[tn] = __builtin_elementwise_max(v1[tn], z4);
      }
      if (r0 < 0) {
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) v1[tn] = z4;
      }
      if constexpr (j >= 1) {
        char* vw = vring + (j & 1) * CROWB;
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
          const half4 vv = __builtin_elementwise_max(prev[tn], __builtin_elementwise_max(v0[tn], v1[tn]));
          const int c = tn * 16 + q * 4;
          *reinterpret_cast<half4*>(vw + crow_swz(wo, c >> 3) + (c & 7) * 2) = vv;
        }
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) prev[tn] = v1[tn];
    }
    if constexpr (j < PBT) store_rows(hs + 9, pf[(j + 1) % D]);
    if constexpr (j <= PBT) lds_barrier();
  });
}

template <int PBT, int D>
static int run_stem(const float* x, int B, int Cin, const _Float16* w, const float* bias, _Float16* out,
                    hipStream_t s) {
  hipLaunchKernelGGL((stem_pool_fp16<PBT, D>), dim3(64 / PBT, B), dim3(stem::NT), 0, s, x, B, Cin, w, bias, out);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

template <int PBT, int D, bool WT = false>
static int run_stem3(const float* x, int B, int Cin, const _Float16* w, const float* bias, _Float16* out,
                     hipStream_t s) {
  PA_CHECK(!WT || (size_t)B * 64 * 64 * 64 * 2 < 0x7fffffffu, "stem: output over 2 GB");
  hipLaunchKernelGGL((stem_pool3_fp16<PBT, D, WT>), dim3(64 / PBT, B), dim3(stem::NT), 0, s, x, B, Cin, w, bias, out);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

template <int PBT, int D>
static int run_stem2(const float* x, int B, int Cin, const _Float16* w, const float* bias, _Float16* out,
                     hipStream_t s) {
  hipLaunchKernelGGL((stem_pool2_fp16<PBT, D>), dim3(64 / PBT, B), dim3(stem::NT), 0, s, x, B, Cin, w, bias, out);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

int launch_stem_pool_fp16(const float* x, int B, int Cin, const _Float16* w, const float* bias, _Float16* out,
                          hipStream_t s) {
  PA_CHECK(Cin >= 1 && Cin <= 4, "stem: Cin %d", Cin);
  if (B <= 0) return PA_OK;
  switch (g_variant[0]) {
    case 1: return run_stem<8, 1>(x, B, Cin, w, bias, out, s);
    case 2: return run_stem<8, 3>(x, B, Cin, w, bias, out, s);
    case 3: return run_stem<16, 2>(x, B, Cin, w, bias, out, s);
    case 4: return run_stem<32, 3>(x, B, Cin, w, bias, out, s);
    case 5: return run_stem<16, 3>(x, B, Cin, w, bias, out, s);
    case 6: return run_stem2<8, 3>(x, B, Cin, w, bias, out, s);
    case 7: return run_stem2<32, 3>(x, B, Cin, w, bias, out, s);
    case 8: return run_stem2<16, 2>(x, B, Cin, w, bias, out, s);
    case 9: return run_stem2<16, 3>(x, B, Cin, w, bias, out, s);
    case 10: return run_stem3<8, 3>(x, B, Cin, w, bias, out, s);
    case 11: return run_stem3<16, 3>(x, B, Cin, w, bias, out, s);
    case 12: return run_stem3<32, 3>(x, B, Cin, w, bias, out, s);
    case 13: return run_stem3<16, 2, false>(x, B, Cin, w, bias, out, s);  // plain (write-back) stores
    default: return run_stem3<16, 2, true>(x, B, Cin, w, bias, out, s);
  }
}

}  // namespace pa
