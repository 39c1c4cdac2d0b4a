// Fused RGBD stem for the fp16 path: conv 7x7 s2 p3 (Cin <= 4 -> 64) + folded BN
// + ReLU + max-pool 3x3 s2 p1, reading the caller's f32 NCHW frames directly and
// writing only the pooled fp16 NHWC map (torchvision resnet18 stem behind
// perseus/detector/models.py:27-28,34-40).  The 128x128x64 conv map never
// touches HBM.
//
// Workgroup = one image x PBT pooled rows (all 64 columns, 64 channels).  Conv
// rows are produced in pairs from a 16-row ring of input rows in LDS (f32->fp16
// converted on the way in, 4 channels interleaved per pixel); each pair needs 9
// input rows and brings in 4 new ones, prefetched D pairs ahead into registers.
// Pooled row p needs conv rows 2p-1, 2p, 2p+1: the previous pair's second row
// and the current pair.  The band recomputes one halo conv pair.
//
// GEMM per pair: M = 256 pixels, N = 64 channels, K = 7 kh x 32 (28 real: 7 kw
// x 4 ch, 4 zero-weight pad) with MFMA A = weights, B = input patch.
// (Versions 1 and 2 -- weights in LDS, conv rows through an LDS ring -- measured
// 59 and 41 us per batch-64 launch against this one's 35; removed.)
#include <type_traits>

#include "conv_gx.h"

namespace pa {

typedef unsigned su32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));

namespace stem {
constexpr int NT = 512;       // 8 waves
constexpr int RING = 16;      // input-row ring
constexpr int PW = 262;       // ring row width in pixels (wi = c - 3)
constexpr int ROWB = PW * 8;  // bytes per ring row (4 x fp16 per pixel)
constexpr int CROWB = 128 * 128;          // one conv row: 128 px x 64 ch fp16
}  // namespace stem

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

// Version 3: weights in VGPRs, vertical pooling in registers.  Wave w owns conv
// columns [16w, 16w + 16) of BOTH rows of every pair (2p, 2p + 1), so it forms the
// vertical max V_p = max(row 2p-1, row 2p, row 2p+1) in registers, keeping row
// 2p + 1 for the next pair.  Only V_p (one 128 x 64 row) goes to LDS (2-slot
// ring) and the pooled row is the horizontal max of 3 V pixels.  The A operand
// (all 7 kh x 64 channels, 112 VGPRs per lane) is loaded once, so the MFMA phase
// reads only the input fragments from LDS.  One LDS-only barrier per pair; waves
// 0-3 do MFMAs then pooling, waves 4-7 the other order (SIMD partners overlap).
// PRE: the input rows come straight from the camera frames (RgbdSrc) through
// preprocess_kernel's arithmetic (conv.hip), so the f32 NCHW frame never exists; the
// values reaching the fp16 ring are the same f32 numbers, hence bit-identical output.
template <int PBT, int D, bool WT = false, int DBG = 0, bool PRE = false>
__global__ __launch_bounds__(512) void stem_pool3_fp16(const float* __restrict__ x, int B, int Cin,
                                                       const _Float16* __restrict__ w, const float* __restrict__ bias,
                                                       _Float16* __restrict__ out, unsigned long long* trace,
                                                       RgbdSrc src) {
  using namespace stem;
  static_assert(RING >= 9 + 4 && D >= 2 && D <= 3, "ring / prefetch depth");
  constexpr int WSTAGE = RING * ROWB + 2 * CROWB + 64 * 4;  // 28 KB weight staging (A fragment order)
  static_assert(WSTAGE % 16 == 0, "staging alignment");
  __shared__ __attribute__((aligned(1024))) char smem[WSTAGE + 28 * 1024];
  if constexpr (DBG == 4) trace_stamp(trace, 0);
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
    if constexpr (PRE) {
      // 4 pixels of row hi, channels 2 lcp and 2 lcp + 1 (R,G or B,depth)
      const int r0 = src.Hs / 2 - 128, c0 = src.Ws / 2 - 128;
      const size_t row = ((size_t)n * src.Hs + hi + r0) * src.Ws + c0 + lcg * 4;
      const int sc0 = lcp ? (src.bgr ? 0 : 2) : (src.bgr ? 2 : 0);  // channel 2 lcp
      constexpr int sc1 = 1;                                        // channel 1 (lcp = 0)
      float a0[4], a1[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint8_t* px = src.rgb + (row + k) * 3;
        a0[k] = (float)((double)px[sc0] / 255.0);  // numpy f64 /255 then .float()
        if (lcp == 0) {
          a1[k] = (float)((double)px[sc1] / 255.0);
        } else {
          float d = src.depth[row + k];
          if (isnan(d) || isinf(d)) d = 0.f;
          d = d / 0.035f;  // streaming.py:76
          if (src.near_m >= 0.f || src.far_m >= 0.f) {
            float sd = 0.035f * d;  // DepthPlaneAugmentation: scale, clip, unscale
            if (src.near_m >= 0.f && sd < src.near_m) sd = 0.f;
            if (src.far_m >= 0.f && sd > src.far_m) sd = 0.f;
            d = sd / 0.035f;
          }
          a1[k] = d;
        }
      }
      v[0] = float4{a0[0], a0[1], a0[2], a0[3]};
      v[1] = float4{a1[0], a1[1], a1[2], a1[3]};
    } else {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int ch = min(2 * lcp + c, Cin - 1);
        v[c] = *reinterpret_cast<const float4*>(xn + ((size_t)ch * 256 + hi) * 256 + lcg * 4);
      }
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
  // prologue, one global round trip: the first 9 input rows, the bias, the weights
  // (A fragments: output channel tn * 16 + r16, k = kh * 32 + 8 q .. + 7) and the
  // first prefetch are all issued before any of them is waited for, the rows first
  // (vmcnt is in order)
  const int hbase = 4 * p0 - 7;
  float4 v0[2], v1[2], v2[2];
  load_rows(hbase, v0);
  load_rows(hbase + 4, v1);
  if (lr == 0) load_rows(hbase + 8, v2);
  float bv = 0.f;
  if (tid < 64) bv = bias[tid];
  // weights: every wave needs all of them (112 VGPRs of A fragments); 8 waves loading
  // 28 KB each through L1 took ~2 us, so the workgroup DMAs them once into LDS in
  // fragment order (block kh * 4 + tn = 64 lanes x 16 B) and each wave reads its copy
  // from there.  These DMAs sit between the row loads and the prefetch loads.
  constexpr int TN = 4;
  char* wst = smem + WSTAGE;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int b = wid + 8 * i;  // block = kh * 4 + tn
    if (b < 28)
      xdma16(w + (size_t)((b & 3) * 16 + r16) * 224 + (b >> 2) * 32 + q * 8, wst + b * 1024);
  }
  float4 pf[D][2];
#pragma unroll
  for (int k = 1; k < D; ++k) load_rows(hbase + 9 + 4 * (k - 1), pf[k]);
  __builtin_amdgcn_sched_barrier(0);
  for (int i = tid; i < RING * 6; i += NT) {
    const int slot = i / 6, k = i - (i / 6) * 6;
    const int px = k < 3 ? k : 256 + k;
    *reinterpret_cast<uint2*>(ring + slot * ROWB + px * 8) = make_uint2(0, 0);
  }
  store_rows(hbase, v0);
  store_rows(hbase + 4, v1);
  if (lr == 0) store_rows(hbase + 8, v2);
  if (tid < 64) bl[tid] = bv;
  xwait_vm<2 * (D - 1)>();  // this wave's weight DMAs (only the prefetch may stay in flight)
  lds_barrier();
  su32x4 wf[7][TN];
#pragma unroll
  for (int kh = 0; kh < 7; ++kh)
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) wf[kh][tn] = *reinterpret_cast<const su32x4*>(wst + (kh * 4 + tn) * 1024 + lane * 16);
  if constexpr (DBG == 4) trace_stamp(trace, 1);

  const int wo = wid * 16 + r16;  // this lane's conv column
  const bool mfma_first = wid < 4;
  const int qc = tid >> 3, c8 = tid & 7;
  half4 prev[TN];  // post-ReLU conv row 2p - 1 (this lane's column, 4 channels per tile)

  stem_for<0, PBT + 2>([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    const int r0 = 2 * p0 - 2 + 2 * j;  // pair j: conv rows r0 = 2p, r0 + 1 (p = p0 - 1 + j)
    const int hs = 4 * p0 - 7 + 4 * j;
    if constexpr (j + D <= PBT && DBG != 3) load_rows(hs + 9 + 4 * (D - 1), pf[j % D]);
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
              if constexpr (DBG != 1)
                acc[t][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, wf[kh][tn]),
                                                                    __builtin_bit_cast(half8, fb[t]), acc[t][tn], 0, 0, 0);
              else
                acc[t][tn][0] += __builtin_bit_cast(f32x4, fb[t])[0];
        }
      }
    };
    auto pool = [&]() __attribute__((always_inline)) {
      if constexpr (j >= 2 && DBG != 2) {
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
      if constexpr (j >= 1 && DBG != 5) {
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
    if constexpr (j < PBT && DBG != 3) store_rows(hs + 9, pf[(j + 1) % D]);
    if constexpr (j <= PBT) lds_barrier();
    if constexpr (DBG == 4) trace_stamp(trace, 2 + j);
  });
  if constexpr (DBG == 4) {
    __builtin_amdgcn_s_waitcnt(0);
    trace_stamp(trace, 63);
  }
}

// Version 4 ("role split"): the same arithmetic as version 3 with the waves split by
// role.  Waves 0-3 (one per SIMD) only convolve: each owns 32 conv columns of both rows
// of a pair (2 x 2 x 4 accumulator tiles, weights in VGPRs, 0.25 LDS reads per MFMA),
// forms the vertical max in registers and writes the V row to LDS.  Waves 4-7 only move
// data: the horizontal max + store of the previous V row, the global loads of the input
// rows D pairs ahead and their fp16 ring stores.  One LDS-only barrier per pair.  In
// version 3 every wave did both halves and the SIMD partners alternated roles; the MFMA
// pipe was busy about half of the launch.  Accumulation order (bias, then kh = 0..6) and
// every rounding step are version 3's, so the pooled map is bit-identical.
// DBG = 4 (timing only): s_memrealtime stamps, 64 per workgroup: slot j = wave 0 (convolving)
// at pair j's barrier, 20 + j = wave 4 (moving) at pair j's barrier, 40 + j = wave 0 past it,
// 60 = start, 61 = prologue barrier passed, 62 = wave 0 done, 63 = wave 4 done; 58 / 59 =
// s_memtime (shader clock) at wave 0's start / end
// XM (A/B): XCD-grouped bands -- workgroup L = blockIdx.y * gridDim.x + blockIdx.x runs on XCD
// L % 8, so the plain (band, image) = (blockIdx.x, blockIdx.y) puts an image's bands on different
// XCDs and the 7 halo input rows between two bands are fetched into two L2s; XM gives the bands of
// one image to workgroups L, L + 8, ... (one XCD).  A bijection when B % 8 == 0, else the identity.
// BR (A/B): the bias in 16 VGPRs as the first tap row's MFMA accumulator input, instead of
// 16 LDS reads per pair into the accumulators (same sum order: bias, then kh = 0..6)
// IL (A/B): column tile 0's epilogue (per 16-channel group: 4 packed converts, 3 packed maxes, a
// V-row write) interleaved in program order between tile 1's tap rows 1..4, one group each, instead
// of after all of tile 1's MFMAs (an in-order wave issues its 56 MFMAs first, so the epilogue
// behind them barely overlapped the pipe)
// (BR and IL shipped this round: 27.3 vs 28.1 us per B = 64 launch, bit-identical, profiles/r05zl_stem_ab.log;
// variant 0:34 is the previous form)
template <int PBT, int D, bool PRE = false, int DBG = 0, bool XM = false, bool BR = true, bool IL = true>
__global__ __launch_bounds__(512) void stem_role_fp16(const float* __restrict__ x, int B, int Cin,
                                                      const _Float16* __restrict__ w, const float* __restrict__ bias,
                                                      _Float16* __restrict__ out, RgbdSrc src,
                                                      unsigned long long* trace) {
  auto stamp = [&](int slot) __attribute__((always_inline)) {
    if constexpr (DBG == 4) {
      if ((threadIdx.x & 63) == 0) trace[(blockIdx.y * gridDim.x + blockIdx.x) * 64 + slot] = __builtin_amdgcn_s_memrealtime();
    }
  };
  using namespace stem;
  static_assert(RING >= 9 + 4 && D >= 2 && D <= 4, "ring / prefetch depth");
  constexpr int WSTAGE = RING * ROWB + 2 * CROWB + 64 * 4;
  __shared__ __attribute__((aligned(1024))) char smem[WSTAGE + 28 * 1024];
  char* ring = smem;
  char* vring = smem + RING * ROWB;
  float* bl = reinterpret_cast<float*>(vring + 2 * CROWB);
  char* wst = smem + WSTAGE;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int q = lane >> 4, r16 = lane & 15;
  int n = blockIdx.y, band = blockIdx.x;
  if constexpr (XM) {
    if (gridDim.y % 8 == 0) {
      const int L = blockIdx.y * gridDim.x + blockIdx.x, m = L >> 3;
      n = (m / (int)gridDim.x) * 8 + (L & 7);
      band = m % (int)gridDim.x;
    }
  }
  const int p0 = band * PBT;
  const bool mover = wid >= 4;
  const int mt = tid & 255;  // thread index within the role
  const float* xn = x + (size_t)n * Cin * 256 * 256;
  const int hbase = 4 * p0 - 7;
  if (wid == 0) stamp(60);
  if constexpr (DBG == 4) {  // shader-clock counter beside the 100 MHz one (slot 58 / 59: start / wave 0 done)
    if (tid == 0) trace[(blockIdx.y * gridDim.x + blockIdx.x) * 64 + 58] = __builtin_amdgcn_s_memtime();
  }

  // movers: thread mt takes pixels 4 lcg .. 4 lcg + 3 (all 4 channels) of row lr of a
  // 4-row group
  const int lr = mt >> 6, lcg = mt & 63;
  auto load_rows = [&](int hi0, float4* v) __attribute__((always_inline)) {
    const int hi = min(max(hi0 + lr, 0), 255);
    if constexpr (PRE) {
      const int r0 = src.Hs / 2 - 128, c0 = src.Ws / 2 - 128;
      const size_t row = ((size_t)n * src.Hs + hi + r0) * src.Ws + c0 + lcg * 4;
      // the 4 pixels' 12 bytes as 3 dwords and their depths as one float4 when aligned (the
      // centre crop of a 4-aligned width always is)
      uint8_t px[12];
      float dp[4];
      const uint8_t* p8 = src.rgb + row * 3;
      if ((((uintptr_t)p8) & 3) == 0 && (((uintptr_t)(src.depth + row)) & 15) == 0) {
        const uint32_t* p32 = reinterpret_cast<const uint32_t*>(p8);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const uint32_t wv = p32[j];
#pragma unroll
          for (int b = 0; b < 4; ++b) px[4 * j + b] = (uint8_t)(wv >> (8 * b));
        }
        const float4 d4 = *reinterpret_cast<const float4*>(src.depth + row);
        dp[0] = d4.x;
        dp[1] = d4.y;
        dp[2] = d4.z;
        dp[3] = d4.w;
      } else {
#pragma unroll
        for (int j = 0; j < 12; ++j) px[j] = p8[j];
#pragma unroll
        for (int k = 0; k < 4; ++k) dp[k] = src.depth[row + k];
      }
      float a[4][4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        // numpy's f64 / 255 then .float(): the correctly rounded f32 quotient is the same
        // value for every byte (checked exhaustively, tests/test_preprocess.py)
        const float c0 = (float)px[3 * k], c2 = (float)px[3 * k + 2];  // constant indices: no scratch array
        a[0][k] = (src.bgr ? c2 : c0) / 255.0f;
        a[1][k] = (float)px[3 * k + 1] / 255.0f;
        a[2][k] = (src.bgr ? c0 : c2) / 255.0f;
        float d = dp[k];
        if (isnan(d) || isinf(d)) d = 0.f;
        d = d / 0.035f;  // streaming.py:76
        if (src.near_m >= 0.f || src.far_m >= 0.f) {
          float sd = 0.035f * d;  // DepthPlaneAugmentation: scale, clip, unscale
          if (src.near_m >= 0.f && sd < src.near_m) sd = 0.f;
          if (src.far_m >= 0.f && sd > src.far_m) sd = 0.f;
          d = sd / 0.035f;
        }
        a[3][k] = d;
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) v[c] = float4{a[c][0], a[c][1], a[c][2], a[c][3]};
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int ch = min(c, Cin - 1);
        v[c] = *reinterpret_cast<const float4*>(xn + ((size_t)ch * 256 + hi) * 256 + lcg * 4);
      }
    }
  };
  auto store_rows = [&](int hi0, const float4* v) __attribute__((always_inline)) {
    const int slot = (hi0 + lr + 64) & (RING - 1);
    char* row = ring + slot * ROWB + (lcg * 4 + 3) * 8;
    const bool rok = (unsigned)(hi0 + lr) < 256u;
    float m[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) m[c] = (rok && c < Cin) ? 1.f : 0.f;
    const float a[4][4] = {{v[0].x, v[0].y, v[0].z, v[0].w}, {v[1].x, v[1].y, v[1].z, v[1].w},
                           {v[2].x, v[2].y, v[2].z, v[2].w}, {v[3].x, v[3].y, v[3].z, v[3].w}};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      half4 h;
#pragma unroll
      for (int c = 0; c < 4; ++c) h[c] = (_Float16)(a[c][k] * m[c]);
      *reinterpret_cast<half4*>(row + k * 8) = h;
    }
  };

  // prologue: movers load the first 9 rows (and the prefetch), every wave DMAs a share of
  // the weights (A-fragment order, as version 3), the bias goes to LDS
  float4 pf[D][4];
  if (mover) {
    load_rows(hbase, pf[0]);
    load_rows(hbase + 4, pf[1]);
  }
  float4 v8[4];
  if (mover && lr == 0) load_rows(hbase + 8, v8);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int b = wid + 8 * i;  // block = kh * 4 + tn
    if (b < 28) xdma16(w + (size_t)((b & 3) * 16 + r16) * 224 + (b >> 2) * 32 + q * 8, wst + b * 1024);
  }
  if (tid < 64) bl[tid] = bias[tid];
  if (mover) {
    for (int i = mt; i < RING * 6; i += 256) {
      const int slot = i / 6, k = i - (i / 6) * 6;
      const int px = k < 3 ? k : 256 + k;
      *reinterpret_cast<uint2*>(ring + slot * ROWB + px * 8) = make_uint2(0, 0);
    }
    store_rows(hbase, pf[0]);
    store_rows(hbase + 4, pf[1]);
    if (lr == 0) store_rows(hbase + 8, v8);
    // prefetch: pair k's new rows (hbase + 9 + 4 (k - 1)) into pf[k % D], k = 1 .. D - 1
#pragma unroll
    for (int k = 1; k < D; ++k)
      if (k <= PBT) load_rows(hbase + 9 + 4 * (k - 1), pf[k % D]);
  }
  // this wave's weight DMAs (the movers' prefetch, issued last, stays in flight)
  if (mover)
    xwait_vm<4 * (D - 1)>();
  else
    xwait_vm<0>();
  lds_barrier();
  if (wid == 0) stamp(61);

  constexpr int TN = 4;
  if (!mover) {
    su32x4 wf[7][TN];
#pragma unroll
    for (int kh = 0; kh < 7; ++kh)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) wf[kh][tn] = *reinterpret_cast<const su32x4*>(wst + (kh * 4 + tn) * 1024 + lane * 16);
    half4 prev[2][TN];  // post-ReLU conv row 2p - 1, per column tile
    f32x4 breg[TN];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) breg[tn] = BR ? *reinterpret_cast<const f32x4*>(bl + tn * 16 + q * 4) : f32x4{};
    stem_for<0, PBT + 1>([&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      const int r0 = 2 * p0 - 2 + 2 * j;  // pair j: conv rows r0 = 2p, r0 + 1 (p = p0 - 1 + j)
      const int hs = 4 * p0 - 7 + 4 * j;
      // column tile c = 0's epilogue (V write) is placed after c = 1's MFMAs are issued, so
      // its VALU work fills the MFMA pipe's shadow instead of following it
      f32x4 acc[2][2][TN];  // [column tile c][row t][tn]
      auto conv_tile = [&](int c, auto&& hook) __attribute__((always_inline)) {
        if constexpr (!BR) {
#pragma unroll
          for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int b = 0; b < TN; ++b) acc[c][t][b] = *reinterpret_cast<const f32x4*>(bl + b * 16 + q * 4);
        }
        // the 9 input rows of this pair (row t + kh for conv row t, tap row kh), each read
        // once and four taps' MFMAs (two tap rows) ahead of its first use
        su32x4 fr[9];
        auto rd = [&](int r) __attribute__((always_inline)) {
          const int slot = (hs + r + 64) & (RING - 1);
          fr[r] = *reinterpret_cast<const su32x4*>(ring + slot * ROWB + (2 * (wid * 32 + c * 16 + r16)) * 8 + q * 16);
        };
#pragma unroll
        for (int r = 0; r < 4; ++r) rd(r);
#pragma unroll
        for (int kh = 0; kh < 7; ++kh) {
          if (kh + 4 <= 8) rd(kh + 4);
          // keep each read two tap rows ahead (the scheduler sank them); VALU / SALU / MFMA may
          // still cross, so the first column tile's epilogue can fill the second tile's MFMA shadow
          __builtin_amdgcn_sched_barrier(0x000E);
          hook(kh);
#pragma unroll
          for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int tn = 0; tn < TN; ++tn)
              acc[c][t][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, wf[kh][tn]),
                                                                     __builtin_bit_cast(half8, fr[kh + 2 * t]),
                                                                     (BR && kh == 0) ? breg[tn] : acc[c][t][tn], 0, 0, 0);
        }
      };
      // rows above the image (only the whole pair r0 = -2, -1 of the first band) are 0 =
      // max-pool's -inf padding, since every window keeps >= 1 real post-ReLU value
      // ReLU commutes with max: relu(max(a, b, c)) = max(a, b, c, 0), so the V row is
      // max(prev, v0, max(v1, 0)) on the raw fp16 conv values, and prev (row 2p + 1) is kept
      // raw as well -- the same fp16 values as ReLU-then-max, one packed max fewer per pair of
      // channels
      // one 16-channel group tn of column tile c (the same operations, per group, as before)
      auto epi_tn = [&](int c, int tn) __attribute__((always_inline)) {
        const half4 z4 = half4{0, 0, 0, 0};
        half4 v0, v1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v0[e] = (_Float16)acc[c][0][tn][e];
          v1[e] = (_Float16)acc[c][1][tn][e];
        }
        if constexpr (j == 0) {
          if (r0 < 0) v1 = z4;
        }
        if constexpr (j >= 1) {
          char* vw = vring + (j & 1) * CROWB;
          const int wo = wid * 32 + c * 16 + r16;
          const half4 vv = __builtin_elementwise_max(__builtin_elementwise_max(prev[c][tn], v0),
                                                     __builtin_elementwise_max(v1, z4));
          const int ch = tn * 16 + q * 4;
          *reinterpret_cast<half4*>(vw + crow_swz(wo, ch >> 3) + (ch & 7) * 2) = vv;
        }
        prev[c][tn] = v1;
      };
      auto epi_tile = [&](int c) __attribute__((always_inline)) {
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) epi_tn(c, tn);
      };
      auto no_hook = [&](int) __attribute__((always_inline)) {};
      conv_tile(0, no_hook);
      if constexpr (IL) {
        conv_tile(1, [&](int kh) __attribute__((always_inline)) {
          if (kh >= 1 && kh <= TN) {
            epi_tn(0, kh - 1);
            __builtin_amdgcn_sched_barrier(0);
          }
        });
      } else {
        conv_tile(1, no_hook);
        epi_tile(0);
      }
      epi_tile(1);
      if (wid == 0) stamp(j);
      lds_barrier();
      if (wid == 0) stamp(40 + j);
    });
    if (wid == 0) stamp(62);
    if constexpr (DBG == 4) {
      if (tid == 0) trace[(blockIdx.y * gridDim.x + blockIdx.x) * 64 + 59] = __builtin_amdgcn_s_memtime();
    }
  } else {
    stem_for<0, PBT + 2>([&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      const int hs = 4 * p0 - 7 + 4 * j;
      if constexpr (DBG == 5) {  // timing only: movers idle (barriers only), wrong results
        if constexpr (j <= PBT) lds_barrier();
        return;
      }
      // the rows of pair j + D (new rows hs + 9 + 4 (D - 1) ..) into pf[j % D]
      if constexpr (j + D <= PBT) load_rows(hs + 9 + 4 * (D - 1), pf[j % D]);
      if constexpr (j >= 2) {  // pooled row p0 + j - 2 from V(j - 1)
        const int p = p0 + j - 2;
        const char* vr = vring + ((j - 1) & 1) * CROWB;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int e = mt + 256 * h, qc = e >> 3, c8 = e & 7;
          half8 m = *reinterpret_cast<const half8*>(vr + crow_swz(2 * qc, c8));
          m = __builtin_elementwise_max(m, *reinterpret_cast<const half8*>(vr + crow_swz(2 * qc + 1, c8)));
          if (qc > 0) m = __builtin_elementwise_max(m, *reinterpret_cast<const half8*>(vr + crow_swz(2 * qc - 1, c8)));
          store16<true>(out, (unsigned)(((((size_t)n * 64 + p) * 64 + qc) * 64 + c8 * 8) * 2), m);
        }
      }
      if constexpr (j < PBT) store_rows(hs + 9, pf[(j + 1) % D]);  // pair j + 1's new rows
      if (wid == 4 && j <= PBT) stamp(20 + j);
      if constexpr (j <= PBT) lds_barrier();
    });
    if constexpr (DBG == 4) {
      __builtin_amdgcn_s_waitcnt(0);
      if (wid == 4) stamp(63);
    }
  }
}

template <int PBT, int D, bool PRE = false, int DBG = 0, bool XM = false, bool BR = true, bool IL = true>
static int run_stem4(const float* x, int B, int Cin, const _Float16* w, const float* bias, _Float16* out, hipStream_t s,
                     RgbdSrc src = RgbdSrc{}, unsigned long long* trace = nullptr) {
  PA_CHECK((size_t)B * 64 * 64 * 64 * 2 < 0x7fffffffu, "stem: output over 2 GB");
  hipLaunchKernelGGL((stem_role_fp16<PBT, D, PRE, DBG, XM, BR, IL>), dim3(64 / PBT, B), dim3(stem::NT), 0, s, x, B, Cin, w, bias, out,
                     src, trace);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

template <int PBT, int D, bool WT = false, int DBG = 0, bool PRE = false>
static int run_stem3(const float* x, int B, int Cin, const _Float16* w, const float* bias, _Float16* out,
                     hipStream_t s, unsigned long long* trace = nullptr, RgbdSrc src = RgbdSrc{}) {
  PA_CHECK(!WT || (size_t)B * 64 * 64 * 64 * 2 < 0x7fffffffu, "stem: output over 2 GB");
  hipLaunchKernelGGL((stem_pool3_fp16<PBT, D, WT, DBG, PRE>), dim3(64 / PBT, B), dim3(stem::NT), 0, s, x, B, Cin, w, bias,
                     out, trace, src);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

int launch_stem_pool_rgbd(const RgbdSrc& src, int B, const _Float16* w, const float* bias, _Float16* out,
                          hipStream_t s) {
  PA_CHECK(src.rgb && src.depth, "stem rgbd: null frame pointer");
  PA_CHECK(src.Hs >= 256 && src.Ws >= 256, "stem rgbd: source %dx%d smaller than 256x256", src.Hs, src.Ws);
  if (B <= 0) return PA_OK;
  // a few frames (the streaming batch): shorter bands, so the grid still covers the chip
  // (B = 3: 96 workgroups of 2 pooled rows instead of 12 of 16; same arithmetic per row)
  // (B <= 4: one pooled row per workgroup -- 192 workgroups at B = 3, 5.6 vs 6.7 us for two rows,
  // bit-identical, profiles/r04stem/)
  if (B <= 4) return run_stem4<1, 2, true>(nullptr, B, 4, w, bias, out, s, src);
  if (B <= 8) return run_stem4<2, 2, true>(nullptr, B, 4, w, bias, out, s, src);
  if (B <= 24) return run_stem4<4, 2, true>(nullptr, B, 4, w, bias, out, s, src);
  return run_stem4<16, 2, true>(nullptr, B, 4, w, bias, out, s, src);
}

int launch_stem_pool_fp16(const float* x, int B, int Cin, const _Float16* w, const float* bias, _Float16* out,
                          hipStream_t s) {
  PA_CHECK(Cin >= 1 && Cin <= 4, "stem: Cin %d", Cin);
  if (B <= 0) return PA_OK;
  switch (g_variant[0]) {
    case 10: return run_stem3<8, 3, true>(x, B, Cin, w, bias, out, s);
    case 11: return run_stem3<16, 3, true>(x, B, Cin, w, bias, out, s);
    case 12: return run_stem3<32, 3, true>(x, B, Cin, w, bias, out, s);
    case 15: return run_stem3<32, 2, true>(x, B, Cin, w, bias, out, s);
    case 13: return run_stem3<16, 2, false>(x, B, Cin, w, bias, out, s);  // plain (write-back) stores
#if PA_TIMING_VARIANTS
    case 21: return run_stem3<16, 2, true, 1>(x, B, Cin, w, bias, out, s);  // timing only: no MFMAs
    case 22: return run_stem3<16, 2, true, 2>(x, B, Cin, w, bias, out, s);  // timing only: no pooling
    case 23: return run_stem3<16, 2, true, 3>(x, B, Cin, w, bias, out, s);  // timing only: no input rows
    case 25: return run_stem3<16, 2, true, 5>(x, B, Cin, w, bias, out, s);  // timing only: no conv-row writes
#endif
    case 14:
      if (g_trace) return run_stem3<16, 2, true, 4>(x, B, Cin, w, bias, out, s, g_trace);  // timestamps
      break;
    case 16: return run_stem3<16, 2, true>(x, B, Cin, w, bias, out, s);  // version 3 (shipped until round 2)
    case 24:
      if (g_trace) return run_stem4<16, 2, false, 4>(x, B, Cin, w, bias, out, s, RgbdSrc{}, g_trace);  // timestamps
      break;
#if PA_TIMING_VARIANTS
    case 26: return run_stem4<16, 2, false, 5>(x, B, Cin, w, bias, out, s);  // timing only: idle movers
#endif
    case 27: return run_stem4<8, 2>(x, B, Cin, w, bias, out, s);  // shorter bands at any batch (A/B)
    case 28: return run_stem4<4, 2>(x, B, Cin, w, bias, out, s);
    case 29: return run_stem4<32, 2>(x, B, Cin, w, bias, out, s);
    case 30: return run_stem4<16, 2, false, 0, true>(x, B, Cin, w, bias, out, s);  // XCD-grouped bands
    case 31: return run_stem4<16, 2, false, 0, false, true, false>(x, B, Cin, w, bias, out, s);  // BR alone
    case 32: return run_stem4<16, 2, false, 0, false, true, true>(x, B, Cin, w, bias, out, s);  // BR + IL
    case 33: return run_stem4<16, 2, false, 0, false, false, true>(x, B, Cin, w, bias, out, s);  // IL
    case 34: return run_stem4<16, 2, false, 0, false, false, false>(x, B, Cin, w, bias, out, s);  // neither (round 4)
    // shipped: version 4, the role split (29.3 vs 31.8 us per B = 64 launch, bit-identical;
    // prefetch depth 3 / 4 measured 29.7 / 30.4 us)
    default: break;
  }
  // small batches: shorter bands (as launch_stem_pool_rgbd)
  if (B <= 4) return run_stem4<1, 2>(x, B, Cin, w, bias, out, s);
  if (B <= 8) return run_stem4<2, 2>(x, B, Cin, w, bias, out, s);
  if (B <= 24) return run_stem4<4, 2>(x, B, Cin, w, bias, out, s);
  return run_stem4<16, 2>(x, B, Cin, w, bias, out, s);  // also variants 14 / 24 without a trace buffer
}

}  // namespace pa
