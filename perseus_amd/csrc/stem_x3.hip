// Fused RGBD stem of the fp16x3 parity mode: conv 7x7 s2 p3 (Cin <= 4 -> 64) + folded
// BN + ReLU + max-pool 3x3 s2 p1 (torchvision resnet18 stem behind
// perseus/detector/models.py:27-28,34-40), with every product formed as
// x_hi w_hi + x_lo w_hi + x_hi w_lo in f32 (conv_gx.h X3): the f32 NCHW input is split
// into an fp16 hi/lo pair on its way into LDS, the weights arrive as the hi/lo planes
// of w * 2^e (per output channel), the ReLU / max-pool run on f32 values and the pooled
// map is written as the (hi, lo) plane pair the layer1 convs read.
//
// Same band decomposition as stem.hip's stem_pool3_fp16 (one image x PBT pooled rows
// per workgroup, conv rows in pairs from a 16-row ring of input rows, each wave owns 16
// conv columns of both rows of a pair and forms the vertical max in registers).  The
// differences are forced by LDS: the two input planes (2 x 33.5 KB), both weight
// planes (2 x 28 KB; 112 VGPRs per plane would not fit next to the f32 epilogue) and
// one f32 V row (32 KB) -- so the V row is single-buffered, and each pair has two
// barriers (V row free / V row written) instead of one.
#include "conv_gx.h"

namespace pa {

typedef _Float16 half2_x __attribute__((ext_vector_type(2)));

namespace stemx3 {
constexpr int NT = 512;
constexpr int RING = 16;
constexpr int PW = 262;               // ring row width in pixels (wi = c - 3)
constexpr int ROWB = PW * 8;          // one plane's ring row: 4 x fp16 per pixel
constexpr int VROWB = 128 * 256;      // f32 V row: 128 px x 64 ch x 4 B
constexpr int WPLANE = 28 * 1024;     // one weight plane in A-fragment order (7 kh x 4 tn blocks)
}  // namespace stemx3

// f32 V row: pixel px = 16 chunks of 16 B (4 channels), XOR-swizzled by px
__device__ __forceinline__ int vswz(int px, int chunk) { return px * 256 + ((chunk ^ (px & 15)) << 4); }

template <int PBT, int D>
__global__ __launch_bounds__(512) void stem_pool3_x3(const float* __restrict__ x, int B, int Cin,
                                                     const _Float16* __restrict__ w, const float* __restrict__ bias_s,
                                                     const float* __restrict__ scale, _Float16* __restrict__ out) {
  using namespace stemx3;
  static_assert(RING >= 9 + 4 && D >= 2 && D <= 3, "ring / prefetch depth");
  __shared__ __attribute__((aligned(1024))) char smem[2 * RING * ROWB + VROWB + 2 * WPLANE + 2 * 64 * 4];
  char* ring = smem;                    // plane 0 (hi), plane 1 (lo) at + RING * ROWB
  char* vrow = smem + 2 * RING * ROWB;  // f32
  char* wst = vrow + VROWB;             // weight planes: hi, lo
  float* bl = reinterpret_cast<float*>(wst + 2 * WPLANE);  // bias * 2^e
  float* sl = bl + 64;                                      // 2^-e

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
      const HiLo s0 = split_x3(a0[k]), s1 = split_x3(a1[k]);
      half2_x h{s0.hi, s1.hi}, l{s0.lo, s1.lo};
      *reinterpret_cast<half2_x*>(row + k * 8) = h;
      *reinterpret_cast<half2_x*>(row + RING * ROWB + k * 8) = l;
    }
  };
  // prologue: the first 9 input rows, the weight planes (DMA), bias / scale, the prefetch
  const int hbase = 4 * p0 - 7;
  float4 v0[2], v1[2], v2[2];
  load_rows(hbase, v0);
  load_rows(hbase + 4, v1);
  if (lr == 0) load_rows(hbase + 8, v2);
  float bv = 0.f, sv = 0.f;
  if (tid < 64) {
    bv = bias_s[tid];
    sv = scale[tid];
  }
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const int b = wid + 8 * i;  // plane (b / 28), block kh * 4 + tn = b % 28
    const int pl = b / 28, bb = b - pl * 28;
    xdma16(w + (size_t)pl * 64 * 224 + (size_t)((bb & 3) * 16 + r16) * 224 + (bb >> 2) * 32 + q * 8,
           wst + b * 1024);
  }
  float4 pf[D][2];
#pragma unroll
  for (int k = 1; k < D; ++k) load_rows(hbase + 9 + 4 * (k - 1), pf[k]);
  __builtin_amdgcn_sched_barrier(0);
  for (int i = tid; i < 2 * RING * 6; i += NT) {
    const int slot = i / 6, k = i - (i / 6) * 6;
    const int px = k < 3 ? k : 256 + k;
    *reinterpret_cast<uint2*>(ring + slot * ROWB + px * 8) = make_uint2(0, 0);
  }
  store_rows(hbase, v0);
  store_rows(hbase + 4, v1);
  if (lr == 0) store_rows(hbase + 8, v2);
  if (tid < 64) {
    bl[tid] = bv;
    sl[tid] = sv;
  }
  xwait_vm<2 * (D - 1)>();  // this wave's weight DMAs (only the prefetch may stay in flight)
  lds_barrier();

  const int wo = wid * 16 + r16;  // this lane's conv column
  const int qc = tid >> 3, c8 = tid & 7;
  constexpr int TN = 4;
  f32x4 prev[TN];  // post-ReLU conv row 2p - 1 (this lane's column, 4 channels per tile)
  f32x4 vv[TN];

  gx_for<0, PBT + 1>([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    const int r0 = 2 * p0 - 2 + 2 * j;  // pair j: conv rows r0 = 2p, r0 + 1 (p = p0 - 1 + j)
    const int hs = 4 * p0 - 7 + 4 * j;
    if constexpr (j + D <= PBT) load_rows(hs + 9 + 4 * (D - 1), pf[j % D]);
    f32x4 acc[2][TN];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) acc[a][b] = *reinterpret_cast<const f32x4*>(bl + b * 16 + q * 4);
#pragma unroll
    for (int kh = 0; kh < 7; ++kh) {
      u32x4 fh[2], fl[2], wh[TN], wl[TN];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int slot = (hs + 2 * t + kh + 64) & (RING - 1);
        fh[t] = *reinterpret_cast<const u32x4*>(ring + slot * ROWB + (2 * wo) * 8 + q * 16);
        fl[t] = *reinterpret_cast<const u32x4*>(ring + RING * ROWB + slot * ROWB + (2 * wo) * 8 + q * 16);
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        wh[tn] = *reinterpret_cast<const u32x4*>(wst + (kh * 4 + tn) * 1024 + lane * 16);
        wl[tn] = *reinterpret_cast<const u32x4*>(wst + WPLANE + (kh * 4 + tn) * 1024 + lane * 16);
      }
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
          const half8 ah = __builtin_bit_cast(half8, wh[tn]), al = __builtin_bit_cast(half8, wl[tn]);
          const half8 bh = __builtin_bit_cast(half8, fh[t]), bo = __builtin_bit_cast(half8, fl[t]);
          acc[t][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc[t][tn], 0, 0, 0);
          acc[t][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bo, acc[t][tn], 0, 0, 0);
          acc[t][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, acc[t][tn], 0, 0, 0);
        }
    }
    // unscale (exact), ReLU; rows above the image (only the pair r0 = -2, -1) are 0 =
    // max-pool's -inf padding, since every window keeps >= 1 real post-ReLU value
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const f32x4 s4 = *reinterpret_cast<const f32x4*>(sl + tn * 16 + q * 4);
      f32x4 a0, a1;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a0[e] = fmaxf(acc[0][tn][e] * s4[e], 0.f);
        a1[e] = r0 < 0 ? 0.f : fmaxf(acc[1][tn][e] * s4[e], 0.f);
      }
      if constexpr (j >= 1) {
#pragma unroll
        for (int e = 0; e < 4; ++e) vv[tn][e] = fmaxf(prev[tn][e], fmaxf(a0[e], a1[e]));
      }
      prev[tn] = a1;
    }
    lds_barrier();  // every wave is past its conv reads (ring) and the last pool's reads (V row)
    if constexpr (j >= 1) {
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) *reinterpret_cast<f32x4*>(vrow + vswz(wo, tn * 4 + q)) = vv[tn];
    }
    if constexpr (j < PBT) store_rows(hs + 9, pf[(j + 1) % D]);
    lds_barrier();
    if constexpr (j >= 1) {  // pooled row p = p0 + j - 1: horizontal max over V pixels 2qc - 1 .. 2qc + 1
      const int p = p0 + j - 1;
      f32x4 m0 = *reinterpret_cast<const f32x4*>(vrow + vswz(2 * qc, 2 * c8));
      f32x4 m1 = *reinterpret_cast<const f32x4*>(vrow + vswz(2 * qc, 2 * c8 + 1));
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        const int px = dx == 0 ? 2 * qc + 1 : 2 * qc - 1;
        if (px < 0) continue;
        const f32x4 a = *reinterpret_cast<const f32x4*>(vrow + vswz(px, 2 * c8));
        const f32x4 b = *reinterpret_cast<const f32x4*>(vrow + vswz(px, 2 * c8 + 1));
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          m0[e] = fmaxf(m0[e], a[e]);
          m1[e] = fmaxf(m1[e], b[e]);
        }
      }
      half8 h, l;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const HiLo s = split_x3(e < 4 ? m0[e] : m1[e - 4]);
        h[e] = s.hi;
        l[e] = s.lo;
      }
      const unsigned o = (unsigned)(((((size_t)n * 64 + p) * 64 + qc) * 128 + c8 * 8) * 2);
      store16<true>(out, o, h);
      store16<true>(out, o + 128, l);
    }
  });
}

// Role split (stem.hip's version 4 for the fp16x3 arithmetic above, bit-identical outputs):
// waves 0-3 (one per SIMD) only convolve, each owning 32 conv columns (two 16-column tiles)
// of both rows of every pair: per tap row 8 weight fragments (hi / lo planes, shared by the
// two tiles and two rows) + 8 input fragments for 48 MFMAs (0.33 LDS reads per MFMA against
// 0.5), the vertical max in registers.  Waves 4-7 only move data: the input rows' global
// loads D pairs ahead, their hi / lo split into the ring, the pooling of the previous V row
// and its stores.  The f32 V row stays single-buffered (LDS), so each pair has two barriers
// as before -- A: the movers are done with V(j - 1) and pair j + 1's ring rows, B: V(j) is
// written -- but the convolving waves reach A straight from their MFMAs, and the movers'
// work runs under them.
template <int PBT, int D>
__global__ __launch_bounds__(512) void stem_role_x3(const float* __restrict__ x, int B, int Cin,
                                                    const _Float16* __restrict__ w, const float* __restrict__ bias_s,
                                                    const float* __restrict__ scale, _Float16* __restrict__ out) {
  using namespace stemx3;
  static_assert(RING >= 9 + 4 && D >= 2 && D <= 3, "ring / prefetch depth");
  __shared__ __attribute__((aligned(1024))) char smem[2 * RING * ROWB + VROWB + 2 * WPLANE + 2 * 64 * 4];
  char* ring = smem;                    // plane 0 (hi), plane 1 (lo) at + RING * ROWB
  char* vrow = smem + 2 * RING * ROWB;  // f32
  char* wst = vrow + VROWB;             // weight planes: hi, lo
  float* bl = reinterpret_cast<float*>(wst + 2 * WPLANE);  // bias * 2^e
  float* sl = bl + 64;                                      // 2^-e

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int q = lane >> 4, r16 = lane & 15;
  const int n = blockIdx.y;
  const int p0 = blockIdx.x * PBT;
  const bool mover = wid >= 4;
  const int mt = tid & 255;
  const float* xn = x + (size_t)n * Cin * 256 * 256;

  // movers: thread mt takes pixels 4 lcg .. 4 lcg + 3 (all 4 channels) of row lr of a 4-row group
  const int lr = mt >> 6, lcg = mt & 63;
  auto load_rows = [&](int hi0, float4* v) __attribute__((always_inline)) {
    const int hi = min(max(hi0 + lr, 0), 255);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int ch = min(c, Cin - 1);
      v[c] = *reinterpret_cast<const float4*>(xn + ((size_t)ch * 256 + hi) * 256 + lcg * 4);
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
      half4 h, l;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const HiLo s = split_x3(a[c][k] * m[c]);
        h[c] = s.hi;
        l[c] = s.lo;
      }
      *reinterpret_cast<half4*>(row + k * 8) = h;
      *reinterpret_cast<half4*>(row + RING * ROWB + k * 8) = l;
    }
  };
  // pooled row p from the V row: thread mt, items e = mt, mt + 256 (column qc = e >> 3, 8 channels c8 = e & 7)
  auto pool_row = [&](int p) __attribute__((always_inline)) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int e = mt + 256 * h, qc = e >> 3, c8 = e & 7;
      f32x4 m0 = *reinterpret_cast<const f32x4*>(vrow + vswz(2 * qc, 2 * c8));
      f32x4 m1 = *reinterpret_cast<const f32x4*>(vrow + vswz(2 * qc, 2 * c8 + 1));
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        const int px = dx == 0 ? 2 * qc + 1 : 2 * qc - 1;
        if (px < 0) continue;
        const f32x4 a = *reinterpret_cast<const f32x4*>(vrow + vswz(px, 2 * c8));
        const f32x4 b = *reinterpret_cast<const f32x4*>(vrow + vswz(px, 2 * c8 + 1));
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          m0[k] = fmaxf(m0[k], a[k]);
          m1[k] = fmaxf(m1[k], b[k]);
        }
      }
      half8 hh, ll;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const HiLo s = split_x3(k < 4 ? m0[k] : m1[k - 4]);
        hh[k] = s.hi;
        ll[k] = s.lo;
      }
      const unsigned o = (unsigned)(((((size_t)n * 64 + p) * 64 + qc) * 128 + c8 * 8) * 2);
      store16<true>(out, o, hh);
      store16<true>(out, o + 128, ll);
    }
  };

  // prologue: movers load the first 9 rows (and the prefetch), every wave DMAs a share of the
  // weight planes, bias / scale to LDS
  const int hbase = 4 * p0 - 7;
  float4 pf[D][4];
  float4 v8[4];
  if (mover) {
    load_rows(hbase, pf[0]);
    load_rows(hbase + 4, pf[1]);
    if (lr == 0) load_rows(hbase + 8, v8);
  }
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const int b = wid + 8 * i;  // plane (b / 28), block kh * 4 + tn = b % 28
    const int pl = b / 28, bb = b - pl * 28;
    xdma16(w + (size_t)pl * 64 * 224 + (size_t)((bb & 3) * 16 + r16) * 224 + (bb >> 2) * 32 + q * 8,
           wst + b * 1024);
  }
  if (tid < 64) {
    bl[tid] = bias_s[tid];
    sl[tid] = scale[tid];
  }
  if (mover) {
    for (int i = mt; i < 2 * RING * 6; i += 256) {
      const int slot = i / 6, k = i - (i / 6) * 6;
      const int px = k < 3 ? k : 256 + k;
      *reinterpret_cast<uint2*>(ring + slot * ROWB + px * 8) = make_uint2(0, 0);
    }
    store_rows(hbase, pf[0]);
    store_rows(hbase + 4, pf[1]);
    if (lr == 0) store_rows(hbase + 8, v8);
#pragma unroll
    for (int k = 1; k < D; ++k)
      if (k <= PBT) load_rows(hbase + 9 + 4 * (k - 1), pf[k % D]);
    xwait_vm<4 * (D - 1)>();  // this wave's weight DMAs (the prefetch, issued last, stays in flight)
  } else {
    xwait_vm<0>();
  }
  lds_barrier();

  constexpr int TN = 4;
  if (!mover) {
    f32x4 prev[2][TN];  // post-ReLU conv row 2p - 1, per column tile
    gx_for<0, PBT + 1>([&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      const int r0 = 2 * p0 - 2 + 2 * j;  // pair j: conv rows r0 = 2p, r0 + 1 (p = p0 - 1 + j)
      const int hs = 4 * p0 - 7 + 4 * j;
      f32x4 acc[2][2][TN];  // [column tile c][row t][tn]
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int b = 0; b < TN; ++b) acc[c][t][b] = *reinterpret_cast<const f32x4*>(bl + b * 16 + q * 4);
#pragma unroll
      for (int kh = 0; kh < 7; ++kh) {
        u32x4 fh[2][2], fl[2][2], wh[TN], wl[TN];
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
          wh[tn] = *reinterpret_cast<const u32x4*>(wst + (kh * 4 + tn) * 1024 + lane * 16);
          wl[tn] = *reinterpret_cast<const u32x4*>(wst + WPLANE + (kh * 4 + tn) * 1024 + lane * 16);
        }
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            const int slot = (hs + 2 * t + kh + 64) & (RING - 1);
            const int wo = wid * 32 + c * 16 + r16;
            fh[c][t] = *reinterpret_cast<const u32x4*>(ring + slot * ROWB + (2 * wo) * 8 + q * 16);
            fl[c][t] = *reinterpret_cast<const u32x4*>(ring + RING * ROWB + slot * ROWB + (2 * wo) * 8 + q * 16);
          }
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
              const half8 ah = __builtin_bit_cast(half8, wh[tn]), al = __builtin_bit_cast(half8, wl[tn]);
              const half8 bh = __builtin_bit_cast(half8, fh[c][t]), bo = __builtin_bit_cast(half8, fl[c][t]);
              acc[c][t][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc[c][t][tn], 0, 0, 0);
              acc[c][t][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bo, acc[c][t][tn], 0, 0, 0);
              acc[c][t][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, acc[c][t][tn], 0, 0, 0);
            }
      }
      // unscale (exact), ReLU, vertical max; rows above the image (only the pair r0 = -2, -1)
      // are 0 = max-pool's -inf padding, since every window keeps >= 1 real post-ReLU value
      f32x4 vv[2][TN];
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
          const f32x4 s4 = *reinterpret_cast<const f32x4*>(sl + tn * 16 + q * 4);
          f32x4 a0, a1;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            a0[e] = fmaxf(acc[c][0][tn][e] * s4[e], 0.f);
            a1[e] = r0 < 0 ? 0.f : fmaxf(acc[c][1][tn][e] * s4[e], 0.f);
          }
          if constexpr (j >= 1) {
#pragma unroll
            for (int e = 0; e < 4; ++e) vv[c][tn][e] = fmaxf(prev[c][tn][e], fmaxf(a0[e], a1[e]));
          }
          prev[c][tn] = a1;
        }
      lds_barrier();  // A: the movers are past V(j - 1) and have stored pair j + 1's rows
      if constexpr (j >= 1) {
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int tn = 0; tn < TN; ++tn)
            *reinterpret_cast<f32x4*>(vrow + vswz(wid * 32 + c * 16 + r16, tn * 4 + q)) = vv[c][tn];
      }
      lds_barrier();  // B: V(j) written
    });
  } else {
    gx_for<0, PBT + 1>([&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      const int hs = 4 * p0 - 7 + 4 * j;
      if constexpr (j + D <= PBT) load_rows(hs + 9 + 4 * (D - 1), pf[j % D]);  // pair j + D's new rows
      if constexpr (j >= 2) pool_row(p0 + j - 2);                               // from V(j - 1)
      if constexpr (j < PBT) store_rows(hs + 9, pf[(j + 1) % D]);                // pair j + 1's new rows
      lds_barrier();  // A
      lds_barrier();  // B
    });
    pool_row(p0 + PBT - 1);  // from V(PBT)
  }
}

int launch_stem_pool_x3(const float* x, int B, int Cin, const _Float16* w, const float* bias_s, const float* scale,
                        _Float16* out, hipStream_t s) {
  PA_CHECK(Cin >= 1 && Cin <= 4, "stem x3: Cin %d", Cin);
  PA_CHECK((size_t)B * 64 * 64 * 128 * 2 < 0x7fffffffu, "stem x3: output over 2 GB");
  if (B <= 0) return PA_OK;
  constexpr int PBT = 16;
  if (g_variant[0] == 30)  // the all-waves form (shipped until round 4)
    hipLaunchKernelGGL((stem_pool3_x3<PBT, 2>), dim3(64 / PBT, B), dim3(stemx3::NT), 0, s, x, B, Cin, w, bias_s, scale,
                       out);
  else
    hipLaunchKernelGGL((stem_role_x3<PBT, 2>), dim3(64 / PBT, B), dim3(stemx3::NT), 0, s, x, B, Cin, w, bias_s, scale,
                       out);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

// latency mode (a few frames): bands of 2 pooled rows, 32 workgroups per frame instead of 4
// (stem.hip's short bands for the fp16 stem); the same arithmetic per pooled row
int launch_stem_pool_x3_small(const float* x, int B, int Cin, const _Float16* w, const float* bias_s,
                              const float* scale, _Float16* out, hipStream_t s) {
  PA_CHECK(Cin >= 1 && Cin <= 4, "stem x3: Cin %d", Cin);
  PA_CHECK((size_t)B * 64 * 64 * 128 * 2 < 0x7fffffffu, "stem x3: output over 2 GB");
  if (B <= 0) return PA_OK;
  constexpr int PBT = 2;
  if (B <= 4 && g_variant[0] != 30) {  // one pooled row per workgroup: 10.1 vs 12.7 us at B = 3 (profiles/r04stem/)
    hipLaunchKernelGGL((stem_role_x3<1, 2>), dim3(64, B), dim3(stemx3::NT), 0, s, x, B, Cin, w, bias_s, scale, out);
    PA_LAUNCH_CHECK();
    return PA_OK;
  }
  if (g_variant[0] == 30)
    hipLaunchKernelGGL((stem_pool3_x3<PBT, 2>), dim3(64 / PBT, B), dim3(stemx3::NT), 0, s, x, B, Cin, w, bias_s, scale,
                       out);
  else
    hipLaunchKernelGGL((stem_role_x3<PBT, 2>), dim3(64 / PBT, B), dim3(stemx3::NT), 0, s, x, B, Cin, w, bias_s, scale,
                       out);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

}  // namespace pa
