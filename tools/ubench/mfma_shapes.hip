// Microbenchmark (round 3): which LDS-fed MFMA loop shape can beat the conv kernels'
// current K loop (v_mfma_f32_16x16x32_f16, 8 waves per CU, 64x32 per wave = 0.75
// ds_read_b128 per 16-cycle MFMA; tools/ubench/mfma_clock.hip measured 0.49-0.54 of
// 2.5 PF for it).  Candidates:
//   * v_mfma_f32_32x32x16_f16 (32 cycles, 2 operand fragments of 1 KB each) at
//     1.5 / 1.0 / 2.0 reads per MFMA — MI355X_MICROARCH.md prices 2 reads per 32-cycle gap
//     at <= 3 cycles;
//   * 16x16x32 register-blocked 128x64 per wave (0.375 reads per MFMA), one wave per SIMD.
// Each wave streams its fragments from a 64 KB LDS image (conflict-free 64 x 16 B rows),
// READS = 0: operands stay in registers; 1: read right before use; 2: read one k-group
// ahead (software pipelined, what the conv kernels do); 3: as 2 for the B (pixel) fragments
// only, the A (weight) fragments stay in registers (round 5: weight-resident-in-VGPR layer1).  Random fp16 operands (clock
// depends on data: MI355X_MICROARCH.md 'DVFS give-back').  Clock = s_memtime /
// s_memrealtime x 100 MHz per wave, median.
//
//   hipcc -O3 --offload-arch=gfx950 tools/ubench/mfma_shapes.hip -o tools/ubench/mfma_shapes
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <vector>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));

template <int S>
struct Acc;
template <>
struct Acc<16> {
  typedef f32x4 T;
  static __device__ T mma(u4 a, u4 b, T c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, a), __builtin_bit_cast(half8, b), c, 0, 0, 0);
  }
  static __device__ float pick(T c) { return c[0] + c[3]; }
};
template <>
struct Acc<32> {
  typedef f32x16 T;
  static __device__ T mma(u4 a, u4 b, T c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, a), __builtin_bit_cast(half8, b), c, 0, 0, 0);
  }
  static __device__ float pick(T c) { return c[0] + c[15]; }
};

// S = MFMA shape (16: 16x16x32, 32: 32x32x16); TM x TN accumulator tiles per wave;
// one k-group = TM + TN fragment reads (READS > 0) and TM * TN MFMAs
template <int S, int TM, int TN, int READS, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void k(const u4* __restrict__ in, float* out, unsigned long long* clk, int iters) {
  typedef typename Acc<S>::T AT;
  __shared__ u4 lds[4096];  // 64 KB
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < 4096; i += WAVES * 64) lds[i] = in[(blockIdx.x * 4096 + i) & 65535];
  __syncthreads();
  u4 fa[TN], fb[TM];
  for (int i = 0; i < TN; ++i) fa[i] = in[(tid * 7 + i) & 65535];
  for (int i = 0; i < TM; ++i) fb[i] = in[(tid * 13 + i + 5) & 65535];
  AT acc[TM][TN];
  for (int i = 0; i < TM; ++i)
    for (int j = 0; j < TN; ++j)
      for (int e = 0; e < (int)(sizeof(AT) / 4); ++e) acc[i][j][e] = 0.f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  const int base = lane + (tid >> 6) * 64 * 3;
  u4 ga[TN], gb[TM];
  if (READS >= 2) {
#pragma unroll
    for (int i = 0; i < TN; ++i) ga[i] = lds[(base + i * 256) & 4095];
#pragma unroll
    for (int i = 0; i < TM; ++i) gb[i] = lds[(base + 2048 + i * 256) & 4095];
  }
  for (int it = 0; it < iters; ++it) {
    const int off = (it & 7) * 64;
    if (READS == 1) {
#pragma unroll
      for (int i = 0; i < TN; ++i) fa[i] = lds[(base + i * 256 + off) & 4095];
#pragma unroll
      for (int i = 0; i < TM; ++i) fb[i] = lds[(base + 2048 + i * 256 + off) & 4095];
    }
    if (READS == 3) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        fb[i] = gb[i];
        gb[i] = lds[(base + 2048 + i * 256 + off + 64) & 4095];
      }
    }
    if (READS == 2) {
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        fa[i] = ga[i];
        ga[i] = lds[(base + i * 256 + off + 64) & 4095];
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        fb[i] = gb[i];
        gb[i] = lds[(base + 2048 + i * 256 + off + 64) & 4095];
      }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = Acc<S>::mma(fa[j], fb[i], acc[i][j]);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  for (int i = 0; i < TM; ++i)
    for (int j = 0; j < TN; ++j) s += Acc<S>::pick(acc[i][j]);
  out[blockIdx.x * 1024 + tid] = s;
  if (lane == 0) {
    clk[2 * (blockIdx.x * 16 + (tid >> 6))] = t1 - t0;
    clk[2 * (blockIdx.x * 16 + (tid >> 6)) + 1] = r1 - r0;
  }
}

template <int S, int TM, int TN, int READS, int WAVES>
void run(const char* name, const u4* in, float* out, unsigned long long* clk) {
  const int grid = 256;
  // flop per MFMA: 16x16x32 and 32x32x16 are 16384 / 32768; keep ~100 ms per run
  const double mflop = 2.0 * S * S * (512 / S);
  const int iters = (int)(2.6e8 / (mflop * TM * TN * WAVES / 8.0));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k<S, TM, TN, READS, WAVES><<<grid, WAVES * 64>>>(in, out, clk, iters);  // warm
  hipEventRecord(e0);
  const int reps = 10;
  for (int r = 0; r < reps; ++r) k<S, TM, TN, READS, WAVES><<<grid, WAVES * 64>>>(in, out, clk, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h(grid * 16 * 2);
  hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost);
  std::vector<double> ghz;
  for (int i = 0; i < grid * WAVES; ++i) {
    const int b = i / WAVES, w = i % WAVES;
    ghz.push_back((double)h[2 * (b * 16 + w)] / (double)h[2 * (b * 16 + w) + 1] * 0.1);
  }
  std::sort(ghz.begin(), ghz.end());
  const double flop = mflop * TM * TN * (double)iters * grid * WAVES * reps;
  const double tf = flop / (ms * 1e-3) / 1e12;
  // reads per 16-cycle MFMA-equivalent (1024 FLOP/clk/SIMD either shape)
  const double rpm = READS ? (double)(READS == 3 ? TM : TM + TN) / (TM * TN) * (16.0 / S) : 0.0;
  const double ghz_med = ghz[ghz.size() / 2];
  printf("%-44s %7.1f TF  %.3f of 2.5PF  %.3f of issue@clk  clk %.3f GHz  reads/16cyc %.3f\n", name, tf, tf / 2500.0,
         tf / (1024.0 * 4 * 256 * ghz_med * 1e-3), ghz_med, rpm);
  fflush(stdout);
}

int main() {
  u4* in;
  float* out;
  unsigned long long* clk;
  hipMalloc(&in, 65536 * 16);
  hipMalloc(&out, 256 * 1024 * 4);
  hipMalloc(&clk, 256 * 16 * 16);
  std::vector<_Float16> h(65536 * 8);
  unsigned s = 12345;
  for (auto& v : h) {
    s = s * 1664525u + 1013904223u;
    v = (_Float16)(((int)(s >> 9) % 2001 - 1000) / 1000.0f);  // uniform [-1, 1]
  }
  hipMemcpy(in, h.data(), h.size() * 2, hipMemcpyHostToDevice);
  if (getenv("SHAPES_R5")) {  // round 5: weights in registers, pixels from LDS
    for (int pass = 0; pass < 2; ++pass) {
      printf("--- pass %d\n", pass);
      run<16, 2, 4, 2, 8>("16x16x32 lds 32x64/wave pref, 8w (c64d now)", in, out, clk);
      run<16, 4, 2, 3, 8>("16x16x32 A regs 64x32/wave, 8w", in, out, clk);
      run<16, 2, 2, 3, 8>("16x16x32 A regs 32x32/wave, 8w", in, out, clk);
      run<16, 4, 4, 3, 8>("16x16x32 A regs 64x64/wave, 8w", in, out, clk);
      run<16, 4, 4, 3, 4>("16x16x32 A regs 64x64/wave, 4w", in, out, clk);
      run<16, 8, 4, 3, 4>("16x16x32 A regs 128x64/wave, 4w", in, out, clk);
      run<16, 2, 4, 3, 4>("16x16x32 A regs 32x64/wave, 4w", in, out, clk);
      run<16, 4, 4, 0, 4>("16x16x32 regs 64x64/wave, 4w", in, out, clk);
    }
    return 0;
  }
  for (int pass = 0; pass < 2; ++pass) {
    printf("--- pass %d\n", pass);
    run<16, 4, 2, 0, 8>("16x16x32 regs 64x32/wave, 8w", in, out, clk);
    run<16, 4, 2, 2, 8>("16x16x32 lds 64x32/wave pref, 8w (current)", in, out, clk);
    run<16, 4, 4, 2, 8>("16x16x32 lds 64x64/wave pref, 8w", in, out, clk);
    run<16, 4, 4, 2, 4>("16x16x32 lds 64x64/wave pref, 4w", in, out, clk);
    run<16, 8, 4, 2, 4>("16x16x32 lds 128x64/wave pref, 4w", in, out, clk);
    run<16, 8, 4, 1, 4>("16x16x32 lds 128x64/wave, 4w", in, out, clk);
    run<32, 1, 1, 0, 8>("32x32x16 regs 32x32/wave, 8w", in, out, clk);
    run<32, 2, 1, 0, 8>("32x32x16 regs 64x32/wave, 8w", in, out, clk);
    run<32, 2, 1, 2, 8>("32x32x16 lds 64x32/wave pref, 8w", in, out, clk);
    run<32, 2, 1, 1, 8>("32x32x16 lds 64x32/wave, 8w", in, out, clk);
    run<32, 1, 1, 2, 8>("32x32x16 lds 32x32/wave pref, 8w (2/mfma)", in, out, clk);
    run<32, 2, 2, 2, 8>("32x32x16 lds 64x64/wave pref, 8w (1/mfma)", in, out, clk);
    run<32, 2, 2, 2, 4>("32x32x16 lds 64x64/wave pref, 4w (1/mfma)", in, out, clk);
    run<32, 4, 2, 2, 4>("32x32x16 lds 128x64/wave pref, 4w", in, out, clk);
    run<32, 2, 1, 2, 4>("32x32x16 lds 64x32/wave pref, 4w", in, out, clk);
  }
  return 0;
}
