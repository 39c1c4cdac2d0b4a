// Microbenchmark: sustained fp16 MFMA rate and the shader clock it runs at, on
// random operands, for (a) MFMAs from registers only and (b) the conv kernels'
// inner-loop shape (8 waves / CU, 16x16x32 MFMAs fed by ds_read_b128 from a
// swizzled LDS image, 0.75 or 0.5 reads per MFMA).  Clock = s_memtime ticks per
// s_memrealtime tick x 100 MHz, stamped by every wave around its loop
// (MI355X_MICROARCH.md 'DVFS give-back' item 6); each run lasts ~100 ms.
//
//   hipcc -O3 --offload-arch=gfx950 tools/ubench/mfma_clock.hip -o /tmp/mfma_clock && /tmp/mfma_clock
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));

// TM x TN accumulators per wave; READS = 0: operands stay in registers; 1: every
// k-group re-reads TM + TN fragments from LDS; 2: the same, one iteration ahead
template <int TM, int TN, int READS>
__global__ __launch_bounds__(512) void k(const u4* __restrict__ in, float* out, unsigned long long* clk, int iters) {
  __shared__ u4 lds[4096];  // 64 KB
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < 4096; i += 512) lds[i] = in[(blockIdx.x * 4096 + i) & 65535];
  __syncthreads();
  u4 fa[TN], fb[TM];
  for (int i = 0; i < TN; ++i) fa[i] = in[(tid * 7 + i) & 65535];
  for (int i = 0; i < TM; ++i) fb[i] = in[(tid * 13 + i + 5) & 65535];
  f32x4 acc[TM][TN];
  for (int i = 0; i < TM; ++i)
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0, 0, 0, 0};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  const int base = lane;  // 64 lanes x 16 B contiguous: conflict-free
  // READS = 2: the fragments of iteration it + 1 are read before iteration it's MFMAs
  u4 ga[TN], gb[TM];
  if (READS == 2) {
#pragma unroll
    for (int i = 0; i < TN; ++i) ga[i] = lds[(base + i * 256) & 4095];
#pragma unroll
    for (int i = 0; i < TM; ++i) gb[i] = lds[(base + 2048 + i * 256) & 4095];
  }
  for (int it = 0; it < iters; ++it) {
    if (READS == 1) {
#pragma unroll
      for (int i = 0; i < TN; ++i) fa[i] = lds[(base + i * 256 + it * 4) & 4095];
#pragma unroll
      for (int i = 0; i < TM; ++i) fb[i] = lds[(base + 2048 + i * 256 + it * 4) & 4095];
    }
    if (READS == 2) {
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        fa[i] = ga[i];
        ga[i] = lds[(base + i * 256 + it * 4 + 4) & 4095];
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        fb[i] = gb[i];
        gb[i] = lds[(base + 2048 + i * 256 + it * 4 + 4) & 4095];
      }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, fa[j]), __builtin_bit_cast(half8, fb[i]),
                                                         acc[i][j], 0, 0, 0);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  for (int i = 0; i < TM; ++i)
    for (int j = 0; j < TN; ++j) s += acc[i][j][0] + acc[i][j][3];
  out[blockIdx.x * 512 + tid] = s;
  if (lane == 0) {
    clk[2 * (blockIdx.x * 8 + (tid >> 6))] = t1 - t0;
    clk[2 * (blockIdx.x * 8 + (tid >> 6)) + 1] = r1 - r0;
  }
}

template <int TM, int TN, int READS>
void run(const char* name, const u4* in, float* out, unsigned long long* clk) {
  const int grid = 256 * 1;
  const int iters = 20000 / (TM * TN) * 16;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k<TM, TN, READS><<<grid, 512>>>(in, out, clk, iters);  // warm
  hipEventRecord(e0);
  const int reps = 20;
  for (int r = 0; r < reps; ++r) k<TM, TN, READS><<<grid, 512>>>(in, out, clk, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h(grid * 8 * 2);
  hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost);
  std::vector<double> ghz;
  for (int i = 0; i < grid * 8; ++i) ghz.push_back((double)h[2 * i] / (double)h[2 * i + 1] * 0.1);
  std::sort(ghz.begin(), ghz.end());
  const double flop = 2.0 * 16 * 16 * 32 * TM * TN * (double)iters * grid * 8 * reps;
  const double tf = flop / (ms * 1e-3) / 1e12;
  printf("%-34s %8.1f TFLOP/s  (%.3f of 2.5 PF)  clock median %.2f GHz  [%.2f, %.2f]  reads/MFMA %.2f\n", name, tf,
         tf / 2500.0, ghz[ghz.size() / 2], ghz.front(), ghz.back(), READS ? (double)(TM + TN) / (TM * TN) : 0.0);
}

int main() {
  u4* in;
  float* out;
  unsigned long long* clk;
  hipMalloc(&in, 65536 * 16);
  hipMalloc(&out, 256 * 512 * 4 * 2);
  hipMalloc(&clk, 256 * 8 * 16 * 2);
  std::vector<_Float16> h(65536 * 8);
  unsigned s = 12345;
  for (auto& v : h) {
    s = s * 1664525u + 1013904223u;
    v = (_Float16)(((int)(s >> 9) % 2001 - 1000) / 1000.0f);  // uniform [-1, 1]
  }
  hipMemcpy(in, h.data(), h.size() * 2, hipMemcpyHostToDevice);
  run<4, 4, 0>("regs 4x4 (16 acc)", in, out, clk);
  run<2, 4, 0>("regs 2x4 (8 acc)", in, out, clk);
  run<4, 2, 1>("lds 4x2 (0.75 reads/mfma)", in, out, clk);
  run<2, 2, 1>("lds 2x2 (1.0 reads/mfma)", in, out, clk);
  run<4, 4, 1>("lds 4x4 (0.5 reads/mfma)", in, out, clk);
  run<4, 2, 2>("lds 4x2 prefetched (0.75)", in, out, clk);
  run<4, 4, 2>("lds 4x4 prefetched (0.5)", in, out, clk);
  return 0;
}
