// Microbenchmark: MFMA 16x16x32 f16 issue rate vs workgroup-barrier frequency.
// grid = 256 WGs x NW waves; each wave runs STEPS x (MPS MFMAs on 4 accumulators [+ s_barrier]).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int MPS, bool BAR>
__global__ void k(const half8* in, float* out, int steps) {
  half8 a = in[threadIdx.x & 63], b = in[(threadIdx.x + 7) & 63];
  f32x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  for (int s = 0; s < steps; ++s) {
#pragma unroll
    for (int i = 0; i < MPS / 4; ++i) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c3, 0, 0, 0);
    }
    if (BAR) __syncthreads();
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
}

template <int MPS, bool BAR>
float run(int nthreads, int steps, const half8* in, float* out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k<MPS, BAR><<<256, nthreads>>>(in, out, steps);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) k<MPS, BAR><<<256, nthreads>>>(in, out, steps);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  half8* in;
  float* out;
  hipMalloc(&in, 64 * sizeof(half8));
  hipMalloc(&out, 256 * 1024 * sizeof(float));
  std::vector<_Float16> h(64 * 8);
  for (int rnd = 0; rnd < 2; ++rnd) {
    for (size_t i = 0; i < h.size(); ++i) h[i] = rnd ? (_Float16)((int)(i * 2654435761u % 1000) / 500.0f - 1.0f) : (_Float16)0;
    hipMemcpy(in, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    const int steps = 720;
    for (int nw : {4, 8}) {
      double mf;
      float t;
      t = run<8, true>(nw * 64, steps, in, out);
      mf = 256.0 * nw * steps * 8;
      printf("%s waves=%d MPS=8  barrier: %8.1f us  %6.1f cyc/MFMA/SIMD @2.1GHz  %6.0f TF\n", rnd ? "rand" : "zero", nw, t * 1e3,
             t * 1e-3 * 2.1e9 / (mf / 1024), mf * 16384 / (t * 1e-3) / 1e12);
      t = run<8, false>(nw * 64, steps, in, out);
      printf("%s waves=%d MPS=8  none   : %8.1f us  %6.1f cyc/MFMA/SIMD  %6.0f TF\n", rnd ? "rand" : "zero", nw, t * 1e3,
             t * 1e-3 * 2.1e9 / (mf / 1024), mf * 16384 / (t * 1e-3) / 1e12);
      t = run<32, true>(nw * 64, steps / 4, in, out);
      printf("%s waves=%d MPS=32 barrier: %8.1f us  %6.1f cyc/MFMA/SIMD  %6.0f TF\n", rnd ? "rand" : "zero", nw, t * 1e3,
             t * 1e-3 * 2.1e9 / (mf / 1024), mf * 16384 / (t * 1e-3) / 1e12);
    }
  }
  return 0;
}
