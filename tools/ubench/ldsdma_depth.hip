// Microbenchmark: per-CU LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave-instruction)
// throughput from an L2-resident buffer against the number of DMAs each wave keeps in
// flight (the conv kernels' weight / patch staging: 8 waves per CU, every wave issuing).
// Each wave issues one DMA, then waits until at most D - 1 of its own are outstanding
// (s_waitcnt vmcnt(D - 1)), so D is the in-flight depth per wave: 8 waves x D KiB per CU.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench/ldsdma_depth.hip -o /tmp/ldsdma_depth && /tmp/ldsdma_depth
#include <hip/hip_runtime.h>

#include <cstdio>

template <int N>
__device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

template <int D>
__global__ __launch_bounds__(512) void stream(const char* __restrict__ src, unsigned slice, int iters, unsigned* out) {
  __shared__ __attribute__((aligned(1024))) char lds[64 * 1024];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nw = blockDim.x >> 6;
  unsigned off = (unsigned)((blockIdx.x * 4096u + threadIdx.x * 16u) % slice);
  for (int it = 0; it < iters; ++it) {
    char* dst = lds + ((it * nw + wave) & 63) * 1024;
    const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(__attribute__((address_space(3))) char*)dst);
    const char* p = src + off;
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(m0), "v"(p) : "memory", "m0");
    wait_vm<D - 1>();
    off += nw * 1024;
    if (off >= slice) off -= slice;
  }
  wait_vm<0>();
  __syncthreads();
  if (lds[lane * 16] == 123 && lds[lane * 16 + 1] == 45) out[0] = 1;
}

template <int D>
void run(const char* src, unsigned slice, unsigned* out, int nt) {
  const int iters = 4096;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  stream<D><<<256, nt>>>(src, slice, iters, out);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) stream<D><<<256, nt>>>(src, slice, iters, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= 5;
  const double bytes = 256.0 * (nt / 64) * iters * 1024.0;
  printf("slice %7u KB  waves %d  depth %2d (%3d KiB/CU in flight): %6.2f TB/s = %5.1f GB/s per CU\n", slice / 1024,
         nt / 64, D, D * nt / 64, bytes / ms / 1e9, bytes / ms / 1e6 / 256);
}

int main() {
  char* src;
  unsigned* out;
  hipMalloc(&src, 64 << 20);
  hipMalloc(&out, 64);
  hipMemset(src, 1, 64 << 20);
  for (unsigned slice : {1u << 20, 32u << 20}) {
    for (int nt : {256, 512}) {
      run<1>(src, slice, out, nt);
      run<2>(src, slice, out, nt);
      run<4>(src, slice, out, nt);
      run<8>(src, slice, out, nt);
      run<16>(src, slice, out, nt);
    }
  }
  return 0;
}
