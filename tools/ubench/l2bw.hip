// Microbenchmark: per-CU load throughput into LDS from an L2/MALL-resident buffer
// (the weight/patch staging pattern of the conv kernels) vs from HBM.
//   mode 0: global_load_dwordx4 -> VGPR -> ds_write_b128 (register staging), DEPTH loads in flight/thread
//   mode 1: global_load_lds_dwordx4 (LDS-DMA), DEPTH instructions in flight per wave
// grid = 256 workgroups x NT threads; each workgroup streams BYTES_PER_WG from buffer
// offset (blockIdx % NSLICE) * slice, so the working set is NSLICE * slice.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned u4 __attribute__((ext_vector_type(4)));

template <int DEPTH>
__global__ __launch_bounds__(512) void regstage(const u4* __restrict__ src, size_t slice_u4, int nslice, int iters,
                                                unsigned* out) {
  __shared__ u4 lds[512 * DEPTH];
  const u4* s = src + (size_t)(blockIdx.x % nslice) * slice_u4;
  const int nt = blockDim.x;
  size_t off = threadIdx.x;
  u4 acc = {0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
    u4 v[DEPTH];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      v[d] = s[off];
      off += nt;
      if (off >= slice_u4) off -= slice_u4;
    }
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) lds[threadIdx.x + d * nt] = v[d];
  }
  __syncthreads();
  acc = lds[(threadIdx.x * 7) % (nt * DEPTH)];
  if (acc[0] == 0x12345678u) out[0] = acc[1];
}

template <int DEPTH>
__global__ __launch_bounds__(512) void ldsdma(const u4* __restrict__ src, size_t slice_u4, int nslice, int iters,
                                              unsigned* out) {
  __shared__ u4 lds[512 * DEPTH];
  const u4* s = src + (size_t)(blockIdx.x % nslice) * slice_u4;
  const int nt = blockDim.x;
  const int wave = threadIdx.x >> 6;
  size_t off = threadIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
#if defined(__HIP_DEVICE_COMPILE__)
      __builtin_amdgcn_global_load_lds(s + off, lds + wave * 64 + d * nt, 16, 0, 0);
#endif
      off += nt;
      if (off >= slice_u4) off -= slice_u4;
    }
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0) (gfx9 encoding: vmcnt low bits 0)
#endif
  }
  __syncthreads();
  u4 acc = lds[(threadIdx.x * 7) % (nt * DEPTH)];
  if (acc[0] == 0x12345678u) out[0] = acc[1];
}

template <typename K>
float timeit(K kern, int nt, const u4* src, size_t slice_u4, int nslice, int iters, unsigned* out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  kern<<<256, nt>>>(src, slice_u4, nslice, iters, out);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) kern<<<256, nt>>>(src, slice_u4, nslice, iters, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  const size_t total = 512ull << 20;  // 512 MB buffer
  u4* src;
  unsigned* out;
  hipMalloc(&src, total);
  hipMalloc(&out, 64);
  hipMemset(src, 1, total);
  struct Cfg {
    const char* name;
    size_t slice;  // bytes per slice
    int nslice;
  } cfgs[] = {{"L2-hot 1 MB shared", 1 << 20, 1},
              {"MALL 32 MB (8 slices x 4 MB)", 4 << 20, 8},
              {"HBM 512 MB (256 slices x 2 MB)", 2 << 20, 256}};
  for (auto& c : cfgs) {
    const size_t slice_u4 = c.slice / 16;
    for (int nt : {256, 512}) {
      const int depth = 8;
      const size_t bytes_per_wg_iter = (size_t)nt * 16 * depth;
      const int iters = (int)((c.slice * 2) / bytes_per_wg_iter);
      const double bytes = 256.0 * iters * bytes_per_wg_iter;
      float t0 = timeit(regstage<8>, nt, src, slice_u4, c.nslice, iters, out);
      auto kd = ldsdma<8>;
      float t1 = timeit(kd, nt, src, slice_u4, c.nslice, iters, out);
      printf("%-32s nt=%d depth=8: regstage %.2f TB/s (%.1f B/clk/CU @2.1GHz) | ldsdma %.2f TB/s (%.1f)\n", c.name, nt,
             bytes / t0 / 1e9, bytes / t0 / 1e-3 / 256 / 2.1e9, bytes / t1 / 1e9, bytes / t1 / 1e-3 / 256 / 2.1e9);
    }
  }
  hipFree(src);
  hipFree(out);
  return 0;
}
