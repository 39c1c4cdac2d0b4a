// Validation loss statistics on the device (perseus/detector/validate.py:162-168):
// over the flattened per-element SmoothL1 losses, mean, unbiased stdev (torch.std),
// min, max and torch.median (the lower middle element, sorted index (n - 1) / 2).
//
// Streaming HBM-bound passes, no host round trip:
//   1. moments: per-workgroup f64 sum + f32 min/max (grid-stride, 16-B loads), a
//      fixed-order final reduction -> mean; then a second pass sums (x - mean)^2 in
//      f64 (two-pass: no cancellation) -> stdev.  Deterministic (no float atomics).
//   2. median by radix select on order-preserving u32 keys, 4 passes of 8 bits:
//      per-workgroup LDS histogram of the keys matching the current prefix, merged
//      with integer atomics, then one workgroup picks the digit holding rank k.
// Workspace (pa_loss_statistics_workspace): partials + histogram + select state.
#include "common.h"

namespace pa {

namespace stats {
constexpr int NT = 256;
constexpr int MAXG = 512;
struct State {
  unsigned prefix, mask, k, pad;
  double mean;
};
struct Partial {
  double s;
  float mn, mx;
};
}  // namespace stats

__device__ __forceinline__ unsigned stat_key(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float stat_unkey(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// pass 0: sum, min, max; pass 1: sum of (x - mean)^2
template <int PASS>
__global__ __launch_bounds__(stats::NT) void stats_moments(const float* __restrict__ x, long long n,
                                                           stats::Partial* __restrict__ part,
                                                           const stats::State* __restrict__ st) {
  using namespace stats;
  __shared__ double ss[NT];
  __shared__ float smn[NT], smx[NT];
  const int tid = threadIdx.x;
  const double mean = PASS ? st->mean : 0.0;
  double s = 0.0;
  float mn = INFINITY, mx = -INFINITY;
  const long long n4 = n / 4;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  const bool aligned = ((size_t)x & 15) == 0;
  const long long stride = (long long)gridDim.x * NT;
  auto acc = [&](float v) {
    if constexpr (PASS == 0) {
      s += (double)v;
      mn = fminf(mn, v);
      mx = fmaxf(mx, v);
    } else {
      const double d = (double)v - mean;
      s += d * d;
    }
  };
  long long tail = 0;
  if (aligned) {
    for (long long i = blockIdx.x * (long long)NT + tid; i < n4; i += stride) {
      const float4 v = x4[i];
      acc(v.x);
      acc(v.y);
      acc(v.z);
      acc(v.w);
    }
    tail = n4 * 4;
  }
  for (long long i = tail + blockIdx.x * (long long)NT + tid; i < n; i += stride) acc(x[i]);
  ss[tid] = s;
  smn[tid] = mn;
  smx[tid] = mx;
  __syncthreads();
  for (int off = NT / 2; off > 0; off >>= 1) {  // fixed tree: deterministic
    if (tid < off) {
      ss[tid] += ss[tid + off];
      smn[tid] = fminf(smn[tid], smn[tid + off]);
      smx[tid] = fmaxf(smx[tid], smx[tid + off]);
    }
    __syncthreads();
  }
  if (tid == 0) part[blockIdx.x] = Partial{ss[0], smn[0], smx[0]};
}

// one workgroup: combine the G partials in index order
template <int PASS>
__global__ __launch_bounds__(64) void stats_combine(const stats::Partial* __restrict__ part, int G, long long n,
                                                    stats::State* __restrict__ st, double* __restrict__ out) {
  if (threadIdx.x != 0) return;
  double s = 0.0;
  float mn = INFINITY, mx = -INFINITY;
  for (int g = 0; g < G; ++g) {
    s += part[g].s;
    mn = fminf(mn, part[g].mn);
    mx = fmaxf(mx, part[g].mx);
  }
  if constexpr (PASS == 0) {
    const double mean = s / (double)n;
    st->mean = mean;
    out[0] = mean;
    out[2] = mn;
    out[3] = mx;
    st->prefix = 0;
    st->mask = 0;
    st->k = (unsigned)((n - 1) / 2);
  } else {
    out[1] = n > 1 ? sqrt(s / (double)(n - 1)) : NAN;  // torch.std: unbiased, NaN for one element
  }
}

__global__ __launch_bounds__(stats::NT) void stats_hist(const float* __restrict__ x, long long n, int shift,
                                                        const stats::State* __restrict__ st,
                                                        unsigned* __restrict__ hist) {
  using namespace stats;
  __shared__ unsigned h[256];
  const int tid = threadIdx.x;
  h[tid] = 0;
  __syncthreads();
  const unsigned prefix = st->prefix, mask = st->mask;
  for (long long i = blockIdx.x * (long long)NT + tid; i < n; i += (long long)gridDim.x * NT) {
    const unsigned k = stat_key(x[i]);
    if ((k & mask) == prefix) atomicAdd(&h[(k >> shift) & 255u], 1u);
  }
  __syncthreads();
  if (h[tid]) atomicAdd(&hist[tid], h[tid]);
}

// one workgroup: the digit whose bucket holds rank k; clears the histogram
__global__ __launch_bounds__(stats::NT) void stats_select(int shift, stats::State* __restrict__ st,
                                                          unsigned* __restrict__ hist, double* __restrict__ out) {
  __shared__ unsigned h[256];
  const int tid = threadIdx.x;
  h[tid] = hist[tid];
  hist[tid] = 0;
  __syncthreads();
  if (tid == 0) {
    unsigned k = st->k, d = 0;
    while (d < 255 && k >= h[d]) {
      k -= h[d];
      ++d;
    }
    st->k = k;
    st->prefix |= d << shift;
    st->mask |= 255u << shift;
    if (shift == 0) out[4] = (double)stat_unkey(st->prefix);
  }
}

static int stats_grid(long long n) {
  const long long g = (n + stats::NT * 4 - 1) / (stats::NT * 4);
  return (int)(g < 1 ? 1 : (g > stats::MAXG ? stats::MAXG : g));
}

size_t loss_statistics_workspace(long long n) {
  (void)n;
  return sizeof(stats::State) + stats::MAXG * sizeof(stats::Partial) + 256 * sizeof(unsigned) + 64;
}

int loss_statistics(const float* x, long long n, double* out, void* ws, size_t ws_bytes, hipStream_t s) {
  using namespace stats;
  PA_CHECK(n > 0, "loss statistics: empty input");
  PA_CHECK(x && out && ws, "loss statistics: null pointer");
  PA_CHECK(ws_bytes >= loss_statistics_workspace(n), "loss statistics: workspace %zu < %zu", ws_bytes,
           loss_statistics_workspace(n));
  PA_CHECK(((size_t)ws & 15) == 0, "loss statistics: workspace not 16-byte aligned");
  char* p = static_cast<char*>(ws);
  State* st = reinterpret_cast<State*>(p);
  Partial* part = reinterpret_cast<Partial*>(p + 32);
  unsigned* hist = reinterpret_cast<unsigned*>(p + 32 + MAXG * sizeof(Partial));
  const int G = stats_grid(n);
  PA_HIP(hipMemsetAsync(hist, 0, 256 * sizeof(unsigned), s));
  hipLaunchKernelGGL(stats_moments<0>, dim3(G), dim3(NT), 0, s, x, n, part, st);
  hipLaunchKernelGGL(stats_combine<0>, dim3(1), dim3(64), 0, s, part, G, n, st, out);
  hipLaunchKernelGGL(stats_moments<1>, dim3(G), dim3(NT), 0, s, x, n, part, st);
  hipLaunchKernelGGL(stats_combine<1>, dim3(1), dim3(64), 0, s, part, G, n, st, out);
  for (int shift = 24; shift >= 0; shift -= 8) {
    hipLaunchKernelGGL(stats_hist, dim3(G), dim3(NT), 0, s, x, n, shift, st, hist);
    hipLaunchKernelGGL(stats_select, dim3(1), dim3(NT), 0, s, shift, st, hist, out);
  }
  PA_LAUNCH_CHECK();
  return PA_OK;
}

}  // namespace pa

extern "C" {

size_t pa_loss_statistics_workspace(long long n) { return pa::loss_statistics_workspace(n); }

int pa_loss_statistics(const float* loss_dev, long long n, double* stats_dev, void* ws_dev, size_t ws_bytes,
                       void* stream) {
  return pa::loss_statistics(loss_dev, n, stats_dev, ws_dev, ws_bytes, (hipStream_t)stream);
}

}  // extern "C"
