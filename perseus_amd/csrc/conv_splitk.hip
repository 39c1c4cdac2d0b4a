// Split-K form of layers 2-4's convs for batches of a few frames (the streaming pose stage:
// one frame per camera per tick, SURVEY.md 8 configs[4]).
//
// At B = 3 the batched kernels (conv_gx.h, conv_s2x.h) give most CUs nothing to do: layer3
// runs 12 workgroups of a 36-step K loop, layer4 16 of 72 steps, so a launch takes as long
// as one workgroup's whole K loop (16-18 us) while the chip idles.  Here the K loop is cut
// into a.Cin / 64 splits of 9 steps (10 for a stride-2 entry: 9 taps + the downsample),
// grid.y = split, every split writes its f32 accumulators to a partial map, and
// splitk_reduce sums the splits in a fixed order (deterministic: same input, same bits) and
// applies the batched kernels' epilogue -- bias, residual, ReLU of models.py's BasicBlock
// convs (torchvision resnet18 via models.py:6-40).
//
// Opt-in per handle (pa_detector_set_split_k): the sum order differs from the
// single-pass kernels', so a split-K forward is not bit-identical to the batched one
// (both are within the fp16 path's error budget).
#include "conv_s2x.h"

namespace pa {

// lo / hi = sum_s part[s][e .. e + 7], s in order 0 .. nsplit - 1 (NS > 0: nsplit == NS, all
// loads issued first)
template <int NS>
__device__ __forceinline__ void splitk_sum(const float* __restrict__ part, int nsplit, unsigned n, unsigned e, f32x4& lo,
                                           f32x4& hi) {
  if constexpr (NS > 0) {
    f32x4 pl[NS], ph[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      pl[s] = *reinterpret_cast<const f32x4*>(part + (size_t)s * n + e);
      ph[s] = *reinterpret_cast<const f32x4*>(part + (size_t)s * n + e + 4);
    }
    lo = pl[0];
    hi = ph[0];
#pragma unroll
    for (int s = 1; s < NS; ++s) {
      lo += pl[s];
      hi += ph[s];
    }
  } else {
    lo = *reinterpret_cast<const f32x4*>(part + e);
    hi = *reinterpret_cast<const f32x4*>(part + e + 4);
    for (int s = 1; s < nsplit; ++s) {
      lo += *reinterpret_cast<const f32x4*>(part + (size_t)s * n + e);
      hi += *reinterpret_cast<const f32x4*>(part + (size_t)s * n + e + 4);
    }
  }
}

// out[p][c] = relu(sum_s part[s][p][c] + bias[c] (+ res[p][c])), 8 channels per thread,
// splits summed in order 0 .. nsplit-1.  With out2 (a stride-2 entry's downsample), the
// threads past n / 8 reduce the second partial set part[nsplit ..] into
// out2[p][c] = sum_s + bias2[c] (no ReLU).
// NS > 0: the split count at compile time -- every partial's loads are issued before the
// first add (with a runtime count the loop waited out one memory latency per split: ~5 us
// per launch at B = 3 whatever the split count); the sum order is the same.
template <int NS>
__global__ __launch_bounds__(256) void splitk_reduce(const float* __restrict__ part, int nsplit, unsigned n,
                                                     const float* __restrict__ bias, const _Float16* __restrict__ res,
                                                     _Float16* __restrict__ out, int Cout, const float* __restrict__ bias2,
                                                     _Float16* __restrict__ out2) {
  unsigned e = (blockIdx.x * 256 + threadIdx.x) * 8;
  const bool second = e >= n;
  if (second) {
    e -= n;
    if (!out2 || e >= n) return;
    part += (size_t)nsplit * n;
    bias = bias2;
    out = out2;
    res = nullptr;
  }
  const int c = (int)(e % (unsigned)Cout);
  f32x4 lo, hi;
  splitk_sum<NS>(part, nsplit, n, e, lo, hi);
  // the batched epilogue's order: (acc + bias) (+ res), then ReLU
  lo += *reinterpret_cast<const f32x4*>(bias + c);
  hi += *reinterpret_cast<const f32x4*>(bias + c + 4);
  half8 r{};
  if (res) r = *reinterpret_cast<const half8*>(res + e);
  half8 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float v0 = lo[j], v1 = hi[j];
    if (res) {
      v0 += (float)r[j];
      v1 += (float)r[j + 4];
    }
    o[j] = (_Float16)(second ? v0 : fmaxf(v0, 0.f));
    o[j + 4] = (_Float16)(second ? v1 : fmaxf(v1, 0.f));
  }
  *reinterpret_cast<half8*>(out + e) = o;
}

static int launch_reduce(const float* part, int nsplit, size_t n, const float* bias, const _Float16* res, _Float16* out,
                         int Cout, const float* bias2, _Float16* out2, hipStream_t s) {
  PA_CHECK(n % 8 == 0 && n < 0x40000000u && Cout % 8 == 0, "split-K reduce: %zu elements", n);
  const size_t threads = (out2 ? 2 * n : n) / 8;
  const dim3 g((unsigned)((threads + 255) / 256));
  switch (g_variant[7] == 5 ? 0 : nsplit) {  // (variant 7:5: the runtime-count loop, A/B)
    case 2: hipLaunchKernelGGL(splitk_reduce<2>, g, dim3(256), 0, s, part, nsplit, (unsigned)n, bias, res, out, Cout, bias2, out2); break;
    case 4: hipLaunchKernelGGL(splitk_reduce<4>, g, dim3(256), 0, s, part, nsplit, (unsigned)n, bias, res, out, Cout, bias2, out2); break;
    case 8: hipLaunchKernelGGL(splitk_reduce<8>, g, dim3(256), 0, s, part, nsplit, (unsigned)n, bias, res, out, Cout, bias2, out2); break;
    default: hipLaunchKernelGGL(splitk_reduce<0>, g, dim3(256), 0, s, part, nsplit, (unsigned)n, bias, res, out, Cout, bias2, out2);
  }
  PA_LAUNCH_CHECK();
  return PA_OK;
}

size_t splitk_part_floats(int B) {
  // per frame, nsplit * H * W * Cout is 2*32*32*128 = 4*16*16*256 = 8*8*8*512 = 262144 for every
  // stride-1 conv, and 2 maps * nsplit * H * W * Cout = 2*4*8*8*512 the same for layer4's entry
  return (size_t)B * 262144;
}

int launch_conv3x3_splitk(const ConvArgs& a, hipStream_t s, bool split_l2) {
  PA_CHECK(a.stride == 1 && a.pad == 1 && (a.epi == EPI_RELU || a.epi == (EPI_RELU | EPI_RES)),
           "split-K conv: stride-1, relu (+residual) only (epi %d)", a.epi);
  PA_CHECK(a.B <= 64, "split-K conv: batch %d above 64", a.B);
  if (a.B <= 0) return PA_OK;
  int rc;
  if (a.Cin == 64 && a.Cout == 64 && a.Hout == 64 && a.Wout == 64) {
    // layer1: the gx kernel on 8 x 16 tiles (4 waves, 9 steps, weights streamed per tap: 96
    // workgroups at B = 3) instead of the weight-resident persistent kernel, whose every
    // workgroup first stages all 73 KB of weights
    if (!split_l2) {
      // 4 x 16 tiles (192 workgroups at B = 3): 4.7-4.9 vs 5.7-5.9 us for 8 x 16 (profiles/r04sm/)
      if (g_variant[1] == 36) return run_gx<2, 16, 1, 64, 2, 2, 64, 3>(a, false, s);  // 2 x 16 tiles: 4.8-5.3 us
      if (g_variant[1] == 35) return run_gx<8, 16, 1, 64, 2, 2, 64, 3>(a, false, s);  // 8 x 16 tiles (A/B)
      return run_gx<4, 16, 1, 64, 2, 2, 64, 3>(a, false, s);
    }
    return launch_conv3x3_c64d(a, 0, s);
  }
  if (a.Cin == 128 && a.Cout == 128 && a.Hout == 32 && a.Wout == 32) {
    // layer2: no split -- the batched kernel's 8 x 16 tile form (gx variant 1, 4 waves, 18 steps:
    // 48 workgroups at B = 3), 9.7 us per forward faster than 2 splits + reduce
    // (profiles/r03aa/ab_l2.log) and bit-identical to the batched path
    // 2 x 16 tiles (192 workgroups at B = 3): 5.1-5.3 us, 4 x 16 5.8-6.1 (variant 1:36), 8 x 16
    // 7.4-7.7 (variant 1:35; profiles/r04sm/)
    if (!split_l2) return launch_conv3x3_gx_l2(a, g_variant[1] == 35 ? 1 : g_variant[1] == 36 ? 5 : 8, s);
    rc = run_gx_part<16, 16, 1, 64, 4, 2, 64, 3, 2>(a, s);
  } else if (a.Cin == 256 && a.Cout == 256 && a.Hout == 16 && a.Wout == 16)
    // 2 x 16 tiles (384 workgroups at B = 3): 8.6-8.7 us with the reduce, 4 x 16 8.8-8.9
    // (variant 3:35), 32-channel 4 x 16 9.4 (3:36), 8 x 16 9.9 (3:39), 16 x 16 11.4 (3:37;
    // profiles/r04sm/)
    if (g_variant[3] == 37)
      rc = run_gx_part<16, 16, 1, 64, 4, 2, 64, 3, 4>(a, s);
    else if (g_variant[3] == 39)
      rc = run_gx_part<8, 16, 1, 64, 2, 2, 64, 3, 4>(a, s);
    else if (g_variant[3] == 35)
      rc = run_gx_part<4, 16, 1, 64, 2, 2, 64, 3, 4>(a, s);
    else
      rc = run_gx_part<2, 16, 1, 64, 2, 2, 64, 3, 4>(a, s);
  else if (a.Cin == 512 && a.Cout == 512 && a.Hout == 8 && a.Wout == 8)
    // 4 x 8 tiles of 2 frames (256 workgroups at B = 3): 9.2 us with the reduce vs 9.9 for
    // 8 x 8 (variant 4:36), 9.2-9.3 for 32-channel 8 x 8 (4:39) and 10.0 for 32-channel 4 x 8
    // (profiles/r04sm/)
    rc = g_variant[4] == 36   ? run_gx_part<8, 8, 2, 64, 4, 2, 64, 3, 8>(a, s)
         : g_variant[4] == 39 ? run_gx_part<8, 8, 2, 32, 4, 1, 64, 3, 8>(a, s)
                              : run_gx_part<4, 8, 2, 64, 2, 2, 64, 3, 8>(a, s);
  else {
    set_error("split-K conv: no configuration for %dx%d x %d -> %d", a.Hout, a.Wout, a.Cin, a.Cout);
    return PA_EINVAL;
  }
  if (rc != PA_OK) return rc;
  return launch_reduce(a.part, a.Cin / 64, (size_t)a.B * a.Hout * a.Wout * a.Cout, a.bias,
                       (const _Float16*)((a.epi & EPI_RES) ? a.res : nullptr), (_Float16*)a.out, a.Cout, nullptr, nullptr, s);
}

// fp16x3 (conv_gx.h X3): out[p] = the (hi, lo) plane pair of relu(sum_s part[s][p][c] *
// scale[c] + bias[c] (+ res_hi + res_lo)), the batched X3 epilogue's operations on the
// split-order sum (the partials carry the weights' 2^e; the unscale is exact).  out / res
// are [pixel][hi (Cout) | lo (Cout)]; with out2 (stride-2 entry) the second partial set is
// the downsample: sum * scale2 + bias2, no ReLU.
template <int NS>
__global__ __launch_bounds__(256) void splitk_reduce_x3(const float* __restrict__ part, int nsplit, unsigned n,
                                                        const float* __restrict__ bias, const float* __restrict__ scale,
                                                        const _Float16* __restrict__ res, _Float16* __restrict__ out,
                                                        int Cout, const float* __restrict__ bias2,
                                                        const float* __restrict__ scale2, _Float16* __restrict__ out2) {
  unsigned e = (blockIdx.x * 256 + threadIdx.x) * 8;
  const bool second = e >= n;
  if (second) {
    e -= n;
    if (!out2 || e >= n) return;
    part += (size_t)nsplit * n;
    bias = bias2;
    scale = scale2;
    out = out2;
    res = nullptr;
  }
  const unsigned pix = e / (unsigned)Cout;
  const int c = (int)(e - pix * (unsigned)Cout);
  f32x4 lo, hi;
  splitk_sum<NS>(part, nsplit, n, e, lo, hi);
  const f32x4 b0 = *reinterpret_cast<const f32x4*>(bias + c), b1 = *reinterpret_cast<const f32x4*>(bias + c + 4);
  const f32x4 s0 = *reinterpret_cast<const f32x4*>(scale + c), s1 = *reinterpret_cast<const f32x4*>(scale + c + 4);
  const size_t o = (size_t)pix * 2 * Cout + c;
  half8 rh{}, rl{};
  if (res) {
    rh = *reinterpret_cast<const half8*>(res + o);
    rl = *reinterpret_cast<const half8*>(res + o + Cout);
  }
  half8 oh, ol;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float v = (j < 4 ? lo[j] : hi[j - 4]) * (j < 4 ? s0[j] : s1[j - 4]) + (j < 4 ? b0[j] : b1[j - 4]);
    if (res) v += (float)rh[j] + (float)rl[j];
    const HiLo hl = split_x3(second ? v : fmaxf(v, 0.f));
    oh[j] = hl.hi;
    ol[j] = hl.lo;
  }
  *reinterpret_cast<half8*>(out + o) = oh;
  *reinterpret_cast<half8*>(out + o + Cout) = ol;
}

static int launch_reduce_x3(const float* part, int nsplit, size_t n, const float* bias, const float* scale,
                            const _Float16* res, _Float16* out, int Cout, const float* bias2, const float* scale2,
                            _Float16* out2, hipStream_t s) {
  PA_CHECK(n % 8 == 0 && n < 0x40000000u && Cout % 8 == 0 && scale && (!out2 || scale2),
           "split-K reduce (fp16x3): %zu elements", n);
  const size_t threads = (out2 ? 2 * n : n) / 8;
  const dim3 g((unsigned)((threads + 255) / 256));
  switch (g_variant[7] == 5 ? 0 : nsplit) {
    case 2: hipLaunchKernelGGL(splitk_reduce_x3<2>, g, dim3(256), 0, s, part, nsplit, (unsigned)n, bias, scale, res, out, Cout, bias2, scale2, out2); break;
    case 4: hipLaunchKernelGGL(splitk_reduce_x3<4>, g, dim3(256), 0, s, part, nsplit, (unsigned)n, bias, scale, res, out, Cout, bias2, scale2, out2); break;
    case 8: hipLaunchKernelGGL(splitk_reduce_x3<8>, g, dim3(256), 0, s, part, nsplit, (unsigned)n, bias, scale, res, out, Cout, bias2, scale2, out2); break;
    default: hipLaunchKernelGGL(splitk_reduce_x3<0>, g, dim3(256), 0, s, part, nsplit, (unsigned)n, bias, scale, res, out, Cout, bias2, scale2, out2);
  }
  PA_LAUNCH_CHECK();
  return PA_OK;
}

// fp16x3 latency mode (the parity-grade streaming tick): the X3 forms of the convs above on
// small tiles, layers 2-4 split-K over the 64-channel input blocks (the merged x_hi steps,
// conv_gx.h XM, in every split) + splitk_reduce_x3.  Not bit-identical to the batched X3
// kernels (another f32 summation order); both stay within the 1e-3 px parity bar.
int launch_conv3x3_splitk_x3(const ConvArgs& a, hipStream_t s, const char** kname) {
  PA_CHECK(a.stride == 1 && a.pad == 1 && (a.epi == EPI_RELU || a.epi == (EPI_RELU | EPI_RES)) && a.scale,
           "split-K conv (fp16x3): stride-1, relu (+residual), scale required (epi %d)", a.epi);
  PA_CHECK(a.B <= 64, "split-K conv: batch %d above 64", a.B);
  if (a.B <= 0) return PA_OK;
  int rc;
  if (a.Cin == 64 && a.Cout == 64 && a.Hout == 64 && a.Wout == 64) {
    // layer1: one 64-channel block, nothing to split; 8 x 16 tiles (4 waves, 18 merged steps)
    if (kname) *kname = "conv3x3x3_l1_small";
    if (g_variant[1] == 36) return run_gx<8, 16, 1, 64, 2, 2, 64, 3, 1, 0, 1, true, true, true>(a, false, s);  // (A/B)
    return run_gx<4, 16, 1, 64, 2, 2, 64, 3, 1, 0, 1, true, true, true>(a, false, s);
  }
  if (a.Cin == 128 && a.Cout == 128 && a.Hout == 32 && a.Wout == 32) {
    if (kname) *kname = "conv3x3x3_l2_splitk";
    // (2 x 16 tiles: 14.2 vs 10.9 us; 32-channel 4 x 16: 11.1, profiles/r04sm/ab_l23s_x3.log)
    rc = g_variant[1] == 36 ? run_gx_part<8, 16, 1, 64, 2, 2, 64, 3, 2, true, true>(a, s)
                            : run_gx_part<4, 16, 1, 64, 2, 2, 64, 3, 2, true, true>(a, s);
  } else if (a.Cin == 256 && a.Cout == 256 && a.Hout == 16 && a.Wout == 16) {
    if (kname) *kname = "conv3x3x3_l3_splitk";
    // (2 x 16 tiles: 14.2 vs 10.9 us; 32-channel 4 x 16: 11.0)
    rc = g_variant[1] == 36 ? run_gx_part<8, 16, 1, 64, 2, 2, 64, 3, 4, true, true>(a, s)
                            : run_gx_part<4, 16, 1, 64, 2, 2, 64, 3, 4, true, true>(a, s);
  } else if (a.Cin == 512 && a.Cout == 512 && a.Hout == 8 && a.Wout == 8) {
    if (kname) *kname = "conv3x3x3_l4_splitk";
    // 32-channel 8 x 8 tiles of 2 frames (256 workgroups at B = 3): 11.1-11.2 us with the reduce
    // vs 12.5-12.7 for 64 channels (variant 4:36) and 11.4-11.5 for 4 x 8 (4:38; profiles/r04sm/)
    // (32-channel 4 x 8: 11.5)
    rc = g_variant[4] == 36   ? run_gx_part<8, 8, 2, 64, 4, 2, 64, 3, 8, true, true>(a, s)
         : g_variant[4] == 38 ? run_gx_part<4, 8, 2, 64, 2, 2, 64, 3, 8, true, true>(a, s)
                              : run_gx_part<8, 8, 2, 32, 4, 1, 64, 3, 8, true, true>(a, s);
  } else {
    set_error("split-K conv (fp16x3): no configuration for %dx%d x %d -> %d", a.Hout, a.Wout, a.Cin, a.Cout);
    return PA_EINVAL;
  }
  if (rc != PA_OK) return rc;
  return launch_reduce_x3(a.part, a.Cin / 64, (size_t)a.B * a.Hout * a.Wout * a.Cout, a.bias, a.scale,
                          (const _Float16*)((a.epi & EPI_RES) ? a.res : nullptr), (_Float16*)a.out, a.Cout, nullptr,
                          nullptr, nullptr, s);
}

int launch_conv3x3s2_small_x3(const ConvS2Args& a, hipStream_t s, const char** kname) {
  PA_CHECK(a.B <= 64, "split-K conv: batch %d above 64", a.B);
  if (a.B <= 0) return PA_OK;
  if (a.Hout == 32 && a.Cin == 64 && a.Cout == 128) {
    // one input-channel block: unsplit, 64-channel tiles on 4 waves (B = 3: 96 workgroups of 30 steps)
    if (kname) *kname = "conv3x3s2x3_l2_small";
    // 2 x 16 tiles (192 workgroups at B = 3): 8.2 vs 10.5 us for 4 x 16 (variant 2:37, profiles/r04sm/)
    if (g_variant[2] == 37) return run_s2x<4, 16, 64, 2, 2, 64, 3, 1, true, true>(a, false, s);
    return run_s2x<2, 16, 64, 2, 2, 64, 3, 1, true, true>(a, false, s);
  }
  int rc, ns;
  if (a.Hout == 16 && a.Cin == 128 && a.Cout == 256) {
    if (kname) *kname = "conv3x3s2x3_l3_splitk";
    ns = 2;
    // 2 x 16 tiles: 11.9 vs 14.2 us with the reduce for 4 x 16 (variant 3:37)
    rc = g_variant[3] == 37 ? run_s2x_part<4, 16, 64, 2, 2, 64, 3, 2, true>(a, s)
                            : run_s2x_part<2, 16, 64, 2, 2, 64, 3, 2, true>(a, s);
  } else if (a.Hout == 8 && a.Cin == 256 && a.Cout == 512) {
    if (kname) *kname = "conv3x3s2x3_l4_splitk";
    ns = 4;
    // 4 x 8 tiles: 11.7 vs 14.1 us with the reduce for 8 x 8 (variant 4:37)
    rc = g_variant[4] == 37 ? run_s2x_part<8, 8, 64, 2, 2, 64, 3, 4, true>(a, s)
                            : run_s2x_part<4, 8, 64, 2, 2, 64, 3, 4, true>(a, s);
  } else {
    set_error("s2x3 small batch: no configuration for %dx%d x %d -> %d", a.Hout, a.Wout, a.Cin, a.Cout);
    return PA_EINVAL;
  }
  if (rc != PA_OK) return rc;
  return launch_reduce_x3(a.part, ns, (size_t)a.B * a.Hout * a.Wout * a.Cout, a.bias, a.scale, nullptr,
                          (_Float16*)a.out, a.Cout, a.bias2, a.scale2, (_Float16*)a.out2, s);
}

int launch_conv3x3s2_small(const ConvS2Args& a, hipStream_t s, const char** kname) {
  PA_CHECK(a.B <= 64, "split-K conv: batch %d above 64", a.B);
  if (a.B <= 0) return PA_OK;
  if (a.Hout == 32 && a.Cin == 64 && a.Cout == 128) {
    // one input-channel block, nothing to split: one 4x16 tile per workgroup (B = 3: 96
    // workgroups of 10 steps, 6.5 us; the batched kernel runs 12 workgroups of 4 tiles, 40
    // steps, 17.8 us)
    if (kname) *kname = "conv3x3s2x_l2_small";
    // 2 x 16 tiles (192 workgroups at B = 3): 4.7 vs 5.8 us for 4 x 16 (variant 2:37, profiles/r04sm/)
    if (g_variant[2] == 37) return run_s2x<4, 16, 64, 2, 2, 64, 3>(a, false, s);
    return run_s2x<2, 16, 64, 2, 2, 64, 3>(a, false, s);
  }
  if (a.Hout == 8 && a.Cin == 256 && a.Cout == 512) {
    if (kname) *kname = "conv3x3s2x_l4_splitk";
    // 4 x 8 tiles: 8.6 vs 10.0 us with the reduce for 8 x 8 (variant 4:37)
    const int rc = g_variant[4] == 37 ? run_s2x_part<8, 8, 64, 2, 2, 64, 3, 4>(a, s)
                                      : run_s2x_part<4, 8, 64, 2, 2, 64, 3, 4>(a, s);
    if (rc != PA_OK) return rc;
    return launch_reduce(a.part, 4, (size_t)a.B * 64 * 512, a.bias, nullptr, (_Float16*)a.out, 512, a.bias2,
                         (_Float16*)a.out2, s);
  }
  set_error("s2x small batch: no configuration for %dx%d x %d -> %d", a.Hout, a.Wout, a.Cin, a.Cout);
  return PA_EINVAL;
}

}  // namespace pa
