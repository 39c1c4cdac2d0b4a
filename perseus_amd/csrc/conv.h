// Launchers for the detector kernels (conv.hip).  Precision is a template
// parameter everywhere: T = _Float16 (fast path) or float (parity path).
#pragma once
#include "common.h"

namespace pa {

// EPI_HEAD (layer4's last conv, conv_gx.h): avgpool + fc in the epilogue instead of the
// activation store (models.py:31-32)
enum { EPI_RELU = 1, EPI_RES = 2, EPI_HEAD = 4 };
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// Kernel-variant selector per layer (A/B timing; 0 = shipped) and the timestamp buffer
// of the tracing variants (launch i of a forward gets g_trace + i * TRACE_LAUNCH;
// nullptr = off).  Both belong to a pa_detector handle (pa_detector_debug_set_variant /
// _set_trace, include/perseus_amd_debug.h): a forward points these thread-locals at its
// handle's settings for the duration of the call, so handles never see each other's.
extern thread_local const int* g_variant;
extern thread_local unsigned long long* g_trace;
constexpr int TRACE_SLOTS = 64, TRACE_LAUNCH = 65536;

// 16-byte store at byte offset `off` from the wave-uniform base `base`; WT = write-through
// (sc1: the line goes on to memory now instead of sitting dirty in this XCD's L2
// until the end-of-kernel write-back)
template <bool WT>
__device__ __forceinline__ void store16(void* base, unsigned off, half8 v) {
  if constexpr (WT) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, (int)off, 0, 16);
  } else {
    *reinterpret_cast<half8*>((char*)base + off) = v;
  }
}

// one s_memrealtime stamp per workgroup (thread 0) into slot `slot`
__device__ __forceinline__ void trace_stamp(unsigned long long* tr, int slot) {
  if (threadIdx.x == 0 && slot < TRACE_SLOTS) tr[(blockIdx.y * gridDim.x + blockIdx.x) * TRACE_SLOTS + slot] = __builtin_amdgcn_s_memrealtime();
}

struct ConvArgs {
  const void* in;     // NHWC [B][Hin][Win][Cin]
  const void* w;      // [Cout][KS][KS][Cin], BatchNorm folded
  const float* bias;  // [Cout], BatchNorm folded
  const float* scale; // fp16x3 only: [Cout] 2^-e, unscales the accumulator (weights hold w * 2^e)
  const void* res;    // NHWC [B][Hout][Wout][Cout] or nullptr
  void* out;          // NHWC [B][Hout][Wout][Cout]
  int B, Hin, Win, Cin, Hout, Wout, Cout, stride, pad, epi, M;
  unsigned long long* trace;  // timing-only variants: s_memrealtime stamps, TRACE_SLOTS per workgroup
  // EPI_HEAD only: pooled means [B][Cout] f32, per-image-pair arrival counters (zero
  // between launches), fc weight [16][Cout] / bias [16], keypoints out [B][16]
  float* pool;
  unsigned* cnt;
  const float* fcw;
  const float* fcb;
  float* y;
  // split-K mode (conv_gx.h PART, small batches): f32 partial sums [split][B][Hout][Wout][Cout],
  // split = blockIdx.y over the input-channel blocks
  float* part;
};

// conv3x3 s2 (+bn, relu) -> out and 1x1 s2 downsample (+bn) -> out2, one pass
struct ConvS2Args {
  const void* in;      // NHWC [B][Hin][Win][Cin]
  const void* w;       // [Cout][3][3][Cin]
  const float* bias;   // [Cout]
  const void* wds;     // [Cout][Cin]
  const float* bias2;  // [Cout]
  const float* scale;  // fp16x3 only: [Cout] 2^-e of w / wds
  const float* scale2;
  void* out;           // NHWC [B][Hout][Wout][Cout]
  void* out2;          // NHWC [B][Hout][Wout][Cout]
  int B, Hin, Win, Cin, Hout, Wout, Cout;
  unsigned long long* trace;  // as ConvArgs::trace
  // split-K mode (conv_s2x.h PART): f32 partials [2][split][B][Hout][Wout][Cout] (conv, then downsample)
  float* part;
  // conv_s2v.hip (the layer2 entry, 64 -> 128): conv + downsample weights in VGPR-fragment order
  // (pa_detector build: [wave 4][fragment 20][tile 2][lane 64][8 fp16])
  const void* wfrag;
};

template <typename T>
int launch_conv3x3s2_ds(const ConvS2Args& a, hipStream_t s, const char** kname);


// fp16, LDS-DMA deep ring (conv_s2x.h, conv_s2x_l.hip), layers 2-4
int launch_conv3x3s2_x(const ConvS2Args& a, int variant, hipStream_t s, const char** kname);
// fp16, 8 x 16 x 128 tiles with the row-split patch (conv_s2w.h), layers 2-3 (shipped there)
int launch_conv3x3s2_w(const ConvS2Args& a, int variant, hipStream_t s, const char** kname);
// fp16 layer2 entry (Cin 64 -> 128) with the weights in VGPRs (conv_s2v.hip; shipped from round 6)
int launch_conv3x3s2_v(const ConvS2Args& a, int variant, hipStream_t s, const char** kname);

template <typename T>
int launch_conv(const ConvArgs& a, int ks, hipStream_t s, const char** kname);

template <typename T>
int launch_conv3x3_s1(const ConvArgs& a, hipStream_t s, const char** kname);


// 3x3 s1, fp16, LDS-DMA with a deep weight ring, fully unrolled (conv_gx.h, conv_gx_l*.hip)
int launch_conv3x3_gx_l2(const ConvArgs& a, int variant, hipStream_t s);
int launch_conv3x3_gx_l3(const ConvArgs& a, int variant, hipStream_t s);
int launch_conv3x3_gx_l4(const ConvArgs& a, int variant, hipStream_t s);
// the same convs split-K + a fixed-order reduce (small batches, conv_splitk.hip): a.part
// holds splitk_part_floats(B) floats
// (layer2 runs unsplit on small tiles unless split_l2, the A/B form)
int launch_conv3x3_splitk(const ConvArgs& a, hipStream_t s, bool split_l2 = false);
// stride-2 block entries for small batches: layer2 on one-tile workgroups, layer4 split-K with
// the conv and the downsample reduced in one pass (layer3's batched kernel is kept)
int launch_conv3x3s2_small(const ConvS2Args& a, hipStream_t s, const char** kname);
size_t splitk_part_floats(int B);
// fp16x3 latency mode: the X3 forms (conv_splitk.hip; same partials buffer)
int launch_conv3x3_splitk_x3(const ConvArgs& a, hipStream_t s, const char** kname);
int launch_conv3x3s2_small_x3(const ConvS2Args& a, hipStream_t s, const char** kname);
int launch_stem_pool_x3_small(const float* x, int B, int Cin, const _Float16* w, const float* bias_s,
                              const float* scale, _Float16* out, hipStream_t s);

// layer1 (Cin = Cout = 64), fp16: weight-resident persistent kernel (conv_c64.hip)
int launch_conv3x3_c64(const ConvArgs& a, int variant, hipStream_t s);
// the same with LDS-DMA staging spread through the K loop (conv_c64d.hip)
int launch_conv3x3_c64d(const ConvArgs& a, int variant, hipStream_t s);
int launch_conv3x3_c64v(const ConvArgs& a, int variant, hipStream_t s);
// CUs a launch on stream s may use (its CU mask, else the device's): persistent grids size by it
int conv_stream_cus(hipStream_t s);


template <typename T>
int launch_stem(const float* x, int B, int Cin, const T* w, const float* bias, T* out, hipStream_t s);

// raw camera frames for the fused-preprocess stem (streaming.py:68-80; conv.hip
// preprocess_kernel's arithmetic): uint8 HWC RGB/BGR + f32 depth [B][Hs][Ws], centre
// crop to 256x256, near/far clip disabled when < 0
struct RgbdSrc {
  const uint8_t* rgb;
  const float* depth;
  int Hs, Ws, bgr;
  float near_m, far_m;
};
int launch_stem_pool_rgbd(const RgbdSrc& src, int B, const _Float16* w, const float* bias, _Float16* out,
                          hipStream_t s);
int launch_stem_pool_fp16(const float* x, int B, int Cin, const _Float16* w, const float* bias, _Float16* out,
                          hipStream_t s);

// fp16x3 parity mode (stem_x3.hip, conv_x3_*.hip, conv.hip head_x3): activations are
// [hi (C) | lo (C)] fp16 plane pairs per pixel, weights hi/lo planes of w * 2^e
int launch_stem_pool_x3(const float* x, int B, int Cin, const _Float16* w, const float* bias_s, const float* scale,
                        _Float16* out, hipStream_t s);
int launch_conv3x3_x3_l1(const ConvArgs& a, hipStream_t s);
int launch_conv3x3_x3v(const ConvArgs& a, hipStream_t s);
int launch_conv3x3_x3_l2(const ConvArgs& a, hipStream_t s);
int launch_conv3x3_x3_l3(const ConvArgs& a, hipStream_t s);
int launch_conv3x3_x3_l4(const ConvArgs& a, hipStream_t s);
int launch_conv3x3s2_x3(const ConvS2Args& a, hipStream_t s, const char** kname);
// px (optional): the keypoints also denormalized to an H x W image (launch_postprocess's values)
int launch_head_x3(const _Float16* in, int B, int HW, int C, const float* fcw, const float* fcb, int nout, float* y,
                   hipStream_t s, float* px = nullptr, int H = 0, int W = 0);

template <typename T>
int launch_maxpool(const T* in, int B, int H, int W, int C, T* out, hipStream_t s);

// px (optional): also the keypoints denormalized to an H x W image (launch_postprocess's values)
template <typename T>
int launch_head(const T* in, int B, int HW, int C, const float* fcw, const float* fcb, int nout, float* y,
                hipStream_t s, float* px = nullptr, int H = 0, int W = 0);

int launch_preprocess(const uint8_t* rgb, const float* depth, int B, int Hs, int Ws, int bgr, float near_m,
                      float far_m, int H, int W, float* x, hipStream_t s);
int launch_postprocess(const float* y, const float* target, int B, int n_kp, int H, int W, float* px,
                       float* loss, hipStream_t s);

}  // namespace pa
