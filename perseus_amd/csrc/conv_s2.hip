// Stride-2 BasicBlock entry conv with the 1x1 stride-2 downsample fused in
// (torchvision resnet18 layer2/3/4 block 0: conv1 3x3 s2 + bn1 + relu, and
// downsample = conv1x1 s2 + bn).
//
// The downsample reads input pixel (2y, 2x), which is exactly the centre tap of
// the 3x3 stride-2 window of output (y, x), so it costs one extra weight tile
// and MFMA set per channel block on the patch that is already in LDS — the
// input is read once for both outputs.
//
// Patch: (2TH+1) x (2TW+1) input pixels per image, columns stored de-interleaved
// (even input columns first, then odd) so that the stride-2 window of 16
// consecutive output columns reads 16 consecutive LDS pixels for every tap
// (conflict-free with the frag_off lane map and the (p>>1)&7 swizzle, as in
// conv_patch.hip).  Weights stream per tap (3 register sets, LDS ring of 2),
// the downsample tile is loaded at tap 1 and staged at tap 3 of each channel
// block; one patch buffer (refilled at channel-block boundaries from registers
// prefetched during the block).
#include <type_traits>

#include "conv.h"

namespace pa {

typedef unsigned s2u4 __attribute__((ext_vector_type(4)));

template <int V>
using sc = std::integral_constant<int, V>;

template <typename T>
struct SElem;
template <>
struct SElem<_Float16> {
  static constexpr int KB = 64;
};
template <>
struct SElem<float> {
  static constexpr int KB = 32;
};

__device__ __forceinline__ int s2swz(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }
__device__ __forceinline__ int s2frag_off(int r) { return r < 4 ? 2 * r : (r < 12 ? 2 * (r - 4) + 1 : 2 * (r - 8)); }

template <typename T>
__device__ __forceinline__ void s2mma(f32x4& acc, const s2u4& a, const s2u4& b);
template <>
__device__ __forceinline__ void s2mma<_Float16>(f32x4& acc, const s2u4& a, const s2u4& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, a), __builtin_bit_cast(half8, b), acc, 0, 0,
                                               0);
}
template <>
__device__ __forceinline__ void s2mma<float>(f32x4& acc, const s2u4& a, const s2u4& b) {
  f32x4 fa = __builtin_bit_cast(f32x4, a), fb = __builtin_bit_cast(f32x4, b);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[0], fb[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[1], fb[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[2], fb[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[3], fb[3], acc, 0, 0, 0);
}

template <typename T>
struct S2R4;
template <>
struct S2R4<_Float16> {
  typedef half4 type;
};
template <>
struct S2R4<float> {
  typedef f32x4 type;
};

template <typename T, int TH, int TW, int NI, int BN, int WM, int WN, int CIN>
__global__ __launch_bounds__(WM* WN * 64) void conv3x3s2_ds(ConvS2Args a) {
  constexpr int NT = WM * WN * 64;
  constexpr int KB = SElem<T>::KB;
  constexpr int CPR = 16 / sizeof(T);
  constexpr int NCB = CIN / KB;
  constexpr int NSTEPS = NCB * 9;
  constexpr int KTOT = 9 * CIN;
  constexpr int PH = 2 * TH + 1, PW = 2 * TW + 1;  // PW = LDS positions per patch row
  constexpr int IMS = (TW == 8) ? ((PH * PW + 7) / 16 * 16 + 8) : PH * PW;
  constexpr int NP = NI * IMS;
  constexpr int BM = NI * TH * TW;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int PCH = (NP * 8 + NT - 1) / NT;
  constexpr int BCH = BN * 8 / NT;
  constexpr int PATCHB = NP * 128;
  constexpr int WB = BN * 128;
  static_assert(BN * 8 % NT == 0, "weight tile / threads");
  static_assert(WTM % 16 == 0 && WTN % 16 == 0, "wave tile");
  static_assert(TW >= 16 || (TW == 8 && NI == 2), "fragment geometry");
  __shared__ __attribute__((aligned(16))) char smem[PATCHB + 3 * WB];
  char* patch = smem;
  char* wbuf = smem + PATCHB;       // 2 tap buffers
  char* dsbuf = smem + PATCHB + 2 * WB;  // downsample tile of the current block

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int q = lane >> 4, r16 = lane & 15;
  const int H = a.Hout, W = a.Wout, Hin = a.Hin, Win = a.Win;
  const int Cout = a.Cout;
  const T* __restrict__ in = (const T*)a.in;
  const T* __restrict__ w = (const T*)a.w;
  const T* __restrict__ wds = (const T*)a.wds;

  const int ntn = Cout / BN;
  const int tn_idx = blockIdx.x % ntn;
  const int sp = blockIdx.x / ntn;
  const int tw_n = W / TW, tpi = (H / TH) * tw_n;
  const int img0 = (sp / tpi) * NI;
  const int rem = sp - (sp / tpi) * tpi;
  const int th0 = (rem / tw_n) * TH, tw0 = (rem - (rem / tw_n) * tw_n) * TW;
  const int n0 = tn_idx * BN;

  s2u4 rp[PCH];
  s2u4 rb[3][BCH];
  s2u4 rds[BCH];
  auto load_patch = [&](int cb) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < PCH; ++i) {
      const int c = tid + i * NT;
      s2u4 v = s2u4{0u, 0u, 0u, 0u};
      if (c < NP * 8) {
        const int p = c >> 3, ch = c & 7;
        const int img = p / IMS, pp = p - (p / IMS) * IMS;
        const int pr = pp / PW, pos = pp - (pp / PW) * PW;
        const int col = pos <= TW ? 2 * pos : 2 * (pos - TW - 1) + 1;  // de-interleaved columns
        const int n = img0 + img, h = 2 * th0 - 1 + pr, x = 2 * tw0 - 1 + col;
        if (pr < PH && n < a.B && (unsigned)h < (unsigned)Hin && (unsigned)x < (unsigned)Win)
          v = *reinterpret_cast<const s2u4*>(in + (((size_t)n * Hin + h) * Win + x) * CIN + cb * KB + ch * CPR);
      }
      rp[i] = v;
    }
  };
  auto store_patch = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < PCH; ++i) {
      const int c = tid + i * NT;
      if (c < NP * 8) *reinterpret_cast<s2u4*>(patch + s2swz(c >> 3, c & 7)) = rp[i];
    }
  };
  auto load_w = [&](int s, auto setc) __attribute__((always_inline)) {
    constexpr int SET = decltype(setc)::value;
    s = s < NSTEPS ? s : NSTEPS - 1;
    const int cb = s / 9, tap = s - (s / 9) * 9;
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int c = tid + i * NT;
      rb[SET][i] = *reinterpret_cast<const s2u4*>(w + (size_t)(n0 + (c >> 3)) * KTOT + tap * CIN + cb * KB + (c & 7) * CPR);
    }
  };
  auto store_w = [&](int buf, auto setc) __attribute__((always_inline)) {
    constexpr int SET = decltype(setc)::value;
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int c = tid + i * NT;
      *reinterpret_cast<s2u4*>(wbuf + buf * WB + s2swz(c >> 3, c & 7)) = rb[SET][i];
    }
  };
  auto load_ds = [&](int cb) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int c = tid + i * NT;
      rds[i] = *reinterpret_cast<const s2u4*>(wds + (size_t)(n0 + (c >> 3)) * CIN + cb * KB + (c & 7) * CPR);
    }
  };
  auto store_ds = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int c = tid + i * NT;
      *reinterpret_cast<s2u4*>(dsbuf + s2swz(c >> 3, c & 7)) = rds[i];
    }
  };

  // lane -> output pixel and its patch position for tap (0,0)
  const int o = s2frag_off(r16);
  int ppix[TM];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int mb = wm * WTM + tm * 16;
    if constexpr (TW == 8) {
      ppix[tm] = (o >> 3) * IMS + (2 * (mb / 16)) * PW + (o & 7);
    } else {
      ppix[tm] = (mb / (TH * TW)) * IMS + (2 * ((mb / TW) % TH)) * PW + mb % TW + o;
    }
  }

  f32x4 acc[TM][TN], accd[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      accd[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

  load_patch(0);
  load_w(0, sc<0>{});
  load_ds(0);
  store_patch();
  store_w(0, sc<0>{});
  store_ds();
  load_w(1, sc<1>{});
  load_w(2, sc<2>{});
  __syncthreads();

  auto step = [&](int cb, auto tapc) __attribute__((always_inline)) {
    constexpr int TAP = decltype(tapc)::value;
    constexpr int KR = TAP / 3, KC = TAP % 3;
    // stride-2 tap -> LDS position offset in the de-interleaved row
    constexpr int COL = KC == 0 ? 0 : (KC == 1 ? TW + 1 : 1);
    const int s = cb * 9 + TAP;
    load_w(s + 3, sc<TAP % 3>{});
    if constexpr (TAP == 0 && NCB > 1) load_patch(cb + 1 < NCB ? cb + 1 : NCB - 1);
    if constexpr (TAP == 1 && NCB > 1) load_ds(cb + 1 < NCB ? cb + 1 : NCB - 1);
    const char* wb = wbuf + (s & 1) * WB;
    s2u4 fa[2][TN], fb[2][TM], fd[2][TN];
#pragma unroll
    for (int g = 0; g < 2; ++g) {
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        fa[g][tn] = *reinterpret_cast<const s2u4*>(wb + s2swz(wn * WTN + tn * 16 + r16, g * 4 + q));
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
        fb[g][tm] = *reinterpret_cast<const s2u4*>(patch + s2swz(ppix[tm] + KR * PW + COL, g * 4 + q));
      if constexpr (TAP == 4) {
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          fd[g][tn] = *reinterpret_cast<const s2u4*>(dsbuf + s2swz(wn * WTN + tn * 16 + r16, g * 4 + q));
      }
    }
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
          s2mma<T>(acc[tm][tn], fa[g][tn], fb[g][tm]);
          if constexpr (TAP == 4) s2mma<T>(accd[tm][tn], fd[g][tn], fb[g][tm]);  // centre tap = 1x1 s2 input
        }
    store_w((s + 1) & 1, sc<(TAP + 1) % 3>{});
    if constexpr (NCB > 1 && TAP == 8) {
      __syncthreads();  // every wave is done with the patch and the ds tile
      if (cb + 1 < NCB) {
        store_patch();
        store_ds();
      }
    }
    __syncthreads();
  };
  for (int cb = 0; cb < NCB; ++cb) {
    step(cb, sc<0>{});
    step(cb, sc<1>{});
    step(cb, sc<2>{});
    step(cb, sc<3>{});
    step(cb, sc<4>{});
    step(cb, sc<5>{});
    step(cb, sc<6>{});
    step(cb, sc<7>{});
    step(cb, sc<8>{});
  }

  // epilogue: conv1 -> relu -> out; downsample -> out2 (no relu), from registers
  typedef typename S2R4<T>::type R4;
  T* __restrict__ out = (T*)a.out;
  T* __restrict__ out2 = (T*)a.out2;
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int mb = wm * WTM + tm * 16;
    int img, y, x;
    if constexpr (TW == 8) {
      y = mb / 16;
      img = o >> 3;
      x = o & 7;
    } else {
      img = mb / (TH * TW);
      y = (mb / TW) % TH;
      x = mb % TW + o;
    }
    const int n = img0 + img;
    if (n >= a.B) continue;
    const size_t pix = (((size_t)n * H + th0 + y) * W + tw0 + x) * Cout;
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int co = n0 + wn * WTN + tn * 16 + q * 4;
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(a.bias + co);
      const f32x4 b2 = *reinterpret_cast<const f32x4*>(a.bias2 + co);
      R4 v1, v2;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v1[j] = (T)fmaxf(acc[tm][tn][j] + b1[j], 0.f);
        v2[j] = (T)(accd[tm][tn][j] + b2[j]);
      }
      *reinterpret_cast<R4*>(out + pix + co) = v1;
      *reinterpret_cast<R4*>(out2 + pix + co) = v2;
    }
  }
}

template <typename T, int TH, int TW, int NI, int BN, int WM, int WN, int CIN>
static int run_s2(const ConvS2Args& a, hipStream_t s) {
  PA_CHECK(a.Cin == CIN, "s2 conv: Cin %d != %d", a.Cin, CIN);
  PA_CHECK(a.Hin == 2 * a.Hout && a.Win == 2 * a.Wout, "s2 conv: %dx%d -> %dx%d", a.Hin, a.Win, a.Hout, a.Wout);
  PA_CHECK(a.Hout % TH == 0 && a.Wout % TW == 0, "s2 conv: %dx%d not tiled by %dx%d", a.Hout, a.Wout, TH, TW);
  PA_CHECK(a.Cout % BN == 0, "s2 conv: Cout %d %% BN %d", a.Cout, BN);
  const int tiles = ((a.B + NI - 1) / NI) * (a.Hout / TH) * (a.Wout / TW) * (a.Cout / BN);
  hipLaunchKernelGGL((conv3x3s2_ds<T, TH, TW, NI, BN, WM, WN, CIN>), dim3(tiles), dim3(WM * WN * 64), 0, s, a);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

// fp16 layer3 / layer4 entries with the weights in VGPRs and K split over the waves by input block
// (conv_s2k.hip)
int launch_conv3x3s2_k(const ConvS2Args& a, int variant, hipStream_t s, const char** kname);

template <typename T>
int launch_conv3x3s2_ds(const ConvS2Args& a, hipStream_t s, const char** kname) {
  if (a.B <= 0) return PA_OK;
  if constexpr (std::is_same<T, _Float16>::value) {
    // shipped: conv_s2w (layers 2 / 3; g_variant[6] = 40..47 its alternatives 0..7) and
    // conv_s2x (layer4; g_variant[6] = 10..39 its alternatives 0..29 on every layer); 3: the
    // one-tile kernel below (bit-identical reference of conv_s2x for the variant test)
    // shipped from round 6: layer2 on conv_s2v.hip (weights in VGPRs; 6:50 its 8-wave 4 x 16 form,
    // 6:52 / 6:53 the two with deferred stores, 6:49 / 6:51 / 6:54 trace variants; layers 3 / 4 as
    // shipped under all of them),
    // layer3 on conv_s2w, layer4 on conv_s2x.  6:40 = conv_s2w on layers 2 and 3 (the round-5
    // kernels, bit-identical to conv_s2v); 48: layers 2 / 3 as shipped, layer4's entry in the 2 x 4
    // XCD split (conv_s2x_l.hip variant 16)
    const int v = g_variant[6];
    // 6:55 / 6:56: layers 3 and 4 on conv_s2k.hip (weights in VGPRs, K split over the waves by
    // input block; 56 with s_memrealtime stamps), layer2 as shipped
    if ((v == 55 || v == 56) && a.Cin >= 128 && a.wfrag) return launch_conv3x3s2_k(a, v - 55, s, kname);
    if ((v == 0 || (v >= 48 && v <= 56)) && a.Cin == 64 && a.Cout == 128 && a.wfrag) {
      if (v >= 55) return launch_conv3x3s2_v(a, 0, s, kname);
      static const int sv[7] = {0, 4, 1, 5, 2, 3, 6};  // 6:48 .. 6:54 -> conv_s2v.hip variant
      // shipped: variant 2, deferred stores (16.0 vs 16.8 us, profiles/r06e/ab.log); 6:48 keeps the
      // stores at the tile end (variant 0)
      return launch_conv3x3s2_v(a, v == 0 ? 2 : sv[v - 48], s, kname);
    }
    const bool w = v == 0 || (v >= 40 && v <= 54);
    if (w && a.Hout != 8) return launch_conv3x3s2_w(a, v == 0 || v >= 48 ? 0 : v - 40, s, kname);
    if (w || (v >= 10 && v <= 39))
      return launch_conv3x3s2_x(a, v >= 10 && v <= 39 ? v - 10 : v == 48 ? 16 : 0, s, kname);
  }
  if (a.Hout == 32) {
    if (kname) *kname = "conv3x3s2ds_l2";
    return run_s2<T, 8, 16, 1, 64, 4, 1, 64>(a, s);
  }
  if (a.Hout == 16) {
    if (kname) *kname = "conv3x3s2ds_l3";
    return run_s2<T, 8, 16, 1, 64, 4, 1, 128>(a, s);
  }
  if (a.Hout == 8) {
    if (kname) *kname = "conv3x3s2ds_l4";
    return run_s2<T, 8, 8, 2, 64, 4, 1, 256>(a, s);
  }
  set_error("s2 conv: no configuration for %dx%d", a.Hout, a.Wout);
  return PA_EINVAL;
}

template int launch_conv3x3s2_ds<_Float16>(const ConvS2Args&, hipStream_t, const char**);
template int launch_conv3x3s2_ds<float>(const ConvS2Args&, hipStream_t, const char**);

}  // namespace pa
