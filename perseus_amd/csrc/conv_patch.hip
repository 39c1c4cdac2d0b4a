// 3x3 stride-1 convolution with an LDS halo patch (the BasicBlock convs of
// torchvision resnet18 after the first block of each stage; 13 of the 20 convs).
//
// Per workgroup: an output tile of NI images x TH x TW pixels x BN channels.
// For every 128-byte channel block cb of the input, the (TH+2) x (TW+2) input
// patch of each image is staged in LDS ONCE and read by all 9 filter taps
// (implicit GEMM re-fetches every input pixel 9x); weights stream per
// (cb, tap) through a 2-deep LDS ring.  Register-staged prefetch: the next
// step's weight tile and, during a whole channel block, the next block's
// patch are in flight while the MFMAs run.  One barrier per step.
//
// MFMA operand roles: A = weights (rows = output channels), B = pixels, so a
// lane's 4 accumulators are 4 consecutive channels of ONE pixel and the
// epilogue stores / residual loads straight from registers (8 B per lane for
// fp16, 16 B for f32), no LDS staging.
#include <type_traits>

#include "conv.h"

namespace pa {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <typename T>
struct PElem;
template <>
struct PElem<_Float16> {
  static constexpr int KB = 64;
};
template <>
struct PElem<float> {
  static constexpr int KB = 32;
};

__device__ __forceinline__ int pswz(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }

template <typename T>
__device__ __forceinline__ void pmma(f32x4& acc, const u32x4& a, const u32x4& b);

template <>
__device__ __forceinline__ void pmma<_Float16>(f32x4& acc, const u32x4& a, const u32x4& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, a), __builtin_bit_cast(half8, b), acc, 0, 0,
                                               0);
}
template <>
__device__ __forceinline__ void pmma<float>(f32x4& acc, const u32x4& a, const u32x4& b) {
  f32x4 fa = __builtin_bit_cast(f32x4, a), fb = __builtin_bit_cast(f32x4, b);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[0], fb[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[1], fb[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[2], fb[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[3], fb[3], acc, 0, 0, 0);
}

// 4 consecutive elements <-> f32
__device__ __forceinline__ void ld4(const _Float16* p, float* v) {
  half4 h = *reinterpret_cast<const half4*>(p);
  v[0] = (float)h[0];
  v[1] = (float)h[1];
  v[2] = (float)h[2];
  v[3] = (float)h[3];
}
__device__ __forceinline__ void ld4(const float* p, float* v) {
  f32x4 a = *reinterpret_cast<const f32x4*>(p);
  v[0] = a[0];
  v[1] = a[1];
  v[2] = a[2];
  v[3] = a[3];
}
__device__ __forceinline__ void st4(_Float16* p, const float* v) {
  half4 h;
  h[0] = (_Float16)v[0];
  h[1] = (_Float16)v[1];
  h[2] = (_Float16)v[2];
  h[3] = (_Float16)v[3];
  *reinterpret_cast<half4*>(p) = h;
}
__device__ __forceinline__ void st4(float* p, const float* v) {
  *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]};
}

// Lane -> pixel map of a 16-pixel MFMA fragment: lanes whose ds_read_b128 lane
// groups read chunk c0 take the even pixel offsets, the others the odd ones, so
// with the (p >> 1) & 7 XOR swizzle every 16-lane group hits 16 distinct bank
// slots for ANY starting pixel (the 9 taps shift the start by 1 and by PW).
__device__ __forceinline__ int frag_off(int r) { return r < 4 ? 2 * r : (r < 12 ? 2 * (r - 4) + 1 : 2 * (r - 8)); }

template <int V>
using ic = std::integral_constant<int, V>;

// KSP = 2: intra-workgroup split-K -- two groups of WM x WN waves compute the
// same output tile, group kg reading only channel half kg of every 64-channel
// block (half the fragment reads per MFMA of a KSP = 1 wave with the same tile,
// twice the waves to hide latency); group 1's accumulators are added into group
// 0's through LDS before the epilogue.
template <typename T, int TH, int TW, int NI, int BN, int WM, int WN, int PBUF, int CIN, int EPI, int TPW, int KSP>
__global__ __launch_bounds__(WM* WN * 64 * KSP) void conv3x3_patch(ConvArgs a, int ntiles) {
  constexpr int NT = WM * WN * 64 * KSP;
  static_assert(KSP == 1 || (KSP == 2 && TPW == 1), "split-K: one tile per workgroup");
  constexpr int KB = PElem<T>::KB;
  constexpr int CPR = 16 / sizeof(T);
  constexpr int NCB = CIN / KB;  // 128-byte channel blocks
  constexpr int SPC = 9;         // steps (filter taps) per channel block
  constexpr int NSTEPS = NCB * SPC;
  constexpr int WD = 3;          // weight register sets (prefetch distance)
  constexpr int KTOT = 9 * CIN;
  constexpr int PH = TH + 2, PW = TW + 2;
  // per-image patch stride in pixels; for 8-wide tiles a fragment pairs one row of
  // two images, which is conflict-free when the image stride is 8 mod 16
  constexpr int IMS = (TW == 8) ? ((PH * PW + 7) / 16 * 16 + 8) : PH * PW;
  constexpr int NP = NI * IMS;  // patch pixels (incl. pad)
  constexpr int BM = NI * TH * TW;
  constexpr int WTM = BM / WM, WTN = BN / WN;  // wave tile
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int PCH = (NP * 8 + NT - 1) / NT;  // patch 16-B chunks per thread
  constexpr int BCH = BN * 8 / NT;             // weight chunks per thread
  static_assert(BN * 8 % NT == 0, "weight tile / threads");
  static_assert(WTM % 16 == 0 && WTN % 16 == 0, "wave tile");
  static_assert(TW >= 16 || (TW == 8 && NI == 2), "fragment geometry");
  static_assert(SPC % WD == 0, "register-set rotation must be static");
  constexpr int PATCHB = NP * 128;
  constexpr int WB = BN * 128;  // one tap's weight tile
  constexpr int REDB = (KSP - 1) * WM * WN * TM * TN * 64 * 16;  // split-K exchange (after the K loop)
  constexpr int STAGEB = PBUF * PATCHB + 2 * WB;
  __shared__ __attribute__((aligned(16))) char smem[STAGEB > REDB ? STAGEB : REDB];
  char* patch = smem;
  char* wbuf = smem + PBUF * PATCHB;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int kg = wid / (WM * WN), wpos = wid - kg * (WM * WN);
  const int wm = wpos / WN, wn = wpos - (wpos / WN) * WN;
  const int q = lane >> 4, r16 = lane & 15;
  const int H = a.Hout, W = a.Wout;
  constexpr int Cin = CIN;
  const int Cout = a.Cout;
  const T* __restrict__ in = (const T*)a.in;
  const T* __restrict__ w = (const T*)a.w;

  // Tiles: N-tiles of one spatial tile are adjacent in the tile index (they share
  // the patch in L2).  A workgroup takes tiles blockIdx.x + t * gridDim.x, t < TPW;
  // gridDim.x is a multiple of the N-tile count, so its output channels (and the
  // streamed weights) are the same for all its tiles, and the next tile's patch is
  // prefetched while the current one computes.
  const int ntn = Cout / BN;
  const int n0 = (blockIdx.x % ntn) * BN;
  const int tw_n = W / TW, tpi = (H / TH) * tw_n;
  struct Tile {
    int img0, th0, tw0;
  };
  auto decode = [&](int tile) __attribute__((always_inline)) {
    const int sp = tile / ntn;
    const int rem = sp - (sp / tpi) * tpi;
    return Tile{(sp / tpi) * NI, (rem / tw_n) * TH, (rem - (rem / tw_n) * tw_n) * TW};
  };

  // ---- staging (register-staged; hipcc counts these loads itself)
  u32x4 rp[PCH];
  u32x4 rb[WD][BCH];
  auto load_patch = [&](const Tile& tl, int cb) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < PCH; ++i) {
      const int c = tid + i * NT;
      u32x4 v = u32x4{0u, 0u, 0u, 0u};
      if (c < NP * 8) {
        const int p = c >> 3, ch = c & 7;
        const int img = p / IMS, pp = p - (p / IMS) * IMS;
        const int pr = pp / PW, pc = pp - (pp / PW) * PW;
        const int n = tl.img0 + img, h = tl.th0 + pr - 1, x = tl.tw0 + pc - 1;
        if (pr < PH && n < a.B && (unsigned)h < (unsigned)H && (unsigned)x < (unsigned)W)
          v = *reinterpret_cast<const u32x4*>(in + (((size_t)n * H + h) * W + x) * Cin + cb * KB + ch * CPR);
      }
      rp[i] = v;
    }
  };
  auto store_patch = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < PCH; ++i) {
      const int c = tid + i * NT;
      if (c < NP * 8) *reinterpret_cast<u32x4*>(patch + buf * PATCHB + pswz(c >> 3, c & 7)) = rp[i];
    }
  };
  auto load_w = [&](int s, auto setc) __attribute__((always_inline)) {
    constexpr int SET = decltype(setc)::value;
    const int cb = s / SPC, tap = s - (s / SPC) * SPC;
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int c = tid + i * NT;
      const int row = c >> 3, ch = c & 7;
      rb[SET][i] = *reinterpret_cast<const u32x4*>(w + (size_t)(n0 + row) * KTOT + tap * Cin + cb * KB + ch * CPR);
    }
  };
  auto store_w = [&](int buf, auto setc) __attribute__((always_inline)) {
    constexpr int SET = decltype(setc)::value;
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int c = tid + i * NT;
      *reinterpret_cast<u32x4*>(wbuf + buf * WB + pswz(c >> 3, c & 7)) = rb[SET][i];
    }
  };

  // per-lane patch pixel (tap (0,0)) of each pixel fragment (tile independent)
  const int o = frag_off(r16);
  int ppix[TM];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int mb = wm * WTM + tm * 16;  // first m of the fragment
    if constexpr (TW == 8) {
      const int y = mb / 16;  // m = (y * 2 + img) * 8 + x
      ppix[tm] = (o >> 3) * IMS + y * PW + (o & 7);
    } else {
      const int img = mb / (TH * TW);
      const int y = (mb / TW) % TH, x = mb % TW + o;
      ppix[tm] = img * IMS + y * PW + x;
    }
  }

  f32x4 acc[TM][TN];
  Tile cur = decode(blockIdx.x);
  const int my_tiles = blockIdx.x + (TPW - 1) * (int)gridDim.x < ntiles
                           ? TPW
                           : (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;

  load_patch(cur, 0);
  load_w(0, ic<0>{});
  store_patch(0);
  store_w(0, ic<0>{});
  load_w(NSTEPS > 1 ? 1 : 0, ic<1>{});
  load_w(NSTEPS > 2 ? 2 : 0, ic<2>{});
  __syncthreads();

  // Weight-step index runs on across tiles (W(s) of tile t+1 = W(s) of tile t),
  // so the prefetch distance WD wraps modulo NSTEPS; gs = global step for the LDS
  // ring parity.
  int gs = 0;
  for (int t = 0; t < TPW; ++t) {
    if (TPW > 1 && t >= my_tiles) break;
    const bool more = TPW > 1 && t + 1 < my_tiles;
    Tile nxt = cur;
    if (more) nxt = decode(blockIdx.x + (t + 1) * (int)gridDim.x);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // One K-step (cb, ST): refill register set ST%3 with W(s+3), MFMAs on the
    // staged W(s) and patch(cb), then W(s+1) (set (ST+1)%3) -> the other LDS
    // buffer.  The next patch (next channel block, or the next tile's first) is
    // loaded at the block's first step and stored after its last.  Every
    // load/store is unconditional (indices are clamped) so that hipcc's vmcnt
    // bookkeeping stays exact.
    auto step = [&](int cb, auto stc) __attribute__((always_inline)) {
      constexpr int ST = decltype(stc)::value;
      const int s = cb * SPC + ST;
      int sw = s + WD;
      if (sw >= NSTEPS) sw = more ? sw - NSTEPS : NSTEPS - 1;
      load_w(sw, ic<ST % WD>{});
      const bool last_cb = cb + 1 == NCB;
      if constexpr (ST == 0 && (NCB > 1 || TPW > 1)) {
        // next channel block, or the next tile's block 0 (clamped: this tile's
        // block 0 again when there is no next tile, nxt == cur)
        load_patch(last_cb ? nxt : cur, last_cb ? 0 : cb + 1);
      }
      const char* pb = patch + (PBUF == 2 ? ((t * NCB + cb) & 1) * PATCHB : 0);
      const char* wb = wbuf + (gs & 1) * WB;
      const int toff = (ST / 3) * PW + (ST % 3);
      constexpr int NG = 2 / KSP;  // 32-channel halves this wave reduces
      u32x4 fa[NG][TN], fb[NG][TM];
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const int gc = (KSP == 2 ? kg : g) * 4 + q;
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          fa[g][tn] = *reinterpret_cast<const u32x4*>(wb + pswz(wn * WTN + tn * 16 + r16, gc));
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
          fb[g][tm] = *reinterpret_cast<const u32x4*>(pb + pswz(ppix[tm] + toff, gc));
      }
#pragma unroll
      for (int g = 0; g < NG; ++g)
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
          for (int tn = 0; tn < TN; ++tn) pmma<T>(acc[tm][tn], fa[g][tn], fb[g][tm]);
      store_w((gs + 1) & 1, ic<(ST + 1) % WD>{});
      ++gs;
      if constexpr (ST == SPC - 1 && (NCB > 1 || TPW > 1)) {
        if (!last_cb || more) {
          if constexpr (PBUF == 2) {
            store_patch((t * NCB + cb + 1) & 1);
            __syncthreads();
          } else {
            __syncthreads();  // single patch buffer: overwrite after every wave is done with it
            store_patch(0);
            __syncthreads();
          }
          return;
        }
      }
      __syncthreads();
    };
    for (int cb = 0; cb < NCB; ++cb) {
      step(cb, ic<0>{});
      step(cb, ic<1>{});
      step(cb, ic<2>{});
      step(cb, ic<3>{});
      step(cb, ic<4>{});
      step(cb, ic<5>{});
      step(cb, ic<6>{});
      step(cb, ic<7>{});
      step(cb, ic<8>{});
    }

    if constexpr (KSP == 2) {
      // the K loop ended with a barrier: the staging LDS is free for the exchange
      f32x4* red = reinterpret_cast<f32x4*>(smem) + (size_t)wpos * TM * TN * 64 + lane;
      if (kg == 1) {
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
          for (int tn = 0; tn < TN; ++tn) red[(tm * TN + tn) * 64] = acc[tm][tn];
      }
      __syncthreads();
      if (kg == 1) return;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) acc[tm][tn] += red[(tm * TN + tn) * 64];
    }
    // ---- epilogue straight from registers: lane holds channels co..co+3 of one pixel.
    // All residual/bias loads are issued before any use (no serial load->use chains).
    const T* __restrict__ res = (const T*)a.res;
    T* __restrict__ out = (T*)a.out;
    size_t pixo[TM];
    bool ok[TM];
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
      const int n = cur.img0 + img;
      ok[tm] = n < a.B;
      pixo[tm] = ((((size_t)(ok[tm] ? n : 0)) * H + cur.th0 + y) * W + cur.tw0 + x) * Cout;
    }
    f32x4 bias[TN];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
      bias[tn] = *reinterpret_cast<const f32x4*>(a.bias + n0 + wn * WTN + tn * 16 + q * 4);
    float rv[TM][TN][4];
    if constexpr (EPI & EPI_RES) {
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) ld4(res + pixo[tm] + n0 + wn * WTN + tn * 16 + q * 4, rv[tm][tn]);
    }
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
      if (!ok[tm]) continue;
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] = acc[tm][tn][j] + bias[tn][j];
          if constexpr (EPI & EPI_RES) v[j] += rv[tm][tn][j];
          if constexpr (EPI & EPI_RELU) v[j] = fmaxf(v[j], 0.f);
        }
        st4(out + pixo[tm] + n0 + wn * WTN + tn * 16 + q * 4, v);
      }
    }
    cur = nxt;
  }
}

template <typename T, int TH, int TW, int NI, int BN, int WM, int WN, int PBUF, int CIN, int TPW = 1, int KSP = 1>
static int run_patch(const ConvArgs& a, hipStream_t s) {
  PA_CHECK(a.epi == EPI_RELU || a.epi == (EPI_RELU | EPI_RES), "patch conv: epilogue %d", a.epi);
  PA_CHECK(a.Cin == CIN, "patch conv: Cin %d != %d", a.Cin, CIN);
  PA_CHECK(a.Hout % TH == 0 && a.Wout % TW == 0, "patch conv: %dx%d not tiled by %dx%d", a.Hout, a.Wout, TH, TW);
  PA_CHECK(a.Cout % BN == 0, "patch conv: Cout %d %% BN %d", a.Cout, BN);
  const int ntn = a.Cout / BN;
  const int tiles = ((a.B + NI - 1) / NI) * (a.Hout / TH) * (a.Wout / TW) * ntn;
  // grid: a multiple of the N-tile count so a workgroup keeps its output channels
  int grid = (tiles + TPW - 1) / TPW;
  grid = (grid + ntn - 1) / ntn * ntn;
  if (a.epi & EPI_RES)
    hipLaunchKernelGGL((conv3x3_patch<T, TH, TW, NI, BN, WM, WN, PBUF, CIN, EPI_RELU | EPI_RES, TPW, KSP>), dim3(grid),
                       dim3(WM * WN * 64 * KSP), 0, s, a, tiles);
  else
    hipLaunchKernelGGL((conv3x3_patch<T, TH, TW, NI, BN, WM, WN, PBUF, CIN, EPI_RELU, TPW, KSP>), dim3(grid),
                       dim3(WM * WN * 64 * KSP), 0, s, a, tiles);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

// Stride-1 3x3 conv, Hin == Hout.  Tile configuration per feature-map size;
// g_variant[layer] (the handle's pa_detector_debug_set_variant) selects alternatives
// for A/B timing.
static const int k_shipped_variants[8] = {0, 0, 0, 0, 0, 0, 0, 0};
thread_local const int* g_variant = k_shipped_variants;
thread_local unsigned long long* g_trace = nullptr;

template <typename T>
int launch_conv3x3_s1(const ConvArgs& a, hipStream_t s, const char** kname) {
  PA_CHECK(a.stride == 1 && a.pad == 1 && a.Hin == a.Hout && a.Win == a.Wout, "patch conv: stride-1 only");
  PA_CHECK(a.Cin % PElem<T>::KB == 0, "patch conv: Cin %d", a.Cin);
  if (a.B <= 0) return PA_OK;
  if constexpr (std::is_same<T, _Float16>::value) {
    const int layer = a.Hout == 64 ? 1 : a.Hout == 32 ? 2 : a.Hout == 16 ? 3 : 4;
    // layers 2-4: conv_gx (deep-ring LDS-DMA, inline-asm DMA, fully unrolled);
    // variants 50-69 pick its alternatives
    if (layer >= 2 && (g_variant[layer] == 0 || (g_variant[layer] >= 50 && g_variant[layer] <= 69))) {
      static const char* names[5] = {"", "conv3x3x_l1", "conv3x3x_l2", "conv3x3x_l3", "conv3x3x_l4"};
      if (kname) *kname = (a.epi & EPI_HEAD) ? "conv3x3x_l4_avgpool_fc" : names[layer];
      // layer4 ships its one-K-group form (conv_gx_l4.hip 15): the K split (0 / 17 there) is faster
      // per launch back to back but 1.4 % slower over whole forwards (profiles/r06t/fwdab.log)
      const int v = g_variant[layer] == 0 ? (layer == 4 ? 15 : 0) : g_variant[layer] - 50;
      if (a.Cin == 128 && a.Hout == 32) return launch_conv3x3_gx_l2(a, v, s);
      if (a.Cin == 256 && a.Hout == 16) return launch_conv3x3_gx_l3(a, v, s);
      if (a.Cin == 512 && a.Hout == 8) return launch_conv3x3_gx_l4(a, v, s);
    }
    // layer1: the weight-resident persistent kernel for all four convs (variant 32
    // keeps the patch kernel for reference timing)
    // shipped: all four on the LDS-DMA variant (interleaved whole-forward A/B after the
    // write-through epilogues: 172.7k vs 171.7k frames/s with the register-staged kernel on
    // the two non-residual convs, profiles/r01f_variant_sweep.log)
    // round 5: conv_c64v.hip (weights in VGPRs): 16-row tiles on the two plain convs, 8-row tiles
    // in two workgroups per CU on the residual ones; the driver's bench command 182.0k vs 179.6k
    // frames/s median over 7 interleaved pairs against conv_c64d (variant 1:60), which 300-step
    // back-to-back forwards still favour by 0.6 % (profiles/r05_c64v/); bit-identical to it
    const bool l1 = a.Hout == 64 && a.Cout == 64 && a.Cin == 64;
    if (l1 && g_variant[1] == 0) {
      if (kname) *kname = "conv3x3c64_l1";
      return launch_conv3x3_c64v(a, 2, s);
    }
    const bool c64 = g_variant[1] >= 30 && g_variant[1] <= 39 && g_variant[1] != 32;
    if (l1 && c64) {
      if (kname) *kname = "conv3x3c64_l1";
      return launch_conv3x3_c64(a, g_variant[1] - 30, s);
    }
    if (l1 && g_variant[1] >= 80 && g_variant[1] <= 89) {
      if (kname) *kname = "conv3x3c64_l1";
      return launch_conv3x3_c64v(a, g_variant[1] - 80, s);
    }
    if (l1 && g_variant[1] >= 93 && g_variant[1] <= 96) {  // conv_c64v.hip 10-13: deferred stores
      if (kname) *kname = "conv3x3c64_l1";
      return launch_conv3x3_c64v(a, g_variant[1] - 83, s);
    }
    if (l1 && g_variant[1] == 99) {  // conv_c64v.hip 15: the plain convs' last row deferred
      if (kname) *kname = "conv3x3c64_l1";
      return launch_conv3x3_c64v(a, 15, s);
    }
    if (a.Hout == 64 && a.Cout == 64 && a.Cin == 64 && g_variant[1] >= 60 && g_variant[1] <= 69) {
      if (kname) *kname = "conv3x3c64_l1";
      return launch_conv3x3_c64d(a, g_variant[1] - 60, s);
    }
  }
  if (a.Hout == 64 && a.Cout == 64) {
    if (kname) *kname = "conv3x3p_l1";
    switch (g_variant[1]) {
      case 1: return run_patch<T, 16, 16, 1, 64, 4, 1, 1, 64, 2>(a, s);
      case 2: return run_patch<T, 16, 16, 1, 64, 4, 1, 2, 64, 2>(a, s);
      case 3: return run_patch<T, 16, 16, 1, 64, 4, 1, 1, 64, 4>(a, s);
      case 4: return run_patch<T, 16, 16, 1, 64, 4, 1, 2, 64, 4>(a, s);
      case 5: return run_patch<T, 16, 16, 1, 64, 8, 1, 2, 64, 4>(a, s);
      case 6: return run_patch<T, 16, 16, 1, 64, 8, 1, 1, 64, 2>(a, s);
      case 7: return run_patch<T, 16, 16, 1, 64, 8, 1, 2, 64, 2>(a, s);
      case 8: return run_patch<T, 16, 16, 1, 64, 8, 1, 1, 64, 1>(a, s);
      case 9: return run_patch<T, 16, 16, 1, 64, 4, 1, 1, 64, 1, 2>(a, s);
      case 32:
      default: return run_patch<T, 16, 16, 1, 64, 4, 1, 1, 64>(a, s);
    }
  }
  if (a.Hout == 32) {
    if (kname) *kname = "conv3x3p_l2";
    switch (g_variant[2]) {
      case 1: return run_patch<T, 16, 16, 1, 128, 4, 2, 2, 128, 2>(a, s);
      case 2: return run_patch<T, 16, 16, 1, 64, 4, 1, 2, 128, 2>(a, s);
      case 3: return run_patch<T, 16, 16, 1, 64, 4, 1, 2, 128, 4>(a, s);
      case 4: return run_patch<T, 16, 16, 1, 64, 8, 1, 2, 128, 2>(a, s);
      case 5: return run_patch<T, 16, 16, 1, 128, 8, 1, 2, 128, 2>(a, s);
      case 6: return run_patch<T, 16, 16, 1, 64, 8, 1, 1, 128, 2>(a, s);
      case 7: return run_patch<T, 16, 16, 1, 64, 4, 1, 1, 128, 1, 2>(a, s);
      case 8: return run_patch<T, 16, 16, 1, 64, 4, 1, 2, 128, 1, 2>(a, s);
      default: return run_patch<T, 16, 16, 1, 128, 4, 2, 2, 128>(a, s);
    }
  }
  if (a.Hout == 16) {
    if (kname) *kname = "conv3x3p_l3";
    switch (g_variant[3]) {
      case 1: return run_patch<T, 16, 16, 1, 64, 4, 2, 2, 256, 2>(a, s);
      case 2: return run_patch<T, 16, 16, 1, 128, 4, 2, 2, 256>(a, s);
      case 3: return run_patch<T, 16, 16, 1, 32, 4, 1, 2, 256>(a, s);
      case 5: return run_patch<T, 16, 16, 1, 64, 4, 1, 1, 256, 1, 2>(a, s);
      default: return run_patch<T, 16, 16, 1, 64, 4, 2, 2, 256>(a, s);
    }
  }
  if (a.Hout == 8) {
    if (kname) *kname = "conv3x3p_l4";
    switch (g_variant[4]) {
      case 1: return run_patch<T, 8, 8, 2, 64, 4, 2, 1, 512, 2>(a, s);
      case 2: return run_patch<T, 8, 8, 2, 64, 2, 2, 1, 512>(a, s);
      case 3: return run_patch<T, 8, 8, 2, 64, 2, 1, 1, 512>(a, s);
      case 4: return run_patch<T, 8, 8, 2, 64, 2, 1, 1, 512, 1, 2>(a, s);
      case 5: return run_patch<T, 8, 8, 2, 64, 2, 1, 2, 512, 1, 2>(a, s);
      case 6: return run_patch<T, 8, 8, 2, 64, 2, 2, 1, 512, 1, 2>(a, s);
      default: return run_patch<T, 8, 8, 2, 64, 4, 2, 1, 512>(a, s);
    }
  }
  set_error("patch conv: no configuration for %dx%d", a.Hout, a.Wout);
  return PA_EINVAL;
}

template int launch_conv3x3_s1<_Float16>(const ConvArgs&, hipStream_t, const char**);
template int launch_conv3x3_s1<float>(const ConvArgs&, hipStream_t, const char**);

}  // namespace pa
