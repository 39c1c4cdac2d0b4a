// Layer1 3x3 stride-1 conv (Cin = Cout = 64), fp16: conv_c64.hip's weight-resident
// persistent kernel with its staging moved onto LDS-DMA (conv_gx.h's inline-asm
// global_load_lds_dwordx4 and explicit vmcnt waits).
//
// conv_c64.hip loads the next tile's 18 x 18 x 64 halo patch into registers at the
// start of a tile (48 KB per CU issued in one burst), then writes it to LDS after
// the MFMAs; timestamps (tools/trace_launch.py) show ~0.6 us per tile in that
// issue burst and the LDS store, outside the MFMA stream.  Here the patch of tile
// t + 1 is DMA'd straight into the idle patch buffer, one wave-instruction every
// other (tap, 32-channel) group of tile t, so the loads overlap the MFMAs and
// nothing is staged through VGPRs.  The weights (9 taps x 64 rows, one DMA per tap
// per lane) and the first patch are DMA'd in the prologue.
//
// LDS: 72 KB weights (row = tap * 64 + permuted output channel) + 2 x 41 KB patch
// buffers (324 patch pixels rounded up to 41 wave-DMAs of 64 x 16 B), the same
// 128-byte swizzled rows, lane -> pixel map and channel-pair permutation as
// conv_gx.h, so the epilogue is c64's.
#include "conv_gx.h"

namespace pa {

namespace c64d {
constexpr int TH = 16, TW = 16, PH = TH + 2, PW = TW + 2, NP = PH * PW;  // 324 patch pixels
constexpr int NWAVE = 8, NT = NWAVE * 64;
constexpr int PJ = (NP * 8 + 63) / 64;  // 41 patch wave-DMAs
constexpr int PATCHB = PJ * 1024;
constexpr int WBYTES = 9 * 64 * 128;  // 73,728
static_assert(PJ == 5 * NWAVE + 1, "patch DMA split: 5 per wave + 1 on wave 0");
static_assert(WBYTES + 2 * PATCHB <= 160 * 1024, "LDS");
}  // namespace c64d

// DBG: 4 = s_memrealtime stamps into a.trace (as conv_c64.hip); timing only (wrong results):
// 5 = the epilogue computed but not stored, 6 = no hand-over barrier between tiles
// PRIO (A/B): 1 = static s_setprio 1 for waves 4-7 (MI355X_MICROARCH.md "Two waves per SIMD" item 4:
// the second-dispatched half loses every arbitration), 2 = for waves 0-3
// XM: XCD-grouped tile order.  Workgroup b runs on XCD b % 8 (round-robin dispatch), so with the
// plain order (tile j = workgroup j + k * grid) the 16 tiles of an image land on 8 XCDs and every
// halo row is fetched into two or three L2s.  XM hands the tiles of one image to workgroups
// j, j + 8, j + 16, ... (one XCD) in the same round: a halo row another tile of the image already
// pulled is an L2 hit.  The map is a bijection on [0, ntiles) when ntiles % (8 * tiles per image)
// == 0 and the identity otherwise; every tile is computed exactly as before.  Shipped (XM = true).
template <int EPI, int DBG = 0, bool WT = false, int PRIO = 0, bool XM = true>
__global__ __launch_bounds__(512) void conv3x3_c64d(ConvArgs a, int ntiles) {
  using namespace c64d;
  constexpr int WTM = TH * TW / NWAVE;  // 32 pixels per wave
  constexpr int TM = WTM / 16, TN = 4;
  __shared__ __attribute__((aligned(1024))) char smem[WBYTES + 2 * PATCHB];
  char* wl = smem;
  char* patch = smem + WBYTES;

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, r16 = lane & 15;
  const int H = a.Hout, W = a.Wout;
  const _Float16* __restrict__ in = (const _Float16*)a.in;
  const _Float16* __restrict__ w = (const _Float16*)a.w;
  const int tw_n = W / TW, tpi = (H / TH) * tw_n;
  const bool xm = XM && ntiles % (8 * tpi) == 0;
  auto tmap = [&](int j) __attribute__((always_inline)) {
    if (!xm) return j;
    const int c = j / (8 * tpi), r = j - c * 8 * tpi;
    return c * 8 * tpi + (r & 7) * tpi + (r >> 3);
  };
  if constexpr (DBG == 4) trace_stamp(a.trace, 0);
  if constexpr (PRIO == 1) {
    if (wid >= 4) __builtin_amdgcn_s_setprio(1);
  } else if constexpr (PRIO == 2) {
    if (wid < 4) __builtin_amdgcn_s_setprio(1);
  }

  // this lane's patch chunks: DMA i of wave wid covers chunk (i * 8 + wid) * 64 + lane
  // (i = 5 only on wave 0); pixel p = chunk >> 3, logical chunk = physical ^ swizzle
  int prow[6], pcol[6], pch[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int c = ((i < 5 ? i * NWAVE + wid : 5 * NWAVE)) * 64 + lane;
    const int p = c >> 3;
    prow[i] = p < NP ? p / PW : 1 << 20;  // rows past the patch: always out of range
    pcol[i] = p - (p / PW) * PW;
    pch[i] = ((c & 7) ^ ((p >> 1) & 7)) * 8;
  }
  // patch DMAs through a buffer resource over the whole input: the halo (and every DMA of a tile
  // that does not exist) reads zeros through an out-of-range offset, so a DMA in the K loop is one
  // offset computation and no branch.  (The pointer form -- the tile decomposed by integer
  // division at every call, a divergent branch around the halo select, the zero line's address
  // loaded through the GOT behind an s_waitcnt lgkmcnt(0) that also drained the fragment reads --
  // cost the K loop of every tile ~1.3 us on the younger waves, r05h trace.)
  const s2w_u4 rsrc = s2w_rsrc(in, (unsigned)((size_t)a.B * H * W * 128 < 0x7fffffffu ? (size_t)a.B * H * W * 128 : 0x7fffffffu));
  struct Org {
    int img, h0, x0;  // patch origin of a tile: image, first input row and column (halo included)
    bool on;          // false: no such tile (every lane reads zeros)
  };
  auto origin = [&](int t, bool on) __attribute__((always_inline)) {
    const int img = t / tpi, rem = t - img * tpi;
    return Org{img, (rem / tw_n) * TH - 1, (rem - (rem / tw_n) * tw_n) * TW - 1, on};
  };
  auto dma_patch = [&](int i, const Org& o, int buf) __attribute__((always_inline)) {
    const int h = o.h0 + prow[i], x = o.x0 + pcol[i];
    const bool ok = o.on && (unsigned)h < (unsigned)H && (unsigned)x < (unsigned)W;
    const unsigned vo = ok ? (unsigned)((((o.img * H + h) * W + x) * 64 + pch[i]) * 2) : S2W_OOB;
    s2w_dma16(rsrc, vo, patch + buf * PATCHB + (i < 5 ? i * NWAVE + wid : 5 * NWAVE) * 1024);
  };

  const int o = xfrag(r16);
  int ppix[TM];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int mb = wid * WTM + tm * 16;
    ppix[tm] = (mb / TW) * PW + mb % TW + o;
  }
  // bias before the DMAs, so that no compiler-visible load sits between them and the
  // per-tap waits of the first tile below
  f32x4 bias[TN];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) bias[tn] = *reinterpret_cast<const f32x4*>(a.bias + (tn >> 1) * 32 + q * 8 + (tn & 1) * 4);
  __builtin_amdgcn_sched_barrier(0);

  // prologue: patch of the first tile, then the 9 weight taps (tap i = DMA i of
  // every wave); the first tile waits for each tap just before it reads it
  int j = blockIdx.x;
  {
    const Org o0 = origin(tmap(j), true);
    if (wid == 0) dma_patch(5, o0, 0);
#pragma unroll
    for (int i = 0; i < 5; ++i) dma_patch(i, o0, 0);
  }
  {
    const int row0 = wid * 8 + (lane >> 3);  // row within the tap
    const int lc = (lane & 7) ^ ((row0 >> 1) & 7);
    const _Float16* src = w + (size_t)xperm(row0) * 576 + lc * 8;
#pragma unroll
    for (int i = 0; i < 9; ++i) xdma16(src + i * 64, wl + (i * NWAVE + wid) * 1024);
  }
  xwait_vm<8>();  // patch + tap 0
  lds_barrier();
  if constexpr (DBG == 4) trace_stamp(a.trace, 1);

  for (int t = 0; j < ntiles; ++t, j += gridDim.x) {
    const int buf = t & 1;
    const int tile = tmap(j);
    const int next = j + gridDim.x;
    const bool has_next = next < ntiles;
    const Org onext = origin(has_next ? tmap(next) : tile, has_next);  // (no next tile: zeros into the idle buffer)
    const int img = tile / tpi, rem = tile - img * tpi;
    const int th0 = (rem / tw_n) * TH, tw0 = (rem - (rem / tw_n) * tw_n) * TW;
    size_t pixo[TM];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
      const int mb = wid * WTM + tm * 16;
      pixo[tm] = (((size_t)img * H + th0 + mb / TW) * W + tw0 + mb % TW + o) * 64 + q * 8;
    }
    half8 rv[TM][TN / 2];
    if constexpr (EPI & EPI_RES) {
      const _Float16* __restrict__ res = (const _Float16*)a.res;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int p = 0; p < TN / 2; ++p) rv[tm][p] = *reinterpret_cast<const half8*>(res + pixo[tm] + p * 32);
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (DBG == 4) trace_stamp(a.trace, 2 + 4 * t);

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* pb = patch + buf * PATCHB;
    xu4 fa[2][TN], fb[2][TM];
    auto rd = [&](auto kc) __attribute__((always_inline)) {
      constexpr int K = decltype(kc)::value, TAP = K >> 1, HG = K & 1, S = K & 1;
      constexpr int TOFF = (TAP / 3) * PW + (TAP % 3);
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        fa[S][tn] = *reinterpret_cast<const xu4*>(wl + xswz(TAP * 64 + tn * 16 + r16, HG * 4 + q));
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) fb[S][tm] = *reinterpret_cast<const xu4*>(pb + xswz(ppix[tm] + TOFF, HG * 4 + q));
    };
    auto mm = [&](auto kc) __attribute__((always_inline)) {
      constexpr int S = decltype(kc)::value & 1;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, fa[S][tn]),
                                                               __builtin_bit_cast(half8, fb[S][tm]), acc[tm][tn], 0, 0, 0);
    };
    rd(xic<0>{});
    gx_for<0, 18>([&](auto kc) __attribute__((always_inline)) {
      constexpr int K = decltype(kc)::value;
      if constexpr (K % 2 == 1 && K + 1 < 18) {
        // first tile: tap (K + 1) / 2's weights.  VMEM ops issued after that DMA:
        // the later taps, the residual loads, and this tile's patch DMAs so far (odd
        // groups < K; wave 0's extra one at group 0 only makes its wait stricter)
        constexpr int TAPN = (K + 1) / 2;
        constexpr int R = (EPI & EPI_RES) ? TM * TN / 2 : 0;
        constexpr int J = K < 5 ? K : 5;  // next-patch DMAs issued at groups 0 .. K - 1 (wave 0's extra at group 5)
        if (t == 0) {
          xwait_vm<8 - TAPN + R + J>();
          lds_barrier();
        }
      }
      if constexpr (K + 1 < 18) rd(xic<K + 1>{});
      // next tile's patch, one DMA per group from group 0 (wave 0's extra at group 5): issued in
      // the first third of the K loop, so it lands before the tile's end (issued at the odd
      // groups up to 9, the epilogue's vmcnt(0) waited ~0.5 us for the last ones, r05k trace)
      if constexpr (K <= 5) {
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (K == 5) {
          if (wid == 0) dma_patch(5, onext, buf ^ 1);
        } else {
          dma_patch(K, onext, buf ^ 1);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      mm(kc);
    });
    if constexpr (DBG == 4) {  // per-wave K-loop end: slot 20 + 8 t + wave
      if (lane == 0 && t < 5)
        a.trace[blockIdx.x * TRACE_SLOTS + 20 + 8 * t + wid] = __builtin_amdgcn_s_memrealtime();
    }
    xwait_vm<0>();  // next patch (+ residual)

    _Float16* __restrict__ out = (_Float16*)a.out;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
      for (int p = 0; p < TN / 2; ++p) {
        half8 hv;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float v = acc[tm][2 * p + (j >> 2)][j & 3] + bias[2 * p + (j >> 2)][j & 3];
          if constexpr (EPI & EPI_RES) v += (float)rv[tm][p][j];
          hv[j] = (_Float16)fmaxf(v, 0.f);
        }
        if (DBG != 5 || a.epi < 0) store16<WT>(out, (unsigned)((pixo[tm] + p * 32) * 2), hv);
      }
    if constexpr (DBG == 4) trace_stamp(a.trace, 3 + 4 * t);
    // every wave's DMAs into buf ^ 1 landed (its wait above) and its reads of buf
    // retired (the MFMAs consumed them): one barrier hands both buffers over
    if constexpr (DBG != 6) lds_barrier();
    if constexpr (DBG == 4) trace_stamp(a.trace, 5 + 4 * t);
  }
  if constexpr (DBG == 4) {
    __builtin_amdgcn_s_waitcnt(0);
    trace_stamp(a.trace, 63);
  }
}

static int num_cus_d() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

// CUs the launch stream may use: a stream created with a CU mask (hipExtStreamCreateWithCUMask,
// e.g. two half-batches on disjoint halves of every XCD) gets one persistent workgroup per CU
// of its mask, not of the device
int conv_stream_cus(hipStream_t s) {
  const int all = num_cus_d();
  uint32_t m[32] = {};
  if (hipExtStreamGetCUMask(s, 32, m) != hipSuccess) return all;
  int n = 0;
  for (int i = 0; i < 32; ++i) n += __builtin_popcount(m[i]);
  return (n > 0 && n < all) ? n : all;
}

template <int DBG, bool WT = false, int PRIO = 0, bool XM = true>
static int run_c64d(const ConvArgs& a, hipStream_t s) {
  PA_CHECK(!WT || (size_t)a.B * a.Hout * a.Wout * 64 * 2 < 0x7fffffffu, "c64d conv: output over 2 GB");
  const int tiles = a.B * (a.Hout / c64d::TH) * (a.Wout / c64d::TW);
  const int cus = conv_stream_cus(s);
  const int grid = tiles < cus ? tiles : cus;
  if (a.epi & EPI_RES)
    hipLaunchKernelGGL((conv3x3_c64d<EPI_RELU | EPI_RES, DBG, WT, PRIO, XM>), dim3(grid), dim3(512), 0, s, a, tiles);
  else
    hipLaunchKernelGGL((conv3x3_c64d<EPI_RELU, DBG, WT, PRIO, XM>), dim3(grid), dim3(512), 0, s, a, tiles);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

int launch_conv3x3_c64d(const ConvArgs& a, int variant, hipStream_t s) {
  PA_CHECK(a.Cin == 64 && a.Cout == 64 && a.stride == 1 && a.pad == 1 && a.Hin == a.Hout && a.Win == a.Wout,
           "c64d conv: Cin=Cout=64 stride-1 only");
  PA_CHECK(a.Hout % c64d::TH == 0 && a.Wout % c64d::TW == 0, "c64d conv: %dx%d not tiled by 16x16", a.Hout, a.Wout);
  PA_CHECK(a.epi == EPI_RELU || a.epi == (EPI_RELU | EPI_RES), "c64d conv: epilogue %d", a.epi);
  if (a.B <= 0) return PA_OK;
  if (variant == 4 && a.trace) return run_c64d<4>(a, s);
#if PA_TIMING_VARIANTS
  if (variant == 5) return run_c64d<5, true>(a, s);  // timing only (wrong results)
  if (variant == 6) return run_c64d<6, true>(a, s);
#endif
  if (variant == 7) return run_c64d<0, true, 1>(a, s);
  if (variant == 8) return run_c64d<0, true, 2>(a, s);
  // shipped: XCD-grouped tile order (FETCH_SIZE 20.0 -> 16.8 MB per launch without the residual,
  // 36.4 -> 33.2 MB with it; -0.5 us on the residual launches, profiles/r05n/); 9 = plain order
  if (variant == 9) return run_c64d<0, true, 0, false>(a, s);
  return variant == 2 ? run_c64d<0, false>(a, s) : run_c64d<0, true>(a, s);  // 2: plain (write-back) stores
}

}  // namespace pa
