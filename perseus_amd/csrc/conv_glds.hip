// 3x3 stride-1 conv with LDS-DMA staging (global_load_lds_dwordx4) and counted
// vmcnt across raw barriers, fp16 (the layer2-4 BasicBlock convs).
//
// Same tiling and LDS images as conv_patch.hip (halo patch per 64-channel block
// reused by the 9 taps, per-tap weight tiles, XOR-swizzled 128-byte rows, MFMA
// A = weights / B = pixels, register epilogue), but nothing is staged through
// registers: the weight tile of tap s+2 and, at the first tap of a block, the
// next block's patch are DMA'd straight into LDS (the swizzle moves to the
// per-lane SOURCE address; out-of-image halo lanes read a zero line).  A step
// waits only for the tile it needs next (`s_waitcnt vmcnt(N)` with N = the DMAs
// issued after it, a compile-time count per tap) and then crosses a bare
// s_barrier, so the prefetch stays in flight across barriers -- hipcc's
// __syncthreads() would drain it (vmcnt(0)) every step
// (cdna_hip_programming.md s5 "Pipelining across barriers").
//
// LDS: 2 patch buffers (block cb, cb+1) + a 3-slot weight ring (taps s, s+1, s+2).
#include <type_traits>

#include "conv.h"

namespace pa {

typedef unsigned gu4 __attribute__((ext_vector_type(4)));

template <int V>
using gic = std::integral_constant<int, V>;

__device__ __attribute__((aligned(128))) unsigned g_zero_line[32];  // 128 zero bytes (halo source)

__device__ __forceinline__ int gswz(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }
__device__ __forceinline__ int gfrag(int r) { return r < 4 ? 2 * r : (r < 12 ? 2 * (r - 4) + 1 : 2 * (r - 8)); }
// weight-row -> output-channel order inside each group of 32 rows: row 16 t + 4 q + v
// holds channel 8 q + 4 t + v, so the accumulators of a lane's tile pair (t = 0, 1)
// are 8 consecutive channels of one pixel (16-byte residual loads / output stores)
__device__ __forceinline__ int gperm(int rho) {
  return (rho & ~31) | (((rho >> 2) & 3) << 3) | (((rho >> 4) & 1) << 2) | (rho & 3);
}

// The LDS-DMA / s_waitcnt builtins exist only for the device target; without the
// guard the host pass silently drops the kernel's launch stub.
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
#if defined(__HIP_DEVICE_COMPILE__)
  // gfx9 s_waitcnt: vmcnt[3:0] bits 3:0, vmcnt[5:4] bits 15:14; expcnt / lgkmcnt left at max
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
#endif
}
// 16 B per lane global -> LDS (wave-uniform LDS base + lane * 16)
__device__ __forceinline__ void dma16(const void* src, char* lds) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
#endif
}

// FP = 1: fragments of step s+1 are read from LDS before step s's MFMAs (two
// fragment register sets), which needs W(s+1) visible one step earlier: weight
// DMA distance 3, 4-slot ring.
template <int TH, int TW, int NI, int BN, int WM, int WN, int CIN, int EPI, int FP>
__global__ __launch_bounds__(WM * WN * 64) void conv3x3_glds(ConvArgs a) {
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int NCB = CIN / 64;
  constexpr int NSTEPS = NCB * 9;
  constexpr int KTOT = 9 * CIN;
  constexpr int PH = TH + 2, PW = TW + 2;
  constexpr int IMS = (TW == 8) ? ((PH * PW + 7) / 16 * 16 + 8) : PH * PW;
  constexpr int NP = NI * IMS;
  constexpr int NPC = (NP * 8 + 63) / 64 * 64;         // patch chunks, padded to whole wave-instructions
  constexpr int PDMA = NPC / 64 / NW + (NPC / 64 % NW ? 1 : 0);  // patch DMA instructions per wave
  constexpr int PATCHB = (PDMA * NW * 64) * 16;          // (incl. the pad the last instructions write)
  constexpr int WB = BN * 128;
  constexpr int WDMA = BN * 8 / NT;                      // weight DMA instructions per wave (per tap)
  constexpr int BM = NI * TH * TW;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  static_assert(BN * 8 % NT == 0 && WDMA >= 1, "weight tile / threads");
  static_assert(WTM % 16 == 0 && WTN % 16 == 0, "wave tile");
  static_assert(TW >= 16 || (TW == 8 && NI == 2), "fragment geometry");
  static_assert(WTN % 32 == 0, "channel-pair permutation needs 32-channel wave tiles");
  // epilogue loads issued during the last block: bias (TN) + residual (TM * TN / 2)
  constexpr int RL = TN + ((EPI & EPI_RES) ? TM * TN / 2 : 0);
  constexpr int NSLOT = FP ? 4 : 3;
  __shared__ __attribute__((aligned(1024))) char smem[2 * PATCHB + NSLOT * WB];
  char* patch = smem;
  char* wring = smem + 2 * PATCHB;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int q = lane >> 4, r16 = lane & 15;
  const int H = a.Hout, W = a.Wout;
  const _Float16* __restrict__ in = (const _Float16*)a.in;
  const _Float16* __restrict__ w = (const _Float16*)a.w;

  const int Cout = a.Cout;
  const int ntn = Cout / BN;
  const int tn_idx = blockIdx.x % ntn;
  const int sp = blockIdx.x / ntn;
  const int tw_n = W / TW, tpi = (H / TH) * tw_n;
  const int img0 = (sp / tpi) * NI;
  const int rem = sp - (sp / tpi) * tpi;
  const int th0 = (rem / tw_n) * TH, tw0 = (rem - (rem / tw_n) * tw_n) * TW;
  const int n0 = tn_idx * BN;

  // per-lane patch DMA sources for block 0 (block cb adds cb * 128 bytes); a lane's
  // LDS slot c = (i * NW + wid) * 64 + lane holds logical chunk (c&7) ^ swz(pixel c>>3)
  const char* psrc[PDMA];
#pragma unroll
  for (int i = 0; i < PDMA; ++i) {
    const int c = (i * NW + wid) * 64 + lane;
    const int p = c >> 3, pc = c & 7;
    const int lc = pc ^ ((p >> 1) & 7);
    const int img = p / IMS, pp = p - (p / IMS) * IMS;
    const int pr = pp / PW, pcl = pp - (pp / PW) * PW;
    const int n = img0 + img, h = th0 + pr - 1, x = tw0 + pcl - 1;
    const bool ok = p < NP && pr < PH && n < a.B && (unsigned)h < (unsigned)H && (unsigned)x < (unsigned)W;
    psrc[i] = ok ? (const char*)(in + (((size_t)n * H + h) * W + x) * CIN + lc * 8) : nullptr;
  }
  auto dma_patch = [&](int cb, int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < PDMA; ++i) {
      const char* s = psrc[i] ? psrc[i] + cb * 128 : (const char*)g_zero_line;
      dma16(s, patch + buf * PATCHB + (i * NW + wid) * 1024);
    }
  };
  // weight DMA: slot c = (i * NW + wid) * 64 + lane -> row co = c >> 3, logical chunk (c&7)^swz(co)
  const _Float16* wsrc[WDMA];
#pragma unroll
  for (int i = 0; i < WDMA; ++i) {
    const int c = (i * NW + wid) * 64 + lane;
    const int co = c >> 3, lc = (c & 7) ^ ((co >> 1) & 7);
    wsrc[i] = w + (size_t)(n0 + gperm(co)) * KTOT + lc * 8;
  }
  auto dma_w = [&](int s, int slot) __attribute__((always_inline)) {
    const int cb = s / 9, tap = s - (s / 9) * 9;
#pragma unroll
    for (int i = 0; i < WDMA; ++i)
      dma16(wsrc[i] + tap * CIN + cb * 64, wring + slot * WB + (i * NW + wid) * 1024);
  };

  const int o = gfrag(r16);
  int ppix[TM];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int mb = wm * WTM + tm * 16;
    if constexpr (TW == 8) {
      ppix[tm] = (o >> 3) * IMS + (mb / 16) * PW + (o & 7);
    } else {
      ppix[tm] = (mb / (TH * TW)) * IMS + ((mb / TW) % TH) * PW + mb % TW + o;
    }
  }

  // epilogue addressing (needed early: the residual is prefetched during the last block)
  const _Float16* __restrict__ res = (const _Float16*)a.res;
  _Float16* __restrict__ out = (_Float16*)a.out;
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
    const int n = img0 + img;
    ok[tm] = n < a.B;
    pixo[tm] = ((((size_t)(ok[tm] ? n : 0)) * H + th0 + y) * W + tw0 + x) * Cout + n0 + wn * WTN + q * 8;
  }
  // bias + residual: RL loads issued right after the DMAs of the last block's
  // first step.  vmcnt is in order, so the waits of that step and the next (the
  // only ones whose awaited DMA is older than these loads) count them too.
  half8 rv[TM][TN / 2];
  f32x4 bias[TN];
  auto load_res = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
      bias[tn] = *reinterpret_cast<const f32x4*>(a.bias + n0 + wn * WTN + (tn >> 1) * 32 + q * 8 + (tn & 1) * 4);
    if constexpr (EPI & EPI_RES) {
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int p = 0; p < TN / 2; ++p) rv[tm][p] = *reinterpret_cast<const half8*>(res + pixo[tm] + p * 32);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if constexpr (!FP) {
    // prologue: patch(0), W(0), W(1) resident
    dma_patch(0, 0);
    dma_w(0, 0);
    if (NSTEPS > 1) dma_w(1, 1);
    wait_vm<0>();
    __builtin_amdgcn_s_barrier();

    // step s = (cb, TAP): DMA W(s+2) (and at TAP 0 the next block's patch), MFMAs on
    // W(s) / patch(cb), then wait for W(s+1) [+ patch(cb+1) after TAP 8] and barrier.
    // LB: cb is the last block (residual prefetch at TAP 0; no wait after TAP 8).
    auto step = [&](int cb, auto tapc, auto lbc) __attribute__((always_inline)) {
      constexpr int TAP = decltype(tapc)::value;
      constexpr bool LB = decltype(lbc)::value;
      constexpr int X = (LB && TAP <= 1) ? RL : 0;
      const int s = cb * 9 + TAP;
      const bool wpre = s + 2 < NSTEPS;
      if (wpre) dma_w(s + 2, (s + 2) % 3);
      const bool ppre = TAP == 0 && cb + 1 < NCB;
      if (ppre) dma_patch(cb + 1, (cb + 1) & 1);
      if constexpr (LB && TAP == 0) load_res();
      const char* pb = patch + (cb & 1) * PATCHB;
      const char* wb = wring + (s % 3) * WB;
      constexpr int TOFF = (TAP / 3) * PW + (TAP % 3);
      gu4 fa[2][TN], fb[2][TM];
#pragma unroll
      for (int g = 0; g < 2; ++g) {
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          fa[g][tn] = *reinterpret_cast<const gu4*>(wb + gswz(wn * WTN + tn * 16 + r16, g * 4 + q));
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
          fb[g][tm] = *reinterpret_cast<const gu4*>(pb + gswz(ppix[tm] + TOFF, g * 4 + q));
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
          for (int tn = 0; tn < TN; ++tn)
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, fa[g][tn]),
                                                                 __builtin_bit_cast(half8, fb[g][tm]), acc[tm][tn], 0, 0,
                                                                 0);
      __builtin_amdgcn_s_setprio(0);
      if constexpr (LB && TAP == 8) return;  // fragments are in registers; nothing left to land
      // W(s+1) was issued one step ago; after it: this step's W(s+2) DMAs and, at TAP 0,
      // the patch DMAs; at TAP 1 the patch DMAs issued at TAP 0 are after it too.
      // Before the last tap of a block everything (incl. the next patch) must land.
      if (!wpre) {
        wait_vm<X>();
      } else if constexpr (TAP == 0 || TAP == 1) {
        if (cb + 1 < NCB)
          wait_vm<WDMA + PDMA + X>();
        else
          wait_vm<WDMA + X>();
      } else {
        wait_vm<WDMA>();
      }
      __builtin_amdgcn_s_barrier();
    };
    auto block = [&](int cb, auto lbc) __attribute__((always_inline)) {
      step(cb, gic<0>{}, lbc);
      step(cb, gic<1>{}, lbc);
      step(cb, gic<2>{}, lbc);
      step(cb, gic<3>{}, lbc);
      step(cb, gic<4>{}, lbc);
      step(cb, gic<5>{}, lbc);
      step(cb, gic<6>{}, lbc);
      step(cb, gic<7>{}, lbc);
      step(cb, gic<8>{}, lbc);
    };
    for (int cb = 0; cb < NCB - 1; ++cb) block(cb, std::false_type{});
    block(NCB - 1, std::true_type{});
  } else {
    // prologue: patch(0), W(0..2) resident
    dma_patch(0, 0);
    dma_w(0, 0);
    if (NSTEPS > 1) dma_w(1, 1);
    if (NSTEPS > 2) dma_w(2, 2);
    wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    gu4 fa[2][2][TN], fb[2][2][TM];
    auto read_frags = [&](int cb, auto tapc, auto setc) __attribute__((always_inline)) {
      constexpr int TAP = decltype(tapc)::value, SET = decltype(setc)::value;
      constexpr int TOFF = (TAP / 3) * PW + (TAP % 3);
      const int s = cb * 9 + TAP;
      const char* pb = patch + (cb & 1) * PATCHB;
      const char* wb = wring + (s & 3) * WB;
#pragma unroll
      for (int g = 0; g < 2; ++g) {
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          fa[SET][g][tn] = *reinterpret_cast<const gu4*>(wb + gswz(wn * WTN + tn * 16 + r16, g * 4 + q));
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
          fb[SET][g][tm] = *reinterpret_cast<const gu4*>(pb + gswz(ppix[tm] + TOFF, g * 4 + q));
      }
    };
    read_frags(0, gic<0>{}, gic<0>{});
    // step (cb, TAP) with fragment set PAR = s & 1 (static: cb pairs are unrolled)
    auto step = [&](int cb, auto tapc, auto parc, auto lbc) __attribute__((always_inline)) {
      constexpr int TAP = decltype(tapc)::value, PAR = decltype(parc)::value;
      constexpr bool LB = decltype(lbc)::value;
      constexpr int X = (LB && TAP <= 1) ? RL : 0;
      const int s = cb * 9 + TAP;
      const bool wpre = s + 3 < NSTEPS;
      if (wpre) dma_w(s + 3, (s + 3) & 3);
      const bool ppre = TAP == 0 && cb + 1 < NCB;
      if (ppre) dma_patch(cb + 1, (cb + 1) & 1);
      if constexpr (LB && TAP == 0) load_res();
      if (s + 1 < NSTEPS) {
        if constexpr (TAP < 8)
          read_frags(cb, gic<TAP + 1>{}, gic<PAR ^ 1>{});
        else
          read_frags(cb + 1, gic<0>{}, gic<PAR ^ 1>{});
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
          for (int tn = 0; tn < TN; ++tn)
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, fa[PAR][g][tn]),
                                                                 __builtin_bit_cast(half8, fb[PAR][g][tm]),
                                                                 acc[tm][tn], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      if constexpr (LB && TAP == 8) return;  // nothing left to land or to protect
      // W(s+2) (read as fragments during step s+1) must have landed; after it were
      // issued: W(s+3) (this step) and, at TAP 0/1, the next block's patch.  The
      // patch itself is retired at TAP 7 (issued before W(s+2) there).
      if constexpr (TAP == 0 || TAP == 1) {
        if (cb + 1 < NCB) {
          if (wpre)
            wait_vm<WDMA + PDMA + X>();
          else
            wait_vm<PDMA + X>();
        } else if (wpre) {
          wait_vm<WDMA + X>();
        } else {
          wait_vm<X>();
        }
      } else {
        if (wpre)
          wait_vm<WDMA>();
        else
          wait_vm<0>();
      }
      __builtin_amdgcn_s_barrier();
    };
    auto block = [&](int cb, auto par0, auto lbc) __attribute__((always_inline)) {
      constexpr int P0 = decltype(par0)::value;
      step(cb, gic<0>{}, gic<P0>{}, lbc);
      step(cb, gic<1>{}, gic<P0 ^ 1>{}, lbc);
      step(cb, gic<2>{}, gic<P0>{}, lbc);
      step(cb, gic<3>{}, gic<P0 ^ 1>{}, lbc);
      step(cb, gic<4>{}, gic<P0>{}, lbc);
      step(cb, gic<5>{}, gic<P0 ^ 1>{}, lbc);
      step(cb, gic<6>{}, gic<P0>{}, lbc);
      step(cb, gic<7>{}, gic<P0 ^ 1>{}, lbc);
      step(cb, gic<8>{}, gic<P0>{}, lbc);
    };
    if constexpr (NCB == 1) {
      block(0, gic<0>{}, std::true_type{});
    } else {
      static_assert(NCB % 2 == 0, "FP blocks run in pairs");
      for (int cb = 0; cb < NCB - 2; cb += 2) {
        block(cb, gic<0>{}, std::false_type{});
        block(cb + 1, gic<1>{}, std::false_type{});
      }
      block(NCB - 2, gic<0>{}, std::false_type{});
      block(NCB - 1, gic<1>{}, std::true_type{});
    }
  }

  // ---- epilogue from registers: lane's channels per tile pair p are pixo + 32 p + [0, 8)
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    if (!ok[tm]) continue;
#pragma unroll
    for (int p = 0; p < TN / 2; ++p) {
      half8 hv;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v = acc[tm][2 * p + (j >> 2)][j & 3] + bias[2 * p + (j >> 2)][j & 3];
        if constexpr (EPI & EPI_RES) v += (float)rv[tm][p][j];
        hv[j] = (_Float16)fmaxf(v, 0.f);
      }
      *reinterpret_cast<half8*>(out + pixo[tm] + p * 32) = hv;
    }
  }
}
template <int TH, int TW, int NI, int BN, int WM, int WN, int CIN, int FP = 0>
static int run_glds(const ConvArgs& a, hipStream_t s) {
  PA_CHECK(a.epi == EPI_RELU || a.epi == (EPI_RELU | EPI_RES), "glds conv: epilogue %d", a.epi);
  PA_CHECK(a.Cin == CIN, "glds conv: Cin %d != %d", a.Cin, CIN);
  PA_CHECK(a.Hout % TH == 0 && a.Wout % TW == 0, "glds conv: %dx%d not tiled by %dx%d", a.Hout, a.Wout, TH, TW);
  PA_CHECK(a.Cout % BN == 0, "glds conv: Cout %d %% BN %d", a.Cout, BN);
  const int tiles = ((a.B + NI - 1) / NI) * (a.Hout / TH) * (a.Wout / TW) * (a.Cout / BN);
  if (a.epi & EPI_RES)
    hipLaunchKernelGGL((conv3x3_glds<TH, TW, NI, BN, WM, WN, CIN, EPI_RELU | EPI_RES, FP>), dim3(tiles),
                       dim3(WM * WN * 64), 0, s, a);
  else
    hipLaunchKernelGGL((conv3x3_glds<TH, TW, NI, BN, WM, WN, CIN, EPI_RELU, FP>), dim3(tiles), dim3(WM * WN * 64), 0, s,
                       a);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

int launch_conv3x3_glds(const ConvArgs& a, int variant, hipStream_t s) {
  if (a.B <= 0) return PA_OK;
  if (a.Hout == 64 && a.Cin == 64) {
    switch (variant) {
      case 1: return run_glds<16, 16, 1, 64, 2, 2, 64>(a, s);
      case 2: return run_glds<16, 16, 1, 64, 4, 1, 64, 1>(a, s);
      default: return run_glds<16, 16, 1, 64, 4, 1, 64>(a, s);
    }
  }
  if (a.Hout == 32) {
    switch (variant) {
      case 1: return run_glds<16, 16, 1, 64, 4, 1, 128>(a, s);
      case 2: return run_glds<16, 16, 1, 128, 4, 2, 128, 1>(a, s);
      case 3: return run_glds<16, 16, 1, 64, 4, 1, 128, 1>(a, s);
      default: return run_glds<16, 16, 1, 128, 4, 2, 128>(a, s);
    }
  }
  if (a.Hout == 16) {
    switch (variant) {
      case 1: return run_glds<16, 16, 1, 64, 4, 1, 256>(a, s);
      case 2: return run_glds<16, 16, 1, 64, 4, 2, 256, 1>(a, s);
      case 3: return run_glds<16, 16, 1, 64, 4, 1, 256, 1>(a, s);
      default: return run_glds<16, 16, 1, 64, 4, 2, 256>(a, s);
    }
  }
  if (a.Hout == 8) {
    switch (variant) {
      case 1: return run_glds<8, 8, 2, 64, 2, 2, 512>(a, s);
      case 2: return run_glds<8, 8, 2, 64, 4, 2, 512, 1>(a, s);
      case 3: return run_glds<8, 8, 2, 64, 2, 2, 512, 1>(a, s);
      default: return run_glds<8, 8, 2, 64, 4, 2, 512>(a, s);
    }
  }
  set_error("glds conv: no configuration for %dx%d", a.Hout, a.Wout);
  return PA_EINVAL;
}

}  // namespace pa
