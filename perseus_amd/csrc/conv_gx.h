// 3x3 stride-1 conv, fp16, LDS-DMA staging with a deep weight ring (the layer2-4
// BasicBlock convs).  LDS images: 128-byte rows (one pixel's or one output
// channel's 64 fp16 of the current 64-channel block), 16-byte chunks XOR-swizzled
// by (row >> 1) & 7; the halo patch is DMA'd with the swizzle applied to the
// per-lane source address.  MFMA A = weights, B = pixels; register epilogue.  An
// earlier version of this kernel (distance-2 ring, looped K) measured 22 us on
// layer3 against this one's 19.5.  The design points:
//
//  * prefetch distance PD: the weight tile of step s + PD is DMA'd at step s into
//    a ring of PD + G slots (G = steps per barrier, below).  An L2-hit LDS-DMA under load takes about a
//    microsecond to land (MI355X_MICROARCH.md, ldsdma-fill), i.e. several steps;
//    distance 2-3 left every step waiting on it.
//  * the K loop is unrolled completely, so every step's `s_waitcnt vmcnt(N)` is a
//    compile-time count of the VMEM ops issued after the newest one the next
//    step's fragment reads need (vm_after() below simulates the issue order).
//  * XCD-aware block order (XG): the Cout/BN workgroups of one spatial tile get
//    consecutive indices within one XCD's round-robin share (blocks b and b + 8
//    share an XCD), so the halo patch they all read is an L2 hit after the first.
//
//  * G steps per barrier: the wait + s_barrier closes every G-th step only.
//
// Step s = (block cb = s / 9, tap = s % 9), one 64-channel K-slice of one tap,
// two half-steps of 32 K.  Per step: read the fragments of half-step 2s+1, MFMAs
// of 2s, read the fragments of 2s+2 (step s + 1); then the DMAs, in issue order
// W(s + PD), at the first group start of a block the next block's patch, RSD steps before the end the bias
// (+ residual) loads; MFMAs of 2s+1; wait for what step s + 2's fragments need and
// cross a bare s_barrier.
//
// X3 (the fp16x3 parity mode): activations are a pair of fp16 planes per
// pixel, [hi (Cin) | lo (Cin)] with hi = fp16(v), lo = fp16(v - hi), and the weights
// [tap][hi (Cin) | lo (Cin)] of w * 2^e_co (e_co per output channel, so lo stays a
// normal fp16).  Each 64-channel block becomes 3 virtual blocks with the products
// x_hi w_hi, x_hi w_lo, x_lo w_hi accumulated in f32 (x_lo w_lo, below 2^-22 relative, is
// dropped); the epilogue unscales by 2^-e_co exactly and writes the result as a new
// (hi, lo) pair.  The K loop machinery is the same, with 3x the steps.
#pragma once
#include <type_traits>

#include "conv.h"

namespace pa {

typedef unsigned xu4 __attribute__((ext_vector_type(4)));

template <int V>
using xic = std::integral_constant<int, V>;

template <int B, int E, typename F>
__device__ __forceinline__ void gx_for(F&& f) {
  if constexpr (B < E) {
    f(xic<B>{});
    gx_for<B + 1, E>(f);
  }
}

// 128 zero bytes (halo source); one copy per translation unit (no relocatable device code)
static __device__ __attribute__((aligned(128))) unsigned gx_zero_line[32];

__device__ __forceinline__ int xswz(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }
__device__ __forceinline__ int xfrag(int r) { return r < 4 ? 2 * r : (r < 12 ? 2 * (r - 4) + 1 : 2 * (r - 8)); }
// weight row 16 t + 4 q + v of each 32-row group holds channel 8 q + 4 t + v: a
// lane's tile pair covers 8 consecutive channels (16-byte epilogue accesses)
__device__ __forceinline__ int xperm(int rho) {
  return (rho & ~31) | (((rho >> 2) & 3) << 3) | (((rho >> 4) & 1) << 2) | (rho & 3);
}

template <int N>
__device__ __forceinline__ void xwait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
#endif
}
// 16 B per lane global -> LDS (wave-uniform LDS base + lane * 16), as inline asm:
// with the builtin, hipcc's waitcnt pass stops counting LDS reads in order once an
// LDS-DMA is pending and waits lgkmcnt(0) at the next use of any LDS read (every
// step, right after the barrier).  The pass does not see these VMEM ops, so every
// wait for DMA'd data is the explicit xwait_vm; its own vmcnt waits (bias,
// residual) only get more conservative.  M0 write -> LDS-DMA needs one wait state.
__device__ __forceinline__ void xdma16(const void* src, char* lds) {
#if defined(__HIP_DEVICE_COMPILE__)
  const unsigned off = __builtin_amdgcn_readfirstlane(
      (unsigned)(size_t)(__attribute__((address_space(3))) char*)lds);
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // m0 is reserved: nothing else in these kernels keeps it live
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(off), "v"(src) : "memory", "m0");
#pragma clang diagnostic pop
#endif
}

// 16 B per lane from a buffer resource -> LDS (wave-uniform LDS base + lane * 16), as inline
// asm like xdma16 (its waits are explicit).  A lane whose 32-bit byte offset is
// out of the resource's range (S2W_OOB) reads zeros: the halo needs no pointer select and
// the per-lane address is one 32-bit VGPR (the 64-bit pointer math of xdma16 kept ~75
// VGPRs live across this kernel's unrolled loop and spilled).
typedef unsigned s2w_u4 __attribute__((ext_vector_type(4)));
constexpr unsigned S2W_OOB = 0x80000000u;
__device__ __forceinline__ s2w_u4 s2w_rsrc(const void* base, unsigned bytes) {
  // wave-uniform by construction; readfirstlane puts it in SGPRs for the asm's "s" operand
  const unsigned long long b = (unsigned long long)base;
  return s2w_u4{(unsigned)__builtin_amdgcn_readfirstlane((unsigned)b),
                (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(b >> 32) & 0xffffu),
                (unsigned)__builtin_amdgcn_readfirstlane(bytes), 0x00020000u};
}
__device__ __forceinline__ void s2w_dma16(s2w_u4 rsrc, unsigned voff, char* lds) {
#if defined(__HIP_DEVICE_COMPILE__)
  const unsigned off = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(__attribute__((address_space(3))) char*)lds);
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // m0 is reserved: nothing else in these kernels keeps it live
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(off), "v"(voff),
               "s"(rsrc) : "memory", "m0");
#pragma clang diagnostic pop
#endif
}

// Issue schedule (per wave), used at compile time.
struct GxPlan {
  int nsteps, ncb, pd, wdma, pdma, rl, rs, g;
  int spb = 9;     // steps per 64-channel block (9 taps; conv_s2x.h adds the downsample)
  int spt = 0;     // multi-tile workgroups (conv_s2x.h TPW > 1): steps per tile; the
  int nstore = 0;  // previous tile's `nstore` output stores open every tile's first step
  int xm = 0;      // X3 merged steps (conv_gx.h XM): the steps of even blocks carry two weight tiles
  // the patch of block c >= 1 is DMA'd at the first group start inside block c - 1
  constexpr int ps(int c) const { return (spb * (c - 1) + g - 1) / g * g; }
  constexpr int ns(int t) const { return (spt && t > 0 && t % spt == 0) ? nstore : 0; }
  constexpr int wc(int s) const { return (xm && (s / spb) % 2 == 0) ? 2 : 1; }
  constexpr int nw(int t) const { return t + pd < nsteps ? wdma * wc(t + pd) : 0; }
  constexpr int np(int t) const { return (t / spb + 1 < ncb && t == ps(t / spb + 1)) ? pdma : 0; }
  constexpr int nr(int t) const { return t == rs ? rl : 0; }
  constexpr int cum(int t) const {  // VMEM ops issued in steps 0..t (prologue excluded: it is drained)
    int c = 0;
    for (int u = 0; u <= t; ++u) c += ns(u) + nw(u) + np(u) + nr(u);
    return c;
  }
  // ops issued after the newest op that the fragments of step v need
  // (W(v), and the patch of block v / spb), counted at the end of step s
  constexpr int vm_after(int s, int v) const {
    int need = 0;  // issue position just past the newest needed op (0 = all in the prologue)
    if (v >= pd) {
      const int t = v - pd;
      const int e = (t > 0 ? cum(t - 1) : 0) + ns(t) + nw(t);
      need = e > need ? e : need;
    }
    const int cb = v / spb;
    if (cb >= 1) {
      const int t = ps(cb);
      const int e = (t > 0 ? cum(t - 1) : 0) + ns(t) + nw(t) + np(t);
      need = e > need ? e : need;
    }
    const int n = cum(s) - need;
    return n < 0 ? 0 : (n > 63 ? 63 : n);
  }
};

// Fused avgpool + fc (models.py:31-32) for layer4's last conv, EPI_HEAD.  The workgroup
// holds two whole 8x8 images x BN channels.  Its rounded fp16 outputs go to LDS instead
// of HBM; the per-channel means are formed with head_fp16's exact arithmetic (conv.hip:
// column sums over pixels g, g+4, .., g+60 in order, then (s0 + s1 + s2 + s3) / 64) and
// written to a.pool; the last of the Cout / BN workgroups of the image pair to arrive
// (agent-scope counter, reset by that workgroup) runs the fc exactly as head_fp16 does,
// so the keypoints are bit-identical to the separate head.  No workgroup waits on another.
template <int TH, int TW, int NI, int BN, int NT, int WTM, int WTN, int TM, int TN, int EPI>
__device__ __forceinline__ void gx_head(const ConvArgs& a, char* smem, const f32x4 (&acc)[TM][TN],
                                        const f32x4 (&bias)[TN], const half8 (&rv)[TM][TN / 2], int img0, int n0,
                                        int ntn, int o) {
  static_assert(TH == 8 && TW == 8 && NI == 2 && BN == 64 && NT == 512, "fused head: 2 whole 8x8 images x 64 ch");
  constexpr int NOUT = 16, HW = 64;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int q = lane >> 4;
  constexpr int WN = BN / WTN;
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  _Float16* tile = reinterpret_cast<_Float16*>(smem);  // [img][pixel][BN]
  float* part = reinterpret_cast<float*>(smem + NI * HW * BN * 2);  // [img][wave][NOUT]
  int* flag = reinterpret_cast<int*>(part + NI * 4 * NOUT);
  __syncthreads();  // every wave is past its last fragment read
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int mb = wm * WTM + tm * 16;
    const int pix = (o >> 3) * HW + (mb / 16) * TW + (o & 7);
#pragma unroll
    for (int p = 0; p < TN / 2; ++p) {
      half8 hv;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v = acc[tm][2 * p + (j >> 2)][j & 3] + bias[2 * p + (j >> 2)][j & 3];
        if constexpr (EPI & EPI_RES) v += (float)rv[tm][p][j];
        hv[j] = (_Float16)fmaxf(v, 0.f);
      }
      *reinterpret_cast<half8*>(tile + pix * BN + wn * WTN + p * 32 + q * 8) = hv;
    }
  }
  // the fc weights of this thread's channel pair (t = tid & 255: channels 2t, 2t + 1),
  // in flight during the pooling; only the pair's last workgroup uses them
  const int t = tid & 255, wi = (tid >> 6) & 3, im = tid >> 8;
  const int Cout = a.Cout;
  float2 fw[NOUT];
#pragma unroll
  for (int j = 0; j < NOUT; ++j) fw[j] = *reinterpret_cast<const float2*>(a.fcw + (size_t)j * Cout + 2 * t);
  // LDS-only barrier: __syncthreads() would also wait for the fc weight loads
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  // thread (image, channel) < NI * BN: head_fp16's 4 pixel-group sums (pixels g, g + 4, ..,
  // g + 60 in order) as 4 independent chains; lanes read consecutive channels (no conflicts)
  const __amdgpu_buffer_rsrc_t pr = __builtin_amdgcn_make_buffer_rsrc(a.pool, 0, 0x7fffffff, 0x00020000);
  if (tid < NI * BN) {
    const int pim = tid / BN, c = tid % BN;
    float cs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < HW / 4; ++u)
#pragma unroll
      for (int g = 0; g < 4; ++g) cs[g] += (float)tile[(pim * HW + g + 4 * u) * BN + c];
    const float inv = 1.0f / (float)HW;
    const float mean = (cs[0] + cs[1] + cs[2] + cs[3]) * inv;
    const int pn = img0 + pim;
    if (pn < a.B)
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, mean), pr,
                                            (int)(((size_t)pn * Cout + n0 + c) * 4), 0, 16);
  }
  const int n = img0 + im;
  // hand-off (MI355X_MICROARCH.md, inter-workgroup visibility): the means are stored
  // write-through (sc1), every wave drains its stores, one lane adds to the pair's
  // agent-scope counter; the last arriver reads them with sc1 loads.  No __threadfence
  // (an L2 write-back per workgroup: 21 -> 63 us for this launch when tried).
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    unsigned* ctr = a.cnt + img0 / NI;
    const unsigned prev = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == (unsigned)(ntn - 1);
    if (last) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch (stream order)
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return;
  // fc, head_fp16's arithmetic: thread t of image im takes channels 2t, 2t + 1
  if (n < a.B) {  // wave-uniform (im = tid >> 8)
    const float2 m = __builtin_bit_cast(
        float2, __builtin_amdgcn_raw_buffer_load_b64(pr, (int)(((size_t)n * Cout + 2 * t) * 4), 0, 16));
#pragma unroll
    for (int j = 0; j < NOUT; ++j) {
      float v = fmaf(fw[j].y, m.y, fw[j].x * m.x);
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
      if (lane == 0) part[(im * 4 + wi) * NOUT + j] = v;
    }
  }
  __syncthreads();
  if (t < NOUT && n < a.B) {
    const float* pp = part + im * 4 * NOUT;
    a.y[(size_t)n * NOUT + t] = pp[t] + pp[NOUT + t] + pp[2 * NOUT + t] + pp[3 * NOUT + t] + a.fcb[t];
  }
}

// DBG (timing experiments only, wrong results): 1 = no waits / barriers in the K loop,
// 2 = also no weight / patch DMAs in the K loop, 3 = no K loop (prologue + epilogue),
// 5 = DMAs and barriers but no vmcnt waits, 6 = barriers only (no DMAs in the K loop);
// 4 = the shipped kernel plus s_memrealtime stamps into a.trace (conv.h trace_stamp)
// FD: fragment reads run FD half-steps ahead of the MFMAs (FD + 1 register sets)
// X3 virtual block vb of a CIN = 64 * NCB conv: the 64-channel block of the activation
// planes [hi | lo] (pblk) and of the weight planes (wblk) it multiplies.
// XM (merged): 2 virtual blocks per 64-channel block b, (x_hi; w_hi, w_lo) then
// (x_lo; w_hi): the steps of the first carry two weight tiles (wblk, wblk2) against
// the same patch fragments, so x_hi is staged and read once for both of its products
// (LDS fragment reads per MFMA: layer3's 64 x 32 wave tile 0.58 instead of 0.75;
// barriers per MFMA: 18 steps per block instead of 27).
template <bool X3, int NCB, bool XM = false>
struct GxBlocks {
  static constexpr int NVB = X3 ? (XM ? 2 : 3) * NCB : NCB;
  static constexpr int pblk(int vb) {
    return X3 ? (XM ? (vb % 2 ? NCB + vb / 2 : vb / 2) : (vb % 3 == 2 ? NCB + vb / 3 : vb / 3)) : vb;
  }
  static constexpr int wblk(int vb) { return X3 ? (XM ? vb / 2 : (vb % 3 == 1 ? NCB + vb / 3 : vb / 3)) : vb; }
  static constexpr bool two(int vb) { return XM && vb % 2 == 0; }  // second weight tile: w_lo of block vb / 2
  static constexpr int wblk2(int vb) { return NCB + vb / 2; }
};

// element offset of 64-channel block b within one pixel / weight tap of a conv whose
// activation / weight planes hold CF channels each: [hi (CF) | lo (CF)]; X3 blocks
// b >= NCB (this launch's channels per plane / 64) are the lo plane's
template <int NCB, int CF>
__device__ __forceinline__ constexpr int gx_boff(int b) {
  return b < NCB ? b * 64 : CF + (b - NCB) * 64;
}

// hi / lo fp16 pair of an f32 value (hi + lo == v to 2^-22 relative)
struct HiLo {
  _Float16 hi, lo;
};
__device__ __forceinline__ HiLo split_x3(float v) {
  const _Float16 h = (_Float16)v;
  return HiLo{h, (_Float16)(v - (float)h)};
}

// PART = NS > 0 (split-K for small batches, conv_splitk.hip): the workgroup runs the CIN
// (= 64 * NCB) input channels of split blockIdx.y of an a.Cin = NS * CIN channel conv and
// writes its f32 accumulators to a.part[split] -- no bias, residual or ReLU (splitk_reduce
// applies them after summing the splits in order).  The K loop is 1 / NS of the full
// conv's, which is the launch's critical path when a batch of a few frames gives every CU at
// most one workgroup.  (A fix-up in the same launch -- write-through partials, a per-tile
// arrival counter, the last arriver summing -- measured slower than the separate reduce:
// 15-19 us against 9 + 4.7 us at B = 3)
//
// KS = 2 (K split inside the workgroup): two groups of WM x WN waves; group kg takes
// half-step kg (K 32 kg .. 32 kg + 31) of every step, so with the same 8 waves a wave's
// tile is twice as tall (layer4: 64 px x 32 ch instead of 32 x 32, 0.75 fragment reads
// per MFMA instead of 1.0; the LDS, not the MFMA, bounds that launch).
// Fragments are read one whole step ahead.  At the end the groups swap the halves of
// their tiles through LDS and each finishes TM / 2 rows as (group 0's sum) + (group 1's):
// a different K order from KS = 1 (not bit-identical; within fp16 rounding).
template <int TH, int TW, int NI, int BN, int WM, int WN, int CIN, int PD, int G, int EPI, int DBG = 0, int FD = 1,
          bool WT = true, bool X3 = false, bool XM = false, int PART = 0, int KS = 1>
__global__ __launch_bounds__(WM * WN * KS * 64) void conv3x3_gx(ConvArgs a, int xg) {
  constexpr int NWG = WM * WN;  // waves per K group
  constexpr int NW = NWG * KS, NT = NW * 64;
  static_assert(KS == 1 || (KS == 2 && FD == 1 && !PART && !(EPI & EPI_HEAD) && (DBG == 0 || DBG == 4)),
                "K split: fragments a step ahead, full epilogue");
  constexpr int NCB = CIN / 64;
  static_assert(!XM || (X3 && FD == 1), "merged X3 steps: fp16x3, fragments half a step ahead");
  static_assert(!PART || EPI == 0, "split-K partials: no epilogue");
  using VB = GxBlocks<X3, NCB, XM>;
  constexpr int XS = X3 ? 2 : 1;  // fp16 planes per activation / weight element
  constexpr int NSTEPS = VB::NVB * 9;
  static_assert(!(X3 && (EPI & EPI_HEAD)), "fused head: fp16 path only");
  constexpr int PH = TH + 2, PW = TW + 2;
  constexpr int IMS = (TW == 8) ? ((PH * PW + 7) / 16 * 16 + 8) : PH * PW;
  constexpr int NP = NI * IMS;
  constexpr int NPC = (NP * 8 + 63) / 64 * 64;
  constexpr int PDMA = NPC / 64 / NW + (NPC / 64 % NW ? 1 : 0);
  constexpr int PATCHB = (PDMA * NW * 64) * 16;
  constexpr int WB = BN * 128;
  constexpr int WDMA = BN * 8 / NT;
  constexpr int BM = NI * TH * TW;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int TME = TM / KS;  // 16-pixel rows a wave finishes in the epilogue
  static_assert(TM % KS == 0, "K split: whole rows per group");
  static_assert(BN * 8 % NT == 0 && WDMA >= 1, "weight tile / threads");
  static_assert(WTM % 16 == 0 && WTN % 32 == 0, "wave tile");
  static_assert(TW >= 16 || (TW == 8 && NI == 2), "fragment geometry");
  static_assert(G >= 1 && G <= 3 && PD >= G + 1 && PD <= 8, "prefetch distance / steps per barrier");
  // slot (t + PD) % NSLOT, written at step t, was last read by step t + PD - NSLOT,
  // which must lie before the last barrier: t - G with a barrier every G steps
  constexpr int NSLOT = PD + G;
  constexpr int RL = PART ? 0 : XS * TN + ((EPI & EPI_RES) ? XS * TME * TN / 2 : 0);
  // epilogue loads (bias, residual) issued RSD steps before the end: early enough to
  // land, late enough not to hold their VGPRs across the whole K loop
  constexpr int RSD = NSTEPS >= 28 ? NSTEPS / 7 : 4;  // ~2 us before the end (layer4: 10 of 72 steps)
  constexpr GxPlan plan{NSTEPS, VB::NVB, PD, WDMA, PDMA, RL, NSTEPS > RSD ? NSTEPS - RSD : 0, G, 9, 0, 0, XM ? 1 : 0};
  constexpr int WSLOT = (XM ? 2 : 1) * WB;  // ring slot: one weight tile, or two (XM)
  static_assert(2 * PATCHB + NSLOT * WSLOT <= 163840, "LDS");
  __shared__ __attribute__((aligned(1024))) char smem[2 * PATCHB + NSLOT * WSLOT];
  char* patch = smem;
  char* wring = smem + 2 * PATCHB;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int kg = KS > 1 ? wid / NWG : 0, wl = wid - kg * NWG;  // K group, wave within it
  const int wm = wl / WN, wn = wl - (wl / WN) * WN;
  const int q = lane >> 4, r16 = lane & 15;
  const int H = a.Hout, W = a.Wout;
  // PART: pixel stride and weight tap stride are the full conv's a.Cin; split blockIdx.y
  // starts at input channel CIN * blockIdx.y
  // CF = the full conv's input channels per plane (PART: NS * CIN, a.Cin); KIN = pixel /
  // weight-tap stride in elements; boff(b) = element offset of 64-channel block b of the
  // [hi (CF) | lo (CF)] planes within a pixel or tap (X3 blocks >= NCB are the lo plane's)
  constexpr int CF = PART ? PART * CIN : CIN;
  constexpr int kin = XS * CF;
  const int kc0 = PART ? CIN * (int)blockIdx.y : 0;
  const _Float16* __restrict__ w = (const _Float16*)a.w + kc0;

  const int Cout = a.Cout;
  const int ntn = Cout / BN;
  int tn_idx, sp;
  if (xg >= 2) {
    // 2-D XCD split: XCD share x = (spatial group sg, channel group cg), XB = xg channel
    // groups, so one XCD streams only ntn / XB of the weights (layer4: 1.2 of 4.7 MB, an
    // L2's worth) and reads 8 / XB of the spatial tiles' inputs
    const int b = blockIdx.x, x8 = b & 7, i = b >> 3;
    const int cg = x8 % xg, sg = x8 / xg, ntx = ntn / xg;
    tn_idx = cg * ntx + i % ntx;
    sp = sg * (((int)gridDim.x / 8) / ntx) + i / ntx;
  } else if (xg) {
    // b = 8 i + x (x: XCD share); i = ntn * j + tn  ->  spatial tile 8 j + x
    const int b = blockIdx.x, x8 = b & 7, i = b >> 3;
    tn_idx = i % ntn;
    sp = (i / ntn) * 8 + x8;
  } else {
    tn_idx = blockIdx.x % ntn;
    sp = blockIdx.x / ntn;
  }
  if constexpr (DBG == 4) trace_stamp(a.trace, 0);
  const int tw_n = W / TW, tpi = (H / TH) * tw_n;
  const int img0 = (sp / tpi) * NI;
  const int rem = sp - (sp / tpi) * tpi;
  const int th0 = (rem / tw_n) * TH, tw0 = (rem - (rem / tw_n) * tw_n) * TW;
  const int n0 = tn_idx * BN;

  // patch DMAs through a buffer resource over this tile's images: one 32-bit byte offset per lane
  // and DMA, computed once; a block adds a constant; halo / padding lanes hold an out-of-range
  // offset (S2W_OOB + a block offset stays out of range) and read zeros (no pointer select)
  const s2w_u4 prs = s2w_rsrc((const _Float16*)a.in + (size_t)img0 * H * W * kin,
                              (unsigned)((size_t)(a.B - img0 < NI ? a.B - img0 : NI) * H * W * kin * 2));
  unsigned poff[PDMA];
#pragma unroll
  for (int i = 0; i < PDMA; ++i) {
    const int c = (i * NW + wid) * 64 + lane;
    const int p = c >> 3, pc = c & 7;
    const int lc = pc ^ ((p >> 1) & 7);
    const int img = p / IMS, pp = p - (p / IMS) * IMS;
    const int pr = pp / PW, pcl = pp - (pp / PW) * PW;
    const int n = img0 + img, h = th0 + pr - 1, x = tw0 + pcl - 1;
    const bool ok = p < NP && pr < PH && n < a.B && (unsigned)h < (unsigned)H && (unsigned)x < (unsigned)W;
    poff[i] = ok ? (unsigned)((((img * H + h) * W + x) * kin + kc0 + lc * 8) * 2) : S2W_OOB;
  }
  auto dma_patch = [&](int vb, int buf) __attribute__((always_inline)) {
    const unsigned bo = (unsigned)(gx_boff<NCB, CF>(VB::pblk(vb)) * 2);
#pragma unroll
    for (int i = 0; i < PDMA; ++i) s2w_dma16(prs, poff[i] + bo, patch + buf * PATCHB + (i * NW + wid) * 1024);
  };
  const _Float16* wsrc[WDMA];
#pragma unroll
  for (int i = 0; i < WDMA; ++i) {
    const int c = (i * NW + wid) * 64 + lane;
    const int co = c >> 3, lc = (c & 7) ^ ((co >> 1) & 7);
    wsrc[i] = w + (size_t)(n0 + xperm(co)) * (9 * kin) + lc * 8;
  }
  auto dma_w = [&](int s) __attribute__((always_inline)) {
    const int vb = s / 9, tap = s % 9;
#pragma unroll
    for (int i = 0; i < WDMA; ++i)
      xdma16(wsrc[i] + tap * kin + gx_boff<NCB, CF>(VB::wblk(vb)), wring + (s % NSLOT) * WSLOT + (i * NW + wid) * 1024);
    if (VB::two(vb))  // compile-time after inlining (s is a step constant)
#pragma unroll
      for (int i = 0; i < WDMA; ++i)
        xdma16(wsrc[i] + tap * kin + gx_boff<NCB, CF>(VB::wblk2(vb)),
               wring + (s % NSLOT) * WSLOT + WB + (i * NW + wid) * 1024);
  };

  const int o = xfrag(r16);
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

  const _Float16* __restrict__ res = (const _Float16*)a.res;
  _Float16* __restrict__ out = (_Float16*)a.out;
  size_t pixo[TME];  // the epilogue's rows: tm = kg * TME + j
  bool ok[TME];
#pragma unroll
  for (int j = 0; j < TME; ++j) {
    const int tm = kg * TME + j;
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
    ok[j] = n < a.B;
    pixo[j] = ((((size_t)(ok[j] ? n : 0)) * H + th0 + y) * W + tw0 + x) * (XS * Cout) + n0 + wn * WTN + q * 8;
  }
  half8 rv[TME][TN / 2];
  half8 rl[X3 ? TME : 1][TN / 2];  // X3: the residual's lo plane
  f32x4 bias[TN];
  f32x4 scl[X3 ? TN : 1];  // X3: 2^-e per output channel
  auto load_epi = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int c = n0 + wn * WTN + (tn >> 1) * 32 + q * 8 + (tn & 1) * 4;
      bias[tn] = *reinterpret_cast<const f32x4*>(a.bias + c);
      if constexpr (X3) scl[tn] = *reinterpret_cast<const f32x4*>(a.scale + c);
    }
    if constexpr (EPI & EPI_RES) {
#pragma unroll
      for (int tm = 0; tm < TME; ++tm)
#pragma unroll
        for (int p = 0; p < TN / 2; ++p) {
          rv[tm][p] = *reinterpret_cast<const half8*>(res + pixo[tm] + p * 32);
          if constexpr (X3) rl[tm][p] = *reinterpret_cast<const half8*>(res + pixo[tm] + Cout + p * 32);
        }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: patch(0) and W(0 .. PD-1), drained
  dma_patch(0, 0);
#pragma unroll
  for (int t = 0; t < PD; ++t)
    if (t < NSTEPS) dma_w(t);
  xwait_vm<0>();
  __builtin_amdgcn_s_barrier();
  if constexpr (DBG == 4) trace_stamp(a.trace, 1);

  // fragments one half-step (32 of the 64 K of a step) ahead: sub-step k = 2 S + g
  // reads into set k % (FD + 1) while the MFMAs of an earlier sub-step run
  static_assert(FD == 1 || FD == 2, "fragment distance");
  constexpr int NSET = FD + 1;
  xu4 fa[NSET][TN], fb[NSET][TM];
  xu4 fa2[XM ? NSET : 1][XM ? TN : 1];  // XM: the second weight tile's fragments
  auto read_frags = [&](auto kc) __attribute__((always_inline)) {
    constexpr int K = decltype(kc)::value;
    constexpr int S = K >> 1, HG = K & 1, CB = S / 9, TAP = S % 9, SET = K % NSET;
    constexpr int TOFF = (TAP / 3) * PW + (TAP % 3);
    const char* pb = patch + (CB & 1) * PATCHB;
    const char* wb = wring + (S % NSLOT) * WSLOT;
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
      fa[SET][tn] = *reinterpret_cast<const xu4*>(wb + xswz(wn * WTN + tn * 16 + r16, HG * 4 + q));
    if constexpr (VB::two(CB))
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        fa2[SET][tn] = *reinterpret_cast<const xu4*>(wb + WB + xswz(wn * WTN + tn * 16 + r16, HG * 4 + q));
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) fb[SET][tm] = *reinterpret_cast<const xu4*>(pb + xswz(ppix[tm] + TOFF, HG * 4 + q));
  };
  auto mfma = [&](auto kc) __attribute__((always_inline)) {
    constexpr int K = decltype(kc)::value;
    constexpr int SET = K % NSET;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, fa[SET][tn]),
                                                             __builtin_bit_cast(half8, fb[SET][tm]), acc[tm][tn], 0, 0, 0);
    // XM: x_hi w_lo after every x_hi w_hi of the half-step (TM x TN independent
    // accumulators between two uses of one)
    if constexpr (VB::two((K >> 1) / 9))
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, fa2[SET][tn]),
                                                               __builtin_bit_cast(half8, fb[SET][tm]), acc[tm][tn], 0, 0, 0);
  };
  // step s + 1's data landed before the barrier that closed step s - 1, so with
  // FD = 2 both its halves are read during step s
  // KS = 2: the fragments of step S (this group's half-step kg) into set S & 1
  auto read_frags_k = [&](auto sc) __attribute__((always_inline)) {
    constexpr int S = decltype(sc)::value;
    constexpr int CB = S / 9, TAP = S % 9, SET = S & 1;
    constexpr int TOFF = (TAP / 3) * PW + (TAP % 3);
    const char* pb = patch + (CB & 1) * PATCHB;
    const char* wb = wring + (S % NSLOT) * WSLOT;
    const int ch = kg * 4 + q;
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) fa[SET][tn] = *reinterpret_cast<const xu4*>(wb + xswz(wn * WTN + tn * 16 + r16, ch));
    if constexpr (VB::two(CB))
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        fa2[SET][tn] = *reinterpret_cast<const xu4*>(wb + WB + xswz(wn * WTN + tn * 16 + r16, ch));
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) fb[SET][tm] = *reinterpret_cast<const xu4*>(pb + xswz(ppix[tm] + TOFF, ch));
  };
  // KS = 2: rows [T0, T1) of step S's MFMAs (XM: x_hi w_lo after x_hi w_hi, as mfma())
  auto mfma_k = [&](auto sc, auto t0, auto t1) __attribute__((always_inline)) {
    constexpr int S = decltype(sc)::value, SET = S & 1;
    constexpr int T0 = decltype(t0)::value, T1 = decltype(t1)::value;
#pragma unroll
    for (int tm = T0; tm < T1; ++tm)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, fa[SET][tn]),
                                                             __builtin_bit_cast(half8, fb[SET][tm]), acc[tm][tn], 0, 0, 0);
    if constexpr (VB::two(S / 9))
#pragma unroll
      for (int tm = T0; tm < T1; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, fa2[SET][tn]),
                                                               __builtin_bit_cast(half8, fb[SET][tm]), acc[tm][tn], 0, 0, 0);
  };
  if constexpr (KS == 2) {
    read_frags_k(xic<0>{});
    gx_for<0, NSTEPS>([&](auto sc) __attribute__((always_inline)) {
      constexpr int S = decltype(sc)::value;
      constexpr int CB = S / 9;
      // step S + 1's data landed before the barrier that closed step S - 1 (as FD = 2)
      if constexpr (S + 1 < NSTEPS) read_frags_k(xic<S + 1>{});
      __builtin_amdgcn_s_setprio(1);
      mfma_k(sc, xic<0>{}, xic<TM / 2>{});
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (S + PD < NSTEPS) dma_w(S + PD);
      if constexpr (CB + 1 < VB::NVB && S == plan.ps(CB + 1)) dma_patch(CB + 1, (CB + 1) & 1);
      if constexpr (S == plan.rs) {
        __builtin_amdgcn_sched_barrier(0);
        load_epi();
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
      mfma_k(sc, xic<TM / 2>{}, xic<TM>{});
      __builtin_amdgcn_s_setprio(0);
      if constexpr ((S + 1) % G == 0 && S + 2 < NSTEPS) {
        constexpr int V = S + G + 1 < NSTEPS ? S + G + 1 : NSTEPS - 1;
        xwait_vm<plan.vm_after(S, V)>();
        __builtin_amdgcn_s_barrier();
      }
    });
  } else {
  read_frags(xic<0>{});
  if constexpr (FD == 2) read_frags(xic<1>{});
  gx_for<0, (DBG == 3 ? 0 : NSTEPS)>([&](auto sc) __attribute__((always_inline)) {
    constexpr int S = decltype(sc)::value;
    constexpr int CB = S / 9, TAP = S % 9;
    if constexpr (FD == 1) read_frags(xic<2 * S + 1>{});
    else if constexpr (S + 1 < NSTEPS) read_frags(xic<2 * S + 2>{});
    __builtin_amdgcn_s_setprio(1);
    mfma(xic<2 * S>{});
    __builtin_amdgcn_s_setprio(0);
    if constexpr (S + 1 < NSTEPS) read_frags(xic<2 * S + 1 + FD>{});
    // DMAs after this step's LDS reads (they are issued by then; see xdma16)
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (S + PD < NSTEPS && (DBG < 2 || DBG == 5)) dma_w(S + PD);
    if constexpr (CB + 1 < VB::NVB && S == plan.ps(CB + 1) && (DBG < 2 || DBG == 5)) dma_patch(CB + 1, (CB + 1) & 1);
    if constexpr (S == plan.rs && !PART) {
      // vm_after() counts these after this step's DMAs: keep the scheduler from
      // moving the (read-only) loads across them
      __builtin_amdgcn_sched_barrier(0);
      load_epi();
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    mfma(xic<2 * S + 1>{});
    __builtin_amdgcn_s_setprio(0);
    if constexpr ((S + 1) % G == 0 && S + 2 < NSTEPS && (DBG == 0 || DBG == 4 || DBG == 5 || DBG == 6)) {
      // the next group (steps s+1 .. s+G) reads the fragments of steps up to s+G+1
      // (first half): those weight tiles and their blocks' patches must have landed
      constexpr int V = S + G + 1 < NSTEPS ? S + G + 1 : NSTEPS - 1;
      if constexpr (DBG != 5) xwait_vm<plan.vm_after(S, V)>();
      __builtin_amdgcn_s_barrier();
    }
  });
  }
  if constexpr (DBG == 3) load_epi();
  if constexpr (DBG == 4) trace_stamp(a.trace, 2);
  xwait_vm<0>();  // bias / residual (also waited for by the compiler at their use)

  // ae[j]: the finished sums of epilogue row kg * TME + j
  f32x4 ae[TME][TN];
  if constexpr (KS == 2) {
    // every wave is past its last fragment read and its DMAs have landed (vmcnt(0)):
    // the patch buffers take the swap; group kg hands over the rows the other finishes
    static_assert(2 * NWG * TME * TN * 1024 <= 2 * PATCHB + NSLOT * WSLOT, "K split swap buffer");
    f32x4* xb = reinterpret_cast<f32x4*>(smem);
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int j = 0; j < TME; ++j)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        xb[(((kg * NWG + wl) * TME + j) * TN + tn) * 64 + lane] = kg ? acc[j][tn] : acc[TME + j][tn];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int j = 0; j < TME; ++j)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const f32x4 o = xb[((((1 - kg) * NWG + wl) * TME + j) * TN + tn) * 64 + lane];
        const f32x4 m = kg ? acc[TME + j][tn] : acc[j][tn];
        ae[j][tn] = kg ? o + m : m + o;  // group 0's partial + group 1's
      }
  } else {
#pragma unroll
    for (int j = 0; j < TME; ++j)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) ae[j][tn] = acc[j][tn];
  }

  if constexpr (EPI & EPI_HEAD) {
    gx_head<TH, TW, NI, BN, NT, WTM, WTN, TM, TN, EPI>(a, smem, acc, bias, rv, img0, n0, ntn, o);
    return;
  }
  if constexpr (PART > 0) {  // f32 partials: acc[tm][tn] = 4 consecutive output channels of one pixel
    float* __restrict__ pt = a.part + (size_t)blockIdx.y * a.B * H * W * Cout;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
      if (!ok[tm]) continue;
      const size_t pix = pixo[tm] / (XS * Cout);  // (n * H + y) * W + x (pixo = pix * XS * Cout + channel < Cout)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int c = n0 + wn * WTN + (tn >> 1) * 32 + q * 8 + (tn & 1) * 4;
        *reinterpret_cast<f32x4*>(pt + pix * Cout + c) = acc[tm][tn];
      }
    }
    return;
  }
#pragma unroll
  for (int tm = 0; tm < TME; ++tm) {
    if (!ok[tm]) continue;
#pragma unroll
    for (int p = 0; p < TN / 2; ++p) {
      half8 hv, lv;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int tn = 2 * p + (j >> 2), e = j & 3;
        if constexpr (X3) {
          float v = ae[tm][tn][e] * scl[tn][e] + bias[tn][e];  // exact unscale (power of 2)
          if constexpr (EPI & EPI_RES) v += (float)rv[tm][p][j] + (float)rl[tm][p][j];
          const HiLo hl = split_x3(fmaxf(v, 0.f));
          hv[j] = hl.hi;
          lv[j] = hl.lo;
        } else {
          float v = ae[tm][tn][e] + bias[tn][e];
          if constexpr (EPI & EPI_RES) v += (float)rv[tm][p][j];
          hv[j] = (_Float16)fmaxf(v, 0.f);
        }
      }
      store16<WT>(out, (unsigned)((pixo[tm] + p * 32) * 2), hv);
      if constexpr (X3) store16<WT>(out, (unsigned)((pixo[tm] + Cout + p * 32) * 2), lv);
    }
  }
  if constexpr (DBG == 4) {
    trace_stamp(a.trace, 3);
    __builtin_amdgcn_s_waitcnt(0);
    trace_stamp(a.trace, 63);
  }
}

// split-K partial launch (PART = NS): grid.y = NS splits of CIN channels, f32 partials to a.part
// (X3: the partial sums of the three products, still scaled by 2^e; the reduce unscales)
template <int TH, int TW, int NI, int BN, int WM, int WN, int CIN, int PD, int NS, bool X3 = false, bool XM = false>
static int run_gx_part(const ConvArgs& a, hipStream_t s) {
  PA_CHECK(a.part && a.Cin == NS * CIN && a.Hout == a.Hin && a.Hout % TH == 0 && a.Wout % TW == 0 && a.Cout % BN == 0,
           "gx split-K: Cin %d Cout %d %dx%d", a.Cin, a.Cout, a.Hout, a.Wout);
  const int ntn = a.Cout / BN;
  const int nsp = ((a.B + NI - 1) / NI) * (a.Hout / TH) * (a.Wout / TW);
  hipLaunchKernelGGL((conv3x3_gx<TH, TW, NI, BN, WM, WN, CIN, PD, 1, 0, 0, 1, true, X3, XM, NS>), dim3(nsp * ntn, NS),
                     dim3(WM * WN * 64), 0, s, a, 0);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

template <int TH, int TW, int NI, int BN, int WM, int WN, int CIN, int PD, int G = 1, int DBG = 0, int FD = 1,
          bool WT = true, bool X3 = false, bool XM = false, int KS = 1>
static int run_gx(const ConvArgs& a, int xg, hipStream_t s) {
  PA_CHECK(a.epi == EPI_RELU || a.epi == (EPI_RELU | EPI_RES) || a.epi == (EPI_RELU | EPI_RES | EPI_HEAD),
           "gx conv: epilogue %d", a.epi);
  PA_CHECK(a.Cin == CIN, "gx conv: Cin %d != %d", a.Cin, CIN);
  PA_CHECK(a.Hout % TH == 0 && a.Wout % TW == 0, "gx conv: %dx%d not tiled by %dx%d", a.Hout, a.Wout, TH, TW);
  PA_CHECK(a.Cout % BN == 0, "gx conv: Cout %d %% BN %d", a.Cout, BN);
  const int ntn = a.Cout / BN;
  const int nsp = ((a.B + NI - 1) / NI) * (a.Hout / TH) * (a.Wout / TW);
  const int tiles = nsp * ntn;
  // whole groups of 8 spatial tiles only; the 2-D split needs XB | ntn and (8 / XB) | nsp
  const int x = xg >= 2 ? ((8 % xg == 0 && ntn % xg == 0 && nsp % (8 / xg) == 0 && ntn >= xg) ? xg : (nsp % 8 == 0))
                        : (xg && nsp % 8 == 0);
  PA_CHECK(!WT || (size_t)a.B * a.Hout * a.Wout * a.Cout * 2 * (X3 ? 2 : 1) < 0x7fffffffu, "gx conv: output over 2 GB");
  PA_CHECK(!X3 || (a.scale && !(a.epi & EPI_HEAD)), "gx conv (fp16x3): scale required, no fused head");
  if (a.epi & EPI_HEAD) {
    if constexpr (TH == 8 && TW == 8 && NI == 2 && BN == 64 && WM * WN == 8 && DBG == 0 && !X3 && KS == 1) {
      PA_CHECK(a.pool && a.cnt && a.fcw && a.fcb && a.y && a.Cout == 512, "gx conv: fused head arguments");
      hipLaunchKernelGGL((conv3x3_gx<TH, TW, NI, BN, WM, WN, CIN, PD, G, EPI_RELU | EPI_RES | EPI_HEAD, DBG, FD, WT>),
                         dim3(tiles), dim3(WM * WN * 64), 0, s, a, x);
    } else {
      PA_CHECK(false, "gx conv: fused head needs the 2 x 8x8 x 64-channel tile");
    }
  } else if (a.epi & EPI_RES)
    hipLaunchKernelGGL((conv3x3_gx<TH, TW, NI, BN, WM, WN, CIN, PD, G, EPI_RELU | EPI_RES, DBG, FD, WT, X3, XM, 0, KS>),
                       dim3(tiles), dim3(WM * WN * KS * 64), 0, s, a, x);
  else
    hipLaunchKernelGGL((conv3x3_gx<TH, TW, NI, BN, WM, WN, CIN, PD, G, EPI_RELU, DBG, FD, WT, X3, XM, 0, KS>),
                       dim3(tiles), dim3(WM * WN * KS * 64), 0, s, a, x);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

}  // namespace pa
