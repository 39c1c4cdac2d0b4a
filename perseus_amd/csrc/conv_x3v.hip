// fp16x3 (parity mode) layer1 3x3 stride-1 conv (Cin = Cout = 64) with the weights in VGPRs:
// conv_c64v.hip's design for the hi / lo planes.
//
// conv_gx X3 runs layer1's 1,024 tiles as four rounds of one-tile workgroups, each round paying
// the prologue (patch + first weight tiles) and the epilogue (stores) of a one-wave-of-workgroups
// launch.  Here one persistent workgroup per CU walks 8-row tiles (2,048 at B = 64, 8 per CU),
// each wave owning 64 pixels x 16 output channels with the hi and lo weights of those channels
// for all 576 K in 144 VGPRs.  The sums follow conv_gx X3 (merged steps, XM) product for product:
// over the 18 (tap, 32-channel) groups w_hi x_hi then w_lo x_hi, then over the 18 groups again
// w_hi x_lo; the epilogue is the same (unscale by 2^-e, bias, residual hi + lo, ReLU, hi / lo
// split), so the output is bit-identical to conv_gx X3's.
//
// Patch: 10 x 18 pixels of 272 bytes (16 chunks: hi 64 channels | lo 64 channels, + 1 pad);
// chunk of hi channels 32 h + 8 q at position 2 q + h, lo at 8 + 2 q + h: one VGPR + ds_read
// immediates address every fragment, conflict-free for ds_read_b128's lane groups (17 P mod 16
// = P, as conv_c64v's 9 P).  Reads: 4 x_hi fragments per 8 MFMAs, then 4 x_lo per 4 (0.67 per
// MFMA).  LDS (all 160 KB): [patch 0 | residual 0 | patch 1 | residual 1], the residual tile
// DMA'd one tile ahead with the patch so the epilogue needs no barrier of its own; the weights
// (147 KB) are staged through [patch 1 | residual 1] in two rounds of 5 and 4 taps; bias and scale
// live in registers.
#include "conv_gx.h"

namespace pa {

namespace x3v {
constexpr int TH = 8, TW = 16, PH = TH + 2, PW = TW + 2, NP = PH * PW;  // 180 patch pixels
constexpr int NWAVE = 8;
constexpr int PXB = 272;                       // bytes per patch pixel (16 chunks + 1 pad)
constexpr int PJ = (NP * 17 + 63) / 64;        // 48 patch wave-DMAs
constexpr int PATCHB = PJ * 1024;
constexpr int PDW = PJ / NWAVE;                // 6 per wave
constexpr int RESB = TH * TW * 256;            // residual tile, hi | lo
constexpr int RDW = RESB / 1024 / NWAVE;       // 4
constexpr int WROW = 256;                      // staged weight row: hi 64 | lo 64
constexpr int WR0 = 5;                         // taps in the first staging round
constexpr int BSTR = PATCHB + RESB;            // [patch b | residual b]
static_assert(PJ == 48 && PJ % NWAVE == 0, "patch DMA split");
static_assert(BSTR >= WR0 * 64 * WROW, "weight staging in patch 1 + residual 1");
static_assert(2 * BSTR <= 160 * 1024, "LDS");
}  // namespace x3v

// weight row co (chunk c of 16) at LDS chunk c ^ (co & 15): a wave's 16 rows at one chunk hit 16
// different bank quads
__device__ __forceinline__ int x3v_wswz(int row, int chunk) { return row * 256 + ((chunk ^ (row & 15)) << 4); }

// DS: a tile's 8 output half4 per lane are stored during the next tile's K loop (steps 6 .. 13, after
// the patch DMAs) instead of at the tile's end (conv_s2v.hip's deferred stores).  Plain convs: held in
// 16 VGPRs.  Residual convs (no VGPRs to spare): staged in place of the residual each lane has just
// read (its own 8 + 8 bytes of the tile's residual buffer); that buffer receives the tile-after-next's
// residual in the next K loop, so there the residual DMAs move behind the staged reads and an LDS
// barrier (steps 14 .. 17).
// NDX < 4 (residual convs): only the tile's last NDX rows deferred, held in VGPRs (2 NDX half4)
template <int EPI, bool DS = false, int NDX = 4>
__global__ __launch_bounds__(512, 2) void conv3x3_x3v(ConvArgs a, int ntiles) {
  using namespace x3v;
  constexpr int TM = 4;
  __shared__ __attribute__((aligned(1024))) char smem[2 * BSTR];
  char* patch = smem;  // patch b at smem + b * BSTR, residual b at smem + b * BSTR + PATCHB
  char* wst = smem + BSTR;

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, r16 = lane & 15;
  const int wn = wid & 3, wm = wid >> 2;  // 16-channel group, pixel rows 4 wm .. 4 wm + 3
  const int H = a.Hout, W = a.Wout;
  const _Float16* __restrict__ in = (const _Float16*)a.in;
  const _Float16* __restrict__ w = (const _Float16*)a.w;
  const int tw_n = W / TW, tpi = (H / TH) * tw_n;
  const bool xm = ntiles % (8 * tpi) == 0;  // XCD-grouped tile order (conv_c64d.hip XM)
  auto tmap = [&](int j) __attribute__((always_inline)) {
    if (!xm) return j;
    const int c = j / (8 * tpi), r = j - c * 8 * tpi;
    return c * 8 * tpi + (r & 7) * tpi + (r >> 3);
  };

  const unsigned abytes = (unsigned)((size_t)a.B * H * W * 256 < 0x7fffffffu ? (size_t)a.B * H * W * 256 : 0x7fffffffu);
  const s2w_u4 rsrc = s2w_rsrc(in, abytes);
  struct Org {
    int img, h0, x0;
    bool on;
  };
  auto origin = [&](int t, bool on) __attribute__((always_inline)) {
    const int img = t / tpi, rem = t - img * tpi;
    return Org{img, (rem / tw_n) * TH - 1, (rem - (rem / tw_n) * tw_n) * TW - 1, on};
  };
  // patch DMA i: LDS slot c = (i * 8 + wid) * 64 + lane holds pixel c / 17, position c % 17 (16:
  // pad); position pos < 8: hi channels 8 ((pos & 1) * 4 + (pos >> 1)), 8 <= pos < 16: lo channels
  // 8 (((pos - 8) & 1) * 4 + ((pos - 8) >> 1)).  Packed per DMA: bits 0-18 offset from the patch
  // origin, 19-23 pr, 24-28 pc, 29 pad / past the patch.
  unsigned pk[PDW];
#pragma unroll
  for (int i = 0; i < PDW; ++i) {
    const int c = (i * NWAVE + wid) * 64 + lane;
    const int p = c / 17, pos = c - p * 17;
    const int pr = p < NP ? p / PW : 0, pc = p < NP ? p - (p / PW) * PW : 0;
    const int pl = pos & 7, ch = (pos >> 3) * 64 + ((pl & 1) * 4 + (pl >> 1)) * 8;
    const unsigned rel = (unsigned)(((pr * W + pc) * 128 + ch) * 2);
    const unsigned bad = (pos >= 16 || p >= NP) ? 1u : 0u;
    pk[i] = (rel & 0x7ffffu) | ((unsigned)pr << 19) | ((unsigned)pc << 24) | (bad << 29);
  }
  auto dma_patch = [&](int i, const Org& o, int buf) __attribute__((always_inline)) {
    const unsigned v = pk[i];
    const int pr = (int)((v >> 19) & 31u), pc = (int)((v >> 24) & 31u);
    const unsigned tb = (unsigned)(((o.img * H + o.h0) * W + o.x0) * 256);  // wave-uniform (may wrap)
    const bool ok = o.on && !(v >> 29) && (unsigned)(o.h0 + pr) < (unsigned)H && (unsigned)(o.x0 + pc) < (unsigned)W;
    s2w_dma16(rsrc, ok ? tb + (v & 0x7ffffu) : S2W_OOB, patch + buf * BSTR + (i * NWAVE + wid) * 1024);
  };
  // residual tile (hi | lo, 256 B per pixel) by DMA i: slot c -> tile pixel c >> 4 = 32 i + m
  // (m = 4 wid + lane / 16), chunk c & 15 stored as logical chunk (c & 15) ^ (pixel & 15)
  const s2w_u4 rres = s2w_rsrc(a.res ? a.res : a.in, abytes);
  const int mres = 4 * wid + (lane >> 4);
  const unsigned rrel = (unsigned)((((mres >> 4) * W + (mres & 15)) * 128 + (((lane & 15) ^ (mres & 15)) * 8)) * 2);
  auto dma_res = [&](int i, int img, int th0, int tw0, int rb) __attribute__((always_inline)) {
    const unsigned tb = (unsigned)((((img * H + th0 + 2 * i) * W + tw0) * 256));
    s2w_dma16(rres, tb + rrel, smem + rb * BSTR + PATCHB + (i * NWAVE + wid) * 1024);
  };

  const int o = xfrag(r16);
  const unsigned rbase = (unsigned)(size_t)(__attribute__((address_space(3))) char*)patch + (unsigned)((wm * 4 * PW + o) * PXB + q * 32);
  const int c0 = wn * 16 + q * 4;  // this lane's 4 consecutive output channels
  const f32x4 bias = *reinterpret_cast<const f32x4*>(a.bias + c0);
  const f32x4 scl = *reinterpret_cast<const f32x4*>(a.scale + c0);
  __builtin_amdgcn_sched_barrier(0);

  int j = blockIdx.x;
  {
    const Org o0 = origin(tmap(j), true);
#pragma unroll
    for (int i = 0; i < PDW; ++i) dma_patch(i, o0, 0);
    if constexpr (EPI & EPI_RES) {
#pragma unroll
      for (int i = 0; i < RDW; ++i) dma_res(i, o0.img, o0.h0 + 1, o0.x0 + 1, 0);
    }
  }
  // weights: row co of tap t = [hi 64 | lo 64] of output channel co (w + co * 1152 + t * 128), staged
  // by LDS-DMA in rounds of taps; fragment (K, h) of this wave = channel 16 wn + r16, tap K / 2,
  // input channels 32 (K & 1) + 8 q .. + 7 of plane h
  xu4 whi[18], wlo[18];
  auto stage = [&](auto t0c, auto t1c) __attribute__((always_inline)) {
    constexpr int T0 = decltype(t0c)::value, T1 = decltype(t1c)::value;
    // tap (64 rows x 256 B = 16 KB) = 16 wave-DMAs of 4 rows: 2 per wave
#pragma unroll
    for (int tap = T0; tap < T1; ++tap)
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        const int row = (d * NWAVE + wid) * 4 + (lane >> 4);  // 0..63
        const int lc = (lane & 15) ^ (row & 15);               // the logical chunk this lane carries
        xdma16(w + (size_t)row * 1152 + tap * 128 + lc * 8, wst + ((tap - T0) * 16 + d * NWAVE + wid) * 1024);
      }
    xwait_vm<0>();
    lds_barrier();
#pragma unroll
    for (int k = 2 * T0; k < 2 * T1; ++k) {
      const int row = ((k >> 1) - T0) * 64 + wn * 16 + r16;
      whi[k] = *reinterpret_cast<const xu4*>(wst + x3v_wswz(row, (k & 1) * 4 + q));
      wlo[k] = *reinterpret_cast<const xu4*>(wst + x3v_wswz(row, 8 + (k & 1) * 4 + q));
    }
    lds_barrier();
  };
  stage(xic<0>{}, xic<WR0>{});
  stage(xic<WR0>{}, xic<9>{});

  constexpr bool DSR = DS && (EPI & EPI_RES) && NDX >= TM;  // staged in the residual buffer
  constexpr int NDR = DS && !DSR && NDX < TM ? NDX : TM;    // rows deferred: TM - NDR .. TM - 1
  constexpr int RD0 = DSR ? PDW + 2 * TM : PDW;             // first residual-DMA step
  constexpr int SS = (DS && !DSR && (EPI & EPI_RES)) ? PDW + RDW : PDW;  // first deferred-store step
  _Float16* __restrict__ out = (_Float16*)a.out;
  // DSR: this lane's staged chunk of tile pixel px, plane pl (the residual read's address)
  auto stg_off = [&](int px, int pl) __attribute__((always_inline)) {
    return px * 256 + (((8 * pl + (c0 >> 3)) ^ (px & 15)) << 4) + (c0 & 4) * 2;
  };
  half4 ph[DS && !DSR ? NDR : 1], pl[DS && !DSR ? NDR : 1];  // DS (VGPRs): the previous tile's hi / lo outputs
  int pend_base = 0;                        // DS: their tile's first element (wave-uniform)
  const int olane = ((wm * 4) * W + o) * 128 + c0;
  for (int t = 0; j < ntiles; ++t, j += gridDim.x) {
    const int buf = t & 1;
    const int tile = tmap(j);
    const int next = j + gridDim.x;
    const bool has_next = next < ntiles;
    const Org onext = origin(has_next ? tmap(next) : tile, has_next);
    const int img = tile / tpi, rem = tile - img * tpi;
    const int th0 = (rem / tw_n) * TH, tw0 = (rem - (rem / tw_n) * tw_n) * TW;

    f32x4 acc[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const __attribute__((address_space(3))) char* pb =
        (const __attribute__((address_space(3))) char*)(size_t)(rbase + buf * BSTR);
    xu4 fb[2][TM];
    // step K < 18: x_hi of group K; K >= 18: x_lo of group K - 18
    auto rd = [&](auto kc) __attribute__((always_inline)) {
      constexpr int K = decltype(kc)::value, G = K % 18, TAP = G >> 1, HG = G & 1, S = K & 1, LO = K >= 18;
      constexpr int TOFF = (TAP / 3) * PW + (TAP % 3);
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
        fb[S][tm] = *reinterpret_cast<const __attribute__((address_space(3))) xu4*>(pb + (tm * PW + TOFF) * PXB + LO * 128 + HG * 16);
    };
    auto mm = [&](auto kc) __attribute__((always_inline)) {
      constexpr int K = decltype(kc)::value, G = K % 18, S = K & 1;
      if constexpr (K < 18) {
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
          acc[tm] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, whi[G]), __builtin_bit_cast(half8, fb[S][tm]),
                                                           acc[tm], 0, 0, 0);
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
          acc[tm] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, wlo[G]), __builtin_bit_cast(half8, fb[S][tm]),
                                                           acc[tm], 0, 0, 0);
      } else {
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
          acc[tm] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, whi[G]), __builtin_bit_cast(half8, fb[S][tm]),
                                                           acc[tm], 0, 0, 0);
      }
    };
    rd(xic<0>{});
    gx_for<0, 36>([&](auto kc) __attribute__((always_inline)) {
      constexpr int K = decltype(kc)::value;
      if constexpr (K + 1 < 36) rd(xic<K + 1>{});
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (K < PDW) {  // the next tile's patch
        __builtin_amdgcn_sched_barrier(0);
        dma_patch(K, onext, buf ^ 1);
        __builtin_amdgcn_sched_barrier(0);
      } else if constexpr ((EPI & EPI_RES) && K >= RD0 && K < RD0 + RDW) {  // the next tile's residual
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (DSR && K == RD0) lds_barrier();  // every wave's staged reads of buf ^ 1 retired
        if (has_next) dma_res(K - RD0, onext.img, onext.h0 + 1, onext.x0 + 1, buf ^ 1);
        __builtin_amdgcn_sched_barrier(0);
      } else if constexpr (DS && K >= SS && K < SS + 2 * NDR) {  // the previous tile's row TM - NDR + (K - SS) / 2
        constexpr int I = K - SS, R = TM - NDR + (I >> 1);
        __builtin_amdgcn_sched_barrier(0);
        if (t > 0) {
          half4 v;
          if constexpr (DSR)
            v = *reinterpret_cast<const half4*>(smem + (buf ^ 1) * BSTR + PATCHB + stg_off((wm * 4 + R) * TW + o, I & 1));
          else
            v = (I & 1) ? pl[I >> 1] : ph[I >> 1];
          *reinterpret_cast<half4*>(out + pend_base + olane + R * W * 128 + (I & 1) * 64) = v;
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      mm(kc);
    });
    // next patch (+ next residual); DS (plain): the previous tile's stores, issued after them, may stay
    // in flight (DSR: the residual DMAs come after them)
    if constexpr (DS && !DSR) {
      if (t > 0)
        xwait_vm<2 * NDR>();
      else
        xwait_vm<0>();
    } else {
      xwait_vm<0>();
    }

    const char* resl = smem + buf * BSTR + PATCHB;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
      const int px = (wm * 4 + tm) * TW + o;  // tile pixel
      half4 rh, rlo;
      if constexpr (EPI & EPI_RES) {
        // hi chunk (c0 / 8) and lo chunk (8 + c0 / 8) of the residual pixel, half (c0 & 4) of each
        const int ch = c0 >> 3, hf = (c0 & 4) * 2;
        rh = *reinterpret_cast<const half4*>(resl + px * 256 + ((ch ^ (px & 15)) << 4) + hf);
        rlo = *reinterpret_cast<const half4*>(resl + px * 256 + (((8 + ch) ^ (px & 15)) << 4) + hf);
      }
      half4 hv, lv;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = acc[tm][e] * scl[e] + bias[e];  // exact unscale (power of 2)
        if constexpr (EPI & EPI_RES) v += (float)rh[e] + (float)rlo[e];
        const HiLo hl = split_x3(fmaxf(v, 0.f));
        hv[e] = hl.hi;
        lv[e] = hl.lo;
      }
      if constexpr (DSR) {  // in place of this lane's residual chunk
        *reinterpret_cast<half4*>(smem + buf * BSTR + PATCHB + stg_off(px, 0)) = hv;
        *reinterpret_cast<half4*>(smem + buf * BSTR + PATCHB + stg_off(px, 1)) = lv;
      } else if (DS && tm >= TM - NDR) {
        ph[DS ? tm - (TM - NDR) : 0] = hv;
        pl[DS ? tm - (TM - NDR) : 0] = lv;
      } else {
        const size_t pix = ((size_t)img * H + th0 + wm * 4 + tm) * W + tw0 + o;
        *reinterpret_cast<half4*>(out + pix * 128 + c0) = hv;
        *reinterpret_cast<half4*>(out + pix * 128 + 64 + c0) = lv;
      }
    }
    if constexpr (DS) pend_base = ((img * H + th0) * W + tw0) * 128;
    lds_barrier();  // patch / residual buf ^ 1 landed everywhere; reads of buf retired
  }
  if constexpr (DS) {  // the last tile's outputs (this lane's own staged chunks)
    if ((int)blockIdx.x < ntiles) {
      const int lb = ((ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x) & 1;  // the last tile's buffer
#pragma unroll
      for (int tm = TM - NDR; tm < TM; ++tm) {
        half4 vh, vl;
        if constexpr (DSR) {
          vh = *reinterpret_cast<const half4*>(smem + lb * BSTR + PATCHB + stg_off((wm * 4 + tm) * TW + o, 0));
          vl = *reinterpret_cast<const half4*>(smem + lb * BSTR + PATCHB + stg_off((wm * 4 + tm) * TW + o, 1));
        } else {
          vh = ph[tm - (TM - NDR)];
          vl = pl[tm - (TM - NDR)];
        }
        *reinterpret_cast<half4*>(out + pend_base + olane + tm * W * 128) = vh;
        *reinterpret_cast<half4*>(out + pend_base + olane + tm * W * 128 + 64) = vl;
      }
    }
  }
}

// ds / dsr: the plain / residual convs with deferred stores (DS); ndr = 1 / 2: the residual convs'
// last 1 / 2 rows deferred in VGPRs
int launch_conv3x3_x3v(const ConvArgs& a, hipStream_t s, bool ds, bool dsr, int ndr) {
  PA_CHECK(a.Cin == 64 && a.Cout == 64 && a.stride == 1 && a.pad == 1 && a.Hin == a.Hout && a.Win == a.Wout,
           "x3v conv: Cin=Cout=64 stride-1 only");
  PA_CHECK(a.Hout % x3v::TH == 0 && a.Wout % x3v::TW == 0 && a.Wout <= 96, "x3v conv: %dx%d", a.Hout, a.Wout);
  PA_CHECK(a.epi == EPI_RELU || a.epi == (EPI_RELU | EPI_RES), "x3v conv: epilogue %d", a.epi);
  PA_CHECK(a.scale, "x3v conv: scale required");
  PA_CHECK((size_t)a.B * a.Hout * a.Wout * 128 * 2 < 0x7fffffffu, "x3v conv: activations over 2 GB");
  if (a.B <= 0) return PA_OK;
  const int tiles = a.B * (a.Hout / x3v::TH) * (a.Wout / x3v::TW);
  const int cus = conv_stream_cus(s);
  const int grid = tiles < cus ? tiles : cus;
  if ((a.epi & EPI_RES) && dsr)
    hipLaunchKernelGGL((conv3x3_x3v<EPI_RELU | EPI_RES, true>), dim3(grid), dim3(512), 0, s, a, tiles);
  else if ((a.epi & EPI_RES) && ndr == 1)
    hipLaunchKernelGGL((conv3x3_x3v<EPI_RELU | EPI_RES, true, 1>), dim3(grid), dim3(512), 0, s, a, tiles);
  else if ((a.epi & EPI_RES) && ndr == 2)
    hipLaunchKernelGGL((conv3x3_x3v<EPI_RELU | EPI_RES, true, 2>), dim3(grid), dim3(512), 0, s, a, tiles);
  else if (a.epi & EPI_RES)
    hipLaunchKernelGGL((conv3x3_x3v<EPI_RELU | EPI_RES>), dim3(grid), dim3(512), 0, s, a, tiles);
  else if (ds)
    hipLaunchKernelGGL((conv3x3_x3v<EPI_RELU, true>), dim3(grid), dim3(512), 0, s, a, tiles);
  else
    hipLaunchKernelGGL((conv3x3_x3v<EPI_RELU>), dim3(grid), dim3(512), 0, s, a, tiles);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

int launch_conv3x3_x3v(const ConvArgs& a, hipStream_t s) { return launch_conv3x3_x3v(a, s, false, false, 0); }

}  // namespace pa
