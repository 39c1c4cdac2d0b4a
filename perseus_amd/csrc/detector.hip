// Host side of the detector: state-dict blob parsing, BatchNorm folding, weight
// packing for the GPU kernels, workspace management and the forward schedule.
// Exposes the C ABI declared in include/perseus_amd.h.
//
// Reference: perseus/detector/models.py:6-40 (KeypointCNN), torchvision
// resnet18 layer graph (stem, 4 stages x 2 BasicBlocks, avgpool, fc).
#include <cmath>
#include <cstdarg>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "conv.h"

namespace pa {

static thread_local std::string g_err;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
}

struct ConvL {
  int cin, cout, ks, stride, pad;
  size_t w_off;   // element offset into the packed weight arrays (w16 / w32)
  size_t b_off;   // element offset into the bias / scale arrays
  size_t w3_off;  // element offset into the fp16x3 weight planes (w3)
  long wk_off = -1;  // layer2 3x3 s1 convs: element offset into pa_detector::wk2 (conv_s1k.hip order)
};

struct Block {
  int conv1, conv2, ds;  // indices into convs; ds = -1 when identity
};

// conv_gx.h xperm on the host (weight packing)
static inline int xperm_host(int rho) { return (rho & ~31) | (((rho >> 2) & 3) << 3) | (((rho >> 4) & 1) << 2) | (rho & 3); }
// layer2's 3x3 s1 convs with the weights in VGPRs (conv_s1k.hip)
int launch_conv3x3_s1k(const ConvArgs& a, const _Float16* wk, int variant, hipStream_t s, const char** kname);

}  // namespace pa

struct pa_detector {
  int in_ch = 4, n_kp = 8, H = 256, W = 256, prec = PA_PREC_FP16;
  std::vector<pa::ConvL> convs;  // convs[0] = stem
  std::vector<pa::Block> blocks;
  _Float16* w16 = nullptr;
  float* w32 = nullptr;
  float* bias = nullptr;
  _Float16* wv2 = nullptr;  // layer2 entry (conv 3x3 s2 + ds, 64 -> 128) in VGPR-fragment order (conv_s2v.hip)
  _Float16* wv3 = nullptr;  // layer3 / layer4 entries (128 -> 256, 256 -> 512) in conv_s2k.hip's order
  _Float16* wv4 = nullptr;
  _Float16* wv2x3 = nullptr;  // fp16x3 layer2 entry's hi / lo planes in conv_x3s2v.hip's register order
  _Float16* wv3x3 = nullptr;  // fp16x3 layer3 entry's in conv_x3s2k.hip's order
  _Float16* wk2 = nullptr;    // layer2's three 3x3 s1 convs in conv_s1k.hip's register order
  _Float16* w3 = nullptr;   // fp16x3: per conv [cout][taps][hi (cin) | lo (cin)] of w * 2^e (stem: hi plane, lo plane)
  float* scl = nullptr;     // fp16x3: 2^-e per output channel (indexed like bias)
  float* bstem3 = nullptr;  // fp16x3 stem: bias * 2^e (the stem's accumulator starts from it)
  float* fcw = nullptr;
  float* fcb = nullptr;
  char* ws = nullptr;
  size_t ws_bytes = 0;
  float* pool = nullptr;     // fused head: pooled means [cap][512] f32
  unsigned* cnt = nullptr;   // fused head: per-image-pair arrival counters, zero between launches
  unsigned* tctr = nullptr;  // layer1 dynamic tile counters (conv_c64v.hip DYN), zero between launches
  int head_cap = 0;          // batch capacity of pool / cnt
  double flops_per_frame = 0;
  int device = 0;
  int variant[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // pa_detector_debug_set_variant (0 = shipped)
  unsigned long long* trace = nullptr;         // pa_detector_debug_set_trace
  int splitk_max = 0;                          // pa_detector_set_split_k: batches <= this run split-K
  float* part = nullptr;                       // its f32 partials (splitk_part_floats(splitk_max))
  float* xin = nullptr;                        // forward_rgbd's f32 input staging (fp16x3 / fp32)
  int xin_cap = 0;
  int reserved = 0;                            // largest pa_detector_reserve batch (clamped to a chunk)
};

namespace pa {

// Parse + fold + pack.  Returns PA_OK or an error code.
static int build(pa_detector* d, const float* blob, size_t nfloats) {
  size_t pos = 0;
  auto take = [&](size_t n) -> const float* {
    if (pos + n > nfloats) return nullptr;
    const float* p = blob + pos;
    pos += n;
    return p;
  };
  std::vector<_Float16> h16, h3;
  std::vector<float> h32, hb, hs, hbs;

  // conv weight + BN -> packed [cout][ks][ks][cin] (stem: [64][7][32])
  auto add_conv = [&](int cin, int cout, int ks, int stride, int pad, bool stem) -> int {
    const float* w = take((size_t)cout * cin * ks * ks);
    const float* g = take(cout);
    const float* b = take(cout);
    const float* mu = take(cout);
    const float* var = take(cout);
    if (!w || !g || !b || !mu || !var) return -1;
    ConvL L{cin, cout, ks, stride, pad, h32.size(), hb.size(), h3.size()};
    const int K = stem ? 7 * 32 : ks * ks * cin;
    std::vector<float> packed((size_t)cout * K, 0.f);
    for (int co = 0; co < cout; ++co) {
      const double scale = (double)g[co] / std::sqrt((double)var[co] + 1e-5);
      hb.push_back((float)((double)b[co] - (double)mu[co] * scale));
      for (int ci = 0; ci < cin; ++ci)
        for (int kr = 0; kr < ks; ++kr)
          for (int kc = 0; kc < ks; ++kc) {
            const double v = (double)w[(((size_t)co * cin + ci) * ks + kr) * ks + kc] * scale;
            size_t k = stem ? (size_t)kr * 32 + kc * 4 + ci : ((size_t)kr * ks + kc) * cin + ci;
            packed[(size_t)co * K + k] = (float)v;
          }
    }
    for (float v : packed) {
      h32.push_back(v);
      h16.push_back((_Float16)v);
    }
    // fp16x3 planes: the f32 folded weights times 2^e_co (max |w| * 2^e in [2^14, 2^15), so
    // the lo parts stay normal fp16), split into hi = fp16(v), lo = fp16(v - hi).  The
    // scaling is exact; the epilogue multiplies by 2^-e_co.
    const size_t base = h3.size();
    h3.resize(base + (size_t)cout * K * 2);
    const int taps = stem ? 7 : ks * ks;
    const int kt = stem ? 32 : cin;  // elements per tap of one plane
    for (int co = 0; co < cout; ++co) {
      float m = 0.f;
      for (int k = 0; k < K; ++k) m = std::fmax(m, std::fabs(packed[(size_t)co * K + k]));
      const int e = m > 0.f ? 14 - std::ilogb(m) : 0;
      hs.push_back(std::ldexp(1.0f, -e));
      if (stem) hbs.push_back(std::ldexp(hb[L.b_off + co], e));
      for (int t = 0; t < taps; ++t)
        for (int c = 0; c < kt; ++c) {
          const float v = std::ldexp(packed[(size_t)co * K + (size_t)t * kt + c], e);
          const _Float16 hi = (_Float16)v, lo = (_Float16)(v - (float)hi);
          if (stem) {  // [plane][64][7][32]
            h3[base + (size_t)co * K + (size_t)t * kt + c] = hi;
            h3[base + (size_t)cout * K + (size_t)co * K + (size_t)t * kt + c] = lo;
          } else {  // [cout][tap][hi (cin) | lo (cin)]
            h3[base + ((size_t)co * taps + t) * 2 * kt + c] = hi;
            h3[base + ((size_t)co * taps + t) * 2 * kt + kt + c] = lo;
          }
        }
    }
    d->convs.push_back(L);
    return (int)d->convs.size() - 1;
  };

  if (add_conv(d->in_ch, 64, 7, 2, 3, true) < 0) return -1;
  int cin = 64;
  const int couts[4] = {64, 128, 256, 512};
  for (int li = 0; li < 4; ++li) {
    for (int bi = 0; bi < 2; ++bi) {
      const int cout = couts[li];
      const int stride = (li > 0 && bi == 0) ? 2 : 1;
      const int bcin = bi == 0 ? cin : cout;
      Block blk;
      blk.conv1 = add_conv(bcin, cout, 3, stride, 1, false);
      blk.conv2 = add_conv(cout, cout, 3, 1, 1, false);
      blk.ds = -1;
      if (blk.conv1 < 0 || blk.conv2 < 0) return -1;
      if (bi == 0 && (stride != 1 || bcin != cout)) {
        blk.ds = add_conv(bcin, cout, 1, stride, 0, false);
        if (blk.ds < 0) return -1;
      }
      d->blocks.push_back(blk);
    }
    cin = couts[li];
  }
  const int nout = 2 * d->n_kp;
  const float* fw = take((size_t)nout * 512);
  const float* fb = take(nout);
  if (!fw || !fb) return -1;
  if (pos != nfloats) return -2;

  // algorithmic FLOPs (2 x MAC; stem at its true K = 49*Cin)
  const int hw_in[4] = {64, 64, 32, 16};
  (void)hw_in;
  double fl = 2.0 * 128 * 128 * 64 * 49.0 * d->in_ch;
  int hw = 64;
  for (const Block& b : d->blocks) {
    const ConvL& c1 = d->convs[b.conv1];
    const int ho = hw / c1.stride;
    fl += 2.0 * ho * ho * c1.cout * 9.0 * c1.cin;
    fl += 2.0 * ho * ho * c1.cout * 9.0 * c1.cout;
    if (b.ds >= 0) fl += 2.0 * ho * ho * c1.cout * (double)c1.cin;
    hw = ho;
  }
  fl += 2.0 * 512 * nout;
  d->flops_per_frame = fl;

  PA_HIP(hipMalloc(&d->w16, h16.size() * sizeof(_Float16)));
  PA_HIP(hipMalloc(&d->w32, h32.size() * sizeof(float)));
  PA_HIP(hipMalloc(&d->bias, hb.size() * sizeof(float)));
  PA_HIP(hipMalloc(&d->fcw, (size_t)nout * 512 * sizeof(float)));
  PA_HIP(hipMalloc(&d->fcb, (size_t)nout * sizeof(float)));
  PA_HIP(hipMemcpy(d->w16, h16.data(), h16.size() * sizeof(_Float16), hipMemcpyHostToDevice));
  PA_HIP(hipMemcpy(d->w32, h32.data(), h32.size() * sizeof(float), hipMemcpyHostToDevice));
  PA_HIP(hipMemcpy(d->bias, hb.data(), hb.size() * sizeof(float), hipMemcpyHostToDevice));
  PA_HIP(hipMemcpy(d->fcw, fw, (size_t)nout * 512 * sizeof(float), hipMemcpyHostToDevice));
  PA_HIP(hipMemcpy(d->fcb, fb, (size_t)nout * sizeof(float), hipMemcpyHostToDevice));
  // the layer2 entry's conv + downsample weights in conv_s2v.hip's register order: for wave wn
  // (channel quarter), fragment k (< 18: tap k / 2, 32-channel half k & 1; 18, 19: the downsample's
  // halves), tile tn, lane (q, r16): 8 fp16 of channel xperm(32 wn + 16 tn + r16), input channels
  // 32 h + 8 q .. + 7 -- each wave-instruction loads 1 KB contiguous straight into the VGPRs the
  // MFMA reads (no LDS staging)
  // The layer3 / layer4 entries' in conv_s2k.hip's order (the same per wave, for its 64-channel
  // input block wb and its workgroup's channel half h): [h][wb][wn][fragment 20][tn 2][lane 64][8]
  // of channel 32 WN h + xperm(32 wn + 16 tn + r16), input channels 64 wb + 32 (k & 1) + 8 q + e.
  auto pack_vgpr = [&](const Block& bk, int wnq, _Float16** dst) -> int {
    const ConvL& c = d->convs[bk.conv1];
    const ConvL& cd = d->convs[bk.ds];
    const int nb = c.cin / 64, nh = c.cout / (32 * wnq);
    std::vector<_Float16> hv((size_t)nh * nb * wnq * 20 * 2 * 64 * 8);
    for (int hh = 0; hh < nh; ++hh)
      for (int wb = 0; wb < nb; ++wb)
        for (int wn = 0; wn < wnq; ++wn)
          for (int k = 0; k < 20; ++k)
            for (int tn = 0; tn < 2; ++tn)
              for (int lane = 0; lane < 64; ++lane)
                for (int e = 0; e < 8; ++e) {
                  const int q = lane >> 4, r16 = lane & 15;
                  const int rho = 32 * wn + 16 * tn + r16;
                  const int co = 32 * wnq * hh + ((rho & ~31) | (((rho >> 2) & 3) << 3) | (((rho >> 4) & 1) << 2) |
                                                  (rho & 3));  // xperm
                  const int ci = 64 * wb + 32 * (k & 1) + 8 * q + e;
                  const _Float16 v = k < 18 ? h16[c.w_off + (size_t)co * 9 * c.cin + (size_t)(k >> 1) * c.cin + ci]
                                            : h16[cd.w_off + (size_t)co * c.cin + ci];
                  hv[((((((size_t)hh * nb + wb) * wnq + wn) * 20 + k) * 2 + tn) * 64 + lane) * 8 + e] = v;
                }
    PA_HIP(hipMalloc(dst, hv.size() * sizeof(_Float16)));
    PA_HIP(hipMemcpy(*dst, hv.data(), hv.size() * sizeof(_Float16), hipMemcpyHostToDevice));
    return PA_OK;
  };
  for (const Block& bk : d->blocks) {
    if (bk.ds < 0) continue;
    const ConvL& c = d->convs[bk.conv1];
    int rc = PA_OK;
    if (c.cin == 64 && c.cout == 128 && !d->wv2) rc = pack_vgpr(bk, 4, &d->wv2);
    if (c.cin == 128 && c.cout == 256 && !d->wv3) rc = pack_vgpr(bk, 4, &d->wv3);
    if (c.cin == 256 && c.cout == 512 && !d->wv4) rc = pack_vgpr(bk, 2, &d->wv4);
    if (rc != PA_OK) return rc;
  }
  // layer2's 3x3 stride-1 convs (128 -> 128) in conv_s1k.hip's order: per conv [h 2][wb 2][wn 2]
  // [fragment 18][tn 2][lane 64][8] of channel 64 h + xperm(32 wn + 16 tn + r16), input channels
  // 64 wb + 32 (k & 1) + 8 q + e, tap k / 2
  {
    std::vector<_Float16> hv;
    for (pa::ConvL& c : d->convs) {
      if (c.cin != 128 || c.cout != 128 || c.ks != 3 || c.stride != 1) continue;
      c.wk_off = (long)hv.size();
      hv.resize(hv.size() + (size_t)2 * 2 * 2 * 18 * 2 * 64 * 8);
      _Float16* dst = hv.data() + c.wk_off;
      for (int hh = 0; hh < 2; ++hh)
        for (int wb = 0; wb < 2; ++wb)
          for (int wn = 0; wn < 2; ++wn)
            for (int k = 0; k < 18; ++k)
              for (int tn = 0; tn < 2; ++tn)
                for (int lane = 0; lane < 64; ++lane)
                  for (int e = 0; e < 8; ++e) {
                    const int q = lane >> 4, r16 = lane & 15;
                    const int co = 64 * hh + pa::xperm_host(32 * wn + 16 * tn + r16);
                    const int ci = 64 * wb + 32 * (k & 1) + 8 * q + e;
                    dst[((((((size_t)hh * 2 + wb) * 2 + wn) * 18 + k) * 2 + tn) * 64 + lane) * 8 + e] =
                        h16[c.w_off + (size_t)co * 9 * 128 + (size_t)(k >> 1) * 128 + ci];
                  }
    }
    if (!hv.empty()) {
      PA_HIP(hipMalloc(&d->wk2, hv.size() * sizeof(_Float16)));
      PA_HIP(hipMemcpy(d->wk2, hv.data(), hv.size() * sizeof(_Float16), hipMemcpyHostToDevice));
    }
  }
  // the fp16x3 layer2 entry's hi / lo planes in conv_x3s2v.hip's register order: [wave 8][fragment
  // 20][plane 2][lane 64][8] of channel 16 wave + r16, input channels 32 (k & 1) + 8 q + e (fragment
  // k < 18: tap k / 2; 18, 19: the downsample)
  for (const Block& bk : d->blocks) {
    const ConvL& c = d->convs[bk.conv1];
    if (bk.ds < 0 || c.cin != 64 || c.cout != 128 || d->wv2x3) continue;
    const ConvL& cd = d->convs[bk.ds];
    std::vector<_Float16> hv((size_t)8 * 20 * 2 * 64 * 8);
    for (int wn = 0; wn < 8; ++wn)
      for (int k = 0; k < 20; ++k)
        for (int pl = 0; pl < 2; ++pl)
          for (int lane = 0; lane < 64; ++lane)
            for (int e = 0; e < 8; ++e) {
              const int q = lane >> 4, r16 = lane & 15, co = 16 * wn + r16, ci = 32 * (k & 1) + 8 * q + e;
              const _Float16 v = k < 18 ? h3[c.w3_off + ((size_t)co * 9 + (k >> 1)) * 128 + pl * 64 + ci]
                                        : h3[cd.w3_off + (size_t)co * 128 + pl * 64 + ci];
              hv[((((size_t)wn * 20 + k) * 2 + pl) * 64 + lane) * 8 + e] = v;
            }
    PA_HIP(hipMalloc(&d->wv2x3, hv.size() * sizeof(_Float16)));
    PA_HIP(hipMemcpy(d->wv2x3, hv.data(), hv.size() * sizeof(_Float16), hipMemcpyHostToDevice));
  }
  // the fp16x3 layer3 entry's in conv_x3s2k.hip's order: [quarter h][block wb][tile wc][fragment
  // 20][plane 2][lane 64][8] of channel 64 h + 16 wc + r16, input channels 64 wb + 32 (k & 1) + 8 q + e
  for (const Block& bk : d->blocks) {
    const ConvL& c = d->convs[bk.conv1];
    if (bk.ds < 0 || c.cin != 128 || c.cout != 256 || d->wv3x3) continue;
    const ConvL& cd = d->convs[bk.ds];
    std::vector<_Float16> hv((size_t)4 * 2 * 4 * 20 * 2 * 64 * 8);
    for (int hh = 0; hh < 4; ++hh)
      for (int wb = 0; wb < 2; ++wb)
        for (int wc = 0; wc < 4; ++wc)
          for (int k = 0; k < 20; ++k)
            for (int pl = 0; pl < 2; ++pl)
              for (int lane = 0; lane < 64; ++lane)
                for (int e = 0; e < 8; ++e) {
                  const int q = lane >> 4, r16 = lane & 15, co = 64 * hh + 16 * wc + r16;
                  const int ci = 64 * wb + 32 * (k & 1) + 8 * q + e;
                  const _Float16 v = k < 18 ? h3[c.w3_off + ((size_t)co * 9 + (k >> 1)) * 256 + pl * 128 + ci]
                                            : h3[cd.w3_off + (size_t)co * 256 + pl * 128 + ci];
                  hv[((((((size_t)hh * 2 + wb) * 4 + wc) * 20 + k) * 2 + pl) * 64 + lane) * 8 + e] = v;
                }
    PA_HIP(hipMalloc(&d->wv3x3, hv.size() * sizeof(_Float16)));
    PA_HIP(hipMemcpy(d->wv3x3, hv.data(), hv.size() * sizeof(_Float16), hipMemcpyHostToDevice));
  }
  PA_HIP(hipMalloc(&d->w3, h3.size() * sizeof(_Float16)));
  PA_HIP(hipMalloc(&d->scl, hs.size() * sizeof(float)));
  PA_HIP(hipMalloc(&d->bstem3, hbs.size() * sizeof(float)));
  PA_HIP(hipMemcpy(d->w3, h3.data(), h3.size() * sizeof(_Float16), hipMemcpyHostToDevice));
  PA_HIP(hipMemcpy(d->scl, hs.data(), hs.size() * sizeof(float), hipMemcpyHostToDevice));
  PA_HIP(hipMemcpy(d->bstem3, hbs.data(), hbs.size() * sizeof(float), hipMemcpyHostToDevice));
  if (!d->tctr) {
    PA_HIP(hipMalloc(&d->tctr, 64 * sizeof(unsigned)));
    PA_HIP(hipMemset(d->tctr, 0, 64 * sizeof(unsigned)));
  }
  return PA_OK;
}

// Activation workspace: 3 ping-pong maps of B x 64x64x64 (the largest; later layers use
// a prefix), plus the 128x128 stem map of the unfused fp32 stem.  Element bytes: fp16 2,
// fp32 4, fp16x3 2 x 2 (hi / lo planes).
static size_t stem_elems(int B, int prec) { return prec == PA_PREC_FP32 ? (size_t)B * 128 * 128 * 64 : 0; }
static size_t ws_need(int B, int prec) {
  const size_t es = prec == PA_PREC_FP16 ? 2 : 4;
  const size_t act = (size_t)B * 64 * 64 * 64;
  return (stem_elems(B, prec) + 3 * act) * es + 1024;
}

static int ensure_head(pa_detector* d, int B);

static int ensure_ws(pa_detector* d, int B) {
  {
    const int rc = ensure_head(d, B);
    if (rc != PA_OK) return rc;
  }
  const size_t need = ws_need(B, d->prec);
  if (need <= d->ws_bytes) return PA_OK;
  if (d->ws) {
    PA_HIP(hipFree(d->ws));
    d->ws = nullptr;
    d->ws_bytes = 0;
  }
  if (hipMalloc(&d->ws, need) != hipSuccess) {
    (void)hipGetLastError();
    set_error("workspace: hipMalloc(%zu) failed", need);
    return PA_ENOMEM;
  }
  d->ws_bytes = need;
  return PA_OK;
}

// fused avgpool + fc (conv_gx.h gx_head): pooled means and zeroed arrival counters
static int ensure_head(pa_detector* d, int B) {
  if (B <= d->head_cap) return PA_OK;
  if (d->pool) PA_HIP(hipFree(d->pool));
  if (d->cnt) PA_HIP(hipFree(d->cnt));
  d->pool = nullptr;
  d->cnt = nullptr;
  d->head_cap = 0;
  const int npair = (B + 1) / 2;
  if (hipMalloc(&d->pool, (size_t)B * 512 * sizeof(float)) != hipSuccess ||
      hipMalloc(&d->cnt, (size_t)npair * sizeof(unsigned)) != hipSuccess) {
    (void)hipGetLastError();
    set_error("head workspace: hipMalloc failed");
    return PA_ENOMEM;
  }
  PA_HIP(hipMemset(d->cnt, 0, (size_t)npair * sizeof(unsigned)));
  PA_HIP(hipDeviceSynchronize());
  d->head_cap = B;
  return PA_OK;
}

// Per-launch device timing.  Mode 1 (target < 0): an event after every launch.
// Mode 2 (target = launch index): that launch is issued `reps` times back to back
// between two events and nothing else is marked, so the average is free of the
// inter-kernel event overhead (~5 us per launch in mode 1).
struct Prof {
  std::vector<hipEvent_t> ev;
  std::vector<const char*> names;
  hipStream_t s;
  int target = -1, reps = 1, cur = 0;
  hipEvent_t t0 = nullptr, t1 = nullptr;
  const char* target_name = nullptr;
  void record(const char* name) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return;
    hipEventRecord(e, s);
    ev.push_back(e);
    names.push_back(name);
  }
  void mark(const char* name) {
    if (target < 0) record(name);
  }
  int count() const { return (target == cur) ? reps : 1; }
  void before() {
    if (target == cur) hipEventRecord(t0, s);
  }
  void after(const char* name) {
    if (target == cur) {
      hipEventRecord(t1, s);
      target_name = name;
    }
    ++cur;
    mark(name);
  }
};

// one timed launch site: runs `call` once (or `reps` times if it is the profiled target)
#define PA_RUN(call, name)                                \
  do {                                                    \
    const int _n = prof ? prof->count() : 1;              \
    if (prof) prof->before();                             \
    for (int _r = 0; _r < _n; ++_r) {                     \
      int _rc = (call);                                   \
      if (_rc != PA_OK) return _rc;                       \
    }                                                     \
    if (prof) prof->after(name);                          \
  } while (0)

#define PA_TRY(x)                \
  do {                           \
    int _rc = (x);               \
    if (_rc != PA_OK) return _rc; \
  } while (0)

// small: the latency mode (pa_detector_set_split_k), decided once per forward call from
// the caller's whole batch (a chunk of a larger batch never switches to it)
template <typename T>
static int forward_t(pa_detector* d, const float* x, int B, float* y, hipStream_t s, Prof* prof, bool small,
                     const RgbdSrc* rgbd = nullptr, float* px = nullptr) {
  const T* wts = std::is_same<T, float>::value ? (const T*)d->w32 : (const T*)d->w16;
  T* S = reinterpret_cast<T*>(d->ws);
  const size_t stem_el = stem_elems(B, d->prec);
  const size_t act_el = (size_t)B * 64 * 64 * 64;
  T* X = S + stem_el;
  T* Tb = X + act_el;
  T* D = Tb + act_el;
  // g_variant[7] == 3: avgpool + fc fused into layer4's last conv (conv_gx.h gx_head).
  // Bit-identical to the separate head_fp16 and measured neutral (27.3 us for the fused
  // launch vs 19.5 + 6.7 us; 176.7k vs 177.3k frames/s interleaved), so not shipped.  It runs
  // with layer4 on its one-K-group form (4:65; the shipped K split has no fused head).
  bool fuse_head = false;
  if constexpr (std::is_same<T, _Float16>::value)
    fuse_head = g_variant[7] == 3 && g_variant[4] == 65 && d->n_kp == 8 && d->H == 256 && d->W == 256 &&
                d->blocks.back().ds < 0;
  if (prof) prof->mark("start");
  const ConvL& st = d->convs[0];
  if constexpr (std::is_same<T, _Float16>::value) {
    // fused conv7x7 + BN + ReLU + maxpool: the 128x128 map stays on chip
    if (rgbd)  // camera frames straight into the stem (preprocess fused into its row loads)
      PA_RUN(launch_stem_pool_rgbd(*rgbd, B, wts + st.w_off, d->bias + st.b_off, X, s), "stem_rgbd_conv7x7_pool");
    else
      PA_RUN(launch_stem_pool_fp16(x, B, d->in_ch, wts + st.w_off, d->bias + st.b_off, X, s), "stem_conv7x7_pool");
  } else {
    PA_RUN(launch_stem<T>(x, B, d->in_ch, wts + st.w_off, d->bias + st.b_off, S, s), "stem_conv7x7");
    PA_RUN(launch_maxpool<T>(S, B, 128, 128, 64, X, s), "maxpool");
  }
  int hw = 64;
  int launch = 1;  // stem = 0
  auto trace = [&]() { return g_trace ? g_trace + (size_t)TRACE_LAUNCH * launch++ : nullptr; };
  // stride-1 convs: split-K form for small batches (pa_detector_set_split_k, conv_splitk.hip)
  auto conv_s1 = [&](ConvArgs& a, const char** kn, const ConvL& cl) -> int {
    if (!(a.epi & EPI_HEAD)) a.cnt = d->tctr;  // (only conv_c64v.hip reads it)
    if constexpr (std::is_same<T, _Float16>::value) {
      const int layer = a.Hout == 64 ? 1 : a.Hout == 32 ? 2 : a.Hout == 16 ? 3 : a.Hout == 8 ? 4 : 0;
      // 2:80 - 2:82 (A/B): layer2 on conv_s1k.hip (weights in VGPRs, K split over the waves)
      if (layer == 2 && g_variant[2] >= 80 && g_variant[2] <= 82 && d->wk2 && cl.wk_off >= 0)
        return launch_conv3x3_s1k(a, d->wk2 + cl.wk_off, g_variant[2] - 80, s, kn);
      // g_variant[layer] == 71 (A/B): layer2 split as well, layer1 on the persistent kernel
      if (layer && small && (g_variant[layer] == 0 || g_variant[layer] == 71 || (g_variant[layer] >= 35 &&
                                                                                   g_variant[layer] <= 39)) &&
          !(a.epi & EPI_HEAD)) {
        const bool split_l2 = g_variant[layer] == 71;
        static const char* names[5] = {"", "conv3x3x_l1_small", "conv3x3x_l2_small", "conv3x3x_l3_splitk",
                                       "conv3x3x_l4_splitk"};
        *kn = (layer == 2 && split_l2) ? "conv3x3x_l2_splitk" : (layer == 1 && split_l2) ? "conv3x3c64_l1" : names[layer];
        a.part = d->part;
        return launch_conv3x3_splitk(a, s, split_l2);
      }
    }
    return launch_conv3x3_s1<T>(a, s, kn);
  };
  for (const Block& b : d->blocks) {
    const ConvL& c1 = d->convs[b.conv1];
    const ConvL& c2 = d->convs[b.conv2];
    const int ho = hw / c1.stride;
    const char* kn = nullptr;
    ConvArgs a{};
    a.B = B;
    a.Hin = hw;
    a.Win = hw;
    a.Hout = ho;
    a.Wout = ho;
    a.M = B * ho * ho;
    const T* res = X;
    T* out = X;  // identity block: residual add in place (same element, same thread)
    if (b.ds >= 0 && g_variant[5] == 0) {
      // conv1 3x3 s2 + bn1 + relu and downsample 1x1 s2 + bn in one pass over X
      const ConvL& cd = d->convs[b.ds];
      ConvS2Args sa{};
      sa.in = X;
      sa.w = wts + c1.w_off;
      sa.bias = d->bias + c1.b_off;
      sa.wds = wts + cd.w_off;
      sa.bias2 = d->bias + cd.b_off;
      if constexpr (std::is_same<T, _Float16>::value)
        sa.wfrag = (c1.cin == 64 && c1.cout == 128)    ? d->wv2   // conv_s2v.hip
                   : (c1.cin == 128 && c1.cout == 256) ? d->wv3   // conv_s2k.hip
                   : (c1.cin == 256 && c1.cout == 512) ? d->wv4
                                                       : nullptr;
      sa.out = Tb;
      sa.out2 = D;
      sa.B = B;
      sa.Hin = hw;
      sa.Win = hw;
      sa.Cin = c1.cin;
      sa.Hout = ho;
      sa.Wout = ho;
      sa.Cout = c1.cout;
      sa.trace = trace();
      bool small_s2 = false;
      if constexpr (std::is_same<T, _Float16>::value) small_s2 = small && g_variant[6] == 0 && ho != 16;
      if (small_s2) {
        sa.part = d->part;
        PA_RUN(launch_conv3x3s2_small(sa, s, &kn), kn);
      } else if (std::is_same<T, _Float16>::value && small && ho == 16 && g_variant[6] == 0) {
        // layer3's entry in the latency mode: conv_s2x.h tiles, 2 x 16 x 64 (96 workgroups at
        // B = 3, vs 12 for the batched conv_s2w.h tiles): 6.2 us vs 7.9 for 4 x 16 x 64 (variant
        // 3:71) and 8.8 for 4 x 16 x 128 (3:38), profiles/r04sm/
        PA_RUN(launch_conv3x3s2_x(sa, g_variant[3] == 38 ? 0 : g_variant[3] == 71 ? 2 : 18, s, &kn), kn);
      } else {
        PA_RUN(launch_conv3x3s2_ds<T>(sa, s, &kn), kn);
      }
      res = D;
      out = D;
    } else {
      // conv1 + bn1 + relu
      a.in = X;
      a.w = wts + c1.w_off;
      a.bias = d->bias + c1.b_off;
      a.res = nullptr;
      a.out = Tb;
      a.Cin = c1.cin;
      a.Cout = c1.cout;
      a.stride = c1.stride;
      a.pad = 1;
      a.epi = EPI_RELU;
      a.trace = trace();
      if (c1.stride == 1)
        PA_RUN(conv_s1(a, &kn, c1), kn);
      else
        PA_RUN(launch_conv<T>(a, 3, s, &kn), kn);
      if (b.ds >= 0) {
        const ConvL& cd = d->convs[b.ds];
        ConvArgs dsa = a;
        dsa.w = wts + cd.w_off;
        dsa.bias = d->bias + cd.b_off;
        dsa.out = D;
        dsa.pad = 0;
        dsa.epi = 0;
        PA_RUN(launch_conv<T>(dsa, 1, s, &kn), kn);
        res = D;
        out = D;
      }
    }
    // conv2 + bn2 + residual + relu
    ConvArgs b2{};
    b2.B = B;
    b2.Hin = ho;
    b2.Win = ho;
    b2.Hout = ho;
    b2.Wout = ho;
    b2.M = B * ho * ho;
    b2.in = Tb;
    b2.w = wts + c2.w_off;
    b2.bias = d->bias + c2.b_off;
    b2.res = res;
    b2.out = out;
    b2.Cin = c2.cin;
    b2.Cout = c2.cout;
    b2.stride = 1;
    b2.pad = 1;
    b2.epi = EPI_RELU | EPI_RES;
    b2.trace = trace();
    if (fuse_head && &b == &d->blocks.back()) {
      b2.epi |= EPI_HEAD;
      b2.pool = d->pool;
      b2.cnt = d->cnt;
      b2.fcw = d->fcw;
      b2.fcb = d->fcb;
      b2.y = y;
    }
    PA_RUN(conv_s1(b2, &kn, c2), kn);
    if (b.ds >= 0) std::swap(X, D);
    hw = ho;
  }
  if (!fuse_head)
    PA_RUN(launch_head<T>(X, B, hw * hw, 512, d->fcw, d->fcb, 2 * d->n_kp, y, s, px, d->H, d->W), "avgpool_fc");
  else if (px)
    PA_RUN(launch_postprocess(y, nullptr, B, d->n_kp, d->H, d->W, px, nullptr, s), "postprocess");
  return PA_OK;
}

// Points the launchers' thread-local variant / trace selectors at this handle's settings
// for one call (conv.h g_variant), restoring the previous ones on exit.
struct HandleScope {
  const int* v;
  unsigned long long* t;
  explicit HandleScope(const pa_detector* d) : v(g_variant), t(g_trace) {
    g_variant = d->variant;
    g_trace = d->trace;
  }
  ~HandleScope() {
    g_variant = v;
    g_trace = t;
  }
};

// Frames per forward_t pass.  Every activation offset in the kernels is 32-bit (buffer
// stores, 2 GB); a batch of B frames needs B * 64*64*64 * 2 bytes per fp16 map (x2 for
// the hi/lo pair of the fp16x3 mode), so larger batches run as consecutive chunks on the
// same stream (each chunk already fills the chip many times over).
constexpr int kChunk = 1024;

// fp16x3 parity mode: every conv as 3 fp16 MFMA products of hi/lo planes,
// f32 accumulate; same schedule and fusions as the fp16 path (stem + pool fused, stride-2
// conv + downsample fused, in-place residual), separate head.
// small: the fp16x3 latency mode (short stem bands, small tiles, layers 2-4 split-K,
// conv_splitk.hip); px (optional): the head also writes the denormalized pixels
static int forward_x3(pa_detector* d, const float* x, int B, float* y, hipStream_t s, Prof* prof, bool small,
                      float* px = nullptr) {
  _Float16* X = reinterpret_cast<_Float16*>(d->ws);
  const size_t act_el = (size_t)B * 64 * 64 * 64 * 2;  // two planes
  _Float16* Tb = X + act_el;
  _Float16* D = Tb + act_el;
  if (prof) prof->mark("start");
  const ConvL& st = d->convs[0];
  if (small)
    PA_RUN(launch_stem_pool_x3_small(x, B, d->in_ch, d->w3 + st.w3_off, d->bstem3, d->scl + st.b_off, X, s),
           "stem_x3_conv7x7_pool_small");
  else
    PA_RUN(launch_stem_pool_x3(x, B, d->in_ch, d->w3 + st.w3_off, d->bstem3, d->scl + st.b_off, X, s),
           "stem_x3_conv7x7_pool");
  int hw = 64;
  int launch = 1;  // stem = 0 (the trace slot of each launch, as forward_t)
  auto trace = [&]() { return g_trace ? g_trace + (size_t)TRACE_LAUNCH * launch++ : nullptr; };
  for (const Block& b : d->blocks) {
    const ConvL& c1 = d->convs[b.conv1];
    const ConvL& c2 = d->convs[b.conv2];
    const int ho = hw / c1.stride;
    const char* kn = nullptr;
    const _Float16* res = X;
    _Float16* out = X;  // identity block: residual add in place (same element, same thread)
    auto s1 = [&](ConvArgs& a) -> int {
      if (small) {
        a.part = d->part;
        return launch_conv3x3_splitk_x3(a, s, &kn);
      }
      switch (a.Hout) {
        case 64: kn = "conv3x3x3_l1"; return launch_conv3x3_x3_l1(a, s);
        case 32: kn = "conv3x3x3_l2"; return launch_conv3x3_x3_l2(a, s);
        case 16: kn = "conv3x3x3_l3"; return launch_conv3x3_x3_l3(a, s);
        case 8: kn = "conv3x3x3_l4"; return launch_conv3x3_x3_l4(a, s);
      }
      set_error("x3 conv: no configuration for %dx%d", a.Hout, a.Wout);
      return PA_EINVAL;
    };
    ConvArgs a{};
    a.B = B;
    a.Hin = hw;
    a.Win = hw;
    a.Hout = ho;
    a.Wout = ho;
    a.M = B * ho * ho;
    a.stride = 1;
    a.pad = 1;
    if (b.ds >= 0) {
      const ConvL& cd = d->convs[b.ds];
      ConvS2Args sa{};
      sa.in = X;
      sa.w = d->w3 + c1.w3_off;
      sa.bias = d->bias + c1.b_off;
      sa.scale = d->scl + c1.b_off;
      sa.wds = d->w3 + cd.w3_off;
      sa.bias2 = d->bias + cd.b_off;
      sa.scale2 = d->scl + cd.b_off;
      sa.wfrag = (c1.cin == 64 && c1.cout == 128)    ? d->wv2x3  // conv_x3s2v.hip
                 : (c1.cin == 128 && c1.cout == 256) ? d->wv3x3  // conv_x3s2k.hip
                                                     : nullptr;
      sa.out = Tb;
      sa.out2 = D;
      sa.B = B;
      sa.Hin = hw;
      sa.Win = hw;
      sa.Cin = c1.cin;
      sa.Hout = ho;
      sa.Wout = ho;
      sa.Cout = c1.cout;
      sa.part = d->part;
      sa.trace = trace();
      if (small)
        PA_RUN(launch_conv3x3s2_small_x3(sa, s, &kn), kn);
      else
        PA_RUN(launch_conv3x3s2_x3(sa, s, &kn), kn);
      res = D;
      out = D;
    } else {
      a.in = X;
      a.w = d->w3 + c1.w3_off;
      a.bias = d->bias + c1.b_off;
      a.scale = d->scl + c1.b_off;
      a.out = Tb;
      a.Cin = c1.cin;
      a.Cout = c1.cout;
      a.epi = EPI_RELU;
      a.trace = trace();
      PA_RUN(s1(a), kn);
    }
    ConvArgs b2 = a;
    b2.Hin = ho;
    b2.Win = ho;
    b2.in = Tb;
    b2.w = d->w3 + c2.w3_off;
    b2.bias = d->bias + c2.b_off;
    b2.scale = d->scl + c2.b_off;
    b2.res = res;
    b2.out = out;
    b2.Cin = c2.cin;
    b2.Cout = c2.cout;
    b2.epi = EPI_RELU | EPI_RES;
    b2.trace = trace();
    PA_RUN(s1(b2), kn);
    if (b.ds >= 0) std::swap(X, D);
    hw = ho;
  }
  PA_RUN(launch_head_x3(X, B, hw * hw, 512, d->fcw, d->fcb, 2 * d->n_kp, y, s, px, d->H, d->W), "avgpool_fc_x3");
  return PA_OK;
}

// the latency mode applies to the whole call (fp16 and fp16x3; fp32 has no such mode)
static bool small_mode(const pa_detector* d, int B) { return B <= d->splitk_max && d->prec != PA_PREC_FP32; }

// one chunk of frames (x: f32 NCHW) in the handle's precision
static int forward_chunk(pa_detector* d, const float* x, int nb, float* y, hipStream_t s, Prof* prof, bool small,
                         float* px) {
  if (d->prec == PA_PREC_FP32) return forward_t<float>(d, x, nb, y, s, prof, false, nullptr, px);
  if (d->prec == PA_PREC_FP16X3) return forward_x3(d, x, nb, y, s, prof, small, px);
  return forward_t<_Float16>(d, x, nb, y, s, prof, small, nullptr, px);
}

static int forward(pa_detector* d, const float* x, int B, float* y, hipStream_t s, Prof* prof, float* px = nullptr) {
  PA_CHECK(d, "null detector");
  PA_CHECK(B >= 0, "batch %d", B);
  if (B == 0) return PA_OK;
  PA_CHECK(x && y, "null input/output pointer");
  PA_TRY(ensure_ws(d, B < kChunk ? B : kChunk));
  HandleScope hs(d);
  const bool small = small_mode(d, B);
  const size_t in_frame = (size_t)d->in_ch * d->H * d->W, out_frame = 2 * (size_t)d->n_kp;
  for (int off = 0; off < B; off += kChunk) {
    const int nb = B - off < kChunk ? B - off : kChunk;
    const int rc = forward_chunk(d, x + off * in_frame, nb, y + off * out_frame, s, prof, small,
                                 px ? px + off * out_frame : nullptr);
    if (rc != PA_OK) return rc;
  }
  return PA_OK;
}

// the f32 (B, 4, 256, 256) input of the non-fused RGBD path (fp16x3 / fp32), grown outside
// any captured graph (the first call of a given batch size allocates)
static int ensure_xin(pa_detector* d, int B) {
  if (B <= d->xin_cap) return PA_OK;
  if (d->xin) PA_HIP(hipFree(d->xin));
  d->xin = nullptr;
  d->xin_cap = 0;
  if (hipMalloc(&d->xin, (size_t)B * 4 * 256 * 256 * sizeof(float)) != hipSuccess) {
    (void)hipGetLastError();
    set_error("forward_rgbd: input staging hipMalloc failed");
    return PA_ENOMEM;
  }
  d->xin_cap = B;
  return PA_OK;
}

// camera frames -> keypoints.  fp16: the preprocess is fused into the stem's row loads;
// fp16x3 / fp32: pa_preprocess_rgbd's kernel into the handle's f32 staging, then the forward
// (4-channel models)
static int forward_rgbd(pa_detector* d, const RgbdSrc& src, int B, float* y, hipStream_t s, float* px = nullptr) {
  PA_CHECK(d, "null detector");
  PA_CHECK(B >= 0, "batch %d", B);
  if (B == 0) return PA_OK;
  PA_CHECK(src.rgb && src.depth && y, "null input/output pointer");
  PA_CHECK(d->in_ch == 4, "forward_rgbd: needs a 4-channel (RGBD) model, have %d", d->in_ch);
  PA_CHECK(src.Hs >= 256 && src.Ws >= 256, "forward_rgbd: source %dx%d smaller than 256x256", src.Hs, src.Ws);
  PA_TRY(ensure_ws(d, B < kChunk ? B : kChunk));
  const bool fused = d->prec == PA_PREC_FP16;
  if (!fused) PA_TRY(ensure_xin(d, B < kChunk ? B : kChunk));
  HandleScope hs(d);
  const bool small = small_mode(d, B);
  const size_t frame = (size_t)src.Hs * src.Ws;
  for (int off = 0; off < B; off += kChunk) {
    const int nb = B - off < kChunk ? B - off : kChunk;
    RgbdSrc c = src;
    c.rgb = src.rgb + off * frame * 3;
    c.depth = src.depth + off * frame;
    float* yc = y + off * 2 * (size_t)d->n_kp;
    float* pc = px ? px + off * 2 * (size_t)d->n_kp : nullptr;
    int rc;
    if (fused) {
      rc = forward_t<_Float16>(d, nullptr, nb, yc, s, nullptr, small, &c, pc);
    } else {
      rc = launch_preprocess(c.rgb, c.depth, nb, c.Hs, c.Ws, c.bgr, c.near_m, c.far_m, d->H, d->W, d->xin, s);
      if (rc == PA_OK) rc = forward_chunk(d, d->xin, nb, yc, s, nullptr, small, pc);
    }
    if (rc != PA_OK) return rc;
  }
  return PA_OK;
}

}  // namespace pa

extern "C" {

int pa_detector_forward_rgbd(pa_detector* d, const uint8_t* rgb_dev, const float* depth_dev, int B, int Hs, int Ws,
                             int bgr, float near_m, float far_m, float* y_dev, void* stream) {
  const pa::RgbdSrc src{rgb_dev, depth_dev, Hs, Ws, bgr, near_m, far_m};
  return pa::forward_rgbd(d, src, B, y_dev, (hipStream_t)stream);
}

int pa_detector_forward_rgbd_px(pa_detector* d, const uint8_t* rgb_dev, const float* depth_dev, int B, int Hs, int Ws,
                                int bgr, float near_m, float far_m, float* y_dev, float* px_dev, void* stream) {
  PA_CHECK(px_dev, "forward_rgbd_px: null pixel output");
  const pa::RgbdSrc src{rgb_dev, depth_dev, Hs, Ws, bgr, near_m, far_m};
  return pa::forward_rgbd(d, src, B, y_dev, (hipStream_t)stream, px_dev);
}

int pa_host_device_pointer(const void* host, void** dev) {
  PA_CHECK(host && dev, "host_device_pointer: null pointer");
  void* p = nullptr;
  const hipError_t e = hipHostGetDevicePointer(&p, const_cast<void*>(host), 0);
  PA_CHECK(e == hipSuccess && p, "hipHostGetDevicePointer: %s (not a mapped pinned host buffer?)", hipGetErrorString(e));
  *dev = p;
  return PA_OK;
}

const char* pa_last_error(void) { return pa::g_err.c_str(); }
const char* pa_version(void) { return "perseus_amd 0.1 gfx950"; }

int pa_detector_create(const float* weights, size_t nbytes, int in_ch, int n_kp, int H, int W, pa_detector** out) {
  PA_CHECK(out, "null out");
  *out = nullptr;
  PA_CHECK(weights, "null weights");
  PA_CHECK(H == 256 && W == 256, "only 256x256 inputs are supported (got %dx%d)", H, W);
  PA_CHECK(in_ch >= 1 && in_ch <= 4, "in_ch %d not in [1,4]", in_ch);
  PA_CHECK(n_kp >= 1 && n_kp <= 16, "n_kp %d not in [1,16]", n_kp);
  PA_CHECK(nbytes % 4 == 0, "nbytes %zu not a multiple of 4", nbytes);
  pa_detector* d = new pa_detector();
  d->in_ch = in_ch;
  d->n_kp = n_kp;
  d->H = H;
  d->W = W;
  if (hipGetDevice(&d->device) != hipSuccess) {
    delete d;
    pa::set_error("hipGetDevice failed (no GPU?)");
    return PA_EHIP;
  }
  int rc = pa::build(d, weights, nbytes / 4);
  if (rc != PA_OK) {
    if (rc == -1 || rc == -2) {
      pa::set_error("weight blob size mismatch: %zu bytes for in_ch=%d n_kp=%d", nbytes, in_ch, n_kp);
      rc = PA_EINVAL;
    }
    pa_detector_destroy(d);
    return rc;
  }
  *out = d;
  return PA_OK;
}

void pa_detector_destroy(pa_detector* d) {
  if (!d) return;
  hipFree(d->w16);
  hipFree(d->w32);
  hipFree(d->bias);
  hipFree(d->fcw);
  hipFree(d->fcb);
  hipFree(d->w3);
  if (d->wv2) hipFree(d->wv2);
  if (d->wv3) hipFree(d->wv3);
  if (d->wv4) hipFree(d->wv4);
  if (d->wv2x3) hipFree(d->wv2x3);
  if (d->wv3x3) hipFree(d->wv3x3);
  if (d->wk2) hipFree(d->wk2);
  hipFree(d->scl);
  hipFree(d->bstem3);
  if (d->ws) hipFree(d->ws);
  if (d->pool) hipFree(d->pool);
  if (d->cnt) hipFree(d->cnt);
  if (d->tctr) hipFree(d->tctr);
  if (d->part) hipFree(d->part);
  if (d->xin) hipFree(d->xin);
  delete d;
}

int pa_detector_reserve(pa_detector* d, int max_batch) {
  PA_CHECK(d && max_batch >= 0, "bad arguments");
  // forward / forward_rgbd never use more than one chunk's workspace
  const int n = max_batch < pa::kChunk ? max_batch : pa::kChunk;
  PA_TRY(pa::ensure_ws(d, n));
  // forward_rgbd's f32 staging (fp16x3 / fp32 on a 4-channel model): reserved here too, so
  // that a graph captured after reserve() never allocates, and never keeps a pointer that a
  // later larger call frees
  if (d->in_ch == 4 && d->prec != PA_PREC_FP16) PA_TRY(pa::ensure_xin(d, n));
  d->reserved = n > d->reserved ? n : d->reserved;
  return PA_OK;
}

int pa_detector_set_split_k(pa_detector* d, int max_batch) {
  PA_CHECK(d, "null detector");
  PA_CHECK(max_batch >= 0 && max_batch <= 64, "split-K max batch %d not in [0,64]", max_batch);
  if (max_batch > d->splitk_max || max_batch == 0) {
    if (d->part) PA_HIP(hipFree(d->part));
    d->part = nullptr;
    d->splitk_max = 0;
    if (max_batch == 0) return PA_OK;
    if (hipMalloc(&d->part, pa::splitk_part_floats(max_batch) * sizeof(float)) != hipSuccess) {
      (void)hipGetLastError();
      pa::set_error("split-K partials: hipMalloc failed");
      return PA_ENOMEM;
    }
  }
  d->splitk_max = max_batch;
  return PA_OK;
}

int pa_detector_set_precision(pa_detector* d, int precision) {
  PA_CHECK(d, "null detector");
  PA_CHECK(precision == PA_PREC_FP16 || precision == PA_PREC_FP32 || precision == PA_PREC_FP16X3, "precision %d",
           precision);
  if (precision != d->prec) {
    // keep the same batch capacity for the new element size
    const size_t old = d->ws_bytes;
    int bcap = 0;
    while (bcap < pa::kChunk && pa::ws_need(bcap + 1, d->prec) <= old) ++bcap;
    d->prec = precision;
    if (bcap > 0) PA_TRY(pa::ensure_ws(d, bcap));
    // a reservation covers forward_rgbd's staging in the new precision too
    if (d->reserved > 0 && d->in_ch == 4 && precision != PA_PREC_FP16) PA_TRY(pa::ensure_xin(d, d->reserved));
  }
  return PA_OK;
}

int pa_detector_forward(pa_detector* d, const float* x_dev, int B, float* y_dev, void* stream) {
  return pa::forward(d, x_dev, B, y_dev, (hipStream_t)stream, nullptr);
}

int pa_detector_profile(pa_detector* d, const float* x_dev, int B, float* y_dev, void* stream, float* ms_out,
                        const char** names_out, int max_n) {
  // one chunk's launch sequence: a larger batch would repeat the marks per chunk
  PA_CHECK(B <= pa::kChunk, "profile: batch %d above the %d-frame chunk (profile one chunk)", B, pa::kChunk);
  pa::Prof p;
  p.s = (hipStream_t)stream;
  int rc = pa::forward(d, x_dev, B, y_dev, p.s, &p);
  if (rc == PA_OK && hipStreamSynchronize(p.s) != hipSuccess) {
    pa::set_error("profile: stream sync failed");
    rc = PA_EHIP;
  }
  int n = 0;
  if (rc == PA_OK) {
    for (size_t i = 1; i < p.ev.size() && n < max_n; ++i, ++n) {
      float ms = 0.f;
      hipEventElapsedTime(&ms, p.ev[i - 1], p.ev[i]);
      if (ms_out) ms_out[n] = ms;
      if (names_out) names_out[n] = p.names[i];
    }
  }
  for (hipEvent_t e : p.ev) hipEventDestroy(e);
  return rc == PA_OK ? n : rc;
}

int pa_detector_time_launch(pa_detector* d, const float* x_dev, int B, float* y_dev, void* stream, int index,
                            int reps, float* avg_ms_out, const char** name_out) {
  PA_CHECK(index >= 0 && reps >= 1, "index %d reps %d", index, reps);
  PA_CHECK(B <= pa::kChunk, "time_launch: batch %d above the %d-frame chunk (time one chunk)", B, pa::kChunk);
  pa::Prof p;
  p.s = (hipStream_t)stream;
  p.target = index;
  p.reps = reps;
  if (hipEventCreate(&p.t0) != hipSuccess || hipEventCreate(&p.t1) != hipSuccess) {
    pa::set_error("time_launch: hipEventCreate failed");
    return PA_EHIP;
  }
  int rc = pa::forward(d, x_dev, B, y_dev, p.s, &p);
  if (rc == PA_OK && !p.target_name) {
    pa::set_error("time_launch: launch index %d out of range (%d launches)", index, p.cur);
    rc = PA_EINVAL;
  }
  if (rc == PA_OK && hipStreamSynchronize(p.s) != hipSuccess) {
    pa::set_error("time_launch: stream sync failed");
    rc = PA_EHIP;
  }
  if (rc == PA_OK) {
    float ms = 0.f;
    hipEventElapsedTime(&ms, p.t0, p.t1);
    if (avg_ms_out) *avg_ms_out = ms / reps;
    if (name_out) *name_out = p.target_name;
  }
  hipEventDestroy(p.t0);
  hipEventDestroy(p.t1);
  return rc;
}

int pa_detector_debug_set_trace(pa_detector* d, unsigned long long* trace_dev) {
  PA_CHECK(d, "null detector");
  d->trace = trace_dev;
  return PA_OK;
}

// Variant ids whose kernels give wrong results by construction (timing experiments: MFMAs,
// DMAs, waits, stores or offset arithmetic removed).  Only a PA_TIMING_VARIANTS build has them;
// the release library refuses the ids, so no public call can reach wrong keypoints.
static bool timing_only_variant(int layer, int v) {
  switch (layer) {
    case 0: return v == 21 || v == 22 || v == 23 || v == 25 || v == 26;  // stem.hip
    case 1: return (v >= 37 && v <= 39) || v == 65 || v == 66 || (v >= 87 && v <= 89);  // c64, c64d, c64v
    case 3: return v >= 58 && v <= 62;  // conv_gx_l3.hip 8-12
    case 4: return v >= 60 && v <= 64;  // conv_gx_l4.hip 10-14
    default: return false;
  }
}

int pa_debug_timing_variants_built(void) { return PA_TIMING_VARIANTS; }

int pa_detector_debug_set_variant(pa_detector* d, int layer, int variant) {
  PA_CHECK(layer >= 0 && layer < 8 && variant >= 0, "layer %d variant %d", layer, variant);
  PA_CHECK(PA_TIMING_VARIANTS || !timing_only_variant(layer, variant),
           "variant %d:%d is timing-only (wrong results): not in the release library (build with "
           "PERSEUS_AMD_TIMING_VARIANTS=1)", layer, variant);
  PA_CHECK(d, "null detector");
  d->variant[layer] = variant;
  return PA_OK;
}

double pa_detector_flops_per_frame(const pa_detector* d) { return d ? d->flops_per_frame : 0.0; }

int pa_preprocess_rgbd(const uint8_t* rgb_dev, const float* depth_dev, int B, int Hs, int Ws, int bgr, float near_m,
                       float far_m, int H, int W, float* x_dev, void* stream) {
  PA_CHECK(B >= 0, "batch");
  if (B == 0) return PA_OK;
  PA_CHECK(rgb_dev && depth_dev && x_dev, "null pointer");
  return pa::launch_preprocess(rgb_dev, depth_dev, B, Hs, Ws, bgr, near_m, far_m, H, W, x_dev, (hipStream_t)stream);
}

int pa_keypoints_postprocess(const float* y_dev, const float* target_dev, int B, int n_kp, int H, int W,
                             float* px_dev, float* loss_dev, void* stream) {
  PA_CHECK(B >= 0 && n_kp > 0, "bad shape");
  if (B == 0) return PA_OK;
  PA_CHECK(y_dev && px_dev, "null pointer");
  return pa::launch_postprocess(y_dev, target_dev, B, n_kp, H, W, px_dev, loss_dev, (hipStream_t)stream);
}

}  // extern "C"
