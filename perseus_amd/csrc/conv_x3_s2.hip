// fp16x3 (parity mode) stride-2 + downsample entry convs.  Layers 2 / 3: conv_s2w.h's
// 8 x 16 x 128 tiles with the row-split patch (shipped; the x_hi patch is staged once for
// its two products); layer4 and the A/B forms: conv_s2x.h (conv_s2x_l.hip's tiles).
#include "conv_s2w.h"
#include "conv_s2x.h"

namespace pa {

// layer2's entry with the hi / lo weights in VGPRs (conv_x3s2v.hip)
int launch_conv3x3s2_v3(const ConvS2Args& a, int variant, hipStream_t s, const char** kname);
// layer3's with the hi / lo weights in VGPRs and K split over the waves by input block (conv_x3s2k.hip)
int launch_conv3x3s2_k3(const ConvS2Args& a, int variant, hipStream_t s, const char** kname);

int launch_conv3x3s2_x3(const ConvS2Args& a, hipStream_t s, const char** kname) {
  if (a.B <= 0) return PA_OK;
  const int v = g_variant[6];
  const bool s2x = v == 44 || v == 45;  // conv_s2x.h forms (A/B; 45 = its shipped tiles)
  // 6:57 / 6:58: layer2 on conv_x3s2v.hip, layer3 on conv_x3s2k.hip (58: with s_memrealtime stamps)
  // shipped from round 6: layer2 on conv_x3s2v.hip (44.6 vs 49.3 us on one box, 46.1 vs 45.7 on another:
  // profiles/r06h/ab.log, r06e/ab_x3.log; its minima 41-42 us against 45-49)
  if ((v == 0 || v == 57 || v == 58 || v == 62) && a.Hout == 32 && a.Cin == 64 && a.wfrag)
    return launch_conv3x3s2_v3(a, v == 58 ? 1 : 0, s, kname);
  // 6:60 / 6:61: layer2 on conv_x3s2v.hip with deferred stores (61: with stamps); layer3 as shipped
  if ((v == 60 || v == 61) && a.Hout == 32 && a.Cin == 64 && a.wfrag) return launch_conv3x3s2_v3(a, v == 60 ? 2 : 3, s, kname);
  // shipped from round 6: layer3 on conv_x3s2k.hip (35.9 vs 39.7 us, profiles/r06e/ab_x3.log); 6:59
  // keeps round 5's conv_s2w.h X3 kernel on layers 2 and 3 (and 6:46 / 44 / 45 below run their own forms)
  // 6:62: layer3's with deferred stores
  if ((v == 0 || (v >= 57 && v <= 62 && v != 59)) && a.Hout == 16 && a.Cin == 128 && a.wfrag)
    return launch_conv3x3s2_k3(a, v == 58 ? 1 : v == 62 ? 2 : 0, s, kname);
  if (a.Hout == 32 && a.Cin == 64) {
    if (!s2x) {
      // 64-channel tiles (the 128-channel X3 tile spills 43-110 VGPRs), two per workgroup (variant 46: one):
      // 49.5 / 52.2 us against 57.8 for conv_s2x.h (profiles/r04e/)
      if (kname) *kname = "conv3x3s2w3_l2";
      if (v == 46) return run_s2w<64, 4, 2, 64, 3, 1, true, true>(a, true, s);
      return run_s2w<64, 4, 2, 64, 3, 2, true, true>(a, true, s);
    }
    if (kname) *kname = "conv3x3s2x3_l2";
    // 8 waves of 32 x 32 (210 VGPRs): 55.1 us against 60.9 for 4 waves of 32 x 64 (366 VGPRs, one
    // wave per SIMD, variant 44); multi-tile workgroups spill here (85 / 77 us)
    if (v == 44) return run_s2x<4, 16, 128, 2, 2, 64, 3, 1, true, true>(a, true, s);
    return run_s2x<4, 16, 128, 2, 4, 64, 3, 1, true, true>(a, true, s);  // 2 patch buffers: 4-row tile
  }
  if (a.Hout == 16 && a.Cin == 128) {
    if (!s2x) {
      if (kname) *kname = "conv3x3s2w3_l3";
      // two tiles per workgroup (4 VGPRs spilled; 43.9 vs 45.2 us for one, variant 46, and 47.4 for
      // conv_s2x.h, profiles/r04e/)
      if (v == 46) return run_s2w<64, 4, 2, 128, 3, 1, true, true>(a, true, s);
      return run_s2w<64, 4, 2, 128, 3, 2, true, true>(a, true, s);
    }
    if (kname) *kname = "conv3x3s2x3_l3";
    return run_s2x<4, 16, 128, 2, 4, 128, 3, 1, true, true>(a, true, s);
  }
  if (a.Hout == 8 && a.Cin == 256) {
    if (kname) *kname = "conv3x3s2x3_l4";
    return run_s2x<8, 8, 128, 2, 4, 256, 3, 1, true, true>(a, true, s);
  }
  set_error("s2x3 conv: no configuration for %dx%d Cin %d", a.Hout, a.Wout, a.Cin);
  return PA_EINVAL;
}

}  // namespace pa
