// conv_s2w.h instantiations: the stride-2 + downsample entries of layer2 and layer3 on
// 8 x 16 x 128 tiles with the row-split patch (shipped; layer4's 8 x 8 entry stays on
// conv_s2x.h), 8 waves of 32 px x 64 ch (the 64 px x 32 ch wave tile spills 28-59 VGPRs at
// the 256-register bound).  variant: 0 shipped, 1 = layer2: one tile per workgroup (two
// rounds) / layer3: prefetch distance 2, 2 = layer2: prefetch distance 2, 4 = XCD-aware order
// off.  (Prefetch distance 4 does not fit beside the 80 KB patch: 164 KB.)
#include "conv_s2w.h"

namespace pa {

int launch_conv3x3s2_w(const ConvS2Args& a, int variant, hipStream_t s, const char** kname) {
  if (a.B <= 0) return PA_OK;
  const bool xg = !(variant & 4);
  if (a.Hout == 32 && a.Cin == 64) {
    // 512 tiles at B = 64: two per workgroup as one step stream (one round of 256 workgroups;
    // variant 1 runs them as two rounds of one-tile workgroups)
    if (kname) *kname = "conv3x3s2w_l2";
    switch (variant & 3) {
      case 1: return run_s2w<128, 4, 2, 64, 3, 1>(a, xg, s);
      case 2: return run_s2w<128, 4, 2, 64, 2, 2>(a, xg, s);  // prefetch distance 2
      default: return run_s2w<128, 4, 2, 64, 3, 2>(a, xg, s);
    }
  }
  if (a.Hout == 16 && a.Cin == 128) {
    if (kname) *kname = "conv3x3s2w_l3";
    switch (variant & 3) {
      case 1: return run_s2w<128, 4, 2, 128, 2, 1>(a, xg, s);  // prefetch distance 2
      default: return run_s2w<128, 4, 2, 128, 3, 1>(a, xg, s);
    }
  }
  set_error("s2w conv: no configuration for %dx%d Cin %d", a.Hout, a.Wout, a.Cin);
  return PA_EINVAL;
}

}  // namespace pa
