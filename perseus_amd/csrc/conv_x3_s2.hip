// conv_s2x.h X3 (fp16x3 parity mode) instantiations: the stride-2 + downsample entry
// conv of layers 2-4, same tiles as the fp16 kernels (conv_s2x_l.hip).
#include "conv_s2x.h"

namespace pa {

int launch_conv3x3s2_x3(const ConvS2Args& a, hipStream_t s, const char** kname) {
  if (a.B <= 0) return PA_OK;
  if (a.Hout == 32 && a.Cin == 64) {
    if (kname) *kname = "conv3x3s2x3_l2";
    // 8 waves of 32 x 32 (210 VGPRs): 55.1 us against 60.9 for 4 waves of 32 x 64 (366 VGPRs, one
    // wave per SIMD, variant 44); multi-tile workgroups spill here (85 / 77 us)
    if (g_variant[6] == 44) return run_s2x<4, 16, 128, 2, 2, 64, 3, 1, true, true>(a, true, s);
    return run_s2x<4, 16, 128, 2, 4, 64, 3, 1, true, true>(a, true, s);  // 2 patch buffers: 4-row tile
  }
  if (a.Hout == 16 && a.Cin == 128) {
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
