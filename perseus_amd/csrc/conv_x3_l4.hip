// conv_gx.h X3 (fp16x3 parity mode) instantiation for layer4's 3x3 stride-1 convs
// (8x8); one file per layer so the fully unrolled kernels compile in parallel.
#include "conv_gx.h"

namespace pa {

int launch_conv3x3_x3_l4(const ConvArgs& a, hipStream_t s) {
  if (a.B <= 0) return PA_OK;
  PA_CHECK(a.Hout == 8 && a.Wout == 8, "x3 conv layer4: %dx%d", a.Hout, a.Wout);
  // merged x_hi steps (conv_gx.h XM) shipped; variant 70 keeps three virtual blocks per 64 channels
  // variant 70 keeps three virtual blocks per 64 channels; 74: merged steps in one K group of 8 waves
  // (32 x 32 wave tiles, shipped until round 6)
  if (g_variant[4] == 70) return run_gx<8, 8, 2, 64, 4, 2, 512, 4, 1, 0, 1, true, true>(a, true, s);
  if (g_variant[4] == 74) return run_gx<8, 8, 2, 64, 4, 2, 512, 4, 1, 0, 1, true, true, true>(a, true, s);
  // shipped (round 6): the K split over two 4-wave groups (conv_gx.h KS = 2, 64 x 32 wave tiles: 0.5
  // fragment reads per MFMA instead of 0.75); 50.8 / 49.7 / 50.8 vs 52.1 / 51.0 / 52.1 us per launch
  // (variant 72 then, profiles/r06o_x3/ab.log); 72 names it explicitly
  return run_gx<8, 8, 2, 64, 2, 2, 512, 4, 1, 0, 1, true, true, true, 2>(a, true, s);
}

}  // namespace pa
