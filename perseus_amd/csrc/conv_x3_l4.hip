// conv_gx.h X3 (fp16x3 parity mode) instantiation for layer4's 3x3 stride-1 convs
// (8x8); one file per layer so the fully unrolled kernels compile in parallel.
#include "conv_gx.h"

namespace pa {

int launch_conv3x3_x3_l4(const ConvArgs& a, hipStream_t s) {
  if (a.B <= 0) return PA_OK;
  PA_CHECK(a.Hout == 8 && a.Wout == 8, "x3 conv layer4: %dx%d", a.Hout, a.Wout);
  // merged x_hi steps (conv_gx.h XM) shipped; variant 70 keeps three virtual blocks per 64 channels
  // variant 72: K split over two 4-wave groups (conv_gx.h KS = 2), 64 x 32 wave tiles
  if (g_variant[4] == 72) return run_gx<8, 8, 2, 64, 2, 2, 512, 4, 1, 0, 1, true, true, true, 2>(a, true, s);
  if (g_variant[4] == 70) return run_gx<8, 8, 2, 64, 4, 2, 512, 4, 1, 0, 1, true, true>(a, true, s);
  return run_gx<8, 8, 2, 64, 4, 2, 512, 4, 1, 0, 1, true, true, true>(a, true, s);
}

}  // namespace pa
