// conv_gx.h X3 (fp16x3 parity mode) instantiation for layer1's 3x3 stride-1 convs
// (64x64); one file per layer so the fully unrolled kernels compile in parallel.
#include "conv_gx.h"

namespace pa {
int launch_conv3x3_x3v(const ConvArgs& a, hipStream_t s, bool ds, bool dsr, int ndr);
}

namespace pa {

int launch_conv3x3_x3_l1(const ConvArgs& a, hipStream_t s) {
  if (a.B <= 0) return PA_OK;
  PA_CHECK(a.Hout == 64 && a.Wout == 64, "x3 conv layer1: %dx%d", a.Hout, a.Wout);
  // merged x_hi steps (conv_gx.h XM) shipped; variant 70 keeps three virtual blocks per 64 channels
  if (g_variant[1] == 70) return run_gx<16, 16, 1, 64, 4, 2, 64, 3, 1, 0, 1, true, true>(a, true, s);
  // shipped (round 5): conv_x3v.hip, weights hi / lo in VGPRs, persistent 8-row tiles, bit-identical to
  // the merged-step gx form (variant 91): layer1 -2.2 to -3.9 us per launch, parity mode +0.7 % on the
  // driver's command, 5 of 6 interleaved pairs (profiles/r05_x3v/)
  if (g_variant[1] == 91) return run_gx<16, 16, 1, 64, 4, 2, 64, 3, 1, 0, 1, true, true, true>(a, true, s);
  // round 6: the plain convs with deferred stores (53.3 vs 56.9 us per launch, profiles/r06j/ab.log;
  // bit-identical); 1:90 keeps their stores at the tile end (1:92 = the shipped form); 1:98: the
  // residual convs' stores deferred as well (staged in place of their residual)
  // shipped (round 6): the residual convs' last row deferred in VGPRs (56.3 / 57.2 vs 59.3 / 60.2 us
  // per launch, profiles/r06m/ab_x3.log; bit-identical); 1:97 keeps all their stores at the tile end,
  // 1:99 defers their last two rows (3 VGPRs spill)
  const int v = g_variant[1];
  return launch_conv3x3_x3v(a, s, v != 90, v == 98, v == 97 ? 0 : v == 99 ? 2 : 1);
}

}  // namespace pa
