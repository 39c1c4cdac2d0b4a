// conv_gx.h instantiations for layer4 (8x8, 512 channels) (one file per layer: the fully unrolled
// kernels compile in parallel).  variant & 1 selects the barrier spacing, variant & 4 turns
// the XCD-aware block order off.
#include "conv_gx.h"

namespace pa {

static int xgv_of(bool xg) { return xg ? 4 : 0; }

int launch_conv3x3_gx_l4(const ConvArgs& a, int variant, hipStream_t s) {
  if (a.B <= 0) return PA_OK;
  const bool xg = variant >= 10 || !(variant & 4);
  // round-1 sweep ("measured and not shipped"): G = 3, fragments a full
  // step ahead, write-back stores, 4-wave tiles and ring distance 6 were removed from
  // the build (each fully unrolled 72-step kernel costs minutes of compile time)
#if PA_TIMING_VARIANTS
  // timing only (wrong results), as layer3's 8-12
  if (variant == 10) return run_gx<8, 8, 2, 64, 4, 2, 512, 4, 1, 1>(a, xgv_of(xg), s);
  if (variant == 11) return run_gx<8, 8, 2, 64, 4, 2, 512, 4, 1, 5>(a, xgv_of(xg), s);
  if (variant == 12) return run_gx<8, 8, 2, 64, 4, 2, 512, 4, 1, 6>(a, xgv_of(xg), s);
  if (variant == 13) return run_gx<8, 8, 2, 64, 4, 2, 512, 4, 1, 2>(a, xgv_of(xg), s);
  if (variant == 14) return run_gx<8, 8, 2, 64, 4, 2, 512, 4, 1, 3>(a, xgv_of(xg), s);
#endif
  // shipped (round 6): the K split over two 4-wave groups (conv_gx.h KS = 2: 64 x 32 wave tiles, 0.75
  // fragment reads per MFMA instead of 1.0), a barrier every 2 steps; 20.5 / 19.9 / 20.5 vs 21.7 / 21.1 /
  // 21.6 us per launch for 15 (profiles/r06o/ab.log); 17 (4:67) names it explicitly.  Measured and
  // removed: the same with a barrier every step (4:66, 21.2 / 20.7 / 21.1 us).
  if (variant == 0 || variant == 17) return run_gx<8, 8, 2, 64, 2, 2, 512, 4, 2, 0, 1, true, false, false, 2>(a, 4, s);
  if (variant == 8 || variant == 9)  // 2-D XCD split: 4 / 2 channel groups per XCD
    return run_gx<8, 8, 2, 64, 4, 2, 512, 4>(a, variant == 8 ? 4 : 2, s);
  // 15 (4:65): shipped until round 6, one K group of 8 waves (32 x 32 wave tiles), 4 channel groups per
  // XCD (round 2: HBM traffic 31-35 MB vs 46-51 per launch with the 1-D order, time unchanged within 1 %,
  // bit-identical); 1 / 5: its barrier every 2 steps (bit-identity cross-check), 4: 1-D order
  const int xgv = xg ? 4 : 0;
  switch (variant & 3) {
    case 1: return run_gx<8, 8, 2, 64, 4, 2, 512, 4, 2>(a, xgv, s);
    default: return run_gx<8, 8, 2, 64, 4, 2, 512, 4>(a, xgv, s);
  }
}

}  // namespace pa
