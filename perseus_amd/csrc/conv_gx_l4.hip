// conv_gx.h instantiations for layer4 (8x8, 512 channels) (one file per layer: the fully unrolled
// kernels compile in parallel).  variant & 3 selects the tile / prefetch distance,
// variant & 4 turns the XCD-aware block order off.
#include "conv_gx.h"

namespace pa {

int launch_conv3x3_gx_l4(const ConvArgs& a, int variant, hipStream_t s) {
  if (a.B <= 0) return PA_OK;
  const bool xg = !(variant & 4);
  if (variant == 6) return run_gx<8, 8, 2, 64, 4, 2, 512, 4, 1, 0, 1, false>(a, true, s);  // plain (write-back) stores
  if (variant == 7 && a.trace) return run_gx<8, 8, 2, 64, 4, 2, 512, 4, 1, 4>(a, true, s);  // timestamps
  if (variant == 8) return run_gx<8, 8, 2, 64, 2, 2, 512, 4>(a, xg, s);  // 4 waves of 64x32 (1 per SIMD)
  if (variant == 9) return run_gx<8, 8, 2, 64, 2, 2, 512, 6>(a, xg, s);  // same, weight ring distance 6
  switch (variant & 3) {
      case 1: return run_gx<8, 8, 2, 64, 4, 2, 512, 4, 2>(a, xg, s);
      case 2: return run_gx<8, 8, 2, 64, 4, 2, 512, 4, 3>(a, xg, s);
      case 3: return run_gx<8, 8, 2, 64, 4, 2, 512, 4, 1, 0, 2>(a, xg, s);
      default: return run_gx<8, 8, 2, 64, 4, 2, 512, 4>(a, xg, s);
  }
}

}  // namespace pa
