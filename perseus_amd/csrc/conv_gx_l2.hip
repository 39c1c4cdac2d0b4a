// conv_gx.h instantiations for layer2 (32x32, 128 channels) (one file per layer: the fully unrolled
// kernels compile in parallel).  variant & 3 selects the tile / prefetch distance,
// variant & 4 turns the XCD-aware block order off.
#include "conv_gx.h"

namespace pa {

int launch_conv3x3_gx_l2(const ConvArgs& a, int variant, hipStream_t s) {
  if (a.B <= 0) return PA_OK;
  const bool xg = !(variant & 4);
  if (variant == 6) return run_gx<16, 16, 1, 128, 4, 2, 128, 3, 1, 0, 1, false>(a, true, s);  // plain (write-back) stores
  if (variant == 7 && a.trace) return run_gx<16, 16, 1, 128, 4, 2, 128, 3, 1, 4>(a, true, s);  // timestamps
  if (variant == 5) return run_gx<4, 16, 1, 64, 2, 2, 128, 3>(a, xg, s);  // 4 x 16 tiles (small batches)
  if (variant == 8) return run_gx<2, 16, 1, 64, 2, 2, 128, 3>(a, xg, s);  // 2 x 16 tiles (small batches, A/B)
  switch (variant & 3) {
      case 1: return run_gx<8, 16, 1, 64, 2, 2, 128, 3>(a, xg, s);  // 80 KB LDS: 2 workgroups per CU
      case 3: return run_gx<16, 16, 1, 64, 4, 2, 128, 3, 1, 0, 2>(a, xg, s);
      default: return run_gx<16, 16, 1, 128, 4, 2, 128, 3>(a, xg, s);
  }
}

}  // namespace pa
