// conv_gx.h instantiations for layer3 (16x16, 256 channels) (one file per layer: the fully unrolled
// kernels compile in parallel).  variant & 3 selects the tile / prefetch distance,
// variant & 4 turns the XCD-aware block order off.
#include "conv_gx.h"

namespace pa {

int launch_conv3x3_gx_l3(const ConvArgs& a, int variant, hipStream_t s) {
  if (a.B <= 0) return PA_OK;
  const bool xg = variant >= 10 || !(variant & 4);
  if (variant == 6) return run_gx<16, 16, 1, 64, 4, 2, 256, 3, 1, 0, 1, false>(a, true, s);  // plain (write-back) stores
  if (variant == 7 && a.trace) return run_gx<16, 16, 1, 64, 4, 2, 256, 3, 1, 4>(a, true, s);  // timestamps
#if PA_TIMING_VARIANTS
  // timing only (wrong results): 8 = no DMAs in the K loop, 9 = no K loop, 10 = DMAs, no waits /
  // barriers; 11 = DMAs + barriers, no vmcnt waits; 12 = barriers only, no DMAs in the K loop
  if (variant == 8) return run_gx<16, 16, 1, 64, 4, 2, 256, 3, 1, 2>(a, xg, s);
  if (variant == 9) return run_gx<16, 16, 1, 64, 4, 2, 256, 3, 1, 3>(a, xg, s);
  if (variant == 10) return run_gx<16, 16, 1, 64, 4, 2, 256, 3, 1, 1>(a, xg, s);
  if (variant == 11) return run_gx<16, 16, 1, 64, 4, 2, 256, 3, 1, 5>(a, xg, s);
  if (variant == 12) return run_gx<16, 16, 1, 64, 4, 2, 256, 3, 1, 6>(a, xg, s);
#endif
  // 16 (3:66): K split over two 4-wave groups (conv_gx.h KS = 2), 64 x 64 wave tiles
  if (variant == 16) return run_gx<16, 16, 1, 64, 4, 1, 256, 3, 1, 0, 1, true, false, false, 2>(a, xg, s);
  switch (variant & 3) {
      case 1: return run_gx<8, 16, 1, 64, 2, 2, 256, 3>(a, xg, s);  // 80 KB LDS: 2 workgroups per CU
      case 2: return run_gx<16, 16, 1, 64, 4, 2, 256, 4, 3>(a, xg, s);
      case 3: return run_gx<16, 16, 1, 64, 4, 2, 256, 3, 1, 0, 2>(a, xg, s);
      default: return run_gx<16, 16, 1, 64, 4, 2, 256, 3>(a, xg, s);
  }
}

}  // namespace pa
