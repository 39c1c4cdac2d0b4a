// conv_s2x.h instantiations: the stride-2 + downsample entry conv of layers 2-4.
// variant & 3 selects the tile / prefetch configuration, variant & 4 turns the
// XCD-aware block order off; 16.. are the multi-tile (TPW) workgroups.
#include "conv_s2x.h"

namespace pa {

int launch_conv3x3s2_x(const ConvS2Args& a, int variant, hipStream_t s, const char** kname) {
  if (a.B <= 0) return PA_OK;
  const bool xg = !(variant & 4);
  if (a.Hout == 32 && a.Cin == 64) {
    // shipped: 4x16 x 128 tiles, 4 per workgroup as one step stream (19.9 vs 21.1 us for
    // one 8x16 tile per workgroup in two rounds; tools/layer_ab.py, r02)
    if (kname) *kname = "conv3x3s2x_l2";
    if (variant & 8) return run_s2x<4, 16, 128, 2, 4, 64, 4, 1, false, false, 0, 4>(a, true, s);  // plain stores
    if (variant == 7 && a.trace) return run_s2x<4, 16, 128, 2, 4, 64, 4, 1, true, false, 4, 4>(a, true, s);  // timestamps
    if (variant == 19 && a.trace) return run_s2x<8, 16, 128, 4, 2, 64, 3, 1, true, false, 4>(a, xg, s);
    if (variant == 16) return run_s2x<4, 16, 128, 2, 2, 64, 3, 1, true, false, 0, 4>(a, true, s);  // 4 waves of 32x64
    if (variant == 17) return run_s2x<4, 16, 128, 2, 4, 64, 3, 1, true, false, 0, 4>(a, true, s);  // distance 3
    switch (variant & 3) {
      case 1: return run_s2x<8, 16, 128, 4, 2, 64, 3>(a, xg, s);  // one 8x16 tile per workgroup (round-1/2 kernel)
      case 2: return run_s2x<8, 16, 64, 4, 1, 64, 3>(a, xg, s);
      case 3: return run_s2x<4, 16, 128, 2, 2, 64, 3>(a, xg, s);
      default: return run_s2x<4, 16, 128, 2, 4, 64, 4, 1, true, false, 0, 4>(a, xg, s);
    }
  }
  if (a.Hout == 16 && a.Cin == 128) {
    if (kname) *kname = "conv3x3s2x_l3";
    if (variant & 8) return run_s2x<4, 16, 128, 2, 4, 128, 3, 1, false>(a, xg, s);  // plain (write-back) stores
    if (variant == 7 && a.trace) return run_s2x<4, 16, 128, 2, 4, 128, 3, 1, true, false, 4>(a, xg, s);  // timestamps
    if (variant == 17) return run_s2x<4, 16, 128, 2, 2, 128, 3, 1, true, false, 0, 2>(a, true, s);  // 19.9 vs 18.4 us
    if (variant == 18) return run_s2x<2, 16, 64, 2, 2, 128, 4>(a, xg, s);  // 2 x 16 x 64 tiles (small batches, A/B)
    switch (variant & 3) {
      case 1: return run_s2x<4, 16, 128, 2, 4, 128, 3, 2>(a, xg, s);
      case 2: return run_s2x<4, 16, 64, 2, 2, 128, 4>(a, xg, s);
      case 3: return run_s2x<4, 16, 128, 2, 2, 128, 3>(a, xg, s);
      default: return run_s2x<4, 16, 128, 2, 4, 128, 3>(a, xg, s);
    }
  }
  if (a.Hout == 8 && a.Cin == 256) {
    if (kname) *kname = "conv3x3s2x_l4";
    if (variant & 8) return run_s2x<8, 8, 128, 2, 4, 256, 3, 1, false>(a, xg, s);  // plain (write-back) stores
    if (variant == 7 && a.trace) return run_s2x<8, 8, 128, 2, 4, 256, 3, 1, true, false, 4>(a, xg, s);  // timestamps
    if (variant == 16) return run_s2x<8, 8, 128, 2, 4, 256, 3>(a, 2, s);  // 2 x 4 XCD split (channel halves x image groups)
    switch (variant & 3) {
      case 1: return run_s2x<8, 8, 128, 2, 4, 256, 2>(a, xg, s);
      case 2: return run_s2x<8, 8, 64, 2, 2, 256, 4>(a, xg, s);
      case 3: return run_s2x<8, 8, 128, 2, 2, 256, 3>(a, xg, s);
      default: return run_s2x<8, 8, 128, 2, 4, 256, 3>(a, xg, s);
    }
  }
  set_error("s2x conv: no configuration for %dx%d Cin %d", a.Hout, a.Wout, a.Cin);
  return PA_EINVAL;
}

}  // namespace pa
