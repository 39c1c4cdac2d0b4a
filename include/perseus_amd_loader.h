/*
 * perseus_amd loader — C ABI of the keypoint-dataset item loader, host side
 * of libperseus_amd.so.  It replaces the per-item file decode of
 *   perseus/detector/data.py:73-102  PrunedKeypointDataset.__getitem__
 *     image  np.asarray(Image.open(png).convert("RGB"), float32).transpose(2, 0, 1) / 255.0
 *     depth  tifffile.TiffFile(tiff).pages[0].asarray()
 *     seg    np.asarray(Image.open(png)) == asset_id + 1  (0 / 1, uint8)
 * with native PNG / TIFF decoders and one call per batch over a pool of host threads.  The
 * HDF5 index (data.py:46-66) stays with the caller: h5py is not part of this image.
 *
 * All pointers are host pointers; outputs are caller-owned.  Return codes and
 * pa_last_error() as in perseus_amd.h.
 *
 * Supported files (PA_EINVAL with a message otherwise):
 *   PNG   bit depth 8 (palette also 1 / 2 / 4), colour types gray, RGB, palette, gray+alpha,
 *         RGBA; not interlaced.
 *   TIFF  one sample per pixel, 8 / 16-bit unsigned or 32-bit float samples, strips (no tiles),
 *         compression none / LZW / Deflate (8, 32946), predictor none / horizontal / floating
 *         point, either byte order.
 */
#ifndef PERSEUS_AMD_LOADER_H
#define PERSEUS_AMD_LOADER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* PNG header: *h, *w, *channels of the samples pa_png_decode(raw = 1) writes (palette: 1) */
int pa_png_info(const uint8_t* buf, size_t n, int* h, int* w, int* channels);

/* Decode a PNG held in memory.  rgb = 1: PIL Image.convert("RGB") — h x w x 3 (gray replicated,
 * alpha dropped, palette looked up); rgb = 0: np.asarray(Image.open()) — the stored samples,
 * palette indices for palette images.  `cap` = bytes available at `out`. */
int pa_png_decode(const uint8_t* buf, size_t n, int rgb, uint8_t* out, size_t cap);

/* TIFF page 0 header: *h, *w */
int pa_tiff_info(const uint8_t* buf, size_t n, int* h, int* w);

/* Decode TIFF page 0 to f32 (h x w); unsigned samples convert exactly. `cap` in floats. */
int pa_tiff_decode_f32(const uint8_t* buf, size_t n, float* out, size_t cap);

/* One batch of data.py items, item i from image_paths[i], depth_paths[i] and
 * seg_paths[i] / asset_ids[i] (any of the three path arrays may be NULL to skip it):
 *   image  [B][3][h][w] f32  = f32(rgb) / 255.0f (data.py:88, numpy f32 division)
 *   depth  [B][h][w]    f32
 *   seg    [B][h][w]    u8   = (sample == asset_id + 1)   (data.py:92-95)
 * Every file must be h x w.  n_threads <= 0: one per core of the affinity mask. */
int pa_load_keypoint_items(const char* const* image_paths, const char* const* depth_paths,
                           const char* const* seg_paths, const int32_t* asset_ids, int B, int h, int w,
                           int n_threads, float* image, float* depth, uint8_t* seg);

#ifdef __cplusplus
}
#endif

#endif /* PERSEUS_AMD_LOADER_H */
