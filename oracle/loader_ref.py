"""ORACLE (test infrastructure only) — the reference's per-item decode, for the loader tests.

Only tests/ and tools/loader_bench.py's reference leg use this.

Restates `perseus/detector/data.py:73-102` (PrunedKeypointDataset.__getitem__) with the
libraries it calls:
  * image: PIL `Image.open(png).convert("RGB")` -> np.float32 -> transpose(2, 0, 1) / 255.0
    (data.py:85, :88; PIL 12.2 is installed here)
  * depth: `tifffile.TiffFile(tiff).pages[0].asarray()` (data.py:86-87).  tifffile is NOT
    installed in this image (unpinned in the reference's pyproject); its values for a
    one-sample float / uint TIFF are the stored samples, so this restatement reads page 0
    with PIL's libtiff-backed TIFF reader instead (mode F / I;16 -> the same samples).
  * segmentation: `np.asarray(Image.open(png))`, zeros_like, `== asset_id + 1` -> 1 (data.py:89,
    :93-95).
"""
from __future__ import annotations

import os

import numpy as np
import torch
from PIL import Image


def read_depth(path: str) -> np.ndarray:
    with Image.open(path) as im:
        return np.asarray(im)


def get_item(root: str, image_name: str, depth_name: str, seg_name: str, asset_id: int, pixel_coordinates):
    image_filename = os.path.join(root, "data", image_name)
    depth_filename = os.path.join(root, "data", depth_name)
    segmentation_filename = os.path.join(root, "data", seg_name)
    _image = np.asarray(Image.open(image_filename).convert("RGB"), dtype=np.float32)
    _depth_image = read_depth(depth_filename)
    original_seg_image = np.asarray(Image.open(segmentation_filename))
    image = torch.from_numpy(_image.transpose(2, 0, 1) / 255.0)
    depth_image = torch.from_numpy(np.array(_depth_image))
    segmentation_image = np.zeros_like(original_seg_image)
    segmentation_image[np.array(original_seg_image) == (asset_id + 1)] = 1
    segmentation_image = torch.from_numpy(segmentation_image)
    return {"image": image, "depth_image": depth_image, "segmentation_image": segmentation_image,
            "pixel_coordinates": pixel_coordinates}
