"""Keypoint-dataset items <- perseus/detector/data.py:14-102.

`KeypointDatasetConfig` and `PrunedKeypointDataset` keep the reference's names, constructor
and `__getitem__` contract (the same dict of tensors, the same dtypes and values); the file
decode is the native loader of libperseus_amd.so (include/perseus_amd_loader.h: PNG and
TIFF decoders, one call per batch over a pool of host threads) instead of PIL + tifffile in
DataLoader worker processes.  `load_batch` returns a whole batch stacked (optionally in
pinned memory, ready for an async copy to the GPU).

One recorded deviation: `depth_image` is always f32.  tifffile returns the page's native
dtype (data.py:79-80), so for the float32 depth TIFFs the reference's datagen writes
(generate_and_label_keypoints.py:93) the items are identical; an integer (e.g. uint16)
depth TIFF would come back as an integer tensor there and as the same values in f32 here.
How tifffile itself decodes float TIFFs with predictor 2 is not pinned by any fixture
(parity unpinned; tests/test_loader.py pins the stored samples instead).

The HDF5 index (data.py:46-66: attrs W / H and, per split, weights, pixel_coordinates,
asset_ids and the three file-name arrays) is read with h5py when it is importable; this
image has no h5py, so `from_index` takes the same arrays directly.
"""

from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

from . import _lib


@dataclass(frozen=True)
class KeypointDatasetConfig:
    """Configuration for the keypoint dataset (data.py:14-19)."""

    dataset_path: str = "data/pruned_dataset/pruned.hdf5"
    lazy: bool = True


def _names(a) -> list[str]:
    return [x.decode("utf-8") if isinstance(x, (bytes, np.bytes_)) else str(x) for x in a]


class PrunedKeypointDataset:
    """A pruned keypoint dataset (data.py:22-102): flattened images with their depth and
    segmentation files, pixel coordinates of the keypoints and per-item asset ids.

    `root` plays the reference's perseus ROOT: relative dataset paths resolve against it and
    the image files live under `root/data/`."""

    def __init__(self, cfg: KeypointDatasetConfig, train: bool = True, root: str | None = None) -> None:
        try:
            import h5py
        except ImportError as e:
            raise ImportError("PrunedKeypointDataset(cfg) reads the HDF5 index with h5py, which is not installed; "
                              "use PrunedKeypointDataset.from_index(...) with the index arrays") from e
        self.cfg = cfg
        self.train = train
        self.root = root if root is not None else os.getcwd()
        path = cfg.dataset_path if cfg.dataset_path.startswith("/") else os.path.join(self.root, cfg.dataset_path)
        with h5py.File(path, "r") as f:
            d = f["train"] if train else f["test"]
            self._set(W=int(f.attrs["W"]), H=int(f.attrs["H"]), weights=d["weights"][()],
                      pixel_coordinates=d["pixel_coordinates"][()], asset_ids=d["asset_ids"][()],
                      image_filenames=d["image_filenames"][()], depth_filenames=d["depth_filenames"][()],
                      segmentation_filenames=d["segmentation_filenames"][()])

    @classmethod
    def from_index(cls, *, image_filenames, depth_filenames, segmentation_filenames, asset_ids, pixel_coordinates,
                   H: int, W: int, weights=None, root: str | None = None, train: bool = True):
        """The dataset from its index arrays (what data.py:46-66 reads from the HDF5 file)."""
        self = cls.__new__(cls)
        self.cfg = None
        self.train = train
        self.root = root if root is not None else os.getcwd()
        self._set(W=int(W), H=int(H), weights=weights, pixel_coordinates=pixel_coordinates, asset_ids=asset_ids,
                  image_filenames=image_filenames, depth_filenames=depth_filenames,
                  segmentation_filenames=segmentation_filenames)
        return self

    def _set(self, *, W, H, weights, pixel_coordinates, asset_ids, image_filenames, depth_filenames,
             segmentation_filenames):
        import torch

        self.W, self.H = W, H
        self.weights = weights
        self.pixel_coordinates = torch.as_tensor(np.asarray(pixel_coordinates))
        self.asset_ids = np.asarray(asset_ids)
        self.image_filenames = _names(image_filenames)
        self.depth_filenames = _names(depth_filenames)
        self.segmentation_filenames = _names(segmentation_filenames)
        n = len(self.image_filenames)
        if not (len(self.depth_filenames) == len(self.segmentation_filenames) == len(self.asset_ids) == n
                and len(self.pixel_coordinates) == n):
            raise ValueError("index arrays differ in length")

    def __len__(self) -> int:
        """The number of images in the dataset."""
        return len(self.image_filenames)

    def _path(self, name: str) -> bytes:
        return os.path.join(self.root, "data", name).encode()

    def load_batch(self, indices, n_threads: int = 0, pin_memory: bool = False) -> dict:
        """Items `indices` stacked: image (B,3,H,W) f32, depth_image (B,H,W) f32,
        segmentation_image (B,H,W) u8, pixel_coordinates (B,...) -- each item what
        data.py:73-102 returns.  n_threads <= 0: one per core of the affinity mask."""
        import torch

        idx = [int(i) for i in np.asarray(indices).reshape(-1)]
        for i in idx:
            if not -len(self) <= i < len(self):
                raise IndexError(i)
        idx = [i % len(self) for i in idx]
        B, H, W = len(idx), self.H, self.W
        image = torch.empty((B, 3, H, W), dtype=torch.float32, pin_memory=pin_memory)
        depth = torch.empty((B, H, W), dtype=torch.float32, pin_memory=pin_memory)
        seg = torch.empty((B, H, W), dtype=torch.uint8, pin_memory=pin_memory)
        arr = C.c_char_p * max(B, 1)
        ip = arr(*[self._path(self.image_filenames[i]) for i in idx])
        dp = arr(*[self._path(self.depth_filenames[i]) for i in idx])
        sp = arr(*[self._path(self.segmentation_filenames[i]) for i in idx])
        aid = np.ascontiguousarray([self.asset_ids[i] for i in idx], dtype=np.int32)
        L = _lib.lib()
        _lib.check(L.pa_load_keypoint_items(ip, dp, sp, aid.ctypes.data if B else None, B, H, W, int(n_threads),
                                            image.data_ptr(), depth.data_ptr(), seg.data_ptr()), "load_batch")
        return {"image": image, "depth_image": depth, "segmentation_image": seg,
                "pixel_coordinates": self.pixel_coordinates[idx]}

    def __getitem__(self, idx: int) -> dict:
        """Get an item from the dataset (data.py:73-102)."""
        b = self.load_batch([idx], n_threads=1)
        return {"image": b["image"][0], "depth_image": b["depth_image"][0],
                "segmentation_image": b["segmentation_image"][0], "pixel_coordinates": self.pixel_coordinates[idx]}


def decode_png(data: bytes, rgb: bool = True) -> np.ndarray:
    """One PNG in memory: PIL `Image.open(...).convert("RGB")` (rgb) or `np.asarray(Image.open(...))`."""
    L = _lib.lib()
    h, w, c = C.c_int(), C.c_int(), C.c_int()
    buf = (C.c_char * len(data)).from_buffer_copy(data)
    _lib.check(L.pa_png_info(buf, len(data), C.byref(h), C.byref(w), C.byref(c)), "png")
    ch = 3 if rgb else c.value
    out = np.empty((h.value, w.value, ch), dtype=np.uint8)
    _lib.check(L.pa_png_decode(buf, len(data), int(rgb), out.ctypes.data, out.nbytes), "png")
    return out if ch > 1 else out[:, :, 0]


def decode_tiff(data: bytes) -> np.ndarray:
    """Page 0 of a one-sample TIFF in memory as f32 (tifffile `pages[0].asarray()` values)."""
    L = _lib.lib()
    h, w = C.c_int(), C.c_int()
    buf = (C.c_char * len(data)).from_buffer_copy(data)
    _lib.check(L.pa_tiff_info(buf, len(data), C.byref(h), C.byref(w)), "tiff")
    out = np.empty((h.value, w.value), dtype=np.float32)
    _lib.check(L.pa_tiff_decode_f32(buf, len(data), out.ctypes.data, out.size), "tiff")
    return out
