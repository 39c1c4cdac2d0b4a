"""Keypoint-dataset loader throughput: the native batch loader
(perseus_amd.data.PrunedKeypointDataset.load_batch, libperseus_amd.so PNG / TIFF decoders
on host threads) against the reference's per-item decode (oracle/loader_ref.get_item: PIL
for the PNGs; PIL's libtiff reader standing in for tifffile, which is not installed).

    python tools/loader_bench.py [--items 256] [--size 256] [--reps 3]

Synthetic files of the dataset's shape in a temporary directory: 256x256 RGB PNG (PIL,
default compression), f32 depth TIFF (Deflate), 8-bit palette segmentation PNG.  Prints
one JSON line: items/s for the native loader at 1 thread and at every core of the
affinity mask, and for the reference decode in one process (the reference runs 8
DataLoader worker processes, validate.py:99-105; its aggregate is at most 8x that).
"""
import argparse
import io
import json
import os
import statistics
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--items", type=int, default=256)
    p.add_argument("--size", type=int, default=256)
    p.add_argument("--reps", type=int, default=3)
    a = p.parse_args()
    import numpy as np
    from PIL import Image

    from oracle import loader_ref
    from perseus_amd.data import PrunedKeypointDataset

    rng = np.random.default_rng(0)
    n, s = a.items, a.size
    with tempfile.TemporaryDirectory() as root:
        os.makedirs(os.path.join(root, "data"))
        names = ([], [], [])
        yy, xx = np.mgrid[0:s, 0:s]
        for i in range(n):
            # smooth images with noise (rendered frames compress, random bytes would not)
            base = (np.sin(xx / (7 + i % 5)) + np.cos(yy / (11 + i % 3))) * 60 + 128
            rgb = np.clip(base[..., None] + rng.normal(0, 8, (s, s, 3)), 0, 255).astype(np.uint8)
            Image.fromarray(rgb, "RGB").save(os.path.join(root, "data", f"{i}.png"))
            depth = (0.12 + 0.36 * (base / 255.0)).astype(np.float32) / np.float32(0.035)
            depth[rng.random((s, s)) < 0.25] = 0.0
            Image.fromarray(depth, "F").save(os.path.join(root, "data", f"{i}_d.tiff"), compression="tiff_deflate")
            seg = np.zeros((s, s), np.uint8)
            seg[s // 4:3 * s // 4, s // 4:3 * s // 4] = 1 + i % 3
            im = Image.fromarray(seg, "P")
            im.putpalette([0, 0, 0, 255, 0, 0, 0, 255, 0, 0, 0, 255] + [0] * 756)
            im.save(os.path.join(root, "data", f"{i}_s.png"))
            names[0].append(f"{i}.png")
            names[1].append(f"{i}_d.tiff")
            names[2].append(f"{i}_s.png")
        aid = np.arange(n) % 3
        ds = PrunedKeypointDataset.from_index(image_filenames=names[0], depth_filenames=names[1],
                                              segmentation_filenames=names[2], asset_ids=aid,
                                              pixel_coordinates=np.zeros((n, 8, 2), np.float32), H=s, W=s, root=root)
        cores = len(os.sched_getaffinity(0))
        threads = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
        idx = list(range(n))

        def rate(fn):
            fn()  # warm the page cache
            t = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                fn()
                t.append(time.perf_counter() - t0)
            return n / statistics.median(t)

        native1 = rate(lambda: ds.load_batch(idx, n_threads=1))
        nativeN = rate(lambda: ds.load_batch(idx, n_threads=threads))
        ref = rate(lambda: [loader_ref.get_item(root, names[0][i], names[1][i], names[2][i], int(aid[i]), None)
                            for i in idx])
        bytes_per_item = sum(os.path.getsize(os.path.join(root, "data", x[0])) for x in zip(*names)) / n
        print(json.dumps({"workload": f"{n} items of {s}x{s}: RGB PNG + f32 Deflate TIFF + palette PNG",
                          "native_items_per_s_1thread": round(native1, 1),
                          "native_items_per_s": round(nativeN, 1), "threads": threads, "affinity_cores": cores,
                          "reference_items_per_s_1process": round(ref, 1),
                          "file_bytes_per_item_png": round(bytes_per_item),
                          "output_bytes_per_item": s * s * (12 + 4 + 1)}))


if __name__ == "__main__":
    main()
