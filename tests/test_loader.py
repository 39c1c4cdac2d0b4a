"""The native keypoint-dataset loader (perseus/detector/data.py:73-102) against
PIL decoding the same bytes, and PrunedKeypointDataset items against the reference's
__getitem__ restated in oracle/loader_ref.py.  Bit-exact throughout (byte / f32 samples).

PNG files come from PIL's encoder and from a hand-written encoder that sets every row
filter (None / Sub / Up / Average / Paeth), splits IDAT, and packs 1 / 2 / 4-bit palette
indices; TIFF files from PIL/libtiff (none, LZW, Deflate) and hand-written strips with the
horizontal and floating-point predictors in both byte orders.  CPU only."""
import io
import os
import struct
import zlib

import numpy as np
import pytest
import torch
from PIL import Image

from oracle import loader_ref
from perseus_amd import _lib
from perseus_amd.data import KeypointDatasetConfig, PrunedKeypointDataset, decode_png, decode_tiff

RNG = np.random.default_rng(11)


# ----------------------------------------------------------------------------- PNG encoders
def _chunk(t: bytes, d: bytes) -> bytes:
    return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    return a if pa <= pb and pa <= pc else (b if pb <= pc else c)


def encode_png(rows: np.ndarray, ctype: int, depth: int = 8, palette=None, filters=None, split: int = 3,
               w: int | None = None) -> bytes:
    """rows: (h, stride) packed sample bytes.  filters: per-row filter types (default cycles 0..4)."""
    h, stride = rows.shape
    ch = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
    bpp = max(1, depth * ch // 8)
    w = stride * 8 // (depth * ch) if w is None else w
    out = bytearray()
    prev = np.zeros(stride, dtype=np.int64)
    for y in range(h):
        f = (y % 5) if filters is None else filters[y]
        row = rows[y].astype(np.int64)
        enc = np.zeros(stride, dtype=np.int64)
        for i in range(stride):
            a = row[i - bpp] if i >= bpp else 0
            b = prev[i]
            c = prev[i - bpp] if i >= bpp else 0
            pred = [0, a, b, (a + b) >> 1, _paeth(a, b, c)][f]
            enc[i] = (row[i] - pred) & 255
        out.append(f)
        out += bytes(enc.astype(np.uint8))
        prev = row
    z = zlib.compress(bytes(out), 6)
    parts = [z[i * len(z) // split:(i + 1) * len(z) // split] for i in range(split)]
    png = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, 0))
    if palette is not None:
        png += _chunk(b"PLTE", bytes(np.asarray(palette, dtype=np.uint8).reshape(-1)))
    for p in parts:
        png += _chunk(b"IDAT", p)
    return png + _chunk(b"IEND", b"")


def pil_png(arr: np.ndarray, mode: str, **kw) -> bytes:
    b = io.BytesIO()
    im = Image.fromarray(arr, mode) if mode != "P" else Image.fromarray(arr, "P")
    if mode == "P":
        im.putpalette(list(RNG.integers(0, 256, 768)))
    im.save(b, format="PNG", **kw)
    return b.getvalue()


def pil_decode(data: bytes, rgb: bool) -> np.ndarray:
    im = Image.open(io.BytesIO(data))
    return np.asarray(im.convert("RGB") if rgb else im)


@pytest.mark.parametrize("shape", [(1, 1), (23, 37), (64, 48)])
@pytest.mark.parametrize("mode", ["RGB", "RGBA", "L", "LA", "P"])
@pytest.mark.parametrize("level", [0, 6, 9])
def test_png_from_pil_matches_pil(mode, shape, level):
    ch = {"RGB": 3, "RGBA": 4, "L": 1, "LA": 2, "P": 1}[mode]
    arr = RNG.integers(0, 256, shape + ((ch,) if ch > 1 else ()), dtype=np.uint8)
    if mode == "LA":  # Image.fromarray has no 2-channel mode: build it
        im = Image.merge("LA", [Image.fromarray(arr[..., 0]), Image.fromarray(arr[..., 1])])
        b = io.BytesIO()
        im.save(b, format="PNG", compress_level=level)
        data = b.getvalue()
    else:
        data = pil_png(arr, mode, compress_level=level)
    for rgb in (True, False):
        np.testing.assert_array_equal(decode_png(data, rgb), pil_decode(data, rgb))


@pytest.mark.parametrize("ctype,ch", [(0, 1), (2, 3), (4, 2), (6, 4)])
def test_png_every_row_filter(ctype, ch):
    h, w = 17, 29
    arr = RNG.integers(0, 256, (h, w * ch), dtype=np.uint8)
    arr[5:9] = arr[4]  # runs, so Up / Paeth see equal neighbours
    for filters in (None, [4] * h, [3] * h, [1] * h):
        data = encode_png(arr, ctype, filters=filters, split=4)
        for rgb in (True, False):
            np.testing.assert_array_equal(decode_png(data, rgb), pil_decode(data, rgb))


@pytest.mark.parametrize("depth", [1, 2, 4, 8])
def test_png_palette_bit_depths(depth):
    h, w = 13, 21
    n = 1 << depth
    idx = RNG.integers(0, n, (h, w), dtype=np.uint8)
    per = 8 // depth
    stride = (w * depth + 7) // 8
    rows = np.zeros((h, stride), dtype=np.uint8)
    for x in range(w):
        rows[:, x // per] |= (idx[:, x] << (8 - depth * (x % per + 1))).astype(np.uint8)
    pal = RNG.integers(0, 256, (n, 3))
    data = encode_png(rows, 3, depth=depth, palette=pal, w=w)
    np.testing.assert_array_equal(decode_png(data, False), idx)
    np.testing.assert_array_equal(decode_png(data, True), pil_decode(data, True))


def test_png_refuses_unsupported_and_corrupt_files():
    b = io.BytesIO()
    Image.fromarray(RNG.integers(0, 65535, (8, 8), dtype=np.uint16)).save(b, format="PNG")
    with pytest.raises(_lib.PerseusError, match="bit depth 16"):
        decode_png(b.getvalue())
    good = encode_png(RNG.integers(0, 256, (4, 12), dtype=np.uint8), 2)
    interlaced = bytearray(good)
    interlaced[8 + 8 + 12] = 1  # IHDR interlace byte
    interlaced[29:33] = struct.pack(">I", zlib.crc32(bytes(interlaced[12:29])) & 0xFFFFFFFF)
    with pytest.raises(_lib.PerseusError, match="interlaced"):
        decode_png(bytes(interlaced))
    with pytest.raises(_lib.PerseusError):
        decode_png(good[: len(good) // 2])
    with pytest.raises(_lib.PerseusError, match="not a PNG"):
        decode_png(b"GIF89a" + b"\0" * 40)


# ---------------------------------------------------------------------------- TIFF encoders
def encode_tiff(arr: np.ndarray, order: str = "<", compression: int = 1, predictor: int = 1, rps: int = 5) -> bytes:
    """One-sample strip TIFF of `arr` (float32 or uint16/uint8)."""
    h, w = arr.shape
    fmt = 3 if arr.dtype == np.float32 else 1
    bps = arr.dtype.itemsize * 8
    strips = []
    for y0 in range(0, h, rps):
        block = arr[y0:y0 + rps]
        rows = []
        for row in block:
            if predictor == 3:
                be = row.astype(">f4").tobytes()
                planes = np.frombuffer(be, dtype=np.uint8).reshape(w, 4).T.reshape(-1).astype(np.int64)
                d = planes.copy()
                d[1:] = planes[1:] - planes[:-1]
                rows.append(bytes((d & 255).astype(np.uint8)))
            elif predictor == 2:
                v = row.astype(np.int64)
                d = v.copy()
                d[1:] = v[1:] - v[:-1]
                rows.append((d % (1 << bps)).astype(row.dtype).astype(row.dtype.newbyteorder(order)).tobytes())
            else:
                rows.append(row.astype(row.dtype.newbyteorder(order)).tobytes())
        raw = b"".join(rows)
        strips.append(zlib.compress(raw) if compression == 8 else raw)
    pk = lambda f, *v: struct.pack(order + f, *v)  # noqa: E731
    tags = [(256, 4, [w]), (257, 4, [h]), (258, 3, [bps]), (259, 3, [compression]), (262, 3, [1]),
            (273, 4, None), (277, 3, [1]), (278, 4, [rps]), (279, 4, [len(s) for s in strips]), (284, 3, [1])]
    if predictor != 1:
        tags.append((317, 3, [predictor]))
    tags.append((339, 3, [fmt]))
    n = len(tags)
    ifd_at = 8
    extra_at = ifd_at + 2 + 12 * n + 4
    extra = b""
    data_at = extra_at + 8 * len(strips) * 2 + 16
    offs, o = [], data_at
    for s in strips:
        offs.append(o)
        o += len(s)
    ifd = pk("H", n)
    for tag, typ, vals in tags:
        vals = offs if tag == 273 else vals
        size = 2 if typ == 3 else 4
        if len(vals) * size <= 4:
            v = b"".join(pk("H" if typ == 3 else "I", x) for x in vals).ljust(4, b"\0")
        else:
            v = pk("I", extra_at + len(extra))
            extra += b"".join(pk("I", x) for x in vals)
        ifd += pk("HHI", tag, typ, len(vals)) + v
    ifd += pk("I", 0)
    head = (b"II" if order == "<" else b"MM") + pk("H", 42) + pk("I", ifd_at)
    body = head + ifd + extra
    body = body.ljust(data_at, b"\0")
    return body + b"".join(strips)


def pil_tiff(data: bytes) -> np.ndarray:
    return np.asarray(Image.open(io.BytesIO(data)))


@pytest.mark.parametrize("compression", [None, "tiff_lzw", "tiff_deflate", "tiff_adobe_deflate"])
@pytest.mark.parametrize("shape", [(1, 1), (31, 17), (96, 80)])
def test_tiff_from_pil_matches_pil(compression, shape):
    arr = (RNG.standard_normal(shape) * 7).astype(np.float32)
    arr.flat[0] = 0.0
    b = io.BytesIO()
    Image.fromarray(arr, "F").save(b, format="TIFF", compression=compression)
    data = b.getvalue()
    np.testing.assert_array_equal(decode_tiff(data), pil_tiff(data))


def test_tiff_uint16_from_pil():
    arr = RNG.integers(0, 65536, (19, 33), dtype=np.uint16)
    b = io.BytesIO()
    Image.fromarray(arr).save(b, format="TIFF", compression="tiff_lzw")
    data = b.getvalue()
    np.testing.assert_array_equal(decode_tiff(data), pil_tiff(data).astype(np.float32))


@pytest.mark.parametrize("order", ["<", ">"])
@pytest.mark.parametrize("compression,predictor", [(1, 1), (8, 1), (8, 3), (1, 3)])
def test_tiff_float_predictor_and_byte_order(order, compression, predictor):
    arr = (RNG.standard_normal((23, 41)) * 3 + 5).astype(np.float32)
    data = encode_tiff(arr, order, compression, predictor, rps=7)
    ours = decode_tiff(data)
    np.testing.assert_array_equal(ours, arr)  # the stored samples: what tifffile's asarray() returns
    # PIL 12.2 reads uncompressed strips itself (ignoring the predictor tag) and swaps
    # big-endian float samples a second time after libtiff has decoded a compressed strip:
    # compared only where PIL reads the file right
    if (order == "<" and (compression != 1 or predictor == 1)) or (compression == 1 and predictor == 1):
        np.testing.assert_array_equal(ours, pil_tiff(data))


@pytest.mark.parametrize("order", ["<", ">"])
def test_tiff_uint16_horizontal_predictor(order):
    arr = RNG.integers(0, 65536, (9, 27), dtype=np.uint16)
    data = encode_tiff(arr, order, 8, 2, rps=4)
    np.testing.assert_array_equal(decode_tiff(data), arr.astype(np.float32))
    np.testing.assert_array_equal(decode_tiff(data), pil_tiff(data).astype(np.float32))


def test_tiff_refuses_unsupported_files():
    rgb = io.BytesIO()
    Image.fromarray(RNG.integers(0, 256, (4, 4, 3), dtype=np.uint8), "RGB").save(rgb, format="TIFF")
    with pytest.raises(_lib.PerseusError, match="samples per pixel"):
        decode_tiff(rgb.getvalue())
    with pytest.raises(_lib.PerseusError, match="not a TIFF"):
        decode_tiff(b"\x89PNG" + b"\0" * 32)


# ------------------------------------------------------------------------------- dataset
def _write_dataset(root, n, h, w):
    os.makedirs(os.path.join(root, "data", "img"), exist_ok=True)
    names = ([], [], [])
    modes = ["RGB", "RGBA", "P", "L"]
    comps = [None, "tiff_lzw", "tiff_deflate", "hand"]
    for i in range(n):
        mode = modes[i % 4]
        ch = {"RGB": 3, "RGBA": 4, "P": 1, "L": 1}[mode]
        arr = RNG.integers(0, 256, (h, w, ch) if ch > 1 else (h, w), dtype=np.uint8)
        open(os.path.join(root, "data", f"img/{i}.png"), "wb").write(pil_png(arr, mode))
        depth = (RNG.uniform(0.12, 0.48, (h, w)) / 0.035).astype(np.float32)
        depth[RNG.random((h, w)) < 0.25] = 0.0
        if comps[i % 4] == "hand":
            data = encode_tiff(depth, "<", 8, 3, rps=3)  # the oracle (PIL) misreads big-endian compressed floats
        else:
            b = io.BytesIO()
            Image.fromarray(depth, "F").save(b, format="TIFF", compression=comps[i % 4])
            data = b.getvalue()
        open(os.path.join(root, "data", f"img/{i}_depth.tiff"), "wb").write(data)
        seg = RNG.integers(0, 4, (h, w), dtype=np.uint8)
        open(os.path.join(root, "data", f"img/{i}_seg.png"), "wb").write(pil_png(seg, "P" if i % 2 else "L"))
        names[0].append(f"img/{i}.png".encode())
        names[1].append(f"img/{i}_depth.tiff".encode())
        names[2].append(f"img/{i}_seg.png".encode())
    return names


def test_dataset_items_match_the_reference_getitem(tmp_path):
    n, h, w = 9, 30, 44
    names = _write_dataset(str(tmp_path), n, h, w)
    asset_ids = RNG.integers(0, 3, n)
    px = torch.from_numpy(RNG.uniform(0, 256, (n, 8, 2)).astype(np.float32))
    ds = PrunedKeypointDataset.from_index(image_filenames=np.array(names[0]), depth_filenames=np.array(names[1]),
                                          segmentation_filenames=np.array(names[2]), asset_ids=asset_ids,
                                          pixel_coordinates=px.numpy(), H=h, W=w, weights=np.ones(n),
                                          root=str(tmp_path))
    assert len(ds) == n
    batch = ds.load_batch(list(range(n)) + [3, -1], n_threads=4)
    for j, i in enumerate(list(range(n)) + [3, n - 1]):
        ref = loader_ref.get_item(str(tmp_path), names[0][i].decode(), names[1][i].decode(), names[2][i].decode(),
                                  int(asset_ids[i]), px[i])
        item = ds[i]
        for k in ("image", "depth_image", "segmentation_image", "pixel_coordinates"):
            assert item[k].dtype == ref[k].dtype and item[k].shape == ref[k].shape, k
            assert torch.equal(item[k], ref[k]), (i, k)
            assert torch.equal(batch[k][j], ref[k]), (i, k)


def test_dataset_errors(tmp_path):
    names = _write_dataset(str(tmp_path), 2, 16, 16)
    ds = PrunedKeypointDataset.from_index(image_filenames=names[0], depth_filenames=names[1],
                                          segmentation_filenames=names[2], asset_ids=[0, 1],
                                          pixel_coordinates=np.zeros((2, 8, 2)), H=16, W=20, root=str(tmp_path))
    with pytest.raises(_lib.PerseusError, match="expected 16 x 20"):
        ds.load_batch([0, 1])
    ds.W = 16
    ds.depth_filenames[1] = "img/missing.tiff"
    with pytest.raises(_lib.PerseusError, match="item 1: cannot open"):
        ds.load_batch([0, 1], n_threads=2)
    with pytest.raises(IndexError):
        ds.load_batch([2])


def test_hdf5_constructor_names_its_dependency():
    try:
        import h5py  # noqa: F401
    except ImportError:
        with pytest.raises(ImportError, match="h5py"):
            PrunedKeypointDataset(KeypointDatasetConfig(), train=False)
    else:
        pytest.skip("h5py present")
