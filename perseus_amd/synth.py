"""Deterministic synthetic weights and RGBD frames for the keypoint path.

The reference's trained checkpoints (`outputs/models/4b8hrqoo.pth`, `1hj7an9g.pth`,
README.md:99) are Git-LFS pointers and its torchvision ImageNet init is a remote
download (`perseus/detector/models.py:20`), so every test, the smoke check and the
bench use weights and frames drawn from a documented counter-based generator.  The
same bytes come out on any machine with numpy, without torch's RNG.

Generator spec:
  * base   = mix64(seed)
  * u[i,j] = (mix64(base + (i << 40) + j) >> 11) * 2**-53     (uniform [0,1), f64)
    where i is the stream id (tensor index in `STATE_KEYS` order, or a fixed id for
    the frame streams) and j the element index in C order; mix64 = splitmix64's
    finaliser.
  * conv weights     U(-a, a), a = sqrt(6 / fan_in)        (He-uniform)
  * BatchNorm        gamma U(0.2,0.6), beta U(-0.1,0.1), mean U(-0.1,0.1), var U(0.5,2)
  * fc               weight U(-FC_SCALE, FC_SCALE), bias U(-0.1, 0.1)
  * frames           RGB = floor(256 u)/255 (PNG /255, `perseus/detector/data.py:78,84`);
                     depth = U(0.12,0.48) m / 0.035 (`augmentations.py:263`), 25 % of
                     pixels 0 (near/far clipped, `augmentations.py:403-431`).
"""

from __future__ import annotations

import hashlib
from collections import OrderedDict

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
_GOLDEN = np.uint64(0x9E3779B97F4A7C15)

# Calibrated once (see oracle/gen_golden.py --calibrate) so that the synthetic
# network's outputs span roughly [-1, 1] like a trained keypoint regressor's.
FC_SCALE = 0.2

STREAM_RGB = 1 << 20
STREAM_DEPTH = (1 << 20) + 1
STREAM_DEPTH_MASK = (1 << 20) + 2
STREAM_TRAJ = (1 << 20) + 3

DEPTH_SCALE = 0.035  # augmentations.py:263 cube_scale; streaming.py:76 `/= 0.035`


def mix64(x: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser on uint64 arrays (wrap-around arithmetic)."""
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def uniform(seed: int, stream: int, n: int) -> np.ndarray:
    """n uniforms in [0,1) (f64) from stream `stream` of generator `seed`."""
    base = mix64(np.uint64(seed & 0xFFFFFFFFFFFFFFFF))
    with np.errstate(over="ignore"):
        ctr = base + (np.uint64(stream) << np.uint64(40)) + np.arange(n, dtype=np.uint64)
    return (mix64(ctr) >> np.uint64(11)).astype(np.float64) * (2.0**-53)


def resnet18_shapes(in_ch: int = 4, n_kp: int = 8) -> "OrderedDict[str, tuple]":
    """State-dict keys/shapes of KeypointCNN (`perseus/detector/models.py:20-32`).

    torchvision's resnet18 naming (`resnet.` prefix); 122 keys incl. the 20
    `num_batches_tracked` int64 scalars.
    """
    shapes: "OrderedDict[str, tuple]" = OrderedDict()

    def bn(prefix: str, c: int) -> None:
        shapes[prefix + ".weight"] = (c,)
        shapes[prefix + ".bias"] = (c,)
        shapes[prefix + ".running_mean"] = (c,)
        shapes[prefix + ".running_var"] = (c,)
        shapes[prefix + ".num_batches_tracked"] = ()

    shapes["resnet.conv1.weight"] = (64, in_ch, 7, 7)
    bn("resnet.bn1", 64)
    cin = 64
    for li, cout in enumerate((64, 128, 256, 512), start=1):
        for bi in range(2):
            stride = 2 if (li > 1 and bi == 0) else 1
            p = f"resnet.layer{li}.{bi}"
            shapes[p + ".conv1.weight"] = (cout, cin if bi == 0 else cout, 3, 3)
            bn(p + ".bn1", cout)
            shapes[p + ".conv2.weight"] = (cout, cout, 3, 3)
            bn(p + ".bn2", cout)
            if bi == 0 and (stride != 1 or cin != cout):
                shapes[p + ".downsample.0.weight"] = (cout, cin, 1, 1)
                bn(p + ".downsample.1", cout)
        cin = cout
    shapes["resnet.fc.weight"] = (2 * n_kp, 512)
    shapes["resnet.fc.bias"] = (2 * n_kp,)
    return shapes


def float_keys(shapes: "OrderedDict[str, tuple]") -> list:
    """Keys that travel in the C-ABI weight blob (everything but num_batches_tracked)."""
    return [k for k in shapes if not k.endswith("num_batches_tracked")]


def synthetic_state_dict(seed: int = 0, in_ch: int = 4, n_kp: int = 8) -> "OrderedDict[str, np.ndarray]":
    """Synthetic KeypointCNN state dict as numpy arrays (f32; int64 counters)."""
    shapes = resnet18_shapes(in_ch, n_kp)
    out: "OrderedDict[str, np.ndarray]" = OrderedDict()
    for i, (k, shp) in enumerate(shapes.items()):
        n = int(np.prod(shp)) if shp else 1
        if k.endswith("num_batches_tracked"):
            out[k] = np.array(0, dtype=np.int64)
            continue
        u = uniform(seed, i, n).reshape(shp)
        if k.endswith("fc.weight"):
            v = (2 * u - 1) * FC_SCALE
        elif k.endswith("fc.bias"):
            v = (2 * u - 1) * 0.1
        elif len(shp) == 4:
            fan_in = shp[1] * shp[2] * shp[3]
            v = (2 * u - 1) * np.sqrt(6.0 / fan_in)
        elif k.endswith(".weight"):
            v = 0.2 + 0.4 * u
        elif k.endswith(".bias"):
            v = (2 * u - 1) * 0.1
        elif k.endswith("running_mean"):
            v = (2 * u - 1) * 0.1
        elif k.endswith("running_var"):
            v = 0.5 + 1.5 * u
        else:  # pragma: no cover
            raise KeyError(k)
        out[k] = v.astype(np.float32)
    return out


def weight_blob(state: "OrderedDict[str, np.ndarray]", in_ch: int = 4, n_kp: int = 8) -> np.ndarray:
    """Flatten a state dict into the C-ABI blob: f32 tensors in `float_keys` order."""
    keys = float_keys(resnet18_shapes(in_ch, n_kp))
    parts = []
    for k in keys:
        a = np.asarray(state[k], dtype=np.float32)
        expect = resnet18_shapes(in_ch, n_kp)[k]
        if tuple(a.shape) != tuple(expect):
            raise ValueError(f"{k}: shape {a.shape} != {expect}")
        parts.append(a.reshape(-1))
    return np.ascontiguousarray(np.concatenate(parts))


def synthetic_frames(seed: int, batch: int, in_ch: int = 4, H: int = 256, W: int = 256,
                     first: int = 0) -> np.ndarray:
    """Frames `first .. first+batch-1` of the synthetic RGBD stream, (B,C,H,W) f32 NCHW.

    Frame f depends only on (seed, f), so shards of a long stream are generated
    independently per rank.
    """
    hw = H * W
    out = np.empty((batch, in_ch, H, W), dtype=np.float32)
    for b in range(batch):
        f = first + b
        ncol = min(in_ch, 3)
        off = f * 3 * hw
        base = mix64(np.uint64(seed & 0xFFFFFFFFFFFFFFFF))
        with np.errstate(over="ignore"):
            ctr = base + (np.uint64(STREAM_RGB) << np.uint64(40)) + np.uint64(off) + np.arange(3 * hw, dtype=np.uint64)
        u = (mix64(ctr) >> np.uint64(11)).astype(np.float64) * (2.0**-53)
        k = np.floor(u * 256.0)
        out[b, :ncol] = (k / 255.0).astype(np.float32).reshape(3, H, W)[:ncol]
        if in_ch > 3:
            with np.errstate(over="ignore"):
                c1 = base + (np.uint64(STREAM_DEPTH) << np.uint64(40)) + np.uint64(f * hw) + np.arange(hw, dtype=np.uint64)
                c2 = base + (np.uint64(STREAM_DEPTH_MASK) << np.uint64(40)) + np.uint64(f * hw) + np.arange(hw, dtype=np.uint64)
            u1 = (mix64(c1) >> np.uint64(11)).astype(np.float64) * (2.0**-53)
            u2 = (mix64(c2) >> np.uint64(11)).astype(np.float64) * (2.0**-53)
            d = (0.12 + 0.36 * u1) / DEPTH_SCALE
            d[u2 < 0.25] = 0.0
            out[b, 3] = d.astype(np.float32).reshape(H, W)
    return out


CUBE_CORNERS = np.array([[x, y, z] for x in (-1, 1) for y in (-1, 1) for z in (-1, 1)], np.float64) * 0.0175
CAMERA_K = np.array([280.0, 280.0, 0.0, 128.0, 128.0])  # Cal3_S2 of the datagen camera


def synthetic_trajectories(seed: int, T: int, L: int, n_kp: int = 8) -> dict:
    """T trajectories x L frames of smoother inputs:
    poses (T*L, 12) with R = Exp(U(-.5,.5)^3) and t = (U(+-.05), U(+-.05), U(.3,.5)) in
    front of the identity camera; vels / angvels U(-1,1)^3; detector-like normalized
    keypoints y U(-1,1) (T*L, 2K) f32."""
    F = T * L
    u = uniform(seed, STREAM_TRAJ, F * (3 + 3 + 3 + 3) + F * 2 * n_kp).astype(np.float64)
    w = (u[:3 * F].reshape(F, 3) - 0.5)
    t = u[3 * F:6 * F].reshape(F, 3)
    t = np.stack([0.1 * t[:, 0] - 0.05, 0.1 * t[:, 1] - 0.05, 0.3 + 0.2 * t[:, 2]], 1)
    vel = 2 * u[6 * F:9 * F].reshape(F, 3) - 1
    ang = 2 * u[9 * F:12 * F].reshape(F, 3) - 1
    y = (2 * u[12 * F:].reshape(F, 2 * n_kp) - 1).astype(np.float32)
    th = np.linalg.norm(w, axis=1)[:, None, None]
    Wx = np.zeros((F, 3, 3))
    Wx[:, 0, 1], Wx[:, 0, 2], Wx[:, 1, 2] = -w[:, 2], w[:, 1], -w[:, 0]
    Wx = Wx - Wx.transpose(0, 2, 1)
    R = np.eye(3) + np.sin(th) / th * Wx + (1 - np.cos(th)) / th ** 2 * (Wx @ Wx)
    poses = np.concatenate([R.reshape(F, 9), t], 1)
    return {"poses": poses, "vels": vel, "angvels": ang, "y": y, "corners": CUBE_CORNERS[:n_kp], "K": CAMERA_K}


def sha256(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
