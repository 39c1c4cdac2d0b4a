"""GPU parity of the fused pre-processing with a numpy restatement of
scripts/streaming.py:59-82 (+ the deterministic near/far clip)."""
import numpy as np
import pytest
import torch

from perseus_amd.detector import preprocess_rgbd

pytestmark = pytest.mark.gpu


def numpy_ref(bgr_u8, depth_m, near=None, far=None):
    frame = bgr_u8[..., ::-1] / 255.0                      # streaming.py:68-69 (f64)
    depth = depth_m.copy()
    depth[np.isnan(depth)] = 0                              # :73-74
    depth[np.isinf(depth)] = 0
    depth /= np.float32(0.035)                              # :76 (f32 array)
    if near is not None or far is not None:
        s = np.float32(0.035) * depth
        if near is not None:
            s = np.where(s < np.float32(near), np.float32(0), s)
        if far is not None:
            s = np.where(s > np.float32(far), np.float32(0), s)
        depth = (s / np.float32(0.035)).astype(np.float32)
    frame = np.concatenate([frame, depth[..., None]], axis=-1)
    H, W = frame.shape[:2]
    frame = frame[H // 2 - 128: H // 2 + 128, W // 2 - 128: W // 2 + 128]  # :79-80
    return torch.from_numpy(frame).permute(2, 0, 1).float().numpy()       # :127


@pytest.mark.parametrize("clip", [(None, None), (0.1, 0.5)])
def test_preprocess_bit_exact(clip):
    rng = np.random.default_rng(0)
    B, Hs, Ws = 2, 376, 672  # ZED VGA
    bgr = rng.integers(0, 256, (B, Hs, Ws, 3), dtype=np.uint8)
    depth = rng.uniform(0.05, 0.6, (B, Hs, Ws)).astype(np.float32)
    depth[0, 180, 300] = np.nan
    depth[1, 190, 330] = np.inf
    x = preprocess_rgbd(torch.from_numpy(bgr).cuda(), torch.from_numpy(depth).cuda(), bgr=True,
                        near=clip[0], far=clip[1]).cpu().numpy()
    for b in range(B):
        ref = numpy_ref(bgr[b], depth[b], *clip)
        np.testing.assert_array_equal(x[b], ref)
