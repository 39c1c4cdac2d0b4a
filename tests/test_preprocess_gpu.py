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


def _frames(seed, B, Hs, Ws):
    rng = np.random.default_rng(seed)
    rgb = rng.integers(0, 256, (B, Hs, Ws, 3), dtype=np.uint8)
    depth = rng.uniform(0.05, 0.6, (B, Hs, Ws)).astype(np.float32)
    depth[0, Hs // 2, Ws // 2 - 7] = np.nan
    depth[-1, Hs // 2 + 3, Ws // 2 + 60] = -np.inf
    return torch.from_numpy(rgb).cuda(), torch.from_numpy(depth).cuda()


def _model(precision="fp16"):
    from perseus_amd import synth
    from perseus_amd.detector import KeypointCNN

    m = KeypointCNN(num_channels=4, precision=precision)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synthetic_state_dict(4).items()})
    return m.eval()


@pytest.mark.parametrize("B,Hs,Ws,bgr,clip", [
    (3, 720, 1280, True, (None, None)),   # configs[4]: 3 x 720p ZED frames
    (2, 376, 672, False, (0.1, 0.5)),     # ZED VGA, RGB order, near/far clip
    (5, 257, 259, True, (0.2, None)),     # odd crop offsets, unaligned rows
    (64, 256, 256, True, (None, 0.4)),    # the benchmark batch, no crop
])
def test_stem_fused_preprocess_bit_exact(B, Hs, Ws, bgr, clip):
    """camera frames into the stem (pa_detector_forward_rgbd) give exactly the
    bits of pa_preprocess_rgbd followed by the f32-input forward."""
    m = _model()
    rgb, depth = _frames(B, B, Hs, Ws)
    ref = m(preprocess_rgbd(rgb, depth, bgr=bgr, near=clip[0], far=clip[1]))
    got = m.forward_rgbd(rgb, depth, bgr=bgr, near=clip[0], far=clip[1])
    assert torch.equal(got, ref)
    prof = [n for n, _ in m.profile(preprocess_rgbd(rgb, depth, bgr=bgr))[0]]
    assert prof[0] == "stem_conv7x7_pool"


def test_stem_fused_preprocess_fp32_and_errors():
    from perseus_amd import _lib

    rgb, depth = _frames(1, 2, 300, 300)
    m32 = _model("fp32")
    ref = m32(preprocess_rgbd(rgb, depth))
    assert torch.equal(m32.forward_rgbd(rgb, depth), ref)  # fp32: the separate preprocess kernel
    m = _model()
    with pytest.raises(RuntimeError):
        m.forward_rgbd(rgb[:, :200], depth[:, :200])  # smaller than 256 x 256
    with pytest.raises(RuntimeError):
        m.forward_rgbd(rgb.float(), depth)
    assert isinstance(_lib.lib().pa_last_error(), bytes)


@pytest.mark.parametrize("split_k", [0, 8])
def test_forward_rgbd_px_fuses_postprocess(split_k):
    """pa_detector_forward_rgbd_px (the streaming tick's call): the same keypoints as
    pa_detector_forward_rgbd, and pixels bit-identical to pa_keypoints_postprocess of them
    (the denormalize runs in the head), in both the batched and the split-K latency mode."""
    from perseus_amd import _lib
    from perseus_amd.detector import denormalize_pixel_coordinates

    m = _model()
    m.set_split_k(split_k)
    rgb, depth = _frames(7, 3, 720, 1280)
    ref = m.forward_rgbd(rgb, depth)
    h = m._ensure_handle(rgb.device)
    y = torch.empty_like(ref)
    px = torch.full((3, 8, 2), float("nan"), device=rgb.device)
    _lib.check(_lib.lib().pa_detector_forward_rgbd_px(h, rgb.data_ptr(), depth.data_ptr(), 3, 720, 1280, 1, -1.0, -1.0,
                                                       y.data_ptr(), px.data_ptr(), _lib.stream_of(rgb.device)),
               "forward_rgbd_px")
    assert torch.equal(y, ref)
    assert torch.equal(px, denormalize_pixel_coordinates(ref))
