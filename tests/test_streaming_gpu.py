"""Config 4 pipeline: graph replay == eager composition, and matches the reference
arithmetic of scripts/streaming.py:59-82 + 126-131 on the same frames."""
import numpy as np
import pytest
import torch

from oracle import resnet_ref as R
from perseus_amd import synth
from perseus_amd.detector import KeypointCNN, preprocess_rgbd
from perseus_amd.streaming import StreamingPipeline

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def model():
    m = KeypointCNN(num_channels=4)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synthetic_state_dict(0).items()})
    return m


def _frames(seed, n=3, Hs=720, Ws=1280):
    rng = np.random.default_rng(seed)
    rgb = rng.integers(0, 256, (n, Hs, Ws, 3), dtype=np.uint8)
    d = rng.uniform(0.12, 0.48, (n, Hs, Ws)).astype(np.float32)
    d[:, ::7, ::5] = np.nan
    d[:, 3::11, ::3] = np.inf
    return rgb, d


@pytest.mark.parametrize("host_crop", [True, False])
def test_graph_matches_eager(model, host_crop):
    rgb, d = _frames(1)
    g = StreamingPipeline(model, host_crop=host_crop, graph=True)
    e = StreamingPipeline(model, host_crop=host_crop, graph=False)
    for seed in (1, 2):
        rgb, d = _frames(seed)
        np.testing.assert_array_equal(g(rgb, d), e(rgb, d))


def test_matches_reference_frame_arithmetic(model):
    rgb, d = _frames(3)
    out = StreamingPipeline(model)(rgb, d)
    # streaming.py:68-80 in numpy, then crop, then the model
    xs = []
    for i in range(3):
        fr = rgb[i][..., ::-1] / 255.0
        dep = d[i].copy()
        dep[np.isnan(dep)] = 0
        dep[np.isinf(dep)] = 0
        dep /= 0.035
        fr = np.concatenate([fr, dep[..., None]], axis=-1)
        H, W = fr.shape[:2]
        fr = fr[H // 2 - 128:H // 2 + 128, W // 2 - 128:W // 2 + 128]
        xs.append(torch.from_numpy(fr).permute(2, 0, 1).float())
    x = torch.stack(xs).cuda()
    x_dev = preprocess_rgbd(torch.as_tensor(rgb).cuda(), torch.as_tensor(d).cuda())
    assert torch.equal(x, x_dev)
    model.set_split_k(3)  # the pipeline's latency mode (pa_detector_set_split_k): same kernels, same bits
    try:
        y = model(x).reshape(3, -1, 2)
    finally:
        model.set_split_k(0)
    np.testing.assert_array_equal(out, R.denormalize_f32(y.cpu().numpy().reshape(3, -1)))


def test_graph_survives_model_reallocation_and_reload():
    """The captured graph holds its own handle: a later larger-batch forward
    (which grows the model's workspace) and a weight reload (which destroys the model's
    handle) must not touch the memory the graph replays into."""
    m = KeypointCNN(num_channels=4)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synthetic_state_dict(0).items()})
    rgb, d = _frames(4)
    g = StreamingPipeline(m, graph=True)
    ref = g(rgb, d)
    m(torch.from_numpy(synth.synthetic_frames(0, 64)).cuda())  # B=64: the model's own workspace grows
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synthetic_state_dict(9).items()})
    m(torch.from_numpy(synth.synthetic_frames(0, 2)).cuda())  # new weights: the model's handle is recreated
    np.testing.assert_array_equal(g(rgb, d), ref)  # the pipeline keeps the weights it was built with
    g.close()


@pytest.mark.parametrize("n", [1, 5])
def test_camera_counts_latency_mode_vs_batched_and_oracle(model, n):
    """Other camera counts through the latency mode: the pipeline's pixels are the bits of
    model.set_split_k(n) + forward on the same frames, within 0.05 px of the batched
    kernels', and within the fp16 budget of the f64 oracle (streaming.py:68-80 arithmetic)."""
    rgb, d = _frames(11, n)
    pipe = StreamingPipeline(model, n_cams=n)
    out = pipe(rgb, d)
    pipe.close()
    x = preprocess_rgbd(torch.as_tensor(rgb).cuda(), torch.as_tensor(d).cuda())
    model.set_split_k(n)
    try:
        y = model(x)
    finally:
        model.set_split_k(0)
    np.testing.assert_array_equal(out, R.denormalize_f32(y.cpu().numpy()).reshape(n, -1, 2))
    yb = model(x).cpu().numpy()
    assert np.abs(R.denormalize_f32(yb).reshape(n, -1, 2) - out).max() <= 0.05
    y64 = R.run(synth.synthetic_state_dict(0), x.cpu().numpy(), torch.float64)
    px64 = R.denormalize_f32(y64.astype(np.float32)).reshape(n, -1, 2)
    assert np.sqrt(((out - px64) ** 2).sum(-1)).max() <= 0.1  # px-L2, the fp16 budget (test_detector_gpu.FP16_PX_MAX)


@pytest.fixture(scope="module")
def model_x3():
    m = KeypointCNN(num_channels=4, precision="fp16x3")
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synthetic_state_dict(0).items()})
    return m


@pytest.mark.parametrize("n", [1, 3, 5])
def test_parity_grade_tick_fp16x3(model_x3, n):
    """The parity-grade streaming tick (fp16x3 in its latency mode): graph replay == eager bit
    for bit, the pixels are model.set_split_k(n) + forward's on the preprocessed frames, and
    every keypoint coordinate is within 1e-3 px of the f64 oracle's (north_star) on the same
    frames (streaming.py:68-80 arithmetic)."""
    rgb, d = _frames(21 + n, n)
    g = StreamingPipeline(model_x3, n_cams=n, graph=True)
    e = StreamingPipeline(model_x3, n_cams=n, graph=False)
    out = g(rgb, d)
    np.testing.assert_array_equal(out, e(rgb, d))
    g.close()
    e.close()
    x = preprocess_rgbd(torch.as_tensor(rgb).cuda(), torch.as_tensor(d).cuda())
    model_x3.set_split_k(n)
    try:
        y = model_x3(x)
    finally:
        model_x3.set_split_k(0)
    np.testing.assert_array_equal(out, R.denormalize_f32(y.cpu().numpy()).reshape(n, -1, 2))
    y64 = R.run(synth.synthetic_state_dict(0), x.cpu().numpy(), torch.float64)
    px64 = ((y64 + 1.0) * 127.5).reshape(n, -1, 2)  # exact denormalize of the f64 outputs
    err = np.abs(out.astype(np.float64) - px64).max()
    print(f"fp16x3 tick, {n} camera(s): max |px - px_f64| = {err:.3e}")
    assert err <= 1e-3


@pytest.mark.parametrize("precision", ["fp16", "fp16x3"])
def test_zero_copy_tick_matches_copying_tick(model, model_x3, precision):
    """zero_copy (the stem / preprocess kernel read the pinned staging over PCIe, no H2D
    copy; the default for fp16x3) against the copying tick: pixels bit for bit, graph and
    eager, with the pose stage."""
    m = model if precision == "fp16" else model_x3
    a = StreamingPipeline(m, n_cams=3, graph=True, zero_copy=False, pose_window=6)
    b = StreamingPipeline(m, n_cams=3, graph=True, zero_copy=True, pose_window=6)
    c = StreamingPipeline(m, n_cams=3, graph=False, zero_copy=True, pose_window=6)
    assert b.zero_copy and not a.zero_copy
    dflt = StreamingPipeline(m, n_cams=1)
    assert dflt.zero_copy == (precision != "fp16")
    dflt.close()
    for seed in range(3):
        rgb, d = _frames(40 + seed, 3)
        ra, rb, rc = a.tick(rgb, d), b.tick(rgb, d), c.tick(rgb, d)
        for x, y, z in zip(ra, rb, rc):
            np.testing.assert_array_equal(x, y)
            np.testing.assert_array_equal(x, z)
    for p in (a, b, c):
        p.close()


@pytest.mark.parametrize("precision", ["fp16x3", "fp32"])
def test_reserve_then_capture_forward_rgbd(precision):
    """reserve() sizes forward_rgbd's f32 staging too, so a graph captured with NO
    eager call before it allocates nothing and replays to the eager bits; a later larger
    eager call may regrow the buffers, so the graph is replayed before it."""
    m = KeypointCNN(num_channels=4, precision=precision)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synthetic_state_dict(0).items()})
    dev = torch.device("cuda", 0)
    rgb, d = _frames(21, n=3, Hs=300, Ws=400)
    rgb_d, d_d = torch.as_tensor(rgb).to(dev), torch.as_tensor(d).to(dev)
    m.reserve(3, dev)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
        y_graph = m.forward_rgbd(rgb_d, d_d)
    g.replay()
    torch.cuda.synchronize(dev)
    got = y_graph.clone()
    want = m.forward_rgbd(rgb_d, d_d)
    torch.cuda.synchronize(dev)
    assert torch.equal(got, want)
    assert torch.isfinite(got).all()
