"""Config 4 pose stage (BASELINE.json configs[4] "end-to-end pose latency"): the
StreamingPipeline tick with pose_window > 0 runs detector -> window advance ->
trajectory linearize (the reference's three factors, perseus/smoother/factors.py:54-142,
160-171, 216-275) -> GN step -> retract in ONE captured graph.

  * graph replay == eager composition, bit for bit, over a sequence of ticks (the fp16 tick
    and the parity-grade fp16x3 tick);
  * one tick's chain against the oracle on a constructed, well-conditioned window (keypoints
    projected from a known trajectory, plus noise): oracle window advance of the previous
    window with the tick's keypoints, the f64 factor restatement (factors_ref), the dense
    GN oracle (gn_ref) of the device's whitened factors, and the oracle retract of the
    advanced window by the device's delta, against the window the tick leaves behind;
  * the first tick after a reset (ONE measured frame: the others carry no projection factor)
    against the same oracle chain;
  * the smoother tracks a pose: 40 ticks of exact keypoints of a known cube trajectory that
    follows the dynamics model, info == 0 on every tick, and the newest pose converges to the
    true one;
  * the fused pose tick (pa_window_pose_tick) equals the four separate launches bit for bit;
  * the split pose tick (pa_window_pose_tick_pre beside the forward, _post after it: the
    default for windows <= 24 frames) equals the fused one up to f64 rounding (another
    elimination order), its first tick's factors bit for bit; with pre_ahead (the next tick's
    pre half right after the results) bit for bit the split tick.
"""
import numpy as np
import pytest
import torch

from oracle import factors_ref as F
from oracle import gn_ref as G
from perseus_amd import synth
from perseus_amd.detector import KeypointCNN
from perseus_amd.streaming import StreamingPipeline

from test_pipeline_gpu import _oracle  # tests/ is on sys.path (rootdir conftest)
from test_streaming_gpu import _frames

pytestmark = pytest.mark.gpu
LW = 6
DT = 1.0 / 30.0
SIG = dict(proj_sigma=2.0, dyn_sigma=0.1, cv_sigma=0.5, lam=1e-2)


def _model(precision="fp16"):
    m = KeypointCNN(num_channels=4, precision=precision)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synthetic_state_dict(0).items()})
    return m


@pytest.fixture(scope="module")
def model():
    return _model()


def _truth(n, ticks, seed=5):
    """Per camera a cube trajectory that follows the PoseDynamicsFactor model exactly
    (factors.py:100-105, world-frame velocity): T_{k+1} = T_k Exp(dt [w; R_k^T v]) with
    constant body angular velocity w and world velocity v.  Returns poses (ticks, n) of
    (R, t), w (n, 3), v (n, 3)."""
    rng = np.random.default_rng(seed)
    w = 0.3 * rng.standard_normal((n, 3))
    v = 0.01 * rng.standard_normal((n, 3))
    poses = []
    cur = []
    for c in range(n):
        R0, _ = F.pose_exp(np.concatenate([0.3 * rng.standard_normal(3), np.zeros(3)]))
        cur.append((R0, np.array([0.0, 0.0, 0.35]) + 0.005 * rng.standard_normal(3)))
    for _ in range(ticks):
        poses.append(list(cur))
        cur = [F.compose(T, F.pose_exp(np.concatenate([DT * w[c], DT * (T[0].T @ v[c])]))) for c, T in enumerate(cur)]
    return poses, w, v


def _keypoints(poses_tick, noise=0.0, rng=None):
    """Normalized keypoints (n, 16) f32 of the cube corners seen by the identity camera
    (Cal3_S2 synth.CAMERA_K): px = pi(K, R p_b + t); n = px / 127.5 - 1 (the inverse of
    kornia's denormalize for a 256 x 256 image, validate.py:144-153)."""
    fx, fy, s, u0, v0 = synth.CAMERA_K
    out = []
    for R, t in poses_tick:
        pc = synth.CUBE_CORNERS @ R.T + t
        assert (pc[:, 2] > 0).all()
        u = fx * pc[:, 0] / pc[:, 2] + s * pc[:, 1] / pc[:, 2] + u0
        v = fy * pc[:, 1] / pc[:, 2] + v0
        px = np.stack([u, v], 1)
        if noise:
            px = px + noise * rng.standard_normal(px.shape)
        assert (px > 0).all() and (px < 255).all()
        out.append((px / 127.5 - 1.0).reshape(-1))
    return np.array(out, np.float32)


def _pipe(model, graph, init=None, **kw):
    p0, v0, w0 = init if init is not None else _init()
    return StreamingPipeline(model, graph=graph, pose_window=LW, init_pose=p0, init_vel=v0, init_angvel=w0,
                             **{**SIG, **kw})


def _init(n=3, seed=5):
    """Initial window state: the true trajectory's first pose, rotated by ~0.1 rad and moved by
    ~1 cm, at rest."""
    poses, _, _ = _truth(n, 1, seed)
    rng = np.random.default_rng(seed + 100)
    p = []
    for R, t in poses[0]:
        Rp, _ = F.pose_exp(np.concatenate([0.1 * rng.standard_normal(3) / np.sqrt(3), np.zeros(3)]))
        p.append(F.pack((R @ Rp, t + 0.01 * rng.standard_normal(3) / np.sqrt(3))))
    return np.array(p), np.zeros((n, 3)), np.zeros((n, 3))


@pytest.mark.parametrize("precision", ["fp16", "fp16x3"])
def test_pose_graph_matches_eager(precision):
    m = _model(precision)
    g, e = _pipe(m, True), _pipe(m, False)
    for seed in range(1, LW + 4):  # past a full window
        rgb, d = _frames(seed)
        pg, qg, ig = g.tick(rgb, d)
        pe, qe, ie = e.tick(rgb, d)
        np.testing.assert_array_equal(pg, pe)
        np.testing.assert_array_equal(qg, qe)
        np.testing.assert_array_equal(ig, ie)
    for k, v in g.window_state().items():
        np.testing.assert_array_equal(v, e.window_state()[k], err_msg=k)
    assert np.isfinite(qg).all()
    # the keypoint-driven pose tick (tick_keypoints: the pose stage's own graph) == eager too
    y = _keypoints(_truth(3, 1)[0][0])
    qg, ig = g.tick_keypoints(y)
    qe, ie = e.tick_keypoints(y)
    np.testing.assert_array_equal(qg, qe)
    np.testing.assert_array_equal(ig, ie)
    g.close()
    e.close()


@pytest.mark.parametrize("graph", [True, False])
def test_fused_pose_tick_matches_four_launches(model, graph):
    """pa_window_pose_tick (advance + linearize, then GN step + retract: two launches, the
    shipped tick for windows <= 24 frames) against the four separate launches, bit for bit:
    poses, info, the window, every factor output and delta, over ticks that fill the window."""
    f, s = _pipe(model, graph, split_pose=False), _pipe(model, graph, split_pose=False)
    assert f.fused_pose and not f.split_pose
    s.fused_pose = False
    truth, _, _ = _truth(3, LW + 3)
    rng = np.random.default_rng(11)
    for k in range(LW + 3):
        y = _keypoints(truth[k], 0.5, rng)
        qf, inf_ = f.tick_keypoints(y)
        qs, ins = s.tick_keypoints(y)
        np.testing.assert_array_equal(qf, qs)
        np.testing.assert_array_equal(inf_, ins)
        for key, v in f.window_state().items():
            np.testing.assert_array_equal(v, s.window_state()[key], err_msg=key)
        for key, v in f.lin.items():
            if isinstance(v, torch.Tensor):
                assert torch.equal(v, s.lin[key]), key
        assert torch.equal(f.gn.out["delta"], s.gn.out["delta"])
    f.close()
    s.close()


@pytest.mark.parametrize("graph", [True, False])
def test_split_pose_tick_matches_fused(model, graph):
    """pa_window_pose_tick_pre + _post against pa_window_pose_tick over ticks that fill the
    window: the same normal equations, eliminated in another order (the newest frame last), so
    delta agrees to f64 rounding; the keypoints, statuses and the first tick's factor outputs
    (the newest frame's projections are evaluated in the post half) are bit-identical."""
    sp, fu = _pipe(model, graph), _pipe(model, graph, split_pose=False)
    assert sp.split_pose and not fu.split_pose
    truth, _, _ = _truth(3, LW + 3)
    rng = np.random.default_rng(11)
    for k in range(LW + 3):
        y = _keypoints(truth[k], 0.5, rng)
        qs, ins = sp.tick_keypoints(y)
        qf, inf_ = fu.tick_keypoints(y)
        np.testing.assert_array_equal(ins, inf_)
        assert (ins == 0).all()
        np.testing.assert_allclose(qs, qf, rtol=0, atol=1e-12)
        ws, wf = sp.window_state(), fu.window_state()
        np.testing.assert_array_equal(ws["y"], wf["y"])
        for key in ("pose", "vel", "angvel"):
            np.testing.assert_allclose(ws[key], wf[key], rtol=0, atol=1e-12, err_msg=key)
        for key, v in sp.lin.items():
            if isinstance(v, torch.Tensor):
                if k == 0 or key == "status":
                    assert torch.equal(v, fu.lin[key]), (k, key)
                else:  # the windows differ by the previous steps' rounding
                    torch.testing.assert_close(v, fu.lin[key], rtol=1e-9, atol=1e-12, msg=f"{k} {key}")
        ds, df = sp.gn.out["delta"], fu.gn.out["delta"]
        assert (ds - df).abs().max().item() <= 1e-9 * df.abs().max().item(), k
    sp.close()
    fu.close()


@pytest.mark.parametrize("graph", [True, False])
def test_pre_ahead_matches_split(model, graph):
    """StreamingPipeline(pre_ahead=True): the next tick's pre half runs right after a tick's
    results (off the latency path).  The same kernels on the same data, so pixels, poses and
    info are bit for bit the split tick's, over camera ticks, keypoint ticks and a reset."""
    a, b = _pipe(model, graph), _pipe(model, graph, pre_ahead=True)
    assert b.pre_ahead and not a.pre_ahead
    truth, _, _ = _truth(3, 6)
    for seed in range(1, 4):
        rgb, d = _frames(seed)
        for x, y_ in zip(a.tick(rgb, d), b.tick(rgb, d)):
            np.testing.assert_array_equal(x, y_)
    for k in range(3):
        y = _keypoints(truth[k])
        for x, y_ in zip(a.tick_keypoints(y), b.tick_keypoints(y)):
            np.testing.assert_array_equal(x, y_)
    a.reset_window()
    b.reset_window()
    for k in range(3, 6):
        y = _keypoints(truth[k])
        for x, y_ in zip(a.tick_keypoints(y), b.tick_keypoints(y)):
            np.testing.assert_array_equal(x, y_)
    a.close()
    b.close()


@pytest.mark.parametrize("precision", ["fp16", "fp16x3"])
def test_zero_copy_out_matches_copy(precision):
    """zero_copy_out (the default: the head writes the pixels and the post half info and the
    newest poses into the pinned output block, no D2H copy) against the copying tick, bit for
    bit, graph replay, over camera ticks and keypoint ticks; also with the fused pose stage
    (pixels zero-copy, info / poses copied)."""
    m = _model(precision)
    for split in (True, False):
        a, b = _pipe(m, True, split_pose=split), _pipe(m, True, split_pose=split, zero_copy_out=False)
        for seed in range(1, 4):
            rgb, d = _frames(seed)
            for x, y_ in zip(a.tick(rgb, d), b.tick(rgb, d)):
                np.testing.assert_array_equal(x, y_)
        y = _keypoints(_truth(3, 1)[0][0])
        for x, y_ in zip(a.tick_keypoints(y), b.tick_keypoints(y)):
            np.testing.assert_array_equal(x, y_)
        a.close()
        b.close()


def _whiten(ref):
    sp, sd, sc = SIG["proj_sigma"], SIG["dyn_sigma"], SIG["cv_sigma"]
    ref["r_proj"], ref["j_proj"] = ref["r_proj"] / sp, ref["j_proj"] / sp
    for k in ("r_dyn", "j_dyn0", "j_dyn1", "j_dyn2", "j_dyn3"):
        ref[k] = ref[k] / sd
    ref["r_cv"] = ref["r_cv"] / sc
    return ref


def _device_lin(p):
    return {k: (v.transpose(1, 2) if k.startswith("j_") else v).cpu().numpy() for k, v in p.lin.items()
            if isinstance(v, torch.Tensor)}


def _check_tick(p, before, y_new, nvalid):
    """The oracle chain of one tick (advance -> factors, with the frames before the window's
    last `nvalid` masked -> dense GN -> retract) against the device's tick."""
    after = p.window_state()
    n, nk = 3, 8
    adv = F.window_advance(before, y_new, p.dt, "world")
    np.testing.assert_array_equal(adv["y"], after["y"])  # keypoints are only moved, never recomputed
    ref = _whiten(_oracle(adv["pose"].reshape(-1, 12), adv["vel"].reshape(-1, 3), adv["angvel"].reshape(-1, 3),
                          adv["y"].reshape(-1, 2 * nk), n, LW, p.dt, "world"))
    off = np.zeros((n, LW, nk), bool)
    off[:, :LW - nvalid] = True
    off = off.reshape(-1)
    ref["status"][off] = 2
    ref["r_proj"][off] = 0.0
    ref["j_proj"][off] = 0.0
    lin = _device_lin(p)
    np.testing.assert_array_equal(lin["status"], ref["status"])
    assert (ref["status"][~off] == 0).all()
    np.testing.assert_array_equal(lin["r_proj"][off], 0.0)
    np.testing.assert_array_equal(lin["j_proj"][off], 0.0)
    np.testing.assert_allclose(lin["r_proj"], ref["r_proj"], atol=1e-9, rtol=0)
    np.testing.assert_allclose(lin["j_proj"], ref["j_proj"], atol=1e-9, rtol=1e-12)
    for k in ("r_dyn", "j_dyn0", "j_dyn1", "j_dyn2", "j_dyn3", "r_cv"):
        np.testing.assert_allclose(lin[k], ref[k], atol=1e-9, rtol=1e-12, err_msg=k)
    # the GN step on the device's own whitened factors, every trajectory well conditioned:
    # backward error (the damped normal equations' residual) and the oracle's step within the
    # forward-error bound 10 cond(M) eps
    H, g, d = G.gn_step(lin, n, LW, nk, SIG["lam"])
    dd = p.gn.out["delta"].cpu().numpy().reshape(n, -1)
    info = p.info_h.numpy().copy()  # (the tick's info output: the pinned block, zero_copy_out)
    eps = np.finfo(np.float64).eps
    for t in range(n):
        M = H[t] + SIG["lam"] * np.eye(H.shape[1])
        cond = np.linalg.cond(M)
        assert cond < 1e10, (t, cond)  # constructed window: well conditioned
        assert info[t] == 0, t
        res = M @ dd[t] + g[t]
        assert np.abs(res).max() <= 1e-11 * (np.abs(M).max() * np.abs(dd[t]).max() + np.abs(g[t]).max()), t
        np.testing.assert_allclose(dd[t], d[t], rtol=0, atol=max(10 * cond * eps, 1e-9) * np.abs(d[t]).max())
    ret = F.window_retract(adv, dd, info)
    for k in ("pose", "vel", "angvel"):
        np.testing.assert_allclose(after[k], ret[k], rtol=0, atol=1e-12, err_msg=k)
    return after


def test_pose_tick_chain_vs_oracle(model):
    """A tick with a full window of consistent measurements (projected truth + 0.5 px noise)."""
    p = _pipe(model, True)
    truth, _, _ = _truth(3, LW + 1)
    rng = np.random.default_rng(7)
    for k in range(LW):  # fill the window with real frames
        p.tick_keypoints(_keypoints(truth[k], 0.5, rng))
    before = p.window_state()
    y_new = _keypoints(truth[LW], 0.5, rng)
    pose, info = p.tick_keypoints(y_new)
    after = _check_tick(p, before, y_new, LW)
    np.testing.assert_array_equal(pose, after["pose"][:, -1])  # the newest poses are the window's last frames
    assert (info == 0).all()
    p.close()


def test_first_tick_after_reset_has_one_measured_frame(model):
    """the frames a reset window holds are the initial state, not measurements.
    The first tick's window has one real frame; the others' projection factors are masked
    (status 2, zero rows) and the step is the oracle's on exactly that factor set."""
    p = _pipe(model, True)
    p.tick_keypoints(_keypoints(_truth(3, 1)[0][0]))  # something to reset from
    p.reset_window()
    before = p.window_state()
    y_new = _keypoints(_truth(3, 1)[0][0])
    p.tick_keypoints(y_new)
    _check_tick(p, before, y_new, 1)
    # two ticks in: two measured frames
    before = p.window_state()
    y2 = _keypoints(_truth(3, 2)[0][1])
    p.tick_keypoints(y2)
    _check_tick(p, before, y2, 2)
    p.close()


def test_pose_tracks_known_trajectory(model):
    """40 ticks of exact keypoints of a trajectory the dynamics model describes exactly,
    from an initial window 0.1 rad / 1 cm off and at rest: the GN step solves (info == 0)
    on every tick, and the newest pose converges to the true pose (rotation < 1e-4 rad,
    translation < 1e-5 m over the last 10 ticks; the measurements are f32 normalized
    coordinates, ~1e-5 px)."""
    n, ticks = 3, 40
    truth, w, v = _truth(n, ticks)
    p = _pipe(model, True, init=_init(n))
    err_r, err_t = [], []
    for k in range(ticks):
        pose, info = p.tick_keypoints(_keypoints(truth[k]))
        assert (info == 0).all(), (k, info)
        er, et = [], []
        for c in range(n):
            R, t = F.unpack(pose[c])
            Rt, tt = truth[k][c]
            er.append(np.linalg.norm(F.rot_log(Rt.T @ R)))
            et.append(np.linalg.norm(t - tt))
        err_r.append(max(er))
        err_t.append(max(et))
    print("rotation error (rad) per tick:", " ".join(f"{e:.1e}" for e in err_r))
    print("translation error (m) per tick:", " ".join(f"{e:.1e}" for e in err_t))
    assert err_r[0] > 1e-3  # it starts off the truth
    assert max(err_r[-10:]) < 1e-4 and max(err_t[-10:]) < 1e-5
    st = p.window_state()
    # the velocities of the last frame pair (frame L-1's own angular velocity is only carried
    # over at the advance: no factor touches it)
    np.testing.assert_allclose(st["angvel"][:, -2], w, atol=1e-3)  # body angular velocity recovered
    np.testing.assert_allclose(st["vel"][:, -2], v, atol=1e-4)     # world velocity recovered
    p.close()


def test_pose_window_rejects_bad_config(model):
    with pytest.raises(ValueError):
        StreamingPipeline(model, pose_window=1)
    with pytest.raises(AssertionError):
        StreamingPipeline(model, pose_window=4, vel_frame="camera")


def test_fused_pose_tick_limits(model):
    """pa_window_pose_tick refuses windows above 24 frames (PA_EINVAL, nothing launched);
    StreamingPipeline then runs the four separate launches, and a 30-frame window still
    solves."""
    from perseus_amd import _lib, pipeline

    p0, v0, w0 = _init()
    p = StreamingPipeline(model, graph=True, pose_window=30, init_pose=p0, init_vel=v0, init_angvel=w0, **SIG)
    assert not p.fused_pose and not p.split_pose
    with pytest.raises(_lib.PerseusError, match="L 30"):
        pipeline.window_pose_tick(p.traj_args, p.y, lam=1e-2, delta=p.gn.out["delta"], info=p.gn.out["info"])
    ws = torch.empty(1 << 22, dtype=torch.uint8, device=p.dev)
    with pytest.raises(_lib.PerseusError, match="L 30"):
        pipeline.window_pose_tick_pre(p.traj_args, ws, lam=1e-2)
    with pytest.raises(_lib.PerseusError, match="L 30"):
        pipeline.window_pose_tick_post(p.traj_args, p.y, ws, delta=p.gn.out["delta"], info=p.gn.out["info"])
    truth, _, _ = _truth(3, 3)
    for k in range(3):
        _, info = p.tick_keypoints(_keypoints(truth[k]))
    assert (info == 0).all()
    p.close()


def test_pre_ahead_request_is_never_dropped_silently(model):
    """pre_ahead needs the split tick; without it the pipeline warns and reports
    pre_ahead False.  With split + zero-copy output, the GN info lives only in the pinned
    block: no stale device buffer is exposed as gn.out['info']."""
    with pytest.warns(RuntimeWarning, match="pre_ahead"):
        p = StreamingPipeline(model, graph=False, pose_window=4, split_pose=False, pre_ahead=True, **SIG)
    assert not p.pre_ahead and not p.split_pose
    p.close()
    p0, v0, w0 = _init()
    q = StreamingPipeline(model, graph=False, pose_window=4, zero_copy_out=True, init_pose=p0, init_vel=v0,
                          init_angvel=w0, **SIG)
    assert q.split_pose and q.gn.out["info"] is None
    truth, _, _ = _truth(3, 3)
    _, info = q.tick_keypoints(_keypoints(truth[0]))
    assert (info == 0).all()
    q.close()
