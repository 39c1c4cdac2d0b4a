"""Config 3 parity: fused trajectory factor linearize (pa_trajectory_linearize) against
the f64 oracle restatement of factors.py fed with the same denormalized keypoints."""
import numpy as np
import pytest
import torch

from oracle import factors_ref as F
from oracle import resnet_ref as R
from perseus_amd import pipeline

pytestmark = pytest.mark.gpu
ATOL = 1e-9
KCAL = np.array([280.0, 280.0, 0.0, 128.0, 128.0])
S = 0.0175
CORNERS = np.array([[x, y, z] for x in (-S, S) for y in (-S, S) for z in (-S, S)])


def _problem(T, L, seed, behind=()):
    rng = np.random.default_rng(seed)
    Fn = T * L
    poses = np.zeros((Fn, 12))
    for f in range(Fn):
        R, _ = F.pose_exp(np.concatenate([0.4 * rng.standard_normal(3), np.zeros(3)]))
        t = np.array([0.05 * rng.standard_normal(), 0.05 * rng.standard_normal(), 0.3 + 0.2 * rng.random()])
        if f in behind:
            t[2] = -0.3  # every corner behind the camera: cheirality
        poses[f] = F.pack((R, t))
    vels = rng.standard_normal((Fn, 3))
    angvels = rng.standard_normal((Fn, 3))
    y = rng.uniform(-1, 1, (Fn, 2 * len(CORNERS))).astype(np.float32)
    return poses, vels, angvels, y


def _denorm(y, H=256, W=256):
    """kornia denormalize_pixel_coordinates in f32 (validate.py:144-153)."""
    return R.denormalize_f32(y, H, W).astype(np.float64)


def _oracle(poses, vels, angvels, y, T, L, dt, vf, Tc=None):
    nk = len(CORNERS)
    z = _denorm(y).reshape(-1, 2)
    Tb = np.repeat(poses, nk, axis=0)
    pb = np.tile(CORNERS, (T * L, 1))
    rp, Jp, st = F.projection_batch(Tb, pb, z, KCAL, Tc)
    idx = np.array([t * L + l for t in range(T) for l in range(L - 1)], dtype=np.int64)
    rd, J0, J1, J2, J3 = F.dynamics_batch(poses[idx], angvels[idx], vels[idx], poses[idx + 1], dt, vf)
    rc = vels[idx + 1] - vels[idx]
    return dict(r_proj=rp, j_proj=Jp, status=st, r_dyn=rd, j_dyn0=J0, j_dyn1=J1, j_dyn2=J2, j_dyn3=J3, r_cv=rc)


def _cmp(out, ref):
    st = out["status"].cpu().numpy()
    np.testing.assert_array_equal(st, ref["status"])
    ok = st == 0
    np.testing.assert_allclose(out["r_proj"].cpu().numpy()[ok], ref["r_proj"][ok], atol=ATOL, rtol=0)
    np.testing.assert_allclose(out["j_proj"].cpu().numpy()[ok], ref["j_proj"][ok], atol=ATOL, rtol=1e-12)
    assert np.isnan(out["r_proj"].cpu().numpy()[~ok]).all()
    for k in ("r_dyn", "j_dyn0", "j_dyn1", "j_dyn2", "j_dyn3", "r_cv"):
        np.testing.assert_allclose(out[k].cpu().numpy(), ref[k], atol=ATOL, rtol=1e-12, err_msg=k)


@pytest.mark.parametrize("vf", ["world", "body"])
def test_trajectory_vs_oracle(vf):
    T, L, dt = 3, 7, 1.0 / 12.0
    poses, vels, angvels, y = _problem(T, L, 11, behind=(5,))
    out = pipeline.linearize_trajectories(torch.as_tensor(y, device="cuda"), poses, vels, angvels, CORNERS, KCAL,
                                          T=T, L=L, dt=dt, vel_frame=vf)
    ref = _oracle(poses, vels, angvels, y, T, L, dt, vf)
    assert ref["status"].sum() == len(CORNERS)
    _cmp(out, ref)
    np.testing.assert_array_equal(out["j_cv0"].cpu().numpy(), np.broadcast_to(-np.eye(3), (T * (L - 1), 3, 3)))
    np.testing.assert_array_equal(out["j_cv1"].cpu().numpy(), np.broadcast_to(np.eye(3), (T * (L - 1), 3, 3)))


def test_trajectory_camera_pose_and_whitening():
    T, L, dt = 2, 5, 0.1
    poses, vels, angvels, y = _problem(T, L, 3)
    Rc, _ = F.pose_exp(np.array([0.02, -0.01, 0.03, 0, 0, 0]))
    Tc = (Rc, np.array([0.01, -0.02, -0.05]))
    sp, sd, sc = np.array([2.0, 3.0]), np.full(6, 0.1), np.array([0.5, 0.25, 1.0])
    out = pipeline.linearize_trajectories(torch.as_tensor(y, device="cuda"), poses, vels, angvels, CORNERS, KCAL,
                                          T=T, L=L, dt=dt, camera_pose=F.pack(Tc), proj_sigmas=sp, dyn_sigmas=sd,
                                          cv_sigmas=sc)
    ref = _oracle(poses, vels, angvels, y, T, L, dt, "world", F.pack(Tc))
    ref["r_proj"] = ref["r_proj"] / sp
    ref["j_proj"] = ref["j_proj"] / sp[:, None]
    for k in ("j_dyn0", "j_dyn1", "j_dyn2", "j_dyn3"):
        ref[k] = ref[k] / sd[:, None]
    ref["r_dyn"] = ref["r_dyn"] / sd
    ref["r_cv"] = ref["r_cv"] / sc
    _cmp(out, ref)
    np.testing.assert_allclose(out["err_proj"].cpu().numpy(), 0.5 * (ref["r_proj"] ** 2).sum(1), rtol=1e-12)
    np.testing.assert_allclose(out["err_dyn"].cpu().numpy(), 0.5 * (ref["r_dyn"] ** 2).sum(1), rtol=1e-12)
    np.testing.assert_allclose(out["err_cv"].cpu().numpy(), 0.5 * (ref["r_cv"] ** 2).sum(1), rtol=1e-12)


def test_single_frame_trajectories_and_no_jacobians():
    T, L = 4, 1
    poses, vels, angvels, y = _problem(T, L, 5)
    out = pipeline.linearize_trajectories(torch.as_tensor(y, device="cuda"), poses, vels, angvels, CORNERS, KCAL,
                                          T=T, L=L, dt=0.1, jacobians=False)
    assert out["r_dyn"].shape == (0, 6) and out["j_proj"] is None
    ref = _oracle(poses, vels, angvels, y, T, L, 0.1, "world")
    np.testing.assert_allclose(out["r_proj"].cpu().numpy(), ref["r_proj"], atol=ATOL, rtol=0)


def test_bad_vel_frame():
    with pytest.raises(AssertionError):
        pipeline.linearize_trajectories(torch.zeros((2, 16), device="cuda"), np.zeros((2, 12)), np.zeros((2, 3)),
                                        np.zeros((2, 3)), CORNERS, KCAL, T=1, L=2, dt=0.1, vel_frame="camera")


def test_detect_and_linearize_uses_device_keypoints():
    from perseus_amd.detector import KeypointCNN
    from perseus_amd.synth import synthetic_frames, synthetic_state_dict

    T, L = 2, 4
    m = KeypointCNN(n_keypoints=8, num_channels=4).cuda()
    m.load_state_dict({k: torch.as_tensor(v) for k, v in synthetic_state_dict(0).items()})
    x = torch.as_tensor(synthetic_frames(1, T * L)).cuda()
    poses, vels, angvels, _ = _problem(T, L, 9)
    out = pipeline.detect_and_linearize(m, x, poses, vels, angvels, CORNERS, KCAL, T=T, L=L, dt=1 / 12)
    y = out["y"].cpu().numpy()
    ref = _oracle(poses, vels, angvels, y, T, L, 1 / 12, "world")
    _cmp(out, ref)


def test_full_size_config3_sampled_vs_oracle():
    """BASELINE configs[3] size (1000 trajectories x 24 frames): a seeded sample of
    every factor type against the oracle, plus properties over all of them."""
    from perseus_amd import synth

    T, L, dt = 1000, 24, 1 / 12
    tr = synth.synthetic_trajectories(5, T, L)
    out = pipeline.linearize_trajectories(torch.as_tensor(tr["y"], device="cuda"), tr["poses"], tr["vels"],
                                          tr["angvels"], tr["corners"], tr["K"], T=T, L=L, dt=dt)
    rng = np.random.default_rng(0)
    nk = 8
    z = _denorm(tr["y"]).reshape(-1, 2)
    for i in rng.choice(T * L * nk, 300, replace=False):
        f, k = divmod(int(i), nk)
        r, H0, st, _ = F.projection(F.unpack(tr["poses"][f]), tr["corners"][k], z[i], tr["K"])
        assert out["status"][i].item() == st == 0
        np.testing.assert_allclose(out["r_proj"][i].cpu().numpy(), r, atol=ATOL, rtol=0)
        np.testing.assert_allclose(out["j_proj"][i].cpu().numpy(), H0, atol=ATOL, rtol=1e-12)
    for j in rng.choice(T * (L - 1), 100, replace=False):
        t, l = divmod(int(j), L - 1)
        f = t * L + l
        r, H = F.dynamics(F.unpack(tr["poses"][f]), tr["angvels"][f], tr["vels"][f], F.unpack(tr["poses"][f + 1]),
                          dt, "world")
        np.testing.assert_allclose(out["r_dyn"][j].cpu().numpy(), r, atol=ATOL, rtol=0)
        for q in range(4):
            np.testing.assert_allclose(out[f"j_dyn{q}"][j].cpu().numpy(), H[q], atol=ATOL, rtol=1e-12)
    # whole-array properties: every corner is in front of the camera; const-vel exact
    assert int(out["status"].sum()) == 0 and torch.isfinite(out["j_proj"]).all()
    v = torch.as_tensor(tr["vels"], device="cuda").reshape(T, L, 3)
    assert torch.equal(out["r_cv"].reshape(T, L - 1, 3), v[:, 1:] - v[:, :-1])


def test_window_retract_newest_vs_oracle():
    """pa_window_retract_newest (the streaming tick's pose output): the window retract of
    oracle/factors_ref.window_retract, plus each trajectory's newest pose after it -- also
    for a trajectory the GN step did not solve (info != 0: window and newest pose unchanged)."""
    T, L = 3, 5
    poses, vels, angvels, _ = _problem(T, L, 9)
    rng = np.random.default_rng(3)
    delta = 0.05 * rng.standard_normal((T * L, 12))
    info = np.array([0, 2, 0], dtype=np.int32)
    win = {"pose": poses.reshape(T, L, 12), "vel": vels.reshape(T, L, 3), "angvel": angvels.reshape(T, L, 3)}
    dwin = {k: torch.as_tensor(np.ascontiguousarray(v), device="cuda") for k, v in win.items()}
    newest = torch.full((T, 12), float("nan"), dtype=torch.float64, device="cuda")
    pipeline.window_retract(dwin, torch.as_tensor(delta, device="cuda"), torch.as_tensor(info, device="cuda"),
                            newest=newest)
    ref = F.window_retract(win, delta, info)
    for k in ("pose", "vel", "angvel"):
        np.testing.assert_allclose(dwin[k].cpu().numpy(), ref[k], rtol=0, atol=1e-12, err_msg=k)
    np.testing.assert_array_equal(newest.cpu().numpy(), dwin["pose"][:, -1].cpu().numpy())
    np.testing.assert_array_equal(newest.cpu().numpy()[1], poses.reshape(T, L, 12)[1, -1])
