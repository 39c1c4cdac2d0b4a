"""GPU parity of the f64 factor kernels against the oracle / golden vectors."""
import os

import numpy as np
import pytest
import torch

from oracle import factors_ref as F
from perseus_amd import smoother

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
ATOL = 1e-9


@pytest.fixture(scope="module")
def g():
    return dict(np.load(os.path.join(GOLD, "factors_golden.npz")))


@pytest.mark.parametrize("vf", ["world", "body"])
def test_dynamics_batch_vs_golden(g, vf):
    out = smoother.linearize_dynamics(g["batch/T1"], g["batch/w"], g["batch/v"], g["batch/T2"], 1.0 / 12.0, vf)
    np.testing.assert_allclose(out["r"].cpu().numpy(), g[f"batch/dyn_{vf}/r"], atol=ATOL)
    for i in range(4):
        np.testing.assert_allclose(out[f"J{i}"].cpu().numpy(), g[f"batch/dyn_{vf}/J{i}"], atol=ATOL)


@pytest.mark.parametrize("vf", ["world", "body"])
def test_dropin_error_func_reference_test_problem(g, vf):
    """tests/test_dynamics_factor.py's problem through the drop-in error_func/H surface,
    checked against the pypose-formulation autodiff at the reference's atol 1e-6."""
    v = smoother.Values()
    T1, T2 = F.unpack(g["test/T1"]), F.unpack(g["test/T2"])
    v.insert("x0", smoother.Pose3(*T1))
    v.insert("x1", smoother.Pose3(*T2))
    v.insert("w0", g["test/ang1"])
    v.insert("v0", g["test/vel1"])
    nm = smoother.noiseModel.Diagonal.Sigmas(np.array([1e-1] * 6))
    f = smoother.PoseDynamicsFactor("x0", "w0", "v0", "x1", nm, 0.1, vel_frame=vf)
    e_plain = f.error_func(f, v)
    H = [np.zeros((6, 6), order="F"), np.zeros((6, 3), order="F"), np.zeros((6, 3), order="F"),
         np.zeros((6, 6), order="F")]
    e = f.error_func(f, v, H)
    ea, Ha = F.autodiff_dynamics(T1, g["test/ang1"], g["test/vel1"], T2, 0.1, vf)
    assert np.allclose(e, ea, atol=1e-6) and np.allclose(e_plain, ea, atol=1e-6)
    for i in range(4):
        assert np.allclose(H[i], Ha[i], atol=1e-6)
    A, b = f.linearize(v)
    np.testing.assert_allclose(b, -e / 0.1, atol=1e-12)
    np.testing.assert_allclose(A[0], H[0] / 0.1, atol=1e-12)
    assert abs(f.error(v) - 0.5 * np.sum((e / 0.1) ** 2)) < 1e-9


def test_const_vel(g):
    out = smoother.linearize_const_vel(g["test/vel1"][None], g["test/vel2"][None])
    np.testing.assert_array_equal(out["r"].cpu().numpy()[0], g["test/vel2"] - g["test/vel1"])
    np.testing.assert_array_equal(out["J0"].cpu().numpy()[0], -np.eye(3))
    np.testing.assert_array_equal(out["J1"].cpu().numpy()[0], np.eye(3))
    v = smoother.Values()
    v.insert(1, g["test/vel1"])
    v.insert(2, g["test/vel2"])
    f = smoother.ConstantVelocityFactor(1, 2, smoother.noiseModel.Diagonal.Sigmas(np.array([0.1] * 3)))
    H = [None, None]
    e = f.error_func(f, v, H)
    np.testing.assert_array_equal(e, g["test/vel2"] - g["test/vel1"])
    np.testing.assert_array_equal(H[1], np.eye(3))


def test_projection_vs_golden_and_cheirality(g):
    out = smoother.linearize_projection(g["proj/T"], g["proj/pb"], g["proj/z"], g["proj/K"])
    st = out["status"].cpu().numpy()
    np.testing.assert_array_equal(st, g["proj/status"])
    ok = st == 0
    np.testing.assert_allclose(out["r"].cpu().numpy()[ok], g["proj/r"][ok], atol=ATOL)
    np.testing.assert_allclose(out["J"].cpu().numpy()[ok], g["proj/J"][ok], atol=ATOL)
    assert np.isnan(out["r"].cpu().numpy()[~ok]).all()


def test_projection_dropin_and_camera_pose(g):
    v = smoother.Values()
    T = F.unpack(g["proj/T"][0])
    v.insert(0, smoother.Pose3(*T))
    K = smoother.Cal3_S2(*g["proj/K"])
    nm = smoother.noiseModel.Isotropic.Sigma(2, 1.5)
    cam = (F.rot_exp(np.array([0.05, -0.02, 0.01])), np.array([0.01, 0.0, -0.02]))
    f = smoother.KeypointProjectionFactor(0, nm, K, g["proj/z"][0], g["proj/pb"][0], smoother.Pose3(*cam))
    H = [None]
    r = f.error_func(f, v, H)
    r0, J0, st, pix = F.projection(T, g["proj/pb"][0], g["proj/z"][0], g["proj/K"], cam)
    np.testing.assert_allclose(r, r0, atol=ATOL)
    np.testing.assert_allclose(H[0], J0, atol=ATOL)
    np.testing.assert_allclose(f.pixel, pix, atol=1e-9)
    # behind the camera -> CheiralityException (GTSAM raises from camera.project)
    v2 = smoother.Values()
    v2.insert(0, smoother.Pose3(np.eye(3), [0, 0, -1.0]))
    f2 = smoother.KeypointProjectionFactor(0, nm, K, [0, 0], [0, 0, 0])
    with pytest.raises(smoother.CheiralityException):
        f2.error_func(f2, v2, [None])


def test_whitening_and_error():
    rng = np.random.default_rng(0)
    n = 1000
    T1 = np.stack([F.pack(F.pose_exp(rng.standard_normal(6))) for _ in range(n)])
    T2 = np.stack([F.pack(F.pose_exp(rng.standard_normal(6))) for _ in range(n)])
    w, v = rng.standard_normal((n, 3)), rng.standard_normal((n, 3))
    isig = np.array([10.0, 10, 10, 5, 5, 5])
    raw = smoother.linearize_dynamics(T1, w, v, T2, 1 / 12)
    wh = smoother.linearize_dynamics(T1, w, v, T2, 1 / 12, inv_sigma=isig)
    torch.testing.assert_close(wh["r"], raw["r"] * torch.tensor(isig, device="cuda"), rtol=1e-14, atol=1e-14)
    torch.testing.assert_close(wh["J0"], raw["J0"] * torch.tensor(isig, device="cuda")[:, None], rtol=1e-14,
                               atol=1e-14)
    torch.testing.assert_close(wh["err"], 0.5 * (wh["r"] ** 2).sum(1), rtol=1e-14, atol=1e-14)
    # spot-check against the oracle
    for i in (0, 499, 999):
        e, H = F.dynamics(F.unpack(T1[i]), w[i], v[i], F.unpack(T2[i]), 1 / 12)
        np.testing.assert_allclose(raw["r"][i].cpu().numpy(), e, atol=ATOL)
        np.testing.assert_allclose(raw["J2"][i].cpu().numpy(), H[2], atol=ATOL)


def test_branches_small_and_near_pi():
    """Log/Exp branch points: identity-ish relative pose (theta < 1e-10), near-pi rotation
    (trace ~ -1 branch) and a zero twist (Expmap small-angle branch)."""
    T1 = np.stack([F.pack((np.eye(3), np.zeros(3))),
                   F.pack((F.rot_exp(np.array([0, 0, np.pi - 1e-6])), np.array([0.1, 0, 0]))),
                   F.pack(F.pose_exp(np.array([0.2, 0.1, -0.3, 1, 2, 3])))])
    w = np.zeros((3, 3))
    v = np.zeros((3, 3))
    T2 = np.stack([F.pack((np.eye(3), np.zeros(3))), F.pack((np.eye(3), np.zeros(3))), T1[2]])
    out = smoother.linearize_dynamics(T1, w, v, T2, 0.1)
    for i in range(3):
        e, H = F.dynamics(F.unpack(T1[i]), w[i], v[i], F.unpack(T2[i]), 0.1)
        np.testing.assert_allclose(out["r"][i].cpu().numpy(), e, atol=1e-8)
        for k in range(4):
            np.testing.assert_allclose(out[f"J{k}"][i].cpu().numpy(), H[k], atol=1e-6)


def test_empty():
    out = smoother.linearize_dynamics(np.zeros((0, 12)), np.zeros((0, 3)), np.zeros((0, 3)), np.zeros((0, 12)), 0.1)
    assert out["r"].shape == (0, 6)
