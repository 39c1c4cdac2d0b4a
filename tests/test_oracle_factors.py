"""Oracle pinning (CPU): closed-form GTSAM restatement vs the autodiff restatement of
tests/test_dynamics_factor.py's pypose oracle (atol 1e-6, the reference's tolerance) and
vs the committed golden vectors."""
import os

import numpy as np
import pytest

from oracle import factors_ref as F

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def g():
    return dict(np.load(os.path.join(GOLD, "factors_golden.npz")))


def test_seeded_problem_is_reference_seed(g):
    # tests/test_dynamics_factor.py:11-21 with np.random.seed(0)
    np.random.seed(0)
    xi1, xi2 = np.random.randn(6), np.random.randn(6)
    vel1, ang1 = np.random.randn(3), np.random.randn(3)
    np.testing.assert_allclose(g["test/T1"], F.pack(F.pose_exp(xi1)))
    np.testing.assert_allclose(g["test/vel1"], vel1)
    np.testing.assert_allclose(g["test/ang1"], ang1)
    np.testing.assert_allclose(xi1[:3], [1.764052, 0.400157, 0.978738], atol=1e-6)


@pytest.mark.parametrize("vf", ["world", "body"])
def test_dynamics_matches_pypose_formulation(g, vf):
    T1, T2 = F.unpack(g["test/T1"]), F.unpack(g["test/T2"])
    e, H = F.dynamics(T1, g["test/ang1"], g["test/vel1"], T2, 0.1, vf)
    ea, Ha = F.autodiff_dynamics(T1, g["test/ang1"], g["test/vel1"], T2, 0.1, vf)
    assert np.allclose(e, ea, atol=1e-6)
    for i in range(4):
        assert np.allclose(H[i], Ha[i], atol=1e-6)
        np.testing.assert_allclose(H[i], g[f"test/dyn_{vf}/H{i}"], atol=1e-12)
    # error-only branch (factors.py:131-140) agrees with the Jacobian branch
    e2, _ = F.dynamics(T1, g["test/ang1"], g["test/vel1"], T2, 0.1, vf, jac=False)
    np.testing.assert_allclose(e2, e, atol=1e-14)


def test_const_vel(g):
    e, H = F.const_vel(g["test/vel1"], g["test/vel2"])
    np.testing.assert_allclose(e, g["test/vel2"] - g["test/vel1"])
    np.testing.assert_array_equal(H[0], -np.eye(3))
    np.testing.assert_array_equal(H[1], np.eye(3))


def test_projection_autodiff_and_cheirality(g):
    r, J, st = F.projection_batch(g["proj/T"], g["proj/pb"], g["proj/z"], g["proj/K"])
    np.testing.assert_array_equal(st, g["proj/status"])
    ok = st == 0
    np.testing.assert_allclose(r[ok], g["proj/r"][ok], atol=1e-12)
    for i in np.nonzero(ok)[0][:8]:
        ra, Ja = F.autodiff_projection(F.unpack(g["proj/T"][i]), g["proj/pb"][i], g["proj/z"][i], g["proj/K"])
        np.testing.assert_allclose(J[i], Ja, atol=1e-6)


def test_datagen_projection_convention():
    """K from data_generation: f = W / (2 tan(fov/2)), fov = 2 atan(16/35) -> 280 px."""
    fov = 2 * np.arctan(16 / 35)
    f = 256 / (2 * np.tan(fov / 2))
    assert abs(f - 280.0) < 1e-9
    # a point on the optical axis projects to the principal point
    r, _, st, pix = F.projection((np.eye(3), np.array([0, 0, 0.5])), [0, 0, 0], [0, 0], (f, f, 0, 128, 128))
    assert st == 0 and np.allclose(pix, [128, 128])


@pytest.mark.parametrize("w", [np.array([1e-9, -2e-9, 0.0]), np.array([0.0, 0.0, np.pi - 1e-5]),
                               np.array([0.3, -2.9, 1.1]) / np.linalg.norm([0.3, -2.9, 1.1]) * (np.pi - 1e-7),
                               np.array([0.4, 0.1, -0.3])])
def test_log_exp_branches(w):
    np.testing.assert_allclose(F.rot_log(F.rot_exp(w)), w, atol=1e-6)
    J = F.rot_dexp(w) @ F.rot_dlog(w)
    if np.linalg.norm(w) < 3.0:
        np.testing.assert_allclose(J, np.eye(3), atol=1e-8)


def test_dexp_q_near_zero_branch_continuity():
    xi_a = np.array([1e-5 * 1.01, 0, 0, 0.3, -0.2, 0.1])
    xi_b = np.array([1e-5 * 0.99, 0, 0, 0.3, -0.2, 0.1])
    np.testing.assert_allclose(F.compute_q(xi_a), F.compute_q(xi_b), atol=1e-6)
