"""pa_trajectory_gn_step with keypoint counts other than 8 (the kernel's general stacked-row
instantiation, RP = 2 * GN_KMAX + 18) against the dense f64 oracle (oracle/gn_ref.py), and
trajectory counts that leave most of the chip idle or oversubscribe it.  Same tolerances
as test_gn_gpu.py."""
import numpy as np
import pytest
import torch

from oracle import gn_ref as G
from perseus_amd import pipeline

from test_pipeline_gpu import CORNERS, KCAL, _problem  # tests/ is on sys.path (rootdir conftest)

pytestmark = pytest.mark.gpu
RTOL = 1e-9
S = 0.0175
FACES = np.array([[S, 0, 0], [-S, 0, 0], [0, S, 0], [0, -S, 0], [0, 0, S], [0, 0, -S]])


def _check(corners, T, L, lam, seed, variant=None):
    K = len(corners)
    poses, vels, angvels, _ = _problem(T, L, seed)
    y = np.random.default_rng(seed + 1).uniform(-1, 1, (T * L, 2 * K)).astype(np.float32)
    lin = pipeline.linearize_trajectories(torch.as_tensor(y, device="cuda"), poses, vels, angvels, corners, KCAL,
                                          T=T, L=L, dt=0.1, proj_sigmas=np.array([2.0, 2.0]),
                                          dyn_sigmas=np.full(6, 0.05), cv_sigmas=np.full(3, 0.5))
    if variant is None:
        out = pipeline.gn_step(lin, T=T, L=L, lam=lam)
    else:
        from perseus_amd import _lib

        L_ = _lib.lib()
        try:
            _lib.check(L_.pa_debug_gn_set_assemblers(variant))
            out = pipeline.gn_step(lin, T=T, L=L, lam=lam)
        finally:
            _lib.check(L_.pa_debug_gn_set_assemblers(0))
    keys = ("r_proj", "j_proj", "status", "r_dyn", "j_dyn0", "j_dyn1", "j_dyn2", "j_dyn3", "r_cv", "j_cv0", "j_cv1")
    H, g, d = G.gn_step({k: lin[k].cpu().numpy() for k in keys}, T, L, K, lam)
    assert (out["info"].cpu().numpy() == 0).all()
    Dd, Ed = out["D"].cpu().numpy(), out["E"].cpu().numpy()
    for t in range(T):
        D, E = G.blocks(H[t], L)
        scale = np.abs(H[t]).max()
        np.testing.assert_allclose(Dd[t * L:(t + 1) * L], D, rtol=RTOL, atol=RTOL * scale)
        if L > 1:
            np.testing.assert_allclose(Ed[t * (L - 1):(t + 1) * (L - 1)], E, rtol=RTOL, atol=RTOL * scale)
    np.testing.assert_allclose(out["g"].cpu().numpy().reshape(T, -1), g, rtol=RTOL, atol=RTOL * np.abs(g).max())
    # delta: the damped normal equations' residual (backward error), and the oracle's step
    # within 1e-9 of its scale or, for the ill-conditioned systems (K = 1: one keypoint per
    # frame leaves the pose weakly constrained), within the forward-error bound 10 cond eps
    dd = out["delta"].cpu().numpy().reshape(T, -1)
    eps = np.finfo(np.float64).eps
    for t in range(T):
        M = H[t] + lam * np.eye(H.shape[1])
        res = M @ dd[t] + g[t]
        assert np.abs(res).max() <= 1e-11 * (np.abs(M).max() * np.abs(dd[t]).max() + np.abs(g[t]).max()), t
        tol = max(1e-9, 10 * np.linalg.cond(M) * eps) * np.abs(d[t]).max()
        np.testing.assert_allclose(dd[t], d[t], rtol=1e-7, atol=tol, err_msg=f"trajectory {t}")


@pytest.mark.parametrize("corners", [CORNERS[:4], np.concatenate([CORNERS, FACES]), CORNERS[:1]],
                         ids=["K4", "K14", "K1"])
def test_gn_step_other_keypoint_counts(corners):
    _check(corners, 3, 7, 1e-3, 21)


def test_gn_step_many_trajectories():
    """600 trajectories: several workgroups per CU, slot reuse over 13 frames."""
    _check(CORNERS, 600, 13, 1e-2, 4)


@pytest.mark.parametrize("L", [2, 3, 4, 25])
def test_gn_step_short_and_odd_windows(L):
    """The two-ended elimination's edge cases (gn_twisted_kernel, merge frame m = L / 2): L = 2
    has no bottom chain, L = 3 a one-frame bottom chain, L = 25 chains of unequal length."""
    _check(CORNERS, 5, L, 1e-3, 30 + L)


def test_gn_step_more_trajectories_than_one_round():
    """1,100 trajectories: more four-wave workgroups than one round holds at four per CU."""
    _check(CORNERS, 1100, 6, 1e-2, 8)


@pytest.mark.parametrize("variant", [16 + 2, 8 + 2])
def test_gn_step_solver_variants_agree(variant):
    """The single-chain solver (16 + NA) and the round-2 block Cholesky (8 + NA), kept as
    pa_debug_gn_set_assemblers variants, against the shipped kernel (cyclic reduction at T = 4)."""
    from perseus_amd import _lib

    poses, vels, angvels, _ = _problem(4, 24, 3)
    y = np.random.default_rng(4).uniform(-1, 1, (4 * 24, 16)).astype(np.float32)
    lin = pipeline.linearize_trajectories(torch.as_tensor(y, device="cuda"), poses, vels, angvels, CORNERS, KCAL,
                                          T=4, L=24, dt=0.1, proj_sigmas=np.array([2.0, 2.0]),
                                          dyn_sigmas=np.full(6, 0.05), cv_sigmas=np.full(3, 0.5))
    ref = pipeline.gn_step(lin, T=4, L=24, lam=1e-3)
    L_ = _lib.lib()
    try:
        _lib.check(L_.pa_debug_gn_set_assemblers(variant))
        out = pipeline.gn_step(lin, T=4, L=24, lam=1e-3)
    finally:
        _lib.check(L_.pa_debug_gn_set_assemblers(0))
    d0, d1 = ref["delta"].cpu().numpy(), out["delta"].cpu().numpy()
    np.testing.assert_allclose(d1, d0, rtol=1e-7, atol=1e-9 * np.abs(d0).max())
    assert torch.equal(ref["D"], out["D"]) and torch.equal(ref["g"], out["g"])


@pytest.mark.parametrize("L", [1, 2, 3, 4, 5, 7, 13, 23, 24])
@pytest.mark.parametrize("variant", [64, 128], ids=["cyclic", "two-ended"])
def test_gn_step_cyclic_reduction_and_two_ended_forms(L, variant):
    """Both solvers at every level shape of the cyclic reduction (n odd: the even positions are
    eliminated, ends included; n even: the odd ones; L = 1: the last-frame solve alone), forced
    through pa_debug_gn_set_assemblers (64: cyclic reduction, 128: the two-ended elimination)."""
    _check(CORNERS, 3, L, 1e-3, 50 + L, variant)


def test_gn_step_cyclic_reduction_many_trajectories():
    """The cyclic-reduction kernel forced at 600 trajectories (several rounds of one
    workgroup per CU)."""
    _check(CORNERS, 600, 24, 1e-2, 6, 64)


@pytest.mark.parametrize("variant", [64, 128], ids=["cyclic", "two-ended"])
def test_gn_step_singular_in_both_forms(variant):
    """lambda = 0: the last frame's angular velocity has no factor; both forms report that
    frame (L) and NaN steps."""
    from perseus_amd import _lib

    T, L = 2, 6
    poses, vels, angvels, y = _problem(T, L, 9)
    lin = pipeline.linearize_trajectories(torch.as_tensor(y, device="cuda"), poses, vels, angvels, CORNERS, KCAL,
                                          T=T, L=L, dt=0.1, proj_sigmas=np.array([2.0, 2.0]),
                                          dyn_sigmas=np.full(6, 0.05), cv_sigmas=np.full(3, 0.5))
    L_ = _lib.lib()
    try:
        _lib.check(L_.pa_debug_gn_set_assemblers(variant))
        out = pipeline.gn_step(lin, T=T, L=L, lam=0.0)
    finally:
        _lib.check(L_.pa_debug_gn_set_assemblers(0))
    assert (out["info"].cpu().numpy() == L).all()
    assert torch.isnan(out["delta"]).all()
