"""GPU parity of the factor-graph consumer (pa_trajectory_gn_step) against
the dense f64 oracle (oracle/gn_ref.py) fed with the device's own whitened factors.

Tolerance: rtol 1e-9 on D, E, g (f64 sums in a different order) and on delta (block vs dense
Cholesky on well-conditioned damped systems)."""
import numpy as np
import pytest
import torch

from oracle import gn_ref as G
from perseus_amd import pipeline

from test_pipeline_gpu import CORNERS, KCAL, _problem  # tests/ is on sys.path (rootdir conftest)

pytestmark = pytest.mark.gpu
RTOL = 1e-9


def _lin(T, L, seed, behind=()):
    poses, vels, angvels, y = _problem(T, L, seed, behind)
    return pipeline.linearize_trajectories(torch.as_tensor(y, device="cuda"), poses, vels, angvels, CORNERS, KCAL,
                                           T=T, L=L, dt=0.1, proj_sigmas=np.array([2.0, 2.0]),
                                           dyn_sigmas=np.full(6, 0.05), cv_sigmas=np.full(3, 0.5))


def _np(lin):
    keys = ("r_proj", "j_proj", "status", "r_dyn", "j_dyn0", "j_dyn1", "j_dyn2", "j_dyn3", "r_cv", "j_cv0", "j_cv1")
    return {k: lin[k].cpu().numpy() for k in keys}


@pytest.mark.parametrize("T,L,lam,behind", [(3, 5, 1e-2, ()), (2, 24, 1e-4, (7,)), (4, 1, 1e-3, ())])
def test_gn_step_matches_dense_oracle(T, L, lam, behind):
    lin = _lin(T, L, 5 + L, behind)
    out = pipeline.gn_step(lin, T=T, L=L, lam=lam)
    K = len(CORNERS)
    H, g, d = G.gn_step(_np(lin), T, L, K, lam)
    assert (out["info"].cpu().numpy() == 0).all()
    Dd, Ed = out["D"].cpu().numpy(), out["E"].cpu().numpy()
    for t in range(T):
        D, E = G.blocks(H[t], L)
        scale = np.abs(H[t]).max()
        np.testing.assert_allclose(Dd[t * L:(t + 1) * L], D, rtol=RTOL, atol=RTOL * scale)
        if L > 1:
            np.testing.assert_allclose(Ed[t * (L - 1):(t + 1) * (L - 1)], E, rtol=RTOL, atol=RTOL * scale)
    np.testing.assert_allclose(out["g"].cpu().numpy().reshape(T, -1), g, rtol=RTOL, atol=RTOL * np.abs(g).max())
    np.testing.assert_allclose(out["delta"].cpu().numpy().reshape(T, -1), d, rtol=1e-7,
                               atol=1e-9 * np.abs(d).max())


def test_gn_step_reports_singular_trajectories():
    """lambda = 0: the last frame's angular velocity has no factor, so its pivot block fails."""
    T, L = 2, 4
    out = pipeline.gn_step(_lin(T, L, 9), T=T, L=L, lam=0.0)
    assert (out["info"].cpu().numpy() == L).all()
    assert torch.isnan(out["delta"]).all()


def test_gn_step_without_block_outputs_is_bit_identical():
    """D, E, g NULL (GNPlan's default, the streaming tick's launch): the blocks stay on chip and
    delta / info are bit for bit those of the launch that also writes them."""
    T, L = 5, 24
    lin = _lin(T, L, 17, behind=(30,))
    ref = pipeline.gn_step(lin, T=T, L=L, lam=1e-3)
    plan = pipeline.GNPlan(lin, T=T, L=L, lam=1e-3)
    assert "D" not in plan.out and "g" not in plan.out
    plan.launch()
    assert torch.equal(plan.out["delta"], ref["delta"]) and torch.equal(plan.out["info"], ref["info"])


def test_gn_step_no_keypoints_null_projection_arrays():
    """n_kp = 0 with NULL r_proj / j_proj / status: only the dynamics and
    constant-velocity factors; against the dense oracle with an empty projection set."""
    from perseus_amd import _lib

    T, L, lam = 3, 6, 1e-2
    lin = _lin(T, L, 23)
    f = _np(lin)
    f["r_proj"], f["j_proj"], f["status"] = (np.zeros((0, 2)), np.zeros((0, 2, 6)), np.zeros(0, np.int32))
    H, g, d = G.gn_step(f, T, L, 0, lam)
    dev = lin["r_dyn"].device
    e = lambda *s: torch.empty(s, dtype=torch.float64, device=dev)  # noqa: E731
    out = {"D": e(T * L, 12, 12), "E": e(T * (L - 1), 12, 12), "g": e(T * L, 12), "delta": e(T * L, 12),
           "info": torch.empty(T, dtype=torch.int32, device=dev)}
    L_ = _lib.lib()
    ws = torch.empty(int(L_.pa_trajectory_gn_workspace(T, L)), dtype=torch.uint8, device=dev)
    p = _lib.ptr
    _lib.check(L_.pa_trajectory_gn_step(T, L, 0, None, None, None, p(lin["r_dyn"]), p(lin["j_dyn0"]),
                                        p(lin["j_dyn1"]), p(lin["j_dyn2"]), p(lin["j_dyn3"]), p(lin["r_cv"]),
                                        p(lin["j_cv0"]), p(lin["j_cv1"]), lam, p(out["D"]), p(out["E"]), p(out["g"]),
                                        p(out["delta"]), p(out["info"]), p(ws), ws.numel(), _lib.stream_of(dev)),
               "gn n_kp=0")
    torch.cuda.synchronize()
    assert (out["info"].cpu().numpy() == 0).all()
    Dd = out["D"].cpu().numpy()
    for t in range(T):
        D, _ = G.blocks(H[t], L)
        np.testing.assert_allclose(Dd[t * L:(t + 1) * L], D, rtol=RTOL, atol=RTOL * np.abs(H[t]).max())
    np.testing.assert_allclose(out["delta"].cpu().numpy().reshape(T, -1), d, rtol=1e-7, atol=1e-9 * np.abs(d).max())
