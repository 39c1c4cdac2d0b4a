"""CPU checks of the GN-step oracle (oracle/gn_ref.py): its normal equations equal a
least-squares solve of the stacked, damped factor rows, and H is block tridiagonal."""
import numpy as np

from oracle import gn_ref as G


def _factors(T, L, K, seed):
    rng = np.random.default_rng(seed)
    n, m = T * L * K, T * (L - 1)
    f = {"r_proj": rng.standard_normal((n, 2)), "j_proj": rng.standard_normal((n, 2, 6)),
         "status": (rng.random(n) < 0.1).astype(np.int32),
         "r_dyn": rng.standard_normal((m, 6)), "j_dyn0": rng.standard_normal((m, 6, 6)),
         "j_dyn1": rng.standard_normal((m, 6, 3)), "j_dyn2": rng.standard_normal((m, 6, 3)),
         "j_dyn3": rng.standard_normal((m, 6, 6)), "r_cv": rng.standard_normal((m, 3)),
         "j_cv0": -np.tile(np.eye(3), (m, 1, 1)), "j_cv1": np.tile(np.eye(3), (m, 1, 1))}
    return f


def test_step_is_damped_least_squares():
    T, L, K, lam = 2, 4, 8, 1e-3
    f = _factors(T, L, K, 0)
    H, g, d = G.gn_step(f, T, L, K, lam)
    for t, (A, r) in enumerate(G.stack(f, T, L, K)):
        Aa = np.concatenate([A, np.sqrt(lam) * np.eye(A.shape[1])])
        ra = np.concatenate([r, np.zeros(A.shape[1])])
        ls = np.linalg.lstsq(Aa, -ra, rcond=None)[0]
        np.testing.assert_allclose(d[t], ls, rtol=1e-8, atol=1e-10)
        # block tridiagonal: nothing beyond the first off-diagonal block
        for i in range(L):
            for j in range(L):
                if abs(i - j) > 1:
                    assert not H[t][i * 12:(i + 1) * 12, j * 12:(j + 1) * 12].any()


def test_undamped_last_angular_velocity_is_singular():
    """No factor touches the last frame's angular velocity: lambda = 0 has no solution."""
    f = _factors(1, 3, 8, 1)
    _, _, d = G.gn_step(f, 1, 3, 8, 0.0)
    assert np.isnan(d).all()
