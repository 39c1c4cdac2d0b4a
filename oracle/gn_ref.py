"""TEST INFRASTRUCTURE ONLY (tests/ and bench cpu legs): dense f64 restatement of one damped
Gauss-Newton / LM step per trajectory over the whitened factors of pa_trajectory_linearize
(include/perseus_amd.h pa_trajectory_gn_step).

Parity unpinned against the reference: perseus has no factor-graph optimizer of its own
(GTSAM's LM runs on the host, `pyproject.toml:21`), so this build defines the step and this
module states it densely: stack every whitened factor row of a trajectory into A (12 L columns,
frame block x_l = [pose tangent 6 | angular velocity 3 | velocity 3]), then
(A^T A + lambda I) delta = -A^T r.  Factor -> key mapping follows factors.py:
KeypointProjectionFactor (:182-275) on pose_l, PoseDynamicsFactor (:8-142) on
(pose_l, angvel_l, vel_l, pose_l+1), ConstantVelocityFactor (:145-171) on (vel_l, vel_l+1).
Jacobians here are (n, rows, cols) arrays (the row-major views pipeline.linearize_trajectories returns).
"""
from __future__ import annotations

import numpy as np

NV = 12


def stack(f: dict, T: int, L: int, K: int):
    """Per trajectory: (A, r) with A (rows, 12 L) and r (rows,); cheirality factors skipped."""
    out = []
    st = f.get("status")
    for t in range(T):
        rows_a, rows_r = [], []
        for l in range(L):
            fr = t * L + l
            for k in range(K):
                u = fr * K + k
                if st is not None and st[u] != 0:
                    continue
                a = np.zeros((2, NV * L))
                a[:, l * NV: l * NV + 6] = f["j_proj"][u]
                rows_a.append(a)
                rows_r.append(f["r_proj"][u])
            if l + 1 < L:
                u = t * (L - 1) + l
                a = np.zeros((6, NV * L))
                a[:, l * NV: l * NV + 6] = f["j_dyn0"][u]
                a[:, l * NV + 6: l * NV + 9] = f["j_dyn1"][u]
                a[:, l * NV + 9: l * NV + 12] = f["j_dyn2"][u]
                a[:, (l + 1) * NV: (l + 1) * NV + 6] = f["j_dyn3"][u]
                rows_a.append(a)
                rows_r.append(f["r_dyn"][u])
                c = np.zeros((3, NV * L))
                c[:, l * NV + 9: l * NV + 12] = f["j_cv0"][u]
                c[:, (l + 1) * NV + 9: (l + 1) * NV + 12] = f["j_cv1"][u]
                rows_a.append(c)
                rows_r.append(f["r_cv"][u])
        out.append((np.concatenate(rows_a, 0), np.concatenate(rows_r, 0)))
    return out


def gn_step(f: dict, T: int, L: int, K: int, lam: float):
    """Returns H (T, 12L, 12L) = A^T A, g (T, 12L) = A^T r, delta (T, 12L) (NaN where
    H + lam I is not positive definite)."""
    Hs, gs, ds = [], [], []
    for A, r in stack(f, T, L, K):
        H = A.T @ A
        g = A.T @ r
        M = H + lam * np.eye(H.shape[0])
        try:
            np.linalg.cholesky(M)
            d = np.linalg.solve(M, -g)
        except np.linalg.LinAlgError:
            d = np.full_like(g, np.nan)
        Hs.append(H)
        gs.append(g)
        ds.append(d)
    return np.stack(Hs), np.stack(gs), np.stack(ds)


def blocks(H: np.ndarray, L: int):
    """Diagonal (L, 12, 12) and super-diagonal (L-1, 12, 12) blocks of one trajectory's H."""
    D = np.stack([H[l * NV:(l + 1) * NV, l * NV:(l + 1) * NV] for l in range(L)])
    E = np.stack([H[l * NV:(l + 1) * NV, (l + 1) * NV:(l + 2) * NV] for l in range(L - 1)]) if L > 1 else None
    return D, E
