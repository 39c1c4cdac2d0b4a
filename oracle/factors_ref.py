"""ORACLE (test infrastructure only) — f64 CPU restatement of the smoother factors.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this.

Restates `perseus/smoother/factors.py`:
  * PoseDynamicsFactor.error_func     `factors.py:54-142` (Jacobian branch :86-130,
    plain branch :131-140)
  * ConstantVelocityFactor.error_func `factors.py:160-171`
  * KeypointProjectionFactor.error_func `factors.py:216-275`
The geometry those call lives in GTSAM (third-party C++, pinned `gtsam>=4.2` at
`pyproject.toml:21`, NOT installed here).  Restated from GTSAM 4.2's published
algorithms: Rot3 Expmap/Logmap (SO3 ExpmapFunctor/DexpFunctor, Logmap incl. the
trace-near--1 branch), SO3 LogmapDerivative, Pose3 Expmap/Logmap (Agrawal06iros
eq. 14), Pose3 ExpmapDerivative/LogmapDerivative with ComputeQforExpmapDerivative
(Barfoot14tro eq. 102, right-Jacobian sign convention, near-zero series below 1e-5),
Pose3 AdjointMap, compose/between/transformFrom/transformTo Jacobians, and
PinholeCamera<Cal3_S2>::project with its point Jacobian and cheirality check.
Tangent order is GTSAM's [omega; v]; perturbations are on the right.

Pinning: `tests/test_dynamics_factor.py:57-71` is the reference's intended oracle
(pypose, torch f64 autodiff; atol 1e-6).  `autodiff_dynamics` below restates it in
plain torch (pypose is absent) and oracle/gen_golden.py + tests/test_oracle_factors.py
check this closed form against it on the test's own seeded problem
(`test_dynamics_factor.py:11-32`).  GTSAM itself cannot run here, so parity beyond that
formulation is unpinned; KeypointProjectionFactor has no reference test at all and is
pinned by the same autodiff method plus the datagen projection convention
(`data_generation/data_utils.py:17-66`).

Pose encoding used everywhere in this repo: 12 f64 = R row-major (9) then t (3).
"""

from __future__ import annotations

import math

import numpy as np

EPS = np.finfo(np.float64).eps


def skew(w):
    return np.array([[0.0, -w[2], w[1]], [w[2], 0.0, -w[0]], [-w[1], w[0], 0.0]])


def rot_exp(w):
    th2 = float(w @ w)
    W = skew(w)
    if th2 <= EPS:
        return np.eye(3) + W
    th = math.sqrt(th2)
    return np.eye(3) + (math.sin(th) / th) * W + ((1 - math.cos(th)) / th2) * (W @ W)


def rot_log(R):
    R11, R12, R13 = R[0]
    R21, R22, R23 = R[1]
    R31, R32, R33 = R[2]
    tr = R11 + R22 + R33
    if tr + 1.0 < 1e-3:
        if R33 > R22 and R33 > R11:
            Wv = R21 - R12
            Q1 = 2.0 + 2.0 * R33
            Q2 = R31 + R13
            Q3 = R23 + R32
            vec = (Q2, Q3, Q1)
        elif R22 > R11:
            Wv = R13 - R31
            Q1 = 2.0 + 2.0 * R22
            Q2 = R23 + R32
            Q3 = R12 + R21
            vec = (Q3, Q1, Q2)
        else:
            Wv = R32 - R23
            Q1 = 2.0 + 2.0 * R11
            Q2 = R12 + R21
            Q3 = R31 + R13
            vec = (Q1, Q2, Q3)
        r = math.sqrt(Q1)
        norm = math.sqrt(Q1 * Q1 + Q2 * Q2 + Q3 * Q3 + Wv * Wv)
        sgn = -1.0 if Wv < 0 else 1.0
        mag = math.pi - (2 * sgn * Wv) / norm
        scale = 0.5 / r * mag
        return sgn * scale * np.array(vec)
    tr3 = tr - 3.0
    if tr3 < -1e-6:
        th = math.acos((tr - 1.0) / 2.0)
        mag = th / (2.0 * math.sin(th))
    else:
        mag = 0.5 - tr3 / 12.0 + tr3 * tr3 / 60.0
    return mag * np.array([R32 - R23, R13 - R31, R21 - R12])


def rot_dexp(w):
    """SO3 ExpmapDerivative = right Jacobian J_r(w)."""
    th2 = float(w @ w)
    W = skew(w)
    if th2 <= EPS:
        return np.eye(3) - 0.5 * W
    th = math.sqrt(th2)
    return np.eye(3) - ((1 - math.cos(th)) / th2) * W + ((th - math.sin(th)) / (th2 * th)) * (W @ W)


def rot_dlog(w):
    """SO3 LogmapDerivative = J_r(w)^-1."""
    th2 = float(w @ w)
    if th2 <= EPS:
        return np.eye(3)
    th = math.sqrt(th2)
    W = skew(w)
    return np.eye(3) + 0.5 * W + (1 / th2 - (1 + math.cos(th)) / (2 * th * math.sin(th))) * (W @ W)


def pose(R, t):
    return (np.asarray(R, dtype=np.float64), np.asarray(t, dtype=np.float64))


def pose_exp(xi):
    w, v = xi[:3], xi[3:]
    R = rot_exp(w)
    th2 = float(w @ w)
    if th2 > EPS:
        wxv = np.cross(w, v)
        t = (wxv - R @ wxv + w * (w @ v)) / th2
    else:
        t = v.copy()
    return R, t


def pose_log(T):
    R, t = T
    w = rot_log(R)
    th = float(np.linalg.norm(w))
    if th < 1e-10:
        return np.concatenate([w, t])
    W = skew(w / th)
    tan_h = math.tan(0.5 * th)
    WT = W @ t
    u = t - (0.5 * th) * WT + (1 - th / (2.0 * tan_h)) * (W @ WT)
    return np.concatenate([w, u])


def compute_q(xi, thresh=1e-5):
    w, v = xi[:3], xi[3:]
    V, W = skew(v), skew(w)
    WVW = W @ V @ W
    phi = float(np.linalg.norm(w))
    if abs(phi) > thresh:
        s, c = math.sin(phi), math.cos(phi)
        p2 = phi * phi
        p3, p4, p5 = p2 * phi, p2 * p2, p2 * p2 * phi
        return (-0.5 * V + (phi - s) / p3 * (W @ V + V @ W - WVW)
                + (1 - p2 / 2 - c) / p4 * (W @ W @ V + V @ W @ W - 3 * WVW)
                - 0.5 * ((1 - p2 / 2 - c) / p4 - 3 * (phi - s - p3 / 6.0) / p5) * (WVW @ W + W @ WVW))
    return (-0.5 * V + 1.0 / 6.0 * (W @ V + V @ W - WVW)
            - 1.0 / 24.0 * (W @ W @ V + V @ W @ W - 3 * WVW)
            + 1.0 / 120.0 * (WVW @ W + W @ WVW))


def pose_dexp(xi):
    Jw = rot_dexp(xi[:3])
    Q = compute_q(xi)
    J = np.zeros((6, 6))
    J[:3, :3] = Jw
    J[3:, 3:] = Jw
    J[3:, :3] = Q
    return J


def pose_dlog(T):
    xi = pose_log(T)
    Jw = rot_dlog(xi[:3])
    Q = compute_q(xi)
    J = np.zeros((6, 6))
    J[:3, :3] = Jw
    J[3:, 3:] = Jw
    J[3:, :3] = -Jw @ Q @ Jw
    return J


def adjoint(T):
    R, t = T
    A = np.zeros((6, 6))
    A[:3, :3] = R
    A[3:, 3:] = R
    A[3:, :3] = skew(t) @ R
    return A


def compose(T1, T2):
    return T1[0] @ T2[0], T1[0] @ T2[1] + T1[1]


def inverse(T):
    return T[0].T, -T[0].T @ T[1]


def between(T1, T2):
    return compose(inverse(T1), T2)


# -------------------------------------------------------------------------------------
# factors
# -------------------------------------------------------------------------------------
def dynamics(T1, w, v, T2, dt, vel_frame="world", jac=True):
    """PoseDynamicsFactor.error_func (`factors.py:54-142`).  Returns r (6,) and
    [H0 6x6, H1 6x3, H2 6x3, H3 6x6] (or None)."""
    R1 = T1[0]
    w = np.asarray(w, dtype=np.float64)
    v = np.asarray(v, dtype=np.float64)
    if vel_frame == "world":
        vb = R1.T @ v                           # transformTo with t = 0 (:100-101)
        dvb_dpose = np.hstack([skew(vb), -np.eye(3)])
        dvb_dvel = R1.T
    else:
        vb = v
    xi = np.concatenate([dt * w, dt * vb])
    inc = pose_exp(xi)                          # Expmap (:104)
    pred = compose(T1, inc)                     # compose (:105)
    rel = between(pred, T2)                     # between (:108)
    err = pose_log(rel)                         # Logmap (:109)
    if not jac:
        return err, None
    Jexp = pose_dexp(xi)
    dpred_dx0 = adjoint(inverse(inc))
    drel_dpred = -adjoint(inverse(rel))
    dlog = pose_dlog(rel)                       # LogmapDerivative (:112)
    H0 = dlog @ drel_dpred @ dpred_dx0          # :114
    dtw = dt * dlog @ drel_dpred @ Jexp         # :117 (dpred_dtwist = I)
    H1 = dtw[:, :3].copy()
    if vel_frame == "world":
        H0[:, :3] += dtw[:, 3:] @ dvb_dpose[:, :3]  # :122
        H2 = dtw[:, 3:] @ dvb_dvel                  # :125
    else:
        H2 = dtw[:, 3:].copy()                      # :128
    H3 = dlog.copy()                                # :130 (drel_dpose2 = I)
    return err, [H0, H1, H2, H3]


def const_vel(v1, v2):
    """ConstantVelocityFactor.error_func (`factors.py:160-171`)."""
    return np.asarray(v2, np.float64) - np.asarray(v1, np.float64), [-np.eye(3), np.eye(3)]


def projection(Tb, p_b, z, K, Tc=None):
    """KeypointProjectionFactor.error_func (`factors.py:216-275`).

    K = (fx, fy, s, u0, v0) (gtsam.Cal3_S2 order).  Returns (r (2,), H0 (2,6), status,
    pixel (2,)); status 1 = GTSAM CheiralityException (depth <= 0 in the camera)."""
    if Tc is None:
        Tc = (np.eye(3), np.zeros(3))
    Rb, tb = Tb
    p_b = np.asarray(p_b, np.float64)
    pw = Rb @ p_b + tb                                  # transformFrom (:257)
    dpc_dpose = np.hstack([Rb @ skew(-p_b), Rb])
    Rc, tc = Tc
    pc = Rc.T @ (pw - tc)                               # camera.project (:260-261)
    if pc[2] <= 0:
        return np.full(2, np.nan), np.full((2, 6), np.nan), 1, np.full(2, np.nan)
    x, y = pc[0] / pc[2], pc[1] / pc[2]
    fx, fy, s, u0, v0 = K
    pix = np.array([fx * x + s * y + u0, fy * y + v0])
    Dcal = np.array([[fx, s], [0.0, fy]])
    Dpn = (1.0 / pc[2]) * np.array([[1.0, 0.0, -x], [0.0, 1.0, -y]])
    dproj_dpoint = Dcal @ Dpn @ Rc.T
    H0 = dproj_dpoint @ dpc_dpose                       # :264
    return pix - np.asarray(z, np.float64), H0, 0, pix


# -------------------------------------------------------------------------------------
# torch f64 autodiff restatement of tests/test_dynamics_factor.py:53-71 (pypose absent)
# -------------------------------------------------------------------------------------
def _torch_helpers():
    import torch

    def hat(w):
        z = torch.zeros((), dtype=w.dtype)
        return torch.stack([torch.stack([z, -w[2], w[1]]), torch.stack([w[2], z, -w[0]]),
                            torch.stack([-w[1], w[0], z])])

    def coeffs(th2):
        small = th2 < 1e-8
        safe = torch.where(small, torch.ones_like(th2), th2)
        th = torch.sqrt(safe)
        A = torch.where(small, 1 - th2 / 6 + th2 * th2 / 120, torch.sin(th) / th)
        B = torch.where(small, 0.5 - th2 / 24 + th2 * th2 / 720, (1 - torch.cos(th)) / safe)
        C = torch.where(small, 1.0 / 6 - th2 / 120 + th2 * th2 / 5040, (th - torch.sin(th)) / (safe * th))
        return A, B, C

    def se3_exp(tau):
        """pypose se3 [rho; phi] -> 4x4."""
        rho, phi = tau[:3], tau[3:]
        W = hat(phi)
        A, B, C = coeffs(phi @ phi)
        I = torch.eye(3, dtype=tau.dtype)
        R = I + A * W + B * (W @ W)
        Jl = I + B * W + C * (W @ W)
        T = torch.eye(4, dtype=tau.dtype)
        T = torch.cat([torch.cat([R, (Jl @ rho)[:, None]], 1), T[3:]], 0)
        return T

    def se3_log(T):
        R, t = T[:3, :3], T[:3, 3]
        c = ((R[0, 0] + R[1, 1] + R[2, 2]) - 1) / 2
        th = torch.acos(torch.clamp(c, -1.0, 1.0))
        vee = torch.stack([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
        phi = th / (2 * torch.sin(th)) * vee
        W = hat(phi)
        th2 = phi @ phi
        I = torch.eye(3, dtype=T.dtype)
        Jinv = I - 0.5 * W + (1 / th2 - (1 + torch.cos(th)) / (2 * th * torch.sin(th))) * (W @ W)
        return torch.cat([Jinv @ t, phi])

    def inv(T):
        R, t = T[:3, :3], T[:3, 3]
        out = torch.eye(4, dtype=T.dtype)
        return torch.cat([torch.cat([R.T, (-R.T @ t)[:, None]], 1), out[3:]], 0)

    def flip(x):
        return torch.cat([x[3:], x[:3]])

    return torch, se3_exp, se3_log, inv, flip


def autodiff_dynamics(T1, w, v, T2, dt, vel_frame="world"):
    """`pypose_error` (`tests/test_dynamics_factor.py:57-71`) + `jacrev` over the zero
    right-perturbations (`:141-143`), in plain torch f64."""
    torch, exp, log, inv, flip = _torch_helpers()

    def mat(T):
        M = np.eye(4)
        M[:3, :3], M[:3, 3] = T
        return torch.tensor(M, dtype=torch.float64)

    x0, x1 = mat(T1), mat(T2)
    w0 = torch.tensor(np.asarray(w, np.float64))
    v0 = torch.tensor(np.asarray(v, np.float64))

    def err(dx0, dw0, dv0, dx1):
        x0p = x0 @ exp(flip(dx0))
        v0p = v0 + dv0
        w0p = w0 + dw0
        x1p = x1 @ exp(flip(dx1))
        if vel_frame == "world":
            v0p = x0p[:3, :3].T @ v0p
        pred = x0p @ exp(dt * torch.cat([v0p, w0p]))
        rel = inv(pred) @ x1p
        return flip(log(rel))

    z6 = torch.zeros(6, dtype=torch.float64)
    z3 = torch.zeros(3, dtype=torch.float64)
    e = err(z6, z3, z3, z6)
    J = torch.func.jacrev(err, argnums=(0, 1, 2, 3))(z6, z3, z3, z6)
    return e.numpy(), [j.numpy() for j in J]


def autodiff_projection(Tb, p_b, z, K, Tc=None):
    """Right-perturbation autodiff of the projection residual (no reference test exists;
    same method as the dynamics test)."""
    torch, exp, log, inv, flip = _torch_helpers()
    if Tc is None:
        Tc = (np.eye(3), np.zeros(3))
    M = np.eye(4)
    M[:3, :3], M[:3, 3] = Tb
    xb = torch.tensor(M, dtype=torch.float64)
    Rc = torch.tensor(Tc[0], dtype=torch.float64)
    tc = torch.tensor(Tc[1], dtype=torch.float64)
    pb = torch.tensor(np.asarray(p_b, np.float64))
    zz = torch.tensor(np.asarray(z, np.float64))
    fx, fy, s, u0, v0 = [float(k) for k in K]

    def err(dx):
        T = xb @ exp(flip(dx))
        pw = T[:3, :3] @ pb + T[:3, 3]
        pc = Rc.T @ (pw - tc)
        x, y = pc[0] / pc[2], pc[1] / pc[2]
        return torch.stack([fx * x + s * y + u0, fy * y + v0]) - zz

    z6 = torch.zeros(6, dtype=torch.float64)
    return err(z6).numpy(), torch.func.jacrev(err)(z6).numpy()


# -------------------------------------------------------------------------------------
# batched drivers (SoA arrays in the repo's pose encoding), used by tests and bench
# -------------------------------------------------------------------------------------
def unpack(p12):
    p12 = np.asarray(p12, np.float64)
    return p12[:9].reshape(3, 3), p12[9:12].copy()


def pack(T):
    return np.concatenate([np.asarray(T[0]).reshape(-1), np.asarray(T[1]).reshape(-1)])


def dynamics_batch(T1, w, v, T2, dt, vel_frame="world"):
    n = T1.shape[0]
    r = np.zeros((n, 6))
    J0, J1, J2, J3 = np.zeros((n, 6, 6)), np.zeros((n, 6, 3)), np.zeros((n, 6, 3)), np.zeros((n, 6, 6))
    for i in range(n):
        r[i], H = dynamics(unpack(T1[i]), w[i], v[i], unpack(T2[i]), dt, vel_frame)
        J0[i], J1[i], J2[i], J3[i] = H
    return r, J0, J1, J2, J3


def projection_batch(Tb, p_b, z, K, Tc=None):
    n = Tb.shape[0]
    r = np.zeros((n, 2))
    J = np.zeros((n, 2, 6))
    st = np.zeros(n, np.int32)
    for i in range(n):
        r[i], J[i], st[i], _ = projection(unpack(Tb[i]), p_b[i], z[i], K,
                                          None if Tc is None else unpack(Tc))
    return r, J, st


# -------------------------------------------------------------------------------------
# fixed-lag window of the config-4 streaming pose stage (include/perseus_amd.h
# pa_window_advance / pa_window_retract); the reference has no smoother loop of its own
# (scripts/streaming.py:121-155 stops at pixels), so these restate the build's definition
# with the reference's dynamics model (factors.py:100-105) and GTSAM's Pose3 retract
# (Expmap chart).  Parity of these two is therefore against the build's spec, not the
# reference.
# -------------------------------------------------------------------------------------
def window_advance(win: dict, y_new, dt, vel_frame="world") -> dict:
    """win: y (T, L, 2K), pose (T, L, 12), angvel / vel (T, L, 3); returns the advanced
    copy: frames shift one towards l = 0, y_new (T, 2K) appended, the new pose =
    pose[L-2] Exp(dt [w; v_b]) with v_b = R^T v (world) or v (body), v = vel[L-2] carried.
    w is the angular velocity of the window's second-to-last frame BEFORE the shift (the
    newest one a PoseDynamicsFactor constrains: the last frame's angular velocity enters no
    factor, so its value holds no information) and becomes the angular velocity of both
    new last frames (L >= 3; L = 2 carries frame 1's)."""
    out = {k: np.array(v, copy=True) for k, v in win.items()}
    for k in out:
        out[k][:, :-1] = win[k][:, 1:]
    out["y"][:, -1] = y_new
    T, L = out["pose"].shape[:2]
    for t in range(T):
        T1 = unpack(out["pose"][t, L - 2])
        w = np.array(win["angvel"][t, L - 2] if L >= 3 else out["angvel"][t, L - 2], copy=True)
        v = out["vel"][t, L - 2]
        vb = T1[0].T @ v if vel_frame == "world" else v
        out["pose"][t, L - 1] = pack(compose(T1, pose_exp(np.concatenate([dt * w, dt * vb]))))
        out["angvel"][t, L - 2] = w
        out["angvel"][t, L - 1] = w
        out["vel"][t, L - 1] = v
    return out


def window_retract(win: dict, delta, info=None) -> dict:
    """pose <- pose Exp(delta[:6]), angvel += delta[6:9], vel += delta[9:12] per frame;
    delta (T*L, 12); trajectories with info != 0 unchanged."""
    out = {k: np.array(v, copy=True) for k, v in win.items()}
    T, L = out["pose"].shape[:2]
    d = np.asarray(delta).reshape(T, L, 12)
    for t in range(T):
        if info is not None and info[t] != 0:
            continue
        for l in range(L):
            out["pose"][t, l] = pack(compose(unpack(out["pose"][t, l]), pose_exp(d[t, l, :6])))
            out["angvel"][t, l] = out["angvel"][t, l] + d[t, l, 6:9]
            out["vel"][t, l] = out["vel"][t, l] + d[t, l, 9:12]
    return out
