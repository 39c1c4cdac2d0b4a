"""Config 3: keypoint forward + per-frame factor linearize, fused on the GPU.

The reference chains these through the host: `KeypointCNN.forward` (models.py:34-40)
-> `.cpu()` -> kornia `denormalize_pixel_coordinates` (validate.py:144-153) -> one
GTSAM `KeypointProjectionFactor` per keypoint (factors.py:182-275) plus one
`PoseDynamicsFactor` (factors.py:8-142) and one `ConstantVelocityFactor`
(factors.py:145-171) per consecutive frame pair, each evaluated through a Python
callback.  Here the detector output never leaves HBM: `pa_trajectory_linearize`
reads it directly, denormalizes in-kernel and evaluates every factor of T
trajectories x L frames in ONE launch on the detector's stream.

Layout (all device, f64 unless noted):
  y        (T*L, 2K) f32   detector output, frame f = t*L + l
  poses    (T*L, 12)       body pose per frame (R row-major, t)
  vels     (T*L, 3)        linear velocity in `vel_frame`
  angvels  (T*L, 3)        body angular velocity
  corners  (K, 3)          keypoints in the body frame
Outputs (factor order: projection f*K + k; dynamics / const-vel t*(L-1) + l):
  proj: r (n,2), J (n,2,6), err (n,), status (n,) int32 (1 = cheirality)
  dyn:  r (m,6), J0 (m,6,6), J1 (m,6,3), J2 (m,6,3), J3 (m,6,6), err (m,)
  cv:   r (m,3), J0 (m,3,3), J1 (m,3,3), err (m,)
Jacobians are whitened (A = H / sigma) and residuals r / sigma when sigmas are given,
matching GTSAM's JacobianFactor (b = -r).
"""

from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib


def _f64(a, dev, shape=None):
    if a is None:
        return None
    t = a if isinstance(a, torch.Tensor) else torch.as_tensor(np.asarray(a, np.float64))
    t = t.to(device=dev, dtype=torch.float64).contiguous()
    if shape is not None:
        t = t.reshape(shape)
    return t


def _isig(sigmas, dim, dev):
    if sigmas is None:
        return None
    s = np.broadcast_to(np.asarray(sigmas, np.float64).reshape(-1), (dim,))
    return torch.as_tensor(1.0 / s, device=dev).contiguous()


def prepare_trajectories(y: torch.Tensor, poses, vels, angvels, corners, K, *, T: int, L: int, dt: float,
                         vel_frame: str = "world", camera_pose=None, H: int = 256, W: int = 256,
                         proj_sigmas=None, dyn_sigmas=None, cv_sigmas=None, jacobians: bool = True,
                         nvalid: torch.Tensor | None = None):
    """Stage inputs on the device and allocate outputs: returns (args, out).  `args`
    (a pa_traj_args) can be launched repeatedly with `launch(args, device)`; `out`
    holds the output tensors (Jacobians as (n, cols, rows) column-major buffers) and
    keeps every staged input alive.  nvalid (optional, int32 (T,) on the device, read at
    every launch): frames with a measurement, counted from the window's end; the projection
    factors of the others get status 2 and zero residual / Jacobian (the GN step skips them)."""
    if y.device.type != "cuda":
        raise RuntimeError("linearize_trajectories expects the detector output on the GPU (no CPU fallback)")
    if vel_frame not in ("world", "body"):
        raise AssertionError("vel_frame must be 'world' or 'body'.")  # factors.py:41
    dev = y.device
    F = T * L
    y = y.to(torch.float32).contiguous()
    if y.dim() != 2 or y.shape[0] != F or y.shape[1] % 2:
        raise ValueError(f"y must be (T*L, 2K) = ({F}, 2K), got {tuple(y.shape)}")
    nk = y.shape[1] // 2
    P = _f64(poses, dev, (F, 12))
    V = _f64(vels, dev, (F, 3))
    Wv = _f64(angvels, dev, (F, 3))
    Cn = _f64(corners, dev, (nk, 3))
    Kt = _f64(K, dev, (5,))
    Tc = _f64(camera_pose, dev, (12,))
    isp, isd, isc = _isig(proj_sigmas, 2, dev), _isig(dyn_sigmas, 6, dev), _isig(cv_sigmas, 3, dev)
    n, m = F * nk, T * max(L - 1, 0)

    def e(*shape, dtype=torch.float64):
        return torch.empty(shape, dtype=dtype, device=dev)

    out = {"r_proj": e(n, 2), "status": e(n, dtype=torch.int32), "err_proj": e(n) if isp is not None else None,
           "r_dyn": e(m, 6), "err_dyn": e(m) if isd is not None else None,
           "r_cv": e(m, 3), "err_cv": e(m) if isc is not None else None}
    for k, shp in _JAC.items():
        out[k] = e(*((n, m)[shp[0]],) + shp[1:]) if jacobians else None

    a = _lib.TrajArgs()
    a.T, a.L, a.n_kp, a.H, a.W = T, L, nk, H, W
    a.y, a.pose, a.vel, a.angvel, a.corners, a.K = (t.data_ptr() for t in (y, P, V, Wv, Cn, Kt))
    a.tcam = _lib.ptr(Tc)
    a.dt = float(dt)
    a.vel_frame = _lib.VEL_WORLD if vel_frame == "world" else _lib.VEL_BODY
    a.isig_proj, a.isig_dyn, a.isig_cv = _lib.ptr(isp), _lib.ptr(isd), _lib.ptr(isc)
    if nvalid is not None and (nvalid.device != dev or nvalid.dtype != torch.int32 or nvalid.numel() != T
                               or not nvalid.is_contiguous()):
        raise RuntimeError(f"nvalid must be a contiguous int32 ({T},) tensor on {dev}")
    a.nvalid = _lib.ptr(nvalid)
    for k in ("r_proj", "err_proj", "status", "r_dyn", "err_dyn", "r_cv", "err_cv", *_JAC):
        setattr(a, k, _lib.ptr(out[k]))
    out["_keep"] = (y, P, V, Wv, Cn, Kt, Tc, isp, isd, isc, nvalid)  # inputs stay alive until the stream drains
    return a, out


# column-major per factor: (0 = proj rows / 1 = dyn,cv rows, cols, rows)
_JAC = {"j_proj": (0, 6, 2), "j_dyn0": (1, 6, 6), "j_dyn1": (1, 3, 6), "j_dyn2": (1, 3, 6), "j_dyn3": (1, 6, 6),
        "j_cv0": (1, 3, 3), "j_cv1": (1, 3, 3)}


def launch(args, device) -> None:
    """One pa_trajectory_linearize launch on `device`'s current stream."""
    with torch.cuda.device(device):
        _lib.check(_lib.lib().pa_trajectory_linearize(C.byref(args), _lib.stream_of(device)),
                   "pa_trajectory_linearize")


def linearize_trajectories(y: torch.Tensor, poses, vels, angvels, corners, K, *, T: int, L: int, dt: float,
                           **kw) -> dict:
    """All factors of T trajectories x L frames from the detector output `y` (device).
    Keywords as `prepare_trajectories`; Jacobians are returned as (n, rows, cols) views."""
    a, out = prepare_trajectories(y, poses, vels, angvels, corners, K, T=T, L=L, dt=dt, **kw)
    launch(a, y.device)
    for k in _JAC:
        if out[k] is not None:
            out[k] = out[k].transpose(1, 2)
    return out


def detect_and_linearize(model, x: torch.Tensor, poses, vels, angvels, corners, K, *, T: int, L: int, dt: float,
                         **kw) -> dict:
    """Config 3 end to end: `model(x)` then `linearize_trajectories` on the same stream;
    the keypoints stay in HBM between the two launches."""
    y = model(x)
    out = linearize_trajectories(y, poses, vels, angvels, corners, K, T=T, L=L, dt=dt, H=model.H, W=model.W, **kw)
    out["y"] = y
    return out


class GNPlan:
    """One damped Gauss-Newton / LM step per trajectory (SURVEY.md 8f.4,
    pa_trajectory_gn_step) over `lin` = the outputs of prepare_trajectories /
    linearize_trajectories run with whitening sigmas and Jacobians, with every output and
    the workspace allocated once, so `launch` can be captured in a HIP graph and replayed
    (the streaming pose stage).  out: delta (T*L,12), info (T,) int32 (0 = solved), and
    with blocks=True also the normal-matrix blocks D (T*L,12,12), E (T*(L-1),12,12) and
    g (T*L,12) (blocks=False: they stay on chip, the launch writes delta and info only).
    Variable block per frame: [pose (6) | angvel (3) | vel (3)]."""

    def __init__(self, lin: dict, *, T: int, L: int, lam: float = 0.0, blocks: bool = False):
        if lin.get("j_proj") is None:
            raise RuntimeError("gn_step needs the Jacobians (linearize with jacobians=True)")
        dev = lin["r_proj"].device
        self.T, self.L, self.lam, self.lin = T, L, float(lam), lin
        self.n_kp = lin["r_proj"].shape[0] // (T * L) if T * L else 0
        m = T * max(L - 1, 0)
        self.m = m

        def e(*shape, dtype=torch.float64):
            return torch.empty(shape, dtype=dtype, device=dev)

        self.out = {"delta": e(T * L, 12), "info": e(T, dtype=torch.int32)}
        if blocks:
            self.out.update(D=e(T * L, 12, 12), E=e(max(m, 1), 12, 12), g=e(T * L, 12))
        L_ = _lib.lib()
        self.ws = torch.empty(max(int(L_.pa_trajectory_gn_workspace(T, L)), 8), dtype=torch.uint8, device=dev)
        self.dev = dev

    def launch(self) -> None:
        """One pa_trajectory_gn_step on the device's current stream."""
        lin, out, p = self.lin, self.out, _lib.ptr
        with torch.cuda.device(self.dev):
            _lib.check(_lib.lib().pa_trajectory_gn_step(
                self.T, self.L, self.n_kp, p(lin["r_proj"]), p(lin["j_proj"]), p(lin.get("status")), p(lin["r_dyn"]),
                p(lin["j_dyn0"]), p(lin["j_dyn1"]), p(lin["j_dyn2"]), p(lin["j_dyn3"]), p(lin["r_cv"]),
                p(lin["j_cv0"]), p(lin["j_cv1"]), self.lam, p(out.get("D")), p(out.get("E")), p(out.get("g")),
                p(out["delta"]),
                p(out["info"]), p(self.ws), self.ws.numel(), _lib.stream_of(self.dev)), "pa_trajectory_gn_step")


def gn_step(lin: dict, *, T: int, L: int, lam: float = 0.0) -> dict:
    """One damped Gauss-Newton / LM step per trajectory on the device (SURVEY.md 8f.4,
    pa_trajectory_gn_step) from `linearize_trajectories(...)` run with whitening sigmas and
    Jacobians.  Returns D (T*L,12,12), E (T*(L-1),12,12), g (T*L,12), delta (T*L,12) and
    info (T,) int32 (0 = solved).  Variable block per frame: [pose (6) | angvel (3) | vel (3)]."""
    plan = GNPlan(lin, T=T, L=L, lam=lam, blocks=True)
    plan.launch()
    out = dict(plan.out)
    out["E"] = out["E"][:plan.m]
    out["_ws"] = plan.ws
    return out


def window_advance(y_new: torch.Tensor, win: dict, *, dt: float, vel_frame: str = "world",
                   nvalid: torch.Tensor | None = None) -> None:
    """pa_window_advance on the device's current stream: every trajectory's window
    (win: y (T, L, 2K) f32, pose (T, L, 12), angvel / vel (T, L, 3) f64) moves one frame,
    y_new (T, 2K) becomes its last frame, whose pose is predicted by the
    PoseDynamicsFactor model (factors.py:100-105).  nvalid (optional, int32 (T,)): the
    window's count of real frames, += 1 up to L (pa_window_advance_n)."""
    T, L, ny = win["y"].shape
    dev = win["y"].device
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().pa_window_advance_n(
            T, L, ny // 2, y_new.data_ptr(), win["y"].data_ptr(), win["pose"].data_ptr(), win["angvel"].data_ptr(),
            win["vel"].data_ptr(), _lib.ptr(nvalid), float(dt),
            _lib.VEL_WORLD if vel_frame == "world" else _lib.VEL_BODY, _lib.stream_of(dev)), "pa_window_advance")


TICK_MAX_L = 24  # pa_window_pose_tick: L <= 24 (the cyclic-reduction GN step), T <= the CU count


def window_pose_tick(args, y_new: torch.Tensor, *, lam: float, delta: torch.Tensor, info: torch.Tensor,
                     newest: torch.Tensor | None = None) -> None:
    """pa_window_pose_tick on the device's current stream: window_advance(y_new) ->
    pa_trajectory_linearize(args) -> pa_trajectory_gn_step (delta, info) ->
    window_retract(newest) in two launches, bit for bit that sequence.  `args` comes from
    prepare_trajectories over the window arrays (with nvalid, whitening sigmas and Jacobians)."""
    dev = y_new.device
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().pa_window_pose_tick(C.byref(args), y_new.data_ptr(), float(lam), delta.data_ptr(),
                                                  info.data_ptr(), _lib.ptr(newest), _lib.stream_of(dev)),
                   "pa_window_pose_tick")


def window_pose_tick_workspace(T: int, L: int, device) -> torch.Tensor:
    """The reduced system pa_window_pose_tick_pre leaves for _post (bytes as a u8 tensor)."""
    n = int(_lib.lib().pa_window_pose_tick_workspace(int(T), int(L)))
    return torch.empty(max(n, 1), dtype=torch.uint8, device=device)


def window_pose_tick_pre(args, ws: torch.Tensor, *, lam: float) -> None:
    """pa_window_pose_tick_pre on the device's current stream: the window advances without the
    new keypoints, every factor but the newest frame's projections, the GN system reduced to
    the newest frame (into ws)."""
    dev = ws.device
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().pa_window_pose_tick_pre(C.byref(args), float(lam), ws.data_ptr(), ws.numel(),
                                                      _lib.stream_of(dev)), "pa_window_pose_tick_pre")


def window_pose_tick_post(args, y_new: torch.Tensor, ws: torch.Tensor, *, delta: torch.Tensor, info: torch.Tensor,
                          newest: torch.Tensor | None = None) -> None:
    """pa_window_pose_tick_post on the device's current stream: y_new lands, the newest frame's
    projection factors join the reduced system, solve (delta, info), retract (newest).  info /
    newest: tensors or device addresses (e.g. of mapped pinned host memory)."""
    dev = y_new.device
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().pa_window_pose_tick_post(C.byref(args), y_new.data_ptr(), ws.data_ptr(), ws.numel(),
                                                       delta.data_ptr(), _lib.ptr(info), _lib.ptr(newest),
                                                       _lib.stream_of(dev)), "pa_window_pose_tick_post")


def window_retract(win: dict, delta: torch.Tensor, info: torch.Tensor | None = None,
                   newest: torch.Tensor | None = None) -> None:
    """pa_window_retract on the device's current stream: pose <- pose Exp(delta[:6]),
    angvel += delta[6:9], vel += delta[9:12]; trajectories with info != 0 unchanged.
    newest (optional, contiguous f64 (T, 12) on the device): each trajectory's last-frame
    pose after the update (pa_window_retract_newest)."""
    T, L = win["pose"].shape[:2]
    dev = win["pose"].device
    if newest is not None and (newest.device != dev or newest.dtype != torch.float64 or newest.numel() != T * 12
                               or not newest.is_contiguous()):
        raise RuntimeError(f"newest must be a contiguous float64 ({T}, 12) tensor on {dev}")
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().pa_window_retract_newest(T, L, delta.data_ptr(), _lib.ptr(info), win["pose"].data_ptr(),
                                                       win["angvel"].data_ptr(), win["vel"].data_ptr(),
                                                       _lib.ptr(newest), _lib.stream_of(dev)),
                   "pa_window_retract")
