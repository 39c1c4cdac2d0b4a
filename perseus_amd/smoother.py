"""Smoother factors on the GPU: drop-in classes for `perseus/smoother/factors.py` plus
the batched structure-of-arrays entry points that are the fast path.

Reference surface mirrored (GTSAM CustomFactor callbacks, `factors.py:8-275`):
  * `PoseDynamicsFactor(pose1, ang_vel1, vel1, pose2, noise_model, dt, vel_frame="world")`
  * `ConstantVelocityFactor(vel1, vel2, noise_model)`
  * `KeypointProjectionFactor(body_pose, noise_model, camera_intrinsics,
     keypoint_measurement, point_body_frame, camera_pose=None)` (sets `.pixel`)
  each with `keys()`, `error_func(this, v, H=None)` (H entries overwritten with f64
  arrays of shape (dim r, dim key), exactly like the reference), `unwhitenedError(v)`,
  `error(v)` = 0.5 ||r / sigma||^2 and `linearize(v)` -> ([A_i], b) with
  A_i = H_i / sigma, b = -r / sigma (GTSAM NoiseModelFactor semantics).

All arithmetic runs in the f64 HIP kernels of libperseus_amd.so; a single-factor call
is a batch of one (correct, not fast); use `linearize_*` for batches.  `Values`,
`Pose3`, `Cal3_S2` and `noiseModel` below are minimal containers standing in for
gtsam's (absent here); real gtsam objects work too (duck typing on
`atPose3/atVector`, `.matrix()`, `.fx()...`, `.sigmas()`).  Errors follow the
reference: vel_frame is asserted, a point behind the camera raises
`CheiralityException` (GTSAM's exception from `camera.project`).
"""

from __future__ import annotations

from typing import List, Optional

import numpy as np
import torch

from . import _lib


class CheiralityException(RuntimeError):
    pass


# ----------------------------------------------------------------- containers
class Pose3:
    """Rigid transform container (R, t) with gtsam.Pose3's accessors used here."""

    def __init__(self, R=None, t=None):
        if R is not None and np.asarray(R).shape == (4, 4):
            M = np.asarray(R, np.float64)
            R, t = M[:3, :3], M[:3, 3]
        self._R = np.eye(3) if R is None else np.array(R, np.float64).reshape(3, 3)
        self._t = np.zeros(3) if t is None else np.array(t, np.float64).reshape(3)

    def rotation(self):
        return self._R.copy()

    def translation(self):
        return self._t.copy()

    def matrix(self):
        M = np.eye(4)
        M[:3, :3], M[:3, 3] = self._R, self._t
        return M


class Cal3_S2:
    """gtsam.Cal3_S2(fx, fy, s, u0, v0)."""

    def __init__(self, fx=1.0, fy=1.0, s=0.0, u0=0.0, v0=0.0):
        self._k = np.array([fx, fy, s, u0, v0], np.float64)

    def fx(self):
        return self._k[0]

    def fy(self):
        return self._k[1]

    def skew(self):
        return self._k[2]

    def px(self):
        return self._k[3]

    def py(self):
        return self._k[4]


class _Diagonal:
    def __init__(self, sigmas):
        self._s = np.asarray(sigmas, np.float64).reshape(-1)

    @classmethod
    def Sigmas(cls, sigmas):
        return cls(sigmas)

    def sigmas(self):
        return self._s.copy()


class _Isotropic(_Diagonal):
    @classmethod
    def Sigma(cls, dim, sigma):
        return cls(np.full(dim, float(sigma)))


class noiseModel:  # noqa: N801  (gtsam.noiseModel namespace)
    Diagonal = _Diagonal
    Isotropic = _Isotropic


class Values:
    """gtsam.Values subset: insert / atPose3 / atVector / exists."""

    def __init__(self):
        self._d = {}

    def insert(self, key, value):
        if key in self._d:
            raise KeyError(f"key {key} already exists")
        self._d[key] = value

    def update(self, key, value):
        self._d[key] = value

    def exists(self, key):
        return key in self._d

    def atPose3(self, key):
        return self._d[key]

    def atVector(self, key):
        return np.asarray(self._d[key], np.float64)


def _pose12(p) -> np.ndarray:
    M = np.asarray(p.matrix(), np.float64)
    return np.concatenate([M[:3, :3].reshape(-1), M[:3, 3]])


def _cal5(K) -> np.ndarray:
    if isinstance(K, Cal3_S2):
        return K._k.copy()
    return np.array([K.fx(), K.fy(), K.skew(), K.px(), K.py()], np.float64)


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("perseus_amd smoother kernels need a ROCm GPU (no CPU fallback)")
    return torch.device("cuda", torch.cuda.current_device())


def _dev(a, device) -> torch.Tensor:
    if isinstance(a, torch.Tensor):
        return a.to(device=device, dtype=torch.float64).contiguous()
    return torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64), device=device)


def _isig(noise, dim, device):
    if noise is None:
        return None
    s = noise.sigmas() if hasattr(noise, "sigmas") else noise
    s = np.asarray(s, np.float64).reshape(-1)
    if s.size != dim:
        raise ValueError(f"noise model dimension {s.size} != factor dimension {dim}")
    return torch.as_tensor(1.0 / s, device=device)


# ---------------------------------------------------------- batched fast path
def linearize_dynamics(T1, w, v, T2, dt: float, vel_frame: str = "world", inv_sigma=None, jacobians=True):
    """Batched PoseDynamicsFactor (factors.py:54-142) on the GPU.

    T1, T2 (n,12) poses; w, v (n,3).  Returns dict of device tensors r (n,6), J0 (n,6,6),
    J1 (n,6,3), J2 (n,6,3), J3 (n,6,6) (row-major views of the column-major buffers)
    and err (n,) when inv_sigma is given (whitened outputs)."""
    assert vel_frame in ["world", "body"], "vel_frame must be 'world' or 'body'."
    dev = _device()
    T1, w, v, T2 = (_dev(a, dev) for a in (T1, w, v, T2))
    n = T1.shape[0]
    isg = None if inv_sigma is None else _dev(inv_sigma, dev)
    r = torch.empty((n, 6), dtype=torch.float64, device=dev)
    J = [torch.empty((n, c, 6), dtype=torch.float64, device=dev) for c in (6, 3, 3, 6)] if jacobians else [None] * 4
    err = torch.empty(n, dtype=torch.float64, device=dev) if isg is not None else None
    _lib.check(_lib.lib().pa_dyn_linearize(
        n, T1.data_ptr(), w.data_ptr(), v.data_ptr(), T2.data_ptr(), float(dt),
        _lib.VEL_WORLD if vel_frame == "world" else _lib.VEL_BODY, _lib.ptr(isg), r.data_ptr(),
        *[_lib.ptr(j) for j in J], _lib.ptr(err), _lib.stream_of(dev)), "pa_dyn_linearize")
    out = {"r": r, "err": err}
    if jacobians:
        for i, j in enumerate(J):
            out[f"J{i}"] = j.transpose(1, 2)  # stored column-major -> (n, 6, cols)
    return out


def linearize_const_vel(v1, v2, inv_sigma=None):
    dev = _device()
    v1, v2 = _dev(v1, dev), _dev(v2, dev)
    n = v1.shape[0]
    isg = None if inv_sigma is None else _dev(inv_sigma, dev)
    r = torch.empty((n, 3), dtype=torch.float64, device=dev)
    J0 = torch.empty((n, 3, 3), dtype=torch.float64, device=dev)
    J1 = torch.empty((n, 3, 3), dtype=torch.float64, device=dev)
    err = torch.empty(n, dtype=torch.float64, device=dev) if isg is not None else None
    _lib.check(_lib.lib().pa_cv_linearize(n, v1.data_ptr(), v2.data_ptr(), _lib.ptr(isg), r.data_ptr(),
                                          J0.data_ptr(), J1.data_ptr(), _lib.ptr(err), _lib.stream_of(dev)),
               "pa_cv_linearize")
    return {"r": r, "J0": J0.transpose(1, 2), "J1": J1.transpose(1, 2), "err": err}


def linearize_projection(Tbody, p_b, z, K, Tcam=None, inv_sigma=None, jacobians=True):
    """Batched KeypointProjectionFactor (factors.py:216-275).  K: (5,) shared or (n,5);
    Tcam: None (identity), (12,) shared or (n,12).  Returns r (n,2), J (n,2,6), status (n,)
    (1 = cheirality), err (n,) if inv_sigma."""
    dev = _device()
    Tb, pb, zz = _dev(Tbody, dev), _dev(p_b, dev), _dev(z, dev)
    n = Tb.shape[0]
    Kt = _dev(K, dev)
    ks = 5 if Kt.dim() == 2 else 0
    Tc = None if Tcam is None else _dev(Tcam, dev)
    ts = 0 if Tc is None or Tc.dim() == 1 else 12
    isg = None if inv_sigma is None else _dev(inv_sigma, dev)
    r = torch.empty((n, 2), dtype=torch.float64, device=dev)
    J = torch.empty((n, 6, 2), dtype=torch.float64, device=dev) if jacobians else None
    st = torch.empty(n, dtype=torch.int32, device=dev)
    err = torch.empty(n, dtype=torch.float64, device=dev) if isg is not None else None
    _lib.check(_lib.lib().pa_proj_linearize(n, Tb.data_ptr(), pb.data_ptr(), zz.data_ptr(), Kt.data_ptr(), ks,
                                            _lib.ptr(Tc), ts, _lib.ptr(isg), r.data_ptr(), _lib.ptr(J),
                                            _lib.ptr(err), st.data_ptr(), _lib.stream_of(dev)), "pa_proj_linearize")
    out = {"r": r, "status": st, "err": err}
    if jacobians:
        out["J"] = J.transpose(1, 2)
    return out


# -------------------------------------------------------- drop-in factor classes
class _Factor:
    dim = 0

    def __init__(self, noise_model, keys):
        self._noise = noise_model
        self._keys = list(keys)

    def keys(self):
        return list(self._keys)

    def noiseModel(self):
        return self._noise

    def dim(self):  # noqa: F811  (gtsam API name)
        return type(self).dim

    def unwhitenedError(self, v, H=None):
        return self.error_func(self, v, H)

    def error(self, v) -> float:
        r = self.error_func(self, v)
        s = self._noise.sigmas() if self._noise is not None else np.ones_like(r)
        rw = r / s
        return 0.5 * float(rw @ rw)

    def linearize(self, v):
        H = [None] * len(self._keys)
        r = self.error_func(self, v, H)
        s = self._noise.sigmas() if self._noise is not None else np.ones_like(r)
        return [h / s[:, None] for h in H], -r / s


class PoseDynamicsFactor(_Factor):
    """factors.py:8-142."""

    dim = 6

    def __init__(self, pose1, ang_vel1, vel1, pose2, noise_model, dt: float, vel_frame: str = "world") -> None:
        assert vel_frame in ["world", "body"], "vel_frame must be 'world' or 'body'."
        super().__init__(noise_model, [pose1, ang_vel1, vel1, pose2])
        self.dt = dt
        self.vel_frame = vel_frame

    def error_func(self, this, v, H: Optional[List[np.ndarray]] = None, dt: Optional[float] = None,
                   vel_frame: Optional[str] = None) -> np.ndarray:
        this = this if this is not None else self
        dt = self.dt if dt is None else dt
        vel_frame = self.vel_frame if vel_frame is None else vel_frame
        k = this.keys()
        T1 = _pose12(v.atPose3(k[0]))[None]
        w = np.asarray(v.atVector(k[1]), np.float64)[None]
        vel = np.asarray(v.atVector(k[2]), np.float64)[None]
        T2 = _pose12(v.atPose3(k[3]))[None]
        out = linearize_dynamics(T1, w, vel, T2, dt, vel_frame, jacobians=bool(H))
        if H:
            for i in range(4):
                H[i] = np.asfortranarray(out[f"J{i}"][0].cpu().numpy())
        return out["r"][0].cpu().numpy()


class ConstantVelocityFactor(_Factor):
    """factors.py:145-171."""

    dim = 3

    def __init__(self, vel1, vel2, noise_model) -> None:
        super().__init__(noise_model, [vel1, vel2])

    def error_func(self, this, v, H: Optional[List[np.ndarray]] = None) -> np.ndarray:
        this = this if this is not None else self
        k = this.keys()
        out = linearize_const_vel(np.asarray(v.atVector(k[0]), np.float64)[None],
                                  np.asarray(v.atVector(k[1]), np.float64)[None])
        if H:
            H[0] = np.asfortranarray(out["J0"][0].cpu().numpy())
            H[1] = np.asfortranarray(out["J1"][0].cpu().numpy())
        return out["r"][0].cpu().numpy()


class KeypointProjectionFactor(_Factor):
    """factors.py:174-275."""

    dim = 2

    def __init__(self, body_pose, noise_model, camera_intrinsics, keypoint_measurement, point_body_frame,
                 camera_pose=None) -> None:
        super().__init__(noise_model, [body_pose])
        self.camera_intrinsics = camera_intrinsics
        self.keypoint_measurement = np.asarray(keypoint_measurement, np.float64).reshape(2)
        self.point_body_frame = np.asarray(point_body_frame, np.float64).reshape(3)
        self.camera_pose = camera_pose if camera_pose is not None else Pose3()
        self.pixel = None

    def error_func(self, this, v, H: Optional[List[np.ndarray]] = None, camera_intrinsics=None,
                   keypoint_measurement=None, point_body_frame=None, camera_pose=None) -> np.ndarray:
        this = this if this is not None else self
        K = _cal5(self.camera_intrinsics if camera_intrinsics is None else camera_intrinsics)
        z = self.keypoint_measurement if keypoint_measurement is None else np.asarray(keypoint_measurement, np.float64)
        pb = self.point_body_frame if point_body_frame is None else np.asarray(point_body_frame, np.float64)
        cam = self.camera_pose if camera_pose is None else camera_pose
        Tb = _pose12(v.atPose3(this.keys()[0]))[None]
        out = linearize_projection(Tb, pb[None], z[None], K, _pose12(cam), jacobians=bool(H))
        if int(out["status"][0].item()) != 0:
            raise CheiralityException("CheiralityException: point behind the camera")
        r = out["r"][0].cpu().numpy()
        if H:
            H[0] = np.asfortranarray(out["J"][0].cpu().numpy())
        self.pixel = r + z
        return r
