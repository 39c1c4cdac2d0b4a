"""Config 4: multi-camera streaming keypoint inference -> pose, one captured HIP graph.

Mirrors the per-frame loop of `scripts/streaming.py:120-131` (grab BGR + depth,
`/255`, depth nan/inf -> 0 and `/0.035`, centre 256x256 crop, `model(x)`, kornia
denormalize) for `n_cams` cameras per tick, batched into one forward, and (with
`pose_window` = L > 0) the pose stage BASELINE.json configs[4] asks for ("end-to-end pose
latency"): a fixed-lag smoother per camera over its last L frames built from the
reference's own factors (perseus/smoother/factors.py: KeypointProjectionFactor :182-275
per keypoint, PoseDynamicsFactor :8-142 and ConstantVelocityFactor :145-171 per frame
pair).  The reference stops at pixels (streaming.py draws them); the factor graph and
its optimizer live in downstream GTSAM code, so this build defines the loop: one damped
Gauss-Newton step per tick.  Per tick:

  host: frames -> pinned staging (centre crop rows only, or the full frame)
  GPU (one hipGraph replay on a private stream): H2D -> pa_detector_forward_rgbd_px
       (B = n_cams; fp16: the preprocess runs inside the stem's row loads; fp16x3 / fp32: the
       preprocess kernel, then the forward; the denormalize in the head), in the small-batch
       latency mode for fp16 and fp16x3 (the parity-grade tick)
       [pose stage] the sequence pa_window_advance_n (window shifts one frame, the new
       keypoints appended, the new pose predicted by the dynamics model, the count of real
       frames + 1) -> pa_trajectory_linearize (whitened factors of every camera's window;
       frames not yet filled by a real tick carry no projection factors) ->
       pa_trajectory_gn_step (delta and info only) -> pa_window_retract_newest (pose
       Exp(delta), velocities += delta, newest poses out), run as the split tick for windows
       <= 24 frames: pa_window_pose_tick_pre (all of it that does not need the new keypoints,
       on the tick's stream while the forward runs on a second one; or, pre_ahead=True, right
       after the previous tick's results) and pa_window_pose_tick_post after the forward
       -> the pixels, info and newest poses land in the pinned output block (zero_copy_out;
       else one D2H), one H2D of [rgb | depth] at the start (or zero-copy reads of it)
  host: wait for the replay, return (n_cams, K, 2) pixel coordinates (and the poses).

The graph removes the per-launch CPU cost of the ~26 launches (the forward at B=3
is launch-bound, not compute-bound).  Workspace and every pose-stage buffer are
allocated before capture so no allocation happens inside the graph.
"""

from __future__ import annotations

import ctypes as C

import warnings

import numpy as np
import torch

from . import _lib, pipeline, synth


class StreamingPipeline:
    """pose_window = L > 0 turns the pose stage on (module docstring).  Its parameters:
    K (fx, fy, s, u0, v0) of the 256x256 crop and the body-frame corners (defaults: the
    datagen camera and cube, synth.CAMERA_K / CUBE_CORNERS); dt = the camera period;
    sigmas of the diagonal noise models (pixels, dynamics tangent, velocity); lam = the
    LM damping; init_pose (n_cams, 12) / init_vel / init_angvel fill every frame of the
    initial window (default: the cube 0.4 m in front of each camera, at rest)."""

    def __init__(self, model, n_cams: int = 3, src_hw=(720, 1280), bgr: bool = True, host_crop: bool = True,
                 graph: bool = True, near: float | None = None, far: float | None = None, device=None,
                 pose_window: int = 0, K=None, corners=None, dt: float = 1.0 / 30.0, vel_frame: str = "world",
                 proj_sigma: float = 1.0, dyn_sigma: float = 0.1, cv_sigma: float = 0.1, lam: float = 1e-2,
                 init_pose=None, init_vel=None, init_angvel=None, split_k: bool = True,
                 zero_copy: bool | None = None, split_pose: bool = True, pre_ahead: bool = False,
                 zero_copy_out: bool = True):
        if not torch.cuda.is_available():
            raise RuntimeError("StreamingPipeline needs a ROCm GPU (no CPU fallback)")
        cam_K = K  # (the name K is the keypoint count below)
        self.dev = torch.device(device or torch.device("cuda", torch.cuda.current_device()))
        self.model = model
        self.n = n_cams
        self.Hs, self.Ws = src_hw
        self.H, self.W = model.H, model.W
        if self.Hs < self.H or self.Ws < self.W:
            raise ValueError(f"source {src_hw} smaller than the model input {self.H}x{self.W}")
        self.bgr = bgr
        self.host_crop = host_crop
        self.near = -1.0 if near is None else float(near)
        self.far = -1.0 if far is None else float(far)
        sh, sw = (self.H, self.W) if host_crop else (self.Hs, self.Ws)
        self.sh, self.sw = sh, sw
        self.r0, self.c0 = self.Hs // 2 - self.H // 2, self.Ws // 2 - self.W // 2
        n, K = n_cams, model.n_keypoints
        # One staging block per direction, so a tick is one H2D and one D2H copy (each copy is a
        # ~5-12 us operation on the stream, and a copy enqueued between kernels stalls them):
        #   in  = [rgb (n, sh, sw, 3) u8 | depth (n, sh, sw) f32]
        #   out = [px (n, K, 2) f32 | info (n,) i32 | pad to 8 B | newest pose (n, 12) f64]
        nr = n * sh * sw * 3
        if nr % 4:
            raise ValueError(f"staging: {n} x {sh} x {sw} RGB bytes not 4-aligned for the depth block")
        nin = nr + n * sh * sw * 4
        self._po = ((n * K * 2 + n) * 4 + 7) // 8 * 8
        self._px_bytes = n * K * 8
        nout = self._po + n * 12 * 8
        self.in_h = torch.empty(nin, dtype=torch.uint8).pin_memory()
        self.in_d = torch.empty(nin, dtype=torch.uint8, device=self.dev)
        self.out_h = torch.zeros(nout, dtype=torch.uint8).pin_memory()
        self.out_d = torch.zeros(nout, dtype=torch.uint8, device=self.dev)

        def views(i, o):
            return (i[:nr].view(n, sh, sw, 3), i[nr:].view(torch.float32).view(n, sh, sw),
                    o[:n * K * 8].view(torch.float32).view(n, K, 2),
                    o[n * K * 8:n * K * 8 + n * 4].view(torch.int32),
                    o[self._po:].view(torch.float64).view(n, 12))

        self.rgb_h, self.depth_h, self.px_h, self.info_h, self.pose_h = views(self.in_h, self.out_h)
        self.rgb_d, self.depth_d, self.px_d, self.info_d, self.pose_d = views(self.in_d, self.out_d)
        # zero_copy: the stem (fp16) / the preprocess kernel (fp16x3, fp32) read the pinned staging
        # over PCIe, no H2D copy in the tick.  None: on for the preprocess-kernel precisions (its
        # coalesced reads beat the copy: fp16x3 pose tick 0.330 -> 0.322 ms device), off for fp16
        # (the stem's row loads over PCIe lose: 0.252 -> 0.267 ms; profiles/r04v/)
        self.zero_copy = (model.precision != "fp16") if zero_copy is None else bool(zero_copy)
        self._src = (self.rgb_d.data_ptr(), self.depth_d.data_ptr())
        if self.zero_copy:
            dp = C.c_void_p()
            _lib.check(_lib.lib().pa_host_device_pointer(C.c_void_p(self.in_h.data_ptr()), C.byref(dp)),
                       "host_device_pointer")
            self._src = (dp.value, dp.value + nr)
        # zero_copy_out: the head writes the pixels, and the split tick's post half info and the
        # newest poses, straight into the pinned output block over PCIe (a few hundred bytes), so
        # the tick has no D2H copy; the fused / four-launch pose stages keep the copy
        self._zc_out = bool(zero_copy_out)
        self._px_out = self.px_d.data_ptr()
        if self._zc_out:
            dp = C.c_void_p()
            _lib.check(_lib.lib().pa_host_device_pointer(C.c_void_p(self.out_h.data_ptr()), C.byref(dp)),
                       "host_device_pointer")
            self._out_dev = dp.value
            self._px_out = dp.value
        self.y = torch.empty((n, 2 * K), dtype=torch.float32, device=self.dev)
        self.y_h = torch.empty((n, 2 * K), dtype=torch.float32).pin_memory()  # tick_keypoints' input
        self.pose_graph = None
        self.stream = torch.cuda.Stream(self.dev)
        # A private handle: the captured graph holds its weight and workspace pointers, so
        # nothing the model does later (a larger batch growing its workspace, a weight
        # reload destroying its handle) may free them under the graph.  Weights are taken
        # as of construction.
        L = _lib.lib()
        self._h = model._new_handle(self.dev)
        _lib.check(L.pa_detector_set_precision(self._h, _lib.precision_code(model.precision)), "set_precision")
        _lib.check(L.pa_detector_reserve(self._h, n), "reserve")
        # latency mode: a batch of n_cams frames leaves most CUs idle in the batched kernels
        # (pa_detector_set_split_k; same results as model.set_split_k(n_cams) + forward;
        # fp16 and fp16x3, fp32 has no such mode)
        self.split_k = bool(split_k) and n <= 64 and model.precision != "fp32"
        _lib.check(L.pa_detector_set_split_k(self._h, n if self.split_k else 0), "set_split_k")
        if model.num_channels != 4:
            raise ValueError("StreamingPipeline feeds RGBD (num_channels=4)")
        self.pose_L = int(pose_window)
        self._split_pose_req = bool(split_pose)
        self._pre_ahead_req = bool(pre_ahead)
        self.fused_pose = self.split_pose = self.pre_ahead = False
        if self.pose_L:
            self._init_pose_stage(cam_K, corners, dt, vel_frame, proj_sigma, dyn_sigma, cv_sigma, lam, init_pose,
                                  init_vel, init_angvel)
        self.graph = None
        self.pre_graph = None
        with torch.cuda.stream(self.stream):
            if self.pre_ahead:
                self._enqueue_pose_pre()
            self._enqueue()  # eager warm-up (also builds the kernels' first-launch state)
        self.stream.synchronize()
        if self.pose_L:
            self.reset_window()  # the warm-up tick advanced it (pre_ahead: and prepares the next tick)
        if graph:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=self.stream):
                self._enqueue()
            self.graph = g
            if self.pre_ahead:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=self.stream):
                    self._enqueue_pose_pre()
                self.pre_graph = g
        self._done = torch.cuda.Event(enable_timing=True)  # (timed: the bench's latency path)

    def _enqueue(self):
        """H2D, preprocess + forward + denormalize, [pose stage], D2H on the current stream.
        Split pose tick: the forward runs on a second stream while this one runs the pre half
        (everything but the newest keypoints); the post half after the join.  (The other
        assignment, pre half on the second stream, measured 0.233 vs 0.218 ms per fp16 tick;
        the pre half is only partly hidden either way: 0.187 ms without it, profiles/r04fork/.)"""
        L = _lib.lib()
        cur = torch.cuda.current_stream(self.dev)
        split = self.pose_L and self.split_pose and not self.pre_ahead
        fw = cur
        if split:
            self.side.wait_stream(cur)
            fw = self.side
        with torch.cuda.stream(fw):
            if not self.zero_copy:
                self.in_d.copy_(self.in_h, non_blocking=True)
            # fp16: the preprocess runs inside the stem's row loads; fp16x3 / fp32: the
            # preprocess kernel into the handle's staging, then the forward; the denormalize in the head
            _lib.check(L.pa_detector_forward_rgbd_px(self._h, self._src[0], self._src[1], self.n,
                                                     self.sh, self.sw, int(self.bgr), self.near, self.far,
                                                     self.y.data_ptr(), self._px_out, fw.cuda_stream),
                       "forward_rgbd_px")
        if split:
            self._enqueue_pose_pre()
            cur.wait_stream(self.side)
            self._enqueue_pose_post()
        elif self.pose_L:
            self._enqueue_pose()  # (pre_ahead: the post half alone)
        self._enqueue_out()

    def _enqueue_out(self):
        """pixels (+ info, newest poses) to the host: one D2H, or nothing (zero_copy_out)."""
        if not self._zc_out:
            self.out_h.copy_(self.out_d, non_blocking=True)
        elif self.pose_L and not self.split_pose:  # the fused / four-launch stages write the device block
            self.out_h[self._px_bytes:].copy_(self.out_d[self._px_bytes:], non_blocking=True)

    def _enqueue_pose_pre(self):
        pipeline.window_pose_tick_pre(self.traj_args, self.tick_ws, lam=self.gn.lam)

    def _enqueue_pose_post(self):
        if self._zc_out:  # info and the newest poses straight into the pinned output block
            info, newest = self._out_dev + self._px_bytes, self._out_dev + self._po
        else:
            info, newest = self.gn.out["info"], self.pose_d
        pipeline.window_pose_tick_post(self.traj_args, self.y, self.tick_ws, delta=self.gn.out["delta"], info=info,
                                       newest=newest)

    def _enqueue_pose(self):
        """The pose stage on the current stream, from the keypoints in self.y (HBM-resident window):
        advance -> linearize -> GN step -> retract, as pa_window_pose_tick_pre + _post (split),
        pa_window_pose_tick's two launches (fused) or the four separate ones (bit-identical to
        the fused form; windows above 24 frames)."""
        if self.split_pose:
            if not self.pre_ahead:
                self._enqueue_pose_pre()
            self._enqueue_pose_post()
            return
        if self.fused_pose:
            pipeline.window_pose_tick(self.traj_args, self.y, lam=self.gn.lam, delta=self.gn.out["delta"],
                                      info=self.gn.out["info"], newest=self.pose_d)
            return
        pipeline.window_advance(self.y, self.win, dt=self.dt, vel_frame=self.vel_frame, nvalid=self.nvalid)
        pipeline.launch(self.traj_args, self.dev)
        self.gn.launch()  # delta, and info straight into the output block
        pipeline.window_retract(self.win, self.gn.out["delta"], self.gn.out["info"], newest=self.pose_d)

    def _init_pose_stage(self, K, corners, dt, vel_frame, proj_sigma, dyn_sigma, cv_sigma, lam, init_pose, init_vel,
                         init_angvel):
        n, Lw, nk, dev = self.n, self.pose_L, self.model.n_keypoints, self.dev
        if Lw < 2:
            raise ValueError("pose_window must be >= 2 frames (the dynamics factors couple frame pairs)")
        if vel_frame not in ("world", "body"):
            raise AssertionError("vel_frame must be 'world' or 'body'.")  # factors.py:41
        self.dt, self.vel_frame = float(dt), vel_frame
        K = synth.CAMERA_K if K is None else np.asarray(K, np.float64)
        corners = synth.CUBE_CORNERS[:nk] if corners is None else np.asarray(corners, np.float64)
        if init_pose is None:
            init_pose = np.tile(np.array([1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0.4], np.float64), (n, 1))
        zeros = np.zeros((n, 3))
        self._init = {"pose": np.asarray(init_pose, np.float64).reshape(n, 12),
                      "vel": np.asarray(zeros if init_vel is None else init_vel, np.float64).reshape(n, 3),
                      "angvel": np.asarray(zeros if init_angvel is None else init_angvel, np.float64).reshape(n, 3)}
        f64 = dict(dtype=torch.float64, device=dev)
        self.win = {"y": torch.zeros((n, Lw, 2 * nk), dtype=torch.float32, device=dev),
                    "pose": torch.empty((n, Lw, 12), **f64), "angvel": torch.empty((n, Lw, 3), **f64),
                    "vel": torch.empty((n, Lw, 3), **f64)}
        # real frames per camera window (from its end): until L ticks have run, the frames
        # before them are the initial state with no measurement, and carry no projection factor
        self.nvalid = torch.zeros(n, dtype=torch.int32, device=dev)
        self.traj_args, self.lin = pipeline.prepare_trajectories(
            self.win["y"].view(n * Lw, 2 * nk), self.win["pose"].view(n * Lw, 12), self.win["vel"].view(n * Lw, 3),
            self.win["angvel"].view(n * Lw, 3), corners, K, T=n, L=Lw, dt=self.dt, vel_frame=vel_frame, H=self.H,
            W=self.W, proj_sigmas=[proj_sigma] * 2, dyn_sigmas=[dyn_sigma] * 6, cv_sigmas=[cv_sigma] * 3,
            nvalid=self.nvalid)
        for k in ("y", "pose", "vel", "angvel"):  # linearize reads the window in place, no staging copy
            assert self.lin["_keep"][("y", "pose", "vel", "angvel").index(k)].data_ptr() == self.win[k].data_ptr()
        self.gn = pipeline.GNPlan(self.lin, T=n, L=Lw, lam=lam)
        self.gn.out["info"] = self.info_d  # the GN step writes info into the output block
        # pa_window_pose_tick: one workgroup per camera of up to 24 frames, at most one per CU
        self.fused_pose = (Lw <= pipeline.TICK_MAX_L
                           and n <= torch.cuda.get_device_properties(dev).multi_processor_count)
        # the split tick (pa_window_pose_tick_pre / _post, same limits): everything but the
        # newest frame's projection factors runs beside the forward, which gets its own stream
        self.split_pose = self.fused_pose and self._split_pose_req
        # pre_ahead: the pre half of tick k + 1 runs right after tick k's results are on the host
        # (in the gap before the next camera frames), so a tick's latency path is H2D, forward,
        # post half, D2H.  The window and factor outputs then already hold the next tick's advance.
        self.pre_ahead = self.split_pose and self._pre_ahead_req
        if self._pre_ahead_req and not self.pre_ahead:  # never drop the request silently
            why = ("split_pose=False" if not self._split_pose_req else
                   f"pose_window {Lw} > {pipeline.TICK_MAX_L}" if Lw > pipeline.TICK_MAX_L else
                   f"{n} cameras > the device's CUs")
            warnings.warn(f"StreamingPipeline: pre_ahead needs the split pose tick ({why}); running the full-latency "
                          f"tick (self.pre_ahead is False)", RuntimeWarning, stacklevel=3)
        if self.split_pose and self._zc_out:
            # the post half writes info and the newest poses straight into the pinned output block
            # (self.info_h / self.pose_h); nothing writes a device copy, so none is exposed
            self.gn.out["info"] = None
        self.tick_ws = pipeline.window_pose_tick_workspace(n, Lw, dev)
        self.side = torch.cuda.Stream(dev)

    def reset_window(self) -> None:
        """Every frame of every camera's window back to the initial state (keypoints 0, no
        real frame: the next tick's window holds one measured frame)."""
        with torch.cuda.stream(self.stream):
            self.win["y"].zero_()
            self.nvalid.zero_()
            for k in ("pose", "vel", "angvel"):
                self.win[k].copy_(torch.as_tensor(self._init[k], device=self.dev)[:, None, :]
                                  .expand_as(self.win[k]))
            if self.pre_ahead:  # the next tick's pre half, from the reset window
                self._enqueue_pose_pre()
        self.stream.synchronize()

    def window_state(self) -> dict:
        """Host copies of the window (y, pose, vel, angvel) after the last tick (pre_ahead: after
        the next tick's advance, whose newest keypoints are not in yet)."""
        self.stream.synchronize()
        return {k: v.cpu().numpy().copy() for k, v in self.win.items()}

    def stage(self, rgb: np.ndarray, depth: np.ndarray) -> None:
        """Copy one tick of camera frames (n, Hs, Ws, 3) uint8 + (n, Hs, Ws) f32 metres
        into the pinned staging buffers (centre crop only when host_crop)."""
        if rgb.shape != (self.n, self.Hs, self.Ws, 3) or depth.shape != (self.n, self.Hs, self.Ws):
            raise ValueError(f"expected ({self.n},{self.Hs},{self.Ws},3) rgb and ({self.n},{self.Hs},{self.Ws}) depth")
        if self.host_crop:
            r0, c0 = self.r0, self.c0
            self.rgb_h.numpy()[:] = rgb[:, r0:r0 + self.H, c0:c0 + self.W]
            self.depth_h.numpy()[:] = depth[:, r0:r0 + self.H, c0:c0 + self.W]
        else:
            self.rgb_h.numpy()[:] = rgb
            self.depth_h.numpy()[:] = depth

    def replay(self) -> None:
        """One tick's device work on the current stream, no wait (pre_ahead: then the next
        tick's pre half, after self._done is recorded)."""
        if self.graph is not None:
            self.graph.replay()
        else:
            self._enqueue()
        if self.pre_ahead:
            self._done.record()
            self._pre()

    def _pre(self):
        if self.pre_graph is not None:
            self.pre_graph.replay()
        else:
            self._enqueue_pose_pre()

    def run(self) -> np.ndarray:
        """Process the staged tick; returns a copy of the (n, K, 2) pixel coordinates."""
        with torch.cuda.stream(self.stream):  # replay() launches on the current stream
            self.replay()
        if self.pre_ahead:
            self._done.synchronize()  # the results; the next tick's pre half keeps running
        else:
            self.stream.synchronize()
        return self.px_h.numpy().copy()

    def __call__(self, rgb: np.ndarray, depth: np.ndarray) -> np.ndarray:
        self.stage(rgb, depth)
        return self.run()

    def tick(self, rgb: np.ndarray, depth: np.ndarray):
        """One camera tick through the pose stage: (pixels (n, K, 2), newest pose of each
        camera's window (n, 12: R row-major, t), GN info (n,) int32, 0 = solved).

        The results are read from the pinned output block (self.px_h / pose_h / info_h), the
        only place every tick form writes them.  With pre_ahead, the next tick's pre half has
        already run when this returns: self.win, self.lin (the factor outputs, status 3 on
        the newest frame's projection factors) and the tick workspace hold the NEXT tick's
        advanced window, not this tick's (window_state() says the same)."""
        if not self.pose_L:
            raise RuntimeError("tick() needs the pose stage (pose_window > 0)")
        px = self(rgb, depth)
        return px, self.pose_h.numpy().copy(), self.info_h.numpy().copy()

    def tick_keypoints(self, y) -> tuple:
        """The pose stage alone on given normalized keypoints y (n, 2K) (the detector's output
        convention, validate.py:139-141): the same launches as a tick's pose stage, from
        self.y, captured as their own graph when graph=True.  Returns (newest pose (n, 12),
        GN info (n,)).  For driving the smoother with known measurements.  As tick(): the
        results come from the pinned output block, and under pre_ahead self.win / self.lin
        already hold the next tick's pre half."""
        if not self.pose_L:
            raise RuntimeError("tick_keypoints() needs the pose stage (pose_window > 0)")
        self.y_h.numpy()[:] = np.asarray(y, np.float32).reshape(self.y_h.shape)

        def enqueue():
            self.y.copy_(self.y_h, non_blocking=True)
            self._enqueue_pose()
            self._enqueue_out()

        with torch.cuda.stream(self.stream):
            if self.graph is not None:
                if self.pose_graph is None:  # captured on first use (every buffer exists already)
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=self.stream):
                        enqueue()
                    self.pose_graph = g
                self.pose_graph.replay()
            else:
                enqueue()
            if self.pre_ahead:
                self._done.record()
                self._pre()
        (self._done if self.pre_ahead else self.stream).synchronize()
        return self.pose_h.numpy().copy(), self.info_h.numpy().copy()

    def close(self) -> None:
        """Drop the graphs, then the handle they captured."""
        self.graph = None
        self.pose_graph = None
        self.pre_graph = None
        if getattr(self, "_h", None) is not None:
            torch.cuda.synchronize(self.dev)
            _lib.lib().pa_detector_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
