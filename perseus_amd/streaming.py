"""Config 4: multi-camera streaming keypoint inference with a captured HIP graph.

Mirrors the per-frame loop of `scripts/streaming.py:120-131` (grab BGR + depth,
`/255`, depth nan/inf -> 0 and `/0.035`, centre 256x256 crop, `model(x)`, kornia
denormalize) for `n_cams` cameras per tick, batched into one forward.  Per tick:

  host: frames -> pinned staging (centre crop rows only, or the full frame)
  GPU (one hipGraph replay on a private stream): H2D -> pa_detector_forward_rgbd
       (B = n_cams; the preprocess runs inside the stem's row loads; fp32: pa_preprocess_rgbd
       + pa_detector_forward) -> pa_keypoints_postprocess -> D2H pixels
  host: wait for the replay, return (n_cams, K, 2) pixel coordinates.

The graph removes the per-launch CPU cost of the ~22 launches (the forward at B=3
is launch-bound, not compute-bound).  Workspace is reserved before capture so no
allocation happens inside the graph.
"""

from __future__ import annotations

import numpy as np
import torch

from . import _lib


class StreamingPipeline:
    def __init__(self, model, n_cams: int = 3, src_hw=(720, 1280), bgr: bool = True, host_crop: bool = True,
                 graph: bool = True, near: float | None = None, far: float | None = None, device=None):
        if not torch.cuda.is_available():
            raise RuntimeError("StreamingPipeline needs a ROCm GPU (no CPU fallback)")
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
        self.rgb_h = torch.empty((n, sh, sw, 3), dtype=torch.uint8).pin_memory()
        self.depth_h = torch.empty((n, sh, sw), dtype=torch.float32).pin_memory()
        self.px_h = torch.empty((n, K, 2), dtype=torch.float32).pin_memory()
        self.rgb_d = torch.empty((n, sh, sw, 3), dtype=torch.uint8, device=self.dev)
        self.depth_d = torch.empty((n, sh, sw), dtype=torch.float32, device=self.dev)
        self.x = torch.empty((n, 4, self.H, self.W), dtype=torch.float32, device=self.dev)
        self.y = torch.empty((n, 2 * K), dtype=torch.float32, device=self.dev)
        self.px_d = torch.empty((n, K, 2), dtype=torch.float32, device=self.dev)
        self.stream = torch.cuda.Stream(self.dev)
        # A private handle: the captured graph holds its weight and workspace pointers, so
        # nothing the model does later (a larger batch growing its workspace, a weight
        # reload destroying its handle) may free them under the graph.  Weights are taken
        # as of construction.
        L = _lib.lib()
        self._h = model._new_handle(self.dev)
        _lib.check(L.pa_detector_set_precision(self._h, _lib.precision_code(model.precision)), "set_precision")
        _lib.check(L.pa_detector_reserve(self._h, n), "reserve")
        if model.num_channels != 4:
            raise ValueError("StreamingPipeline feeds RGBD (num_channels=4)")
        self.graph = None
        with torch.cuda.stream(self.stream):
            self._enqueue()  # eager warm-up (also builds the kernels' first-launch state)
        self.stream.synchronize()
        if graph:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=self.stream):
                self._enqueue()
            self.graph = g

    def _enqueue(self):
        """H2D, preprocess, forward, postprocess, D2H on the current stream."""
        L = _lib.lib()
        s = torch.cuda.current_stream(self.dev).cuda_stream
        self.rgb_d.copy_(self.rgb_h, non_blocking=True)
        self.depth_d.copy_(self.depth_h, non_blocking=True)
        if self.model.precision != "fp16":  # fp32 / fp16x3: preprocess kernel, then the forward
            _lib.check(L.pa_preprocess_rgbd(self.rgb_d.data_ptr(), self.depth_d.data_ptr(), self.n, self.sh, self.sw,
                                            int(self.bgr), self.near, self.far, self.H, self.W, self.x.data_ptr(), s),
                       "preprocess")
            _lib.check(L.pa_detector_forward(self._h, self.x.data_ptr(), self.n, self.y.data_ptr(), s), "forward")
        else:  # fp16: the preprocess runs inside the stem's row loads
            _lib.check(L.pa_detector_forward_rgbd(self._h, self.rgb_d.data_ptr(), self.depth_d.data_ptr(), self.n,
                                                  self.sh, self.sw, int(self.bgr), self.near, self.far,
                                                  self.y.data_ptr(), s), "forward_rgbd")
        _lib.check(L.pa_keypoints_postprocess(self.y.data_ptr(), None, self.n, self.model.n_keypoints, self.H, self.W,
                                              self.px_d.data_ptr(), None, s), "postprocess")
        self.px_h.copy_(self.px_d, non_blocking=True)

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

    def run(self) -> np.ndarray:
        """Process the staged tick; returns a copy of the (n, K, 2) pixel coordinates."""
        with torch.cuda.stream(self.stream):  # replay() launches on the current stream
            if self.graph is not None:
                self.graph.replay()
            else:
                self._enqueue()
        self.stream.synchronize()
        return self.px_h.numpy().copy()

    def __call__(self, rgb: np.ndarray, depth: np.ndarray) -> np.ndarray:
        self.stage(rgb, depth)
        return self.run()

    def close(self) -> None:
        """Drop the graph, then the handle it captured."""
        self.graph = None
        if getattr(self, "_h", None) is not None:
            torch.cuda.synchronize(self.dev)
            _lib.lib().pa_detector_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
