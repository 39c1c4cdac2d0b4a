"""Drop-in `KeypointCNN` backed by the gfx950 HIP kernels of libperseus_amd.so.

Mirrors `perseus/detector/models.py:6-40`:
  * `KeypointCNN(n_keypoints=8, num_channels=3, H=256, W=256)` with attributes
    `.n_keypoints .num_channels .H .W` (read by validate.py:176, streaming.py:130);
  * `state_dict()` / `load_state_dict()` with torchvision resnet18 key names under
    `resnet.` (122 keys incl. 20 `num_batches_tracked`), so checkpoints saved by the
    reference's train.py (`torch.save(model.state_dict())`, train.py:351-355) load
    unchanged after the callers' own `module.` stripping (validate.py:93-97);
  * `forward(x)`: x (B, C, H, W) f32 -> (B, 2K) f32 normalized keypoints.

Nothing here computes on the CPU: the parameters are plain containers (there is no
torch conv graph behind them), and forward calls the C ABI.  A CPU input tensor (as in
scripts/streaming.py:126-128, which never moves the model) is copied to the current
GPU, run there, and the result copied back to the input's device.

Differences from the reference (documented in DESIGN.md): inference only (no
autograd, `train()` mode is not supported), only 256x256 inputs, num_channels 1-4.
"""

from __future__ import annotations

import numpy as np
import torch
from torch import nn

from . import _lib
from .synth import float_keys, resnet18_shapes


# Bumped whenever any module registers (or re-assigns) a parameter or buffer, so a
# model's cached tensor list for the weight fingerprint is rebuilt after structural
# changes; in-place updates (load_state_dict copies) show in each tensor's _version.
_REG_EPOCH = [0]


def _bump_epoch(*_args, **_kw):
    _REG_EPOCH[0] += 1


torch.nn.modules.module.register_module_parameter_registration_hook(_bump_epoch)
torch.nn.modules.module.register_module_buffer_registration_hook(_bump_epoch)


class _Conv(nn.Module):
    def __init__(self, shape):
        super().__init__()
        self.weight = nn.Parameter(torch.zeros(shape), requires_grad=False)


class _BN(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(c), requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(c), requires_grad=False)
        self.register_buffer("running_mean", torch.zeros(c))
        self.register_buffer("running_var", torch.ones(c))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))


class _Linear(nn.Module):
    def __init__(self, out_f, in_f):
        super().__init__()
        self.weight = nn.Parameter(torch.zeros(out_f, in_f), requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(out_f), requires_grad=False)


class _Block(nn.Module):
    def __init__(self, cin, cout, ds):
        super().__init__()
        self.conv1 = _Conv((cout, cin, 3, 3))
        self.bn1 = _BN(cout)
        self.conv2 = _Conv((cout, cout, 3, 3))
        self.bn2 = _BN(cout)
        if ds:
            self.downsample = nn.ModuleDict({"0": _Conv((cout, cin, 1, 1)), "1": _BN(cout)})


class _ResNet18Params(nn.Module):
    """Parameter tree with torchvision.models.resnet18's names (no forward)."""

    def __init__(self, in_ch, n_out):
        super().__init__()
        self.conv1 = _Conv((64, in_ch, 7, 7))
        self.bn1 = _BN(64)
        cin = 64
        for li, cout in enumerate((64, 128, 256, 512), start=1):
            ds = li > 1
            self.add_module(f"layer{li}", nn.ModuleDict({"0": _Block(cin, cout, ds), "1": _Block(cout, cout, False)}))
            cin = cout
        self.fc = _Linear(n_out, 512)


class KeypointCNN(nn.Module):
    """Default perseus keypoint CNN (ResNet-18 regressor), HIP/MFMA implementation."""

    def __init__(self, n_keypoints: int = 8, num_channels: int = 3, H: int = 256, W: int = 256,
                 precision: str = "fp16") -> None:
        super().__init__()
        if (H, W) != (256, 256):
            raise ValueError(f"only 256x256 inputs are supported, got {H}x{W}")
        if not 1 <= num_channels <= 4:
            raise ValueError(f"num_channels must be in [1, 4], got {num_channels}")
        self.resnet = _ResNet18Params(num_channels, 2 * n_keypoints)
        self.n_keypoints = n_keypoints
        self.num_channels = num_channels
        self.H = H
        self.W = W
        self.precision = precision
        self._handle = None
        self._handle_dev = None
        self._stamp = None
        self._variants = {}
        self._split_k = 0
        self.eval()

    # -------------------------------------------------------------- weights
    def _fingerprint(self):
        # state_dict() walks the module tree (~130 us per forward); the tensor list is
        # cached until a parameter/buffer registration anywhere bumps _REG_EPOCH
        if getattr(self, "_fp_epoch", None) != _REG_EPOCH[0]:
            self._fp_tensors = list(self.state_dict(keep_vars=True).values())
            self._fp_epoch = _REG_EPOCH[0]
        return tuple((t._version, t.data_ptr()) for t in self._fp_tensors)

    def _blob(self) -> np.ndarray:
        sd = self.state_dict()
        shapes = resnet18_shapes(self.num_channels, self.n_keypoints)
        parts = [sd[k].detach().to("cpu", torch.float32).reshape(-1).numpy() for k in float_keys(shapes)]
        return np.ascontiguousarray(np.concatenate(parts))

    def _new_handle(self, device: torch.device):
        """A fresh pa_detector handle on `device` holding the current weights (the
        caller owns it: pa_detector_destroy)."""
        L = _lib.lib()
        blob = self._blob()
        h = _lib.C.c_void_p()
        with torch.cuda.device(device):
            _lib.check(L.pa_detector_create(blob.ctypes.data, blob.nbytes, self.num_channels, self.n_keypoints,
                                            self.H, self.W, _lib.C.byref(h)), "pa_detector_create")
        for layer in range(8):
            _lib.check(L.pa_detector_debug_set_variant(h, layer, self._variants.get(layer, 0)), "set_variant")
        if self._split_k:
            _lib.check(L.pa_detector_set_split_k(h, self._split_k), "set_split_k")
        return h

    def _ensure_handle(self, device: torch.device):
        stamp = self._fingerprint()
        if self._handle is not None and self._stamp == stamp and self._handle_dev == device:
            return self._handle
        self._release()
        h = self._new_handle(device)
        self._handle = h
        self._handle_dev = device
        self._stamp = stamp
        return h

    def refresh_weights(self) -> None:
        """Re-upload the weights on the next forward.  Needed only after writes that
        bypass the version counters the fingerprint reads (`param.data[...] = v`,
        `param.data.copy_(v)`); load_state_dict and in-place ops on the parameters
        themselves are picked up automatically."""
        self._stamp = None

    def set_variants(self, variants: "dict[int, int] | None" = None) -> None:
        """Tuning hook (include/perseus_amd_debug.h): kernel variant per layer for THIS
        model's handle; {} / None restores the shipped kernels."""
        self._variants = dict(variants or {})
        if self._handle is not None:
            L = _lib.lib()
            for layer in range(8):
                _lib.check(L.pa_detector_debug_set_variant(self._handle, layer, self._variants.get(layer, 0)),
                           "set_variant")

    def set_split_k(self, max_batch: int) -> None:
        """Latency mode (pa_detector_set_split_k): fp16 and fp16x3 forwards of at most
        `max_batch` frames run short stem bands, small tiles and layers 2-4's convs split-K
        (fills the chip at a few frames; deterministic, not bit-identical to the batched
        kernels; fp16x3 keeps its 1e-3 px parity).  0 turns it off."""
        if not 0 <= max_batch <= 64:
            raise ValueError(f"split-K max batch {max_batch} not in [0, 64]")
        self._split_k = int(max_batch)
        if self._handle is not None:
            _lib.check(_lib.lib().pa_detector_set_split_k(self._handle, self._split_k), "set_split_k")

    def set_trace(self, trace: "torch.Tensor | None") -> None:
        """Timestamp buffer of the tracing kernel variants (None = off)."""
        dev = trace.device if trace is not None else torch.device("cuda", torch.cuda.current_device())
        _lib.check(_lib.lib().pa_detector_debug_set_trace(self._ensure_handle(dev),
                                                           None if trace is None else trace.data_ptr()), "set_trace")

    def _release(self):
        if self._handle is not None:
            _lib.lib().pa_detector_destroy(self._handle)
            self._handle = None

    def __del__(self):
        try:
            self._release()
        except Exception:
            pass

    def train(self, mode: bool = True):
        if mode:
            raise NotImplementedError("perseus_amd.KeypointCNN is inference-only (train.py is out of scope)")
        return super().train(False)

    def reserve(self, max_batch: int, device=None):
        """pa_detector_reserve in this model's precision: the workspace (and for fp16x3 / fp32
        the RGBD staging of forward_rgbd) for batches up to `max_batch`, so that a graph
        captured afterwards allocates nothing."""
        device = torch.device(device or torch.device("cuda", torch.cuda.current_device()))
        h = self._ensure_handle(device)
        L = _lib.lib()
        _lib.check(L.pa_detector_set_precision(h, _lib.precision_code(self.precision)), "set_precision")
        _lib.check(L.pa_detector_reserve(h, max_batch), "reserve")

    def flops_per_frame(self) -> float:
        dev = torch.device("cuda", torch.cuda.current_device())
        return _lib.lib().pa_detector_flops_per_frame(self._ensure_handle(dev))

    # -------------------------------------------------------------- forward
    def _prep(self, x: torch.Tensor):
        if x.dim() != 4 or x.shape[1] != self.num_channels or x.shape[2] != self.H or x.shape[3] != self.W:
            raise RuntimeError(f"expected input of shape (B, {self.num_channels}, {self.H}, {self.W}), "
                               f"got {tuple(x.shape)}")
        out_dev = x.device
        if x.device.type != "cuda":
            if not torch.cuda.is_available():
                raise RuntimeError("perseus_amd.KeypointCNN needs a ROCm GPU (no CPU fallback)")
            x = x.to(torch.device("cuda", torch.cuda.current_device()), non_blocking=False)
        x = x.to(torch.float32).contiguous()
        return x, out_dev

    def forward(self, x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """`out` (optional, not in the reference signature): a contiguous f32 (B, 16) tensor on
        the input's GPU that the keypoints are written into (no extra copy kernel)."""
        x, out_dev = self._prep(x)
        dev = x.device
        h = self._ensure_handle(dev)
        L = _lib.lib()
        _lib.check(L.pa_detector_set_precision(h, _lib.precision_code(self.precision)),
                   "set_precision")
        shape = (x.shape[0], 2 * self.n_keypoints)
        if out is not None:
            if (out.device != dev or out.dtype != torch.float32 or tuple(out.shape) != shape
                    or not out.is_contiguous()):
                raise RuntimeError(f"out must be a contiguous float32 {shape} tensor on {dev}")
            y = out
        else:
            y = torch.empty(shape, dtype=torch.float32, device=dev)
        with torch.cuda.device(dev):
            _lib.check(L.pa_detector_forward(h, x.data_ptr(), x.shape[0], y.data_ptr(), _lib.stream_of(dev)),
                       "pa_detector_forward")
        return y if out_dev == dev else y.to(out_dev)

    def forward_rgbd(self, rgb: torch.Tensor, depth: torch.Tensor, bgr: bool = True, near: float | None = None,
                     far: float | None = None) -> torch.Tensor:
        """Camera frames -> keypoints (streaming.py:68-80 then :128): uint8 (B,Hs,Ws,3) + f32
        metres (B,Hs,Ws) on the GPU, centre-cropped to 256x256, through pa_detector_forward_rgbd:
        fp16: the preprocess runs inside the stem's row loads (no f32 input tensor); fp16x3 /
        fp32: the preprocess kernel into the handle's staging, then the forward.  All give the
        bits of forward(preprocess_rgbd(rgb, depth, ...))."""
        if rgb.device.type != "cuda" or depth.device.type != "cuda":
            raise RuntimeError("forward_rgbd expects device tensors")
        if self.num_channels != 4:
            return self.forward(preprocess_rgbd(rgb, depth, self.H, self.W, bgr=bgr, near=near, far=far))
        rgb = rgb.contiguous()
        depth = depth.contiguous().float()
        if rgb.dtype != torch.uint8 or rgb.dim() != 4 or rgb.shape[-1] != 3 or depth.shape != rgb.shape[:3]:
            raise RuntimeError(f"expected uint8 (B,Hs,Ws,3) + (B,Hs,Ws) depth, got {tuple(rgb.shape)} "
                               f"{rgb.dtype} / {tuple(depth.shape)}")
        B, Hs, Ws, _ = rgb.shape
        dev = rgb.device
        h = self._ensure_handle(dev)
        L = _lib.lib()
        _lib.check(L.pa_detector_set_precision(h, _lib.precision_code(self.precision)), "set_precision")
        y = torch.empty((B, 2 * self.n_keypoints), dtype=torch.float32, device=dev)
        with torch.cuda.device(dev):
            _lib.check(L.pa_detector_forward_rgbd(h, rgb.data_ptr(), depth.data_ptr(), B, Hs, Ws, int(bgr),
                                                  -1.0 if near is None else float(near),
                                                  -1.0 if far is None else float(far), y.data_ptr(),
                                                  _lib.stream_of(dev)), "pa_detector_forward_rgbd")
        return y

    def profile(self, x: torch.Tensor, max_kernels: int = 64):
        """Per-kernel device times (ms) of one forward, via HIP events in the library."""
        x, _ = self._prep(x)
        dev = x.device
        h = self._ensure_handle(dev)
        L = _lib.lib()
        _lib.check(L.pa_detector_set_precision(h, _lib.precision_code(self.precision)),
                   "set_precision")
        y = torch.full((x.shape[0], 2 * self.n_keypoints), float("nan"), dtype=torch.float32, device=dev)
        ms = (_lib.C.c_float * max_kernels)()
        names = (_lib.C.c_char_p * max_kernels)()
        with torch.cuda.device(dev):
            n = _lib.check(L.pa_detector_profile(h, x.data_ptr(), x.shape[0], y.data_ptr(), _lib.stream_of(dev),
                                                 ms, names, max_kernels), "pa_detector_profile")
        return [(names[i].decode(), ms[i]) for i in range(n)], y


    def time_launch(self, x: torch.Tensor, index: int, reps: int = 20):
        """(name, avg ms) of launch `index` of the forward, issued `reps` times back to
        back between two HIP events on the current stream (no per-launch event gaps)."""
        x, _ = self._prep(x)
        dev = x.device
        h = self._ensure_handle(dev)
        L = _lib.lib()
        _lib.check(L.pa_detector_set_precision(h, _lib.precision_code(self.precision)),
                   "set_precision")
        y = torch.empty((x.shape[0], 2 * self.n_keypoints), dtype=torch.float32, device=dev)
        ms = _lib.C.c_float()
        name = _lib.C.c_char_p()
        with torch.cuda.device(dev):
            _lib.check(L.pa_detector_time_launch(h, x.data_ptr(), x.shape[0], y.data_ptr(), _lib.stream_of(dev),
                                                 index, reps, _lib.C.byref(ms), _lib.C.byref(name)),
                       "pa_detector_time_launch")
        return name.value.decode(), ms.value


def denormalize_pixel_coordinates(y: torch.Tensor, H: int = 256, W: int = 256, target: torch.Tensor | None = None):
    """Device post-processing (validate.py:130-153): normalized (B,2K) -> px (B,K,2),
    plus SmoothL1(beta=1, reduction='none') against normalized targets if given."""
    if y.device.type != "cuda":
        raise RuntimeError("denormalize_pixel_coordinates expects a device tensor")
    y = y.contiguous().float()
    B, n2 = y.shape
    px = torch.empty((B, n2 // 2, 2), dtype=torch.float32, device=y.device)
    loss = None
    tptr = None
    if target is not None:
        target = target.reshape(B, n2).contiguous().float()
        loss = torch.empty_like(y)
        tptr = target.data_ptr()
    _lib.check(_lib.lib().pa_keypoints_postprocess(y.data_ptr(), tptr, B, n2 // 2, H, W, px.data_ptr(),
                                                   None if loss is None else loss.data_ptr(),
                                                   _lib.stream_of(y.device)), "postprocess")
    return px if loss is None else (px, loss)


def loss_statistics(losses: torch.Tensor) -> dict:
    """The "Validation Loss" block of validate.py:162-168 on the device: mean, stdev
    (unbiased, as torch.std), min, max and median (torch.median: the lower middle element)
    of the flattened losses, computed by the library's HIP kernels (pa_loss_statistics)
    with one device->host copy of the five results.  Raises on an empty tensor."""
    if losses.device.type != "cuda":
        raise RuntimeError("loss_statistics expects a device tensor")
    x = losses.reshape(-1).contiguous().float()
    n = x.numel()
    if n == 0:
        raise RuntimeError("loss_statistics: empty input")
    L = _lib.lib()
    ws = torch.empty(int(L.pa_loss_statistics_workspace(n)), dtype=torch.uint8, device=x.device)
    out = torch.empty(5, dtype=torch.float64, device=x.device)
    _lib.check(L.pa_loss_statistics(x.data_ptr(), n, out.data_ptr(), ws.data_ptr(), ws.numel(),
                                    _lib.stream_of(x.device)), "loss_statistics")
    mean, std, mn, mx, med = out.cpu().tolist()
    # the reference prints torch f32 reductions (validate.py:165): the f64 results rounded
    # once to f32 are what an exact f32 reduction returns (torch's own order may differ
    # from them by a few f32 ulps; tests/test_stats_gpu.py bounds that)
    f32 = {k: float(np.float32(v)) for k, v in (("mean", mean), ("std", std))}
    return {"mean": mean, "std": std, "min": mn, "max": mx, "median": med, "mean_f32": f32["mean"],
            "std_f32": f32["std"]}


def validation_report(losses: torch.Tensor) -> str:
    """The "Validation Loss" block validate.py:162-168 prints, from loss_statistics (device
    reductions, one 40-byte copy back); values are f32 tensors as torch prints them."""
    st = loss_statistics(losses)
    t = lambda v: torch.tensor(v, dtype=torch.float32)  # noqa: E731
    return "\n".join(["=" * 80, "Validation Loss", f"Mean +/- Stdev: {t(st['mean_f32'])} +/- {t(st['std_f32'])}",
                      f"Min: {t(st['min'])}", f"Max: {t(st['max'])}", f"Median: {t(st['median'])}", "=" * 80])


def preprocess_rgbd(rgb: torch.Tensor, depth: torch.Tensor, H: int = 256, W: int = 256, bgr: bool = True,
                    near: float | None = None, far: float | None = None) -> torch.Tensor:
    """Device version of ZEDCamera.get_frame's arithmetic (streaming.py:59-82) +
    deterministic near/far clip: uint8 (B,Hs,Ws,3) + f32 metres (B,Hs,Ws) ->
    (B,4,H,W) f32 model input."""
    if rgb.device.type != "cuda" or depth.device.type != "cuda":
        raise RuntimeError("preprocess_rgbd expects device tensors")
    rgb = rgb.contiguous()
    depth = depth.contiguous().float()
    B, Hs, Ws, _ = rgb.shape
    x = torch.empty((B, 4, H, W), dtype=torch.float32, device=rgb.device)
    _lib.check(_lib.lib().pa_preprocess_rgbd(rgb.data_ptr(), depth.data_ptr(), B, Hs, Ws, int(bgr),
                                             -1.0 if near is None else near, -1.0 if far is None else far,
                                             H, W, x.data_ptr(), _lib.stream_of(rgb.device)), "preprocess")
    return x
