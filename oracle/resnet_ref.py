"""ORACLE (test infrastructure only) — CPU restatement of the KeypointCNN forward.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / the timed CPU baseline.  The product path
(`perseus_amd.detector`) never calls it.

What it restates
  * `perseus/detector/models.py:6-40` — KeypointCNN: torchvision resnet18 (`:20`),
    conv1 -> Conv2d(C,64,7,s2,p3,bias=False) when C != 3 (`:27-28`),
    AdaptiveAvgPool2d((1,1)) (`:31`), fc 512 -> 2K (`:32`), forward = resnet(x) (`:34-40`).
  * torchvision.models.resnet18 (third-party, pinned `torchvision>=0.16.2` at
    `pyproject.toml:19`, NOT installed here): stem conv/bn/relu/maxpool(3,s2,p1),
    4 stages x 2 BasicBlocks (conv3x3-bn-relu-conv3x3-bn, +identity or
    1x1-s2-conv+bn downsample, relu), avgpool, flatten, fc.  BatchNorm in eval
    mode with torch's default eps=1e-5.
It runs on torch's CPU ATen kernels exactly as the reference's CPU path does
(`scripts/streaming.py:104,126-128` runs the model on CPU), in f32 (the reference
dtype) or f64 (the accuracy yardstick).

Pinning: oracle/gen_golden.py checks this restatement against (1) the reference's own
`KeypointCNN` imported from /root/reference with `ResNet18Standin` below injected as
`torchvision.models` (pins the wrapper: conv1 swap, avgpool/fc replacement, state-dict
keys), and (2) HuggingFace transformers' independent ResNet implementation
(`transformers.ResNetModel`, layer_type="basic", depths [2,2,2,2]) with the same
weights (pins the ResNet-18 internals).  Outputs of (1) are committed as
tests/golden/detector_golden.npz.
"""

from __future__ import annotations

from collections import OrderedDict

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

BN_EPS = 1e-5


def _bn(x, sd, p):
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"],
                        sd[p + ".bias"], training=False, eps=BN_EPS)


def forward(sd: "dict[str, torch.Tensor]", x: torch.Tensor) -> torch.Tensor:
    """ResNet-18 keypoint forward on CPU: x (B,C,256,256) -> (B,2K).

    `sd` holds `resnet.*` tensors of the same dtype as x.
    """
    r = "resnet."
    h = F.conv2d(x, sd[r + "conv1.weight"], stride=2, padding=3)
    h = F.relu(_bn(h, sd, r + "bn1"))
    h = F.max_pool2d(h, kernel_size=3, stride=2, padding=1)
    for li in range(1, 5):
        for bi in range(2):
            p = f"{r}layer{li}.{bi}"
            stride = 2 if (li > 1 and bi == 0) else 1
            idn = h
            o = F.conv2d(h, sd[p + ".conv1.weight"], stride=stride, padding=1)
            o = F.relu(_bn(o, sd, p + ".bn1"))
            o = F.conv2d(o, sd[p + ".conv2.weight"], stride=1, padding=1)
            o = _bn(o, sd, p + ".bn2")
            if (p + ".downsample.0.weight") in sd:
                idn = F.conv2d(h, sd[p + ".downsample.0.weight"], stride=stride)
                idn = _bn(idn, sd, p + ".downsample.1")
            h = F.relu(o + idn)
    h = torch.flatten(F.adaptive_avg_pool2d(h, (1, 1)), 1)
    return F.linear(h, sd[r + "fc.weight"], sd[r + "fc.bias"])


def to_torch(state: "dict[str, np.ndarray]", dtype=torch.float32) -> "dict[str, torch.Tensor]":
    return {k: torch.from_numpy(np.asarray(v)).to(dtype) for k, v in state.items()
            if not k.endswith("num_batches_tracked")}


def run(state, x: np.ndarray, dtype=torch.float32, threads: int | None = None) -> np.ndarray:
    """Convenience: numpy in, numpy out (B,2K)."""
    if threads is not None:
        torch.set_num_threads(threads)
    sd = to_torch(state, dtype)
    with torch.no_grad():
        y = forward(sd, torch.from_numpy(np.ascontiguousarray(x)).to(dtype))
    return y.numpy()


def denormalize(y: np.ndarray, H: int = 256, W: int = 256) -> np.ndarray:
    """kornia.geometry.denormalize_pixel_coordinates restated (`validate.py:144-153`,
    `streaming.py:129-131`): (B,2K) normalized -> (B,K,2) px, px = (n+1)(S-1)/2."""
    y = np.asarray(y, dtype=np.float64).reshape(y.shape[0], -1, 2)
    scale = np.array([(W - 1) / 2.0, (H - 1) / 2.0])
    return (y + 1.0) * scale


def denormalize_f32(y: np.ndarray, H: int = 256, W: int = 256) -> np.ndarray:
    """kornia.geometry.conversions.denormalize_pixel_coordinates (kornia, unpinned
    version: absent here) operation for operation in f32, as validate.py:144-153 and
    streaming.py:129-131 run it on f32 model outputs:
        hw = stack([W, H]); factor = 2 / (hw - 1).clamp(eps); px = 1 / factor * (n + 1)
    (1 / f32(2/255) = 127.49999237, so this differs from 127.5 (n+1) by <= 1.6e-5 px)."""
    y = np.asarray(y, dtype=np.float32).reshape(np.shape(y)[0], -1, 2)
    hw = np.array([W, H], np.float32)
    factor = np.float32(2.0) / np.maximum(hw - np.float32(1), np.float32(1e-8))
    return (np.float32(1.0) / factor) * (y + np.float32(1.0))


# --------------------------------------------------------------------------------------
# torchvision.models stand-in (module tree with torchvision's names; no weight download).
# Used ONLY by oracle/gen_golden.py to import the reference's KeypointCNN here.
# --------------------------------------------------------------------------------------
class _Block(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        idn = x if self.downsample is None else self.downsample(x)
        o = self.relu(self.bn1(self.conv1(x)))
        o = self.bn2(self.conv2(o))
        return self.relu(o + idn)


class ResNet18Standin(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        cin = 64
        for li, cout in enumerate((64, 128, 256, 512), start=1):
            s = 1 if li == 1 else 2
            setattr(self, f"layer{li}", nn.Sequential(_Block(cin, cout, s), _Block(cout, cout, 1)))
            cin = cout
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512, 1000)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


def standin_resnet18(weights=None, **_):
    return ResNet18Standin()


def hf_resnet_forward(state, x: np.ndarray, in_ch: int = 4) -> np.ndarray:
    """Independent third-party implementation (HuggingFace transformers ResNet) with the
    same weights; fc applied on the pooled features.  f64."""
    from transformers import ResNetConfig, ResNetModel

    cfg = ResNetConfig(num_channels=in_ch, embedding_size=64, hidden_sizes=[64, 128, 256, 512],
                       depths=[2, 2, 2, 2], layer_type="basic", hidden_act="relu",
                       downsample_in_first_stage=False)
    m = ResNetModel(cfg).double().eval()
    sd = OrderedDict()

    def bn(dst, src):
        for a in ("weight", "bias", "running_mean", "running_var"):
            sd[f"{dst}.{a}"] = torch.from_numpy(np.asarray(state[f"{src}.{a}"])).double()

    sd["embedder.embedder.convolution.weight"] = torch.from_numpy(state["resnet.conv1.weight"]).double()
    bn("embedder.embedder.normalization", "resnet.bn1")
    for li in range(4):
        for bi in range(2):
            src = f"resnet.layer{li + 1}.{bi}"
            dst = f"encoder.stages.{li}.layers.{bi}"
            sd[f"{dst}.layer.0.convolution.weight"] = torch.from_numpy(state[src + ".conv1.weight"]).double()
            bn(f"{dst}.layer.0.normalization", src + ".bn1")
            sd[f"{dst}.layer.1.convolution.weight"] = torch.from_numpy(state[src + ".conv2.weight"]).double()
            bn(f"{dst}.layer.1.normalization", src + ".bn2")
            if (src + ".downsample.0.weight") in state:
                sd[f"{dst}.shortcut.convolution.weight"] = torch.from_numpy(state[src + ".downsample.0.weight"]).double()
                bn(f"{dst}.shortcut.normalization", src + ".downsample.1")
    missing, unexpected = m.load_state_dict(sd, strict=False)
    missing = [k for k in missing if not k.endswith("num_batches_tracked")]
    assert not missing and not unexpected, (missing, unexpected)
    with torch.no_grad():
        pooled = m(torch.from_numpy(x).double()).pooler_output.flatten(1)
        y = F.linear(pooled, torch.from_numpy(state["resnet.fc.weight"]).double(),
                     torch.from_numpy(state["resnet.fc.bias"]).double())
    return y.numpy()
