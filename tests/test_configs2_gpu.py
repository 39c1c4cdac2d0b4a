"""configs[2] on one GPU: one rank's shard of the 24-frame x 1k-trajectory set
(shard.trajectory_range(1000, 24, 8, r) = 125 whole trajectories = 3,000 frames)
through forward + pa_trajectory_linearize, checked against the oracle, and the RCCL
branch of shard.gather_keypoints exercised on device tensors (nccl process group of
world size 1, forced through the collective)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

from oracle import factors_ref as F
from oracle import resnet_ref as R
from perseus_amd import pipeline, shard, synth
from perseus_amd.detector import KeypointCNN

pytestmark = pytest.mark.gpu
ATOL = 1e-9
FP16_PX_MAX = 0.09  # fp16 mode regression bound (test_detector_gpu.FP16_PX_MAX)


def _model(precision="fp16"):
    m = KeypointCNN(num_channels=4, precision=precision)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synthetic_state_dict(0).items()})
    return m.eval()


def test_rank_shard_3000_frames_forward_and_linearize():
    T, L, world, rank = 1000, 24, 8, 3
    f0, f1 = shard.trajectory_range(T, L, world, rank)
    n = f1 - f0
    assert (n, f0 % L) == (3000, 0)
    t_local = n // L
    # 100 distinct seeded frames tiled over the shard (generating 3,000 on the host takes
    # minutes; a 100-frame period is coprime to the library's 1024-frame chunks)
    x = torch.from_numpy(synth.synthetic_frames(4, 100, first=f0)).cuda().repeat(30, 1, 1, 1)
    m = _model()
    y = m(x)
    assert y.shape == (n, 16) and torch.isfinite(y).all()
    # sampled frames against the f64 oracle at the fp16 bound; chunk boundaries included
    idx = np.array([0, 1, 1023, 1024, 2047, 2048, n - 1])
    y64 = R.run(synth.synthetic_state_dict(0), x[idx].cpu().numpy(), torch.float64)
    d = np.abs(y[idx].cpu().numpy() - y64).reshape(len(idx), -1, 2) * 127.5
    assert np.sqrt((d ** 2).sum(-1)).max() <= FP16_PX_MAX
    # batch-invariance across the library's 1024-frame chunks
    assert torch.equal(m(x[1000:1100]), y[1000:1100])
    tr = synth.synthetic_trajectories(rank, t_local, L)
    out = pipeline.linearize_trajectories(y, tr["poses"], tr["vels"], tr["angvels"], tr["corners"], tr["K"],
                                          T=t_local, L=L, dt=1 / 12)
    z = R.denormalize_f32(y.cpu().numpy()).astype(np.float64).reshape(-1, 2)
    rng = np.random.default_rng(1)
    for i in rng.choice(n * 8, 200, replace=False):
        f, k = divmod(int(i), 8)
        r, H0, st, _ = F.projection(F.unpack(tr["poses"][f]), tr["corners"][k], z[i], tr["K"])
        assert out["status"][i].item() == st
        if st == 0:
            np.testing.assert_allclose(out["r_proj"][i].cpu().numpy(), r, atol=ATOL, rtol=0)
            np.testing.assert_allclose(out["j_proj"][i].cpu().numpy(), H0, atol=ATOL, rtol=1e-12)
    for j in rng.choice(t_local * (L - 1), 60, replace=False):
        t, l = divmod(int(j), L - 1)
        f = t * L + l
        r, H = F.dynamics(F.unpack(tr["poses"][f]), tr["angvels"][f], tr["vels"][f], F.unpack(tr["poses"][f + 1]),
                          1 / 12, "world")
        np.testing.assert_allclose(out["r_dyn"][j].cpu().numpy(), r, atol=ATOL, rtol=0)
        for q in range(4):
            np.testing.assert_allclose(out[f"j_dyn{q}"][j].cpu().numpy(), H[q], atol=ATOL, rtol=1e-12)


def test_fp16x3_batch_over_one_chunk():
    """The parity mode over a batch larger than the library's 1024-frame chunk: same bits
    per frame as a small batch, within 1e-3 px of the f64 oracle."""
    x = torch.from_numpy(synth.synthetic_frames(6, 50)).cuda().repeat(21, 1, 1, 1)  # 1050 frames
    m = _model("fp16x3")
    y = m(x)
    assert torch.equal(m(x[1020:1030]), y[1020:1030])
    idx = np.array([0, 1023, 1024, 1049])
    y64 = R.run(synth.synthetic_state_dict(0), x[idx].cpu().numpy(), torch.float64)
    assert np.abs(y[idx].cpu().numpy() - y64).max() * 127.5 <= 1e-3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_gather_keypoints_over_rccl_world_size_1():
    """shard.gather_keypoints' nccl branch on device tensors: with static counts exactly
    one all_gather_into_tensor (RCCL), without them a count exchange first; world size 1
    is the most one GPU can host, so the single-rank short-circuit is bypassed with
    force=True."""
    assert not dist.is_initialized()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        y = torch.randn(37, 16, device="cuda")
        calls = []
        orig = {n: getattr(dist, n) for n in ("all_gather", "all_gather_into_tensor")}
        for n, f in orig.items():
            setattr(dist, n, lambda *a, _f=f, _n=n, **k: (calls.append(_n), _f(*a, **k))[1])
        try:
            g = shard.gather_keypoints(y, force=True, counts=shard.shard_counts(37, 1))
            assert calls == ["all_gather_into_tensor"], calls
            g2 = shard.gather_keypoints(y, force=True)
            assert calls == ["all_gather_into_tensor", "all_gather", "all_gather_into_tensor"], calls
        finally:
            for n, f in orig.items():
                setattr(dist, n, f)
        assert g.device.type == "cuda" and torch.equal(g, y) and torch.equal(g2, y)
        assert shard.gather_keypoints(y) is y  # default single-rank short-circuit
    finally:
        dist.destroy_process_group()
