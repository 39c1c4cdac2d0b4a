"""Frame sharding across GPUs: one process per GPU, weights replicated,
frames partitioned with no data-path collective; one all-gather of predicted keypoints
when a consumer needs every frame (configs[2]).

The reference has no multi-GPU inference (validate.py runs one DataLoader on one
device, validate.py:100-129); this module is the build's own partitioning:
  * `frame_range`       contiguous, balanced frame ranges (config 1: weak scaling);
  * `trajectory_range`  whole trajectories per rank, so PoseDynamicsFactor /
                        ConstantVelocityFactor pairs (factors.py:8-171) never span ranks;
  * `gather_keypoints`  ONE all_gather (RCCL over xGMI for device tensors, gloo for CPU)
                        of uneven per-rank (n_i, 2K) f32 blocks -> (sum n_i, 2K) in rank order.
"""

from __future__ import annotations

import torch
import torch.distributed as dist


def frame_range(n_frames: int, world: int, rank: int) -> tuple[int, int]:
    """[start, stop) of rank's contiguous share; sizes differ by at most one."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    q, r = divmod(n_frames, world)
    start = rank * q + min(rank, r)
    return start, start + q + (1 if rank < r else 0)


def trajectory_range(n_traj: int, traj_len: int, world: int, rank: int) -> tuple[int, int]:
    """Frame range [start, stop) holding whole trajectories t in frame_range(n_traj)."""
    t0, t1 = frame_range(n_traj, world, rank)
    return t0 * traj_len, t1 * traj_len


def shard_counts(n_frames: int, world: int, traj_len: int = 1) -> list[int]:
    """Rows every rank holds under frame_range (traj_len = 1) or trajectory_range
    (whole trajectories of traj_len frames; n_frames = trajectories x traj_len): the
    `counts` argument of gather_keypoints, known statically by every rank."""
    if traj_len > 1:
        if n_frames % traj_len:
            raise ValueError(f"{n_frames} frames is not whole trajectories of {traj_len}")
        spans = [trajectory_range(n_frames // traj_len, traj_len, world, r) for r in range(world)]
    else:
        spans = [frame_range(n_frames, world, r) for r in range(world)]
    return [b - a for a, b in spans]


def gather_keypoints(y_local: torch.Tensor, group=None, force: bool = False,
                     counts: list[int] | None = None) -> torch.Tensor:
    """All-gather (n_i, D) blocks of every rank -> (sum n_i, D), rank order.

    `counts` = every rank's n_i (shard_counts: each caller knows them from
    frame_range / trajectory_range), so the data path is exactly ONE all_gather
    (all_gather_into_tensor on RCCL): blocks are padded to the largest and trimmed
    after it.  Without `counts` they are exchanged first (a second, tiny all_gather)
    — kept only for callers whose shard sizes are data-dependent.  On device tensors
    with the nccl backend this is RCCL.  A single-rank group returns y_local unless
    `force` (tests run the collective path at world size 1, the most one GPU can host)."""
    if not dist.is_initialized() or (dist.get_world_size(group) == 1 and not force):
        return y_local
    world = dist.get_world_size(group)
    y_local = y_local.contiguous()
    if counts is None:
        n = torch.tensor([y_local.shape[0]], dtype=torch.int64, device=y_local.device)
        cts = [torch.empty_like(n) for _ in range(world)]
        dist.all_gather(cts, n, group=group)
        counts = [int(c.item()) for c in cts]
    else:
        counts = [int(c) for c in counts]
        if len(counts) != world:
            raise ValueError(f"counts has {len(counts)} entries for a world of {world}")
        me = dist.get_rank(group)
        if counts[me] != y_local.shape[0]:
            raise ValueError(f"rank {me}: counts[{me}] = {counts[me]} but the local block has {y_local.shape[0]} rows")
    nmax = max(counts)
    if y_local.shape[0] < nmax:
        pad = torch.zeros((nmax - y_local.shape[0],) + tuple(y_local.shape[1:]), dtype=y_local.dtype,
                          device=y_local.device)
        send = torch.cat([y_local, pad])
    else:
        send = y_local
    out = torch.empty((world * nmax,) + tuple(y_local.shape[1:]), dtype=y_local.dtype, device=y_local.device)
    if _has_into(y_local):
        dist.all_gather_into_tensor(out, send, group=group)
    else:
        dist.all_gather(list(out.chunk(world)), send, group=group)
    return torch.cat([out[r * nmax:r * nmax + c] for r, c in enumerate(counts)])


def _has_into(t: torch.Tensor) -> bool:
    # gloo has no all_gather_into_tensor; RCCL does (one contiguous output buffer)
    return t.device.type == "cuda" and dist.get_backend() == "nccl"
