"""Multi-rank path on CPU: gloo, world_size 2 (and 3 for uneven shards)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from perseus_amd import shard


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_frame_range_partitions():
    for n in (0, 1, 7, 64, 24000, 24001):
        for w in (1, 2, 3, 8):
            rs = [shard.frame_range(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            sizes = [b - a for a, b in rs]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard.frame_range(10, 2, 2)


def test_trajectory_range_keeps_trajectories_whole():
    L = 24
    for w in (1, 2, 3, 8):
        rs = [shard.trajectory_range(1000, L, w, r) for r in range(w)]
        assert rs[-1][1] == 24000
        for a, b in rs:
            assert a % L == 0 and b % L == 0
    assert shard.trajectory_range(1000, 24, 8, 3) == (375 * 24, 500 * 24)


def test_shard_counts_match_ranges():
    for n, w in ((128, 2), (7, 2), (10, 3), (24000, 8), (1, 2)):
        assert shard.shard_counts(n, w) == [b - a for a, b in (shard.frame_range(n, w, r) for r in range(w))]
    assert shard.shard_counts(24000, 8, traj_len=24) == [3000] * 8
    assert shard.shard_counts(240, 7, traj_len=24) == [48, 48, 48, 24, 24, 24, 24]
    with pytest.raises(ValueError):
        shard.shard_counts(25, 2, traj_len=24)


def _count_collectives():
    """Wrap every torch.distributed collective gather_keypoints could issue; returns
    the call log."""
    log = []
    for name in ("all_gather", "all_gather_into_tensor", "all_gather_object", "broadcast", "all_reduce"):
        orig = getattr(dist, name)

        def wrap(*a, _orig=orig, _name=name, **k):
            log.append(_name)
            return _orig(*a, **k)

        setattr(dist, name, wrap)
    return log


def _worker(rank, world, port, n_total, traj_len, static, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if traj_len > 1:
            a, b = shard.trajectory_range(n_total // traj_len, traj_len, world, rank)
        else:
            a, b = shard.frame_range(n_total, world, rank)
        y = torch.arange(a * 16, b * 16, dtype=torch.float32).reshape(b - a, 16)
        log = _count_collectives()
        counts = shard.shard_counts(n_total, world, traj_len=traj_len) if static else None
        g = shard.gather_keypoints(y, counts=counts)
        q.put((rank, g.shape, bool(torch.equal(g, torch.arange(n_total * 16, dtype=torch.float32)
                                                 .reshape(n_total, 16))), list(log)))
    finally:
        dist.destroy_process_group()


def _run(world, n_total, traj_len=1, static=True):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, n_total, traj_len, static, q)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    return sorted(q.get(timeout=5) for _ in range(world))


@pytest.mark.parametrize("world,n_total", [(2, 128), (2, 7), (3, 10), (2, 1)])
def test_gather_keypoints_gloo(world, n_total):
    """Static counts (the callers' form): the data path is exactly ONE collective."""
    for rank, shape, ok, log in _run(world, n_total):
        assert tuple(shape) == (n_total, 16) and ok, (rank, shape)
        assert log == ["all_gather"], (rank, log)  # gloo has no all_gather_into_tensor


@pytest.mark.parametrize("world", [2, 3])
def test_gather_trajectory_shards_one_collective(world):
    """configs[2]-shaped shards (whole 24-frame trajectories, uneven at world 3)."""
    n = 7 * 24
    for rank, shape, ok, log in _run(world, n, traj_len=24):
        assert tuple(shape) == (n, 16) and ok, (rank, shape)
        assert log == ["all_gather"], (rank, log)


def test_gather_keypoints_gloo_count_exchange():
    """Without counts (data-dependent shard sizes) the sizes are exchanged first."""
    for rank, shape, ok, log in _run(3, 10, static=False):
        assert tuple(shape) == (10, 16) and ok, (rank, shape)
        assert log == ["all_gather", "all_gather"], (rank, log)


def test_gather_rejects_wrong_counts():
    y = torch.ones(3, 16)
    assert shard.gather_keypoints(y, counts=[5, 5]) is y  # single process: no collective, no check


def test_gather_single_process_is_identity():
    y = torch.ones(3, 16)
    assert shard.gather_keypoints(y) is y
