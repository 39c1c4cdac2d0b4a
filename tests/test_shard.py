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


def _worker(rank, world, port, n_total, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        a, b = shard.frame_range(n_total, world, rank)
        y = torch.arange(a * 16, b * 16, dtype=torch.float32).reshape(b - a, 16)
        g = shard.gather_keypoints(y)
        q.put((rank, g.shape, bool(torch.equal(g, torch.arange(n_total * 16, dtype=torch.float32)
                                                 .reshape(n_total, 16)))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_total", [(2, 128), (2, 7), (3, 10), (2, 1)])
def test_gather_keypoints_gloo(world, n_total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=5) for _ in range(world))
    for rank, shape, ok in res:
        assert tuple(shape) == (n_total, 16) and ok, (rank, shape)


def test_gather_single_process_is_identity():
    y = torch.ones(3, 16)
    assert shard.gather_keypoints(y) is y
