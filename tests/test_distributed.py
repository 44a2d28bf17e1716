"""world_size-2 gloo test of the multi-GPU episode exchange (CPU; the GPU run uses RCCL)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mj_envs_amd.dist import EpisodeGather, Shard, rank_seed


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sh = Shard(rank=rank, world=world, local_rank=rank, envs_per_rank=n)
        g = EpisodeGather(n, world, "cpu")
        ret = torch.arange(n, dtype=torch.float32) + 1000 * rank
        goal = torch.full((n,), 10 * (rank + 1), dtype=torch.int32)
        r, gl = g(ret, goal)
        q.put((rank, sh.env_offset, rank_seed(1, rank), r.tolist(), gl.tolist(), g.success_rate(15)))
    finally:
        dist.destroy_process_group()


def test_episode_gather_world2():
    world, n = 2, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort()
    expect_ret = [float(i) for i in range(n)] + [1000.0 + i for i in range(n)]
    for rank, off, seed, r, gl, sr in out:
        assert off == rank * n
        assert seed == 1 + rank
        assert r == expect_ret                      # every rank sees the global vector, rank order
        assert gl == [10] * n + [20] * n
        assert sr == pytest.approx(0.5)             # rank 1's envs (20 goal steps) exceed 15


def test_single_rank_gather_is_copy():
    g = EpisodeGather(3, 1, "cpu")
    r, gl = g(torch.tensor([1.0, 2.0, 3.0]), torch.tensor([0, 30, 26], dtype=torch.int32))
    assert r.tolist() == [1.0, 2.0, 3.0]
    assert g.success_rate(25) == pytest.approx(2 / 3)
