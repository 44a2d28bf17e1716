"""world_size-2 gloo tests of the multi-GPU layout (CPU; the GPU run uses RCCL over xGMI)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mj_envs_amd.dist import EpisodeTotals, Shard, stagger_phases


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
        g = EpisodeTotals(n, world, "cpu")
        # rank r: env i finished (i % 3) episodes, returns 1000 r + i each, successes of rank 1's
        ep = torch.tensor([i % 3 for i in range(n)], dtype=torch.int32)
        ret = ep.float() * (torch.arange(n, dtype=torch.float32) + 1000 * rank)
        suc = ep if rank == 1 else torch.zeros(n, dtype=torch.int32)
        e, r, s = g(ep, ret, suc)
        ph = stagger_phases(n, sh.env_offset, 200)
        q.put((rank, sh.env_offset, e.tolist(), r.tolist(), s.tolist(), g.summary(), ph.tolist()))
    finally:
        dist.destroy_process_group()


def test_episode_totals_world2():
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
    ep = [i % 3 for i in range(n)] * 2
    ret = [float((i % 3) * i) for i in range(n)] + [float((i % 3) * (1000 + i)) for i in range(n)]
    one = stagger_phases(world * n, 0, 200).tolist()       # the unsharded batch
    for rank, off, e, r, s, summ, ph in out:
        assert off == rank * n
        assert e == ep and r == ret                          # every rank sees the global vectors
        assert s == [0] * n + [i % 3 for i in range(n)]
        assert summ["episodes"] == sum(ep)
        assert summ["success_pct"] == pytest.approx(50.0)
        assert summ["mean_return"] == pytest.approx(sum(ret) / sum(ep))
        assert ph == one[rank * n:(rank + 1) * n]            # phases keyed by the global env id


def test_single_rank_totals_is_copy():
    g = EpisodeTotals(3, 1, "cpu")
    e, r, s = g(torch.tensor([1, 2, 0], dtype=torch.int32), torch.tensor([1.0, 2.0, 0.0]),
                torch.tensor([1, 0, 0], dtype=torch.int32))
    assert e.tolist() == [1, 2, 0] and r.tolist() == [1.0, 2.0, 0.0]
    assert g.summary()["success_pct"] == pytest.approx(100 / 3)


def test_stagger_phases_cover_horizon():
    ph = stagger_phases(65536, 0, 200)
    assert ph.min() == 0 and ph.max() == 199
    counts = np.bincount(ph, minlength=200)
    assert counts.min() > 0.8 * 65536 / 200 and counts.max() < 1.2 * 65536 / 200
