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


# --- bench.py's own launcher: `--gpus N` starts N ranks itself -----------------
import json
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*argv, timeout=180):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *argv], capture_output=True,
                          text=True, timeout=timeout, env=env, cwd=REPO)


def test_bench_launcher_dry_run_world2():
    """--gpus 2 outside torchrun: two child ranks (distinct pids), env offsets 0 and E, world 2,
    and the packed [3, E] exchange delivers every rank's block in global env order."""
    E = 16
    p = _bench("--gpus", "2", "--dry-run", "--envs-per-gpu", str(E))
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1                                   # rank 0 prints the one line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "env-shard x2"
    ranks = sorted(d["ranks"], key=lambda r: r["rank"])
    assert [(r["rank"], r["local_rank"], r["world"], r["env_offset"]) for r in ranks] == [(0, 0, 2, 0), (1, 1, 2, E)]
    assert ranks[0]["pid"] != ranks[1]["pid"] and os.getpid() not in (ranks[0]["pid"], ranks[1]["pid"])
    x = d["exchange"]
    assert x["backend"] == "gloo" and x["calls"] == 1 and x["bytes_per_rank_per_call"] == 3 * 4 * E
    assert x["episodes_ok"] and x["returns_ok"] and x["successes_ok"]
    g = np.arange(2 * E)
    assert x["summary"]["episodes"] == int((g % 3).sum())


def test_bench_launcher_strong_scaling_shards():
    """--gpus 2 --total-envs 262144 (SURVEY C4's strong-scaling total): 131 072 envs per rank at
    global offsets 0 and 131 072, the exchange over both ranks' blocks."""
    p = _bench("--gpus", "2", "--dry-run", "--total-envs", "262144")
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    d = json.loads(lines[0])
    ranks = sorted(d["ranks"], key=lambda r: r["rank"])
    assert [(r["env_offset"], r["envs"]) for r in ranks] == [(0, 131072), (131072, 131072)]
    assert d["config"]["total_envs"] == 262144 and d["config"]["envs_per_gpu"] == 131072
    x = d["exchange"]
    assert x["episodes_ok"] and x["returns_ok"] and x["successes_ok"]
    assert x["bytes_per_rank_per_call"] == 3 * 4 * 131072


def test_count_gpus_without_hip(monkeypatch):
    """The launcher parent counts GPUs through AMD SMI / the KFD topology, never a HIP call, and
    applies the visibility variables; with neither source it raises instead of guessing."""
    from mj_envs_amd import dist
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1")
    assert dist._visible(8) == 2
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "3")
    assert dist._visible(8) == 1
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES")
    try:
        n = dist.count_gpus()
        assert n >= 0
    except RuntimeError as e:
        assert "neither" in str(e)
    import torch
    assert not torch.cuda.is_initialized()


def test_bench_launcher_refuses_missing_gpus():
    """Never a silent fall-back to fewer ranks: with fewer visible GPUs than --gpus it exits non-zero."""
    import torch
    n = max(2, torch.cuda.device_count() + 1)
    p = _bench("--gpus", str(n), "--steps", "1", "--warmup", "0", "--envs-per-gpu", "8")
    assert p.returncode != 0
    assert "refusing" in (p.stdout + p.stderr)


def test_launch_ranks_propagates_failure(tmp_path):
    """A failing rank's exit code is the launcher's; the other ranks are stopped."""
    from mj_envs_amd.dist import launch_ranks
    script = tmp_path / "rank.py"
    script.write_text("import os, sys, time\n"
                      "r = int(os.environ['RANK'])\n"
                      "assert os.environ['WORLD_SIZE'] == '3' and os.environ['MASTER_ADDR'] == '127.0.0.1'\n"
                      "if r == 1: sys.exit(3)\n"
                      "time.sleep(60)\n")
    import time
    t0 = time.time()
    assert launch_ranks(3, [], str(script)) == 3
    assert time.time() - t0 < 30


def test_bench_world_mismatch_refused():
    env = dict(os.environ, RANK="0", WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="1")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "4", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=REPO)
    assert p.returncode != 0 and "WORLD_SIZE" in p.stderr


@pytest.mark.gpu
def test_bench_launcher_one_gpu_rccl():
    """`bench.py --gpus 1 --launch` through the same launcher code the N-GPU run uses: one child
    rank, an RCCL process group of one, the packed episode-totals all-gather every horizon."""
    p = _bench("--gpus", "1", "--launch", "--steps", "20", "--warmup", "2", "--preroll", "200",
               "--envs-per-gpu", "4096", "--no-cpu-baseline", "--no-parity", "--no-config2", timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    print(json.dumps(dict(value=d["value"], exchange=d["exchange"], episodes=d["episodes"])))
    assert d["n_gpus"] == 1 and d["config"]["parallelism"] == "env-shard x1"
    assert d["config"]["total_envs"] == 4096 and d["value"] > 0 and d["finite"]
    x = d["exchange"]
    assert x["backend"] == "nccl" and x["collective"] == "all_gather_into_tensor" and x["world"] == 1
    assert x["calls"] == 3 and x["bytes_per_rank_per_call"] == 3 * 4 * 4096
    assert x["gathered_equals_rank_sums"]
    assert x["global_episodes"] >= 4096                   # every env ended >= 1 episode in the pre-roll
    assert 0 < d["episodes"]["finished_in_timed_window"] <= 4096


def test_bench_default_preroll_times_one_exchange():
    """whatever --warmup / --steps the driver passes, the default pre-roll puts one
    horizon boundary (the episode-totals all-gather) inside the timed window"""
    from bench import default_preroll
    for horizon in (100, 200):
        for warmup in (0, 5, 20, 300):
            for steps in (1, 2, 20, 400, 1000):
                p = default_preroll(horizon, warmup, steps)
                window = range(p + warmup, p + warmup + steps)
                assert p >= horizon
                assert any((k + 1) % horizon == 0 for k in window), (horizon, warmup, steps, p)
