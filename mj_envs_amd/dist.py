"""Multi-GPU layout: one process per GPU, envs sharded in contiguous blocks.

Envs are independent: rank r owns envs [r * E, (r + 1) * E) of the global batch and keys every
Philox stream (reset draws, random actions, policy noise) by the GLOBAL env id
(``aw_set_env_offset``), so a run on N GPUs reproduces the one-GPU run of the same global batch
bit for bit.  The only collective is the episode bookkeeping exchange the reference's drivers do
on the host: every rank contributes its block's per-env totals over finished episodes (count,
summed return, successes) and all ranks receive the global vectors -- ONE all-gather of a packed
[3, E] int32 block per exchange (RCCL over xGMI on MI355X; gloo in the CPU tests).

The reference never parallelised its drivers (``mj_envs_vision/run.py:48``: "TODO: create worker
setup and parallelise"); ``launch_ranks`` is the one-process-per-GPU launcher ``bench.py --gpus N``
uses when it is not already running under ``torch.distributed.run``.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time
from dataclasses import dataclass


@dataclass
class Shard:
    rank: int
    world: int
    local_rank: int
    envs_per_rank: int

    @property
    def env_offset(self) -> int:
        """Global id of this rank's first env (Philox streams are keyed by the global id)."""
        return self.rank * self.envs_per_rank

    @property
    def total_envs(self) -> int:
        return self.world * self.envs_per_rank


def shard_from_env(envs_per_rank: int) -> Shard:
    return Shard(rank=int(os.environ.get("RANK", "0")), world=int(os.environ.get("WORLD_SIZE", "1")),
                 local_rank=int(os.environ.get("LOCAL_RANK", "0")), envs_per_rank=envs_per_rank)


def under_launcher() -> bool:
    """True inside a rank started by torch.distributed.run or by ``launch_ranks``."""
    return "WORLD_SIZE" in os.environ and "RANK" in os.environ


def stagger_phases(n: int, env_offset: int, horizon: int, seed: int = 0x5A66):
    """Per-env starting step of the first episode, a hash of the global env id modulo the horizon
    (independent of the sharding): envs then reach their horizon -- and auto-reset -- on
    different steps, so any window of steps sees every episode phase (benchmark steady state)."""
    import numpy as np
    g = (np.arange(n, dtype=np.uint64) + np.uint64(env_offset) + np.uint64(seed)) * np.uint64(0x9E3779B97F4A7C15)
    g ^= g >> np.uint64(29)
    g *= np.uint64(0xBF58476D1CE4E5B9)
    g ^= g >> np.uint64(32)
    return (g % np.uint64(max(horizon, 1))).astype(np.int32)


class EpisodeTotals:
    """Preallocated exchange of the per-env totals over finished episodes (``aw_episode_totals``):
    every finished episode is counted exactly once, whenever it ended.

    The send block is one int32 [3, E] tensor -- row 0 episode counts, row 1 the fp32 bits of the
    summed returns, row 2 successes -- whose rows ``rows()`` hands to the kernel as three contiguous
    vectors, so a rank's contribution is written in place and leaves in ONE all-gather of 12 E
    bytes per horizon (768 KiB per rank at 65 536 envs; SURVEY §5 sizes the exchange).  With
    no process group (a single process) the exchange is a local copy."""

    def __init__(self, envs_per_rank: int, world: int, device, group=None, collective: bool | None = None):
        import torch
        import torch.distributed as dist
        self.world = world
        self.envs = envs_per_rank
        self.group = group
        self.collective = (dist.is_available() and dist.is_initialized()) if collective is None else collective
        if world > 1 and not self.collective:
            raise RuntimeError("EpisodeTotals: world > 1 needs an initialised process group")
        self.send = torch.zeros(3, envs_per_rank, dtype=torch.int32, device=device)
        self.recv = torch.zeros(world, 3, envs_per_rank, dtype=torch.int32, device=device)
        self.calls = 0

    def rows(self):
        """(episodes int32, sum_return float32, successes int32) views of the send block."""
        import torch
        return self.send[0], self.send[1].view(torch.float32), self.send[2]

    @property
    def bytes_per_rank(self) -> int:
        return self.send.numel() * self.send.element_size()

    def __call__(self, episodes=None, sum_return=None, successes=None):
        """Exchange (optionally copying the given per-env vectors into the send block first) and
        return the global (episodes, sum_return, successes) vectors in global env order."""
        import torch
        import torch.distributed as dist
        e, r, s = self.rows()
        for dst, src in ((e, episodes), (r, sum_return), (s, successes)):
            if src is not None and src.data_ptr() != dst.data_ptr():
                dst.copy_(src)
        if self.collective:
            dist.all_gather_into_tensor(self.recv.view(-1), self.send.view(-1), group=self.group)
        else:
            self.recv[0].copy_(self.send)
        self.calls += 1
        g = self.recv.transpose(0, 1)                     # [3, world, E]
        return (g[0].reshape(-1), g[1].reshape(-1).view(torch.float32), g[2].reshape(-1))

    def summary(self) -> dict:
        """global episode count, mean return per finished episode, success rate (%)"""
        import torch
        e, r, s = self.recv[:, 0], self.recv[:, 1].contiguous().view(torch.float32), self.recv[:, 2]
        n = int(e.sum())
        return dict(episodes=n, mean_return=float(r.double().sum()) / max(n, 1),
                    success_pct=100.0 * int(s.sum()) / max(n, 1))


def _visible(n_phys: int) -> int:
    """devices left by the HIP / ROCr / CUDA visibility lists (the runtime applies them in turn)"""
    n = n_phys
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is None:
            continue
        ids = [x for x in v.split(",") if x.strip() != ""]
        n = min(n, len(ids))
    return n


def count_gpus() -> int:
    """GPUs this process may use, counted WITHOUT a HIP call (the launcher parent must never
    initialise the GPU it hands to its child ranks): AMD SMI's processor handles, else the KFD
    topology (nodes with SIMDs), then the visibility variables.  Raises RuntimeError when neither
    source answers -- never falls back to the HIP runtime."""
    n = None
    try:
        import amdsmi
        amdsmi.amdsmi_init()
        try:
            n = len(amdsmi.amdsmi_get_processor_handles())
        finally:
            amdsmi.amdsmi_shut_down()
    except Exception:
        n = None
    if n is None:
        root = "/sys/class/kfd/kfd/topology/nodes"
        try:
            n = 0
            for d in os.listdir(root):
                with open(os.path.join(root, d, "properties")) as f:
                    props = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
                n += int(props.get("simd_count", "0")) > 0
        except OSError:
            n = None
    if n is None:
        raise RuntimeError("count_gpus: neither AMD SMI nor the KFD topology is available")
    return _visible(n)


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(nproc: int, argv: list[str], script: str, env_extra: dict | None = None,
                 poll_s: float = 0.2) -> int:
    """Start ``nproc`` ranks of ``script`` (one process per GPU, ranks 0..nproc-1 on local devices
    0..nproc-1) with torch.distributed.run's environment contract (RANK, LOCAL_RANK, WORLD_SIZE,
    LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT) and wait for them.  The caller must not
    have touched the GPU (the ranks are children, never an exec of this process).  If a rank
    fails, the others are terminated (by their own handles) and its exit code is returned."""
    port = free_port()
    procs = []
    for r in range(nproc):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nproc),
                   LOCAL_WORLD_SIZE=str(nproc), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), **(env_extra or {}))
        procs.append(subprocess.Popen([sys.executable, script, *argv], env=env))
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in live:
                        q.terminate()
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc if rc >= 0 else 128 - rc
