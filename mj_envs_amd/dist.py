"""Multi-GPU layout: one process per GPU, envs sharded in contiguous blocks.

Envs are independent: rank r owns envs [r * E, (r + 1) * E) of the global batch and keys every
Philox stream (reset draws, random actions, policy noise) by the GLOBAL env id
(``aw_set_env_offset``), so a run on N GPUs reproduces the one-GPU run of the same global batch
bit for bit.  The only collective is the episode bookkeeping exchange the reference's drivers do
on the host: every rank contributes its block's per-env totals over finished episodes (count,
summed return, successes) and all ranks receive the global vectors (RCCL all-gather over xGMI on
MI355X; gloo in the CPU tests).
"""
from __future__ import annotations

import os
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
    """Preallocated all-gather of the per-env totals over finished episodes
    (``aw_episode_totals``): every finished episode is counted exactly once, whenever it ended."""

    def __init__(self, envs_per_rank: int, world: int, device, group=None):
        import torch
        self.world = world
        self.group = group
        self.episodes = torch.zeros(world * envs_per_rank, dtype=torch.int32, device=device)
        self.sum_return = torch.zeros(world * envs_per_rank, dtype=torch.float32, device=device)
        self.successes = torch.zeros(world * envs_per_rank, dtype=torch.int32, device=device)

    def __call__(self, episodes, sum_return, successes):
        import torch.distributed as dist
        if self.world == 1:
            self.episodes.copy_(episodes)
            self.sum_return.copy_(sum_return)
            self.successes.copy_(successes)
        else:
            dist.all_gather_into_tensor(self.episodes, episodes, group=self.group)
            dist.all_gather_into_tensor(self.sum_return, sum_return, group=self.group)
            dist.all_gather_into_tensor(self.successes, successes, group=self.group)
        return self.episodes, self.sum_return, self.successes

    def summary(self) -> dict:
        """global episode count, mean return per finished episode, success rate (%)"""
        n = int(self.episodes.sum())
        return dict(episodes=n, mean_return=float(self.sum_return.double().sum()) / max(n, 1),
                    success_pct=100.0 * int(self.successes.sum()) / max(n, 1))
