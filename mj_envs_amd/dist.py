"""Multi-GPU layout: one process per GPU, envs sharded in contiguous blocks.

Envs are independent, so the only collective is the episode-boundary exchange the reference's
drivers do on the host: every rank contributes the returns / goal-step counts of its block and
all ranks receive the global vectors (RCCL all-gather over xGMI on MI355X; gloo on CPU tests).
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


def rank_seed(base_seed: int, rank: int) -> int:
    """Per-rank Philox key for reset draws (distinct streams per rank)."""
    return base_seed + rank


class EpisodeGather:
    """Preallocated all-gather of per-env episode returns and goal counts."""

    def __init__(self, envs_per_rank: int, world: int, device, group=None):
        import torch
        self.world = world
        self.group = group
        self.ret = torch.empty(world * envs_per_rank, dtype=torch.float32, device=device)
        self.goal = torch.empty(world * envs_per_rank, dtype=torch.int32, device=device)

    def __call__(self, last_ret, last_goal):
        import torch.distributed as dist
        if self.world == 1:
            self.ret.copy_(last_ret)
            self.goal.copy_(last_goal)
        else:
            dist.all_gather_into_tensor(self.ret, last_ret, group=self.group)
            dist.all_gather_into_tensor(self.goal, last_goal, group=self.group)
        return self.ret, self.goal

    def success_rate(self, success_steps: int) -> float:
        """Fraction of envs whose last episode had > success_steps goal steps (evaluate_success)."""
        return float((self.goal > success_steps).float().mean())
