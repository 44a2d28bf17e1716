"""On-device Gaussian MLP policy.

Restates mjrl's ``gaussian_mlp.MLP`` (third-party, unpinned git master), which the reference's
DAPG baseline builds as ``MLP(env_spec, hidden_sizes=(32, 32), seed=seed, init_log_std=-1.0)``
(``mj_envs_vision/algos/baselines.py:67-70``) and queries with ``get_action(obs)``
(``:82-86``: ``[1]['evaluation']`` = the mean for ``act``, ``[0]`` = mean + exp(log_std) N(0,1)
for ``sample_action``).  Network (mjrl ``FCNetwork``): ``(obs - in_shift) / (in_scale + 1e-8)``,
tanh hidden layers, linear output, ``* out_scale + out_shift``; at construction the seed is
applied with ``torch.manual_seed``, layers take torch's ``nn.Linear`` default init, and the last
layer's weight and bias are scaled by 1e-2.

The forward pass runs in the HIP kernel ``k_mlp`` (``aw_policy_mlp``, one thread per env).
``GaussianMLP.from_npz`` loads the reference's pretrained DAPG policies
(``algos/dapg_pretrained/*.pickle``) from the inert fixtures ``tests/golden/dapg_<task>.npz``
that ``tests/golden/make_dapg.py`` extracted WITHOUT unpickling (opcode-level data walk, tensors
through ``torch.load(weights_only=True)``): hammer / door / relocate 32x32, pen 64x64.
"""
from __future__ import annotations

import ctypes
from typing import Sequence

import numpy as np

from . import _native


class GaussianMLP:
    def __init__(self, obs_dim: int, act_dim: int, hidden_sizes: Sequence[int] = (32, 32),
                 init_log_std: float = -1.0, seed: int | None = None, device: int = 0):
        import torch
        hs = tuple(hidden_sizes)
        if len(hs) != 2 or hs[0] != hs[1] or hs[0] not in (32, 64):
            raise ValueError("aw_policy_mlp supports two equal hidden layers of width 32 or 64")
        self.obs_dim, self.act_dim, self.hidden = obs_dim, act_dim, hs[0]
        if seed is not None:
            torch.manual_seed(seed)
            np.random.seed(seed)
        sizes = (obs_dim,) + hs + (act_dim,)
        layers = [torch.nn.Linear(sizes[i], sizes[i + 1]) for i in range(len(sizes) - 1)]
        with torch.no_grad():
            layers[-1].weight.mul_(1e-2)
            layers[-1].bias.mul_(1e-2)
        self.weights = [(l.weight.detach().double().numpy(), l.bias.detach().double().numpy()) for l in layers]
        self.in_shift = np.zeros(obs_dim)
        self.in_scale = np.ones(obs_dim)
        self.out_shift = np.zeros(act_dim)
        self.out_scale = np.ones(act_dim)
        self.log_std = np.full(act_dim, float(init_log_std))
        self.device = device
        self._dev = None
        self.upload()

    @classmethod
    def from_npz(cls, path: str, device: int = 0) -> "GaussianMLP":
        """Pretrained weights (``W0 b0 W1 b1 W2 b2`` in nn.Linear [out, in] layout, ``in_shift
        in_scale out_shift out_scale log_std``), e.g. tests/golden/dapg_hammer.npz."""
        d = np.load(path, allow_pickle=False)
        sizes = tuple(int(x) for x in d["layer_sizes"])
        self = cls.__new__(cls)
        self.obs_dim, self.act_dim = sizes[0], sizes[-1]
        hs = sizes[1:-1]
        if len(hs) != 2 or hs[0] != hs[1] or hs[0] not in (32, 64):
            raise ValueError(f"aw_policy_mlp supports two equal hidden layers of width 32 or 64, got {hs}")
        self.hidden = hs[0]
        self.weights = [(np.asarray(d[f"W{i}"], np.float64), np.asarray(d[f"b{i}"], np.float64)) for i in range(3)]
        for k in ("in_shift", "in_scale", "out_shift", "out_scale", "log_std"):
            setattr(self, k, np.asarray(d[k], np.float64))
        self.device = device
        self._dev = None
        self.upload()
        return self

    def mean_np(self, obs: np.ndarray) -> np.ndarray:
        """fp64 host forward of the mean (mjrl FCNetwork.forward), for checks."""
        (W0, b0), (W1, b1), (W2, b2) = self.weights
        x = (np.asarray(obs, np.float64) - self.in_shift) / (self.in_scale + 1e-8)
        x = np.tanh(x @ W0.T + b0)
        x = np.tanh(x @ W1.T + b1)
        return (x @ W2.T + b2) * self.out_scale + self.out_shift

    def flat_params(self) -> np.ndarray:
        """Parameter block in the aw_policy_mlp layout (aw_policy.h)."""
        (W0, b0), (W1, b1), (W2, b2) = self.weights
        parts = [self.in_shift, self.in_scale, W0.ravel(), b0, W1.ravel(), b1, W2.ravel(), b2,
                 self.out_scale, self.out_shift, self.log_std]
        return np.concatenate([np.asarray(p, np.float64).ravel() for p in parts]).astype(np.float32)

    def upload(self):
        import torch
        self._dev = torch.tensor(self.flat_params(), device=torch.device("cuda", self.device))

    def act(self, obs, out=None, sample: bool = False, seed: int = 0, step: int = 0, env_offset: int = 0):
        """actions [n, act_dim] (device) from obs [n, obs_dim] (device fp32): the mean, or with
        sample=True mean + exp(log_std) * N(0, 1) from Philox (seed, (env_offset + env, step))."""
        import torch
        n = obs.shape[0]
        assert obs.shape[1] == self.obs_dim and obs.is_contiguous() and obs.dtype == torch.float32
        if out is None:
            out = torch.empty(n, self.act_dim, dtype=torch.float32, device=obs.device)
        L = _native.load()
        _native._check(L.aw_policy_mlp(n, self.obs_dim, self.hidden, self.act_dim, self._dev.data_ptr(),
                                       obs.data_ptr(), out.data_ptr(), int(sample), ctypes.c_uint64(seed),
                                       ctypes.c_uint64(step), ctypes.c_uint64(env_offset), _native._stream()))
        return out
