"""Running mean / variance normaliser with rl_games 1.6.1 semantics.

rl_games is a third-party trainer (``rl-games==1.6.1``, ``isaaclab_rl/setup.py:46``) that is absent
from this image; this restates its ``algos_torch/running_mean_std.py::RunningMeanStd`` as the
reference agent config uses it (``normalize_input`` / ``normalize_value``,
``allsteps/agents/rl_games_ppo_cfg.yaml``):

* statistics in float64 (``running_mean``, ``running_var``, ``count`` initialised to 1);
* in training mode every forward folds the batch moments in (batch variance unbiased) with the
  parallel-variance formula, then normalises with the UPDATED statistics;
* normalise: ``clamp((x - mean) / sqrt(var + 1e-5), -5, 5)``; denormalise:
  ``sqrt(var + 1e-5) * clamp(x, -5, 5) + mean``.

The buffer names match rl_games' so checkpoints interoperate (``running_mean_std.running_mean`` ...).
Everything stays on the device: no host synchronisation.
"""

from __future__ import annotations

import torch
from torch import nn


class RunningMeanStd(nn.Module):
    def __init__(self, insize, epsilon: float = 1e-5):
        super().__init__()
        self.insize = tuple(insize) if not isinstance(insize, int) else (insize,)
        self.epsilon = epsilon
        self.axis = [0]
        self.register_buffer("running_mean", torch.zeros(self.insize, dtype=torch.float64))
        self.register_buffer("running_var", torch.ones(self.insize, dtype=torch.float64))
        self.register_buffer("count", torch.ones((), dtype=torch.float64))

    @torch.no_grad()
    def update(self, x: torch.Tensor) -> None:
        batch_mean = x.mean(self.axis)
        batch_var = x.var(self.axis)
        batch_count = x.size(0)
        delta = batch_mean - self.running_mean
        tot = self.count + batch_count
        new_mean = self.running_mean + delta * batch_count / tot
        m2 = self.running_var * self.count + batch_var * batch_count + delta ** 2 * self.count * batch_count / tot
        self.running_mean.copy_(new_mean)
        self.running_var.copy_(m2 / tot)
        self.count.copy_(tot)

    def forward(self, x: torch.Tensor, denorm: bool = False) -> torch.Tensor:
        if self.training and not denorm:
            self.update(x)
        mean = self.running_mean.float()
        std = torch.sqrt(self.running_var.float() + self.epsilon)
        if denorm:
            return std * torch.clamp(x, -5.0, 5.0) + mean
        return torch.clamp((x - mean) / std, -5.0, 5.0)
