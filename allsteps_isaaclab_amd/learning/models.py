"""Actor-critic network of the Allsteps rl_games agent (``continuous_a2c_logstd`` + ``actor_critic``).

Restates rl_games 1.6.1 ``algos_torch/network_builder.py::A2CBuilder.Network`` and
``algos_torch/models.py::ModelA2CContinuousLogStd`` for the configuration the reference trains with
(``allsteps/agents/rl_games_ppo_cfg.yaml:13-35``): shared trunk (``separate: False``), MLP
[256] x 5 with ELU, linear ``mu`` (no activation), scalar value head, state-independent
``sigma`` parameter (``fixed_sigma: True``, constant 0 = log-std), PyTorch default weight init with
zero biases, obs / value running normalisers.

Module and parameter names are rl_games' (``a2c_network.actor_mlp.0.weight``, ``a2c_network.mu.bias``,
``a2c_network.sigma``, ``running_mean_std.*``, ``value_mean_std.*``) so a checkpoint written by
either trainer loads in the other.

All parameters live in ONE flat fp32 buffer (``FlatParams``): the gradient all-reduce, the norm
clip and the Adam step each touch one contiguous tensor, never a per-parameter list.
"""

from __future__ import annotations

import math

import torch
from torch import nn

from .running_mean_std import RunningMeanStd

_LOG_2PI = math.log(2.0 * math.pi)

_ACT = {"elu": nn.ELU, "relu": nn.ReLU, "tanh": nn.Tanh, "selu": nn.SELU, "None": nn.Identity, None: nn.Identity}


class A2CNetwork(nn.Module):
    """``A2CBuilder.Network`` for a flat observation, shared trunk, fixed sigma."""

    def __init__(self, obs_dim: int, actions_num: int, units=(256, 256, 256, 256, 256), activation: str = "elu",
                 sigma_init: float = 0.0, fixed_sigma: bool = True, separate: bool = False):
        super().__init__()
        if separate:
            raise NotImplementedError("separate actor / critic trunks (the Allsteps agent uses a shared trunk)")
        if not fixed_sigma:
            raise NotImplementedError("state-dependent sigma (the Allsteps agent uses fixed_sigma: True)")
        # registration order follows rl_games (sigma is a direct parameter -> first in state_dict)
        self.sigma = nn.Parameter(torch.full((actions_num,), float(sigma_init)))
        layers: list[nn.Module] = []
        n_in = obs_dim
        for u in units:
            layers += [nn.Linear(n_in, u), _ACT[activation]()]
            n_in = u
        self.actor_mlp = nn.Sequential(*layers)
        self.critic_mlp = nn.Sequential()
        self.value = nn.Linear(n_in, 1)
        self.value_act = nn.Identity()
        self.mu = nn.Linear(n_in, actions_num)
        self.mu_act = nn.Identity()
        self.sigma_act = nn.Identity()
        for m in self.modules():  # mlp_init 'default' keeps torch's init; biases zeroed (network_builder.py)
            if isinstance(m, nn.Linear) and m.bias is not None:
                nn.init.zeros_(m.bias)

    def forward(self, obs: torch.Tensor):
        out = self.actor_mlp(obs.flatten(1))
        # heads in fp32 even under fp16 / bf16 autocast: mu feeds the PPO ratio exp(old_neglogp - neglogp)
        with torch.autocast(device_type=out.device.type, enabled=False):
            out = out.float()
            value = self.value_act(self.value(out))
            mu = self.mu_act(self.mu(out))
        logstd = mu * 0.0 + self.sigma_act(self.sigma)
        return mu, logstd, value


def neglogp(x: torch.Tensor, mean: torch.Tensor, std: torch.Tensor, logstd: torch.Tensor) -> torch.Tensor:
    """ModelA2CContinuousLogStd.Network.neglogp: -log N(x; mean, std) summed over the action axis."""
    return (0.5 * (((x - mean) / std) ** 2).sum(dim=-1) + 0.5 * _LOG_2PI * x.size(-1) + logstd.sum(dim=-1))


class ModelA2CContinuousLogStd(nn.Module):
    """rl_games ``ModelA2CContinuousLogStd.Network``: normalisers around the A2C network.

    ``forward({'is_train': True, 'prev_actions': a, 'obs': o})`` -> prev_neglogp / values (normalised) /
    entropy / mus / sigmas; ``forward({'is_train': False, 'obs': o})`` -> sampled actions, neglogpacs,
    values (denormalised), mus, sigmas.
    """

    def __init__(self, obs_dim: int, actions_num: int, normalize_input: bool = True, normalize_value: bool = True,
                 **net_kwargs):
        super().__init__()
        self.a2c_network = A2CNetwork(obs_dim, actions_num, **net_kwargs)
        self.normalize_input = normalize_input
        self.normalize_value = normalize_value
        self.running_mean_std = RunningMeanStd((obs_dim,)) if normalize_input else None
        self.value_mean_std = RunningMeanStd((1,)) if normalize_value else None

    def norm_obs(self, obs: torch.Tensor) -> torch.Tensor:
        if self.running_mean_std is None:
            return obs
        with torch.no_grad():
            return self.running_mean_std(obs)

    def denorm_value(self, value: torch.Tensor) -> torch.Tensor:
        if self.value_mean_std is None:
            return value
        with torch.no_grad():
            return self.value_mean_std(value, denorm=True)

    def forward(self, input_dict: dict, generator: torch.Generator | None = None) -> dict:
        is_train = input_dict.get("is_train", True)
        obs = self.norm_obs(input_dict["obs"])
        mu, logstd, value = self.a2c_network(obs)
        sigma = torch.exp(logstd)
        if is_train:
            prev = input_dict["prev_actions"]
            entropy = (0.5 + 0.5 * _LOG_2PI + torch.log(sigma)).sum(dim=-1)  # Normal(mu, sigma).entropy()
            return {"prev_neglogp": neglogp(prev, mu, sigma, logstd), "values": value, "entropy": entropy,
                    "rnn_states": None, "mus": mu, "sigmas": sigma}
        actions = torch.normal(mu, sigma, generator=generator)
        return {"neglogpacs": neglogp(actions, mu, sigma, logstd), "values": self.denorm_value(value),
                "actions": actions, "rnn_states": None, "mus": mu, "sigmas": sigma}


class FlatParams:
    """Re-home every parameter of ``module`` (and its gradient) into one contiguous fp32 buffer.

    ``params`` / ``grads`` are the flat views; each ``p.data`` / ``p.grad`` is a view into them, so
    autograd accumulates straight into ``grads`` (zero it, never set grads to None).  ``bucket`` is
    ``grads`` followed by ``extra`` scalar slots that travel in the same collective.
    """

    def __init__(self, module: nn.Module, extra: int = 0, order: list | None = None):
        ps = [p for p in module.parameters() if p.requires_grad] if order is None else list(order)
        if order is not None and {id(p) for p in ps} != {id(p) for p in module.parameters() if p.requires_grad}:
            raise ValueError("FlatParams order must list every trainable parameter exactly once")
        n = sum(p.numel() for p in ps)
        dev = ps[0].device
        self.params = torch.empty(n, dtype=torch.float32, device=dev)
        self.bucket = torch.zeros(n + extra, dtype=torch.float32, device=dev)
        self.grads = self.bucket[:n]
        self.extra = self.bucket[n:]
        self.slices: list[tuple[int, int]] = []
        off = 0
        for p in ps:
            k = p.numel()
            self.params[off:off + k].copy_(p.data.reshape(-1))
            p.data = self.params[off:off + k].view_as(p)
            p.grad = self.grads[off:off + k].view_as(p)
            self.slices.append((off, k))
            off += k
        self.tensors = ps
        self.numel = n

    def offset(self, p: torch.Tensor) -> int:
        for q, (off, _) in zip(self.tensors, self.slices):
            if q is p:
                return off
        raise KeyError("parameter not in the flat buffer")

    def zero_grad(self) -> None:
        self.bucket.zero_()

    def rebind(self) -> None:
        """Re-point .data / .grad at the flat buffers (after load_state_dict copied into them)."""
        for p, (off, k) in zip(self.tensors, self.slices):
            if p.data.data_ptr() != self.params[off:off + k].data_ptr():
                self.params[off:off + k].copy_(p.data.reshape(-1))
                p.data = self.params[off:off + k].view_as(p)
            if p.grad is None or p.grad.data_ptr() != self.grads[off:off + k].data_ptr():
                p.grad = self.grads[off:off + k].view_as(p)


def env_signature(vec_env, obs_shape, actions_num: int) -> dict:
    """What a checkpoint's policy was trained against: observation / action sizes, the env cfg's class
    and its action_scale (the C5 task's actuator scaling) -- stored in every checkpoint so that a
    policy is never restored silently into an env whose observation layout or action scaling changed
    under the same task id."""
    uw = getattr(getattr(vec_env, "env", None), "unwrapped", None)
    cfg = getattr(uw, "cfg", None)
    sig = {"obs_dim": int(obs_shape[0]), "actions_num": int(actions_num)}
    if cfg is not None:
        sig["env_cfg"] = type(cfg).__name__
        scale = getattr(cfg, "action_scale", None)
        if scale is not None:
            sig["action_scale"] = float(scale)
    return sig


def check_env_signature(saved: dict | None, current: dict, fn: str) -> None:
    """Refuse a checkpoint whose stored env signature differs from the env it is restored into (keys
    present on both sides; checkpoints written before the signature existed are accepted)."""
    if not isinstance(saved, dict):
        return
    bad = {k: (saved[k], current[k]) for k in saved.keys() & current.keys() if saved[k] != current[k]}
    if bad:
        diff = ", ".join(f"{k}: checkpoint {a!r} vs env {b!r}" for k, (a, b) in sorted(bad.items()))
        raise ValueError(f"checkpoint {fn} was trained against another env ({diff}): its policy does not fit this task")
