"""PPO agent for Allsteps-v0 with rl_games 1.6.1 ``a2c_continuous`` semantics, MI355X-first.

rl_games is third-party (``rl-games==1.6.1``, ``isaaclab_rl/setup.py:46``) and absent from this image;
the reference trains Allsteps with it through ``scripts/reinforcement_learning/rl_games/train.py:157-178``
and ``allsteps/learning/a2c_ppo_mirroring.py:5-37``.  This module restates
the parts of ``common/a2c_common.py`` (``A2CBase`` / ``ContinuousA2CBase``) and
``algos_torch/a2c_continuous.py`` (``A2CAgent``) that the reference config
(``allsteps/agents/rl_games_ppo_cfg.yaml``) exercises -- parity unpinned (no rl_games output exists
offline); the unit tests check each formula against an independent statement:

* rollout: ``horizon_length`` steps of (policy sample -> ``vec_env.step``), rewards shaped by
  ``scale_value``, ``value_bootstrap`` adds ``gamma * V(s) * time_out``; initial dones = 1;
* GAE(``gamma``, ``tau``) with rl_games' done convention (``mb_dones[t]`` = done flag of the obs at t);
* dataset: returns / values normalised by the value normaliser (train mode, both calls update it),
  advantages standardised; minibatches are contiguous slices of the env-major flattened batch
  (``PPODataset``, no shuffle), ``mu`` / ``sigma`` written back per minibatch (``update_mu_sigma``);
* loss ``a_loss + 0.5 critic_coef c_loss - entropy_coef H + bounds_loss_coef b_loss`` with clipped
  ratio, clipped value loss (``clip_value``), soft bound loss at +-1.1;
* obs normaliser updated by the train-mode forwards of the FIRST mini-epoch only;
* Adam (eps 1e-8), grad-norm clip ``grad_norm``, adaptive LR (``kl_threshold``; x1.5 / /1.5 within
  [1e-6, 1e-2]) after EVERY minibatch (``schedule_type: legacy``) from the rank-averaged KL.

MI355X-specific design (no change of the maths):

* No host synchronisation in the training loop: episode statistics (``AverageMeter``), the KL and
  the adaptive learning rate live on the device (rl_games calls ``.item()`` / ``nonzero`` several
  times per minibatch); the host only reads the statistics once per epoch for the log line.
* Parameters and gradients in ONE flat fp32 buffer (``FlatParams``): the multi-GPU gradient
  exchange is ONE RCCL all-reduce per minibatch of [grads | kl] (rl_games: a cat + all-reduce +
  per-parameter copy, then a second all-reduce + broadcast for the KL / LR), the norm clip is one
  reduction and Adam one pass over the buffer.
* ``mixed_precision``: as rl_games, fp16 autocast for the 256-wide trunk GEMMs (MFMA) with
  ``torch.cuda.amp.GradScaler``'s dynamic loss scale (2^16, x2 after 2000 good steps, x0.5 and the
  step skipped on a non-finite gradient) held on the device, so no host sync is added; the mu / value
  heads run in fp32 (a 16-bit mu would put ~0.4 % noise into the PPO ratio).  ``mixed_precision_dtype:
  bfloat16`` selects bf16 instead.
* Multi-GPU: ``multi_gpu_mode: allreduce`` (default, rl_games ``multi_gpu`` semantics: per-rank
  minibatches, averaged gradients) or ``allgather`` (BASELINE north star: the rollout tensors of all
  ranks are all-gathered over RCCL at the PPO boundary and every rank runs the identical update on
  the global batch with a world-size-scaled minibatch; no gradient exchange).
"""

from __future__ import annotations

import math
import os
import time

import torch
import torch.distributed as dist

from .fused import SCALER_GROWTH_INTERVAL, SCALER_INIT
from .models import FlatParams, ModelA2CContinuousLogStd, check_env_signature, env_signature


def fused_param_order(model) -> list:
    """Flat-buffer order for the fused step: trunk (W, b per layer), [mu.w | value.w] as one 22 x 256
    head matrix, [mu.b | value.b], sigma."""
    net = model.a2c_network
    order = []
    for m in net.actor_mlp:
        if isinstance(m, torch.nn.Linear):
            order += [m.weight, m.bias]
    return order + [net.mu.weight, net.value.weight, net.mu.bias, net.value.bias, net.sigma]

# ------------------------------------------------------------------------------------------------
# helpers (rl_games common/*)


def swap_and_flatten01(arr: torch.Tensor) -> torch.Tensor:
    """(H, N, ...) -> (N * H, ...), env-major (a2c_common.swap_and_flatten01)."""
    s = arr.size()
    return arr.transpose(0, 1).reshape(s[0] * s[1], *s[2:])


def policy_kl(p0_mu, p0_sigma, p1_mu, p1_sigma, reduce: bool = True):
    """torch_ext.policy_kl."""
    c1 = torch.log(p1_sigma / p0_sigma + 1e-5)
    c2 = (p0_sigma ** 2 + (p1_mu - p0_mu) ** 2) / (2.0 * (p1_sigma ** 2 + 1e-5))
    kl = (c1 + c2 - 0.5).sum(dim=-1)
    return kl.mean() if reduce else kl


def actor_loss(old_neglogp, neglogp, advantage, is_ppo: bool, e_clip: float):
    """common_losses.actor_loss."""
    if not is_ppo:
        return neglogp * advantage
    ratio = torch.exp(old_neglogp - neglogp)
    surr1 = advantage * ratio
    surr2 = advantage * torch.clamp(ratio, 1.0 - e_clip, 1.0 + e_clip)
    return torch.max(-surr1, -surr2)


def critic_loss(value_preds, values, e_clip: float, returns, clip_value: bool):
    """common_losses.critic_loss."""
    if clip_value:
        clipped = value_preds + (values - value_preds).clamp(-e_clip, e_clip)
        return torch.max((values - returns) ** 2, (clipped - returns) ** 2)
    return (returns - values) ** 2


def bound_loss(mu, soft_bound: float = 1.1):
    """A2CAgent.bound_loss."""
    return (torch.clamp_max(mu + soft_bound, 0.0) ** 2 + torch.clamp_min(mu - soft_bound, 0.0) ** 2).sum(dim=-1)


class RewardsShaper:
    """tr_helpers.DefaultRewardsShaper."""

    def __init__(self, scale_value=1.0, shift_value=0.0, min_val=-math.inf, max_val=math.inf, is_torch=True):
        self.scale_value, self.shift_value, self.min_val, self.max_val = scale_value, shift_value, min_val, max_val

    def __call__(self, reward):
        reward = (reward + self.shift_value) * self.scale_value
        if self.min_val != -math.inf or self.max_val != math.inf:
            reward = torch.clamp(reward, self.min_val, self.max_val)
        return reward


class AverageMeter:
    """torch_ext.AverageMeter (mean of the last ``max_size`` finished episodes), kept on the device:
    ``update(values, mask)`` folds in the masked rows without a host round trip (rl_games indexes with
    ``dones.nonzero()``)."""

    def __init__(self, in_shape: int, max_size: int, device):
        self.max_size = max_size
        self.mean = torch.zeros(in_shape, dtype=torch.float32, device=device)
        self.current_size = torch.zeros((), dtype=torch.float32, device=device)

    def update(self, values: torch.Tensor, mask: torch.Tensor) -> None:
        m = mask.float()
        size = m.sum()
        v = values.float().reshape(values.shape[0], -1)
        new_mean = (v * m[:, None]).sum(0) / size.clamp_min(1.0)
        size = size.clamp(0, self.max_size)
        old_size = torch.minimum(self.max_size - size, self.current_size)
        size_sum = old_size + size
        upd = size > 0
        self.mean.copy_(torch.where(upd, (self.mean * old_size + new_mean * size) / size_sum.clamp_min(1.0),
                                    self.mean))
        self.current_size.copy_(torch.where(upd, size_sum, self.current_size))

    def clear(self) -> None:
        self.mean.zero_()
        self.current_size.zero_()

    def get_mean(self):
        return self.mean.cpu().numpy()


class AdaptiveScheduler:
    """schedulers.AdaptiveScheduler on a device fp64 scalar (no .item() per minibatch)."""

    def __init__(self, kl_threshold: float = 0.008, min_lr: float = 1e-6, max_lr: float = 1e-2):
        self.kl_threshold, self.min_lr, self.max_lr = kl_threshold, min_lr, max_lr

    def update_(self, lr: torch.Tensor, kl: torch.Tensor) -> None:
        k = kl.to(lr.dtype)
        new = torch.where(k > 2.0 * self.kl_threshold, torch.clamp_min(lr / 1.5, self.min_lr), lr)
        new = torch.where(k < 0.5 * self.kl_threshold, torch.clamp_max(lr * 1.5, self.max_lr), new)
        lr.copy_(new)


class IdentityScheduler:
    def update_(self, lr, kl) -> None:
        pass


class FlatAdam:
    """torch.optim.Adam (amsgrad off, weight_decay 0) over one flat parameter buffer with a device-side
    learning rate and step count: bias corrections, step size and update are device ops, so the step
    never synchronises and can be captured in a HIP graph."""

    def __init__(self, flat: FlatParams, lr: torch.Tensor, betas=(0.9, 0.999), eps: float = 1e-8):
        self.flat = flat
        self.lr = lr
        self.beta1, self.beta2 = betas
        self.eps = eps
        self.exp_avg = torch.zeros_like(flat.params)
        self.exp_avg_sq = torch.zeros_like(flat.params)
        self.step_t = torch.zeros((), dtype=torch.float64, device=flat.params.device)

    @torch.no_grad()
    def step(self) -> None:
        g, p = self.flat.grads, self.flat.params
        self.step_t += 1
        self.exp_avg.lerp_(g, 1.0 - self.beta1)
        self.exp_avg_sq.mul_(self.beta2).addcmul_(g, g, value=1.0 - self.beta2)
        bc1 = 1.0 - torch.pow(self.beta1, self.step_t)
        bc2_sqrt = torch.sqrt(1.0 - torch.pow(self.beta2, self.step_t))
        step_size = (self.lr / bc1).float()
        denom = (self.exp_avg_sq.sqrt() / bc2_sqrt.float()).add_(self.eps)
        p.sub_(step_size * (self.exp_avg / denom))

    def state_dict(self) -> dict:
        return {"exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq, "step": self.step_t, "lr": self.lr}

    def load_state_dict(self, sd: dict) -> None:
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        self.step_t.copy_(sd["step"])
        self.lr.copy_(sd["lr"])


class PPODataset:
    """datasets.PPODataset (non-recurrent): minibatch i = rows [i m, (i + 1) m) of the flat batch."""

    def __init__(self, batch_size: int, minibatch_size: int):
        if batch_size % minibatch_size:
            raise ValueError(f"batch size {batch_size} is not a multiple of minibatch_size {minibatch_size}")
        self.batch_size, self.minibatch_size = batch_size, minibatch_size
        self.length = batch_size // minibatch_size
        self.values_dict: dict | None = None
        self.last_range = (0, 0)

    def update_values_dict(self, values_dict) -> None:
        self.values_dict = values_dict

    def update_mu_sigma(self, mu, sigma) -> None:
        s, e = self.last_range
        self.values_dict["mu"][s:e] = mu
        self.values_dict["sigma"][s:e] = sigma

    def __len__(self) -> int:
        return self.length

    def __getitem__(self, idx: int) -> dict:
        s, e = idx * self.minibatch_size, (idx + 1) * self.minibatch_size
        self.last_range = (s, e)
        return {k: v[s:e] for k, v in self.values_dict.items() if v is not None}


class DefaultAlgoObserver:
    """rl_games.common.algo_observer.DefaultAlgoObserver surface (hooks are no-ops)."""

    def before_init(self, base_name, config, experiment_name):
        pass

    def after_init(self, algo):
        self.algo = algo

    def process_infos(self, infos, done_indices):
        pass

    def after_steps(self):
        pass

    def after_print_stats(self, frame, epoch_num, total_time):
        pass


# ------------------------------------------------------------------------------------------------


class A2CAgent:
    """rl_games ``A2CAgent(base_name, params)`` for a continuous action space."""

    def __init__(self, base_name: str, params: dict):
        from ..rl_games import vecenv

        self.params = params
        self.config = config = params["config"]
        self.base_name = base_name
        self.name = config.get("name", base_name)
        self.ppo = config.get("ppo", True)
        self.multi_gpu = bool(config.get("multi_gpu", False))
        self.rank, self.world_size, self.local_rank = 0, 1, 0
        if self.multi_gpu:
            from ..distributed import init_process_group

            info = init_process_group()
            self.rank, self.world_size, self.local_rank = info.rank, info.world, info.local_rank
            if torch.cuda.is_available():
                config["device"] = f"cuda:{self.local_rank}"
        self.multi_gpu_mode = config.get("multi_gpu_mode", "allreduce")
        if self.multi_gpu_mode not in ("allreduce", "allgather"):
            raise ValueError(f"multi_gpu_mode must be 'allreduce' or 'allgather', got {self.multi_gpu_mode!r}")
        self.device = torch.device(config.get("device", "cuda:0"))
        self.ppo_device = self.device
        self.env_name = config["env_name"]
        self.num_actors = int(config["num_actors"])
        self.env_config = config.get("env_config", {})
        self.vec_env = config.get("vec_env") or vecenv.create_vec_env(self.env_name, self.num_actors,
                                                                       **self.env_config)
        self.env_info = self.vec_env.get_env_info()
        self.obs_shape = tuple(self.env_info["observation_space"].shape)
        action_space = self.env_info["action_space"]
        self.actions_num = int(action_space.shape[0])
        self.actions_low = torch.as_tensor(action_space.low, dtype=torch.float32, device=self.device)
        self.actions_high = torch.as_tensor(action_space.high, dtype=torch.float32, device=self.device)
        self.clip_actions = bool(config.get("clip_actions", True))
        self._unit_box = bool(torch.all(self.actions_low == -1.0) and torch.all(self.actions_high == 1.0))
        self.num_agents = int(self.env_info.get("agents", 1))
        self.value_size = int(self.env_info.get("value_size", 1))

        self.horizon_length = int(config["horizon_length"])
        self.batch_size = self.horizon_length * self.num_actors * self.num_agents
        self.batch_size_envs = self.horizon_length * self.num_actors
        self.minibatch_size = int(config.get("minibatch_size", self.num_actors * config.get("minibatch_size_per_env", 0)))
        self.mini_epochs_num = int(config["mini_epochs"])
        self.gamma = float(config["gamma"])
        self.tau = float(config["tau"])
        self.e_clip = float(config["e_clip"])
        self.clip_value = bool(config.get("clip_value", False))
        self.critic_coef = float(config["critic_coef"])
        self.entropy_coef = float(config["entropy_coef"])
        self.bounds_loss_coef = config.get("bounds_loss_coef", None)
        self.bound_loss_type = config.get("bound_loss_type", "bound")
        self.grad_norm = float(config.get("grad_norm", 1.0))
        self.truncate_grads = bool(config.get("truncate_grads", False))
        self.normalize_advantage = bool(config["normalize_advantage"])
        self.normalize_input = bool(config["normalize_input"])
        self.normalize_value = bool(config.get("normalize_value", False))
        self.value_bootstrap = bool(config.get("value_bootstrap", False))
        self.mixed_precision = bool(config.get("mixed_precision", False)) and self.device.type == "cuda"
        mpd = config.get("mixed_precision_dtype", "float16")
        if mpd not in ("float16", "bfloat16"):
            raise ValueError(f"mixed_precision_dtype must be float16 or bfloat16, got {mpd!r}")
        self.mixed_precision_dtype = torch.float16 if mpd == "float16" else torch.bfloat16
        # GradScaler(enabled=mixed_precision) state on the device: [scale, growth tracker].  `grad_scaler:
        # False` (not an rl_games key; a measurement knob) runs the 16-bit trunk unscaled
        self.scaler_state = (torch.tensor([SCALER_INIT, 0.0], device=self.device)
                             if self.mixed_precision and bool(config.get("grad_scaler", True)) else None)
        self.max_epochs = int(config.get("max_epochs", -1))
        self.save_freq = int(config.get("save_frequency", 0))
        self.save_best_after = int(config.get("save_best_after", 100))
        self.print_stats = bool(config.get("print_stats", True)) and self.rank == 0
        self.score_to_win = config.get("score_to_win", math.inf)
        self.games_to_track = int(config.get("games_to_track", 100))
        rs = config.get("reward_shaper", {}) or {}
        self.rewards_shaper = RewardsShaper(**rs)
        self.schedule_type = config.get("schedule_type", "legacy")
        if config.get("lr_schedule") == "adaptive":
            self.scheduler = AdaptiveScheduler(float(config.get("kl_threshold", 0.008)))
        else:
            self.scheduler = IdentityScheduler()
        self.train_dir = config.get("train_dir", "runs")
        self.experiment_name = config.get("full_experiment_name", self.name)
        self.experiment_dir = os.path.join(self.train_dir, self.experiment_name)
        self.nn_dir = os.path.join(self.experiment_dir, "nn")

        net = params["network"]
        mlp = net.get("mlp", {})
        space = net.get("space", {}).get("continuous", {})
        sigma_init = space.get("sigma_init", {})
        self.model = ModelA2CContinuousLogStd(
            self.obs_shape[0], self.actions_num, normalize_input=self.normalize_input,
            normalize_value=self.normalize_value, units=tuple(mlp.get("units", (256, 256, 256, 256, 256))),
            activation=mlp.get("activation", "elu"),
            sigma_init=float(sigma_init.get("val", 0.0)) if sigma_init.get("name") == "const_initializer" else 0.0,
            fixed_sigma=bool(space.get("fixed_sigma", True)), separate=bool(net.get("separate", False)),
        ).to(self.device)
        # fused HIP-graph minibatch step (learning/fused.py) on the device; autograd path elsewhere
        self.fused_update = bool(config.get("fused_update", self.device.type == "cuda"))
        order = fused_param_order(self.model) if self.fused_update else None
        self.flat = FlatParams(self.model, extra=1, order=order)  # [grads | kl]: one collective per minibatch
        self._bucket, self._kl_slot = self.flat.bucket, self.flat.extra
        self.last_lr = float(config["learning_rate"])
        self.lr = torch.tensor(self.last_lr, dtype=torch.float64, device=self.device)
        self.optimizer = FlatAdam(self.flat, self.lr, eps=1e-8)

        self.algo_observer = params.get("algo_observer") or DefaultAlgoObserver()
        self.epoch_num = 0
        self.frame = 0
        self.last_mean_rewards = -100500.0
        self.rnn_states = None
        self.is_rnn = False
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(int(params.get("seed", 0)) + 7919 * self.rank)
        self.algo_observer.after_init(self)

    # ------------------------------------------------------------------ tensors
    def init_tensors(self) -> None:
        H, N, dev = self.horizon_length, self.num_actors * self.num_agents, self.device
        A = self.actions_num
        self.tensor_dict = {
            "obses": torch.zeros((H, N) + self.obs_shape, device=dev),
            "rewards": torch.zeros(H, N, self.value_size, device=dev),
            "values": torch.zeros(H, N, self.value_size, device=dev),
            "neglogpacs": torch.zeros(H, N, device=dev),
            "dones": torch.zeros(H, N, dtype=torch.uint8, device=dev),
            "actions": torch.zeros(H, N, A, device=dev),
            "mus": torch.zeros(H, N, A, device=dev),
            "sigmas": torch.zeros(H, N, A, device=dev),
        }
        self.tensor_list = ["actions", "neglogpacs", "values", "mus", "sigmas", "obses", "dones"]
        self.current_rewards = torch.zeros(N, self.value_size, device=dev)
        self.current_shaped_rewards = torch.zeros(N, self.value_size, device=dev)
        self.current_lengths = torch.zeros(N, device=dev)
        self.dones = torch.ones(N, dtype=torch.uint8, device=dev)
        self.game_rewards = AverageMeter(self.value_size, self.games_to_track, dev)
        self.game_shaped_rewards = AverageMeter(self.value_size, self.games_to_track, dev)
        self.game_lengths = AverageMeter(1, self.games_to_track, dev)
        world_mb = self.world_size if (self.multi_gpu and self.multi_gpu_mode == "allgather") else 1
        self.dataset = PPODataset(self.batch_size * world_mb, self.minibatch_size * world_mb)
        self._play_graphs = None
        uw = getattr(getattr(self.vec_env, "env", None), "unwrapped", None)
        if self.fused_update and self.config.get("rollout_graphs", True) and getattr(uw, "graph_safe_step", False):
            # one HIP graph per rollout step index: policy forward + sampling + env step + bookkeeping
            uw.set_graph_capture(True)
            self._uw = uw
            self._play_graphs = {}
            self._obs_buf = torch.zeros((N,) + self.obs_shape, device=dev)
            self._dones_buf = torch.ones(N, dtype=torch.uint8, device=dev)
        self.fused = None
        if self.fused_update:
            from .fused import FusedPPOUpdate

            self.fused = FusedPPOUpdate(self, compute_dtype=self.mixed_precision_dtype if self.mixed_precision
                                        else torch.float32, use_graphs=bool(self.config.get("hip_graphs", True)),
                                        scaler=self.scaler_state)
            self._ds_static: dict = {}
            if self._play_graphs is not None:
                self.fused.init_rollout(N, int(self.params.get("seed", 0)) * 7919 + self.rank)
                self.fused.init_bookkeeping(self)

    # ------------------------------------------------------------------ env / policy
    def obs_to_tensors(self, obs):
        if isinstance(obs, dict):
            return {"obs": obs["obs"], "states": obs.get("states")}
        return {"obs": obs}

    def env_reset(self):
        return self.obs_to_tensors(self.vec_env.reset())

    def preprocess_actions(self, actions: torch.Tensor) -> torch.Tensor:
        if not self.clip_actions:
            return actions
        a = torch.clamp(actions, -1.0, 1.0)
        if self._unit_box:  # rescale_actions to [-1, 1] is the identity
            return a
        d = (self.actions_high - self.actions_low) / 2.0
        m = (self.actions_high + self.actions_low) / 2.0
        return a * d + m

    def env_step(self, actions: torch.Tensor):
        obs, rewards, dones, infos = self.vec_env.step(self.preprocess_actions(actions))
        if self.value_size == 1:
            rewards = rewards.unsqueeze(1)
        return self.obs_to_tensors(obs), rewards.to(self.ppo_device), dones.to(self.ppo_device), infos

    @torch.no_grad()
    def get_action_values(self, obs: dict) -> dict:
        self.model.eval()
        return self.model({"is_train": False, "prev_actions": None, "obs": obs["obs"]}, generator=self.gen)

    @torch.no_grad()
    def get_values(self, obs: dict) -> torch.Tensor:
        self.model.eval()
        return self.model({"is_train": False, "prev_actions": None, "obs": obs["obs"]}, generator=self.gen)["values"]

    # ------------------------------------------------------------------ rollout
    def discount_values(self, fdones, last_values, mb_fdones, mb_values, mb_rewards):
        lastgaelam = 0
        mb_advs = torch.zeros_like(mb_rewards)
        for t in reversed(range(self.horizon_length)):
            if t == self.horizon_length - 1:
                nextnonterminal = 1.0 - fdones
                nextvalues = last_values
            else:
                nextnonterminal = 1.0 - mb_fdones[t + 1]
                nextvalues = mb_values[t + 1]
            nextnonterminal = nextnonterminal.unsqueeze(1)
            delta = mb_rewards[t] + self.gamma * nextvalues * nextnonterminal - mb_values[t]
            mb_advs[t] = lastgaelam = delta + self.gamma * self.tau * nextnonterminal * lastgaelam
        return mb_advs

    def _play_step_body(self, n: int) -> None:
        """Rollout step n on static buffers (the captured form of one play_steps iteration)."""
        td = self.tensor_dict
        obs = self._obs_buf
        res = {k: td[k][n] for k in ("actions", "neglogpacs", "values", "mus", "sigmas")}
        self.fused.policy_act(obs, res)  # trunk + heads + Philox sampling straight into the buffers
        td["obses"][n].copy_(obs)
        td["dones"][n].copy_(self._dones_buf)
        obs2, rewards, dones, infos = self.env_step(res["actions"])
        # shaping + value bootstrap + episode sums + AverageMeters: two launches (fused.rollout_post)
        self.fused.rollout_post(self, rewards.reshape(-1), dones, infos.get("time_outs"), res["values"].reshape(-1),
                                td["rewards"][n].reshape(-1))
        self._obs_buf.copy_(obs2["obs"])
        self._dones_buf.copy_(dones)

    def _play_step_graph(self, n: int) -> None:
        """First call: eager (warm-up, real step).  Second: capture (no execution) + replay.  Later:
        replay, then advance the env's host-side counters the replay did not touch."""
        g = self._play_graphs.get(n)
        if g is None:
            self._play_step_body(n)
            self._play_graphs[n] = "warm"
            return
        if g == "warm":
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._play_step_body(n)  # the env's Python counters advance here, once
            self._play_graphs[n] = g
            g.replay()
            return
        g.replay()
        self._uw.account_steps(1)

    @torch.no_grad()
    def play_steps(self) -> dict:
        td = self.tensor_dict
        step_time = 0.0
        if self._play_graphs is not None:
            self.model.eval()
            if self.obs["obs"].data_ptr() != self._obs_buf.data_ptr():
                self._obs_buf.copy_(self.obs["obs"])
            if self.dones.data_ptr() != self._dones_buf.data_ptr():
                self._dones_buf.copy_(self.dones)
            for n in range(self.horizon_length):
                self._play_step_graph(n)
            self.obs = {"obs": self._obs_buf}
            self.dones = self._dones_buf
            return self._finish_rollout(step_time)
        for n in range(self.horizon_length):
            res = self.get_action_values(self.obs)
            td["obses"][n] = self.obs["obs"]
            td["dones"][n] = self.dones
            for k in ("actions", "neglogpacs", "values", "mus", "sigmas"):
                td[k][n] = res[k]
            t0 = time.perf_counter()
            self.obs, rewards, self.dones, infos = self.env_step(res["actions"])
            step_time += time.perf_counter() - t0
            shaped = self.rewards_shaper(rewards)
            if self.value_bootstrap and "time_outs" in infos:
                shaped = shaped + self.gamma * res["values"] * infos["time_outs"].unsqueeze(1).float()
            td["rewards"][n] = shaped
            self.current_rewards += rewards
            self.current_shaped_rewards += shaped
            self.current_lengths += 1
            done = self.dones.bool()
            self.game_rewards.update(self.current_rewards, done)
            self.game_shaped_rewards.update(self.current_shaped_rewards, done)
            self.game_lengths.update(self.current_lengths.unsqueeze(1), done)
            self.algo_observer.process_infos(infos, done)
            not_dones = 1.0 - self.dones.float()
            self.current_rewards *= not_dones.unsqueeze(1)
            self.current_shaped_rewards *= not_dones.unsqueeze(1)
            self.current_lengths *= not_dones
        return self._finish_rollout(step_time)

    def _finish_rollout(self, step_time: float) -> dict:
        td = self.tensor_dict
        if self._play_graphs is not None:
            last_values = self.fused.policy_values(self.obs["obs"])
        else:
            last_values = self.get_values(self.obs)
        mb_advs = self.discount_values(self.dones.float(), last_values, td["dones"].float(), td["values"],
                                       td["rewards"])
        mb_returns = mb_advs + td["values"]
        batch = {k: swap_and_flatten01(td[k]) for k in self.tensor_list}
        batch["returns"] = swap_and_flatten01(mb_returns)
        batch["played_frames"] = self.batch_size
        batch["step_time"] = step_time
        return batch

    def gather_batch(self, batch: dict) -> dict:
        """allgather mode: concatenate every rank's flattened rollout (env-major ⇒ global env order)
        with one RCCL all-gather per dtype (distributed.RolloutGather)."""
        from ..distributed import RolloutGather

        if not hasattr(self, "_gather"):
            self._gather = RolloutGather(env_axis=0)
        keys = self.tensor_list + ["returns"]
        out = self._gather.gather({k: batch[k] for k in keys})
        out["played_frames"] = batch["played_frames"]
        out["step_time"] = batch["step_time"]
        return out

    # ------------------------------------------------------------------ update
    def prepare_dataset(self, batch: dict) -> None:
        values, returns = batch["values"], batch["returns"]
        advantages = returns - values
        if self.normalize_value:
            vms = self.model.value_mean_std
            vms.train()
            values = vms(values)
            returns = vms(returns)
            vms.eval()
        advantages = torch.sum(advantages, dim=1)
        if self.normalize_advantage:
            advantages = (advantages - advantages.mean()) / (advantages.std() + 1e-8)
        ds = {"old_values": values, "old_logp_actions": batch["neglogpacs"], "advantages": advantages,
              "returns": returns, "actions": batch["actions"], "obs": batch["obses"], "dones": batch["dones"],
              "mu": batch["mus"], "sigma": batch["sigmas"]}
        if self.fused is not None:  # static buffers: the captured graphs address them by pointer
            st = self._ds_static
            for k, v in ds.items():
                v = v.reshape(v.shape[0], -1) if v.dim() > 1 else v
                if k not in st or st[k].shape != v.shape or st[k].dtype != v.dtype:
                    st[k] = torch.empty_like(v, memory_format=torch.contiguous_format)
                st[k].copy_(v)
            ds = dict(st)
            self.fused.set_dataset(ds)
        self.dataset.update_values_dict(ds)

    def _exchange_grads(self) -> None:
        if self.multi_gpu and self.multi_gpu_mode == "allreduce" and self.world_size > 1:
            dist.all_reduce(self._bucket, op=dist.ReduceOp.SUM)
            self._bucket.div_(self.world_size)

    def calc_gradients(self, input_dict: dict):
        value_preds = input_dict["old_values"]
        old_neglogp = input_dict["old_logp_actions"]
        advantage = input_dict["advantages"]
        old_mu, old_sigma = input_dict["mu"], input_dict["sigma"]
        return_batch = input_dict["returns"]
        actions = input_dict["actions"]
        obs = input_dict["obs"]
        with torch.autocast(device_type=self.device.type, dtype=self.mixed_precision_dtype, enabled=self.mixed_precision):
            res = self.model({"is_train": True, "prev_actions": actions, "obs": obs})
            neglogp, values, entropy = res["prev_neglogp"], res["values"], res["entropy"]
            mu, sigma = res["mus"], res["sigmas"]
            a_loss = actor_loss(old_neglogp, neglogp, advantage, self.ppo, self.e_clip).mean()
            c_loss = critic_loss(value_preds, values, self.e_clip, return_batch, self.clip_value).mean()
            if self.bound_loss_type == "bound" and self.bounds_loss_coef is not None:
                b_loss = bound_loss(mu).mean()
            elif self.bound_loss_type == "regularisation":
                b_loss = (mu * mu).sum(dim=-1).mean()
            else:
                b_loss = torch.zeros((), device=self.device)
            entropy = entropy.mean()
            loss = (a_loss + 0.5 * c_loss * self.critic_coef - entropy * self.entropy_coef
                    + b_loss * float(self.bounds_loss_coef or 0.0))
        self.flat.zero_grad()
        if self.scaler_state is not None:
            (loss * self.scaler_state[0]).backward()  # scaler.scale(loss).backward()
        else:
            loss.backward()
        with torch.no_grad():
            kl = policy_kl(mu.detach().float(), sigma.detach().float(), old_mu, old_sigma, True)
            self._kl_slot.copy_(kl.reshape(1))
        self._exchange_grads()
        skip = False
        if self.scaler_state is not None:  # scaler.unscale_ / scaler.step / scaler.update
            with torch.no_grad():
                g = self.flat.grads
                found_inf = ~torch.isfinite(g).all()
                g.mul_(1.0 / self.scaler_state[0])
                skip = bool(found_inf.item())  # (GradScaler.step reads found_inf on the host too)
                self._scaler_update(skip)
        if not skip:
            if self.truncate_grads:
                g = self.flat.grads
                coef = torch.clamp(self.grad_norm / (torch.linalg.vector_norm(g) + 1e-6), max=1.0)
                g.mul_(coef)
            self.optimizer.step()
        return (a_loss.detach(), c_loss.detach(), entropy.detach(), self._kl_slot[0].clone(),
                mu.detach(), sigma.detach(), b_loss.detach())

    @torch.no_grad()
    def _scaler_update(self, found_inf: bool) -> None:
        """GradScaler.update (backoff 0.5, growth 2 after SCALER_GROWTH_INTERVAL good steps in a row); the
        fused path does the same in ppo_tail."""
        st = self.scaler_state
        if found_inf:
            st[0] *= 0.5
            st[1] = 0.0
        elif float(st[1]) + 1.0 >= SCALER_GROWTH_INTERVAL:
            st[0] *= 2.0
            st[1] = 0.0
        else:
            st[1] += 1.0

    def train_epoch(self):
        self.model.eval()
        t_play = time.perf_counter()
        batch = self.play_steps()
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)  # play / update split of the epoch time (once per epoch)
        if self.multi_gpu and self.multi_gpu_mode == "allgather" and self.world_size > 1:
            batch = self.gather_batch(batch)
        t_update = time.perf_counter()
        self.model.train()
        self.curr_frames = batch.pop("played_frames")
        step_time = batch.pop("step_time")
        self.prepare_dataset(batch)
        self.algo_observer.after_steps()
        if self.fused is not None:
            return self._train_epoch_fused(t_play, t_update, step_time)
        a_losses, c_losses, b_losses, entropies, kls = [], [], [], [], []
        for _ in range(self.mini_epochs_num):
            ep_kls = []
            for i in range(len(self.dataset)):
                a_loss, c_loss, entropy, kl, cmu, csigma, b_loss = self.calc_gradients(self.dataset[i])
                a_losses.append(a_loss)
                c_losses.append(c_loss)
                b_losses.append(b_loss)
                entropies.append(entropy)
                ep_kls.append(kl)
                self.dataset.update_mu_sigma(cmu, csigma)
                if self.schedule_type == "legacy":
                    self.scheduler.update_(self.lr, kl)
            av_kls = torch.stack(ep_kls).mean()
            if self.schedule_type == "standard":
                self.scheduler.update_(self.lr, av_kls)
            kls.append(av_kls)
            if self.normalize_input:
                self.model.running_mean_std.eval()  # statistics from the first mini-epoch only
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        t_end = time.perf_counter()
        stats = {k: torch.stack(v).mean() for k, v in
                 (("a_loss", a_losses), ("c_loss", c_losses), ("b_loss", b_losses), ("entropy", entropies),
                  ("kl", kls))}
        return step_time, t_update - t_play, t_end - t_update, t_end - t_play, stats

    def _train_epoch_fused(self, t_play: float, t_update: float, step_time: float):
        """Minibatch loop on the HIP graphs of learning/fused.py: graph A (forward, losses, backward),
        the bucket all-reduce (allreduce mode), graph B (clip, Adam, adaptive LR, counters)."""
        f = self.fused
        f.begin_epoch()
        n_mb = len(self.dataset)
        # `exchange_schedule` (agent config, diagnostic): run the allreduce mode's schedule -- per-minibatch
        # graphs A / exchange / B, the separate norm pass -- at world 1 too, so its one-GPU cost is measured
        # (scripts/price_exchange.sh); the exchange itself is then a no-op
        exchange = (self.multi_gpu and self.multi_gpu_mode == "allreduce" and self.world_size > 1) or bool(
            self.config.get("exchange_schedule", False))
        for ep in range(self.mini_epochs_num):
            rms_train = self.normalize_input and ep == 0
            if not exchange:  # nothing between A and B: the whole mini-epoch is one graph
                f.run_minibatches(n_mb, rms_train)
            else:
                for _ in range(n_mb):
                    f.step_a(rms_train)
                    self._exchange_grads()
                    f.step_b()
            if self.schedule_type == "standard":
                s0 = ep * n_mb
                self.scheduler.update_(self.lr, f.stats[s0:s0 + n_mb, 4].mean())
        if self.normalize_input:
            self.model.running_mean_std.eval()
        torch.cuda.synchronize(self.device)
        t_end = time.perf_counter()
        st = f.stats[: self.mini_epochs_num * n_mb]
        kls = st[:, 4].view(self.mini_epochs_num, n_mb).mean(1)
        stats = {"a_loss": st[:, 0].mean(), "c_loss": st[:, 1].mean(), "b_loss": st[:, 2].mean(),
                 "entropy": st[:, 3].mean(), "kl": kls.mean()}
        return step_time, t_update - t_play, t_end - t_update, t_end - t_play, stats

    # ------------------------------------------------------------------ loop
    def update_epoch(self) -> int:
        self.epoch_num += 1
        return self.epoch_num

    def train(self):
        self.init_tensors()
        self.last_mean_rewards = -100500.0
        total_time = 0.0
        self.obs = self.env_reset()
        self.curr_frames = self.batch_size_envs
        if self.multi_gpu and self.world_size > 1:
            dist.broadcast(self.flat.params, 0)
            for b in self.model.buffers():
                dist.broadcast(b, 0)
        if self.fused is not None:
            self.fused.refresh_mirror()
        while True:
            epoch_num = self.update_epoch()
            step_time, play_time, update_time, sum_time, stats = self.train_epoch()
            total_time += sum_time
            curr_frames = self.curr_frames * (self.world_size if self.multi_gpu else 1)
            self.frame += curr_frames
            should_exit = False
            if step_time <= 0.0:  # graph replays: env steps are not separately timed
                step_time = play_time
            self.last_stats = {"epoch": epoch_num, "frames": self.frame, "play_time": play_time,
                               "update_time": update_time, "step_time": step_time,
                               "fps_step": curr_frames / max(step_time, 1e-9),
                               "fps_total": curr_frames / max(sum_time, 1e-9),
                               "lr": float(self.lr), **{k: float(v) for k, v in stats.items()}}
            if self.rank == 0:
                if self.print_stats:
                    print(f"fps step: {self.last_stats['fps_step']:.0f} fps total: "
                          f"{self.last_stats['fps_total']:.0f} epoch: {epoch_num}/{self.max_epochs} "
                          f"frames: {self.frame}", flush=True)
                if float(self.game_rewards.current_size) > 0:
                    mean_rewards = self.game_rewards.get_mean()
                    self.mean_rewards = float(mean_rewards[0])
                    self.last_stats["mean_rewards"] = self.mean_rewards
                    self.last_stats["mean_lengths"] = float(self.game_lengths.get_mean()[0])
                    name = f"{self.name}_ep_{epoch_num}_rew_{self.mean_rewards}"
                    if self.save_freq > 0 and epoch_num % self.save_freq == 0 and \
                            self.mean_rewards <= self.last_mean_rewards:
                        self.save(os.path.join(self.nn_dir, "last_" + name))
                    if self.mean_rewards > self.last_mean_rewards and epoch_num >= self.save_best_after:
                        self.last_mean_rewards = self.mean_rewards
                        self.save(os.path.join(self.nn_dir, self.name))
                        if self.last_mean_rewards > self.score_to_win:
                            self.save(os.path.join(self.nn_dir, name))
                            should_exit = True
                self._log_metrics()
                if self.max_epochs != -1 and epoch_num >= self.max_epochs:
                    mean = self.game_rewards.get_mean()[0] if float(self.game_rewards.current_size) > 0 else -math.inf
                    self.save(os.path.join(self.nn_dir, f"last_{self.name}_ep_{epoch_num}_rew_{mean}"))
                    should_exit = True
            if self.multi_gpu and self.world_size > 1:
                t = torch.tensor([float(should_exit)], device=self.device)
                dist.broadcast(t, 0)
                should_exit = bool(t.item())
            if should_exit:
                return self.last_mean_rewards, epoch_num

    def _log_metrics(self) -> None:
        """rl_games writes its per-epoch scalars to TensorBoard (absent here): one JSON line per epoch
        in <train_dir>/<experiment>/summaries/metrics.jsonl (losses, lr, kl, fps, episode stats)."""
        if not self.config.get("write_metrics", True):
            return
        import json

        d = os.path.join(self.experiment_dir, "summaries")
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "metrics.jsonl"), "a") as f:
            f.write(json.dumps({k: (round(v, 6) if isinstance(v, float) else v) for k, v in self.last_stats.items()})
                    + "\n")

    # ------------------------------------------------------------------ checkpoints (rl_games layout)
    def get_weights(self) -> dict:
        return {"model": self.model.state_dict()}

    def set_weights(self, weights: dict) -> None:
        self.model.load_state_dict(weights["model"])
        self.flat.rebind()
        if getattr(self, "fused", None) is not None:
            self.fused.refresh_mirror()

    def get_full_state_weights(self) -> dict:
        state = self.get_weights()
        state.update(epoch=self.epoch_num, frame=self.frame, last_mean_rewards=self.last_mean_rewards,
                     optimizer=self.optimizer.state_dict(), env_state=None,
                     env_signature=env_signature(self.vec_env, self.obs_shape, self.actions_num))
        if self.scaler_state is not None:  # rl_games: state['scaler'] = self.scaler.state_dict()
            state["scaler"] = {"scale": float(self.scaler_state[0]), "growth_factor": 2.0, "backoff_factor": 0.5,
                               "growth_interval": SCALER_GROWTH_INTERVAL,
                               "_growth_tracker": int(self.scaler_state[1])}
        return state

    def save(self, fn: str) -> None:
        os.makedirs(os.path.dirname(fn) or ".", exist_ok=True)
        torch.save(self.get_full_state_weights(), fn + ".pth")

    def restore(self, fn: str, set_epoch: bool = True) -> None:
        ckpt = torch.load(fn, map_location=self.device, weights_only=True)
        check_env_signature(ckpt.get("env_signature"), env_signature(self.vec_env, self.obs_shape, self.actions_num), fn)
        self.set_weights(ckpt)
        if set_epoch:
            self.epoch_num = int(ckpt.get("epoch", 0))
            self.frame = int(ckpt.get("frame", 0))
        opt = ckpt.get("optimizer")
        if isinstance(opt, dict) and "exp_avg" in opt:
            self.optimizer.load_state_dict(opt)
        sc = ckpt.get("scaler")
        if self.scaler_state is not None and isinstance(sc, dict) and "scale" in sc:
            self.scaler_state[0] = float(sc["scale"])
            self.scaler_state[1] = float(sc.get("_growth_tracker", 0))
