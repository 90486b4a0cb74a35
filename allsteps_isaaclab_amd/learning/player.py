"""rl_games ``PpoPlayerContinuous`` surface used by the reference's play.py (play.py:140-201):
``runner.create_player()``, ``restore(path)``, ``reset()``, ``get_batch_size(obs, 1)``,
``obs_to_torch(obs)``, ``get_action(obs, is_deterministic)``, ``is_rnn``, ``states``.

Deterministic play returns ``mu``; stochastic play samples ``N(mu, sigma)``; either way clamped to
[-1, 1] and rescaled to the action bounds (players.py ``rescale_actions``).  Checkpoints are rl_games'
layout (``{'model': state_dict, ...}``) loaded with ``weights_only=True``.
"""

from __future__ import annotations

import torch

from .models import ModelA2CContinuousLogStd, check_env_signature, env_signature


class PpoPlayerContinuous:
    def __init__(self, params: dict):
        from ..rl_games import vecenv

        self.params = params
        self.config = config = params["config"]
        self.player_config = config.get("player", {}) or {}
        self.device = torch.device(config.get("device", "cuda:0"))
        self.env_name = config["env_name"]
        self.num_actors = int(config.get("num_actors", 1))
        self.env = config.get("vec_env") or vecenv.create_vec_env(self.env_name, self.num_actors,
                                                                   **config.get("env_config", {}))
        info = self.env.get_env_info()
        self.obs_shape = tuple(info["observation_space"].shape)
        space = info["action_space"]
        self.actions_num = int(space.shape[0])
        self.actions_low = torch.as_tensor(space.low, dtype=torch.float32, device=self.device)
        self.actions_high = torch.as_tensor(space.high, dtype=torch.float32, device=self.device)
        self.clip_actions = bool(config.get("clip_actions", True))
        self.is_deterministic = bool(self.player_config.get("deterministic", True))
        self.games_num = int(self.player_config.get("games_num", 2000))
        net = params["network"]
        mlp = net.get("mlp", {})
        cont = net.get("space", {}).get("continuous", {})
        sig = cont.get("sigma_init", {})
        self.model = ModelA2CContinuousLogStd(
            self.obs_shape[0], self.actions_num, normalize_input=bool(config["normalize_input"]),
            normalize_value=bool(config.get("normalize_value", False)),
            units=tuple(mlp.get("units", (256, 256, 256, 256, 256))), activation=mlp.get("activation", "elu"),
            sigma_init=float(sig.get("val", 0.0)) if sig.get("name") == "const_initializer" else 0.0,
        ).to(self.device).eval()
        self.is_rnn = False
        self.states = None
        self.has_batch_dimension = False
        self.batch_size = 1
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(int(params.get("seed", 0)))

    def restore(self, fn: str) -> None:
        ckpt = torch.load(fn, map_location=self.device, weights_only=True)
        check_env_signature(ckpt.get("env_signature"), env_signature(self.env, self.obs_shape, self.actions_num), fn)
        self.model.load_state_dict(ckpt["model"])
        if "running_mean_std" in ckpt and self.model.running_mean_std is not None:
            self.model.running_mean_std.load_state_dict(ckpt["running_mean_std"])

    def reset(self) -> None:
        self.states = None

    def init_rnn(self) -> None:
        pass

    def get_batch_size(self, obs, batch_size: int) -> int:
        o = obs["obs"] if isinstance(obs, dict) else obs
        if len(o.size()) > len(self.obs_shape):
            batch_size = o.size(0)
            self.has_batch_dimension = True
        self.batch_size = batch_size
        return batch_size

    def obs_to_torch(self, obs):
        if isinstance(obs, dict):
            obs = obs["obs"]
        return torch.as_tensor(obs, device=self.device).float()

    @torch.no_grad()
    def get_action(self, obs: torch.Tensor, is_deterministic: bool = False) -> torch.Tensor:
        if not self.has_batch_dimension:
            obs = obs.unsqueeze(0)
        res = self.model({"is_train": False, "prev_actions": None, "obs": obs}, generator=self.gen)
        a = res["mus"] if is_deterministic else res["actions"]
        if not self.has_batch_dimension:
            a = a.squeeze(0)
        if not self.clip_actions:
            return a
        a = torch.clamp(a, -1.0, 1.0)
        return a * (self.actions_high - self.actions_low) / 2.0 + (self.actions_high + self.actions_low) / 2.0

    def run(self, max_steps: int | None = None) -> dict:
        """BasePlayer.run, reduced: step the batched env with the policy until ``games_num`` episodes
        finished (or ``max_steps``); returns mean episode reward / length (device-side sums)."""
        obs = self.obs_to_torch(self.env.reset())
        self.get_batch_size(obs, 1)
        n = obs.shape[0]
        cur_r = torch.zeros(n, device=self.device)
        cur_l = torch.zeros(n, device=self.device)
        sum_r = torch.zeros((), device=self.device)
        sum_l = torch.zeros((), device=self.device)
        games = torch.zeros((), device=self.device)
        steps = 0
        while True:
            a = self.get_action(obs, self.is_deterministic)
            obs, r, done, _ = self.env.step(a)
            obs = self.obs_to_torch(obs)
            cur_r += r
            cur_l += 1
            d = done.float()
            sum_r += (cur_r * d).sum()
            sum_l += (cur_l * d).sum()
            games += d.sum()
            cur_r *= 1.0 - d
            cur_l *= 1.0 - d
            steps += 1
            if (max_steps is not None and steps >= max_steps) or (steps % 64 == 0 and float(games) >= self.games_num):
                break
        g = max(float(games), 1.0)
        return {"games": float(games), "mean_reward": float(sum_r) / g, "mean_length": float(sum_l) / g,
                "steps": steps}
