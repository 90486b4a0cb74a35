"""rl_games VecEnv surface for the Allsteps env (isaaclab_rl/rl_games.py:80-360 behaviour).

``RlGamesVecEnvWrapper`` is what ``scripts/reinforcement_learning/rl_games/train.py`` wraps the env
in (train.py:140-150): it clamps actions to ``clip_actions``, steps the env, clamps observations to
``clip_obs``, returns ``dones = terminated | truncated`` and, for infinite-horizon tasks
(``cfg.is_finite_horizon`` False, the Allsteps default), ``extras["time_outs"] = truncated``
(rl_games.py:238-268).  ``RlGamesGpuEnv`` is the thin ``IVecEnv`` rl_games' runner instantiates
through ``env_configurations`` (rl_games.py:320-360).

rl_games itself (1.6.1) is a third-party trainer that is not installed in this image; when it is
importable its ``IVecEnv`` / ``env_configurations`` are used, otherwise stand-ins with the same
names keep the surface importable.
"""

from __future__ import annotations

import torch

from .envs.direct_rl_env import DirectRLEnv
from .envs.spaces import Box

try:  # pragma: no cover - depends on the image
    import rl_games as _rlg  # type: ignore

    if getattr(_rlg, "ALLSTEPS_COMPAT", False):  # our own opt-in shim (compat/site/rl_games)
        raise ImportError
    from rl_games.common import env_configurations, vecenv  # type: ignore
    from rl_games.common.vecenv import IVecEnv  # type: ignore

    HAVE_RL_GAMES = True
except Exception:  # rl_games absent: the stand-ins of _vecenv
    HAVE_RL_GAMES = False
    from ._vecenv import IVecEnv, env_configurations, vecenv


class RlGamesVecEnvWrapper(IVecEnv):
    """Isaac-Lab-style env -> rl_games vectorised env (rl_games.py:80-120)."""

    def __init__(self, env, rl_device: str, clip_obs: float, clip_actions: float):
        if not isinstance(env.unwrapped, DirectRLEnv):
            raise ValueError(f"The environment must be inherited from DirectRLEnv. Environment type: {type(env)}")
        self.env = env
        self._rl_device = rl_device
        self._clip_obs = clip_obs
        self._clip_actions = clip_actions
        self._sim_device = env.unwrapped.device
        space = self.state_space
        self.rlg_num_states = 0 if space is None else space.shape[0]

    def __str__(self):
        return (f"<{type(self).__name__}{self.env}>\n\tObservations clipping: {self._clip_obs}"
                f"\n\tActions clipping     : {self._clip_actions}\n\tAgent device         : {self._rl_device}"
                f"\n\tAsymmetric-learning  : {self.rlg_num_states != 0}")

    __repr__ = __str__

    # ---- gym.Wrapper-like properties
    @property
    def render_mode(self):
        return self.env.render_mode

    @property
    def unwrapped(self):
        return self.env.unwrapped

    @property
    def num_envs(self) -> int:
        return self.unwrapped.num_envs

    @property
    def device(self):
        return self.unwrapped.device

    @classmethod
    def class_name(cls) -> str:
        return cls.__name__

    def _box(self, space, bound: float, what: str) -> Box:
        if not hasattr(space, "shape") or not hasattr(space, "low"):
            raise NotImplementedError(f"The RL-Games wrapper does not support {what} space: '{type(space)}'.")
        return Box(-bound, bound, space.shape)

    @property
    def observation_space(self) -> Box:
        return self._box(self.unwrapped.single_observation_space["policy"], self._clip_obs, "observation")

    @property
    def action_space(self) -> Box:
        return self._box(self.unwrapped.single_action_space, self._clip_actions, "action")

    @property
    def state_space(self) -> Box | None:
        critic = self.unwrapped.single_observation_space.get("critic")
        return None if critic is None else self._box(critic, self._clip_obs, "state")

    def get_number_of_agents(self) -> int:
        return getattr(self, "num_agents", 1)

    def get_env_info(self) -> dict:
        return {"observation_space": self.observation_space, "action_space": self.action_space,
                "state_space": self.state_space}

    # ---- MDP
    def seed(self, seed: int = -1) -> int:
        return self.unwrapped.seed(seed)

    def reset(self):
        obs_dict, _ = self.env.reset()
        return self._process_obs(obs_dict)

    def step(self, actions: torch.Tensor):
        # clamp returns a new tensor (the reference's detach().clone() + clamp in one op)
        a = torch.clamp(actions.detach().to(device=self._sim_device), -self._clip_actions, self._clip_actions)
        obs_dict, rew, terminated, truncated, extras = self.env.step(a)
        if not self.unwrapped.cfg.is_finite_horizon:
            extras["time_outs"] = truncated.to(device=self._rl_device)
        obs = self._process_obs(obs_dict)
        rew = rew.to(device=self._rl_device)
        dones = (terminated | truncated).to(device=self._rl_device)
        extras = {k: v.to(device=self._rl_device, non_blocking=True) if hasattr(v, "to") else v
                  for k, v in extras.items()}
        if "log" in extras:
            extras["episode"] = extras.pop("log")
        if "mean_curriculum" in extras:
            print(f"The current mean curriculum is:{extras['mean_curriculum']}.")
        return obs, rew, dones, extras

    def close(self):
        return self.env.close()

    def _process_obs(self, obs_dict):
        o = obs_dict["policy"]
        # clamp to +-inf is the identity (NaN stays NaN): then only the reference's defensive clone
        obs = (o.clone() if self._clip_obs == float("inf") else torch.clamp(o, -self._clip_obs, self._clip_obs)
               ).to(device=self._rl_device)
        if self.rlg_num_states == 0:
            return obs
        if "critic" not in obs_dict:
            raise NotImplementedError("Environment does not define key 'critic' for privileged observations.")
        states = torch.clamp(obs_dict["critic"], -self._clip_obs, self._clip_obs).to(self._rl_device).clone()
        return {"obs": obs, "states": states}


class RlGamesGpuEnv(IVecEnv):
    """The ``IVecEnv`` rl_games' runner creates from ``env_configurations`` (rl_games.py:320-360)."""

    def __init__(self, config_name: str, num_actors: int, **kwargs):
        self.env: RlGamesVecEnvWrapper = env_configurations.configurations[config_name]["env_creator"](**kwargs)

    def step(self, action):
        return self.env.step(action)

    def reset(self):
        return self.env.reset()

    def get_number_of_agents(self) -> int:
        return self.env.get_number_of_agents()

    def get_env_info(self) -> dict:
        return self.env.get_env_info()
