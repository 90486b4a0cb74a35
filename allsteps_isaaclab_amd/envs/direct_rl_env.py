"""``DirectRLEnv`` -- the direct-workflow env contract of the reference, MI355X-native.

Mirrors the caller-visible surface of ``isaaclab/envs/direct_rl_env.py`` (``step``, ``reset``,
``seed``, ``close``, spaces, counters; SURVEY.md §8b ring 2).  Unlike the reference there is no
Omniverse simulation context: a subclass owns a native step backend and implements
``_step_impl`` / ``_reset_impl``; the base class keeps the bookkeeping (episode counters, spaces,
``extras``, device placement) so that wrappers written for the reference run unchanged.
"""

from __future__ import annotations

import math
from typing import Any

import torch

from .scene import SceneView
from .spaces import Box, Dict, batch_box


class DirectRLEnv:
    """Base class of direct-workflow environments (direct_rl_env.py:53-670)."""

    is_vector_env = True
    metadata: dict = {"render_modes": [None, "rgb_array"], "isaac_sim_version": None}

    def __init__(self, cfg, render_mode: str | None = None, **kwargs):
        self.cfg = cfg
        self.render_mode = render_mode
        self._is_closed = False
        if cfg.seed is not None:
            cfg.seed = self.seed(cfg.seed)
        self._device = torch.device(cfg.sim.device)
        self.num_envs = int(cfg.scene.num_envs)
        self.scene = SceneView(cfg.scene, self._device)  # env_origins: the reference's world offsets
        self.common_step_counter = 0
        self._sim_step_counter = 0
        self.extras: dict = {}
        self._configure_gym_env_spaces()

    # ------------------------------------------------------------------ properties
    @property
    def device(self) -> str:
        return str(self._device)

    @property
    def physics_dt(self) -> float:
        return self.cfg.sim.dt

    @property
    def step_dt(self) -> float:
        return self.cfg.sim.dt * self.cfg.decimation

    @property
    def max_episode_length_s(self) -> float:
        return self.cfg.episode_length_s

    @property
    def max_episode_length(self) -> int:
        # direct_rl_env.py:247-250
        return math.ceil(self.max_episode_length_s / (self.cfg.sim.dt * self.cfg.decimation))

    @property
    def unwrapped(self) -> "DirectRLEnv":
        return self

    # ------------------------------------------------------------------ spaces (direct_rl_env.py:523-561)
    def _configure_gym_env_spaces(self):
        inf = math.inf
        self.single_observation_space = Dict()
        self.single_observation_space["policy"] = Box(-inf, inf, (int(self.cfg.observation_space),))
        self.single_action_space = Box(-inf, inf, (int(self.cfg.action_space),))
        # direct_rl_env.py:551-552: the batched observation space is the policy Box, not a Dict
        self.observation_space = batch_box(self.single_observation_space["policy"], self.num_envs)
        self.action_space = batch_box(self.single_action_space, self.num_envs)
        self.state_space = None
        if getattr(self.cfg, "state_space", 0):
            self.single_observation_space["critic"] = Box(-inf, inf, (int(self.cfg.state_space),))
            self.state_space = batch_box(self.single_observation_space["critic"], self.num_envs)

    # ------------------------------------------------------------------ operations
    def reset(self, seed: int | None = None, options: dict[str, Any] | None = None):
        """direct_rl_env.py:256-294: reset all envs and return (observations, extras)."""
        if seed is not None:
            self.seed(seed)
            self._reseed(seed)
        obs = self._reset_impl()
        return obs, self.extras

    def step(self, action: torch.Tensor):
        """direct_rl_env.py:296-383: one env step (decimation physics substeps inside)."""
        action = action.to(self._device)
        self._sim_step_counter += self.cfg.decimation
        out = self._step_impl(action)
        self.common_step_counter += 1
        return out

    @staticmethod
    def seed(seed: int = -1) -> int:
        """direct_rl_env.py:390-407: seed torch / numpy / random (no replicator here)."""
        import random

        import numpy as np

        if seed == -1:
            seed = np.random.randint(0, 10_000)
        random.seed(seed)
        np.random.seed(seed)
        torch.manual_seed(seed)
        return seed

    def render(self, recompute: bool = False):
        """``rgb_array``: an (H, W, 3) uint8 frame of env 0 (envs/render.py; direct_rl_env.py:508-548
        returns the viewport capture there).  None without a render mode."""
        if self.render_mode is None:
            return None
        if self.render_mode != "rgb_array":
            raise NotImplementedError(f"render_mode={self.render_mode!r}: only 'rgb_array' is supported (headless)")
        return self._render_rgb(0)

    def _render_rgb(self, env_id: int):
        raise NotImplementedError(f"{type(self).__name__} has no renderer")

    def close(self):
        self._is_closed = True

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ subclass hooks
    def _reseed(self, seed: int):
        pass

    def _reset_impl(self):
        raise NotImplementedError

    def _step_impl(self, action: torch.Tensor):
        raise NotImplementedError
