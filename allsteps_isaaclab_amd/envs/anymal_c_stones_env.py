"""``AnymalCStonesEnv`` -- BASELINE C5 behind the direct-workflow env surface (registered as
``Allsteps-AnymalC-v0``), so ``RlGamesVecEnvWrapper``, ``train.py`` and ``play.py`` drive it like Allsteps-v0.

One ``step(actions)`` is ``as_quad_step`` on the HIP device: ``decimation`` substeps of ``k_step<18>``
(6 + 12 generalized velocities) with IsaacLab's DC motor evaluated in every substep on the position targets
``default_q + action_scale * a`` (anymal_c_env.py:73-78), four foot sensors, then ``k_quad``: target
stones, potentials, rewards, dones, in-kernel resets of done envs (stand pose + Philox joint noise, actions
observed as zero: anymal_c_env.py:171-172) and the 64-float observation.  Simulation settings are ANYmal-C's
(``AnymalCStonesEnvCfg``: dt 1/200, friction 1.0 multiply, max depenetration velocity 1.0).  There is no
CPU fallback: without the HIP library or a gfx950 device the constructor raises ``NativeError``.
"""

from __future__ import annotations

import numpy as np
import torch

from .. import _native
from ..model import ANYMAL_C_JSON, load_model
from .anymal_c_stones_env_cfg import AnymalCStonesEnvCfg
from .direct_rl_env import DirectRLEnv


def stand_pose(dof_names: list[str], init: dict) -> np.ndarray:
    """Default joint positions in the model's cfg DOF order from ANYMAL_C_CFG's regex-style table
    (HAA, {F,H}_HFE, {F,H}_KFE)."""
    q = np.zeros(len(dof_names), np.float32)
    for k, name in enumerate(dof_names):
        leg, joint = name.split("_")
        q[k] = init["HAA"] if joint == "HAA" else init[f"{leg[1]}_{joint}"]
    return q


def level0_stones(n: int, num_steps: int = 20) -> np.ndarray:
    """steps_pos of curriculum level 0 ([3 * num_steps][n]): x = 0.75 k, y = 0, z = 0.75 k cos(pi/2)."""
    st = np.zeros((3 * num_steps, n), np.float32)
    for k in range(num_steps):
        st[3 * k] = 0.75 * k
        st[3 * k + 2] = np.float32(k * 0.75) * np.cos(np.float32(np.pi / 2), dtype=np.float32)
    return st


class AnymalCStonesEnv(DirectRLEnv):
    """The C5 task env: ``reset() -> ({"policy": obs}, extras)``, ``step(a) -> ({"policy": obs}, reward,
    terminated, truncated, extras)``; every buffer on the device."""

    cfg: AnymalCStonesEnvCfg

    def __init__(self, cfg: AnymalCStonesEnvCfg | None = None, render_mode: str | None = None, **kwargs):
        cfg = cfg or AnymalCStonesEnvCfg()
        super().__init__(cfg, render_mode, **kwargs)
        dev = self._device
        if dev.type != "cuda" or not torch.cuda.is_available():
            raise _native.NativeError(f"AnymalCStonesEnv runs on the HIP backend only (device={dev}, HIP device "
                                      f"available: {torch.cuda.is_available()}); there is no CPU fallback")
        self.model = load_model(ANYMAL_C_JSON)
        if not cfg.robot.enabled_self_collisions:  # ArticulationRootPropertiesCfg.enabled_self_collisions
            self.model = dict(self.model, num_self_pairs=0, self_pair=[0] * len(self.model["self_pair"]))
        n = self.num_envs
        self.num_dof = self.model["num_hinges"]
        if self.num_dof != cfg.action_space:
            raise ValueError(f"model has {self.num_dof} hinges, cfg.action_space = {cfg.action_space}")
        self.state: dict[str, torch.Tensor] = {}
        for name, rows, t in _native.STATE_LAYOUT:
            self.state[name] = torch.zeros((rows, n) if rows > 1 else (n,), device=dev,
                                           dtype=torch.float32 if t == "f" else torch.int32)
        self.state["curriculum"] = torch.zeros(1, dtype=torch.int32, device=dev)
        self.state["contact_mask_hind"] = torch.zeros((2, n), dtype=torch.int32, device=dev)  # sensors RH, LH
        self.state["feet"] = torch.zeros((8, n), dtype=torch.int32, device=dev)  # per-foot targets | reach counts
        self.state["stones"][:] = torch.as_tensor(level0_stones(n, cfg.num_steps), device=dev)
        with torch.cuda.device(dev):
            self._native = _native.NativeEnv(n, self.model, cfg, self.state, int(cfg.seed or 0),
                                             dev.index if dev.index is not None else torch.cuda.current_device())
        self.default_joint_pos = torch.as_tensor(stand_pose(self.model["dof_names"], cfg.robot.init_joint_pos),
                                                 device=dev)
        self._native.set_actuator(_native.ACT_DC_MOTOR, action_scale=cfg.action_scale,
                                  default_q=self.default_joint_pos.cpu().tolist(), **cfg.actuator())
        self._native.set_quad_task(**cfg.quad_task())
        # articulation.py:1262-1266: mean -+ 0.5 range * factor (data only, as in IsaacLab)
        lo = torch.tensor([self.model["lower"][self.model["cfg_dof_link"][k]] for k in range(self.num_dof)])
        hi = torch.tensor([self.model["upper"][self.model["cfg_dof_link"][k]] for k in range(self.num_dof)])
        mean, rng = (lo + hi) / 2, hi - lo
        f = cfg.robot.soft_joint_pos_limit_factor
        self.soft_joint_pos_limits = torch.stack([mean - 0.5 * rng * f, mean + 0.5 * rng * f], -1).to(dev)
        self.soft_joint_pos_limits = self.soft_joint_pos_limits.unsqueeze(0).expand(n, -1, -1)
        self.obs_buf = torch.zeros((n, _native.QUAD_OBS_DIM), dtype=torch.float32, device=dev)
        self.reward_buf = torch.zeros(n, dtype=torch.float32, device=dev)
        # k_quad writes 0 / 1 bytes straight into the bool buffers (torch.bool is one byte, as AllstepsEnv)
        self.reset_terminated = torch.zeros(n, dtype=torch.bool, device=dev)
        self.reset_time_outs = torch.zeros(n, dtype=torch.bool, device=dev)
        # persistent reset_buf (DirectRLEnv keeps one): filled from terminated | truncated on the first
        # access after a step, so in-place writes (env.reset_buf[ids] = 1) stick until the next step
        self._reset_buf = torch.zeros(n, dtype=torch.bool, device=dev)
        self._reset_buf_stale = False
        self.extras = {}
        self._native.quad_reset_all(self.obs_buf, stream=self._stream())
        # the ArticulationData views (ring 1 zero-copy, ring 2 -- the 13 MJCF bodies -- by as_body_state on
        # demand), as the walker's env serves them (envs/allsteps_env.py)
        from .allsteps_env import _RobotView

        self.robot = _RobotView(self)

    def _stream(self) -> int:
        return torch.cuda.current_stream(self._device).cuda_stream

    @property
    def episode_length_buf(self) -> torch.Tensor:
        return self.state["ep_len"]

    @property
    def target_index(self) -> torch.Tensor:
        return self.state["idx"]

    @property
    def reset_buf(self) -> torch.Tensor:
        """terminated | truncated of the last step: one persistent buffer, formed on the first access after
        a step (no kernel in the step itself); writes into it persist until the next step."""
        if self._reset_buf_stale:
            torch.logical_or(self.reset_terminated, self.reset_time_outs, out=self._reset_buf)
            self._reset_buf_stale = False
        return self._reset_buf

    @reset_buf.setter
    def reset_buf(self, value) -> None:
        self._reset_buf.copy_(torch.as_tensor(value, device=self._reset_buf.device).to(torch.bool).expand_as(
            self._reset_buf))
        self._reset_buf_stale = False

    @property
    def foot_targets(self) -> torch.Tensor:
        """(N, 4) target stone of each sensor foot (RF, LF, RH, LH); target_index is the front pair's min"""
        return self.state["feet"][:4].T

    @property
    def contact_mask(self) -> torch.Tensor:
        """(N, 4) stone bitmasks of the four sensor feet (RF, LF, RH, LH) in the last substep."""
        return torch.cat([self.state["contact_mask"], self.state["contact_mask_hind"]], dim=0).T

    def _render_rgb(self, env_id: int):
        from .render import render_frame

        st = {k: self.state[k][..., env_id].detach().cpu().numpy() for k in ("root_pos", "root_quat", "q", "stones")}
        half = [0.5 * v for v in self.cfg.step_size]
        return render_frame(self.model, st["root_pos"], st["root_quat"], st["q"], st["stones"].reshape(-1, 3), half,
                            target=int(self.state["idx"][env_id]))

    def get_state(self) -> dict:
        return {k: v.clone() for k, v in self.state.items()}

    def _reseed(self, seed: int):
        self._native.set_seed(seed)

    def _reset_impl(self):
        self._native.quad_reset_all(self.obs_buf, stream=self._stream())
        self._reset_buf_stale = True
        return {"policy": self.obs_buf}

    def _step_impl(self, action: torch.Tensor):
        if action.shape != (self.num_envs, self.num_dof):
            raise ValueError(f"actions must be ({self.num_envs}, {self.num_dof}), got {tuple(action.shape)}")
        a = action.to(torch.float32).contiguous()
        self._native.quad_step(a, self.obs_buf, self.reward_buf, self.reset_terminated, self.reset_time_outs,
                               stream=self._stream())
        self._reset_buf_stale = True
        return {"policy": self.obs_buf}, self.reward_buf, self.reset_terminated, self.reset_time_outs, self.extras

    def close(self):
        if getattr(self, "_native", None) is not None:
            self._native.close()
            self._native = None
        super().close()
