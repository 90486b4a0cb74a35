"""BASELINE C5: an ANYmal-C-like quadruped on the ALLSTEPS stones.

The reference's C5 row ("Anymal-C quadruped on ALLSTEPS stones, 16384 envs, 4-foot contact, different
DoF count") has no model source offline (the ANYmal-C USD and actuator net are Nucleus-only,
``isaaclab_assets/robots/anymal.py:47,95``) and no task: ``direct/anymal_c/anymal_c_env.py`` is a
flat-ground velocity-tracking task.  What this module provides is the part of that row that lives on
the hot path: the same ``k_step`` physics (Featherstone dynamics, stone contacts, PGS) instantiated for
18 generalized velocities (6 + 12 hinges, ``model/anymal_c.xml``), stepped by ``as_physics_step`` over
the same SoA state and stone courses as the walker, four feet in contact with two stones.

``QuadrupedStonesEnv`` owns the device state; ``step(actions)`` applies tau = 1.2 * gear * clip(a)
(the Allsteps actuation, gear 80/1.2 N m) for ``decimation`` substeps of 1/240 s.  ``stand_actions``
is a joint-space PD on top of it (the ANYmal default stance), used by the physics tests to keep the
robots standing on the stones.

The C5 task env (the DC motor actuator, the stepping-stone task epilogue, ANYmal-C's simulation
settings, the direct-workflow surface) is ``envs/anymal_c_stones_env.py`` (``Allsteps-AnymalC-v0``).
"""

from __future__ import annotations

import numpy as np
import torch

from .. import _native
from ..model import ANYMAL_C_JSON, load_model
from .allsteps_env_cfg import AllstepsEnvCfg
from .anymal_c_stones_env import level0_stones  # noqa: F401  (re-exported for the physics tests)
from .anymal_c_stones_env import stand_pose as _stand_pose

# ANYmal default stance (IsaacLab ANYMAL_C_CFG init_state: HAA 0, front HFE 0.4 / KFE -0.8, hind HFE
# -0.4 / KFE 0.8), in the model's cfg DOF order
STAND_Q = {"HAA": 0.0, "F_HFE": 0.4, "H_HFE": -0.4, "F_KFE": -0.8, "H_KFE": 0.8}
# base pose over the level-0 line of stones (x = 0.75 k, top at 0.1125): hind feet on stone 0, front
# feet on stone 1, base at the stance height (hip-to-sole 0.574 m) + 1 cm
STAND_ROOT = (0.375, 0.0, 0.1125 + 0.574 + 0.01)
ACT_SCALE = 80.0  # N m per unit action (1.2 * gear)


def stand_pose(dof_names: list[str]) -> np.ndarray:
    return _stand_pose(dof_names, STAND_Q)


class QuadrupedStonesEnv:
    """Physics-only vectorised quadruped on stepping stones (HIP, k_step<18>)."""

    def __init__(self, num_envs: int, device: str = "cuda:0", seed: int = 42, cfg: AllstepsEnvCfg | None = None):
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise _native.NativeError("QuadrupedStonesEnv runs on the HIP backend only; there is no CPU fallback")
        self.cfg = cfg or AllstepsEnvCfg()
        self.model = load_model(ANYMAL_C_JSON)
        self.num_envs = n = int(num_envs)
        self.num_dof = self.model["num_hinges"]
        dev = self.device
        self.state: dict[str, torch.Tensor] = {}
        for name, rows, t in _native.STATE_LAYOUT:
            dt = torch.float32 if t == "f" else torch.int32
            self.state[name] = torch.zeros((rows, n) if rows > 1 else (n,), dtype=dt, device=dev)
        self.state["curriculum"] = torch.zeros(1, dtype=torch.int32, device=dev)
        self.state["contact_mask_hind"] = torch.zeros((2, n), dtype=torch.int32, device=dev)  # sensors RH, LH
        with torch.cuda.device(dev):
            self._native = _native.NativeEnv(n, self.model, self.cfg, self.state, seed,
                                             dev.index if dev.index is not None else torch.cuda.current_device())
        self.q_stand = torch.as_tensor(stand_pose(self.model["dof_names"]), device=dev)
        self.reset()

    def reset(self, stones: torch.Tensor | None = None) -> None:
        """Every env standing in the default stance over stones 0 (hind feet) and 1 (front feet)."""
        s, n = self.state, self.num_envs
        for k in ("root_lin", "root_ang", "qd", "q"):
            s[k].zero_()
        s["root_pos"][:] = torch.tensor(STAND_ROOT, device=self.device).view(3, 1)
        s["root_quat"].zero_()
        s["root_quat"][0] = 1.0
        s["q"][: self.num_dof] = self.q_stand.view(-1, 1)
        s["contact_mask"].zero_()
        s["contact_mask_hind"].zero_()
        s["stones"][:] = stones if stones is not None else torch.as_tensor(level0_stones(n), device=self.device)

    def stand_actions(self, kp: float = 150.0, kd: float = 4.0) -> torch.Tensor:
        """(N, 12) actions of a joint PD on the default stance: a = (kp (q* - q) - kd qd) / 80 N m."""
        q = self.state["q"][: self.num_dof]
        qd = self.state["qd"][: self.num_dof]
        tau = kp * (self.q_stand.view(-1, 1) - q) - kd * qd
        return (tau / ACT_SCALE).T.contiguous()

    def step(self, actions: torch.Tensor) -> None:
        if actions.shape != (self.num_envs, self.num_dof) or actions.dtype != torch.float32:
            raise ValueError(f"actions must be float32 ({self.num_envs}, {self.num_dof}), got "
                             f"{tuple(actions.shape)} {actions.dtype}")
        self._native.physics_step(actions.contiguous(), stream=torch.cuda.current_stream(self.device).cuda_stream)

    @property
    def root_pos(self) -> torch.Tensor:
        return self.state["root_pos"].T

    @property
    def contact_mask(self) -> torch.Tensor:
        """(N, 4) stone bitmasks of the four sensor feet (RF, LF, RH, LH) in the last substep."""
        return torch.cat([self.state["contact_mask"], self.state["contact_mask_hind"]], dim=0).T

    def close(self) -> None:
        if getattr(self, "_native", None) is not None:
            self._native.close()
            self._native = None
