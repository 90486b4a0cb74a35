"""The ``as_task_t`` table from an env cfg -- one helper for the HIP path (``_native.make_task``) and the
CPU oracle (``oracle/oracle.py::make_task``), so the two structs cannot drift.

Dispatch is on the cfg type, never on attribute presence:

* ``AllstepsEnvCfg`` (Allsteps-v0, allsteps_env_cfg.py:54-234): every field is the walker task's;
* ``AnymalCStonesEnvCfg`` (BASELINE C5): ``as_task_t`` carries only the stones / timing block the
  physics reads (``num_steps``, ``step_dt``); the task itself is ``as_quad_task_t``
  (``AnymalCStonesEnvCfg.quad_task``), and the walker-only entries (reward scales, curriculum, reset
  pose, mirror tables) are the walker's defaults, which no quadruped kernel reads;
* anything else raises ``TypeError``.
"""

from __future__ import annotations

import numpy as np


def linspace_f32(start: float, end: float, steps: int) -> np.ndarray:
    """float32 torch.linspace (ATen RangeFactories: start+i*step for the first half, end-(n-1-i)*step after)."""
    s, e = np.float32(start), np.float32(end)
    step = (e - s) / np.float32(steps - 1)
    return np.array([s + step * np.float32(i) if i < steps // 2 else e - step * np.float32(steps - i - 1)
                     for i in range(steps)], np.float32)


def task_fields(cfg, dof_names: list) -> dict:
    """as_task_t field -> value (scalars and lists), for ctypes structs of either side."""
    from .allsteps_env_cfg import AllstepsEnvCfg, running_start_pose
    from .anymal_c_stones_env_cfg import AnymalCStonesEnvCfg

    if isinstance(cfg, AllstepsEnvCfg):
        w = cfg
    elif isinstance(cfg, AnymalCStonesEnvCfg):
        w = AllstepsEnvCfg()  # walker-only entries: unread by k_step<18> / k_quad (as_quad_task_t holds the task)
    else:
        raise TypeError(f"no as_task_t for a {type(cfg).__name__}: expected AllstepsEnvCfg or AnymalCStonesEnvCfg")
    f = {
        "num_steps": cfg.num_steps,
        "step_radius": w.step_radius,
        "stop_frames": w.stop_frames,
        "eps": w.epsilon,
        "alive": w.alive_reward_scale, "energy": w.energy_cost_scale, "action": w.actions_cost_scale,
        "joint_limit": w.joint_at_limit_cost_scale, "death": w.death_cost,
        "dof_vel_scale": w.dof_vel_scale, "fall_abs": w.termination_height_absolute,
        "step_dt": float(np.float32(cfg.sim.dt * cfg.decimation)),
        "max_episode_length": w.max_episode_length,
        "max_curriculum": w.max_curriculum,
        "curriculum_threshold": w.curriculum_progress_threshold,
        "term_curriculum": [float(x) for x in linspace_f32(0.75, 0.45, w.max_curriculum + 1)],
        "gain_curriculum": [float(x) for x in linspace_f32(1.2, 1.2, w.max_curriculum + 1)],
        "init_root": list(w.init_root_pos),
        "init_q": [float(np.float32(x)) for x in running_start_pose()],
        "noise_lo": w.initial_joint_angle_range[0], "noise_hi": w.initial_joint_angle_range[1],
        "clip_lo": w.initial_joint_angle_clip_range[0], "clip_hi": w.initial_joint_angle_clip_range[1],
        "regen_footsteps": int(bool(getattr(w, "regenerate_footsteps", False))),
    }
    if all(x in dof_names for x in (*w.right_body_names, *w.left_body_names, *w.negation_body_names)):
        J = dof_names.index
        f["right_idx"] = [J(x) for x in w.right_body_names]
        f["left_idx"] = [J(x) for x in w.left_body_names]
        f["neg_idx"] = [J(x) for x in w.negation_body_names]
    # else: a model without the walker's joints (the quadruped) never reads the reset mirror tables
    return f


def fill(struct, fields: dict):
    """Copy task_fields() into a ctypes struct (arrays element-wise)."""
    for k, v in fields.items():
        if isinstance(v, list):
            getattr(struct, k)[:] = v
        else:
            setattr(struct, k, v)
    return struct
