"""``AnymalCStonesEnvCfg`` -- BASELINE C5: the ANYmal-C quadruped on the ALLSTEPS stones, on ANYmal-C's own
simulation settings.

The simulation and robot fields follow the reference's ANYmal-C direct task and asset, not the walker's:

* ``direct/anymal_c/anymal_c_env_cfg.py:51-95`` (``AnymalCFlatEnvCfg``): episode 20 s, decimation 4,
  12 actions (its action scale 0.5 is raised to 1.0 here: the stones' stride needs the range),
  ``SimulationCfg(dt=1/200)``, physics material static = dynamic friction
  1.0 with the "multiply" combine mode on both the robot's default material and the terrain -- the
  contact friction is 1.0 x 1.0 = 1.0 (the walker uses 0.85 from the "average" combine);
* ``isaaclab_assets/robots/anymal.py`` ``ANYMAL_C_CFG``: rigid bodies with max_depenetration_velocity
  1.0 (the walker: 10), self-collision on, 4 position / 0 velocity solver iterations, the default stance
  (HAA 0, front HFE 0.4 / KFE -0.8, hind HFE -0.4 / KFE 0.8), ``soft_joint_pos_limit_factor=0.95``;
* the actuator: IsaacLab's DC motor with the ANYdrive 3 "simple" gains (``ANYDRIVE_3_SIMPLE_ACTUATOR_CFG``).
  The reference's ANYMAL_C_CFG uses the actuator network (``ANYDRIVE_3_LSTM_ACTUATOR_CFG``), whose
  weights are Nucleus-only (``anymal.py:47``); the DC motor is the documented analytical stand-in.

The stepping-stone task itself is authored (the reference has no quadruped stepping-stone task; DESIGN.md
§7b): stones as in Allsteps-v0 (20 boxes 0.5 x 0.8 x 0.225 m); the reference's target machine run per foot (every
foot has its own target stone -- the front feet start aiming at stone 2, the hind feet at stone 1 -- and
advances it after pushing on it within ``step_radius`` of its aim point for ``stop_frames`` steps; the
front pair's common target is the env's target index); the ALLSTEPS reward terms -- alive, potential
progress (body to the target stone, plus ``foot_progress`` x the feet's distances to their aim points),
energy, action cost, step hit 50 exp(-d / 0.25) per foot, last-stone bonus, death cost
(allsteps_env.py:347-394); death on tilt or a base height below the target stone.  The soft joint limits are data (``AnymalCStonesEnv
.soft_joint_pos_limits``): as in IsaacLab they do not enter the physics (articulation.py:1262-1266 only
stores them; PhysX gets the hard limits), and the direct ANYmal-C task never reads them.
"""

from __future__ import annotations

from dataclasses import dataclass, field

from .allsteps_env_cfg import InteractiveSceneCfg, SimulationCfg


def anymal_c_sim_cfg() -> SimulationCfg:
    return SimulationCfg(
        dt=1.0 / 200.0,                    # anymal_c_env_cfg.py: SimulationCfg(dt=1 / 200)
        render_interval=4,
        friction=1.0 * 1.0,                # "multiply" combine of robot 1.0 and terrain 1.0
        max_depenetration_velocity=1.0,    # anymal.py ANYMAL_C_CFG rigid_props
        solver_position_iteration_count=4,  # articulation_props: 4 position / 0 velocity iterations
    )


@dataclass
class AnymalCRobotCfg:
    """The articulation: default stance (ANYMAL_C_CFG.init_state), soft joint limit factor, actuator."""

    init_joint_pos: dict = field(default_factory=lambda: {"HAA": 0.0, "F_HFE": 0.4, "H_HFE": -0.4, "F_KFE": -0.8,
                                                          "H_KFE": 0.8})
    soft_joint_pos_limit_factor: float = 0.95
    # ANYDRIVE_3_SIMPLE_ACTUATOR_CFG (DCMotorCfg): kp, kd, saturation effort, effort limit, velocity limit
    stiffness: float = 40.0
    damping: float = 5.0
    saturation_effort: float = 120.0
    effort_limit: float = 80.0
    velocity_limit: float = 7.5
    enabled_self_collisions: bool = True


@dataclass
class AnymalCStonesEnvCfg:
    # env (anymal_c_env_cfg.py AnymalCFlatEnvCfg)
    episode_length_s: float = 20.0
    decimation: int = 4
    # anymal_c_env_cfg.py uses 0.5 for flat-ground velocity tracking; position targets within +-0.5 rad
    # of the stance cannot make the 0.75 m stride of the stones (the leg must reach 0.45 m behind and
    # ahead of its hip), and a 1000-epoch run at 0.5 only learns to stand (DESIGN.md §7b, r04d curves)
    action_scale: float = 1.0
    action_space: int = 12
    observation_space: int = 64
    state_space: int = 0
    seed: int | None = 42
    is_finite_horizon: bool = False

    sim: SimulationCfg = field(default_factory=anymal_c_sim_cfg)
    scene: InteractiveSceneCfg = field(default_factory=lambda: InteractiveSceneCfg(num_envs=16384))  # BASELINE C5
    robot: AnymalCRobotCfg = field(default_factory=AnymalCRobotCfg)

    # stones (as Allsteps-v0: allsteps_env_cfg.py:90-97), level-0 line
    num_steps: int = 20
    step_size: tuple = (0.5, 0.8, 0.225)

    # the stepping-stone task (authored; include/allsteps.h as_quad_task_t): the ALLSTEPS target
    # machine and reward terms (allsteps_env.py:347-394, 418-457) on four feet
    stop_frames: int = 2          # steps the swing foot must push on its target stone (allsteps_env_cfg: 2)
    step_radius: float = 0.25     # allsteps_env_cfg.py:97
    alive_reward: float = 0.5     # authored for the quadruped (the walker's alive_reward_scale is 2.0)
    energy_cost: float = 0.009    # energy_cost_scale (allsteps_env_cfg.py:222): sum |qd a|
    action_cost: float = 0.01     # actions_cost_scale (allsteps_env_cfg.py:223): ||a||
    death_reward: float = -1.0    # death_cost (allsteps_env_cfg.py:228)
    step_reward: float = 50.0     # allsteps_env.py:380: 50 exp(-d / 0.25) on a fresh reach
    step_sigma: float = 0.25
    target_bonus: float = 10.0    # allsteps_env.py:383, last stone with the body within 0.15 m
    bonus_radius: float = 0.15
    foot_progress: float = 0.5    # weight of the feet's distances to their aim points in the potential
    # aim point of each sensor foot (RF, LF, RH, LH) on its stone: the centre + this lateral offset,
    # the feet's stance width in model/anymal_c.xml (hip 0.1 + abduction link 0.1 either side)
    foot_offset_y: tuple = (-0.2, 0.2, -0.2, 0.2)
    min_height: float = 0.25      # base below target stone + this: terminated
    up_z_min: float = 0.5         # projected gravity z above -this (tilt past 60 degrees): terminated
    stand_height: float = 0.584   # reset: base this far above the higher of stones 0 / 1 (top face)
    joint_noise: float = 0.05     # reset: U(-1, 1) x this on every joint

    @property
    def max_episode_length(self) -> int:
        import math

        return math.ceil(self.episode_length_s / (self.sim.dt * self.decimation))

    def quad_task(self) -> dict:
        """The as_quad_task_t fields (_native.NativeEnv.set_quad_task / oracle OrQuadTask)."""
        import numpy as np

        return {"stop_frames": self.stop_frames, "alive": self.alive_reward, "action_cost": self.action_cost,
                "death": self.death_reward, "min_height": self.min_height, "up_z_min": self.up_z_min,
                "max_episode_length": self.max_episode_length,
                "step_dt": float(np.float32(self.sim.dt * self.decimation)), "stand_height": self.stand_height,
                "joint_noise": self.joint_noise, "energy_cost": self.energy_cost, "step_radius": self.step_radius,
                "step_reward": self.step_reward, "step_sigma": self.step_sigma, "target_bonus": self.target_bonus,
                "bonus_radius": self.bonus_radius, "foot_progress": self.foot_progress,
                "foot_offset_y": list(self.foot_offset_y)}

    def actuator(self) -> dict:
        r = self.robot
        return {"stiffness": r.stiffness, "damping": r.damping, "saturation_effort": r.saturation_effort,
                "effort_limit": r.effort_limit, "velocity_limit": r.velocity_limit}
