"""``AllstepsEnvCfg`` -- the configuration surface of the reference task, MI355X-native backend.

Mirrors ``isaaclab_tasks/direct/allsteps/allsteps_env_cfg.py:51-235`` field for field where the
field means something without Omniverse (env counts, timing, reward scales, names, reset ranges),
plus the physics constants that replace the PhysX scene/articulation settings
(``simulation_cfg.py``, ``walker3d.py:21-46``).  USD/visual fields (markers, lights, materials,
prim paths) have no meaning here and are not carried.
"""

from __future__ import annotations

import dataclasses
import math
from dataclasses import dataclass, field


@dataclass
class SimulationCfg:
    """Physics constants (``isaaclab/sim/simulation_cfg.py``; ``walker3d.py:21-46``)."""

    dt: float = 1.0 / 240.0                 # allsteps_env_cfg.py:62
    render_interval: int = 4
    device: str = "cuda:0"
    gravity: tuple = (0.0, 0.0, -9.81)      # simulation_cfg.py gravity
    # Contact / solver settings replacing PhysX TGS (walker3d.py:26-32: 4 position iterations,
    # max_depenetration_velocity 10).  Friction: "average" combine of the MJCF geom friction 1.2
    # and the PhysX default material 0.5 (simulation_cfg.py default material) -> 0.85.
    friction: float = 0.85
    contact_margin: float = 0.01
    baumgarte: float = 0.2
    slop: float = 0.002
    max_depenetration_velocity: float = 10.0
    solver_position_iteration_count: int = 4
    max_joint_velocity: float = 100.0


@dataclass
class InteractiveSceneCfg:
    num_envs: int = 4096                    # allsteps_env_cfg.py:78
    env_spacing: float = 4.0
    replicate_physics: bool = True


@dataclass
class AllstepsEnvCfg:
    # env (allsteps_env_cfg.py:53-59)
    episode_length_s: float = 15.0
    decimation: int = 4
    action_scale: float = 1.0
    action_space: int = 21
    observation_space: int = 59
    state_space: int = 0
    seed: int | None = 42
    is_finite_horizon: bool = False          # direct_rl_env_cfg.py:59

    sim: SimulationCfg = field(default_factory=SimulationCfg)
    scene: InteractiveSceneCfg = field(default_factory=InteractiveSceneCfg)

    # steps (allsteps_env_cfg.py:90-97)
    num_steps: int = 20
    step_size: tuple = (0.5, 0.8, 0.225)
    step_radius: float = 0.25
    camera_pos: tuple = (1.5, -4.0, 1.5)
    # Curriculum level the stones are generated at.  The reference generates them once at level 0
    # (allsteps_env.py:71) and never regenerates; C3 uses 9 as an init knob.
    initial_stone_curriculum: int = 0
    # The reference never regenerates stones (its _reset_idx resets curr_target_index before testing
    # it, allsteps_env.py:492-500).  True = the intended behaviour: a reset env
    # whose target index was past half the stones gets a new course at the current curriculum level.
    regenerate_footsteps: bool = False

    # joint gears, cfg/PhysX dof order (allsteps_env_cfg.py:133-155)
    joint_gears: list = field(default_factory=lambda: [
        60, 80, 60, 50, 60, 60, 50, 60, 60, 60, 60, 80, 100, 60, 80, 100, 60, 90, 90, 60, 60])
    force_scale: float = 1.5

    torso_name: str = "torso"
    foot_names: list = field(default_factory=lambda: ["right_foot", "left_foot"])
    hip_y_names: list = field(default_factory=lambda: ["right_hip_y", "left_hip_y"])
    right_body_names: list = field(default_factory=lambda: [
        "right_shoulder_x", "right_shoulder_y", "right_shoulder_z", "right_elbow", "right_hip_x",
        "right_hip_y", "right_hip_z", "right_knee", "right_ankle"])
    left_body_names: list = field(default_factory=lambda: [
        "left_shoulder_x", "left_shoulder_y", "left_shoulder_z", "left_elbow", "left_hip_x",
        "left_hip_y", "left_hip_z", "left_knee", "left_ankle"])
    negation_body_names: list = field(default_factory=lambda: ["abdomen_z", "abdomen_x"])

    # reward scales (allsteps_env_cfg.py:222-234)
    energy_cost_scale: float = 0.009
    actions_cost_scale: float = 0.01
    alive_reward_scale: float = 2.0
    dof_vel_scale: float = 0.1
    joint_at_limit_cost_scale: float = 0.1
    death_cost: float = -1.0
    termination_height_absolute: float = 0.4
    angular_velocity_scale: float = 0.25
    initial_joint_angle_range: list = field(default_factory=lambda: [-0.1, 0.1])
    initial_joint_angle_clip_range: list = field(default_factory=lambda: [-0.95, 0.95])

    # task constants hard-coded in allsteps_env.py:29-60
    epsilon: float = 1e-4
    stop_frames: int = 2
    max_curriculum: int = 9
    curriculum_progress_threshold: int = 12
    init_root_pos: tuple = (0.2, 0.0, 1.5)   # walker3d.py:37

    def replace(self, **kw) -> "AllstepsEnvCfg":
        return dataclasses.replace(self, **kw)

    @property
    def step_dt(self) -> float:
        return self.sim.dt * self.decimation

    @property
    def max_episode_length(self) -> int:
        # direct_rl_env.py:247-250
        return math.ceil(self.episode_length_s / (self.sim.dt * self.decimation))


def running_start_pose() -> list:
    """allsteps_env.py:505-511: running-start joint pose, cfg dof order."""
    q = [0.0] * 21
    q[12] = q[17] = -math.pi / 8
    q[15] = math.pi / 10
    q[2] = q[5] = math.pi / 3
    q[4] = -math.pi / 6
    q[7] = math.pi / 6
    q[9] = q[10] = math.pi / 3
    return q
