"""``AllstepsEnv`` -- the Allsteps-v0 stepping-stone task on the MI355X-native step kernels.

Drop-in for ``isaaclab_tasks/direct/allsteps/allsteps_env.py:34-567`` (``AllstepsEnv``): same
constructor (``cfg, render_mode``), same ``step``/``reset`` results (policy obs (N, 59), reward,
terminated, truncated, extras), same task buffers (``curr_target_index``, ``swing_leg``,
``potentials`` ...), same mirror indices and symmetry functions.  Underneath, the whole
``DirectRLEnv.step`` -- actuation, 4 physics substeps, contacts, foot-state machine, rewards,
dones, resets, observations -- is two HIP kernels (``liballsteps_hip.so``) over a struct-of-arrays
state that stays resident in HBM; there is no PhysX, no Python per-step logic and no host sync.
"""

from __future__ import annotations

from typing import Tuple

import torch

from .. import _native
from ..model import joint_limits_cfg, load_model
from .allsteps_env_cfg import AllstepsEnvCfg
from .direct_rl_env import DirectRLEnv

RIGHT_FOOT = 0
LEFT_FOOT = 1
EPSILON = 1e-4

_FLOAT_FIELDS = [(n, r) for n, r, t in _native.STATE_LAYOUT if t == "f"]
_INT_FIELDS = [(n, r) for n, r, t in _native.STATE_LAYOUT if t == "i"]


class _RobotData:
    """The ``ArticulationData`` views (articulation_data.py:364-601).  Ring 1 -- what the task reads --
    as zero-copy (N, k) views of the SoA state (k-major storage, so rows are strided).  Ring 2 -- the
    body views of every MJCF body (``body_names``: the walker's 17, document order) -- computed on demand
    by the ``as_body_state`` HIP kernel (the step kernel's own FK of the state as it stands) each time one
    is read; the step never computes them (include/allsteps.h)."""

    def __init__(self, env: "AllstepsEnv"):
        self._env = env
        s = env.state
        n = env.num_envs
        self.joint_names = list(env.model["dof_names"])
        self.body_names = list(env.model["body_names"])
        self.num_bodies = len(self.body_names)
        self._body_table = _native.make_body_table(env.model)
        self._body_out = None
        nd = self._nd = int(env.model["num_hinges"])
        lim = torch.as_tensor(joint_limits_cfg(env.model), device=env._device)
        self.joint_pos_limits = lim.unsqueeze(0).expand(n, -1, -1)
        djp = getattr(env, "default_joint_pos", None)  # the quadruped's stand pose; the walker's is zero
        self.default_joint_pos = (djp.reshape(1, nd).expand(n, nd).clone() if torch.is_tensor(djp)
                                  else torch.zeros(n, nd, device=env._device))
        self.default_joint_vel = torch.zeros(n, nd, device=env._device)
        self.default_root_state = torch.zeros(n, 13, device=env._device)
        if getattr(env.cfg, "init_root_pos", None) is not None:
            self.default_root_state[:, :3] = torch.tensor(env.cfg.init_root_pos, device=env._device)
        self.default_root_state[:, 3] = 1.0
        self._s = s

    root_pos_w = property(lambda self: self._s["root_pos"].T)
    root_quat_w = property(lambda self: self._s["root_quat"].T)
    root_lin_vel_w = property(lambda self: self._s["root_lin"].T)
    root_ang_vel_w = property(lambda self: self._s["root_ang"].T)
    joint_pos = property(lambda self: self._s["q"][: self._nd].T)  # the state's rows past the model's hinges unused
    joint_vel = property(lambda self: self._s["qd"][: self._nd].T)

    @property
    def root_state_w(self) -> torch.Tensor:
        s = self._s
        return torch.cat([s["root_pos"], s["root_quat"], s["root_lin"], s["root_ang"]], 0).T.contiguous()

    def _bodies(self) -> torch.Tensor:
        """(16, B, N) as_body_state rows of the current state: pos 3 | quat 4 | frame lin vel 3 | ang vel 3 |
        COM lin vel 3 (one launch on the env's stream)."""
        env = self._env
        if self._body_out is None:
            self._body_out = torch.empty(_native.BODY_STATE_ROWS, self.num_bodies, env.num_envs, device=env._device)
        env._native.body_state(self._body_table, self._body_out, stream=env._stream())
        return self._body_out

    def _rows(self, lo: int, hi: int) -> torch.Tensor:
        return self._bodies()[lo:hi].permute(2, 1, 0).contiguous()

    @property
    def body_pos_w(self) -> torch.Tensor:
        """(N, B, 3) body (link-frame) positions, all bodies; rows torso / right_foot / left_foot equal the
        state's body_pos (the step's FK after the last substep) bit for bit."""
        return self._rows(0, 3)

    @property
    def body_quat_w(self) -> torch.Tensor:
        """(N, B, 4) body orientations (w, x, y, z)."""
        return self._rows(3, 7)

    @property
    def body_lin_vel_w(self) -> torch.Tensor:
        """(N, B, 3) linear velocities of the bodies' centres of mass (PhysX link velocities)."""
        return self._rows(13, 16)

    @property
    def body_ang_vel_w(self) -> torch.Tensor:
        return self._rows(10, 13)

    @property
    def body_state_w(self) -> torch.Tensor:
        """(N, B, 13) [pos, quat, lin_vel, ang_vel]: link-frame pose, centre-of-mass velocity
        (articulation_data.py:430-447)."""
        b = self._bodies()
        return torch.cat([b[0:7], b[13:16], b[10:13]], 0).permute(2, 1, 0).contiguous()

    @property
    def body_link_state_w(self) -> torch.Tensor:
        """(N, B, 13) link-frame pose and the link frame's own velocity (articulation_data.py:449-470)."""
        return self._rows(0, 13)

    @property
    def body_link_pos_w(self) -> torch.Tensor:
        return self._rows(0, 3)

    @property
    def body_link_vel_w(self) -> torch.Tensor:
        return self._rows(7, 13)

    @property
    def body_com_pos_w(self) -> torch.Tensor:
        """(N, B, 3) the bodies' own centres of mass (as_body_table_t.com, from the MJCF geoms)."""
        b = self._bodies()
        q = b[3:7].permute(2, 1, 0)
        com = torch.as_tensor(self._env.model["body_com"][: self.num_bodies], device=b.device)
        w, v = q[..., :1], q[..., 1:]
        c = com.expand_as(v)
        t = 2.0 * torch.linalg.cross(v, c, dim=-1)
        return b[0:3].permute(2, 1, 0) + c + w * t + torch.linalg.cross(v, t, dim=-1)


class _SensorData:
    def __init__(self, sensor: "_FootSensor"):
        self._sensor = sensor

    @property
    def force_matrix_w(self) -> torch.Tensor | None:
        """(N, B, 20, 3) FLAG-VALUED force matrix of the stones (filter_prim_paths_expr = the 20 steps):
        (0, 0, 1) N where the foot pushed on that stone with |F| > 1e-4 N in the env step's last
        substep (contact_sensor.py:341 with the contact solve's impulse / dt), 0 elsewhere.  The force
        itself is not kept by the step (only the flag the task reads: allsteps_env.py:421-425 tests
        ``vector_norm(force_matrix_w) > EPSILON``, which this view answers exactly).  None for the
        unfiltered two-foot sensor, as in the reference."""
        return self._sensor._force_matrix()

    @property
    def net_forces_w(self):
        raise _native.NativeError(
            "ContactSensor.data.net_forces_w is not available: the MI355X step keeps the per-stone contact "
            "flags of each foot (force_matrix_w, flag-valued), not net contact forces (INTEGRATION.md §C3)")


class _FootSensor:
    """The reference's foot ContactSensors (allsteps_env_cfg.py:119-130; contact_sensor.py:320-343):
    ``sensor_right`` / ``sensor_left`` (one foot, filtered by the 20 stones) and ``sensor`` (both feet,
    unfiltered), over the state's per-foot stone bitmasks (contact_mask)."""

    def __init__(self, env: "AllstepsEnv", feet: list, names: list, filtered: bool):
        self._env, self._feet, self._filtered = env, feet, filtered
        self.body_names = list(names)
        self.num_bodies = len(feet)
        self.data = _SensorData(self)

    def _force_matrix(self):
        if not self._filtered:
            return None
        env = self._env
        m = env.state["contact_mask"]  # (2, N) int32, bit s = stone s
        bits = torch.arange(env.num_steps, device=m.device, dtype=torch.int32)
        f = torch.zeros(env.num_envs, self.num_bodies, env.num_steps, 3, device=m.device)
        for k, foot in enumerate(self._feet):
            f[:, k, :, 2] = ((m[foot].unsqueeze(1) >> bits) & 1).float()
        return f


class _RobotView:
    """Minimal ``Articulation`` surface: ``data`` plus the state writers used on reset."""

    def __init__(self, env: "AllstepsEnv"):
        self._env = env
        self.data = _RobotData(env)
        self._ALL_INDICES = torch.arange(env.num_envs, dtype=torch.long, device=env._device)

    def write_root_pose_to_sim(self, root_pose: torch.Tensor, env_ids=None):
        ids = self._ALL_INDICES if env_ids is None else env_ids
        s = self._env.state
        s["root_pos"][:, ids] = root_pose[:, :3].T.to(s["root_pos"].dtype)
        s["root_quat"][:, ids] = root_pose[:, 3:7].T.to(s["root_quat"].dtype)

    def write_root_velocity_to_sim(self, root_velocity: torch.Tensor, env_ids=None):
        ids = self._ALL_INDICES if env_ids is None else env_ids
        s = self._env.state
        s["root_lin"][:, ids] = root_velocity[:, :3].T.float()
        s["root_ang"][:, ids] = root_velocity[:, 3:6].T.float()

    def write_joint_state_to_sim(self, position, velocity, joint_ids=None, env_ids=None):
        ids = self._ALL_INDICES if env_ids is None else env_ids
        s = self._env.state
        s["q"][:, ids] = position.T.float()
        s["qd"][:, ids] = velocity.T.float()


class AllstepsEnv(DirectRLEnv):
    cfg: AllstepsEnvCfg

    def __init__(self, cfg: AllstepsEnvCfg | None = None, render_mode: str | None = None, *,
                 env_id_offset: int = 0, model: dict | None = None, **kwargs):
        cfg = cfg if cfg is not None else AllstepsEnvCfg()
        super().__init__(cfg, render_mode, **kwargs)
        if self._device.type != "cuda" or not torch.cuda.is_available():
            raise _native.NativeError(
                f"AllstepsEnv runs on the HIP backend only (device={self._device}, HIP device available: "
                f"{torch.cuda.is_available()}); there is no CPU fallback")
        self.model = model if model is not None else load_model()
        n = self.num_envs
        dev = self._device
        # ---- SoA state, resident in HBM ([field][env])
        nf = sum(r for _, r in _FLOAT_FIELDS)
        ni = sum(r for _, r in _INT_FIELDS)
        self._fbuf = torch.zeros((nf, n), dtype=torch.float32, device=dev)
        self._ibuf = torch.zeros((ni, n), dtype=torch.int32, device=dev)
        self.state: dict[str, torch.Tensor] = {}
        o = 0
        for name, r in _FLOAT_FIELDS:
            self.state[name] = self._fbuf[o:o + r] if r > 1 else self._fbuf[o]
            o += r
        o = 0
        for name, r in _INT_FIELDS:
            self.state[name] = self._ibuf[o:o + r] if r > 1 else self._ibuf[o]
            o += r
        self.state["curriculum"] = torch.zeros(1, dtype=torch.int32, device=dev)
        self.state["root_quat"][0] = 1.0
        self.state["idx"][:] = 1
        self.state["next"][:] = 2
        self.env_id_offset = int(env_id_offset)
        self._seed_value = int(cfg.seed if cfg.seed is not None else 0)
        with torch.cuda.device(dev):
            self._native = _native.NativeEnv(n, self.model, cfg, self.state, self._seed_value,
                                             dev.index if dev.index is not None else torch.cuda.current_device(),
                                             self.env_id_offset)
            # footsteps generated once at init (allsteps_env.py:71), curriculum level 0 by default
            self._native.generate_stones(int(cfg.initial_stone_curriculum), stream=self._stream())
        # ---- DirectRLEnv buffers (direct_rl_env.py:179-185)
        self.reset_terminated = torch.zeros(n, dtype=torch.bool, device=dev)
        self.reset_time_outs = torch.zeros(n, dtype=torch.bool, device=dev)
        self.reward_buf = torch.zeros(n, dtype=torch.float32, device=dev)
        self.obs_buf = {"policy": torch.zeros(n, cfg.observation_space, device=dev)}
        self._actions = torch.zeros(n, cfg.action_space, device=dev)
        # ---- task constants / names (allsteps_env.py:41-92)
        self.num_steps = cfg.num_steps
        self.step_radius = cfg.step_radius
        self.stop_frames = cfg.stop_frames
        self.max_curriculum = torch.tensor(cfg.max_curriculum, dtype=torch.int64, device=dev)
        self.termination_curriculum = torch.as_tensor(_native.linspace_f32(0.75, 0.45, cfg.max_curriculum + 1),
                                                      device=dev)
        self.applied_gain_curriculum = torch.as_tensor(_native.linspace_f32(1.2, 1.2, cfg.max_curriculum + 1),
                                                       device=dev)
        self.joint_gears = torch.tensor(cfg.joint_gears, dtype=torch.float32, device=dev)
        self.robot = _RobotView(self)
        # foot contact sensors (allsteps_env.py:224-226): right = sensor foot 0, left = 1
        self.sensor_right = _FootSensor(self, [0], ["right_foot"], True)
        self.sensor_left = _FootSensor(self, [1], ["left_foot"], True)
        self.sensor = _FootSensor(self, [0, 1], ["right_foot", "left_foot"], False)
        jn = self.robot.data.joint_names
        self.foot_names = list(cfg.foot_names)
        self.foot_indices = [self.robot.data.body_names.index(x) for x in self.foot_names]
        self.torso_index = self.robot.data.body_names.index(cfg.torso_name)
        L = lambda names: torch.tensor([jn.index(x) for x in names], dtype=torch.int64, device=dev)  # noqa: E731
        self.hip_y_index = L(cfg.hip_y_names)
        self.right_body_indices = L(cfg.right_body_names)
        self.left_body_indices = L(cfg.left_body_names)
        self.negation_body_indices = L(cfg.negation_body_names)

    # ------------------------------------------------------------------ task buffers (views)
    episode_length_buf = property(lambda self: self.state["ep_len"])
    curr_target_index = property(lambda self: self.state["idx"])
    prev_target_index = property(lambda self: self.state["prev"])
    next_target_index = property(lambda self: self.state["next"])
    target_reach_count = property(lambda self: self.state["count"])
    swing_leg = property(lambda self: self.state["swing"])
    potentials = property(lambda self: self.state["pot"])
    old_potentials = property(lambda self: self.state["old_pot"])
    foot_contact = property(lambda self: self.state["foot_contact"].T)

    @property
    def curriculum(self) -> torch.Tensor:
        """Per-env curriculum level (all envs share one level in the reference, allsteps_env.py:472)."""
        return self.state["curriculum"].expand(self.num_envs)

    def _render_rgb(self, env_id: int):
        from .render import render_frame

        st = {k: self.state[k][..., env_id].detach().cpu().numpy() for k in ("root_pos", "root_quat", "q", "stones")}
        half = [0.5 * v for v in self.cfg.step_size]
        return render_frame(self.model, st["root_pos"], st["root_quat"], st["q"], st["stones"].reshape(-1, 3), half,
                            target=int(self.state["idx"][env_id]))

    @property
    def steps_pos(self) -> torch.Tensor:
        """(N, 20, 3) stepping-stone centres, env-local frame."""
        return self.state["stones"].view(self.num_steps, 3, -1).permute(2, 0, 1)

    @property
    def actions(self) -> torch.Tensor:
        return torch.clamp(self._actions, -1.0, 1.0)

    @property
    def reset_buf(self) -> torch.Tensor:
        return self.reset_terminated | self.reset_time_outs

    @property
    def targets_w(self) -> torch.Tensor:
        """(N, 3, 3) previous / current / next target stone (allsteps_env.py:459-467)."""
        sp = self.steps_pos
        ar = torch.arange(self.num_envs, device=self._device)
        idx = [self.state[k].long() for k in ("prev", "idx", "next")]
        return torch.stack([sp[ar, i] for i in idx], 1)

    # ------------------------------------------------------------------ native backend
    def _stream(self):
        return torch.cuda.current_stream(self._device).cuda_stream

    def _reseed(self, seed: int):
        self._seed_value = int(seed)
        self._native.set_seed(self._seed_value)

    def _reset_impl(self, reset_draws: torch.Tensor | None = None):
        obs = torch.empty(self.num_envs, self.cfg.observation_space, device=self._device)
        self._native.reset_all(obs, reset_draws, stream=self._stream())
        self.obs_buf = {"policy": obs}
        return self.obs_buf

    def _reset_idx(self, env_ids, reset_draws: torch.Tensor | None = None):
        """AllstepsEnv._reset_idx(env_ids) (allsteps_env.py:469-567): reset the given envs (curriculum
        gate and second foot-state tick for all envs, as the reference does), then refresh the
        observation buffer.  ``env_ids``: indices, a bool mask, or None (all envs)."""
        if env_ids is None:
            return self._reset_impl(reset_draws)
        ids = torch.as_tensor(env_ids, device=self._device)
        if ids.dtype == torch.bool:
            if ids.shape != (self.num_envs,):
                raise ValueError(f"env_ids mask must be ({self.num_envs},), got {tuple(ids.shape)}")
            mask = ids.to(torch.uint8).contiguous()
        else:
            ids = ids.long().reshape(-1)
            if ids.numel() and (int(ids.min()) < 0 or int(ids.max()) >= self.num_envs):
                raise IndexError(f"env_ids out of range [0, {self.num_envs})")
            mask = torch.zeros(self.num_envs, dtype=torch.uint8, device=self._device)
            mask[ids] = 1
        obs = torch.empty(self.num_envs, self.cfg.observation_space, device=self._device)
        d = None if reset_draws is None else reset_draws.to(self._device).float().contiguous()
        self._native.reset_mask(mask, obs, d, stream=self._stream())
        self.obs_buf = {"policy": obs}
        return self.obs_buf

    def _step_impl(self, action: torch.Tensor, reset_draws: torch.Tensor | None = None):
        a = action if (action.dtype == torch.float32 and action.is_contiguous()) else action.float().contiguous()
        if a.shape != (self.num_envs, self.cfg.action_space):
            raise ValueError(f"actions must be ({self.num_envs}, {self.cfg.action_space}), got {tuple(a.shape)}")
        obs = torch.empty(self.num_envs, self.cfg.observation_space, device=self._device)
        rew = torch.empty(self.num_envs, device=self._device)
        self._native.step(a, obs, rew, self.reset_terminated, self.reset_time_outs, reset_draws,
                          stream=self._stream())
        self._actions = a
        self.obs_buf = {"policy": obs}
        self.reward_buf = rew
        return self.obs_buf, rew, self.reset_terminated, self.reset_time_outs, self.extras

    # ---- HIP-graph capture of step() (trainer rollout graphs)
    graph_safe_step = True  # step() launches only stream-ordered work with no host synchronisation

    def set_graph_capture(self, on: bool = True) -> None:
        """Make ``step`` replayable from a captured HIP graph (as_set_graph_safe: fixed counter bank,
        cleared by a memset node per call)."""
        self._native.set_graph_safe(on)

    def account_steps(self, k: int = 1) -> None:
        """Advance the host-side step counters for ``k`` steps replayed from a graph (the replay runs
        the device work of ``step`` but not its Python bookkeeping)."""
        self._sim_step_counter += self.cfg.decimation * k
        self.common_step_counter += k

    def step_with_draws(self, action: torch.Tensor, reset_draws: torch.Tensor):
        """``step`` with injected reset draws ((N, 22) U[0,1): mirror, 21 joint noise) -- parity tests."""
        self._sim_step_counter += self.cfg.decimation
        out = self._step_impl(action.to(self._device), reset_draws.to(self._device).float().contiguous())
        self.common_step_counter += 1
        return out

    def reset_with_draws(self, reset_draws: torch.Tensor):
        return self._reset_impl(reset_draws.to(self._device).float().contiguous()), self.extras

    def task_step(self, action: torch.Tensor, reset_draws: torch.Tensor | None = None):
        """Post-physics half of ``step`` on the current state (body_pos / contact_mask as written)."""
        a = action.to(self._device).float().contiguous()
        obs = torch.empty(self.num_envs, self.cfg.observation_space, device=self._device)
        rew = torch.empty(self.num_envs, device=self._device)
        d = None if reset_draws is None else reset_draws.to(self._device).float().contiguous()
        self._native.task_step(a, obs, rew, self.reset_terminated, self.reset_time_outs, d, stream=self._stream())
        return {"policy": obs}, rew, self.reset_terminated, self.reset_time_outs, self.extras

    def physics_step(self, action: torch.Tensor):
        """Physics only (4 substeps, no task logic) -- known-answer tests / profiling."""
        a = action.to(self._device).float().contiguous()
        self._native.physics_step(a, stream=self._stream())

    def generate_foot_steps(self, level: int, draws: torch.Tensor | None = None):
        """_generate_foot_steps_allsteps at `level` for every env (allsteps_env.py:106-174)."""
        d = None if draws is None else draws.to(self._device).float().contiguous()
        self._native.generate_stones(int(level), d, stream=self._stream())

    def dropped_contacts(self) -> int:
        """Contacts the constraint budget (AS_MAX_CONTACTS contacts, AS_MAX_ROWS rows incl. the joint
        limits) cut in the last step, over all envs and substeps -- PhysX keeps every contact
        (simulation_cfg.py:110), so this is the step's deviation from it in contact count.  Reads the
        device counter (as_step_counters word 3): synchronises the env's stream."""
        return int(self._native.counters_host(self._stream())[3])

    def get_state(self) -> dict:
        """Copy of the full SoA state (field -> (rows, N) tensor)."""
        return {k: v.clone() for k, v in self.state.items()}

    def set_state(self, state: dict):
        for k, v in state.items():
            self.state[k].copy_(torch.as_tensor(v).to(self.state[k].device, self.state[k].dtype).reshape(
                self.state[k].shape))

    def close(self):
        if getattr(self, "_native", None) is not None:
            self._native.close()
            self._native = None
        super().close()


# ------------------------------------------------------------------------------------------------
# mirror augmentation (allsteps_env.py:570-660)

def _mirror_indices(env, obs_dim: int, act_dim: int, device):
    uw = env.unwrapped
    right, left, neg = uw.right_body_indices, uw.left_body_indices, uw.negation_body_indices
    K = 2 if obs_dim == 56 else 3
    steps_neg = torch.tensor([K * i + 1 for i in range(3)], dtype=torch.int64, device=device)
    root_neg = torch.tensor([1, 4], dtype=torch.int64, device=device)
    r_obs = torch.cat((right + 6, right + 6 + act_dim, torch.tensor([6 + act_dim * 2], device=device)))
    l_obs = torch.cat((left + 6, left + 6 + act_dim, torch.tensor([6 + act_dim * 2 + 1], device=device)))
    n_obs = torch.cat((root_neg, 6 + neg, 6 + act_dim + neg, 6 + act_dim * 2 + 2 + steps_neg))
    return right, left, neg, r_obs, l_obs, n_obs


def _mirror(x, right, left, neg):
    y = x.clone()
    y[:, right] = x[:, left]
    y[:, left] = x[:, right]
    y[:, neg] = -x[:, neg]
    return y


def get_symmetric_states_rsl_rl(obs, actions, env, is_critic: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
    uw = env.unwrapped
    dev = uw.right_body_indices.device
    right, left, neg, r_obs, l_obs, n_obs = _mirror_indices(env, uw.observation_space.shape[1],
                                                            uw.action_space.shape[1], dev)
    ro = None if obs is None else torch.vstack((obs, _mirror(obs, r_obs, l_obs, n_obs)))
    ra = None if actions is None else torch.vstack((actions, _mirror(actions, right, left, neg)))
    return ro, ra


def get_symmetric_states_rl_games(obs, actions, env, is_critic: bool, mus):
    ro, ra = get_symmetric_states_rsl_rl(obs, actions, env, is_critic)
    if mus is None:
        return ro, ra, None
    uw = env.unwrapped
    rm = torch.vstack((mus, _mirror(mus, uw.right_body_indices, uw.left_body_indices, uw.negation_body_indices)))
    return ro, ra, rm
