"""ctypes binding of the CPU oracle (TEST INFRASTRUCTURE ONLY -- see oracle.h).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg import this
module, as the checker / reported CPU baseline.  The product (``allsteps_isaaclab_amd``) never
imports it.
"""

from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liballsteps_oracle.so")

MAXL, MAXG, MAXSP = 32, 32, 256
f3 = C.c_float * 3


class OrModel(C.Structure):
    _fields_ = [
        ("num_links", C.c_int32), ("num_hinges", C.c_int32), ("parent", C.c_int32 * MAXL),
        ("offset_pos", (C.c_float * 3) * MAXL), ("offset_quat", (C.c_float * 4) * MAXL),
        ("axis", (C.c_float * 3) * MAXL), ("anchor", (C.c_float * 3) * MAXL), ("mass", C.c_float * MAXL),
        ("com", (C.c_float * 3) * MAXL), ("inertia", (C.c_float * 6) * MAXL), ("armature", C.c_float * MAXL),
        ("lower", C.c_float * MAXL), ("upper", C.c_float * MAXL), ("cfg_dof_link", C.c_int32 * MAXL),
        ("gear", C.c_float * MAXL), ("num_geoms", C.c_int32), ("geom_link", C.c_int32 * MAXG),
        ("geom_type", C.c_int32 * MAXG), ("geom_foot", C.c_int32 * MAXG), ("geom_radius", C.c_float * MAXG),
        ("geom_p0", (C.c_float * 3) * MAXG), ("geom_p1", (C.c_float * 3) * MAXG), ("torso_link", C.c_int32),
        ("foot_link", C.c_int32 * 2), ("num_priority_geoms", C.c_int32), ("num_self_pairs", C.c_int32),
        ("self_pair", C.c_int32 * MAXSP),
    ]


class OrSim(C.Structure):
    _fields_ = [
        ("dt", C.c_float), ("substeps", C.c_int32), ("gravity", C.c_float), ("friction", C.c_float),
        ("margin", C.c_float), ("baumgarte", C.c_float), ("slop", C.c_float), ("max_depen_vel", C.c_float),
        ("pgs_iters", C.c_int32), ("stone_half", C.c_float * 3), ("max_joint_vel", C.c_float),
    ]


class OrTask(C.Structure):
    _fields_ = [
        ("num_steps", C.c_int32), ("step_radius", C.c_float), ("stop_frames", C.c_int32), ("eps", C.c_float),
        ("alive", C.c_float), ("energy", C.c_float), ("action", C.c_float), ("joint_limit", C.c_float),
        ("death", C.c_float), ("dof_vel_scale", C.c_float), ("fall_abs", C.c_float), ("step_dt", C.c_float),
        ("max_episode_length", C.c_int32), ("max_curriculum", C.c_int32), ("curriculum_threshold", C.c_int32),
        ("term_curriculum", C.c_float * 10), ("gain_curriculum", C.c_float * 10), ("init_root", C.c_float * 3),
        ("init_q", C.c_float * 21), ("right_idx", C.c_int32 * 9), ("left_idx", C.c_int32 * 9),
        ("neg_idx", C.c_int32 * 2), ("noise_lo", C.c_float), ("noise_hi", C.c_float), ("clip_lo", C.c_float),
        ("clip_hi", C.c_float), ("regen_footsteps", C.c_int32),
    ]


MAXC = 10  # oracle.h OR_MAX_CONTACTS


class OrProbe(C.Structure):
    _fields_ = [
        ("nfound", C.c_int32), ("nself_found", C.c_int32), ("ncap", C.c_int32), ("nlim", C.c_int32),
        ("ncontact", C.c_int32), ("link", C.c_int32 * MAXC), ("link2", C.c_int32 * MAXC),
        ("stone", C.c_int32 * MAXC), ("foot", C.c_int32 * MAXC), ("sep", C.c_float * MAXC),
        ("nrm", (C.c_float * 3) * MAXC), ("lam_n", C.c_float * MAXC), ("mask", C.c_uint32 * 2),
        ("stone_impulse", (C.c_float * 3) * 20), ("net_impulse", C.c_float * 3), ("recorded", C.c_int32),
    ]


FP = C.POINTER(C.c_float)
IP = C.POINTER(C.c_int32)
UP = C.POINTER(C.c_uint32)


class OrState(C.Structure):
    _fields_ = [
        ("n", C.c_int32), ("root_pos", FP), ("root_quat", FP), ("root_lin", FP), ("root_ang", FP), ("q", FP),
        ("qd", FP), ("stones", FP), ("pot", FP), ("old_pot", FP), ("foot_contact", FP), ("body_pos", FP),
        ("idx", IP), ("prev", IP), ("next", IP), ("count", IP), ("swing", IP), ("ep_len", IP), ("episode", UP),
        ("contact_mask", UP), ("curriculum", IP), ("contact_mask_hind", UP), ("feet", IP),
    ]


class OrActuator(C.Structure):
    _fields_ = [("mode", C.c_int32), ("action_scale", C.c_float), ("default_q", C.c_float * 21),
                ("stiffness", C.c_float), ("damping", C.c_float), ("saturation_effort", C.c_float),
                ("effort_limit", C.c_float), ("velocity_limit", C.c_float)]


QUAD_OBS = 64  # include/allsteps.h AS_QUAD_OBS_DIM


class OrQuadTask(C.Structure):
    _fields_ = [("stop_frames", C.c_int32), ("alive", C.c_float), ("action_cost", C.c_float), ("death", C.c_float),
                ("min_height", C.c_float), ("up_z_min", C.c_float), ("max_episode_length", C.c_int32),
                ("step_dt", C.c_float), ("stand_height", C.c_float), ("joint_noise", C.c_float),
                ("energy_cost", C.c_float), ("step_radius", C.c_float), ("step_reward", C.c_float),
                ("step_sigma", C.c_float), ("target_bonus", C.c_float), ("bonus_radius", C.c_float),
                ("foot_progress", C.c_float), ("foot_offset_y", C.c_float * 4)]


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_LIB = None


def lib() -> C.CDLL:
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            build()
        _LIB = C.CDLL(LIB_PATH)
        L = _LIB
        V = C.c_void_p
        L.or_task_post_physics.argtypes = [V, V, V, FP, FP, FP, FP, C.c_uint64, V, V, FP, FP,
                                           C.POINTER(C.c_uint8), C.POINTER(C.c_uint8), IP]
        L.or_task_reset_all.argtypes = [V, V, V, FP, C.c_uint64, FP]
        L.or_task_reset_mask.argtypes = [V, V, V, C.POINTER(C.c_uint8), FP, C.c_uint64, FP]
        L.or_env_step.argtypes = [V, V, V, V, FP, FP, C.c_uint64, FP, FP, C.POINTER(C.c_uint8),
                                  C.POINTER(C.c_uint8), IP, C.POINTER(C.c_int64), C.c_int]
        L.or_physics_step.restype = C.c_int
        L.or_physics_step_act.restype = C.c_int
        L.or_env_reset_all.argtypes = [V, V, V, V, FP, C.c_uint64, FP]
        L.or_math_batch.argtypes = [C.c_int, FP, FP, FP, FP, FP]
        L.or_sft_batch.argtypes = [C.c_int, FP, FP, FP, FP]
        L.or_footsteps.argtypes = [V, C.c_int, C.c_int, FP, FP, FP]
        L.or_fk_bodies.argtypes = [V, FP, FP, FP, FP]
        L.or_mass_matrix.argtypes = [V, FP, FP, FP, FP, FP]
        L.or_bias_forces.argtypes = [V, FP, FP, FP, FP, C.c_float, FP]
        L.or_philox_uniform.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_int, FP]
        L.or_physics_step.argtypes = [V, V, V, V, C.c_int, FP]
        L.or_probe_substep.argtypes = [V, V, V, V, C.c_int, FP, V]
        L.or_physics_step_act.argtypes = [V, V, V, V, V, C.c_int, FP]
        L.or_dc_motor_batch.argtypes = [C.c_int, FP, FP, FP, V, FP]
        L.or_quad_post_physics.argtypes = [V, V, V, V, V, V, FP, C.c_int, C.c_uint64, FP, FP,
                                           C.POINTER(C.c_uint8), C.POINTER(C.c_uint8)]
        L.or_link_point.argtypes = [V, V, C.c_int, C.c_int, FP, FP]
        L.or_quad_step.argtypes = [V, V, V, V, V, V, FP, C.c_uint64, FP, FP, C.POINTER(C.c_uint8),
                                   C.POINTER(C.c_uint8), C.c_int]
    return _LIB


def fp(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(FP)


def ip(a: np.ndarray):
    assert a.dtype == np.int32 and a.flags.c_contiguous
    return a.ctypes.data_as(IP)


def up(a: np.ndarray):
    assert a.dtype == np.uint32 and a.flags.c_contiguous
    return a.ctypes.data_as(UP)


def u8p(a: np.ndarray):
    assert a.dtype == np.uint8 and a.flags.c_contiguous
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


# ---------------------------------------------------------------------------------- constructors

def make_model(m: dict) -> OrModel:
    M = OrModel()
    M.num_links = m["num_links"]
    M.num_hinges = m["num_hinges"]
    for name in ("parent", "cfg_dof_link", "geom_link", "geom_type", "geom_foot"):
        getattr(M, name)[:] = [int(x) for x in m[name]]
    for name in ("mass", "armature", "lower", "upper", "gear", "geom_radius"):
        getattr(M, name)[:] = [float(x) for x in m[name]]
    for name in ("offset_pos", "offset_quat", "axis", "anchor", "com", "inertia", "geom_p0", "geom_p1"):
        arr = getattr(M, name)
        for i, row in enumerate(m[name]):
            arr[i][:] = [float(x) for x in row]
    M.num_geoms = m["num_geoms"]
    M.num_priority_geoms = int(m["num_priority_geoms"])
    M.num_self_pairs = int(m["num_self_pairs"])
    M.self_pair[:] = [int(x) for x in m["self_pair"]]
    M.torso_link = int(m["torso_link"])
    M.foot_link[:] = [int(x) for x in m["foot_link"]]
    return M


def make_task(cfg, dof_names: list) -> OrTask:
    """as_task_t from the cfg (envs/task_table.py: shared with the HIP path, dispatched on the cfg type)."""
    from allsteps_isaaclab_amd.envs.task_table import fill, task_fields

    return fill(OrTask(), task_fields(cfg, dof_names))


def make_sim(cfg) -> OrSim:
    S = OrSim()
    s = cfg.sim
    S.dt = s.dt
    S.substeps = cfg.decimation
    S.gravity = s.gravity[2]
    S.friction = s.friction
    S.margin = s.contact_margin
    S.baumgarte = s.baumgarte
    S.slop = s.slop
    S.max_depen_vel = s.max_depenetration_velocity
    S.pgs_iters = s.solver_position_iteration_count
    sz = cfg.step_size
    S.stone_half[:] = [sz[0] / 2, sz[1] / 2, sz[2] / 2]
    S.max_joint_vel = s.max_joint_velocity
    return S


class OracleState:
    """Numpy-owned SoA state ([field][n]) bound to an OrState struct."""

    FIELDS_F = {"root_pos": 3, "root_quat": 4, "root_lin": 3, "root_ang": 3, "q": 21, "qd": 21, "stones": 60,
                "pot": 1, "old_pot": 1, "foot_contact": 2, "body_pos": 9}
    FIELDS_I = {"idx": 1, "prev": 1, "next": 1, "count": 1, "swing": 1, "ep_len": 1, "feet": 8}
    FIELDS_U = {"episode": 1, "contact_mask": 2, "contact_mask_hind": 2}

    def __init__(self, n: int):
        self.n = n
        self.a = {}
        for k, w in self.FIELDS_F.items():
            self.a[k] = np.zeros((w, n) if w > 1 else (n,), np.float32)
        for k, w in self.FIELDS_I.items():
            self.a[k] = np.zeros((w, n) if w > 1 else (n,), np.int32)
        for k, w in self.FIELDS_U.items():
            self.a[k] = np.zeros((w, n) if w > 1 else (n,), np.uint32)
        self.a["curriculum"] = np.zeros(1, np.int32)
        self.a["root_quat"][0] = 1.0
        self.a["idx"][:] = 1
        self.a["next"][:] = 2
        self.s = OrState()
        self.s.n = n
        for k in self.FIELDS_F:
            setattr(self.s, k, fp(self.a[k]))
        for k in list(self.FIELDS_I) + ["curriculum"]:
            setattr(self.s, k, ip(self.a[k]))
        for k in self.FIELDS_U:
            setattr(self.s, k, up(self.a[k]))

    def __getitem__(self, k):
        return self.a[k]

    @property
    def ptr(self):
        return C.byref(self.s)


class Oracle:
    """Bundle of model/sim/task structs + convenience calls."""

    def __init__(self, cfg=None, model: dict | None = None):
        from allsteps_isaaclab_amd.envs.allsteps_env_cfg import AllstepsEnvCfg
        from allsteps_isaaclab_amd.model import load_model

        self.cfg = cfg or AllstepsEnvCfg()
        self.m = model or load_model()
        self.model = make_model(self.m)
        self.task = make_task(self.cfg, self.m["dof_names"])
        self.sim = make_sim(self.cfg)
        self.L = lib()

    def state(self, n: int) -> OracleState:
        return OracleState(n)

    def env_step(self, st: OracleState, actions: np.ndarray, seed: int = 42, reset_draws=None, nthreads: int = 1):
        n = st.n
        actions = np.ascontiguousarray(actions, np.float32)
        obs = np.zeros((n, 59), np.float32)
        rew = np.zeros(n, np.float32)
        term = np.zeros(n, np.uint8)
        trunc = np.zeros(n, np.uint8)
        anyr = np.zeros(1, np.int32)
        drop = C.c_int64(0)
        rd = fp(np.ascontiguousarray(reset_draws, np.float32)) if reset_draws is not None else None
        self.L.or_env_step(C.byref(self.model), C.byref(self.sim), C.byref(self.task), st.ptr, fp(actions), rd,
                           seed, fp(obs), fp(rew), u8p(term), u8p(trunc), ip(anyr), C.byref(drop), nthreads)
        self.last_dropped = int(drop.value)  # contacts the row budget cut in this step (as_step_counters [3])
        return obs, rew, term.astype(bool), trunc.astype(bool), bool(anyr[0])

    def physics_step(self, st: OracleState, actions: np.ndarray) -> int:
        """Physics only (decimation substeps), no task logic: for known-answer tests.  Returns the
        contacts the row budget cut over all envs and substeps."""
        a = np.clip(np.ascontiguousarray(actions, np.float32), -1, 1)
        drop = 0
        for e in range(st.n):
            row = np.ascontiguousarray(a[e])
            drop += self.L.or_physics_step(C.byref(self.model), C.byref(self.sim), C.byref(self.task), st.ptr, e,
                                           fp(row))
        return drop

    def physics_step_act(self, st: OracleState, act: OrActuator, actions):
        """Physics only with an actuator (or_physics_step_act)."""
        a = np.clip(np.ascontiguousarray(actions, np.float32), -1, 1)
        for e in range(st.n):
            row = np.ascontiguousarray(a[e])
            self.L.or_physics_step_act(C.byref(self.model), C.byref(self.sim), C.byref(self.task), C.byref(act),
                                       st.ptr, e, fp(row))

    def quad_step(self, st: OracleState, act: OrActuator, q: OrQuadTask, actions, seed: int = 42, nthreads: int = 1):
        n = st.n
        obs = np.zeros((n, QUAD_OBS), np.float32)
        rew = np.zeros(n, np.float32)
        term = np.zeros(n, np.uint8)
        trunc = np.zeros(n, np.uint8)
        self.L.or_quad_step(C.byref(self.model), C.byref(self.sim), C.byref(self.task), C.byref(act), C.byref(q),
                            st.ptr, fp(np.ascontiguousarray(actions, np.float32)), seed, fp(obs), fp(rew), u8p(term),
                            u8p(trunc), nthreads)
        return obs, rew, term.astype(bool), trunc.astype(bool)

    def quad_reset_all(self, st: OracleState, act: OrActuator, q: OrQuadTask, seed: int = 42):
        obs = np.zeros((st.n, QUAD_OBS), np.float32)
        z = np.zeros(1, np.float32)
        self.L.or_quad_post_physics(C.byref(self.model), C.byref(self.sim), C.byref(self.task), C.byref(act),
                                    C.byref(q), st.ptr, fp(z), 1, seed, fp(obs), None, None, None)
        return obs

    def probe(self, st: OracleState, e: int = 0, actions=None) -> dict:
        """The constraint set and contact impulses of env e's first substep, plus the stone impulses
        summed over the env step's substeps (or_probe_substep); the state is not advanced."""
        nh = self.m["num_hinges"]
        a = np.zeros(nh, np.float32) if actions is None else np.clip(np.asarray(actions, np.float32), -1, 1)
        P = OrProbe()
        self.L.or_probe_substep(C.byref(self.model), C.byref(self.sim), C.byref(self.task), st.ptr, e,
                                fp(np.ascontiguousarray(a)), C.byref(P))
        k = P.ncontact
        return {"nfound": P.nfound, "nself_found": P.nself_found, "ncap": P.ncap, "nlim": P.nlim, "ncontact": k,
                "link": np.array(P.link[:k]), "link2": np.array(P.link2[:k]), "stone": np.array(P.stone[:k]),
                "foot": np.array(P.foot[:k]), "sep": np.array(P.sep[:k], np.float32),
                "nrm": np.array([list(P.nrm[c]) for c in range(k)], np.float32).reshape(k, 3),
                "lam_n": np.array(P.lam_n[:k], np.float32), "mask": (P.mask[0], P.mask[1]),
                "stone_impulse": np.array([list(P.stone_impulse[s]) for s in range(20)], np.float32),
                "net_impulse": np.array(list(P.net_impulse), np.float32)}

    def reset_all(self, st: OracleState, seed: int = 42, reset_draws=None):
        obs = np.zeros((st.n, 59), np.float32)
        rd = fp(np.ascontiguousarray(reset_draws, np.float32)) if reset_draws is not None else None
        self.L.or_env_reset_all(C.byref(self.model), C.byref(self.sim), C.byref(self.task), st.ptr, rd, seed,
                                fp(obs))
        return obs

    def reset_mask(self, st: OracleState, mask, seed: int = 42, reset_draws=None):
        """_reset_idx on the envs with mask != 0, then the observations (or_task_reset_mask)."""
        obs = np.zeros((st.n, 59), np.float32)
        m = np.ascontiguousarray(np.asarray(mask) != 0, np.uint8)
        rd = fp(np.ascontiguousarray(reset_draws, np.float32)) if reset_draws is not None else None
        self.L.or_task_reset_mask(C.byref(self.model), C.byref(self.task), st.ptr, u8p(m), rd, seed, fp(obs))
        return obs

    def footsteps(self, n: int, level: int, draws: np.ndarray):
        pos = np.zeros((n, self.cfg.num_steps, 3), np.float32)
        dphi = np.zeros((n, self.cfg.num_steps), np.float32)
        self.L.or_footsteps(C.byref(self.task), n, level, fp(np.ascontiguousarray(draws, np.float32)), fp(pos),
                            fp(dphi))
        return pos, dphi

    def mass_matrix(self, root_quat, q_int):
        nv = 6 + self.m["num_hinges"]
        H = np.zeros((nv, nv), np.float32)
        com = np.zeros(3, np.float32)
        rp = np.zeros(3, np.float32)
        self.L.or_mass_matrix(C.byref(self.model), fp(rp), fp(np.asarray(root_quat, np.float32)),
                              fp(np.ascontiguousarray(q_int, np.float32)), fp(H), fp(com))
        return H, com

    def bias_forces(self, root_quat, q_int, u, gravity=-9.81):
        nv = 6 + self.m["num_hinges"]
        Cv = np.zeros(nv, np.float32)
        rp = np.zeros(3, np.float32)
        self.L.or_bias_forces(C.byref(self.model), fp(rp), fp(np.asarray(root_quat, np.float32)),
                              fp(np.ascontiguousarray(q_int, np.float32)), fp(np.ascontiguousarray(u, np.float32)),
                              gravity, fp(Cv))
        return Cv

    def fk_bodies(self, root_pos, root_quat, q_cfg):
        out = np.zeros(9, np.float32)
        self.L.or_fk_bodies(C.byref(self.model), fp(np.asarray(root_pos, np.float32)),
                            fp(np.asarray(root_quat, np.float32)), fp(np.ascontiguousarray(q_cfg, np.float32)),
                            fp(out))
        return out.reshape(3, 3)

    def link_point(self, st: OracleState, e: int, link: int, pl=(0.0, 0.0, 0.0)):
        """World position of pl (link frame) on `link` of env e (the C5 task's foot-tip FK)."""
        out = np.zeros(3, np.float32)
        self.L.or_link_point(C.byref(self.model), st.ptr, e, link, fp(np.asarray(pl, np.float32)), fp(out))
        return out

    def philox(self, seed: int, env: int, episode: int, k: int = 22):
        out = np.zeros(k, np.float32)
        self.L.or_philox_uniform(seed, env, episode, k, fp(out))
        return out
