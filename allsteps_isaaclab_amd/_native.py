"""ctypes binding of ``liballsteps_hip.so`` (the C ABI of ``include/allsteps.h``).

The product path has no fallback: if the HIP library is missing or no gfx950 device is present the
calls raise :class:`NativeError` -- nothing silently runs on the CPU.
"""

from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG, "liballsteps_hip.so")
PPO_LIB_PATH = os.path.join(PKG, "libppo_hip.so")
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(os.path.dirname(PKG), "include")

MAXL, MAXG, MAXSP = 32, 32, 256
ABI_VERSION = 5

EXPORTED_SYMBOLS = [
    "as_create", "as_destroy", "as_reset_all", "as_step", "as_physics_step", "as_generate_stones",
    "as_step_counters", "as_get_curriculum_host", "as_abi_version", "as_last_error", "as_task_step",
    "as_set_seed", "as_profile", "as_profile_read", "as_debug_stamps", "as_reset_mask", "as_set_graph_safe",
    "as_profile_sampled", "as_hbm_copy", "as_set_actuator", "as_set_quad_task", "as_quad_step", "as_quad_reset_all",
    "as_build_id", "as_step_counters_host", "as_body_state", "as_sweep_plan",
]
MAXB = 32  # AS_MAX_BODIES
BODY_STATE_ROWS = 16  # AS_BODY_STATE_ROWS: pos 3 | quat 4 | frame lin vel 3 | ang vel 3 | COM lin vel 3


class NativeError(RuntimeError):
    pass


class AsBodyTable(C.Structure):
    """as_body_table_t (include/allsteps.h): the model's bodies for as_body_state."""
    _fields_ = [("num_bodies", C.c_int32), ("link", C.c_int32 * MAXB), ("offset_pos", (C.c_float * 3) * MAXB),
                ("offset_quat", (C.c_float * 4) * MAXB), ("com", (C.c_float * 3) * MAXB)]


def make_body_table(m: dict) -> AsBodyTable:
    t = AsBodyTable()
    nb = int(m["num_bodies"])
    t.num_bodies = nb
    for k in range(nb):
        t.link[k] = int(m["body_link"][k])
        t.offset_pos[k][:] = [float(x) for x in m["body_offset_pos"][k]]
        t.offset_quat[k][:] = [float(x) for x in m["body_offset_quat"][k]]
        t.com[k][:] = [float(x) for x in m["body_com"][k]]
    return t


class AsModel(C.Structure):
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


class AsSim(C.Structure):
    _fields_ = [
        ("dt", C.c_float), ("substeps", C.c_int32), ("gravity", C.c_float), ("friction", C.c_float),
        ("margin", C.c_float), ("baumgarte", C.c_float), ("slop", C.c_float), ("max_depen_vel", C.c_float),
        ("pgs_iters", C.c_int32), ("stone_half", C.c_float * 3), ("max_joint_vel", C.c_float),
    ]


class AsTask(C.Structure):
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


VP = C.c_void_p


class AsState(C.Structure):
    _fields_ = [(name, VP) for name in (
        "root_pos", "root_quat", "root_lin", "root_ang", "q", "qd", "stones", "pot", "old_pot", "foot_contact",
        "body_pos", "idx", "prev", "next", "count", "swing", "ep_len", "episode", "contact_mask", "curriculum",
        "contact_mask_hind", "feet")]


class AsActuator(C.Structure):
    _fields_ = [("mode", C.c_int32), ("action_scale", C.c_float), ("default_q", C.c_float * 21),
                ("stiffness", C.c_float), ("damping", C.c_float), ("saturation_effort", C.c_float),
                ("effort_limit", C.c_float), ("velocity_limit", C.c_float)]


class AsQuadTask(C.Structure):
    _fields_ = [("stop_frames", C.c_int32), ("alive", C.c_float), ("action_cost", C.c_float), ("death", C.c_float),
                ("min_height", C.c_float), ("up_z_min", C.c_float), ("max_episode_length", C.c_int32),
                ("step_dt", C.c_float), ("stand_height", C.c_float), ("joint_noise", C.c_float),
                ("energy_cost", C.c_float), ("step_radius", C.c_float), ("step_reward", C.c_float),
                ("step_sigma", C.c_float), ("target_bonus", C.c_float), ("bonus_radius", C.c_float),
                ("foot_progress", C.c_float), ("foot_offset_y", C.c_float * 4)]


ACT_TORQUE, ACT_DC_MOTOR = 0, 1
QUAD_OBS_DIM = 64


# (field, rows, dtype) of the SoA state, in as_state_t order
STATE_LAYOUT = [
    ("root_pos", 3, "f"), ("root_quat", 4, "f"), ("root_lin", 3, "f"), ("root_ang", 3, "f"), ("q", 21, "f"),
    ("qd", 21, "f"), ("stones", 60, "f"), ("pot", 1, "f"), ("old_pot", 1, "f"), ("foot_contact", 2, "f"),
    ("body_pos", 9, "f"), ("idx", 1, "i"), ("prev", 1, "i"), ("next", 1, "i"), ("count", 1, "i"),
    ("swing", 1, "i"), ("ep_len", 1, "i"), ("episode", 1, "i"), ("contact_mask", 2, "i"),
]

_LIB = None


def lib_path() -> str:
    return os.environ.get("ALLSTEPS_HIP_LIB", LIB_PATH)


def source_digest() -> str:
    """Provenance digest of the native sources: sha256 over every csrc/*.hip, csrc/*.h and include/*.h
    (name + bytes, sorted by name) and both libraries' compile flags (include path excluded, so the
    digest is the same in any checkout), first 16 hex digits.  build_native() compiles it into
    both libraries (as_build_id / ppo_build_id); load() refuses a library whose id differs."""
    import hashlib

    h = hashlib.sha256()
    files = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".h"))]
    files += [os.path.join(INCLUDE, f) for f in os.listdir(INCLUDE) if f.endswith(".h")]
    for path in sorted(files, key=os.path.basename):
        h.update(os.path.basename(path).encode() + b"\0")
        with open(path, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    for flags in (STEP_FLAGS, PPO_FLAGS):
        h.update(" ".join(x for x in flags if x != INCLUDE).encode() + b"\0")
    return h.hexdigest()[:16]


def check_build_id(lib_id: bytes | str, path: str, env_var: str) -> None:
    """Raise NativeError when the library at `path` was not built from this tree's sources, unless the
    caller chose the library explicitly through `env_var` (A/B variants, diagnostic builds)."""
    if env_var in os.environ:
        return
    got = lib_id.decode(errors="replace") if isinstance(lib_id, bytes) else str(lib_id)
    want = source_digest()
    if got != want:
        raise NativeError(f"{path} was built from other sources (build id {got}, this tree {want}): rebuild it "
                          f"(`python -c 'import __graft_entry__ as g; g.build()'`), or set {env_var} to load a "
                          f"variant on purpose")


def load() -> C.CDLL:
    """Load liballsteps_hip.so (raises NativeError if it is missing: build it with build_native())."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = lib_path()
    if not os.path.exists(path):
        raise NativeError(f"{path} not found: the HIP extension is not built "
                          f"(run `python -c 'import __graft_entry__ as g; g.build()'`)")
    L = C.CDLL(path)
    V, I32, I64, U64 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint64
    L.as_create.argtypes = [I32, V, V, V, V, U64, I32, I64, C.POINTER(V)]
    L.as_destroy.argtypes = [V]
    L.as_reset_all.argtypes = [V, V, V, V]
    L.as_reset_mask.argtypes = [V, V, V, V, V]
    L.as_step.argtypes = [V, V, V, V, V, V, V, V]
    L.as_physics_step.argtypes = [V, V, V]
    L.as_task_step.argtypes = [V, V, V, V, V, V, V, V]
    L.as_set_seed.argtypes = [V, U64]
    L.as_set_graph_safe.argtypes = [V, I32]
    L.as_profile.argtypes = [V, I32]
    L.as_profile_sampled.argtypes = [V, I32, I32]
    L.as_debug_stamps.argtypes = [V, V]
    L.as_profile_read.argtypes = [V, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(I32)]
    L.as_generate_stones.argtypes = [V, I32, V, V]
    L.as_step_counters.argtypes = [V, C.POINTER(V)]
    L.as_get_curriculum_host.argtypes = [V, C.POINTER(I32)]
    L.as_step_counters_host.argtypes = [V, C.POINTER(I32), V]
    L.as_hbm_copy.argtypes = [V, V, I64, V]
    L.as_set_actuator.argtypes = [V, V]
    L.as_set_quad_task.argtypes = [V, V]
    L.as_quad_step.argtypes = [V, V, V, V, V, V, V]
    L.as_quad_reset_all.argtypes = [V, V, V]
    L.as_body_state.argtypes = [V, V, V, V]
    L.as_sweep_plan.argtypes = [V, C.POINTER(C.c_uint64)]
    L.as_last_error.restype = C.c_char_p
    L.as_build_id.restype = C.c_char_p
    for name in EXPORTED_SYMBOLS:
        if name not in ("as_last_error", "as_build_id"):
            getattr(L, name).restype = C.c_int
    if L.as_abi_version() != ABI_VERSION:
        raise NativeError(f"ABI version mismatch: library {L.as_abi_version()} != {ABI_VERSION}")
    check_build_id(L.as_build_id(), path, "ALLSTEPS_HIP_LIB")
    _LIB = L
    return L


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().as_last_error().decode(errors="replace")
        raise NativeError(f"{what} failed ({rc}): {msg}")


def hbm_copy_bandwidth(device, nbytes: int = 2 << 30, iters: int = 20) -> float:
    """Achievable HBM bandwidth (GB/s, read + write bytes) of the in-tree STREAM-copy kernel
    (as_hbm_copy) between two `nbytes` device buffers, timed with HIP events on the current stream."""
    import torch

    L = load()
    n16 = nbytes // 16
    src = torch.empty(n16 * 4, dtype=torch.float32, device=device).uniform_()
    dst = torch.empty_like(src)
    stream = torch.cuda.current_stream(device)
    sp = C.c_void_p(stream.cuda_stream)
    for _ in range(3):
        check(L.as_hbm_copy(C.c_void_p(dst.data_ptr()), C.c_void_p(src.data_ptr()), n16, sp), "as_hbm_copy")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(iters):
        check(L.as_hbm_copy(C.c_void_p(dst.data_ptr()), C.c_void_p(src.data_ptr()), n16, sp), "as_hbm_copy")
    e1.record(stream)
    e1.synchronize()
    ok = bool(torch.equal(src, dst))
    ms = e0.elapsed_time(e1) / iters
    del src, dst
    if not ok:
        raise NativeError("as_hbm_copy: destination differs from source")
    return 2.0 * n16 * 16 / (ms * 1e-3) / 1e9


# the step library's device-code flags (tests/test_kernel_budget.py compiles with exactly these):
# -ffp-contract=off: no implicit FMA contraction -- every FMA of the physics path is an explicit fmaf()
# in the order include/as_detmath.h fixes, so the oracle (built the same way) rounds identically and
# HIP <-> oracle parity is bit-exact.  -fno-slp-vectorize: the SLP pairs of the step kernel's scalar
# code cost more register moves than they save (launch -2 %); the packed math that pays
# (sweep, W rows) is written out as 2-vectors
STEP_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize", "-I", INCLUDE]
PPO_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fno-slp-vectorize", "-I", INCLUDE]


def build_native(verbose: bool = False) -> str:
    """Compile liballsteps_hip.so and libppo_hip.so for gfx950 in-tree (hipcc)."""
    import subprocess

    srcs = [os.path.join(CSRC, f) for f in ("allsteps_kernels.hip", "allsteps_abi.hip")]
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    digest = source_digest()
    cmd = [hipcc, *STEP_FLAGS, f'-DAS_BUILD_ID="{digest}"', "-fPIC", "-shared", "-Wno-unused-result", "-o",
           LIB_PATH] + srcs
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    # PPO-update kernels (include/ppo.h) -> libppo_hip.so
    cmd = [hipcc, *PPO_FLAGS, f'-DPPO_BUILD_ID="{digest}"', "-fPIC", "-shared", "-Wno-unused-result",
           "-o", PPO_LIB_PATH, os.path.join(CSRC, "ppo_kernels.hip"), os.path.join(CSRC, "ppo_mlp.hip"),
           os.path.join(CSRC, "ppo_wgrad.hip")]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    return LIB_PATH


# ------------------------------------------------------------------------------------------ structs

def sweep_plan(m: dict) -> tuple[int, int]:
    """as_sweep_plan: (1 if the step kernel's compiled sweep skips hold for model `m`, else 0; the mask of
    column quads that are exactly zero for it).  Host-only (no device)."""
    L = load()
    M = make_model(m)
    mask = C.c_uint64(0)
    rc = L.as_sweep_plan(C.byref(M), C.byref(mask))
    if rc < 0:
        raise NativeError(L.as_last_error().decode())
    return rc, int(mask.value)


def make_model(m: dict) -> AsModel:
    M = AsModel()
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


from .envs.task_table import linspace_f32  # noqa: E402  (re-exported: allsteps_env.py)


def make_task(cfg, dof_names: list) -> AsTask:
    """as_task_t from the cfg (envs/task_table.py: shared with the oracle, dispatched on the cfg type)."""
    from allsteps_isaaclab_amd.envs.task_table import fill, task_fields

    return fill(AsTask(), task_fields(cfg, dof_names))


def make_sim(cfg) -> AsSim:
    S = AsSim()
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


class NativeEnv:
    """Owns an ``as_env_t`` handle over caller-owned (torch) SoA state tensors."""

    def __init__(self, n: int, model: dict, cfg, state: dict, seed: int, device_index: int, env_offset: int = 0):
        self.L = load()
        self.n = n
        self._model = make_model(model)
        self._sim = make_sim(cfg)
        self._task = make_task(cfg, model["dof_names"])
        self._state_tensors = state  # keep alive
        S = AsState()
        for name, _, _ in STATE_LAYOUT:
            setattr(S, name, state[name].data_ptr())
        S.curriculum = state["curriculum"].data_ptr()
        S.contact_mask_hind = state["contact_mask_hind"].data_ptr() if "contact_mask_hind" in state else None
        S.feet = state["feet"].data_ptr() if "feet" in state else None
        self._state = S
        h = C.c_void_p()
        check(self.L.as_create(n, C.byref(self._model), C.byref(self._sim), C.byref(self._task), C.byref(S),
                               seed & 0xFFFFFFFFFFFFFFFF, device_index, env_offset, C.byref(h)), "as_create")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.L.as_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def step(self, actions, obs, rew, term, trunc, reset_draws=None, stream=None):
        check(self.L.as_step(self.h, actions.data_ptr(), obs.data_ptr(), rew.data_ptr(), term.data_ptr(),
                             trunc.data_ptr(), reset_draws.data_ptr() if reset_draws is not None else None,
                             stream), "as_step")

    def task_step(self, actions, obs, rew, term, trunc, reset_draws=None, stream=None):
        check(self.L.as_task_step(self.h, actions.data_ptr(), obs.data_ptr(), rew.data_ptr(), term.data_ptr(),
                                  trunc.data_ptr(), reset_draws.data_ptr() if reset_draws is not None else None,
                                  stream), "as_task_step")

    def set_seed(self, seed: int):
        check(self.L.as_set_seed(self.h, seed & 0xFFFFFFFFFFFFFFFF), "as_set_seed")

    def set_graph_safe(self, on: bool):
        check(self.L.as_set_graph_safe(self.h, int(bool(on))), "as_set_graph_safe")

    def reset_all(self, obs, reset_draws=None, stream=None):
        check(self.L.as_reset_all(self.h, obs.data_ptr(),
                                  reset_draws.data_ptr() if reset_draws is not None else None, stream),
              "as_reset_all")

    def reset_mask(self, mask, obs, reset_draws=None, stream=None):
        check(self.L.as_reset_mask(self.h, mask.data_ptr(), obs.data_ptr(),
                                   reset_draws.data_ptr() if reset_draws is not None else None, stream),
              "as_reset_mask")

    def physics_step(self, actions, stream=None):
        check(self.L.as_physics_step(self.h, actions.data_ptr(), stream), "as_physics_step")

    def body_state(self, table: "AsBodyTable", out, stream=None):
        """as_body_state: out [BODY_STATE_ROWS][num_bodies][n] fp32 on the device (ring-2 body views)."""
        check(self.L.as_body_state(self.h, C.byref(table), out.data_ptr(), stream), "as_body_state")

    def set_actuator(self, mode: int, action_scale: float = 0.0, default_q=(), stiffness: float = 0.0,
                     damping: float = 0.0, saturation_effort: float = 0.0, effort_limit: float = 0.0,
                     velocity_limit: float = 0.0):
        A = AsActuator()
        A.mode, A.action_scale = mode, action_scale
        A.default_q[: len(default_q)] = [float(x) for x in default_q]
        A.stiffness, A.damping = stiffness, damping
        A.saturation_effort, A.effort_limit, A.velocity_limit = saturation_effort, effort_limit, velocity_limit
        self._act = A
        check(self.L.as_set_actuator(self.h, C.byref(A)), "as_set_actuator")

    def set_quad_task(self, **kw):
        Q = AsQuadTask()
        for k, v in kw.items():
            if isinstance(v, (list, tuple)):
                getattr(Q, k)[:] = [float(x) for x in v]
            else:
                setattr(Q, k, v)
        self._quad = Q
        check(self.L.as_set_quad_task(self.h, C.byref(Q)), "as_set_quad_task")

    def quad_step(self, actions, obs, rew, term, trunc, stream=None):
        check(self.L.as_quad_step(self.h, actions.data_ptr(), obs.data_ptr(), rew.data_ptr(), term.data_ptr(),
                                  trunc.data_ptr(), stream), "as_quad_step")

    def quad_reset_all(self, obs, stream=None):
        check(self.L.as_quad_reset_all(self.h, obs.data_ptr(), stream), "as_quad_reset_all")

    def generate_stones(self, level: int, draws=None, stream=None):
        check(self.L.as_generate_stones(self.h, level, draws.data_ptr() if draws is not None else None, stream),
              "as_generate_stones")

    def profile_sampled(self, max_records: int, stride: int):
        check(self.L.as_profile_sampled(self.h, max_records, stride), "as_profile_sampled")

    def profile(self, max_launches: int):
        check(self.L.as_profile(self.h, max_launches), "as_profile")

    def profile_read(self):
        a, b, k = C.c_double(), C.c_double(), C.c_int32()
        check(self.L.as_profile_read(self.h, C.byref(a), C.byref(b), C.byref(k)), "as_profile_read")
        return a.value, b.value, k.value

    def debug_stamps(self, buf):
        check(self.L.as_debug_stamps(self.h, None if buf is None else buf.data_ptr()), "as_debug_stamps")

    def counters_host(self, stream=None) -> list:
        """The last step's counter words [any reset, target-index sum, regen level, contacts dropped]
        (synchronises `stream`)."""
        out = (C.c_int32 * 4)()
        check(self.L.as_step_counters_host(self.h, out, stream), "as_step_counters_host")
        return list(out)

    def counters_ptr(self) -> int:
        p = C.c_void_p()
        check(self.L.as_step_counters(self.h, C.byref(p)), "as_step_counters")
        return p.value
