"""Known-answer bounds on the contact solver that stands in for PhysX TGS (DESIGN.md §4 "Solver").

The reference steps the walker with PhysX 5's TGS solver (``PhysxCfg.solver_type = 1``,
simulation_cfg.py:37), 4 position / 0 velocity iterations, ``enable_stabilization`` on, and the
articulation's ``sleep_threshold = 0.005`` / ``stabilization_threshold = 0.001`` (walker3d.py:26-32).  The
spec here is a velocity-level PGS (4 sweeps) with a Baumgarte position bias (0.2, slop 0.002, capped at
``max_depenetration_velocity``), and no sleeping.  No PhysX output exists offline, so the difference is
bounded by what the two must agree on:

* resting contact: penetration at rest within the slop (TGS resolves to ~0 through its position
  iterations; the bias here leaves at most ``slop`` + the PGS residual), no drift, kinetic energy per unit
  mass far below the PhysX sleep threshold (a body PhysX would put to sleep stays put here too);
* Coulomb friction: a sliding sphere reaches rolling without slipping at 5/7 of its initial speed
  (t* = 2 v0 / (7 mu g)) and keeps it (no rolling friction in either solver);
* articulations: a free two-capsule hinge pair dropped on a stone settles below the sleep threshold; the
  PD-held ANYmal stance (an articulated robot on four feet over two stones) rests 10 s with every foot
  within the slop and a millimetre of base creep.

The oracle runs the bounds on the CPU; ``-m gpu`` mirrors replay the same scenarios through the HIP
``as_physics_step`` and require the device state to equal the oracle's bit for bit at every second, so
the bounds hold for the kernel as well.
"""

import numpy as np
import pytest

from _models import STONE_TOP, GpuPhysics, level0_stones, padded_model, sphere_model

SLOP = 0.002          # AllstepsEnvCfg.sim.slop
SLEEP = 0.005         # walker3d.py:30 sleep_threshold: mass-normalised kinetic energy, m^2/s^2
STEPS_10S = 600       # physics steps of 4 x 1/240 s
SETTLE = 120          # 2 s
MU = 0.85


def _cap_mass(r, L):
    return 1000.0 * (np.pi * r * r * L + 4.0 / 3.0 * np.pi * r ** 3)


def _cap_inertia(m, r, L, axis):
    """solid cylinder of the capsule's length about its centre (a stand-in: only the resting answer matters)"""
    ia, it = 0.5 * m * r * r, m * (3 * r * r + L * L) / 12.0
    i = [it, it, it]
    i["xyz".index(axis)] = ia
    return tuple(i)


# ------------------------------------------------------------------------------------------- scenarios
# each returns (model, init(st)); the stones are the level-0 line (stone 3 centred at x = 2.25)

def scenario_sphere():
    m, _ = sphere_model(0.1)

    def init(st):
        st["root_pos"][:, 0] = [2.3, 0.1, STONE_TOP + 0.1 + 0.02]
    return m, init


def scenario_capsule():
    r, L = 0.05, 0.4
    mass = _cap_mass(r, L)
    root = {"mass": mass, "com": (0.0, 0.0, 0.0), "inertia": _cap_inertia(mass, r, L, "y")}
    m = padded_model([root], [{"link": 0, "type": 1, "radius": r, "p0": (0.0, -L / 2, 0.0), "p1": (0.0, L / 2, 0.0),
                               "foot": 0}])

    def init(st):
        st["root_pos"][:, 0] = [2.25, 0.0, STONE_TOP + r + 0.01]
    return m, init


def scenario_rolling(v0=0.5):
    m, _ = sphere_model(0.1)

    def init(st):
        st["root_pos"][:, 0] = [2.25, -0.3, STONE_TOP + 0.1]
        st["root_lin"][1, 0] = v0
    return m, init


def scenario_hinge_pair():
    r, L = 0.04, 0.2
    m1 = _cap_mass(r, L)
    root = {"mass": m1, "com": (0.0, 0.0, 0.0), "inertia": _cap_inertia(m1, r, L, "x")}
    link = {"parent": 0, "offset": (0.12, 0.0, 0.0), "axis": (0.0, 1.0, 0.0), "mass": m1, "com": (0.12, 0.0, 0.0),
            "inertia": _cap_inertia(m1, r, L, "x"), "lower": -1.0, "upper": 1.0}
    geoms = [{"link": 0, "type": 1, "radius": r, "p0": (-0.1, 0.0, 0.0), "p1": (0.1, 0.0, 0.0), "foot": 0},
             {"link": 1, "type": 1, "radius": r, "p0": (0.02, 0.0, 0.0), "p1": (0.22, 0.0, 0.0), "foot": 0}]
    m = padded_model([root, link], geoms)

    def init(st):
        st["root_pos"][:, 0] = [2.15, 0.0, STONE_TOP + r + 0.05]
        st["q"][0, 0] = 0.3
    return m, init


SCENARIOS = {"sphere": scenario_sphere, "capsule": scenario_capsule, "rolling": scenario_rolling,
             "hinge_pair": scenario_hinge_pair}


def run_oracle(oracle_mod, name, steps=STEPS_10S):
    """(per-step series, final state): root pos, root (lin, ang), q, qd of dof 0, min contact separation"""
    m, init = SCENARIOS[name]()
    orc = oracle_mod.Oracle(model=m)
    st = orc.state(1)
    st["stones"][:] = level0_stones(1)
    init(st)
    act = np.zeros((1, 21), np.float32)
    s = {"pos": [], "vel": [], "q": [], "qd": [], "sep": []}
    for _ in range(steps):
        orc.physics_step(st, act)
        p = orc.probe(st)
        s["pos"].append(st["root_pos"][:, 0].copy())
        s["vel"].append(np.r_[st["root_lin"][:, 0], st["root_ang"][:, 0]])
        s["q"].append(st["q"][0, 0])
        s["qd"].append(st["qd"][0, 0])
        s["sep"].append(p["sep"][: p["ncontact"]].min() if p["ncontact"] else np.inf)
    return {k: np.array(v) for k, v in s.items()}, orc, st


def _resting_bounds(s, r_lin_max):
    pen = -s["sep"][SETTLE:].min()
    drift = np.abs(s["pos"][SETTLE:] - s["pos"][SETTLE]).max()
    v = s["vel"][SETTLE:, :3]
    ke = 0.5 * (v * v).sum(1).max()
    assert np.isfinite(s["sep"][SETTLE:]).all(), "contact lost while resting"
    assert pen <= SLOP + 5e-5, pen
    assert drift <= r_lin_max, drift
    assert ke < 1e-3 * SLEEP, ke
    return pen, drift, ke


def test_resting_sphere_10s(oracle_mod):
    s, _, _ = run_oracle(oracle_mod, "sphere")
    _resting_bounds(s, 1e-5)
    assert np.abs(s["vel"][SETTLE:]).max() < 1e-4


def test_resting_capsule_10s(oracle_mod):
    """a capsule lying on its side: two contacts (bisection minimum + end points) share the load"""
    s, _, _ = run_oracle(oracle_mod, "capsule")
    _resting_bounds(s, 2e-3)  # neutral rolling about its own axis: sub-mm creep, no rolling friction
    z = s["pos"][SETTLE:, 2]
    assert (z >= STONE_TOP + 0.05 - SLOP - 5e-5).all() and (z <= STONE_TOP + 0.05 + 1e-4).all()


def test_sliding_sphere_reaches_rolling(oracle_mod):
    """Coulomb box friction: v -> 5/7 v0 and w = -v / r by t* = 2 v0 / (7 mu g) = 17 ms (2 env steps), then
    steady rolling"""
    v0, r = 0.5, 0.1
    s, _, _ = run_oracle(oracle_mod, "rolling", steps=12)
    vy, wx = s["vel"][:, 1], s["vel"][:, 3]
    assert 2 * v0 / (7 * MU * 9.81) < 2 / 60
    np.testing.assert_allclose(vy[2:], 5.0 / 7.0 * v0, rtol=5e-3)
    np.testing.assert_allclose(wx[2:] * r, -vy[2:], atol=1e-5)
    assert np.ptp(vy[2:]) < 1e-6  # no rolling friction
    # the sliding phase decelerates at mu g at most
    assert vy[0] >= v0 - MU * 9.81 / 60 - 1e-4


def test_hinge_pair_settles_below_sleep_threshold(oracle_mod):
    s, _, _ = run_oracle(oracle_mod, "hinge_pair")
    late = slice(STEPS_10S - 60, STEPS_10S)
    assert np.abs(s["vel"][late]).max() < 1e-3
    assert np.abs(s["qd"][late]).max() < 1e-3
    assert 0.5 * (s["vel"][late, :3] ** 2).sum(1).max() < 1e-3 * SLEEP
    assert np.abs(s["pos"][180:] - s["pos"][180]).max() < 2e-3
    assert -s["sep"][SETTLE:].min() <= SLOP + 5e-5
    assert abs(s["q"][-1]) < 0.05  # both capsules flat on the stone


# ------------------------------------------------------------------------------------- ANYmal stance

def _quad_stand(oracle_mod):
    from allsteps_isaaclab_amd.envs.quadruped import STAND_ROOT, stand_pose
    from allsteps_isaaclab_amd.model import ANYMAL_C_JSON, load_model

    m = load_model(ANYMAL_C_JSON)
    orc = oracle_mod.Oracle(model=m)
    st = orc.state(1)
    st["stones"][:] = level0_stones(1)
    st["root_pos"][:] = np.array(STAND_ROOT, np.float32)[:, None]
    q0 = stand_pose(m["dof_names"])
    st["q"][:12] = q0[:, None]
    return orc, st, q0


def _quad_pd(q, qd, q0):
    return ((150.0 * (q0 - q) - 4.0 * qd) / 80.0).astype(np.float32)


def test_anymal_stance_rests_10s(oracle_mod):
    orc, st, q0 = _quad_stand(oracle_mod)
    pos, vel, qd, sep = [], [], [], []
    for _ in range(STEPS_10S):
        orc.physics_step(st, _quad_pd(st["q"][:12].T, st["qd"][:12].T, q0))
        p = orc.probe(st)
        assert p["ncontact"] == 4 and sorted(p["foot"][:4].tolist()) == [0, 1, 2, 3]
        pos.append(st["root_pos"][:, 0].copy())
        vel.append(np.r_[st["root_lin"][:, 0], st["root_ang"][:, 0]])
        qd.append(st["qd"][:12, 0].copy())
        sep.append(p["sep"][:4].min())
    pos, vel, qd, sep = map(np.array, (pos, vel, qd, sep))
    assert -sep[SETTLE:].min() <= SLOP + 5e-5
    assert np.abs(pos[SETTLE:] - pos[SETTLE]).max() < 1.5e-3
    assert np.abs(pos[300:] - pos[300]).max() < 5e-4
    assert np.abs(vel[300:]).max() < 1e-3 and np.abs(qd[300:]).max() < 2e-3
    assert 0.5 * (vel[300:, :3] ** 2).sum(1).max() < 1e-3 * SLEEP


# ------------------------------------------------------------------------------------------------ GPU

FIELDS = ("root_pos", "root_quat", "root_lin", "root_ang", "q", "qd", "body_pos")


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_solver_bounds_gpu_bit_exact(oracle_mod, name):
    """the HIP path replays each scenario; every second its state equals the oracle's, so the bounds above
    hold on the device"""
    m, init = SCENARIOS[name]()
    orc = oracle_mod.Oracle(model=m)
    st = orc.state(1)
    st["stones"][:] = level0_stones(1)
    init(st)
    gpu = GpuPhysics(m, 1)
    gpu.load_oracle(st)
    act = np.zeros((1, 21), np.float32)
    steps = 12 if name == "rolling" else STEPS_10S
    for t in range(steps):
        gpu.step(act)
        orc.physics_step(st, act)
        if t % 60 == 59 or t == steps - 1:
            g = gpu.get()
            for k in FIELDS:
                assert np.array_equal(g[k], st[k]), (name, t, k, np.abs(g[k] - st[k]).max())
    gpu.close()


@pytest.mark.gpu
def test_anymal_stance_gpu_bit_exact(oracle_mod):
    import torch

    from allsteps_isaaclab_amd.envs.quadruped import QuadrupedStonesEnv

    orc, st, q0 = _quad_stand(oracle_mod)
    env = QuadrupedStonesEnv(1, "cuda:0")
    for k, v in env.state.items():
        if k in st.a and k != "curriculum":
            a = np.ascontiguousarray(st[k]).reshape(v.shape)
            v.copy_(torch.from_numpy(a.view(np.int32) if a.dtype == np.uint32 else a))
    for t in range(STEPS_10S):
        g = {k: env.state[k].cpu().numpy() for k in ("q", "qd")}
        a = _quad_pd(g["q"][:12].T, g["qd"][:12].T, q0)
        env.step(torch.from_numpy(a).to("cuda:0"))
        orc.physics_step(st, a)
        if t % 60 == 59:
            torch.cuda.synchronize()
            for k in FIELDS:
                gk = env.state[k].cpu().numpy().reshape(st[k].shape)
                assert np.array_equal(gk, st[k]), (t, k, np.abs(gk - st[k]).max())
    env.close()
