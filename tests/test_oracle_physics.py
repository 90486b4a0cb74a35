"""Known-answer tests for the oracle's articulated-body physics (PhysX parity is unpinned).

Modelled on the reference's generic physics tests: analytic free fall, a body at
rest on a stone (contact force = m g, filtered-contact flag set), conservation of momentum and
energy in zero gravity (ties the CRBA inertia H to the RNEA bias C), and H's structure.
"""

import copy

import numpy as np
import pytest


def _level0_stones(st):
    for k in range(20):
        st["stones"][3 * k + 0][:] = 0.75 * k
        st["stones"][3 * k + 2][:] = 0.0


def _q_int(orc, q_cfg):
    q = np.zeros(orc.m["num_hinges"], np.float32)
    for k in range(orc.m["num_hinges"]):
        q[orc.m["cfg_dof_link"][k] - 1] = q_cfg[k]
    return q


def _u(orc, st, e=0):
    nh = orc.m["num_hinges"]
    u = np.zeros(6 + nh, np.float32)
    u[:3] = st["root_lin"][:, e]
    u[3:6] = st["root_ang"][:, e]
    for k in range(nh):
        u[6 + orc.m["cfg_dof_link"][k] - 1] = st["qd"][k, e]
    return u


def test_mass_matrix_structure(orc):
    rng = np.random.default_rng(0)
    q = rng.uniform(-0.5, 0.5, 21).astype(np.float32)
    quat = rng.normal(size=4).astype(np.float32)
    quat /= np.linalg.norm(quat)
    H, com = orc.mass_matrix(quat, q)
    assert np.abs(H - H.T).max() < 1e-5
    ev = np.linalg.eigvalsh(H.astype(np.float64))
    assert ev.min() > 1e-3
    M = orc.m["total_mass"]
    np.testing.assert_allclose(np.diag(H)[:3], M, rtol=1e-5)
    np.testing.assert_allclose(H[:3, :3] - np.diag(np.diag(H)[:3]), 0, atol=1e-5)
    # arm dofs do not couple with leg dofs (disjoint subtrees)
    names = orc.m["link_names"]
    arm = [6 + i - 1 for i, nm in enumerate(names) if "shoulder" in nm or "elbow" in nm]
    leg = [6 + i - 1 for i, nm in enumerate(names) if "hip" in nm or "knee" in nm or "ankle" in nm]
    assert np.abs(H[np.ix_(arm, leg)]).max() == 0.0


def test_free_fall(orc):
    st = orc.state(4)
    _level0_stones(st)
    st["root_pos"][2][:] = 10.0
    act = np.zeros((4, 21), np.float32)
    orc.env_step(st, act)
    g, dt = 9.81, 4 / 240
    np.testing.assert_allclose(st["root_lin"][2], -g * dt, rtol=1e-5)
    np.testing.assert_allclose(st["root_lin"][:2], 0, atol=1e-6)
    assert np.abs(st["qd"]).max() < 1e-4
    assert st["contact_mask"].max() == 0
    # semi-implicit Euler: z drop = g dt_sub^2 (1+2+3+4)
    dts = 1 / 240
    np.testing.assert_allclose(10.0 - st["root_pos"][2], g * dts * dts * 10, rtol=1e-3)


@pytest.mark.parametrize("seed", [0, 1])
def test_zero_gravity_conservation(oracle_mod, seed):
    orc = oracle_mod.Oracle()
    orc.sim.gravity = 0.0
    st = orc.state(1)
    _level0_stones(st)
    st["root_pos"][2][:] = 50.0  # far from every stone: no contacts
    rng = np.random.default_rng(seed)
    st["qd"][:, 0] = rng.uniform(-1.0, 1.0, 21)
    st["root_lin"][:, 0] = rng.uniform(-0.3, 0.3, 3)
    st["root_ang"][:, 0] = rng.uniform(-0.5, 0.5, 3)

    def momentum_energy():
        q = _q_int(orc, st["q"][:, 0])
        H, com = orc.mass_matrix(st["root_quat"][:, 0], q)
        u = _u(orc, st)
        p = H[:3] @ u           # linear momentum (conjugate to root translation)
        return p, 0.5 * u @ H @ u

    p0, e0 = momentum_energy()
    act = np.zeros((1, 21), np.float32)
    for _ in range(15):  # 60 substeps, well inside the joint limits
        orc.env_step(st, act)
    p1, e1 = momentum_energy()
    assert np.abs(p1 - p0).max() < 2e-2 * (np.abs(p0).max() + 1.0)
    assert abs(e1 - e0) < 3e-2 * e0


def _sphere_model(orc_mod):
    """A single free sphere (radius 0.1, density 1000) -- the root link only."""
    from allsteps_isaaclab_amd.model import load_model

    m = copy.deepcopy(load_model())
    r = 0.1
    mass = 1000.0 * 4 / 3 * np.pi * r ** 3
    m["num_links"] = 1
    m["num_hinges"] = 0
    m["mass"][:] = 0
    m["mass"][0] = mass
    m["com"][:] = 0
    m["inertia"][:] = 0
    m["inertia"][0, :3] = 0.4 * mass * r * r
    m["num_geoms"] = 1
    m["geom_link"][0] = 0
    m["geom_type"][0] = 0
    m["geom_foot"][0] = 0
    m["geom_radius"][0] = r
    m["geom_p0"][0] = 0
    m["geom_p1"][0] = 0
    m["cfg_dof_link"][:] = 0
    return m, mass


def test_sphere_resting_contact(oracle_mod):
    m, mass = _sphere_model(oracle_mod)
    orc = oracle_mod.Oracle(model=m)
    st = orc.state(1)
    _level0_stones(st)
    top = 0.225 / 2
    st["root_pos"][:, 0] = [0.75 * 3 + 0.05, 0.1, top + 0.1 + 0.05]  # 5 cm above stone 3
    act = np.zeros((1, 21), np.float32)
    for _ in range(60):  # 1 s
        orc.physics_step(st, act)
    z = st["root_pos"][2, 0]
    assert abs(z - (top + 0.1)) < 3e-3, z           # resting on the top face (small penetration)
    assert np.abs(st["root_lin"][:, 0]).max() < 1e-2  # at rest
    assert st["contact_mask"][0, 0] == (1 << 3)     # filtered contact with stone 3 only


def test_zero_torque_collapse_no_tunnelling(orc):
    """Robot dropped in the reset pose onto level-0 stones stays above the stone tops."""
    n = 16
    st = orc.state(n)
    _level0_stones(st)
    orc.reset_all(st, seed=3)
    act = np.zeros((n, 21), np.float32)
    lowest = np.inf
    for _ in range(40):
        obs, rew, term, trunc, anyr = orc.env_step(st, act)
        assert np.isfinite(obs).all() and np.isfinite(rew).all()
        over = (np.abs(st["body_pos"][3] - np.round(st["body_pos"][3] / 0.75) * 0.75) < 0.2) & ~term
        if over.any():
            lowest = min(lowest, st["body_pos"][5][over].min())
    # foot-frame origin sits 0.025 below the capsule bottom: allow 2 cm of penetration
    assert lowest > 0.1125 - 0.025 - 0.02, lowest


def _fk64(m, root_pos, root_quat, q_cfg):
    """float64 root -> link walk: R_i = R_parent Roff_i Rj_i, p_i = p_parent + R_parent (offset_pos +
    Roff (anchor - Rj anchor)) -- the textbook recursion the spec's pointer jumping reassociates."""
    def quat(q):
        w, x, y, z = q
        return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                         [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                         [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])

    def axang(a, t):
        a = np.asarray(a, np.float64)
        K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
        return np.eye(3) + np.sin(t) * K + (1 - np.cos(t)) * K @ K

    nl = m["num_links"]
    q_int = np.zeros(nl)
    for k in range(m["num_hinges"]):
        q_int[m["cfg_dof_link"][k]] = q_cfg[k]
    R = [None] * nl
    p = [None] * nl
    R[0], p[0] = quat(np.asarray(root_quat, np.float64)), np.asarray(root_pos, np.float64)
    for i in range(1, nl):
        Roff, Rj = quat(np.asarray(m["offset_quat"][i], np.float64)), axang(m["axis"][i], q_int[i])
        an = np.asarray(m["anchor"][i], np.float64)
        t = np.asarray(m["offset_pos"][i], np.float64) + Roff @ (an - Rj @ an)
        pa = m["parent"][i]
        R[i], p[i] = R[pa] @ Roff @ Rj, p[pa] + R[pa] @ t
    return R, p


def test_fk_pointer_jumping_matches_a_float64_walk(orc):
    """The spec's FK (pointer jumping over the tree, float32) places the torso and feet where a float64
    root -> link recursion does, to float32 rounding, at random poses of the walker."""
    rng = np.random.default_rng(11)
    m = orc.m
    worst = 0.0
    for _ in range(20):
        q = rng.uniform(-1.5, 1.5, m["num_hinges"]).astype(np.float32)
        rp = rng.uniform(-2, 2, 3).astype(np.float32)
        qt = rng.normal(size=4)
        rq = (qt / np.linalg.norm(qt)).astype(np.float32)
        bp = orc.fk_bodies(rp, rq, q)
        _, p64 = _fk64(m, rp, rq, q)
        for b, link in enumerate((m["torso_link"], *m["foot_link"])):
            worst = max(worst, float(np.abs(bp[b] - p64[link]).max()))
    assert worst < 5e-6, worst
