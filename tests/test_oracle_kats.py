"""Physics known-answer tests modelled on the reference's own, on the oracle (CPU);
tests/test_gpu_constraints.py runs the same models through the HIP kernels.

* jointed pendulum (source/isaaclab/test/assets/test_articulation.py:1342-1456, the single-joint
  articulation under gravity): period 2 pi sqrt(L/g) (1 + theta0^2/16), energy conserved, and the
  bob's velocity from finite differences of its position equals L * qd (the body-state /
  joint-state consistency that test checks);
* filtered contact forces (source/isaaclab/test/sensors/test_contact_sensor.py:249-382): a resting
  body's per-(sensor, stone) flag is set exactly for the stone it touches, the filtered force equals
  the net contact force, zero contact gives a zero flag, and the summed normal force at rest is m g.
"""

import numpy as np

from _models import PEND_L, PEND_M, PEND_ROOT, STONE_TOP, level0_stones, pendulum_model, sphere_model

G = 9.81


def _pendulum(oracle_mod, theta0):
    orc = oracle_mod.Oracle(model=pendulum_model())
    st = orc.state(1)
    st["stones"][:] = level0_stones(1)
    st["root_pos"][:, 0] = PEND_ROOT
    st["q"][0, 0] = theta0
    return orc, st


def _bob(st, q):
    """bob position (y, z) relative to the hinge for hinge angle q about +x (arm along -z at q = 0)"""
    return np.array([PEND_L * np.sin(q), -PEND_L * np.cos(q)])


def pendulum_series(step, st, steps):
    q, qd, root = [], [], []
    for _ in range(steps):
        step()
        q.append(float(st["q"][0, 0]))
        qd.append(float(st["qd"][0, 0]))
        root.append(st["root_pos"][:, 0].copy())
    return np.array(q), np.array(qd), np.array(root)


def check_pendulum(q, qd, root, theta0, dt=4 / 240):
    # the base stays put (10 t on its tripod)
    assert np.abs(root - root[0]).max() < 2e-3
    # period from the upward zero crossings of q
    t = np.arange(1, len(q) + 1) * dt
    up = np.nonzero((q[:-1] < 0) & (q[1:] >= 0))[0]
    tc = t[up] + (0 - q[up]) / (q[up + 1] - q[up]) * dt
    T = np.diff(tc).mean()
    T_ref = 2 * np.pi * np.sqrt(PEND_L / G) * (1 + theta0 ** 2 / 16)
    assert abs(T - T_ref) < 5e-3 * T_ref, (T, T_ref)
    # energy of the bob (point mass on a massless arm)
    E = 0.5 * PEND_M * (PEND_L * qd) ** 2 + PEND_M * G * PEND_L * (1 - np.cos(q))
    # semi-implicit Euler: the energy oscillates by O(omega dt) ~ 2 % around its initial value
    assert np.abs(E - E[0]).max() < 3e-2 * E[0], (E.min(), E.max())
    # body velocity vs joint state: |d bob / dt| (central differences) = L |qd|
    p = np.stack([_bob(None, x) for x in q])
    v = (p[2:] - p[:-2]) / (2 * dt)
    np.testing.assert_allclose(np.linalg.norm(v, axis=1), PEND_L * np.abs(qd[1:-1]), atol=0.03 * PEND_L * np.abs(qd).max())


def test_pendulum_period_energy_velocity(oracle_mod):
    theta0 = 0.3
    orc, st = _pendulum(oracle_mod, theta0)
    act = np.zeros((1, 21), np.float32)
    q, qd, root = pendulum_series(lambda: orc.physics_step(st, act), st, 240)  # 4 s, ~2.8 periods
    check_pendulum(q, qd, root, theta0)
    # the tripod rests on stone 2: flag set for stone 2 only, on sensor 0
    assert st["contact_mask"][0, 0] == 1 << 2 and st["contact_mask"][1, 0] == 0


def _sphere(oracle_mod, z_gap):
    m, mass = sphere_model(0.1)
    orc = oracle_mod.Oracle(model=m)
    st = orc.state(1)
    st["stones"][:] = level0_stones(1)
    st["root_pos"][:, 0] = [0.75 * 3 + 0.05, 0.1, STONE_TOP + 0.1 + z_gap]
    return orc, st, mass


def mean_normal_force(orc, st, steps=10):
    """vertical contact force: the stone impulses summed over every substep of `steps` env steps
    (or_probe_substep's net_impulse; physics advanced in between) / elapsed time"""
    act = np.zeros((1, 21), np.float32)
    jz = 0.0
    for _ in range(steps):
        jz += float(orc.probe(st)["net_impulse"][2])
        orc.physics_step(st, act)
    return jz / (steps * orc.sim.substeps * orc.sim.dt)


def test_filtered_contact_force_resting(oracle_mod):
    orc, st, mass = _sphere(oracle_mod, 0.02)
    act = np.zeros((1, 21), np.float32)
    for _ in range(60):
        orc.physics_step(st, act)
    p = orc.probe(st)
    assert p["ncontact"] >= 1 and set(p["stone"].tolist()) == {3} and set(p["foot"].tolist()) == {0}
    # filtered (sensor 0, stone 3) force = net contact force (every contact is on stone 3)
    f_net = (p["lam_n"][:, None] * p["nrm"]).sum(axis=0) / orc.sim.dt
    f_stone3 = (p["lam_n"][p["stone"] == 3][:, None] * p["nrm"][p["stone"] == 3]).sum(axis=0) / orc.sim.dt
    np.testing.assert_array_equal(f_net, f_stone3)
    assert np.abs(f_net[:2]).max() < 0.05 * mass * G
    assert p["mask"] == (1 << 3, 0) and st["contact_mask"][0, 0] == 1 << 3
    # at rest the normal force carries the weight
    assert abs(mean_normal_force(orc, st) - mass * G) < 0.03 * mass * G


def test_zero_contact_zero_flag(oracle_mod):
    orc, st, _ = _sphere(oracle_mod, 0.5)  # 0.5 m above the stone: free fall for a few steps
    act = np.zeros((1, 21), np.float32)
    for _ in range(5):
        orc.physics_step(st, act)
        assert st["contact_mask"][:, 0].tolist() == [0, 0]
    p = orc.probe(st)
    assert p["ncontact"] == 0 and p["mask"] == (0, 0)


def test_filtered_forces_sum_to_net_two_stones(oracle_mod):
    """A ball resting in the gap between stones 3 and 4 (on both edges): one filtered force per
    stone, each pushing up and towards the gap's centre, summing to the net contact force; the
    sensor flags both stones and no other."""
    m, mass = sphere_model(0.2)
    orc = oracle_mod.Oracle(model=m)
    st = orc.state(1)
    st["stones"][:] = level0_stones(1)
    x_gap = 0.75 * 3 + 0.375  # the 0.25 m gap between the stone boxes (0.5 long)
    st["root_pos"][:, 0] = [x_gap, 0.0, STONE_TOP + 0.16]
    act = np.zeros((1, 21), np.float32)
    for _ in range(90):
        orc.physics_step(st, act)
    assert abs(st["root_pos"][0, 0] - x_gap) < 1e-3 and np.abs(st["root_lin"][:, 0]).max() < 1e-2
    p = orc.probe(st)
    assert set(p["stone"].tolist()) == {3, 4}
    f = {s: p["stone_impulse"][s] for s in range(20)}
    f_net = p["net_impulse"]
    assert not np.any([f[s].any() for s in range(20) if s not in (3, 4)])
    np.testing.assert_allclose(f[3] + f[4], f_net, rtol=1e-5, atol=1e-6)
    assert f[3][0] > 0 and f[4][0] < 0 and f[3][2] > 0 and f[4][2] > 0  # towards the centre, upwards
    assert p["mask"] == ((1 << 3) | (1 << 4), 0)
    # (wedged on two edges, friction carries part of the weight: the normal forces alone do not sum
    # to m g here -- the flat case in test_filtered_contact_force_resting checks that)
