"""HIP kernels on the constraint-budget states and the physics known-answer models (-m gpu).

* the walker fixtures of tests/golden/constraint_states.npz (self-contact arm, crowded feet, fallen
  with limit rows), 64 envs each with per-env random actions: every state field and contact flag
  bit-identical to the oracle after each of 5 physics steps;
* the pendulum and the resting / falling / wedged spheres of tests/test_oracle_kats.py (padded to 21
  hinges, tests/_models.py): the same known answers on the GPU, bit-identical to the oracle;
* a clump of 14 crossing capsules (91 overlapping self pairs): more pairs pass the bounding-sphere
  filter than the kernel's one-pass list holds, so its word-by-word path runs -- bit-identical too;
* the contacts the constraint budget cuts (as_step_counters word 3, env.dropped_contacts()) equal the
  oracle's count in every step of the "crowded" and "fallen" fixtures through the full env step.
"""

import numpy as np
import pytest

from _models import (GpuPhysics, PEND_ROOT, STONE_TOP, constraint_fixture, level0_stones, pendulum_model,
                     put_oracle, sphere_model)
from test_oracle_kats import check_pendulum, pendulum_series

pytestmark = pytest.mark.gpu

FLOAT_FIELDS = ("root_pos", "root_quat", "root_lin", "root_ang", "q", "qd", "body_pos")


def _assert_same(g, st, what):
    for k in FLOAT_FIELDS:
        assert np.array_equal(g[k], st[k]), (what, k, np.abs(g[k] - st[k]).max())
    assert np.array_equal(g["contact_mask"].view(np.uint32), st["contact_mask"]), (what, "contact_mask")


@pytest.mark.parametrize("name", ["self_arm", "crowded", "fallen"])
def test_constraint_states_bit_exact(orc, name):
    n, steps = 64, 5
    snap = constraint_fixture(name)
    st = orc.state(n)
    for e in range(n):
        put_oracle(st, snap, e)
    gpu = GpuPhysics(orc.m, n)
    gpu.load_oracle(st)
    rng = np.random.default_rng(3)
    for t in range(steps):
        act = rng.uniform(-1, 1, (n, 21)).astype(np.float32)
        act[0] = 0.0  # env 0: the fixture's own motion
        gpu.step(act)
        orc.physics_step(st, act)
        _assert_same(gpu.get(), st, f"{name} step {t}")
    if name == "self_arm":  # the self-contact pushed the arm out of the torso on the GPU as well
        q_arm = [orc.m["dof_names"].index(k) for k in ("right_shoulder_x", "right_shoulder_y", "right_shoulder_z",
                                                        "right_elbow")]
        assert np.abs(gpu.get()["q"][q_arm, 0] - snap["q"][q_arm]).max() > 1e-3
    gpu.close()


def test_pendulum_gpu(oracle_mod):
    theta0 = 0.3
    m = pendulum_model()
    orc = oracle_mod.Oracle(model=m)
    st = orc.state(1)
    st["stones"][:] = level0_stones(1)
    st["root_pos"][:, 0] = PEND_ROOT
    st["q"][0, 0] = theta0
    gpu = GpuPhysics(m, 1)
    gpu.load_oracle(st)
    act = np.zeros((1, 21), np.float32)
    s = {}

    def step():
        gpu.step(act)
        s.update(gpu.get())
        orc.physics_step(st, act)
        _assert_same(s, st, "pendulum")

    class View:  # pendulum_series reads the GPU state after each step
        def __getitem__(self, k):
            return s[k]

    q, qd, root = pendulum_series(step, View(), 240)
    check_pendulum(q, qd, root, theta0)
    assert s["contact_mask"][0, 0] == 1 << 2 and s["contact_mask"][1, 0] == 0
    gpu.close()


@pytest.mark.parametrize("case", ["resting", "falling", "wedged"])
def test_sphere_flags_gpu(oracle_mod, case):
    r = 0.2 if case == "wedged" else 0.1
    m, _ = sphere_model(r)
    orc = oracle_mod.Oracle(model=m)
    st = orc.state(1)
    st["stones"][:] = level0_stones(1)
    pos = {"resting": [0.75 * 3 + 0.05, 0.1, STONE_TOP + 0.1 + 0.02],
           "falling": [0.75 * 3 + 0.05, 0.1, STONE_TOP + 0.1 + 0.5],
           "wedged": [0.75 * 3 + 0.375, 0.0, STONE_TOP + 0.16]}[case]
    st["root_pos"][:, 0] = pos
    gpu = GpuPhysics(m, 1)
    gpu.load_oracle(st)
    act = np.zeros((1, 21), np.float32)
    steps = {"resting": 60, "falling": 5, "wedged": 90}[case]
    for _ in range(steps):
        gpu.step(act)
        orc.physics_step(st, act)
        g = gpu.get()
        _assert_same(g, st, case)
        if case == "falling":
            assert g["contact_mask"][:, 0].tolist() == [0, 0]
    want = {"resting": 1 << 3, "falling": 0, "wedged": (1 << 3) | (1 << 4)}[case]
    assert int(g["contact_mask"][0, 0]) == want and int(g["contact_mask"][1, 0]) == 0
    gpu.close()


def _clump_model(nlinks: int = 14) -> dict:
    """nlinks capsules on sibling hinge links, all near the root origin in a star of directions:
    every one of the C(nlinks, 2) self pairs overlaps, so more pairs pass the bounding-sphere filter
    than the kernel's one-pass pair list holds (64) and it takes the word-by-word path."""
    from _models import padded_model

    root = {"mass": 10.0, "com": (0.0, 0.0, 0.0), "inertia": (0.1, 0.1, 0.1)}
    links, geoms = [root], []
    rng = np.random.default_rng(5)
    for i in range(nlinks):
        d = rng.normal(size=3)
        d /= np.linalg.norm(d)
        links.append({"parent": 0, "offset": (0.0, 0.0, 0.0), "axis": tuple(np.roll((1.0, 0.0, 0.0), i % 3)),
                      "mass": 0.5, "com": tuple(0.05 * d), "inertia": (1e-3, 1e-3, 1e-3), "lower": -3.0,
                      "upper": 3.0})
        o = 0.01 * rng.normal(size=3)  # off the common centre: no two axes meet (a zero distance has no normal)
        geoms.append({"link": i + 1, "type": 1, "radius": 0.03, "p0": tuple(o - 0.15 * d), "p1": tuple(o + 0.15 * d)})
    m = padded_model(links, geoms)
    pairs = [(a, b) for a in range(nlinks) for b in range(a + 1, nlinks)]
    m["num_self_pairs"] = len(pairs)
    for p, (a, b) in enumerate(pairs):
        m["self_pair"][p] = a | (b << 8)
    return m


def test_self_pairs_past_the_list_capacity(oracle_mod):
    m = _clump_model()
    assert m["num_self_pairs"] > 64
    n, steps = 4, 3
    orc = oracle_mod.Oracle(model=m)
    st = orc.state(n)
    st["stones"][:] = level0_stones(n)
    st["root_pos"][:, :] = np.array([[1.5], [0.0], [2.0]], np.float32)  # in the air: self-contacts only
    gpu = GpuPhysics(m, n)
    gpu.load_oracle(st)
    rng = np.random.default_rng(11)
    moved = 0.0
    for t in range(steps):
        act = rng.uniform(-1, 1, (n, 21)).astype(np.float32)
        gpu.step(act)
        orc.physics_step(st, act)
        g = gpu.get()
        _assert_same(g, st, f"clump step {t}")
        moved = max(moved, float(np.abs(g["qd"][:14]).max()))
    assert moved > 0.0  # the self-contacts (at most the budget's 10) push the links apart
    gpu.close()


@pytest.mark.parametrize("name", ["crowded", "fallen"])
def test_dropped_contacts_equal_oracle(orc, name):
    """the device count of contacts cut by the 10-contact / 30-row budget (PhysX keeps every
    one, simulation_cfg.py:110) equals the oracle's in every step, and the fixtures do cut some."""
    import os

    import torch

    from allsteps_isaaclab_amd.envs.allsteps_env import AllstepsEnv
    from allsteps_isaaclab_amd.envs.allsteps_env_cfg import AllstepsEnvCfg

    n, steps = 64, 5
    cfg = AllstepsEnvCfg()
    cfg.scene.num_envs = n
    cfg.sim.device = "cuda:0"
    cfg.seed = 42
    env = AllstepsEnv(cfg)
    env.reset()
    torch.cuda.synchronize()
    st = orc.state(n)
    for k, v in env.get_state().items():
        st[k][...] = v.cpu().numpy().reshape(st[k].shape).view(st[k].dtype)
    snap = constraint_fixture(name)
    for e in range(n):
        put_oracle(st, snap, e)
    env.set_state({k: st[k].view(np.int32) if st[k].dtype == np.uint32 else st[k] for k in env.get_state()})
    rng = np.random.default_rng(3)
    total = 0
    for t in range(steps):
        act = rng.uniform(-1, 1, (n, 21)).astype(np.float32)
        act[0] = 0.0
        env.step(torch.from_numpy(act).cuda())
        orc.env_step(st, act, seed=42, nthreads=max(1, min(16, os.cpu_count() or 1)))
        g = env.dropped_contacts()
        print(f"[dropped {name}] step {t}: gpu {g} oracle {orc.last_dropped}")
        assert g == orc.last_dropped, (t, g, orc.last_dropped)
        total += g
    _assert_same({k: v.cpu().numpy() for k, v in env.get_state().items()}, st, name)
    assert total > 0
    env.close()
