"""BASELINE C5 (quadruped on the stones, physics only).

The model is an authored ANYmal-C approximation (``model/anymal_c.xml``: the vendor USD is Nucleus-only),
so parity with the real robot / PhysX is unpinned.  What is pinned:
  * CPU: the compiled tables (12 hinges in IsaacLab's ANYmal joint order, four feet first under the
    contact cap, mass from the geoms), and known answers of the oracle on this model -- free fall, a
    PD-held stance that rests on two stones with both sensor feet in contact;
  * GPU: k_step<18> against the oracle from identical states (same tolerances as the walker's
    tests/test_gpu_parity.py: positions 2e-3, velocities 1e-2, contact bits >= 99 % exact), the stance
    on the GPU, and size-independent properties at the C5 size (16384 envs): finite state, no envs
    through a stone, all feet supported.
"""

import numpy as np
import pytest
import torch

from allsteps_isaaclab_amd.envs.quadruped import STAND_ROOT, level0_stones, stand_pose
from allsteps_isaaclab_amd.model import ANYMAL_C_JSON, load_model

STONE_TOP = 0.1125


@pytest.fixture(scope="module")
def qmodel():
    return load_model(ANYMAL_C_JSON)


@pytest.fixture(scope="module")
def qorc(oracle_mod, qmodel):
    return oracle_mod.Oracle(model=qmodel)


def _stand_state(orc, m, n):
    st = orc.state(n)
    st["stones"][:] = level0_stones(n)
    st["root_pos"][:] = np.array(STAND_ROOT, np.float32)[:, None]
    st["q"][:12] = stand_pose(m["dof_names"])[:, None]
    return st


def _pd(st, q0, kp=150.0, kd=4.0):
    q, qd = st["q"][:12].T, st["qd"][:12].T
    return ((kp * (q0 - q) - kd * qd) / 80.0).astype(np.float32)


def test_quadruped_model_tables(qmodel):
    m = qmodel
    assert m["num_links"] == 13 and m["num_hinges"] == 12
    assert m["dof_names"][:4] == ["LF_HAA", "LH_HAA", "RF_HAA", "RH_HAA"]
    assert m["dof_names"][8:] == ["LF_KFE", "LH_KFE", "RF_KFE", "RH_KFE"]
    assert 45.0 < m["total_mass"] < 52.0
    # the four feet are the first geoms (a foot contact is never dropped for a body contact)
    assert m["geom_name"][:4] == ["LF_FOOT", "LH_FOOT", "RF_FOOT", "RH_FOOT"]
    # sensor feet: RF -> 0, LF -> 1, RH -> 2, LH -> 3
    foot = dict(zip(m["geom_name"], m["geom_foot"][: m["num_geoms"]]))
    assert foot["RF_FOOT"] == 0 and foot["LF_FOOT"] == 1 and foot["RH_FOOT"] == 2 and foot["LH_FOOT"] == 3
    assert foot["base_geom"] == -1
    np.testing.assert_allclose(m["gear"][:12], 80.0 / 1.2, rtol=1e-6)


def test_quadruped_free_fall(qorc, qmodel):
    st = _stand_state(qorc, qmodel, 3)
    st["root_pos"][2] = 10.0
    qorc.physics_step(st, np.zeros((3, 12), np.float32))
    np.testing.assert_allclose(st["root_lin"][2], -9.81 * 4 / 240, rtol=1e-5)
    assert st["contact_mask"].max() == 0


def test_quadruped_zero_gravity_conservation(oracle_mod, qmodel):
    """No gravity, no contacts, no torque: linear momentum H[:3] u and kinetic energy u^T H u / 2 are
    conserved (ties the CRBA H to the RNEA bias C on this model, as for the walker)."""
    orc = oracle_mod.Oracle(model=qmodel)
    orc.sim.gravity = 0.0
    st = _stand_state(orc, qmodel, 1)
    st["root_pos"][2] = 50.0
    rng = np.random.default_rng(3)
    st["qd"][:12, 0] = rng.uniform(-1.0, 1.0, 12)
    st["root_lin"][:, 0] = rng.uniform(-0.3, 0.3, 3)
    st["root_ang"][:, 0] = rng.uniform(-0.5, 0.5, 3)

    def momentum_energy():
        q = np.zeros(12, np.float32)
        u = np.zeros(18, np.float32)
        u[:3], u[3:6] = st["root_lin"][:, 0], st["root_ang"][:, 0]
        for k in range(12):
            li = qmodel["cfg_dof_link"][k]
            q[li - 1] = st["q"][k, 0]
            u[6 + li - 1] = st["qd"][k, 0]
        H, _ = orc.mass_matrix(st["root_quat"][:, 0], q)
        return H[:3] @ u, 0.5 * u @ H @ u

    p0, e0 = momentum_energy()
    for _ in range(10):  # 40 substeps, inside the joint limits
        orc.physics_step(st, np.zeros((1, 12), np.float32))
    p1, e1 = momentum_energy()
    assert np.abs(p1 - p0).max() < 2e-2 * (np.abs(p0).max() + 1.0)
    assert abs(e1 - e0) < 3e-2 * e0


def test_quadruped_stance_rests_on_two_stones(qorc, qmodel):
    st = _stand_state(qorc, qmodel, 2)
    q0 = stand_pose(qmodel["dof_names"])
    for _ in range(90):
        qorc.physics_step(st, _pd(st, q0))
    z = st["root_pos"][2]
    assert ((z > 0.64) & (z < 0.70)).all(), z
    assert (np.abs(st["root_quat"][1:]) < 5e-3).all()  # level base
    assert (np.abs(st["root_lin"]) < 2e-2).all()       # at rest
    assert (st["contact_mask"] == 2).all()             # RF and LF on stone 1
    assert np.abs(st["q"][:12].T - q0).max() < 0.1     # PD sag under gravity only


# ------------------------------------------------------------------------------------------------ GPU


def _gpu_env(n):
    from allsteps_isaaclab_amd.envs.quadruped import QuadrupedStonesEnv

    return QuadrupedStonesEnv(n, "cuda:0")


def _to_oracle(env, st):
    for k, v in env.state.items():
        if k in ("curriculum",):
            continue
        st[k][...] = v.cpu().numpy().reshape(st[k].shape).view(st[k].dtype)


@pytest.mark.gpu
@pytest.mark.parametrize("warm", [0, 20])
def test_quadruped_gpu_matches_oracle(qorc, qmodel, warm):
    n = 256
    env = _gpu_env(n)
    gen = torch.Generator(device="cuda:0").manual_seed(warm)
    for _ in range(warm):  # warm up into a perturbed, contact-rich state
        env.step((env.stand_actions() + 0.3 * (torch.rand(n, 12, device="cuda:0", generator=gen) * 2 - 1)))
    torch.cuda.synchronize()
    st = qorc.state(n)
    _to_oracle(env, st)
    act = (env.stand_actions() + 0.5 * (torch.rand(n, 12, device="cuda:0", generator=gen) * 2 - 1)).contiguous()
    env.step(act)
    torch.cuda.synchronize()
    qorc.physics_step(st, act.cpu().numpy())
    g = {k: v.cpu().numpy() for k, v in env.state.items()}
    mask_eq = ((g["contact_mask"].view(np.uint32) == st["contact_mask"]).all(axis=0)
               & (g["contact_mask_hind"].view(np.uint32) == st["contact_mask_hind"]).all(axis=0))
    print(f"quadruped parity warm={warm}: contact bits differ on {np.count_nonzero(~mask_eq)} of {n} envs")
    assert mask_eq.all(), f"contact bits differ on {np.count_nonzero(~mask_eq)} envs"
    # the same float32 operations in the same order on both sides (include/as_detmath.h): bit-exact
    for k in ("root_pos", "root_quat", "q", "root_lin", "root_ang", "qd", "body_pos"):
        assert np.array_equal(g[k], st[k]), (k, np.abs(g[k] - st[k]).max())
    env.close()


@pytest.mark.gpu
def test_quadruped_gpu_stance_and_c5_size_properties():
    n = 16384  # BASELINE C5
    env = _gpu_env(n)
    gen = torch.Generator(device="cuda:0").manual_seed(5)
    for _ in range(60):
        env.step(env.stand_actions())
    torch.cuda.synchronize()
    z = env.root_pos[:, 2]
    assert bool(((z > 0.64) & (z < 0.70)).all())
    # sensors RF, LF on stone 1; RH, LH on stone 0
    assert bool((env.contact_mask == torch.tensor([2, 2, 1, 1], device="cuda:0", dtype=torch.int32)).all())
    # perturbed stepping (the bench's protocol): every env stays finite, nearly all keep standing,
    # and no base (capsule radius 0.12) sinks into a stone it is above (a robot may legitimately
    # slip into the 0.25 m gap between stones and fall below their tops)
    for _ in range(60):
        env.step(env.stand_actions() + 0.3 * (torch.rand(n, 12, device="cuda:0", generator=gen) * 2 - 1))
    torch.cuda.synchronize()
    for k, v in env.state.items():
        if v.dtype == torch.float32:
            assert bool(torch.isfinite(v).all()), k
    p = env.root_pos
    assert float((p[:, 2] > 0.5).float().mean()) > 0.99
    dx = torch.remainder(p[:, 0] + 0.375, 0.75) - 0.375  # x offset from the nearest stone centre
    over = (dx.abs() < 0.25) & (p[:, 1].abs() < 0.4) & (p[:, 0] > -0.25) & (p[:, 0] < 14.5)
    assert bool((p[over, 2] > STONE_TOP + 0.12 - 0.02).all())
    env.close()


@pytest.mark.gpu
def test_quadruped_rejects_bad_actions():
    env = _gpu_env(8)
    with pytest.raises(ValueError):
        env.step(torch.zeros(8, 21, device="cuda:0"))
    env.close()
