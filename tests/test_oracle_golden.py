"""Pin the CPU oracle's task logic to golden vectors from the reference's own code.

The vectors were produced by importing the reference ``allsteps_env.py`` / ``utils/math.py``
(``tests/golden/gen_golden.py``).  Integer and boolean outputs must match exactly; float outputs
within 2e-5 relative + 2e-5 absolute (float32, same operation order; the only differences are
libm vs ATen transcendental rounding and reduction order inside ``vector_norm``).
"""

import ctypes as C

import numpy as np
import pytest

from conftest import golden

RTOL, ATOL = 2e-5, 2e-5


def test_math_helpers(orc, oracle_mod):
    g = golden("math")
    q, v = g["m_q"], g["m_v"]
    n = len(q)
    rpy = np.zeros((n, 3), np.float32)
    qri = np.zeros((n, 3), np.float32)
    qr = np.zeros((n, 3), np.float32)
    O = oracle_mod
    orc.L.or_math_batch(n, O.fp(q), O.fp(v), O.fp(rpy), O.fp(qri), O.fp(qr))
    # roll/pitch/yaw are in [0, 2pi) (math.py:444); compare on the circle to tolerate 0 <-> 2pi
    for k, name in enumerate(("m_roll", "m_pitch", "m_yaw")):
        d = np.abs(rpy[:, k] - g[name])
        d = np.minimum(d, np.abs(d - 2 * np.pi))
        assert d.max() < 1e-5, name
    # the quirk: small negative roll/pitch come out near 2pi
    assert rpy[4, 0] > 6.0 and rpy[4, 1] > 6.0
    np.testing.assert_allclose(qri, g["m_qri"], rtol=RTOL, atol=1e-5)
    np.testing.assert_allclose(qr, g["m_qr"], rtol=RTOL, atol=1e-5)
    out = np.zeros((n, 3), np.float32)
    orc.L.or_sft_batch(n, O.fp(g["m_t01"]), O.fp(g["m_qs"]), O.fp(g["m_t02"]), O.fp(out))
    np.testing.assert_allclose(out, g["m_sft"], rtol=RTOL, atol=1e-5)
    # scale / unscale
    lib = orc.L
    lib.or_scale_transform.restype = C.c_float
    lib.or_scale_transform.argtypes = [C.c_float] * 3
    lib.or_unscale_transform.restype = C.c_float
    lib.or_unscale_transform.argtypes = [C.c_float] * 3
    x, lim = g["m_x"], g["m_lim"]
    sc = np.array([[lib.or_scale_transform(float(x[i, k]), float(lim[k, 0]), float(lim[k, 1]))
                    for k in range(21)] for i in range(0, len(x), 16)], np.float32)
    us = np.array([[lib.or_unscale_transform(float(x[i, k]), float(lim[k, 0]), float(lim[k, 1]))
                    for k in range(21)] for i in range(0, len(x), 16)], np.float32)
    np.testing.assert_array_equal(sc, g["m_scale"][::16])
    np.testing.assert_array_equal(us, g["m_unscale"][::16])


@pytest.mark.parametrize("level", [0, 3, 9])
def test_footsteps(orc, level):
    g = golden("footsteps")
    draws = g[f"fs{level}_draws"]
    n = draws.shape[1]
    pos, dphi = orc.footsteps(n, level, draws)
    np.testing.assert_allclose(pos, g[f"fs{level}_pos"], rtol=1e-5, atol=2e-6)
    np.testing.assert_allclose(dphi, g[f"fs{level}_dphi"], rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(g[f"fs{level}_swing"], np.array([1, 0] * 10))
    if level == 0:
        # RNG-independent straight line; z = k * 0.75 * cos(fp32 pi/2) quirk
        np.testing.assert_allclose(pos[:, :, 0], np.broadcast_to(0.75 * np.maximum(np.arange(20), 0), (n, 20)),
                                   atol=1e-5)
        assert np.all(pos[:, 1:, 2] < 0)


def _load_seq_state(orc, g):
    n = g["init_idx"].shape[0]
    st = orc.state(n)
    for k in ("idx", "prev", "next", "count", "swing", "ep_len"):
        st[k][:] = g["init_" + k]
    st["pot"][:] = g["init_pot"]
    st["old_pot"][:] = g["init_old_pot"]
    st["curriculum"][0] = g["init_curriculum"][0]
    st["stones"][:] = g["steps_pos"].reshape(n, 60).T
    return st, n


@pytest.mark.parametrize("fixture", ["task_seq", "gates"])
def test_task_sequence(orc, oracle_mod, fixture):
    """task_seq: 40-step DirectRLEnv.step post-physics sequence: dones -> rewards -> resets -> obs.
    gates: one step on states whose roll / pitch straddle the reward gates (allsteps_env.py:356-359)
    by 10 ulp .. 0.01 rad: the oracle's gate decisions are the reference's (a flipped gate moves the
    reward by ~0.4, far outside the tolerance)."""
    O = oracle_mod
    g = golden(fixture)
    st, n = _load_seq_state(orc, g)
    T = g["seq_obs"].shape[0]
    post = {}

    CB = C.CFUNCTYPE(None, C.c_void_p, C.c_int, C.POINTER(C.c_float))

    def post_fk(ctx, e, out):
        vals = post["bp"][e]
        for i in range(9):
            out[i] = float(vals[i])

    cb = CB(post_fk)
    steps_with_reset = 0
    for t in range(T):
        rs = g["seq_root_state"][t]
        st["root_pos"][:] = rs[:, 0:3].T
        st["root_quat"][:] = rs[:, 3:7].T
        st["root_lin"][:] = rs[:, 7:10].T
        st["root_ang"][:] = rs[:, 10:13].T
        st["q"][:] = g["seq_joint_pos"][t].T
        st["qd"][:] = g["seq_joint_vel"][t].T
        st["body_pos"][:] = np.concatenate([g["seq_torso"][t], g["seq_rfoot"][t], g["seq_lfoot"][t]], 1).T
        post["bp"] = np.concatenate([g["seq_post_torso"][t], g["seq_post_rfoot"][t], g["seq_post_lfoot"][t]], 1)
        fm_r = np.ascontiguousarray(g["seq_fm_r"][t], np.float32)
        fm_l = np.ascontiguousarray(g["seq_fm_l"][t], np.float32)
        act = np.ascontiguousarray(g["seq_actions"][t], np.float32)
        draws = np.ascontiguousarray(g["seq_reset_draws"][t], np.float32)
        obs = np.zeros((n, 59), np.float32)
        rew = np.zeros(n, np.float32)
        term = np.zeros(n, np.uint8)
        trunc = np.zeros(n, np.uint8)
        anyr = np.zeros(1, np.int32)
        orc.L.or_task_post_physics(C.byref(orc.model), C.byref(orc.task), st.ptr, O.fp(act), O.fp(fm_r), O.fp(fm_l),
                                   O.fp(draws), 0, C.cast(cb, C.c_void_p), None, O.fp(obs), O.fp(rew), O.u8p(term),
                                   O.u8p(trunc), O.ip(anyr))
        msg = f"step {t}"
        np.testing.assert_array_equal(term.astype(bool), g["seq_terminated"][t], msg)
        np.testing.assert_array_equal(trunc.astype(bool), g["seq_truncated"][t], msg)
        assert bool(anyr[0]) == bool(g["seq_any_reset"][t]), msg
        steps_with_reset += int(anyr[0])
        for k in ("idx", "prev", "next", "count", "swing", "ep_len"):
            np.testing.assert_array_equal(st[k], g["seq_" + k][t], f"{msg} {k}")
        assert st["curriculum"][0] == g["seq_curriculum"][t][0], msg
        np.testing.assert_allclose(rew, g["seq_reward"][t], rtol=RTOL, atol=5e-5, err_msg=msg)
        np.testing.assert_allclose(st["pot"], g["seq_pot"][t], rtol=RTOL, atol=ATOL, err_msg=msg)
        np.testing.assert_allclose(st["old_pot"], g["seq_old_pot"][t], rtol=RTOL, atol=ATOL, err_msg=msg)
        np.testing.assert_array_equal(st["foot_contact"].T, g["seq_foot_contact"][t], msg)
        # obs: angles on the circle, everything else plain
        go = g["seq_obs"][t]
        d = np.abs(obs[:, 1:3] - go[:, 1:3])
        d = np.minimum(d, np.abs(d - 2 * np.pi))
        assert d.max() < 2e-5, msg
        np.testing.assert_allclose(np.delete(obs, [1, 2], 1), np.delete(go, [1, 2], 1), rtol=RTOL, atol=5e-5,
                                   err_msg=msg)
        # reset state
        prs = g["seq_post_root_state"][t]
        np.testing.assert_allclose(st["root_pos"].T, prs[:, :3], atol=1e-6, err_msg=msg)
        np.testing.assert_array_equal(np.signbit(st["root_quat"].T), np.signbit(prs[:, 3:7]), msg)
        np.testing.assert_allclose(st["q"].T, g["seq_post_joint_pos"][t], rtol=1e-6, atol=1e-6, err_msg=msg)
        np.testing.assert_array_equal(st["qd"].T, g["seq_post_joint_vel"][t], msg)
    if fixture == "task_seq":
        assert 0 < steps_with_reset < T
    else:
        assert np.array_equal(obs[:, 1] > 0.4, g["gate_roll"] > 0.4)
        assert np.array_equal(obs[:, 2] > 0.4, g["gate_pitch"] > 0.4)
        assert 0 < int((g["gate_roll"] > 0.4).sum()) < len(obs)


def test_philox_uniform_range(orc):
    d = np.concatenate([orc.philox(42, e, ep) for e in range(64) for ep in range(4)])
    assert d.min() >= 0.0 and d.max() < 1.0
    assert abs(d.mean() - 0.5) < 0.02
    a = orc.philox(42, 3, 1)
    np.testing.assert_array_equal(a, orc.philox(42, 3, 1))
    assert not np.array_equal(a, orc.philox(42, 3, 2))
    assert not np.array_equal(a, orc.philox(43, 3, 1))


def _stepped_state(orc, n, steps, seed):
    st = orc.state(n)
    rng = np.random.default_rng(seed)
    orc.reset_all(st, reset_draws=rng.uniform(0, 1, (n, 22)).astype(np.float32))
    for _ in range(steps):
        orc.env_step(st, rng.uniform(-1, 1, (n, 21)).astype(np.float32),
                     reset_draws=rng.uniform(0, 1, (n, 22)).astype(np.float32))
    return st


def test_reset_mask_matches_reset_all_and_noop(orc):
    """_reset_idx(all ids) == reset(); _reset_idx(no ids) changes nothing; a subset resets exactly
    the masked envs (the foot-state tick and the curriculum gate apply to all, as in the reference)."""
    n = 24
    draws = np.random.default_rng(1).uniform(0, 1, (n, 22)).astype(np.float32)
    a, b = _stepped_state(orc, n, 6, 9), _stepped_state(orc, n, 6, 9)
    oa = orc.reset_all(a, reset_draws=draws)
    ob = orc.reset_mask(b, np.ones(n, bool), reset_draws=draws)
    for k in ("q", "qd", "root_pos", "root_quat", "idx", "prev", "next", "count", "swing", "pot", "old_pot",
              "episode", "ep_len", "curriculum", "body_pos", "foot_contact"):
        np.testing.assert_array_equal(a[k], b[k], k)
    np.testing.assert_array_equal(oa, ob)
    c = _stepped_state(orc, n, 6, 9)
    before = {k: np.array(c[k]) for k in ("q", "qd", "root_pos", "idx", "count", "swing", "pot", "old_pot",
                                          "ep_len", "episode", "foot_contact")}
    oc = orc.reset_mask(c, np.zeros(n, bool), reset_draws=draws)
    for k, v in before.items():
        np.testing.assert_array_equal(c[k], v, k)
    assert np.isfinite(oc).all()
    # partial: masked envs get the reset pose of the full reset, the others keep their joints
    d = _stepped_state(orc, n, 6, 9)
    q0 = np.array(d["q"])
    m = np.arange(n) % 3 == 0
    orc.reset_mask(d, m, reset_draws=draws)
    np.testing.assert_array_equal(d["q"][:, m], a["q"][:, m])
    np.testing.assert_array_equal(d["q"][:, ~m], q0[:, ~m])
    np.testing.assert_array_equal(d["ep_len"][m], 0)
