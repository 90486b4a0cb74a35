"""Property tests (hypothesis) of the CPU oracle: invariants that hold for every input, not only for
the golden vectors (SURVEY.md §4 "property tests with hypothesis").  The oracle is the checker the
GPU parity tests trust, so these pin it beyond the reference's fixtures:

* H(q) (CRBA, oracle/physics.c) is symmetric positive definite in every pose, its linear block is
  M I;
* the RNEA bias C(q, u) is the gravity wrench at rest (linear part (0, 0, M g)), zero with neither
  gravity nor velocity, and quadratic in u without gravity (C(2u) = 4 C(u));
* quaternion helpers (utils/math.py:546-565, 414-444 restated in oracle/task.c) preserve length,
  invert each other, and return Euler angles in [0, 2 pi);
* footsteps (allsteps_env.py:125-174): stones 0-2 fixed at x = 0, 0.75, 1.5, every later stride in
  [0.75, linspace(0.75, 0.9, 10)[level]];
* the task state machine (allsteps_env.py:418-467) keeps prev = idx - 1, next = min(idx + 1, 19),
  idx in [1, 19], count and swing in {0, 1}, finite observations / rewards, for any action sequence.
"""

import numpy as np
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as S

SET = settings(max_examples=30, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])

f32 = dict(allow_nan=False, allow_infinity=False, width=32)
quats = S.lists(S.floats(-1, 1, **f32), min_size=4, max_size=4).filter(lambda v: np.linalg.norm(v) > 0.2)
poses = S.lists(S.floats(-1.25, 1.25, **f32), min_size=21, max_size=21)
vels = S.lists(S.floats(-2, 2, **f32), min_size=27, max_size=27)


def _unit(v):
    v = np.asarray(v, np.float32)
    return (v / np.linalg.norm(v)).astype(np.float32)


@SET
@given(quats, poses)
def test_mass_matrix_spd_in_every_pose(orc, qv, q):
    H, _ = orc.mass_matrix(_unit(qv), np.asarray(q, np.float32))
    scale = np.abs(H).max()
    assert np.abs(H - H.T).max() <= 1e-6 * scale
    assert np.linalg.eigvalsh(H.astype(np.float64)).min() > 0.0
    M = orc.m["total_mass"]
    np.testing.assert_allclose(H[:3, :3], M * np.eye(3), atol=1e-4 * M)


@SET
@given(quats, poses)
def test_bias_at_rest_is_the_gravity_wrench(orc, qv, q):
    quat, q = _unit(qv), np.asarray(q, np.float32)
    zero = np.zeros(27, np.float32)
    Cg = orc.bias_forces(quat, q, zero)
    M = orc.m["total_mass"]
    np.testing.assert_allclose(Cg[:3], [0.0, 0.0, M * 9.81], atol=1e-4 * M * 9.81)
    assert np.abs(orc.bias_forces(quat, q, zero, gravity=0.0)).max() == 0.0


@SET
@given(quats, poses, vels)
def test_bias_is_quadratic_in_velocity_without_gravity(orc, qv, q, u):
    quat, q, u = _unit(qv), np.asarray(q, np.float32), np.asarray(u, np.float32)
    c1 = orc.bias_forces(quat, q, u, gravity=0.0).astype(np.float64)
    c2 = orc.bias_forces(quat, q, 2.0 * u, gravity=0.0).astype(np.float64)
    np.testing.assert_allclose(c2, 4.0 * c1, rtol=1e-4, atol=1e-4 * max(np.abs(c2).max(), 1.0))


@SET
@given(S.lists(quats, min_size=1, max_size=8), S.data())
def test_quaternion_helpers(orc, oracle_mod, qs, data):
    O = oracle_mod
    n = len(qs)
    q = np.stack([_unit(v) for v in qs])
    v = np.asarray(data.draw(S.lists(S.lists(S.floats(-5, 5, **f32), min_size=3, max_size=3), min_size=n,
                                     max_size=n)), np.float32)
    rpy, qri, qr = (np.zeros((n, 3), np.float32) for _ in range(3))
    orc.L.or_math_batch(n, O.fp(q), O.fp(v), O.fp(rpy), O.fp(qri), O.fp(qr))
    nv = np.linalg.norm(v, axis=1)
    np.testing.assert_allclose(np.linalg.norm(qr, axis=1), nv, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(np.linalg.norm(qri, axis=1), nv, rtol=1e-5, atol=1e-5)
    assert (rpy >= 0).all() and (rpy < 2 * np.pi + 1e-6).all()
    back = np.zeros((n, 3), np.float32)
    orc.L.or_math_batch(n, O.fp(q), O.fp(np.ascontiguousarray(qr)), O.fp(rpy), O.fp(back), O.fp(qr))
    np.testing.assert_allclose(back, v, rtol=1e-5, atol=2e-5)


@SET
@given(S.integers(0, 9), S.integers(0, 2**31 - 1))
def test_footstep_strides(orc, level, seed):
    n = 4
    draws = np.random.default_rng(seed).uniform(0, 1, (5, n, 20)).astype(np.float32)
    pos, _ = orc.footsteps(n, level, draws)
    np.testing.assert_allclose(pos[:, :3, 0], np.broadcast_to([0.0, 0.75, 1.5], (n, 3)), atol=1e-6)
    np.testing.assert_allclose(pos[:, :3, 1], 0.0, atol=1e-6)
    stride = np.linalg.norm(np.diff(pos.astype(np.float64), axis=1), axis=2)
    hi = np.linspace(0.75, 0.9, 10, dtype=np.float32)[level]
    assert stride.min() >= 0.75 - 1e-5 and stride.max() <= hi + 1e-5


@settings(max_examples=8, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(S.integers(0, 2**31 - 1), S.floats(0.1, 1.0))
def test_task_state_machine_invariants(orc, seed, amp):
    n = 8
    st = orc.state(n)
    for k in range(20):
        st["stones"][3 * k + 0][:] = 0.75 * k
    orc.reset_all(st, seed=seed % 1000)
    rng = np.random.default_rng(seed)
    for _ in range(12):
        act = (rng.uniform(-1, 1, (n, 21)) * amp).astype(np.float32)
        obs, rew, term, trunc, _ = orc.env_step(st, act, seed=seed % 1000)
        idx, prev, nxt = st["idx"], st["prev"], st["next"]
        assert np.isfinite(obs).all() and np.isfinite(rew).all()
        assert ((idx >= 1) & (idx <= 19)).all()
        assert (prev == idx - 1).all() and (nxt == np.minimum(idx + 1, 19)).all()
        assert np.isin(st["count"], [0, 1]).all() and np.isin(st["swing"], [0, 1]).all()
        assert (rew[term] == -1.0).all()
        assert not trunc.any()  # 12 steps << 899
