"""GPU parity: the HIP step kernels vs the CPU oracle (and the reference golden vectors).

Tolerances (float32 on both sides, the same operations in the same order: -ffp-contract=off plus
the explicit fmaf of include/as_detmath.h on both, the kernel's lane reductions restated serially in
the oracle -- see tests/test_gpu_exact.py for the multi-step trajectories):
  * task logic on identical inputs: ints / bools exact, floats rtol 1e-5 / atol 1e-4 (vs the
    reference's own torch outputs);
  * one full env step (4 physics substeps) from an identical state: discrete outputs (terminated,
    truncated, target index, reach count, swing leg, contact flags) equal for every env, and the
    physical state, observations and rewards bit-identical (the transcendentals are the shared
    deterministic forms of include/as_detmath.h, the reward sums the kernel's lane tree).
"""

import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu


def _env(n, level=0, seed=42):
    from allsteps_isaaclab_amd.envs.allsteps_env import AllstepsEnv
    from allsteps_isaaclab_amd.envs.allsteps_env_cfg import AllstepsEnvCfg

    cfg = AllstepsEnvCfg()
    cfg.scene.num_envs = n
    cfg.sim.device = "cuda:0"
    cfg.seed = seed
    cfg.initial_stone_curriculum = level
    return AllstepsEnv(cfg)


def _to_oracle(env, st):
    for k, v in env.get_state().items():
        st[k][...] = v.cpu().numpy().reshape(st[k].shape).view(st[k].dtype)


def _from_oracle(env, st):
    s = {}
    for k in env.state:
        a = np.ascontiguousarray(st[k])
        if a.dtype == np.uint32:
            a = a.view(np.int32)
        s[k] = torch.from_numpy(a)
    env.set_state(s)


def _gpu_state(env):
    return {k: v.cpu().numpy() for k, v in env.get_state().items()}


def test_library_exports_and_loads():
    from allsteps_isaaclab_amd import _native

    L = _native.load()
    assert L.as_abi_version() == _native.ABI_VERSION


@pytest.mark.parametrize("n16", [1, 1023, 1024 * 256 * 40 + 7])
def test_hbm_copy_probe(n16):
    """as_hbm_copy (bench.py's measured HBM peak) copies every 16-B element, ragged tails included,
    and rejects misaligned pointers."""
    import ctypes as C

    from allsteps_isaaclab_amd import _native

    L = _native.load()
    src = torch.randint(-2**31, 2**31 - 1, (n16 * 4 + 4,), dtype=torch.int32, device="cuda:0")
    dst = torch.zeros_like(src)
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    _native.check(L.as_hbm_copy(C.c_void_p(dst.data_ptr()), C.c_void_p(src.data_ptr()), n16, s), "as_hbm_copy")
    torch.cuda.synchronize()
    assert torch.equal(dst[: n16 * 4], src[: n16 * 4])
    assert not dst[n16 * 4:].any(), "copy wrote past n16 elements"
    assert L.as_hbm_copy(C.c_void_p(dst.data_ptr() + 4), C.c_void_p(src.data_ptr()), 1, s) != 0


@pytest.mark.parametrize("level", [0, 3, 9])
def test_stones_vs_golden(orc, level):
    """k_stones vs the reference's own courses (within the transcendental's ulps) and vs the oracle's
    (bit-identical: both use as_sincosf)."""
    g = golden("footsteps")
    draws = torch.from_numpy(g[f"fs{level}_draws"])
    n = draws.shape[1]
    env = _env(n)
    env.generate_foot_steps(level, draws)
    torch.cuda.synchronize()
    pos = env.steps_pos.cpu().numpy()
    np.testing.assert_allclose(pos, g[f"fs{level}_pos"], rtol=1e-5, atol=5e-6)
    pos_c, _ = orc.footsteps(n, level, g[f"fs{level}_draws"])
    assert np.array_equal(pos, pos_c), np.abs(pos - pos_c).max()
    env.close()


@pytest.mark.parametrize("fixture", ["task_seq", "gates"])
def test_task_logic_golden_replay(orc, oracle_mod, fixture):
    """Replay the reference task sequences through the GPU task kernel (physics bypassed): ints /
    bools exact and floats near-exact vs the reference's own outputs (until the first reset; post-
    reset body positions come from real FK on the GPU, fake FK in the fixture), and observations and
    rewards bit-identical to the oracle's on the same inputs (gates: roll / pitch straddling the
    reward gates by 10 ulp .. 0.01 rad)."""
    g = golden(fixture)
    n = g["init_idx"].shape[0]
    env = _env(n)
    st = orc.state(n)
    for k in ("idx", "prev", "next", "count", "swing", "ep_len"):
        st[k][:] = g["init_" + k]
    st["pot"][:] = g["init_pot"]
    st["old_pot"][:] = g["init_old_pot"]
    st["stones"][:] = g["steps_pos"].reshape(n, 60).T
    T = g["seq_obs"].shape[0]
    for t in range(T):
        rs = g["seq_root_state"][t]
        st["root_pos"][:] = rs[:, 0:3].T
        st["root_quat"][:] = rs[:, 3:7].T
        st["root_lin"][:] = rs[:, 7:10].T
        st["root_ang"][:] = rs[:, 10:13].T
        st["q"][:] = g["seq_joint_pos"][t].T
        st["qd"][:] = g["seq_joint_vel"][t].T
        st["body_pos"][:] = np.concatenate([g["seq_torso"][t], g["seq_rfoot"][t], g["seq_lfoot"][t]], 1).T
        for f, key in ((0, "seq_fm_r"), (1, "seq_fm_l")):
            nrm = np.linalg.norm(g[key][t], axis=-1) > 1e-4          # (n, 20) force-matrix flags
            st["contact_mask"][f] = (nrm * (1 << np.arange(20))).sum(1).astype(np.uint32)
        _from_oracle(env, st)
        act = g["seq_actions"][t]
        draws = g["seq_reset_draws"][t]
        o_g, r_g, t_g, tr_g, _ = env.task_step(torch.from_numpy(act), torch.from_numpy(draws))
        torch.cuda.synchronize()
        # oracle, same inputs, physics FK for reset envs
        import ctypes as C
        O = oracle_mod
        obs = np.zeros((n, 59), np.float32)
        rew = np.zeros(n, np.float32)
        term = np.zeros(n, np.uint8)
        trunc = np.zeros(n, np.uint8)
        anyr = np.zeros(1, np.int32)
        orc.L.or_task_post_physics(C.byref(orc.model), C.byref(orc.task), st.ptr, O.fp(np.ascontiguousarray(act)),
                                   None, None, O.fp(np.ascontiguousarray(draws)), 0, None, None, O.fp(obs),
                                   O.fp(rew), O.u8p(term), O.u8p(trunc), O.ip(anyr))
        msg = f"step {t}"
        np.testing.assert_array_equal(t_g.cpu().numpy(), g["seq_terminated"][t], msg)
        np.testing.assert_array_equal(tr_g.cpu().numpy(), g["seq_truncated"][t], msg)
        np.testing.assert_allclose(r_g.cpu().numpy(), g["seq_reward"][t], rtol=1e-5, atol=1e-4, err_msg=msg)
        gs = _gpu_state(env)
        for k in ("idx", "prev", "next", "count", "swing", "ep_len"):
            np.testing.assert_array_equal(gs[k], st[k], f"{msg} {k}")
        assert gs["curriculum"][0] == st["curriculum"][0] == g["seq_curriculum"][t][0], msg
        og = o_g["policy"].cpu().numpy()
        # the same arithmetic on both sides (include/as_detmath.h transcendentals, the kernel's reward
        # tree restated in oracle/task.c): == (only the sign of a zero may differ)
        assert np.array_equal(og, obs), (msg, np.abs(og - obs).max())
        assert np.array_equal(r_g.cpu().numpy(), rew), (msg, np.abs(r_g.cpu().numpy() - rew).max())
        if not g["seq_any_reset"][t]:
            np.testing.assert_allclose(np.delete(og, [1, 2], 1), np.delete(g["seq_obs"][t], [1, 2], 1), rtol=1e-5,
                                       atol=1e-4, err_msg=msg)
        # continue the replay from the fixture's own post-step task state
        for k in ("idx", "prev", "next", "count", "swing", "ep_len"):
            st[k][:] = g["seq_" + k][t]
        st["pot"][:] = g["seq_pot"][t]
        st["old_pot"][:] = g["seq_old_pot"][t]
        st["curriculum"][0] = g["seq_curriculum"][t][0]
    env.close()


def _random_states(orc, n, steps, seed, level=0):
    """Reference-distribution states: oracle reset then `steps` random-action env steps, on the
    level-0 straight line or on stones generated at curriculum `level`."""
    st = orc.state(n)
    if level == 0:
        for k in range(20):
            st["stones"][3 * k + 0][:] = 0.75 * k
            st["stones"][3 * k + 2][:] = np.float32(k * 0.75) * np.cos(np.float32(np.pi / 2), dtype=np.float32)
    else:
        rng = np.random.default_rng(seed + 1000)
        pos, _ = orc.footsteps(n, level, rng.uniform(0, 1, (5, n, 20)).astype(np.float32))
        st["stones"][:] = pos.reshape(n, 60).T
    orc.reset_all(st, seed=seed)
    rng = np.random.default_rng(seed)
    for _ in range(steps):
        orc.env_step(st, rng.uniform(-1, 1, (n, 21)).astype(np.float32), seed=seed)
    return st


@pytest.mark.parametrize("warm,level", [(0, 0), (10, 0), (40, 0), (10, 9), (40, 9)])
def test_env_step_parity(orc, warm, level):
    n = 256
    st = _random_states(orc, n, warm, seed=7 + warm, level=level)
    env = _env(n)
    _from_oracle(env, st)
    rng = np.random.default_rng(100 + warm)
    act = rng.uniform(-1, 1, (n, 21)).astype(np.float32)
    draws = rng.uniform(0, 1, (n, 22)).astype(np.float32)
    o_g, r_g, t_g, tr_g, _ = env.step_with_draws(torch.from_numpy(act), torch.from_numpy(draws))
    torch.cuda.synchronize()
    o_c, r_c, t_c, tr_c, _ = orc.env_step(st, act, reset_draws=draws)
    gs = _gpu_state(env)
    disc = np.ones(n, bool)
    disc &= t_g.cpu().numpy() == t_c
    disc &= tr_g.cpu().numpy() == tr_c
    for k in ("idx", "count", "swing"):
        disc &= gs[k] == st[k]
    disc &= (gs["contact_mask"].view(np.uint32) == st["contact_mask"]).all(0)
    print(f"env_step parity warm={warm} level={level}: {int((~disc).sum())} of {n} envs with a discrete mismatch")
    assert disc.all(), f"discrete mismatch on {np.flatnonzero(~disc)}"
    for k in ("root_pos", "root_quat", "q", "body_pos", "root_lin", "root_ang", "qd", "pot", "old_pot"):
        assert np.array_equal(gs[k], st[k]), (k, np.abs(gs[k] - st[k]).max())
    og = o_g["policy"].cpu().numpy()
    assert np.array_equal(og, o_c), np.abs(og - o_c).max()
    assert np.array_equal(r_g.cpu().numpy(), r_c), np.abs(r_g.cpu().numpy() - r_c).max()
    env.close()


@pytest.mark.parametrize("n", [1, 2, 3, 65])
def test_env_step_parity_ragged(orc, n):
    """Env counts that leave the last two-env workgroup half empty (and a single env): the idle half
    must neither write nor disturb its neighbour; every env is checked exactly as above."""
    st = _random_states(orc, n, 10, seed=11 + n)
    env = _env(n)
    _from_oracle(env, st)
    rng = np.random.default_rng(200 + n)
    act = rng.uniform(-1, 1, (n, 21)).astype(np.float32)
    draws = rng.uniform(0, 1, (n, 22)).astype(np.float32)
    o_g, r_g, t_g, tr_g, _ = env.step_with_draws(torch.from_numpy(act), torch.from_numpy(draws))
    torch.cuda.synchronize()
    o_c, r_c, t_c, tr_c, _ = orc.env_step(st, act, reset_draws=draws)
    gs = _gpu_state(env)
    np.testing.assert_array_equal(t_g.cpu().numpy(), t_c)
    np.testing.assert_array_equal(tr_g.cpu().numpy(), tr_c)
    for k in ("idx", "count", "swing", "ep_len"):
        np.testing.assert_array_equal(gs[k], st[k], k)
    np.testing.assert_array_equal(gs["contact_mask"].view(np.uint32), st["contact_mask"])
    for k in ("root_pos", "root_quat", "q", "body_pos", "root_lin", "root_ang", "qd"):
        assert np.array_equal(gs[k], st[k]), (k, np.abs(gs[k] - st[k]).max())
    og = o_g["policy"].cpu().numpy()
    assert np.array_equal(og, o_c), np.abs(og - o_c).max()
    assert np.array_equal(r_g.cpu().numpy(), r_c)
    env.close()


def test_reset_all_parity(orc):
    n = 128
    env = _env(n)
    st = orc.state(n)
    _to_oracle(env, st)
    rng = np.random.default_rng(3)
    draws = rng.uniform(0, 1, (n, 22)).astype(np.float32)
    o_g, _ = env.reset_with_draws(torch.from_numpy(draws))
    torch.cuda.synchronize()
    o_c = orc.reset_all(st, reset_draws=draws)
    gs = _gpu_state(env)
    for k in ("idx", "prev", "next", "count", "swing", "ep_len"):
        np.testing.assert_array_equal(gs[k], st[k], k)
    for k in ("q", "body_pos", "root_pos", "root_quat"):
        assert np.array_equal(gs[k], st[k]), k
    assert np.array_equal(o_g["policy"].cpu().numpy(), o_c)
    # running-start pose quirk: the mirrored half has the swing leg flipped
    assert set(np.unique(gs["swing"])) == {0, 1}
    env.close()


@pytest.mark.parametrize("kind", ["partial", "none", "all"])
def test_reset_mask_parity(orc, kind):
    """_reset_idx(env_ids) on a subset (as_reset_mask) vs the oracle's masked reset, from states
    reached by random stepping (non-trivial foot state for the second tick)."""
    n = 128
    st = _random_states(orc, n, 12, seed=31)
    env = _env(n)
    _from_oracle(env, st)
    rng = np.random.default_rng(5)
    mask = {"partial": rng.uniform(size=n) < 0.3, "none": np.zeros(n, bool), "all": np.ones(n, bool)}[kind]
    draws = rng.uniform(0, 1, (n, 22)).astype(np.float32)
    before = _gpu_state(env)
    o_g = env._reset_idx(torch.from_numpy(mask), reset_draws=torch.from_numpy(draws))
    torch.cuda.synchronize()
    o_c = orc.reset_mask(st, mask, reset_draws=draws)
    gs = _gpu_state(env)
    for k in ("idx", "prev", "next", "count", "swing", "ep_len", "episode", "curriculum"):
        np.testing.assert_array_equal(gs[k], st[k], k)
    for k in ("q", "qd", "root_pos", "root_quat", "root_lin", "root_ang"):
        assert np.array_equal(gs[k], st[k]), k
        # envs outside the mask keep their physical state bit for bit
        np.testing.assert_array_equal(gs[k][..., ~mask], before[k][..., ~mask], k)
    assert np.array_equal(gs["body_pos"], st["body_pos"])
    assert np.array_equal(gs["pot"], st["pot"])
    og = o_g["policy"].cpu().numpy()
    assert np.array_equal(og, o_c), np.abs(og - o_c).max()
    if kind == "none":
        for k in before:
            np.testing.assert_array_equal(gs[k], before[k], k)
    env.close()


def test_philox_reset_draws_match_oracle(orc):
    """Without injected draws both sides use Philox(seed, env, episode): resets agree."""
    n = 64
    env = _env(n, seed=1234)
    st = orc.state(n)
    _to_oracle(env, st)
    o_g, _ = env.reset()
    torch.cuda.synchronize()
    o_c = orc.reset_all(st, seed=1234)
    assert np.array_equal(env.get_state()["q"].cpu().numpy(), st["q"])
    assert np.array_equal(o_g["policy"].cpu().numpy(), o_c)
    env.close()


def test_free_fall_gpu():
    n = 64
    env = _env(n)
    s = env.get_state()
    s["root_pos"][2] = 10.0
    env.set_state(s)
    env.physics_step(torch.zeros(n, 21))
    torch.cuda.synchronize()
    st = env.get_state()
    np.testing.assert_allclose(st["root_lin"][2].cpu().numpy(), -9.81 * 4 / 240, rtol=1e-5)
    assert st["qd"].abs().max().item() < 1e-4
    assert int(st["contact_mask"].abs().max()) == 0
    env.close()


def test_determinism_and_long_rollout():
    """Two envs, same seed, same actions: bitwise identical; 300 random steps stay finite."""
    n = 1024
    outs = []
    for _ in range(2):
        env = _env(n, seed=42)
        env.reset()
        gen = torch.Generator(device="cuda").manual_seed(0)
        for t in range(300):
            a = torch.rand(n, 21, device="cuda", generator=gen) * 2 - 1
            obs, rew, term, trunc, _ = env.step(a)
        torch.cuda.synchronize()
        o = obs["policy"].cpu().numpy()
        assert np.isfinite(o).all() and np.isfinite(rew.cpu().numpy()).all()
        outs.append((o, env.get_state()["q"].cpu().numpy()))
        env.close()
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1], outs[1][1])


def _env_off(n, offset, seed=42):
    from allsteps_isaaclab_amd.envs.allsteps_env import AllstepsEnv
    from allsteps_isaaclab_amd.envs.allsteps_env_cfg import AllstepsEnvCfg

    cfg = AllstepsEnvCfg()
    cfg.scene.num_envs = n
    cfg.sim.device = "cuda:0"
    cfg.seed = seed
    return AllstepsEnv(cfg, env_id_offset=offset)


def test_shards_match_unsharded():
    """Weak-scaling layout: two shards (global env ids [0, n/2), [n/2, n)) stepped side by side give
    bitwise the same trajectories as one env of n (Philox reset draws keyed by global env id)."""
    n, h, steps = 1024, 512, 120
    full = _env_off(n, 0)
    parts = [_env_off(h, 0), _env_off(h, h)]
    full.reset()
    for p in parts:
        p.reset()
    gen = torch.Generator(device="cuda").manual_seed(7)
    resets = 0
    for _ in range(steps):
        a = torch.rand(n, 21, device="cuda", generator=gen) * 2 - 1
        of, rf, tf, uf, _ = full.step(a)
        outs = [p.step(a[i * h:(i + 1) * h]) for i, p in enumerate(parts)]
        torch.testing.assert_close(torch.cat([o[0]["policy"] for o in outs]), of["policy"], rtol=0, atol=0)
        torch.testing.assert_close(torch.cat([o[1] for o in outs]), rf, rtol=0, atol=0)
        assert torch.equal(torch.cat([o[2] for o in outs]), tf) and torch.equal(torch.cat([o[3] for o in outs]), uf)
        resets += int((tf | uf).sum())
    assert resets > 0, "no env reset: the test did not exercise the Philox reset path"
    sf = full.get_state()
    for k in ("q", "qd", "root_pos", "idx", "episode"):
        cat = torch.cat([p.get_state()[k].reshape(-1, h) for p in parts], dim=1)
        assert torch.equal(cat.reshape(sf[k].shape), sf[k]), k
    for e in [full] + parts:
        e.close()


def test_c3_large_config_invariants():
    """C3 (32768 envs, stone curriculum level 9): size-independent invariants of the task state
    after 60 steps of random actions (allsteps_env.py semantics): finite outputs, stones never
    regenerated, target indices consistent, done envs restarted, episode counters bounded."""
    n = 32768
    env = _env(n, level=9)
    stones0 = env.state["stones"].clone()
    env.reset()
    gen = torch.Generator(device="cuda").manual_seed(3)
    for _ in range(60):
        a = torch.rand(n, 21, device="cuda", generator=gen) * 2 - 1
        obs, rew, term, trunc, _ = env.step(a)
        done = term | trunc
        assert torch.isfinite(obs["policy"]).all() and torch.isfinite(rew).all()
        ep = env.episode_length_buf
        assert bool((ep[done] == 0).all()) and int(ep.max()) <= 899
    assert torch.equal(env.state["stones"], stones0)
    idx, prev, nxt = (env.state[k] for k in ("idx", "prev", "next"))
    assert int(idx.min()) >= 1 and int(idx.max()) <= 19
    assert torch.equal(prev, idx - 1) and torch.equal(nxt, torch.clamp(idx + 1, max=19))
    assert 0 <= int(env.state["curriculum"][0]) <= 9
    assert bool(((env.state["swing"] == 0) | (env.state["swing"] == 1)).all())
    env.close()


def test_bench_two_ranks_one_gpu():
    """Rehearsal of the driver's multi-GPU bench launch (torch.distributed.run, one process per rank,
    barrier + max-over-ranks timing) with two ranks sharing cuda:0 over gloo: rank 0 prints ONE JSON
    line whose value counts both ranks' envs, with the env + PPO `train` leg measured on both ranks."""
    import json
    import os
    import socket
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ, ALLSTEPS_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "20",
           "--warmup", "3", "--num-envs", "256", "--no-cpu-baseline", "--no-c5", "--train-envs", "1024",
           "--multi-gpu-mode", "allgather"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = lines[0]
    assert line["n_gpus"] == 2 and line["config"]["global_envs"] == 512 and line["scaling"] == "weak"
    assert abs(line["value"] - 512 * 20 / (line["ms_per_step"] * 20 / 1e3)) / line["value"] < 1e-2
    # C4's env + PPO leg runs at N ranks too (the trainer's --distributed path), counting both ranks
    tr = line["train"]
    assert "error" not in tr, (tr, r.stderr[-2000:])
    assert tr["n_gpus"] == 2 and tr["global_envs"] == 2048 and tr["value"] > 0
    assert tr["multi_gpu_mode"] == "allgather"  # the north star's exchange, selected explicitly


def test_bench_gpus_flag_launches_ranks_itself():
    """`python bench.py --gpus 2` with NO launcher in the command (the driver's and a user's plain
    invocation): bench.py starts torch.distributed.run as a child, the two ranks (sharing cuda:0 over
    gloo here) form the job, and the relayed line reports both GPUs' envs."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["ALLSTEPS_DIST_BACKEND"] = "gloo"
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "20", "--warmup", "3",
           "--num-envs", "256", "--no-cpu-baseline", "--no-c5", "--train-envs", "1024"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = lines[0]
    assert line["n_gpus"] == 2 and line["config"]["global_envs"] == 2 * line["config"]["num_envs_per_gpu"] == 512
    tr = line["train"]
    assert "error" not in tr, (tr, r.stderr[-2000:])
    assert tr["n_gpus"] == 2 and tr["multi_gpu_mode"] == "allreduce"  # bench default
    tg = line["train_allgather"]  # the north star's exchange, reported beside the default
    assert "error" not in tg, (tg, r.stderr[-2000:])
    assert tg["n_gpus"] == 2 and tg["multi_gpu_mode"] == "allgather"
    assert line["no_preheat"]["value"] > 0
    # the kernel timings come from a bit-exact replay of each rank's timed window, >= 200 launches
    km = line["kernels_ms"]
    assert km["replay_exact"] and km["sampled_launches"] >= 200


@pytest.mark.gpu
def test_bench_single_gpu_driver_shape():
    """The driver's own invocation shape (K = 20, W = 5): the replay of the timed window is bit-exact,
    >= 200 launches are event-timed whatever K is, and the event figures account for the timed loop's
    wall clock (bench.events_consistent); the roofline's duration is the event average."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--steps", "20", "--warmup", "5", "--no-cpu-baseline",
           "--no-c5", "--no-train"]
    r = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    km = line["kernels_ms"]
    print(json.dumps(km))
    assert km["replay_exact"] and km["sampled_launches"] == 200
    assert km["events_consistent"], km
    assert line["roofline"]["duration_ms"] == km["k_step_ms"]
    assert "error" not in (line["roofline"]["latency"] or {})
    assert line["contacts_dropped"]["total"] >= 0
