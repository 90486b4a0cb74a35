"""Bit-exact HIP <-> oracle parity over multi-step trajectories (SURVEY §8c tier B).

The HIP step kernels (liballsteps_hip.so, called through the C ABI) and the CPU oracle
(oracle/physics.c + task.c) compute the same float32 operations in the same order: both are built
with -ffp-contract=off, every FMA is an explicit fmaf of include/as_detmath.h, sin/cos are the shared
as_sincosf, and the oracle restates the kernel's cross-lane reductions (32-lane trees, two-partial W
rows, triplet PGS) serially.  So from an identical state, with the same actions and the same Philox
reset stream, every step must give:

  * discrete outputs -- terminated, truncated, target index / prev / next, reach count, swing leg,
    episode length, reset counter, per-(foot, stone) contact masks, curriculum level -- equal for
    100 % of the envs (allsteps_env.py:396-457 decisions on the physics state);
  * the physical state (root pose / velocity, joint angles / velocities, body positions, potentials,
    foot contact flags) bit-identical (compared with ==, so only the sign of a zero may differ);
  * observations and rewards == as well: roll / pitch use the shared deterministic atan2 / asin /
    remainder of include/as_detmath.h, the step reward its exp, and the oracle restates the
    kernel's 32-lane tree for the per-env action / energy sums (oracle/task.c half_tree32).

The mismatch counts are printed for every step of every run.  Sizes: C1 (2 envs, level 0), C2
(4096 envs, level 0) and C3 (32768 envs, stone level 9) from reset, and C2 / C3 from a warm state
(120 GPU steps of random actions first: fallen robots, contact-saturated envs, resets in flight).
"""

import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

INT_FIELDS = ("idx", "prev", "next", "count", "swing", "ep_len", "episode", "contact_mask")
FLOAT_FIELDS = ("root_pos", "root_quat", "root_lin", "root_ang", "q", "qd", "body_pos", "pot", "old_pot",
                "foot_contact", "stones")
THREADS = max(1, min(16, os.cpu_count() or 1))


def _env(n, level, seed):
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


def _mismatch(gs, st, n):
    """Per field: the envs whose entries differ (== comparison)."""
    out = {}
    for k in INT_FIELDS + FLOAT_FIELDS:
        g = gs[k].reshape(-1, n)
        c = st[k].reshape(-1, n)
        if k in INT_FIELDS:
            g = g.view(np.uint32)
            c = c.view(np.uint32)
        bad = (g != c).any(0)
        out[k] = np.flatnonzero(bad)
    out["curriculum"] = np.array([], int) if int(gs["curriculum"][0]) == int(st["curriculum"][0]) else np.array([0])
    return out


def _describe(gs, st, n, bad):
    lines = []
    for k, ids in bad.items():
        if len(ids) == 0 or k == "curriculum":
            continue
        e = int(ids[0])
        g = gs[k].reshape(-1, n)[:, e]
        c = st[k].reshape(-1, n)[:, e]
        if k in FLOAT_FIELDS:
            d = np.abs(g.astype(np.float64) - c.astype(np.float64))
            lines.append(f"  {k}: {len(ids)} envs, first env {e}, max |diff| {d.max():.3e} at row {int(d.argmax())}")
        else:
            lines.append(f"  {k}: {len(ids)} envs, first env {e}: gpu {g.tolist()} oracle {c.tolist()}")
    return "\n".join(lines)


def _run(orc, capsys, n, level, steps, warm, seed=42, near_timeout=False):
    env = _env(n, level, seed)
    env.reset()
    gen = torch.Generator(device="cuda").manual_seed(seed + warm)
    for _ in range(warm):  # GPU alone: reach a contact-rich, mid-episode state
        env.step(torch.rand(n, 21, device="cuda", generator=gen) * 2.4 - 1.2)
    if near_timeout:  # episode counters 890..898: every env meets the 899-step time-out inside the window
        env.set_state({"ep_len": (890 + torch.arange(n, device="cuda") % 9).to(torch.int32).reshape(1, n)})
    torch.cuda.synchronize()
    st = orc.state(n)
    _to_oracle(env, st)
    rng = np.random.default_rng(1000 + n + level + warm)
    resets = contacts = dropped = truncs = 0
    for t in range(steps):
        act = rng.uniform(-1.2, 1.2, (n, 21)).astype(np.float32)
        o_g, r_g, t_g, tr_g, _ = env.step(torch.from_numpy(act).cuda())
        torch.cuda.synchronize()
        o_c, r_c, t_c, tr_c, _ = orc.env_step(st, act, seed=seed, nthreads=THREADS)
        gs = {k: v.cpu().numpy() for k, v in env.get_state().items()}
        bad = _mismatch(gs, st, n)
        bad["terminated"] = np.flatnonzero(t_g.cpu().numpy() != t_c)
        bad["truncated"] = np.flatnonzero(tr_g.cpu().numpy() != tr_c)
        og = o_g["policy"].cpu().numpy()
        bad["obs"] = np.flatnonzero((og != o_c).any(1))
        rg = r_g.cpu().numpy()
        bad["reward"] = np.flatnonzero(rg != r_c)
        nbad = len(set().union(*[set(v.tolist()) for v in bad.values()]))
        # contacts cut by the constraint budget this step: the device counter == the oracle's count
        d_g = env.dropped_contacts()
        assert d_g == orc.last_dropped, (t, d_g, orc.last_dropped)
        dropped += d_g
        resets += int((t_c | tr_c).sum())
        truncs += int(tr_c.sum())
        contacts += int((st["contact_mask"] != 0).any(0).sum())
        with capsys.disabled():
            print(f"[exact n={n} level={level} warm={warm}] step {t}: {nbad} of {n} envs mismatched "
                  f"(resets {int((t_c | tr_c).sum())}, envs in contact {int((st['contact_mask'] != 0).any(0).sum())}, "
                  f"contacts dropped {d_g} = oracle {orc.last_dropped})")
        assert nbad == 0, f"step {t}: {nbad} envs differ\n" + _describe(gs, st, n, bad) + "\n" + \
            "\n".join(f"  {k}: {len(v)} envs" for k, v in bad.items() if len(v) and k in ("terminated", "truncated",
                                                                                          "obs", "reward"))
    env.close()
    return resets, contacts, dropped, truncs


@pytest.mark.parametrize("n,level,steps,warm", [
    (2, 0, 40, 0),          # C1 size
    (4096, 0, 40, 0),       # C2 from reset: the drop onto the stones
    (4096, 0, 20, 120),     # C2 warm: fallen robots, saturated contact sets, resets in flight
    (32768, 9, 20, 0),      # C3 from reset
    (32768, 9, 20, 120),    # C3 warm
    (1024, 0, 400, 0),      # long horizon: 400 consecutive steps, every env through falls and resets
])
def test_trajectory_bit_exact(orc, capsys, n, level, steps, warm):
    resets, contacts, dropped, _ = _run(orc, capsys, n, level, steps, warm)
    if n >= 4096:
        assert contacts > 0, "no env ever touched a stone: the trajectory did not exercise the contact path"
    if n == 32768 and warm:
        assert dropped > 0, "the C3 warm trajectory never hit the constraint budget: the drop count is untested"
    if warm:
        assert resets > 0, "no env reset during the compared steps"


@pytest.mark.parametrize("n,level", [(4096, 0), (32768, 9)])
def test_time_out_path_bit_exact(orc, capsys, n, level):
    """Full steps (physics + task) across the 899-step time-out (allsteps_env.py:399 with direct_rl_env.py:248-250, truncated =
    episode_length_buf >= max_episode_length - 1): episode counters preset to 890..898 after a warm-up,
    then 12 steps in lock-step with the oracle -- every env that has not fallen is truncated and reset
    inside the window (the random-action trajectories above fall long before 899 steps)."""
    resets, contacts, dropped, truncs = _run(orc, capsys, n, level, 12, 60, near_timeout=True)
    assert truncs > 0, "no time-out inside the window"
    with capsys.disabled():
        print(f"[time-out n={n}] {truncs} time-outs, {resets} resets, {dropped} contacts dropped in 12 steps")
