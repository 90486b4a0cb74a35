"""Diagnostic: per-phase cycles of k_step from in-kernel s_memtime stamps (as_debug_stamps).

Runs in the per-wave record mode (slot 31 set): every wave of a launch stores its own record with
plain stores (no atomics, which would queue in front of the late waves' memory traffic and distort
the tail).  The records of each of the last `steps` launches are read back after the launch and
aggregated here: mean / max cycles per phase over all waves, the distribution of per-wave totals,
and the slowest waves of the slowest launch with their SIMD partner (same HW_ID / XCC_ID key).
"""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from allsteps_isaaclab_amd.envs.allsteps_env import AllstepsEnv  # noqa: E402
from allsteps_isaaclab_amd.envs.allsteps_env_cfg import AllstepsEnvCfg  # noqa: E402

PHASES = ["load", "fk", "rnea", "hrow", "sweep", "solve", "collide", "rows", "wsolve", "pgs", "integrate", "fkfinal",
          "task", "reset", "store"]
NP = len(PHASES)
BASE, WORDS = 64, 26


def simd_key(r):
    hw = r[:, NP + 3]
    simd, cu, sh, se = (hw >> 4) & 3, (hw >> 8) & 15, (hw >> 12) & 1, (hw >> 13) & 7
    xcc = r[:, NP + 4] & 15
    return ((xcc * 8 + se) * 2 + sh) * 16 * 4 + cu * 4 + simd


def launch_summary(r, top=6):
    tot = r[:, NP]
    key = simd_key(r)
    rows = np.maximum(r[:, NP + 5], r[:, NP + 6])
    out = []
    for i in np.argsort(-tot)[:top]:
        mates = np.where((key == key[i]) & (np.arange(len(r)) != i))[0]
        out.append({"blk": int(i), "tot": int(tot[i]), "rows": [int(r[i, NP + 5]), int(r[i, NP + 6])],
                    "cons": [int(r[i, NP + 7]), int(r[i, NP + 8])],
                    "mates": [[int(tot[j]), int(rows[j]), int(r[j, NP + 1]) - int(r[i, NP + 1])] for j in mates],
                    "phases": {PHASES[k]: int(r[i, k]) for k in range(NP)}})
    return out


def wave_records(env, acts) -> np.ndarray:
    """[launches, waves, WORDS] per-wave records of k_step for one env.step per action row of `acts`
    (as_debug_stamps in record mode; the stamps add a few s_memtime reads per phase)."""
    n = env.num_envs
    nblk = (n + 1) // 2
    buf = torch.zeros(BASE + nblk * WORDS, dtype=torch.int64, device=env.device)
    buf[31] = 1
    env._native.debug_stamps(buf)
    recs = []
    try:
        for a in acts:
            env.step(a)
            torch.cuda.synchronize()
            recs.append(buf[BASE:].view(nblk, WORDS).cpu().numpy().astype(np.int64).copy())
    finally:
        env._native.debug_stamps(None)
    return np.stack(recs)


def latency_summary(R) -> dict:
    """Latency-side figures of k_step (bench.py roofline.latency): per-wave cycles (mean, slowest),
    the launch's span in cycles (first wave start to last wave end), the mean / slowest wave's share
    of the span, and the slowest wave's phases."""
    tot = R[:, :, NP]
    # the launch span from s_memrealtime (a 100 MHz clock common to the chip; s_memtime counts each
    # CU's own shader clock and is not aligned across CUs), in shader cycles at the waves' own clock
    rt = (R[:, :, NP + 10] - R[:, :, NP + 9]).astype(np.float64)
    clk = np.median((R[:, :, NP + 2] - R[:, :, NP + 1]) / np.maximum(rt, 1) * 100e6)
    span = float(np.mean((R[:, :, NP + 10].max(axis=1) - R[:, :, NP + 9].min(axis=1)) / 100e6 * clk))
    worst = int(np.argmax(tot.max(axis=1)))
    i = int(np.argmax(R[worst, :, NP]))
    return {"avg_wave_cycles": int(tot.mean()), "max_wave_cycles": int(tot.max(axis=1).mean()),
            "launch_cycles": int(span), "clock_ghz": round(clk / 1e9, 3), "avg_wave_over_launch": round(float(tot.mean()) / span, 3),
            "max_wave_over_launch": round(float(tot.max(axis=1).mean()) / span, 3),
            "critical_path_phases": {PHASES[k]: int(R[worst, i, k]) for k in range(NP)},
            "critical_path_rows": [int(R[worst, i, NP + 5]), int(R[worst, i, NP + 6])],
            "mean_phases": {PHASES[k]: int(R[:, :, k].mean()) for k in range(NP)},
            "launches": int(R.shape[0])}


def main(n=4096, steps=30, warm=10, no_self=False):
    cfg = AllstepsEnvCfg()
    cfg.scene.num_envs = n
    cfg.sim.device = "cuda:0"
    model = None
    if no_self:  # ablation: the same kernel without self-collision pairs
        from allsteps_isaaclab_amd.model import load_model

        model = load_model()
        model["num_self_pairs"] = 0
    env = AllstepsEnv(cfg, model=model)
    env.reset()
    gen = torch.Generator(device="cuda").manual_seed(0)
    acts = torch.rand(steps + warm, n, 21, device="cuda", generator=gen) * 2 - 1
    for t in range(warm):
        env.step(acts[t])
    R = wave_records(env, acts[warm:])
    ph = R[:, :, :NP]
    tot = R[:, :, NP]
    rows = np.maximum(R[:, :, NP + 5], R[:, :, NP + 6]).ravel()
    worst = int(np.argmax(tot.max(axis=1)))
    per = {PHASES[k]: int(ph[:, :, k].mean()) for k in range(NP)}
    s = max(sum(per.values()), 1)
    print(json.dumps({
        "n": n, "no_self": no_self, "launches": steps, "cycles_per_wave_step": s,
        "max_wave_step_total_mean": int(tot.max(axis=1).mean()), "max_wave_step_total": int(tot.max()),
        "total_pct": {q: int(np.percentile(tot, q)) for q in (10, 50, 90, 99)},
        "corr_total_rows": round(float(np.corrcoef(tot.ravel(), rows)[0, 1]), 3),
        "latency": latency_summary(R),
        "per_phase": per, "share": {k: round(v / s, 3) for k, v in per.items()},
        "per_phase_max": {PHASES[k]: int(ph[:, :, k].max()) for k in range(NP)},
        "per_phase_p99": {PHASES[k]: int(np.percentile(ph[:, :, k], 99)) for k in range(NP)},
        "worst_launch_top": launch_summary(R[worst])}))
    env.close()


if __name__ == "__main__":
    main(no_self="noself" in sys.argv[1:])
    main(n=512, no_self="noself" in sys.argv[1:])
