"""Diagnostic: how much does a k_step wave's SIMD partner cost it, and can the partner be chosen?

Per-wave records of k_step (scripts/stamps.py wave_records, C2: 4096 envs, level 0) give, for every
launch, each wave's cycles, its two envs' constraint rows (summed over the substeps) and its SIMD
(HW_ID / XCC_ID).  Printed (one JSON line):
  * placement: whether the same workgroups share a SIMD in every launch (then a pairing of env pairs
    with SIMD partners could be planned from the block index alone), and the block-index distance
    between partners;
  * a least-squares fit of a wave's cycles on its own heavier env's rows and its partner's rows;
  * predictability: the correlation of an env's rows in one launch with the next launch's.
"""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from stamps import NP, PHASES, simd_key, wave_records  # noqa: E402
from allsteps_isaaclab_amd.envs.allsteps_env import AllstepsEnv  # noqa: E402
from allsteps_isaaclab_amd.envs.allsteps_env_cfg import AllstepsEnvCfg  # noqa: E402


def xcd_block(b, nb):
    q, r, x, slot = nb >> 3, nb & 7, b & 7, b >> 3
    return (x * (q + 1) if x < r else r * (q + 1) + (x - r) * q) + slot


def main(n=4096, steps=30, warm=20):
    cfg = AllstepsEnvCfg()
    cfg.scene.num_envs = n
    cfg.sim.device = "cuda:0"
    env = AllstepsEnv(cfg)
    env.reset()
    gen = torch.Generator(device="cuda").manual_seed(0)
    acts = torch.rand(steps + warm, n, 21, device="cuda", generator=gen) * 2 - 1
    for t in range(warm):
        env.step(acts[t])
    R = wave_records(env, acts[warm:])  # [L, nb, words]
    L, nb = R.shape[0], R.shape[1]
    tot = R[:, :, NP].astype(np.float64)
    rows = R[:, :, NP + 5: NP + 7].astype(np.float64)  # [L, nb, 2] (env halves)
    own = rows.max(axis=2)
    # partners per launch
    same, dist, mate_rows, mate_tot, waves_per_simd = 0, [], np.zeros((L, nb)), np.zeros((L, nb)), []
    mates0 = None
    for li in range(L):
        key = simd_key(R[li])
        order = np.argsort(key, kind="stable")
        ks = key[order]
        groups = np.split(order, np.flatnonzero(np.diff(ks)) + 1)
        waves_per_simd.append(np.bincount([len(g) for g in groups]).tolist())
        mates = np.full(nb, -1)
        for g in groups:
            if len(g) == 2:
                mates[g[0]], mates[g[1]] = g[1], g[0]
                dist.append(abs(int(g[1]) - int(g[0])))
        has = mates >= 0
        mate_rows[li, has] = own[li, mates[has]]
        mate_tot[li, has] = tot[li, mates[has]]
        if mates0 is None:
            mates0 = mates
        else:
            same += int(np.sum(mates == mates0))
    X = np.stack([np.ones(L * nb), own.ravel(), mate_rows.ravel()], axis=1)
    coef, *_ = np.linalg.lstsq(X, tot.ravel(), rcond=None)
    # CU level: the rows of the other waves on the same CU (other SIMDs), and the block -> CU pattern
    cu_rows = np.zeros((L, nb))
    cu_of = []
    for li in range(L):
        ck = simd_key(R[li]) // 4
        cu_of.append(ck)
        sums = np.bincount(ck, weights=own[li], minlength=ck.max() + 1)
        cu_rows[li] = sums[ck] - own[li] - mate_rows[li]
    X2 = np.stack([np.ones(L * nb), own.ravel(), mate_rows.ravel(), cu_rows.ravel()], axis=1)
    coef2, *_ = np.linalg.lstsq(X2, tot.ravel(), rcond=None)
    ck0 = cu_of[0]
    cu_blocks = [sorted(np.flatnonzero(ck0 == c).tolist()) for c in np.unique(ck0)[:3]]
    # env rows launch to launch (env id of block b, half h)
    # (only with the fixed placement: under the cost-balanced wave map the env of a block moves)
    c1 = None
    if os.environ.get("ALLSTEPS_WAVE_MAP") == "0":
        eid = np.array([[xcd_block(b, nb) * 2 + h for h in range(2)] for b in range(nb)])
        er = np.zeros((L, n))
        er[:, eid.ravel()] = rows.reshape(L, -1)
        c1 = round(float(np.corrcoef(er[:-1].ravel(), er[1:].ravel())[0, 1]), 3)
    worst = np.argmax(tot, axis=1)
    d = {"n": n, "launches": L, "waves_per_simd_hist": waves_per_simd[0],
         "mates_same_as_launch0": round(same / max((L - 1) * nb, 1), 3),
         "mate_block_distance_top": [[int(k), int(v)] for k, v in sorted(zip(*np.unique(dist, return_counts=True)), key=lambda kv: -kv[1])[:10]],
         "fit_cycles": {"const": round(coef[0]), "per_own_row": round(coef[1], 1), "per_mate_row": round(coef[2], 1)},
         "fit_cycles_cu": {"const": round(coef2[0]), "per_own_row": round(coef2[1], 1), "per_mate_row": round(coef2[2], 1),
                           "per_cu_other_row": round(coef2[3], 1)},
         "cu_same_as_launch0": round(float(np.mean([np.mean(c == ck0) for c in cu_of[1:]])), 3),
         "cu_blocks_example": cu_blocks,
         "rows_mean": round(float(own.mean()), 2), "rows_p99": float(np.percentile(own, 99)),
         "env_rows_corr_next_launch": c1,
         "pairs_own_mate_rows_corr": round(float(np.corrcoef(own.ravel(), mate_rows.ravel())[0, 1]), 3),
         "slowest": [{"tot": int(tot[li, w]), "own": int(own[li, w]), "mate": int(mate_rows[li, w]),
                      "mate_tot": int(mate_tot[li, w])} for li, w in enumerate(worst)][:10],
         "mean_tot": int(tot.mean()), "max_tot_mean": int(tot.max(axis=1).mean()),
         "top_waves_by_launch": [[[int(tot[li, w]), int(own[li, w]), int(mate_rows[li, w])] for w in np.argsort(-tot[li])[:8]]
                                 for li in range(3)],
         "mean_phases": {PHASES[k]: int(R[:, :, k].mean()) for k in range(NP)},
         "slowest_phases": [{PHASES[k]: int(R[li, w, k]) for k in range(NP)} for li, w in enumerate(worst)][:6],
         "slowest_cons": [[int(R[li, w, NP + 7]), int(R[li, w, NP + 8])] for li, w in enumerate(worst)][:10]}
    # counterfactual from the fit: the slowest wave if its partner were the lightest
    print(json.dumps(d))
    env.close()


if __name__ == "__main__":
    main()
