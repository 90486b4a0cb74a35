"""Diagnostic: per-phase cycles of k_step from in-kernel s_memtime stamps (as_debug_stamps)."""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from allsteps_isaaclab_amd.envs.allsteps_env import AllstepsEnv  # noqa: E402
from allsteps_isaaclab_amd.envs.allsteps_env_cfg import AllstepsEnvCfg  # noqa: E402

PHASES = ["load", "fk", "rnea", "hrow", "sweep", "solve", "collide", "rows", "wsolve", "pgs", "integrate", "task",
          "reset", "store"]


def main(n=4096, steps=50):
    cfg = AllstepsEnvCfg()
    cfg.scene.num_envs = n
    cfg.sim.device = "cuda:0"
    env = AllstepsEnv(cfg)
    env.reset()
    gen = torch.Generator(device="cuda").manual_seed(0)
    acts = torch.rand(steps + 10, n, 21, device="cuda", generator=gen) * 2 - 1
    for t in range(10):
        env.step(acts[t])
    buf = torch.zeros(32, dtype=torch.int64, device="cuda")
    env._native.debug_stamps(buf)
    for t in range(steps):
        env.step(acts[10 + t])
    torch.cuda.synchronize()
    env._native.debug_stamps(None)
    waves = (n + 1) // 2 * steps
    tot = buf.cpu().tolist()
    per = {PHASES[i]: round(tot[i] / waves) for i in range(len(PHASES))}
    s = sum(per.values())
    mx = {PHASES[i]: tot[16 + i] for i in range(len(PHASES))}
    print(json.dumps({"n": n, "cycles_per_wave_step": s, "max_wave_step_total": tot[len(PHASES)], "per_phase_max": mx,
                      "per_phase": per,
                      "share": {k: round(v / s, 3) for k, v in per.items()}}))
    env.close()


if __name__ == "__main__":
    main()
    main(n=512)
