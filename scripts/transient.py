"""Per-step cost of env.step from reset (DESIGN §3 "The driver's window"): HIP events (torch's current
stream, which the env launches on) around every env.step of one run from env.reset(), U(-1, 1)
actions as bench.py draws them; prints the mean step time per window of step indices, the resets per
step, and where the driver's `--steps 20 --warmup 5` window (steps 5..24) sits against the
steady state.

    python scripts/transient.py [num_envs] [steps] [level]
"""

from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1200
    level = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    from allsteps_isaaclab_amd.envs.allsteps_env import AllstepsEnv
    from allsteps_isaaclab_amd.envs.allsteps_env_cfg import AllstepsEnvCfg

    dev = torch.device("cuda:0")
    cfg = AllstepsEnvCfg()
    cfg.scene.num_envs = n
    cfg.sim.device = str(dev)
    cfg.seed = 42
    cfg.initial_stone_curriculum = level
    env = AllstepsEnv(cfg)
    gen = torch.Generator(device=dev).manual_seed(1000)
    actions = torch.rand(steps, n, 21, device=dev, generator=gen) * 2.0 - 1.0
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    resets = torch.zeros(steps, dtype=torch.int32, device=dev)
    env.reset()
    torch.cuda.synchronize()
    for t in range(steps):
        ev[t][0].record()
        _, _, term, trunc, _ = env.step(actions[t])
        ev[t][1].record()
        resets[t] = (term | trunc).sum()
    torch.cuda.synchronize()
    ms = [a.elapsed_time(b) for a, b in ev]
    rs = resets.cpu().tolist()
    edges = [0, 5, 10, 15, 25, 50, 100, 200, 400, 800, steps]
    rows = []
    for a, b in zip(edges[:-1], edges[1:]):
        if a >= steps:
            break
        b = min(b, steps)
        rows.append({"steps": f"{a}..{b - 1}", "ms_per_step": round(sum(ms[a:b]) / (b - a), 5),
                     "resets_per_step": round(sum(rs[a:b]) / (b - a), 1)})
    drv = sum(ms[5:25]) / 20
    steady = sum(ms[steps // 2:]) / (steps - steps // 2)
    out = {"num_envs": n, "level": level, "windows": rows, "driver_window_5_24_ms": round(drv, 5),
           "steady_second_half_ms": round(steady, 5), "driver_over_steady": round(drv / steady, 4)}
    print(json.dumps(out), flush=True)
    env.close()


if __name__ == "__main__":
    main()
