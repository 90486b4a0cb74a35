"""BASELINE C5 throughput: the quadruped (model/anymal_c.xml) on the stones, physics only, 1 GPU.

    python scripts/bench_quadruped.py [--num_envs 16384] [--steps 500] [--warmup 20]

A step = 4 substeps of k_step<18> for every env (as_physics_step) under a joint PD on the ANYmal
stance plus fresh U(-0.3, 0.3) perturbation actions (pre-drawn on the device); the PD's few torch
elementwise ops are inside the timed region.  No task / resets (the reference has no Allsteps task
for ANYmal), so this is the physics half of C5 only.  Prints one JSON line.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def measure(num_envs: int = 16384, steps: int = 500, warmup: int = 20, device: str = "cuda:0") -> dict:
    from allsteps_isaaclab_amd.envs.quadruped import QuadrupedStonesEnv

    env = QuadrupedStonesEnv(num_envs, device)
    gen = torch.Generator(device=device).manual_seed(7)
    noise = (torch.rand(steps + warmup, num_envs, 12, device=device, generator=gen) * 2 - 1) * 0.3
    for t in range(warmup):
        env.step(env.stand_actions() + noise[steps + t])
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for t in range(steps):
        env.step(env.stand_actions() + noise[t])
    torch.cuda.synchronize(device)
    el = time.perf_counter() - t0
    standing = float((env.root_pos[:, 2] > 0.5).float().mean())
    env.close()
    return {"metric": "env-steps/sec, quadruped (ANYmal-C approximation) on ALLSTEPS stones, physics only",
            "value": round(num_envs * steps / el, 1), "unit": "env-steps/s", "n_gpus": 1, "num_envs": num_envs,
            "steps": steps, "ms_per_step": round(el / steps * 1e3, 4), "dof": 12, "kernel": "k_step<18>",
            "standing_fraction_end": round(standing, 4),
            "data": "synthetic (PD stance + U(-0.3,0.3) perturbations, level-0 stones)"}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--num_envs", type=int, default=16384)
    p.add_argument("--steps", type=int, default=500)
    p.add_argument("--warmup", type=int, default=20)
    a = p.parse_args()
    print(json.dumps(measure(a.num_envs, a.steps, a.warmup)), flush=True)


if __name__ == "__main__":
    main()
