"""BASELINE C5 throughput: the quadruped (model/anymal_c.xml) on the stones with its task, 1 GPU.

    python scripts/bench_quadruped.py [--num_envs 16384] [--steps 500] [--warmup 100]

A step = ``AnymalCStonesEnv.step`` (``Allsteps-AnymalC-v0``, ANYmal-C's sim settings: dt 1/200, friction
1.0, max depenetration velocity 1.0) = as_quad_step: 4 substeps of k_step<18> for every env with the DC
motor actuator evaluated in each substep (position targets default + 0.5 a), then k_quad (target
stones, potentials, rewards, dones, in-kernel resets, the 64-float observation).  Actions: U(-1, 1),
fresh every step (pre-drawn on the device).  Episodes end and reset inside the timed region.  Prints
one JSON line.
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


def measure(num_envs: int = 16384, steps: int = 500, warmup: int = 100, device: str = "cuda:0") -> dict:
    from allsteps_isaaclab_amd import registry

    cfg = registry.load_cfg_from_registry("Allsteps-AnymalC-v0", "env_cfg_entry_point")
    cfg.scene.num_envs = num_envs
    cfg.sim.device = device
    env = registry.make("Allsteps-AnymalC-v0", cfg=cfg)
    env.reset()
    gen = torch.Generator(device=device).manual_seed(7)
    acts = torch.rand(steps + 20, num_envs, 12, device=device, generator=gen) * 2 - 1
    # (100 warm-up steps: a cold box's first ~20 steps run at well under half the steady rate)
    for t in range(warmup):
        env.step(acts[steps + t % 20])
    torch.cuda.synchronize(device)
    # resets counted on every 10th step only: the count's own kernels (or / sum / add, ~4 us each) would
    # otherwise be a few per cent of the step they measure
    dones = torch.zeros((), dtype=torch.int64, device=device)
    sampled = 0
    t0 = time.perf_counter()
    for t in range(steps):
        _, _, term, trunc, _ = env.step(acts[t])
        if t % 10 == 0:
            dones += (term | trunc).sum()
            sampled += 1
    torch.cuda.synchronize(device)
    el = time.perf_counter() - t0
    env.close()
    return {"metric": "env-steps/sec, quadruped (ANYmal-C approximation) stepping-stone task (DC motor, 4 foot "
                      "sensors, resets in the loop)",
            "task": "Allsteps-AnymalC-v0",
            "config": {"env_cfg": "AnymalCStonesEnvCfg", "dt": cfg.sim.dt, "decimation": cfg.decimation,
                       "friction": cfg.sim.friction, "friction_combine": "multiply (1.0 x 1.0)",
                       "max_depenetration_velocity": cfg.sim.max_depenetration_velocity,
                       "soft_joint_pos_limit_factor": cfg.robot.soft_joint_pos_limit_factor},
            "value": round(num_envs * steps / el, 1), "unit": "env-steps/s", "n_gpus": 1, "num_envs": num_envs,
            "steps": steps, "ms_per_step": round(el / steps * 1e3, 4), "dof": 12, "kernels": "k_step<18> + k_quad",
            "resets_per_step": round(float(dones.item()) / max(sampled, 1), 1),
            "data": "synthetic (U(-1,1) actions, level-0 stones, stand-pose resets)"}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--num_envs", type=int, default=16384)
    p.add_argument("--steps", type=int, default=500)
    p.add_argument("--warmup", type=int, default=100)
    a = p.parse_args()
    print(json.dumps(measure(a.num_envs, a.steps, a.warmup)), flush=True)


if __name__ == "__main__":
    main()
