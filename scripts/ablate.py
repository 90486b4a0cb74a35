"""Runtime ablation of k_step: time the kernel (HIP events per launch) under knobs that switch
phases off without rebuilding: PGS sweeps, contacts (stones moved out of reach), substeps."""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from allsteps_isaaclab_amd.envs.allsteps_env import AllstepsEnv  # noqa: E402
from allsteps_isaaclab_amd.envs.allsteps_env_cfg import AllstepsEnvCfg  # noqa: E402


def run(name, n=4096, steps=100, pgs=4, decimation=4, far=False, level=0):
    cfg = AllstepsEnvCfg()
    cfg.scene.num_envs = n
    cfg.sim.device = "cuda:0"
    cfg.sim.solver_position_iteration_count = pgs
    cfg.decimation = decimation
    cfg.initial_stone_curriculum = level
    env = AllstepsEnv(cfg)
    if far:
        env.state["stones"][2::3] -= 100.0
    env.reset()
    gen = torch.Generator(device="cuda").manual_seed(0)
    acts = torch.rand(steps + 10, n, 21, device="cuda", generator=gen) * 2 - 1
    for t in range(10):
        env.step(acts[t])
    torch.cuda.synchronize()
    env._native.profile(steps)
    for t in range(steps):
        env.step(acts[10 + t])
    k, o, cnt = env._native.profile_read()
    env.close()
    r = {"case": name, "n": n, "k_step_ms": round(k / cnt, 4), "k_obs_ms": round(o / cnt, 4)}
    print(json.dumps(r), flush=True)
    return r


if __name__ == "__main__":
    run("full")
    run("pgs0", pgs=0)
    run("no_contacts", far=True)
    run("no_contacts_pgs0", far=True, pgs=0)
    run("substeps1", decimation=1)
    run("n1024", n=1024)
    run("n16384", n=16384)
    run("n32768_L9", n=32768, level=9)
