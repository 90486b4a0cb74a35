"""Diagnostic: per-phase cycles of the C5 quadruped's k_step<18> (scripts/stamps.py records).

    python scripts/stamps_c5.py [num_envs] [steps]

One JSON line: bench.py's `roofline.latency` object (mean / slowest wave, their phases) for
`Allsteps-AnymalC-v0` under U(-1, 1) actions after a warm-up second, as `scripts/bench_quadruped.py`
drives it.  The stamps add a few s_memtime reads per phase.
"""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import torch  # noqa: E402

import stamps  # noqa: E402


def main(n: int = 16384, steps: int = 20, warm: int = 50):
    from allsteps_isaaclab_amd import registry

    cfg = registry.load_cfg_from_registry("Allsteps-AnymalC-v0", "env_cfg_entry_point")
    cfg.scene.num_envs = n
    cfg.sim.device = "cuda:0"
    env = registry.make("Allsteps-AnymalC-v0", cfg=cfg)
    env.reset()
    gen = torch.Generator(device="cuda:0").manual_seed(7)
    acts = torch.rand(steps + warm, n, 12, device="cuda:0", generator=gen) * 2 - 1
    for t in range(warm):
        env.step(acts[t])
    torch.cuda.synchronize()
    R = stamps.wave_records(env.unwrapped if hasattr(env, "unwrapped") else env, acts[warm:])
    print(json.dumps({"task": "Allsteps-AnymalC-v0", "num_envs": n, "launches": steps,
                      "latency": stamps.latency_summary(R)}), flush=True)
    env.close()


if __name__ == "__main__":
    a = [int(x) for x in sys.argv[1:3]]
    main(*a)
