"""Is the driver's window (bench.py --steps 20 --warmup 5: steps 5..24 after reset) slower because of
the physics of the landing or because the GPU is still clocking up?  Times the same 20-step window
three ways in one process (DESIGN §3 "The driver's window"): (a) as bench.py does it, (b) after 300 ms
of unrelated GPU load (matmuls) right before the warm-up, (c) the window steps 500..519 instead.
Prints ms per step of each, best of 3 repetitions (a fresh env.reset() each)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from allsteps_isaaclab_amd.envs.allsteps_env import AllstepsEnv  # noqa: E402
from allsteps_isaaclab_amd.envs.allsteps_env_cfg import AllstepsEnvCfg  # noqa: E402

cfg = AllstepsEnvCfg()
cfg.scene.num_envs = 4096
cfg.sim.device = "cuda:0"
cfg.seed = 42
env = AllstepsEnv(cfg)
acts = torch.rand(525, 4096, 21, device="cuda:0", generator=torch.Generator(device="cuda:0").manual_seed(1000)) * 2 - 1
m = torch.randn(4096, 4096, device="cuda:0")


def window(warm: int, heat: bool) -> float:
    env.set_state({k: v for k, v in s0.items()})
    env.reset()
    torch.cuda.synchronize()
    if heat:
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.3:
            for _ in range(8):
                m @ m
            torch.cuda.synchronize()
    for t in range(warm):
        env.step(acts[t % 500])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(20):
        env.step(acts[warm + t])
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / 20 * 1e3


env.reset()
s0 = env.get_state()
time.sleep(1.0)  # let the GPU idle down as after env construction
out = {}
for name, warm, heat in (("a_driver_window", 5, False), ("b_preheated", 5, True), ("c_steps_500", 500, False)):
    r = []
    for _ in range(3):
        time.sleep(0.5)
        r.append(window(warm, heat))
    out[name] = round(min(r), 5)
print(json.dumps(out))
