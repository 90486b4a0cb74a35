import os, sys, time, json
sys.path.insert(0, os.getcwd())
import torch
from allsteps_isaaclab_amd.envs.allsteps_env import AllstepsEnv
from allsteps_isaaclab_amd.envs.allsteps_env_cfg import AllstepsEnvCfg
cfg = AllstepsEnvCfg(); cfg.scene.num_envs = 4096; cfg.sim.device = "cuda:0"; cfg.seed = 42
env = AllstepsEnv(cfg)
a = torch.rand(1100, 4096, 21, device="cuda:0") * 2 - 1
env.reset(); torch.cuda.synchronize()
host = []
for t in range(1100):
    t0 = time.perf_counter(); env.step(a[t]); host.append(time.perf_counter() - t0)
torch.cuda.synchronize()
# fixed overhead: an empty timed region
ov = []
for _ in range(20):
    torch.cuda.synchronize(); t0 = time.perf_counter(); torch.cuda.synchronize(); ov.append(time.perf_counter() - t0)
one = []
for _ in range(20):
    torch.cuda.synchronize(); t0 = time.perf_counter(); env.step(a[0]); torch.cuda.synchronize(); one.append(time.perf_counter() - t0)
print(json.dumps({"host_us_steps_0_25": round(1e6 * sum(host[:25]) / 25, 1), "host_us_steady": round(1e6 * sum(host[100:]) / 1000, 1),
                  "empty_region_us": round(1e6 * sorted(ov)[10], 1), "one_step_synced_us": round(1e6 * sorted(one)[10], 1)}))
