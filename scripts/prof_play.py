"""Rollout-only timing (play_steps with rollout graphs) at N envs: wall per step, for rocprofv3."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts", "reinforcement_learning", "rl_games"))
import torch  # noqa: E402

import train  # noqa: E402
from allsteps_isaaclab_amd.learning import a2c_continuous as A  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
captured = {}
orig_train = A.A2CAgent.train


def only_play(self):
    self.init_tensors()
    self.obs = self.env_reset()
    for ep in range(6):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        self.play_steps()
        torch.cuda.synchronize()
        print(f"play epoch {ep}: {(time.perf_counter() - t0) * 1e3 / self.horizon_length:.3f} ms/step", flush=True)
    return 0, 0


A.A2CAgent.train = only_play
train.main(["--task", "Allsteps-v0", "--num_envs", str(N), "--max_iterations", "1", "--log_root", "/tmp/pp"])
