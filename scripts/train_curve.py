"""Learning-curve run of the full stack (native env + PPO trainer) on one GPU: the reference agent
config, N envs, E epochs; prints per-epoch mean episode reward / length / curriculum target index as
JSON lines (the evidence that physics + task + trainer learn together).

    python scripts/train_curve.py [num_envs] [epochs] [every] [task] [env.<k>=<v> | agent.<k>=<v> ...]
    (task: Allsteps-v0 or Allsteps-AnymalC-v0, the C5 quadruped behind the same env surface; the seed is 42
    unless CURVE_SEED is set)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts", "reinforcement_learning", "rl_games"))
import torch  # noqa: E402

import train  # noqa: E402
from allsteps_isaaclab_amd.learning import a2c_continuous as A  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
E = int(sys.argv[2]) if len(sys.argv) > 2 else 300
EVERY = int(sys.argv[3]) if len(sys.argv) > 3 else 10
TASK = sys.argv[4] if len(sys.argv) > 4 else "Allsteps-v0"
orig = A.A2CAgent.train_epoch
t0 = time.perf_counter()


def logged(self):
    out = orig(self)
    if self.epoch_num % EVERY == 0 or self.epoch_num == 1:
        uw = self._uw if getattr(self, "_uw", None) is not None else self.vec_env.env.unwrapped
        ti = uw.curr_target_index if hasattr(uw, "curr_target_index") else uw.target_index
        rec = {"epoch": self.epoch_num, "frames": self.frame + self.curr_frames, "wall_s": round(time.perf_counter() - t0, 2),
               "mean_reward": round(float(self.game_rewards.mean.reshape(-1)[0]), 3),
               "mean_length": round(float(self.game_lengths.mean.reshape(-1)[0]), 1),
               "mean_target_index": round(float(ti.float().mean()), 3),
               "max_target_index": int(ti.max()),
               "curriculum": int(uw.state["curriculum"][0]), "lr": float(self.lr), "kl": round(float(out[4]["kl"]), 5)}
        print(json.dumps(rec), flush=True)
    return out


A.A2CAgent.train_epoch = logged
with open(os.devnull, "w") as dn:
    import contextlib

    with contextlib.redirect_stdout(sys.stderr):
        pass
# past the four positional arguments: hydra-style overrides (env.<path>=<value>, agent.<path>=<value>)
train.main(["--task", TASK, "--num_envs", str(N), "--max_iterations", str(E), "--seed", os.environ.get("CURVE_SEED", "42"),
            "--log_root", "/tmp/curve_logs", *sys.argv[5:]])
