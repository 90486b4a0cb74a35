"""Env + PPO throughput (BASELINE C4 per GPU; SURVEY.md §8d "report env-only throughput, and
separately env+PPO"): the reference train.py flow with the reference agent config (horizon 32,
minibatch 32768, 10 mini-epochs, MLP 5 x 256), timed per epoch after warm-up epochs.

    python scripts/bench_train.py --num_envs 32768 --epochs 5 --warmup 2

Prints one JSON line: env-steps/s including the PPO update, the play / update split, and the
env-only step rate inside the rollout (rl_games' "fps step")."""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts", "reinforcement_learning", "rl_games"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--num_envs", type=int, default=32768)
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--level", type=int, default=None, help="initial stone curriculum level (C3: 9)")
    args = ap.parse_args()
    import torch

    import train
    from allsteps_isaaclab_amd.learning import a2c_continuous as A

    samples = []
    orig = A.A2CAgent.train_epoch

    def timed(self):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = orig(self)
        torch.cuda.synchronize()
        samples.append((time.perf_counter() - t0, out[0], out[1], out[2]))
        print(json.dumps({"epoch": self.epoch_num, "s": round(samples[-1][0], 4), "play_s": round(out[1], 4),
                          "update_s": round(out[2], 4)}), flush=True)
        return out

    A.A2CAgent.train_epoch = timed
    argv = ["--task", "Allsteps-v0", "--headless", "--num_envs", str(args.num_envs), "--max_iterations",
            str(args.epochs + args.warmup), "--seed", "42", "--log_root", "/tmp/bench_train_logs"]
    if args.level is not None:
        argv += ["--stone_level", str(args.level)]
    runner, _ = train.main(argv)
    agent = runner.agent
    t = samples[args.warmup:]
    frames = agent.batch_size * len(t)
    wall = sum(x[0] for x in t)
    print(json.dumps({
        "metric": "env-steps/sec incl. PPO update (rl_games agent config), Allsteps-v0",
        "value": round(frames / wall, 1), "unit": "env-steps/s", "n_gpus": 1, "num_envs": args.num_envs,
        "epochs": len(t), "horizon": agent.horizon_length, "minibatch": agent.minibatch_size,
        "mini_epochs": agent.mini_epochs_num, "s_per_epoch": round(wall / len(t), 4),
        "play_s": round(sum(x[2] for x in t) / len(t), 4), "update_s": round(sum(x[3] for x in t) / len(t), 4),
        "env_step_s_in_play": round(sum(x[1] for x in t) / len(t), 4),
        "mixed_precision": agent.mixed_precision, "data": "synthetic (random-init policy)"}))


if __name__ == "__main__":
    main()
