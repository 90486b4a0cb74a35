"""Env + PPO throughput (BASELINE C4 per GPU; SURVEY.md §8d "report env-only throughput, and
separately env+PPO"): the reference train.py flow with the reference agent config (horizon 32,
minibatch 32768, 10 mini-epochs, MLP 5 x 256), timed per epoch after warm-up epochs (the first
epoch runs eagerly, the second captures the rollout / update HIP graphs).

    python scripts/bench_train.py --num_envs 32768 --epochs 5 --warmup 2 [agent.params.config.<key>=<value> ...]

Prints one JSON line: env-steps/s including the PPO update and the play / update split."""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts", "reinforcement_learning", "rl_games"))


def measure(num_envs: int = 32768, epochs: int = 3, warmup: int = 2, level: int | None = None,
            log_root: str = "/tmp/bench_train_logs", verbose: bool = True, distributed: bool = False,
            multi_gpu_mode: str = "allgather", overrides: list[str] | None = None) -> dict:
    """num_envs per rank; with distributed=True (under torch.distributed.run) every rank trains with
    train.py --distributed --multi_gpu_mode <mode> and the result counts all ranks' env-steps over the
    slowest rank's time.  "allgather" (default) is the north star's exchange: one RCCL all-gather of the
    rollout tensors at the PPO boundary, identical replicated updates; "allreduce" is rl_games' own
    (per-rank minibatches, averaged gradients)."""
    import torch
    import torch.distributed as dist

    import train
    from allsteps_isaaclab_amd.learning import a2c_continuous as A

    samples = []
    orig = A.A2CAgent.train_epoch

    def timed(self):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = orig(self)
        torch.cuda.synchronize()
        samples.append((time.perf_counter() - t0, out[1], out[2]))
        if verbose:
            print(json.dumps({"epoch": self.epoch_num, "s": round(samples[-1][0], 4), "play_s": round(out[1], 4),
                              "update_s": round(out[2], 4)}), flush=True)
        return out

    A.A2CAgent.train_epoch = timed
    try:
        argv = ["--task", "Allsteps-v0", "--headless", "--num_envs", str(num_envs), "--max_iterations",
                str(epochs + warmup), "--seed", "42", "--log_root", log_root]
        if level is not None:
            argv += ["--stone_level", str(level)]
        if distributed:
            argv += ["--distributed", "--multi_gpu_mode", multi_gpu_mode]
        argv += list(overrides or [])
        if verbose:
            runner, _ = train.main(argv)
        else:  # keep stdout to the caller's single JSON line
            import contextlib
            import io

            with contextlib.redirect_stdout(io.StringIO()):
                runner, _ = train.main(argv)
    finally:
        A.A2CAgent.train_epoch = orig
    agent = runner.agent
    t = samples[warmup:]
    world = dist.get_world_size() if distributed and dist.is_initialized() else 1
    frames = agent.horizon_length * num_envs * world * len(t)
    wall = sum(x[0] for x in t)
    if world > 1:  # the slowest rank's time
        dev = agent.device if dist.get_backend() == "nccl" else "cpu"
        w = torch.tensor([wall], dtype=torch.float64, device=dev)
        dist.all_reduce(w, op=dist.ReduceOp.MAX)
        wall = float(w.item())
    return {
        "metric": "env-steps/sec incl. PPO update (rl_games agent config), Allsteps-v0",
        "value": round(frames / wall, 1), "unit": "env-steps/s", "n_gpus": world, "num_envs": num_envs,
        "global_envs": num_envs * world, "multi_gpu_mode": getattr(agent, "multi_gpu_mode", None) if world > 1 else None,
        "epochs": len(t), "horizon": agent.horizon_length, "minibatch": agent.minibatch_size,
        "mini_epochs": agent.mini_epochs_num, "s_per_epoch": round(wall / len(t), 4),
        "play_s": round(sum(x[1] for x in t) / len(t), 4), "update_s": round(sum(x[2] for x in t) / len(t), 4),
        "mixed_precision": agent.mixed_precision, "grad_scaler": agent.scaler_state is not None,
        "hip_graphs": agent._play_graphs is not None,
        "precision": (("fp16" if agent.mixed_precision_dtype == torch.float16 else "bf16") if agent.mixed_precision
                      else "fp32") + " MLP trunk and heads on MFMA (fp32 accumulate; heads rounded to 16 bit as under autocast), fp32 losses / Adam / normalisers, "
                     "device-side GradScaler (rl_games mixed_precision=True: fp16 autocast; DESIGN.md §7)",
        "data": "synthetic (random-init policy, reference reset distribution)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--num_envs", type=int, default=32768)
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--level", type=int, default=None, help="initial stone curriculum level (C3: 9)")
    ap.add_argument("--distributed", action="store_true", help="one rank per GPU under torch.distributed.run")
    ap.add_argument("--multi_gpu_mode", choices=("allgather", "allreduce"), default="allgather",
                    help="--distributed exchange: RCCL all-gather of rollouts (north star) or gradient all-reduce")
    ap.add_argument("--quiet", action="store_true", help="only the result line (rank 0)")
    # the rest of the command line: hydra-style overrides that train.py applies (agent.<path>=<value>,
    # env.<path>=<value>), e.g. agent.params.config.mixed_precision_dtype=bfloat16
    args, extra = ap.parse_known_args()
    bad = [a for a in extra if "=" not in a or a.startswith("-")]
    if bad:
        ap.error(f"unrecognized arguments: {' '.join(bad)}")
    out = measure(args.num_envs, args.epochs, args.warmup, args.level, verbose=not args.quiet,
                  distributed=args.distributed, multi_gpu_mode=args.multi_gpu_mode, overrides=extra)
    import torch.distributed as dist

    if not (dist.is_initialized() and dist.get_rank() != 0):
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
