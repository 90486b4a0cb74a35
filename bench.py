"""Allsteps-v0 step throughput on MI355X: env-steps/s (whole job), 4096 envs per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--num-envs 4096] [--level 0]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

Protocol (after scripts/benchmarks/benchmark_non_rl.py:155-179): --preheat-ms of untimed
env steps (GPU clocks to steady state), env.reset(), W untimed warm-up steps, then K timed
``env.step`` calls bracketed by a barrier + device synchronize on both sides;
fresh U(-1, 1) actions every step (pre-drawn on the device before the timed region); seed 42 + rank;
episodes terminate and reset naturally inside the timed region.  Envs are sharded per rank (weak
scaling, no collective in the step).  value = all ranks' env-steps / max-over-ranks wall time.

Extra objects on the JSON line:
  roofline     -- k_step (the dominant kernel): algorithmic bytes per launch / its HIP-event-timed
                  average duration over a replay of the timed window (>= 200 sampled launches, on the
                  env's stream; kernel_times), vs 8 TB/s HBM;
                  `latency`: per-wave cycle records of the timed window's first (up to 20) launches,
                  replayed (mean / slowest wave vs the launch span, the slowest wave's phases:
                  scripts/stamps.py).
  cpu_baseline -- rank 0, N = 1: the CPU oracle (oracle/, a port of the same step) timed on this
                  host's cores on a bounded sample.
  train        -- every rank (BASELINE C4, SURVEY §8d "env+PPO separately"): env-steps/s of the PPO
                  trainer over all ranks (scripts/bench_train.py: reference agent config, 32768 envs
                  per rank, horizon 32, 10 mini-epochs; N > 1: the --distributed path), one child
                  process per rank with a time limit (train_leg) -- reported beside `value`, never as
                  `value`.
  c5           -- rank 0, N = 1 (BASELINE C5): the quadruped (model/anymal_c.xml) stepping-stone task
                  (DC motor actuator in every substep, four foot sensors, task epilogue and resets in
                  the timed loop), 16384 envs (scripts/bench_quadruped.py) -- beside `value`.
"""

from __future__ import annotations

import argparse
import datetime
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
# BASELINE.json "metric" (the driver compares the line against it)
BASELINE_METRIC = "env-steps/sec (whole node), Allsteps-v0 at 4096 envs, 1/2/4/8 MI355X"

# Algorithmic bytes per env per launch: every state byte the kernel must read
# or write once, from the SoA layout of include/allsteps.h.
K_STEP_READ = 84 + 52 + 168 + 240 + 8 + 24 + 8 + 8 + 4    # actions, root, q/qd, stones, masks, ints, pots, contact, episode
K_STEP_WRITE = 52 + 168 + 36 + 8 + 24 + 8 + 8 + 4 + 6 + 236  # root, q/qd, body_pos, masks, ints, pots, contact, episode, rew/term/trunc, obs row
K_STEP_BYTES = K_STEP_READ + K_STEP_WRITE


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=1000)
    p.add_argument("--warmup", type=int, default=50)
    p.add_argument("--num-envs", type=int, default=4096)
    p.add_argument("--level", type=int, default=0, help="stone curriculum level (C3: 9)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=None,
                   help="oracle OpenMP threads (default: OMP_NUM_THREADS, else nproc; BASELINE.md §3)")
    p.add_argument("--no-train", action="store_true", help="skip the env+PPO trainer measurement")
    p.add_argument("--train-envs", type=int, default=32768)
    p.add_argument("--multi-gpu-mode", dest="multi_gpu_mode", choices=("allgather", "allreduce"), default="allreduce",
                   help="N > 1 train leg: RCCL gradient all-reduce per minibatch (rl_games --distributed, default: "
                        "it scales, DESIGN.md §6) or the north star's all-gather of rollouts (every rank then "
                        "runs the whole update on W x the data)")
    p.add_argument("--no-c5", action="store_true", help="skip the quadruped (BASELINE C5) task measurement")
    p.add_argument("--preheat-ms", type=float, default=250.0,
                   help="untimed env steps before env.reset() that bring the GPU to its steady clocks (DESIGN.md §3 "
                        "'The driver's window'); 0 disables")
    return p.parse_args()


def pmc_record(num_envs: int) -> dict:
    """The committed rocprofv3 PMC figures of k_step (scripts/profile.sh writes
    profiles/traffic_k_step.json): HBM bytes per launch (FETCH_SIZE x 2 + WRITE_SIZE) and the VALU
    issue fraction (SQ_INSTS_VALU vs the SIMDs' cycles); empty when absent or for another size."""
    try:
        with open(os.path.join(ROOT, "profiles", "traffic_k_step.json")) as f:
            t = json.load(f)
        return t if int(t["num_envs"]) == num_envs else {}
    except (OSError, KeyError, ValueError):
        return {}


def kernel_times(ms_per_step: float, k_ms: float, o_ms: float, launches: int) -> dict:
    """Per-launch durations (ms) of the step's two kernels over the timed window.

    `k_ms` / `o_ms` are the summed HIP-event spans of k_step / k_obs over `launches` launches of a
    replay of the timed window (same start state, same actions: the run is deterministic, so the
    replay launches the very kernels the timed loop launched), recorded on the env's stream.  The
    roofline's duration is the k_step event average (`k_step_ms`).  The events span each kernel plus
    its own dispatch, so event k_step + event k_obs is checked against the timed loop's wall clock
    (`event_sum_over_wall`, an independent measurement: events_consistent); `k_step_period_ms` = wall
    ms_per_step - event k_obs is the step period left to k_step (kernel + launch gap), kept beside it."""
    n = max(launches, 1)
    k_ev, o_ev = k_ms / n, o_ms / n
    return {"k_step_ms": round(k_ev, 5), "k_obs_ms": round(o_ev, 5), "sampled_launches": launches,
            "k_step_period_ms": round(ms_per_step - o_ev, 5),
            "event_sum_over_wall": round((k_ev + o_ev) / ms_per_step, 4) if ms_per_step > 0 else None,
            "method": "HIP events on the env's stream around every k_step / k_obs launch of a replay of the "
                      "timed window (state restored to the window's start, same actions, repeated until >= 200 "
                      "launches are sampled; no events inside the timed loop itself); k_step_ms includes the "
                      "launch's dispatch"}


def events_consistent(t: dict, lo: float = 0.9, hi: float = 1.1) -> bool:
    """The event-timed kernels of the replay account for the timed loop's wall clock: their sum per
    step lies within [lo, hi] x ms_per_step (events over-read by their own dispatch, a few per cent;
    a replay that diverged from the timed window, or events that missed launches, fall outside)."""
    r = t.get("event_sum_over_wall")
    return r is not None and lo <= r <= hi


def measured_hbm_peak(device) -> float | None:
    """Achievable HBM GB/s of the in-tree STREAM-copy kernel (as_hbm_copy, 2 x 2 GiB buffers)."""
    from allsteps_isaaclab_amd import _native

    try:
        return round(_native.hbm_copy_bandwidth(device), 1)
    except Exception as e:  # reported, never fatal for the env metric
        print(f"bench: as_hbm_copy probe failed: {e}", file=sys.stderr)
        return None


def host_cpu() -> dict:
    """nproc (affinity), os.cpu_count(), the CPU model and socket count (lscpu's fields, from
    /proc/cpuinfo) of the host the CPU baseline runs on."""
    model, sockets = None, set()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                k, _, v = line.partition(":")
                k = k.strip()
                if k == "model name" and model is None:
                    model = v.strip()
                elif k == "physical id":
                    sockets.add(v.strip())
    except OSError:
        pass
    return {"nproc": len(os.sched_getaffinity(0)), "cpu_count": os.cpu_count(), "model": model,
            "sockets": len(sockets) or None}


def cpu_baseline(num_envs: int, level: int, threads: int | None, warm_steps: int = 50, samples: int = 3,
                 min_wall_s: float = 7.0, min_steps: int = 20, max_wall_s: float = 60.0) -> dict:
    """The oracle (CPU port of the same step) on the host cores, timed after `warm_steps` steps past the
    from-reset transient (the falling start), in `samples` back-to-back samples of at least `min_wall_s`
    of wall clock and `min_steps` steps each (at most `max_wall_s`): >= 21 s of CPU work in all.  The
    value is the median sample's rate; the spread (min, max) is reported beside it because the host's
    other tenants share these cores (benchmark_non_rl.py:155-179 times one long run; three samples
    make the noise visible instead).

    Threads: OMP_NUM_THREADS when set, else nproc.  On the GPU box OMP_NUM_THREADS is
    the job's CPU share per GPU (16) and is kept: nproc there counts every CPU of the host, which other
    jobs share, so more threads would measure contention, not the port."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle as O

    host = host_cpu()
    env_threads = os.environ.get("OMP_NUM_THREADS")
    if threads is None:
        threads = int(env_threads or host["nproc"])
    why = ("OMP_NUM_THREADS (the job's CPU share; nproc counts the whole shared host)" if env_threads
           else "nproc")
    O.build()
    orc = O.Oracle()
    n = num_envs
    st = orc.state(n)
    if level == 0:
        for k in range(20):
            st["stones"][3 * k + 0][:] = 0.75 * k
            st["stones"][3 * k + 2][:] = np.float32(k * 0.75) * np.cos(np.float32(np.pi / 2), dtype=np.float32)
    else:
        rng = np.random.default_rng(0)
        pos, _ = orc.footsteps(n, level, rng.uniform(0, 1, (5, n, 20)).astype(np.float32))
        st["stones"][:] = pos.reshape(n, 60).T
    orc.reset_all(st, seed=42)
    rng = np.random.default_rng(42)
    acts = [rng.uniform(-1, 1, (n, 21)).astype(np.float32) for _ in range(4)]
    for t in range(warm_steps):  # past the from-reset transient: envs fall, reset, walk at random
        orc.env_step(st, acts[t % 4], nthreads=threads)
    rates, total_steps, total_s, k = [], 0, 0.0, 0
    for _ in range(samples):
        steps, t0 = 0, time.perf_counter()
        while True:
            orc.env_step(st, acts[k % 4], nthreads=threads)
            steps += 1
            k += 1
            el = time.perf_counter() - t0
            if (el >= min_wall_s and steps >= min_steps) or el >= max_wall_s:
                break
        rates.append(n * steps / el)
        total_steps += steps
        total_s += el
    med = float(np.median(rates))
    return {"value": round(med, 1), "unit": "env-steps/s", "cores": threads, "kind": "port",
            "kind_detail": "bit-exact serial restatement of the HIP step (oracle/: the kernel's lane trees, "
                           "MFMA fmaf chains and two-partial sums restated serially, -ffp-contract=off), not a "
                           "tuned CPU simulator; the reference's PhysX CPU pipeline cannot run here",
            "samples": [round(r, 1) for r in rates], "spread": round((max(rates) - min(rates)) / med, 4),
            "threads_from": why, "host": host,
            "sample": f"oracle/ C port, {n} envs, {samples} samples, {total_steps} steps in {total_s:.2f} s wall "
                      f"(level {level}, U(-1,1) actions, timed after {warm_steps} warm-up steps), OpenMP {threads} "
                      f"threads; value = median sample, spread = (max - min) / median"}


def train_leg(args, world: int, rank: int, backend: str, device, timeout_s: float = 300.0) -> dict:
    """env + PPO (BASELINE C4) in a child process per rank (scripts/bench_train.py; at N ranks its own
    process group on a fresh port, the trainer's --distributed path with --multi_gpu_mode allreduce:
    one RCCL all-reduce of the [grads | kl] bucket per minibatch, rl_games' own multi_gpu exchange and
    the one that scales -- DESIGN.md §6 prices it against the north star's all-gather of rollouts,
    which replicates the whole update on every rank; --multi-gpu-mode allgather selects that).  A child that fails or stalls is killed after `timeout_s` and reported
    as an error: the env metric on the line never waits on the trainer's collectives."""
    import signal
    import socket
    import subprocess

    port = 0
    if rank == 0:
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
    if world > 1:  # every rank's child joins rank 0's port
        t = torch.tensor([port], dtype=torch.int64, device=device if backend == "nccl" else "cpu")
        dist.broadcast(t, 0)
        port = int(t.item())
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TORCHELASTIC_USE_AGENT_STORE="False",
               ALLSTEPS_DIST_TIMEOUT_S=str(int(timeout_s)))
    cmd = [sys.executable, os.path.join(ROOT, "scripts", "bench_train.py"), "--num_envs", str(args.train_envs),
           "--epochs", "2", "--warmup", "2", "--quiet"]
    if world > 1:  # north star: the RCCL all-gather of rollout tensors at the PPO boundary
        cmd += ["--distributed", "--multi_gpu_mode", args.multi_gpu_mode]
    p = subprocess.Popen(cmd, env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         start_new_session=True)
    try:
        out, err = p.communicate(timeout=timeout_s)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        p.communicate()
        return {"error": f"train child exceeded {timeout_s:.0f} s and was killed"}
    if p.returncode != 0:
        return {"error": f"train child exit {p.returncode}: {err.strip()[-600:]}"}
    if rank != 0:
        return {}
    try:
        return json.loads(out.strip().splitlines()[-1])
    except (IndexError, ValueError):
        return {"error": f"train child printed no result line: {out[-300:]} {err[-300:]}"}


def launcher_cmd(gpus: int, argv: list[str], port: int) -> list[str]:
    """The one-process-per-GPU launch of this script (the reference's multi-GPU recipe,
    docs/source/features/multi_gpu.rst:58, scripts/reinforcement_learning/rl_games/train.py:99-105):
    torch.distributed.run on one node, rendezvous on 127.0.0.1, the same bench arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(gpus),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]


def self_launch(gpus: int, argv: list[str]) -> int:
    """`python bench.py --gpus N` without a launcher: start torch.distributed.run as a CHILD process
    (never exec: this parent has made no HIP call, and stays that way) and relay its output and exit
    code.  The child's stdout is inherited, so rank 0's single JSON line is this command's line."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    p = subprocess.Popen(launcher_cmd(gpus, argv, port), env=env, cwd=ROOT)
    try:
        return p.wait()
    except KeyboardInterrupt:
        p.terminate()
        return p.wait()


def check_world(gpus: int, environ) -> tuple[int, str | None]:
    """(world, error): the process group size the ranks will form, and why this invocation must not
    run.  `--gpus` is the requested GPU count; under a launcher WORLD_SIZE must equal it, so a line
    can never report a different GPU count than the one asked for."""
    if gpus < 1:
        return 0, f"bench: --gpus must be >= 1 (got {gpus})"
    ws = environ.get("WORLD_SIZE")
    if ws is None:
        return gpus, None
    if int(ws) != gpus:
        return int(ws), (f"bench: WORLD_SIZE={ws} from the launcher but --gpus {gpus}; pass the same count to "
                         f"both (or run `python bench.py --gpus N` and let it launch the N ranks itself)")
    return gpus, None


def main():
    args = parse()
    world, err = check_world(args.gpus, os.environ)
    if err:
        print(err, file=sys.stderr, flush=True)
        sys.exit(2)
    if "WORLD_SIZE" not in os.environ and world > 1:
        sys.exit(self_launch(world, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; ALLSTEPS_DIST_BACKEND=gloo lets ranks share one GPU (the rehearsal in
    # tests/test_gpu_parity.py::test_bench_two_ranks_one_gpu), the default is RCCL ("nccl")
    backend = os.environ.get("ALLSTEPS_DIST_BACKEND", "nccl")
    if backend == "nccl" and local >= torch.cuda.device_count():  # device_count() makes no HIP call
        print(f"bench: rank {rank} needs GPU {local} but {torch.cuda.device_count()} are visible", file=sys.stderr,
              flush=True)
        sys.exit(2)
    device = torch.device(f"cuda:{local % max(torch.cuda.device_count(), 1) if backend == 'gloo' else local}")
    torch.cuda.set_device(device)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        timeout = datetime.timedelta(seconds=600)  # a stalled rank ends the job instead of hanging it
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device, timeout=timeout)
        else:
            dist.init_process_group(backend, timeout=timeout)

    from allsteps_isaaclab_amd.envs.allsteps_env import AllstepsEnv
    from allsteps_isaaclab_amd.envs.allsteps_env_cfg import AllstepsEnvCfg

    n = args.num_envs
    cfg = AllstepsEnvCfg()
    cfg.scene.num_envs = n
    cfg.sim.device = str(device)
    cfg.seed = 42 + rank
    cfg.initial_stone_curriculum = args.level
    env = AllstepsEnv(cfg, env_id_offset=rank * n)
    gen = torch.Generator(device=device).manual_seed(1000 + rank)
    K, W = args.steps, args.warmup
    actions = torch.rand(K + W, n, 21, device=device, generator=gen) * 2.0 - 1.0
    # GPU clocks: a timed region of a few ms right after construction would run while the GPU is still
    # clocking up from idle (measured: the 20-step driver window 0.1428 ms/step cold, 0.1317 warm,
    # scripts/window_clock.py).  Steps of the env itself, BEFORE env.reset(), keep the part afterwards --
    # reset, W warm-up steps, K timed steps -- exactly the protocol; they are reported on the line.
    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(device)

    # the protocol without the pre-heat, first, on the GPU as it comes (benchmark_non_rl.py:145-166 starts
    # timing right after env.reset()): reported beside the line's value, never as it
    cold = None
    if args.preheat_ms > 0:
        env.reset()
        for t in range(W):
            env.step(actions[K + t])
        env._native.profile(0)
        barrier()
        t0 = time.perf_counter()
        for t in range(K):
            env.step(actions[t])
        barrier()
        cold = time.perf_counter() - t0
        if world > 1:
            tt = torch.tensor([cold], device=device if backend == "nccl" else "cpu", dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            cold = float(tt.item())
    preheat_steps = 0
    if args.preheat_ms > 0:
        env.reset()
        t_heat = time.perf_counter()
        while time.perf_counter() - t_heat < args.preheat_ms / 1e3:
            for _ in range(10):
                env.step(actions[preheat_steps % (K + W)])
                preheat_steps += 1
            torch.cuda.synchronize(device)
    env.reset()
    for t in range(W):
        env.step(actions[K + t])
    torch.cuda.synchronize(device)
    env._native.profile(0)  # no HIP events inside the timed loop (each adds a launch gap to its step)
    s_start = env.get_state()  # the timed window's start state: replayed below for the kernel timings

    barrier()
    t0 = time.perf_counter()
    for t in range(K):
        env.step(actions[t])
    barrier()
    el = time.perf_counter() - t0
    s_end = env.get_state()
    resets = int(env.reset_buf.sum().item())
    # kernel durations over the timed window itself: replay it from its start state with HIP events
    # around every launch, as often as needed for >= 200 sampled launches whatever K is (the step is
    # deterministic, so the replay runs the timed loop's launches again; replay_exact checks that)
    reps = max(1, -(-200 // K))
    env._native.profile(reps * K)
    for _ in range(reps):
        env.set_state(s_start)
        for t in range(K):
            env.step(actions[t])
    torch.cuda.synchronize(device)
    k_ms, o_ms, launches = env._native.profile_read()
    env._native.profile(0)
    replay_exact = all(torch.equal(v, s_end[k]) for k, v in env.get_state().items())
    if world > 1:
        tt = torch.tensor([el], device=device if backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    # contacts the constraint budget cut in the timed window (as_step_counters word 3 per step), on
    # one more replay: the read synchronises every step, so it stays out of the timed and event loops
    env.set_state(s_start)
    dropped = 0
    for t in range(K):
        env.step(actions[t])
        dropped += env.dropped_contacts()
    # latency side of k_step: per-wave records of the timed window's first launches (replayed again)
    latency = None
    if rank == 0:
        sys.path.insert(0, os.path.join(ROOT, "scripts"))
        import stamps

        try:
            env.set_state(s_start)
            latency = stamps.latency_summary(stamps.wave_records(env, actions[:min(K, 20)]))
        except Exception as e:  # reported, never fatal for the env metric
            latency = {"error": f"{type(e).__name__}: {e}"}

    if rank == 0:
        value = n * world * K / el
        t = kernel_times(el / K * 1e3, k_ms, o_ms, launches)
        t["replay_exact"] = replay_exact
        t["events_consistent"] = events_consistent(t)
        achieved = K_STEP_BYTES * n / (t["k_step_ms"] / 1e3) / 1e9
        pmc = pmc_record(n)
        line = {
            "metric": BASELINE_METRIC,
            "value": round(value, 1),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": round(el / K * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (U(-1,1) actions, reference reset distribution, natural resets)",
            "config": {
                "workload": f"Allsteps-v0 biped walker, {n} envs/GPU, stone curriculum level {args.level}, "
                            f"decimation 4 x dt 1/240",
                "num_envs_per_gpu": n,
                "global_envs": n * world,
                "parallelism": f"dp{world} (env shards, no collective in step)",
            },
            "kernels_ms": t,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "duration_ms": t["k_step_ms"], "duration_method": t["method"],
                         "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": pmc.get("traffic_bytes_per_launch"),
                         "traffic_unit": "bytes per launch (rocprofv3 PMC, profiles/traffic_k_step.json)",
                         "kernel": "k_step", "bytes_per_env": K_STEP_BYTES,
                         "peak_measured": measured_hbm_peak(device),
                         "peak_measured_method": "in-tree STREAM copy (as_hbm_copy), read + write GB/s",
                         "valu_issue_frac": pmc.get("valu_issue_frac"),
                         # latency-bound kernel: the launch lasts as long as its slowest wave
                         "latency": latency},
            "cpu_baseline": None,
            "resets_last_step": resets,
            # PhysX keeps every contact (simulation_cfg.py:110); this build's 30-row budget cuts these
            "gpu_preheat": {"ms": args.preheat_ms, "env_steps": preheat_steps,
                            "what": "untimed env steps before env.reset() (GPU clocks to steady state); then reset, "
                                    "W warm-up steps, K timed steps"},
            "no_preheat": None if cold is None else {
                "value": round(n * world * K / cold, 1), "ms_per_step": round(cold / K * 1e3, 4),
                "what": "the same protocol (reset, W warm-up steps, K timed steps, same actions) run first, before "
                        "the pre-heat, on the GPU as it comes: the reference protocol's number "
                        "(benchmark_non_rl.py:145-166); beside `value`, never as it"},
            "contacts_dropped": {"total": dropped, "per_step": round(dropped / K, 2),
                                 "per_env_step": round(dropped / (K * n), 6),
                                 "method": "as_step_counters word 3 summed over the timed window's K steps "
                                           "(replayed from its start state): contacts the narrowphase found "
                                           "beyond the 10-contact / 30-row cap, all envs and substeps"},
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(n, args.level, args.cpu_threads)
    env.close()
    del env, actions
    torch.cuda.empty_cache()
    if not args.no_train:
        train = train_leg(args, world, rank, backend, device)
        if rank == 0:
            line["train"] = train
        elif "error" in train:
            print(f"bench rank {rank}: train leg failed: {train['error']}", file=sys.stderr, flush=True)
        if world > 1:  # both exchange modes on the line: the other one beside the default
            other = "allgather" if args.multi_gpu_mode == "allreduce" else "allreduce"
            train2 = train_leg(argparse.Namespace(**{**vars(args), "multi_gpu_mode": other}), world, rank, backend,
                               device)
            if rank == 0:
                line["train_" + other] = train2
    if rank == 0:
        if world == 1 and not args.no_c5:
            sys.path.insert(0, os.path.join(ROOT, "scripts"))
            import bench_quadruped

            try:
                line["c5"] = bench_quadruped.measure(16384, steps=300, warmup=100, device=str(device))
            except Exception as e:  # reported, never fatal for the env metric
                line["c5"] = {"error": f"{type(e).__name__}: {e}"}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
