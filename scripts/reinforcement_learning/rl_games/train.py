"""Train Allsteps-v0 with the rl_games-semantics PPO agent (reference: scripts/reinforcement_learning/rl_games/train.py).

Same CLI and the same steps as the reference script (train.py:76-178): load the env / agent configs
from the task registry, apply the CLI overrides, under ``--distributed`` offset the seed by the global
rank and put env + agent on ``cuda:<local_rank>`` with ``multi_gpu: True``, wrap the env in
``RlGamesVecEnvWrapper``, register it as ``rlgpu``, build the ``Runner`` with the mirror agent and
train.  Kit / app-launcher flags (``--headless`` ...) are accepted and ignored (there is no simulator
app); ``--video`` is not supported (no renderer).

    python scripts/reinforcement_learning/rl_games/train.py --task Allsteps-v0 --headless
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
        scripts/reinforcement_learning/rl_games/train.py --task Allsteps-v0 --headless --distributed
"""

from __future__ import annotations

import argparse
import dataclasses
import math
import os
import random
import sys
from datetime import datetime

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, ROOT)


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="Train an RL agent with RL-Games.")
    p.add_argument("--video", action="store_true", default=False)
    p.add_argument("--video_length", type=int, default=200)
    p.add_argument("--video_interval", type=int, default=2000)
    p.add_argument("--num_envs", type=int, default=None)
    p.add_argument("--task", type=str, default="Allsteps-v0")
    p.add_argument("--seed", type=int, default=None)
    p.add_argument("--distributed", action="store_true", default=False)
    p.add_argument("--checkpoint", type=str, default=None)
    p.add_argument("--sigma", type=str, default=None)
    p.add_argument("--max_iterations", type=int, default=None)
    p.add_argument("--device", type=str, default=None)
    p.add_argument("--multi_gpu_mode", choices=("allreduce", "allgather"), default=None,
                   help="gradient all-reduce (rl_games multi_gpu) or rollout all-gather at the PPO boundary")
    p.add_argument("--stone_level", type=int, default=None,
                   help="init-time stone curriculum level (BASELINE C3 knob; the reference always starts at 0)")
    p.add_argument("--log_root", type=str, default=os.path.join("logs", "rl_games"))
    args, _unknown = p.parse_known_args(argv)  # app-launcher flags (--headless, --enable_cameras ...) ignored
    return args


def _to_dict(obj):
    if dataclasses.is_dataclass(obj):
        return {f.name: _to_dict(getattr(obj, f.name)) for f in dataclasses.fields(obj)}
    if isinstance(obj, (list, tuple)):
        return [_to_dict(x) for x in obj]
    if isinstance(obj, dict):
        return {k: _to_dict(v) for k, v in obj.items()}
    return obj if isinstance(obj, (int, float, str, bool, type(None))) else repr(obj)


def main(argv=None):
    import yaml

    from allsteps_isaaclab_amd import registry
    from allsteps_isaaclab_amd.distributed import init_process_group
    from allsteps_isaaclab_amd.learning import Runner
    from allsteps_isaaclab_amd.learning.a2c_ppo_mirroring import A2CAgentSymmetry
    from allsteps_isaaclab_amd.rl_games import RlGamesGpuEnv, RlGamesVecEnvWrapper, env_configurations, vecenv

    args = parse_args(argv)
    if args.video:
        raise SystemExit("--video: there is no renderer in the MI355X build")
    env_cfg = registry.load_cfg_from_registry(args.task, "env_cfg_entry_point")
    agent_cfg = registry.load_cfg_from_registry(args.task, "rl_games_cfg_entry_point")
    # hydra-style overrides (env.<path>=<value> / agent.<path>=<value>), as the reference's @hydra_task_config
    registry.apply_overrides(env_cfg, agent_cfg, registry.override_tokens(sys.argv[1:] if argv is None else argv))
    env_cfg.scene.num_envs = args.num_envs if args.num_envs is not None else env_cfg.scene.num_envs
    env_cfg.sim.device = args.device if args.device is not None else env_cfg.sim.device
    if args.stone_level is not None:
        env_cfg.initial_stone_curriculum = args.stone_level
    if args.seed == -1:
        args.seed = random.randint(0, 10000)
    params = agent_cfg["params"]
    params["seed"] = args.seed if args.seed is not None else params["seed"]
    params["config"]["max_epochs"] = args.max_iterations if args.max_iterations is not None else params["config"]["max_epochs"]
    if args.checkpoint is not None:
        params["load_checkpoint"] = True
        params["load_path"] = args.checkpoint
    train_sigma = float(args.sigma) if args.sigma is not None else None
    env_kwargs = {}
    if args.distributed:
        info = init_process_group()
        params["seed"] += info.rank
        params["config"]["device"] = params["config"]["device_name"] = f"cuda:{info.local_rank}"
        params["config"]["multi_gpu"] = True
        env_cfg.sim.device = f"cuda:{info.local_rank}"
        env_kwargs["env_id_offset"] = info.rank * int(env_cfg.scene.num_envs)
    if args.multi_gpu_mode is not None:
        params["config"]["multi_gpu_mode"] = args.multi_gpu_mode
    env_cfg.seed = params["seed"]

    log_root = os.path.abspath(os.path.join(args.log_root, params["config"]["name"]))
    log_dir = params["config"].get("full_experiment_name", datetime.now().strftime("%Y-%m-%d_%H-%M-%S"))
    params["config"]["train_dir"] = log_root
    params["config"]["full_experiment_name"] = log_dir
    os.makedirs(os.path.join(log_root, log_dir, "params"), exist_ok=True)
    with open(os.path.join(log_root, log_dir, "params", "env.yaml"), "w") as f:
        yaml.safe_dump(_to_dict(env_cfg), f)
    with open(os.path.join(log_root, log_dir, "params", "agent.yaml"), "w") as f:
        yaml.safe_dump(_to_dict(agent_cfg), f)

    rl_device = params["config"]["device"]
    clip_obs = params["env"].get("clip_observations", math.inf)
    clip_actions = params["env"].get("clip_actions", math.inf)
    env = registry.make(args.task, cfg=env_cfg, render_mode=None, **env_kwargs)
    env = RlGamesVecEnvWrapper(env, rl_device, clip_obs, clip_actions)
    vecenv.register("IsaacRlgWrapper", lambda config_name, num_actors, **kw: RlGamesGpuEnv(config_name, num_actors, **kw))
    env_configurations.register("rlgpu", {"vecenv_type": "IsaacRlgWrapper", "env_creator": lambda **kw: env})
    params["config"]["num_actors"] = env.unwrapped.num_envs

    runner = Runner()
    runner.algo_factory.register_builder("a2c_continuous_mirroring", lambda **kw: A2CAgentSymmetry(**kw))
    runner.load(agent_cfg)
    runner.reset()
    run_args = {"train": True, "play": False, "sigma": train_sigma}
    if args.checkpoint is not None:
        run_args["checkpoint"] = args.checkpoint
    result = runner.run(run_args)
    env.close()
    return runner, result


if __name__ == "__main__":
    main()
