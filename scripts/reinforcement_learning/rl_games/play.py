"""Play a checkpoint of the Allsteps-v0 rl_games agent (reference: scripts/reinforcement_learning/rl_games/play.py).

Same flow as the reference (play.py:100-201): load the configs from the task registry, wrap the env
in ``RlGamesVecEnvWrapper``, register it as ``rlgpu``, ``runner.create_player()``,
``agent.restore(checkpoint)``, then step ``obs -> agent.get_action(obs, is_deterministic) ->
env.step`` in inference mode.  There is no simulator app to keep running, so the loop runs
``--steps`` steps (the reference runs until the app window closes) and prints the mean episode
reward / length of the episodes that finished.  ``--video`` (play.py:111-127, 189-193) makes the env with
``render_mode="rgb_array"``, wraps it in ``RecordVideo`` (step 0 trigger, ``--video_length`` frames of env
0, written under ``<run dir>/videos/play`` -- as an animated GIF: no MP4 encoder in this image) and stops
after ``--video_length`` steps.
Checkpoints are rl_games' layout ({'model': state_dict, ...}), so a checkpoint trained by the
reference's rl_games loads here and vice versa.

    python scripts/reinforcement_learning/rl_games/play.py --task Allsteps-v0 --checkpoint runs/.../nn/allsteps.pth
"""

from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, ROOT)


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="Play a checkpoint of an RL agent from RL-Games.")
    p.add_argument("--video", action="store_true", default=False)
    p.add_argument("--video_length", type=int, default=200)
    p.add_argument("--num_envs", type=int, default=None)
    p.add_argument("--task", type=str, default="Allsteps-v0")
    p.add_argument("--checkpoint", type=str, required=True)
    p.add_argument("--use_last_checkpoint", action="store_true")
    p.add_argument("--real-time", action="store_true", default=False)
    p.add_argument("--steps", type=int, default=1000)
    p.add_argument("--stochastic", action="store_true", help="sample actions instead of the mean")
    p.add_argument("--device", type=str, default=None)
    args, _unknown = p.parse_known_args(argv)
    return args


def main(argv=None):
    import torch

    from allsteps_isaaclab_amd import registry
    from allsteps_isaaclab_amd.learning import Runner
    from allsteps_isaaclab_amd.rl_games import RlGamesGpuEnv, RlGamesVecEnvWrapper, env_configurations, vecenv

    args = parse_args(argv)
    env_cfg = registry.load_cfg_from_registry(args.task, "env_cfg_entry_point")
    agent_cfg = registry.load_cfg_from_registry(args.task, "rl_games_cfg_entry_point")
    env_cfg.scene.num_envs = args.num_envs if args.num_envs is not None else env_cfg.scene.num_envs
    env_cfg.sim.device = args.device if args.device is not None else env_cfg.sim.device
    params = agent_cfg["params"]
    rl_device = params["config"]["device"]
    clip_obs = params["env"].get("clip_observations", math.inf)
    clip_actions = params["env"].get("clip_actions", math.inf)
    env = registry.make(args.task, cfg=env_cfg, render_mode="rgb_array" if args.video else None)
    video = None
    if args.video:
        from allsteps_isaaclab_amd.envs.record_video import RecordVideo

        log_dir = os.path.dirname(os.path.dirname(os.path.abspath(args.checkpoint)))
        env = video = RecordVideo(env, video_folder=os.path.join(log_dir, "videos", "play"),
                                  step_trigger=lambda step: step == 0, video_length=args.video_length,
                                  disable_logger=True)
    env = RlGamesVecEnvWrapper(env, rl_device, clip_obs, clip_actions)
    vecenv.register("IsaacRlgWrapper", lambda config_name, num_actors, **kw: RlGamesGpuEnv(config_name, num_actors, **kw))
    env_configurations.register("rlgpu", {"vecenv_type": "IsaacRlgWrapper", "env_creator": lambda **kw: env})
    params["load_checkpoint"] = True
    params["load_path"] = args.checkpoint
    params["config"]["num_actors"] = env.unwrapped.num_envs
    runner = Runner()
    runner.load(agent_cfg)
    agent = runner.create_player()
    agent.restore(args.checkpoint)
    agent.reset()
    dt = env.unwrapped.step_dt
    obs = env.reset()
    if isinstance(obs, dict):
        obs = obs["obs"]
    _ = agent.get_batch_size(obs, 1)
    deterministic = agent.is_deterministic and not args.stochastic
    n = env.unwrapped.num_envs
    cur_r = torch.zeros(n, device=env.unwrapped.device)
    cur_l = torch.zeros(n, device=env.unwrapped.device)
    sums = torch.zeros(3, device=env.unwrapped.device)  # reward, length, episodes
    steps = min(args.steps, args.video_length) if args.video else args.steps
    for _ in range(steps):
        t0 = time.time()
        with torch.inference_mode():
            obs = agent.obs_to_torch(obs)
            actions = agent.get_action(obs, is_deterministic=deterministic)
            obs, rew, dones, _ = env.step(actions)
            cur_r += rew
            cur_l += 1
            d = dones.float()
            sums += torch.stack([(cur_r * d).sum(), (cur_l * d).sum(), d.sum()])
            cur_r *= 1 - d
            cur_l *= 1 - d
        sleep = dt - (time.time() - t0)
        if args.real_time and sleep > 0:
            time.sleep(sleep)
    r, l, k = sums.tolist()
    env.close()
    out = {"steps": steps, "num_envs": n, "episodes": int(k), "mean_reward": r / max(k, 1.0),
           "mean_length": l / max(k, 1.0), "deterministic": deterministic}
    if video is not None:
        out["video"] = video.saved
    print(json.dumps(out))
    return out


if __name__ == "__main__":
    main()
