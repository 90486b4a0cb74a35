"""CPU test double with the rl_games VecEnv surface (get_env_info / reset / step -> obs, rew, dones,
{'time_outs'}): a batch of 2-D point masses steered to a goal.  Used only to exercise the PPO trainer
on CPU; the product env (AllstepsEnv) runs on the HIP backend only."""

import torch

from allsteps_isaaclab_amd.envs.spaces import Box


class ToyReachEnv:
    def __init__(self, num_envs: int = 64, seed: int = 0, horizon: int = 40, device: str = "cpu"):
        self.n, self.T, self.device = num_envs, horizon, torch.device(device)
        self.g = torch.Generator(device=self.device).manual_seed(seed)
        self.x = torch.zeros(num_envs, 2, device=self.device)
        self.goal = torch.zeros(num_envs, 2, device=self.device)
        self.t = torch.zeros(num_envs, device=self.device)

    def get_env_info(self):
        return {"observation_space": Box(-float("inf"), float("inf"), (5,)), "action_space": Box(-1.0, 1.0, (2,)),
                "state_space": None}

    def _reset(self, mask):
        m = mask.unsqueeze(1)
        self.x = torch.where(m, torch.rand(self.n, 2, generator=self.g, device=self.device) * 2 - 1, self.x)
        self.goal = torch.where(m, torch.rand(self.n, 2, generator=self.g, device=self.device) * 2 - 1, self.goal)
        self.t = torch.where(mask, torch.zeros_like(self.t), self.t)

    def _obs(self):
        return torch.cat([self.x, self.goal, (self.t / self.T).unsqueeze(1)], 1)

    def reset(self):
        self._reset(torch.ones(self.n, dtype=torch.bool, device=self.device))
        return self._obs()

    def step(self, actions):
        self.x = self.x + 0.1 * torch.clamp(actions, -1, 1)
        self.t += 1
        d = torch.linalg.vector_norm(self.x - self.goal, dim=1)
        rew = 1.0 - d
        term = d < 0.05
        trunc = self.t >= self.T
        done = term | trunc
        self._reset(done)
        return self._obs(), rew, done, {"time_outs": trunc & ~term}


def agent_params(num_envs: int, **overrides):
    """The Allsteps agent config (rl_games_ppo_cfg.yaml) scaled to the toy env."""
    import yaml

    from allsteps_isaaclab_amd import registry

    cfg = registry.load_cfg_from_registry("Allsteps-v0", "rl_games_cfg_entry_point")
    p = cfg["params"]
    p["network"]["mlp"]["units"] = [64, 64]
    c = p["config"]
    c.update(device="cpu", num_actors=num_envs, horizon_length=16, minibatch_size=num_envs * 4, mini_epochs=4,
             max_epochs=3, print_stats=False, save_frequency=0, train_dir="/tmp/allsteps_ppo_test")
    c.update(overrides)
    return yaml.safe_load(yaml.safe_dump(p))
