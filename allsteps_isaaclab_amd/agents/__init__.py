"""Agent configurations for Allsteps-v0 (rl_games PPO: rl_games_ppo_cfg.yaml)."""
