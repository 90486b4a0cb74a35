"""Shim of ``isaaclab_rl.rl_games`` (isaaclab_rl/rl_games.py): the wrapper classes of
allsteps_isaaclab_amd.rl_games."""

from allsteps_isaaclab_amd.rl_games import RlGamesGpuEnv, RlGamesVecEnvWrapper

__all__ = ["RlGamesGpuEnv", "RlGamesVecEnvWrapper"]
