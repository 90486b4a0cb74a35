"""Shim of ``rl_games.torch_runner.Runner``."""

from allsteps_isaaclab_amd.learning.runner import Runner

__all__ = ["Runner"]
