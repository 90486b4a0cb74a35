"""Shim of ``rl_games.algos_torch.players`` (``PpoPlayerContinuous``)."""

from allsteps_isaaclab_amd.learning.player import PpoPlayerContinuous

__all__ = ["PpoPlayerContinuous"]
