"""Shim of ``rl_games.common.player`` (``BasePlayer`` for the scripts' annotations)."""

from allsteps_isaaclab_amd.learning.player import PpoPlayerContinuous as BasePlayer

__all__ = ["BasePlayer"]
