"""Shim of ``rl_games.algos_torch``."""

from . import players  # noqa: F401
