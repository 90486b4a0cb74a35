"""Shim of ``rl_games.common``."""

from . import env_configurations, vecenv  # noqa: F401
