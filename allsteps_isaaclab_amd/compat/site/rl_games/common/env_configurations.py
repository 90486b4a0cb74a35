"""Shim of ``rl_games.common.env_configurations`` (module-level ``register`` / ``configurations``)."""

from allsteps_isaaclab_amd._vecenv import env_configurations as _reg

configurations = _reg.configurations


def register(name: str, config: dict) -> None:
    _reg.register(name, config)
