"""Shim of ``rl_games.common.vecenv`` (module-level ``register`` / ``create_vec_env``, ``IVecEnv``)."""

from allsteps_isaaclab_amd._vecenv import IVecEnv  # noqa: F401
from allsteps_isaaclab_amd._vecenv import vecenv as _reg

vecenv_config = _reg.vecenv_config


def register(config_name: str, func) -> None:
    _reg.register(config_name, func)


def create_vec_env(config_name: str, num_actors: int, **kwargs):
    return _reg.create_vec_env(config_name, num_actors, **kwargs)
