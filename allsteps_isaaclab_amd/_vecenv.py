"""Stand-ins for rl_games' env registries (``rl_games.common.env_configurations`` /
``rl_games.common.vecenv``, rl_games 1.6.1) used when rl_games is not installed: ``register`` /
``configurations`` and ``register`` / ``create_vec_env`` with rl_games' semantics.  The opt-in shim
package ``rl_games`` (allsteps_isaaclab_amd.compat) exposes these same objects, so a script that
registers its env through ``rl_games.common`` reaches this package's trainer."""

from __future__ import annotations


class IVecEnv:  # noqa: D101 - rl_games.common.ivecenv.IVecEnv surface
    pass


class Configurations:
    def __init__(self):
        self.configurations: dict[str, dict] = {}

    def register(self, name: str, config: dict):
        self.configurations[name] = config


class VecEnvRegistry:
    """rl_games.common.vecenv: ``register(type_name, creator)`` / ``create_vec_env(config_name, n)``."""

    def __init__(self):
        self.vecenv_config: dict = {}

    def register(self, config_name: str, func) -> None:
        self.vecenv_config[config_name] = func

    def create_vec_env(self, config_name: str, num_actors: int, **kwargs):
        vec_env_name = env_configurations.configurations[config_name]["vecenv_type"]
        return self.vecenv_config[vec_env_name](config_name, num_actors, **kwargs)


env_configurations = Configurations()
vecenv = VecEnvRegistry()
