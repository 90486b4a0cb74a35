"""``A2CAgentSymmetry`` -- the reference's mirror-augmented PPO agent (``allsteps/learning/a2c_ppo_mirroring.py:5-37``).

With ``config.symmetry`` on, every rollout batch is doubled with its left/right mirror image
(``get_symmetric_states_rl_games``, allsteps_env.py:570-660): obs / actions / mus mirrored, returns /
dones / values / sigmas / neglogpacs repeated, batch and dataset sizes doubled.  The reference config
ships with ``symmetry: False`` (``rl_games_ppo_cfg.yaml:76``), in which case this is ``A2CAgent``.
"""

from __future__ import annotations

from ..envs.allsteps_env import get_symmetric_states_rl_games
from .a2c_continuous import A2CAgent


class A2CAgentSymmetry(A2CAgent):
    def __init__(self, base_name: str, params: dict):
        super().__init__(base_name, params)
        self.symmetry = bool(params["config"].get("symmetry", False))
        if self.symmetry:
            self.batch_size *= 2
            self.batch_size_envs *= 2

    def play_steps(self) -> dict:
        batch = super().play_steps()
        if self.symmetry:
            batch["returns"] = batch["returns"].repeat(2, 1)
            batch["dones"] = batch["dones"].repeat(2)
            batch["values"] = batch["values"].repeat(2, 1)
            batch["sigmas"] = batch["sigmas"].repeat(2, 1)
            batch["neglogpacs"] = batch["neglogpacs"].repeat(2)
            batch["obses"], batch["actions"], batch["mus"] = get_symmetric_states_rl_games(
                batch["obses"], batch["actions"], self.vec_env.env, False, batch["mus"])
        return batch
