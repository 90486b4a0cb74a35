"""Shim of ``rl_games.common.algo_observer``: the observer hooks (no-ops; the trainer keeps its own
episode statistics on the device)."""

from allsteps_isaaclab_amd.learning.a2c_continuous import DefaultAlgoObserver


class AlgoObserver(DefaultAlgoObserver):
    pass


class IsaacAlgoObserver(DefaultAlgoObserver):
    """isaaclab's rl_games observer (episode-info logging) -- statistics come from the trainer here."""


__all__ = ["AlgoObserver", "DefaultAlgoObserver", "IsaacAlgoObserver"]
