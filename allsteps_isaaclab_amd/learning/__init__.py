"""PPO trainer for Allsteps-v0 with rl_games 1.6.1 semantics (rl_games is
absent from this image).  ``Runner`` / ``A2CAgent`` / ``A2CAgentSymmetry`` / ``PpoPlayerContinuous``
keep the names the reference's train.py / play.py use."""

from .a2c_continuous import A2CAgent  # noqa: F401
from .a2c_ppo_mirroring import A2CAgentSymmetry  # noqa: F401
from .player import PpoPlayerContinuous  # noqa: F401
from .runner import Runner  # noqa: F401
