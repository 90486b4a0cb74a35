"""Shim of ``isaaclab_tasks/direct/allsteps/learning/a2c_ppo_mirroring.py``: the mirror agent."""

from allsteps_isaaclab_amd.learning.a2c_ppo_mirroring import A2CAgentSymmetry

__all__ = ["A2CAgentSymmetry"]
