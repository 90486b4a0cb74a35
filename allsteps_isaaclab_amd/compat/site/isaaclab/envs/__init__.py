"""Shim of ``isaaclab.envs``: the direct-workflow base over allsteps_isaaclab_amd.envs.  Multi-agent
and manager-based workflows are out of scope: their names exist for the scripts'
isinstance checks and annotations only."""

from allsteps_isaaclab_amd.envs.allsteps_env_cfg import AllstepsEnvCfg as DirectRLEnvCfg
from allsteps_isaaclab_amd.envs.direct_rl_env import DirectRLEnv


class DirectMARLEnv:  # no multi-agent task on this path: isinstance(env.unwrapped, DirectMARLEnv) is False
    pass


class DirectMARLEnvCfg:
    pass


class ManagerBasedRLEnvCfg:
    pass


def multi_agent_to_single_agent(env, state_as_observation: bool = False):
    raise NotImplementedError("multi-agent envs are out of scope of the MI355X build (SURVEY §8)")


__all__ = ["DirectRLEnv", "DirectRLEnvCfg", "DirectMARLEnv", "DirectMARLEnvCfg", "ManagerBasedRLEnvCfg",
           "multi_agent_to_single_agent"]
