"""Shim of the third-party ``rl_games`` (1.6.1, absent offline) over allsteps_isaaclab_amd: the env
registries, ``Runner`` and the continuous PPO player, whose maths allsteps_isaaclab_amd.learning
restates.  A real rl_games installation takes precedence (compat.install appends
this directory to the end of sys.path)."""

ALLSTEPS_COMPAT = True
