"""Minimal ``gymnasium`` shim (gymnasium is absent offline): ``register`` / ``make`` / ``spec`` /
``registry`` over allsteps_isaaclab_amd.registry, ``spaces`` over allsteps_isaaclab_amd.envs.spaces.
``wrappers.RecordVideo`` records ``env.render()`` frames (envs/record_video.py)."""

from allsteps_isaaclab_amd.envs import spaces  # noqa: F401
from allsteps_isaaclab_amd.registry import make, register, spec  # noqa: F401
from allsteps_isaaclab_amd.registry import registry  # noqa: F401

from . import wrappers  # noqa: F401,E402

ALLSTEPS_COMPAT = True


class Env:  # annotation / isinstance surface
    pass
