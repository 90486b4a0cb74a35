"""Shim of ``gymnasium.wrappers``: ``RecordVideo`` is allsteps_isaaclab_amd.envs.record_video's (GIF frames
of the software renderer, envs/render.py)."""

from allsteps_isaaclab_amd.envs.record_video import RecordVideo  # noqa: F401
