"""Shim of ``isaaclab_tasks``: importing it registers Allsteps-v0 (isaaclab_tasks/direct/allsteps/
__init__.py:13-22) with the task registry (and gymnasium)."""

import allsteps_isaaclab_amd.registry  # noqa: F401
