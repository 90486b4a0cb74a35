"""Shim of ``isaaclab_tasks.direct.allsteps.learning``."""
