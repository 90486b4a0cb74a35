"""Shim of ``isaaclab_rl``."""
