"""Shim of the ``isaaclab.utils`` helpers the scripts import."""
