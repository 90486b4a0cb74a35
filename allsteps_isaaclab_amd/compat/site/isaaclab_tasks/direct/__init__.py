"""Shim package (allsteps_isaaclab_amd.compat)."""
