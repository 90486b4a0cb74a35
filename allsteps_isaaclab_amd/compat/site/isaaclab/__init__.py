"""Shim (allsteps_isaaclab_amd.compat): the parts of Isaac Lab's ``isaaclab`` package the Allsteps
train / play scripts import, over allsteps_isaaclab_amd."""
