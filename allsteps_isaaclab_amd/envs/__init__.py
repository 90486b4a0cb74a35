"""Environments: DirectRLEnv base + AllstepsEnv (the Allsteps-v0 task)."""
