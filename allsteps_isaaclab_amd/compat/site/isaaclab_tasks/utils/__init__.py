"""Shim of ``isaaclab_tasks.utils`` (parse_cfg.py): cfg loading from the registry, ``parse_env_cfg``
and ``get_checkpoint_path``."""

from __future__ import annotations

import os
import re

from allsteps_isaaclab_amd.registry import load_cfg_from_registry


def parse_env_cfg(task_name: str, device: str = "cuda:0", num_envs: int | None = None,
                  use_fabric: bool | None = None):
    cfg = load_cfg_from_registry(task_name, "env_cfg_entry_point")
    cfg.sim.device = device
    if num_envs is not None:
        cfg.scene.num_envs = num_envs
    return cfg


def get_checkpoint_path(log_path: str, run_dir: str = ".*", checkpoint: str = ".*",
                        other_dirs: list[str] | None = None, sort_alpha: bool = True) -> str:
    """parse_cfg.py get_checkpoint_path: the last run matching run_dir, its last checkpoint matching
    `checkpoint` (under other_dirs)."""
    try:
        runs = [os.path.join(log_path, r) for r in os.listdir(log_path)
                if os.path.isdir(os.path.join(log_path, r)) and re.match(run_dir, r)]
    except FileNotFoundError:
        runs = []
    if not runs:
        raise ValueError(f"No runs present in the directory: '{log_path}' match: '{run_dir}'.")
    runs.sort() if sort_alpha else runs.sort(key=os.path.getmtime)
    run_path = os.path.join(runs[-1], *(other_dirs or []))
    models = [f for f in os.listdir(run_path) if re.match(checkpoint, f)]
    if not models:
        raise ValueError(f"No checkpoints in the directory: '{run_path}' match '{checkpoint}'.")
    models.sort(key=lambda m: f"{m:0>15}")
    return os.path.join(run_path, models[-1])


__all__ = ["get_checkpoint_path", "load_cfg_from_registry", "parse_env_cfg"]
