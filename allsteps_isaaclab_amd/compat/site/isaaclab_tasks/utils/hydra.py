"""Shim of ``isaaclab_tasks.utils.hydra.hydra_task_config`` without hydra (absent offline): the
decorated ``main(env_cfg, agent_cfg)`` receives the task's registry configs with the command line's
hydra-style overrides applied (``env.<path>=<value>`` / ``agent.<path>=<value>``, values parsed as
YAML scalars), which is how Isaac Lab's hydra integration addresses the two configs."""

from __future__ import annotations

import functools
import sys

from allsteps_isaaclab_amd.registry import apply_overrides, load_cfg_from_registry, override_tokens  # noqa: F401


def hydra_task_config(task_name: str, agent_cfg_entry_point: str):
    def decorator(func):
        @functools.wraps(func)
        def wrapper(*args, **kwargs):
            env_cfg = load_cfg_from_registry(task_name, "env_cfg_entry_point")
            agent_cfg = load_cfg_from_registry(task_name, agent_cfg_entry_point)
            apply_overrides(env_cfg, agent_cfg, override_tokens(sys.argv[1:]))
            return func(env_cfg, agent_cfg, *args, **kwargs)

        return wrapper

    return decorator
