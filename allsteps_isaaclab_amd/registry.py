"""Task registry: ``gym.register(id="Allsteps-v0", ...)`` / ``gym.make``.

Mirrors ``isaaclab_tasks/direct/allsteps/__init__.py:13-22`` (entry point, ``disable_env_checker``,
``env_cfg_entry_point`` / ``rl_games_cfg_entry_point`` kwargs) and ``train.py:134``
(``gym.make(task, cfg=env_cfg, render_mode=None)``).  When ``gymnasium`` is installed the task is
registered there too, so ``gymnasium.make("Allsteps-v0", cfg=...)`` works unchanged; this image has
no gymnasium, so the same ``register`` / ``make`` / ``spec`` surface is provided here.
"""

from __future__ import annotations

import importlib
from dataclasses import dataclass, field


@dataclass
class EnvSpec:
    id: str
    entry_point: str
    disable_env_checker: bool = True
    kwargs: dict = field(default_factory=dict)


registry: dict[str, EnvSpec] = {}


def _resolve(entry: str):
    mod, _, attr = entry.partition(":")
    obj = importlib.import_module(mod)
    for part in attr.split("."):
        obj = getattr(obj, part)
    return obj


def register(id: str, entry_point: str, disable_env_checker: bool = True, kwargs: dict | None = None) -> None:
    registry[id] = EnvSpec(id, entry_point, disable_env_checker, dict(kwargs or {}))
    try:  # pragma: no cover - gymnasium absent in this image
        import gymnasium

        if getattr(gymnasium, "ALLSTEPS_COMPAT", False):  # the opt-in shim (compat/site) IS this registry
            return
        if id not in gymnasium.registry:
            gymnasium.register(id=id, entry_point=entry_point, disable_env_checker=disable_env_checker,
                               kwargs=dict(kwargs or {}))
    except ImportError:
        pass


def spec(id: str) -> EnvSpec:
    if id not in registry:
        raise KeyError(f"environment {id!r} is not registered (known: {sorted(registry)})")
    return registry[id]


def load_cfg_from_registry(task_name: str, entry_point_key: str):
    """isaaclab_tasks/utils/parse_cfg.py:19 load_cfg_from_registry: instantiate the cfg entry point."""
    ep = spec(task_name).kwargs[entry_point_key]
    if isinstance(ep, str) and ep.endswith((".yaml", ".yml")):
        import yaml

        mod, _, fname = ep.partition(":")
        import os

        path = os.path.join(os.path.dirname(importlib.import_module(mod).__file__), fname)
        with open(path) as f:
            return yaml.safe_load(f)
    obj = _resolve(ep) if isinstance(ep, str) else ep
    return obj() if callable(obj) else obj


def make(id: str, cfg=None, render_mode: str | None = None, **kwargs):
    """gym.make(id, cfg=env_cfg, render_mode=None)."""
    s = spec(id)
    if cfg is None and "env_cfg_entry_point" in s.kwargs:
        cfg = load_cfg_from_registry(id, "env_cfg_entry_point")
    cls = _resolve(s.entry_point)
    return cls(cfg=cfg, render_mode=render_mode, **kwargs)


register(
    id="Allsteps-v0",
    entry_point="allsteps_isaaclab_amd.envs.allsteps_env:AllstepsEnv",
    disable_env_checker=True,
    kwargs={
        "env_cfg_entry_point": "allsteps_isaaclab_amd.envs.allsteps_env_cfg:AllstepsEnvCfg",
        "rl_games_cfg_entry_point": "allsteps_isaaclab_amd.agents:rl_games_ppo_cfg.yaml",
    },
)

# BASELINE C5: the ANYmal-C quadruped on the stones, on ANYmal-C's simulation settings (authored task id:
# the reference registers its ANYmal-C tasks as Isaac-Velocity-*-Anymal-C-Direct-v0, flat-ground velocity
# tracking, anymal_c/__init__.py:17-41)
register(
    id="Allsteps-AnymalC-v0",
    entry_point="allsteps_isaaclab_amd.envs.anymal_c_stones_env:AnymalCStonesEnv",
    disable_env_checker=True,
    kwargs={
        "env_cfg_entry_point": "allsteps_isaaclab_amd.envs.anymal_c_stones_env_cfg:AnymalCStonesEnvCfg",
        "rl_games_cfg_entry_point": "allsteps_isaaclab_amd.agents:rl_games_anymal_c_stones_ppo_cfg.yaml",
    },
)


def _set(obj, path: list[str], value) -> None:
    for k in path[:-1]:
        obj = obj[k] if isinstance(obj, dict) else getattr(obj, k)
    if isinstance(obj, dict):
        obj[path[-1]] = value
    else:
        if not hasattr(obj, path[-1]):
            raise AttributeError(f"{type(obj).__name__} has no field {path[-1]!r}")
        setattr(obj, path[-1], value)


OVERRIDE_PREFIXES = ("env.", "agent.", "+env.", "+agent.")


def override_tokens(argv: list[str]) -> list[str]:
    """The hydra-style override tokens of a command line: only ``[+]env.<path>=<v>`` /
    ``[+]agent.<path>=<v>`` (a flag's value that happens to contain '=', e.g. ``--checkpoint a=b.pth``,
    is not an override)."""
    return [a for a in argv if "=" in a and a.startswith(OVERRIDE_PREFIXES)]


def apply_overrides(env_cfg, agent_cfg, overrides: list[str]) -> None:
    """Hydra-style command-line overrides (``env.<path>=<value>`` / ``agent.<path>=<value>``, values
    parsed as YAML scalars) -- how Isaac Lab's hydra integration addresses the two configs."""
    import yaml

    for ov in overrides:
        key, sep, val = ov.partition("=")
        if not sep or "." not in key:
            raise ValueError(f"unsupported override {ov!r} (expected env.<path>=<value> or agent.<path>=<value>)")
        root, *path = key.lstrip("+").split(".")
        target = {"env": env_cfg, "agent": agent_cfg}.get(root)
        if target is None:
            raise ValueError(f"override {ov!r} must start with env. or agent.")
        _set(target, path, yaml.safe_load(val))
