"""Opt-in import shims: the reference's module paths over this package, so that the reference's own
``scripts/reinforcement_learning/rl_games/train.py`` / ``play.py`` run without editing their import
blocks (``train.py:13,48-73``, ``play.py:12,50-69``; north_star "train.py runs unchanged").

``site/`` holds top-level packages named as the reference's dependencies -- ``isaaclab`` (``app``,
``envs``, ``utils``), ``isaaclab_rl.rl_games``, ``isaaclab_tasks`` (registration, ``utils``,
``utils.hydra``, ``direct.allsteps.learning``), ``rl_games`` (``common``, ``torch_runner``,
``algos_torch.players``) and a minimal ``gymnasium`` -- each a thin re-export of this package's own
implementation (``registry``, ``envs``, ``rl_games``, ``learning``).  Nothing is importable under those
names until :func:`install` is called, and ``install`` appends ``site/`` to the END of ``sys.path``,
so a real Isaac Lab / rl_games / gymnasium installation always wins: the shims never shadow one.

    python -m allsteps_isaaclab_amd.compat <reference>/scripts/reinforcement_learning/rl_games/train.py \\
        --task Allsteps-v0 --headless --num_envs 4096
"""

from __future__ import annotations

import os
import runpy
import sys

SITE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "site")
SHIMMED = ("isaaclab", "isaaclab_rl", "isaaclab_tasks", "rl_games", "gymnasium")


def install() -> list[str]:
    """Make the shim packages importable (lowest priority).  Returns the names a real installation
    already provides (those keep resolving to the real package)."""
    import importlib.util

    real = [m for m in SHIMMED if SITE not in sys.path and importlib.util.find_spec(m) is not None]
    if SITE not in sys.path:
        sys.path.append(SITE)
    return real


def installed() -> bool:
    return SITE in sys.path


def run_script(path: str, argv: list[str] | None = None) -> None:
    """Run a reference script unchanged (as ``__main__``) with the shims installed."""
    install()
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    if root not in sys.path:
        sys.path.insert(0, root)
    sys.argv = [path] + list(argv or [])
    runpy.run_path(path, run_name="__main__")
