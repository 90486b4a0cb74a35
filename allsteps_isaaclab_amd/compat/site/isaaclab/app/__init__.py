"""Shim of ``isaaclab.app.AppLauncher`` (isaaclab/app/app_launcher.py): there is no Omniverse Kit app in
the MI355X build, so launching is a no-op; the CLI flags are accepted (and ``--device`` honoured by
the scripts), ranks come from the torch.distributed.run environment."""

from __future__ import annotations

import argparse
import os


class _SimulationApp:
    """``SimulationApp`` surface used by the scripts: ``is_running()`` / ``close()``.  ``is_running``
    stays True (play.py's loop runs until interrupted, as under Kit) unless ALLSTEPS_APP_MAX_FRAMES
    bounds it."""

    def __init__(self):
        self._frames = 0
        self._max = int(os.environ.get("ALLSTEPS_APP_MAX_FRAMES", "0"))

    def is_running(self) -> bool:
        self._frames += 1
        return self._max <= 0 or self._frames <= self._max

    def close(self) -> None:
        pass


class AppLauncher:
    def __init__(self, launcher_args=None, **kwargs):
        args = vars(launcher_args) if isinstance(launcher_args, argparse.Namespace) else dict(launcher_args or {})
        args.update(kwargs)
        self.device = args.get("device", "cuda:0")
        self.local_rank = int(os.environ.get("LOCAL_RANK", 0))
        self.global_rank = int(os.environ.get("RANK", 0))
        self.app = _SimulationApp()

    @staticmethod
    def add_app_launcher_args(parser: argparse.ArgumentParser) -> None:
        g = parser.add_argument_group("app_launcher arguments (accepted, no Kit app in the MI355X build)")
        g.add_argument("--headless", action="store_true", default=False)
        g.add_argument("--livestream", type=int, default=-1)
        g.add_argument("--enable_cameras", action="store_true", default=False)
        g.add_argument("--xr", action="store_true", default=False)
        g.add_argument("--device", type=str, default="cuda:0")
        g.add_argument("--verbose", action="store_true", default=False)
        g.add_argument("--info", action="store_true", default=False)
        g.add_argument("--experience", type=str, default="")
        g.add_argument("--rendering_mode", type=str, default=None)
        g.add_argument("--kit_args", type=str, default="")
