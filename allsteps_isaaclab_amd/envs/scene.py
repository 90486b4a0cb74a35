"""``InteractiveScene``'s caller-visible geometry (isaaclab/scene/interactive_scene.py:292-302).

The step runs every env in its own frame: an env's positions (``root_pos_w``, ``body_pos_w``,
``steps_pos``, ...) are relative to its origin, which the reference adds on reset
(allsteps_env.py:111,515) and then subtracts again everywhere the task reads them (targets, distances and
potentials are differences; heights are the z of a ground plane at z = 0).  The reference's world
coordinates are these plus ``scene.env_origins``.
"""

from __future__ import annotations

import math

import torch


def grid_env_origins(num_envs: int, env_spacing: float, device="cpu") -> torch.Tensor:
    """(num_envs, 3) origins of a plane terrain's env grid, the rule of TerrainImporter
    ._compute_env_origins_grid (isaaclab/terrains/terrain_importer.py:349-361): rows = ceil(N /
    floor(sqrt(N))), cols = ceil(N / rows), env k at row k // cols, column k % cols; x = -(row - (rows -
    1) / 2) * spacing, y = (col - (cols - 1) / 2) * spacing, z = 0."""
    n = int(num_envs)
    rows = math.ceil(n / int(math.sqrt(n)))
    cols = math.ceil(n / rows)
    k = torch.arange(n, device=device)
    row = torch.div(k, cols, rounding_mode="floor").to(torch.float32)
    col = (k % cols).to(torch.float32)
    out = torch.zeros(n, 3, device=device)
    out[:, 0] = -(row - (rows - 1) / 2) * env_spacing
    out[:, 1] = (col - (cols - 1) / 2) * env_spacing
    return out


class SceneView:
    """``env.scene``: ``num_envs``, ``cfg`` and ``env_origins`` (the plane terrain's grid)."""

    def __init__(self, cfg, device):
        self.cfg = cfg
        self.device = str(device)
        self._origins = None

    @property
    def num_envs(self) -> int:
        return int(self.cfg.num_envs)

    @property
    def env_origins(self) -> torch.Tensor:
        if self._origins is None:
            self._origins = grid_env_origins(self.num_envs, float(self.cfg.env_spacing), self.device)
        return self._origins
