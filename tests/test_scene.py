"""env.scene.env_origins: the plane terrain's env grid (terrain_importer.py:349-361), restated in
envs/scene.py; pinned here to hand-worked values and to a meshgrid statement of the same rule."""

import numpy as np
import torch

from allsteps_isaaclab_amd.envs.allsteps_env_cfg import InteractiveSceneCfg
from allsteps_isaaclab_amd.envs.scene import SceneView, grid_env_origins


def _meshgrid_rule(n, spacing):
    rows = np.ceil(n / int(np.sqrt(n)))
    cols = np.ceil(n / rows)
    ii, jj = np.meshgrid(np.arange(rows), np.arange(cols), indexing="ij")
    out = np.zeros((n, 3), np.float32)
    out[:, 0] = -(ii.flatten()[:n] - (rows - 1) / 2) * spacing
    out[:, 1] = (jj.flatten()[:n] - (cols - 1) / 2) * spacing
    return out


def test_grid_origins_hand_worked():
    # 5 envs: rows = ceil(5 / 2) = 3, cols = ceil(5 / 3) = 2
    o = grid_env_origins(5, 4.0)
    want = [[4, -2, 0], [4, 2, 0], [0, -2, 0], [0, 2, 0], [-4, -2, 0]]
    assert torch.equal(o, torch.tensor(want, dtype=torch.float32))


def test_grid_origins_match_the_meshgrid_rule():
    for n in (1, 2, 3, 7, 64, 1000, 4096, 32768):
        for sp in (4.0, 2.5):
            np.testing.assert_array_equal(grid_env_origins(n, sp).numpy(), _meshgrid_rule(n, sp))


def test_scene_view_uses_the_cfg_spacing():
    s = SceneView(InteractiveSceneCfg(num_envs=4096, env_spacing=4.0), "cpu")
    o = s.env_origins
    assert s.num_envs == 4096 and o.shape == (4096, 3)
    assert float(o[:, 0].max()) == 126.0 and float(o[:, 1].min()) == -126.0 and float(o[:, 2].abs().max()) == 0.0
    assert s.env_origins is o  # computed once
