"""The ``rgb_array`` renderer behind play.py --video (envs/render.py, envs/record_video.py), on the CPU.

* its host forward kinematics puts the torso and feet where the stepped state's ``body_pos`` has them
  (the oracle's step writes body_pos from the same FK the kernel runs), within float32 rounding;
* a frame is an (H, W, 3) uint8 image with the robot and the stones drawn;
* RecordVideo writes ``video_length`` frames as an animated GIF from the trigger step on.
"""

import os

import numpy as np
import pytest

from allsteps_isaaclab_amd.envs.render import link_poses, render_frame
from allsteps_isaaclab_amd.model import load_model


def _stepped_state(oracle_mod, n=4, steps=30):
    orc = oracle_mod.Oracle()
    st = orc.state(n)
    for k in range(20):
        st["stones"][3 * k] = 0.75 * k
    orc.reset_all(st, seed=3)
    rng = np.random.default_rng(1)
    for _ in range(steps):
        orc.env_step(st, rng.uniform(-1, 1, (n, 21)).astype(np.float32))
    return orc, st


def test_host_fk_matches_the_stepped_body_positions(oracle_mod):
    m = load_model()
    _, st = _stepped_state(oracle_mod)
    for e in range(st["root_pos"].shape[1]):
        R, p = link_poses(m, st["root_pos"][:, e], st["root_quat"][:, e], st["q"][:, e])
        for b, link in enumerate([int(m["torso_link"]), int(m["foot_link"][0]), int(m["foot_link"][1])]):
            np.testing.assert_allclose(p[link], st["body_pos"][3 * b:3 * b + 3, e], atol=2e-5)
        for i in range(int(m["num_links"])):
            np.testing.assert_allclose(R[i] @ R[i].T, np.eye(3), atol=1e-6)  # float32 root quaternion


def test_frame_draws_robot_and_stones(oracle_mod):
    m = load_model()
    _, st = _stepped_state(oracle_mod, n=1, steps=5)
    img = render_frame(m, st["root_pos"][:, 0], st["root_quat"][:, 0], st["q"][:, 0],
                       st["stones"][:, 0].reshape(-1, 3), (0.25, 0.4, 0.1125), target=1)
    assert img.shape == (360, 640, 3) and img.dtype == np.uint8
    robot = (img[..., 0] == 40) & (img[..., 1] == 90) & (img[..., 2] == 170)
    target = (img[..., 0] == 200) & (img[..., 1] == 120) & (img[..., 2] == 60)
    assert robot.sum() > 500 and target.sum() > 100


def test_record_video_writes_gif(tmp_path):
    from PIL import Image

    from allsteps_isaaclab_amd.envs.record_video import RecordVideo

    class Fake:
        render_mode = "rgb_array"
        step_dt = 1.0 / 60.0
        unwrapped = property(lambda self: self)

        def __init__(self):
            self.t = 0

        def render(self):
            f = np.zeros((8, 8, 3), np.uint8)
            f[..., 0] = self.t
            return f

        def reset(self):
            self.t = 0
            return None

        def step(self, a):
            self.t += 1
            return None

        def close(self):
            pass

    env = RecordVideo(Fake(), video_folder=str(tmp_path / "videos"), step_trigger=lambda s: s == 0, video_length=5)
    env.reset()
    for _ in range(9):
        env.step(None)
    env.close()
    assert len(env.saved) == 1 and os.path.basename(env.saved[0]) == "rl-video-step-0.gif"
    im = Image.open(env.saved[0])
    assert im.n_frames == 5
    with pytest.raises(ValueError):
        RecordVideo(type("E", (), {"render_mode": None})(), video_folder=str(tmp_path))
