"""``RecordVideo`` -- the gymnasium wrapper play.py puts around the env for ``--video`` (play.py:117-127):
from the step ``step_trigger`` accepts, record ``video_length`` frames of ``env.render()`` and write them to
``video_folder``.  gymnasium encodes MP4 through moviepy / ffmpeg, which this image lacks; the frames are
written as an animated GIF (PIL) with the env's step period, ``<name_prefix>-step-<n>.gif``.
Every other attribute is the wrapped env's."""

from __future__ import annotations

import os


class RecordVideo:
    def __init__(self, env, video_folder: str, episode_trigger=None, step_trigger=None, video_length: int = 0,
                 name_prefix: str = "rl-video", fps: int | None = None, disable_logger: bool = True, **_):
        if getattr(env, "render_mode", None) != "rgb_array":
            raise ValueError("RecordVideo needs an env made with render_mode='rgb_array'")
        self.env = env
        self.video_folder = os.path.abspath(video_folder)
        os.makedirs(self.video_folder, exist_ok=True)
        self.step_trigger = step_trigger or (lambda step: step == 0)
        self.video_length = int(video_length) if video_length else 200
        self.name_prefix = name_prefix
        dt = float(getattr(getattr(env, "unwrapped", env), "step_dt", 1.0 / 60.0))
        self.fps = int(fps) if fps else max(1, round(1.0 / dt))
        self.step_id = 0
        self.frames: list = []
        self.recording = False
        self.saved: list[str] = []

    def __getattr__(self, name):  # everything else is the env's
        # only reached for names not on the wrapper; before __init__ has set `env` (a failed __init__,
        # copy / pickle) there is nothing to forward to, and looking `env` up here would recurse
        if name == "env" or "env" not in self.__dict__:
            raise AttributeError(name)
        return getattr(self.env, name)

    @property
    def unwrapped(self):
        return self.env.unwrapped

    def _capture(self) -> None:
        if not self.recording and self.step_trigger(self.step_id):
            self.recording, self.frames, self._start = True, [], self.step_id
        if self.recording:
            self.frames.append(self.env.render())
            if len(self.frames) >= self.video_length:
                self._save()

    def _save(self) -> None:
        from PIL import Image

        if not self.frames:
            return
        path = os.path.join(self.video_folder, f"{self.name_prefix}-step-{self._start}.gif")
        imgs = [Image.fromarray(f) for f in self.frames]
        imgs[0].save(path, save_all=True, append_images=imgs[1:], duration=int(1000 / self.fps), loop=0)
        self.saved.append(path)
        self.recording, self.frames = False, []

    def reset(self, *args, **kwargs):
        out = self.env.reset(*args, **kwargs)
        self._capture()
        return out

    def step(self, action):
        out = self.env.step(action)
        self.step_id += 1
        self._capture()
        return out

    def close(self):
        if self.recording:
            self._save()
        return self.env.close()
