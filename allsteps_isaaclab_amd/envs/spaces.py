"""Gym spaces: ``gymnasium.spaces`` when installed, else a minimal Box with the same surface.

The reference builds its spaces with ``gymnasium.spaces.Box(-inf, inf, shape)``
(``isaaclab/envs/utils/spaces.py:31-32``) and batches them with ``gym.vector.utils.batch_space``.
"""

from __future__ import annotations

import numpy as np

try:  # pragma: no cover - depends on the image
    import gymnasium as _gym

    Box = _gym.spaces.Box
    Dict = _gym.spaces.Dict
    HAVE_GYMNASIUM = True
except Exception:  # gymnasium is not installed in this image
    HAVE_GYMNASIUM = False

    class Box:  # noqa: D101 - mirrors gymnasium.spaces.Box
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.shape = tuple(shape) if shape is not None else np.shape(low)
            self.dtype = np.dtype(dtype)
            self.low = np.full(self.shape, low, self.dtype) if np.isscalar(low) else np.asarray(low, self.dtype)
            self.high = np.full(self.shape, high, self.dtype) if np.isscalar(high) else np.asarray(high, self.dtype)

        def sample(self):
            lo = np.where(np.isfinite(self.low), self.low, -1.0)
            hi = np.where(np.isfinite(self.high), self.high, 1.0)
            return np.random.uniform(lo, hi).astype(self.dtype)

        def contains(self, x) -> bool:
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

        def __repr__(self):
            return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"

        def __eq__(self, other):
            return isinstance(other, Box) and self.shape == other.shape and np.array_equal(self.low, other.low) \
                and np.array_equal(self.high, other.high)

    class Dict(dict):  # noqa: D101 - mirrors gymnasium.spaces.Dict (mapping of spaces)
        pass


def batch_box(space: Box, n: int) -> Box:
    """gym.vector.utils.batch_space for a Box."""
    low = np.broadcast_to(space.low, (n,) + space.shape)
    high = np.broadcast_to(space.high, (n,) + space.shape)
    return Box(low=np.array(low), high=np.array(high), shape=(n,) + space.shape, dtype=space.dtype)
