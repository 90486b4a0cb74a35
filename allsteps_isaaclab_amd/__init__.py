"""allsteps_isaaclab_amd -- MI355X-native Allsteps-v0 (stepping-stone humanoid) environment.

``import allsteps_isaaclab_amd`` registers ``Allsteps-v0`` (as ``import isaaclab_tasks`` does in
the reference).  The step runs in ``liballsteps_hip.so`` (HIP, gfx950); see ``include/allsteps.h``.
"""

from . import registry  # noqa: F401  (registers Allsteps-v0)
from .registry import make, register  # noqa: F401

__all__ = ["make", "register", "registry"]
