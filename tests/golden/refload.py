"""Load the reference Allsteps task module with stub Isaac modules (golden-fixture generation only).

Used ONLY by ``gen_golden.py`` in the build container, where ``/root/reference`` exists.  Nothing
here is imported by the product, the GPU tests, ``smoke()`` or ``bench.py``.  The recipe is the one
SURVEY.md §8(c) verified: the Isaac/Omniverse packages are replaced by empty stub modules in
``sys.modules``; ``isaaclab/utils/math.py`` and ``allsteps_env.py`` are the reference's own files,
loaded as text from their paths.  Physics is absent; the callers feed synthetic robot/sensor data.
"""

from __future__ import annotations

import importlib.util
import sys
import types

REF = "/root/reference/source"
MATH_PY = f"{REF}/isaaclab/isaaclab/utils/math.py"
ENV_PY = f"{REF}/isaaclab_tasks/isaaclab_tasks/direct/allsteps/allsteps_env.py"
RLG_PY = f"{REF}/isaaclab_rl/isaaclab_rl/rl_games.py"


def _mod(name: str, **attrs) -> types.ModuleType:
    m = types.ModuleType(name)
    m.__path__ = []  # behave like a package for submodule imports
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


class _Any:
    def __init__(self, *a, **k):
        pass

    def __getattr__(self, name):
        return _Any()

    def __call__(self, *a, **k):
        return _Any()


class DirectRLEnvStub:
    """Stand-in for isaaclab.envs.DirectRLEnv: only the pieces AllstepsEnv calls via super()."""

    def _reset_idx(self, env_ids):  # direct_rl_env.py:563-584 (scene.reset + ep_len = 0)
        self.episode_length_buf[env_ids] = 0


def load_math():
    if "isaaclab.utils.math" in sys.modules and hasattr(sys.modules["isaaclab.utils.math"], "quat_apply"):
        return sys.modules["isaaclab.utils.math"]
    _mod("isaaclab")
    _mod("isaaclab.utils")
    spec = importlib.util.spec_from_file_location("isaaclab.utils.math", MATH_PY)
    m = importlib.util.module_from_spec(spec)
    sys.modules["isaaclab.utils.math"] = m
    spec.loader.exec_module(m)
    sys.modules["isaaclab.utils"].math = m
    return m


def load_allsteps_env():
    math_mod = load_math()
    gym = _mod("gymnasium", spaces=_Any())
    _ = gym
    sim = _mod("isaaclab.sim", DomeLightCfg=_Any)
    sys.modules["isaaclab"].sim = sim
    _mod("isaaclab.sim.spawners")
    _mod("isaaclab.sim.spawners.from_files", GroundPlaneCfg=_Any, spawn_ground_plane=_Any())
    _mod("isaaclab.assets", Articulation=_Any, RigidObject=_Any, RigidObjectCollection=_Any)
    _mod("isaaclab.envs", DirectRLEnv=DirectRLEnvStub)
    _mod("isaaclab.markers", VisualizationMarkers=_Any)
    _mod("isaaclab.sensors", ContactSensor=_Any)
    _mod("isaaclab_rl")
    _mod("isaaclab_rl.rsl_rl")
    _mod("isaaclab_rl.rsl_rl.vecenv_wrapper", RslRlVecEnvWrapper=_Any)
    _mod("isaaclab_rl.rl_games", RlGamesVecEnvWrapper=_Any)
    _mod("isaaclab_tasks")
    _mod("isaaclab_tasks.direct")
    _mod("isaaclab_tasks.direct.allsteps")
    _mod("isaaclab_tasks.direct.allsteps.allsteps_env_cfg", AllstepsEnvCfg=_Any)
    name = "isaaclab_tasks.direct.allsteps.allsteps_env"
    spec = importlib.util.spec_from_file_location(name, ENV_PY)
    m = importlib.util.module_from_spec(spec)
    m.__package__ = "isaaclab_tasks.direct.allsteps"
    sys.modules[name] = m
    spec.loader.exec_module(m)
    return m, math_mod


def load_rl_games_wrapper(direct_env_cls):
    """Load the reference RlGamesVecEnvWrapper with gym/gymnasium/rl_games stubbed."""

    class Box:
        def __init__(self, low, high, shape=None, dtype=None):
            self.low, self.high, self.shape = low, high, tuple(shape) if shape is not None else None

    spaces = types.SimpleNamespace(Box=Box)
    gym = _mod("gym", spaces=spaces)
    _mod("gym.spaces", Box=Box)
    gym.spaces = spaces
    g2 = sys.modules.get("gymnasium") or _mod("gymnasium")
    g2.spaces = spaces
    _mod("rl_games")
    _mod("rl_games.common")
    _mod("rl_games.common.env_configurations", configurations={})
    _mod("rl_games.common.vecenv", IVecEnv=object)
    sys.modules["rl_games.common"].env_configurations = sys.modules["rl_games.common.env_configurations"]
    envs = sys.modules.get("isaaclab.envs") or _mod("isaaclab.envs")
    envs.DirectRLEnv = direct_env_cls
    envs.ManagerBasedRLEnv = type("ManagerBasedRLEnv", (), {})
    envs.VecEnvObs = dict
    name = "isaaclab_rl.rl_games_ref"
    spec = importlib.util.spec_from_file_location(name, RLG_PY)
    m = importlib.util.module_from_spec(spec)
    sys.modules[name] = m
    spec.loader.exec_module(m)
    return m, Box
