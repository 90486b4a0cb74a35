"""Host-side surface of the drop-in, on CPU: mirror augmentation, the rl_games VecEnv wrapper, the
task registry / configs, and the loud failure of the product path without a gfx950 device.

Fixtures (tests/golden/gen_golden.py, produced by importing the reference modules):
  mirror.npz      -- get_symmetric_states_rl_games / _rsl_rl (allsteps_env.py:570-660)
  rlg_wrapper.npz -- RlGamesVecEnvWrapper.step I/O (isaaclab_rl/rl_games.py:238-312) on a fake env
"""

import math
import types

import numpy as np
import pytest
import torch

from allsteps_isaaclab_amd import registry
from allsteps_isaaclab_amd.envs.allsteps_env import get_symmetric_states_rl_games, get_symmetric_states_rsl_rl
from allsteps_isaaclab_amd.envs.allsteps_env_cfg import AllstepsEnvCfg
from allsteps_isaaclab_amd.envs.direct_rl_env import DirectRLEnv
from allsteps_isaaclab_amd.envs.spaces import Box
from allsteps_isaaclab_amd.model.mjcf import CFG_DOF_ORDER
from allsteps_isaaclab_amd.rl_games import RlGamesGpuEnv, RlGamesVecEnvWrapper, env_configurations

from conftest import golden


def _mirror_env():
    cfg = AllstepsEnvCfg()
    J = CFG_DOF_ORDER.index
    uw = types.SimpleNamespace(
        right_body_indices=torch.tensor([J(x) for x in cfg.right_body_names]),
        left_body_indices=torch.tensor([J(x) for x in cfg.left_body_names]),
        negation_body_indices=torch.tensor([J(x) for x in cfg.negation_body_names]),
        observation_space=types.SimpleNamespace(shape=(64, 59)),
        action_space=types.SimpleNamespace(shape=(64, 21)),
    )
    return types.SimpleNamespace(unwrapped=uw, device="cpu")


def test_mirror_rl_games_matches_reference():
    g = golden("mirror")
    obs, act, mus = (torch.from_numpy(g[k]) for k in ("mir_obs", "mir_act", "mir_mus"))
    o, a, m = get_symmetric_states_rl_games(obs, act, _mirror_env(), False, mus)
    np.testing.assert_array_equal(o.numpy(), g["mir_out_obs"])
    np.testing.assert_array_equal(a.numpy(), g["mir_out_act"])
    np.testing.assert_array_equal(m.numpy(), g["mir_out_mus"])


def test_mirror_rsl_rl_matches_reference():
    g = golden("mirror")
    o, a = get_symmetric_states_rsl_rl(torch.from_numpy(g["mir_obs"]), torch.from_numpy(g["mir_act"]), _mirror_env())
    np.testing.assert_array_equal(o.numpy(), g["mir_rsl_obs"])
    np.testing.assert_array_equal(a.numpy(), g["mir_rsl_act"])


def test_mirror_is_an_involution():
    g = golden("mirror")
    obs = torch.from_numpy(g["mir_obs"])
    o, _ = get_symmetric_states_rsl_rl(obs, None, _mirror_env())
    back, _ = get_symmetric_states_rsl_rl(o[64:], None, _mirror_env())
    torch.testing.assert_close(back[64:], obs, rtol=0, atol=0)


class _FakeEnv(DirectRLEnv):
    """Replays the fixture's env outputs; records the actions it was stepped with."""

    def __init__(self, g):
        self.num_envs = 16
        self._device = torch.device("cpu")
        self.render_mode = None
        self.cfg = types.SimpleNamespace(is_finite_horizon=False)
        self.single_observation_space = {"policy": Box(-math.inf, math.inf, (59,))}
        self.single_action_space = Box(-math.inf, math.inf, (21,))
        self.g = g
        self.seen = None
        self.obs_seq = [g["rlg_env_obs"], g["rlg_clip_env_obs"]]  # the env's observations, call by call

    def step(self, a):
        self.seen = a.clone()
        g = self.g
        obs = self.obs_seq.pop(0)
        return ({"policy": torch.from_numpy(obs)}, torch.from_numpy(g["rlg_env_rew"]),
                torch.from_numpy(g["rlg_env_term"]), torch.from_numpy(g["rlg_env_trunc"]), {})

    def close(self):
        pass


def test_rl_games_wrapper_step_matches_reference():
    g = golden("rlg_wrapper")
    fe = _FakeEnv(g)
    w = RlGamesVecEnvWrapper(fe, "cpu", math.inf, 1.0)
    o, r, d, ex = w.step(torch.from_numpy(g["rlg_actions"]))
    np.testing.assert_array_equal(fe.seen.numpy(), g["rlg_seen_actions"])
    np.testing.assert_array_equal(o.numpy(), g["rlg_obs"])
    np.testing.assert_array_equal(r.numpy(), g["rlg_rew"])
    np.testing.assert_array_equal(d.numpy(), g["rlg_dones"])
    np.testing.assert_array_equal(ex["time_outs"].numpy(), g["rlg_time_outs"])
    w2 = RlGamesVecEnvWrapper(fe, "cpu", 10.0, 0.5)
    o2, _, _, _ = w2.step(torch.from_numpy(g["rlg_actions"]))
    np.testing.assert_array_equal(o2.numpy(), g["rlg_clip_obs10"])
    np.testing.assert_array_equal(fe.seen.numpy(), g["rlg_seen_actions_05"])


def test_rl_games_wrapper_spaces_and_env_info():
    fe = _FakeEnv(golden("rlg_wrapper"))
    w = RlGamesVecEnvWrapper(fe, "cpu", 10.0, 1.0)
    info = w.get_env_info()
    assert info["observation_space"].shape == (59,) and info["action_space"].shape == (21,)
    assert float(info["observation_space"].high.max()) == 10.0 and float(info["action_space"].low.min()) == -1.0
    assert info["state_space"] is None and w.rlg_num_states == 0
    assert w.get_number_of_agents() == 1 and w.num_envs == 16
    env_configurations.register("rlgpu_test", {"vecenv_type": "IsaacRlgWrapper", "env_creator": lambda **kw: w})
    ge = RlGamesGpuEnv("rlgpu_test", 16)
    assert ge.get_env_info()["action_space"].shape == (21,)


def test_rl_games_wrapper_rejects_foreign_env():
    with pytest.raises(ValueError):
        RlGamesVecEnvWrapper(types.SimpleNamespace(unwrapped=object()), "cpu", 1.0, 1.0)


def test_registry_and_cfg():
    s = registry.spec("Allsteps-v0")
    assert s.entry_point.endswith("allsteps_env:AllstepsEnv") and s.disable_env_checker
    cfg = registry.load_cfg_from_registry("Allsteps-v0", "env_cfg_entry_point")
    assert isinstance(cfg, AllstepsEnvCfg)
    assert (cfg.decimation, cfg.action_space, cfg.observation_space) == (4, 21, 59)
    assert abs(cfg.sim.dt - 1 / 240) < 1e-12 and cfg.episode_length_s == 15.0
    agent = registry.load_cfg_from_registry("Allsteps-v0", "rl_games_cfg_entry_point")
    assert agent["params"]["config"]["horizon_length"] == 32
    with pytest.raises(KeyError):
        registry.spec("Nope-v0")


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-device path")
def test_make_fails_loudly_without_device():
    from allsteps_isaaclab_amd._native import NativeError

    cfg = AllstepsEnvCfg()
    cfg.scene.num_envs = 4
    with pytest.raises((NativeError, RuntimeError)):
        registry.make("Allsteps-v0", cfg=cfg)
