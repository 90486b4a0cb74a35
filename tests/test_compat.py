"""The opt-in import shims (allsteps_isaaclab_amd.compat): the reference's own rl_games train / play
scripts run unchanged over this package (north_star "train.py runs unchanged").

The reference scripts are read from /root/reference when present (this container only: the reference
never travels to the GPU box) and executed AS THEY ARE through ``python -m allsteps_isaaclab_amd.compat``.
Without a HIP device they get through every line before the environment -- argument parsing, the
AppLauncher, the rl_games / isaaclab / isaaclab_tasks / hydra imports, the registry cfgs with hydra
overrides, the log dumps (train.py:76-134; play.py:71-111) -- and stop at gym.make with the product's
loud NativeError (no CPU fallback).
"""

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_RLG = "/root/reference/scripts/reinforcement_learning/rl_games"
needs_ref = pytest.mark.skipif(not os.path.isdir(REF_RLG), reason="reference scripts absent (GPU box)")


def _py(code: str, cwd: str, extra_path: str | None = None) -> subprocess.CompletedProcess:
    env = dict(os.environ, PYTHONPATH=os.pathsep.join(p for p in (ROOT, extra_path) if p))
    return subprocess.run([sys.executable, "-c", code], cwd=cwd, env=env, capture_output=True, text=True, timeout=120)


def test_shims_are_opt_in(tmp_path):
    r = _py("import importlib.util as u; print([u.find_spec(m) is None for m in "
            "('isaaclab', 'isaaclab_rl', 'isaaclab_tasks', 'rl_games')])", str(tmp_path))
    assert r.returncode == 0 and r.stdout.strip() == "[True, True, True, True]", r.stdout + r.stderr
    r = _py("from allsteps_isaaclab_amd import compat; compat.install()\n"
            "import isaaclab.app, isaaclab.envs, isaaclab_rl.rl_games, isaaclab_tasks, rl_games.torch_runner\n"
            "from isaaclab_tasks.utils.hydra import hydra_task_config\n"
            "from rl_games.common import env_configurations, vecenv\n"
            "import allsteps_isaaclab_amd.rl_games as R, allsteps_isaaclab_amd._vecenv as V\n"
            "assert R.vecenv is V.vecenv and R.env_configurations is V.env_configurations\n"
            "import gymnasium; print(gymnasium.spec('Allsteps-v0').entry_point)", str(tmp_path))
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip() == "allsteps_isaaclab_amd.envs.allsteps_env:AllstepsEnv"


def test_install_never_shadows_a_real_package(tmp_path):
    fake = tmp_path / "real"
    (fake / "rl_games").mkdir(parents=True)
    (fake / "rl_games" / "__init__.py").write_text("REAL = True\n")
    r = _py("from allsteps_isaaclab_amd import compat; print(compat.install())\n"
            "import rl_games; print(getattr(rl_games, 'REAL', False))", str(tmp_path), extra_path=str(fake))
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == ["['rl_games']", "True"]


def test_hydra_overrides(tmp_path):
    r = _py("from allsteps_isaaclab_amd import compat; compat.install()\n"
            "import sys; sys.argv = ['x', '--headless', 'env.scene.num_envs=128', 'agent.params.config.horizon_length=16',"
            " '--checkpoint', '/tmp/a=b.pth']\n"
            "from isaaclab_tasks.utils.hydra import hydra_task_config\n"
            "@hydra_task_config('Allsteps-v0', 'rl_games_cfg_entry_point')\n"
            "def main(env_cfg, agent_cfg):\n"
            "    print(env_cfg.scene.num_envs, agent_cfg['params']['config']['horizon_length'])\n"
            "main()", str(tmp_path))
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.split() == ["128", "16"]


def test_override_tokens_ignore_flag_values_with_equals():
    """a flag's value containing '=' (a checkpoint path) is not a hydra override."""
    from allsteps_isaaclab_amd.registry import override_tokens

    argv = ["--task", "Allsteps-v0", "--checkpoint", "/tmp/run=3/model.pth", "--log_root", "a=b", "env.scene.num_envs=64",
            "+agent.params.config.minibatch_size=2048", "agent.params.seed=1"]
    assert override_tokens(argv) == ["env.scene.num_envs=64", "+agent.params.config.minibatch_size=2048",
                                     "agent.params.seed=1"]


def _run_reference(script: str, args: list[str], cwd) -> subprocess.CompletedProcess:
    env = dict(os.environ, PYTHONPATH=ROOT, HIP_VISIBLE_DEVICES=os.environ.get("HIP_VISIBLE_DEVICES", ""))
    return subprocess.run([sys.executable, "-m", "allsteps_isaaclab_amd.compat", os.path.join(REF_RLG, script), *args],
                          cwd=str(cwd), env=env, capture_output=True, text=True, timeout=300)


@needs_ref
def test_reference_train_py_runs_unchanged_to_the_env(tmp_path):
    r = _run_reference("train.py", ["--task", "Allsteps-v0", "--headless", "--num_envs", "64", "--max_iterations",
                                    "1", "agent.params.config.minibatch_size=2048"], tmp_path)
    assert r.returncode != 0
    assert "NativeError: AllstepsEnv runs on the HIP backend only" in r.stderr, r.stderr[-3000:]
    runs = list((tmp_path / "logs" / "rl_games" / "allsteps").iterdir())
    assert len(runs) == 1
    params = sorted(p.name for p in (runs[0] / "params").iterdir())
    assert params == ["agent.pkl", "agent.yaml", "env.pkl", "env.yaml"]
    import yaml

    agent = yaml.safe_load((runs[0] / "params" / "agent.yaml").read_text())
    assert agent["params"]["config"]["minibatch_size"] == 2048 and agent["params"]["config"]["max_epochs"] == 1
    env = yaml.safe_load((runs[0] / "params" / "env.yaml").read_text())
    assert env["scene"]["num_envs"] == 64


@needs_ref
def test_reference_play_py_runs_unchanged_to_the_env(tmp_path):
    (tmp_path / "model.pth").write_bytes(b"")
    r = _run_reference("play.py", ["--task", "Allsteps-v0", "--headless", "--num_envs", "16", "--checkpoint",
                                   "model.pth"], tmp_path)
    assert r.returncode != 0
    assert "NativeError: AllstepsEnv runs on the HIP backend only" in r.stderr, r.stderr[-3000:]
    assert "Loading model checkpoint from" in r.stdout or "Loading experiment" in r.stdout


# The shimmed call sequence of the reference train.py (train.py:76-178), run on the device.  The
# reference script itself never travels to the GPU box, so this driver (written here, not copied) makes
# the same calls in the same order through the same import names: hydra_task_config over the registry
# cfgs, gym.make, RlGamesVecEnvWrapper, the vecenv / env_configurations registrations, Runner with
# IsaacAlgoObserver, the a2c_continuous_mirroring builder, load / reset / run.
_DRIVER = '''
import math, os, sys
import gymnasium as gym
from rl_games.common import env_configurations, vecenv
from rl_games.common.algo_observer import IsaacAlgoObserver
from rl_games.torch_runner import Runner
from isaaclab_rl.rl_games import RlGamesGpuEnv, RlGamesVecEnvWrapper
import isaaclab_tasks  # noqa: F401
from isaaclab_tasks.utils.hydra import hydra_task_config
from isaaclab_tasks.direct.allsteps.learning import a2c_ppo_mirroring

@hydra_task_config("Allsteps-v0", "rl_games_cfg_entry_point")
def main(env_cfg, agent_cfg):
    env_cfg.scene.num_envs = 64
    env_cfg.sim.device = "cuda:0"
    agent_cfg["params"]["config"]["max_epochs"] = 1
    env_cfg.seed = agent_cfg["params"]["seed"]
    root = os.path.abspath(os.path.join("logs", "rl_games", agent_cfg["params"]["config"]["name"]))
    agent_cfg["params"]["config"]["train_dir"] = root
    agent_cfg["params"]["config"]["full_experiment_name"] = "gpu_flow"
    rl_device = agent_cfg["params"]["config"]["device"]
    clip_obs = agent_cfg["params"]["env"].get("clip_observations", math.inf)
    clip_actions = agent_cfg["params"]["env"].get("clip_actions", math.inf)
    env = gym.make("Allsteps-v0", cfg=env_cfg, render_mode=None)
    env = RlGamesVecEnvWrapper(env, rl_device, clip_obs, clip_actions)
    vecenv.register("IsaacRlgWrapper", lambda config_name, num_actors, **kw: RlGamesGpuEnv(config_name, num_actors, **kw))
    env_configurations.register("rlgpu", {"vecenv_type": "IsaacRlgWrapper", "env_creator": lambda **kw: env})
    agent_cfg["params"]["config"]["num_actors"] = env.unwrapped.num_envs
    runner = Runner(IsaacAlgoObserver())
    runner.algo_factory.register_builder("a2c_continuous_mirroring", lambda **kw: a2c_ppo_mirroring.A2CAgentSymmetry(**kw))
    runner.load(agent_cfg)
    runner.reset()
    runner.run({"train": True, "play": False, "sigma": None})
    env.close()
    print("FLOW_OK")

main()
'''


@pytest.mark.gpu
def test_shimmed_train_flow_on_gpu(tmp_path):
    """the compat path end to end on the device -- the rl_games.torch_runner shim,
    IsaacAlgoObserver, isaaclab_rl's RlGamesVecEnvWrapper / RlGamesGpuEnv and the mirror-agent builder
    -- one PPO epoch at 64 envs (agent minibatch 64 x 32 steps), and a checkpoint written."""
    script = tmp_path / "flow.py"
    script.write_text(_DRIVER)
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", "allsteps_isaaclab_amd.compat", str(script), "--headless",
                        "agent.params.config.minibatch_size=2048"], cwd=str(tmp_path), env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "FLOW_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])
    ckpts = list((tmp_path / "logs" / "rl_games" / "allsteps" / "gpu_flow" / "nn").glob("*.pth"))
    assert ckpts, "no checkpoint written"
