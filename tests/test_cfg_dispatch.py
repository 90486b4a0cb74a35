"""Host-side cfg plumbing: the as_task_t table is dispatched on the cfg type (one helper for the HIP
path and the oracle), the C5 robot's self-collision switch reaches the model, and the video wrapper
fails cleanly when it has no env."""

import copy
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def test_task_table_is_shared_and_dispatched_on_type():
    import oracle as O

    from allsteps_isaaclab_amd import _native
    from allsteps_isaaclab_amd.envs.allsteps_env_cfg import AllstepsEnvCfg
    from allsteps_isaaclab_amd.envs.anymal_c_stones_env_cfg import AnymalCStonesEnvCfg
    from allsteps_isaaclab_amd.model import ANYMAL_C_JSON, load_model

    walker, quad = load_model(), load_model(ANYMAL_C_JSON)
    for cfg, m in ((AllstepsEnvCfg(), walker), (AnymalCStonesEnvCfg(), quad)):
        a, b = _native.make_task(cfg, m["dof_names"]), O.make_task(cfg, m["dof_names"])
        assert bytes(a) == bytes(b)  # the same struct image on both sides
    q = _native.make_task(AnymalCStonesEnvCfg(), quad["dof_names"])
    assert q.num_steps == AnymalCStonesEnvCfg().num_steps
    assert q.step_dt == pytest.approx(1 / 200 * 4)

    class NotACfg:  # has the walker's field names, but is neither cfg: no silent defaults
        alive_reward_scale = 2.0
        num_steps = 20

    for make in (_native.make_task, O.make_task):
        with pytest.raises(TypeError):
            make(NotACfg(), walker["dof_names"])


def test_record_video_without_env_raises_attribute_error():
    from allsteps_isaaclab_amd.envs.record_video import RecordVideo

    class NoRender:
        render_mode = None

    with pytest.raises(ValueError):
        RecordVideo(NoRender(), "/tmp/unused_video_dir")
    bare = RecordVideo.__new__(RecordVideo)  # as copy / pickle create it: no __init__
    with pytest.raises(AttributeError):
        bare.step_trigger_missing  # noqa: B018
    with pytest.raises(AttributeError):
        copy.copy(bare).anything  # noqa: B018


@pytest.mark.gpu
def test_anymal_self_collision_switch_reaches_the_model():
    from allsteps_isaaclab_amd.envs.anymal_c_stones_env import AnymalCStonesEnv
    from allsteps_isaaclab_amd.envs.anymal_c_stones_env_cfg import AnymalCStonesEnvCfg

    cfg = AnymalCStonesEnvCfg()
    cfg.scene.num_envs = 64
    env = AnymalCStonesEnv(cfg)
    assert env.model["num_self_pairs"] == 66
    env.close()
    cfg.robot.enabled_self_collisions = False
    env = AnymalCStonesEnv(cfg)
    assert env.model["num_self_pairs"] == 0
    env.step(__import__("torch").zeros(64, 12, device="cuda:0"))
    env.close()
