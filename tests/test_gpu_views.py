"""Ring-2 views off the hot path: ``robot.data.body_*`` for every MJCF body through
the ``as_body_state`` HIP kernel, and the foot sensors' ``force_matrix_w``.

Checked against an independent float64 numpy forward kinematics of the model tables (positions and
orientations) and, for the velocities, against finite differences of that FK along the state's own
velocity (root linear / angular velocity, qd); the torso / feet rows against the state's body_pos bit for
bit; the flag-valued force matrix against the contact masks the task uses.
"""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _quat_mat(q):
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def _axis_angle(a, t):
    a = np.asarray(a, float)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + np.sin(t) * K + (1 - np.cos(t)) * K @ K


def _fk_bodies(m, root_pos, root_quat, q_cfg):
    """float64 FK: world pose of every body (link walk in topological order)."""
    nl = m["num_links"]
    qi = np.zeros(nl)
    for k in range(m["num_hinges"]):
        qi[m["cfg_dof_link"][k]] = q_cfg[k]
    R0 = _quat_mat(root_quat)
    R = [None] * nl
    p = [None] * nl
    R[0], p[0] = R0, np.zeros(3)
    for i in range(1, nl):
        par = m["parent"][i]
        Roff = _quat_mat(np.asarray(m["offset_quat"][i], float))
        Rj = _axis_angle(m["axis"][i], qi[i])
        an = np.asarray(m["anchor"][i], float)
        A = Roff @ Rj
        t = Roff @ (an - Rj @ an) + np.asarray(m["offset_pos"][i], float)
        R[i] = R[par] @ A
        p[i] = p[par] + R[par] @ t
    pos, rot = [], []
    for b in range(m["num_bodies"]):
        L = m["body_link"][b]
        pos.append(np.asarray(root_pos, float) + p[L] + R[L] @ np.asarray(m["body_offset_pos"][b], float))
        rot.append(R[L] @ _quat_mat(np.asarray(m["body_offset_quat"][b], float)))
    return np.array(pos), np.array(rot)


def _quat_mul(a, b):
    w1, x1, y1, z1 = a
    w2, x2, y2, z2 = b
    return np.array([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                     w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2])


@pytest.fixture(scope="module")
def env():
    from allsteps_isaaclab_amd.envs.allsteps_env import AllstepsEnv
    from allsteps_isaaclab_amd.envs.allsteps_env_cfg import AllstepsEnvCfg

    cfg = AllstepsEnvCfg()
    cfg.scene.num_envs = 256
    cfg.sim.device = "cuda:0"
    e = AllstepsEnv(cfg)
    e.reset()
    g = torch.Generator(device="cuda:0").manual_seed(3)
    for _ in range(40):
        e.step(torch.rand(256, 21, device="cuda:0", generator=g) * 2 - 1)
    torch.cuda.synchronize()
    yield e
    e.close()


def test_body_names_and_shapes(env):
    d = env.robot.data
    assert len(d.body_names) == 17 and d.body_names[0] == "walker3d"
    assert {"torso", "right_foot", "left_foot", "head", "right_hand", "left_hand", "pelvis"} <= set(d.body_names)
    for v in (d.body_pos_w, d.body_lin_vel_w, d.body_ang_vel_w):
        assert v.shape == (256, 17, 3)
    assert d.body_quat_w.shape == (256, 17, 4)
    assert d.body_state_w.shape == (256, 17, 13) and d.body_link_state_w.shape == (256, 17, 13)
    # the task's own lookups (allsteps_env.py:87-88) resolve into these views
    assert env.foot_indices == [d.body_names.index("right_foot"), d.body_names.index("left_foot")]


def test_task_bodies_equal_state_body_pos_bit_for_bit(env):
    """torso / right_foot / left_foot rows: the step's own FK of the final pose (state body_pos)."""
    d = env.robot.data
    bp = env.state["body_pos"].view(3, 3, -1).permute(2, 0, 1)
    idx = [d.body_names.index(x) for x in ("torso", "right_foot", "left_foot")]
    assert torch.equal(d.body_pos_w[:, idx], bp)


def test_body_poses_match_float64_fk(env):
    m = env.model
    d = env.robot.data
    pos, quat = d.body_pos_w.cpu().numpy(), d.body_quat_w.cpu().numpy()
    st = {k: env.state[k].cpu().numpy() for k in ("root_pos", "root_quat", "q")}
    for e in range(0, 256, 17):
        p_ref, R_ref = _fk_bodies(m, st["root_pos"][:, e], st["root_quat"][:, e], st["q"][:, e])
        np.testing.assert_allclose(pos[e], p_ref, atol=2e-5)
        for b in range(17):
            np.testing.assert_allclose(_quat_mat(quat[e, b].astype(np.float64)), R_ref[b], atol=2e-5)
            assert quat[e, b, 0] >= 0.0 and abs(np.linalg.norm(quat[e, b]) - 1.0) < 1e-5


def test_body_velocities_are_the_derivative_of_fk(env):
    """Frame and COM velocities against a central difference of the float64 FK along the state's velocity:
    root COM velocity (root_lin) / angular velocity (root_ang) and qd."""
    m = env.model
    d = env.robot.data
    ls = d.body_link_state_w.cpu().numpy()
    bs = d.body_state_w.cpu().numpy()
    st = {k: env.state[k].cpu().numpy().astype(np.float64) for k in ("root_pos", "root_quat", "q", "qd", "root_lin",
                                                                      "root_ang")}
    h = 1e-6
    com_b = np.asarray(m["body_com"][:17], float)
    for e in range(0, 256, 23):
        rp, rq, q, qd = st["root_pos"][:, e], st["root_quat"][:, e], st["q"][:, e], st["qd"][:, e]
        w0, vc0 = st["root_ang"][:, e], st["root_lin"][:, e]
        c0 = _quat_mat(rq) @ np.asarray(m["com"][0], float)
        vO = vc0 - np.cross(w0, c0)  # the root origin's velocity

        def pose(s):
            th = np.linalg.norm(w0) * s
            dq = np.concatenate([[np.cos(th / 2)], np.sin(th / 2) * w0 / max(np.linalg.norm(w0), 1e-300)])
            return _fk_bodies(m, rp + vO * s, _quat_mul(dq, rq), q + qd * s)

        (p1, R1), (p0, R0) = pose(h), pose(-h)
        v_frame = (p1 - p0) / (2 * h)
        c1 = p1 + np.einsum("bij,bj->bi", R1, com_b)
        c0b = p0 + np.einsum("bij,bj->bi", R0, com_b)
        v_com = (c1 - c0b) / (2 * h)
        scale = 1.0 + np.abs(v_frame).max()
        np.testing.assert_allclose(ls[e, :, 7:10], v_frame, atol=2e-3 * scale)
        np.testing.assert_allclose(bs[e, :, 7:10], v_com, atol=2e-3 * scale)
        # angular velocity: dR/dt R^T = [w]x
        for b in range(17):
            W = (R1[b] - R0[b]) / (2 * h) @ ((R1[b] + R0[b]) / 2).T
            w_ref = np.array([W[2, 1] - W[1, 2], W[0, 2] - W[2, 0], W[1, 0] - W[0, 1]]) / 2
            np.testing.assert_allclose(ls[e, b, 10:13], w_ref, atol=2e-3 * (1 + np.abs(w_ref).max()))


def test_foot_sensor_force_matrix_is_the_task_flag(env):
    """force_matrix_w (flag-valued): ||F|| > EPSILON exactly where the state's contact mask has the stone
    bit -- the test allsteps_env.py:421-425 applies; the unfiltered sensor has none (as the reference)."""
    from allsteps_isaaclab_amd import _native

    m = env.state["contact_mask"].long()
    for foot, sens in ((0, env.sensor_right), (1, env.sensor_left)):
        fm = sens.data.force_matrix_w
        assert fm.shape == (256, 1, 20, 3)
        flag = torch.linalg.vector_norm(fm, dim=-1).squeeze(1) > 1e-4
        bits = ((m[foot].unsqueeze(1) >> torch.arange(20, device=m.device)) & 1).bool()
        assert torch.equal(flag, bits)
    assert env.sensor.data.force_matrix_w is None
    with pytest.raises(_native.NativeError):
        env.sensor_left.data.net_forces_w


def test_quadruped_body_views_match_float64_fk():
    """The C5 env serves the same views for its 13 bodies (AnymalCStonesEnv.robot.data)."""
    from allsteps_isaaclab_amd.envs.anymal_c_stones_env import AnymalCStonesEnv
    from allsteps_isaaclab_amd.envs.anymal_c_stones_env_cfg import AnymalCStonesEnvCfg

    cfg = AnymalCStonesEnvCfg()
    cfg.scene.num_envs = 128
    cfg.sim.device = "cuda:0"
    env = AnymalCStonesEnv(cfg)
    env.reset()
    g = torch.Generator(device="cuda:0").manual_seed(5)
    for _ in range(20):
        env.step(torch.rand(128, 12, device="cuda:0", generator=g) * 2 - 1)
    torch.cuda.synchronize()
    d, m = env.robot.data, env.model
    assert d.body_names[0] == "base" and len(d.body_names) == 13
    assert d.body_pos_w.shape == (128, 13, 3) and d.joint_pos.shape == (128, 12)
    assert torch.equal(d.default_joint_pos[0], env.default_joint_pos)
    pos = d.body_pos_w.cpu().numpy()
    st = {k: env.state[k].cpu().numpy() for k in ("root_pos", "root_quat", "q")}
    for e in range(0, 128, 13):
        p_ref, _ = _fk_bodies(m, st["root_pos"][:, e], st["root_quat"][:, e], st["q"][:, e])
        np.testing.assert_allclose(pos[e], p_ref, atol=2e-5)
    env.close()
