"""``render_mode="rgb_array"`` for the direct-workflow envs: a software rasteriser of one env's robot and
stepping stones (the reference renders through Isaac Sim's RTX viewport, absent offline; play.py's
``--video`` records what ``env.render()`` returns, ``play.py:111-127``).

The frame is a side view (world x right, z up) of env ``env_id`` with a top view (x right, y up) inset:
stones as boxes, the robot's sphere / capsule geoms as discs / stadiums.  Link poses come from a host
forward kinematics of the device state (root pose + joint angles) over the model tables -- the same
local-transform composition as the k_step FK (``csrc/allsteps_kernels.hip`` fk), evaluated in float64 for
one env per frame.  Rendering is a viewer, not part of the stepped path: it reads the state and draws.
"""

from __future__ import annotations

import numpy as np


def _quat_mat(q) -> np.ndarray:
    w, x, y, z = (float(v) for v in q)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def _axis_angle(a, t) -> np.ndarray:
    a = np.asarray(a, np.float64)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + np.sin(t) * K + (1 - np.cos(t)) * K @ K


def link_poses(model: dict, root_pos, root_quat, q_cfg) -> tuple[np.ndarray, np.ndarray]:
    """World rotation (nl, 3, 3) and origin (nl, 3) of every link.  q_cfg: joint angles in cfg dof order."""
    nl = int(model["num_links"])
    qi = np.zeros(nl)
    for k in range(int(model["num_hinges"])):
        qi[int(model["cfg_dof_link"][k])] = float(q_cfg[k])
    R = np.zeros((nl, 3, 3))
    p = np.zeros((nl, 3))
    R[0], p[0] = _quat_mat(root_quat), np.asarray(root_pos, np.float64)
    for i in range(1, nl):
        par = int(model["parent"][i])
        Roff = _quat_mat(model["offset_quat"][i])
        Rj = _axis_angle(model["axis"][i], qi[i])
        an = np.asarray(model["anchor"][i], np.float64)
        Rl = Roff @ Rj
        pl = Roff @ (an - Rj @ an) + np.asarray(model["offset_pos"][i], np.float64)
        R[i] = R[par] @ Rl
        p[i] = p[par] + R[par] @ pl
    return R, p


def geom_segments(model: dict, R: np.ndarray, p: np.ndarray) -> list[tuple[np.ndarray, np.ndarray, float]]:
    """(end a, end b, radius) of every geom in world coordinates (a sphere: a == b)."""
    out = []
    for g in range(int(model["num_geoms"])):
        l = int(model["geom_link"][g])
        a = p[l] + R[l] @ np.asarray(model["geom_p0"][g], np.float64)
        b = a if int(model["geom_type"][g]) == 0 else p[l] + R[l] @ np.asarray(model["geom_p1"][g], np.float64)
        out.append((a, b, float(model["geom_radius"][g])))
    return out


def render_frame(model: dict, root_pos, root_quat, q_cfg, stones, stone_half, target: int | None = None,
                 size: tuple[int, int] = (640, 360)) -> np.ndarray:
    """(H, W, 3) uint8 frame: side view over x-z, a top-view inset over x-y.  stones: (S, 3) centres."""
    from PIL import Image, ImageDraw

    W, H = size
    img = Image.new("RGB", (W, H), (235, 238, 242))
    d = ImageDraw.Draw(img)
    R, p = link_poses(model, root_pos, root_quat, q_cfg)
    segs = geom_segments(model, R, p)
    cx, cz = float(root_pos[0]), float(root_pos[2])
    scale = H / 3.0  # 3 m of height in view

    def side(x, z):
        return (W * 0.5 + (x - cx) * scale, H * 0.62 - (z - max(cz - 1.0, 0.0) - 0.6) * scale)

    hx, hy, hz = (float(v) for v in stone_half)
    for k, c in enumerate(np.asarray(stones)):
        x0, y0 = side(c[0] - hx, c[2] + hz)
        x1, y1 = side(c[0] + hx, c[2] - hz)
        d.rectangle([x0, y0, x1, y1], fill=(200, 120, 60) if k == target else (150, 150, 160), outline=(90, 90, 100))
    for a, b, r in segs:
        pa, pb = side(a[0], a[2]), side(b[0], b[2])
        w = max(int(2 * r * scale), 1)
        d.line([pa, pb], fill=(40, 90, 170), width=w)
        for q in (pa, pb):
            d.ellipse([q[0] - r * scale, q[1] - r * scale, q[0] + r * scale, q[1] + r * scale], fill=(40, 90, 170))
    # top view inset (upper right): x right, y up, 4 m x 2 m around the root
    iw, ih, ts = W // 3, H // 3, (W // 3) / 4.0
    ox, oy = W - iw - 8, 8
    d.rectangle([ox, oy, ox + iw, oy + ih], fill=(250, 250, 252), outline=(120, 120, 130))

    def top(x, y):
        return (ox + iw * 0.5 + (x - cx) * ts, oy + ih * 0.5 - (y - float(root_pos[1])) * ts)

    for k, c in enumerate(np.asarray(stones)):
        x0, y0 = top(c[0] - hx, c[1] + hy)
        x1, y1 = top(c[0] + hx, c[1] - hy)
        if x1 < ox or x0 > ox + iw:
            continue
        d.rectangle([max(x0, ox), max(y0, oy), min(x1, ox + iw), min(y1, oy + ih)],
                    fill=(200, 120, 60) if k == target else (170, 170, 180))
    for a, b, r in segs:
        d.line([top(a[0], a[1]), top(b[0], b[1])], fill=(40, 90, 170), width=max(int(2 * r * ts), 1))
    return np.asarray(img, np.uint8)
