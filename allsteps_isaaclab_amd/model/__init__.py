"""Model tables for the Allsteps walker (compiled from the reference MJCF by ``mjcf.py``).

``load_model()`` flattens ``walker3d.json`` into the fixed-size arrays of the C-ABI model struct
(``include/allsteps.h`` :c:type:`as_model_t`): links in topological (parent-before-child) order,
link 0 the floating root, link i >= 1 carrying hinge dof i-1; geoms ordered feet first
(``num_priority_geoms``): their stone contacts are emitted before every other geom's, so the contact cap
(``AS_MAX_CONTACTS``) never drops a foot contact in favour of another body's; and the self-collision
pair table (``self_pair``).
"""

from __future__ import annotations

import json
import os

import numpy as np

MAX_LINKS = 32
MAX_GEOMS = 32
MAX_SELF_PAIRS = 256  # include/allsteps.h AS_MAX_SELF_PAIRS
MAX_BODIES = 32  # include/allsteps.h AS_MAX_BODIES
HERE = os.path.dirname(os.path.abspath(__file__))
WALKER_JSON = os.path.join(HERE, "walker3d.json")
ANYMAL_C_JSON = os.path.join(HERE, "anymal_c.json")  # BASELINE C5 quadruped (authored approximation)


def load_json(path: str = WALKER_JSON) -> dict:
    with open(path) as f:
        return json.load(f)


def load_model(path: str = WALKER_JSON) -> dict:
    """Return the flat model tables (numpy, float32 / int32) used by the kernels and the oracle."""
    j = load_json(path)
    links = j["links"]
    nl = len(links)
    if nl > MAX_LINKS:
        raise ValueError(f"model has {nl} links > {MAX_LINKS}")
    m = {
        "num_links": nl,
        "num_hinges": nl - 1,
        "parent": np.full(MAX_LINKS, -1, np.int32),
        "offset_pos": np.zeros((MAX_LINKS, 3), np.float32),
        "offset_quat": np.zeros((MAX_LINKS, 4), np.float32),
        "axis": np.zeros((MAX_LINKS, 3), np.float32),
        "anchor": np.zeros((MAX_LINKS, 3), np.float32),
        "mass": np.zeros(MAX_LINKS, np.float32),
        "com": np.zeros((MAX_LINKS, 3), np.float32),
        "inertia": np.zeros((MAX_LINKS, 6), np.float32),
        "armature": np.zeros(MAX_LINKS, np.float32),
        "lower": np.zeros(MAX_LINKS, np.float32),
        "upper": np.zeros(MAX_LINKS, np.float32),
        "cfg_dof_link": np.zeros(MAX_LINKS, np.int32),
        "gear": np.zeros(MAX_LINKS, np.float32),
    }
    m["offset_quat"][:, 0] = 1.0
    for i, L in enumerate(links):
        if L["parent"] >= i:
            raise ValueError("links must be in topological order")
        m["parent"][i] = L["parent"]
        m["offset_pos"][i] = L["offset_pos"]
        m["offset_quat"][i] = L["offset_quat"]
        m["mass"][i] = L["mass"]
        m["com"][i] = L["com"]
        I = np.array(L["inertia"])
        m["inertia"][i] = [I[0, 0], I[1, 1], I[2, 2], I[0, 1], I[0, 2], I[1, 2]]
        if L["joint"] is not None:
            jt = L["joint"]
            m["axis"][i] = jt["axis"]
            m["anchor"][i] = jt["anchor"]
            m["armature"][i] = jt["armature"]
            m["lower"][i], m["upper"][i] = jt["range"]
    m["cfg_dof_link"][: nl - 1] = j["cfg_dof_link"]
    m["gear"][: nl - 1] = j["gears"]

    # geoms: feet first (the walker: right then left; the quadruped: its four feet), then every other
    # geom in link order; the two sensor feet get geom_foot 0 / 1 (contact-sensor bitmasks)
    bl = j["body_link"]
    foot_link = [bl[b] for b in j.get("sensor_feet", ["right_foot", "left_foot"])]
    first = [bl[b] for b in j.get("contact_first", ["right_foot", "left_foot"])]
    geoms = []
    for i, L in enumerate(links):
        for g in L["geoms"]:
            foot = foot_link.index(i) if i in foot_link else -1
            geoms.append((0 if i in first else 1, first.index(i) if i in first else 0, i, foot, g))
    geoms.sort(key=lambda t: (t[0], t[1], t[2]))
    geoms = [(t[0], t[3], t[2], t[4]) for t in geoms]
    if len(geoms) > MAX_GEOMS:
        raise ValueError("too many geoms")
    m["num_geoms"] = len(geoms)
    m["geom_link"] = np.zeros(MAX_GEOMS, np.int32)
    m["geom_type"] = np.zeros(MAX_GEOMS, np.int32)
    m["geom_foot"] = np.full(MAX_GEOMS, -1, np.int32)
    m["geom_radius"] = np.zeros(MAX_GEOMS, np.float32)
    m["geom_p0"] = np.zeros((MAX_GEOMS, 3), np.float32)
    m["geom_p1"] = np.zeros((MAX_GEOMS, 3), np.float32)
    m["geom_name"] = []
    for k, (_, foot, li, g) in enumerate(geoms):
        m["geom_link"][k] = li
        m["geom_type"][k] = 0 if g["type"] == "sphere" else 1
        m["geom_foot"][k] = foot
        m["geom_radius"][k] = g["radius"]
        m["geom_p0"][k] = g["p0"]
        m["geom_p1"][k] = g["p1"]
        m["geom_name"].append(g["name"])
    m["num_priority_geoms"] = sum(1 for t in geoms if t[0] == 0)
    m["self_pair"], m["num_self_pairs"] = self_collision_pairs(links, [(t[2], t[3]) for t in geoms])
    m["torso_link"] = bl[j.get("torso", "torso")]
    m["foot_link"] = np.array(foot_link[:2], np.int32)  # body_pos FK slots (as_model_t.foot_link[2])
    m["sensor_links"] = list(foot_link)
    m["link_names"] = [L["name"] for L in links]
    # the MJCF bodies (document order) for the ArticulationData body views (ring 2, as_body_state):
    # the link whose frame carries each body, the body frame in it, the body's own COM (body frame)
    bodies = j.get("bodies") or [{"name": b, "link": li, "offset_pos": [0.0] * 3, "offset_quat": [1.0, 0.0, 0.0, 0.0],
                                   "mass": 0.0, "com": [0.0] * 3} for b, li in bl.items()]
    if len(bodies) > MAX_BODIES:
        raise ValueError(f"model has {len(bodies)} bodies > {MAX_BODIES}")
    m["body_names"] = [b["name"] for b in bodies]
    m["num_bodies"] = len(bodies)
    m["body_link"] = np.zeros(MAX_BODIES, np.int32)
    m["body_offset_pos"] = np.zeros((MAX_BODIES, 3), np.float32)
    m["body_offset_quat"] = np.zeros((MAX_BODIES, 4), np.float32)
    m["body_offset_quat"][:, 0] = 1.0
    m["body_com"] = np.zeros((MAX_BODIES, 3), np.float32)
    for k, b in enumerate(bodies):
        m["body_link"][k] = b["link"]
        m["body_offset_pos"][k] = b["offset_pos"]
        m["body_offset_quat"][k] = b["offset_quat"]
        m["body_com"][k] = b["com"]
    m["dof_names"] = list(j["cfg_dof_order"])
    m["total_mass"] = float(j["total_mass"])
    return m


def self_collision_pairs(links: list, geoms: list) -> tuple[np.ndarray, int]:
    """Geom pairs (g1 < g2, ascending) the robot collides with itself: ``walker3d.py:27``
    ``enabled_self_collisions=True`` on a robot imported from ``walker3d.xml``.

    A pair is kept when its geoms sit on different weld bodies (a jointed MJCF body together with the
    joint-less bodies merged into it: head / torso on the root, the hands on the forearms) that are not
    parent and child (PhysX never collides the two links of a joint; MuJoCo's parent filter), and when
    the MJCF filter bits admit it: ``(contype1 & conaffinity2) | (contype2 & conaffinity1)``
    (``walker3d.xml:5,34,41,44``: torso / butt carry 1, waist 2, everything else 3).
    Packed as ``g1 | g2 << 8`` (``include/allsteps.h`` ``as_model_t.self_pair``)."""
    def weld_parent(i: int):
        body = links[i]["body"]
        while links[i]["parent"] >= 0 and links[links[i]["parent"]]["body"] == body:
            i = links[i]["parent"]
        p = links[i]["parent"]
        return links[p]["body"] if p >= 0 else None

    out = []
    for g1 in range(len(geoms)):
        for g2 in range(g1 + 1, len(geoms)):
            (l1, a), (l2, b) = geoms[g1], geoms[g2]
            w1, w2 = links[l1]["body"], links[l2]["body"]
            if w1 == w2 or weld_parent(l1) == w2 or weld_parent(l2) == w1:
                continue
            if not ((a.get("contype", 1) & b.get("conaffinity", 1)) | (b.get("contype", 1) & a.get("conaffinity", 1))):
                continue
            out.append(g1 | (g2 << 8))
    if len(out) > MAX_SELF_PAIRS:
        raise ValueError(f"{len(out)} self-collision pairs > {MAX_SELF_PAIRS}")
    arr = np.zeros(MAX_SELF_PAIRS, np.int32)
    arr[: len(out)] = out
    return arr, len(out)


def joint_limits_cfg(m: dict) -> np.ndarray:
    """(21, 2) joint position limits in cfg/PhysX dof order (ArticulationData.joint_pos_limits)."""
    nh = m["num_hinges"]
    lim = np.zeros((nh, 2), np.float32)
    for k in range(nh):
        li = m["cfg_dof_link"][k]
        lim[k] = (m["lower"][li], m["upper"][li])
    return lim
