"""MJCF -> reduced-coordinate model tables for the Allsteps walker.

The reference spawns the robot from ``data/usd/walker3d.usd`` (``isaaclab_assets/robots/walker3d.py:20``),
which is not in the tree; the only model source is ``isaaclab_assets/data/mjcf/walker3d.xml``
(SURVEY.md §0.8, Appendix B).  This module compiles that MJCF into the constant tables the HIP
step kernel and the CPU oracle consume:

* one *link* per hinge joint (a body with k hinges becomes a chain of k links; the first k-1 are
  massless and the last one carries the body's geoms, mass and inertia), plus the floating root;
* bodies without joints (head, torso, hands) are merged into their parent link (fixed joints);
* mass / COM / inertia from geoms at density 1000 (MuJoCo ``inertiafromgeom="true"``);
* joint axis / anchor in the link frame, limits in radians (``compiler angle="degree"``), armature
  from the joint default classes;
* the DOF permutation to the PhysX/cfg DOF order of ``allsteps_env_cfg.py:133-155``.

Run ``python -m allsteps_isaaclab_amd.model.mjcf <walker3d.xml> <out.json>`` to regenerate
``walker3d.json`` (committed; the GPU box has no ``/root/reference``), and
``python -m allsteps_isaaclab_amd.model.mjcf anymal_c.xml anymal_c.json anymal_c`` for the BASELINE C5
quadruped (an authored approximation, ``anymal_c.xml``).
"""

from __future__ import annotations

import json
import math
import sys
import xml.etree.ElementTree as ET

import numpy as np

DENSITY = 1000.0

# PhysX / cfg DOF order: allsteps_env_cfg.py:133-155 (joint_gears comments), consistent with the
# reset indices at allsteps_env.py:505-511.
CFG_DOF_ORDER = [
    "abdomen_z", "abdomen_y",
    "right_shoulder_x", "right_shoulder_y", "right_shoulder_z",
    "left_shoulder_x", "left_shoulder_y", "left_shoulder_z",
    "abdomen_x", "right_elbow", "left_elbow",
    "right_hip_x", "right_hip_y", "right_hip_z",
    "left_hip_x", "left_hip_y", "left_hip_z",
    "right_knee", "left_knee", "right_ankle", "left_ankle",
]
# allsteps_env_cfg.py:133-155
CFG_GEARS = [60, 80, 60, 50, 60, 60, 50, 60, 60, 60, 60, 80, 100, 60, 80, 100, 60, 90, 90, 60, 60]

# Per-model compile options: DOF order, gears, the torso body and the two contact-sensor feet
# (geom_foot 0 / 1), and the bodies whose geoms are ordered first under the contact cap.
WALKER = {"source": "isaaclab_assets/data/mjcf/walker3d.xml", "dof_order": CFG_DOF_ORDER, "gears": CFG_GEARS,
          "torso": "torso", "sensor_feet": ["right_foot", "left_foot"], "contact_first": ["right_foot", "left_foot"]}
# BASELINE C5 quadruped (model/anymal_c.xml, an authored approximation): IsaacLab's ANYmal joint order
# (PhysX breadth-first: all HAA, then HFE, then KFE, legs LF, LH, RF, RH); gear 66.67 so that the
# Allsteps actuation 1.2 * gear * a reaches 80 N m; the four feet carry contact sensors 0..3 (RF, LF, RH,
# LH: the front pair in the walker's two sensor slots).
_LEGS = ["LF", "LH", "RF", "RH"]
ANYMAL_C = {"source": "allsteps_isaaclab_amd/model/anymal_c.xml (authored; the vendor USD is Nucleus-only)",
            "dof_order": [f"{leg}_{j}" for j in ("HAA", "HFE", "KFE") for leg in _LEGS],
            "gears": [80.0 / 1.2] * 12, "torso": "base", "sensor_feet": ["RF_SHANK", "LF_SHANK", "RH_SHANK", "LH_SHANK"],
            "contact_first": [f"{leg}_SHANK" for leg in _LEGS]}


def _floats(s: str | None, n: int | None = None) -> list[float]:
    if s is None:
        return None
    v = [float(x) for x in s.split()]
    if n is not None and len(v) != n:
        raise ValueError(f"expected {n} floats, got {s!r}")
    return v


def quat_to_mat(q) -> np.ndarray:
    w, x, y, z = q
    n = math.sqrt(w * w + x * x + y * y + z * z)
    w, x, y, z = w / n, x / n, y / n, z / n
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
        [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
        [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)],
    ])


def mat_to_quat(R) -> list[float]:
    """(w, x, y, z) of a rotation matrix, w >= 0 (Shepperd's branch on the largest diagonal term)."""
    R = np.asarray(R, float)
    t = np.trace(R)
    if t > 0:
        s = math.sqrt(t + 1.0) * 2
        q = [0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s]
    else:
        i = int(np.argmax(np.diag(R)))
        j, k = (i + 1) % 3, (i + 2) % 3
        s = math.sqrt(1.0 + R[i, i] - R[j, j] - R[k, k]) * 2
        q = [0.0] * 4
        q[0] = (R[k, j] - R[j, k]) / s
        q[1 + i] = 0.25 * s
        q[1 + j] = (R[j, i] + R[i, j]) / s
        q[1 + k] = (R[k, i] + R[i, k]) / s
    q = np.array(q)
    q = q / np.linalg.norm(q)
    return (q if q[0] >= 0 else -q).tolist()


def _frame_from_z(d: np.ndarray) -> np.ndarray:
    """Rotation whose third column is the unit vector d."""
    z = d / np.linalg.norm(d)
    a = np.array([1.0, 0.0, 0.0]) if abs(z[0]) < 0.9 else np.array([0.0, 1.0, 0.0])
    x = np.cross(a, z)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    return np.stack([x, y, z], axis=1)


def geom_mass_inertia(g: dict) -> tuple[float, np.ndarray, np.ndarray]:
    """(mass, com, inertia about com) of one geom in its body frame (MuJoCo inertiafromgeom)."""
    r = g["radius"]
    if g["type"] == "sphere":
        m = DENSITY * 4.0 / 3.0 * math.pi * r ** 3
        return m, np.array(g["p0"]), np.eye(3) * (0.4 * m * r * r)
    p0, p1 = np.array(g["p0"]), np.array(g["p1"])
    d = p1 - p0
    h = float(np.linalg.norm(d))  # cylinder height
    m_sph = DENSITY * 4.0 * math.pi * r ** 3 / 3.0
    m_cyl = DENSITY * math.pi * r * r * h
    m = m_sph + m_cyl
    ixx = m_cyl * (3 * r * r + h * h) / 12.0 + m_sph * (2 * r * r / 5.0 + h * h / 4.0 + 3 * h * r / 8.0)
    izz = m_cyl * r * r / 2.0 + m_sph * 2 * r * r / 5.0
    R = _frame_from_z(d)
    I = R @ np.diag([ixx, ixx, izz]) @ R.T
    return m, 0.5 * (p0 + p1), I


def combine(parts):
    """Sum (mass, com, inertia-about-com) triples with the parallel-axis theorem."""
    m = sum(p[0] for p in parts)
    if m == 0.0:
        return 0.0, np.zeros(3), np.zeros((3, 3))
    c = sum(p[0] * p[1] for p in parts) / m
    I = np.zeros((3, 3))
    for mi, ci, Ii in parts:
        r = ci - c
        I += Ii + mi * (np.dot(r, r) * np.eye(3) - np.outer(r, r))
    return m, c, I


class _Defaults:
    def __init__(self, root: ET.Element):
        self.joint = {}
        self.geom = {}
        self.classes = {}
        d = root.find("default")
        if d is not None:
            j = d.find("joint")
            if j is not None:
                self.joint = dict(j.attrib)
            g = d.find("geom")
            if g is not None:
                self.geom = dict(g.attrib)
            for cls in d.findall("default"):
                cj = cls.find("joint")
                self.classes[cls.get("class")] = dict(cj.attrib) if cj is not None else {}

    def joint_attr(self, j: ET.Element, key: str, fallback=None):
        if key in j.attrib:
            return j.get(key)
        cls = j.get("class")
        if cls is not None and key in self.classes.get(cls, {}):
            return self.classes[cls][key]
        return self.joint.get(key, fallback)

    def geom_attr(self, g: ET.Element, key: str, fallback=None):
        return g.get(key, self.geom.get(key, fallback))


def compile_mjcf(path: str, opts: dict | None = None) -> dict:
    opts = opts or WALKER
    root = ET.parse(path).getroot()
    comp = root.find("compiler")
    deg = comp is None or comp.get("angle", "degree") == "degree"
    defaults = _Defaults(root)
    world = root.find("worldbody")
    base = world.find("body")

    links: list[dict] = []
    # every MJCF body in document order: the link whose frame carries it, its frame in that link's frame,
    # and the mass / COM of its own geoms (body frame) -- the ArticulationData body views (ring 2)
    bodies: list[dict] = []

    def add_body_entry(body: ET.Element, link: int, R_b: np.ndarray, p_b: np.ndarray) -> None:
        parts = [geom_mass_inertia(g) for g in parse_geoms(body, np.eye(3), np.zeros(3))]
        m, c, _ = combine(parts) if parts else (0.0, np.zeros(3), np.zeros((3, 3)))
        bodies.append({"name": body.get("name"), "link": link, "offset_pos": np.asarray(p_b, float).tolist(),
                       "offset_quat": mat_to_quat(R_b), "mass": float(m), "com": np.asarray(c, float).tolist()})

    def parse_geoms(body: ET.Element, R_off: np.ndarray, p_off: np.ndarray) -> list[dict]:
        """Geoms of `body`, expressed in a frame where body-frame point x maps to R_off x + p_off."""
        out = []
        for g in body.findall("geom"):
            gtype = g.get("type", "sphere")
            size = _floats(g.get("size"))
            # MuJoCo collision filter bits (default 1 / 1; walker3d.xml:5 sets 3 / 3, torso / butt 1, waist 2)
            filt = {"contype": int(defaults.geom_attr(g, "contype", "1")),
                    "conaffinity": int(defaults.geom_attr(g, "conaffinity", "1"))}
            if gtype == "sphere":
                p = np.array(_floats(g.get("pos", "0 0 0"), 3))
                out.append({"name": g.get("name"), "type": "sphere", "radius": size[0],
                            "p0": (R_off @ p + p_off).tolist(), "p1": (R_off @ p + p_off).tolist(), **filt})
            elif gtype == "capsule":
                ft = _floats(g.get("fromto"), 6)
                a, b = np.array(ft[:3]), np.array(ft[3:])
                out.append({"name": g.get("name"), "type": "capsule", "radius": size[0],
                            "p0": (R_off @ a + p_off).tolist(), "p1": (R_off @ b + p_off).tolist(), **filt})
            else:
                raise ValueError(f"unsupported geom type {gtype}")
        return out

    def body_offset(body: ET.Element):
        pos = np.array(_floats(body.get("pos", "0 0 0"), 3))
        quat = _floats(body.get("quat", "1 0 0 0"), 4)
        return pos, quat

    def add_body(body: ET.Element, parent_link: int, R_acc: np.ndarray, p_acc: np.ndarray):
        """Add links for `body`. (R_acc, p_acc) maps body-frame points into the frame of
        `parent_link` when the body has no joints (merged fixed bodies)."""
        pos, quat = body_offset(body)
        joints = body.findall("joint")
        if not joints:
            # fixed body: merge geoms into parent_link, recurse with accumulated transform
            R_b = R_acc @ quat_to_mat(quat)
            p_b = R_acc @ pos + p_acc
            add_body_entry(body, parent_link, R_b, p_b)
            links[parent_link]["geoms"].extend(parse_geoms(body, R_b, p_b))
            links[parent_link]["merged"].append(body.get("name"))
            for child in body.findall("body"):
                add_body(child, parent_link, R_b, p_b)
            return
        if not np.allclose(R_acc, np.eye(3)) or not np.allclose(p_acc, 0):
            raise ValueError("jointed body under a merged fixed body is not supported")
        qn = np.array(quat) / np.linalg.norm(quat)
        prev = parent_link
        for k, j in enumerate(joints):
            if j.get("type", "hinge") != "hinge":
                raise ValueError("only hinge joints below the free root are supported")
            axis = np.array(_floats(j.get("axis", "0 0 1"), 3))
            axis = axis / np.linalg.norm(axis)
            rng = _floats(defaults.joint_attr(j, "range"), 2)
            if deg:
                rng = [math.radians(rng[0]), math.radians(rng[1])]
            link = {
                "name": j.get("name"),
                "body": body.get("name"),
                "parent": prev,
                "offset_pos": pos.tolist() if k == 0 else [0.0, 0.0, 0.0],
                "offset_quat": qn.tolist() if k == 0 else [1.0, 0.0, 0.0, 0.0],
                "joint": {
                    "name": j.get("name"),
                    "axis": axis.tolist(),
                    "anchor": _floats(j.get("pos", "0 0 0"), 3),
                    "range": rng,
                    "armature": float(defaults.joint_attr(j, "armature", "0")),
                    "damping_mjcf": float(defaults.joint_attr(j, "damping", "0")),
                    "stiffness_mjcf": float(defaults.joint_attr(j, "stiffness", "0")),
                },
                "geoms": [],
                "merged": [],
                "is_body_frame": k == len(joints) - 1,
            }
            links.append(link)
            prev = len(links) - 1
        add_body_entry(body, prev, np.eye(3), np.zeros(3))
        links[prev]["geoms"].extend(parse_geoms(body, np.eye(3), np.zeros(3)))
        for child in body.findall("body"):
            add_body(child, prev, np.eye(3), np.zeros(3))

    # floating root
    if base.find("freejoint") is None:
        raise ValueError("expected a freejoint root")
    pos, quat = body_offset(base)
    links.append({"name": "root", "body": base.get("name"), "parent": -1,
                  "offset_pos": [0.0, 0.0, 0.0], "offset_quat": [1.0, 0.0, 0.0, 0.0],
                  "joint": None, "geoms": [], "merged": [], "is_body_frame": True})
    add_body_entry(base, 0, np.eye(3), np.zeros(3))
    links[0]["geoms"].extend(parse_geoms(base, np.eye(3), np.zeros(3)))
    for child in base.findall("body"):
        add_body(child, 0, np.eye(3), np.zeros(3))

    # mass properties
    for L in links:
        parts = [geom_mass_inertia(g) for g in L["geoms"]]
        m, c, I = combine(parts) if parts else (0.0, np.zeros(3), np.zeros((3, 3)))
        L["mass"] = float(m)
        L["com"] = c.tolist()
        L["inertia"] = I.tolist()

    # body -> link of its frame
    body_link = {}
    for i, L in enumerate(links):
        if L["is_body_frame"]:
            body_link[L["body"]] = i
        for mb in L["merged"]:
            body_link.setdefault(mb, i)

    # DOF permutation: link i (i>=1) carries internal hinge dof i-1
    jname_to_link = {L["joint"]["name"]: i for i, L in enumerate(links) if L["joint"] is not None}
    cfg_to_link = [jname_to_link[n] for n in opts["dof_order"]]

    out = {
        "source": opts["source"],
        "density": DENSITY,
        "links": links,
        "body_link": body_link,
        "cfg_dof_order": list(opts["dof_order"]),
        "cfg_dof_link": cfg_to_link,
        "gears": list(opts["gears"]),
        "mjcf_base_pos": pos.tolist(),
        "total_mass": float(sum(L["mass"] for L in links)),
        "bodies": bodies,
    }
    if opts is not WALKER:  # the walker's json predates these keys; load_model defaults to them
        out.update(torso=opts["torso"], sensor_feet=opts["sensor_feet"], contact_first=opts["contact_first"])
    return out


def main(argv: list[str]) -> None:
    src, dst = argv[1], argv[2]
    model = compile_mjcf(src, ANYMAL_C if len(argv) > 3 and argv[3] == "anymal_c" else WALKER)
    with open(dst, "w") as f:
        json.dump(model, f, indent=1)
    print(f"wrote {dst}: {len(model['links'])} links, total mass {model['total_mass']:.3f} kg")


if __name__ == "__main__":
    main(sys.argv)
