"""Small physics models and fixture plumbing shared by the oracle (CPU) and HIP (GPU) known-answer tests.

The HIP step kernel is compiled for 27 generalized velocities (the walker: 6 + 21 hinges) and 18 (the
C5 quadruped), so a small test model (a pendulum, a free sphere) runs on BOTH sides padded to 21 hinges
with inert dummy links: parent = root, COM on the hinge axis through the root origin (no gravity
torque), 1 g, no geoms, limits far outside any reachable angle.  Their only effect is a few grams of
extra root mass.
"""

from __future__ import annotations

import copy
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
STONE_TOP = 0.225 / 2


def _blank_walker_tables():
    from allsteps_isaaclab_amd.model import load_model

    return copy.deepcopy(load_model())


def padded_model(links: list[dict], geoms: list[dict], nh_total: int = 21) -> dict:
    """Model tables (the load_model dict) from explicit links (link 0 = root) and geoms, padded with
    dummy hinge links to `nh_total` hinges.  A link: mass, com (3), inertia (xx, yy, zz); hinge links
    also parent, offset (3), axis (3), lower, upper.  A geom: link, type (0 sphere / 1 capsule),
    radius, p0, p1, foot."""
    m = _blank_walker_tables()
    L = list(links)
    while len(L) < nh_total + 1:
        L.append({"parent": 0, "offset": (0.0, 0.0, 0.0), "axis": (1.0, 0.0, 0.0), "mass": 1e-3,
                  "com": (0.0, 0.0, 0.0), "inertia": (1e-5, 1e-5, 1e-5), "lower": -50.0, "upper": 50.0})
    nl = len(L)
    m["num_links"], m["num_hinges"] = nl, nl - 1
    for key in ("parent", "offset_pos", "axis", "anchor", "mass", "com", "inertia", "armature", "lower", "upper",
                "gear"):
        m[key][...] = 0
    m["offset_quat"][...] = 0
    m["offset_quat"][:, 0] = 1.0
    m["parent"][0] = -1
    for i, l in enumerate(L):
        m["mass"][i] = l["mass"]
        m["com"][i] = l["com"]
        m["inertia"][i, :3] = l["inertia"]
        if i > 0:
            m["parent"][i] = l["parent"]
            m["offset_pos"][i] = l["offset"]
            m["axis"][i] = l["axis"]
            m["lower"][i], m["upper"][i] = l["lower"], l["upper"]
    m["cfg_dof_link"][...] = 0
    m["cfg_dof_link"][: nl - 1] = np.arange(1, nl)
    m["num_geoms"] = len(geoms)
    for key in ("geom_link", "geom_type", "geom_radius", "geom_p0", "geom_p1"):
        m[key][...] = 0
    m["geom_foot"][...] = -1
    for g, d in enumerate(geoms):
        m["geom_link"][g] = d["link"]
        m["geom_type"][g] = d["type"]
        m["geom_radius"][g] = d["radius"]
        m["geom_p0"][g] = d["p0"]
        m["geom_p1"][g] = d.get("p1", d["p0"])
        m["geom_foot"][g] = d.get("foot", -1)
    m["num_priority_geoms"] = 0
    m["num_self_pairs"] = 0
    m["self_pair"][...] = 0
    m["torso_link"] = 0
    m["foot_link"] = np.zeros(2, np.int32)
    m["total_mass"] = float(sum(l["mass"] for l in L))
    return m


def sphere_model(r: float = 0.1) -> tuple[dict, float]:
    """One free sphere (radius r, density 1000) on the root, its geom wired to contact sensor 0."""
    mass = 1000.0 * 4.0 / 3.0 * np.pi * r ** 3
    root = {"mass": mass, "com": (0.0, 0.0, 0.0), "inertia": (0.4 * mass * r * r,) * 3}
    return padded_model([root], [{"link": 0, "type": 0, "radius": r, "p0": (0.0, 0.0, 0.0), "foot": 0}]), mass


# the pendulum (modelled on test_articulation.py:1342-1456 "single_joint" + gravity): a 10 t base
# standing on three small spheres on a stone (in effect fixed), a massless arm of length PEND_L from a
# hinge about x at y = +0.3 from the base (past the stone's edge) to a 1 kg bob
PEND_L = 0.5
PEND_M = 1.0
PEND_ROOT = (1.5, 0.2, STONE_TOP + 0.05 + 0.02)  # tripod sphere bottoms on stone 2's top face


def pendulum_model() -> dict:
    root = {"mass": 1.0e4, "com": (0.0, 0.0, 0.0), "inertia": (1.0e4, 1.0e4, 1.0e4)}
    arm = {"parent": 0, "offset": (0.0, 0.3, 0.0), "axis": (1.0, 0.0, 0.0), "mass": PEND_M,
           "com": (0.0, 0.0, -PEND_L), "inertia": (1e-6, 1e-6, 1e-6), "lower": -50.0, "upper": 50.0}
    feet = [(0.1, 0.0, -0.05), (-0.1, 0.08, -0.05), (-0.1, -0.08, -0.05)]
    geoms = [{"link": 0, "type": 0, "radius": 0.02, "p0": p, "foot": 0} for p in feet]
    return padded_model([root, arm], geoms)


def level0_stones(n: int) -> np.ndarray:
    st = np.zeros((60, n), np.float32)
    for k in range(20):
        st[3 * k] = 0.75 * k
    return st


# ---------------------------------------------------------------------------------- walker fixtures

def constraint_fixture(name: str) -> dict:
    """One env's state (tests/golden/constraint_states.npz, gen_constraint_states.py) as [rows] arrays."""
    z = np.load(os.path.join(HERE, "golden", "constraint_states.npz"), allow_pickle=False)
    return {k.split("/", 1)[1]: z[k] for k in z.files if k.startswith(name + "/")}


def put_oracle(st, snap: dict, e: int = 0) -> None:
    for k, v in snap.items():
        a = st[k]
        if a.ndim > 1:
            a[:, e] = v
        else:
            a[e] = v[0]


class GpuPhysics:
    """A physics-only HIP handle for any model (as_physics_step through the C-ABI; no task logic),
    with its SoA state as torch tensors on cuda:0 -- the GPU side of the known-answer tests."""

    def __init__(self, model: dict, n: int, seed: int = 42):
        import torch

        from allsteps_isaaclab_amd import _native
        from allsteps_isaaclab_amd.envs.allsteps_env_cfg import AllstepsEnvCfg

        self.n = n
        self.state = {}
        for name, rows, t in _native.STATE_LAYOUT:
            self.state[name] = torch.zeros((rows, n) if rows > 1 else (n,),
                                           dtype=torch.float32 if t == "f" else torch.int32, device="cuda:0")
        self.state["curriculum"] = torch.zeros(1, dtype=torch.int32, device="cuda:0")
        self.state["root_quat"][0] = 1.0
        self.native = _native.NativeEnv(n, model, AllstepsEnvCfg(), self.state, seed, 0)

    def load_oracle(self, st) -> None:
        """copy an oracle state (same n) to the device"""
        import torch

        for k, v in self.state.items():
            if k == "curriculum":
                continue
            a = np.ascontiguousarray(st[k]).reshape(v.shape)
            v.copy_(torch.from_numpy(a.view(np.int32) if a.dtype == np.uint32 else a))

    def step(self, actions) -> None:
        import torch

        a = torch.as_tensor(actions, dtype=torch.float32, device="cuda:0").contiguous()
        self.native.physics_step(a, stream=torch.cuda.current_stream().cuda_stream)

    def get(self) -> dict:
        import torch

        torch.cuda.synchronize()
        return {k: v.cpu().numpy() for k, v in self.state.items()}

    def close(self) -> None:
        self.native.close()
