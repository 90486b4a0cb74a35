"""Generate tests/golden/constraint_states.npz: walker states that exercise the constraint budget.

The fixtures are states of OUR oracle (not reference outputs -- PhysX is absent), found
by a seeded search and committed so that the CPU and GPU constraint tests start from the same bytes.
The committed bytes ARE the fixture: the search was run on the round-2 oracle, and the oracle's
arithmetic has changed since (round 4: FK by pointer jumping), so a regeneration on a later oracle
finds other states -- equally valid ones, meeting the same acceptance predicates below.  Those
predicates (`self_arm_ok`, `crowded_ok`, `fallen_ok`) are what the fixture promises; they are checked
on the committed states on HEAD's oracle by tests/test_oracle_constraints.py::test_fixture_claims, and
`python tests/golden/gen_constraint_states.py --check` runs the same check.

  self_arm    -- the robot high in the air (no stone within reach), right arm folded so that the
                 forearm / hand penetrates the torso: exactly one contact, a self-contact between
                 the right forearm link and the root link (walker3d.py:27 enabled_self_collisions);
  crowded     -- a natural rollout state whose first substep finds more contacts than the budget
                 keeps, with a foot contact on a higher-index stone than some non-foot contact that
                 is kept and pushes (lam_n > 0), i.e. a state where a stone-major emission order would
                 have let other bodies crowd out the foot (VERDICT r01 "what's missing" 2);
  fallen      -- a natural rollout state with more contacts than the budget AND several active
                 joint-limit rows (all of which must be kept).

    python tests/golden/gen_constraint_states.py            # search and (re)write the fixture
    python tests/golden/gen_constraint_states.py --check    # the committed states meet the predicates
"""

from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402  (test infrastructure)

FIELDS = list(O.OracleState.FIELDS_F) + list(O.OracleState.FIELDS_I) + list(O.OracleState.FIELDS_U)


def snapshot(st, e) -> dict:
    out = {}
    for k in FIELDS:
        a = st[k]
        out[k] = np.ascontiguousarray(a[..., e]) if a.ndim > 1 else np.array([a[e]])
    return out


def level0(st):
    for k in range(20):
        st["stones"][3 * k + 0][:] = 0.75 * k
        st["stones"][3 * k + 2][:] = 0.0


def self_arm_ok(orc, p) -> bool:
    """Exactly one contact, a self-contact between the root link and the right forearm, penetrating."""
    m = orc.m
    elbow = m["cfg_dof_link"][m["dof_names"].index("right_elbow")]
    return bool(p["ncontact"] == 1 and p["link2"][0] >= 0 and p["sep"][0] < -0.01
                and {int(p["link"][0]), int(p["link2"][0])} == {0, elbow})


def crowded_ok(p) -> bool:
    """More contacts found than the budget keeps, and a kept foot contact on a higher-index stone than
    some kept non-foot stone contact, pushing (lam_n > 0): the state in which a stone-major emission
    order would have let other bodies crowd out the foot."""
    if p["nfound"] <= p["ncap"]:
        return False
    feet = p["foot"] >= 0
    others = ~feet & (p["stone"] >= 0)
    if not feet.any() or not others.any():
        return False
    hi_foot = p["stone"][feet].max()
    return bool(hi_foot > p["stone"][others].min() and (p["lam_n"][feet & (p["stone"] == hi_foot)] > 0).any())


def fallen_ok(p) -> bool:
    """More contacts found than the budget keeps AND at least three active joint-limit rows."""
    return bool(p["nfound"] > p["ncap"] and p["nlim"] >= 3)


def find_self_arm(orc) -> dict:
    m = orc.m
    names = m["dof_names"]
    link_of = {nm: m["cfg_dof_link"][k] for k, nm in enumerate(names)}
    arm = ["right_shoulder_x", "right_shoulder_y", "right_shoulder_z", "right_elbow"]
    lim = {nm: (m["lower"][link_of[nm]], m["upper"][link_of[nm]]) for nm in arm}
    rng = np.random.default_rng(7)
    st = orc.state(1)
    level0(st)
    for _ in range(20000):
        st["q"][:] = 0.0
        for nm in arm:
            lo, hi = lim[nm]
            st["q"][names.index(nm), 0] = rng.uniform(lo + 0.05, hi - 0.05)
        st["root_pos"][:, 0] = [0.0, 0.0, 5.0]
        if self_arm_ok(orc, orc.probe(st, 0)):
            return snapshot(st, 0)
    raise RuntimeError("no self-contact pose found")


def find_rollout_states(orc, n=512, steps=400) -> tuple[dict, dict]:
    st = orc.state(n)
    level0(st)
    orc.reset_all(st, seed=11)
    rng = np.random.default_rng(11)
    crowded = fallen = None
    for _ in range(steps):
        orc.env_step(st, rng.uniform(-1, 1, (n, 21)).astype(np.float32))
        for e in range(n):
            p = orc.probe(st, e)
            if crowded is None and crowded_ok(p):
                crowded = snapshot(st, e)
            if fallen is None and fallen_ok(p):
                fallen = snapshot(st, e)
        if crowded is not None and fallen is not None:
            return crowded, fallen
    raise RuntimeError(f"not found: crowded {crowded is not None}, fallen {fallen is not None}")


def check(orc, path=None) -> dict:
    """Each committed state against its acceptance predicate on this oracle: {name: bool}."""
    z = np.load(path or os.path.join(HERE, "constraint_states.npz"), allow_pickle=False)
    out = {}
    for name, ok in (("self_arm", lambda p: self_arm_ok(orc, p)), ("crowded", crowded_ok), ("fallen", fallen_ok)):
        st = orc.state(1)
        for k in z.files:
            if k.startswith(name + "/"):
                a, v = st[k.split("/", 1)[1]], z[k]
                if a.ndim > 1:
                    a[:, 0] = v
                else:
                    a[0] = v[0]
        out[name] = ok(orc.probe(st, 0))
    return out


def main():
    O.build()
    orc = O.Oracle()
    if "--check" in sys.argv:
        res = check(orc)
        print(res)
        sys.exit(0 if all(res.values()) else 1)
    out = {}
    for name, snap in [("self_arm", find_self_arm(orc)), *zip(("crowded", "fallen"), find_rollout_states(orc))]:
        for k, v in snap.items():
            out[f"{name}/{k}"] = v
    path = os.path.join(HERE, "constraint_states.npz")
    np.savez(path, **out)
    print(f"wrote {path}: {sorted({k.split('/')[0] for k in out})}")


if __name__ == "__main__":
    main()
