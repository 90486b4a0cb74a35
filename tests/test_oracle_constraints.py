"""The constraint set on the oracle (CPU): self-collision, the row budget, and foot priority.

States come from tests/golden/constraint_states.npz (found by tests/golden/gen_constraint_states.py);
the per-substep constraint set is read through the oracle's probe (or_probe_substep).  The same states
are stepped on the HIP kernels in tests/test_gpu_constraints.py, bit-exact against these.
"""

import copy

import numpy as np
import pytest

from _models import constraint_fixture, put_oracle

MAXC, MAXR = 10, 30  # include/allsteps.h AS_MAX_CONTACTS / AS_MAX_ROWS


def _state(orc, name):
    st = orc.state(1)
    put_oracle(st, constraint_fixture(name))
    return st


def test_self_pair_table(orc):
    """walker3d.py:27 self-collision on a robot imported from walker3d.xml: 190 pairs; no pair on one
    weld body or across a joint; torso / butt (contype 1) never meet the waist (contype 2)."""
    m = orc.m
    names, links = m["geom_name"], m["geom_link"]
    pairs = [(int(e) & 255, int(e) >> 8) for e in m["self_pair"][: m["num_self_pairs"]]]
    assert len(pairs) == 190 and pairs == sorted(pairs)
    named = {(names[a], names[b]) for a, b in pairs} | {(names[b], names[a]) for a, b in pairs}
    assert ("torso", "waist") not in named and ("butt", "waist") not in named   # filter bits 1 vs 2
    assert ("torso", "butt") in named and ("right_hand", "left_hand") in named
    assert ("right_hand", "right_larm") not in named      # merged into one weld body
    assert ("right_uarm1", "right_larm") not in named     # elbow joint: parent / child
    assert ("head", "right_uarm1") not in named           # shoulder joint: root / upper arm
    assert ("right_shin1", "right_foot_1") not in named   # ankle
    assert ("right_thigh1", "right_foot_1") in named      # two joints apart: collide
    for a, b in pairs:
        assert links[a] != links[b]


def test_self_contact_arm_torso_impulse(oracle_mod, orc):
    """Forearm folded into the torso, robot in the air: one self-contact, a positive normal impulse,
    and the penetration shrinks; with the pair table emptied the arm stays inside the torso."""
    st = _state(orc, "self_arm")
    p = orc.probe(st)
    assert p["ncontact"] == 1 and p["nself_found"] == 1 and p["stone"][0] == -1 and p["foot"][0] == -1
    assert {int(p["link"][0]), int(p["link2"][0])} == {0, 17}
    assert p["sep"][0] < -0.01 and p["lam_n"][0] > 0.0
    assert p["mask"] == (0, 0)  # self-contacts never reach the foot sensors

    m0 = copy.deepcopy(orc.m)
    m0["num_self_pairs"] = 0
    orc0 = oracle_mod.Oracle(model=m0)
    st0 = _state(orc0, "self_arm")
    act = np.zeros((1, 21), np.float32)
    for _ in range(3):
        orc.physics_step(st, act)
        orc0.physics_step(st0, act)
    p1 = orc.probe(st)
    sep1 = p1["sep"][0] if p1["ncontact"] else np.inf
    assert sep1 > p["sep"][0] + 5e-3, (p["sep"][0], sep1)
    # without the pair the arm keeps (free-fall: no relative motion) its penetration
    q_arm = [orc.m["dof_names"].index(n) for n in ("right_shoulder_x", "right_shoulder_y", "right_shoulder_z",
                                                    "right_elbow")]
    q_init = constraint_fixture("self_arm")["q"][q_arm]
    assert np.abs(st0["q"][q_arm, 0] - q_init).max() < 1e-4
    assert np.abs(st["q"][q_arm, 0] - q_init).max() > 1e-3


def test_budget_keeps_every_limit_row(orc):
    """A fallen robot: more contacts than rows, several joint limits active -- every limit row is kept
    and the contacts fill exactly what the limits leave."""
    st = _state(orc, "fallen")
    p = orc.probe(st)
    assert p["nlim"] >= 3
    assert p["nfound"] > p["ncap"]
    assert p["ncap"] == min(MAXC, (MAXR - p["nlim"]) // 3)
    assert p["ncontact"] == p["ncap"]
    assert 3 * p["ncontact"] + p["nlim"] <= MAXR


def _classes(p, m):
    npri = m["num_priority_geoms"]
    feet_links = set(int(m["geom_link"][g]) for g in range(npri))
    cls = []
    for c in range(p["ncontact"]):
        if p["stone"][c] < 0:
            cls.append(2)
        else:
            cls.append(0 if int(p["link"][c]) in feet_links else 1)
    return cls


def test_feet_first_under_the_cap(orc):
    """More contacts than the budget, a foot pushing on a higher-index stone than another body's
    contact: the kept list is feet first (then other bodies, then self-contacts), the foot's contact
    survives and its (foot, stone) sensor bit fires (allsteps_env.py:421-425 reads it)."""
    st = _state(orc, "crowded")
    p = orc.probe(st)
    assert p["nfound"] > p["ncap"]
    cls = _classes(p, orc.m)
    assert cls == sorted(cls)
    feet = p["foot"] >= 0
    hi = p["stone"][feet].max()
    assert (p["stone"][~feet & (p["stone"] >= 0)] < hi).any()
    f = int(p["foot"][feet & (p["stone"] == hi)][0])
    assert (p["mask"][f] >> hi) & 1
    # within a class: stone-major, ascending
    for c in (0, 1):
        s = [int(p["stone"][i]) for i in range(p["ncontact"]) if cls[i] == c]
        assert s == sorted(s)


@pytest.mark.parametrize("name", ["self_arm", "crowded", "fallen"])
def test_fixture_states_are_valid(orc, name):
    snap = constraint_fixture(name)
    assert abs(np.linalg.norm(snap["root_quat"]) - 1.0) < 1e-5
    assert np.isfinite(np.concatenate([v.astype(np.float64).ravel() for v in snap.values()])).all()


@pytest.mark.parametrize("name", ["fallen", "crowded"])
def test_dropped_contacts_counted(orc, name):
    """The oracle searches every pair past the cap and counts what it cuts (as_step_counters word 3 on
    the device): at least the first substep's found - kept, and the physics-only and full env steps
    agree on it; cutting does not change which contacts are kept (the probe's list is the same)."""
    st = _state(orc, name)
    p = orc.probe(st)
    first = p["nfound"] - p["ncontact"]
    assert first > 0
    st2 = _state(orc, name)
    act = np.zeros((1, 21), np.float32)
    drop = orc.physics_step(st2, act)
    assert drop >= first
    st3 = _state(orc, name)
    st3["idx"][:] = 1
    st3["next"][:] = 2
    orc.env_step(st3, act)
    assert orc.last_dropped == drop


def test_fixture_claims(orc):
    """the committed constraint states are a search result of an earlier oracle
    (tests/golden/gen_constraint_states.py cannot regenerate the same bytes on HEAD's oracle), so the
    generator's acceptance predicates -- the promises of its docstring -- are checked here on the
    committed bytes with HEAD's oracle: the arm penetrates the torso as the only contact; the crowded
    state finds more contacts than the budget and keeps a pushing foot contact on a higher stone than a
    kept non-foot contact; the fallen state finds more contacts than the budget with >= 3 limit rows
    (every one kept: test_budget_keeps_every_limit_row)."""
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import gen_constraint_states as G

    assert G.check(orc) == {"self_arm": True, "crowded": True, "fallen": True}
    p = orc.probe(_state(orc, "crowded"))
    assert p["ncontact"] == p["ncap"] and p["nfound"] > p["ncap"]  # contacts beyond the budget are cut
