"""Constraint-budget sizing: how many contacts / joint-limit rows a substep needs.

Builds a statistics variant of the oracle (-DOR_STATS, contact storage 64) in /tmp, runs the full
env step (physics + task, natural resets) on random U(-1, 1) actions from reset, and prints per
substep the histograms of contacts found before the cap, active limit rows, self-contacts found and
contacts kept under AS_MAX_CONTACTS / AS_MAX_ROWS, plus how often the cap dropped a contact.

    python scripts/contact_stats.py [num_envs] [steps] [level]
"""

from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402  (test infrastructure: statistics only)


def build_stats_lib() -> str:
    out = "/tmp/liballsteps_oracle_stats.so"
    src = os.path.join(ROOT, "oracle")
    subprocess.run(["gcc", "-O2", "-mfma", "-fPIC", "-std=c11", "-ffp-contract=off", "-shared", "-DOR_STATS",
                    "-DOR_MAX_CONTACTS=64", "-o", out, os.path.join(src, "task.c"), os.path.join(src, "physics.c"),
                    os.path.join(src, "quad.c"),
                    "-lm"], check=True)
    return out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    level = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    O.LIB_PATH = build_stats_lib()
    orc = O.Oracle()
    st = orc.state(n)
    rng = np.random.default_rng(0)
    if level == 0:
        for k in range(20):
            st["stones"][3 * k + 0][:] = 0.75 * k
            st["stones"][3 * k + 2][:] = np.float32(k * 0.75) * np.cos(np.float32(np.pi / 2), dtype=np.float32)
    else:
        pos, _ = orc.footsteps(n, level, rng.uniform(0, 1, (5, n, 20)).astype(np.float32))
        st["stones"][:] = pos.reshape(n, 60).T
    orc.reset_all(st, seed=42)
    for _ in range(steps):
        orc.env_step(st, rng.uniform(-1, 1, (n, 21)).astype(np.float32))
    hist = np.ctypeslib.as_array((C.c_longlong * (6 * 256)).in_dll(orc.L, "or_stats_hist")).reshape(6, 256)
    tot = hist[0].sum()
    names = ["contacts found", "limit rows", "contacts kept", "self-contacts found", None, "self pairs past filter"]
    print(f"{n} envs x {steps} steps (level {level}) = {tot} substeps")
    for i, name in enumerate(names):
        if name is None:
            continue
        h = hist[i]
        nz = np.nonzero(h)[0]
        q = np.searchsorted(np.cumsum(h), [0.5 * tot, 0.99 * tot, 0.999 * tot, tot])
        print(f"  {name:20s} mean {np.dot(np.arange(256), h) / tot:6.2f}  p50 {q[0]}  p99 {q[1]}  p99.9 {q[2]}  "
              f"max {nz.max() if len(nz) else 0}")
    m = orc.m
    top = np.argsort(-hist[4])[:8]
    print("  most frequent self-contact pairs (per substep):",
          ", ".join(f"{m['geom_name'][m['self_pair'][p] & 255]}/{m['geom_name'][m['self_pair'][p] >> 8]} "
                    f"{hist[4][p] / tot:.3f}" for p in top if hist[4][p]))
    found = np.dot(np.arange(256), hist[0])
    kept = np.dot(np.arange(256), hist[2])
    print(f"  contacts dropped by the cap: {found - kept} of {found} ({100.0 * (found - kept) / max(found, 1):.3f} %)")


if __name__ == "__main__":
    main()
