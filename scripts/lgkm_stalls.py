"""Static scan of a kernel's assembly for LDS reads waited on too soon.

For every ``s_waitcnt lgkmcnt(N)`` it finds the LDS instructions (``ds_*``) that must have completed
(the in-order LDS queue: all but the last N issued) and reports the ones issued fewer than ``--min``
instructions earlier in the same basic block -- their latency (~100+ cycles) is exposed.  SMEM loads
also count in lgkmcnt but complete out of order; a block that mixes them is approximate.

    python scripts/lgkm_stalls.py k.s --func _ZN2as6k_stepILi27EEEvNS_8StepArgsE [--min 8]
"""
import argparse
import re
import sys


def scan(lines: list[str], func: str, min_gap: int = 8) -> list[tuple[str, int, int, str]]:
    """(block, 1-based line, instructions between issue and wait, instruction) of every LDS read that a
    `s_waitcnt lgkmcnt(N)` retires fewer than `min_gap` instructions after its issue."""
    start = next(i for i, l in enumerate(lines) if l.startswith(func + ":"))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    q = []  # (index of instruction, line) of outstanding LDS ops in issue order
    n = 0
    block = ""
    hits = []
    for i in range(start, end):
        l = lines[i]
        if re.match(r"^\.LBB", l):
            block = l.split(":")[0]
            q = []  # conservative: a new block starts with nothing tracked
            continue
        s = l.strip()
        if not s or s.startswith(";") or s.startswith("."):
            continue
        n += 1
        if s.startswith("ds_"):
            q.append((n, i, s))
        m = re.match(r"s_waitcnt\s+.*lgkmcnt\((\d+)\)", s)
        if m:
            keep = int(m.group(1))
            done = q[: max(len(q) - keep, 0)]
            q = q[max(len(q) - keep, 0):]
            for (k, li, ins) in done:
                if n - k < min_gap and ins.startswith("ds_read"):
                    hits.append((block, li + 1, n - k, ins))
    return hits


def main():
    p = argparse.ArgumentParser()
    p.add_argument("asm")
    p.add_argument("--func", default="_ZN2as6k_stepILi27EEEvNS_8StepArgsE")
    p.add_argument("--min", type=int, default=8)
    a = p.parse_args()
    hits = scan(open(a.asm).read().split("\n"), a.func, a.min)
    for h in hits:
        print(f"{h[0]} line {h[1]}: waited {h[2]} instructions after {h[3]}")
    print(f"{len(hits)} early waits on LDS reads", file=sys.stderr)


if __name__ == "__main__":
    main()
