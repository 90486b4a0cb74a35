"""CPU baseline (the oracle port, bench.cpu_baseline) at SURVEY §8d's three sizes on this host's cores:
C1 (2 envs, level 0), C2 (4096 envs, level 0), C3 (32768 envs, level 9) -- the same protocol as the bench
line's cpu_baseline object (median of 3 samples of >= 7 s after 50 warm-up steps, OMP_NUM_THREADS
threads).  One JSON line per size (the bench line keeps 4096).

    python scripts/cpu_baseline_sizes.py > profiles/r06_cpu_baseline.jsonl
"""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

for name, n, level in (("C1", 2, 0), ("C2", 4096, 0), ("C3", 32768, 9)):
    r = bench.cpu_baseline(n, level, None)
    r.update(config=name, num_envs=n, level=level)
    print(json.dumps(r), flush=True)
