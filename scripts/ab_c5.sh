#!/bin/bash
# C5 (quadruped, 16384 envs) A/B of the wave placement: ALLSTEPS_WAVE_MAP=0 / 1, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/ab_c5.log
for rep in 1 2; do
  for v in 0 1; do
    ALLSTEPS_WAVE_MAP=$v timeout -k 10 200 python bench.py --no-train --no-cpu-baseline --steps 20 > gpurun_out/ab_one.log 2>&1 || { tail -5 gpurun_out/ab_one.log; exit 1; }
    tail -1 gpurun_out/ab_one.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); c=d['c5']
print('map$v', 'c2 %.4g' % d['value'], 'c5', {k: c[k] for k in c if not isinstance(c[k], (dict, list))})" | tee -a gpurun_out/ab_c5.log
  done
done
