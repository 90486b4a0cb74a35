#!/bin/bash
# bench.py A/B on one box: the tree's bench.py against abtest/<name>.py, alternating, two repetitions
# (C2, env leg only).  -> gpurun_out/bench_ab.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/bench_ab.log
: > $OUT
for rep in 1 2; do
  for b in bench.py "$@"; do
    f=$b; [ "$b" = bench.py ] || f=abtest/$b.py
    timeout -k 10 200 python $f --no-train --no-c5 --no-cpu-baseline > gpurun_out/bench_ab_one.log 2>&1 || { tail -5 gpurun_out/bench_ab_one.log; exit 1; }
    tail -1 gpurun_out/bench_ab_one.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print('$b', 'value %.5g' % d['value'], 'ms', d['ms_per_step'], d['kernels_ms'])" | tee -a $OUT
  done
done
