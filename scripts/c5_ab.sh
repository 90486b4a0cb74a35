#!/bin/bash
# C5 A/B: scripts/bench_quadruped.py (16384 envs) and the per-phase stamps (scripts/stamps_c5.py) of
# abtest/<name>.so candidates, alternating, two repetitions.  -> gpurun_out/c5_ab.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/c5_ab.log
: > $OUT
for rep in 1 2; do
  for lib in "$@"; do
    ALLSTEPS_HIP_LIB=$PWD/abtest/$lib.so timeout -k 10 200 python scripts/bench_quadruped.py --steps 300 \
      > gpurun_out/c5_one.log 2>&1 || { tail -5 gpurun_out/c5_one.log; exit 1; }
    tail -1 gpurun_out/c5_one.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print('$lib', 'value %.4g' % d['value'], 'ms', d['ms_per_step'], 'resets', d['resets_per_step'])" | tee -a $OUT
    if [ $rep = 1 ]; then
      ALLSTEPS_HIP_LIB=$PWD/abtest/$lib.so timeout -k 10 200 python scripts/stamps_c5.py 16384 20 \
        > gpurun_out/c5_one.log 2>&1 || { tail -5 gpurun_out/c5_one.log; exit 1; }
      tail -1 gpurun_out/c5_one.log | python -c "
import json,sys
L=json.loads(sys.stdin.read())['latency']
print('$lib', 'avg', L['avg_wave_cycles'], 'max', L['max_wave_cycles'], 'launch', L['launch_cycles'])
print('  mean', L['mean_phases'])" | tee -a $OUT
    fi
  done
done
