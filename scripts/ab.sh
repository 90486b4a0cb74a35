#!/bin/bash
# A/B timing of candidate libraries against base.so on one box: alternating runs, C2 and C3.
# Usage: bash scripts/ab.sh cand1 [cand2 ...]   (names of abtest/<name>.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/ab.log
: > $OUT
run() {  # lib size level steps
  ALLSTEPS_HIP_LIB=$PWD/abtest/$1.so timeout -k 10 200 python bench.py --no-train --no-c5 --no-cpu-baseline \
    --num-envs $2 --level $3 --steps $4 > gpurun_out/ab_one.log 2>&1 || { tail -5 gpurun_out/ab_one.log; exit 1; }
  tail -1 gpurun_out/ab_one.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); L=d['roofline']['latency']
print('$1 N=$2', 'value %.4g' % d['value'], 'k_step', d['kernels_ms']['k_step_ms'], 'period', d['kernels_ms']['k_step_period_ms'], 'k_obs', d['kernels_ms']['k_obs_ms'], 'ms', d['ms_per_step'],
      'crit', {k: L['critical_path_phases'][k] for k in ('collide','pgs','sweep','wsolve','rows')},
      'meancollide', L['mean_phases']['collide'], 'meanpgs', L['mean_phases']['pgs'], 'meansweep', L['mean_phases']['sweep'], 'max', L['max_wave_cycles'], 'avg', L['avg_wave_cycles'])" | tee -a $OUT
}
for rep in 1 2; do
  for lib in base "$@"; do
    run $lib 4096 0 1000 || exit 1
  done
  for lib in base "$@"; do
    run $lib 32768 9 300 || exit 1
  done
done
