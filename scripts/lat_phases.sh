#!/bin/bash
# Per-phase latency records (bench.py roofline.latency: mean wave and the slowest wave's phases) of the
# in-tree library and of abtest/<name>.so candidates, C2 (4096 envs, level 0).  -> gpurun_out/lat_phases.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in "$@"; do
  ALLSTEPS_HIP_LIB=$PWD/abtest/$lib.so timeout -k 10 200 python bench.py --no-train --no-c5 --no-cpu-baseline \
    --steps 300 > gpurun_out/lat_one.log 2>&1 || { tail -5 gpurun_out/lat_one.log; exit 1; }
  tail -1 gpurun_out/lat_one.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); L=d['roofline']['latency']
print('$lib', 'value %.4g' % d['value'], 'max', L['max_wave_cycles'], 'avg', L['avg_wave_cycles'], 'rows', L['critical_path_rows'])
print('  crit', L['critical_path_phases'])
print('  mean', L['mean_phases'])" | tee -a gpurun_out/lat_phases.log
done
