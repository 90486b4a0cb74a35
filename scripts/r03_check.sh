#!/bin/bash
# Kernel-change check on the GPU box: the bit-exact trajectory / constraint / quadruped tests, then a
# short bench line (k_step timing + per-wave latency records).  Stops on a fault, abort or time-out.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TESTS=${TESTS:-"tests/test_gpu_exact.py tests/test_gpu_constraints.py tests/test_quadruped_task.py"}
timeout -k 10 600 python -u -m pytest -v --timeout 400 --timeout-method thread -s -m gpu $TESTS > gpurun_out/r03_exact.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|mismatch|differ" gpurun_out/r03_exact.log | grep -v " 0 of " | head -40; tail -3 gpurun_out/r03_exact.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-train --no-c5 --no-cpu-baseline --steps ${STEPS:-1000} ${BENCH_ARGS} > gpurun_out/r03_bench.log 2>&1
rc2=$?; tail -1 gpurun_out/r03_bench.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); L=d['roofline']['latency']
print('value', d['value'], 'k_step', d['kernels_ms'])
print('latency', {k: L[k] for k in ('avg_wave_cycles','max_wave_cycles','launch_cycles','clock_ghz')})
print('crit', L['critical_path_phases'], L['critical_path_rows'])
print('mean', L['mean_phases'])" || tail -5 gpurun_out/r03_bench.log
[ $rc2 -eq 0 ] || exit $rc2
if [ -n "$C3" ]; then
  timeout -k 10 300 python bench.py --no-train --no-c5 --no-cpu-baseline --num-envs 32768 --level 9 --steps 300 > gpurun_out/r03_c3.log 2>&1
  rc3=$?; tail -1 gpurun_out/r03_c3.log | cut -c1-300; exit $rc3
fi
exit $rc
