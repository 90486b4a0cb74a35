#!/bin/bash
# Exact-parity check on the GPU box: the trajectory tests, then a short bench (k_step timing).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -v --timeout 400 --timeout-method thread -s tests/test_gpu_exact.py ${EXACT_ARGS} > gpurun_out/exact.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error|mismatched|differ|  [a-z_]+:" gpurun_out/exact.log | grep -v " 0 of " | head -60; tail -3 gpurun_out/exact.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-train --no-c5 --no-cpu-baseline --steps 500 > gpurun_out/exact_bench.log 2>&1
rc=$?; tail -1 gpurun_out/exact_bench.log | cut -c1-400; exit $rc
