#!/bin/bash
# GPU round: pytest -m gpu, smoke, bench. Each GPU step has its own time limit; stop on a fault,
# abort, segfault or time-out (exit >= 124 or 134/139), continue past ordinary test failures.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
echo "== pytest -m gpu"; date
timeout -k 10 ${PYTEST_TIMEOUT:-600} python -m pytest tests -m gpu -q -x ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"; ok $rc || exit $rc
echo "== smoke"; date
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -5 gpurun_out/smoke.log; echo "smoke rc=$rc"; ok $rc || exit $rc
echo "== bench"; date
timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; tail -5 gpurun_out/bench.log; echo "bench rc=$rc"
exit $rc
