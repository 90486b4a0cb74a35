#!/bin/bash
# Full GPU test suite on the box (one pytest process), then smoke.  Stops on a fault / abort / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -15; echo "pytest rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc2=$?; tail -2 gpurun_out/smoke.log; echo "smoke rc=$rc2"
exit $(( rc > rc2 ? rc : rc2 ))
