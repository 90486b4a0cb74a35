#!/bin/bash
# Diagnostic: bench.py under each scheduling variant of k_step (AS_TUNE, see StepArgs::tune).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for t in ${TUNES:-0 1}; do
  echo "== tune $t"
  AS_TUNE=$t timeout -k 10 120 python bench.py --steps 300 --no-cpu-baseline > gpurun_out/tune_$t.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/tune_$t.log').read().strip().splitlines()[-1]);print(d['value'], d['kernels_ms'])"
done
