#!/bin/bash
# Round-5 first GPU call: GPU suite + smoke, the driver-shaped bench (K 20 / W 5) and the long default
# bench on the same box, and the from-reset transient (where the driver's window sits).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_tests.sh || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-train --no-c5 > gpurun_out/r05a_bench_k20.log 2>&1 || { tail -5 gpurun_out/r05a_bench_k20.log; exit 1; }
tail -1 gpurun_out/r05a_bench_k20.log | cut -c1-600
timeout -k 10 300 python bench.py --no-train --no-c5 --no-cpu-baseline > gpurun_out/r05a_bench_k1000.log 2>&1 || { tail -5 gpurun_out/r05a_bench_k1000.log; exit 1; }
tail -1 gpurun_out/r05a_bench_k1000.log | cut -c1-600
timeout -k 10 200 python scripts/transient.py 4096 1200 0 > gpurun_out/r05a_transient.log 2>&1 || { tail -5 gpurun_out/r05a_transient.log; exit 1; }
cat gpurun_out/r05a_transient.log
TAG=r05a bash scripts/price_exchange.sh || exit 1
