#!/bin/bash
# trainer experiment: fused-kernel GPU tests, then the env+PPO throughput at 32768 envs and a kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_learning.py -k "fused or weight or mlp or deterministic" > gpurun_out/exp_learn.log 2>&1 || { tail -30 gpurun_out/exp_learn.log; exit 1; }
tail -2 gpurun_out/exp_learn.log
timeout -k 10 200 python scripts/bench_train.py --num_envs 32768 --epochs 3 --warmup 2 2>/dev/null | tail -1
TAG=_exp bash scripts/prof_train.sh 2>&1 | sed -n 2,9p
