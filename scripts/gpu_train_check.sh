#!/bin/bash
# GPU: trainer tests, env+PPO throughput at 4096 and 32768 envs (scripts/bench_train.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_learning.py -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_learn.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_learn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_train.py --num_envs 4096 --epochs 4 --warmup 2 > gpurun_out/bt4096.log 2>&1 || exit $?
tail -1 gpurun_out/bt4096.log
timeout -k 10 400 python -u scripts/bench_train.py --num_envs 32768 --epochs 3 --warmup 1 > gpurun_out/bt32768.log 2>&1 || exit $?
tail -1 gpurun_out/bt32768.log
