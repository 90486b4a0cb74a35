#!/bin/bash
# Learning curves of the full stack on one GPU (scripts/train_curve.py, the reference agent configs):
# Allsteps-v0 at 4096 and 32768 envs, and the C5 quadruped (Allsteps-AnymalC-v0) at 4096 envs.
# One JSON line per logged epoch -> gpurun_out/<TAG>_train_curve_*.jsonl.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-r04}
run() {  # name envs epochs every task limit
  echo "== $1"; date
  timeout -k 10 $6 python -u scripts/train_curve.py $2 $3 $4 $5 > gpurun_out/${T}_train_curve_$1.jsonl \
    2> gpurun_out/${T}_train_curve_$1.log || { rc=$?; tail -20 gpurun_out/${T}_train_curve_$1.log; exit $rc; }
  tail -1 gpurun_out/${T}_train_curve_$1.jsonl
}
run 4096 4096 1000 25 Allsteps-v0 300 || exit $?
run 32768 32768 500 10 Allsteps-v0 400 || exit $?
run c5_4096 4096 1000 25 Allsteps-AnymalC-v0 400 || exit $?
date
