#!/bin/bash
# rocprofv3 kernel trace of scripts/bench_train.py (1 warm-up + 1 timed epoch); summary to stdout.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/prof_train${TAG}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 $R/scripts/bench_train.py --num_envs ${NUM_ENVS:-32768} --epochs 1 --warmup 1 ${OVR} > $R/gpurun_out/prof_train${TAG}.log 2>&1 || exit $?
rm -f $O/run_kernel_trace.csv
tail -1 $R/gpurun_out/prof_train${TAG}.log
python3 $R/scripts/kstats.py $O/run_kernel_stats.csv 30
