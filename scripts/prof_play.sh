#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/prof_play
timeout -k 10 300 python3 $R/scripts/prof_play.py ${NUM_ENVS:-32768} || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 $R/scripts/prof_play.py ${NUM_ENVS:-32768} > $R/gpurun_out/prof_play.log 2>&1 || exit $?
rm -f $O/run_kernel_trace.csv
python3 $R/scripts/kstats.py $O/run_kernel_stats.csv 25
