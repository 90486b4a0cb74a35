#!/bin/bash
# rocprofv3 kernel trace of the C5 quadruped bench (k_step<18>, 16384 envs) -> gpurun_out/prof_c5_$TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/prof_c5_${TAG:-r01h}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 $R/scripts/bench_quadruped.py --num_envs 16384 --steps 200 > $O.log 2>&1 || exit $?
rm -f $O/run_kernel_trace.csv
tail -1 $O.log
python3 $R/scripts/kstats.py $O/run_kernel_stats.csv 8
