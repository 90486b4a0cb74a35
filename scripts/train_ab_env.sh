#!/bin/bash
# A/B of a trainer environment switch with one library: each setting in its own processes,
# alternated over two rounds (bench_train.py update_s at 32768 envs), then one rocprofv3 kernel-stats pass
# per setting.  Usage: bash scripts/train_ab_env.sh VAR   (setting A: VAR=0, setting B: VAR=1)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
VAR=$1
for rep in 1 2; do
  for val in 0 1; do
    env $VAR=$val timeout -k 10 300 python scripts/bench_train.py --num_envs 32768 --epochs 3 --warmup 1 \
      > gpurun_out/train_ab_one.log 2>&1 || { tail -5 gpurun_out/train_ab_one.log; exit 1; }
    tail -1 gpurun_out/train_ab_one.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$VAR=$val rep $rep update_s', d['update_s'], 'value', d['value'])"
  done
done
cd /tmp && export TMPDIR=/tmp
for val in 0 1; do
  O=$R/gpurun_out/train_ab_prof_${VAR}_$val
  export $VAR=$val
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- \
    python3 $R/scripts/bench_train.py --num_envs 32768 --epochs 1 --warmup 1 > $O.log 2>&1 || exit $?
  rm -f $O/run_kernel_trace.csv
  echo "== $VAR=$val"
  python3 $R/scripts/kstats.py $O/run_kernel_stats.csv 9 | grep -v k_step
done
