#!/bin/bash
# bench.py (env-only, cpu_baseline on) at the SURVEY §8d sizes: C1 N = 2 (level 0), C2 N = 4096
# (level 0), C3 N = 32768 (level 9).  One JSON line per size -> gpurun_out/sizes_$TAG.jsonl.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/sizes_${TAG:-r01}.jsonl
: > $OUT
for cfg in "2 0" "4096 0" "32768 9"; do
  set -- $cfg
  echo "== N=$1 level=$2"; date
  timeout -k 10 300 python bench.py --num-envs $1 --level $2 --no-train --no-c5 --steps ${STEPS:-1000} \
    > gpurun_out/sizes_$1.log 2>&1 || { rc=$?; tail -5 gpurun_out/sizes_$1.log; exit $rc; }
  grep '^{' gpurun_out/sizes_$1.log >> $OUT
done
cat $OUT
