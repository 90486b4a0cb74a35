#!/bin/bash
# the one-GPU cost of the allreduce mode's schedule -- per-minibatch graphs A / (exchange) /
# B and the separate gradient-norm pass (fuse_norm off) -- against the default one-graph-per-mini-epoch
# schedule, at 32768 envs with the reference agent config; world 1, so the exchange itself is a no-op
# (agent.params.config.exchange_schedule=True).  Two alternating repetitions.  One JSON line per run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-r06}_allreduce_schedule.jsonl
: > $OUT
for rep in 1 2; do
  for sched in False True; do
    timeout -k 10 300 python scripts/bench_train.py --num_envs 32768 --epochs 4 --warmup 2 --quiet \
      agent.params.config.exchange_schedule=$sched > gpurun_out/sched_$sched.log 2>&1 || { tail -5 gpurun_out/sched_$sched.log; exit 1; }
    tail -1 gpurun_out/sched_$sched.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); d['exchange_schedule']=$sched; d['rep']=$rep; print(json.dumps(d))" | tee -a $OUT
  done
done
