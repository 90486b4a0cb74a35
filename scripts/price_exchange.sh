#!/bin/bash
# DESIGN §6 "Pricing the C4 exchange" (VERDICT r04 item 1): on ONE GPU, the PPO update each rank of a
# W-GPU job would run per epoch.  allgather (north star): every rank updates on the gathered W x batch
# with a W x minibatch -- emulated here by one rank with W x 32768 envs and minibatch W x 32768 (the same
# rows, minibatch count and mini-epochs); allreduce (rl_games multi_gpu): the W = 1 update per rank plus
# one gradient all-reduce per minibatch (modelled in DESIGN §6, no second GPU here).  Reference agent
# config otherwise (horizon 32, 10 mini-epochs).  One JSON line per W.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-r05}_price_exchange.jsonl
: > $OUT
for W in 1 2 4 8; do
  N=$((W * 32768))
  timeout -k 10 300 python scripts/bench_train.py --num_envs $N --epochs 3 --warmup 2 --quiet \
    agent.params.config.minibatch_size=$N > gpurun_out/price_w$W.log 2>&1 || { tail -5 gpurun_out/price_w$W.log; exit 1; }
  tail -1 gpurun_out/price_w$W.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); d['emulated_world']=$W; print(json.dumps(d))" | tee -a $OUT
done
