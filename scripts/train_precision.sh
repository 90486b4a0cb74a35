#!/bin/bash
# Trainer leg (scripts/bench_train.py, 32768 envs, reference agent config) under the precision knobs,
# alternating, two repetitions: fp16 + GradScaler (the default: rl_games mixed_precision=True), fp16
# without the scaler, bf16 with / without it, fp32.  One JSON line each -> gpurun_out/<TAG>_train_precision.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-r04}_train_precision.jsonl
: > $OUT
C=agent.params.config
for rep in 1 2; do
  for cfg in "fp16_scaler:" "fp16_noscaler:$C.grad_scaler=False" "bf16_scaler:$C.mixed_precision_dtype=bfloat16" \
             "bf16_noscaler:$C.mixed_precision_dtype=bfloat16 $C.grad_scaler=False" "fp32:$C.mixed_precision=False"; do
    name=${cfg%%:*}; ovr=${cfg#*:}
    echo "== $name rep $rep"; date
    timeout -k 10 240 python scripts/bench_train.py --num_envs 32768 --epochs 6 --warmup 2 --quiet $ovr \
      > gpurun_out/train_prec_one.log 2>&1 || { tail -5 gpurun_out/train_prec_one.log; exit 1; }
    tail -1 gpurun_out/train_prec_one.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); d['case']='$name'; d['rep']=$rep
print(json.dumps(d))" | tee -a $OUT | cut -c1-200
  done
done
