#!/bin/bash
# C5 learning-curve variants (scripts/train_curve.py, Allsteps-AnymalC-v0, 4096 envs, EPOCHS epochs), one
# JSON-lines file each -> gpurun_out/<TAG>_c5_<name>.jsonl; the variants are hydra-style env overrides.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-r04}
E=${EPOCHS:-1000}
for v in "$@"; do
  name=${v%%:*}; ovr=${v#*:}
  echo "== $name: $ovr"; date
  timeout -k 10 300 python -u scripts/train_curve.py 4096 $E 50 Allsteps-AnymalC-v0 $ovr \
    > gpurun_out/${T}_c5_$name.jsonl 2> gpurun_out/${T}_c5_$name.log || { tail -5 gpurun_out/${T}_c5_$name.log; exit 1; }
  python - gpurun_out/${T}_c5_$name.jsonl <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
for r in rows[:: max(1, len(rows) // 6)] + rows[-1:]:
    print(r["epoch"], r["mean_reward"], r["mean_length"], r["mean_target_index"], r["max_target_index"])
PY
done
