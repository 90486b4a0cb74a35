#!/bin/bash
# HBM traffic of the trainer's minibatch kernels: rocprofv3 FETCH_SIZE and WRITE_SIZE in
# separate passes over one bench_train.py epoch at 32768 envs, per-dispatch averages per kernel, FETCH_SIZE
# doubled (MI355X_MICROARCH.md gfx950 correction).  Summary JSON lines to stdout.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/prof_train_pmc${TAG}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $O/$P -o run -- python3 $R/scripts/bench_train.py \
    --num_envs 32768 --epochs 1 --warmup 0 > $O/$P.log 2>&1 || { echo "pmc $P failed rc=$?"; tail -5 $O/$P.log; exit 1; }
done
python3 - "$O" <<'PY'
import collections, csv, glob, json, sys
o = sys.argv[1]
keys = ("k_mlp_fwd<2, 21>", "k_mlp_bwd<2>", "k_wgrad<2>", "k_reduce_rows", "k_adam<true>", "k_step<27")
res = collections.defaultdict(dict)
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"{o}/{c}/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != c:
                continue
            for k in keys:
                if k in r["Kernel_Name"]:
                    per[k][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for k, d in per.items():
        res[k][c] = sum(d.values()) / max(len(d), 1)
        res[k]["dispatches"] = len(d)
for k in keys:
    v = res.get(k)
    if not v or "FETCH_SIZE" not in v or "WRITE_SIZE" not in v:
        continue
    rd, wr = 2.0 * v["FETCH_SIZE"] * 1024.0, v["WRITE_SIZE"] * 1024.0
    print(json.dumps({"kernel": k, "dispatches": v["dispatches"], "read_mb": round(rd / 1e6, 2),
                      "write_mb": round(wr / 1e6, 2), "traffic_mb": round((rd + wr) / 1e6, 2),
                      "method": "FETCH_SIZE x 2 + WRITE_SIZE (KB), per-dispatch mean"}))
PY
