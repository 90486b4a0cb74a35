#!/bin/bash
# rocprofv3 kernel trace + PMC passes of bench.py (one GPU call).  Output: gpurun_out/prof_$TAG/
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${TAG:-r01}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps ${STEPS:-100} --warmup 10 --no-cpu-baseline --no-train --no-c5 ${BENCH_ARGS}"
set -o pipefail
echo "== kernel trace"; date
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B > $OUT/trace.log 2>&1 || exit $?
tail -2 $OUT/trace.log
for P in "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  T=$(echo $P | tr ' ' '_' | cut -c1-40)
  echo "== pmc $P"; date
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc_$T -o run -- $B > $OUT/pmc_$T.log 2>&1 || { echo "pmc pass failed rc=$?"; tail -5 $OUT/pmc_$T.log; exit 1; }
done
echo "== ablation"; date
timeout -k 10 300 python3 $R/scripts/ablate.py > $OUT/ablate.log 2>&1; cat $OUT/ablate.log
# per-launch HBM traffic of k_step from the FETCH_SIZE / WRITE_SIZE passes (bench.py's roofline.traffic)
python3 - "$OUT" "${NUM_ENVS:-4096}" > $OUT/traffic_k_step.json <<'PY'
import csv, glob, json, sys
out, n = sys.argv[1], int(sys.argv[2])
def per_dispatch(c):
    """average over k_step dispatches of counter c (summed over its instances in a dispatch)"""
    files = [f for f in glob.glob(f"{out}/pmc_*/run_counter_collection.csv")]
    for f in files:
        rows = [r for r in csv.DictReader(open(f))
                if r["Kernel_Name"].startswith(("void as::k_step<27>", "void as::k_step<27, ")) and r["Counter_Name"] == c]
        if rows:
            per = {}
            for r in rows:
                per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
            return sum(per.values()) / max(len(per), 1)
    return None
vals = {c: per_dispatch(c) for c in ("FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_VALU", "GRBM_GUI_ACTIVE")}
traffic = (2.0 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024.0
cyc = vals["GRBM_GUI_ACTIVE"] / 8.0  # summed over the 8 XCDs
print(json.dumps({"kernel": "k_step<27, *>", "num_envs": n, "fetch_kb": round(vals["FETCH_SIZE"], 1),
                  "write_kb": round(vals["WRITE_SIZE"], 1), "traffic_bytes_per_launch": round(traffic),
                  "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; FETCH_SIZE doubled "
                            "(MI355X_MICROARCH.md gfx950 correction), WRITE_SIZE as reported",
                  "valu_insts_per_launch": vals["SQ_INSTS_VALU"], "clock_cycles_per_launch": round(cyc),
                  "valu_issue_frac": round(vals["SQ_INSTS_VALU"] * 2 / (1024 * cyc), 4),
                  "valu_method": "SQ_INSTS_VALU (chip-wide wave-level VALU instructions) x 2 issue cycles per "
                                 "wave64 VALU instruction (MI355X_MICROARCH.md) / (1024 SIMDs x GRBM_GUI_ACTIVE/8)"}))
PY
cat $OUT/traffic_k_step.json
