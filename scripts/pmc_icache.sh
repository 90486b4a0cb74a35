#!/bin/bash
# Instruction-cache counters of k_step (one GPU call): list the SQC / IFETCH counters the box offers,
# then one rocprofv3 --pmc pass per available group over a short bench.py run.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$R/gpurun_out/icache_${TAG:-r03}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/avail.txt 2>&1 || { echo "list failed"; tail -5 $OUT/avail.txt; exit 1; }
grep -oE "\b(SQC_[A-Z0-9_]+|SQ_IFETCH[A-Z_]*|SQ_INSTS_[A-Z_]+|SQ_WAIT_[A-Z_]+)\b" $OUT/avail.txt | sort -u > $OUT/names.txt
cat $OUT/names.txt | tr '\n' ' '; echo
B="python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-train --no-c5 ${BENCH_ARGS}"
# two counters per pass (the SQC block's per-pass limit is not documented in the guide)
PASSES=${PASSES:-"SQC_ICACHE_REQ:SQC_ICACHE_MISSES SQC_ICACHE_HITS:SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH_LEVEL:SQ_INSTS_VALU"}
for PP in $PASSES; do
  P=$(echo $PP | tr ':' ' ')
  ok=1; for c in $P; do grep -qx "$c" $OUT/names.txt || ok=0; done
  [ $ok = 1 ] || { echo "skip $P (not all available)"; continue; }
  T=$(echo $P | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc_$T -o run -- $B > $OUT/pmc_$T.log 2>&1 || { echo "pmc $P failed"; tail -5 $OUT/pmc_$T.log; exit 1; }
  python3 - $OUT/pmc_$T <<'PY'
import csv, glob, sys
per = {}
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith(("void as::k_step<27>", "void as::k_step<27, ")):
            k = (r["Dispatch_Id"], r["Counter_Name"])
            per[k] = per.get(k, 0.0) + float(r["Counter_Value"])
tot = {}
for (d, c), v in per.items():
    tot.setdefault(c, []).append(v)
for c, v in sorted(tot.items()):
    print(f"k_step<27> {c}: {sum(v)/len(v):.1f} per dispatch over {len(v)}")
PY
done
