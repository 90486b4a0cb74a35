#!/bin/bash
# rocprofv3 kernel trace + PMC passes of bench.py (one GPU call).  Output: gpurun_out/prof_$TAG/
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${TAG:-r01}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps ${STEPS:-100} --warmup 10 --no-cpu-baseline ${BENCH_ARGS}"
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
