#!/bin/bash
# Extra PMC passes (one counter group per pass) on a short bench run: instruction-cache, scalar
# cache, vector L1 and wait-state counters.  Output: gpurun_out/pmc_probe_$TAG/
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${TAG:-probe}
OUT=$R/gpurun_out/pmc_probe_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline ${BENCH_ARGS}"
timeout -k 10 120 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
i=0
for P in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" \
         "SQ_IFETCH SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_INSTS_VMEM" \
         "SQC_DCACHE_HITS SQC_DCACHE_MISSES" \
         "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
         "SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_VMEM" \
         "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  echo "== pmc $P"
  timeout -k 10 180 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- $B > $OUT/p$i.log 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
done
exit 0
