#!/bin/bash
# Traffic calibration on the GPU box (one call): the probe (scripts/probes/traffic_calib, built on the
# CPU side: hipcc --offload-arch=gfx950 -O3 -o scripts/probes/traffic_calib scripts/probes/traffic_calib.hip)
# under separate rocprofv3 FETCH_SIZE and WRITE_SIZE passes at N envs x F fields, reduced by
# scripts/traffic_calib.py (with k_step's own counters if $KSTEP_TRAFFIC names a traffic_k_step.json).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${TAG:-r03}
N=${N:-4096}
F=${F:-32}
OUT=$R/gpurun_out/calib_${TAG}_n$N
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P="$R/scripts/probes/traffic_calib $N $F 20"
timeout -k 10 60 $P > $OUT/probe.json || exit $?
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_$C -o run -- $P > $OUT/pmc_$C.log 2>&1 || { echo "pmc $C failed"; tail -5 $OUT/pmc_$C.log; exit 1; }
done
python3 $R/scripts/traffic_calib.py $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE "$(cat $OUT/probe.json)" $KSTEP_TRAFFIC > $OUT/calib.json
cat $OUT/calib.json
