#!/bin/bash
# Round-end measurement of HEAD in one GPU call: the full GPU suite + smoke, the C2 rocprofv3 trace /
# PMC passes / ablation / trainer stats (prof_all.sh), the C3 trace + traffic passes, the C5 trace, the three
# SURVEY sizes with the CPU baseline beside each, and the default bench line.  Every GPU step has its
# own time limit; the chain stops at the first failure.  TAG names the outputs (gpurun_out/<TAG>_*).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
T=${TAG:-r04}
mkdir -p gpurun_out
echo "== gpu suite"; date
bash scripts/gpu_tests.sh || exit $?
cp gpurun_out/pytest_gpu.log gpurun_out/${T}_pytest_gpu.log
echo "== C2 profiles"; date
TAG=$T bash scripts/prof_all.sh || exit $?
cp gpurun_out/prof_$T/trace/run_kernel_stats.csv gpurun_out/${T}_kernel_stats.csv
cp gpurun_out/prof_$T/traffic_k_step.json gpurun_out/${T}_traffic_k_step.json
# the bench lines below read profiles/traffic_k_step.json: refresh it from THIS tree's PMC passes first
cp gpurun_out/prof_$T/traffic_k_step.json profiles/traffic_k_step.json
cp gpurun_out/prof_$T/ablate.log gpurun_out/${T}_ablate.log
echo "== C3 profiles"; date
NUM_ENVS=32768 BENCH_ARGS="--num-envs 32768 --level 9" STEPS=30 TAG=${T}_c3 bash scripts/profile.sh \
  > gpurun_out/profile_${T}_c3.log 2>&1 || { tail -20 gpurun_out/profile_${T}_c3.log; exit 1; }
rm -f gpurun_out/prof_${T}_c3/trace/run_kernel_trace.csv
cp gpurun_out/prof_${T}_c3/trace/run_kernel_stats.csv gpurun_out/${T}_c3_kernel_stats.csv
cp gpurun_out/prof_${T}_c3/traffic_k_step.json gpurun_out/${T}_c3_traffic_k_step.json
echo "== C5 trace"; date
TAG=$T bash scripts/prof_c5.sh > gpurun_out/${T}_c5_kernel_stats.txt 2>&1 || { tail -20 gpurun_out/${T}_c5_kernel_stats.txt; exit 1; }
echo "== sizes"; date
TAG=$T bash scripts/sizes.sh > gpurun_out/sizes_${T}.log 2>&1 || { tail -20 gpurun_out/sizes_${T}.log; exit 1; }
cp gpurun_out/sizes_$T.jsonl gpurun_out/${T}_sizes.jsonl
echo "== default bench"; date
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench_default.log 2>&1 || { tail -20 gpurun_out/${T}_bench_default.log; exit 1; }
tail -1 gpurun_out/${T}_bench_default.log | cut -c1-400
date
