set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/prof_train
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_train.py --num_envs 32768 --epochs 1 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_train.log 2>&1 || exit $?
rm -f $O/run_kernel_trace.csv
head -40 $O/run_kernel_stats.csv
