set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=r01f bash $R/scripts/profile.sh > $R/gpurun_out/profile_r01f.log 2>&1 || { tail -20 $R/gpurun_out/profile_r01f.log; exit 1; }
tail -5 $R/gpurun_out/profile_r01f.log
rm -f $R/gpurun_out/prof_r01f/trace/run_kernel_trace.csv
python3 $R/scripts/pmc_summary.py $R/gpurun_out/prof_r01f > $R/gpurun_out/r01f_pmc_summary.txt || exit 1
NUM_ENVS=32768 TAG=_r01f bash $R/scripts/prof_train.sh > $R/gpurun_out/r01f_train_kernel_stats.txt 2>&1 || exit 1
tail -3 $R/gpurun_out/r01f_train_kernel_stats.txt
