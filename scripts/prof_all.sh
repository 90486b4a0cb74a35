# Round profiles: k_step kernel trace + PMC passes of bench.py (profile.sh), the PMC summary, and the
# trainer's kernel stats.  TAG names the round (profiles/<TAG>_*).
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${TAG:-r01h}
TAG=$T bash $R/scripts/profile.sh > $R/gpurun_out/profile_$T.log 2>&1 || { tail -20 $R/gpurun_out/profile_$T.log; exit 1; }
tail -5 $R/gpurun_out/profile_$T.log
rm -f $R/gpurun_out/prof_$T/trace/run_kernel_trace.csv
python3 $R/scripts/pmc_summary.py $R/gpurun_out/prof_$T > $R/gpurun_out/${T}_pmc_summary.txt || exit 1
NUM_ENVS=32768 TAG=_$T bash $R/scripts/prof_train.sh > $R/gpurun_out/${T}_train_kernel_stats.txt 2>&1 || exit 1
tail -3 $R/gpurun_out/${T}_train_kernel_stats.txt
