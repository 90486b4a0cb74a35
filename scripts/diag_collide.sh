cd "${GRAFT_REPO_ROOT}"
# Diagnostic collide split: needs abtest/diag.so, built by applying profiles/r06z6_collide_diag.patch to a copy
# of the kernel at 4c782d5 and `bash scripts/ab_build.sh diag <that copy>` (timing only).
mkdir -p gpurun_out
for lib in base diag; do for cfg in "4096 0 1000" "32768 9 300"; do set -- $cfg
ALLSTEPS_HIP_LIB=$PWD/abtest/$lib.so timeout -k 10 200 python bench.py --no-train --no-c5 --no-cpu-baseline --num-envs $1 --level $2 --steps $3 > gpurun_out/d1.log 2>&1 || exit 1
tail -1 gpurun_out/d1.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); L=d['roofline']['latency']
print('$lib', $1, 'mean', L['mean_phases']); print('   crit', L['critical_path_phases'])" | tee -a gpurun_out/diag.log
done; done
