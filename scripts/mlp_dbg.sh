#!/bin/bash
# variants of the fused MLP forward for timing (debug only)
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
for d in ${DBGS:-0 1 2 4 7}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DPPO_MLP_DBG=$d -I $R/include -o /tmp/libppo_dbg$d.so $R/allsteps_isaaclab_amd/csrc/ppo_kernels.hip $R/allsteps_isaaclab_amd/csrc/ppo_mlp.hip $R/allsteps_isaaclab_amd/csrc/ppo_wgrad.hip
  echo "dbg=$d"; PPO_HIP_LIB=/tmp/libppo_dbg$d.so timeout -k 10 60 python $R/scripts/mlp_fwd_bench.py ${ROWS:-4096}
done
