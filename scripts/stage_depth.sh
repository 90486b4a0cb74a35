#!/bin/bash
# staging depth variants of the fused MLP kernels (PPO_STAGE_DEPTH loads in flight per thread), timed
# by scripts/mlp_fwd_bench.py (forward) -- debug only
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
for d in ${DEPTHS:-8 16 32}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DPPO_STAGE_DEPTH=$d -I $R/include -o /tmp/libppo_sd$d.so $R/allsteps_isaaclab_amd/csrc/ppo_kernels.hip $R/allsteps_isaaclab_amd/csrc/ppo_mlp.hip $R/allsteps_isaaclab_amd/csrc/ppo_wgrad.hip
  echo "depth=$d"; PPO_HIP_LIB=/tmp/libppo_sd$d.so timeout -k 10 60 python $R/scripts/mlp_fwd_bench.py ${ROWS:-32768}
done
