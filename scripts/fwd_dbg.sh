#!/bin/bash
# Timing-only variants of the fused trunk forward (PPO_FWD_DBG in csrc/ppo_mlp.hip: 1 no weight reloads,
# 2 no exp, 4 no stores; results are wrong by construction), timed by scripts/mlp_ab.py against the
# round-4 library (abtest/ppo_r04.so, built from git by hand) at 32768 and 1000 rows.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
for d in ${DBGS:-0 1 2 4 7}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DPPO_FWD_DBG=$d -I include \
    -o /tmp/libppo_fdbg$d.so allsteps_isaaclab_amd/csrc/ppo_kernels.hip allsteps_isaaclab_amd/csrc/ppo_mlp.hip \
    allsteps_isaaclab_amd/csrc/ppo_wgrad.hip || exit 1
  for n in 32768 1000; do
    echo -n "dbg=$d rows=$n "; timeout -k 10 60 python scripts/mlp_ab.py abtest/ppo_r04.so /tmp/libppo_fdbg$d.so $n f16 \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('fwd_us', d['fwd_us'], 'h', d['h_maxdiff'], 'head', round(d['head_maxdiff'],4))" || exit 1
  done
done
