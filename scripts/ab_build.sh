#!/bin/bash
# build an A/B candidate step library into abtest/ (scratch, git-ignored): bash scripts/ab_build.sh NAME KERNELS.hip [extra hipcc flags]
# (KERNELS.hip: a copy of csrc/allsteps_kernels.hip; its includes are rewritten to this tree's paths)
set -e
cd "$(dirname "$0")/.."
N=$1; SRC=$2; shift 2
T=abtest/.src_$N.hip
sed 's#"../../include/allsteps.h"#"../include/allsteps.h"#; s#"allsteps_device.h"#"../allsteps_isaaclab_amd/csrc/allsteps_device.h"#; s#"allsteps_kernels.h"#"../allsteps_isaaclab_amd/csrc/allsteps_kernels.h"#' $SRC > $T
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -I include \
  -DAS_BUILD_ID=\"abtest-$N\" -fPIC -shared -Wno-unused-result "$@" -o abtest/$N.so $T allsteps_isaaclab_amd/csrc/allsteps_abi.hip
echo built abtest/$N.so
