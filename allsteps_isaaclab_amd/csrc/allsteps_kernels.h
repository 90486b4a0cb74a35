// allsteps_kernels.h -- host/device interface of the step kernels (internal to liballsteps_hip.so).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/allsteps.h"

namespace as {

constexpr int kMaxLinks = 24;  // LDS sizing of the step kernel (walker: 22 links)
constexpr int kMaxDofs = 6 + kMaxLinks - 1;

enum { kModeStep = 0, kModeReset = 1, kModePhysics = 2, kModeTask = 3 };

// Everything the kernels read that does not change per step: model tables + the tree plan
// derived from them on the host.  The plan is bitmasks over links / dofs: every tree pass of the
// step kernel is a walk over one lane's own ancestor path or subtree (no level barriers), and
// each lane keeps its own masks in registers for the whole launch.
struct Consts {
  as_model_t model;
  as_sim_t sim;
  as_task_t task;
  as_actuator_t act;               // as_set_actuator (mode AS_ACT_TORQUE after as_create)
  as_quad_task_t quad;             // as_set_quad_task (BASELINE C5)
  int32_t nv;
  int32_t st_has_hind;             // the state carries contact_mask_hind (sensors 2, 3)
  int32_t max_path;                // longest root->link path, root excluded (links)
  int32_t max_sub;                 // largest subtree of a non-root link, itself excluded
  uint32_t root_kids;              // links whose parent is the root
  uint32_t lpath[kMaxLinks];       // links on the path root..link, both included
  uint32_t lsub[kMaxLinks];        // links in the subtree of link, itself included
  uint32_t ancmask[kMaxLinks];     // dofs on the path root..link (root dofs 0-5 always set)
  uint32_t dsub[kMaxDofs];         // links moved by dof j (subtree of its link; root dofs: all)
  uint32_t ddesc[kMaxDofs];        // dofs k whose link path contains dof j (bit k)
  // FK by pointer jumping (k_step fk): jump[i] byte r = the 2^r-th ancestor of link i, the root (0)
  // once the path is exhausted; fk_rounds = ceil(log2(max_path)) rounds cover every path
  uint32_t jump[kMaxLinks];
  int32_t fk_rounds;
};

struct StepArgs {
  const Consts* consts;
  as_state_t st;
  int32_t n;
  int32_t mode;
  const float* actions;
  float* reward;
  float* obs;                  // [n][59] observation rows (speculative second tick, see k_step)
  uint32_t* side;              // [kSideWords][n]: tick-#1 state and observation entries for k_obs
  uint8_t* terminated;
  uint8_t* truncated;
  const float* reset_draws;
  const uint8_t* reset_mask;   // kModeReset: envs to reset (null: all)
  int32_t* counters;  // one bank (kCntBank ints, zero at launch: see k_obs), layout below
  uint64_t seed;
  int64_t env_offset;
  unsigned long long* stamps;  // diagnostic phase timing (s_memtime deltas summed over waves) or null
  const int32_t* wave_map;     // [2 * blocks] env of each workgroup half (see kMapEnvs) or null: xcd_block
};

// phase ids of the diagnostic stamps (as_debug_stamps)
enum {
  kStLoad = 0, kStFK, kStLinkQ, kStDyn, kStChol, kStSolve, kStCollide, kStRows, kStWsolve, kStPGS,
  kStIntegrate, kStFKFinal, kStTask, kStReset, kStStore, kNumStamps
};

// Step counters, one bank per launch (two banks alternate; k_obs clears the next one):
//   [0]  any env reset (plain store of 1)
//   [1]  sum of curr_target_index over all envs, published by k_obs from the partial sums
//   [2]  kCntLevel (regen_footsteps)
//   [3]  contacts cut by the row budget in this launch, all envs and substeps (kCntDropped)
//   [kCntStride * (1 + i)], i < kCntSlots: partial sums, one atomic per wave into slot block % kCntSlots
//        (one 64-B line each: 4096 same-address atomics serialise at the memory side)
constexpr int kCntSlots = 16;
constexpr int kCntStride = 16;
constexpr int kCntBank = kCntStride * (1 + kCntSlots);

// side buffer of k_step -> k_obs: idx, prev, next, count, swing, pot, old_pot, foot_contact[2]
// (tick-#1 state) and foot_contact[2], targets[9] (tick-#1 observation entries 48..58)
constexpr int kSideState = 9;
constexpr int kSideObs = 11;
constexpr int kSideRegen = kSideState + kSideObs;  // 1 = reset env due new stones (regen_footsteps)
constexpr int kSideCost = kSideRegen + 1;   // constraint rows of the env over this launch's substeps
constexpr int kSideWords = kSideCost + 1;

// Cost-balanced wave placement (k_obs / k_quad -> the next k_step; placement only, never results).
// k_obs ranks each chunk of kMapEnvs consecutive envs by the constraint rows they had in this launch,
// puts ranks 2p and 2p + 1 in one wave (pair p, 0 = heaviest) and places pair p of chunk w at workgroup
//   resident grid (the whole grid fits the chip, 8 one-wave workgroups per CU):
//     p < 16: p C + w,   p >= 16: n / 4 + (31 - p) C + w        (C = n / 64 chunks)
//   -- workgroups b and b + n / 4 share a SIMD (measured, scripts/simd_mates.py), and a wave's cycles
//   grow with its PARTNER's rows more than with its own, so the heaviest wave gets the lightest partner;
//   streamed grid (more workgroups than slots): p C + w, so the dispatcher starts the heaviest pairs of
//   every chunk first and the lightest last (longest-processing-time-first order).
// Either way workgroup b runs on XCD b % 8 = w % 8 (C is a multiple of 8): a chunk's envs stay in one
// XCD's L2.  wave_map[2 b + h] = the env of workgroup b's half h.
constexpr int kMapEnvs = 64;
__host__ __device__ inline bool wave_map_fits(int n) { return n > 0 && n % (8 * kMapEnvs) == 0; }
__host__ __device__ inline int wave_map_block(int w, int p, int n, bool streamed) {
  const int C = n / kMapEnvs;
  if (streamed || p < kMapEnvs / 4) return p * C + w;
  return (n >> 2) + (kMapEnvs / 2 - 1 - p) * C + w;
}
constexpr int kCntLevel = 2;  // counter-bank word: the curriculum level k_step saw (k_obs regen level)
constexpr int kCntDropped = 3;  // counter-bank word: contacts found past the row budget (as_step_counters [3])

// k_quad (BASELINE C5 task epilogue, one env per lane)
struct QuadArgs {
  const Consts* consts;
  as_state_t st;
  int32_t n;
  int32_t reset_all;           // 1: reset every env (as_quad_reset_all), no task step
  const float* actions;        // [n][nh]
  float* obs;                  // [n][AS_QUAD_OBS_DIM]
  float* reward;
  uint8_t* terminated;
  uint8_t* truncated;
  uint64_t seed;
  int64_t env_offset;
  const uint32_t* side;        // k_step's side buffer (the row counts of the placement)
  int32_t* wave_map;           // null, or rebuilt here for the next k_step (kMapEnvs)
  int32_t map_streamed;        // wave_map_block
};

struct ObsArgs {
  const Consts* consts;
  as_state_t st;
  int32_t n;
  int32_t* counters;       // this launch's bank (k_obs publishes the sum into [1])
  int32_t* next_counters;  // the other bank, cleared here for the next launch
  float* obs;
  const uint32_t* side;
  uint64_t seed;
  int64_t env_offset;
  int32_t* wave_map;       // null, or rebuilt here for the next k_step from the side buffer's row counts
  int32_t map_streamed;    // wave_map_block: the grid streams through the chip (LPT order)
};

struct StonesArgs {
  const Consts* consts;
  float* stones;
  int32_t n;
  int32_t level;
  const float* draws;
  uint64_t seed;
  int64_t env_offset;
};

// k_body_state (ring-2 views, as_body_state): the step kernel's FK of the current state, then every
// body's pose and velocities
struct BodyArgs {
  const Consts* consts;
  as_state_t st;
  int32_t n;
  float* out;                  // [AS_BODY_STATE_ROWS][nb][n]
  as_body_table_t bodies;
};

// The H^-1 sweep's skipped column quads (allsteps_kernels.hip sweep_inverse; bit r (NB - 1) + jb: round
// r, quad jb of the rotated row), compiled for the Allsteps walker (27 dofs) and the C5 quadruped (18):
// the quads in which the pivot rows are structurally zero for those trees.  as_create runs the
// structural sweep for the model it is given (sweep_skip_mask) and launches the skipping kernel only if
// every compiled bit is also set for that model.
constexpr uint64_t kSweepSkip27 = 207817167ull;  // 14 of the walker's 42 quad updates
constexpr uint64_t kSweepSkip18 = 3219ull;       // 6 of the quadruped's 20
uint64_t sweep_skip_mask(const as_model_t& m);  // the model's exactly-zero quads (host)

bool step_supported_nv(int nv);
hipError_t launch_body_state(const BodyArgs& a, hipStream_t stream);
hipError_t launch_step(const StepArgs& a, int nv, bool sweep_skip, hipStream_t stream);
hipError_t launch_obs(const ObsArgs& a, hipStream_t stream);
hipError_t launch_stones(const StonesArgs& a, hipStream_t stream);
hipError_t launch_quad(const QuadArgs& a, hipStream_t stream);
// zero n int32 words with a kernel (graph-safe stepping: a kernel node instead of a memset node)
hipError_t launch_zero(int32_t* p, int n, hipStream_t stream);
size_t step_lds_bytes();

}  // namespace as
