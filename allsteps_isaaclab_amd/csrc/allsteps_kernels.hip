// allsteps_kernels.hip -- MI355X (gfx950) step kernels for Allsteps-v0.
//
// k_step (K1): one env per 32-lane group (two envs per 64-lane wave, one wave per workgroup).
//   For each env: load the SoA state once, run `decimation` physics substeps, then the task
//   epilogue of DirectRLEnv.step (direct_rl_env.py:349-364): episode counter, foot-state tick #1,
//   targets, potentials, dones, rewards and -- for envs that are done -- the in-kernel reset
//   (allsteps_env.py:469-565) with Philox draws and an FK of the new pose.  The state is read and
//   written exactly once per env step.
//   One substep (oracle/physics.c is its serial restatement):
//     FK (level-synchronous, lanes = links) -> link inertias / motion subspaces -> RNEA bias and
//     composite inertias (lanes = links) -> joint-space inertia rows H_j (lane = dof j, from the
//     ancestor bitmasks) -> H^-1 by in-register Gauss-Jordan (one row per lane, pivot row broadcast
//     through LDS) -> u* = u + dt H^-1 (tau - C) -> stone contacts + joint-limit rows ->
//     W = H^-1 J^T (lane = dof, J and W columns in VGPRs) -> projected Gauss-Seidel on the impulses
//     with DPP cross-lane reductions -> semi-implicit integration.
// k_obs (K2): one env per lane.  If any env reset this step (device counter written by K1), the
//   second _compute_useful_values over ALL envs (allsteps_env.py:567: foot-state tick #2 with the
//   stale last-substep contacts, targets, potentials) and the curriculum gate
//   (allsteps_env.py:471-479); then the observation (allsteps_env.py:326-345).
// k_stones: _generate_foot_steps_allsteps (allsteps_env.py:125-174), one env per lane.
#include <hip/hip_runtime.h>

#include "../../include/allsteps.h"
#include "allsteps_device.h"
#include "allsteps_kernels.h"

namespace as {

constexpr int G = 32;               // lanes per env
constexpr int EPB = 2;              // envs per 64-lane workgroup
constexpr int LMAX = kMaxLinks;     // links (walker: 22)
constexpr int NVMAX = 6 + LMAX - 1; // generalized velocities
constexpr int MAXC = AS_MAX_CONTACTS;
constexpr int MAXR = AS_MAX_ROWS;
constexpr int NST = AS_NUM_STONES;
constexpr int kBisectIters = 12;    // capsule minimum: slope-sign bisection, interval 2^-12 = 2.4e-4
constexpr int kPairsPerChunk = G;   // one lane per (stone, geom) pair in the exact test
static_assert(kPairsPerChunk - 1 + G <= 64, "pending pair list (PhaseScratch::col.pl)");
constexpr int kSweepB = 4;        // pivot block of the H^-1 sweep
typedef float v4f __attribute__((ext_vector_type(4)));  // native 16-B vector (LDS b128 accesses)
typedef float v2f __attribute__((ext_vector_type(2)));  // register pair (packed FP32 math)

static_assert(NVMAX <= G, "one lane per generalized velocity");
static_assert(LMAX <= G, "one lane per link");
static_assert(MAXR <= G, "one row per lane in the row builders");
static_assert(MAXR <= 3 * MAXC, "a row index / 3 is a valid contact slot");

// ------------------------------------------------------------------------------------------------
// per-env LDS scratch.  Occupancy at 4096 envs is set by LDS: two envs per 64-lane workgroup must
// stay <= 20 KB so that 8 workgroups (2 waves/SIMD) fit a CU and 4096 envs run in one round.  The
// phase-local arrays therefore share one union: FK (Rl) -> dynamics (c, Ib, Ic, V, A, F) ->
// sweep (piv) -> constraint rows (Jm, Wm); each phase ends before the next one writes.
constexpr int kPrioRows = 9;          // constraint rows per issue-priority level (see substep; 4 / 6 / 9 / 12 / 15 timed)
constexpr int kRowGroup = 3;          // constraint rows per J / W / PGS group (a contact triplet)
constexpr int LDJ = 28;               // J / W row stride (>= NV = 27)
struct DynScratch {
  float c[LMAX][3];
  float Ib[LMAX][10];
  float Ic[LMAX][10];
  float Sq[LMAX][6];    // S_i qd_i, later the subtree force sums F_i
  union {
    float Rl[LMAX][12]; // FK: local joint transforms (R 9, p 3); dead before cr / f are written
    struct {
      float cr[LMAX][6];  // V_i x_m S_i qd_i
    } b;
    // subtree sums: body force (6) and spatial inertia (10) of every link, transposed and split by
    // link parity ([quantity][l & 1][l >> 1]: the MFMA's A operand runs, read as 16-B vectors),
    // written after the last read of cr
    alignas(16) float xt[16][2][LMAX / 2];
  };
};
struct alignas(16) ConScratch {
  float Jm[MAXR][LDJ];  // J rows (lane = dof column); W = H^-1 J^T stays in registers (lane = dof)
};
union alignas(16) PhaseScratch {
  DynScratch d;
  float obs[64];        // epilogue: observation row staging
  struct {
    // collide: geom segment endpoints, radius, packed type/foot/link; row stride 12 floats (16-B
    // aligned): geoms g and g + 8 land on different banks of the pair passes' gathered reads
    alignas(16) float g[32][12];
    alignas(16) float bs[32][4];  //  bounding sphere (segment midpoint, half length + radius)
    int pl[64];         //          pending (stone << 8 | geom) pairs (< 32 + G), then self pairs
    uint32_t need[NST]; //          per candidate stone: geoms past the bounding test
    alignas(16) float cc[NST][4];  //   per candidate stone: its center relative to the root
  } col;
  struct alignas(16) {
    // sweep: every lane's (rotated) row, rewritten each round, so the publishing stores need no
    // pivot-lane branch; rows are read by the next round's pivot indices.  Row stride 28 floats: the
    // 8-lane groups of a ds_write_b128 then cover 8 distinct 4-bank quads
    float rows[G][28];
  } sw;                 // aliases the dynamics scratch, dead by then
  ConScratch k;
  // contact flags: per contact lambda_n n (3) and its (foot, stone) key, written after the PGS
  alignas(16) float cf[MAXC][4];
};

// The constants block is read-only for the whole launch: address space 4 (constant) lets uniform
// loads become scalar loads and keeps lane-varying ones global (not flat) loads.
using CK = const __attribute__((address_space(4))) Consts;

// Per-lane tree plan and joint constants, read once per launch and kept in registers
// (lane = link for the l* fields, lane = dof for the d* fields, lane = hinge for lo / hi).
struct Topo {
  uint32_t lpath;  // links on the path root..link(lane)
  uint32_t lsub;   // subtree of link(lane)
  uint32_t dsub;   // links moved by dof lane
  float lo, hi;    // limits of hinge lane (link lane + 1)
  float arm;       // armature of dof lane (0 on the root dofs)
  uint32_t jump;   // FK pointer jumping: byte r = the 2^r-th ancestor of link lane (Consts::jump)
};

__device__ Topo load_topo(const Consts& K, int lane) {
  const as_model_t& m = K.model;
  const int nl = m.num_links, nv = K.nv;
  Topo t;
  const int l = lane < nl ? lane : 0;
  const int j = lane < nv ? lane : 0;
  const int hl = lane + 1 < nl ? lane + 1 : 0;
  t.lpath = lane < nl ? K.lpath[l] : 0u;
  t.lsub = lane < nl ? K.lsub[l] : 0u;
  t.dsub = lane < nv ? K.dsub[j] : 0u;
  t.lo = m.lower[hl];
  t.hi = m.upper[hl];
  t.arm = lane >= 6 && lane < nv ? m.armature[lane - 5] : 0.f;
  t.jump = lane < nl ? K.jump[l] : 0u;
  return t;
}

struct EnvS {
  float R[LMAX][9];
  float p[LMAX][3];
  float c0[3];          // root COM (relative), kept past the dynamics phase for integration
  // motion subspace [w; v_O] per dof.  Rows of 12 floats (48 B, two 16-B stores / loads): 16 lanes at
  // that stride cover 16 distinct 16-B slots of the 64 read banks and 8 of the 32 write banks, where a
  // 32-B stride put dofs j and j + 4 (stores) or j + 8 (loads) on the same banks
  alignas(16) float S[NVMAX][12];
  float b[32];          // tau - C
  PhaseScratch x;
  // per row: 1/A_rr, target, bound parameter, in-group coupling.  The bound parameter is what the
  // PGS needs of the row's group: on row 1 of a group mu for a contact triplet (0 otherwise), on
  // row 2 the upper-bound offset, 0 for a contact triplet (+-mu ln) and +inf otherwise ([0, inf))
  alignas(16) float rmeta[MAXR][4];
  float cdir[MAXC][3][3];  // contact frame: normal, tangent 1, tangent 2
  int rlink[MAXR];      // contact rows: link | (link2 + 1) << 8 (link2 = -1: stone); limit rows: -1 - dof
  float rsign[MAXR];
  float cpt[MAXC][3], cn[MAXC][3], csep[MAXC];
  int clink[MAXC], clink2[MAXC], cstone[MAXC], cfoot[MAXC];  // clink2 / cstone: -1 unless self / stone
  float u[NVMAX];
  float qi[LMAX];       // hinge angles, link order (link i -> qi[i-1])
  float tau[LMAX];
  float qt[LMAX];       // AS_ACT_DC_MOTOR: joint position targets (link order)
  float act[AS_ACT_DIM];
  float stones[NST * 3];
  float root_pos[3], root_quat[4];
  int cand[NST];
  uint32_t mask[4];     // contact sensors 0..3 (2, 3: a quadruped's hind feet)
  int ndrop;            // contacts cut by the row budget over this launch's substeps (counters[kCntDropped])
  int nrows;            // constraint rows over this launch's substeps (the next launch's placement cost)
};

struct Smem {
  EnvS env[EPB];
  Topo topo[G];  // per-lane tree plan (shared by both envs; registers cannot hold it)
  unsigned long long stamp_acc[kNumStamps];
  int maxrow;
};

// ------------------------------------------------------------------------------------------------
// cross-lane helpers

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  // bound_ctrl: the quad permutes and row mirrors used here never read outside the row, so the
  // "old" operand is dead and the move folds into the consuming v_add_f32_dpp
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}

__device__ __forceinline__ float readlane_f(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }

// Sum over the 32 lanes of this env's half-wave: DPP butterfly inside each 16-lane row
// (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror), then v_permlane16_swap exchanges the
// two rows of each half so that every lane adds (row 0 + row 1) of its half -- no SGPR round trip.
// Every lane of a half gets the bit-identical value.
__device__ __forceinline__ float row_pair_sum(float v) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
  return __int_as_float(p[0]) + __int_as_float(p[1]);
}

__device__ __forceinline__ float half_sum(float v) {
  v += dpp<0xB1>(v);
  v += dpp<0x4E>(v);
  v += dpp<0x141>(v);
  v += dpp<0x140>(v);
  return row_pair_sum(v);
}

// Sums over the half-wave of N independent values (the W pass and the PGS), two at a time: the
// first v_permlane16_swap exchanges row 1 of value a with row 0 of value b, so one add leaves
// a_l + a_(l+16) in row 0 and b_l + b_(l+16) in row 1; the DPP butterfly then finishes both sums at
// once (A in every lane of row 0, B in row 1), and a second swap hands A and B to every lane of the
// half.  A pair costs 8 instructions instead of 14; an odd last value takes the swap with itself
// first (7).  The tree: the cross-row add, then a balanced tree over the 16 row lanes (oracle
// tree32); every lane gets the bit-identical value.
template <int N>
__device__ __forceinline__ void half_sum_n(float (&v)[N]) {
  constexpr int P = (N + 1) / 2;
  float c[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int b = 2 * p + 1 < N ? 2 * p + 1 : 2 * p;
    const auto s = __builtin_amdgcn_permlane16_swap(__float_as_int(v[2 * p]), __float_as_int(v[b]), false, false);
    c[p] = __int_as_float(s[0]) + __int_as_float(s[1]);
  }
#pragma unroll
  for (int p = 0; p < P; ++p) c[p] += dpp<0xB1>(c[p]);
#pragma unroll
  for (int p = 0; p < P; ++p) c[p] += dpp<0x4E>(c[p]);
#pragma unroll
  for (int p = 0; p < P; ++p) c[p] += dpp<0x141>(c[p]);
#pragma unroll
  for (int p = 0; p < P; ++p) c[p] += dpp<0x140>(c[p]);
#pragma unroll
  for (int p = 0; p < P; ++p) {
    if (2 * p + 1 < N) {
      const auto s = __builtin_amdgcn_permlane16_swap(__float_as_int(c[p]), __float_as_int(c[p]), false, false);
      v[2 * p] = __int_as_float(s[0]);
      v[2 * p + 1] = __int_as_float(s[1]);
    } else {
      v[2 * p] = c[p];
    }
  }
}

// Exclusive prefix sum over this env's half-wave of a count c in [0, 3], and the half's total:
// two ballots (bit 0 and bit 1 of c) and popcounts, no cross-lane data movement.
__device__ __forceinline__ int half_scan3(int c, int& total) {
  const int sh = threadIdx.x & 32;
  const uint32_t m0 = (uint32_t)(__ballot((c & 1) != 0) >> sh);
  const uint32_t m1 = (uint32_t)(__ballot((c & 2) != 0) >> sh);
  const uint32_t lt = (1u << (threadIdx.x & 31)) - 1u;
  total = __popc(m0) + 2 * __popc(m1);
  return __popc(m0 & lt) + 2 * __popc(m1 & lt);
}

template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, true);
}

// OR over the half-wave of two values at once (the pairing of half_sum_n)
__device__ __forceinline__ void half_or2(uint32_t& x, uint32_t& y) {
  const auto s = __builtin_amdgcn_permlane16_swap((int)x, (int)y, false, false);
  uint32_t c = (uint32_t)s[0] | (uint32_t)s[1];
  c |= dpp_u<0xB1>(c);
  c |= dpp_u<0x4E>(c);
  c |= dpp_u<0x141>(c);
  c |= dpp_u<0x140>(c);
  const auto t = __builtin_amdgcn_permlane16_swap((int)c, (int)c, false, false);
  x = (uint32_t)t[0];
  y = (uint32_t)t[1];
}

// half_min of N values two at a time (the pairing of half_sum_n; min is exact, so any order gives
// the same value)
template <int N>
__device__ __forceinline__ void half_min_n(float (&v)[N]) {
  static_assert(N % 2 == 0, "pairs");
  constexpr int P = N / 2;
  float c[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const auto s = __builtin_amdgcn_permlane16_swap(__float_as_int(v[2 * p]), __float_as_int(v[2 * p + 1]), false, false);
    c[p] = fminf(__int_as_float(s[0]), __int_as_float(s[1]));
  }
#pragma unroll
  for (int p = 0; p < P; ++p) c[p] = fminf(c[p], dpp<0xB1>(c[p]));
#pragma unroll
  for (int p = 0; p < P; ++p) c[p] = fminf(c[p], dpp<0x4E>(c[p]));
#pragma unroll
  for (int p = 0; p < P; ++p) c[p] = fminf(c[p], dpp<0x141>(c[p]));
#pragma unroll
  for (int p = 0; p < P; ++p) c[p] = fminf(c[p], dpp<0x140>(c[p]));
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const auto s = __builtin_amdgcn_permlane16_swap(__float_as_int(c[p]), __float_as_int(c[p]), false, false);
    v[2 * p] = __int_as_float(s[0]);
    v[2 * p + 1] = __int_as_float(s[1]);
  }
}

// diagnostic phase stamps (off when p == nullptr): each wave accumulates its s_memtime deltas per
// phase in LDS and adds them to the device counters once, at the end of the launch -- a global
// atomic per phase boundary would put a contended memory round trip into the next phase.
// With p[kWaveRecFlag] != 0 each wave also writes a record of its own (the last launch's waves:
// phase cycles, total, start / end time, HW_ID / XCC_ID, rows and contacts summed over substeps per
// env) at p + kWaveRecBase + block * kWaveRecWords, for tail analysis (scripts/stamps.py).
constexpr int kWaveRecFlag = 31, kWaveRecBase = 64, kWaveRecWords = 26;
static_assert(16 + kNumStamps <= kWaveRecFlag && kNumStamps + 11 <= kWaveRecWords, "stamp slots");
struct Stamp {
  unsigned long long* p;
  unsigned long long* acc;  // LDS, kNumStamps
  unsigned long long t;
  unsigned long long t0 = 0ull, rt0 = 0ull;  // s_memtime / s_memrealtime (100 MHz) at the start
  unsigned rows = 0u, cons = 0u;
  __device__ void start() {
    if (p) {
      if (threadIdx.x < kNumStamps) acc[threadIdx.x] = 0ull;
      t = t0 = __builtin_amdgcn_s_memtime();
      rt0 = __builtin_amdgcn_s_memrealtime();
    }
  }
  __device__ void count(int nrow, int nc) {
    if (p) {
      rows += (unsigned)nrow;
      cons += (unsigned)nc;
    }
  }
  __device__ void mark(int k) {
    if (p) {
      unsigned long long now = __builtin_amdgcn_s_memtime();
      if (threadIdx.x == 0) acc[k] += now - t;
      t = now;
    }
  }
  __device__ void flush() {
    if (p) {
      __syncthreads();
      unsigned long long tot = 0;
      for (int k = 0; k < kNumStamps; ++k) tot += acc[k];
      if (p[kWaveRecFlag]) {
        // per-wave records, plain stores only: the atomics of the aggregate mode would queue in
        // front of the late waves' own memory traffic and distort exactly the tail being measured
        unsigned long long* rec = p + kWaveRecBase + (size_t)blockIdx.x * kWaveRecWords;
        const unsigned long long now = __builtin_amdgcn_s_memtime();
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
        const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
        const int k = threadIdx.x;
        if (k < kNumStamps) rec[k] = acc[k];
        if (k == 0) {
          rec[kNumStamps] = tot; rec[kNumStamps + 1] = t0; rec[kNumStamps + 2] = now;
          rec[kNumStamps + 9] = rt0; rec[kNumStamps + 10] = __builtin_amdgcn_s_memrealtime();
          rec[kNumStamps + 3] = hw; rec[kNumStamps + 4] = xcc;
          rec[kNumStamps + 5] = rows; rec[kNumStamps + 7] = cons;
        }
        if (k == 32) { rec[kNumStamps + 6] = rows; rec[kNumStamps + 8] = cons; }
      } else {
        if (threadIdx.x < kNumStamps) {
          atomicAdd(p + threadIdx.x, acc[threadIdx.x]);
          atomicMax(p + 16 + threadIdx.x, acc[threadIdx.x]);  // slots 16..: per-phase maximum
        }
        if (threadIdx.x == 0) atomicMax(p + kNumStamps, tot);  // slot kNumStamps: the slowest wave's total
      }
    }
  }
};

// ------------------------------------------------------------------------------------------------
// Mask walks.  take_bit pops the lowest set bit (0 and !valid once the mask is empty); the walks run
// a wave-uniform number of iterations (the model's longest path / largest subtree) with several
// rows loaded per iteration, and add an invalid row as +0 (no-op), so the LDS loads of one
// iteration are independent of each other and of the running sum.
__device__ __forceinline__ int take_bit(uint32_t& m, bool& valid) {
  valid = m != 0u;
  const int l = valid ? __builtin_ctz(m) : 0;
  m &= m - 1u;
  return l;
}

// The dynamics walks read an invalid slot from row kZeroRow of their tables, which holds +0 (written
// in every substep by lane kZeroRow): adding it is the +0 a select would add, without the select.
// num_hinges <= AS_ACT_DIM keeps that row past every model's links.
constexpr int kZeroRow = LMAX - 1;
static_assert(AS_ACT_DIM + 1 <= kZeroRow, "zero row past the links");
__device__ __forceinline__ int take_bit_z(uint32_t& m) {
  const int l = m != 0u ? __builtin_ctz(m) : kZeroRow;
  m &= m - 1u;
  return l;
}

// acc += sum of rows[l] over the set bits l of `mask`, ascending, U rows per iteration.
template <int W, int U>
__device__ __forceinline__ void path_sum(uint32_t mask, int n_max, float (&acc)[W], const float (*rows)[W]) {
  for (int it = 0; it < n_max; it += U) {
    int l[U];
#pragma unroll
    for (int u = 0; u < U; ++u) l[u] = take_bit_z(mask);
    float x[U][W];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < W; ++k) x[u][k] = rows[l[u]][k];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < W; ++k) acc[k] += x[u][k];
  }
}

// FK by ancestor-path walks.  Local joint transforms are formed in parallel (lane = link); then
// lane i composes the transforms on its own path root -> i, which is the same sequence of products
// a level-by-level pass would form (R_i = R_parent Rl_i, p_i = p_parent + R_parent t_i), with no
// level barriers: the tree depth only sets the length of the longest lane's loop.
// kDyn: also the link's spatial quantities for the dynamics (COM, spatial inertia at O, motion
// subspace of its hinge, S_i qd_i) from the registers of the walk, and the six root columns.
// Per-lane joint constants of the local transform (lane = link), read once per launch and kept in
// registers across the substeps (as lane-varying global loads they were an L2 round trip at the head
// of every substep's FK)
struct LinkC {
  float oq[4], ax[3], an[3], op[3];
};
__device__ __forceinline__ LinkC load_link(const Consts& K, int lane) {
  const as_model_t& m = K.model;
  const int i = lane >= 1 && lane < m.num_links ? lane : 0;
  LinkC c;
#pragma unroll
  for (int k = 0; k < 4; ++k) c.oq[k] = m.offset_quat[i][k];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    c.ax[k] = m.axis[i][k];
    c.an[k] = m.anchor[i][k];
    c.op[k] = m.offset_pos[i][k];
  }
  return c;
}

template <bool kDyn>
__device__ __forceinline__ void fk(const Consts& K, EnvS& s, int lane, const Topo& tp, LinkC lc, int max_path) {
  const as_model_t& m = K.model;
  const int nl = m.num_links;
  DynScratch& d = s.x.d;
  // opaque per call: nothing derived from them is hoisted out of the substep loop
  asm volatile("" : "+v"(lc.oq[0]), "+v"(lc.oq[1]), "+v"(lc.oq[2]), "+v"(lc.oq[3]), "+v"(lc.ax[0]),
               "+v"(lc.ax[1]), "+v"(lc.ax[2]));
  asm volatile("" : "+v"(lc.an[0]), "+v"(lc.an[1]), "+v"(lc.an[2]), "+v"(lc.op[0]), "+v"(lc.op[1]),
               "+v"(lc.op[2]));
  // lane i: its joint's local transform A = (Rl, tl) (rotation row-major, translation), the identity
  // on the root lane; then pointer jumping over the tree (fk_rounds rounds): A_i <- A_a o A_i with a
  // the 2^r-th ancestor of i (the root's identity past the path), so after round r A_i is the product
  // of the 2^(r+1) transforms ending at i, and after the last one the whole path root -> i -- three
  // dependent compositions for the walker's 8-link paths instead of eight.  (Ra, ta) o (Rb, tb) =
  // (Ra Rb, ta + Ra tb), as_matmul3 / as_matvec3 operations; oracle/physics.c kinematics forms the same
  // products in the same association.
  float A[12];
#pragma unroll
  for (int k = 0; k < 12; ++k) A[k] = k == 0 || k == 4 || k == 8 ? 1.f : 0.f;
  if (lane >= 1 && lane < nl) {
    const int i = lane;
    float Roff[9], Rj[9], Ro[3], t[3], tmp[3];
    quat_to_mat(lc.oq, Roff);
    axis_angle_mat(lc.ax, s.qi[i - 1], Rj);
    matmul3(Roff, Rj, A);
    matvec3(Rj, lc.an, Ro);
    for (int k = 0; k < 3; ++k) t[k] = lc.an[k] - Ro[k];
    matvec3(Roff, t, tmp);
    for (int k = 0; k < 3; ++k) A[9 + k] = tmp[k] + lc.op[k];
  }
  __syncthreads();  // (also publishes the actuator's tau before the dynamics read it)
  {
    const int rounds = __builtin_amdgcn_readfirstlane(K.fk_rounds);
    const uint32_t jw = tp.jump;
    typedef __attribute__((address_space(3))) v4f* lds_v4p_t;
    for (int r = 0; r < rounds; ++r) {
      // publish this round's A (rows of 12 floats: three 16-B stores), read the ancestor's.  One wave:
      // its LDS operations complete in issue order, so the reads see this round's stores and the next
      // round's stores cannot overtake them; the empty asm keeps the compiler from reordering them
      if (lane < nl) {
        lds_v4p_t own = (lds_v4p_t)(&d.Rl[lane][0]);
        own[0] = v4f{A[0], A[1], A[2], A[3]};
        own[1] = v4f{A[4], A[5], A[6], A[7]};
        own[2] = v4f{A[8], A[9], A[10], A[11]};
      }
      asm volatile("" ::: "memory");
      const int anc = (jw >> (8 * r)) & 0xff;
      const lds_v4p_t ar = (lds_v4p_t)(&d.Rl[anc][0]);
      const v4f q0 = ar[0], q1 = ar[1], q2 = ar[2];
      asm volatile("" ::: "memory");
      const float Ra[9] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x};
      const float ta[3] = {q2.y, q2.z, q2.w};
      float Rn[9], w[3];
      matmul3(Ra, A, Rn);
      matvec3(Ra, A + 9, w);
#pragma unroll
      for (int k = 0; k < 9; ++k) A[k] = Rn[k];
#pragma unroll
      for (int k = 0; k < 3; ++k) A[9 + k] = ta[k] + w[k];
    }
  }
  float R0[9];
  quat_to_mat(s.root_quat, R0);
  if (lane < nl) {
    // the world pose: R = R0 A_R, p = R0 A_t (relative to the root origin)
    float R[9], p[3];
    matmul3(R0, A, R);
    matvec3(R0, A + 9, p);
#pragma unroll
    for (int k = 0; k < 9; ++k) s.R[lane][k] = R[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) s.p[lane][k] = p[k];
    if (kDyn) {
      const int i = lane;
      float cw[3];
      matvec3(R, m.com[i], cw);
      const float c[3] = {p[0] + cw[0], p[1] + cw[1], p[2] + cw[2]};
      d.c[i][0] = c[0]; d.c[i][1] = c[1]; d.c[i][2] = c[2];
      const float* Il = m.inertia[i];
      const float Im[9] = {Il[0], Il[3], Il[4], Il[3], Il[1], Il[5], Il[4], Il[5], Il[2]};
      const float Rt[9] = {R[0], R[3], R[6], R[1], R[4], R[7], R[2], R[5], R[8]};
      float T[9], Iw[9];
      matmul3(R, Im, T);
      matmul3(T, Rt, Iw);
      const float mass = m.mass[i], cc = dot3(c, c);
      float* B = d.Ib[i];
      B[0] = mass;
      B[1] = mass * c[0]; B[2] = mass * c[1]; B[3] = mass * c[2];
      B[4] = Iw[0] + mass * (cc - c[0] * c[0]);
      B[5] = Iw[4] + mass * (cc - c[1] * c[1]);
      B[6] = Iw[8] + mass * (cc - c[2] * c[2]);
      B[7] = Iw[1] - mass * c[0] * c[1];
      B[8] = Iw[2] - mass * c[0] * c[2];
      B[9] = Iw[5] - mass * c[1] * c[2];
      if (i > 0) {
        float a[3], o[3];
        matvec3(R, lc.ax, a);
        matvec3(R, lc.an, o);
        for (int k = 0; k < 3; ++k) o[k] += p[k];
        float S[6] = {a[0], a[1], a[2], 0.f, 0.f, 0.f};
        cross3(o, a, S + 3);
        const float qd = s.u[6 + i - 1];
        *reinterpret_cast<v4f*>(&s.S[6 + i - 1][0]) = v4f{S[0], S[1], S[2], S[3]};
        *reinterpret_cast<v4f*>(&s.S[6 + i - 1][4]) = v4f{S[4], S[5], 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 6; ++k) d.Sq[i][k] = S[k] * qd;
      }
    }
  }
  if (kDyn && lane == kZeroRow) {  // the walks' +0 rows (see take_bit_z)
#pragma unroll
    for (int k = 0; k < 10; ++k) d.Ib[kZeroRow][k] = 0.f;
#pragma unroll
    for (int k = 0; k < 6; ++k) d.Sq[kZeroRow][k] = 0.f;
  }
  if (kDyn) {
    // root columns need the root COM c0 = R0 com_0 (p_0 = 0): every lane forms it itself
    float c0[3];
    matvec3(R0, m.com[0], c0);
    if (lane < 3) s.c0[lane] = c0[lane];
    if (lane < 6) {
      float S[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      const int k = lane % 3;
      if (lane < 3) {
        S[3 + k] = 1.f;
      } else {
        float e[3] = {0.f, 0.f, 0.f};
        e[k] = 1.f;
        S[k] = 1.f;
        cross3(c0, e, S + 3);
      }
      *reinterpret_cast<v4f*>(&s.S[lane][0]) = v4f{S[0], S[1], S[2], S[3]};
      *reinterpret_cast<v4f*>(&s.S[lane][4]) = v4f{S[4], S[5], 0.f, 0.f};
    }
  }
  __syncthreads();
}

// Two-block f32 MFMA (v_mfma_f32_32x32x1_2b_f32): one 32 x 32 block per env (block b = lanes
// 32b..32b+31), K = 1 per instruction, lane l supplying A[l % 32][k] and B[k][l % 32] of its own env;
// the result is bit for bit an fmaf chain over k (scripts/probes/mfma_2b_probe.hip).  Register v of
// block b holds row 8(v/4) + 4h + v%4 on lane half h, column lane % 32; one v_permlane32_swap per
// register pair (blocks 0 and 1 trade halves) leaves lane n with column n of its own env's block.
typedef float f32x32 __attribute__((ext_vector_type(32)));
__device__ __forceinline__ void mfma_columns(const f32x32& acc, float (&col)[32]) {
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    const auto p = __builtin_amdgcn_permlane32_swap(__float_as_int(acc[v]), __float_as_int(acc[16 + v]), false, false);
    const int r0 = 8 * (v >> 2) + (v & 3);
    col[r0] = __int_as_float(p[0]);
    col[r0 + 4] = __int_as_float(p[1]);
  }
}

// RNEA bias forces (qdd = 0) and composite inertias by path / subtree walks (lanes = links):
//   V_i  = V_0 + sum_{l on path, root->i} S_l qd_l            (= V_parent + S_i qd_i)
//   A_i  = A_0 + sum_{l on path} V_l x_m S_l qd_l             (= A_parent + V_i x S_i qd_i)
//   f_i  = I_i A_i + V_i x_f I_i V_i - gravity wrench
//   F_i  = sum_{l in subtree(i) (i included), ascending} f_l,  likewise Ic_i from the I_l
// The subtree sums are one matrix product per env on the matrix cores: with X the 16 x LMAX table of
// every link's (f, I) and M_il = [l in subtree(i)], the two-block f32 MFMA forms (X M^T) over LMAX K
// steps, an fmaf chain over l ascending from +0 for every (quantity, link) -- the root's row is the
// whole tree (oracle/physics.c subtree_sums restates the chain).  Then per dof j: C_j = S_j . F_link(j),
// b_j = tau_j - C_j (returned, also in LDS), Fh_j = Ic_link(j) S_j.
template <int NV>
__device__ __forceinline__ float dynamics(const Consts& K, EnvS& s, int lane, const Topo& tp, float gravity,
                                          float (&Sj)[6], float (&Fj)[6], int max_path) {
  const as_model_t& m = K.model;
  const int nl = m.num_links, nv = K.nv;
  DynScratch& d = s.x.d;
  float V[6], A[6];
  {
    const float* u = s.u;
    float wxc[3], vxw[3];
    cross3(s.c0, u + 3, wxc);
    cross3(u, u + 3, vxw);
    for (int k = 0; k < 3; ++k) {
      V[k] = u[3 + k];
      V[3 + k] = u[k] + wxc[k];
      A[k] = 0.f;
      A[3 + k] = vxw[k];
    }
  }
  if (lane < nl) {
    path_sum<6, 4>(tp.lpath & ~1u, max_path, V, d.Sq);
    if (lane > 0) {
      float Sq[6], cr[6];
#pragma unroll
      for (int k = 0; k < 6; ++k) Sq[k] = d.Sq[lane][k];
      crm(V, Sq, cr);
#pragma unroll
      for (int k = 0; k < 6; ++k) d.b.cr[lane][k] = cr[k];
    }
  }
  if (lane == kZeroRow) {  // the walks' +0 row (see take_bit_z); FK's Rl, which b aliases, is dead
#pragma unroll
    for (int k = 0; k < 6; ++k) d.b.cr[kZeroRow][k] = 0.f;
  }
  __syncthreads();
  float f[6], Ib[10];
  if (lane < nl) {
    path_sum<6, 4>(tp.lpath & ~1u, max_path, A, d.b.cr);
#pragma unroll
    for (int k = 0; k < 10; ++k) Ib[k] = d.Ib[lane][k];
    float IA[6], IV[6], x[6];
    inertia_mul(Ib, A, IA);
    inertia_mul(Ib, V, IV);
    crf(V, IV, x);
    const float mg[3] = {0.f, 0.f, Ib[0] * gravity};
    float cxmg[3];
    cross3(d.c[lane], mg, cxmg);
    for (int k = 0; k < 3; ++k) {
      f[k] = IA[k] + x[k] - cxmg[k];
      f[3 + k] = IA[3 + k] + x[3 + k] - mg[k];
    }
  }
  // every link's (f, I) into the transposed table; links past nl (and the lanes up to LMAX) add +0
  if (lane < LMAX) {
    const bool lv = lane < nl;
#pragma unroll
    for (int k = 0; k < 6; ++k) d.xt[k][lane & 1][lane >> 1] = lv ? f[k] : 0.f;
#pragma unroll
    for (int k = 0; k < 10; ++k) d.xt[6 + k][lane & 1][lane >> 1] = lv ? Ib[k] : 0.f;
  }
  __syncthreads();
  {
    // Both envs in one single-block v_mfma_f32_32x32x2_f32 (K = 2 per instruction, an fmaf chain over
    // its two K entries in order: scripts/probes/mfma_x2_probe.hip): row r = 16 env + quantity, column
    // = link i, instruction t takes link slots 2t (lanes 0-31) and 2t + 1 (lanes 32-63).  A operand:
    // lane l supplies X_env(r)[r % 16][2t + l / 32] (r = l % 32, the env's table in LDS); B operand:
    // lane l supplies M_{i, 2t + l / 32}, i = l % 32.  D row r, column i sits at register v of lane
    // half h with r = 8 (v / 4) + 4 h + v % 4: one v_permlane32_swap per register pair leaves lane
    // (env e, link i) with its 16 sums.
    const int tid = threadIdx.x, h = tid >> 5, r = tid & 31;
    EnvS* envs = &s - h;  // sm.env[0]
    const float* xr = envs[r >> 4].x.d.xt[r & 15][h];
    const uint32_t sub = (lane < nl ? tp.lsub : 0u) >> h;
    float xa[LMAX / 2];
    // the three 16-B reads issued together and passed through an empty asm (one wait): left to the
    // scheduler, each read reused the previous one's registers and waited under the MFMA chain
    static_assert(LMAX / 2 == 12, "three quads");
    v4f xq[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) xq[t] = *reinterpret_cast<const v4f*>(xr + 4 * t);
    asm volatile("" : "+v"(xq[0]), "+v"(xq[1]), "+v"(xq[2]));
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      xa[4 * t] = xq[t].x; xa[4 * t + 1] = xq[t].y; xa[4 * t + 2] = xq[t].z; xa[4 * t + 3] = xq[t].w;
    }
    typedef float f32x16 __attribute__((ext_vector_type(16)));
    f32x16 acc = {};
    // only the instructions that hold a link: num_links = NV - 5 (as_create: one hinge per non-root
    // link), and a slot past it adds +0 products to an accumulator that started at +0 -- the same bits
    // (the walker's 22 links use 11 of the 12 steps, the quadruped's 13 links 7)
    constexpr int kSubSteps = (NV - 5 + 1) / 2;
    static_assert(kSubSteps <= LMAX / 2, "link slots");
#pragma unroll
    for (int t = 0; t < kSubSteps; ++t)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xa[t], (float)((sub >> (2 * t)) & 1u), acc, 0, 0, 0);
    float col[16];
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      const auto pr = __builtin_amdgcn_permlane32_swap(__float_as_int(acc[w]), __float_as_int(acc[8 + w]), false, false);
      const int q0 = 8 * (w >> 2) + (w & 3);
      col[q0] = __int_as_float(pr[0]);
      col[q0 + 4] = __int_as_float(pr[1]);
    }
    if (lane < nl) {  // lane i: F_i (0..5), Ic_i (6..15)
#pragma unroll
      for (int k = 0; k < 6; ++k) d.Sq[lane][k] = col[k];  // Sq is dead: F_i
#pragma unroll
      for (int k = 0; k < 10; ++k) d.Ic[lane][k] = col[6 + k];
    }
  }
  __syncthreads();
  float bj = 0.f;
  if (lane < nv) {
    const int j = lane;
    const int link = j < 6 ? 0 : j - 5;
    float F[6], Ic[10], S[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) F[k] = d.Sq[link][k];
#pragma unroll
    for (int k = 0; k < 10; ++k) Ic[k] = d.Ic[link][k];
#pragma unroll
    for (int k = 0; k < 6; ++k) S[k] = s.S[j][k];
    const float Cj = dot6(S, F);
    bj = (j < 6 ? 0.f : s.tau[j - 6]) - Cj;
    s.b[j] = bj;
    inertia_mul(Ic, S, Fj);
#pragma unroll
    for (int k = 0; k < 6; ++k) Sj[k] = S[k];
  } else {
    if (lane < 32) s.b[lane] = 0.f;
#pragma unroll
    for (int k = 0; k < 6; ++k) Sj[k] = Fj[k] = 0.f;
  }
  __syncthreads();
  return bj;
}

// Row j of the joint-space inertia H (lane j):
//   H_jk = S_k . (Ic_link(j) S_j)  if dof k is on the path of link(j) (k ancestor-or-self),
//        = S_j . (Ic_link(k) S_k)  if dof j is on the path of link(k),   else 0;  + armature.
// Every product P_kj = S_k . Fh_j (Fh_j = Ic_link(j) S_j) comes from six K steps of the two-block
// f32 MFMA (one block per env; A: lane k's S_k, B: lane j's Fh_j, both in registers from dynamics):
// P_kj is an fmaf chain over the six spatial components (oracle/physics.c chain6).  After the
// column shuffle lane j holds P_kj for every k: the path-side entries of its row.  Lane j publishes
// its row masked to its path, (k on path(j)) ? P_kj (+ armature on the diagonal) : +0, in LDS; the
// other side is the transposed entry of that matrix (lane k's P_jk for j on path(k)), one b32 read
// per column.  Lanes past NV read the all-zero padding column NV.
template <int NV>
__device__ __forceinline__ void h_row(EnvS& s, int lane, const Topo& tp, uint32_t anc_j, const float (&Sj)[6],
                                      const float (&Fj)[6], float (&Hr)[NV]) {
  static_assert(NV < LDJ, "padding column");
  // opaque per substep: the 27 column masks derived from it would otherwise be hoisted out of the
  // substep loop as SGPR pairs and spilled to VGPR lanes (a readlane per column per substep)
  asm volatile("" : "+v"(anc_j));
  const int j = lane < NV ? lane : 0;
  f32x32 acc = {};
#pragma unroll
  for (int a = 0; a < 6; ++a) acc = __builtin_amdgcn_mfma_f32_32x32x1f32(Sj[a], Fj[a], acc, 0, 0, 0);
  float col[32];
  mfma_columns(acc, col);
  const float arm = tp.arm;
  const uint32_t on = lane < NV ? anc_j : 0u;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const float h = k == j ? col[k] + arm : col[k];
    Hr[k] = (on >> k) & 1u ? h : 0.f;
  }
  float(*M)[LDJ] = s.x.k.Jm;
  if (lane < NV) {
#pragma unroll
    for (int q = 0; q < LDJ / 4; ++q) {
      float e[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) e[c] = 4 * q + c < NV ? Hr[4 * q + c] : 0.f;
      *reinterpret_cast<v4f*>(&M[lane][4 * q]) = v4f{e[0], e[1], e[2], e[3]};
    }
  }
  // the root's six dofs are on every dof's path (ancmask bits 0-5, as_create), so their entries are
  // never taken from the transpose: those reads and selects are not issued (lanes >= NV keep the +0 of
  // the select above, as before)
  constexpr int kRootDofs = 6;
  const int jj = lane < NV ? lane : NV;
  float t[NV];
#pragma unroll
  for (int k = kRootDofs; k < NV; ++k) t[k] = M[k][jj];
  // (a register value, not a load: a select between two loads becomes a load from a selected
  // address, which puts Hr in scratch)
#pragma unroll
  for (int k = kRootDofs; k < NV; ++k) {
    asm volatile("" : "+v"(t[k]));
    Hr[k] = (on >> k) & 1u ? Hr[k] : t[k];
  }
}

// H^-1 by the block sweep operator on BxB pivot blocks, with column rotation (same arithmetic as
// oracle/physics.c sweep_inverse).  H is padded to an order NP (a multiple of B) with identity rows
// and columns.  Lane i holds row i in Hr, rotated so that the current pivot columns are always
// Hr[0..B-1]: a round shifts every row left by B and appends the B new pivot-column entries, so the
// register row is only indexed by compile-time constants, no per-column select is needed and (B
// even) pairs stay aligned for packed FMAs.  Round on pivots P = {p..p+B-1}, D = (H_PP)^-1:
//   the pivot lanes publish their rows without the pivot columns (Q) and H_PP (Pb);
//   every lane forms D (in-register sweep of the uniform BxB block);
//   row'_j = alpha row_j - sum_c beta_c Q_cj, new pivot-column entries = beta, with
//     (alpha, beta) = (1, a_iP D)  for i not in P   (a_ij - a_iP D a_Pj;  a_iP <- a_iP D)
//     (alpha, beta) = (0, -D_t)    for pivot lane t (D a_Pj;  a_PP <- -D).
// After all rounds the rotation is back to the identity and the rows hold -H^-1.
// 4x4 SPD inverse by 2x2 blocks (Schur complement): two 2x2 determinant inverses instead of four
// sequential pivots, so the chain on each sweep round's critical path is two divisions deep.
//   M = [A B; C D]:  Ai = A^-1, X = Ai B, Y = C Ai, S = D - C X, Si = S^-1,
//   M^-1 = [Ai + (X Si) Y, -(X Si); -(Si Y), Si]       (oracle/physics.c block_inverse: same order)
// The 2x2 blocks are kept as rows of packed pairs: a row of a product is one v_pk_mul + one
// v_pk_fma (per element the same mul and fmaf as the scalar form), the Schur difference and the
// final sum one v_pk_add each.
__device__ __forceinline__ void inv2(float a, float b, float c, float d, v2f (&o)[2]) {
  const float id = 1.0f / fmaf(a, d, -(b * c));
  o[0] = v2f{d, -b} * v2f{id, id};
  o[1] = v2f{-c, a} * v2f{id, id};
}
__device__ __forceinline__ void mul2(const v2f (&x)[2], const v2f (&y)[2], v2f (&o)[2]) {
#pragma unroll
  for (int i = 0; i < 2; ++i)
    o[i] = __builtin_elementwise_fma(v2f{x[i].y, x[i].y}, y[1], v2f{x[i].x, x[i].x} * y[0]);
}
template <int B>
__device__ __forceinline__ void block_inverse(float (&M)[B][B]) {  // M <- M^-1 (SPD)
  static_assert(B == 4, "2x2-block Schur inverse");
  const v2f A[2] = {v2f{M[0][0], M[0][1]}, v2f{M[1][0], M[1][1]}};
  const v2f Bm[2] = {v2f{M[0][2], M[0][3]}, v2f{M[1][2], M[1][3]}};
  const v2f C[2] = {v2f{M[2][0], M[2][1]}, v2f{M[3][0], M[3][1]}};
  const v2f D[2] = {v2f{M[2][2], M[2][3]}, v2f{M[3][2], M[3][3]}};
  v2f Ai[2], X[2], Y[2], CX[2], S[2], Si[2], XS[2], XSY[2], SY[2];
  inv2(A[0].x, A[0].y, A[1].x, A[1].y, Ai);
  mul2(Ai, Bm, X);
  mul2(C, Ai, Y);
  mul2(C, X, CX);
#pragma unroll
  for (int i = 0; i < 2; ++i) S[i] = D[i] - CX[i];
  inv2(S[0].x, S[0].y, S[1].x, S[1].y, Si);
  mul2(X, Si, XS);
  mul2(XS, Y, XSY);
  mul2(Si, Y, SY);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const v2f top = Ai[i] + XSY[i];
    M[i][0] = top.x; M[i][1] = top.y;
    M[i][2] = -XS[i].x; M[i][3] = -XS[i].y;
    M[2 + i][0] = -SY[i].x; M[2 + i][1] = -SY[i].y;
    M[2 + i][2] = Si[i].x; M[2 + i][3] = Si[i].y;
  }
}

// The sweep's layout (include/as_detmath.h AS_SWEEP_PAD): the NV dofs padded to NP with identity rows /
// columns at padded index PAD, the NB = NP / 4 pivot blocks swept LAST block first (the limbs before the
// root).  A lane keeps ITS dof's row (lane k < NV: dof k, padded row padded(k); lane NV + q: pad row
// PAD + q), so no row moves between lanes; the columns start in the round-0 rotated order -- blocks
// NB - 1, NB - 2, ..., 0, natural order inside a block -- which the rotation below returns to after the
// last round.  SKIP bit r (NB - 1) + jb: in round r the pivot rows are exactly zero in column quad jb
// (as_create's structural check, sweep_skip_mask): that quad's update is the identity and is not issued
// (the pivot rows' zeros are +0 and stay +0, so every skipped fmaf would have returned its addend bit for
// bit; the oracle performs them).
template <int NV>
struct SweepLayout {
  static constexpr int NP = (NV + kSweepB - 1) / kSweepB * kSweepB;
  static constexpr int NB = NP / kSweepB;
  static constexpr int NQ = NB - 1;
  static constexpr int PAD = AS_SWEEP_PAD(NV);
  static constexpr int padded(int k) { return k < PAD ? k : k + (NP - NV); }
  static constexpr int pos(int P) { return (NB - 1 - P / kSweepB) * kSweepB + P % kSweepB; }  // round-0 register
};

// Software-pipelined and branch-free.  Every lane publishes its whole rotated row each round (no
// pivot-lane branch: the sweep is one basic block, so the scheduler can interleave across rounds), and
// its new leading quad -- the next round's pivot columns -- first: right after that store every lane
// reads the next pivot block back and inverts it, and the 4x4 inverse's division chain overlaps the
// round's remaining column updates instead of heading the next round.  Per element the operations
// and their order are those of oracle/physics.c sweep_inverse: only the issue order changes.
template <int NV, uint64_t SKIP>
__device__ void sweep_inverse(EnvS& s, int lane, float (&Hr)[SweepLayout<NV>::NP]) {
  typedef SweepLayout<NV> L;
  constexpr int NP = L::NP, NB = L::NB, NQ = L::NQ, B = kSweepB;
  static_assert(B == 4, "16-B pivot rows");
  static_assert(NP <= 28, "row buffer stride");
  static_assert(NQ * NB <= 64, "skip mask bits");
  // this lane's padded row
  const int prow = lane < NV ? (lane < L::PAD ? lane : lane + (NP - NV)) : (lane < NP ? L::PAD + (lane - NV) : lane);
  // LDS operations of a wave complete in issue order: a round's stores cannot overtake the previous
  // round's reads of the same rows.  Explicit 16-B accesses on a native 4-vector type (float4 is a
  // struct whose copies SROA splits into b96 + b32 pairs)
  float(*Rw)[28] = s.x.sw.rows;
  v4f* own = reinterpret_cast<v4f*>(Rw[prow]);
  // a row quad is stored only if the next round reads it: round r reads quad jb of its pivot rows
  // unless SKIP says those are +0 (the rows are LDS scratch, dead after the sweep)
#pragma unroll
  for (int j = 0; j < NP; j += 4)
    if (j == 0 || !((SKIP >> (j / 4 - 1)) & 1ull)) own[j / 4] = v4f{Hr[j], Hr[j + 1], Hr[j + 2], Hr[j + 3]};
  __syncthreads();
  float D[B][B];
#pragma unroll
  for (int a = 0; a < B; ++a) {
    const v4f d = *reinterpret_cast<const v4f*>(Rw[(NB - 1) * B + a]);
    D[a][0] = d.x; D[a][1] = d.y; D[a][2] = d.z; D[a][3] = d.w;
  }
  block_inverse<B>(D);
  // unrolled over the rounds: the column rotation is then register renaming and the pivot lanes /
  // padding / skipped quads are known per round
#pragma unroll
  for (int r = 0; r < NB; ++r) {
    const int p = (NB - 1 - r) * B;  // the pivot block's padded rows
    const int t = prow - p;
    const bool piv = (unsigned)t < (unsigned)B;
    // the pivot rows' other columns (stored last round, or above for r = 0); a skipped quad's are
    // never read
    v4f x[NQ][B];
#pragma unroll
    for (int jb = 0; jb < NQ; ++jb)
#pragma unroll
      for (int c = 0; c < B; ++c)
        if (!((SKIP >> (r * NQ + jb)) & 1ull)) x[jb][c] = *reinterpret_cast<const v4f*>(&Rw[p + c][B + 4 * jb]);
    // packed pairs written out (the file is built without the SLP vectorizer, which elsewhere paid
    // for its pairs with register moves); per element the same operations in the same order
    float alpha = 1.f, beta[B];
    v2f vb[B / 2] = {v2f{0.f, 0.f}, v2f{0.f, 0.f}};
#pragma unroll
    for (int e = 0; e < B; ++e)
#pragma unroll
      for (int c2 = 0; c2 < B / 2; ++c2)
        vb[c2] = __builtin_elementwise_fma(v2f{Hr[e], Hr[e]}, v2f{D[e][2 * c2], D[e][2 * c2 + 1]}, vb[c2]);
#pragma unroll
    for (int c = 0; c < B; ++c) {
      const float v = c & 1 ? vb[c / 2].y : vb[c / 2].x;
      float pv = -D[0][c];
#pragma unroll
      for (int e = 1; e < B; ++e) pv = t == e ? -D[e][c] : pv;
      beta[c] = piv ? pv : v;
    }
    if (piv) alpha = 0.f;
    float Dn[B][B];
#pragma unroll
    for (int jb = 0; jb < NQ; ++jb) {
      const int j = B + 4 * jb;
      v2f lo, hi;
      if ((SKIP >> (r * NQ + jb)) & 1ull) {
        // the pivot rows are +0 in this quad: alpha a - sum (+-0) = a, for the pivot lanes too (their
        // own entries here are those +0)
        lo = v2f{Hr[j], Hr[j + 1]};
        hi = v2f{Hr[j + 2], Hr[j + 3]};
      } else {
        lo = v2f{alpha, alpha} * v2f{Hr[j], Hr[j + 1]};
        hi = v2f{alpha, alpha} * v2f{Hr[j + 2], Hr[j + 3]};
#pragma unroll
        for (int c = 0; c < B; ++c) {
          lo = __builtin_elementwise_fma(v2f{-beta[c], -beta[c]}, x[jb][c].xy, lo);
          hi = __builtin_elementwise_fma(v2f{-beta[c], -beta[c]}, x[jb][c].zw, hi);
        }
      }
      Hr[j - B] = lo.x; Hr[j + 1 - B] = lo.y; Hr[j + 2 - B] = hi.x; Hr[j + 3 - B] = hi.y;
      if (jb == 0 && r + 1 < NB) {
        // the next round's pivot block (padded rows p - B ..): published, read back and inverted under
        // the rest of the round
        own[0] = v4f{lo.x, lo.y, hi.x, hi.y};
        __builtin_amdgcn_wave_barrier();  // one wave: the store above reaches LDS before these reads
#pragma unroll
        for (int a = 0; a < B; ++a) {
          const v4f d = *reinterpret_cast<const v4f*>(Rw[p - B + a]);
          Dn[a][0] = d.x; Dn[a][1] = d.y; Dn[a][2] = d.z; Dn[a][3] = d.w;
        }
        block_inverse<B>(Dn);
      }
    }
#pragma unroll
    for (int c = 0; c < B; ++c) Hr[NP - B + c] = beta[c];
    if (r + 1 < NB) {
#pragma unroll
      for (int j = B; j < NP; j += 4)
        if (!((SKIP >> ((r + 1) * NQ + j / 4 - 1)) & 1ull)) own[j / 4] = v4f{Hr[j], Hr[j + 1], Hr[j + 2], Hr[j + 3]};
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int a = 0; a < B; ++a)
#pragma unroll
        for (int c = 0; c < B; ++c) D[a][c] = Dn[a][c];
    }
  }
  __syncthreads();
}

// ------------------------------------------------------------------------------------------------
// contacts: robot geoms vs axis-aligned stone boxes

__device__ void emit_contact(EnvS& s, int slot, int ncap, int link, int link2, int stone, int foot, const float* P,
                             const float* n, float sep, float r) {
  if (slot >= ncap) return;
  s.clink[slot] = link; s.clink2[slot] = link2; s.cstone[slot] = stone; s.cfoot[slot] = foot; s.csep[slot] = sep;
  for (int k = 0; k < 3; ++k) { s.cn[slot][k] = n[k]; s.cpt[slot][k] = P[k] - n[k] * r; }
}

// Per-lane constants read from the constants block once per launch and kept in registers across the
// substeps (lane-varying global loads every substep were an L2 round trip at the head of collide and
// of the H rows): the geom of lane g, and the H-row masks of dof lane j.
struct GeomC {
  int link, type, foot;
  float r, p0[3], p1[3];
  uint32_t anc;  // h_row: dofs on the path of dof j's link
};
__device__ __forceinline__ GeomC load_geom(const Consts& K, int lane) {
  const as_model_t& m = K.model;
  const int g = lane < m.num_geoms ? lane : 0;
  GeomC c;
  c.link = m.geom_link[g];
  c.type = m.geom_type[g];
  c.foot = m.geom_foot[g];
  c.r = m.geom_radius[g];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    c.p0[k] = m.geom_p0[g][k];
    c.p1[k] = m.geom_p1[g][k];
  }
  const int j = lane < K.nv ? lane : 0;
  c.anc = K.ancmask[j < 6 ? 0 : j - 5];
  // opaque: the values are not rematerialised from memory inside the substep loop
  asm volatile("" : "+v"(c.link), "+v"(c.type), "+v"(c.foot), "+v"(c.r), "+v"(c.anc));
  asm volatile("" : "+v"(c.p0[0]), "+v"(c.p0[1]), "+v"(c.p0[2]), "+v"(c.p1[0]), "+v"(c.p1[1]), "+v"(c.p1[2]));
  return c;
}

// as_capsule_contact (include/as_detmath.h) without branches: every lane forms the three quotients of
// the main path (s, then t, then the clamped-end s) and selects; the degenerate cases (a sphere: a or e
// <= eps) reuse the same quotients with their own numerators.  The values selected are the same
// operations on the same operands as the branchy form, so the same bits; a wave whose pairs take
// different branches runs three divisions instead of up to six.
__device__ __forceinline__ float capsule_contact_sel(const float* a1, const float* b1, float r1, const float* a2,
                                                     const float* b2, float r2, float* P, float* n) {
  float d1[3], d2[3], r[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    d1[k] = b1[k] - a1[k];
    d2[k] = b2[k] - a2[k];
    r[k] = a1[k] - a2[k];
  }
  const float a = as_dot3(d1, d1), e = as_dot3(d2, d2), f = as_dot3(d2, r);
  const float eps = 1e-12f;
  const bool pa = a <= eps, pe = e <= eps, gen = !pa && !pe;
  const float c = as_dot3(d1, r);
  const float b = as_dot3(d1, d2);
  const float den = fmaf(a, e, -(b * b));
  const float sm = den > 0.f ? as_clamp01(fmaf(b, f, -(c * e)) / den) : 0.f;
  const float tq = (pa ? f : fmaf(b, sm, f)) / e;
  const bool lo = gen && tq < 0.f, hi = gen && tq > 1.f;
  const float sq = as_clamp01((hi ? b - c : -c) / a);
  const float s = pa ? 0.f : (pe || lo || hi) ? sq : sm;
  const float t = pa ? (pe ? 0.f : as_clamp01(tq)) : pe ? 0.f : lo ? 0.f : hi ? 1.f : tq;
  float c1[3], c2[3], w[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    c1[k] = fmaf(s, d1[k], a1[k]);
    c2[k] = fmaf(t, d2[k], a2[k]);
    w[k] = c1[k] - c2[k];
  }
  const float dist = sqrtf(as_dot3(w, w));
  const bool nz = dist > 1e-9f;
  const float inv = 1.0f / dist;
  n[0] = nz ? w[0] * inv : 0.f;
  n[1] = nz ? w[1] * inv : 0.f;
  n[2] = nz ? w[2] * inv : 1.f;
  const float sep = dist - r1 - r2;
  const float off = fmaf(0.5f, sep, r2);
#pragma unroll
  for (int k = 0; k < 3; ++k) P[k] = fmaf(off, n[k], c2[k]);
  return sep;
}

// At most ncap contacts, in priority order (oracle/physics.c collide() emits the same list); every
// pair is still tested past the cap, and the contacts found beyond it are counted in s.ndrop:
//   1. the priority geoms (the feet: geoms [0, num_priority_geoms)) against the candidate stones,
//      stone-major, geom-minor;  2. every other geom against the candidate stones, likewise;
//   3. robot self-contacts, one per self-collision pair in table order.
__device__ __forceinline__ int collide(const Consts& K, EnvS& s, int lane, int ncap, const GeomC& gc, const float* h,
                                       float margin) {
  const as_model_t& m = K.model;
  const int nst = K.task.num_steps, ng = m.num_geoms, npri = m.num_priority_geoms, nsp = m.num_self_pairs;
  // self-collision pair words of this lane (pairs lane, lane + 32, ...), loaded first so that their
  // latency hides behind the stone contacts
  constexpr int kSelfW = AS_MAX_SELF_PAIRS / G;
  int spw[kSelfW];
#pragma unroll
  for (int i = 0; i < kSelfW; ++i) spw[i] = G * i + lane < nsp ? m.self_pair[G * i + lane] : 0;
  // geom segment in the O frame (lane = geom), formed once for all candidate stones
  const bool gv = lane < ng;
  const int link = gc.link, gtype = gc.type, foot = gc.foot;
  const float r = gc.r;
  float a[3], bb[3];
  {
    float t0[3], t1[3];
    matvec3(s.R[link], gc.p0, t0);
    matvec3(s.R[link], gc.p1, t1);
    for (int k = 0; k < 3; ++k) { a[k] = s.p[link][k] + t0[k]; bb[k] = s.p[link][k] + t1[k]; }
  }
  const float L = sqrtf((bb[0] - a[0]) * (bb[0] - a[0]) + (bb[1] - a[1]) * (bb[1] - a[1]) +
                        (bb[2] - a[2]) * (bb[2] - a[2]));
  const float mid[3] = {0.5f * (a[0] + bb[0]), 0.5f * (a[1] + bb[1]), 0.5f * (a[2] + bb[2])};
  // broadphase (lane = stone): stone boxes that come within the contact margin of the robot's
  // bounding box (union of the geoms' boxes).  Conservative: every pair the narrowphase would
  // turn into a contact survives, so the contact set and order match the oracle's.
  // the six extents reduced in three pairs, the maxima as minima of the negated values (exact)
  float blo[3], bhi[3], ext[6];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float e = gtype == 0 ? a[k] : fminf(a[k], bb[k]);
    const float f = gtype == 0 ? a[k] : fmaxf(a[k], bb[k]);
    ext[k] = gv ? e - r : 1e30f;
    ext[3 + k] = gv ? -(f + r) : 1e30f;
  }
  half_min_n(ext);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    blo[k] = ext[k] - margin;
    bhi[k] = -ext[3 + k] + margin;
  }
  bool isc = false;
  float cst[3] = {0.f, 0.f, 0.f};
  if (lane < nst) {
    isc = true;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      cst[k] = s.stones[3 * lane + k] - s.root_pos[k];
      isc = isc && (cst[k] - h[k] <= bhi[k]) && (cst[k] + h[k] >= blo[k]);
    }
  }
  uint64_t bal = __ballot(isc);
  const int half = (threadIdx.x >> 5) & 1;
  uint32_t mine = (uint32_t)(bal >> (32 * half));
  if (isc) {
    const int pos = __popc(mine & ((1u << lane) - 1u));
    s.cand[pos] = lane;
    // the candidate's relative center for pass A (one 16-B broadcast read per candidate there)
    *reinterpret_cast<v4f*>(s.x.col.cc[pos]) = v4f{cst[0], cst[1], cst[2], 0.f};
  }
  const int ncand = __popc(mine);
  // narrowphase in two passes.  (A) lane = geom, loop over the candidate stones (once for the
  // priority geoms, once for the rest): the cheap bounding test (spheres: the exact separation)
  // appends the surviving (stone, geom) pairs to a list in LDS, in emission order.  (B) lane = pair,
  // in chunks of kPairsPerChunk: the exact test (capsules: slope bisection for the segment's closest
  // point) and the contacts, emitted in list order by a prefix sum.  A chunk is flushed as soon as
  // either env of the wave has kPairsPerChunk pairs pending, by both envs together (the other one
  // flushes its partial list: chunk boundaries change neither the contacts nor their order, and one
  // flush for the wave replaces one per env under divergence), so the list never exceeds 32 + 22
  // entries; the search runs over every pair even past ncap contacts (the surplus is counted, not
  // emitted).
  {
    float* gs = s.x.col.g[lane];  // staging of this lane's geom for pass B and the self pairs
    if (gv) {
      gs[0] = a[0]; gs[1] = a[1]; gs[2] = a[2];
      gs[3] = bb[0]; gs[4] = bb[1]; gs[5] = bb[2];
      gs[6] = r;
      gs[7] = __int_as_float(gtype | ((foot + 1) << 4) | (link << 8));
      *reinterpret_cast<v4f*>(s.x.col.bs[lane]) = v4f{mid[0], mid[1], mid[2], 0.5f * L + r};
    }
  }
  int* pl = s.x.col.pl;
  int pend = 0, base = 0;
  auto flush = [&](int npairs) {  // pass B over pl[0, npairs) (npairs <= kPairsPerChunk), shift the rest
    int cnt = 0, plink = 0, pst = 0, pfoot = -1;
    float P0[3], N0[3], P1[3], N1[3], P2[3], N2[3], SEP0 = 0.f, SEP1 = 0.f, SEP2 = 0.f, pr = 0.f;
    const bool act = lane < npairs;
    const int e = act ? pl[lane] : 0;  // (an env with nothing pending flushes too: stone 0, geom 0)
    const int gi = e & 0xff;
    pst = e >> 8;
    const float* gq = s.x.col.g[gi];
    const float A[3] = {gq[0], gq[1], gq[2]}, Bb[3] = {gq[3], gq[4], gq[5]};
    pr = gq[6];
    const int meta = __float_as_int(gq[7]);
    const int pty = meta & 15;
    pfoot = ((meta >> 4) & 15) - 1;
    plink = meta >> 8;
    float c[3];
    for (int k = 0; k < 3; ++k) c[k] = s.stones[3 * pst + k] - s.root_pos[k];
    // capsule: minimum of the (convex) signed distance along the segment by bisection on the sign
    // of its slope.  Runs for every lane (the result is only used by capsule pairs); unrolled by 4
    // (by 2: +0.6 % step time, profiles/r06z7_ab_flush_unroll.log).
    float lo = 0.f, hi = 1.f;
#pragma unroll 4
    for (int it = 0; it < kBisectIters; ++it) {
      const float t = 0.5f * (lo + hi);
      const bool up = sd_box_slope(A, Bb, t, c, h) > 0.f;
      hi = up ? t : hi;
      lo = up ? lo : t;
    }
    if (act) {
      // the segment's first point: the sphere's test and the capsule's t = 0 end are the same value
      float n0[3];
      const float s0 = sd_box(A, c, h, n0) - pr;
      if (pty == 0) {
        if (s0 < margin) {
          for (int k = 0; k < 3; ++k) { P0[k] = A[k]; N0[k] = n0[k]; }
          SEP0 = s0;
          cnt = 1;
        }
      } else {
        float n1[3];
        float s1 = sd_box(Bb, c, h, n1) - pr;
        float ts = 0.5f * (lo + hi), Ps[3], ns[3];
        for (int k = 0; k < 3; ++k) Ps[k] = A[k] + ts * (Bb[k] - A[k]);
        float ss = sd_box(Ps, c, h, ns) - pr;
        bool e0 = s0 < margin, e1 = s1 < margin;
        bool es = ss < margin && ss < fminf(s0, s1) - 0.002f;
        // pack the emitted contacts in (t=0, t=1, t*) order into slots 0..2
        for (int k = 0; k < 3; ++k) { P0[k] = A[k]; N0[k] = n0[k]; }
        SEP0 = s0;
        if (e0) {
          for (int k = 0; k < 3; ++k) { P1[k] = Bb[k]; N1[k] = n1[k]; P2[k] = Ps[k]; N2[k] = ns[k]; }
          SEP1 = s1; SEP2 = ss;
          if (!e1) { for (int k = 0; k < 3; ++k) { P1[k] = Ps[k]; N1[k] = ns[k]; } SEP1 = ss; }
        } else {
          for (int k = 0; k < 3; ++k) { P0[k] = Bb[k]; N0[k] = n1[k]; P1[k] = Ps[k]; N1[k] = ns[k]; }
          SEP0 = s1; SEP1 = ss;
          if (!e1) { for (int k = 0; k < 3; ++k) { P0[k] = Ps[k]; N0[k] = ns[k]; } SEP0 = ss; }
        }
        cnt = (int)e0 + (int)e1 + (int)es;
      }
    }
    int total;
    const int slot = base + half_scan3(cnt, total);
    if (cnt > 0) emit_contact(s, slot, ncap, plink, -1, pst, pfoot, P0, N0, SEP0, pr);
    if (cnt > 1) emit_contact(s, slot + 1, ncap, plink, -1, pst, pfoot, P1, N1, SEP1, pr);
    if (cnt > 2) emit_contact(s, slot + 2, ncap, plink, -1, pst, pfoot, P2, N2, SEP2, pr);
    base += total;
    // shift the unprocessed tail (< 32 entries) to the front
    const int rest = pend - npairs;
    const int tail = lane < rest ? pl[npairs + lane] : 0;
    __syncthreads();
    if (lane < rest) pl[lane] = tail;
    pend = rest;
    __syncthreads();
  };
  __syncthreads();
  // pass A (lane = geom): one bounding test per (candidate stone, geom), kept as a per-stone mask of
  // the surviving geoms; the masks then become the pair list class by class (feet first),
  // stone-major, geom-minor
  uint32_t* cneed = s.x.col.need;
  const float pa[3] = {gtype == 0 ? a[0] : mid[0], gtype == 0 ? a[1] : mid[1], gtype == 0 ? a[2] : mid[2]};
  const float cap_lim = 0.5f * L + r + margin;
#pragma unroll 1
  for (int ci = 0; ci < ncand; ++ci) {
    const v4f cv = *reinterpret_cast<const v4f*>(s.x.col.cc[ci]);
    const float c[3] = {cv.x, cv.y, cv.z};
    float nr[3];
    // one distance per lane: the sphere's center, or the capsule's midpoint for its bounding test
    const float sd = sd_box(pa, c, h, nr);
    bool need = false;
    if (gv) need = gtype == 0 ? sd - r < margin : sd <= cap_lim;
    const uint32_t bl = (uint32_t)(__ballot(need) >> (32 * half));
    if (lane == 0) cneed[ci] = bl;
  }
  __syncthreads();
  const uint32_t primask = npri >= 32 ? ~0u : (1u << npri) - 1u;
  const int wcand = max(__builtin_amdgcn_readlane(ncand, 0), __builtin_amdgcn_readlane(ncand, 32));
#pragma unroll 1
  for (int cls = 0; cls < 2; ++cls) {
#pragma unroll 1
    for (int ci = 0; ci < wcand; ++ci) {
      const uint32_t bl = ci < ncand ? cneed[ci] & (cls == 0 ? primask : ~primask) : 0u;
      if ((bl >> lane) & 1u) pl[pend + __popc(bl & ((1u << lane) - 1u))] = (s.cand[ci] << 8) | lane;
      pend += __popc(bl);  // no barrier: the single wave's LDS operations complete in issue order
      // wave-uniform flush decision (see above); the candidate loop runs to the wave's larger count
      if (max(__builtin_amdgcn_readlane(pend, 0), __builtin_amdgcn_readlane(pend, 32)) >= kPairsPerChunk)
        flush(pend < kPairsPerChunk ? pend : kPairsPerChunk);
    }
  }
  if (pend > 0) flush(pend);
  // self-contacts.  (A) lane = pair: the bounding-sphere filter; the surviving pairs are appended to
  // the pending list in table order.  (B) lane = pending pair, in chunks of G: the capsule-capsule
  // closest points (capsule_contact_sel: as_detmath.h's as_capsule_contact, which the oracle runs, in
  // selects), emitted in list order.
  pend = 0;
  auto flush_self = [&](int npairs) {
    const bool act = lane < npairs;
    const int e = pl[act ? lane : 0];
    const int g1 = e & 0xff, g2 = e >> 8;
    int cnt = 0, l1 = 0, l2 = 0;
    float P[3], n[3], sep = 0.f;
    if (act) {
      const float* q1 = s.x.col.g[g1];
      const float* q2 = s.x.col.g[g2];
      sep = capsule_contact_sel(q1, q1 + 3, q1[6], q2, q2 + 3, q2[6], P, n);
      cnt = sep < margin;
      l1 = __float_as_int(q1[7]) >> 8;
      l2 = __float_as_int(q2[7]) >> 8;
    }
    int total;
    const int slot = base + half_scan3(cnt, total);
    if (cnt) emit_contact(s, slot, ncap, l1, l2, -1, -1, P, n, sep, 0.f);
    base += total;
    const int rest = pend - npairs;
    const int tail = lane < rest ? pl[npairs + lane] : 0;
    __syncthreads();
    if (lane < rest) pl[lane] = tail;
    pend = rest;
    __syncthreads();
  };
  // all filter tests first (their LDS reads overlap), then the list is appended to without a
  // barrier per word (LDS operations of the single wave complete in issue order)
  // Every lane reads both spheres of every word (a word past nsp reads geom 0's twice: spw = 0) and
  // the reads are passed through an empty asm, four words at a time: each batch waits once.  (With
  // `pv && test` the compiler put each word's reads behind a branch on pv and waited on them word by
  // word: one LDS latency per word.)
  // Batches past the table (the quadruped's 66 pairs fill one of the two) are skipped by a scalar
  // branch; their words stay empty.
  uint32_t hbl[kSelfW];
  static_assert(kSelfW % 4 == 0, "batches of four words");
#pragma unroll
  for (int i = 0; i < kSelfW; ++i) hbl[i] = 0u;
#pragma unroll
  for (int i0 = 0; i0 < kSelfW; i0 += 4) {
    if (G * i0 >= nsp) break;
    v4f s1[4], s2[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      s1[i] = *reinterpret_cast<const v4f*>(s.x.col.bs[spw[i0 + i] & 0xff]);
      s2[i] = *reinterpret_cast<const v4f*>(s.x.col.bs[spw[i0 + i] >> 8]);
    }
    asm volatile("" : "+v"(s1[0]), "+v"(s1[1]), "+v"(s1[2]), "+v"(s1[3]), "+v"(s2[0]), "+v"(s2[1]), "+v"(s2[2]),
                 "+v"(s2[3]));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool pv = G * (i0 + i) + lane < nsp;
      const float m1[3] = {s1[i].x, s1[i].y, s1[i].z}, m2[3] = {s2[i].x, s2[i].y, s2[i].z};
      const bool hit = as_sphere_bound(m1, s1[i].w, m2, s2[i].w, margin);
      hbl[i0 + i] = (uint32_t)(__ballot(pv & hit) >> (32 * half));
    }
  }
  // The survivors' list positions in table order (word-major, lane-minor) by prefix counts, and all
  // of them written at once when neither env has more than the list holds (64; a random-action run
  // has 7 on average, 31 at p99.9: DESIGN §4), then tested 32 at a time -- the same chunks and
  // contact order as appending word by word.  More survivors: word by word, flushing every 32.
  const uint32_t lt = (1u << lane) - 1u;
  int tot = 0, at[kSelfW];
#pragma unroll
  for (int i = 0; i < kSelfW; ++i) {
    at[i] = tot + __popc(hbl[i] & lt);
    tot += __popc(hbl[i]);
  }
  if (max(__builtin_amdgcn_readlane(tot, 0), __builtin_amdgcn_readlane(tot, 32)) <= 64) {
#pragma unroll
    for (int i = 0; i < kSelfW; ++i)
      if ((hbl[i] >> lane) & 1u) pl[at[i]] = spw[i];
    pend = tot;
    while (pend > 0) flush_self(pend < G ? pend : G);
  } else {
    // a rolled loop (one copy of flush_self: code size is instruction-cache footprint); word i of
    // the register arrays by a select chain
#pragma unroll 1
    for (int i = 0; i < kSelfW; ++i) {
      if (G * i >= nsp) break;
      uint32_t bl = hbl[0];
      int w = spw[0];
#pragma unroll
      for (int k = 1; k < kSelfW; ++k) {
        bl = i == k ? hbl[k] : bl;
        w = i == k ? spw[k] : w;
      }
      if ((bl >> lane) & 1u) pl[pend + __popc(bl & lt)] = w;
      pend += __popc(bl);
      if (pend >= G) flush_self(G);
    }
    if (pend > 0) flush_self(pend);
  }
  // the search runs to the end: contacts past the cap are found, not emitted, and counted
  if (lane == 0 && base > ncap) s.ndrop += base - ncap;
  __syncthreads();
  return base < ncap ? base : ncap;  // uniform over the env's half-wave
}

__device__ void tangents(const float* n, float* t1, float* t2) {
  float e[3] = {1.f, 0.f, 0.f};
  if (fabsf(n[0]) > 0.9f) { e[0] = 0.f; e[1] = 1.f; }
  cross3(n, e, t1);
  float inv = 1.0f / sqrtf(dot3(t1, t1));
  for (int k = 0; k < 3; ++k) t1[k] *= inv;
  cross3(n, t1, t2);
}

// Contact-sensor flag of lane c's contact (c < nce, a foot contact): |sum lambda_n n| / dt over the
// contacts c2 < nce with its (foot, stone) pair, in ascending order; NC = the wave's larger nce.  Each
// contact's products lambda_n n and its pair key come from one 16-B LDS row (EnvS::x.cf; the same
// products the per-term form rounded; keys past nce never match), so a term is one read.
template <int NC>
__device__ __forceinline__ void contact_flag(const EnvS& s, int lane, int nce, float dt, uint32_t (&b)[4]) {
  static_assert(NC <= MAXC, "contacts");
  const int cl = lane < MAXC ? lane : 0;
  const int f = s.cfoot[cl], st = s.cstone[cl];
  const int key = __float_as_int(s.x.cf[cl][3]);
  float fx = 0.f, fy = 0.f, fz = 0.f;
  // all rows read first and passed through an empty asm, so that one wait covers every read (left to
  // the scheduler, each read was issued only when the previous term's registers freed: one LDS latency
  // per term)
  v4f t[NC];
#pragma unroll
  for (int c2 = 0; c2 < NC; ++c2) t[c2] = *reinterpret_cast<const v4f*>(s.x.cf[c2]);
  static_assert(NC == 10, "operand list below");
  asm volatile("" : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]), "+v"(t[4]), "+v"(t[5]), "+v"(t[6]), "+v"(t[7]),
               "+v"(t[8]), "+v"(t[9]));
#pragma unroll
  for (int c2 = 0; c2 < NC; ++c2) {
    const v4f v = t[c2];
    const bool same = __float_as_int(v.w) == key;
    fx += same ? v.x : 0.f;
    fy += same ? v.y : 0.f;
    fz += same ? v.z : 0.f;
  }
  if (lane < nce && f >= 0 && sqrtf(fx * fx + fy * fy + fz * fz) / dt > 1e-4f) b[f & 3] = 1u << st;
}

// Dot product of two padded rows held as packed pairs: two interleaved partial sums (even / odd
// element, fmaf chains ascending; v_pk_fma_f32 is the two fmafs), added at the end.  oracle/physics.c
// dot_pairs is the same arithmetic.
template <int NPR>
__device__ __forceinline__ float dot_pairs(const v2f (&a)[NPR], const v2f (&b)[NPR]) {
  v2f p = v2f{0.f, 0.f};
#pragma unroll
  for (int i = 0; i < NPR; ++i) p = __builtin_elementwise_fma(a[i], b[i], p);
  return p.x + p.y;
}

// W = H^-1 J^T for both envs of the wave on the matrix cores: v_mfma_f32_32x32x1_2b_f32 holds one
// 32 x 32 block per env (block b = lanes 32b..32b+31), K = 1 per instruction, so step k takes lane r's
// J_rk as the A operand (the lane built row r: no data movement) and lane j's (H^-1)_jk as the B
// operand (lane j holds row j of H^-1 after the sweep), and after NV steps block b holds
//   W_r[j] = sum_k J_rk (H^-1)_jk,   an fmaf chain over k ascending (gfx950 f32 MFMA numerics:
// bit for bit D = fma(a_k, b_k, C) per step -- scripts/probes/mfma_2b_probe.hip checks the layout and
// the chain on hardware; oracle/physics.c forms the same chain).  The result's layout (register v of
// block b: row 8(v/4) + 4h + v%4 on lane half h, column j = lane % 32) is brought to "lane j holds W_rj
// for every row r of its own env" by one v_permlane32_swap per register pair (blocks 0 and 1 trade
// their upper / lower halves).  The projections then need W by rows: lane j stores its column into
// the J image (after lane j has read its J column, the PGS's Jc), and
//   lane r forms A_rr = J_r . W_r and the in-triplet projections A_sr = J_s . W_r (r < s; lane s, from
//   the W rows of the two rows before it): each row's PGS coupling x_s A_sr is formed and stored by
//   that lane (no lane reads another lane's LDS result without a barrier in between).
// Cost per substep: NV MFMAs (64 cycles each on the SIMD's matrix pipe), independent of the row
// count; the LDS carries only the transposes.
template <int NV>
__device__ __forceinline__ void w_rows(EnvS& s, int lane, int nrow, const float* Hr, const v2f (&Jr)[LDJ / 2],
                                       float (&Jc)[MAXR], float (&Wc)[MAXR], uint32_t jmask) {
  static_assert(NV < LDJ, "padding column NV");
  static_assert(MAXR <= 32, "rows of one MFMA block");
  constexpr int NQ = (NV + 3) / 4;  // 16-B quads of a row that hold dofs
  float(*M)[LDJ] = s.x.k.Jm;
  const int jc = lane < NV ? lane : NV;  // column NV is +0 in the J image
#pragma unroll
  for (int r = 0; r < MAXR; ++r) Jc[r] = M[r][jc];
  // (an empty volatile asm orders memory operations: the J column reads issue here, and their latency
  // hides under the MFMA chain instead of heading the barrier below)
  float j0 = Jr[0].x;  // the MFMA chain's first operand, through the asm: the chain starts after it
  asm volatile("" : "+v"(j0));
  f32x32 acc = {};
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const float jk = k == 0 ? j0 : k & 1 ? Jr[k >> 1].y : Jr[k >> 1].x;
    // K step k only when some live row of either env can be nonzero at dof k (jmask, uniform): every
    // other step would add J_rk (H^-1)_jk = +0 x h to an accumulator that started at +0 and so is never
    // -0 -- the same bits (C3 +1.6 %, C2 +0.4 %: r06u)
    if ((jmask >> k) & 1u) acc = __builtin_amdgcn_mfma_f32_32x32x1f32(jk, Hr[k], acc, 0, 0, 0);
  }
  float wr[32];
  mfma_columns(acc, wr);
#pragma unroll
  for (int r = 0; r < MAXR; ++r) Wc[r] = wr[r];
  __syncthreads();  // every lane's J column reads are done
  if (lane < LDJ) {
#pragma unroll
    for (int r = 0; r < MAXR; ++r) M[r][lane] = wr[r];
  }
  __syncthreads();
  v2f jn[2 * NQ];
#pragma unroll
  for (int i = 0; i < 2 * NQ; ++i) jn[i] = Jr[i];
  const int r0 = lane < MAXR ? lane : 0;
  const int r1 = lane >= 1 ? min(lane - 1, MAXR - 1) : 0, r2 = lane >= 2 ? min(lane - 2, MAXR - 1) : 0;
  v2f w0[2 * NQ], w1[2 * NQ], w2[2 * NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const v4f c = *reinterpret_cast<const v4f*>(&M[r0][4 * q]);
    const v4f a = *reinterpret_cast<const v4f*>(&M[r1][4 * q]);
    const v4f b = *reinterpret_cast<const v4f*>(&M[r2][4 * q]);
    w0[2 * q] = c.xy; w0[2 * q + 1] = c.zw;
    w1[2 * q] = a.xy; w1[2 * q + 1] = a.zw;
    w2[2 * q] = b.xy; w2[2 * q + 1] = b.zw;
  }
  const float arr = dot_pairs(jn, w0);  // A_{lane, lane}
  const float a1 = dot_pairs(jn, w1);   // A_{lane, lane-1}
  const float a2 = dot_pairs(jn, w2);   // A_{lane, lane-2}
  if (lane < MAXR) {
    const float x = lane < nrow ? 1.0f / (arr + 1e-9f) : 0.f;
    s.rmeta[lane][0] = x;
    if (lane >= nrow) { s.rmeta[lane][1] = 0.f; s.rmeta[lane][2] = lane % 3 == 2 ? __builtin_inff() : 0.f; }
    // the PGS coupling factors x_s A_sr: row r0 holds x_1 A_10, row r0 + 1 x_2 A_20, row r0 + 2 x_2 A_21
    const int t = lane % 3;
    if (t == 1) s.rmeta[lane - 1][3] = x * a1;
    if (t == 2) {
      s.rmeta[lane - 1][3] = x * a2;
      s.rmeta[lane][3] = x * a1;
    }
  }
}

// PGS sweeps over NG row groups (see substep): rows in order, contacts as (normal, tangent, tangent)
// triplets, then joint limits; lane j holds u_j and every lane of an env all its impulses.  A group
// takes its three velocities J_r . u from the u at its start (three interleaved half-wave reductions)
// and adds the in-group couplings A_sr dlambda_r of the rows before it -- the Gauss-Seidel sweep row
// by row (J_s . (u + W_r dl_r) = J_s . u + A_sr dl_r) with one reduction latency per group.
template <int NG>
__device__ __forceinline__ void pgs_sweeps(const EnvS& s, int iters, float& uj, float (&lamr)[MAXR],
                                           const float (&Jc)[MAXR], const float (&Wc)[MAXR]) {
  typedef __attribute__((address_space(3))) const v4f* lds_v4p;
  lds_v4p meta = (lds_v4p)(&s.rmeta[0][0]);
  // Software-pipelined metadata: group g+1's three rows are read at the head of group g (between two
  // empty volatile asm statements, which order memory operations: the reads issue before group g's
  // reductions start) and consumed after group g+1's reductions, so the LDS latency is hidden by a
  // whole group.  Reading them at the head of their own group left each group waiting on the read
  // (its destination registers were reused as soon as the unused lane-0 bound field died).  The row
  // metadata is the same in every sweep, so the last group reads group 0 for the next sweep.
  v4f n0 = meta[0], n1 = meta[1], n2 = meta[2];
#pragma unroll 1
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int r = kRowGroup * g;
      // the group's rows pass through the asm: no use of them is hoisted into the previous group
      // (where it would wait on the read), and every field's register -- m0.z too, a bound that row 0
      // of a group never uses -- stays allocated to the read until the read has landed
      v4f m0 = n0, m1 = n1, m2 = n2;
      asm volatile("" : "+v"(meta), "+v"(uj), "+v"(m0), "+v"(m1), "+v"(m2));
      {
        const int rn = g + 1 < NG ? r + kRowGroup : 0;
        n0 = meta[rn];
        n1 = meta[rn + 1];
        n2 = meta[rn + 2];
      }
      asm volatile("" : "+v"(uj));
      float vg[3] = {Jc[r] * uj, Jc[r + 1] * uj, Jc[r + 2] * uj};
      half_sum_n(vg);
      // t_s = lambda_s + (target_s - v_s - sum_{r<s} A_sr dl_r) x_s, with the parts that do not
      // depend on this sweep's impulse changes formed first: the chain from one row's dl to the
      // next row's clamp is a single FMA
      const float k10 = m0.w, k20 = m1.w, k21 = m2.w;  // x_s A_sr, formed after the W pass
      float t1 = fmaf(-vg[1], m1.x, fmaf(m1.y, m1.x, lamr[r + 1]));
      float t2 = fmaf(-vg[2], m2.x, fmaf(m2.y, m2.x, lamr[r + 2]));
      // Row types by group: a contact triplet is (normal, tangent, tangent), every other group holds
      // limit rows (or the zero rows past nrow); contacts come first.  So row 0 always clamps to
      // [0, inf) and its impulse ln bounds only this triplet's tangents, and rows 1 and 2 share one
      // pair of bounds, +-mu ln for a contact triplet and [0, inf) otherwise -- the bounds a per-row
      // clamp forms, bit for bit (fmaf(-0, ln, 0) = +0 for the finite ln >= 0); the two bound
      // parameters were stored with the rows (EnvS::rmeta), so no type test runs in the sweep.
      const float mu_g = m1.z, off_g = m2.z;
      const float l0 = __builtin_amdgcn_fmed3f(fmaf(-vg[0], m0.x, fmaf(m0.y, m0.x, lamr[r])), 0.f, __builtin_inff());
      const float d0 = l0 - lamr[r];
      lamr[r] = l0;
      const float blo = fmaf(-mu_g, l0, 0.f), bhi = fmaf(mu_g, l0, off_g);
      t1 = fmaf(-k10, d0, t1);
      t2 = fmaf(-k20, d0, t2);
      uj = fmaf(Wc[r], d0, uj);
      const float l1 = __builtin_amdgcn_fmed3f(t1, blo, bhi);
      const float d1 = l1 - lamr[r + 1];
      lamr[r + 1] = l1;
      t2 = fmaf(-k21, d1, t2);
      uj = fmaf(Wc[r + 1], d1, uj);
      const float l2 = __builtin_amdgcn_fmed3f(t2, blo, bhi);
      const float d2 = l2 - lamr[r + 2];
      lamr[r + 2] = l2;
      uj = fmaf(Wc[r + 2], d2, uj);
    }
  }
}

template <int NV, uint64_t SKIP>
__device__ void substep(const Consts& K0, Smem& sm, EnvS& s, int lane0, const Topo& tp0, const GeomC& gc,
                        const LinkC& lc, uint32_t (&mask_out)[4], Stamp& ts) {
  // Opaque copies of the constants pointer and the lane id: everything derived from them below
  // (model-table loads, LDS addresses, lane masks) is loop-invariant, and without this the
  // compiler hoists all of it out of the substep loop and spills it.
  CK* kp = (CK*)(&K0);
  int lane = lane0;
  asm volatile("" : "+s"(kp), "+v"(lane));
  const Consts& K = *(const Consts*)(kp);
  const Topo& tp = tp0;  // LDS (Smem::topo)
  const as_model_t& m = K.model;
  const float dt = K.sim.dt;
  const int nh = m.num_hinges;
  // Scalars of the model loaded in groups just ahead of the phases that use them, each group passed
  // through an empty asm: one wait per group instead of a scalar load and a wait beside each use (a
  // wait on the scalar loads also waits on every LDS read in flight, so each one exposed an LDS
  // latency too).  Short live ranges: held across the whole substep they pushed the epilogue's SGPRs
  // into spills.
  int smp = K.max_path;
  asm volatile("" : "+s"(smp));
  if (K.act.mode == AS_ACT_DC_MOTOR && lane < nh) {  // the actuator runs in every substep (lane = hinge)
    const as_actuator_t& A = K.act;
    s.tau[lane] = as_dc_motor(s.qt[lane], s.qi[lane], s.u[6 + lane], A.stiffness, A.damping, A.saturation_effort,
                              A.effort_limit, A.velocity_limit);
  }
  fk<true>(K, s, lane, tp, lc, smp);  // (its first barrier publishes tau before the dynamics read it)
  ts.mark(kStFK);
  float Sj[6], Fj[6];  // dof lane j: S_j and Ic_link(j) S_j for the H rows
  dynamics<NV>(K, s, lane, tp, K.sim.gravity, Sj, Fj, smp);
  ts.mark(kStLinkQ);
  typedef SweepLayout<NV> SL;
  constexpr int NP = SL::NP;
  float Hr[NP];
  h_row<NV>(s, lane, tp, gc.anc, Sj, Fj, *reinterpret_cast<float(*)[NV]>(Hr));
  ts.mark(kStDyn);
  {
    // into the sweep's round-0 column order with the identity pad rows / columns (register renaming),
    // the sweep, and back: row `lane` of H^-1 in dof order
    float Hs[NP];
#pragma unroll
    for (int k = 0; k < NV; ++k) Hs[SL::pos(SL::padded(k))] = Hr[k];
#pragma unroll
    for (int q = 0; q < NP - NV; ++q) Hs[SL::pos(SL::PAD + q)] = lane == NV + q ? 1.f : 0.f;
    sweep_inverse<NV, SKIP>(s, lane, Hs);  // Hs <- this lane's row of -H^-1
#pragma unroll
    for (int k = 0; k < NV; ++k) Hr[k] = lane < NV ? -Hs[SL::pos(SL::padded(k))] : 0.f;
#pragma unroll
    for (int k = NV; k < NP; ++k) Hr[k] = 0.f;
  }
  ts.mark(kStChol);
  // u* = u + dt H^-1 b   (b broadcast from LDS)
  float uj = 0.f;
  {
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) acc = fmaf(Hr[k], s.b[k], acc);
    if (lane < NV) {
      uj = fmaf(dt, acc, s.u[lane]);
      s.u[lane] = uj;
    }
  }
  __syncthreads();
  ts.mark(kStSolve);
  // ---- constraints.  Joint-limit rows first counted (every one is kept), then the contacts fill the
  //      remaining rows, at most MAXC; rows are ordered contacts (normal, tangent, tangent), then the
  //      limits (lane h = hinge: lower then upper, in hinge order)
  int lo_v = 0, hi_v = 0;
  float err_lo = 0.f, err_hi = 0.f;
  if (lane < nh) {
    float qv = s.qi[lane], pred = qv + dt * s.u[6 + lane];
    err_lo = tp.lo - qv;
    err_hi = qv - tp.hi;
    lo_v = pred < tp.lo;
    hi_v = pred > tp.hi;
  }
  int ltotal;
  const int lpos = half_scan3(lo_v + hi_v, ltotal);
  const int nlim = ltotal < MAXR ? ltotal : MAXR;
  const int ncap = (MAXR - nlim) / 3 < MAXC ? (MAXR - nlim) / 3 : MAXC;
  float sb = K.sim.baumgarte, ssl = K.sim.slop, smd = K.sim.max_depen_vel, sfr = K.sim.friction, smg = K.sim.margin;
  float sh[3] = {K.sim.stone_half[0], K.sim.stone_half[1], K.sim.stone_half[2]};
  asm volatile("" : "+s"(sb), "+s"(ssl), "+s"(smd), "+s"(sfr), "+s"(smg), "+s"(sh[0]), "+s"(sh[1]), "+s"(sh[2]));
  const int nc = collide(K, s, lane, ncap, gc, sh, smg);
  ts.mark(kStCollide);

  if (lane < nc) {  // contact rows 3c..3c+2: normal, tangent 1, tangent 2
    float t1[3], t2[3];
    tangents(s.cn[lane], t1, t2);
    const float* dirs[3] = {s.cn[lane], t1, t2};
    float sp = s.csep[lane];
    const int lk = s.clink[lane] | ((s.clink2[lane] + 1) << 8);
    for (int d = 0; d < 3; ++d) {
      int r = 3 * lane + d;
      for (int k = 0; k < 3; ++k) s.cdir[lane][d][k] = dirs[d][k];
      s.rlink[r] = lk;
      s.rsign[r] = 0.f;
      // one division for both branches: (sp < 0 ? min(b max(-sp - slop, 0) / dt, vmax) : -sp / dt)
      const float num = sp < 0.f ? sb * fmaxf(-sp - ssl, 0.f) : -sp;
      const float tv = num / dt;
      s.rmeta[r][1] = d == 0 ? (sp < 0.f ? fminf(tv, smd) : tv) : 0.f;
      s.rmeta[r][2] = d == 1 ? sfr : 0.f;
    }
  }
  const int crow = 3 * nc;
  int slot = crow + lpos;
  for (int sd = 0; sd < 2; ++sd) {
    int viol = sd == 0 ? lo_v : hi_v;
    if (!viol) continue;
    if (slot < MAXR) {
      float err = sd == 0 ? err_lo : err_hi;
      s.rlink[slot] = -1 - (6 + lane);
      s.rsign[slot] = sd == 0 ? 1.f : -1.f;
      const float tv = (err > 0.f ? sb * err : err) / dt;  // one division, both branches
      s.rmeta[slot][1] = err > 0.f ? fminf(tv, smd) : tv;
      s.rmeta[slot][2] = slot % 3 == 2 ? __builtin_inff() : 0.f;
    }
    ++slot;
  }
  const int nrow = crow + nlim;  // uniform over the env's half-wave
  ts.count(nrow, nc);
  if (lane == 0) s.nrows += nrow;  // (the last substep's rows, or the peak, predict no better: r06j)
  const int maxrow = max(__builtin_amdgcn_readlane(nrow, 0), __builtin_amdgcn_readlane(nrow, 32));
  __syncthreads();  // the row metadata above, for the J build
  // Issue priority by constraint load: the two waves of a SIMD are arbitrated by priority, then
  // age, so a contact-heavy wave that happens to be the younger one would get only the leftover
  // issue slots and set the launch's tail.  The heavier wave of the pair takes precedence for the
  // rest of this substep and the fixed-cost phases of the next (scalar branch: s_setprio is not
  // masked by EXEC, so exactly one of them may execute).
  {
    const int lvl = __builtin_amdgcn_readfirstlane(maxrow) / kPrioRows;
    if (lvl >= 3) __builtin_amdgcn_s_setprio(3);
    else if (lvl == 2) __builtin_amdgcn_s_setprio(2);
    else if (lvl == 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
  }
  // ---- J rows, one lane per row (lane r < MAXR), kept in LDS [row][dof]: a contact row is
  //      J_rj = S_j . f6_r for the dofs whose link lies on the path root..link(r) (lpath of the
  //      row's link; dof j < 6 moves every link), minus the same on the second link's path for a
  //      self contact; a limit row is +-1 at its dof.  Every row < MAXR is written (zero past nrow),
  //      all rows at once: no per-row LDS round trip, no loop.  Lane r keeps its row in registers
  //      for W_r (w_rows).
  v2f Jr[LDJ / 2];
  uint32_t jmask = ~0u;
  {
    const int rr = lane < MAXR ? lane : 0;
    const int c = rr / 3, u = rr - 3 * c;
    const int lk = s.rlink[rr];
    const float sg = s.rsign[rr];
    float P[3], f6[6];  // spatial force direction [P x d; d]
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      P[k] = s.cpt[c][k];
      f6[3 + k] = s.cdir[c][u][k];
    }
    // lane j's motion-subspace row for the MFMA below, read with the row metadata; the empty volatile
    // asm orders memory operations, so these reads issue before the path-mask reads that depend on lk
    // (one LDS latency for both instead of one after the other)
    const int jo = lane < NV ? lane : 0;
    const v4f s0 = *reinterpret_cast<const v4f*>(&s.S[jo][0]);
    const v4f s1 = *reinterpret_cast<const v4f*>(&s.S[jo][4]);
    asm volatile("");
    cross3(P, f6 + 3, f6);
    const bool con = lk >= 0;
    const int l2 = (lk >> 8) - 1;
    // Every lane loads and computes everything; the selects are bit masks (exact: x & ~0 = x,
    // x & 0 = +0), so that no branch around the loads serialises one LDS round trip per column.
    const uint32_t pm1 = sm.topo[con ? lk & 31 : 0].lpath & (con ? ~0u : 0u);
    const uint32_t pm2 = sm.topo[con && l2 >= 0 ? l2 & 31 : 0].lpath & (con && l2 >= 0 ? ~0u : 0u);
    const uint32_t live = lane < nrow ? ~0u : 0u;
    // S_j . f6_r for every (dof j, row r) of both envs: six K steps of the two-block MFMA (A: lane j's
    // own motion subspace row, B: lane r's f6), an fmaf chain over the components (oracle chain6);
    // after the column shuffle lane r holds its row's products for every dof
    float Pj[32];
    {
      const float z = lane < NV ? 1.f : 0.f;
      const float Sa[6] = {s0.x * z, s0.y * z, s0.z * z, s0.w * z, s1.x * z, s1.y * z};
      f32x32 acc = {};
#pragma unroll
      for (int a = 0; a < 6; ++a) acc = __builtin_amdgcn_mfma_f32_32x32x1f32(Sa[a], f6[a], acc, 0, 0, 0);
      mfma_columns(acc, Pj);
    }
#pragma unroll
    for (int q = 0; q < LDJ / 4; ++q) {
      float jq[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int j = 4 * q + e;
        if (j < NV) {
          const uint32_t jb = __float_as_uint(Pj[j]);
          const int lnk = j < 6 ? 0 : j - 5;  // the link dof j moves with
          // contact row: (on path 1 ? jcon : 0) - (on path 2 ? jcon : 0), +0 on a limit row (pm = 0);
          // limit row: sign at its dof, +0 elsewhere and on every contact row (lk >= 0 > -1 - lk)
          const float jc1 = __uint_as_float(jb & (0u - ((pm1 >> lnk) & 1u)));
          const float jc2 = __uint_as_float(jb & (0u - ((pm2 >> lnk) & 1u)));
          const uint32_t jl = __float_as_uint(sg) & (-1 - lk == j ? ~0u : 0u);
          jq[e] = __uint_as_float(((__float_as_uint(jc1 - jc2)) | jl) & live);
        } else {
          jq[e] = 0.f;
        }
      }
      Jr[2 * q] = v2f{jq[0], jq[1]};
      Jr[2 * q + 1] = v2f{jq[2], jq[3]};
      if (lane < MAXR) *reinterpret_cast<v4f*>(&s.x.k.Jm[lane][4 * q]) = v4f{jq[0], jq[1], jq[2], jq[3]};
    }
    // the dofs any live row of either env can be nonzero at (structural: its links' root paths, or its
    // limit dof), OR-reduced over the wave: W's MFMA K steps outside it add +0 products only
    const uint32_t pm = pm1 | pm2;
    uint32_t dm = ((pm & 1u) ? 0x3Fu : 0u) | ((pm >> 1) << 6);
    if (!con && lane < MAXR) dm = 1u << ((-1 - lk) & 31);
    dm = lane < nrow ? dm : 0u;
    uint32_t dd = 0u;
    half_or2(dm, dd);
    jmask = (uint32_t)__builtin_amdgcn_readlane((int)dm, 0) | (uint32_t)__builtin_amdgcn_readlane((int)dm, 32);
  }
  __syncthreads();
  ts.mark(kStRows);
  // W = H^-1 J^T, A_rr and the in-triplet couplings (w_rows: one row per lane); lane j's W and J
  // columns go to registers for the PGS.  Hr is zero on lanes >= NV.
  float Wc[MAXR], Jc[MAXR];
  w_rows<NV>(s, lane, nrow, Hr, Jr, Jc, Wc, jmask);
  __syncthreads();
  ts.mark(kStWsolve);
  // ---- projected Gauss-Seidel (lane j holds u_j; every lane of an env holds all its impulses).
  // Rows in order: contacts as (normal, tangent, tangent) triplets, then joint limits; a tangent
  // row's bound uses the impulse of the most recent normal row (ln).  Lane j's J / W columns of
  // every row sit in registers (kept from the W pass).  A group of three rows takes the three
  // velocities J_r . u from the u at its start (three independent reductions) and adds the
  // in-group coupling A_sr dlambda_r of the rows before it, which is the Gauss-Seidel sweep row by
  // row (J_s . (u + W_r dl_r) = J_s . u + A_sr dl_r) with one reduction latency per group instead
  // of one per row.  The row loop is unrolled with an exit per group; rows in [maxrow, group end)
  // have zero J / W / metadata and leave everything unchanged.
  const int iters = K.sim.pgs_iters;
  float lamr[MAXR];
#pragma unroll
  for (int r = 0; r < MAXR; ++r) lamr[r] = 0.f;
  // one instantiation per group count (maxrow is wave-uniform): the groups run without a skip test,
  // so the sweep state needs no copies at per-group joins
  static_assert(MAXR / kRowGroup == 10, "group-count dispatch");
  switch ((__builtin_amdgcn_readfirstlane(maxrow) + kRowGroup - 1) / kRowGroup) {
    case 1: pgs_sweeps<1>(s, iters, uj, lamr, Jc, Wc); break;
    case 2: pgs_sweeps<2>(s, iters, uj, lamr, Jc, Wc); break;
    case 3: pgs_sweeps<3>(s, iters, uj, lamr, Jc, Wc); break;
    case 4: pgs_sweeps<4>(s, iters, uj, lamr, Jc, Wc); break;
    case 5: pgs_sweeps<5>(s, iters, uj, lamr, Jc, Wc); break;
    case 6: pgs_sweeps<6>(s, iters, uj, lamr, Jc, Wc); break;
    case 7: pgs_sweeps<7>(s, iters, uj, lamr, Jc, Wc); break;
    case 8: pgs_sweeps<8>(s, iters, uj, lamr, Jc, Wc); break;
    case 9: pgs_sweeps<9>(s, iters, uj, lamr, Jc, Wc); break;
    case 10: pgs_sweeps<10>(s, iters, uj, lamr, Jc, Wc); break;
    default: break;
  }
  // contact c's normal impulse (row 3c; every lane of an env holds all its impulses) times its normal,
  // and its (foot, stone) key, one 16-B row per contact for the flags; contacts past the solved
  // normal rows (nce) get a key no contact has
  const int nce = min(nc, (nrow + kRowGroup - 1) / kRowGroup);  // contacts whose normal row was solved
  if (lane < NV) s.u[lane] = uj;
  if (lane < MAXC) {
    float ln = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) ln = lane == c ? lamr[3 * c] : ln;
    ln = 3 * lane < nrow ? ln : 0.f;
    const int key = lane < nce ? ((s.cfoot[lane] + 1) << 8) | (s.cstone[lane] + 1) : -1;
    *reinterpret_cast<v4f*>(s.x.cf[lane]) =
        v4f{ln * s.cn[lane][0], ln * s.cn[lane][1], ln * s.cn[lane][2], __int_as_float(key)};
  }
  __syncthreads();
  ts.mark(kStPGS);
  // ---- contact-sensor flags of this substep (force_matrix_w = impulse / dt, > eps): lane c sums
  //      lambda_n n over the contacts with its (foot, stone) pair in ascending order, and the
  //      per-foot stone bits are OR-reduced over the half-wave
  {
    // All MAXC terms (one 16-B read each; the terms past an env's own count add +0 to a sum that is
    // never -0: the same bits) and no per-count dispatch: the flags, the hind-feet masks (zero for a
    // biped) and the root update below are one basic block, so the scheduler interleaves the root
    // update's serial chain with the flag sums.
    uint32_t b[4] = {0u, 0u, 0u, 0u};
    contact_flag<MAXC>(s, lane, nce, dt, b);
    half_or2(b[0], b[1]);
    half_or2(b[2], b[3]);
#pragma unroll
    for (int k = 0; k < 4; ++k) mask_out[k] = b[k];
  }
  // ---- integrate.  The root update is formed by every lane of the env (no lane-0 branch; the
  //      small-angle case by selects, the same values) and stored by lane 0
  float rq[4], rp[3];
  {
    const float* u = s.u;
    float c0w[3];
    for (int k = 0; k < 3; ++k) c0w[k] = fmaf(dt, u[k], s.root_pos[k] + s.c0[k]);
    const float* w = u + 3;
    const float wn = sqrtf(dot3(w, w));
    const float th = wn * dt;
    float sn, cs;
    as_sincosf(0.5f * th, &sn, &cs);
    const float sc = sn / wn;
    const bool big = th > 1e-12f;
    const float dq[4] = {big ? cs : 1.f, big ? w[0] * sc : 0.5f * dt * w[0], big ? w[1] * sc : 0.5f * dt * w[1],
                         big ? w[2] * sc : 0.5f * dt * w[2]};
    const float* q0 = s.root_quat;
    float nq[4] = {dq[0] * q0[0] - dq[1] * q0[1] - dq[2] * q0[2] - dq[3] * q0[3],
                   dq[0] * q0[1] + dq[1] * q0[0] + dq[2] * q0[3] - dq[3] * q0[2],
                   dq[0] * q0[2] - dq[1] * q0[3] + dq[2] * q0[0] + dq[3] * q0[1],
                   dq[0] * q0[3] + dq[1] * q0[2] - dq[2] * q0[1] + dq[3] * q0[0]};
    const float qn = 1.0f / sqrtf(nq[0] * nq[0] + nq[1] * nq[1] + nq[2] * nq[2] + nq[3] * nq[3]);
    for (int k = 0; k < 4; ++k) rq[k] = nq[k] * qn;
    float Rn[9], cl[3];
    quat_to_mat(rq, Rn);
    matvec3(Rn, m.com[0], cl);
    for (int k = 0; k < 3; ++k) rp[k] = c0w[k] - cl[k];
  }
  if (lane < nh) {
    float v = fminf(fmaxf(s.u[6 + lane], -K.sim.max_joint_vel), K.sim.max_joint_vel);
    s.u[6 + lane] = v;
    s.qi[lane] = fmaf(dt, v, s.qi[lane]);
  }
  if (lane == 0) {
    for (int k = 0; k < 4; ++k) s.root_quat[k] = rq[k];
    for (int k = 0; k < 3; ++k) s.root_pos[k] = rp[k];
  }
  __syncthreads();
  ts.mark(kStIntegrate);
}

// ------------------------------------------------------------------------------------------------
// task logic helpers (allsteps_env.py)

struct Useful {
  float h, roll, pitch, body_dist, dist_s;  // dist_s: swing-foot xy distance to the target
  int reached;
};

// allsteps_env.py:418-457 foot-state tick + 459-467 targets + 407-416 potentials (one env, serial).
// dist_s is the swing foot's distance with the swing leg AFTER the tick (allsteps_env.py:371).
__device__ void compute_useful(const Consts& K, const float* root_pos, const float* root_quat, const float* bp,
                               const float* stones_env, int stride, uint32_t mask_r, uint32_t mask_l, int& idx,
                               int& prev, int& next, int& count, int& swing, float& pot, float& old_pot,
                               float* foot_contact, bool tick, Useful& u) {
  const as_task_t& T = K.task;
  const int N = T.num_steps;
  float lower = fminf(bp[8], bp[5]);   // minimum(left_z, right_z)
  u.h = bp[2] - lower;
  euler_rp_from_quat(root_quat, &u.roll, &u.pitch);
  u.reached = 0;
  u.dist_s = 0.f;
  if (tick) {
    float cf0 = ((mask_r >> idx) & 1u) ? 1.f : 0.f;
    float cf1 = ((mask_l >> idx) & 1u) ? 1.f : 0.f;
    foot_contact[0] = cf0;
    foot_contact[1] = cf1;
    float tx = stones_env[(idx * 3 + 0) * stride], ty = stones_env[(idx * 3 + 1) * stride];
    float dx0 = bp[3] - tx, dy0 = bp[4] - ty, dx1 = bp[6] - tx, dy1 = bp[7] - ty;
    float d0 = sqrtf(dx0 * dx0 + dy0 * dy0), d1 = sqrtf(dx1 * dx1 + dy1 * dy1);
    float cfs = swing == 0 ? cf0 : cf1;
    float ds = swing == 0 ? d0 : d1;
    u.reached = (cfs > 0.f) && (ds < T.step_radius);
    if (u.reached) count += 1;
    if (count >= T.stop_frames) {
      swing ^= 1;
      int ni = min(max(idx + 1, 0), N - 1);
      idx = ni;
      prev = min(max(ni - 1, 0), N - 1);
      next = min(max(ni + 1, 0), N - 1);
      count = 0;
    }
    u.dist_s = swing == 0 ? d0 : d1;
  }
  float dx = stones_env[(next * 3 + 0) * stride] - root_pos[0];
  float dy = stones_env[(next * 3 + 1) * stride] - root_pos[1];
  u.body_dist = sqrtf(dx * dx + dy * dy);
  old_pot = pot;
  pot = -(u.body_dist) / T.step_dt;
}

// ------------------------------------------------------------------------------------------------
// XCD-aware env mapping.  Workgroup b is dispatched to XCD b % 8; a 128-B line of an SoA field
// holds 32 consecutive envs = 16 workgroups, which with the identity mapping would be split over all
// eight per-XCD L2s (each fetching and writing back the whole line for 16 useful bytes).  Give XCD x
// a contiguous range of env pairs instead (a bijection for any grid size; placement only affects
// speed, never results).
__device__ __forceinline__ int xcd_block(int b, int nb) {
  const int q = nb >> 3, r = nb & 7, x = b & 7, slot = b >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + slot;
}

// k_step's workgroup is exactly ONE wave: its __syncthreads are LDS fences only, and the FK pointer
// jumping relies on a single wave's LDS operations completing in issue order (no barrier between
// rounds).  Launch and launch bound both use this constant; widening it must add those barriers.
constexpr int kStepThreads = 64;
static_assert(kStepThreads == 64, "k_step assumes a one-wave (wave64) workgroup: see the FK rounds");

template <int NV, uint64_t SKIP>
__global__ __launch_bounds__(kStepThreads) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_step(StepArgs P) {
  __shared__ Smem sm;
  // model / plan constants stay in global memory (5.7 KB, L1/K$-resident): LDS is the occupancy
  // budget, see EnvS
  const Consts& K = *(const Consts*)(CK*)P.consts;
  const int el = threadIdx.x >> 5, lane = threadIdx.x & 31;
  const int n = P.n;
  const int e_raw = P.wave_map ? P.wave_map[EPB * blockIdx.x + el] : xcd_block(blockIdx.x, gridDim.x) * EPB + el;
  const bool valid = e_raw < n;
  const int e = valid ? e_raw : n - 1;
  EnvS& s = sm.env[el];
  const as_state_t& st = P.st;
  Stamp ts{P.stamps, sm.stamp_acc, 0ull};
  ts.start();
  // Under the wave map the second half of the grid holds the predicted-light waves, each the SIMD
  // partner of a heavy one.  The light wave starts with issue priority, until the first substep's row
  // count sets the rule below: with the heavy wave ahead from the first instruction the light partner
  // finished last (a wave's cycles grow more with its partner's rows than with its own, r06j), and
  // light-first for the opening phases only (not every substep's, nor the first two) measured best (r06k).
  if (P.wave_map && blockIdx.x >= (gridDim.x >> 1)) __builtin_amdgcn_s_setprio(1);
  __syncthreads();
  const as_model_t& m = K.model;
  const int nh = m.num_hinges;
  const as_task_t& T = K.task;
  if (el == 0) sm.topo[lane] = load_topo(K, lane);
  const Topo& tp = sm.topo[lane];
  // ---- load
  if (lane < 3) {
    s.root_pos[lane] = st.root_pos[lane * n + e];
    s.u[lane] = st.root_lin[lane * n + e];
    s.u[3 + lane] = st.root_ang[lane * n + e];
  }
  if (lane < 4) s.root_quat[lane] = st.root_quat[lane * n + e];
  if (lane == 0) { s.ndrop = 0; s.nrows = 0; }
  const int cur = st.curriculum[0];
  const float gain = T.gain_curriculum[cur];
  if (lane < nh) {
    int i = m.cfg_dof_link[lane] - 1;
    s.qi[i] = st.q[lane * n + e];
    s.u[6 + i] = st.qd[lane * n + e];
    float a = 0.f;
    if (P.mode != kModeReset) a = P.actions[(size_t)e * nh + lane];
    a = fminf(fmaxf(a, -1.f), 1.f);                      // allsteps_env.py:267-268
    s.act[lane] = a;
    s.tau[i] = gain * m.gear[lane] * a;                  // allsteps_env.py:273
    s.qt[i] = K.act.action_scale * a + K.act.default_q[lane];  // AS_ACT_DC_MOTOR (anymal_c_env.py:73-74)
  }
  for (int k = lane; k < 3 * T.num_steps; k += G) s.stones[k] = st.stones[k * n + e];
  uint32_t mask[4] = {st.contact_mask[e], st.contact_mask[n + e], 0u, 0u};
  __syncthreads();
  ts.mark(kStLoad);
  const bool do_physics = P.mode == kModeStep || P.mode == kModePhysics;
  const LinkC lc = load_link(K, lane);
  // ---- physics
  if (do_physics) {
    const GeomC gc = load_geom(K, lane);
    for (int sub = 0; sub < K.sim.substeps; ++sub) substep<NV, SKIP>(K, sm, s, lane, tp, gc, lc, mask, ts);
  }
  // This lane's reset constants (joint `lane` in cfg order: its link and limits, the start pose plain and
  // mirrored), loaded ahead of the final FK so that their global loads (L2 round trips) run under it
  // instead of heading the reset (the memory clobber keeps them there, not sunk into the reset
  // branch); the limits then come from the tree plan in LDS.  The task's reward and the observation
  // use the same link and limits.
  int rs_li = 1, rs_src = lane;
  float rs_q = 0.f, rs_qm = 0.f, rs_sg = 1.f, rs_lo = 0.f, rs_hi = 0.f;
  {
    // the mirror map through the constant address space (uniform: scalar loads, all issued together),
    // applied by selects in the reference's order (the later match wins, as the sequential ifs)
    const __attribute__((address_space(4))) as_task_t* Tc = &((CK*)P.consts)->task;
    int rmap[9], lmap[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) { rmap[t] = Tc->right_idx[t]; lmap[t] = Tc->left_idx[t]; }
    const int ng0 = Tc->neg_idx[0], ng1 = Tc->neg_idx[1];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      rs_src = rmap[t] == lane ? lmap[t] : rs_src;
      rs_src = lmap[t] == lane ? rmap[t] : rs_src;
    }
    rs_sg = ng0 == lane || ng1 == lane ? -1.f : 1.f;
    if (lane < nh) {
      rs_q = T.init_q[lane] * 1.f;
      rs_qm = T.init_q[rs_src] * rs_sg;
      rs_li = m.cfg_dof_link[lane];
    }
  }
  asm volatile("" ::: "memory");
  if (do_physics) {
    fk<false>(K, s, lane, tp, lc, K.max_path);  // FK of the final pose for body_pos_w (articulation_data.py:439)
    if (lane == 0) { s.mask[0] = mask[0]; s.mask[1] = mask[1]; s.mask[2] = mask[2]; s.mask[3] = mask[3]; }
  }
  ts.mark(kStFKFinal);
  if (lane < nh) {  // m.lower / upper[li] as copied into the tree plan (Topo: hinge li - 1 is link li)
    rs_lo = sm.topo[rs_li - 1].lo;
    rs_hi = sm.topo[rs_li - 1].hi;
  }
  if (lane == 0 && !do_physics) { s.mask[0] = mask[0]; s.mask[1] = mask[1]; }
  __syncthreads();
  float bp[9];
  if (do_physics) {
    const int ls[3] = {m.torso_link, m.foot_link[0], m.foot_link[1]};
    for (int b = 0; b < 3; ++b)
      for (int k = 0; k < 3; ++k) bp[3 * b + k] = s.root_pos[k] + s.p[ls[b]][k];
  } else {
    for (int k = 0; k < 9; ++k) bp[k] = st.body_pos[k * n + e];
  }
  // ---- task epilogue (direct_rl_env.py:349-364)
  int idx = st.idx[e], prev = st.prev[e], next = st.next[e], count = st.count[e], swing = st.swing[e];
  int ep_len = st.ep_len[e];
  float pot = st.pot[e], old_pot = st.old_pot[e];
  float fc[2] = {st.foot_contact[e], st.foot_contact[n + e]};
  uint32_t episode = st.episode[e];
  bool done = false;
  if (P.mode == kModeStep || P.mode == kModeTask) {
    ep_len += 1;                                         // direct_rl_env.py:351
    Useful u;
    compute_useful(K, s.root_pos, s.root_quat, bp, s.stones, 1, s.mask[0], s.mask[1], idx, prev, next, count,
                   swing, pot, old_pot, fc, true, u);    // allsteps_env.py:397 tick #1
    // lane-parallel pieces of the reward: sum a^2, sum |qd a|, #(|q_scaled| > 0.99)
    float a2 = 0.f, en = 0.f;
    int atlim = 0;
    if (lane < nh) {
      const int li = rs_li;
      float a = s.act[lane];
      a2 = a * a;
      en = fabsf(s.u[6 + li - 1] * a);
      atlim = fabsf(scale_transform(s.qi[li - 1], rs_lo, rs_hi)) > 0.99f;
    }
    a2 = half_sum(a2);
    en = half_sum(en);
    uint64_t bl = __ballot(atlim != 0);
    int nlim = __popcll(bl >> (32 * el) & 0xffffffffull);
    const float* lv = s.u;
    float speed = sqrtf(lv[0] * lv[0] + lv[1] * lv[1] + lv[2] * lv[2]);
    bool time_out = ep_len >= T.max_episode_length - 1;  // allsteps_env.py:399
    bool fell = u.h < T.term_curriculum[cur];            // :401
    bool so_fast = speed > 5.0f;                         // :402
    bool died = s.root_pos[2] < T.fall_abs;              // :403
    bool terminated = fell || so_fast || died;
    // allsteps_env.py:347-394
    float progress = pot - old_pot;
    bool roll_v = (u.roll > 0.4f) || (u.roll < -0.4f);
    bool pitch_v = (u.pitch > 0.4f) || (u.pitch < -0.2f);
    float roll_cost = roll_v ? fabsf(u.roll) : 0.f;
    float pitch_cost = pitch_v ? fabsf(u.pitch) : 0.f;
    float speed_cost = speed > 1.6f ? speed - 1.6f : 0.f;
    float action_cost = T.action * sqrtf(a2);
    float energy_cost = T.energy * en;
    float limit_cost = (float)nlim * T.joint_limit;
    bool cond = u.reached && count == 1 && idx < T.num_steps - 1;
    float step_rew = cond ? 50.0f * as_expf(-u.dist_s / 0.25f) : 0.f;  // shared deterministic exp
    bool bonus_c = idx == T.num_steps - 1 && u.body_dist < 0.15f;
    float total = T.alive + progress;
    total = total - roll_cost;
    total = total - pitch_cost;
    total = total - speed_cost;
    total = total - energy_cost;
    total = total - action_cost;
    total = total - limit_cost;
    total = total + step_rew;
    total = total + (bonus_c ? 10.0f : 0.f);
    float rew = terminated ? T.death : total;
    done = terminated || time_out;
    if (valid && lane == 0) {
      P.reward[e] = rew;
      P.terminated[e] = terminated ? 1 : 0;
      P.truncated[e] = time_out ? 1 : 0;
    }
  } else if (P.mode == kModeReset) {
    done = P.reset_mask == nullptr || P.reset_mask[e] != 0;
  }
  if (P.mode != kModePhysics) {
    // curriculum mean over the tick-#1 indices and the any-reset flag: one atomic per wave into a
    // striped partial sum, the flag by plain store
    const int cidx = valid ? idx : 0;
    const bool vdone = valid && done;
    const int wsum = __builtin_amdgcn_readlane(cidx, 0) + __builtin_amdgcn_readlane(cidx, 32);
    const bool wdone = __any(vdone);
    // contacts the row budget cut in this launch (rare: one same-address atomic per wave that had any)
    const int ndr = valid ? s.ndrop : 0;
    const int wdrop = __builtin_amdgcn_readlane(ndr, 0) + __builtin_amdgcn_readlane(ndr, 32);
    if (threadIdx.x == 0) {
      atomicAdd(&P.counters[kCntStride * (1 + (int)(blockIdx.x % kCntSlots))], wsum);
      if (wdrop) atomicAdd(&P.counters[kCntDropped], wdrop);
      if (wdone) P.counters[0] = 1;
      if (T.regen_footsteps) P.counters[kCntLevel] = P.st.curriculum[0];  // same value from every wave
    }
  }
  ts.mark(kStTask);
  // ---- in-kernel reset (allsteps_env.py:481-565)
  const bool any_done = __any(done);  // wave-uniform: both envs of the wave enter the FK together
  // regen_footsteps: the over-half test on the PRE-reset target index (allsteps_env.py:497-500 as
  // intended); k_obs draws the new course once the launch-wide curriculum gate is known
  const bool regen = T.regen_footsteps && P.mode != kModePhysics && done && idx > T.num_steps / 2;
  if (P.mode != kModePhysics && any_done) {
    if (done) {
      float dm = 0.f, dn = 0.f;  // mirror draw, this lane's joint-noise draw
      if (P.reset_draws) {
        dm = P.reset_draws[(size_t)e * 22];
        if (lane < nh) dn = P.reset_draws[(size_t)e * 22 + 1 + lane];
      } else {
        float blk[4];
        philox_block(P.seed, (uint32_t)(P.env_offset + e), episode, 0u, kResetTag, blk);
        dm = blk[0];
        if (lane < nh) {  // draw k = 1 + lane lives in block (1 + lane) / 4, slot (1 + lane) % 4
          const int k = 1 + lane;
          philox_block(P.seed, (uint32_t)(P.env_offset + e), episode, (uint32_t)(k >> 2), kResetTag, blk);
          const int sl = k & 3;
          dn = sl == 0 ? blk[0] : (sl == 1 ? blk[1] : (sl == 2 ? blk[2] : blk[3]));
        }
      }
      ep_len = 0;
      old_pot = 0.f; pot = 0.f; count = 0; swing = 0; idx = 1; prev = 0; next = 2;
      const bool mirror = dm > 0.5f;
      if (mirror) swing ^= 1;
      if (lane < nh) {
        // joint `lane` (cfg order): running-start pose, mirrored, noise, clip (allsteps_env.py:505-560)
        // (the mirror map, start pose and limits were loaded ahead: rs_*)
        const float sign = mirror ? rs_sg : 1.f;
        float jp = mirror ? rs_qm : rs_q;
        float jv = 0.f * sign;
        int li = rs_li;
        float x = jp + (dn * (T.noise_hi - T.noise_lo) + T.noise_lo);
        float sc = fminf(fmaxf(scale_transform(x, rs_lo, rs_hi), T.clip_lo), T.clip_hi);
        s.qi[li - 1] = unscale_transform(sc, rs_lo, rs_hi);
        s.u[6 + li - 1] = jv;
      }
      if (lane < 3) {
        s.root_pos[lane] = T.init_root[lane];
        s.u[lane] = 0.f;
        s.u[3 + lane] = 0.f;
      }
      if (lane == 0) {
        float sg = mirror ? -1.f : 1.f;
        s.root_quat[0] = 1.f;
        s.root_quat[1] = 0.f * sg;
        s.root_quat[2] = 0.f * sg;
        s.root_quat[3] = 0.f * sg;
      }
      episode += 1u;
    }
    __syncthreads();
    fk<false>(K, s, lane, tp, lc, K.max_path);  // body_pos of the reset pose (write_joint_state_to_sim invalidates FK)
    if (done) {
      const int ls[3] = {m.torso_link, m.foot_link[0], m.foot_link[1]};
      for (int b = 0; b < 3; ++b)
        for (int k = 0; k < 3; ++k) bp[3 * b + k] = s.root_pos[k] + s.p[ls[b]][k];
    }
  }
  __syncthreads();
  // ---- observation with a speculative second tick (allsteps_env.py:326-345, 567).  The reference
  //      re-runs _compute_useful_values for ALL envs when ANY env reset this step -- a launch-wide
  //      condition.  The tick is applied here as if some env reset (true at any realistic env
  //      count); the tick-#1 state and the tick-dependent observation entries (foot contact,
  //      targets) go to a side buffer, and k_obs restores them in a launch where no env reset.
  if (P.obs) {
    int i2 = idx, p2 = prev, n2 = next, c2 = count, w2 = swing;
    float pot2 = pot, op2 = old_pot, fc2[2] = {fc[0], fc[1]};
    Useful u2;
    compute_useful(K, s.root_pos, s.root_quat, bp, s.stones, 1, s.mask[0], s.mask[1], i2, p2, n2, c2, w2, pot2,
                   op2, fc2, true, u2);
    float* ob = s.x.obs;
    uint32_t* side = P.side;
    if (lane == 0) {
      ob[0] = u2.h;
      ob[1] = u2.roll;
      ob[2] = u2.pitch;
      float vb[3];
      quat_rotate_inverse(s.root_quat, s.u, vb);
      ob[3] = vb[0]; ob[4] = vb[1]; ob[5] = vb[2];
      ob[48] = fc2[0];
      ob[49] = fc2[1];
    }
    if (lane < nh) {
      const int li = rs_li;
      ob[6 + lane] = scale_transform(s.qi[li - 1], rs_lo, rs_hi);
      ob[27 + lane] = fminf(fmaxf(s.u[6 + li - 1] * T.dof_vel_scale, -5.f), 5.f);
    }
    if (lane < 6) {  // lanes 0-2: targets after the second tick, lanes 3-5: after the first
      const int t = lane < 3 ? lane : lane - 3;
      const int ti = lane < 3 ? (t == 0 ? p2 : (t == 1 ? i2 : n2)) : (t == 0 ? prev : (t == 1 ? idx : next));
      const float tw[3] = {s.stones[3 * ti], s.stones[3 * ti + 1], s.stones[3 * ti + 2]};
      float o3[3];
      subtract_frame_transforms(s.root_pos, s.root_quat, tw, o3);
      if (lane < 3) {
        for (int k = 0; k < 3; ++k) ob[50 + 3 * t + k] = o3[k];
      } else if (valid) {
        for (int k = 0; k < 3; ++k) side[(kSideState + 2 + 3 * t + k) * n + e] = __float_as_uint(o3[k]);
      }
    }
    __syncthreads();
    if (valid) {
      float* orow = P.obs + (size_t)e * AS_OBS_DIM;
      orow[lane] = ob[lane];
      if (lane < AS_OBS_DIM - 32) orow[32 + lane] = ob[32 + lane];
      if (lane == 0) {
        const uint32_t sv[kSideState + 2] = {(uint32_t)idx, (uint32_t)prev, (uint32_t)next, (uint32_t)count,
                                             (uint32_t)swing, __float_as_uint(pot), __float_as_uint(old_pot),
                                             __float_as_uint(fc[0]), __float_as_uint(fc[1]),
                                             __float_as_uint(fc[0]), __float_as_uint(fc[1])};
        for (int k = 0; k < kSideState + 2; ++k) side[k * n + e] = sv[k];
        side[kSideRegen * n + e] = regen ? 1u : 0u;
      }
    }
    idx = i2; prev = p2; next = n2; count = c2; swing = w2;
    pot = pot2; old_pot = op2; fc[0] = fc2[0]; fc[1] = fc2[1];
  }
  ts.mark(kStReset);
  // ---- store
  if (valid) {
    if (lane < 3) {
      st.root_pos[lane * n + e] = s.root_pos[lane];
      st.root_lin[lane * n + e] = s.u[lane];
      st.root_ang[lane * n + e] = s.u[3 + lane];
    }
    if (lane < 4) st.root_quat[lane * n + e] = s.root_quat[lane];
    if (lane < nh) {
      int i = rs_li - 1;
      st.q[lane * n + e] = s.qi[i];
      st.qd[lane * n + e] = s.u[6 + i];
    }
    if (lane < 9) {
      float v = bp[0];
#pragma unroll
      for (int k = 1; k < 9; ++k) v = (lane == k) ? bp[k] : v;
      st.body_pos[lane * n + e] = v;
    }
    if (lane == 0) {
      // an env reset in this launch starts the next one from the spawn pose in the air: no rows
      // (its fallen-state rows predicted a heavy wave that was not; C3 +1 %, r06q)
      P.side[kSideCost * n + e] = done ? 0u : (uint32_t)s.nrows;
      st.contact_mask[e] = s.mask[0];
      st.contact_mask[n + e] = s.mask[1];
      if (st.contact_mask_hind) {
        st.contact_mask_hind[e] = s.mask[2];
        st.contact_mask_hind[n + e] = s.mask[3];
      }
      if (P.mode != kModePhysics) {
        st.idx[e] = idx; st.prev[e] = prev; st.next[e] = next; st.count[e] = count; st.swing[e] = swing;
        st.ep_len[e] = ep_len; st.pot[e] = pot; st.old_pot[e] = old_pot;
        st.foot_contact[e] = fc[0]; st.foot_contact[n + e] = fc[1];
        st.episode[e] = episode;
      }
    }
  }
  ts.mark(kStStore);
  ts.flush();
}

// ------------------------------------------------------------------------------------------------
// K2: the launch-wide part of the observation step.  If any env reset this step (device counter
// written by k_step): the curriculum gate (allsteps_env.py:471-479, evaluated on the tick-#1 target
// indices) -- k_step has already applied the second tick.  If none did: restore the tick-#1 state
// and observation entries k_step saved in the side buffer.
__device__ void gen_stones(const as_task_t& T, int level, uint64_t seed, uint32_t env, uint32_t episode,
                           const float* draws, float* stones, int n, int e);

// The next k_step's placement (kMapEnvs), by one wave (t = lane): env chunk w's 64 envs ranked by their
// constraint rows in this launch (a bitonic sort of (rows, lane) keys across the wave, unique keys:
// deterministic), rank q -> pair q / 2, half q % 2 (rows is at most substeps x 30: 16 bits hold it).
__device__ __forceinline__ void build_wave_map(const uint32_t* side, int32_t* wave_map, int n, bool streamed, int w,
                                               int t) {
  static_assert(kMapEnvs == 64, "one wave per env chunk");
  const uint32_t rows = min(side[kSideCost * n + w * kMapEnvs + t], 0xFFFFu);
  uint32_t key = rows << 6 | (uint32_t)(63 - t);  // descending rows, ascending env on ties
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1)
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const uint32_t o = (uint32_t)__shfl_xor((int)key, j);
      const bool desc = (t & k) == 0, first = (t & j) == 0;  // descending overall
      key = first == desc ? max(key, o) : min(key, o);
    }
  wave_map[EPB * wave_map_block(w, t >> 1, n, streamed) + (t & 1)] = w * kMapEnvs + 63 - (int)(key & 63u);
}

__global__ __launch_bounds__(64) void k_obs(ObsArgs P) {
  const Consts& K = *(const Consts*)(CK*)P.consts;
  const as_task_t& T = K.task;
  const int n = P.n;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int any_reset = P.counters[0];
  if (P.wave_map) build_wave_map(P.side, P.wave_map, n, P.map_streamed != 0, blockIdx.x, threadIdx.x);
  if (blockIdx.x == 0) {
    // the gate's inputs in one memory round trip: lane i < kCntSlots reads partial sum i, lane
    // kCntSlots the curriculum level (all issued before any store: the stores below may alias them)
    const int t = threadIdx.x;
    int v = 0;
    if (t < kCntSlots) v = P.counters[kCntStride * (1 + t)];
    else if (t == kCntSlots) v = P.st.curriculum[0];
    const int c = __shfl(v, kCntSlots);
    int part = t < kCntSlots ? v : 0;
#pragma unroll
    for (int off = kCntSlots / 2; off > 0; off >>= 1) part += __shfl_xor(part, off);
    const int sum = __builtin_amdgcn_readfirstlane(part);  // lanes 0..15 hold the total (exact integers)
    if (t == 0) {
      P.counters[1] = sum;
      // (regen below recomputes this gate per thread from the bank, race-free)
      if (any_reset && (float)sum / (float)n > (float)T.curriculum_threshold)
        P.st.curriculum[0] = min(c + 1, T.max_curriculum);
    }
  }
  // the next launch's bank (this launch reads the other one)
  for (int k = e; k < kCntBank; k += gridDim.x * blockDim.x) P.next_counters[k] = 0;
  if (any_reset && T.regen_footsteps && e < n && P.side[kSideRegen * n + e]) {
    int sum = 0;
    for (int i = 0; i < kCntSlots; ++i) sum += P.counters[kCntStride * (1 + i)];
    const int c0 = P.counters[kCntLevel];
    const int level = (float)sum / (float)n > (float)T.curriculum_threshold ? min(c0 + 1, T.max_curriculum) : c0;
    gen_stones(T, level, P.seed, (uint32_t)(P.env_offset + e), P.st.episode[e], nullptr, P.st.stones, n, e);
  }
  if (any_reset) return;
  if (e >= n) return;
  const as_state_t& st = P.st;
  const uint32_t* sd = P.side;
  st.idx[e] = (int)sd[e];
  st.prev[e] = (int)sd[n + e];
  st.next[e] = (int)sd[2 * n + e];
  st.count[e] = (int)sd[3 * n + e];
  st.swing[e] = (int)sd[4 * n + e];
  st.pot[e] = __uint_as_float(sd[5 * n + e]);
  st.old_pot[e] = __uint_as_float(sd[6 * n + e]);
  st.foot_contact[e] = __uint_as_float(sd[7 * n + e]);
  st.foot_contact[n + e] = __uint_as_float(sd[8 * n + e]);
  float* o = P.obs + (size_t)e * AS_OBS_DIM;
  for (int k = 0; k < kSideObs; ++k) o[48 + k] = __uint_as_float(sd[(kSideState + k) * n + e]);
}

// ------------------------------------------------------------------------------------------------
// allsteps_env.py:125-174 _generate_foot_steps_allsteps (+ env origin = 0)
__device__ float lerp_t(float a, float b, float w) {  // torch.lerp (ATen Lerp.h)
  return fabsf(w) < 0.5f ? a + w * (b - a) : b - (b - a) * (1.0f - w);
}

// one env's course at `level`: draws[3][n][N] if given, else Philox (seed, env, episode, k, "Ston")
__device__ void gen_stones(const as_task_t& T, int level, uint64_t seed, uint32_t env, uint32_t episode,
                           const float* draws, float* stones, int n, int e) {
  const int N = T.num_steps, maxc = T.max_curriculum;
  const int c = min(level, maxc);
  const float ratio = (float)c / (float)maxc;
  const float step = (0.9f - 0.75f) / (float)maxc;  // torch.linspace(0.75, 0.9, 10)[c]
  const float dist_hi = c < (maxc + 1) / 2 ? 0.75f + step * (float)c : 0.9f - step * (float)(maxc - c);
  const float d2r = 0.01745329251994329577f;
  const float yaw_lo = (-20.0f * ratio) * d2r, yaw_hi = (20.0f * ratio) * d2r;
  const float p_lo = (-30.0f * ratio) * d2r + 1.57079632679489661923f;
  const float p_hi = (30.0f * ratio) * d2r + 1.57079632679489661923f;
  float x = 0.f, y = 0.f, z = 0.f, phi = 0.f;
  for (int k = 0; k < N; ++k) {
    float w[3];
    if (draws) {
      for (int j = 0; j < 3; ++j) w[j] = draws[((size_t)j * n + e) * N + k];
    } else {
      float blk[4];
      philox_block(seed, env, episode, (uint32_t)k, kStonesTag, blk);
      w[0] = blk[0]; w[1] = blk[1]; w[2] = blk[2];
    }
    float dr = lerp_t(0.75f, dist_hi, w[0]);
    float dph = lerp_t(yaw_lo, yaw_hi, w[1]);
    float dth = lerp_t(p_lo, p_hi, w[2]);
    if (k == 0) { dr = 0.f; dph = 0.f; dth = 1.57079632679489661923f; }
    if (k == 1 || k == 2) { dr = 0.75f; dph = 0.f; dth = 1.57079632679489661923f; }
    phi += dph;
    float st_, ct_, sp, cp;
    as_sincosf(dth, &st_, &ct_);
    as_sincosf(phi, &sp, &cp);
    x += dr * st_ * cp;
    y += dr * st_ * sp;
    z += dr * ct_;
    stones[(k * 3 + 0) * n + e] = x;
    stones[(k * 3 + 1) * n + e] = y;
    stones[(k * 3 + 2) * n + e] = z;
  }
}

__global__ __launch_bounds__(256) void k_stones(StonesArgs P) {
  const as_task_t& T = ((const Consts*)(CK*)P.consts)->task;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= P.n) return;
  gen_stones(T, P.level, P.seed, (uint32_t)(P.env_offset + e), 0u, P.draws, P.stones, P.n, e);
}

// ------------------------------------------------------------------------------------------------
// k_quad: the BASELINE C5 task epilogue (include/allsteps.h as_quad_task_t), one env per lane, after
// the physics substeps of k_step<18> (AS_ACT_DC_MOTOR); oracle/quad.c or_quad_post_physics is its
// serial restatement.  Coalesced SoA loads / stores (64-thread workgroups, like k_obs).
constexpr uint32_t kQuadTag = 0x51756164u;  // "Quad": reset-draw stream of the quadruped task

// k_quad: 64 envs per 256-thread workgroup.  The four feet's tips (FK of a 3-link chain each) run one
// thread per (env, foot) -- as one thread per env they were 11 % of the C5 step, a quarter of the
// SIMDs busy -- with the model tables they walk staged in LDS; the task logic then runs one thread
// per env.  Phases: (1) tips of the stepped state; (2) target ticks, rewards, dones, the reset of done
// envs (its joint angles also to LDS); (3) tips of the reset pose for the reset envs; (4) their
// potential, the state and the observation.  Per element the operations are as_link_point's
// (include/as_detmath.h, shared with oracle/quad.c) in the same order.
constexpr int kQuadEnvs = 64;
struct QuadSmem {
  int32_t parent[AS_MAX_LINKS], link_dof[AS_MAX_LINKS];
  float off_pos[AS_MAX_LINKS][3], off_quat[AS_MAX_LINKS][4], axis[AS_MAX_LINKS][3], anchor[AS_MAX_LINKS][3];
  int32_t foot_link[4];
  float foot_p1[4][3];
  float tip[kQuadEnvs][4][3];
  float root[kQuadEnvs][7];   // reset envs: the stand pose (position, quaternion)
  float qres[kQuadEnvs][AS_ACT_DIM];
  int32_t reset[kQuadEnvs];
  float obs[kQuadEnvs][AS_QUAD_OBS_DIM + 1];  // observation rows, written out coalesced (+1: banks)
};

__global__ __launch_bounds__(4 * kQuadEnvs) void k_quad(QuadArgs P) {
  const Consts& K = *(const Consts*)(CK*)P.consts;
  const as_model_t& m = K.model;
  const as_quad_task_t& Q = K.quad;
  __shared__ QuadSmem qs;
  const int tid = threadIdx.x;
  const int n = P.n, nh = m.num_hinges, N = K.task.num_steps;
  const as_state_t& st = P.st;
  static_assert(kQuadEnvs == kMapEnvs, "a workgroup's envs are one placement chunk");
  if (P.wave_map && tid < kMapEnvs) build_wave_map(P.side, P.wave_map, n, P.map_streamed != 0, blockIdx.x, tid);  // (wave 0)
  // ---- the model tables of the feet's chains, once per workgroup
  if (tid == 0) as_link_dof_map(m.cfg_dof_link, nh, AS_MAX_LINKS, qs.link_dof);
  if (tid < AS_MAX_LINKS) {
    const int i = tid;
    qs.parent[i] = m.parent[i];
    for (int k = 0; k < 3; ++k) {
      qs.off_pos[i][k] = m.offset_pos[i][k];
      qs.axis[i][k] = m.axis[i][k];
      qs.anchor[i][k] = m.anchor[i][k];
    }
    for (int k = 0; k < 4; ++k) qs.off_quat[i][k] = m.offset_quat[i][k];
  }
  if (tid < 4) {  // sensor foot f's geom: its link and capsule end p1
    int g = 0;
    for (int j = 0; j < m.num_geoms; ++j)
      if (m.geom_foot[j] == tid) { g = j; break; }
    qs.foot_link[tid] = m.geom_link[g];
    for (int k = 0; k < 3; ++k) qs.foot_p1[tid][k] = m.geom_p1[g][k];
  }
  __syncthreads();
  // foot f's tip from the joint-angle column q_col[k * stride] and the root pose
  auto tip_of = [&](int f, const float* q_col, int stride, const float* rp, const float* rq, float* tip) {
    as_link_point(qs.parent, qs.link_dof, &qs.off_pos[0][0], &qs.off_quat[0][0], &qs.axis[0][0],
                  &qs.anchor[0][0], q_col, stride, qs.foot_link[f], rp, rq, qs.foot_p1[f], tip);
  };
  // ---- (1) tips of the stepped state, thread = (env, foot)
  {
    const int le = tid >> 2, f = tid & 3, e = blockIdx.x * kQuadEnvs + le;
    if (!P.reset_all && e < n) {
      float rp[3], rq[4];
      for (int k = 0; k < 3; ++k) rp[k] = st.root_pos[k * n + e];
      for (int k = 0; k < 4; ++k) rq[k] = st.root_quat[k * n + e];
      tip_of(f, st.q + e, n, rp, rq, qs.tip[le][f]);
    }
  }
  __syncthreads();
  // ---- (2) task logic, thread = env
  const int le = tid, e = blockIdx.x * kQuadEnvs + le;
  const bool live = tid < kQuadEnvs && e < n;
  auto stone = [&](int k, int c) { return st.stones[(3 * k + c) * n + e]; };
  // xy distance of foot f's tip to the aim point on stone k
  auto aim_dist = [&](int f, int k, const float* tip) {
    const float fx = tip[0] - stone(k, 0), fy = tip[1] - (stone(k, 1) + Q.foot_offset_y[f]);
    return sqrtf(fx * fx + fy * fy);
  };
  float rp[3], rq[4], lin[3], ang[3], a[AS_ACT_DIM], q[AS_ACT_DIM], qd[AS_ACT_DIM];
  int idx = 0, ep_len = 0, t[4], c[4];
  uint32_t episode = 0u, mk[4];
  float pot = 0.f, old_pot = 0.f;
  bool was_reset = false;
  if (live) {
    for (int k = 0; k < 3; ++k) {
      rp[k] = st.root_pos[k * n + e];
      lin[k] = st.root_lin[k * n + e];
      ang[k] = st.root_ang[k * n + e];
    }
    for (int k = 0; k < 4; ++k) rq[k] = st.root_quat[k * n + e];
    for (int k = 0; k < nh; ++k) {
      const float x = P.reset_all ? 0.f : P.actions[(size_t)e * nh + k];
      a[k] = fminf(fmaxf(x, -1.f), 1.f);
    }
    idx = st.idx[e];
    ep_len = st.ep_len[e];
    for (int f = 0; f < 4; ++f) {
      t[f] = st.feet[f * n + e];
      c[f] = st.feet[(4 + f) * n + e];
    }
    episode = st.episode[e];
    mk[0] = st.contact_mask[e];
    mk[1] = st.contact_mask[n + e];
    mk[2] = st.contact_mask_hind[e];
    mk[3] = st.contact_mask_hind[n + e];
    pot = st.pot[e];
    old_pot = st.old_pot[e];
    bool term = false, trunc = false;
    if (!P.reset_all) {
      ep_len += 1;
      // target tick per foot (allsteps_env.py:418-440) and the step reward of a fresh reach (:377-380)
      float step_hit = 0.f, fsum = 0.f;
      for (int f = 0; f < 4; ++f) {
        const float* tip = qs.tip[le][f];
        const float d = aim_dist(f, t[f], tip);
        const bool reached = ((mk[f] >> t[f]) & 1u) && d < Q.step_radius;
        if (reached) c[f] += 1;
        if (c[f] >= Q.stop_frames) {
          c[f] = 0;
          t[f] = min(t[f] + 1, N - 1);
        }
        if (reached && c[f] == 1 && t[f] < N - 1) step_hit += Q.step_reward * as_expf(-d / Q.step_sigma);
        fsum += aim_dist(f, t[f], tip);  // to the (updated) target: the potential
      }
      idx = min(t[0], t[1]);
      old_pot = pot;
      const float dx = stone(idx, 0) - rp[0], dy = stone(idx, 1) - rp[1];
      const float bd = sqrtf(dx * dx + dy * dy);
      pot = -(bd + Q.foot_progress * fsum) / Q.step_dt;
      const float down[3] = {0.f, 0.f, -1.f};
      float gb[3];
      quat_rotate_inverse(rq, down, gb);
      term = gb[2] > -Q.up_z_min || rp[2] < stone(idx, 2) + Q.min_height;
      trunc = ep_len >= Q.max_episode_length;
      float a2 = 0.f, en = 0.f;
      for (int k = 0; k < nh; ++k) {
        a2 += a[k] * a[k];
        en += fabsf(st.qd[k * n + e] * a[k]);
      }
      const float bonus = idx == N - 1 && bd < Q.bonus_radius ? Q.target_bonus : 0.f;
      const float progress = pot - old_pot;
      P.reward[e] = term ? Q.death
                         : (((Q.alive + progress) - Q.energy_cost * en) - Q.action_cost * sqrtf(a2)) + step_hit + bonus;
      P.terminated[e] = term;
      P.truncated[e] = trunc;
    }
    for (int k = 0; k < nh; ++k) {
      q[k] = st.q[k * n + e];
      qd[k] = st.qd[k * n + e];
    }
    was_reset = P.reset_all || term || trunc;
    if (was_reset) {
      // the stand pose over stones 0 (hind feet) and 1 (front feet), joints + U(-1, 1) * noise
      float blk[4];
      for (int k = 0; k < nh; ++k) {
        if ((k & 3) == 0) philox_block(P.seed, (uint32_t)(P.env_offset + e), episode, (uint32_t)(k >> 2), kQuadTag, blk);
        q[k] = K.act.default_q[k] + Q.joint_noise * (2.f * blk[k & 3] - 1.f);
        qd[k] = 0.f;
        st.q[k * n + e] = q[k];
        st.qd[k * n + e] = 0.f;
        qs.qres[le][k] = q[k];
      }
      episode += 1u;
      rp[0] = 0.5f * (stone(0, 0) + stone(1, 0));
      rp[1] = 0.5f * (stone(0, 1) + stone(1, 1));
      rp[2] = fmaxf(stone(0, 2), stone(1, 2)) + K.sim.stone_half[2] + Q.stand_height;
      rq[0] = 1.f; rq[1] = rq[2] = rq[3] = 0.f;
      for (int k = 0; k < 3; ++k) {
        lin[k] = ang[k] = 0.f;
        st.root_pos[k * n + e] = rp[k];
        st.root_lin[k * n + e] = 0.f;
        st.root_ang[k * n + e] = 0.f;
        qs.root[le][k] = rp[k];
      }
      for (int k = 0; k < 4; ++k) {
        st.root_quat[k * n + e] = rq[k];
        qs.root[le][3 + k] = rq[k];
      }
    }
  }
  if (tid < kQuadEnvs) qs.reset[tid] = was_reset;
  __syncthreads();
  // ---- (3) tips of the reset pose (joint angles from LDS), thread = (env, foot)
  {
    const int le3 = tid >> 2, f = tid & 3;
    if (qs.reset[le3]) tip_of(f, qs.qres[le3], 1, &qs.root[le3][0], &qs.root[le3][3], qs.tip[le3][f]);
  }
  __syncthreads();
  // ---- (4) the reset envs' targets and potential; the state and the observation, thread = env
  if (live) {
    if (was_reset) {
      ep_len = 0;
      float fsum = 0.f;
      for (int f = 0; f < 4; ++f) {
        t[f] = min(f < 2 ? 2 : 1, N - 1);
        c[f] = 0;
        fsum += aim_dist(f, t[f], qs.tip[le][f]);
      }
      idx = min(t[0], t[1]);
      const float dx = stone(idx, 0) - rp[0], dy = stone(idx, 1) - rp[1];
      pot = -(sqrtf(dx * dx + dy * dy) + Q.foot_progress * fsum) / Q.step_dt;
      old_pot = pot;
      for (int k = 0; k < 4; ++k) mk[k] = 0u;
      st.contact_mask[e] = 0u;
      st.contact_mask[n + e] = 0u;
      st.contact_mask_hind[e] = 0u;
      st.contact_mask_hind[n + e] = 0u;
    }
    st.idx[e] = idx;
    for (int f = 0; f < 4; ++f) {
      st.feet[f * n + e] = t[f];
      st.feet[(4 + f) * n + e] = c[f];
    }
    st.ep_len[e] = ep_len;
    st.episode[e] = episode;
    st.pot[e] = pot;
    st.old_pot[e] = old_pot;
    // observation [64]: lin / ang velocity (body), projected gravity, each foot's aim point and stone
    // idx + 1 relative to the root (body), each foot on its target stone, q - default, qd, actions --
    // staged in LDS, then the block's rows (contiguous in memory) written by all 256 threads
    float* o = qs.obs[le];
    float v[3];
    quat_rotate_inverse(rq, lin, v);
    o[0] = v[0]; o[1] = v[1]; o[2] = v[2];
    quat_rotate_inverse(rq, ang, v);
    o[3] = v[0]; o[4] = v[1]; o[5] = v[2];
    const float down[3] = {0.f, 0.f, -1.f};
    quat_rotate_inverse(rq, down, v);
    o[6] = v[0]; o[7] = v[1]; o[8] = v[2];
    for (int f = 0; f < 5; ++f) {
      const int k = f < 4 ? t[f] : min(idx + 1, N - 1);
      const float oy = f < 4 ? Q.foot_offset_y[f] : 0.f;
      const float d[3] = {stone(k, 0) - rp[0], (stone(k, 1) + oy) - rp[1], stone(k, 2) - rp[2]};
      quat_rotate_inverse(rq, d, v);
      o[9 + 3 * f] = v[0]; o[10 + 3 * f] = v[1]; o[11 + 3 * f] = v[2];
    }
    for (int f = 0; f < 4; ++f) o[24 + f] = (mk[f] >> t[f]) & 1u ? 1.f : 0.f;
    for (int k = 0; k < nh; ++k) {
      o[28 + k] = q[k] - K.act.default_q[k];
      o[28 + nh + k] = qd[k];
      o[28 + 2 * nh + k] = was_reset ? 0.f : a[k];  // _reset_idx zeroes _actions (anymal_c_env.py:171-172)
    }
  }
  __syncthreads();
  const int e0 = blockIdx.x * kQuadEnvs, rows = min(kQuadEnvs, n - e0);
  float* ob = P.obs + (size_t)e0 * AS_QUAD_OBS_DIM;
  for (int x = tid; x < rows * AS_QUAD_OBS_DIM; x += 4 * kQuadEnvs)
    ob[x] = qs.obs[x / AS_QUAD_OBS_DIM][x % AS_QUAD_OBS_DIM];
}

hipError_t launch_quad(const QuadArgs& a, hipStream_t stream) {
  hipLaunchKernelGGL(k_quad, dim3((a.n + kQuadEnvs - 1) / kQuadEnvs), dim3(4 * kQuadEnvs), 0, stream, a);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// NV = 27: the Allsteps walker (6 + 21 hinges); NV = 18: the quadruped of BASELINE C5
// (model/anymal_c.xml, 6 + 12 hinges), stepped through as_physics_step.
bool step_supported_nv(int nv) { return nv == 27 || nv == 18; }

// The structural sweep (host): which column quads of which rounds the pivot rows are exactly zero in,
// for this model's tree under the sweep's layout and round order (SweepLayout).  H_ij is nonzero only
// when the links of dofs i and j are on one root path (h_row writes +0 elsewhere); a round on block P
// leaves (i, j) zero unless it was nonzero or both a_iP and a_Pj have a nonzero entry, sets the pivot
// columns where a_iP has one and the pivot rows where a_Pj has one -- a zero stays +0 through every such
// update (its products all have a +0 factor and start from +0), which is what makes a skipped quad exact.
uint64_t sweep_skip_mask(const as_model_t& m) {
  const int nl = m.num_links, nv = 6 + m.num_hinges;
  const int NP = (nv + kSweepB - 1) / kSweepB * kSweepB, NB = NP / kSweepB, NQ = NB - 1, PAD = AS_SWEEP_PAD(nv);
  if (NP > 32 || NQ * NB > 64 || nl < 1 || nl > kMaxLinks) return 0ull;
  auto padded = [&](int k) { return k < PAD ? k : k + (NP - nv); };
  auto link = [](int d) { return d < 6 ? 0 : d - 5; };
  auto on_path = [&](int a, int l) {  // a is l or one of its ancestors
    for (int x = l; x >= 0; x = x > 0 ? m.parent[x] : -1)
      if (x == a) return true;
    return false;
  };
  bool S[32][32] = {};
  for (int i = 0; i < nv; ++i)
    for (int j = 0; j < nv; ++j)
      S[padded(i)][padded(j)] = on_path(link(i), link(j)) || on_path(link(j), link(i));
  for (int q = 0; q < NP - nv; ++q) S[PAD + q][PAD + q] = true;
  uint64_t mask = 0ull;
  for (int r = 0; r < NB; ++r) {
    const int b = NB - 1 - r, p = kSweepB * b;
    bool colany[32] = {}, rowany[32] = {};
    for (int c = 0; c < kSweepB; ++c)
      for (int k = 0; k < NP; ++k) {
        colany[k] = colany[k] || S[p + c][k];
        rowany[k] = rowany[k] || S[k][p + c];
      }
    for (int jb = 0; jb < NQ; ++jb) {
      const int bb = ((b - 1 - jb) % NB + NB) % NB;
      bool any = false;
      for (int c = 0; c < kSweepB; ++c) any = any || colany[kSweepB * bb + c];
      if (!any) mask |= 1ull << (r * NQ + jb);
    }
    for (int i = 0; i < NP; ++i)
      for (int j = 0; j < NP; ++j) {
        const bool pi = i >= p && i < p + kSweepB, pj = j >= p && j < p + kSweepB;
        S[i][j] = pi && pj ? true : pj ? rowany[i] : pi ? colany[j] : (S[i][j] || (rowany[i] && colany[j]));
      }
  }
  return mask;
}

hipError_t launch_step(const StepArgs& a, int nv, bool sweep_skip, hipStream_t stream) {
  int blocks = (a.n + EPB - 1) / EPB;
  if (nv == 27 && sweep_skip)
    hipLaunchKernelGGL((k_step<27, kSweepSkip27>), dim3(blocks), dim3(kStepThreads), 0, stream, a);
  else if (nv == 27)
    hipLaunchKernelGGL((k_step<27, 0ull>), dim3(blocks), dim3(kStepThreads), 0, stream, a);
  else if (nv == 18 && sweep_skip)
    hipLaunchKernelGGL((k_step<18, kSweepSkip18>), dim3(blocks), dim3(kStepThreads), 0, stream, a);
  else if (nv == 18)
    hipLaunchKernelGGL((k_step<18, 0ull>), dim3(blocks), dim3(kStepThreads), 0, stream, a);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_obs(const ObsArgs& a, hipStream_t stream) {
  // 64-thread workgroups: one wave per CU spreads the (latency-bound, one env per lane) work over
  // 4x as many CUs and their L1 / address paths
  int blocks = (a.n + 63) / 64;
  hipLaunchKernelGGL(k_obs, dim3(blocks), dim3(64), 0, stream, a);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Ring-2 views (as_body_state, include/allsteps.h): the ArticulationData body poses and velocities of
// every model body, from the state as it stands.  Off the hot path (launched when a view is read); the
// launch shape is k_step's (two envs per one-wave workgroup) so the FK is k_step's own fk<false>.
__device__ void mat_to_quat(const float* R, float* q) {  // (w, x, y, z), w >= 0
  const float t = R[0] + R[4] + R[8];
  float w, x, y, z;
  if (t > 0.f) {
    const float r = 2.f * sqrtf(t + 1.f);
    w = 0.25f * r; x = (R[7] - R[5]) / r; y = (R[2] - R[6]) / r; z = (R[3] - R[1]) / r;
  } else if (R[0] >= R[4] && R[0] >= R[8]) {
    const float r = 2.f * sqrtf(1.f + R[0] - R[4] - R[8]);
    w = (R[7] - R[5]) / r; x = 0.25f * r; y = (R[1] + R[3]) / r; z = (R[2] + R[6]) / r;
  } else if (R[4] >= R[8]) {
    const float r = 2.f * sqrtf(1.f + R[4] - R[0] - R[8]);
    w = (R[2] - R[6]) / r; x = (R[1] + R[3]) / r; y = 0.25f * r; z = (R[5] + R[7]) / r;
  } else {
    const float r = 2.f * sqrtf(1.f + R[8] - R[0] - R[4]);
    w = (R[3] - R[1]) / r; x = (R[2] + R[6]) / r; y = (R[5] + R[7]) / r; z = 0.25f * r;
  }
  const float sg = w < 0.f ? -1.f : 1.f, nn = sg / sqrtf(w * w + x * x + y * y + z * z);
  q[0] = w * nn; q[1] = x * nn; q[2] = y * nn; q[3] = z * nn;
}

__global__ __launch_bounds__(kStepThreads) void k_body_state(BodyArgs P) {
  __shared__ Smem sm;
  const Consts& K = *(const Consts*)(CK*)P.consts;
  const int el = threadIdx.x >> 5, lane = threadIdx.x & 31;
  const int n = P.n;
  const int e_raw = blockIdx.x * EPB + el;
  const bool valid = e_raw < n;
  const int e = valid ? e_raw : n - 1;
  EnvS& s = sm.env[el];
  const as_state_t& st = P.st;
  const as_model_t& m = K.model;
  const int nh = m.num_hinges, nl = m.num_links;
  if (el == 0) sm.topo[lane] = load_topo(K, lane);
  if (lane < 3) s.root_pos[lane] = st.root_pos[lane * n + e];
  if (lane < 4) s.root_quat[lane] = st.root_quat[lane * n + e];
  if (lane < nh) {
    const int i = m.cfg_dof_link[lane] - 1;
    s.qi[i] = st.q[lane * n + e];
    s.u[6 + i] = st.qd[lane * n + e];
  }
  float v0[3], w0[3];  // the root COM's linear velocity (root_lin) and the angular velocity
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    v0[k] = st.root_lin[k * n + e];
    w0[k] = st.root_ang[k * n + e];
  }
  __syncthreads();
  const LinkC lc = load_link(K, lane);
  fk<false>(K, s, lane, sm.topo[lane], lc, K.max_path);
  // lane i >= 1: its hinge's world axis and anchor (relative to the root origin) and qd, into the
  // dynamics scratch (free after fk<false>)
  DynScratch& d = s.x.d;
  if (lane >= 1 && lane < nl) {
    float a[3], o[3];
    matvec3(s.R[lane], lc.ax, a);
    matvec3(s.R[lane], lc.an, o);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      d.c[lane][k] = a[k];
      d.Sq[lane][k] = o[k] + s.p[lane][k];
    }
    d.Sq[lane][3] = s.u[6 + lane - 1];
  }
  __syncthreads();
  const int nb = P.bodies.num_bodies;
  if (lane < nb && valid) {
    const int b = lane, L = P.bodies.link[b];
    float R0[9], c0[3];
    quat_to_mat(s.root_quat, R0);
    matvec3(R0, m.com[0], c0);
    // the root origin's velocity: v_O = v_com0 - w0 x c0
    float vO[3], t[3];
    cross3(w0, c0, t);
#pragma unroll
    for (int k = 0; k < 3; ++k) vO[k] = v0[k] - t[k];
    const float* RL = s.R[L];
    float po[3], pb[3];
    matvec3(RL, P.bodies.offset_pos[b], po);
#pragma unroll
    for (int k = 0; k < 3; ++k) pb[k] = s.p[L][k] + po[k];
    float w[3] = {w0[0], w0[1], w0[2]}, v[3];
    cross3(w0, pb, t);
#pragma unroll
    for (int k = 0; k < 3; ++k) v[k] = vO[k] + t[k];
    uint32_t path = sm.topo[L].lpath & ~1u;  // hinges on the path root..L (link j >= 1 carries hinge j - 1)
    while (path) {
      const int j = __builtin_ctz(path);
      path &= path - 1u;
      const float nj[3] = {d.c[j][0], d.c[j][1], d.c[j][2]};
      const float qd = d.Sq[j][3];
      const float r[3] = {pb[0] - d.Sq[j][0], pb[1] - d.Sq[j][1], pb[2] - d.Sq[j][2]};
      cross3(nj, r, t);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        w[k] += nj[k] * qd;
        v[k] += t[k] * qd;
      }
    }
    float Ro[9], Rb[9], q[4];
    quat_to_mat(P.bodies.offset_quat[b], Ro);
    matmul3(RL, Ro, Rb);
    mat_to_quat(Rb, q);
    float cw[3], vc[3];
    matvec3(Rb, P.bodies.com[b], cw);
    cross3(w, cw, t);
#pragma unroll
    for (int k = 0; k < 3; ++k) vc[k] = v[k] + t[k];
    const float row[AS_BODY_STATE_ROWS] = {s.root_pos[0] + pb[0], s.root_pos[1] + pb[1], s.root_pos[2] + pb[2],
                                           q[0], q[1], q[2], q[3], v[0], v[1], v[2], w[0], w[1], w[2],
                                           vc[0], vc[1], vc[2]};
#pragma unroll
    for (int r = 0; r < AS_BODY_STATE_ROWS; ++r) P.out[((size_t)r * nb + b) * n + e] = row[r];
  }
}

hipError_t launch_body_state(const BodyArgs& a, hipStream_t stream) {
  const int blocks = (a.n + EPB - 1) / EPB;
  hipLaunchKernelGGL(k_body_state, dim3(blocks), dim3(kStepThreads), 0, stream, a);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_zero(int32_t* p, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) p[i] = 0;
}

hipError_t launch_zero(int32_t* p, int n, hipStream_t stream) {
  hipLaunchKernelGGL(k_zero, dim3(1), dim3(256), 0, stream, p, n);
  return hipGetLastError();
}

hipError_t launch_stones(const StonesArgs& a, hipStream_t stream) {
  int blocks = (a.n + 255) / 256;
  hipLaunchKernelGGL(k_stones, dim3(blocks), dim3(256), 0, stream, a);
  return hipGetLastError();
}

size_t step_lds_bytes() { return sizeof(Smem) + sizeof(Consts); }

}  // namespace as
