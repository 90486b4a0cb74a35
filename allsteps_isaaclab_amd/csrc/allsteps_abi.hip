// allsteps_abi.hip -- extern "C" implementation of include/allsteps.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/allsteps.h"
#include "allsteps_kernels.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                        \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess) return fail(AS_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(_e)); \
  } while (0)

// STREAM-style copy: each thread moves 4 x 16 B per iteration (loads issued before stores), grid
// stride over the whole buffer, non-temporal so the copy does not thrash the MALL it measures past.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_hbm_copy(u32x4* __restrict__ dst, const u32x4* __restrict__ src,
                                                   int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * 256 * 4;
  for (int64_t base = (int64_t)blockIdx.x * 256 * 4 + threadIdx.x; base < n; base += stride) {
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (base + u * 256 < n) v[u] = __builtin_nontemporal_load(src + base + u * 256);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (base + u * 256 < n) __builtin_nontemporal_store(v[u], dst + base + u * 256);
  }
}

}  // namespace

struct as_env {
  int32_t n;
  int32_t device;
  uint64_t seed;
  int64_t env_offset;
  as_state_t st;
  as::Consts* consts_dev;
  int32_t* counters_dev;  // two banks of kCntBank: step t uses bank t % 2, k_obs clears the other
  int32_t bank = 0, last_bank = 0;
  int32_t graph_safe = 0;  // as_set_graph_safe: fixed bank 0 + memset per call
  uint32_t* side_dev = nullptr;  // [kSideWords][n] k_step -> k_obs
  int32_t* wave_map_dev = nullptr;  // [n] cost-balanced placement (kMapEnvs), or null: xcd_block
  int32_t map_streamed = 0;         // k_step's grid is larger than the chip's workgroup slots
  bool sweep_skip = false;          // the model admits the compiled sweep skips (as_sweep_plan)
  int32_t num_steps;
  int32_t nv;
  as::Consts host;        // host copy of consts_dev (as_set_actuator / as_set_quad_task re-upload it)
  int32_t quad_ready = 0; // as_set_quad_task called
  // optional per-launch timing (as_profile): event triples around k_step / k_obs
  std::vector<hipEvent_t> ev;
  unsigned long long* stamps = nullptr;  // diagnostic (as_debug_stamps)
  int32_t prof_cap = 0, prof_n = 0, prof_stride = 1, prof_calls = 0;
};

extern "C" {

int as_abi_version(void) { return AS_ABI_VERSION; }

#ifndef AS_BUILD_ID
#define AS_BUILD_ID "unversioned"
#endif
const char* as_build_id(void) { return AS_BUILD_ID; }

int as_hbm_copy(void* dst, const void* src, int64_t n16, void* stream) {
  if (!dst || !src || n16 < 0) return fail(AS_ERR_INVALID, "as_hbm_copy: null pointer or negative size");
  if (((uintptr_t)dst | (uintptr_t)src) & 15) return fail(AS_ERR_INVALID, "as_hbm_copy: pointers must be 16-B aligned");
  if (n16 == 0) return AS_OK;
  const int64_t per_block = 256 * 4;
  const int64_t blocks = std::min<int64_t>((n16 + per_block - 1) / per_block, 1 << 20);
  hipLaunchKernelGGL(k_hbm_copy, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, (u32x4*)dst,
                     (const u32x4*)src, n16);
  HIP_TRY(hipGetLastError());
  return AS_OK;
}

const char* as_last_error(void) { return g_err.c_str(); }

int as_sweep_plan(const as_model_t* model, uint64_t* skip_mask) {
  if (!model) return fail(AS_ERR_INVALID, "as_sweep_plan: null model");
  const int nv = 6 + model->num_hinges;
  if (!as::step_supported_nv(nv) || model->num_links < 1 || model->num_links > as::kMaxLinks)
    return fail(AS_ERR_INVALID, "as_sweep_plan: no k_step instantiation for this model");
  for (int i = 1; i < model->num_links; ++i)
    if (model->parent[i] < 0 || model->parent[i] >= i) return fail(AS_ERR_INVALID, "as_sweep_plan: parent not topological");
  const uint64_t valid = as::sweep_skip_mask(*model);
  const uint64_t compiled = nv == 27 ? as::kSweepSkip27 : as::kSweepSkip18;
  if (skip_mask) *skip_mask = valid;
  return (compiled & ~valid) == 0ull ? 1 : 0;
}

int as_create(int32_t num_envs, const as_model_t* model, const as_sim_t* sim, const as_task_t* task,
              const as_state_t* state, uint64_t seed, int32_t device, int64_t env_id_offset, as_env_t** out) {
  if (!out || !model || !sim || !task || !state) return fail(AS_ERR_INVALID, "as_create: null argument");
  *out = nullptr;
  if (num_envs <= 0) return fail(AS_ERR_INVALID, "as_create: num_envs must be > 0");
  if (num_envs > AS_MAX_ENVS)
    return fail(AS_ERR_INVALID, "as_create: num_envs > AS_MAX_ENVS (" + std::to_string(AS_MAX_ENVS) +
                                    "): the kernels' state offsets are 32-bit; shard the envs over more handles");
  if (model->num_links < 1 || model->num_links > as::kMaxLinks)
    return fail(AS_ERR_INVALID, "as_create: num_links out of range (1.." + std::to_string(as::kMaxLinks) + ")");
  if (model->num_hinges != model->num_links - 1 || model->num_hinges > AS_ACT_DIM)
    return fail(AS_ERR_INVALID, "as_create: num_hinges must be num_links-1 <= 21");
  if (model->num_geoms < 0 || model->num_geoms > AS_MAX_GEOMS) return fail(AS_ERR_INVALID, "as_create: num_geoms");
  if (task->num_steps < 1 || task->num_steps > AS_NUM_STONES) return fail(AS_ERR_INVALID, "as_create: num_steps");
  if (sim->substeps < 1 || sim->pgs_iters < 0) return fail(AS_ERR_INVALID, "as_create: substeps/pgs_iters");
  const void* ptrs[] = {state->root_pos, state->root_quat, state->root_lin, state->root_ang, state->q,
                        state->qd, state->stones, state->pot, state->old_pot, state->foot_contact,
                        state->body_pos, state->idx, state->prev, state->next, state->count, state->swing,
                        state->ep_len, state->episode, state->contact_mask, state->curriculum};
  for (const void* p : ptrs)
    if (!p) return fail(AS_ERR_INVALID, "as_create: null state field");
  // every model field the kernels index with: a malformed model is rejected here instead of becoming
  // an out-of-bounds LDS / register access (geoms: 32 LDS slots, foot id packed in 4 bits into the
  // per-foot sensor masks; self pairs: 8-bit geom indices, 6 words per lane)
  if (model->num_priority_geoms < 0 || model->num_priority_geoms > model->num_geoms)
    return fail(AS_ERR_INVALID, "as_create: num_priority_geoms outside [0, num_geoms]");
  const int max_foot = state->contact_mask_hind ? 3 : 1;
  for (int g = 0; g < model->num_geoms; ++g) {
    if (model->geom_link[g] < 0 || model->geom_link[g] >= model->num_links)
      return fail(AS_ERR_INVALID, "as_create: geom_link[" + std::to_string(g) + "] outside [0, num_links)");
    if (model->geom_type[g] != 0 && model->geom_type[g] != 1)
      return fail(AS_ERR_INVALID, "as_create: geom_type[" + std::to_string(g) + "] not 0 (sphere) / 1 (capsule)");
    if (model->geom_foot[g] < -1 || model->geom_foot[g] > max_foot)
      return fail(AS_ERR_INVALID, "as_create: geom_foot[" + std::to_string(g) + "] outside [-1, " +
                                      std::to_string(max_foot) + "] (2, 3 need contact_mask_hind)");
  }
  if (model->num_self_pairs < 0 || model->num_self_pairs > AS_MAX_SELF_PAIRS)
    return fail(AS_ERR_INVALID, "as_create: num_self_pairs outside [0, AS_MAX_SELF_PAIRS]");
  for (int i = 0; i < model->num_self_pairs; ++i) {
    const int w = model->self_pair[i], g1 = w & 0xff, g2 = w >> 8;
    if (w < 0 || g1 >= g2 || g2 >= model->num_geoms)
      return fail(AS_ERR_INVALID, "as_create: self_pair[" + std::to_string(i) + "] is not g1 | g2 << 8 with g1 < g2 < num_geoms");
  }

  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(AS_ERR_NO_DEVICE, "as_create: no HIP device");
  if (device < 0 || device >= ndev) return fail(AS_ERR_INVALID, "as_create: bad device index");
  HIP_TRY(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(AS_ERR_NO_DEVICE, std::string("as_create: device is ") + prop.gcnArchName + ", built for gfx950");

  // tree plan
  as::Consts h{};
  h.model = *model;
  h.sim = *sim;
  h.task = *task;
  h.nv = 6 + model->num_hinges;
  h.act.mode = AS_ACT_TORQUE;
  h.st_has_hind = state->contact_mask_hind != nullptr;
  const int nl = model->num_links;
  for (int i = 0; i < nl; ++i) {
    int pa = model->parent[i];
    if (i == 0 ? pa != -1 : (pa < 0 || pa >= i)) return fail(AS_ERR_INVALID, "as_create: parent not topological");
    h.lpath[i] = (i == 0 ? 0u : h.lpath[pa]) | (1u << i);
    if (i > 0 && pa == 0) h.root_kids |= 1u << i;
  }
  for (int i = 0; i < nl; ++i)
    for (int l = 0; l < nl; ++l)
      if ((h.lpath[l] >> i) & 1u) h.lsub[i] |= 1u << l;
  for (int j = 0; j < h.nv; ++j) h.dsub[j] = j < 6 ? h.lsub[0] : h.lsub[j - 5];
  for (int i = 0; i < nl; ++i) {
    h.max_path = std::max(h.max_path, __builtin_popcount(h.lpath[i]) - 1);
    if (i > 0) h.max_sub = std::max(h.max_sub, __builtin_popcount(h.lsub[i]) - 1);
  }
  while ((1 << h.fk_rounds) < h.max_path) ++h.fk_rounds;
  if (h.fk_rounds > 4) return fail(AS_ERR_INVALID, "as_create: tree deeper than 16 links");
  for (int i = 0; i < nl; ++i) {
    int a = i > 0 ? model->parent[i] : 0;
    for (int r = 0; r < 4; ++r) {  // a = the 2^r-th ancestor (0 past the root)
      h.jump[i] |= (uint32_t)a << (8 * r);
      for (int k = 0; k < (1 << r); ++k) a = a > 0 ? model->parent[a] : 0;
    }
  }
  for (int k = 0; k < model->num_hinges; ++k) {
    int li = model->cfg_dof_link[k];
    if (li < 1 || li >= model->num_links) return fail(AS_ERR_INVALID, "as_create: cfg_dof_link");
  }
  for (int l = 0; l < model->num_links; ++l) {
    uint32_t mask = 0x3Fu;
    for (int i = l; i > 0; i = model->parent[i]) mask |= 1u << (6 + i - 1);
    h.ancmask[l] = mask;
  }
  for (int j = 0; j < h.nv; ++j)
    for (int k = 0; k < h.nv; ++k) {
      const int lk = k < 6 ? 0 : k - 5;
      if ((h.ancmask[lk] >> j) & 1u) h.ddesc[j] |= 1u << k;
    }
  if (!as::step_supported_nv(h.nv))
    return fail(AS_ERR_INVALID, "as_create: no k_step instantiation for " + std::to_string(h.nv) + " dofs");

  as_env* env = new as_env();
  env->n = num_envs;
  env->device = device;
  env->seed = seed;
  env->env_offset = env_id_offset;
  env->st = *state;
  env->num_steps = task->num_steps;
  env->nv = h.nv;
  env->host = h;
  env->sweep_skip = as_sweep_plan(model, nullptr) == 1;
  if (hipMalloc(&env->consts_dev, sizeof(as::Consts)) != hipSuccess ||
      hipMalloc(&env->counters_dev, 2 * as::kCntBank * sizeof(int32_t)) != hipSuccess ||
      hipMalloc(&env->side_dev, (size_t)as::kSideWords * num_envs * sizeof(uint32_t)) != hipSuccess) {
    (void)hipFree(env->consts_dev);
    (void)hipFree(env->counters_dev);
    delete env;
    return fail(AS_ERR_HIP, "as_create: hipMalloc failed");
  }
  HIP_TRY(hipMemcpy(env->consts_dev, &h, sizeof(as::Consts), hipMemcpyHostToDevice));
  HIP_TRY(hipMemset(env->counters_dev, 0, 2 * as::kCntBank * sizeof(int32_t)));
  HIP_TRY(hipMemset(env->side_dev, 0, (size_t)as::kSideWords * num_envs * sizeof(uint32_t)));
  // cost-balanced placement (placement only: results are the same under any map); ALLSTEPS_WAVE_MAP=0
  // keeps the fixed XCD-contiguous placement (A/B timing)
  const char* wm = std::getenv("ALLSTEPS_WAVE_MAP");
  if (as::wave_map_fits(num_envs) && !(wm && std::strcmp(wm, "0") == 0)) {
    // k_step: one-wave workgroups of 2 envs, 8 per CU (LDS-bound, tests/kernel_budget.json)
    // (ALLSTEPS_WAVE_MAP=resident keeps the resident layout on a streamed grid: A/B timing)
    env->map_streamed = num_envs / 2 > 8 * prop.multiProcessorCount && !(wm && std::strcmp(wm, "resident") == 0);
    std::vector<int32_t> map((size_t)num_envs);  // the map k_obs builds from all-zero row counts (2 envs per workgroup)
    for (int w = 0; w < num_envs / as::kMapEnvs; ++w)
      for (int t = 0; t < as::kMapEnvs; ++t)
        map[(size_t)2 * as::wave_map_block(w, t >> 1, num_envs, env->map_streamed) + (t & 1)] = w * as::kMapEnvs + t;
    if (hipMalloc(&env->wave_map_dev, map.size() * sizeof(int32_t)) != hipSuccess) {
      (void)as_destroy(env);
      return fail(AS_ERR_HIP, "as_create: hipMalloc failed");
    }
    HIP_TRY(hipMemcpy(env->wave_map_dev, map.data(), map.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  }
  *out = env;
  return AS_OK;
}

int as_destroy(as_env_t* env) {
  if (!env) return AS_OK;
  (void)hipSetDevice(env->device);
  for (hipEvent_t e : env->ev) (void)hipEventDestroy(e);
  (void)hipFree(env->consts_dev);
  (void)hipFree(env->counters_dev);
  (void)hipFree(env->side_dev);
  (void)hipFree(env->wave_map_dev);
  delete env;
  return AS_OK;
}

static int run(as_env_t* env, int mode, const float* actions, float* obs, float* reward, uint8_t* term,
               uint8_t* trunc, const float* reset_draws, void* stream, const uint8_t* reset_mask = nullptr) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // no memset per step: this launch's counter bank was cleared by the previous launch's k_obs
  // (physics-only launches do not touch the counters and keep the bank)
  if (env->graph_safe && mode != as::kModePhysics) {
    env->bank = 0;
    // a kernel node, not hipMemsetAsync: replaying a captured memset node next to other graphs was
    // observed to leave the bank holding pointer-sized garbage on this ROCm build
    HIP_TRY(as::launch_zero(env->counters_dev, as::kCntBank, s));
  }
  int32_t* cnt = env->counters_dev + as::kCntBank * env->bank;
  as::StepArgs a{};
  a.consts = env->consts_dev;
  a.st = env->st;
  a.n = env->n;
  a.mode = mode;
  a.actions = actions;
  a.reward = reward;
  a.terminated = term;
  a.truncated = trunc;
  a.reset_draws = reset_draws;
  a.reset_mask = reset_mask;
  a.counters = cnt;
  a.seed = env->seed;
  a.env_offset = env->env_offset;
  a.stamps = env->stamps;
  a.obs = mode == as::kModePhysics ? nullptr : obs;
  a.side = env->side_dev;
  a.wave_map = env->wave_map_dev;
  const bool prof = env->prof_n < env->prof_cap && (env->prof_calls++ % env->prof_stride) == 0;
  if (prof) HIP_TRY(hipEventRecord(env->ev[3 * env->prof_n], s));
  HIP_TRY(as::launch_step(a, env->nv, env->sweep_skip, s));
  if (prof) HIP_TRY(hipEventRecord(env->ev[3 * env->prof_n + 1], s));
  if (mode == as::kModePhysics) {
    if (prof) {
      HIP_TRY(hipEventRecord(env->ev[3 * env->prof_n + 2], s));
      ++env->prof_n;
    }
    return AS_OK;
  }
  as::ObsArgs o{};
  o.consts = env->consts_dev;
  o.st = env->st;
  o.n = env->n;
  o.counters = cnt;
  o.next_counters = env->counters_dev + as::kCntBank * (env->bank ^ 1);
  env->last_bank = env->bank;
  if (!env->graph_safe) env->bank ^= 1;
  o.obs = obs;
  o.side = env->side_dev;
  o.seed = env->seed;
  o.env_offset = env->env_offset;
  o.wave_map = env->wave_map_dev;
  o.map_streamed = env->map_streamed;
  HIP_TRY(as::launch_obs(o, s));
  if (prof) {
    HIP_TRY(hipEventRecord(env->ev[3 * env->prof_n + 2], s));
    ++env->prof_n;
  }
  return AS_OK;
}

int as_debug_stamps(as_env_t* env, uint64_t* stamps_dev) {
  if (!env) return fail(AS_ERR_INVALID, "as_debug_stamps: null handle");
  env->stamps = reinterpret_cast<unsigned long long*>(stamps_dev);
  return AS_OK;
}

int as_profile(as_env_t* env, int32_t max_launches) {
  if (!env || max_launches < 0) return fail(AS_ERR_INVALID, "as_profile: bad argument");
  HIP_TRY(hipSetDevice(env->device));
  for (hipEvent_t e : env->ev) HIP_TRY(hipEventDestroy(e));
  env->ev.assign(3 * (size_t)max_launches, nullptr);
  for (auto& e : env->ev) HIP_TRY(hipEventCreate(&e));
  env->prof_cap = max_launches;
  env->prof_n = 0;
  env->prof_stride = 1;
  env->prof_calls = 0;
  return AS_OK;
}

int as_profile_sampled(as_env_t* env, int32_t max_records, int32_t stride) {
  if (!env || stride < 1) return fail(AS_ERR_INVALID, "as_profile_sampled: bad argument");
  const int rc = as_profile(env, max_records);
  if (rc != AS_OK) return rc;
  env->prof_stride = stride;
  return AS_OK;
}

int as_profile_read(as_env_t* env, double* step_kernel_ms, double* obs_kernel_ms, int32_t* launches) {
  if (!env || !step_kernel_ms || !obs_kernel_ms || !launches) return fail(AS_ERR_INVALID, "as_profile_read: null");
  double a = 0.0, b = 0.0;
  if (env->prof_n > 0) HIP_TRY(hipEventSynchronize(env->ev[3 * env->prof_n - 1]));
  for (int i = 0; i < env->prof_n; ++i) {
    float t1 = 0.f, t2 = 0.f;
    HIP_TRY(hipEventElapsedTime(&t1, env->ev[3 * i], env->ev[3 * i + 1]));
    HIP_TRY(hipEventElapsedTime(&t2, env->ev[3 * i + 1], env->ev[3 * i + 2]));
    a += t1;
    b += t2;
  }
  *step_kernel_ms = a;
  *obs_kernel_ms = b;
  *launches = env->prof_n;
  env->prof_n = 0;
  return AS_OK;
}

int as_step(as_env_t* env, const float* actions, float* obs, float* reward, uint8_t* terminated, uint8_t* truncated,
            const float* reset_draws, void* stream) {
  if (!env || !actions || !obs || !reward || !terminated || !truncated)
    return fail(AS_ERR_INVALID, "as_step: null argument");
  return run(env, as::kModeStep, actions, obs, reward, terminated, truncated, reset_draws, stream);
}

int as_task_step(as_env_t* env, const float* actions, float* obs, float* reward, uint8_t* terminated,
                 uint8_t* truncated, const float* reset_draws, void* stream) {
  if (!env || !actions || !obs || !reward || !terminated || !truncated)
    return fail(AS_ERR_INVALID, "as_task_step: null argument");
  return run(env, as::kModeTask, actions, obs, reward, terminated, truncated, reset_draws, stream);
}

int as_set_seed(as_env_t* env, uint64_t seed) {
  if (!env) return fail(AS_ERR_INVALID, "as_set_seed: null handle");
  env->seed = seed;
  return AS_OK;
}

int as_reset_all(as_env_t* env, float* obs, const float* reset_draws, void* stream) {
  if (!env || !obs) return fail(AS_ERR_INVALID, "as_reset_all: null argument");
  return run(env, as::kModeReset, nullptr, obs, nullptr, nullptr, nullptr, reset_draws, stream);
}

int as_reset_mask(as_env_t* env, const uint8_t* mask, float* obs, const float* reset_draws, void* stream) {
  if (!env || !mask || !obs) return fail(AS_ERR_INVALID, "as_reset_mask: null argument");
  return run(env, as::kModeReset, nullptr, obs, nullptr, nullptr, nullptr, reset_draws, stream, mask);
}

int as_physics_step(as_env_t* env, const float* actions, void* stream) {
  if (!env || !actions) return fail(AS_ERR_INVALID, "as_physics_step: null argument");
  return run(env, as::kModePhysics, actions, nullptr, nullptr, nullptr, nullptr, nullptr, stream);
}

int as_set_actuator(as_env_t* env, const as_actuator_t* act) {
  if (!env || !act) return fail(AS_ERR_INVALID, "as_set_actuator: null argument");
  if (act->mode != AS_ACT_TORQUE && act->mode != AS_ACT_DC_MOTOR) return fail(AS_ERR_INVALID, "as_set_actuator: mode");
  if (act->mode == AS_ACT_DC_MOTOR && !(act->velocity_limit > 0.f && act->effort_limit >= 0.f))
    return fail(AS_ERR_INVALID, "as_set_actuator: the DC motor needs velocity_limit > 0 and effort_limit >= 0");
  HIP_TRY(hipSetDevice(env->device));
  env->host.act = *act;
  // ordered on the null stream with respect to every earlier launch (hipMemcpy synchronises)
  // setup call, not stream-ordered: every launch still queued on any stream (torch's pool streams are
  // non-blocking, so a plain hipMemcpy would not wait for them) finishes before the block changes
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(env->consts_dev, &env->host, sizeof(as::Consts), hipMemcpyHostToDevice));
  return AS_OK;
}

int as_set_quad_task(as_env_t* env, const as_quad_task_t* q) {
  if (!env || !q) return fail(AS_ERR_INVALID, "as_set_quad_task: null argument");
  if (env->host.model.num_hinges != 12 || 28 + 3 * env->host.model.num_hinges != AS_QUAD_OBS_DIM)
    return fail(AS_ERR_INVALID, "as_set_quad_task: the task is defined for a 12-hinge quadruped");
  if (!env->st.contact_mask_hind || !env->st.feet)
    return fail(AS_ERR_INVALID, "as_set_quad_task: state->contact_mask_hind / state->feet is NULL");
  if (q->stop_frames < 1 || q->max_episode_length < 1 || !(q->step_dt > 0.f) || env->num_steps < 3 ||
      !(q->step_sigma > 0.f))
    return fail(AS_ERR_INVALID, "as_set_quad_task: stop_frames / max_episode_length / step_dt / num_steps / step_sigma");
  for (int f = 0; f < 4; ++f) {  // k_quad takes each swing foot's tip from its sensor geom
    bool found = false;
    for (int g = 0; g < env->host.model.num_geoms; ++g) found = found || env->host.model.geom_foot[g] == f;
    if (!found) return fail(AS_ERR_INVALID, "as_set_quad_task: the model needs a foot geom for each sensor 0..3");
  }
  HIP_TRY(hipSetDevice(env->device));
  env->host.quad = *q;
  // setup call, not stream-ordered: every launch still queued on any stream (torch's pool streams are
  // non-blocking, so a plain hipMemcpy would not wait for them) finishes before the block changes
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(env->consts_dev, &env->host, sizeof(as::Consts), hipMemcpyHostToDevice));
  env->quad_ready = 1;
  return AS_OK;
}

static int quad(as_env_t* env, int reset_all, const float* actions, float* obs, float* reward, uint8_t* term,
                uint8_t* trunc, void* stream) {
  if (!env->quad_ready) return fail(AS_ERR_INVALID, "as_quad_*: call as_set_quad_task first");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (!reset_all) {
    const int rc = run(env, as::kModePhysics, actions, nullptr, nullptr, nullptr, nullptr, nullptr, stream);
    if (rc != AS_OK) return rc;
  }
  as::QuadArgs a{};
  a.consts = env->consts_dev;
  a.st = env->st;
  a.n = env->n;
  a.reset_all = reset_all;
  a.actions = actions;
  a.obs = obs;
  a.reward = reward;
  a.terminated = term;
  a.truncated = trunc;
  a.seed = env->seed;
  a.env_offset = env->env_offset;
  a.side = env->side_dev;
  a.wave_map = env->wave_map_dev;
  a.map_streamed = env->map_streamed;
  HIP_TRY(as::launch_quad(a, s));
  return AS_OK;
}

int as_quad_step(as_env_t* env, const float* actions, float* obs, float* reward, uint8_t* terminated,
                 uint8_t* truncated, void* stream) {
  if (!env || !actions || !obs || !reward || !terminated || !truncated)
    return fail(AS_ERR_INVALID, "as_quad_step: null argument");
  return quad(env, 0, actions, obs, reward, terminated, truncated, stream);
}

int as_quad_reset_all(as_env_t* env, float* obs, void* stream) {
  if (!env || !obs) return fail(AS_ERR_INVALID, "as_quad_reset_all: null argument");
  return quad(env, 1, nullptr, obs, nullptr, nullptr, nullptr, stream);
}

int as_generate_stones(as_env_t* env, int32_t level, const float* draws, void* stream) {
  if (!env) return fail(AS_ERR_INVALID, "as_generate_stones: null handle");
  if (level < 0) return fail(AS_ERR_INVALID, "as_generate_stones: level < 0");
  as::StonesArgs a{};
  a.consts = env->consts_dev;
  a.stones = env->st.stones;
  a.n = env->n;
  a.level = level;
  a.draws = draws;
  a.seed = env->seed;
  a.env_offset = env->env_offset;
  HIP_TRY(as::launch_stones(a, reinterpret_cast<hipStream_t>(stream)));
  return AS_OK;
}

int as_body_state(as_env_t* env, const as_body_table_t* bodies_host, float* out, void* stream) {
  if (!env || !bodies_host || !out) return fail(AS_ERR_INVALID, "as_body_state: null argument");
  const as_body_table_t& b = *bodies_host;
  if (b.num_bodies < 1 || b.num_bodies > AS_MAX_BODIES)
    return fail(AS_ERR_INVALID, "as_body_state: num_bodies out of range [1, AS_MAX_BODIES]");
  for (int i = 0; i < b.num_bodies; ++i)
    if (b.link[i] < 0 || b.link[i] >= env->host.model.num_links)
      return fail(AS_ERR_INVALID, "as_body_state: body link out of range");
  as::BodyArgs a{};
  a.consts = env->consts_dev;
  a.st = env->st;
  a.n = env->n;
  a.out = out;
  a.bodies = b;
  HIP_TRY(as::launch_body_state(a, reinterpret_cast<hipStream_t>(stream)));
  return AS_OK;
}

int as_set_graph_safe(as_env_t* env, int32_t on) {
  if (!env) return fail(AS_ERR_INVALID, "as_set_graph_safe: null handle");
  env->graph_safe = on != 0;
  return AS_OK;
}

int as_step_counters(as_env_t* env, const int32_t** counters_dev) {
  if (!env || !counters_dev) return fail(AS_ERR_INVALID, "as_step_counters: null argument");
  *counters_dev = env->counters_dev + as::kCntBank * env->last_bank;
  return AS_OK;
}

int as_step_counters_host(as_env_t* env, int32_t* out_host, void* stream) {
  if (!env || !out_host) return fail(AS_ERR_INVALID, "as_step_counters_host: null argument");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  HIP_TRY(hipMemcpyAsync(out_host, env->counters_dev + as::kCntBank * env->last_bank, 4 * sizeof(int32_t),
                         hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  return AS_OK;
}

int as_get_curriculum_host(as_env_t* env, int32_t* level_host) {
  if (!env || !level_host) return fail(AS_ERR_INVALID, "as_get_curriculum_host: null argument");
  HIP_TRY(hipMemcpy(level_host, env->st.curriculum, sizeof(int32_t), hipMemcpyDeviceToHost));
  return AS_OK;
}

}  // extern "C"
