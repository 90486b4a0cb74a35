/*
 * allsteps.h -- C ABI of the MI355X-native Allsteps-v0 step (liballsteps_hip.so).
 *
 * The reference's hot path is DirectRLEnv.step (isaaclab/envs/direct_rl_env.py:296-383) over the
 * Allsteps task (isaaclab_tasks/direct/allsteps/allsteps_env.py:257-567), whose physics half is
 * the omni.physics.tensors / PhysX operator surface (SURVEY.md §8b "Ring 3"):
 *   set_dof_actuation_forces      (articulation.py:195)          -> as_step (actions in, torque inside)
 *   SimulationContext.step / simulate(dt) x decimation (simulation_context.py:453-478) -> as_step
 *   get_root_transforms / get_root_velocities / get_dof_positions / get_dof_velocities
 *       (articulation_data.py:374-376, 533, 542)                -> state views (as_state_t)
 *   update_articulations_kinematic (articulation_data.py:439)   -> fused FK inside as_step
 *   RigidContactView.get_contact_force_matrix (contact_sensor.py:341) -> contact_mask (as_state_t)
 *   set_root_* / set_dof_* on reset (articulation.py:316-341, 400-420, 472-551) -> in-kernel reset
 * and the task code around it (_apply_action, _get_dones, _get_rewards, _reset_idx,
 * _get_observations), fused into two kernels per env step.
 *
 * Conventions: every buffer argument is a DEVICE pointer unless its name ends in _host; the caller
 * owns all buffers (state included, see as_state_t) and keeps them alive for the handle's life;
 * `stream` is a hipStream_t (NULL = default stream).  Calls on one handle are serialised by the
 * caller.  No call synchronises the stream except as_get_curriculum_host.  Every function returns 0
 * on success or a negative AS_ERR_* code; as_last_error() gives a message (thread-local).
 */
#ifndef ALLSTEPS_H
#define ALLSTEPS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AS_ABI_VERSION 5
#define AS_MAX_LINKS 32
#define AS_MAX_GEOMS 32
#define AS_MAX_SELF_PAIRS 256
/* envs per handle: the kernels index the field-major state and the [5][n][20] draw tables with 32-bit
 * offsets (row * n + env, < 2^31); 2^24 envs is ~22 GB of state, far past one GPU's useful launch */
#define AS_MAX_ENVS (1 << 24)
#define AS_NUM_STONES 20
/* Constraint budget per env and substep: every active joint-limit row is kept (a walker has at most
 * 21, one side per hinge); contacts fill the remaining rows three at a time up to AS_MAX_CONTACTS, in
 * priority order: feet on stones, other geoms on stones, robot self-contacts. */
#define AS_MAX_CONTACTS 10
#define AS_MAX_ROWS 30
#define AS_OBS_DIM 59
#define AS_ACT_DIM 21
#define AS_QUAD_OBS_DIM 64

enum {
  AS_OK = 0,
  AS_ERR_INVALID = -1,   /* bad argument (null pointer, size out of range, model too large) */
  AS_ERR_HIP = -2,       /* HIP runtime error (message has the hipError string) */
  AS_ERR_NO_DEVICE = -3, /* no gfx950 device / code object for this device */
};

/* Robot model tables (allsteps_isaaclab_amd/model/walker3d.json; compiled from walker3d.xml). */
typedef struct {
  int32_t num_links;                  /* incl. floating root = link 0; link i >= 1 carries hinge i-1 */
  int32_t num_hinges;                 /* num_links - 1 (== AS_ACT_DIM for the walker) */
  int32_t parent[AS_MAX_LINKS];       /* topological: parent[i] < i */
  float offset_pos[AS_MAX_LINKS][3];
  float offset_quat[AS_MAX_LINKS][4]; /* (w, x, y, z) */
  float axis[AS_MAX_LINKS][3];
  float anchor[AS_MAX_LINKS][3];
  float mass[AS_MAX_LINKS];
  float com[AS_MAX_LINKS][3];
  float inertia[AS_MAX_LINKS][6];     /* about COM, link frame: xx yy zz xy xz yz */
  float armature[AS_MAX_LINKS];
  float lower[AS_MAX_LINKS];
  float upper[AS_MAX_LINKS];
  int32_t cfg_dof_link[AS_MAX_LINKS]; /* PhysX/cfg dof k -> link */
  float gear[AS_MAX_LINKS];           /* cfg order (allsteps_env_cfg.py:133-155) */
  int32_t num_geoms;
  int32_t geom_link[AS_MAX_GEOMS];
  int32_t geom_type[AS_MAX_GEOMS];    /* 0 sphere, 1 capsule */
  int32_t geom_foot[AS_MAX_GEOMS];    /* contact sensor 0..3 or -1 (walker: 0 right, 1 left foot;
                                         quadruped: RF, LF, RH, LH) */
  float geom_radius[AS_MAX_GEOMS];
  float geom_p0[AS_MAX_GEOMS][3];
  float geom_p1[AS_MAX_GEOMS][3];
  int32_t torso_link;
  int32_t foot_link[2];
  int32_t num_priority_geoms;         /* geoms [0, n) (the feet) emit their stone contacts first */
  int32_t num_self_pairs;             /* self-collision geom pairs (walker3d.py:27 enabled_self_collisions) */
  int32_t self_pair[AS_MAX_SELF_PAIRS]; /* g1 | g2 << 8, g1 < g2, ascending (model/__init__.py) */
} as_model_t;

/* Physics constants (simulation_cfg.py; walker3d.py:21-46; allsteps_env_cfg.py:62). */
typedef struct {
  float dt;
  int32_t substeps;
  float gravity;
  float friction;
  float margin;
  float baumgarte;
  float slop;
  float max_depen_vel;
  int32_t pgs_iters;
  float stone_half[3];
  float max_joint_vel;
} as_sim_t;

/* Task constants (allsteps_env.py:29-60; allsteps_env_cfg.py:54-234). */
typedef struct {
  int32_t num_steps;
  float step_radius;
  int32_t stop_frames;
  float eps;
  float alive, energy, action, joint_limit, death, dof_vel_scale, fall_abs;
  float step_dt;
  int32_t max_episode_length;
  int32_t max_curriculum;
  int32_t curriculum_threshold;
  float term_curriculum[10];
  float gain_curriculum[10];
  float init_root[3];
  float init_q[21];
  int32_t right_idx[9], left_idx[9], neg_idx[2];
  float noise_lo, noise_hi, clip_lo, clip_hi;
  /* 0 = reference behaviour (stones never regenerate: _reset_idx resets curr_target_index before its
   * over-half test, allsteps_env.py:492-500); 1 = the intended behaviour: a reset
   * env whose target index was > num_steps / 2 gets new stones at the (post-gate) curriculum level */
  int32_t regen_footsteps;
} as_task_t;

/* Per-env state: structure of arrays, field-major / env-minor ([field][num_envs]), device memory,
 * caller-owned.  These are the ArticulationData views of the reference:
 *   root_pos/root_quat  = root_state_w[:, 0:7]  (root link frame, quat w,x,y,z)
 *   root_lin/root_ang   = root_state_w[:, 7:13] (root link COM velocity, world)
 *   q / qd              = joint_pos / joint_vel (cfg dof order)
 *   body_pos            = body_pos_w[:, {torso, right_foot, left_foot}]
 * and the AllstepsEnv task buffers (allsteps_env.py:66-96). */
typedef struct {
  float* root_pos;      /* [3][n] */
  float* root_quat;     /* [4][n] */
  float* root_lin;      /* [3][n] */
  float* root_ang;      /* [3][n] */
  float* q;             /* [21][n] */
  float* qd;            /* [21][n] */
  float* stones;        /* [20*3][n]  steps_pos, env-local frame (env origin = 0) */
  float* pot;           /* [n] potentials */
  float* old_pot;       /* [n] old_potentials */
  float* foot_contact;  /* [2][n] */
  float* body_pos;      /* [9][n] */
  int32_t* idx;         /* [n] curr_target_index */
  int32_t* prev;        /* [n] */
  int32_t* next;        /* [n] */
  int32_t* count;       /* [n] target_reach_count */
  int32_t* swing;       /* [n] swing_leg */
  int32_t* ep_len;      /* [n] episode_length_buf */
  uint32_t* episode;    /* [n] reset counter: Philox stream of the reset draws */
  uint32_t* contact_mask; /* [2][n] per-foot bitmask of stones with force > eps, last substep */
  int32_t* curriculum;  /* [1] */
  uint32_t* contact_mask_hind; /* [2][n] contact sensors 2 and 3 (a quadruped's hind feet), or NULL */
  int32_t* feet;        /* [8][n] the quadruped task's per-foot target stones (rows 0..3, sensor order)
                           and reach counts (rows 4..7), or NULL (the walker) */
} as_state_t;

/* Actuation of the physics step (as_set_actuator; as_create starts in AS_ACT_TORQUE).
 *   AS_ACT_TORQUE:   tau = gain_curriculum[level] * gear * clip(a, -1, 1)  (the Allsteps walker,
 *                    allsteps_env.py:267-274, an ImplicitActuator with kp = kd = 0);
 *   AS_ACT_DC_MOTOR: joint position targets q* = default_q + action_scale * clip(a, -1, 1)
 *                    (anymal_c_env.py:73-78), tracked by IsaacLab's DCMotor actuator evaluated in
 *                    every physics substep: tau = kp (q* - q) + kd (0 - qd)  (IdealPD,
 *                    actuator_pd.py:184-199), clipped to [tau_min(qd), tau_max(qd)] with
 *                    tau_max = clip(sat (1 - qd / v_max), 0, effort_limit),
 *                    tau_min = clip(sat (-1 - qd / v_max), -effort_limit, 0)  (actuator_pd.py:264-275). */
enum { AS_ACT_TORQUE = 0, AS_ACT_DC_MOTOR = 1 };
typedef struct {
  int32_t mode;
  float action_scale;
  float default_q[AS_ACT_DIM];   /* cfg dof order */
  float stiffness, damping;
  float saturation_effort, effort_limit, velocity_limit;
} as_actuator_t;

/* The BASELINE C5 task: a quadruped crossing the Allsteps stones with the ALLSTEPS reward terms
 * (allsteps_env.py:347-394) and the reference's target machine (:418-457) run per foot (authored here --
 * the reference has no quadruped stepping-stone task; its ANYmal-C task is flat-ground velocity
 * tracking).  Per env step, after the physics substeps:
 *   feet: every sensor foot f (0..3 = RF, LF, RH, LH) has its own target stone t_f (state.feet rows
 *     0..3; 2 for the front feet and 1 for the hind feet after a reset: they stand on stones 1 / 0) and
 *     reach count c_f (rows 4..7); its aim point is stone t_f's centre + (0, foot_offset_y[f]), its
 *     position the tip of its sensor geom (the capsule end p1, FK from q: as_link_point);
 *   target tick per foot (allsteps_env.py:418-440): reached = f pushes on t_f (contact mask bit) and
 *     its xy distance d to the aim point < step_radius; c_f += reached; c_f >= stop_frames: c_f = 0,
 *     t_f += 1 (clamped); the front pair's target idx = min(t_RF, t_LF) (state.idx);
 *   potential (:441-448): pot = -(|stone[idx] - root|_xy + foot_progress sum_f d_f) / step_dt, d_f
 *     the foot's distance to its (updated) aim point;
 *   terminated = body tilted past up_z_min or below the target stone + min_height; truncated at
 *     max_episode_length;
 *   reward (:347-394) = alive + (pot - old_pot) - energy_cost sum|qd a| - action_cost ||a||
 *     + sum_f step_reward exp(-d_f / step_sigma) over the feet with a fresh reach (c_f == 1, t_f <
 *     num_steps - 1) + target_bonus when idx is the last stone and the root is within bonus_radius of
 *     it (xy); death on termination;
 * reset of done envs to the stand pose over stones 0 / 1 (+ U(-1,1) * joint_noise, Philox); observation
 * [64] = root linear / angular velocity (body frame), projected gravity, each foot's aim point and
 * stone idx + 1 relative to the root (body frame), each foot's contact with its target stone [4],
 * q - default_q, qd, the clipped actions. */
typedef struct {
  int32_t stop_frames;
  float alive, action_cost, death;
  float min_height, up_z_min;
  int32_t max_episode_length;
  float step_dt;
  float stand_height;       /* root z above the higher of stones 0 / 1's top face at reset */
  float joint_noise;
  float energy_cost;        /* energy_cost_scale (allsteps_env_cfg.py:222) */
  float step_radius;        /* allsteps_env_cfg.py:97 */
  float step_reward;        /* 50 (allsteps_env.py:380) */
  float step_sigma;         /* 0.25 */
  float target_bonus;       /* 10 (allsteps_env.py:383) */
  float bonus_radius;       /* 0.15 */
  float foot_progress;      /* weight of the feet's distances in the potential */
  float foot_offset_y[4];   /* aim point lateral offset per sensor foot (RF, LF, RH, LH) */
} as_quad_task_t;

typedef struct as_env as_env_t;

/* Create a handle for `num_envs` envs on HIP device `device`.  `env_id_offset` is this shard's
 * first global env id (Philox stream = (seed, env_id_offset + e, episode)), so a sharded run is
 * bit-identical to an unsharded one.  The state pointers are stored, not copied.  The model's
 * 6 + num_hinges must have a compiled step kernel: 27 (the Allsteps walker, as_step / as_task_step /
 * as_physics_step) or 18 (the BASELINE C5 quadruped, as_physics_step); otherwise AS_ERR_INVALID. */
int as_create(int32_t num_envs, const as_model_t* model_host, const as_sim_t* sim_host,
              const as_task_t* task_host, const as_state_t* state, uint64_t seed, int32_t device,
              int64_t env_id_offset, as_env_t** out);
int as_destroy(as_env_t* env);

/* DirectRLEnv.reset (direct_rl_env.py:256-294): _reset_idx(all) -> FK -> observations. */
int as_reset_all(as_env_t* env, float* obs, const float* reset_draws, void* stream);

/* AllstepsEnv._reset_idx(env_ids) (allsteps_env.py:469-567, direct_rl_env.py:563-584) on the envs
 * with mask[e] != 0 (device, [n] uint8), then _get_observations for all envs into obs [n][59].
 * Like the reference's _reset_idx it applies the curriculum gate (mean target index over all envs)
 * and the second foot-state tick to every env; an all-zero mask changes nothing (the reference
 * never calls _reset_idx with no ids).  reset_draws as in as_step. */
int as_reset_mask(as_env_t* env, const uint8_t* mask, float* obs, const float* reset_draws, void* stream);

/* DirectRLEnv.step (direct_rl_env.py:296-383) for all envs: actions [n][21] (any range, clamped
 * to [-1,1] inside) -> obs [n][59], reward [n], terminated [n], truncated [n] (uint8 0/1).
 * reset_draws: NULL (Philox) or [n][22] U[0,1) draws (mirror, 21 joint-noise) for envs that reset
 * this step -- the reference's torch.rand(K) / rand(K,21) (allsteps_env.py:518,542). */
int as_step(as_env_t* env, const float* actions, float* obs, float* reward, uint8_t* terminated,
            uint8_t* truncated, const float* reset_draws, void* stream);

/* Task logic only (the post-physics half of as_step): body_pos / contact_mask are taken from the
 * state as the caller wrote them -- the operator a task-logic golden replay drives. */
int as_task_step(as_env_t* env, const float* actions, float* obs, float* reward, uint8_t* terminated,
                 uint8_t* truncated, const float* reset_draws, void* stream);

/* Re-seed the Philox reset-draw stream (DirectRLEnv.seed / reset(seed=...)). */
int as_set_seed(as_env_t* env, uint64_t seed);

/* Physics only (decimation substeps, no task logic): for known-answer tests and profiling. */
int as_physics_step(as_env_t* env, const float* actions, void* stream);

/* Select the actuation of the physics step (AS_ACT_TORQUE / AS_ACT_DC_MOTOR, see as_actuator_t).
 * as_set_actuator and as_set_quad_task are setup calls: they synchronize the device (every queued
 * launch on every stream finishes first) and then rewrite the handle's constants block.  Not graph-
 * safe: a captured graph keeps reading the block and sees the new values on its next replay. */
int as_set_actuator(as_env_t* env, const as_actuator_t* act_host);
/* BASELINE C5: the quadruped stepping-stone task (as_quad_task_t).  as_quad_step = physics substeps
 * (with the handle's actuator) + the task epilogue of every env, reset of done envs and the
 * observation [n][AS_QUAD_OBS_DIM]; as_quad_reset_all resets every env.  Needs a model whose sensor
 * feet 0..3 are the four feet and state->contact_mask_hind != NULL. */
int as_set_quad_task(as_env_t* env, const as_quad_task_t* task_host);
int as_quad_step(as_env_t* env, const float* actions, float* obs, float* reward, uint8_t* terminated,
                 uint8_t* truncated, void* stream);
int as_quad_reset_all(as_env_t* env, float* obs, void* stream);

/* _generate_foot_steps_allsteps (allsteps_env.py:125-174) on the device at curriculum `level`;
 * draws: [5][n][20] U[0,1) (NULL = Philox stream (seed, env, 0xF007)). Writes state->stones. */
int as_generate_stones(as_env_t* env, int32_t level, const float* draws, void* stream);

/* Ring-2 views, off the hot path (round 6).  The reference's ArticulationData body views
 * (articulation_data.py:430-447 body_state_w -- link-frame pose, COM velocity -- and body_link_state_w --
 * link-frame pose and velocity; body_pos_w = body_state_w[..., :3]) for EVERY body of the model (the
 * walker's 17 MJCF bodies), computed on demand from the SoA state as it stands: root pose / velocity
 * (root_lin is the root COM's velocity, as in the state), q, qd.  FK with the step kernel's own
 * arithmetic, so rows of bodies whose frame is the torso / a foot link equal state->body_pos bit for bit;
 * then per body b, with L = link[b]:
 *   pos  = root_pos + p_L + R_L offset_pos[b]             rot = R_L R(offset_quat[b])  (quat w, x, y, z)
 *   w    = root angular velocity + sum over the hinges j on the path of L of axis_j(world) * qd_j
 *   vfrm = velocity of the body frame's origin             vcom = velocity of the body's own COM (com[b])
 * out: device [AS_BODY_STATE_ROWS][num_bodies][n] fp32 = pos 3 | quat 4 | vfrm 3 | w 3 | vcom 3.
 * as_step never runs it; the caller launches it when a view is read (envs/allsteps_env.py). */
#define AS_MAX_BODIES 32
#define AS_BODY_STATE_ROWS 16
typedef struct {
  int32_t num_bodies;
  int32_t link[AS_MAX_BODIES];          /* the link whose frame carries the body (model body_link) */
  float offset_pos[AS_MAX_BODIES][3];   /* body frame in that link's frame */
  float offset_quat[AS_MAX_BODIES][4];  /* (w, x, y, z) */
  float com[AS_MAX_BODIES][3];          /* the body's own centre of mass, body frame */
} as_body_table_t;
int as_body_state(as_env_t* env, const as_body_table_t* bodies_host, float* out, void* stream);

/* The H^-1 sweep plan for a model (round 6, ABI 5; no device needed).  The step kernel sweeps the
 * padded joint-space inertia last block first and, for the trees it is compiled for (the walker, the
 * C5 quadruped), skips the column quads in which the pivot rows are structurally zero -- an exact
 * identity, so results do not depend on it.  Returns 1 when the compiled skips hold for `model` (as_create
 * then launches the skipping kernel), 0 when they do not (the full sweep runs), <0 on an invalid model;
 * *skip_mask (if not NULL) receives the quads that are zero for this model (bit r (NB-1) + q: round r,
 * quad q).  Replaces nothing in the reference: PhysX factors the articulation internally. */
int as_sweep_plan(const as_model_t* model, uint64_t* skip_mask);

/* Per-launch timing: record HIP events around the step kernel (k_step) and the observation
 * kernel (k_obs) of the next `max_launches` calls on their own stream; as_profile_read
 * synchronises on the last event and returns the summed durations (ms) and the launch count. */
int as_profile(as_env_t* env, int32_t max_launches);
/* Sampled form: time every `stride`-th call only (up to `max_records` of them), so the events'
 * launch gaps touch 1 / stride of the calls of a timed loop. */
int as_profile_sampled(as_env_t* env, int32_t max_records, int32_t stride);
int as_profile_read(as_env_t* env, double* step_kernel_ms, double* obs_kernel_ms, int32_t* launches);

/* Diagnostic: when stamps_dev (device, >= 32 uint64) is non-null, every k_step wave adds the
 * s_memtime cycles of each of its 15 phases (load, fk, rnea, H rows, H^-1 sweep, solve, collide,
 * rows, W, pgs, integrate, final fk, task, reset, store) to slots 0..14; slot 15 keeps the largest
 * single-wave total of any launch and slots 16..30 the largest single-wave cycles of each phase
 * (atomicMax).  If slot 31 is non-zero on entry, the buffer must hold 64 + 26 * ceil(num_envs / 2)
 * words and each wave instead stores (no atomics) a 26-word record of its own at 64 + 26 * block
 * (phases, total, start / end s_memtime, HW_ID, XCC_ID, rows and contacts per env, start / end
 * s_memrealtime), overwritten by every launch (scripts/stamps.py).  Pass NULL to switch off. */
int as_debug_stamps(as_env_t* env, uint64_t* stamps_dev);

/* Graph-safe stepping (on != 0): every as_step / as_task_step / as_reset_* uses the SAME counter bank,
 * cleared by a one-block kernel at the start of the call, instead of alternating two banks from host
 * state -- so a call captured once in a HIP graph (hipStreamBeginCapture) can be replayed any number
 * of times.  Off (default): two banks, no memset (lowest eager launch count). */
int as_set_graph_safe(as_env_t* env, int32_t on);

/* Device counters of the last step: [0] = any env reset, [1] = sum of curr_target_index, [3] = contacts
 * the constraint budget cut (found by the narrowphase beyond the AS_MAX_CONTACTS / AS_MAX_ROWS - limit
 * rows cap, summed over the step's envs and substeps; PhysX keeps every contact,
 * simulation_cfg.py:110 gpu_max_rigid_contact_count = 2**23).  Valid until the step after next. */
int as_step_counters(as_env_t* env, const int32_t** counters_dev);
/* The same four words [0..3] copied to the host after `stream` (the stream the step ran on) drains;
 * synchronises the stream -- a diagnostic read (tests, bench), never inside a timed step. */
int as_step_counters_host(as_env_t* env, int32_t* out_host, void* stream);
int as_get_curriculum_host(as_env_t* env, int32_t* level_host); /* synchronises the stream */

/* Diagnostic (SURVEY §8d "confirm with an in-repo STREAM-copy kernel"): dst[i] = src[i] for
 * n16 16-byte elements (both device pointers 16-B aligned, non-overlapping), a grid-stride copy
 * with non-temporal loads/stores sized to fill all 256 CUs.  bench.py times it with HIP events to
 * report the achievable HBM bandwidth beside the 8 TB/s spec peak. */
int as_hbm_copy(void* dst, const void* src, int64_t n16, void* stream);

int as_abi_version(void);
const char* as_last_error(void);
/* Provenance: the source digest the library was compiled from (-DAS_BUILD_ID, computed by
 * allsteps_isaaclab_amd/_native.py::source_digest over csrc/ + include/ + the compile flags).  The
 * Python loader refuses a library whose digest differs from the tree's, so a stale or variant build
 * is never run silently ("unversioned" when built without the define). */
const char* as_build_id(void);

#ifdef __cplusplus
}
#endif
#endif
