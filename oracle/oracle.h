/*
 * oracle.h -- CPU restatement of the Allsteps-v0 env step (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity oracle for the HIP step kernels of allsteps_isaaclab_amd.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only as the checker /
 * the reported CPU baseline -- never as the product path.
 *
 * Two halves:
 *   task logic (task.c)  -- a plain-C restatement of the reference task code
 *       source/isaaclab_tasks/isaaclab_tasks/direct/allsteps/allsteps_env.py and the
 *       isaaclab/utils/math.py helpers it calls.  PINNED: tests/test_oracle_golden.py checks it
 *       against golden vectors produced by importing the reference module itself
 *       (tests/golden/gen_golden.py).
 *   physics (physics.c)  -- the articulated-body dynamics that replace PhysX (the reference calls
 *       an external closed binary, isaacsim 4.5 / omni.physx, absent offline).  PARITY UNPINNED
 *       against PhysX: no reference output exists for it.  It is checked by analytic known-answer
 *       tests (free fall, resting contact force = m g, momentum/energy conservation, CRBA vs RNEA
 *       consistency) instead; see DESIGN.md §Parity.
 */
#ifndef ALLSTEPS_ORACLE_H
#define ALLSTEPS_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OR_MAX_LINKS 32
#define OR_MAX_GEOMS 32
#define OR_MAX_STONES 20
#define OR_NDOF_ROOT 6
#define OR_MAX_SELF_PAIRS 256
/* include/allsteps.h AS_MAX_CONTACTS / AS_MAX_ROWS: limits always kept, contacts fill the remaining
 * rows (feet on stones, others, self).  Overridable only for the cap-sizing statistics build
 * (scripts/contact_stats.py, -DOR_STATS), never for parity. */
#ifndef OR_MAX_CONTACTS
#define OR_MAX_CONTACTS 10
#endif
#ifndef OR_MAX_ROWS
#define OR_MAX_ROWS 30
#endif

/* Model tables compiled from walker3d.xml (allsteps_isaaclab_amd/model/walker3d.json). */
typedef struct {
  int32_t num_links;                 /* incl. the floating root (link 0) */
  int32_t num_hinges;                /* = num_links - 1: link i>=1 carries hinge i-1 */
  int32_t parent[OR_MAX_LINKS];
  float offset_pos[OR_MAX_LINKS][3]; /* parent link frame -> this link's pre-joint frame */
  float offset_quat[OR_MAX_LINKS][4];/* (w, x, y, z) */
  float axis[OR_MAX_LINKS][3];       /* hinge axis, link frame */
  float anchor[OR_MAX_LINKS][3];     /* hinge anchor, link frame */
  float mass[OR_MAX_LINKS];
  float com[OR_MAX_LINKS][3];
  float inertia[OR_MAX_LINKS][6];    /* about COM, link frame: xx yy zz xy xz yz */
  float armature[OR_MAX_LINKS];
  float lower[OR_MAX_LINKS];
  float upper[OR_MAX_LINKS];
  int32_t cfg_dof_link[OR_MAX_LINKS];/* cfg/PhysX dof k -> link index */
  float gear[OR_MAX_LINKS];          /* cfg order */
  int32_t num_geoms;
  int32_t geom_link[OR_MAX_GEOMS];
  int32_t geom_type[OR_MAX_GEOMS];   /* 0 sphere, 1 capsule */
  int32_t geom_foot[OR_MAX_GEOMS];   /* -1, 0 right foot, 1 left foot */
  float geom_radius[OR_MAX_GEOMS];
  float geom_p0[OR_MAX_GEOMS][3];
  float geom_p1[OR_MAX_GEOMS][3];
  int32_t torso_link;
  int32_t foot_link[2];              /* right, left */
  int32_t num_priority_geoms;        /* geoms [0, n) emit their stone contacts first */
  int32_t num_self_pairs;            /* self-collision pairs g1 | g2 << 8 (model/__init__.py) */
  int32_t self_pair[OR_MAX_SELF_PAIRS];
} or_model_t;

/* Simulation constants (walker3d.py:21-46, simulation_cfg.py, allsteps_env_cfg.py:62). */
typedef struct {
  float dt;             /* 1/240 */
  int32_t substeps;     /* decimation 4 */
  float gravity;        /* -9.81 (z) */
  float friction;       /* Coulomb mu */
  float margin;         /* speculative contact distance */
  float baumgarte;      /* penetration / limit correction per step */
  float slop;
  float max_depen_vel;  /* max_depenetration_velocity = 10 */
  int32_t pgs_iters;    /* solver_position_iteration_count = 4 */
  float stone_half[3];  /* 0.25, 0.4, 0.1125 */
  float max_joint_vel;
} or_sim_t;

/* Task constants (allsteps_env.py:29-60, allsteps_env_cfg.py:54-234). */
typedef struct {
  int32_t num_steps;            /* 20 */
  float step_radius;            /* 0.25 */
  int32_t stop_frames;          /* 2 */
  float eps;                    /* 1e-4 */
  float alive, energy, action, joint_limit, death, dof_vel_scale, fall_abs;
  float step_dt;                /* 1/60 */
  int32_t max_episode_length;   /* 900 */
  int32_t max_curriculum;       /* 9 */
  int32_t curriculum_threshold; /* 12 */
  float term_curriculum[10];
  float gain_curriculum[10];
  float init_root[3];           /* (0.2, 0, 1.5) */
  float init_q[21];             /* running-start pose, cfg order */
  int32_t right_idx[9], left_idx[9], neg_idx[2];
  float noise_lo, noise_hi, clip_lo, clip_hi;
  int32_t regen_footsteps; /* as_task_t.regen_footsteps: fix of allsteps_env.py:492-500 behind a flag */
} or_task_t;

/* Per-env state, structure of arrays: field-major, env-minor ([field][num_envs]). */
typedef struct {
  int32_t n;
  float *root_pos, *root_quat, *root_lin, *root_ang;   /* [3][n] [4][n] [3][n] [3][n] */
  float *q, *qd;                                       /* [21][n] cfg order */
  float *stones;                                       /* [20][3][n] env-local */
  float *pot, *old_pot;                                /* [n] */
  float *foot_contact;                                 /* [2][n] */
  float *body_pos;                                     /* [3][3][n]: torso, rfoot, lfoot */
  int32_t *idx, *prev, *next, *count, *swing, *ep_len; /* [n] */
  uint32_t *episode;                                   /* [n] reset counter (RNG stream) */
  uint32_t *contact_mask;                              /* [2][n] stone bitmask, last substep */
  int32_t *curriculum;                                 /* [1] */
  uint32_t *contact_mask_hind;                         /* [2][n] sensors 2, 3 (quadruped) or NULL */
  int32_t *feet;                                       /* [8][n] quadruped per-foot targets / counts or NULL */
} or_state_t;

/* include/allsteps.h as_actuator_t / as_quad_task_t, field for field */
typedef struct {
  int32_t mode; /* 0 torque (tau = gain gear a), 1 DC motor on position targets */
  float action_scale;
  float default_q[21];
  float stiffness, damping;
  float saturation_effort, effort_limit, velocity_limit;
} or_actuator_t;
typedef struct {
  int32_t stop_frames;
  float alive, action_cost, death;
  float min_height, up_z_min;
  int32_t max_episode_length;
  float step_dt;
  float stand_height;
  float joint_noise;
  float energy_cost, step_radius, step_reward, step_sigma, target_bonus, bonus_radius, foot_progress;
  float foot_offset_y[4];
} or_quad_task_t;

/* ---- math helpers (isaaclab/utils/math.py) ---- */
void or_euler_xyz_from_quat(const float q[4], float* roll, float* pitch, float* yaw);
void or_quat_rotate_inverse(const float q[4], const float v[3], float out[3]);
void or_quat_rotate(const float q[4], const float v[3], float out[3]);
void or_subtract_frame_transforms(const float t01[3], const float q01[4], const float t02[3], float out[3]);
float or_scale_transform(float x, float lo, float hi);
float or_unscale_transform(float x, float lo, float hi);

/* ---- batched helpers for the golden tests ---- */
void or_math_batch(int n, const float* q, const float* v, float* rpy, float* qri, float* qr);
void or_detmath_eval(int fn, int n, const float* a, const float* b, float* out);
void or_sft_batch(int n, const float* t01, const float* q01, const float* t02, float* out);
void or_footsteps(const or_task_t* task, int n, int level, const float* draws /* [5][n][20] */,
                  float* pos /* [n][20][3] */, float* dphi /* [n][20] */);

/* ---- task logic (post-physics part of DirectRLEnv.step) ----
 * Inputs are the post-physics robot state in `st` (root, q, qd, body_pos) and the per-(foot,
 * stone) contact force matrices fm_r/fm_l ([n][20][3], may be NULL when contact_mask is used).
 * reset_draws: [n][22] (mirror draw, 21 noise draws) for envs that reset, or NULL -> Philox.
 * post_fk: callback giving torso/foot positions for a freshly reset env (NULL -> physics FK). */
typedef void (*or_post_fk_fn)(void* ctx, int env, float body_pos[9]);
void or_task_post_physics(const or_model_t* model, const or_task_t* task, or_state_t* st,
                          const float* actions, const float* fm_r, const float* fm_l,
                          const float* reset_draws, uint64_t seed, or_post_fk_fn post_fk, void* ctx,
                          float* obs, float* rew, uint8_t* term, uint8_t* trunc, int32_t* any_reset);

void or_task_reset_all(const or_model_t* model, const or_task_t* task, or_state_t* st, const float* reset_draws,
                       uint64_t seed, float* obs);
/* ENV:469-567 _reset_idx on the envs with mask[e] != 0 (curriculum gate and second tick for all
 * envs), then _get_observations; an all-zero mask leaves the state unchanged. */
void or_task_reset_mask(const or_model_t* model, const or_task_t* task, or_state_t* st, const uint8_t* mask,
                        const float* reset_draws, uint64_t seed, float* obs);

/* ---- physics ---- */
void or_fk_bodies(const or_model_t* m, const float root_pos[3], const float root_quat[4], const float* q_cfg,
                  float body_pos[9]);
/* physics of env `env` (decimation substeps); returns the contacts the row budget cut over its substeps
 * (contacts found - contacts kept: the kernel's as_step_counters word 3 summed over envs) */
int or_physics_step(const or_model_t* m, const or_sim_t* sim, const or_task_t* task, or_state_t* st,
                    int env, const float* act_clamped);
/* the same with an actuator (act NULL = torque mode): AS_ACT_DC_MOTOR recomputes the joint torques from
 * the position targets default_q + action_scale a in every substep */
int or_physics_step_act(const or_model_t* m, const or_sim_t* sim, const or_task_t* task, const or_actuator_t* act,
                        or_state_t* st, int env, const float* act_clamped);
void or_dc_motor_batch(int n, const float* qt, const float* q, const float* qd, const or_actuator_t* act, float* tau);
/* ---- BASELINE C5 quadruped task (quad.c; the HIP k_quad kernel's restatement) ---- */
void or_quad_post_physics(const or_model_t* m, const or_sim_t* sim, const or_task_t* task, const or_actuator_t* act,
                          const or_quad_task_t* q, or_state_t* st, const float* actions, int reset_all,
                          uint64_t seed, float* obs, float* rew, uint8_t* term, uint8_t* trunc);
/* physics substeps (DC motor) + task epilogue, every env; actions [n][12] */
/* test hook: world position of point pl (link frame) on `link` of env e (include/as_detmath.h as_link_point) */
void or_link_point(const or_model_t* m, const or_state_t* st, int e, int link, const float* pl, float* out);
void or_quad_step(const or_model_t* m, const or_sim_t* sim, const or_task_t* task, const or_actuator_t* act,
                  const or_quad_task_t* q, or_state_t* st, const float* actions, uint64_t seed, float* obs,
                  float* rew, uint8_t* term, uint8_t* trunc, int nthreads);
/* full env step: physics (decimation substeps) + task logic; obs [n][59]; *dropped (if non-null) = the
 * contacts the row budget cut over all envs and substeps */
void or_env_step(const or_model_t* m, const or_sim_t* sim, const or_task_t* task, or_state_t* st,
                 const float* actions, const float* reset_draws, uint64_t seed, float* obs, float* rew,
                 uint8_t* term, uint8_t* trunc, int32_t* any_reset, int64_t* dropped, int nthreads);
/* reset all envs (env.reset()): ep_len=0 + reset pose + tick #2 semantics + obs */
void or_env_reset_all(const or_model_t* m, const or_sim_t* sim, const or_task_t* task, or_state_t* st,
                      const float* reset_draws, uint64_t seed, float* obs);

/* ---- physics internals exposed for known-answer tests ---- */
void or_mass_matrix(const or_model_t* m, const float root_pos[3], const float root_quat[4], const float* q_int,
                    float* H /* [nv][nv] */, float* com0 /* [3] */);
void or_bias_forces(const or_model_t* m, const float root_pos[3], const float root_quat[4], const float* q_int,
                    const float* u /* nv */, float gravity, float* C /* nv */);
void or_philox_uniform(uint64_t seed, uint32_t env, uint32_t episode, int k, float* out);
void or_philox_block(uint64_t seed, uint32_t env, uint32_t episode, uint32_t b, uint32_t tag, float out[4]);
/* every env's course at `level` from the Philox "Ston" stream of (seed, env, episode[e] or 0) */
void or_stones_philox(const or_task_t* task, int n, int level, uint64_t seed, const uint32_t* episode, float* stones);

/* ---- known-answer probe: the constraint set and contact impulses of ONE substep ---- */
typedef struct {
  int32_t nfound;       /* contacts the narrowphase finds (no cap, no early exit) */
  int32_t nself_found;  /* of which robot self-contacts */
  int32_t ncap;         /* contact budget left by the limit rows: min(MAX_CONTACTS, (MAX_ROWS - nlim) / 3) */
  int32_t nlim;         /* joint-limit rows (all kept) */
  int32_t ncontact;     /* contacts kept */
  int32_t link[OR_MAX_CONTACTS], link2[OR_MAX_CONTACTS], stone[OR_MAX_CONTACTS], foot[OR_MAX_CONTACTS];
  float sep[OR_MAX_CONTACTS], nrm[OR_MAX_CONTACTS][3];
  float lam_n[OR_MAX_CONTACTS]; /* normal impulse after the PGS sweeps (force = lam_n / dt) */
  uint32_t mask[2];             /* contact-sensor bits of this substep */
  /* over ALL substeps of the env step: stone contact impulses summed per stone and in total (the
   * environment's push on the robot; self-contacts are internal and excluded) */
  float stone_impulse[OR_MAX_STONES][3];
  float net_impulse[3];
  int32_t recorded;             /* internal: the first substep has been recorded */
} or_probe_t;
/* Run one env step's physics (all substeps) of env e (act_clamped in cfg order) on a copy of its
 * state and report its first substep plus the impulse sums; `st` is not modified. */
void or_probe_substep(const or_model_t* m, const or_sim_t* sim, const or_task_t* task, const or_state_t* st, int e,
                      const float* act_clamped, or_probe_t* out);

#ifdef OR_STATS
/* per-substep histograms (single-threaded runs): [0] contacts the narrowphase found (before the cap),
 * [1] active joint-limit rows, [2] contacts kept, [3] self-contacts found */
extern long long or_stats_hist[6][256]; /* [4]: self-contacts per pair index, [5]: pairs past the sphere filter */
#endif

#ifdef __cplusplus
}
#endif
#endif
