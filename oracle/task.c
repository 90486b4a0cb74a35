/*
 * task.c -- CPU restatement of the Allsteps-v0 task logic (TEST INFRASTRUCTURE; see oracle.h).
 *
 * Every function cites the reference it restates.  Paths are relative to /root/reference/source:
 *   ENV  = isaaclab_tasks/isaaclab_tasks/direct/allsteps/allsteps_env.py
 *   MATH = isaaclab/isaaclab/utils/math.py
 *   DRL  = isaaclab/isaaclab/envs/direct_rl_env.py
 * Arithmetic is float32 in the reference's operation order so that integer / boolean outputs are
 * exact and floats agree to a few ulp with the golden vectors.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"
#include "../include/as_detmath.h"

#define PI_F 3.14159265358979323846f

/* ------------------------------------------------------------------ math helpers (MATH) */

/* MATH:413-444 euler_xyz_from_quat: atan2/asin, then "% 2pi" (torch.remainder).  The transcendentals
 * are the shared deterministic forms of include/as_detmath.h (the HIP kernel computes the same bits;
 * within a few ulp of torch's, tests/test_oracle_golden.py); the remainder is the identity + 2 pi
 * fold on their [-pi, pi] range. */
void or_euler_xyz_from_quat(const float q[4], float* roll, float* pitch, float* yaw) {
  float qw = q[0], qx = q[1], qy = q[2], qz = q[3];
  float sin_roll = 2.0f * (qw * qx + qy * qz);
  float cos_roll = 1.0f - 2.0f * (qx * qx + qy * qy);
  float r = as_atan2f(sin_roll, cos_roll);
  float sin_pitch = 2.0f * (qw * qy - qz * qx);
  float p;
  if (fabsf(sin_pitch) >= 1.0f) /* copysign(pi/2, sin_pitch): |mag| * sign(x)  (MATH:121-140) */
    p = (float)(3.14159265358979323846 / 2.0) * (sin_pitch > 0.0f ? 1.0f : -1.0f);
  else
    p = as_asinf(sin_pitch);
  float sin_yaw = 2.0f * (qw * qz + qx * qy);
  float cos_yaw = 1.0f - 2.0f * (qy * qy + qz * qz);
  float y = as_atan2f(sin_yaw, cos_yaw);
  *roll = as_rem2pi(r);
  *pitch = as_rem2pi(p);
  *yaw = as_rem2pi(y);
}

static void cross3(const float a[3], const float b[3], float o[3]) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}

/* MATH:605-625 quat_rotate_inverse: a - b + c with a = v(2w^2-1), b = 2w (qv x v), c = 2 qv (qv.v) */
void or_quat_rotate_inverse(const float q[4], const float v[3], float out[3]) {
  float w = q[0];
  const float* qv = q + 1;
  float s = 2.0f * (w * w) - 1.0f;
  float cr[3];
  cross3(qv, v, cr);
  float d = qv[0] * v[0] + qv[1] * v[1] + qv[2] * v[2];
  for (int i = 0; i < 3; ++i) {
    float a = v[i] * s;
    float b = cr[i] * w * 2.0f;
    float c = qv[i] * d * 2.0f;
    out[i] = a - b + c;
  }
}

/* MATH:582-602 quat_rotate */
void or_quat_rotate(const float q[4], const float v[3], float out[3]) {
  float w = q[0];
  const float* qv = q + 1;
  float s = 2.0f * (w * w) - 1.0f;
  float cr[3];
  cross3(qv, v, cr);
  float d = qv[0] * v[0] + qv[1] * v[1] + qv[2] * v[2];
  for (int i = 0; i < 3; ++i) out[i] = v[i] * s + cr[i] * w * 2.0f + qv[i] * d * 2.0f;
}

/* MATH:785-818 subtract_frame_transforms (translation part):
 * q10 = quat_inv(q01) = normalize(conjugate(q01)) (MATH:224-249, 82-93), t12 = quat_apply(q10, t02-t01)
 * quat_apply (MATH:546-565): t = 2 xyz x v; v + w t + xyz x t */
void or_subtract_frame_transforms(const float t01[3], const float q01[4], const float t02[3], float out[3]) {
  float c[4] = {q01[0], -q01[1], -q01[2], -q01[3]};
  float nrm = sqrtf(c[0] * c[0] + c[1] * c[1] + c[2] * c[2] + c[3] * c[3]);
  if (nrm < 1e-9f) nrm = 1e-9f;
  float q10[4] = {c[0] / nrm, c[1] / nrm, c[2] / nrm, c[3] / nrm};
  float v[3] = {t02[0] - t01[0], t02[1] - t01[1], t02[2] - t01[2]};
  float t[3], t2[3];
  cross3(q10 + 1, v, t);
  t[0] *= 2.0f; t[1] *= 2.0f; t[2] *= 2.0f;
  cross3(q10 + 1, t, t2);
  for (int i = 0; i < 3; ++i) out[i] = v[i] + q10[0] * t[i] + t2[i];
}

/* MATH:22-40 */
float or_scale_transform(float x, float lo, float hi) {
  float offset = (lo + hi) * 0.5f;
  return 2.0f * (x - offset) / (hi - lo);
}

/* MATH:43-61 */
float or_unscale_transform(float x, float lo, float hi) {
  float offset = (lo + hi) * 0.5f;
  return x * (hi - lo) * 0.5f + offset;
}

void or_math_batch(int n, const float* q, const float* v, float* rpy, float* qri, float* qr) {
  for (int i = 0; i < n; ++i) {
    or_euler_xyz_from_quat(q + 4 * i, rpy + 3 * i, rpy + 3 * i + 1, rpy + 3 * i + 2);
    or_quat_rotate_inverse(q + 4 * i, v + 3 * i, qri + 3 * i);
    or_quat_rotate(q + 4 * i, v + 3 * i, qr + 3 * i);
  }
}

void or_sft_batch(int n, const float* t01, const float* q01, const float* t02, float* out) {
  for (int i = 0; i < n; ++i) or_subtract_frame_transforms(t01 + 3 * i, q01 + 4 * i, t02 + 3 * i, out + 3 * i);
}

/* ------------------------------------------------------------------ footsteps (ENV:125-174) */

/* torch.lerp CPU formula (ATen Lerp.h): weight < 0.5 ? a + w (b-a) : b - (b-a)(1-w) */
static float lerpf_t(float a, float b, float w) {
  return (fabsf(w) < 0.5f) ? a + w * (b - a) : b - (b - a) * (1.0f - w);
}

/* torch.linspace(start, end, steps) float32 (ATen RangeFactories): step = (end-start)/(steps-1);
 * i < steps/2 ? start + i*step : end - (steps-1-i)*step */
static float linspace_at(float start, float end, int steps, int i) {
  float step = (end - start) / (float)(steps - 1);
  int halfway = steps / 2;
  return (i < halfway) ? start + step * (float)i : end - step * (float)(steps - i - 1);
}

void or_footsteps(const or_task_t* task, int n, int level, const float* draws, float* pos, float* dphi_out) {
  const int N = task->num_steps;
  const int maxc = task->max_curriculum;
  int c = level < maxc ? level : maxc;
  float ratio = (float)c / (float)maxc;                       /* ENV:127 */
  float dist_lo = 0.75f, dist_hi = linspace_at(0.75f, 0.9f, maxc + 1, c); /* ENV:129-130 */
  const float d2r = (float)(3.14159265358979323846 / 180.0);
  float yaw_lo = (-20.0f * ratio) * d2r, yaw_hi = (20.0f * ratio) * d2r;  /* ENV:131 */
  float p_lo = (-30.0f * ratio) * d2r + (float)(3.14159265358979323846 / 2.0);
  float p_hi = (30.0f * ratio) * d2r + (float)(3.14159265358979323846 / 2.0);
  const float half_pi = (float)(3.14159265358979323846 / 2.0);
  for (int e = 0; e < n; ++e) {
    float x = 0.f, y = 0.f, z = 0.f, phi = 0.f;
    for (int k = 0; k < N; ++k) {
      float wdr = draws[(0 * n + e) * N + k];
      float wph = draws[(1 * n + e) * N + k];
      float wth = draws[(2 * n + e) * N + k];
      float dr = lerpf_t(dist_lo, dist_hi, wdr);                  /* ENV:137 */
      float dph = lerpf_t(yaw_lo, yaw_hi, wph);                   /* ENV:138 */
      float dth = lerpf_t(p_lo, p_hi, wth);                       /* ENV:139 */
      if (k == 0) { dr = 0.f; dph = 0.f; dth = half_pi; }         /* ENV:144-146 */
      if (k == 1 || k == 2) { dr = 0.75f; dph = 0.f; dth = half_pi; } /* ENV:148-150 */
      phi += dph;                                                 /* ENV:155 cumsum */
      float st_, ct_, sp, cp;                                     /* the kernel's shared sin / cos */
      as_sincosf(dth, &st_, &ct_);
      as_sincosf(phi, &sp, &cp);
      float dx = dr * st_ * cp;                                   /* ENV:157-159 */
      float dy = dr * st_ * sp;
      float dz = dr * ct_;
      x += dx; y += dy; z += dz;                                  /* ENV:165-167 */
      pos[(e * N + k) * 3 + 0] = x;
      pos[(e * N + k) * 3 + 1] = y;
      pos[(e * N + k) * 3 + 2] = z;
      dphi_out[e * N + k] = phi;
    }
  }
}

/* ------------------------------------------------------------------ Philox4x32-10 reset draws */

static void philox4x32_10(uint32_t ctr[4], const uint32_t key_in[2]) {
  uint32_t k0 = key_in[0], k1 = key_in[1];
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * ctr[0];
    uint64_t p1 = (uint64_t)0xCD9E8D57u * ctr[2];
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ ctr[1] ^ k0, n1 = lo1, n2 = hi0 ^ ctr[3] ^ k1, n3 = lo0;
    ctr[0] = n0; ctr[1] = n1; ctr[2] = n2; ctr[3] = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

/* 4 uniforms of block b of the (env, episode) stream with counter tag `tag` (the kernels' philox_block) */
void or_philox_block(uint64_t seed, uint32_t env, uint32_t episode, uint32_t b, uint32_t tag, float out[4]) {
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t ctr[4] = {env, episode, b, tag};
  philox4x32_10(ctr, key);
  for (int j = 0; j < 4; ++j) out[j] = (float)(ctr[j] >> 8) * (1.0f / 16777216.0f);
}

/* draws k = 0..21 of env `env`'s `episode`-th reset: U[0,1) with 24-bit mantissa */
void or_philox_uniform(uint64_t seed, uint32_t env, uint32_t episode, int k, float* out) {
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  for (int b = 0; b * 4 < k; ++b) {
    uint32_t ctr[4] = {env, episode, (uint32_t)b, 0x416c6c73u /* "Alls" */};
    philox4x32_10(ctr, key);
    for (int j = 0; j < 4 && b * 4 + j < k; ++j) out[b * 4 + j] = (float)(ctr[j] >> 8) * (1.0f / 16777216.0f);
  }
}

/* One env's course at `level` from Philox draws keyed (seed, env, episode, block k, "Ston"): the
 * kernel's k_stones / k_obs regeneration stream (ENV:125-174 formulas, as or_footsteps). */
static void stones_philox(const or_task_t* task, int n, int e, int level, uint64_t seed, uint32_t env,
                          uint32_t episode, float* stones /* [60][n] */) {
  const int N = task->num_steps, maxc = task->max_curriculum;
  const int c = level < maxc ? level : maxc;
  const float ratio = (float)c / (float)maxc;
  const float dist_hi = linspace_at(0.75f, 0.9f, maxc + 1, c);
  const float d2r = (float)(3.14159265358979323846 / 180.0);
  const float yaw_lo = (-20.0f * ratio) * d2r, yaw_hi = (20.0f * ratio) * d2r;
  const float half_pi = (float)(3.14159265358979323846 / 2.0);
  const float p_lo = (-30.0f * ratio) * d2r + half_pi, p_hi = (30.0f * ratio) * d2r + half_pi;
  const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  float x = 0.f, y = 0.f, z = 0.f, phi = 0.f;
  for (int k = 0; k < N; ++k) {
    uint32_t ctr[4] = {env, episode, (uint32_t)k, 0x53746f6eu /* "Ston" */};
    philox4x32_10(ctr, key);
    float w[3];
    for (int j = 0; j < 3; ++j) w[j] = (float)(ctr[j] >> 8) * (1.0f / 16777216.0f);
    float dr = lerpf_t(0.75f, dist_hi, w[0]), dph = lerpf_t(yaw_lo, yaw_hi, w[1]), dth = lerpf_t(p_lo, p_hi, w[2]);
    if (k == 0) { dr = 0.f; dph = 0.f; dth = half_pi; }
    if (k == 1 || k == 2) { dr = 0.75f; dph = 0.f; dth = half_pi; }
    phi += dph;
    float st_, ct_, sp, cp;
    as_sincosf(dth, &st_, &ct_);
    as_sincosf(phi, &sp, &cp);
    x += dr * st_ * cp;
    y += dr * st_ * sp;
    z += dr * ct_;
    stones[(size_t)(3 * k + 0) * n + e] = x;
    stones[(size_t)(3 * k + 1) * n + e] = y;
    stones[(size_t)(3 * k + 2) * n + e] = z;
  }
}

void or_stones_philox(const or_task_t* task, int n, int level, uint64_t seed, const uint32_t* episode,
                      float* stones) {
  for (int e = 0; e < n; ++e) stones_philox(task, n, e, level, seed, (uint32_t)e, episode ? episode[e] : 0u, stones);
}

/* ------------------------------------------------------------------ task logic */

#define F(arr, f, n, e) (arr)[(size_t)(f) * (n) + (e)]

static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

typedef struct {
  float h, roll, pitch, vb[3], qs[21], targets_b[9], body_dist_xy, dist_f[2];
  int reached;
} useful_t;

static float norm3(float a, float b, float c) { return sqrtf(a * a + b * b + c * c); }

/* ENV:418-457 _calculate_foot_state for one env.  contact[f] comes from the force matrix entry of
 * the current target stone (norm > EPSILON). */
static void foot_state(const or_task_t* task, or_state_t* st, int e, const float* fm_r, const float* fm_l,
                       useful_t* u) {
  const int n = st->n, N = task->num_steps;
  int idx = st->idx[e];
  float cf[2];
  if (fm_r) {
    const float* a = fm_r + ((size_t)e * N + idx) * 3;
    const float* b = fm_l + ((size_t)e * N + idx) * 3;
    cf[0] = norm3(a[0], a[1], a[2]) > task->eps ? 1.0f : 0.0f;  /* ENV:421-425 */
    cf[1] = norm3(b[0], b[1], b[2]) > task->eps ? 1.0f : 0.0f;
  } else {
    cf[0] = ((F(st->contact_mask, 0, n, e) >> idx) & 1u) ? 1.0f : 0.0f;
    cf[1] = ((F(st->contact_mask, 1, n, e) >> idx) & 1u) ? 1.0f : 0.0f;
  }
  F(st->foot_contact, 0, n, e) = cf[0];
  F(st->foot_contact, 1, n, e) = cf[1];
  float tx = F(st->stones, idx * 3 + 0, n, e), ty = F(st->stones, idx * 3 + 1, n, e); /* ENV:429 */
  for (int f = 0; f < 2; ++f) {                                                         /* ENV:430-431 */
    float dx = F(st->body_pos, 3 + 3 * f + 0, n, e) - tx;
    float dy = F(st->body_pos, 3 + 3 * f + 1, n, e) - ty;
    u->dist_f[f] = sqrtf(dx * dx + dy * dy);
  }
  int sw = st->swing[e];
  u->reached = (cf[sw] > 0.0f) && (u->dist_f[sw] < task->step_radius); /* ENV:433 */
  if (u->reached) st->count[e] += 1;                                    /* ENV:435 */
  if (st->count[e] >= task->stop_frames) {                              /* ENV:437-457 */
    st->swing[e] = sw ^ 1;
    int ni = clampi(idx + 1, 0, N - 1);
    st->idx[e] = ni;
    st->prev[e] = clampi(ni - 1, 0, N - 1);
    st->next[e] = clampi(ni + 1, 0, N - 1);
    st->count[e] = 0;
  }
}

/* ENV:276-324 _compute_useful_values for one env (incl. foot-state tick, targets, potentials). */
static void useful_values(const or_model_t* model, const or_task_t* task, or_state_t* st, int e,
                          const float* fm_r, const float* fm_l, useful_t* u, int tick) {
  const int n = st->n;
  float rz = F(st->body_pos, 3 + 2, n, e), lz = F(st->body_pos, 6 + 2, n, e);
  float lower = lz < rz ? lz : rz;                                      /* ENV:281 minimum(left, right) */
  u->h = F(st->body_pos, 2, n, e) - lower;                              /* ENV:283 */
  float q[4] = {F(st->root_quat, 0, n, e), F(st->root_quat, 1, n, e), F(st->root_quat, 2, n, e),
                F(st->root_quat, 3, n, e)};
  float yaw;
  or_euler_xyz_from_quat(q, &u->roll, &u->pitch, &yaw);                 /* ENV:285 */
  for (int k = 0; k < 21; ++k) {                                        /* ENV:287-291 */
    int li = model->cfg_dof_link[k];
    u->qs[k] = or_scale_transform(F(st->q, k, n, e), model->lower[li], model->upper[li]);
  }
  float v[3] = {F(st->root_lin, 0, n, e), F(st->root_lin, 1, n, e), F(st->root_lin, 2, n, e)};
  or_quat_rotate_inverse(q, v, u->vb);                                  /* ENV:293 */
  if (tick) foot_state(task, st, e, fm_r, fm_l, u);                     /* ENV:298 */
  const int N = task->num_steps;
  int tix[3] = {st->prev[e], st->idx[e], st->next[e]};                  /* ENV:459-467 */
  float rp[3] = {F(st->root_pos, 0, n, e), F(st->root_pos, 1, n, e), F(st->root_pos, 2, n, e)};
  float tw[3][3];
  for (int k = 0; k < 3; ++k) {
    for (int c = 0; c < 3; ++c) tw[k][c] = F(st->stones, tix[k] * 3 + c, n, e);
    or_subtract_frame_transforms(rp, q, tw[k], u->targets_b + 3 * k);   /* ENV:302-316 */
  }
  (void)N;
  float dx = tw[2][0] - rp[0], dy = tw[2][1] - rp[1];                   /* ENV:407-416 */
  u->body_dist_xy = sqrtf(dx * dx + dy * dy);
  if (!tick) return;
  st->old_pot[e] = st->pot[e];
  st->pot[e] = -(u->body_dist_xy) / task->step_dt;
}

/* ENV:276-324 _compute_useful_values (foot-state tick and potentials included). */
static void compute_useful(const or_model_t* model, const or_task_t* task, or_state_t* st, int e,
                           const float* fm_r, const float* fm_l, useful_t* u) {
  useful_values(model, task, st, e, fm_r, fm_l, u, 1);
}

/* The observation inputs of the current state without a foot-state tick (no _compute_useful_values
 * call: an empty reset set). */
static void useful_no_tick(const or_model_t* model, const or_task_t* task, or_state_t* st, int e, useful_t* u) {
  useful_values(model, task, st, e, NULL, NULL, u, 0);
}

/* ENV:326-345 _get_observations for one env. */
static void write_obs(const or_task_t* task, const or_state_t* st, int e, const useful_t* u, float* o) {
  const int n = st->n;
  o[0] = u->h;
  o[1] = u->roll;
  o[2] = u->pitch;
  for (int i = 0; i < 3; ++i) o[3 + i] = u->vb[i];
  for (int k = 0; k < 21; ++k) o[6 + k] = u->qs[k];
  for (int k = 0; k < 21; ++k) {
    float x = F(st->qd, k, n, e) * task->dof_vel_scale;
    o[27 + k] = x < -5.0f ? -5.0f : (x > 5.0f ? 5.0f : x);
  }
  o[48] = F(st->foot_contact, 0, n, e);
  o[49] = F(st->foot_contact, 1, n, e);
  for (int i = 0; i < 9; ++i) o[50 + i] = u->targets_b[i];
}

/* Sum of n <= 32 per-dof terms (lane k = cfg dof k) as the HIP kernel forms it (k_step half_sum: DPP
 * butterflies = balanced pairwise trees over lanes 0..15 and 16..31, then row 0 + row 1; lanes past n
 * add +0).  torch sums in its own reduction order; the golden vectors absorb the difference. */
static float half_tree32(const float* v, int n) {
  float a[32] = {0.0f};
  for (int i = 0; i < n; ++i) a[i] = v[i];
  for (int w = 1; w < 16; w *= 2)
    for (int i = 0; i < 32; i += 2 * w) a[i] = a[i] + a[i + w];
  return a[0] + a[16];
}

/* ENV:347-394 _get_rewards for one env. */
static float reward(const or_task_t* task, const or_state_t* st, int e, const useful_t* u, const float* a,
                    int terminated) {
  const int n = st->n;
  float alive = 1.0f * task->alive;
  float progress = st->pot[e] - st->old_pot[e];
  int roll_v = (u->roll > 0.4f) || (u->roll < -0.4f);
  int pitch_v = (u->pitch > 0.4f) || (u->pitch < -0.2f);
  float roll_cost = roll_v ? fabsf(u->roll) : 0.0f;
  float pitch_cost = pitch_v ? fabsf(u->pitch) : 0.0f;
  float lv[3] = {F(st->root_lin, 0, n, e), F(st->root_lin, 1, n, e), F(st->root_lin, 2, n, e)};
  float speed = norm3(lv[0], lv[1], lv[2]);
  float speed_cost = speed > 1.6f ? speed - 1.6f : 0.0f;
  float sq[21], ea[21];
  for (int k = 0; k < 21; ++k) {
    sq[k] = a[k] * a[k];
    ea[k] = fabsf(F(st->qd, k, n, e) * a[k]);
  }
  const float ss = half_tree32(sq, 21), en = half_tree32(ea, 21); /* the kernel's lane tree */
  float action_cost = task->action * sqrtf(ss);
  float energy_cost = task->energy * en;
  int nlim = 0;
  for (int k = 0; k < 21; ++k) nlim += fabsf(u->qs[k]) > 0.99f;
  float limit_cost = (float)nlim * task->joint_limit;
  int cond = u->reached && (st->count[e] == 1) && (st->idx[e] < task->num_steps - 1);
  float dist = u->dist_f[st->swing[e]];
  float step_rew = cond ? 50.0f * as_expf(-dist / 0.25f) : 0.0f;     /* shared deterministic exp */
  int bonus_cond = (st->idx[e] == task->num_steps - 1) && (u->body_dist_xy < 0.15f);
  float bonus = bonus_cond ? 10.0f : 0.0f;
  float total = alive + progress;
  total = total - roll_cost;
  total = total - pitch_cost;
  total = total - speed_cost;
  total = total - energy_cost;
  total = total - action_cost;
  total = total - limit_cost;
  total = total + step_rew;
  total = total + bonus;
  return terminated ? task->death * 1.0f : total;
}

/* ENV:469-567 _reset_idx body for one env (after the curriculum check), draws[0] = mirror draw,
 * draws[1..21] = noise draws.  Writes root/joint state; the body positions are refreshed by the
 * caller (FK), then the caller runs the second _compute_useful_values over all envs. */
static void reset_env(const or_model_t* model, const or_task_t* task, or_state_t* st, int e, const float* draws) {
  const int n = st->n;
  st->ep_len[e] = 0;                                                    /* DRL:584 */
  st->old_pot[e] = 0.0f;                                                /* ENV:487-494 */
  st->pot[e] = 0.0f;
  st->count[e] = 0;
  st->swing[e] = 0;
  st->idx[e] = 1;
  st->prev[e] = 0;
  st->next[e] = 2;
  float jp[21], jv[21];
  for (int k = 0; k < 21; ++k) { jp[k] = task->init_q[k]; jv[k] = 0.0f; } /* ENV:505-513 */
  float rootq[4] = {1.0f, 0.0f, 0.0f, 0.0f};
  int mirror = draws[0] > 0.5f;                                         /* ENV:518 */
  if (mirror) {                                                          /* ENV:522-538 */
    float mp[21], mv[21];
    memcpy(mp, jp, sizeof mp);
    memcpy(mv, jv, sizeof mv);
    for (int i = 0; i < 9; ++i) {
      mp[task->right_idx[i]] = jp[task->left_idx[i]];
      mp[task->left_idx[i]] = jp[task->right_idx[i]];
      mv[task->right_idx[i]] = jv[task->left_idx[i]];
      mv[task->left_idx[i]] = jv[task->right_idx[i]];
    }
    for (int i = 0; i < 2; ++i) { mp[task->neg_idx[i]] *= -1.0f; mv[task->neg_idx[i]] *= -1.0f; }
    memcpy(jp, mp, sizeof mp);
    memcpy(jv, mv, sizeof mv);
    rootq[1] *= -1.0f; rootq[2] *= -1.0f; rootq[3] *= -1.0f;
    st->swing[e] ^= 1;
  }
  for (int k = 0; k < 21; ++k) {                                        /* ENV:542-560 */
    int li = model->cfg_dof_link[k];
    float x = jp[k] + (draws[1 + k] * (task->noise_hi - task->noise_lo) + task->noise_lo);
    float s = or_scale_transform(x, model->lower[li], model->upper[li]);
    s = s < task->clip_lo ? task->clip_lo : (s > task->clip_hi ? task->clip_hi : s);
    F(st->q, k, n, e) = or_unscale_transform(s, model->lower[li], model->upper[li]);
    F(st->qd, k, n, e) = jv[k];
  }
  for (int c = 0; c < 3; ++c) {                                         /* ENV:514-515, 563-564 */
    F(st->root_pos, c, n, e) = task->init_root[c];
    F(st->root_lin, c, n, e) = 0.0f;
    F(st->root_ang, c, n, e) = 0.0f;
  }
  for (int c = 0; c < 4; ++c) F(st->root_quat, c, n, e) = rootq[c];
  st->episode[e] += 1u;
}

/* ENV:469-567 _reset_idx(ids) + ENV:567 second _compute_useful_values over ALL envs. */
static void reset_and_tick2(const or_model_t* model, const or_task_t* task, or_state_t* st, const uint8_t* done,
                            long long idx_sum, const float* reset_draws, uint64_t seed, or_post_fk_fn post_fk,
                            void* ctx, const float* fm_r, const float* fm_l, useful_t* u) {
  const int n = st->n;
  /* ENV:471-479 curriculum: mean over ALL envs of the current target index > 12 */
  if ((float)idx_sum / (float)n > (float)task->curriculum_threshold) {
    int c = st->curriculum[0] + 1;
    st->curriculum[0] = c > task->max_curriculum ? task->max_curriculum : c;
  }
  for (int e = 0; e < n; ++e) {
    if (!done[e]) continue;
    float d[22];
    if (reset_draws)
      memcpy(d, reset_draws + (size_t)e * 22, sizeof d);
    else
      or_philox_uniform(seed, (uint32_t)e, st->episode[e], 22, d);
    /* ENV:497-500 as intended (flag): the over-half test on the PRE-reset target index */
    const int regen = task->regen_footsteps && st->idx[e] > task->num_steps / 2;
    reset_env(model, task, st, e, d);
    /* stones 0..2 are the same for every course, so the reset observation / potentials (targets
     * 0..2 after a reset) do not change; the new course is keyed by the new episode */
    if (regen) stones_philox(task, n, e, st->curriculum[0], seed, (uint32_t)e, st->episode[e], st->stones);
    float bp[9];
    if (post_fk) {
      post_fk(ctx, e, bp);
    } else {
      float rp[3], rq[4], qc[21];
      for (int c = 0; c < 3; ++c) rp[c] = F(st->root_pos, c, n, e);
      for (int c = 0; c < 4; ++c) rq[c] = F(st->root_quat, c, n, e);
      for (int k = 0; k < 21; ++k) qc[k] = F(st->q, k, n, e);
      or_fk_bodies(model, rp, rq, qc, bp);
    }
    for (int c = 0; c < 9; ++c) F(st->body_pos, c, n, e) = bp[c];
  }
  /* stale contacts: the sensor re-reads the last substep's matrix (contact_sensor.py:142-161) */
  for (int e = 0; e < n; ++e) compute_useful(model, task, st, e, fm_r, fm_l, &u[e]);
}

void or_task_reset_all(const or_model_t* model, const or_task_t* task, or_state_t* st, const float* reset_draws,
                       uint64_t seed, float* obs) {
  /* DRL:256-294 reset(): _reset_idx(all envs) -> write_data_to_sim/forward -> _get_observations */
  const int n = st->n;
  useful_t* u = (useful_t*)malloc(sizeof(useful_t) * (size_t)n);
  uint8_t* done = (uint8_t*)calloc((size_t)n + 1, 1);
  long long idx_sum = 0;
  for (int e = 0; e < n; ++e) { done[e] = 1; idx_sum += st->idx[e]; }
  reset_and_tick2(model, task, st, done, idx_sum, reset_draws, seed, NULL, NULL, NULL, NULL, u);
  for (int e = 0; e < n; ++e) write_obs(task, st, e, &u[e], obs + (size_t)e * 59);
  free(u);
  free(done);
}

void or_task_reset_mask(const or_model_t* model, const or_task_t* task, or_state_t* st, const uint8_t* mask,
                        const float* reset_draws, uint64_t seed, float* obs) {
  /* ENV:469-567 _reset_idx(env_ids) then ENV:326-345 _get_observations; an empty id set is a no-op
   * (DRL:361 only calls _reset_idx when some env is done) */
  const int n = st->n;
  int any = 0;
  long long idx_sum = 0;
  for (int e = 0; e < n; ++e) { any |= mask[e] != 0; idx_sum += st->idx[e]; }
  useful_t* u = (useful_t*)malloc(sizeof(useful_t) * (size_t)n);
  if (any) {
    reset_and_tick2(model, task, st, mask, idx_sum, reset_draws, seed, NULL, NULL, NULL, NULL, u);
  } else {
    /* no reset: the observation of the current state, no foot-state tick */
    for (int e = 0; e < n; ++e) useful_no_tick(model, task, st, e, &u[e]);
  }
  for (int e = 0; e < n; ++e) write_obs(task, st, e, &u[e], obs + (size_t)e * 59);
  free(u);
}

void or_task_post_physics(const or_model_t* model, const or_task_t* task, or_state_t* st, const float* actions,
                          const float* fm_r, const float* fm_l, const float* reset_draws, uint64_t seed,
                          or_post_fk_fn post_fk, void* ctx, float* obs, float* rew, uint8_t* term,
                          uint8_t* trunc, int32_t* any_reset) {
  const int n = st->n;
  useful_t* u = (useful_t*)malloc(sizeof(useful_t) * (size_t)n);
  uint8_t* done = (uint8_t*)calloc((size_t)n + 1, 1);
  float a[21];
  int nreset = 0;
  long long idx_sum = 0;
  const int cur = st->curriculum[0];
  for (int e = 0; e < n; ++e) {
    for (int k = 0; k < 21; ++k) {                                      /* ENV:267-268 clamp */
      float x = actions[(size_t)e * 21 + k];
      a[k] = x < -1.0f ? -1.0f : (x > 1.0f ? 1.0f : x);
    }
    st->ep_len[e] += 1;                                                 /* DRL:351 */
    compute_useful(model, task, st, e, fm_r, fm_l, &u[e]);              /* ENV:396-397 tick #1 */
    int time_out = st->ep_len[e] >= task->max_episode_length - 1;       /* ENV:399 */
    int fell = u[e].h < task->term_curriculum[cur];                     /* ENV:401 */
    float lv0 = F(st->root_lin, 0, n, e), lv1 = F(st->root_lin, 1, n, e), lv2 = F(st->root_lin, 2, n, e);
    int so_fast = norm3(lv0, lv1, lv2) > 5.0f;                          /* ENV:402 */
    int died = F(st->root_pos, 2, n, e) < task->fall_abs;               /* ENV:403 */
    term[e] = (uint8_t)(fell || so_fast || died);
    trunc[e] = (uint8_t)time_out;
    rew[e] = reward(task, st, e, &u[e], a, term[e]);                    /* DRL:355 */
    done[e] = term[e] | trunc[e];
    nreset += done[e];
    idx_sum += st->idx[e];
  }
  *any_reset = nreset > 0;
  if (nreset > 0)                                                       /* DRL:359-364 */
    reset_and_tick2(model, task, st, done, idx_sum, reset_draws, seed, post_fk, ctx, fm_r, fm_l, u);
  for (int e = 0; e < n; ++e) write_obs(task, st, e, &u[e], obs + (size_t)e * 59); /* DRL:373 */
  free(u);
  free(done);
}

/* ------------------------------------------------------------------ shared transcendentals (tests) */

/* Evaluate one of include/as_detmath.h's deterministic functions on n inputs (tests/test_detmath.py
 * measures their accuracy): fn 0 atan2(a, b), 1 asin(a), 2 exp(a), 3 sin(a), 4 cos(a), 5 rem2pi(a). */
void or_detmath_eval(int fn, int n, const float* a, const float* b, float* out) {
  for (int i = 0; i < n; ++i) {
    float s, c;
    switch (fn) {
      case 0: out[i] = as_atan2f(a[i], b[i]); break;
      case 1: out[i] = as_asinf(a[i]); break;
      case 2: out[i] = as_expf(a[i]); break;
      case 3: as_sincosf(a[i], &s, &c); out[i] = s; break;
      case 4: as_sincosf(a[i], &s, &c); out[i] = c; break;
      default: out[i] = as_rem2pi(a[i]); break;
    }
  }
}
