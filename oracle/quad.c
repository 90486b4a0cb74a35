/*
 * quad.c -- CPU restatement of the BASELINE C5 quadruped task (TEST INFRASTRUCTURE; see oracle.h).
 *
 * The serial form of the HIP kernel k_quad (allsteps_isaaclab_amd/csrc/allsteps_kernels.hip) and of
 * include/allsteps.h as_quad_task_t.  The reference has no quadruped stepping-stone task (its ANYmal-C
 * task, isaaclab_tasks/direct/anymal_c/anymal_c_env.py, is flat-ground velocity tracking): the task is
 * authored here from the Allsteps task's pieces (target stones, potentials, allsteps_env.py:347-457)
 * and the ANYmal task's actuation / observation terms (anymal_c_env.py:73-110): the ALLSTEPS reward
 * terms (step hit, progress, energy, alive, target bonus; allsteps_env.py:347-394) and the target machine
 * (:418-457) run per foot (each foot its own target stone and reach count).  PARITY UNPINNED
 * against any reference output; the HIP kernel is checked against this file bit for bit.
 */
#include <math.h>
#include <stddef.h>

#include "oracle.h"
#include "../include/as_detmath.h"

#define F(arr, f, n, e) (arr)[(size_t)(f) * (n) + (e)]
#define QUAD_TAG 0x51756164u /* "Quad" */
#define QUAD_OBS 64

static int imin(int a, int b) { return a < b ? a : b; }

/* foot f's tip (its sensor geom's capsule end p1) in env e, root pose (rp, rq) */
static void quad_tip(const or_model_t* m, const or_state_t* st, int e, int f, const float* rp, const float* rq,
                     float* tip) {
  int g = 0;
  for (int j = 0; j < m->num_geoms; ++j)
    if (m->geom_foot[j] == f) { g = j; break; }
  int32_t link_dof[OR_MAX_LINKS];
  as_link_dof_map(m->cfg_dof_link, m->num_hinges, OR_MAX_LINKS, link_dof);
  as_link_point(m->parent, link_dof, &m->offset_pos[0][0], &m->offset_quat[0][0], &m->axis[0][0], &m->anchor[0][0],
                st->q + e, st->n, m->geom_link[g], rp, rq, m->geom_p1[g], tip);
}

void or_quad_post_physics(const or_model_t* m, const or_sim_t* sim, const or_task_t* task, const or_actuator_t* act,
                          const or_quad_task_t* Q, or_state_t* st, const float* actions, int reset_all,
                          uint64_t seed, float* obs, float* rew, uint8_t* term_out, uint8_t* trunc_out) {
  const int n = st->n, nh = m->num_hinges, N = task->num_steps;
  const float half_z = sim->stone_half[2];
  for (int e = 0; e < n; ++e) {
#define STONE(k, c) F(st->stones, 3 * (k) + (c), n, e)
#define AIM_DIST(f, k, tip) \
  sqrtf(((tip)[0] - STONE(k, 0)) * ((tip)[0] - STONE(k, 0)) + \
        ((tip)[1] - (STONE(k, 1) + Q->foot_offset_y[f])) * ((tip)[1] - (STONE(k, 1) + Q->foot_offset_y[f])))
    float rp[3], rq[4], lin[3], ang[3], a[21];
    for (int k = 0; k < 3; ++k) {
      rp[k] = F(st->root_pos, k, n, e);
      lin[k] = F(st->root_lin, k, n, e);
      ang[k] = F(st->root_ang, k, n, e);
    }
    for (int k = 0; k < 4; ++k) rq[k] = F(st->root_quat, k, n, e);
    for (int k = 0; k < nh; ++k) {
      const float x = reset_all ? 0.f : actions[(size_t)e * nh + k];
      a[k] = fminf(fmaxf(x, -1.f), 1.f);
    }
    int idx = st->idx[e], ep_len = st->ep_len[e], t[4], c[4];
    for (int f = 0; f < 4; ++f) {
      t[f] = F(st->feet, f, n, e);
      c[f] = F(st->feet, 4 + f, n, e);
    }
    uint32_t episode = st->episode[e];
    uint32_t mk[4] = {F(st->contact_mask, 0, n, e), F(st->contact_mask, 1, n, e), F(st->contact_mask_hind, 0, n, e),
                      F(st->contact_mask_hind, 1, n, e)};
    float pot = st->pot[e], old_pot = st->old_pot[e];
    int term = 0, trunc = 0;
    if (!reset_all) {
      ep_len += 1;
      /* ENV:418-440 target tick per foot; ENV:377-380 step reward of a fresh reach */
      float step_hit = 0.f, fsum = 0.f;
      for (int f = 0; f < 4; ++f) {
        float tip[3];
        quad_tip(m, st, e, f, rp, rq, tip);
        const float d = AIM_DIST(f, t[f], tip);
        const int reached = ((mk[f] >> t[f]) & 1u) && d < Q->step_radius;
        if (reached) c[f] += 1;
        if (c[f] >= Q->stop_frames) {
          c[f] = 0;
          t[f] = imin(t[f] + 1, N - 1);
        }
        if (reached && c[f] == 1 && t[f] < N - 1) step_hit += Q->step_reward * as_expf(-d / Q->step_sigma);
        fsum += AIM_DIST(f, t[f], tip);
      }
      idx = imin(t[0], t[1]);
      old_pot = pot;
      const float dx = STONE(idx, 0) - rp[0], dy = STONE(idx, 1) - rp[1];
      const float bd = sqrtf(dx * dx + dy * dy);
      pot = -(bd + Q->foot_progress * fsum) / Q->step_dt;
      const float down[3] = {0.f, 0.f, -1.f};
      float gb[3];
      or_quat_rotate_inverse(rq, down, gb);
      term = gb[2] > -Q->up_z_min || rp[2] < STONE(idx, 2) + Q->min_height;
      trunc = ep_len >= Q->max_episode_length;
      float a2 = 0.f, en = 0.f;
      for (int k = 0; k < nh; ++k) {
        a2 += a[k] * a[k];
        en += fabsf(F(st->qd, k, n, e) * a[k]);
      }
      const float bonus = idx == N - 1 && bd < Q->bonus_radius ? Q->target_bonus : 0.f;
      const float progress = pot - old_pot;
      rew[e] = term ? Q->death
                    : (((Q->alive + progress) - Q->energy_cost * en) - Q->action_cost * sqrtf(a2)) + step_hit + bonus;
      term_out[e] = (uint8_t)term;
      trunc_out[e] = (uint8_t)trunc;
    }
    float q[21], qd[21];
    for (int k = 0; k < nh; ++k) {
      q[k] = F(st->q, k, n, e);
      qd[k] = F(st->qd, k, n, e);
    }
    const int was_reset = reset_all || term || trunc;
    if (was_reset) {
      float blk[4];
      for (int k = 0; k < nh; ++k) {
        if ((k & 3) == 0) or_philox_block(seed, (uint32_t)e, episode, (uint32_t)(k >> 2), QUAD_TAG, blk);
        q[k] = act->default_q[k] + Q->joint_noise * (2.f * blk[k & 3] - 1.f);
        qd[k] = 0.f;
        F(st->q, k, n, e) = q[k];
        F(st->qd, k, n, e) = 0.f;
      }
      episode += 1u;
      rp[0] = 0.5f * (STONE(0, 0) + STONE(1, 0));
      rp[1] = 0.5f * (STONE(0, 1) + STONE(1, 1));
      rp[2] = fmaxf(STONE(0, 2), STONE(1, 2)) + half_z + Q->stand_height;
      rq[0] = 1.f; rq[1] = rq[2] = rq[3] = 0.f;
      for (int k = 0; k < 3; ++k) {
        lin[k] = ang[k] = 0.f;
        F(st->root_pos, k, n, e) = rp[k];
        F(st->root_lin, k, n, e) = 0.f;
        F(st->root_ang, k, n, e) = 0.f;
      }
      for (int k = 0; k < 4; ++k) F(st->root_quat, k, n, e) = rq[k];
      ep_len = 0;
      float fsum = 0.f;
      for (int f = 0; f < 4; ++f) {
        t[f] = imin(f < 2 ? 2 : 1, N - 1);
        c[f] = 0;
        float tip[3];
        quad_tip(m, st, e, f, rp, rq, tip); /* the reset pose (q written above) */
        fsum += AIM_DIST(f, t[f], tip);
      }
      idx = imin(t[0], t[1]);
      const float dx = STONE(idx, 0) - rp[0], dy = STONE(idx, 1) - rp[1];
      pot = -(sqrtf(dx * dx + dy * dy) + Q->foot_progress * fsum) / Q->step_dt;
      old_pot = pot;
      for (int k = 0; k < 4; ++k) mk[k] = 0u;
      F(st->contact_mask, 0, n, e) = F(st->contact_mask, 1, n, e) = 0u;
      F(st->contact_mask_hind, 0, n, e) = F(st->contact_mask_hind, 1, n, e) = 0u;
    }
    st->idx[e] = idx;
    for (int f = 0; f < 4; ++f) {
      F(st->feet, f, n, e) = t[f];
      F(st->feet, 4 + f, n, e) = c[f];
    }
    st->ep_len[e] = ep_len;
    st->episode[e] = episode;
    st->pot[e] = pot;
    st->old_pot[e] = old_pot;
    float* o = obs + (size_t)e * QUAD_OBS;
    float v[3];
    or_quat_rotate_inverse(rq, lin, v);
    o[0] = v[0]; o[1] = v[1]; o[2] = v[2];
    or_quat_rotate_inverse(rq, ang, v);
    o[3] = v[0]; o[4] = v[1]; o[5] = v[2];
    const float down[3] = {0.f, 0.f, -1.f};
    or_quat_rotate_inverse(rq, down, v);
    o[6] = v[0]; o[7] = v[1]; o[8] = v[2];
    for (int f = 0; f < 5; ++f) {
      const int k = f < 4 ? t[f] : imin(idx + 1, N - 1);
      const float oy = f < 4 ? Q->foot_offset_y[f] : 0.f;
      const float d[3] = {STONE(k, 0) - rp[0], (STONE(k, 1) + oy) - rp[1], STONE(k, 2) - rp[2]};
      or_quat_rotate_inverse(rq, d, v);
      o[9 + 3 * f] = v[0]; o[10 + 3 * f] = v[1]; o[11 + 3 * f] = v[2];
    }
    for (int f = 0; f < 4; ++f) o[24 + f] = (mk[f] >> t[f]) & 1u ? 1.f : 0.f;
    for (int k = 0; k < nh; ++k) {
      o[28 + k] = q[k] - act->default_q[k];
      o[28 + nh + k] = qd[k];
      o[28 + 2 * nh + k] = was_reset ? 0.f : a[k]; /* _reset_idx zeroes _actions (anymal_c_env.py:171-172) */
    }
#undef AIM_DIST
#undef STONE
  }
}

void or_quad_step(const or_model_t* m, const or_sim_t* sim, const or_task_t* task, const or_actuator_t* act,
                  const or_quad_task_t* q, or_state_t* st, const float* actions, uint64_t seed, float* obs,
                  float* rew, uint8_t* term, uint8_t* trunc, int nthreads) {
  const int n = st->n, nh = m->num_hinges;
  (void)nthreads;
#pragma omp parallel for num_threads(nthreads > 0 ? nthreads : 1) schedule(static)
  for (int e = 0; e < n; ++e) {
    float a[21];
    for (int k = 0; k < nh; ++k) {
      const float x = actions[(size_t)e * nh + k];
      a[k] = x < -1.f ? -1.f : (x > 1.f ? 1.f : x);
    }
    or_physics_step_act(m, sim, task, act, st, e, a);
  }
  or_quad_post_physics(m, sim, task, act, q, st, actions, 0, seed, obs, rew, term, trunc);
}

/* test hook: as_link_point on env e's state (the C5 task's foot-tip FK) */
void or_link_point(const or_model_t* m, const or_state_t* st, int e, int link, const float* pl, float* out) {
  const int n = st->n;
  float rp[3], rq[4];
  for (int k = 0; k < 3; ++k) rp[k] = F(st->root_pos, k, n, e);
  for (int k = 0; k < 4; ++k) rq[k] = F(st->root_quat, k, n, e);
  int32_t link_dof[OR_MAX_LINKS];
  as_link_dof_map(m->cfg_dof_link, m->num_hinges, OR_MAX_LINKS, link_dof);
  as_link_point(m->parent, link_dof, &m->offset_pos[0][0], &m->offset_quat[0][0], &m->axis[0][0], &m->anchor[0][0],
                st->q + e, n, link, rp, rq, pl, out);
}
