// allsteps_device.h -- device-side math for the Allsteps step kernels (gfx950).
//
// Small fixed-size vector / spatial-algebra helpers, the isaaclab.utils.math formulas the task
// uses (isaaclab/utils/math.py:22-61, 224-249, 413-444, 546-625, 785-818), and the Philox4x32-10
// counter RNG that replaces torch.rand in the reset path (allsteps_env.py:518, 542).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/as_detmath.h"

namespace as {

#define AS_DEV __device__ __forceinline__

// Physics-path primitives: the fmaf-ordered arithmetic of include/as_detmath.h, shared with the
// oracle (oracle/physics.c) so both sides round identically (the library is built with
// -ffp-contract=off, so nothing else is contracted).
AS_DEV void cross3(const float* a, const float* b, float* o) { as_cross3(a, b, o); }
AS_DEV float dot3(const float* a, const float* b) { return as_dot3(a, b); }
AS_DEV float dot6(const float* a, const float* b) { return as_dot6(a, b); }
AS_DEV void quat_to_mat(const float* q, float* R) { as_quat_to_mat(q, R); }
AS_DEV void axis_angle_mat(const float* a, float ang, float* R) { as_axis_angle_mat(a, ang, R); }
AS_DEV void matmul3(const float* A, const float* B, float* C) { as_matmul3(A, B, C); }
AS_DEV void matvec3(const float* A, const float* v, float* o) { as_matvec3(A, v, o); }
AS_DEV void inertia_mul(const float* I, const float* V, float* out) { as_inertia_mul(I, V, out); }
AS_DEV void crm(const float* V, const float* M, float* o) { as_crm(V, M, o); }
AS_DEV void crf(const float* V, const float* Fv, float* o) { as_crf(V, Fv, o); }

// Task-path cross product (isaaclab.utils.math uses torch.cross: plain products and a difference,
// oracle/task.c cross3)
AS_DEV void task_cross3(const float* a, const float* b, float* o) {
  float x = a[1] * b[2] - a[2] * b[1], y = a[2] * b[0] - a[0] * b[2], z = a[0] * b[1] - a[1] * b[0];
  o[0] = x; o[1] = y; o[2] = z;
}

// signed distance from p to an axis-aligned box (center c, half extents h); outward normal
// Slope sign carrier of t -> sd_box(a + t (b - a)) (convex in t): outside the box (some slab
// distance d_k > 0) sum_k o_k s_k D_k, half the derivative of the squared distance; inside the
// derivative of the deepest slab term, s_ax D_ax (ties to the lowest axis).  Only its sign is used
// (oracle sd_box_slope, same operations): the offset a - c and D are loop-invariant in the bisection,
// so a round is one FMA per axis for the point, a max3 for the outside test and an FMA chain for the sum.
AS_DEV float sd_box_slope(const float* a, const float* b, float t, const float* c, const float* h) {
  float d[3], sD[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float D = b[k] - a[k];
    const float r = fmaf(t, D, a[k] - c[k]);
    sD[k] = r >= 0.f ? D : -D;
    d[k] = fabsf(r) - h[k];
  }
  const float o0 = fmaxf(d[0], 0.f), o1 = fmaxf(d[1], 0.f), o2 = fmaxf(d[2], 0.f);
  const float g_out = fmaf(o2, sD[2], fmaf(o1, sD[1], o0 * sD[0]));
  int ax = 0;
  if (d[1] > d[ax]) ax = 1;
  if (d[2] > d[ax]) ax = 2;
  const float g_in = ax == 0 ? sD[0] : (ax == 1 ? sD[1] : sD[2]);
  return fmaxf(d[0], fmaxf(d[1], d[2])) > 0.f ? g_out : g_in;
}

AS_DEV float sd_box(const float* p, const float* c, const float* h, float* nrm) {
  float d[3], s[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    float r = p[k] - c[k];
    s[k] = r >= 0.f ? 1.f : -1.f;
    d[k] = fabsf(r) - h[k];
  }
  float o0 = fmaxf(d[0], 0.f), o1 = fmaxf(d[1], 0.f), o2 = fmaxf(d[2], 0.f);
  float out = sqrtf(o0 * o0 + o1 * o1 + o2 * o2);
  if (out > 0.f) {
    float inv = 1.0f / out;
    nrm[0] = s[0] * o0 * inv; nrm[1] = s[1] * o1 * inv; nrm[2] = s[2] * o2 * inv;
    return out;
  }
  int ax = 0;
  if (d[1] > d[ax]) ax = 1;
  if (d[2] > d[ax]) ax = 2;
  nrm[0] = ax == 0 ? s[0] : 0.f;
  nrm[1] = ax == 1 ? s[1] : 0.f;
  nrm[2] = ax == 2 ? s[2] : 0.f;
  return ax == 0 ? d[0] : (ax == 1 ? d[1] : d[2]);
}

// ---------------------------------------------------------------- isaaclab.utils.math (math.py)

// math.py:413-444 euler_xyz_from_quat (roll, pitch), "% 2pi" = torch.remainder; atan2 / asin / remainder
// are the shared deterministic forms of include/as_detmath.h (the oracle computes the same bits)
AS_DEV void euler_rp_from_quat(const float* q, float* roll, float* pitch) {
  float qw = q[0], qx = q[1], qy = q[2], qz = q[3];
  float sin_roll = 2.0f * (qw * qx + qy * qz);
  float cos_roll = 1.0f - 2.0f * (qx * qx + qy * qy);
  float r = as_atan2f(sin_roll, cos_roll);
  float sin_pitch = 2.0f * (qw * qy - qz * qx);
  float p = fabsf(sin_pitch) >= 1.0f ? 1.57079632679489661923f * (sin_pitch > 0.0f ? 1.0f : -1.0f)
                                    : as_asinf(sin_pitch);
  *roll = as_rem2pi(r);
  *pitch = as_rem2pi(p);
}

// math.py:605-625 quat_rotate_inverse
AS_DEV void quat_rotate_inverse(const float* q, const float* v, float* out) {
  float w = q[0];
  const float* qv = q + 1;
  float s = 2.0f * (w * w) - 1.0f;
  float cr[3];
  task_cross3(qv, v, cr);
  float d = qv[0] * v[0] + qv[1] * v[1] + qv[2] * v[2];
#pragma unroll
  for (int i = 0; i < 3; ++i) out[i] = v[i] * s - cr[i] * w * 2.0f + qv[i] * d * 2.0f;
}

// math.py:785-818 subtract_frame_transforms (translation): quat_apply(normalize(conj(q01)), t02 - t01)
AS_DEV void subtract_frame_transforms(const float* t01, const float* q01, const float* t02, float* out) {
  float c0 = q01[0], c1 = -q01[1], c2 = -q01[2], c3 = -q01[3];
  float nrm = fmaxf(sqrtf(c0 * c0 + c1 * c1 + c2 * c2 + c3 * c3), 1e-9f);
  float q10[4] = {c0 / nrm, c1 / nrm, c2 / nrm, c3 / nrm};
  float v[3] = {t02[0] - t01[0], t02[1] - t01[1], t02[2] - t01[2]};
  float t[3], t2[3];
  task_cross3(q10 + 1, v, t);
  t[0] *= 2.0f; t[1] *= 2.0f; t[2] *= 2.0f;
  task_cross3(q10 + 1, t, t2);
#pragma unroll
  for (int i = 0; i < 3; ++i) out[i] = v[i] + q10[0] * t[i] + t2[i];
}

// math.py:22-61
AS_DEV float scale_transform(float x, float lo, float hi) { return 2.0f * (x - (lo + hi) * 0.5f) / (hi - lo); }
AS_DEV float unscale_transform(float x, float lo, float hi) { return x * (hi - lo) * 0.5f + (lo + hi) * 0.5f; }

// ---------------------------------------------------------------- Philox4x32-10

AS_DEV void philox4x32_10(uint32_t* ctr, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t lo0 = 0xD2511F53u * ctr[0], hi0 = __umulhi(0xD2511F53u, ctr[0]);
    uint32_t lo1 = 0xCD9E8D57u * ctr[2], hi1 = __umulhi(0xCD9E8D57u, ctr[2]);
    uint32_t n0 = hi1 ^ ctr[1] ^ k0, n2 = hi0 ^ ctr[3] ^ k1;
    ctr[0] = n0; ctr[1] = lo1; ctr[2] = n2; ctr[3] = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

// 4 uniforms in [0,1) of block b of the (env, episode) stream
AS_DEV void philox_block(uint64_t seed, uint32_t env, uint32_t episode, uint32_t b, uint32_t tag, float* out4) {
  uint32_t ctr[4] = {env, episode, b, tag};
  philox4x32_10(ctr, (uint32_t)seed, (uint32_t)(seed >> 32));
#pragma unroll
  for (int j = 0; j < 4; ++j) out4[j] = (float)(ctr[j] >> 8) * (1.0f / 16777216.0f);
}

constexpr uint32_t kResetTag = 0x416c6c73u;  // "Alls"
constexpr uint32_t kStonesTag = 0x53746f6eu; // "Ston"

}  // namespace as
