/*
 * as_detmath.h -- the float32 arithmetic specification shared by the HIP step kernels
 * (allsteps_isaaclab_amd/csrc) and the CPU oracle (oracle/physics.c).
 *
 * Bit-exact HIP <-> oracle parity needs every float operation
 * on the physics path to be the same correctly rounded IEEE-754 operation in the same order on both
 * sides.  Both sides are compiled with -ffp-contract=off, so a * b + c is a multiply and an add
 * everywhere; where an FMA is wanted it is written as fmaf() (v_fma_f32 on gfx950, the correctly
 * rounded fmaf of C99 on the host), in the order fixed here.  Division and sqrtf are correctly
 * rounded on both sides (HIP's default -fhip-fp32-correctly-rounded-divide-sqrt; IEEE on x86-64).
 *
 * Library transcendentals differ between the device math library and the host libm by an ulp, so
 * the physics path uses as_sincosf below instead: Cody-Waite reduction by pi/2 and minimax
 * polynomials on [-pi/4, pi/4], built only from rintf / multiply / fmaf (max error ~2 ulp for
 * |x| < 1e4; the path's arguments are joint angles, half rotation angles and stone bearings).
 *
 * Plain C99 + HIP: every function is usable from gcc (oracle) and hipcc (device and host).
 */
#ifndef AS_DETMATH_H
#define AS_DETMATH_H

#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define AS_HD __host__ __device__ __forceinline__
#else
#define AS_HD static inline
#endif

/* The H^-1 sweep's layout (csrc/allsteps_kernels.hip sweep_inverse, oracle/physics.c sweep_inverse):
 * the nv dofs are padded to a multiple of 4 with identity rows / columns inserted at padded index
 * AS_SWEEP_PAD(nv) (dof k < pad -> k, else k + the pad count), and the 4 x 4 pivot blocks are swept
 * LAST block first -- the limbs (the high dof indices of a topological order) before the root, so the
 * columns of the other limbs stay exactly zero through the first rounds.  The pad position aligns the
 * walker's arms (dofs 19-22, 23-26) and the quadruped's last leg to whole blocks. */
#define AS_SWEEP_PAD(nv) ((nv) == 27 ? 19 : (nv) == 18 ? 15 : (nv))

/* dot products: fmaf chain from the first product, ascending index */
AS_HD float as_dot3(const float* a, const float* b) { return fmaf(a[2], b[2], fmaf(a[1], b[1], a[0] * b[0])); }

AS_HD float as_dot6(const float* a, const float* b) {
  float s = a[0] * b[0];
  s = fmaf(a[1], b[1], s);
  s = fmaf(a[2], b[2], s);
  s = fmaf(a[3], b[3], s);
  s = fmaf(a[4], b[4], s);
  return fmaf(a[5], b[5], s);
}

/* a x b, each component as fmaf(p, q, -(r s)) */
AS_HD void as_cross3(const float* a, const float* b, float* o) {
  const float x = fmaf(a[1], b[2], -(a[2] * b[1]));
  const float y = fmaf(a[2], b[0], -(a[0] * b[2]));
  const float z = fmaf(a[0], b[1], -(a[1] * b[0]));
  o[0] = x; o[1] = y; o[2] = z;
}

/* row-major 3x3 */
AS_HD void as_matvec3(const float* A, const float* v, float* o) {
  const float x = as_dot3(A, v), y = as_dot3(A + 3, v), z = as_dot3(A + 6, v);
  o[0] = x; o[1] = y; o[2] = z;
}

AS_HD void as_matmul3(const float* A, const float* B, float* C) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      C[3 * i + j] = fmaf(A[3 * i + 2], B[6 + j], fmaf(A[3 * i + 1], B[3 + j], A[3 * i] * B[j]));
}

/* symmetric (xx yy zz xy xz yz) times vector */
AS_HD void as_sym_mul(const float* I, const float* w, float* o) {
  const float x = fmaf(I[4], w[2], fmaf(I[3], w[1], I[0] * w[0]));
  const float y = fmaf(I[5], w[2], fmaf(I[1], w[1], I[3] * w[0]));
  const float z = fmaf(I[2], w[2], fmaf(I[5], w[1], I[4] * w[0]));
  o[0] = x; o[1] = y; o[2] = z;
}

/* spatial inertia (m, h, Io) x motion [w; v] = [Io w + h x v; m v - h x w] */
AS_HD void as_inertia_mul(const float* I, const float* V, float* out) {
  float Iw[3], hv[3], hw[3];
  as_sym_mul(I + 4, V, Iw);
  as_cross3(I + 1, V + 3, hv);
  as_cross3(I + 1, V, hw);
  for (int k = 0; k < 3; ++k) {
    out[k] = Iw[k] + hv[k];
    out[3 + k] = fmaf(I[0], V[3 + k], -hw[k]);
  }
}

/* [w;v] x_m [w2;v2] = [w x w2; w x v2 + v x w2] */
AS_HD void as_crm(const float* V, const float* M, float* o) {
  float a[3], b[3], c[3];
  as_cross3(V, M, a);
  as_cross3(V, M + 3, b);
  as_cross3(V + 3, M, c);
  for (int k = 0; k < 3; ++k) { o[k] = a[k]; o[3 + k] = b[k] + c[k]; }
}

/* [w;v] x_f [n;f] = [w x n + v x f; w x f] */
AS_HD void as_crf(const float* V, const float* Fv, float* o) {
  float a[3], b[3], c[3];
  as_cross3(V, Fv, a);
  as_cross3(V + 3, Fv + 3, b);
  as_cross3(V, Fv + 3, c);
  for (int k = 0; k < 3; ++k) { o[k] = a[k] + b[k]; o[3 + k] = c[k]; }
}

/* unit quaternion (w, x, y, z) -> row-major rotation matrix */
AS_HD void as_quat_to_mat(const float* q, float* R) {
  const float w = q[0], x = q[1], y = q[2], z = q[3];
  const float xx = x * x, yy = y * y, zz = z * z;
  const float xy = x * y, xz = x * z, yz = y * z, wx = w * x, wy = w * y, wz = w * z;
  R[0] = 1.f - 2.f * (yy + zz); R[1] = 2.f * (xy - wz);       R[2] = 2.f * (xz + wy);
  R[3] = 2.f * (xy + wz);       R[4] = 1.f - 2.f * (xx + zz); R[5] = 2.f * (yz - wx);
  R[6] = 2.f * (xz - wy);       R[7] = 2.f * (yz + wx);       R[8] = 1.f - 2.f * (xx + yy);
}

/* sin and cos of x: k = rint(x 2/pi), r = x - k pi/2 in three fmaf steps (Cody-Waite), minimax
 * polynomials in r^2 on [-pi/4, pi/4], quadrant select by k mod 4. */
AS_HD void as_sincosf(float x, float* sn, float* cs) {
  const float k = rintf(x * 0.636619772f);
  float r = fmaf(-k, 1.57079625e+00f, x);
  r = fmaf(-k, 7.54978942e-08f, r);
  r = fmaf(-k, 5.39030253e-15f, r);
  const float z = r * r;
  float ps = fmaf(-1.9515296e-04f, z, 8.3321608e-03f);
  ps = fmaf(ps, z, -1.6666655e-01f);
  const float s = fmaf(ps * z, r, r);
  float pc = fmaf(2.4433157e-05f, z, -1.3887316e-03f);
  pc = fmaf(pc, z, 4.1666646e-02f);
  const float c = fmaf(pc * z, z, fmaf(-0.5f, z, 1.0f));
  const int q = ((int)k) & 3;
  const float s1 = (q & 1) ? c : s;
  const float c1 = (q & 1) ? s : c;
  *sn = (q & 2) ? -s1 : s1;
  *cs = ((q + 1) & 2) ? -c1 : c1;
}

/* ---- the task path's transcendentals (allsteps_env.py rewards / observations).  Same construction
 * as as_sincosf: range reduction and minimax polynomials from +, *, fmaf, division and sqrtf only,
 * all correctly rounded on both sides, so the device and the host produce the same bits.  Accuracy
 * (vs double precision): as_atan2f <= 2.5 ulp, as_asinf <= 3 ulp, as_expf <= 2 ulp on the domains
 * the task uses (Cephes-style coefficients; tests/test_detmath.py measures them). */

/* atan(t) for t in [0, 1]: t > tan(pi/8) is reduced by atan(t) = pi/4 + atan((t - 1) / (t + 1)) */
AS_HD float as_atan01f(float t) {
  const int red = t > 0.414213562f;
  const float z = red ? (t - 1.0f) / (t + 1.0f) : t;
  const float z2 = z * z;
  float p = fmaf(8.05374449538e-2f, z2, -1.38776856032e-1f);
  p = fmaf(p, z2, 1.99777106478e-1f);
  p = fmaf(p, z2, -3.33329491539e-1f);
  const float y = fmaf(p * z2, z, z);
  return red ? y + 0.785398163397448309616f : y;
}

/* atan2(y, x) with C's signed-zero cases (atan2(+-0, +0) = +-0, atan2(+-0, -0) = +-pi); quadrants
 * from |y| vs |x| and the signs; the pi/2 and pi complements in two parts (hi + lo) */
AS_HD float as_atan2f(float y, float x) {
  const float ax = fabsf(x), ay = fabsf(y);
  const int ysign = signbit(y) != 0;
  if (ax == 0.0f && ay == 0.0f) {
    const float r = signbit(x) ? 3.14159265358979323846f : 0.0f;
    return ysign ? -r : r;
  }
  const int swap = ay > ax;
  const float a = as_atan01f(swap ? ax / ay : ay / ax);
  float r = swap ? (1.57079637050628662109f - a) + -4.37113900018624283e-08f : a;
  if (signbit(x)) r = (3.14159274101257324219f - r) + -8.74227800037248566e-08f;
  return ysign ? -r : r;
}

/* asin(s) for |s| < 1: |s| > 0.5 uses asin(s) = pi/2 - 2 asin(sqrt((1 - |s|) / 2)) */
AS_HD float as_asinf(float s) {
  const float a = fabsf(s);
  const int big = a > 0.5f;
  const float z = big ? 0.5f * (1.0f - a) : a * a;
  const float x = big ? sqrtf(z) : a;
  float p = fmaf(4.2163199048e-2f, z, 2.4181311049e-2f);
  p = fmaf(p, z, 4.5470025998e-2f);
  p = fmaf(p, z, 7.4953002686e-2f);
  p = fmaf(p, z, 1.6666752422e-1f);
  float r = fmaf(p * z, x, x);
  if (big) r = (1.57079637050628662109f - (r + r)) + -4.37113900018624283e-08f;
  return signbit(s) ? -r : r;
}

/* exp(x) for x <= 0 (the step reward's exp(-d / 0.25)): k = rint(x log2 e), r = x - k ln 2 in two
 * fmaf steps, a degree-6 polynomial for e^r on [-ln2/2, ln2/2], scaled by 2^k (ldexpf, exact for the
 * normal results kept here); x < -87 (e^x below the normal range) gives +0; NaN passes through
 * (a float-to-int of NaN differs between the device and x86, so it must never reach ldexpf) */
AS_HD float as_expf(float x) {
  if (!(x == x)) return x;
  if (x < -87.0f) return 0.0f;
  const float k = rintf(x * 1.44269504088896341f);
  float r = fmaf(-k, 0.693359375f, x);
  r = fmaf(-k, -2.12194440e-4f, r);
  float p = fmaf(1.9875691500e-4f, r, 1.3981999507e-3f);
  p = fmaf(p, r, 8.3334519073e-3f);
  p = fmaf(p, r, 4.1665795894e-2f);
  p = fmaf(p, r, 1.6666665459e-1f);
  p = fmaf(p, r, 5.0000001201e-1f);
  const float y = fmaf(p, r * r, r) + 1.0f;
  return ldexpf(y, (int)k);
}

/* torch.remainder(a, 2 pi) for |a| <= pi (euler_xyz_from_quat's atan2 / asin results, math.py:444):
 * fmod is the identity there, so the remainder is a + 2 pi for a < 0 and a otherwise (-0 stays -0) */
AS_HD float as_rem2pi(float a) { return a < 0.0f ? a + 6.28318530717958647692f : a; }

/* Rodrigues rotation about the unit axis a by ang (as_sincosf) */
AS_HD void as_axis_angle_mat(const float* a, float ang, float* R) {
  float s, c;
  as_sincosf(ang, &s, &c);
  const float t = 1.f - c;
  const float tx = t * a[0], ty = t * a[1], tz = t * a[2];
  R[0] = fmaf(tx, a[0], c);           R[1] = fmaf(tx, a[1], -(s * a[2])); R[2] = fmaf(tx, a[2], s * a[1]);
  R[3] = fmaf(tx, a[1], s * a[2]);    R[4] = fmaf(ty, a[1], c);          R[5] = fmaf(ty, a[2], -(s * a[0]));
  R[6] = fmaf(tx, a[2], -(s * a[1])); R[7] = fmaf(ty, a[2], s * a[0]);   R[8] = fmaf(tz, a[2], c);
}

/* World position of the point pl (link frame) on `link`: the root pose (rp, unit quaternion rq), then
 * the walk root -> link with every link's joint transform as the physics' FK forms it
 * (oracle/physics.c kinematics): Rl = Roff(offset_quat) Rj(axis, q), tl = offset_pos + Roff (anchor -
 * Rj anchor); p += R tl, R = R Rl; out = rp + (p + R pl).  The hinge angle of link i is read from the
 * state column q_col[link_dof[i] * q_stride], link_dof the inverse of cfg_dof_link (as_link_dof_map).
 * Model tables flattened row-major ([link][3] / [link][4]). */
AS_HD void as_link_point(const int32_t* parent, const int32_t* link_dof, const float* offset_pos,
                         const float* offset_quat, const float* axis, const float* anchor, const float* q_col,
                         int q_stride, int link, const float* rp, const float* rq, const float* pl, float* out) {
  int depth = 0;
  for (int l = link; l > 0; l = parent[l]) ++depth;
  float R[9], p[3] = {0.f, 0.f, 0.f};
  as_quat_to_mat(rq, R);
  for (int s = depth - 1; s >= 0; --s) {
    int i = link;
    for (int j = 0; j < s; ++j) i = parent[i];  /* the ancestor s links above `link` */
    const float qi = q_col[link_dof[i] * q_stride];
    float Roff[9], Rj[9], Rl[9], Ro[3], t[3], tl[3], wp[3], Rn[9];
    as_quat_to_mat(offset_quat + 4 * i, Roff);
    as_axis_angle_mat(axis + 3 * i, qi, Rj);
    as_matmul3(Roff, Rj, Rl);
    as_matvec3(Rj, anchor + 3 * i, Ro);
    for (int k = 0; k < 3; ++k) t[k] = anchor[3 * i + k] - Ro[k];
    as_matvec3(Roff, t, tl);
    for (int k = 0; k < 3; ++k) tl[k] = tl[k] + offset_pos[3 * i + k];
    as_matvec3(R, tl, wp);
    for (int k = 0; k < 3; ++k) p[k] = p[k] + wp[k];
    as_matmul3(R, Rl, Rn);
    for (int k = 0; k < 9; ++k) R[k] = Rn[k];
  }
  float w[3];
  as_matvec3(R, pl, w);
  for (int k = 0; k < 3; ++k) out[k] = rp[k] + (p[k] + w[k]);
}

/* link_dof[i] = the cfg dof k with cfg_dof_link[k] == i (0 for the root and unused links) */
AS_HD void as_link_dof_map(const int32_t* cfg_dof_link, int nh, int nlinks, int32_t* link_dof) {
  for (int i = 0; i < nlinks; ++i) link_dof[i] = 0;
  for (int k = 0; k < nh; ++k) link_dof[cfg_dof_link[k]] = k;
}

/* ---- actuators (include/allsteps.h as_actuator_t) */

/* IsaacLab's DCMotor on a position target (actuator_pd.py:184-199, 264-275), torch's float32 order:
 * tau = kp (q* - q) + kd (0 - qd) + 0, clipped to [clip(sat (-1 - qd / vmax), -lim, 0),
 * clip(sat (1 - qd / vmax), 0, lim)] */
AS_HD float as_dc_motor(float qt, float q, float qd, float kp, float kd, float sat, float lim, float vmax) {
  const float tau = kp * (qt - q) + kd * (0.f - qd) + 0.f;
  const float r = qd / vmax;
  const float hi = fminf(fmaxf(sat * (1.f - r), 0.f), lim);
  const float lo = fminf(fmaxf(sat * (-1.f - r), -lim), 0.f);
  return fminf(fmaxf(tau, lo), hi);
}

/* ---- robot self-collision (walker3d.py:27 enabled_self_collisions; shared by kernel and oracle) */

AS_HD float as_clamp01(float x) { return fminf(fmaxf(x, 0.f), 1.f); }

/* Pair filter: the bounding spheres (segment midpoint m, half length + radius R) of two geoms come
 * within `margin`.  Conservative for the exact test below up to rounding; both sides apply it in the
 * same arithmetic, so they keep the same pairs. */
AS_HD int as_sphere_bound(const float* m1, float R1, const float* m2, float R2, float margin) {
  const float d0 = m1[0] - m2[0], d1 = m1[1] - m2[1], d2 = m1[2] - m2[2];
  const float lim = R1 + R2 + margin;
  return d0 * d0 + d1 * d1 + d2 * d2 <= lim * lim;
}

/* Contact of two capsules (a sphere is a capsule with a == b): closest points of the segments
 * [a1, b1] and [a2, b2] (Ericson, Real-Time Collision Detection, 5.1.9: s, t clamped to [0, 1]),
 * separation |c1 - c2| - r1 - r2 (returned), unit normal n from geom 2 towards geom 1 (+z if the axes
 * touch), contact point P midway between the two surfaces along n. */
AS_HD float as_capsule_contact(const float* a1, const float* b1, float r1, const float* a2, const float* b2,
                               float r2, float* P, float* n) {
  float d1[3], d2[3], r[3];
  for (int k = 0; k < 3; ++k) {
    d1[k] = b1[k] - a1[k];
    d2[k] = b2[k] - a2[k];
    r[k] = a1[k] - a2[k];
  }
  const float a = as_dot3(d1, d1), e = as_dot3(d2, d2), f = as_dot3(d2, r);
  const float eps = 1e-12f;
  float s = 0.f, t = 0.f;
  if (a <= eps) {
    t = e <= eps ? 0.f : as_clamp01(f / e);
  } else {
    const float c = as_dot3(d1, r);
    if (e <= eps) {
      s = as_clamp01(-c / a);
    } else {
      const float b = as_dot3(d1, d2);
      const float den = fmaf(a, e, -(b * b));
      s = den > 0.f ? as_clamp01(fmaf(b, f, -(c * e)) / den) : 0.f;
      t = fmaf(b, s, f) / e;
      if (t < 0.f) {
        t = 0.f;
        s = as_clamp01(-c / a);
      } else if (t > 1.f) {
        t = 1.f;
        s = as_clamp01((b - c) / a);
      }
    }
  }
  float c1[3], c2[3], w[3];
  for (int k = 0; k < 3; ++k) {
    c1[k] = fmaf(s, d1[k], a1[k]);
    c2[k] = fmaf(t, d2[k], a2[k]);
    w[k] = c1[k] - c2[k];
  }
  const float dist = sqrtf(as_dot3(w, w));
  if (dist > 1e-9f) {
    const float inv = 1.0f / dist;
    n[0] = w[0] * inv; n[1] = w[1] * inv; n[2] = w[2] * inv;
  } else {
    n[0] = 0.f; n[1] = 0.f; n[2] = 1.f;
  }
  const float sep = dist - r1 - r2;
  const float off = fmaf(0.5f, sep, r2);
  for (int k = 0; k < 3; ++k) P[k] = fmaf(off, n[k], c2[k]);
  return sep;
}

#endif /* AS_DETMATH_H */
