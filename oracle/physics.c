/*
 * physics.c -- CPU restatement of the articulated-body step that replaces PhysX
 * (TEST INFRASTRUCTURE; see oracle.h).
 *
 * The reference steps PhysX 5 (isaacsim 4.5 / omni.physx, external, absent offline) through
 * isaaclab/sim/simulation_context.py:453-478 with the articulation configured at
 * isaaclab_assets/robots/walker3d.py:21-46 (self-collision on, 4 position / 0 velocity solver
 * iterations, gyroscopic forces on, max_depenetration_velocity 10, implicit actuators with
 * kp = kd = 0 so the effort target is the joint torque).  PARITY UNPINNED against PhysX.
 *
 * Algorithm (one substep, dt = 1/240; DESIGN.md §Dynamics is the spec the HIP kernel follows):
 *   1. FK of all links, spatial quantities in a world-aligned frame with origin at the root link
 *      origin (O).  Generalised velocity u = [v_com0 (3), w0 (3), qd hinges (nh)].
 *   2. RNEA with qdd = 0 -> bias C(q, u) (Coriolis, centrifugal, gyroscopic, gravity).
 *   3. CRBA -> joint-space inertia H (+ armature on the hinge diagonal); H^-1 by the symmetric
 *      sweep operator.  Subtree sums (composite inertias, RNEA forces) in the kernel's order.
 *   4. u* = u + dt H^-1 (tau - C).
 *   5. Contacts (robot spheres/capsules vs the 20 axis-aligned stone boxes, speculative margin)
 *      and joint-limit rows; projected Gauss-Seidel on impulses (normal >= 0, box friction,
 *      Baumgarte bias capped at max_depenetration_velocity), pgs_iters sweeps.
 *   6. Semi-implicit integration: hinges q += dt u, root COM += dt v, orientation by exp map.
 *   The per-(foot, stone) normal impulse of the last substep gives the contact-sensor flags
 *   (contact_sensor.py:320-343: force_matrix_w = impulse / dt, tested > 1e-4 at
 *   allsteps_env.py:421-425).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"
#include "../include/as_detmath.h"

#define NV_MAX (OR_NDOF_ROOT + OR_MAX_LINKS)
#define F(arr, f, n, e) (arr)[(size_t)(f) * (n) + (e)]

typedef struct {
  int nl, nv;
  float R[OR_MAX_LINKS][9];  /* link rotation (world) */
  float p[OR_MAX_LINKS][3];  /* link origin, relative to O */
  float c[OR_MAX_LINKS][3];  /* link COM, relative to O */
  float S[NV_MAX][6];        /* motion subspace [w; v_O] per dof */
  float Ic[OR_MAX_LINKS][10];/* spatial inertia at O: m, h(3), Io(6) (xx yy zz xy xz yz) */
  float Ib[OR_MAX_LINKS][10];/* single-body spatial inertia at O */
  float c0[3];               /* root COM from the root quaternion's matrix (root columns, velocities) */
} kin_t;

/* The primitives of the shared float32 arithmetic specification (include/as_detmath.h): explicit
 * fmaf in a fixed order, everything else uncontracted (-ffp-contract=off), identical to the HIP
 * kernel's rounding. */
#define quat_to_mat as_quat_to_mat
#define axis_angle_mat as_axis_angle_mat
#define matmul3 as_matmul3
#define matvec3 as_matvec3
#define cross as_cross3
#define dot3 as_dot3
#define dot6 as_dot6
#define inertia_mul as_inertia_mul
#define crm as_crm
#define crf as_crf

/* Sum of 32 lane values as the kernel's paired half-wave reduction forms it (half_sum_n: lane l of
 * row 0 adds lane l + 16 of row 1, then DPP butterflies over lane pairs, quads, 8-lane halves and the
 * 16-lane row): the cross-row add, then a balanced binary tree over the 16 partial sums in index
 * order.  Lanes past the row's width carry 0. */
static float tree32(const float* v) {
  float a[16];
  for (int i = 0; i < 16; ++i) a[i] = v[i] + v[i + 16];
  for (int w = 1; w < 16; w *= 2)
    for (int i = 0; i < 16; i += 2 * w) a[i] = a[i] + a[i + w];
  return a[0];
}

/* Dot product over n (even) entries as the kernel's dot_pairs forms it: two interleaved fmaf chains
 * (even / odd entries, ascending), added at the end. */
static float dot_pairs(const float* a, const float* b, int n) {
  float e = 0.f, o = 0.f;
  for (int k = 0; k < n; k += 2) {
    e = fmaf(a[k], b[k], e);
    o = fmaf(a[k + 1], b[k + 1], o);
  }
  return e + o;
}

static int is_ancestor(const or_model_t* m, int a, int l) {
  while (l > a) l = m->parent[l];
  return l == a;
}

/* Subtree sums as the HIP kernel's matrix product forms them (dynamics() in
 * csrc/allsteps_kernels.hip: the two-block f32 MFMA over OR_SUBTREE_STEPS K steps, one per link
 * slot): for every link i, one fmaf chain from +0 over the link slots l ascending,
 * acc = fmaf(x_l, [l in subtree(i)], acc), with x_l = 0 past the model's links; subtree(i) includes
 * i, and the root's is the whole tree. */
#define OR_SUBTREE_STEPS 24 /* the kernel's kMaxLinks */
static void subtree_sums(const or_model_t* m, int nl, int w, const float* own, float* tot) {
  for (int i = 0; i < nl; ++i)
    for (int k = 0; k < w; ++k) {
      float acc = 0.f;
      for (int l = 0; l < OR_SUBTREE_STEPS; ++l) {
        const float x = l < nl ? own[l * w + k] : 0.f;
        const float mk = l < nl && is_ancestor(m, i, l) ? 1.f : 0.f;
        acc = fmaf(x, mk, acc);
      }
      tot[i * w + k] = acc;
    }
}

/* FK + motion subspace + spatial inertias. q_int: hinge angles in link order (link i -> q_int[i-1]).
 * Link i's pose is the kernel's pointer jumping (k_step fk): A_i = its joint's local transform (Rl, tl)
 * (the identity for the root); for r < ceil(log2(max_path)) rounds, every link at once, A_i <- A_a o A_i
 * with a = the 2^r-th ancestor of i (the root past the path) and the round-r values on both sides;
 * (Ra, ta) o (Rb, tb) = (Ra Rb, ta + Ra tb).  Then R_i = R0 A_i.R, p_i = R0 A_i.t. */
static void kinematics(const or_model_t* m, const float root_quat[4], const float* q_int, kin_t* K) {
  const int nl = m->num_links;
  K->nl = nl;
  K->nv = OR_NDOF_ROOT + m->num_hinges;
  float R0[9];
  quat_to_mat(root_quat, R0);
  float A[OR_MAX_LINKS][12], An[OR_MAX_LINKS][12];
  int anc[OR_MAX_LINKS], depth_max = 0;
  for (int i = 0; i < nl; ++i) {
    for (int k = 0; k < 12; ++k) A[i][k] = k == 0 || k == 4 || k == 8 ? 1.f : 0.f;
    anc[i] = i > 0 ? m->parent[i] : 0;
    int dpt = 0;
    for (int l = i; l > 0; l = m->parent[l]) ++dpt;
    if (dpt > depth_max) depth_max = dpt;
  }
  for (int i = 1; i < nl; ++i) {
    float Roff[9], Rj[9], t[3], Ro[3];
    quat_to_mat(m->offset_quat[i], Roff);
    axis_angle_mat(m->axis[i], q_int[i - 1], Rj);
    matmul3(Roff, Rj, A[i]);
    /* joint translation t_j = o - Rj o; local origin = offset_pos + Roff t_j */
    matvec3(Rj, m->anchor[i], Ro);
    for (int k = 0; k < 3; ++k) t[k] = m->anchor[i][k] - Ro[k];
    matvec3(Roff, t, A[i] + 9);
    for (int k = 0; k < 3; ++k) A[i][9 + k] += m->offset_pos[i][k];
  }
  int rounds = 0;
  while ((1 << rounds) < depth_max) ++rounds;
  for (int r = 0; r < rounds; ++r) {
    int an2[OR_MAX_LINKS];
    for (int i = 0; i < nl; ++i) {
      const float* Aa = A[anc[i]];
      float w[3];
      matmul3(Aa, A[i], An[i]);
      matvec3(Aa, A[i] + 9, w);
      for (int k = 0; k < 3; ++k) An[i][9 + k] = Aa[9 + k] + w[k];
      an2[i] = anc[anc[i]];
    }
    memcpy(A, An, sizeof(float) * 12 * (size_t)nl);
    for (int i = 0; i < nl; ++i) anc[i] = an2[i];
  }
  for (int i = 0; i < nl; ++i) {
    matmul3(R0, A[i], K->R[i]);
    matvec3(R0, A[i] + 9, K->p[i]);
  }
  matvec3(R0, m->com[0], K->c0);
  for (int i = 0; i < nl; ++i) {
    float cw[3];
    matvec3(K->R[i], m->com[i], cw);
    for (int k = 0; k < 3; ++k) K->c[i][k] = K->p[i][k] + cw[k];
    /* world inertia about COM: R I R^T */
    const float* Il = m->inertia[i];
    float Im[9] = {Il[0], Il[3], Il[4], Il[3], Il[1], Il[5], Il[4], Il[5], Il[2]};
    float T[9], Iw[9], Rt[9];
    const float* R = K->R[i];
    Rt[0] = R[0]; Rt[1] = R[3]; Rt[2] = R[6]; Rt[3] = R[1]; Rt[4] = R[4]; Rt[5] = R[7];
    Rt[6] = R[2]; Rt[7] = R[5]; Rt[8] = R[8];
    matmul3(R, Im, T);
    matmul3(T, Rt, Iw);
    float mass = m->mass[i], *c = K->c[i];
    float cc = dot3(c, c);
    float* B = K->Ib[i];
    B[0] = mass;
    B[1] = mass * c[0]; B[2] = mass * c[1]; B[3] = mass * c[2];
    B[4] = Iw[0] + mass * (cc - c[0] * c[0]);
    B[5] = Iw[4] + mass * (cc - c[1] * c[1]);
    B[6] = Iw[8] + mass * (cc - c[2] * c[2]);
    B[7] = Iw[1] - mass * c[0] * c[1];
    B[8] = Iw[2] - mass * c[0] * c[2];
    B[9] = Iw[5] - mass * c[1] * c[2];
  }
  /* motion subspace (root columns from the root quaternion's COM, as the kernel's s.c0) */
  const float* c0 = K->c0;
  for (int k = 0; k < 3; ++k) {
    float* Sl = K->S[k];
    float* Sa = K->S[3 + k];
    for (int j = 0; j < 6; ++j) Sl[j] = Sa[j] = 0.f;
    Sl[3 + k] = 1.f;
    float e[3] = {0.f, 0.f, 0.f};
    e[k] = 1.f;
    Sa[k] = 1.f;
    cross(c0, e, Sa + 3);
  }
  for (int i = 1; i < nl; ++i) {
    float a[3], o[3], Ro[3];
    matvec3(K->R[i], m->axis[i], a);
    matvec3(K->R[i], m->anchor[i], Ro);
    for (int k = 0; k < 3; ++k) o[k] = K->p[i][k] + Ro[k];
    float* S = K->S[OR_NDOF_ROOT + i - 1];
    S[0] = a[0]; S[1] = a[1]; S[2] = a[2];
    cross(o, a, S + 3);
  }
  /* composite inertias (world frame: plain sums over the subtree) */
  subtree_sums(m, nl, 10, &K->Ib[0][0], &K->Ic[0][0]);
}

/* dofs influencing link i: hinge dofs on the path to the root (deepest first), then root dofs */
static int chain_dofs(const or_model_t* m, int link, int* out) {
  int n = 0;
  for (int l = link; l > 0; l = m->parent[l]) out[n++] = OR_NDOF_ROOT + l - 1;
  for (int k = OR_NDOF_ROOT - 1; k >= 0; --k) out[n++] = k;
  return n;
}

/* S_k . F as the kernel's two-block MFMA forms it (h_row): one fmaf chain over the six spatial
 * components, ascending, from +0 */
static float chain6(const float* s, const float* f) {
  float a = 0.f;
  for (int c = 0; c < 6; ++c) a = fmaf(s[c], f[c], a);
  return a;
}

static void crba(const or_model_t* m, const kin_t* K, float* H) {
  const int nv = K->nv;
  memset(H, 0, sizeof(float) * (size_t)nv * nv);
  int chain[NV_MAX];
  for (int j = 0; j < nv; ++j) {
    int link = j < OR_NDOF_ROOT ? 0 : j - OR_NDOF_ROOT + 1;
    float Fj[6];
    inertia_mul(K->Ic[link], K->S[j], Fj);
    int nc = chain_dofs(m, link, chain);
    for (int t = 0; t < nc; ++t) {
      int k = chain[t];
      if (k > j) continue; /* fill lower triangle (k <= j) and mirror */
      float h = chain6(K->S[k], Fj);
      H[j * nv + k] = h;
      H[k * nv + j] = h;
    }
  }
  /* root block: the kernel's row j (lane j) forms every root column k from its own column force,
   * H_jk = S_k . (Ic_0 S_j), so its upper triangle is not the mirror of the lower one */
  for (int j = 0; j < OR_NDOF_ROOT; ++j) {
    float Fj[6];
    inertia_mul(K->Ic[0], K->S[j], Fj);
    for (int k = j + 1; k < OR_NDOF_ROOT; ++k) H[j * nv + k] = chain6(K->S[k], Fj);
  }
  for (int i = 1; i < m->num_links; ++i) {
    int j = OR_NDOF_ROOT + i - 1;
    H[j * nv + j] += m->armature[i];
  }
}

static void link_velocities(const or_model_t* m, const kin_t* K, const float* u, float V[][6]) {
  const float* c0 = K->c0;
  float wxc[3];
  cross(c0, u + 3, wxc);
  for (int k = 0; k < 3; ++k) { V[0][k] = u[3 + k]; V[0][3 + k] = u[k] + wxc[k]; }
  for (int i = 1; i < K->nl; ++i) {
    float qd = u[OR_NDOF_ROOT + i - 1];
    const float* S = K->S[OR_NDOF_ROOT + i - 1];
    for (int k = 0; k < 6; ++k) V[i][k] = V[m->parent[i]][k] + S[k] * qd;
  }
}

static void rnea_bias(const or_model_t* m, const kin_t* K, const float* u, float gravity, float* C) {
  float V[OR_MAX_LINKS][6], A[OR_MAX_LINKS][6], fb[OR_MAX_LINKS][6], Fl[OR_MAX_LINKS][6];
  link_velocities(m, K, u, V);
  /* A_0 = [0; v_c0 x w] */
  float vxw[3];
  cross(u, u + 3, vxw);
  for (int k = 0; k < 3; ++k) { A[0][k] = 0.f; A[0][3 + k] = vxw[k]; }
  for (int i = 1; i < K->nl; ++i) {
    float qd = u[OR_NDOF_ROOT + i - 1];
    const float* S = K->S[OR_NDOF_ROOT + i - 1];
    float Sq[6], cr[6];
    for (int k = 0; k < 6; ++k) Sq[k] = S[k] * qd;
    crm(V[i], Sq, cr);
    for (int k = 0; k < 6; ++k) A[i][k] = A[m->parent[i]][k] + cr[k];
  }
  for (int i = 0; i < K->nl; ++i) {
    float IA[6], IV[6], x[6];
    inertia_mul(K->Ib[i], A[i], IA);
    inertia_mul(K->Ib[i], V[i], IV);
    crf(V[i], IV, x);
    float mg[3] = {0.f, 0.f, m->mass[i] * gravity};
    float cxmg[3];
    cross(K->c[i], mg, cxmg);
    for (int k = 0; k < 3; ++k) {
      fb[i][k] = IA[k] + x[k] - cxmg[k];
      fb[i][3 + k] = IA[3 + k] + x[3 + k] - mg[k];
    }
  }
  subtree_sums(m, K->nl, 6, &fb[0][0], &Fl[0][0]);
  for (int j = 0; j < K->nv; ++j) {
    int link = j < OR_NDOF_ROOT ? 0 : j - OR_NDOF_ROOT + 1;
    C[j] = dot6(K->S[j], Fl[link]);
  }
}

/* Inverse of the SPD joint-space inertia by the block sweep operator on SWEEP_B x SWEEP_B pivot
 * blocks (no pivoting needed for SPD), in the arithmetic of the HIP kernel (sweep_inverse /
 * block_inverse in csrc/allsteps_kernels.hip).  The matrix is padded to a multiple of SWEEP_B with
 * identity rows/columns at AS_SWEEP_PAD(n), and the blocks are swept last block first (the limbs
 * before the root).  Round on P = {p..p+B-1}: D = (a_PP)^-1 by 2x2-block Schur complement;
 * row'_j = alpha a_ij - sum_c beta_c a_Pc,j for j not in P, row'_P = beta, where
 * (alpha, beta) = (1, a_iP D) for i not in P and (0, -D_t) for pivot row t.  After all rounds
 * a = -H^-1; the result is negated. */
#define SWEEP_B 4
/* 4x4 SPD inverse by 2x2 blocks (Schur complement), the kernel's block_inverse:
 *   M = [A B; C D]: Ai = A^-1, X = Ai B, Y = C Ai, S = D - C X, Si = S^-1,
 *   M^-1 = [Ai + (X Si) Y, -(X Si); -(Si Y), Si]. */
static void inv2(float a, float b, float c, float d, float o[2][2]) {
  const float id = 1.0f / fmaf(a, d, -(b * c));
  o[0][0] = d * id; o[0][1] = -b * id; o[1][0] = -c * id; o[1][1] = a * id;
}
static void mul2(const float x[2][2], const float y[2][2], float o[2][2]) {
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j) o[i][j] = fmaf(x[i][1], y[1][j], x[i][0] * y[0][j]);
}
static void block_inverse(float M[SWEEP_B][SWEEP_B]) {
  float A[2][2] = {{M[0][0], M[0][1]}, {M[1][0], M[1][1]}};
  float Bm[2][2] = {{M[0][2], M[0][3]}, {M[1][2], M[1][3]}};
  float C[2][2] = {{M[2][0], M[2][1]}, {M[3][0], M[3][1]}};
  float D[2][2] = {{M[2][2], M[2][3]}, {M[3][2], M[3][3]}};
  float Ai[2][2], X[2][2], Y[2][2], CX[2][2], S[2][2], Si[2][2], XS[2][2], XSY[2][2], SY[2][2];
  inv2(A[0][0], A[0][1], A[1][0], A[1][1], Ai);
  mul2(Ai, Bm, X);
  mul2(C, Ai, Y);
  mul2(C, X, CX);
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j) S[i][j] = D[i][j] - CX[i][j];
  inv2(S[0][0], S[0][1], S[1][0], S[1][1], Si);
  mul2(X, Si, XS);
  mul2(XS, Y, XSY);
  mul2(Si, Y, SY);
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j) {
      M[i][j] = Ai[i][j] + XSY[i][j];
      M[i][2 + j] = -XS[i][j];
      M[2 + i][j] = -SY[i][j];
      M[2 + i][2 + j] = Si[i][j];
    }
}

/* dof k's row / column in the padded order (AS_SWEEP_PAD, include/as_detmath.h) */
static int sweep_padded(int k, int n, int np) { return k < AS_SWEEP_PAD(n) ? k : k + (np - n); }

static void sweep_inverse(float* h, int n) {
  const int np = (n + SWEEP_B - 1) / SWEEP_B * SWEEP_B;
  float a[NV_MAX + SWEEP_B][NV_MAX + SWEEP_B];
  float out[NV_MAX + SWEEP_B];
  for (int i = 0; i < np; ++i)
    for (int j = 0; j < np; ++j) a[i][j] = i == j ? 1.f : 0.f;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) a[sweep_padded(i, n, np)][sweep_padded(j, n, np)] = h[i * n + j];
  /* the last pivot block first (the kernel's round order) */
  for (int p = np - SWEEP_B; p >= 0; p -= SWEEP_B) {
    float D[SWEEP_B][SWEEP_B], Q[SWEEP_B][NV_MAX + SWEEP_B];
    for (int x = 0; x < SWEEP_B; ++x)
      for (int c = 0; c < SWEEP_B; ++c) D[x][c] = a[p + x][p + c];
    block_inverse(D);
    for (int x = 0; x < SWEEP_B; ++x)
      for (int j = 0; j < np; ++j) Q[x][j] = a[p + x][j];
    for (int i = 0; i < np; ++i) {
      const int t = i - p;
      const int piv = t >= 0 && t < SWEEP_B;
      float alpha = piv ? 0.f : 1.f, beta[SWEEP_B];
      for (int c = 0; c < SWEEP_B; ++c) {
        float v = 0.f;
        for (int e = 0; e < SWEEP_B; ++e) v = fmaf(a[i][p + e], D[e][c], v);
        beta[c] = piv ? -D[t][c] : v;
      }
      for (int j = 0; j < np; ++j) {
        if (j >= p && j < p + SWEEP_B) {
          out[j] = beta[j - p];
        } else {
          float v = alpha * a[i][j];
          for (int c = 0; c < SWEEP_B; ++c) v = fmaf(-beta[c], Q[c][j], v);
          out[j] = v;
        }
      }
      for (int j = 0; j < np; ++j) a[i][j] = out[j];
    }
  }
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) h[i * n + j] = -a[sweep_padded(i, n, np)][sweep_padded(j, n, np)];
}

/* x = A b (row-major, fmaf chain ascending in k) */
static void matvec_n(const float* A, int n, const float* b, float* x) {
  for (int i = 0; i < n; ++i) {
    float s = 0.f;
    for (int k = 0; k < n; ++k) s = fmaf(A[i * n + k], b[k], s);
    x[i] = s;
  }
}

/* ---------------------------------------------------------------- collision (boxes, spheres, capsules) */

/* signed distance from p to an axis-aligned box (center c, half extents h); normal out of box */
/* Slope sign carrier of t -> sd_box(a + t (b - a)), convex in t: outside the box (some slab
 * distance d_k > 0) sum_k o_k s_k D_k (half the derivative of the squared distance, o_k = max(d_k, 0)),
 * inside s_ax D_ax of the deepest slab (ties to the lowest axis).  Only its sign is used.  The point
 * offset is fmaf(t, D, a - c), the sum an fmaf chain: the HIP kernel's form (allsteps_device.h). */
static float sd_box_slope(const float a[3], const float b[3], float t, const float c[3], const float h[3]) {
  float d[3], sD[3];
  for (int k = 0; k < 3; ++k) {
    const float D = b[k] - a[k];
    const float r = fmaf(t, D, a[k] - c[k]);
    sD[k] = r >= 0.f ? D : -D;
    d[k] = fabsf(r) - h[k];
  }
  if (fmaxf(d[0], fmaxf(d[1], d[2])) > 0.f) {
    float o0 = d[0] > 0.f ? d[0] : 0.f, o1 = d[1] > 0.f ? d[1] : 0.f, o2 = d[2] > 0.f ? d[2] : 0.f;
    return fmaf(o2, sD[2], fmaf(o1, sD[1], o0 * sD[0]));
  }
  int ax = 0;
  if (d[1] > d[ax]) ax = 1;
  if (d[2] > d[ax]) ax = 2;
  return sD[ax];
}

static float sd_box(const float p[3], const float c[3], const float h[3], float nrm[3]) {
  float d[3], s[3];
  for (int k = 0; k < 3; ++k) {
    float r = p[k] - c[k];
    s[k] = r >= 0.f ? 1.f : -1.f;
    d[k] = fabsf(r) - h[k];
  }
  float o0 = d[0] > 0.f ? d[0] : 0.f, o1 = d[1] > 0.f ? d[1] : 0.f, o2 = d[2] > 0.f ? d[2] : 0.f;
  float out = sqrtf(o0 * o0 + o1 * o1 + o2 * o2);
  if (out > 0.f) {
    float inv = 1.0f / out;
    nrm[0] = s[0] * o0 * inv; nrm[1] = s[1] * o1 * inv; nrm[2] = s[2] * o2 * inv;
    return out;
  }
  int ax = 0;
  if (d[1] > d[ax]) ax = 1;
  if (d[2] > d[ax]) ax = 2;
  nrm[0] = nrm[1] = nrm[2] = 0.f;
  nrm[ax] = s[ax];
  return d[ax];
}

#ifdef OR_STATS
long long or_stats_hist[6][256];
#endif

static __thread or_probe_t* g_probe; /* or_probe_substep: record this substep, find every contact */

typedef struct {
  int n, tried, tried_self; /* tried: contacts found before the cap (statistics, probe) */
  int link[OR_MAX_CONTACTS], link2[OR_MAX_CONTACTS], stone[OR_MAX_CONTACTS], foot[OR_MAX_CONTACTS];
  float pt[OR_MAX_CONTACTS][3], nrm[OR_MAX_CONTACTS][3], sep[OR_MAX_CONTACTS];
} contacts_t;

/* link2 = -1 for a stone contact (the stone is kinematic), else the second robot link of a
 * self-contact (stone = foot = -1), which takes the opposite impulse */
static void add_contact(contacts_t* C, int ncap, int link, int link2, int stone, int foot, const float P[3],
                        const float nrm[3], float sep, float r) {
  C->tried++;
  C->tried_self += stone < 0;
  if (C->n >= ncap) return;
  int c = C->n++;
  C->link[c] = link; C->link2[c] = link2; C->stone[c] = stone; C->foot[c] = foot; C->sep[c] = sep;
  for (int k = 0; k < 3; ++k) { C->nrm[c][k] = nrm[k]; C->pt[c][k] = P[k] - nrm[k] * r; }
}

#define BISECT_ITERS 12

/* Contacts of one substep, at most ncap, in priority order (the HIP kernel's collide() emits the same
 * list):
 *   1. the priority geoms (the feet, geoms [0, num_priority_geoms)) against the candidate stones,
 *      stone-major (ascending), geom-minor;
 *   2. every other geom against the candidate stones, stone-major, geom-minor;
 *   3. robot self-contacts, one per self-collision pair in table order (model self_pair). */
static void collide(const or_model_t* m, const or_sim_t* sim, const kin_t* K, const float* stones_rel, int nst,
                    int ncap, contacts_t* C) {
  C->n = C->tried = C->tried_self = 0;
#ifdef OR_STATS
  ncap = OR_MAX_CONTACTS; /* find everything, keep ncap (below) */
#endif
  const int keep = ncap;          /* add_contact keeps ncap; the search runs to the end and counts the */
  ncap = 1 << 30;                 /* contacts past the cap (tried - n: dropped, as_step_counters [3]) */

  const float* h = sim->stone_half;
  /* geom segments in the O frame, their midpoints / lengths, and the robot's bounding box */
  float ga[OR_MAX_GEOMS][3], gb[OR_MAX_GEOMS][3], gL[OR_MAX_GEOMS], gm[OR_MAX_GEOMS][3];
  float blo[3] = {1e30f, 1e30f, 1e30f}, bhi[3] = {-1e30f, -1e30f, -1e30f};
  for (int g = 0; g < m->num_geoms; ++g) {
    int l = m->geom_link[g];
    float t0[3], t1[3];
    matvec3(K->R[l], m->geom_p0[g], t0);
    matvec3(K->R[l], m->geom_p1[g], t1);
    for (int k = 0; k < 3; ++k) { ga[g][k] = K->p[l][k] + t0[k]; gb[g][k] = K->p[l][k] + t1[k]; }
    const float* a = ga[g];
    const float* b = gb[g];
    gL[g] = sqrtf((b[0] - a[0]) * (b[0] - a[0]) + (b[1] - a[1]) * (b[1] - a[1]) + (b[2] - a[2]) * (b[2] - a[2]));
    for (int k = 0; k < 3; ++k) gm[g][k] = 0.5f * (a[k] + b[k]);
    const float r = m->geom_radius[g];
    for (int k = 0; k < 3; ++k) {
      const float e = m->geom_type[g] == 0 ? a[k] : fminf(a[k], b[k]);
      const float f = m->geom_type[g] == 0 ? a[k] : fmaxf(a[k], b[k]);
      blo[k] = fminf(blo[k], e - r);
      bhi[k] = fmaxf(bhi[k], f + r);
    }
  }
  /* broadphase: stones whose box comes within the margin of the robot's bounding box (conservative:
   * every (stone, geom) pair the narrowphase would turn into a contact survives) */
  int cand[OR_MAX_STONES], nc = 0;
  for (int s = 0; s < nst; ++s) {
    const float* c = stones_rel + 3 * s;
    int in = 1;
    for (int k = 0; k < 3; ++k)
      in = in && (c[k] - h[k] <= bhi[k] + sim->margin) && (c[k] + h[k] >= blo[k] - sim->margin);
    if (in) cand[nc++] = s;
  }
  const int npri = m->num_priority_geoms;
  for (int cls = 0; cls < 2; ++cls) {
    const int g0 = cls == 0 ? 0 : npri, g1 = cls == 0 ? npri : m->num_geoms;
    for (int ci = 0; ci < nc && C->n < ncap; ++ci) {
      int s = cand[ci];
      const float* c = stones_rel + 3 * s;
      for (int g = g0; g < g1; ++g) {
        int l = m->geom_link[g];
        float r = m->geom_radius[g];
        const float* a = ga[g];
        const float* b = gb[g];
        float nr[3];
        if (m->geom_type[g] == 0) {
          float sd = sd_box(a, c, h, nr) - r;
          if (sd < sim->margin) add_contact(C, keep, l, -1, s, m->geom_foot[g], a, nr, sd, r);
          continue;
        }
        /* capsule: bounding test on the segment midpoint */
        float nm[3];
        if (sd_box(gm[g], c, h, nm) > 0.5f * gL[g] + r + sim->margin) continue;
        float n0[3], n1[3];
        float s0 = sd_box(a, c, h, n0) - r;
        float s1 = sd_box(b, c, h, n1) - r;
        /* minimum of the (convex) sd along the segment: bisection on the sign of its slope
         * (sd_box_slope), BISECT_ITERS rounds, the HIP kernel's form */
        float lo = 0.f, hi = 1.f;
        for (int it = 0; it < BISECT_ITERS; ++it) {
          const float t = 0.5f * (lo + hi);
          if (sd_box_slope(a, b, t, c, h) > 0.f) hi = t; else lo = t;
        }
        float ts = 0.5f * (lo + hi), Ps[3], ns[3];
        for (int k = 0; k < 3; ++k) Ps[k] = a[k] + ts * (b[k] - a[k]);
        float ss = sd_box(Ps, c, h, ns) - r;
        if (s0 < sim->margin) add_contact(C, keep, l, -1, s, m->geom_foot[g], a, n0, s0, r);
        if (s1 < sim->margin) add_contact(C, keep, l, -1, s, m->geom_foot[g], b, n1, s1, r);
        float smin = s0 < s1 ? s0 : s1;
        if (ss < sim->margin && ss < smin - 0.002f) add_contact(C, keep, l, -1, s, m->geom_foot[g], Ps, ns, ss, r);
      }
    }
  }
  /* self-contacts: bounding-sphere filter, then the capsule-capsule closest points (as_detmath.h) */
#ifdef OR_STATS
  int nbound = 0;
#endif
  for (int p = 0; p < m->num_self_pairs && C->n < ncap; ++p) {
    const int g1 = m->self_pair[p] & 0xff, g2 = m->self_pair[p] >> 8;
    const float R1 = 0.5f * gL[g1] + m->geom_radius[g1], R2 = 0.5f * gL[g2] + m->geom_radius[g2];
    if (!as_sphere_bound(gm[g1], R1, gm[g2], R2, sim->margin)) continue;
#ifdef OR_STATS
    nbound++;
#endif
    float P[3], n[3];
    const float sep = as_capsule_contact(ga[g1], gb[g1], m->geom_radius[g1], ga[g2], gb[g2], m->geom_radius[g2], P, n);
    if (sep < sim->margin) {
#ifdef OR_STATS
      or_stats_hist[4][p]++;
#endif
      add_contact(C, keep, m->geom_link[g1], m->geom_link[g2], -1, -1, P, n, sep, 0.f);
    }
  }
#ifdef OR_STATS
  or_stats_hist[5][nbound < 255 ? nbound : 255]++;
#endif
}

/* ---------------------------------------------------------------- one env step (decimation substeps) */

typedef struct {
  int nrow;
  int type[OR_MAX_ROWS];     /* 0 normal, 1 tangent, 2 limit */
  int contact[OR_MAX_ROWS];
  float target[OR_MAX_ROWS];
  float J[OR_MAX_ROWS][NV_MAX];
  float W[OR_MAX_ROWS][NV_MAX];
  float Ad[OR_MAX_ROWS];
  float lam[OR_MAX_ROWS];
} rows_t;

/* J_j = S_j . f6 (f6 = [P x d; d]) for the dofs on link's path, minus the same for link2's path (a
 * self-contact's second body takes the opposite impulse; dofs on both paths cancel to 0) */
static void contact_row(const or_model_t* m, const kin_t* K, int link, int link2, const float P[3], const float d[3],
                        float* J) {
  float f6[6];
  cross(P, d, f6);
  f6[3] = d[0]; f6[4] = d[1]; f6[5] = d[2];
  int on1[NV_MAX] = {0}, on2[NV_MAX] = {0};
  int chain[NV_MAX];
  int nc = chain_dofs(m, link, chain);
  for (int t = 0; t < nc; ++t) on1[chain[t]] = 1;
  if (link2 >= 0) {
    nc = chain_dofs(m, link2, chain);
    for (int t = 0; t < nc; ++t) on2[chain[t]] = 1;
  }
  for (int j = 0; j < K->nv; ++j) {
    const float v = chain6(K->S[j], f6);  /* the kernel's MFMA chain */
    J[j] = (on1[j] ? v : 0.f) - (on2[j] ? v : 0.f);
  }
}

static void tangents(const float n[3], float t1[3], float t2[3]) {
  float e[3] = {1.f, 0.f, 0.f};
  if (fabsf(n[0]) > 0.9f) { e[0] = 0.f; e[1] = 1.f; }
  cross(n, e, t1);
  float inv = 1.0f / sqrtf(dot3(t1, t1));
  for (int k = 0; k < 3; ++k) t1[k] *= inv;
  cross(n, t1, t2);
}

/* returns the contacts the row budget cut in this substep (found - kept) */
static int substep(const or_model_t* m, const or_sim_t* sim, const or_actuator_t* act, const float* qt_int,
                    float root_pos[3], float root_quat[4], float* q_int, float* u, float* tau_int,
                    const float* stones_w, int nst, uint32_t mask[4]) {
  if (act && act->mode == 1) /* the DC motor runs in every substep (as_dc_motor, include/as_detmath.h) */
    for (int i = 0; i < m->num_hinges; ++i)
      tau_int[i] = as_dc_motor(qt_int[i], q_int[i], u[OR_NDOF_ROOT + i], act->stiffness, act->damping,
                               act->saturation_effort, act->effort_limit, act->velocity_limit);
  kin_t K;
  kinematics(m, root_quat, q_int, &K);
  const int nv = K.nv, nh = m->num_hinges;
  const float dt = sim->dt;
  float H[NV_MAX * NV_MAX], C[NV_MAX], b[NV_MAX], acc[NV_MAX];
  crba(m, &K, H);
  rnea_bias(m, &K, u, sim->gravity, C);
  for (int j = 0; j < nv; ++j) b[j] = (j < OR_NDOF_ROOT ? 0.f : tau_int[j - OR_NDOF_ROOT]) - C[j];
  sweep_inverse(H, nv); /* H <- H^-1 */
  matvec_n(H, nv, b, acc);
  for (int j = 0; j < nv; ++j) u[j] = fmaf(dt, acc[j], u[j]);

  /* constraints: joint-limit rows first counted (all of them are kept), then the contacts fill the
   * remaining rows; rows are ordered contacts (normal, tangent, tangent) then limits (hinge order,
   * lower before upper) */
  int lim_dof[OR_MAX_ROWS], lim_side[OR_MAX_ROWS], nlim = 0;
  for (int i = 1; i <= nh; ++i) {
    int j = OR_NDOF_ROOT + i - 1;
    float qv = q_int[i - 1], pred = qv + dt * u[j];
    for (int side = 0; side < 2; ++side) {
      int viol = side == 0 ? pred < m->lower[i] : pred > m->upper[i];
      if (!viol || nlim >= OR_MAX_ROWS) continue;
      lim_dof[nlim] = i;
      lim_side[nlim++] = side;
    }
  }
  int ncap = (OR_MAX_ROWS - nlim) / 3;
  if (ncap > OR_MAX_CONTACTS) ncap = OR_MAX_CONTACTS;
  float stones_rel[OR_MAX_STONES * 3];
  for (int s = 0; s < nst; ++s)
    for (int k = 0; k < 3; ++k) stones_rel[3 * s + k] = stones_w[3 * s + k] - root_pos[k];
  contacts_t Cn;
  collide(m, sim, &K, stones_rel, nst, ncap, &Cn);
  if (g_probe && !g_probe->recorded) {
    or_probe_t* P = g_probe;
    P->nfound = Cn.tried; P->nself_found = Cn.tried_self; P->ncap = ncap; P->nlim = nlim; P->ncontact = Cn.n;
    for (int c = 0; c < Cn.n; ++c) {
      P->link[c] = Cn.link[c]; P->link2[c] = Cn.link2[c]; P->stone[c] = Cn.stone[c]; P->foot[c] = Cn.foot[c];
      P->sep[c] = Cn.sep[c];
      for (int k = 0; k < 3; ++k) P->nrm[c][k] = Cn.nrm[c][k];
    }
  }
#ifdef OR_STATS
  or_stats_hist[0][Cn.tried < 255 ? Cn.tried : 255]++;
  or_stats_hist[1][nlim]++;
  or_stats_hist[3][Cn.tried_self < 255 ? Cn.tried_self : 255]++;
  if (Cn.n > ncap) Cn.n = ncap;
  or_stats_hist[2][Cn.n]++;
#endif
  const int dropped = Cn.tried - Cn.n;
  static __thread rows_t Rw;
  rows_t* R = &Rw;
  R->nrow = 0;
  for (int c = 0; c < Cn.n; ++c) {
    float t1[3], t2[3];
    tangents(Cn.nrm[c], t1, t2);
    const float* dirs[3] = {Cn.nrm[c], t1, t2};
    for (int d = 0; d < 3; ++d) {
      int r = R->nrow++;
      R->type[r] = d == 0 ? 0 : 1;
      R->contact[r] = c;
      contact_row(m, &K, Cn.link[c], Cn.link2[c], Cn.pt[c], dirs[d], R->J[r]);
      float s = Cn.sep[c];
      if (d == 0)
        R->target[r] = s < 0.f ? fminf(sim->baumgarte * fmaxf(-s - sim->slop, 0.f) / dt, sim->max_depen_vel)
                               : -s / dt;
      else
        R->target[r] = 0.f;
    }
  }
  for (int l = 0; l < nlim; ++l) {
    const int i = lim_dof[l], side = lim_side[l], j = OR_NDOF_ROOT + i - 1;
    const float qv = q_int[i - 1];
    float err = side == 0 ? m->lower[i] - qv : qv - m->upper[i];
    int r = R->nrow++;
    R->type[r] = 2;
    R->contact[r] = -1;
    for (int k = 0; k < nv; ++k) R->J[r][k] = 0.f;
    R->J[r][j] = side == 0 ? 1.f : -1.f;
    R->target[r] = err > 0.f ? fminf(sim->baumgarte * err / dt, sim->max_depen_vel) : err / dt;
  }
  /* W_r = H^-1 J_r^T (the kernel's w_rows(): f32 MFMA, bit for bit an fmaf chain): W_r[i] = sum_k J_rk
   * (H^-1)_ik as one fmaf chain over k ascending, row i of H^-1 as the sweep left it; rows are padded
   * with +0 to the 16-B width npad.  The projections
   * A_rr = J_r . W_r and the in-triplet couplings A_sr = J_s . W_r (s > r in the same row triplet) as
   * two interleaved partial sums over the padded width (dot_pairs). */
  const int ngrp = (R->nrow + 2) / 3, nr3 = 3 * ngrp;
  const int npad = (nv + 3) / 4 * 4;
  for (int r = R->nrow; r < nr3; ++r) {
    for (int k = 0; k < NV_MAX; ++k) R->J[r][k] = 0.f;
    R->type[r] = 0;
    R->target[r] = 0.f;
  }
  float cpl[OR_MAX_ROWS + 3];
  for (int r = 0; r < nr3; ++r) {
    for (int k = nv; k < npad; ++k) R->J[r][k] = 0.f;
    for (int i = 0; i < npad; ++i) {
      float w = 0.f;
      if (i < nv)
        for (int k = 0; k < nv; ++k) w = fmaf(R->J[r][k], H[i * nv + k], w);
      R->W[r][i] = w;
    }
    R->Ad[r] = r < R->nrow ? 1.0f / (dot_pairs(R->J[r], R->W[r], npad) + 1e-9f) : 0.f;
    R->lam[r] = 0.f;
  }
  for (int g = 0; g < ngrp; ++g) {
    const int r0 = 3 * g;
    const int ps[3][2] = {{1, 0}, {2, 0}, {2, 1}}; /* (s, r): A_10, A_20, A_21 */
    for (int c = 0; c < 3; ++c) cpl[r0 + c] = dot_pairs(R->J[r0 + ps[c][0]], R->W[r0 + ps[c][1]], npad);
  }
  /* projected Gauss-Seidel, row triplets (the kernel's PGS loop): the three velocities J_r . u of a
   * triplet come from the u at its start, rows 2 and 3 add the in-triplet couplings of this sweep's
   * impulse changes; t = lambda + (target - v) / A_rr as fmaf chains; normal and limit rows clamp to
   * [0, inf), tangent rows to +-mu * (the latest normal impulse). */
  for (int it = 0; it < sim->pgs_iters; ++it) {
    float ln = 0.f;
    for (int g = 0; g < ngrp; ++g) {
      const int r0 = 3 * g;
      float vg[3];
      for (int c = 0; c < 3; ++c) {
        float pr[32] = {0.f};
        for (int k = 0; k < nv; ++k) pr[k] = R->J[r0 + c][k] * u[k];
        vg[c] = tree32(pr);
      }
      const float* x = R->Ad + r0;
      const float* y = R->target + r0;
      const float k10 = x[1] * cpl[r0], k20 = x[2] * cpl[r0 + 1], k21 = x[2] * cpl[r0 + 2];
      float t[3];
      for (int c = 0; c < 3; ++c) t[c] = fmaf(-vg[c], x[c], fmaf(y[c], x[c], R->lam[r0 + c]));
      for (int c = 0; c < 3; ++c) {
        const int r = r0 + c;
        float l1;
        if (R->type[r] == 1) {
          const float lo = fmaf(-sim->friction, ln, 0.f), hi = fmaf(sim->friction, ln, 0.f);
          l1 = t[c] < lo ? lo : (t[c] > hi ? hi : t[c]);
        } else {
          l1 = t[c] > 0.f ? t[c] : 0.f;
        }
        if (R->type[r] == 0) ln = l1;
        const float dl = l1 - R->lam[r];
        R->lam[r] = l1;
        if (c == 0) { t[1] = fmaf(-k10, dl, t[1]); t[2] = fmaf(-k20, dl, t[2]); }
        if (c == 1) t[2] = fmaf(-k21, dl, t[2]);
        for (int k = 0; k < nv; ++k) u[k] = fmaf(R->W[r][k], dl, u[k]);
      }
    }
  }
  /* contact sensor flags of this substep: |sum_n lambda_n n| / dt > eps per (foot, stone) */
  mask[0] = mask[1] = mask[2] = mask[3] = 0u;
  for (int c = 0; c < Cn.n; ++c) {
    if (Cn.foot[c] < 0) continue;
    float fx = 0.f, fy = 0.f, fz = 0.f;
    for (int c2 = 0; c2 < Cn.n; ++c2) {
      if (Cn.foot[c2] != Cn.foot[c] || Cn.stone[c2] != Cn.stone[c]) continue;
      float l = R->lam[3 * c2];
      fx += l * Cn.nrm[c2][0]; fy += l * Cn.nrm[c2][1]; fz += l * Cn.nrm[c2][2];
    }
    float fn = sqrtf(fx * fx + fy * fy + fz * fz) / dt;
    if (fn > 1e-4f) mask[Cn.foot[c] & 3] |= 1u << Cn.stone[c];
  }
  if (g_probe) {
    or_probe_t* P = g_probe;
    if (!P->recorded) {
      for (int c = 0; c < Cn.n; ++c) P->lam_n[c] = R->lam[3 * c];
      P->mask[0] = mask[0];
      P->mask[1] = mask[1];
      P->recorded = 1;
    }
    for (int c = 0; c < Cn.n; ++c) {
      if (Cn.stone[c] < 0) continue;
      for (int k = 0; k < 3; ++k) {
        P->stone_impulse[Cn.stone[c]][k] += R->lam[3 * c] * Cn.nrm[c][k];
        P->net_impulse[k] += R->lam[3 * c] * Cn.nrm[c][k];
      }
    }
  }
  /* clamp joint speeds, integrate */
  for (int i = 0; i < nh; ++i) {
    float* v = &u[OR_NDOF_ROOT + i];
    if (*v > sim->max_joint_vel) *v = sim->max_joint_vel;
    if (*v < -sim->max_joint_vel) *v = -sim->max_joint_vel;
    q_int[i] = fmaf(dt, *v, q_int[i]);
  }
  float c0w[3];
  for (int k = 0; k < 3; ++k) c0w[k] = fmaf(dt, u[k], root_pos[k] + K.c0[k]);
  const float* w = u + 3;
  float wn = sqrtf(dot3(w, w));
  float th = wn * dt, dq[4];
  if (th > 1e-12f) {
    float sn, cs;
    as_sincosf(0.5f * th, &sn, &cs);
    float s = sn / wn;
    dq[0] = cs; dq[1] = w[0] * s; dq[2] = w[1] * s; dq[3] = w[2] * s;
  } else {
    dq[0] = 1.f; dq[1] = 0.5f * dt * w[0]; dq[2] = 0.5f * dt * w[1]; dq[3] = 0.5f * dt * w[2];
  }
  const float* q0 = root_quat;
  float nq[4] = {dq[0] * q0[0] - dq[1] * q0[1] - dq[2] * q0[2] - dq[3] * q0[3],
                 dq[0] * q0[1] + dq[1] * q0[0] + dq[2] * q0[3] - dq[3] * q0[2],
                 dq[0] * q0[2] - dq[1] * q0[3] + dq[2] * q0[0] + dq[3] * q0[1],
                 dq[0] * q0[3] + dq[1] * q0[2] - dq[2] * q0[1] + dq[3] * q0[0]};
  float qn = 1.0f / sqrtf(nq[0] * nq[0] + nq[1] * nq[1] + nq[2] * nq[2] + nq[3] * nq[3]);
  for (int k = 0; k < 4; ++k) root_quat[k] = nq[k] * qn;
  float Rn[9], cl[3];
  quat_to_mat(root_quat, Rn);
  matvec3(Rn, m->com[0], cl);
  for (int k = 0; k < 3; ++k) root_pos[k] = c0w[k] - cl[k];
  return dropped;
}

void or_fk_bodies(const or_model_t* m, const float root_pos[3], const float root_quat[4], const float* q_cfg,
                  float body_pos[9]) {
  float q_int[OR_MAX_LINKS];
  for (int k = 0; k < m->num_hinges; ++k) q_int[m->cfg_dof_link[k] - 1] = q_cfg[k];
  kin_t K;
  kinematics(m, root_quat, q_int, &K);
  int ls[3] = {m->torso_link, m->foot_link[0], m->foot_link[1]};
  for (int b = 0; b < 3; ++b)
    for (int k = 0; k < 3; ++k) body_pos[3 * b + k] = root_pos[k] + K.p[ls[b]][k];
}

int or_physics_step_act(const or_model_t* m, const or_sim_t* sim, const or_task_t* task, const or_actuator_t* act,
                        or_state_t* st, int e, const float* act_clamped) {
  const int n = st->n, nh = m->num_hinges;
  float rp[3], rq[4], q_int[OR_MAX_LINKS], u[NV_MAX], tau[OR_MAX_LINKS], qt[OR_MAX_LINKS], stones[OR_MAX_STONES * 3];
  for (int k = 0; k < 3; ++k) rp[k] = F(st->root_pos, k, n, e);
  for (int k = 0; k < 4; ++k) rq[k] = F(st->root_quat, k, n, e);
  for (int k = 0; k < 3; ++k) { u[k] = F(st->root_lin, k, n, e); u[3 + k] = F(st->root_ang, k, n, e); }
  /* ENV:270-274 _apply_action: tau = gain[curriculum] * gear * a (ImplicitActuator pass-through); with a
   * DC motor, position targets default + scale a (anymal_c_env.py:73-74) */
  float gain = task->gain_curriculum[st->curriculum[0]];
  for (int k = 0; k < nh; ++k) {
    int i = m->cfg_dof_link[k] - 1;
    q_int[i] = F(st->q, k, n, e);
    u[OR_NDOF_ROOT + i] = F(st->qd, k, n, e);
    tau[i] = gain * m->gear[k] * act_clamped[k];
    qt[i] = act ? act->action_scale * act_clamped[k] + act->default_q[k] : 0.f;
  }
  const int nst = task->num_steps;
  for (int s = 0; s < nst; ++s)
    for (int k = 0; k < 3; ++k) stones[3 * s + k] = F(st->stones, s * 3 + k, n, e);
  uint32_t mask[4] = {0u, 0u, 0u, 0u};
  int dropped = 0;
  for (int s = 0; s < sim->substeps; ++s) dropped += substep(m, sim, act, qt, rp, rq, q_int, u, tau, stones, nst, mask);
  for (int k = 0; k < 3; ++k) {
    F(st->root_pos, k, n, e) = rp[k];
    F(st->root_lin, k, n, e) = u[k];
    F(st->root_ang, k, n, e) = u[3 + k];
  }
  for (int k = 0; k < 4; ++k) F(st->root_quat, k, n, e) = rq[k];
  for (int k = 0; k < nh; ++k) {
    int i = m->cfg_dof_link[k] - 1;
    F(st->q, k, n, e) = q_int[i];
    F(st->qd, k, n, e) = u[OR_NDOF_ROOT + i];
  }
  F(st->contact_mask, 0, n, e) = mask[0];
  F(st->contact_mask, 1, n, e) = mask[1];
  if (st->contact_mask_hind) {
    F(st->contact_mask_hind, 0, n, e) = mask[2];
    F(st->contact_mask_hind, 1, n, e) = mask[3];
  }
  float bp[9], qc[OR_MAX_LINKS];
  for (int k = 0; k < nh; ++k) qc[k] = F(st->q, k, n, e);
  or_fk_bodies(m, rp, rq, qc, bp);
  for (int c = 0; c < 9; ++c) F(st->body_pos, c, n, e) = bp[c];
  return dropped;
}

/* known-answer hook: the DC motor torque of include/as_detmath.h for n inputs */
void or_dc_motor_batch(int n, const float* qt, const float* q, const float* qd, const or_actuator_t* act, float* tau) {
  for (int i = 0; i < n; ++i)
    tau[i] = as_dc_motor(qt[i], q[i], qd[i], act->stiffness, act->damping, act->saturation_effort, act->effort_limit,
                         act->velocity_limit);
}

int or_physics_step(const or_model_t* m, const or_sim_t* sim, const or_task_t* task, or_state_t* st, int e,
                    const float* act_clamped) {
  return or_physics_step_act(m, sim, task, NULL, st, e, act_clamped);
}

/* ---------------------------------------------------------------- env-level API */

void or_probe_substep(const or_model_t* m, const or_sim_t* sim, const or_task_t* task, const or_state_t* st, int e,
                      const float* act_clamped, or_probe_t* out) {
  /* the env's state as or_physics_step loads it, one substep, nothing written back */
  const int n = st->n, nh = m->num_hinges;
  float rp[3], rq[4], q_int[OR_MAX_LINKS], u[NV_MAX], tau[OR_MAX_LINKS], stones[OR_MAX_STONES * 3];
  for (int k = 0; k < 3; ++k) rp[k] = F(st->root_pos, k, n, e);
  for (int k = 0; k < 4; ++k) rq[k] = F(st->root_quat, k, n, e);
  for (int k = 0; k < 3; ++k) { u[k] = F(st->root_lin, k, n, e); u[3 + k] = F(st->root_ang, k, n, e); }
  float gain = task->gain_curriculum[st->curriculum[0]];
  for (int k = 0; k < nh; ++k) {
    int i = m->cfg_dof_link[k] - 1;
    q_int[i] = F(st->q, k, n, e);
    u[OR_NDOF_ROOT + i] = F(st->qd, k, n, e);
    tau[i] = gain * m->gear[k] * act_clamped[k];
  }
  const int nst = task->num_steps;
  for (int s = 0; s < nst; ++s)
    for (int k = 0; k < 3; ++k) stones[3 * s + k] = F(st->stones, s * 3 + k, n, e);
  memset(out, 0, sizeof(*out));
  uint32_t mask[4] = {0u, 0u, 0u, 0u};
  g_probe = out;
  for (int sub = 0; sub < sim->substeps; ++sub) substep(m, sim, NULL, NULL, rp, rq, q_int, u, tau, stones, nst, mask);
  g_probe = NULL;
}

void or_env_step(const or_model_t* m, const or_sim_t* sim, const or_task_t* task, or_state_t* st,
                 const float* actions, const float* reset_draws, uint64_t seed, float* obs, float* rew,
                 uint8_t* term, uint8_t* trunc, int32_t* any_reset, int64_t* dropped, int nthreads) {
  const int n = st->n;
  (void)nthreads;
  long long drop = 0;
#pragma omp parallel for num_threads(nthreads > 0 ? nthreads : 1) schedule(static) reduction(+ : drop)
  for (int e = 0; e < n; ++e) {
    float a[OR_MAX_LINKS];
    for (int k = 0; k < m->num_hinges; ++k) {
      float x = actions[(size_t)e * m->num_hinges + k];
      a[k] = x < -1.f ? -1.f : (x > 1.f ? 1.f : x);
    }
    drop += or_physics_step(m, sim, task, st, e, a);
  }
  if (dropped) *dropped = drop;
  or_task_post_physics(m, task, st, actions, NULL, NULL, reset_draws, seed, NULL, NULL, obs, rew, term, trunc,
                       any_reset);
}

void or_env_reset_all(const or_model_t* m, const or_sim_t* sim, const or_task_t* task, or_state_t* st,
                      const float* reset_draws, uint64_t seed, float* obs) {
  (void)sim;
  or_task_reset_all(m, task, st, reset_draws, seed, obs);
}

/* ---------------------------------------------------------------- known-answer test hooks */

void or_mass_matrix(const or_model_t* m, const float root_pos[3], const float root_quat[4], const float* q_int,
                    float* H, float* com0) {
  (void)root_pos;
  kin_t K;
  kinematics(m, root_quat, q_int, &K);
  crba(m, &K, H);
  for (int k = 0; k < 3; ++k) com0[k] = K.c[0][k];
}

void or_bias_forces(const or_model_t* m, const float root_pos[3], const float root_quat[4], const float* q_int,
                    const float* u, float gravity, float* C) {
  (void)root_pos;
  kin_t K;
  kinematics(m, root_quat, q_int, &K);
  rnea_bias(m, &K, u, gravity, C);
}
