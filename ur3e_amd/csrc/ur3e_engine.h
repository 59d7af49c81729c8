/*
 * ur3e_engine.h — per-environment FP64 rigid-body step for gfx950.
 *
 * Execution model: ONE environment per wavefront lane.  Each lane keeps its
 * environment's working set (kinematic tree, mass matrix, contact list,
 * constraint rows, Newton state) in a private `KData` (lane-private scratch,
 * which gfx950 interleaves per lane at dword granularity, i.e. every access is
 * a coalesced 256-B wave transaction).  The model image (ur3e_model_t) is read
 * through wave-uniform addresses, so its loads become scalar (SMEM) loads
 * shared by the 64 lanes.
 *
 * Numerics: every stage below follows the operation order of the CPU oracle
 * (oracle/ur3e_oracle.c) so results are bit-identical; build with
 * -ffp-contract=off.  Where the kernel differs structurally it keeps the
 * per-element accumulation order: e.g. constraint rows compute efc_vel, aref
 * and R at creation (the oracle does it in a second pass), contacts keep a
 * pair index instead of copies of the pair parameters.
 *
 * Semantics: MuJoCo 3.3.3 mj_step as driven by the reference
 * (gymnasium_env/envs/ur3e_env2.py:83 do_simulation; controller/move_l_mug.py:78);
 * see SURVEY.md §2.2 for the stage list.
 */
#ifndef UR3E_ENGINE_H
#define UR3E_ENGINE_H

#include <hip/hip_runtime.h>

#include "../../include/ur3e_model.h"
#include "detmath.h"
#include "convex.h"

/* kernel capacities: the largest reference model (main.xml: nq 21, nv 20, 25 bodies) */
#define K_NQ 21
/* stale-kinematics carry per env: tcp xpos(3), xmat(9), arm Jacobian 6x6, qfrc_bias[0:6] */
#define NCARRY 54
#define K_NV 20
#define K_NB 25
#define K_NJ 16
#define K_NG 16
#define K_NS 12
#define K_NU 7
#define K_MAXCON UR3E_MAXCON
#define K_MAXEFC UR3E_MAXEFC

#define K_MINVAL 1e-15
#define K_MINIMP 0.0001
#define K_MAXIMP 0.9999
#define K_MAXVAL 1e10

#define CN_EQUALITY 0
#define CN_FRICTION_DOF 1
#define CN_LIMIT_JOINT 3
#define CN_CONTACT_ELLIPTIC 7
#define ST_SATISFIED 0
#define ST_QUADRATIC 1
#define ST_LINEARNEG 2
#define ST_LINEARPOS 3
#define ST_CONE 4

#define KD __device__ static inline
#define KDN __device__ static __attribute__((noinline))
/* n / d from r = 1.0 / d (itself a correctly rounded division), d > 0 finite: q0 = n r is within an
   ulp of n / d, the residual d q0 - n is exact in one fma, and q0 - e r rounds to the correctly rounded
   quotient (Markstein's theorem: r within half an ulp of 1/d, q0 within an ulp of n/d; no underflow or
   overflow).  Signed zeros: n = -0 gives q0 = -0, e = +0, -0 - (+0) r = -0, as -0 / d.  Three
   operations instead of the ~11 of a full division, so several quotients by one divisor cost one
   division and three operations each.  The theorem needs the residual to stay out of the subnormal
   range: with |n| below 2^-960 (subnormal numerators included) it does not hold (the host check finds
   one-ulp misses there), nor for |n| above 2^960 or infinite, so those numerators -- never seen on the
   path, but possible -- take the true division behind a branch that no lane normally enters.
   tools/div_rcp_check.c checks the whole function against n / d over random and structured operand
   pairs, subnormal, tiny, huge and infinite numerators included, for the divisor ranges the callers
   use (Cholesky pivots >= sqrt(mjMINVAL), norms >= mjMINVAL; tests/test_div_rcp.py). */
#define K_RCP_NLO 0x1p-960
#define K_RCP_NHI 0x1p+960
/* numerators outside Markstein's range (zero is inside: it gives the signed zero exactly) */
KD bool k_rcp_unsafe(double n) {
  const double an = __builtin_fabs(n);
  return an > 0.0 && (an < K_RCP_NLO || an > K_RCP_NHI);
}
/* the three operations alone: callers that check k_rcp_unsafe on the numerators they keep themselves */
KD double k_div_rcp_raw(double n, double d, double r) {
  const double q0 = n * r;
  const double e = __builtin_fma(d, q0, -n);
  return __builtin_fma(-e, r, q0);
}
KD double k_div_rcp(double n, double d, double r) {
  double q = k_div_rcp_raw(n, d, r);
  if (__builtin_expect(k_rcp_unsafe(n), 0)) q = n / d;
  return q;
}
/* this lane's index within the workgroup, opaque to the optimiser: a value derived from
   threadIdx.x alone is loop-invariant, and LICM would hoist all of them out of the per-substep
   loop and keep them live (spilled) across the whole forward pass; reading the lane through an
   empty asm makes each stage derive its lane constants where it uses them */
__device__ __forceinline__ int w_lane() {
  int l = (int)threadIdx.x;
  asm volatile("" : "+v"(l));
  return l;
}

typedef const ur3e_model_t* __restrict__ KModel;

struct KContact {
  double pos[3];
  double frame[9];
  double dist;
  double mu;
  double friction[5];
  int dim;
  int geom1, geom2;
  int cpair;
  int efc_address;
};

struct KData {
  double qpos[K_NQ];
  double qvel[K_NV];
  double qacc_warmstart[K_NV];
  double ctrl[K_NU];
  /* position stage */
  double xpos[K_NB][3];
  double xquat[K_NB][4];
  double xmat[K_NB][9];
  double xipos[K_NB][3];
  double ximat[K_NB][9];
  double xanchor[K_NJ][3];
  double xaxis[K_NJ][3];
  double geom_xpos[K_NG][3];
  double geom_xmat[K_NG][9];
  double site_xpos[K_NS][3];
  double site_xmat[K_NS][9];
  double subtree_com[K_NB][3];
  double cinert[K_NB][10];
  double cdof[K_NV][6];
  double actuator_length[K_NU];
  double qM[K_NV][K_NV];
  double qLD[K_NV][K_NV];
  double qLDiagInv[K_NV];
  /* contacts */
  int ncon;
  KContact contact[K_MAXCON];
  /* constraint rows */
  int nefc;
  int efc_type[K_MAXEFC];
  int efc_id[K_MAXEFC];
  int efc_state[K_MAXEFC];
  double efc_J[K_MAXEFC][K_NV];
  double efc_R[K_MAXEFC];
  double efc_D[K_MAXEFC];
  double efc_aref[K_MAXEFC];
  double efc_floss[K_MAXEFC];
  double efc_force[K_MAXEFC];
  double touch[UR3E_MAXTOUCH];
  double jar[K_MAXEFC];
  double Jv[K_MAXEFC];
  /* velocity stage */
  double cvel[K_NB][6];
  double cdof_dot[K_NV][6];
  double qfrc_bias[K_NV];
  double qfrc_passive[K_NV];
  double qfrc_smooth[K_NV];
  double qacc_smooth[K_NV];
  double qfrc_constraint[K_NV];
  double qacc[K_NV];
  /* Newton */
  double H[K_NV][K_NV];
  double Ma[K_NV];
  double grad[K_NV];
  double search[K_NV];
  double Mv[K_NV];
  double gauss, cost, scale;
  int nwarn;
};

/* ================================================================== */
/* small vector helpers                                                */
/* ================================================================== */
KD void k_mul_quat(double res[4], const double a[4], const double b[4]) {
  double r0 = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  double r1 = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  double r2 = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  double r3 = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  res[0] = r0; res[1] = r1; res[2] = r2; res[3] = r3;
}

/* The small quaternion helpers below keep MuJoCo's special cases (zero vector, identity quaternion,
   degenerate norm, zero angle) as selects instead of branches: the values are identical, and arrays
   written on both sides of a branch no longer end up in private (scratch) memory. */
KD void k_rot_vec_quat(double res[3], const double v[3], const double q[4]) {
  const double v0 = v[0], v1 = v[1], v2 = v[2];
  const bool vz = v0 == 0 && v1 == 0 && v2 == 0;
  const bool qi = q[0] == 1 && q[1] == 0 && q[2] == 0 && q[3] == 0;
  double t0 = q[0] * v0 + q[2] * v2 - q[3] * v1;
  double t1 = q[0] * v1 + q[3] * v0 - q[1] * v2;
  double t2 = q[0] * v2 + q[1] * v1 - q[2] * v0;
  double r0 = v0 + 2 * (q[2] * t2 - q[3] * t1);
  double r1 = v1 + 2 * (q[3] * t0 - q[1] * t2);
  double r2 = v2 + 2 * (q[1] * t1 - q[2] * t0);
  res[0] = vz ? 0.0 : (qi ? v0 : r0);
  res[1] = vz ? 0.0 : (qi ? v1 : r1);
  res[2] = vz ? 0.0 : (qi ? v2 : r2);
}

KD void k_quat2mat(double r[9], const double q[4]) {
  const bool qi = q[0] == 1 && q[1] == 0 && q[2] == 0 && q[3] == 0;
  double q00 = q[0] * q[0], q01 = q[0] * q[1], q02 = q[0] * q[2], q03 = q[0] * q[3];
  double q11 = q[1] * q[1], q12 = q[1] * q[2], q13 = q[1] * q[3];
  double q22 = q[2] * q[2], q23 = q[2] * q[3], q33 = q[3] * q[3];
  const double m0 = q00 + q11 - q22 - q33;
  const double m4 = q00 - q11 + q22 - q33;
  const double m8 = q00 - q11 - q22 + q33;
  const double m1 = 2 * (q12 - q03);
  const double m2 = 2 * (q13 + q02);
  const double m3 = 2 * (q12 + q03);
  const double m5 = 2 * (q23 - q01);
  const double m6 = 2 * (q13 - q02);
  const double m7 = 2 * (q23 + q01);
  r[0] = qi ? 1.0 : m0; r[1] = qi ? 0.0 : m1; r[2] = qi ? 0.0 : m2;
  r[3] = qi ? 0.0 : m3; r[4] = qi ? 1.0 : m4; r[5] = qi ? 0.0 : m5;
  r[6] = qi ? 0.0 : m6; r[7] = qi ? 0.0 : m7; r[8] = qi ? 1.0 : m8;
}

/* mju_normalize4's tests on n = sqrt(s) as comparisons on s = |q|^2 (sqrt is correctly rounded and
   monotonic): n < K_MINVAL <=> s < K_NRM_TINY, |n - 1| <= K_MINVAL <=> K_NRM_LO <= s <= K_NRM_HI.
   Exact doubles from tools/normalize_thresholds.py (tests/test_normalize_thresholds.py) */
#define K_NRM_TINY 0x1.4484bfeebc2a0p-100
#define K_NRM_LO 0x1.fffffffffffeep-1
#define K_NRM_HI 0x1.0000000000009p+0
KD void k_normalize4(double q[4]) {
  const double a = q[0], b = q[1], c = q[2], d = q[3];
  const double s = a * a + b * b + c * c + d * d;
  const bool tiny = s < K_NRM_TINY;
  double ra = a, rb = b, rc = c, rd = d;
  /* the square root and the divisions stay behind a branch (skipped when no lane needs them: an
     already unit quaternion, the common case); only scalars are assigned in it.  NaN: no rescale,
     as fabs(NaN - 1) > K_MINVAL is false */
  if (!tiny && (s < K_NRM_LO || s > K_NRM_HI)) {
    const double n = sqrt(s);
    const double r = 1.0 / n;
    ra = k_div_rcp(a, n, r); rb = k_div_rcp(b, n, r); rc = k_div_rcp(c, n, r); rd = k_div_rcp(d, n, r);
  }
  q[0] = tiny ? 1.0 : ra;
  q[1] = tiny ? 0.0 : rb;
  q[2] = tiny ? 0.0 : rc;
  q[3] = tiny ? 0.0 : rd;
}

KD double k_normalize3(double v[3]) {
  const double a = v[0], b = v[1], c = v[2];
  double n = sqrt(a * a + b * b + c * c);
  const bool tiny = n < K_MINVAL;
  double ra = 1, rb = 0, rc = 0;
  if (!tiny) {
    const double r = 1.0 / n;
    ra = k_div_rcp(a, n, r); rb = k_div_rcp(b, n, r); rc = k_div_rcp(c, n, r);
  }
  v[0] = tiny ? 1.0 : ra;
  v[1] = tiny ? 0.0 : rb;
  v[2] = tiny ? 0.0 : rc;
  return tiny ? 0.0 : n;
}

KD void k_axis_angle_quat(double q[4], const double axis[3], double angle) {
  double c = 1, x = 0, y = 0, z = 0;
  if (angle != 0) {
    double s = ur3e_sin(angle * 0.5);
    c = ur3e_cos(angle * 0.5);
    x = axis[0] * s; y = axis[1] * s; z = axis[2] * s;
  }
  q[0] = c; q[1] = x; q[2] = y; q[3] = z;
}

KD void k_mat_vec3(double r[3], const double m[9], const double v[3]) {
  double r0 = m[0] * v[0] + m[1] * v[1] + m[2] * v[2];
  double r1 = m[3] * v[0] + m[4] * v[1] + m[5] * v[2];
  double r2 = m[6] * v[0] + m[7] * v[1] + m[8] * v[2];
  r[0] = r0; r[1] = r1; r[2] = r2;
}

KD void k_mat_t_vec3(double r[3], const double m[9], const double v[3]) {
  double r0 = m[0] * v[0] + m[3] * v[1] + m[6] * v[2];
  double r1 = m[1] * v[0] + m[4] * v[1] + m[7] * v[2];
  double r2 = m[2] * v[0] + m[5] * v[1] + m[8] * v[2];
  r[0] = r0; r[1] = r1; r[2] = r2;
}

KD void k_cross3(double r[3], const double a[3], const double b[3]) {
  double r0 = a[1] * b[2] - a[2] * b[1];
  double r1 = a[2] * b[0] - a[0] * b[2];
  double r2 = a[0] * b[1] - a[1] * b[0];
  r[0] = r0; r[1] = r1; r[2] = r2;
}

KD double k_dot3(const double a[3], const double b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

KD void k_local2global(double xp[3], double xm[9], const double bxpos[3], const double bxquat[4],
                       const double bxmat[9], const double lpos[3], const double lquat[4]) {
  double t[3], q[4];
  k_mat_vec3(t, bxmat, lpos);
  xp[0] = bxpos[0] + t[0]; xp[1] = bxpos[1] + t[1]; xp[2] = bxpos[2] + t[2];
  k_mul_quat(q, bxquat, lquat);
  k_normalize4(q);
  k_quat2mat(xm, q);
}

KD void k_mul_inert_vec(double r[6], const double i[10], const double v[6]) {
  double r0 = i[0] * v[0] + i[3] * v[1] + i[4] * v[2] - i[8] * v[4] + i[7] * v[5];
  double r1 = i[3] * v[0] + i[1] * v[1] + i[5] * v[2] + i[8] * v[3] - i[6] * v[5];
  double r2 = i[4] * v[0] + i[5] * v[1] + i[2] * v[2] - i[7] * v[3] + i[6] * v[4];
  double r3 = i[8] * v[1] - i[7] * v[2] + i[9] * v[3];
  double r4 = i[6] * v[2] - i[8] * v[0] + i[9] * v[4];
  double r5 = i[7] * v[0] - i[6] * v[1] + i[9] * v[5];
  r[0] = r0; r[1] = r1; r[2] = r2; r[3] = r3; r[4] = r4; r[5] = r5;
}

KD void k_cross_motion(double r[6], const double v[6], const double u[6]) {
  double r0 = -v[2] * u[1] + v[1] * u[2];
  double r1 = v[2] * u[0] - v[0] * u[2];
  double r2 = -v[1] * u[0] + v[0] * u[1];
  double r3 = -v[2] * u[4] + v[1] * u[5];
  double r4 = v[2] * u[3] - v[0] * u[5];
  double r5 = -v[1] * u[3] + v[0] * u[4];
  r3 += -v[5] * u[1] + v[4] * u[2];
  r4 += v[5] * u[0] - v[3] * u[2];
  r5 += -v[4] * u[0] + v[3] * u[1];
  r[0] = r0; r[1] = r1; r[2] = r2; r[3] = r3; r[4] = r4; r[5] = r5;
}

KD void k_cross_force(double r[6], const double v[6], const double f[6]) {
  double r0 = -v[2] * f[1] + v[1] * f[2];
  double r1 = v[2] * f[0] - v[0] * f[2];
  double r2 = -v[1] * f[0] + v[0] * f[1];
  double r3 = -v[2] * f[4] + v[1] * f[5];
  double r4 = v[2] * f[3] - v[0] * f[5];
  double r5 = -v[1] * f[3] + v[0] * f[4];
  r0 += -v[5] * f[4] + v[4] * f[5];
  r1 += v[5] * f[3] - v[3] * f[5];
  r2 += -v[4] * f[3] + v[3] * f[4];
  r[0] = r0; r[1] = r1; r[2] = r2; r[3] = r3; r[4] = r4; r[5] = r5;
}

KD double k_dot6(const double a[6], const double b[6]) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5];
}

/* ================================================================== */
/* position stage                                                      */
/* ================================================================== */
KDN void k_kinematics(KModel m, KData* d) {
  d->xpos[0][0] = d->xpos[0][1] = d->xpos[0][2] = 0;
  d->xquat[0][0] = 1; d->xquat[0][1] = d->xquat[0][2] = d->xquat[0][3] = 0;
  k_quat2mat(d->xmat[0], d->xquat[0]);
  d->xipos[0][0] = d->xipos[0][1] = d->xipos[0][2] = 0;
  k_quat2mat(d->ximat[0], d->xquat[0]);
  const int nb = m->nbody;
  for (int i = 1; i < nb; i++) {
    int pid = m->body_parentid[i];
    double xpos[3], xquat[4];
    int jfirst = m->body_jntadr[i];
    if (m->body_jntnum[i] == 1 && m->jnt_type[jfirst] == UR3E_JNT_FREE) {
      int a = m->jnt_qposadr[jfirst];
      xpos[0] = d->qpos[a]; xpos[1] = d->qpos[a + 1]; xpos[2] = d->qpos[a + 2];
      xquat[0] = d->qpos[a + 3]; xquat[1] = d->qpos[a + 4]; xquat[2] = d->qpos[a + 5]; xquat[3] = d->qpos[a + 6];
      k_normalize4(xquat);
      d->xanchor[jfirst][0] = xpos[0]; d->xanchor[jfirst][1] = xpos[1]; d->xanchor[jfirst][2] = xpos[2];
      d->xaxis[jfirst][0] = 0; d->xaxis[jfirst][1] = 0; d->xaxis[jfirst][2] = 1;
    } else {
      double t[3];
      k_mat_vec3(t, d->xmat[pid], m->body_pos[i]);
      xpos[0] = d->xpos[pid][0] + t[0]; xpos[1] = d->xpos[pid][1] + t[1]; xpos[2] = d->xpos[pid][2] + t[2];
      k_mul_quat(xquat, d->xquat[pid], m->body_quat[i]);
      for (int k = 0; k < m->body_jntnum[i]; k++) {
        int j = jfirst + k;
        double xaxis[3], xanchor[3], qloc[4], vec[3];
        k_rot_vec_quat(xaxis, m->jnt_axis[j], xquat);
        k_rot_vec_quat(xanchor, m->jnt_pos[j], xquat);
        xanchor[0] += xpos[0]; xanchor[1] += xpos[1]; xanchor[2] += xpos[2];
        int a = m->jnt_qposadr[j];
        k_axis_angle_quat(qloc, m->jnt_axis[j], d->qpos[a] - m->qpos0[a]);
        k_mul_quat(xquat, xquat, qloc);
        k_rot_vec_quat(vec, m->jnt_pos[j], xquat);
        xpos[0] = xanchor[0] - vec[0]; xpos[1] = xanchor[1] - vec[1]; xpos[2] = xanchor[2] - vec[2];
        for (int c = 0; c < 3; c++) { d->xanchor[j][c] = xanchor[c]; d->xaxis[j][c] = xaxis[c]; }
      }
    }
    k_normalize4(xquat);
    for (int c = 0; c < 3; c++) d->xpos[i][c] = xpos[c];
    for (int c = 0; c < 4; c++) d->xquat[i][c] = xquat[c];
    k_quat2mat(d->xmat[i], xquat);
    k_local2global(d->xipos[i], d->ximat[i], d->xpos[i], d->xquat[i], d->xmat[i], m->body_ipos[i],
                   m->body_iquat[i]);
  }
  for (int g = 0; g < m->ngeom; g++) {
    int b = m->geom_bodyid[g];
    k_local2global(d->geom_xpos[g], d->geom_xmat[g], d->xpos[b], d->xquat[b], d->xmat[b], m->geom_pos[g],
                   m->geom_quat[g]);
  }
  for (int s = 0; s < m->nsite; s++) {
    int b = m->site_bodyid[s];
    k_local2global(d->site_xpos[s], d->site_xmat[s], d->xpos[b], d->xquat[b], d->xmat[b], m->site_pos[s],
                   m->site_quat[s]);
  }
}

KDN void k_com_pos(KModel m, KData* d) {
  const int nb = m->nbody;
  for (int i = 0; i < nb; i++) {
    d->subtree_com[i][0] = d->xipos[i][0] * m->body_mass[i];
    d->subtree_com[i][1] = d->xipos[i][1] * m->body_mass[i];
    d->subtree_com[i][2] = d->xipos[i][2] * m->body_mass[i];
  }
  for (int i = nb - 1; i > 0; i--) {
    int p = m->body_parentid[i];
    d->subtree_com[p][0] += d->subtree_com[i][0];
    d->subtree_com[p][1] += d->subtree_com[i][1];
    d->subtree_com[p][2] += d->subtree_com[i][2];
  }
  for (int i = 0; i < nb; i++) {
    if (m->body_subtreemass[i] < K_MINVAL) {
      d->subtree_com[i][0] = d->xipos[i][0]; d->subtree_com[i][1] = d->xipos[i][1];
      d->subtree_com[i][2] = d->xipos[i][2];
    } else {
      double s = 1.0 / m->body_subtreemass[i];
      d->subtree_com[i][0] *= s; d->subtree_com[i][1] *= s; d->subtree_com[i][2] *= s;
    }
  }
  for (int k = 0; k < 10; k++) d->cinert[0][k] = 0;
  for (int i = 1; i < nb; i++) {
    const double* mat = d->ximat[i];
    const double* in = m->body_inertia[i];
    const double* c = d->subtree_com[m->body_rootid[i]];
    double dif[3] = {d->xipos[i][0] - c[0], d->xipos[i][1] - c[1], d->xipos[i][2] - c[2]};
    double mass = m->body_mass[i];
    double tmp[9] = {mat[0] * in[0], mat[3] * in[0], mat[6] * in[0], mat[1] * in[1], mat[4] * in[1],
                     mat[7] * in[1], mat[2] * in[2], mat[5] * in[2], mat[8] * in[2]};
    double* r = d->cinert[i];
    r[0] = mat[0] * tmp[0] + mat[1] * tmp[3] + mat[2] * tmp[6];
    r[1] = mat[3] * tmp[1] + mat[4] * tmp[4] + mat[5] * tmp[7];
    r[2] = mat[6] * tmp[2] + mat[7] * tmp[5] + mat[8] * tmp[8];
    r[3] = mat[0] * tmp[1] + mat[1] * tmp[4] + mat[2] * tmp[7];
    r[4] = mat[0] * tmp[2] + mat[1] * tmp[5] + mat[2] * tmp[8];
    r[5] = mat[3] * tmp[2] + mat[4] * tmp[5] + mat[5] * tmp[8];
    r[0] += mass * (dif[1] * dif[1] + dif[2] * dif[2]);
    r[1] += mass * (dif[0] * dif[0] + dif[2] * dif[2]);
    r[2] += mass * (dif[0] * dif[0] + dif[1] * dif[1]);
    r[3] -= mass * dif[0] * dif[1];
    r[4] -= mass * dif[0] * dif[2];
    r[5] -= mass * dif[1] * dif[2];
    r[6] = mass * dif[0];
    r[7] = mass * dif[1];
    r[8] = mass * dif[2];
    r[9] = mass;
  }
  for (int j = 0; j < m->njnt; j++) {
    int b = m->jnt_bodyid[j];
    int da = m->jnt_dofadr[j];
    const double* c = d->subtree_com[m->body_rootid[b]];
    double off[3] = {c[0] - d->xanchor[j][0], c[1] - d->xanchor[j][1], c[2] - d->xanchor[j][2]};
    if (m->jnt_type[j] == UR3E_JNT_FREE) {
      for (int k = 0; k < 3; k++) {
        for (int r = 0; r < 6; r++) d->cdof[da + k][r] = 0;
        d->cdof[da + k][3 + k] = 1;
      }
      for (int k = 0; k < 3; k++) {
        double ax[3] = {d->xmat[b][k], d->xmat[b][3 + k], d->xmat[b][6 + k]};
        double cr[3];
        k_cross3(cr, ax, off);
        d->cdof[da + 3 + k][0] = ax[0]; d->cdof[da + 3 + k][1] = ax[1]; d->cdof[da + 3 + k][2] = ax[2];
        d->cdof[da + 3 + k][3] = cr[0]; d->cdof[da + 3 + k][4] = cr[1]; d->cdof[da + 3 + k][5] = cr[2];
      }
    } else {
      double cr[3];
      k_cross3(cr, d->xaxis[j], off);
      d->cdof[da][0] = d->xaxis[j][0]; d->cdof[da][1] = d->xaxis[j][1]; d->cdof[da][2] = d->xaxis[j][2];
      d->cdof[da][3] = cr[0]; d->cdof[da][4] = cr[1]; d->cdof[da][5] = cr[2];
    }
  }
}

KD int k_dof_qposadr(KModel m, int dof) {
  int j = m->dof_jntid[dof];
  return m->jnt_qposadr[j] + (dof - m->jnt_dofadr[j]);
}

/* actuator lengths (fixed tendons folded in); moments are model constants */
KD void k_transmission(KModel m, KData* d) {
  for (int a = 0; a < m->nu; a++) {
    double g = m->act_gear[a];
    if (m->act_trntype[a] == UR3E_TRN_JOINT) {
      int j = m->act_trnid[a];
      d->actuator_length[a] = d->qpos[m->jnt_qposadr[j]] * g;
    } else {
      int t = m->act_trnid[a];
      double len = 0;
      for (int k = 0; k < m->ten_num[t]; k++) len += m->ten_coef[t][k] * d->qpos[k_dof_qposadr(m, m->ten_dof[t][k])];
      d->actuator_length[a] = len * g;
    }
  }
}

KDN void k_crb(KModel m, KData* d) {
  const int nb = m->nbody, nv = m->nv;
  double crb[K_NB][10];
  for (int i = 0; i < nb; i++)
    for (int k = 0; k < 10; k++) crb[i][k] = d->cinert[i][k];
  for (int i = nb - 1; i > 0; i--) {
    int p = m->body_parentid[i];
    if (p > 0)
      for (int k = 0; k < 10; k++) crb[p][k] += crb[i][k];
  }
  for (int i = 0; i < nv; i++)
    for (int j = 0; j < nv; j++) d->qM[i][j] = 0;
  for (int i = 0; i < nv; i++) {
    double buf[6];
    k_mul_inert_vec(buf, crb[m->dof_bodyid[i]], d->cdof[i]);
    d->qM[i][i] = m->dof_armature[i];
    for (int j = i; j >= 0; j = m->dof_parentid[j]) {
      d->qM[i][j] += k_dot6(d->cdof[j], buf);
      d->qM[j][i] = d->qM[i][j];
    }
  }
}

KD void k_factor_tree(KModel m, double A[K_NV][K_NV], double diaginv[K_NV]) {
  const int nv = m->nv;
  for (int k = nv - 1; k >= 0; k--) {
    if (A[k][k] < K_MINVAL) A[k][k] = K_MINVAL;
    for (int i = m->dof_parentid[k]; i >= 0; i = m->dof_parentid[i]) {
      double tmp = A[k][i] / A[k][k];
      for (int j = i; j >= 0; j = m->dof_parentid[j]) A[i][j] -= A[k][j] * tmp;
      A[k][i] = tmp;
    }
  }
  for (int i = 0; i < nv; i++) diaginv[i] = 1.0 / A[i][i];
}

KD void k_solve_tree(KModel m, const double A[K_NV][K_NV], const double diaginv[K_NV], double* x,
                     const double* b) {
  const int nv = m->nv;
  for (int i = 0; i < nv; i++) x[i] = b[i];
  for (int i = nv - 1; i >= 0; i--)
    for (int j = m->dof_parentid[i]; j >= 0; j = m->dof_parentid[j]) x[j] -= A[i][j] * x[i];
  for (int i = 0; i < nv; i++) x[i] *= diaginv[i];
  /* forward pass: ancestors farthest-first (increasing index), so the GPU can run it as a
     column sweep with the same per-element operation order */
  for (int i = 0; i < nv; i++) {
    int anc[UR3E_MAXNV], na = 0;
    for (int j = m->dof_parentid[i]; j >= 0; j = m->dof_parentid[j]) anc[na++] = j;
    for (int t = na - 1; t >= 0; t--) x[i] -= A[i][anc[t]] * x[anc[t]];
  }
}

/* r = M v, dense row order (exact zeros add nothing) */
KD void k_mul_M(KModel m, const KData* d, double* r, const double* v) {
  const int nv = m->nv;
  for (int i = 0; i < nv; i++) {
    double s = 0;
    for (int j = 0; j < nv; j++) s += d->qM[i][j] * v[j];
    r[i] = s;
  }
}

/* translational point Jacobian of `body` at p into jacp[3][K_NV] (full rows, zero outside the chain) */
KD void k_jac_point(KModel m, const KData* d, int body, const double p[3], double jacp[3][K_NV],
                    double jacr[3][K_NV]) {
  const int nv = m->nv;
  for (int k = 0; k < nv; k++) {
    jacp[0][k] = 0; jacp[1][k] = 0; jacp[2][k] = 0;
    if (jacr) { jacr[0][k] = 0; jacr[1][k] = 0; jacr[2][k] = 0; }
  }
  int dof = -1;
  for (int b = body; b > 0 && dof < 0; b = m->body_parentid[b])
    if (m->body_dofnum[b]) dof = m->body_dofadr[b] + m->body_dofnum[b] - 1;
  const double* c = d->subtree_com[m->body_rootid[body]];
  double off[3] = {p[0] - c[0], p[1] - c[1], p[2] - c[2]};
  for (int j = dof; j >= 0; j = m->dof_parentid[j]) {
    const double* cd = d->cdof[j];
    double cr[3];
    k_cross3(cr, cd, off);
    jacp[0][j] = cd[3] + cr[0];
    jacp[1][j] = cd[4] + cr[1];
    jacp[2][j] = cd[5] + cr[2];
    if (jacr) { jacr[0][j] = cd[0]; jacr[1][j] = cd[1]; jacr[2][j] = cd[2]; }
  }
}

KD void k_site_velocity(KModel m, const KData* d, int site, double res[6]) {
  int b = m->site_bodyid[site];
  const double* cv = d->cvel[b];
  const double* c = d->subtree_com[m->body_rootid[b]];
  double dif[3] = {d->site_xpos[site][0] - c[0], d->site_xpos[site][1] - c[1], d->site_xpos[site][2] - c[2]};
  double cr[3];
  k_cross3(cr, dif, cv);
  res[0] = cv[0]; res[1] = cv[1]; res[2] = cv[2];
  res[3] = cv[3] - cr[0]; res[4] = cv[4] - cr[1]; res[5] = cv[5] - cr[2];
}

/* ================================================================== */
/* collision                                                           */
/* ================================================================== */
struct KRaw {
  double pos[3];
  double n[3];
  double dist;
};

/* rows 1 and 2 of a contact frame whose row 0 (the unit normal) is already in f[0..2] */
KD void k_frame_rest(double f[9]) {
  double y[3];
  if (fabs(f[1]) < 0.5) { y[0] = 0; y[1] = 1; y[2] = 0; }
  else { y[0] = 0; y[1] = 0; y[2] = 1; }
  double dd = f[0] * y[0] + f[1] * y[1] + f[2] * y[2];
  y[0] -= f[0] * dd; y[1] -= f[1] * dd; y[2] -= f[2] * dd;
  k_normalize3(y);
  f[3] = y[0]; f[4] = y[1]; f[5] = y[2];
  double z[3];
  k_cross3(z, f, y);
  f[6] = z[0]; f[7] = z[1]; f[8] = z[2];
}

KD void k_make_frame(double f[9], const double n[3]) {
  f[0] = n[0]; f[1] = n[1]; f[2] = n[2];
  k_normalize3(f);
  k_frame_rest(f);
}

/* Narrowphase routines are templated on where their intermediate polygons live (Clip) and where
   their contacts go (Emit), so the compact tier can keep both in LDS (dynamic indices there are
   plain ds_read/ds_write addresses) while the other tiers keep private arrays.  The arithmetic and
   its order are the same for every instantiation.
     Clip: double get(int buf, int v, int c) / void set(int buf, int v, int c, double x),
           buf in {0, 1} (ping-pong), v < 8, c < 3
     Emit: void operator()(int k, const double pos[3], const double n[3], double dist) */
struct KRawEmit {
  KRaw* out;
  __device__ __forceinline__ void operator()(int k, const double pos[3], const double n[3], double dist) const {
    out[k].pos[0] = pos[0]; out[k].pos[1] = pos[1]; out[k].pos[2] = pos[2];
    out[k].n[0] = n[0]; out[k].n[1] = n[1]; out[k].n[2] = n[2];
    out[k].dist = dist;
  }
};
struct KPrivClip {
  double b[2][8][3];
  __device__ __forceinline__ double get(int buf, int v, int c) const { return b[buf][v][c]; }
  __device__ __forceinline__ void set(int buf, int v, int c, double x) { b[buf][v][c] = x; }
};

/* column i (i in 0..2, may be lane-varying) of a row-major 3x3 matrix read straight from where the
   matrix lives (LDS / global): the frame axes of the box-box test without a dynamically indexed
   private array */
__device__ __forceinline__ void k_col3(double out[3], const double* R, int i) {
  out[0] = R[i]; out[1] = R[3 + i]; out[2] = R[6 + i];
}

template <class Emit>
__device__ static __forceinline__ int k_plane_box_t(const double pp[3], const double pm[9], const double bp[3],
                                                     const double bm[9], const double bs[3], double margin,
                                                     const Emit& emit) {
  double n[3] = {pm[2], pm[5], pm[8]};
  double dif[3] = {bp[0] - pp[0], bp[1] - pp[1], bp[2] - pp[2]};
  double dist = k_dot3(n, dif);
  int cnt = 0;
  for (int i = 0; i < 8; i++) {
    double v[3] = {(i & 1) ? bs[0] : -bs[0], (i & 2) ? bs[1] : -bs[1], (i & 4) ? bs[2] : -bs[2]};
    double corner[3];
    k_mat_vec3(corner, bm, v);
    double ld = k_dot3(n, corner);
    if (dist + ld > margin || ld > 0) continue;
    const double cd = dist + ld;
    double h = cd * 0.5;
    double pos[3] = {corner[0] - n[0] * h + bp[0], corner[1] - n[1] * h + bp[1], corner[2] - n[2] * h + bp[2]};
    emit(cnt, pos, n, cd);
    if (++cnt >= 4) return cnt;
  }
  return cnt;
}

KD int k_plane_box(const double pp[3], const double pm[9], const double bp[3], const double bm[9],
                   const double bs[3], double margin, KRaw* out) {
  return k_plane_box_t(pp, pm, bp, bm, bs, margin, KRawEmit{out});
}

template <class Clip, class Emit>
__device__ static __forceinline__ int k_box_box_t(const double p1[3], const double R1[9], const double s1[3],
                                                   const double p2[3], const double R2[9], const double s2[3],
                                                   double margin, Clip& clip, const Emit& emit) {
  double a[3][3], b[3][3];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    a[k][0] = R1[k]; a[k][1] = R1[3 + k]; a[k][2] = R1[6 + k];
    b[k][0] = R2[k]; b[k][1] = R2[3 + k]; b[k][2] = R2[6 + k];
  }
  double pp[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  double best = -1e300;
  int bestcode = -1;
  double bestax[3] = {0, 0, 0};
#pragma unroll
  for (int code = 0; code < 6; code++) {
    const double* ax = code < 3 ? a[code] : b[code - 3];
    double ext = 0;
#pragma unroll
    for (int k = 0; k < 3; k++) ext += s1[k] * fabs(k_dot3(a[k], ax));
#pragma unroll
    for (int k = 0; k < 3; k++) ext += s2[k] * fabs(k_dot3(b[k], ax));
    double s = fabs(k_dot3(pp, ax)) - ext;
    if (s > margin) return 0;
    if (s > best) {
      best = s; bestcode = code;
      bestax[0] = ax[0]; bestax[1] = ax[1]; bestax[2] = ax[2];
    }
  }
#pragma unroll
  for (int i = 0; i < 3; i++) {
#pragma unroll
    for (int j = 0; j < 3; j++) {
      double u[3];
      k_cross3(u, a[i], b[j]);
      double len = sqrt(k_dot3(u, u));
      if (len < 1e-6) continue;
      const double rlen = 1.0 / len;
      u[0] = k_div_rcp(u[0], len, rlen); u[1] = k_div_rcp(u[1], len, rlen); u[2] = k_div_rcp(u[2], len, rlen);
      double ext = 0;
#pragma unroll
      for (int k = 0; k < 3; k++) ext += s1[k] * fabs(k_dot3(a[k], u));
#pragma unroll
      for (int k = 0; k < 3; k++) ext += s2[k] * fabs(k_dot3(b[k], u));
      double s = fabs(k_dot3(pp, u)) - ext;
      if (s > margin) return 0;
      if (s * 1.05 > best) {
        best = s; bestcode = 6 + 3 * i + j;
        bestax[0] = u[0]; bestax[1] = u[1]; bestax[2] = u[2];
      }
    }
  }
  double n[3] = {bestax[0], bestax[1], bestax[2]};
  if (k_dot3(pp, n) < 0) { n[0] = -n[0]; n[1] = -n[1]; n[2] = -n[2]; }

  if (bestcode >= 6) {
    int i = (bestcode - 6) / 3, j = (bestcode - 6) % 3;
    double ai[3], bj[3];
    k_col3(ai, R1, i);
    k_col3(bj, R2, j);
    double pa[3] = {p1[0], p1[1], p1[2]}, pb[3] = {p2[0], p2[1], p2[2]};
#pragma unroll
    for (int k = 0; k < 3; k++) {
      if (k != i) {
        double sg = k_dot3(n, a[k]) > 0 ? 1.0 : -1.0;
        pa[0] += sg * s1[k] * a[k][0]; pa[1] += sg * s1[k] * a[k][1]; pa[2] += sg * s1[k] * a[k][2];
      }
      if (k != j) {
        double sg = k_dot3(n, b[k]) > 0 ? -1.0 : 1.0;
        pb[0] += sg * s2[k] * b[k][0]; pb[1] += sg * s2[k] * b[k][1]; pb[2] += sg * s2[k] * b[k][2];
      }
    }
    double w[3] = {pa[0] - pb[0], pa[1] - pb[1], pa[2] - pb[2]};
    double uaub = k_dot3(ai, bj);
    double q1 = k_dot3(ai, w), q2 = k_dot3(bj, w);
    double den = 1.0 - uaub * uaub;
    double t = 0, u = 0;
    if (den > 1e-12) {
      t = (uaub * q2 - q1) / den;
      u = (q2 - uaub * q1) / den;
    }
    double ca[3] = {pa[0] + t * ai[0], pa[1] + t * ai[1], pa[2] + t * ai[2]};
    double cb[3] = {pb[0] + u * bj[0], pb[1] + u * bj[1], pb[2] + u * bj[2]};
    double pos[3] = {0.5 * (ca[0] + cb[0]), 0.5 * (ca[1] + cb[1]), 0.5 * (ca[2] + cb[2])};
    emit(0, pos, n, best);
    return 1;
  }

  int ref_is_1 = bestcode < 3;
  int fk = ref_is_1 ? bestcode : bestcode - 3;
  const double* rp = ref_is_1 ? p1 : p2;
  const double* ip = ref_is_1 ? p2 : p1;
  const double* rs = ref_is_1 ? s1 : s2;
  const double* is = ref_is_1 ? s2 : s1;
  const double* rR = ref_is_1 ? R1 : R2; /* ra[k] = column k of rR */
  const double* iR = ref_is_1 ? R2 : R1; /* ia[k] = column k of iR */
  double nr[3] = {ref_is_1 ? n[0] : -n[0], ref_is_1 ? n[1] : -n[1], ref_is_1 ? n[2] : -n[2]};
  double rafk[3];
  k_col3(rafk, rR, fk);
  const double rsfk = rs[fk];
  double rsg = k_dot3(nr, rafk) > 0 ? 1.0 : -1.0;
  double cr[3] = {rp[0] + rsg * rsfk * rafk[0], rp[1] + rsg * rsfk * rafk[1], rp[2] + rsg * rsfk * rafk[2]};
  int t1 = (fk + 1) % 3, t2 = (fk + 2) % 3;
  double rat1[3], rat2[3];
  k_col3(rat1, rR, t1);
  k_col3(rat2, rR, t2);
  const double rst1 = rs[t1], rst2 = rs[t2];
  int im = 0;
  double bd = -1;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    double iak[3];
    k_col3(iak, iR, k);
    const double dmk = k_dot3(iak, nr);
    if (fabs(dmk) > bd) { bd = fabs(dmk); im = k; }
  }
  double iaim[3], iau1[3], iau2[3];
  k_col3(iaim, iR, im);
  const double dmim = k_dot3(iaim, nr); /* = dm[im], recomputed from the same operands */
  double isg = dmim > 0 ? -1.0 : 1.0;
  const double isim = is[im];
  double ic[3] = {ip[0] + isg * isim * iaim[0], ip[1] + isg * isim * iaim[1], ip[2] + isg * isim * iaim[2]};
  int u1 = (im + 1) % 3, u2 = (im + 2) % 3;
  k_col3(iau1, iR, u1);
  k_col3(iau2, iR, u2);
  const double isu1 = is[u1], isu2 = is[u2];
  /* a quad clipped by the 4 half-planes of a rectangle never exceeds 8 vertices (each clip adds
     at most one), so 8-point buffers hold every intermediate polygon; clip e reads buffer e & 1
     and writes the other one */
  int np = 4;
  const double sx[4] = {1, -1, -1, 1}, sy[4] = {1, 1, -1, -1};
#pragma unroll
  for (int k = 0; k < 4; k++) {
    double v[3];
#pragma unroll
    for (int c = 0; c < 3; c++) v[c] = ic[c] + sx[k] * isu1 * iau1[c] + sy[k] * isu2 * iau2[c] - cr[c];
    clip.set(0, k, 0, k_dot3(v, rat1));
    clip.set(0, k, 1, k_dot3(v, rat2));
    clip.set(0, k, 2, k_dot3(v, nr));
  }
#pragma unroll
  for (int e = 0; e < 4; e++) {
    const int ax = e >> 1, src = e & 1, dst = src ^ 1;
    double sgn = (e & 1) ? -1.0 : 1.0;
    double lim = ax == 0 ? rst1 : rst2;
    int nn = 0;
    for (int k = 0; k < np; k++) {
      const int kq = k + 1 < np ? k + 1 : 0;
      double P[3] = {clip.get(src, k, 0), clip.get(src, k, 1), clip.get(src, k, 2)};
      double Q[3] = {clip.get(src, kq, 0), clip.get(src, kq, 1), clip.get(src, kq, 2)};
      double dp = sgn * P[ax] - lim, dq = sgn * Q[ax] - lim;
      if (dp <= 0) {
        clip.set(dst, nn, 0, P[0]); clip.set(dst, nn, 1, P[1]); clip.set(dst, nn, 2, P[2]);
        nn++;
      }
      if ((dp <= 0) != (dq <= 0)) {
        double tt = dp / (dp - dq);
        clip.set(dst, nn, 0, P[0] + tt * (Q[0] - P[0]));
        clip.set(dst, nn, 1, P[1] + tt * (Q[1] - P[1]));
        clip.set(dst, nn, 2, P[2] + tt * (Q[2] - P[2]));
        nn++;
      }
    }
    np = nn;
    if (np == 0) break;
  }
  /* after the fourth clip the polygon is in buffer 0 (np == 0 after an early break) */
  int cnt = 0;
  for (int k = 0; k < np && cnt < 8; k++) {
    const double x = clip.get(0, k, 0), y = clip.get(0, k, 1), h = clip.get(0, k, 2);
    if (h > margin) continue;
    double w[3];
#pragma unroll
    for (int c = 0; c < 3; c++) w[c] = cr[c] + x * rat1[c] + y * rat2[c] + (h * 0.5) * nr[c];
    emit(cnt, w, n, h);
    cnt++;
  }
  return cnt;
}

__device__ static __forceinline__ int k_box_box_inl(const double p1[3], const double R1[9], const double s1[3],
                                                     const double p2[3], const double R2[9], const double s2[3],
                                                     double margin, KRaw* out) {
  KPrivClip clip;
  return k_box_box_t(p1, R1, s1, p2, R2, s2, margin, clip, KRawEmit{out});
}

/* out-of-line copy for the multi-call-site paths (keeps those kernels' code size down) */
KDN int k_box_box(const double p1[3], const double R1[9], const double s1[3], const double p2[3],
                  const double R2[9], const double s2[3], double margin, KRaw* out) {
  return k_box_box_inl(p1, R1, s1, p2, R2, s2, margin, out);
}

KDN void k_collision(KModel m, KData* d) {
  d->ncon = 0;
  KRaw raw[8];
  const int npair = m->ncpair;
  for (int p = 0; p < npair; p++) {
    int g1 = m->cpair_geom1[p], g2 = m->cpair_geom2[p];
    double margin = m->cpair_margin[p];
    double rb1 = m->geom_rbound[g1], rb2 = m->geom_rbound[g2];
    if (rb1 > 0 && rb2 > 0) {
      double dx = d->geom_xpos[g1][0] - d->geom_xpos[g2][0];
      double dy = d->geom_xpos[g1][1] - d->geom_xpos[g2][1];
      double dz = d->geom_xpos[g1][2] - d->geom_xpos[g2][2];
      double lim = rb1 + rb2 + margin;
      if (dx * dx + dy * dy + dz * dz > lim * lim) continue;
    }
    int n = 0;
    int t1 = m->geom_type[g1], t2 = m->geom_type[g2];
    if (t1 == UR3E_GEOM_PLANE && t2 == UR3E_GEOM_BOX) {
      n = k_plane_box(d->geom_xpos[g1], d->geom_xmat[g1], d->geom_xpos[g2], d->geom_xmat[g2], m->geom_size[g2],
                      margin, raw);
    } else if (t1 == UR3E_GEOM_BOX && t2 == UR3E_GEOM_BOX) {
      n = k_box_box(d->geom_xpos[g1], d->geom_xmat[g1], m->geom_size[g1], d->geom_xpos[g2], d->geom_xmat[g2],
                    m->geom_size[g2], margin, raw);
    }
    for (int k = 0; k < n; k++) {
      if (d->ncon >= K_MAXCON) break;
      KContact* c = d->contact + d->ncon++;
      c->pos[0] = raw[k].pos[0]; c->pos[1] = raw[k].pos[1]; c->pos[2] = raw[k].pos[2];
      k_make_frame(c->frame, raw[k].n);
      c->dist = raw[k].dist;
      for (int f = 0; f < 5; f++) c->friction[f] = m->cpair_friction[p][f];
      c->dim = m->cpair_condim[p];
      c->geom1 = g1; c->geom2 = g2;
      c->cpair = p;
      c->mu = 0;
      c->efc_address = -1;
    }
  }
}

/* ================================================================== */
/* constraints                                                         */
/* ================================================================== */
KD double k_get_impedance(const double* solimp, double pos, double margin) {
  double dmin = solimp[0], dmax = solimp[1], width = solimp[2], mid = solimp[3], power = solimp[4];
  if (dmin < K_MINIMP) dmin = K_MINIMP;
  if (dmin > K_MAXIMP) dmin = K_MAXIMP;
  if (dmax < K_MINIMP) dmax = K_MINIMP;
  if (dmax > K_MAXIMP) dmax = K_MAXIMP;
  if (dmin == dmax || width <= K_MINVAL) return 0.5 * (dmin + dmax);
  double x = (pos - margin) / width;
  if (x < 0) x = -x;
  if (x >= 1) return dmax;
  if (x <= 0) return dmin;
  double y;
  if (power == 1) {
    y = x;
  } else if (x <= mid) {
    int ip = (int)power;
    double a = 1.0, xp = 1.0;
    for (int k = 0; k < ip - 1; k++) a *= mid;
    a = 1.0 / a;
    for (int k = 0; k < ip; k++) xp *= x;
    y = a * xp;
  } else {
    int ip = (int)power;
    double b = 1.0, xp = 1.0;
    for (int k = 0; k < ip - 1; k++) b *= (1 - mid);
    b = 1.0 / b;
    for (int k = 0; k < ip; k++) xp *= (1 - x);
    y = 1 - b * xp;
  }
  return dmin + y * (dmax - dmin);
}

/* finalize row r: efc_vel -> aref, R (mj_makeImpedance / mj_referenceConstraint) */
KD void k_row_impedance(KModel m, KData* d, int r, const double* sref, const double* simp, double pos,
                        double margin, double diag, int friction_row) {
  const int nv = m->nv;
  double vel = 0;
  for (int k = 0; k < nv; k++) vel += d->efc_J[r][k] * d->qvel[k];
  double imp = k_get_impedance(simp, pos, margin);
  double dmax = simp[1];
  if (dmax < K_MINIMP) dmax = K_MINIMP;
  if (dmax > K_MAXIMP) dmax = K_MAXIMP;
  double K, B;
  if (sref[0] > 0) {
    double tc = sref[0];
    if (tc < 2 * m->timestep) tc = 2 * m->timestep;
    double dr = sref[1];
    K = 1.0 / (dmax * dmax * tc * tc * dr * dr);
    B = 2.0 / (dmax * tc);
  } else {
    K = -sref[0] / (dmax * dmax);
    B = -sref[1] / dmax;
  }
  if (friction_row)
    d->efc_aref[r] = -B * vel;
  else
    d->efc_aref[r] = -B * vel - K * imp * (pos - margin);
  double R = (1 - imp) * diag / imp;
  d->efc_R[r] = R < K_MINVAL ? K_MINVAL : R;
}

KD int k_add_row(KData* d, int type, int id, double floss) {
  if (d->nefc >= K_MAXEFC) return -1;
  int r = d->nefc++;
  d->efc_type[r] = type;
  d->efc_id[r] = id;
  d->efc_floss[r] = floss;
  return r;
}

KDN void k_make_constraint(KModel m, KData* d) {
  const int nv = m->nv;
  d->nefc = 0;
  double jp1[3][K_NV], jp2[3][K_NV];
  for (int e = 0; e < m->neq; e++) {
    if (m->eq_type[e] == UR3E_EQ_CONNECT) {
      int b1 = m->eq_obj1[e], b2 = m->eq_obj2[e];
      double p1[3], p2[3];
      k_mat_vec3(p1, d->xmat[b1], m->eq_data[e]);
      p1[0] += d->xpos[b1][0]; p1[1] += d->xpos[b1][1]; p1[2] += d->xpos[b1][2];
      k_mat_vec3(p2, d->xmat[b2], m->eq_data[e] + 3);
      p2[0] += d->xpos[b2][0]; p2[1] += d->xpos[b2][1]; p2[2] += d->xpos[b2][2];
      k_jac_point(m, d, b1, p1, jp1, nullptr);
      k_jac_point(m, d, b2, p2, jp2, nullptr);
      double diag = m->body_invweight0[b1][0] + m->body_invweight0[b2][0];
      if (d->nefc + 3 > K_MAXEFC) return;
      for (int k = 0; k < 3; k++) {
        int r = k_add_row(d, CN_EQUALITY, e, 0);
        if (r < 0) return;
        for (int v = 0; v < nv; v++) d->efc_J[r][v] = jp1[k][v] - jp2[k][v];
        k_row_impedance(m, d, r, m->eq_solref[e], m->eq_solimp[e], p1[k] - p2[k], 0, diag, 0);
      }
    } else if (m->eq_type[e] == UR3E_EQ_JOINT) {
      int j1 = m->eq_obj1[e], j2 = m->eq_obj2[e];
      const double* c = m->eq_data[e];
      int a1 = m->jnt_qposadr[j1];
      double q1 = d->qpos[a1] - m->qpos0[a1];
      double pos, dpoly = 0;
      double diag = m->dof_invweight0[m->jnt_dofadr[j1]];
      if (j2 >= 0) {
        int a2 = m->jnt_qposadr[j2];
        double q2 = d->qpos[a2] - m->qpos0[a2];
        pos = q1 - (c[0] + q2 * (c[1] + q2 * (c[2] + q2 * (c[3] + q2 * c[4]))));
        dpoly = c[1] + q2 * (2 * c[2] + q2 * (3 * c[3] + q2 * 4 * c[4]));
        diag += m->dof_invweight0[m->jnt_dofadr[j2]];
      } else {
        pos = q1 - c[0];
      }
      int r = k_add_row(d, CN_EQUALITY, e, 0);
      if (r < 0) return;
      for (int v = 0; v < nv; v++) d->efc_J[r][v] = 0;
      d->efc_J[r][m->jnt_dofadr[j1]] = 1;
      if (j2 >= 0) d->efc_J[r][m->jnt_dofadr[j2]] = -dpoly;
      k_row_impedance(m, d, r, m->eq_solref[e], m->eq_solimp[e], pos, 0, diag, 0);
    }
  }
  for (int v = 0; v < nv; v++) {
    if (m->dof_frictionloss[v] > 0) {
      int r = k_add_row(d, CN_FRICTION_DOF, v, m->dof_frictionloss[v]);
      if (r < 0) return;
      for (int k = 0; k < nv; k++) d->efc_J[r][k] = 0;
      d->efc_J[r][v] = 1;
      k_row_impedance(m, d, r, m->dof_solref[v], m->dof_solimp[v], 0, 0, m->dof_invweight0[v], 1);
    }
  }
  for (int j = 0; j < m->njnt; j++) {
    if (!m->jnt_limited[j]) continue;
    if (m->jnt_type[j] != UR3E_JNT_HINGE && m->jnt_type[j] != UR3E_JNT_SLIDE) continue;
    double q = d->qpos[m->jnt_qposadr[j]];
    for (int side = -1; side <= 1; side += 2) {
      double dist = side * (m->jnt_range[j][(side + 1) / 2] - q);
      if (dist < m->jnt_margin[j]) {
        int dof = m->jnt_dofadr[j];
        int r = k_add_row(d, CN_LIMIT_JOINT, j, 0);
        if (r < 0) return;
        for (int k = 0; k < nv; k++) d->efc_J[r][k] = 0;
        d->efc_J[r][dof] = -(double)side;
        k_row_impedance(m, d, r, m->jnt_solref[j], m->jnt_solimp[j], dist, m->jnt_margin[j],
                        m->dof_invweight0[dof], 0);
      }
    }
  }
  for (int ci = 0; ci < d->ncon; ci++) {
    KContact* c = d->contact + ci;
    if (c->dim != 3) continue;
    int p = c->cpair;
    int b1 = m->geom_bodyid[c->geom1], b2 = m->geom_bodyid[c->geom2];
    k_jac_point(m, d, b1, c->pos, jp1, nullptr);
    k_jac_point(m, d, b2, c->pos, jp2, nullptr);
    double diag = m->body_invweight0[b1][0] + m->body_invweight0[b2][0];
    double incl = m->cpair_margin[p] - m->cpair_gap[p];
    if (d->nefc + 3 > K_MAXEFC) return;
    c->efc_address = d->nefc;
    for (int k = 0; k < 3; k++) {
      int r = k_add_row(d, CN_CONTACT_ELLIPTIC, ci, 0);
      if (r < 0) { c->efc_address = -1; return; }
      for (int v = 0; v < nv; v++) {
        double dj0 = jp2[0][v] - jp1[0][v];
        double dj1 = jp2[1][v] - jp1[1][v];
        double dj2 = jp2[2][v] - jp1[2][v];
        d->efc_J[r][v] = c->frame[3 * k] * dj0 + c->frame[3 * k + 1] * dj1 + c->frame[3 * k + 2] * dj2;
      }
      k_row_impedance(m, d, r, m->cpair_solref[p], m->cpair_solimp[p], c->dist, incl, diag, k > 0);
    }
    int a = c->efc_address;
    d->efc_R[a + 1] = d->efc_R[a] / m->impratio;
    c->mu = c->friction[0] * sqrt(d->efc_R[a + 1] / d->efc_R[a]);
    for (int j = 1; j < c->dim - 1; j++)
      d->efc_R[a + j + 1] = d->efc_R[a + 1] * c->friction[0] * c->friction[0] / (c->friction[j] * c->friction[j]);
  }
  for (int i = 0; i < d->nefc; i++) d->efc_D[i] = 1.0 / d->efc_R[i];
}

/* ================================================================== */
/* velocity stage                                                      */
/* ================================================================== */
KDN void k_com_vel(KModel m, KData* d) {
  for (int k = 0; k < 6; k++) d->cvel[0][k] = 0;
  const int nb = m->nbody;
  for (int i = 1; i < nb; i++) {
    double cv[6];
    for (int k = 0; k < 6; k++) cv[k] = d->cvel[m->body_parentid[i]][k];
    int bda = m->body_dofadr[i];
    for (int j = 0; j < m->body_dofnum[i]; j++) {
      int dof = bda + j;
      int jt = m->jnt_type[m->dof_jntid[dof]];
      if (jt == UR3E_JNT_FREE) {
        for (int k = 0; k < 3; k++)
          for (int r = 0; r < 6; r++) d->cdof_dot[dof + k][r] = 0;
        double tmp[6] = {0, 0, 0, 0, 0, 0};
        for (int k = 0; k < 3; k++)
          for (int r = 0; r < 6; r++) tmp[r] += d->cdof[dof + k][r] * d->qvel[dof + k];
        for (int r = 0; r < 6; r++) cv[r] += tmp[r];
        for (int k = 3; k < 6; k++) k_cross_motion(d->cdof_dot[dof + k], cv, d->cdof[dof + k]);
        for (int r = 0; r < 6; r++) tmp[r] = 0;
        for (int k = 3; k < 6; k++)
          for (int r = 0; r < 6; r++) tmp[r] += d->cdof[dof + k][r] * d->qvel[dof + k];
        for (int r = 0; r < 6; r++) cv[r] += tmp[r];
        j += 5;
      } else {
        k_cross_motion(d->cdof_dot[dof], cv, d->cdof[dof]);
        for (int r = 0; r < 6; r++) cv[r] += d->cdof[dof][r] * d->qvel[dof];
      }
    }
    for (int k = 0; k < 6; k++) d->cvel[i][k] = cv[k];
  }
}

KDN void k_rne(KModel m, KData* d) {
  double cacc[K_NB][6], cfrc[K_NB][6];
  cacc[0][0] = cacc[0][1] = cacc[0][2] = 0;
  cacc[0][3] = -m->gravity[0]; cacc[0][4] = -m->gravity[1]; cacc[0][5] = -m->gravity[2];
  for (int k = 0; k < 6; k++) cfrc[0][k] = 0;
  const int nb = m->nbody;
  for (int i = 1; i < nb; i++) {
    double tmp[6] = {0, 0, 0, 0, 0, 0};
    int bda = m->body_dofadr[i];
    for (int j = 0; j < m->body_dofnum[i]; j++)
      for (int r = 0; r < 6; r++) tmp[r] += d->cdof_dot[bda + j][r] * d->qvel[bda + j];
    int p = m->body_parentid[i];
    for (int r = 0; r < 6; r++) cacc[i][r] = cacc[p][r] + tmp[r];
    double f1[6], f2[6], f3[6];
    k_mul_inert_vec(f1, d->cinert[i], cacc[i]);
    k_mul_inert_vec(f2, d->cinert[i], d->cvel[i]);
    k_cross_force(f3, d->cvel[i], f2);
    for (int r = 0; r < 6; r++) cfrc[i][r] = f1[r] + f3[r];
  }
  for (int i = nb - 1; i > 0; i--) {
    int p = m->body_parentid[i];
    if (p > 0)
      for (int r = 0; r < 6; r++) cfrc[p][r] += cfrc[i][r];
  }
  for (int v = 0; v < m->nv; v++) d->qfrc_bias[v] = k_dot6(d->cdof[v], cfrc[m->dof_bodyid[v]]);
}

KD void k_passive(KModel m, KData* d) {
  for (int v = 0; v < m->nv; v++) d->qfrc_passive[v] = 0;
  for (int j = 0; j < m->njnt; j++) {
    double k = m->jnt_stiffness[j];
    if (k == 0) continue;
    if (m->jnt_type[j] == UR3E_JNT_HINGE || m->jnt_type[j] == UR3E_JNT_SLIDE) {
      int a = m->jnt_qposadr[j];
      d->qfrc_passive[m->jnt_dofadr[j]] = -k * (d->qpos[a] - m->qpos_spring[a]);
    }
  }
  for (int v = 0; v < m->nv; v++) {
    double b = m->dof_damping[v];
    if (b != 0) d->qfrc_passive[v] -= b * d->qvel[v];
  }
}

/* actuation; moment rows are constants of the model (joint gear / fixed tendon coef * gear) */
KD void k_actuation(KModel m, KData* d, double qfrc_actuator[K_NV]) {
  const int nv = m->nv;
  double force[K_NU];
  for (int a = 0; a < m->nu; a++) {
    double g = m->act_gear[a];
    double vel = 0;
    if (m->act_trntype[a] == UR3E_TRN_JOINT) {
      int dof = m->jnt_dofadr[m->act_trnid[a]];
      for (int v = 0; v < nv; v++) vel += (v == dof ? g : 0.0) * d->qvel[v];
    } else {
      int t = m->act_trnid[a];
      for (int v = 0; v < nv; v++) {
        double mom = 0;
        for (int k = 0; k < m->ten_num[t]; k++)
          if (m->ten_dof[t][k] == v) mom = m->ten_coef[t][k] * g;
        vel += mom * d->qvel[v];
      }
    }
    double ctrl = d->ctrl[a];
    if (m->act_ctrllimited[a]) {
      if (ctrl < m->act_ctrlrange[a][0]) ctrl = m->act_ctrlrange[a][0];
      if (ctrl > m->act_ctrlrange[a][1]) ctrl = m->act_ctrlrange[a][1];
    }
    double f = m->act_gainprm[a][0] * ctrl;
    if (m->act_biastype[a] == UR3E_BIAS_AFFINE)
      f += m->act_biasprm[a][0] + m->act_biasprm[a][1] * d->actuator_length[a] + m->act_biasprm[a][2] * vel;
    if (m->act_forcelimited[a]) {
      if (f < m->act_forcerange[a][0]) f = m->act_forcerange[a][0];
      if (f > m->act_forcerange[a][1]) f = m->act_forcerange[a][1];
    }
    force[a] = f;
  }
  for (int v = 0; v < nv; v++) {
    double s = 0;
    for (int a = 0; a < m->nu; a++) {
      double mom;
      if (m->act_trntype[a] == UR3E_TRN_JOINT) {
        mom = (v == m->jnt_dofadr[m->act_trnid[a]]) ? m->act_gear[a] : 0.0;
      } else {
        int t = m->act_trnid[a];
        mom = 0;
        for (int k = 0; k < m->ten_num[t]; k++)
          if (m->ten_dof[t][k] == v) mom = m->ten_coef[t][k] * m->act_gear[a];
      }
      s += mom * force[a];
    }
    qfrc_actuator[v] = s;
  }
}

/* ================================================================== */
/* Newton solver                                                       */
/* ================================================================== */
KDN double k_constraint_update(KModel m, KData* d) {
  double cost = 0;
  const int nefc = d->nefc;
  for (int i = 0; i < nefc; i++) {
    int t = d->efc_type[i];
    double D = d->efc_D[i], R = d->efc_R[i];
    double jar = d->jar[i];
    if (t == CN_EQUALITY) {
      d->efc_force[i] = -D * jar;
      cost += 0.5 * D * jar * jar;
      d->efc_state[i] = ST_QUADRATIC;
    } else if (t == CN_FRICTION_DOF) {
      double fl = d->efc_floss[i];
      if (jar <= -R * fl) {
        d->efc_force[i] = fl;
        cost += -0.5 * R * fl * fl - fl * jar;
        d->efc_state[i] = ST_LINEARNEG;
      } else if (jar >= R * fl) {
        d->efc_force[i] = -fl;
        cost += -0.5 * R * fl * fl + fl * jar;
        d->efc_state[i] = ST_LINEARPOS;
      } else {
        d->efc_force[i] = -D * jar;
        cost += 0.5 * D * jar * jar;
        d->efc_state[i] = ST_QUADRATIC;
      }
    } else if (t == CN_LIMIT_JOINT) {
      if (jar >= 0) {
        d->efc_force[i] = 0;
        d->efc_state[i] = ST_SATISFIED;
      } else {
        d->efc_force[i] = -D * jar;
        cost += 0.5 * D * jar * jar;
        d->efc_state[i] = ST_QUADRATIC;
      }
    } else {
      KContact* c = d->contact + d->efc_id[i];
      int dim = c->dim;
      double mu = c->mu;
      double U[6];
      U[0] = d->jar[i] * mu;
      for (int j = 1; j < dim; j++) U[j] = d->jar[i + j] * c->friction[j - 1];
      double N = U[0];
      double T2 = 0;
      for (int j = 1; j < dim; j++) T2 += U[j] * U[j];
      double T = sqrt(T2);
      if (N >= mu * T || (T <= 0 && N >= 0)) {
        for (int j = 0; j < dim; j++) {
          d->efc_force[i + j] = 0;
          d->efc_state[i + j] = ST_SATISFIED;
        }
      } else if (mu * N + T <= 0 || (T <= 0 && N < 0)) {
        for (int j = 0; j < dim; j++) {
          d->efc_force[i + j] = -d->efc_D[i + j] * d->jar[i + j];
          cost += 0.5 * d->efc_D[i + j] * d->jar[i + j] * d->jar[i + j];
          d->efc_state[i + j] = ST_QUADRATIC;
        }
      } else {
        double Dm = d->efc_D[i] / (mu * mu * (1 + mu * mu));
        double NT = N - mu * T;
        cost += 0.5 * Dm * NT * NT;
        d->efc_force[i] = -Dm * NT * mu;
        for (int j = 1; j < dim; j++) d->efc_force[i + j] = Dm * NT * mu * U[j] / T * c->friction[j - 1];
        for (int j = 0; j < dim; j++) d->efc_state[i + j] = ST_CONE;
      }
      i += dim - 1;
    }
  }
  return cost;
}

KDN void k_eval_state(KModel m, KData* d, const double* qacc) {
  const int nv = m->nv;
  k_mul_M(m, d, d->Ma, qacc);
  for (int i = 0; i < d->nefc; i++) {
    double v = 0;
    for (int k = 0; k < nv; k++) v += d->efc_J[i][k] * qacc[k];
    d->jar[i] = v - d->efc_aref[i];
  }
  double g = 0;
  for (int k = 0; k < nv; k++) g += (d->Ma[k] - d->qfrc_smooth[k]) * (qacc[k] - d->qacc_smooth[k]);
  d->gauss = 0.5 * g;
  d->cost = d->gauss + k_constraint_update(m, d);
}

KD void k_compute_grad(KModel m, KData* d) {
  const int nv = m->nv;
  for (int k = 0; k < nv; k++) {
    double f = 0;
    for (int i = 0; i < d->nefc; i++) f += d->efc_J[i][k] * d->efc_force[i];
    d->qfrc_constraint[k] = f;
  }
  for (int k = 0; k < nv; k++) d->grad[k] = d->Ma[k] - d->qfrc_smooth[k] - d->qfrc_constraint[k];
}

KDN void k_hessian_factor(KModel m, KData* d) {
  const int nv = m->nv;
  for (int r = 0; r < nv; r++)
    for (int c = 0; c < nv; c++) d->H[r][c] = d->qM[r][c];
  for (int i = 0; i < d->nefc; i++) {
    int st = d->efc_state[i];
    if (st == ST_QUADRATIC) {
      double D = d->efc_D[i];
      for (int r = 0; r < nv; r++) {
        double jr = d->efc_J[i][r];
        if (jr == 0) continue;
        double djr = D * jr;
        for (int c = 0; c <= r; c++) d->H[r][c] += djr * d->efc_J[i][c];
      }
    } else if (st == ST_CONE && d->efc_type[i] == CN_CONTACT_ELLIPTIC) {
      KContact* c = d->contact + d->efc_id[i];
      int dim = c->dim;
      double mu = c->mu;
      double U[6], sc[6];
      sc[0] = mu;
      U[0] = d->jar[i] * mu;
      for (int j = 1; j < dim; j++) {
        sc[j] = c->friction[j - 1];
        U[j] = d->jar[i + j] * sc[j];
      }
      double T2 = 0;
      for (int j = 1; j < dim; j++) T2 += U[j] * U[j];
      double T = sqrt(T2);
      double N = U[0];
      double Dm = d->efc_D[i] / (mu * mu * (1 + mu * mu));
      double Hc[6][6];
      Hc[0][0] = 1;
      for (int j = 1; j < dim; j++) {
        Hc[0][j] = -mu * U[j] / T;
        Hc[j][0] = Hc[0][j];
      }
      double muNT = mu * N / T;
      for (int j = 1; j < dim; j++)
        for (int k = 1; k < dim; k++) Hc[j][k] = (j == k ? mu * mu - muNT : 0.0) + muNT * U[j] * U[k] / T2;
      for (int j = 0; j < dim; j++)
        for (int k = 0; k < dim; k++) Hc[j][k] = Hc[j][k] * Dm * sc[j] * sc[k];
      for (int r = 0; r < nv; r++) {
        double t[6];
        for (int j = 0; j < dim; j++) {
          double acc = 0;
          for (int k = 0; k < dim; k++) acc += Hc[j][k] * d->efc_J[i + k][r];
          t[j] = acc;
        }
        for (int cc = 0; cc <= r; cc++) {
          double acc = 0;
          for (int j = 0; j < dim; j++) acc += d->efc_J[i + j][cc] * t[j];
          d->H[r][cc] += acc;
        }
      }
      i += dim - 1;
    } else if (d->efc_type[i] == CN_CONTACT_ELLIPTIC) {
      i += d->contact[d->efc_id[i]].dim - 1;
    }
  }
  for (int j = 0; j < nv; j++) {
    double sum = d->H[j][j];
    for (int k = 0; k < j; k++) sum -= d->H[j][k] * d->H[j][k];
    if (sum < K_MINVAL) sum = K_MINVAL;
    double ljj = sqrt(sum);
    d->H[j][j] = ljj;
    for (int i = j + 1; i < nv; i++) {
      double v = d->H[i][j];
      for (int k = 0; k < j; k++) v -= d->H[i][k] * d->H[j][k];
      d->H[i][j] = v / ljj;
    }
  }
}

KD void k_hessian_solve(KModel m, const KData* d, double* x, const double* b) {
  const int nv = m->nv;
  for (int i = 0; i < nv; i++) {
    double v = b[i];
    for (int k = 0; k < i; k++) v -= d->H[i][k] * x[k];
    x[i] = v / d->H[i][i];
  }
  for (int i = nv - 1; i >= 0; i--) {
    double v = x[i];
    for (int k = nv - 1; k > i; k--) v -= d->H[k][i] * x[k];
    x[i] = v / d->H[i][i];
  }
}

KDN void k_ls_eval(KModel m, const KData* d, double a, double* f, double* df, double* d2f) {
  const int nv = m->nv;
  double g1 = 0, g2 = 0, g0 = d->gauss;
  for (int k = 0; k < nv; k++) {
    g1 += d->search[k] * (d->Ma[k] - d->qfrc_smooth[k]);
    g2 += d->search[k] * d->Mv[k];
  }
  double F = g0 + a * g1 + 0.5 * a * a * g2;
  double dF = g1 + a * g2;
  double d2F = g2;
  for (int i = 0; i < d->nefc; i++) {
    int t = d->efc_type[i];
    double D = d->efc_D[i], R = d->efc_R[i];
    double x = d->jar[i] + a * d->Jv[i];
    double v = d->Jv[i];
    if (t == CN_EQUALITY) {
      F += 0.5 * D * x * x; dF += D * x * v; d2F += D * v * v;
    } else if (t == CN_FRICTION_DOF) {
      double fl = d->efc_floss[i];
      if (x <= -R * fl) { F += -0.5 * R * fl * fl - fl * x; dF += -fl * v; }
      else if (x >= R * fl) { F += -0.5 * R * fl * fl + fl * x; dF += fl * v; }
      else { F += 0.5 * D * x * x; dF += D * x * v; d2F += D * v * v; }
    } else if (t == CN_LIMIT_JOINT) {
      if (x < 0) { F += 0.5 * D * x * x; dF += D * x * v; d2F += D * v * v; }
    } else {
      const KContact* c = d->contact + d->efc_id[i];
      int dim = c->dim;
      double mu = c->mu;
      double U[6], V[6];
      U[0] = (d->jar[i] + a * d->Jv[i]) * mu;
      V[0] = d->Jv[i] * mu;
      for (int j = 1; j < dim; j++) {
        U[j] = (d->jar[i + j] + a * d->Jv[i + j]) * c->friction[j - 1];
        V[j] = d->Jv[i + j] * c->friction[j - 1];
      }
      double N = U[0];
      double T2 = 0;
      for (int j = 1; j < dim; j++) T2 += U[j] * U[j];
      double T = sqrt(T2);
      if (N >= mu * T || (T <= 0 && N >= 0)) {
      } else if (mu * N + T <= 0 || (T <= 0 && N < 0)) {
        for (int j = 0; j < dim; j++) {
          double xj = d->jar[i + j] + a * d->Jv[i + j];
          double vj = d->Jv[i + j];
          double Dj = d->efc_D[i + j];
          F += 0.5 * Dj * xj * xj; dF += Dj * xj * vj; d2F += Dj * vj * vj;
        }
      } else {
        double Dm = d->efc_D[i] / (mu * mu * (1 + mu * mu));
        double UV = 0, VV = 0;
        for (int j = 1; j < dim; j++) { UV += U[j] * V[j]; VV += V[j] * V[j]; }
        double NT = N - mu * T;
        double dNT = V[0] - mu * UV / T;
        double d2NT = -mu * (VV * T2 - UV * UV) / (T2 * T);
        F += 0.5 * Dm * NT * NT;
        dF += Dm * NT * dNT;
        d2F += Dm * (dNT * dNT + NT * d2NT);
      }
      i += dim - 1;
    }
  }
  *f = F; *df = dF; *d2f = d2F;
}

KDN double k_line_search(KModel m, KData* d) {
  const int nv = m->nv;
  double snorm = 0;
  for (int k = 0; k < nv; k++) snorm += d->search[k] * d->search[k];
  snorm = sqrt(snorm);
  if (snorm < K_MINVAL) return 0;
  k_mul_M(m, d, d->Mv, d->search);
  for (int i = 0; i < d->nefc; i++) {
    double v = 0;
    for (int k = 0; k < nv; k++) v += d->efc_J[i][k] * d->search[k];
    d->Jv[i] = v;
  }
  double gtol = m->tolerance * m->ls_tolerance * snorm / d->scale;
  double f0, d0, h0;
  k_ls_eval(m, d, 0.0, &f0, &d0, &h0);
  if (d0 >= 0) return 0;
  double lo = 0.0, dlo = d0, hlo = h0;
  double hi = -1.0, dhi = 0, hhi = 0;
  double bestA = 0.0, bestF = f0;
  double a = -d0 / h0;
  for (int it = 0; it < m->ls_iterations; it++) {
    double f, df, d2f;
    k_ls_eval(m, d, a, &f, &df, &d2f);
    if (f < bestF) { bestF = f; bestA = a; }
    if (fabs(df) < gtol) return (f <= bestF) ? a : bestA;
    if (df < 0) { lo = a; dlo = df; hlo = d2f; }
    else { hi = a; dhi = df; hhi = d2f; }
    double na;
    if (hi < 0) {
      na = a - df / d2f;
      if (!(na > a)) na = 2 * a;
    } else {
      double c1 = lo - dlo / hlo;
      double c2 = hi - dhi / hhi;
      if (c1 > lo && c1 < hi) na = c1;
      else if (c2 > lo && c2 < hi) na = c2;
      else na = 0.5 * (lo + hi);
    }
    a = na;
  }
  return bestA;
}

KDN void k_solve_newton(KModel m, KData* d) {
  const int nv = m->nv;
  if (d->nefc == 0) {
    for (int k = 0; k < nv; k++) d->qacc[k] = d->qacc_smooth[k];
    for (int k = 0; k < nv; k++) d->qfrc_constraint[k] = 0;
    return;
  }
  d->scale = 1.0 / (m->meaninertia * (nv > 1 ? nv : 1));
  double qacc[K_NV];
  for (int k = 0; k < nv; k++) qacc[k] = d->qacc_warmstart[k];
  k_eval_state(m, d, qacc);
  double cost_ws = d->cost;
  k_eval_state(m, d, d->qacc_smooth);
  double cost_sm = d->cost;
  if (cost_ws > cost_sm) {
    for (int k = 0; k < nv; k++) qacc[k] = d->qacc_smooth[k];
  } else {
    k_eval_state(m, d, qacc);
  }
  k_compute_grad(m, d);
  k_hessian_factor(m, d);
  double Mgrad[K_NV];
  k_hessian_solve(m, d, Mgrad, d->grad);
  for (int k = 0; k < nv; k++) d->search[k] = -Mgrad[k];
  for (int iter = 0; iter < m->iterations; iter++) {
    double alpha = k_line_search(m, d);
    if (alpha == 0) break;
    for (int k = 0; k < nv; k++) qacc[k] += alpha * d->search[k];
    double oldcost = d->cost;
    k_eval_state(m, d, qacc);
    k_compute_grad(m, d);
    double gn = 0;
    for (int k = 0; k < nv; k++) gn += d->grad[k] * d->grad[k];
    double improvement = d->scale * (oldcost - d->cost);
    double gradient = d->scale * sqrt(gn);
    if (improvement < m->tolerance || gradient < m->tolerance) break;
    k_hessian_factor(m, d);
    k_hessian_solve(m, d, Mgrad, d->grad);
    for (int k = 0; k < nv; k++) d->search[k] = -Mgrad[k];
  }
  for (int k = 0; k < nv; k++) d->qacc[k] = qacc[k];
}

/* ================================================================== */
/* forward / step                                                      */
/* ================================================================== */
/* touch sensor ray test (mj_sensorAcc mjSENS_TOUCH): does the ray from p along dir hit the site box */
KD int k_ray_box_hit(const double sp[3], const double sm[9], const double ss[3], const double p[3],
                     const double dir[3]) {
  double lp[3], ld[3], dp[3] = {p[0] - sp[0], p[1] - sp[1], p[2] - sp[2]};
  k_mat_t_vec3(lp, sm, dp);
  k_mat_t_vec3(ld, sm, dir);
  double tmin = 0.0, tmax = 1e300;
  for (int k = 0; k < 3; k++) {
    if (fabs(ld[k]) < K_MINVAL) {
      if (lp[k] < -ss[k] || lp[k] > ss[k]) return 0;
    } else {
      double t1 = (-ss[k] - lp[k]) / ld[k], t2 = (ss[k] - lp[k]) / ld[k];
      if (t1 > t2) { double tt = t1; t1 = t2; t2 = tt; }
      if (t1 > tmin) tmin = t1;
      if (t2 < tmax) tmax = t2;
      if (tmin > tmax) return 0;
    }
  }
  return 1;
}

/* touch sensors, oracle sensor_touch (oracle/ur3e_oracle.c) */
KD void k_touch(KModel m, KData* d) {
  for (int s = 0; s < m->ntouch; s++) {
    int site = m->touch_site[s];
    int body = m->site_bodyid[site];
    double sum = 0;
    for (int ci = 0; ci < d->ncon; ci++) {
      const KContact* c = d->contact + ci;
      if (c->efc_address < 0) continue;
      int b1 = m->geom_bodyid[c->geom1], b2 = m->geom_bodyid[c->geom2];
      if (body != b1 && body != b2) continue;
      double fn = d->efc_force[c->efc_address];
      if (fn <= 0) continue;
      double ray[3] = {c->frame[0], c->frame[1], c->frame[2]};
      if (body == b2) { ray[0] = -ray[0]; ray[1] = -ray[1]; ray[2] = -ray[2]; }
      if (k_ray_box_hit(d->site_xpos[site], d->site_xmat[site], m->site_size[site], c->pos, ray)) sum += fn;
    }
    d->touch[s] = sum;
  }
}

KDN void k_forward(KModel m, KData* d) {
  const int nv = m->nv;
  k_kinematics(m, d);
  k_com_pos(m, d);
  k_transmission(m, d);
  k_crb(m, d);
  for (int i = 0; i < nv; i++)
    for (int j = 0; j < nv; j++) d->qLD[i][j] = d->qM[i][j];
  k_factor_tree(m, d->qLD, d->qLDiagInv);
  k_collision(m, d);
  k_make_constraint(m, d);
  k_com_vel(m, d);
  k_passive(m, d);
  k_rne(m, d);
  double qfrc_act[K_NV];
  k_actuation(m, d, qfrc_act);
  for (int k = 0; k < nv; k++) d->qfrc_smooth[k] = d->qfrc_passive[k] - d->qfrc_bias[k] + qfrc_act[k];
  k_solve_tree(m, d->qLD, d->qLDiagInv, d->qacc_smooth, d->qfrc_smooth);
  k_solve_newton(m, d);
  k_touch(m, d);
}

KD int k_is_bad(double x) { return x != x || x > K_MAXVAL || x < -K_MAXVAL; }

KD void k_reset_bad(KModel m, KData* d) {
  for (int k = 0; k < m->nq; k++) d->qpos[k] = m->qpos0[k];
  for (int k = 0; k < m->nv; k++) { d->qvel[k] = 0; d->qacc_warmstart[k] = 0; }
  d->nwarn++;
}

/* mj_step: check, forward, check, Euler with implicit damping */
KDN void k_step(KModel m, KData* d) {
  const int nq = m->nq, nv = m->nv;
  int bad = 0;
  for (int k = 0; k < nq; k++) bad |= k_is_bad(d->qpos[k]);
  for (int k = 0; k < nv; k++) bad |= k_is_bad(d->qvel[k]);
  if (bad) k_reset_bad(m, d);
  k_forward(m, d);
  bad = 0;
  for (int k = 0; k < nv; k++) bad |= k_is_bad(d->qacc[k]);
  if (bad) {
    k_reset_bad(m, d);
    k_forward(m, d);
  }
  double qacc_int[K_NV];
  int damped = 0;
  for (int k = 0; k < nv; k++) damped |= m->dof_damping[k] > 0;
  if (damped) {
    /* reuse H as the implicit-damping factor buffer (Newton state is dead here) */
    double hinv[K_NV], f[K_NV];
    for (int i = 0; i < nv; i++)
      for (int j = 0; j < nv; j++) d->H[i][j] = d->qM[i][j];
    for (int k = 0; k < nv; k++) d->H[k][k] += m->timestep * m->dof_damping[k];
    k_factor_tree(m, d->H, hinv);
    for (int k = 0; k < nv; k++) f[k] = d->qfrc_smooth[k] + d->qfrc_constraint[k];
    k_solve_tree(m, d->H, hinv, qacc_int, f);
  } else {
    for (int k = 0; k < nv; k++) qacc_int[k] = d->qacc[k];
  }
  double h = m->timestep;
  for (int k = 0; k < nv; k++) d->qvel[k] += h * qacc_int[k];
  for (int j = 0; j < m->njnt; j++) {
    int a = m->jnt_qposadr[j], v = m->jnt_dofadr[j];
    if (m->jnt_type[j] == UR3E_JNT_FREE) {
      d->qpos[a] += h * d->qvel[v];
      d->qpos[a + 1] += h * d->qvel[v + 1];
      d->qpos[a + 2] += h * d->qvel[v + 2];
      double w[3] = {d->qvel[v + 3], d->qvel[v + 4], d->qvel[v + 5]};
      double ang = h * k_normalize3(w);
      double qr[4];
      k_axis_angle_quat(qr, w, ang);
      double q[4] = {d->qpos[a + 3], d->qpos[a + 4], d->qpos[a + 5], d->qpos[a + 6]};
      k_normalize4(q);
      k_mul_quat(q, q, qr);
      d->qpos[a + 3] = q[0]; d->qpos[a + 4] = q[1]; d->qpos[a + 5] = q[2]; d->qpos[a + 6] = q[3];
    } else {
      d->qpos[a] += h * d->qvel[v];
    }
  }
  for (int k = 0; k < nv; k++) d->qacc_warmstart[k] = d->qacc[k];
}

#endif /* UR3E_ENGINE_H */
