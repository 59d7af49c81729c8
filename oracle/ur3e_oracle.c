/*
 * ur3e_oracle.c — CPU ORACLE (test infrastructure only; see ur3e_oracle.h).
 *
 * Scalar FP64 restatement of the MuJoCo 3.3.3 pipeline stages used by the
 * reference's env step plus the reference controller and
 * UR3eEnv2 epilogue.  Compile with -ffp-contract=off: the MI355X kernels in
 * ur3e_amd/csrc mirror the operation order of every function below so that
 * results agree bit-for-bit.
 */
#include "ur3e_oracle.h"

#include <math.h>
#include <string.h>

#include "../ur3e_amd/csrc/detmath.h"
#include "../ur3e_amd/csrc/convex.h"

#define MINVAL 1e-15
#define MINIMP 0.0001
#define MAXIMP 0.9999
#define MAXVAL 1e10

/* ===================================================================== */
/* small vector helpers (MuJoCo mju_* semantics)                          */
/* ===================================================================== */
static void mul_quat(double res[4], const double a[4], const double b[4]) {
  double r0 = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  double r1 = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  double r2 = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  double r3 = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  res[0] = r0; res[1] = r1; res[2] = r2; res[3] = r3;
}

static void rot_vec_quat(double res[3], const double v[3], const double q[4]) {
  if (v[0] == 0 && v[1] == 0 && v[2] == 0) {
    res[0] = res[1] = res[2] = 0;
  } else if (q[0] == 1 && q[1] == 0 && q[2] == 0 && q[3] == 0) {
    res[0] = v[0]; res[1] = v[1]; res[2] = v[2];
  } else {
    double t0 = q[0] * v[0] + q[2] * v[2] - q[3] * v[1];
    double t1 = q[0] * v[1] + q[3] * v[0] - q[1] * v[2];
    double t2 = q[0] * v[2] + q[1] * v[1] - q[2] * v[0];
    double r0 = v[0] + 2 * (q[2] * t2 - q[3] * t1);
    double r1 = v[1] + 2 * (q[3] * t0 - q[1] * t2);
    double r2 = v[2] + 2 * (q[1] * t1 - q[2] * t0);
    res[0] = r0; res[1] = r1; res[2] = r2;
  }
}

static void quat2mat(double r[9], const double q[4]) {
  if (q[0] == 1 && q[1] == 0 && q[2] == 0 && q[3] == 0) {
    r[0] = 1; r[1] = 0; r[2] = 0; r[3] = 0; r[4] = 1; r[5] = 0; r[6] = 0; r[7] = 0; r[8] = 1;
    return;
  }
  double q00 = q[0] * q[0], q01 = q[0] * q[1], q02 = q[0] * q[2], q03 = q[0] * q[3];
  double q11 = q[1] * q[1], q12 = q[1] * q[2], q13 = q[1] * q[3];
  double q22 = q[2] * q[2], q23 = q[2] * q[3], q33 = q[3] * q[3];
  r[0] = q00 + q11 - q22 - q33;
  r[4] = q00 - q11 + q22 - q33;
  r[8] = q00 - q11 - q22 + q33;
  r[1] = 2 * (q12 - q03);
  r[2] = 2 * (q13 + q02);
  r[3] = 2 * (q12 + q03);
  r[5] = 2 * (q23 - q01);
  r[6] = 2 * (q13 - q02);
  r[7] = 2 * (q23 + q01);
}

static void normalize4(double q[4]) {
  double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < MINVAL) {
    q[0] = 1; q[1] = q[2] = q[3] = 0;
  } else if (fabs(n - 1.0) > MINVAL) {
    q[0] /= n; q[1] /= n; q[2] /= n; q[3] /= n;
  }
}

static double normalize3(double v[3]) {
  double n = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
  if (n < MINVAL) {
    v[0] = 1; v[1] = 0; v[2] = 0;
    return 0;
  }
  v[0] /= n; v[1] /= n; v[2] /= n;
  return n;
}

static void axis_angle_quat(double q[4], const double axis[3], double angle) {
  if (angle == 0) {
    q[0] = 1; q[1] = q[2] = q[3] = 0;
    return;
  }
  double s = ur3e_sin(angle * 0.5);
  q[0] = ur3e_cos(angle * 0.5);
  q[1] = axis[0] * s; q[2] = axis[1] * s; q[3] = axis[2] * s;
}

static void mat_vec3(double r[3], const double m[9], const double v[3]) {
  double r0 = m[0] * v[0] + m[1] * v[1] + m[2] * v[2];
  double r1 = m[3] * v[0] + m[4] * v[1] + m[5] * v[2];
  double r2 = m[6] * v[0] + m[7] * v[1] + m[8] * v[2];
  r[0] = r0; r[1] = r1; r[2] = r2;
}

static void mat_t_vec3(double r[3], const double m[9], const double v[3]) {
  double r0 = m[0] * v[0] + m[3] * v[1] + m[6] * v[2];
  double r1 = m[1] * v[0] + m[4] * v[1] + m[7] * v[2];
  double r2 = m[2] * v[0] + m[5] * v[1] + m[8] * v[2];
  r[0] = r0; r[1] = r1; r[2] = r2;
}

static void cross3(double r[3], const double a[3], const double b[3]) {
  double r0 = a[1] * b[2] - a[2] * b[1];
  double r1 = a[2] * b[0] - a[0] * b[2];
  double r2 = a[0] * b[1] - a[1] * b[0];
  r[0] = r0; r[1] = r1; r[2] = r2;
}

static double dot3(const double a[3], const double b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

/* local -> global pose of an object attached to body b */
static void local2global(double xp[3], double xm[9], const double bxpos[3], const double bxquat[4],
                         const double bxmat[9], const double lpos[3], const double lquat[4]) {
  double t[3], q[4];
  mat_vec3(t, bxmat, lpos);
  xp[0] = bxpos[0] + t[0]; xp[1] = bxpos[1] + t[1]; xp[2] = bxpos[2] + t[2];
  mul_quat(q, bxquat, lquat);
  normalize4(q);
  quat2mat(xm, q);
}

/* ===================================================================== */
/* spatial algebra (MuJoCo conventions, [angular; linear])                */
/* ===================================================================== */
static void mul_inert_vec(double r[6], const double i[10], const double v[6]) {
  double r0 = i[0] * v[0] + i[3] * v[1] + i[4] * v[2] - i[8] * v[4] + i[7] * v[5];
  double r1 = i[3] * v[0] + i[1] * v[1] + i[5] * v[2] + i[8] * v[3] - i[6] * v[5];
  double r2 = i[4] * v[0] + i[5] * v[1] + i[2] * v[2] - i[7] * v[3] + i[6] * v[4];
  double r3 = i[8] * v[1] - i[7] * v[2] + i[9] * v[3];
  double r4 = i[6] * v[2] - i[8] * v[0] + i[9] * v[4];
  double r5 = i[7] * v[0] - i[6] * v[1] + i[9] * v[5];
  r[0] = r0; r[1] = r1; r[2] = r2; r[3] = r3; r[4] = r4; r[5] = r5;
}

static void cross_motion(double r[6], const double v[6], const double u[6]) {
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

static void cross_force(double r[6], const double v[6], const double f[6]) {
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

static double dot6(const double a[6], const double b[6]) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5];
}

/* ===================================================================== */
/* mj_kinematics                                                          */
/* ===================================================================== */
static void kinematics(const ur3e_model_t* m, ur3o_data* d) {
  d->xpos[0][0] = d->xpos[0][1] = d->xpos[0][2] = 0;
  d->xquat[0][0] = 1; d->xquat[0][1] = d->xquat[0][2] = d->xquat[0][3] = 0;
  quat2mat(d->xmat[0], d->xquat[0]);
  d->xipos[0][0] = d->xipos[0][1] = d->xipos[0][2] = 0;
  quat2mat(d->ximat[0], d->xquat[0]);
  for (int i = 1; i < m->nbody; i++) {
    int pid = m->body_parentid[i];
    double xpos[3], xquat[4];
    int jfirst = m->body_jntadr[i];
    if (m->body_jntnum[i] == 1 && m->jnt_type[jfirst] == UR3E_JNT_FREE) {
      int a = m->jnt_qposadr[jfirst];
      xpos[0] = d->qpos[a]; xpos[1] = d->qpos[a + 1]; xpos[2] = d->qpos[a + 2];
      xquat[0] = d->qpos[a + 3]; xquat[1] = d->qpos[a + 4]; xquat[2] = d->qpos[a + 5]; xquat[3] = d->qpos[a + 6];
      normalize4(xquat);
      d->xanchor[jfirst][0] = xpos[0]; d->xanchor[jfirst][1] = xpos[1]; d->xanchor[jfirst][2] = xpos[2];
      d->xaxis[jfirst][0] = 0; d->xaxis[jfirst][1] = 0; d->xaxis[jfirst][2] = 1;
    } else {
      double t[3];
      mat_vec3(t, d->xmat[pid], m->body_pos[i]);
      xpos[0] = d->xpos[pid][0] + t[0]; xpos[1] = d->xpos[pid][1] + t[1]; xpos[2] = d->xpos[pid][2] + t[2];
      mul_quat(xquat, d->xquat[pid], m->body_quat[i]);
      for (int k = 0; k < m->body_jntnum[i]; k++) {
        int j = jfirst + k;
        double xaxis[3], xanchor[3], qloc[4], vec[3];
        rot_vec_quat(xaxis, m->jnt_axis[j], xquat);
        rot_vec_quat(xanchor, m->jnt_pos[j], xquat);
        xanchor[0] += xpos[0]; xanchor[1] += xpos[1]; xanchor[2] += xpos[2];
        /* hinge only (ball/slide unused by the UR3e models) */
        int a = m->jnt_qposadr[j];
        axis_angle_quat(qloc, m->jnt_axis[j], d->qpos[a] - m->qpos0[a]);
        mul_quat(xquat, xquat, qloc);
        rot_vec_quat(vec, m->jnt_pos[j], xquat);
        xpos[0] = xanchor[0] - vec[0]; xpos[1] = xanchor[1] - vec[1]; xpos[2] = xanchor[2] - vec[2];
        memcpy(d->xanchor[j], xanchor, sizeof(xanchor));
        memcpy(d->xaxis[j], xaxis, sizeof(xaxis));
      }
    }
    normalize4(xquat);
    memcpy(d->xpos[i], xpos, sizeof(xpos));
    memcpy(d->xquat[i], xquat, sizeof(xquat));
    quat2mat(d->xmat[i], xquat);
    local2global(d->xipos[i], d->ximat[i], d->xpos[i], d->xquat[i], d->xmat[i], m->body_ipos[i], m->body_iquat[i]);
  }
  for (int g = 0; g < m->ngeom; g++) {
    int b = m->geom_bodyid[g];
    local2global(d->geom_xpos[g], d->geom_xmat[g], d->xpos[b], d->xquat[b], d->xmat[b], m->geom_pos[g],
                 m->geom_quat[g]);
  }
  for (int s = 0; s < m->nsite; s++) {
    int b = m->site_bodyid[s];
    local2global(d->site_xpos[s], d->site_xmat[s], d->xpos[b], d->xquat[b], d->xmat[b], m->site_pos[s],
                 m->site_quat[s]);
  }
}

/* ===================================================================== */
/* mj_comPos                                                              */
/* ===================================================================== */
static void com_pos(const ur3e_model_t* m, ur3o_data* d) {
  for (int i = 0; i < m->nbody; i++) {
    d->subtree_com[i][0] = d->xipos[i][0] * m->body_mass[i];
    d->subtree_com[i][1] = d->xipos[i][1] * m->body_mass[i];
    d->subtree_com[i][2] = d->xipos[i][2] * m->body_mass[i];
  }
  for (int i = m->nbody - 1; i > 0; i--) {
    int p = m->body_parentid[i];
    d->subtree_com[p][0] += d->subtree_com[i][0];
    d->subtree_com[p][1] += d->subtree_com[i][1];
    d->subtree_com[p][2] += d->subtree_com[i][2];
  }
  for (int i = 0; i < m->nbody; i++) {
    if (m->body_subtreemass[i] < MINVAL) {
      d->subtree_com[i][0] = d->xipos[i][0]; d->subtree_com[i][1] = d->xipos[i][1];
      d->subtree_com[i][2] = d->xipos[i][2];
    } else {
      double s = 1.0 / m->body_subtreemass[i];
      d->subtree_com[i][0] *= s; d->subtree_com[i][1] *= s; d->subtree_com[i][2] *= s;
    }
  }
  /* cinert: inertia about the root subtree com, world orientation */
  for (int i = 0; i < 10; i++) d->cinert[0][i] = 0;
  for (int i = 1; i < m->nbody; i++) {
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
  /* cdof */
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
        cross3(cr, ax, off);
        d->cdof[da + 3 + k][0] = ax[0]; d->cdof[da + 3 + k][1] = ax[1]; d->cdof[da + 3 + k][2] = ax[2];
        d->cdof[da + 3 + k][3] = cr[0]; d->cdof[da + 3 + k][4] = cr[1]; d->cdof[da + 3 + k][5] = cr[2];
      }
    } else {
      double cr[3];
      cross3(cr, d->xaxis[j], off);
      d->cdof[da][0] = d->xaxis[j][0]; d->cdof[da][1] = d->xaxis[j][1]; d->cdof[da][2] = d->xaxis[j][2];
      d->cdof[da][3] = cr[0]; d->cdof[da][4] = cr[1]; d->cdof[da][5] = cr[2];
    }
  }
}

/* ===================================================================== */
/* fixed tendons + actuator transmission                                  */
/* ===================================================================== */
static int dof_qposadr(const ur3e_model_t* m, int dof) {
  int j = m->dof_jntid[dof];
  return m->jnt_qposadr[j] + (dof - m->jnt_dofadr[j]);
}

static void tendon_transmission(const ur3e_model_t* m, ur3o_data* d) {
  for (int t = 0; t < m->ntendon; t++) {
    double len = 0;
    for (int k = 0; k < m->ten_num[t]; k++) len += m->ten_coef[t][k] * d->qpos[dof_qposadr(m, m->ten_dof[t][k])];
    d->ten_length[t] = len;
  }
  for (int a = 0; a < m->nu; a++) {
    for (int v = 0; v < m->nv; v++) d->actuator_moment[a][v] = 0;
    double g = m->act_gear[a];
    if (m->act_trntype[a] == UR3E_TRN_JOINT) {
      int j = m->act_trnid[a];
      d->actuator_length[a] = d->qpos[m->jnt_qposadr[j]] * g;
      d->actuator_moment[a][m->jnt_dofadr[j]] = g;
    } else {
      int t = m->act_trnid[a];
      d->actuator_length[a] = d->ten_length[t] * g;
      for (int k = 0; k < m->ten_num[t]; k++) d->actuator_moment[a][m->ten_dof[t][k]] = m->ten_coef[t][k] * g;
    }
  }
}

/* ===================================================================== */
/* mj_crb / mj_factorM / mj_solveM                                        */
/* ===================================================================== */
static void crb(const ur3e_model_t* m, ur3o_data* d) {
  memcpy(d->crb, d->cinert, sizeof(double) * 10 * m->nbody);
  for (int i = m->nbody - 1; i > 0; i--) {
    int p = m->body_parentid[i];
    if (p > 0)
      for (int k = 0; k < 10; k++) d->crb[p][k] += d->crb[i][k];
  }
  for (int i = 0; i < m->nv; i++)
    for (int j = 0; j < m->nv; j++) d->qM[i][j] = 0;
  for (int i = 0; i < m->nv; i++) {
    double buf[6];
    mul_inert_vec(buf, d->crb[m->dof_bodyid[i]], d->cdof[i]);
    d->qM[i][i] = m->dof_armature[i];
    for (int j = i; j >= 0; j = m->dof_parentid[j]) {
      d->qM[i][j] += dot6(d->cdof[j], buf);
      d->qM[j][i] = d->qM[i][j];
    }
  }
}

/* reverse-order sparse-tree LDL' (MuJoCo mj_factorI) on a dense array */
static void factor_tree(const ur3e_model_t* m, double A[UR3E_MAXNV][UR3E_MAXNV], double diaginv[UR3E_MAXNV]) {
  int nv = m->nv;
  for (int k = nv - 1; k >= 0; k--) {
    if (A[k][k] < MINVAL) A[k][k] = MINVAL;
    for (int i = m->dof_parentid[k]; i >= 0; i = m->dof_parentid[i]) {
      double tmp = A[k][i] / A[k][k];
      for (int j = i; j >= 0; j = m->dof_parentid[j]) A[i][j] -= A[k][j] * tmp;
      A[k][i] = tmp;
    }
  }
  for (int i = 0; i < nv; i++) diaginv[i] = 1.0 / A[i][i];
}

static void solve_tree(const ur3e_model_t* m, const double A[UR3E_MAXNV][UR3E_MAXNV],
                       const double diaginv[UR3E_MAXNV], double* x, const double* b) {
  int nv = m->nv;
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

static void mul_M(const ur3e_model_t* m, const ur3o_data* d, double* r, const double* v) {
  for (int i = 0; i < m->nv; i++) {
    double s = 0;
    for (int j = 0; j < m->nv; j++) s += d->qM[i][j] * v[j];
    r[i] = s;
  }
}

/* ===================================================================== */
/* Jacobians / object velocity                                            */
/* ===================================================================== */
/* dense point Jacobian of `body` at world point p: jacp/jacr 3 x nv, row-major, stride nv */
static void jac_point(const ur3e_model_t* m, const ur3o_data* d, int body, const double p[3], double* jacp,
                      double* jacr) {
  int nv = m->nv;
  if (jacp) for (int k = 0; k < 3 * nv; k++) jacp[k] = 0;
  if (jacr) for (int k = 0; k < 3 * nv; k++) jacr[k] = 0;
  /* last dof in the chain of `body` */
  int dof = -1;
  for (int b = body; b > 0 && dof < 0; b = m->body_parentid[b])
    if (m->body_dofnum[b]) dof = m->body_dofadr[b] + m->body_dofnum[b] - 1;
  const double* c = d->subtree_com[m->body_rootid[body]];
  double off[3] = {p[0] - c[0], p[1] - c[1], p[2] - c[2]};
  for (int j = dof; j >= 0; j = m->dof_parentid[j]) {
    const double* cd = d->cdof[j];
    if (jacp) {
      double cr[3];
      cross3(cr, cd, off);
      jacp[0 * nv + j] = cd[3] + cr[0];
      jacp[1 * nv + j] = cd[4] + cr[1];
      jacp[2 * nv + j] = cd[5] + cr[2];
    }
    if (jacr) {
      jacr[0 * nv + j] = cd[0];
      jacr[1 * nv + j] = cd[1];
      jacr[2 * nv + j] = cd[2];
    }
  }
}

void ur3o_jac_site(const ur3e_model_t* m, const ur3o_data* d, int site, double* jacp, double* jacr) {
  jac_point(m, d, m->site_bodyid[site], d->site_xpos[site], jacp, jacr);
}

/* mj_objectVelocity(mjOBJ_SITE, flg_local=0): [w, v] in world frame from cvel */
void ur3o_site_velocity(const ur3e_model_t* m, const ur3o_data* d, int site, double res[6]) {
  int b = m->site_bodyid[site];
  const double* cv = d->cvel[b];
  const double* c = d->subtree_com[m->body_rootid[b]];
  double dif[3] = {d->site_xpos[site][0] - c[0], d->site_xpos[site][1] - c[1], d->site_xpos[site][2] - c[2]};
  double cr[3];
  cross3(cr, dif, cv);
  res[0] = cv[0]; res[1] = cv[1]; res[2] = cv[2];
  res[3] = cv[3] - cr[0]; res[4] = cv[4] - cr[1]; res[5] = cv[5] - cr[2];
}

/* ===================================================================== */
/* collision                                                              */
/* ===================================================================== */
static void make_frame(double f[9], const double n[3]) {
  f[0] = n[0]; f[1] = n[1]; f[2] = n[2];
  normalize3(f);
  double y[3];
  if (fabs(f[1]) < 0.5) { y[0] = 0; y[1] = 1; y[2] = 0; }
  else { y[0] = 0; y[1] = 0; y[2] = 1; }
  double dd = f[0] * y[0] + f[1] * y[1] + f[2] * y[2];
  y[0] -= f[0] * dd; y[1] -= f[1] * dd; y[2] -= f[2] * dd;
  normalize3(y);
  f[3] = y[0]; f[4] = y[1]; f[5] = y[2];
  double z[3];
  cross3(z, f, y);
  f[6] = z[0]; f[7] = z[1]; f[8] = z[2];
}

typedef struct {
  double pos[3];
  double n[3];
  double dist;
} rawcon;

/* mjc_PlaneBox: plane (geom1) vs box (geom2); at most 4 corners */
static int plane_box(const double pp[3], const double pm[9], const double bp[3], const double bm[9],
                     const double bs[3], double margin, rawcon* out) {
  double n[3] = {pm[2], pm[5], pm[8]};
  double dif[3] = {bp[0] - pp[0], bp[1] - pp[1], bp[2] - pp[2]};
  double dist = dot3(n, dif);
  int cnt = 0;
  for (int i = 0; i < 8; i++) {
    double v[3] = {(i & 1) ? bs[0] : -bs[0], (i & 2) ? bs[1] : -bs[1], (i & 4) ? bs[2] : -bs[2]};
    double corner[3];
    mat_vec3(corner, bm, v);
    double ld = dot3(n, corner);
    if (dist + ld > margin || ld > 0) continue;
    rawcon* c = out + cnt;
    c->dist = dist + ld;
    c->n[0] = n[0]; c->n[1] = n[1]; c->n[2] = n[2];
    double h = c->dist * 0.5;
    c->pos[0] = corner[0] - n[0] * h + bp[0];
    c->pos[1] = corner[1] - n[1] * h + bp[1];
    c->pos[2] = corner[2] - n[2] * h + bp[2];
    if (++cnt >= 4) return cnt;
  }
  return cnt;
}

/* box-box: separating-axis test (3+3 face axes, 9 edge axes), face contacts
   by clipping the incident face against the reference face, edge-edge by
   closest points.  Normal points from box1 to box2; dist < 0 = penetration;
   pos = midpoint between the surfaces.  <= 8 contacts. */
static int box_box(const double p1[3], const double R1[9], const double s1[3], const double p2[3],
                   const double R2[9], const double s2[3], double margin, rawcon* out) {
  double a[3][3], b[3][3];
  for (int k = 0; k < 3; k++) {
    a[k][0] = R1[k]; a[k][1] = R1[3 + k]; a[k][2] = R1[6 + k];
    b[k][0] = R2[k]; b[k][1] = R2[3 + k]; b[k][2] = R2[6 + k];
  }
  double pp[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  double best = -1e300;
  int bestcode = -1;
  double bestax[3] = {0, 0, 0};
  /* face axes */
  for (int code = 0; code < 6; code++) {
    const double* ax = code < 3 ? a[code] : b[code - 3];
    double ext = 0;
    for (int k = 0; k < 3; k++) ext += s1[k] * fabs(dot3(a[k], ax));
    for (int k = 0; k < 3; k++) ext += s2[k] * fabs(dot3(b[k], ax));
    double s = fabs(dot3(pp, ax)) - ext;
    if (s > margin) return 0;
    if (s > best) {
      best = s; bestcode = code;
      bestax[0] = ax[0]; bestax[1] = ax[1]; bestax[2] = ax[2];
    }
  }
  /* edge axes */
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) {
      double u[3];
      cross3(u, a[i], b[j]);
      double len = sqrt(dot3(u, u));
      if (len < 1e-6) continue;
      u[0] /= len; u[1] /= len; u[2] /= len;
      double ext = 0;
      for (int k = 0; k < 3; k++) ext += s1[k] * fabs(dot3(a[k], u));
      for (int k = 0; k < 3; k++) ext += s2[k] * fabs(dot3(b[k], u));
      double s = fabs(dot3(pp, u)) - ext;
      if (s > margin) return 0;
      if (s * 1.05 > best) {
        best = s; bestcode = 6 + 3 * i + j;
        bestax[0] = u[0]; bestax[1] = u[1]; bestax[2] = u[2];
      }
    }
  }
  /* normal from box1 to box2 */
  double n[3] = {bestax[0], bestax[1], bestax[2]};
  if (dot3(pp, n) < 0) { n[0] = -n[0]; n[1] = -n[1]; n[2] = -n[2]; }

  if (bestcode >= 6) {
    int i = (bestcode - 6) / 3, j = (bestcode - 6) % 3;
    double pa[3] = {p1[0], p1[1], p1[2]}, pb[3] = {p2[0], p2[1], p2[2]};
    for (int k = 0; k < 3; k++) {
      if (k != i) {
        double sg = dot3(n, a[k]) > 0 ? 1.0 : -1.0;
        pa[0] += sg * s1[k] * a[k][0]; pa[1] += sg * s1[k] * a[k][1]; pa[2] += sg * s1[k] * a[k][2];
      }
      if (k != j) {
        double sg = dot3(n, b[k]) > 0 ? -1.0 : 1.0;
        pb[0] += sg * s2[k] * b[k][0]; pb[1] += sg * s2[k] * b[k][1]; pb[2] += sg * s2[k] * b[k][2];
      }
    }
    /* closest points of lines pa + t*ua and pb + u*ub */
    double w[3] = {pa[0] - pb[0], pa[1] - pb[1], pa[2] - pb[2]};
    double uaub = dot3(a[i], b[j]);
    double q1 = dot3(a[i], w), q2 = dot3(b[j], w);
    double den = 1.0 - uaub * uaub;
    double t = 0, u = 0;
    if (den > 1e-12) {
      t = (uaub * q2 - q1) / den;
      u = (q2 - uaub * q1) / den;
    }
    double ca[3] = {pa[0] + t * a[i][0], pa[1] + t * a[i][1], pa[2] + t * a[i][2]};
    double cb[3] = {pb[0] + u * b[j][0], pb[1] + u * b[j][1], pb[2] + u * b[j][2]};
    out[0].pos[0] = 0.5 * (ca[0] + cb[0]);
    out[0].pos[1] = 0.5 * (ca[1] + cb[1]);
    out[0].pos[2] = 0.5 * (ca[2] + cb[2]);
    out[0].n[0] = n[0]; out[0].n[1] = n[1]; out[0].n[2] = n[2];
    out[0].dist = best;
    return 1;
  }

  /* face contact: reference box owns the axis */
  int ref_is_1 = bestcode < 3;
  int fk = ref_is_1 ? bestcode : bestcode - 3;
  const double* rp = ref_is_1 ? p1 : p2;
  const double* ip = ref_is_1 ? p2 : p1;
  const double* rs = ref_is_1 ? s1 : s2;
  const double* is = ref_is_1 ? s2 : s1;
  double (*ra)[3] = ref_is_1 ? a : b;
  double (*ia)[3] = ref_is_1 ? b : a;
  /* outward normal of the reference face, toward the incident box */
  double nr[3] = {ref_is_1 ? n[0] : -n[0], ref_is_1 ? n[1] : -n[1], ref_is_1 ? n[2] : -n[2]};
  double rsg = dot3(nr, ra[fk]) > 0 ? 1.0 : -1.0;
  double cr[3] = {rp[0] + rsg * rs[fk] * ra[fk][0], rp[1] + rsg * rs[fk] * ra[fk][1], rp[2] + rsg * rs[fk] * ra[fk][2]};
  int t1 = (fk + 1) % 3, t2 = (fk + 2) % 3;
  /* incident face: most anti-parallel to nr */
  int im = 0;
  double bd = -1;
  double dm[3];
  for (int k = 0; k < 3; k++) {
    dm[k] = dot3(ia[k], nr);
    if (fabs(dm[k]) > bd) { bd = fabs(dm[k]); im = k; }
  }
  double isg = dm[im] > 0 ? -1.0 : 1.0;
  double ic[3] = {ip[0] + isg * is[im] * ia[im][0], ip[1] + isg * is[im] * ia[im][1], ip[2] + isg * is[im] * ia[im][2]};
  int u1 = (im + 1) % 3, u2 = (im + 2) % 3;
  /* incident quad in reference-face coordinates (x, y, h) */
  double poly[16][3], tmp[16][3];
  int np = 4;
  static const double sx[4] = {1, -1, -1, 1}, sy[4] = {1, 1, -1, -1};
  for (int k = 0; k < 4; k++) {
    double v[3];
    for (int c = 0; c < 3; c++) v[c] = ic[c] + sx[k] * is[u1] * ia[u1][c] + sy[k] * is[u2] * ia[u2][c] - cr[c];
    poly[k][0] = dot3(v, ra[t1]);
    poly[k][1] = dot3(v, ra[t2]);
    poly[k][2] = dot3(v, nr);
  }
  /* clip against |x| <= rs[t1], |y| <= rs[t2] */
  for (int e = 0; e < 4; e++) {
    int ax = e >> 1;                 /* 0: x, 1: y */
    double sgn = (e & 1) ? -1.0 : 1.0; /* keep sgn*coord <= lim */
    double lim = ax == 0 ? rs[t1] : rs[t2];
    int nn = 0;
    for (int k = 0; k < np; k++) {
      const double* P = poly[k];
      const double* Q = poly[(k + 1) % np];
      double dp = sgn * P[ax] - lim, dq = sgn * Q[ax] - lim;
      if (dp <= 0) {
        tmp[nn][0] = P[0]; tmp[nn][1] = P[1]; tmp[nn][2] = P[2];
        nn++;
      }
      if ((dp <= 0) != (dq <= 0)) {
        double tt = dp / (dp - dq);
        tmp[nn][0] = P[0] + tt * (Q[0] - P[0]);
        tmp[nn][1] = P[1] + tt * (Q[1] - P[1]);
        tmp[nn][2] = P[2] + tt * (Q[2] - P[2]);
        nn++;
      }
    }
    np = nn;
    for (int k = 0; k < np; k++) { poly[k][0] = tmp[k][0]; poly[k][1] = tmp[k][1]; poly[k][2] = tmp[k][2]; }
    if (np == 0) break;
  }
  int cnt = 0;
  for (int k = 0; k < np && cnt < 8; k++) {
    double h = poly[k][2];
    if (h > margin) continue;
    double w[3];
    for (int c = 0; c < 3; c++) w[c] = cr[c] + poly[k][0] * ra[t1][c] + poly[k][1] * ra[t2][c] + (h * 0.5) * nr[c];
    out[cnt].pos[0] = w[0]; out[cnt].pos[1] = w[1]; out[cnt].pos[2] = w[2];
    out[cnt].n[0] = n[0]; out[cnt].n[1] = n[1]; out[cnt].n[2] = n[2];
    out[cnt].dist = h;
    cnt++;
  }
  return cnt;
}

/* a geom as a convex shape: box (half sizes) or the hull of its mesh, at its current pose */
static void geom_convex(const ur3e_model_t* m, const ur3o_data* d, int g, ur3e_cvx* c) {
  if (m->geom_type[g] == UR3E_GEOM_MESH) {
    const int id = m->geom_dataid[g];
    c->v = &m->mesh_vert[m->mesh_vertadr[id]][0];
    c->nv = m->mesh_vertnum[id];
  } else {
    c->v = 0;
    c->nv = 0;
  }
  for (int k = 0; k < 3; k++) { c->size[k] = m->geom_size[g][k]; c->pos[k] = d->geom_xpos[g][k]; }
  for (int k = 0; k < 9; k++) c->mat[k] = d->geom_xmat[g][k];
}

/* convex mesh pairs (convex.h): plane-mesh (<= UR3E_CVX_PLANE_MAX contacts), box-mesh and mesh-mesh
   (GJK + EPA, one contact) */
static int mesh_collide(const ur3e_model_t* m, const ur3o_data* d, int g1, int g2, double margin, rawcon* out) {
  ur3e_cvx b;
  geom_convex(m, d, g2, &b);
  if (m->geom_type[g1] == UR3E_GEOM_PLANE) {
    double pos[UR3E_CVX_PLANE_MAX][3], nrm[UR3E_CVX_PLANE_MAX][3], dist[UR3E_CVX_PLANE_MAX];
    const int n = ur3e_plane_convex(d->geom_xpos[g1], d->geom_xmat[g1], &b, margin, pos, nrm, dist);
    for (int k = 0; k < n; k++) {
      memcpy(out[k].pos, pos[k], sizeof(out[k].pos));
      memcpy(out[k].n, nrm[k], sizeof(out[k].n));
      out[k].dist = dist[k];
    }
    return n;
  }
  ur3e_cvx a;
  geom_convex(m, d, g1, &a);
  ur3e_epa scratch;
  return ur3e_convex_convex(&a, &b, margin, &scratch, out[0].pos, out[0].n, &out[0].dist);
}

static void collision(const ur3e_model_t* m, ur3o_data* d) {
  d->ncon = 0;
  d->con_overflow = 0;
  rawcon raw[8];
  for (int p = 0; p < m->ncpair; p++) {
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
      n = plane_box(d->geom_xpos[g1], d->geom_xmat[g1], d->geom_xpos[g2], d->geom_xmat[g2], m->geom_size[g2], margin, raw);
    } else if (t1 == UR3E_GEOM_BOX && t2 == UR3E_GEOM_BOX) {
      n = box_box(d->geom_xpos[g1], d->geom_xmat[g1], m->geom_size[g1], d->geom_xpos[g2], d->geom_xmat[g2],
                  m->geom_size[g2], margin, raw);
    } else if (t2 == UR3E_GEOM_MESH) {
      n = mesh_collide(m, d, g1, g2, margin, raw);
    }
    for (int k = 0; k < n; k++) {
      if (d->ncon >= UR3E_MAXCON) { d->con_overflow = 1; break; }
      ur3o_contact* c = d->contact + d->ncon++;
      memcpy(c->pos, raw[k].pos, sizeof(c->pos));
      make_frame(c->frame, raw[k].n);
      c->dist = raw[k].dist;
      c->includemargin = margin - m->cpair_gap[p];
      for (int f = 0; f < 5; f++) c->friction[f] = m->cpair_friction[p][f];
      c->solref[0] = m->cpair_solref[p][0]; c->solref[1] = m->cpair_solref[p][1];
      for (int f = 0; f < 5; f++) c->solimp[f] = m->cpair_solimp[p][f];
      c->dim = m->cpair_condim[p];
      c->geom1 = g1; c->geom2 = g2;
      c->mu = 0;
      c->efc_address = -1;
    }
  }
}

/* ===================================================================== */
/* constraints: mj_makeConstraint + mj_makeImpedance / reference          */
/* ===================================================================== */
static int add_row(ur3o_data* d, int type, int id, double pos, double margin, double floss, double diag) {
  if (d->nefc >= UR3E_MAXEFC) { d->efc_overflow = 1; return -1; }
  int r = d->nefc++;
  d->efc_type[r] = type; d->efc_id[r] = id;
  d->efc_pos[r] = pos; d->efc_margin[r] = margin; d->efc_frictionloss[r] = floss; d->efc_diagApprox[r] = diag;
  return r;
}

static void make_constraint(const ur3e_model_t* m, ur3o_data* d) {
  int nv = m->nv;
  d->nefc = 0;
  d->efc_overflow = 0;
  double jp1[3 * UR3E_MAXNV], jp2[3 * UR3E_MAXNV];
  /* equality */
  for (int e = 0; e < m->neq; e++) {
    if (m->eq_type[e] == UR3E_EQ_CONNECT) {
      int b1 = m->eq_obj1[e], b2 = m->eq_obj2[e];
      double p1[3], p2[3];
      mat_vec3(p1, d->xmat[b1], m->eq_data[e]);
      p1[0] += d->xpos[b1][0]; p1[1] += d->xpos[b1][1]; p1[2] += d->xpos[b1][2];
      mat_vec3(p2, d->xmat[b2], m->eq_data[e] + 3);
      p2[0] += d->xpos[b2][0]; p2[1] += d->xpos[b2][1]; p2[2] += d->xpos[b2][2];
      jac_point(m, d, b1, p1, jp1, 0);
      jac_point(m, d, b2, p2, jp2, 0);
      double diag = m->body_invweight0[b1][0] + m->body_invweight0[b2][0];
      if (d->nefc + 3 > UR3E_MAXEFC) { d->efc_overflow = 1; return; }
      for (int k = 0; k < 3; k++) {
        int r = add_row(d, UR3O_CNSTR_EQUALITY, e, p1[k] - p2[k], 0, 0, diag);
        if (r < 0) return;
        for (int v = 0; v < nv; v++) d->efc_J[r][v] = jp1[k * nv + v] - jp2[k * nv + v];
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
      int r = add_row(d, UR3O_CNSTR_EQUALITY, e, pos, 0, 0, diag);
      if (r < 0) return;
      for (int v = 0; v < nv; v++) d->efc_J[r][v] = 0;
      d->efc_J[r][m->jnt_dofadr[j1]] = 1;
      if (j2 >= 0) d->efc_J[r][m->jnt_dofadr[j2]] = -dpoly;
    }
  }
  /* dof friction loss */
  for (int v = 0; v < nv; v++) {
    if (m->dof_frictionloss[v] > 0) {
      int r = add_row(d, UR3O_CNSTR_FRICTION_DOF, v, 0, 0, m->dof_frictionloss[v], m->dof_invweight0[v]);
      if (r < 0) return;
      for (int k = 0; k < nv; k++) d->efc_J[r][k] = 0;
      d->efc_J[r][v] = 1;
    }
  }
  /* joint limits (hinge/slide) */
  for (int j = 0; j < m->njnt; j++) {
    if (!m->jnt_limited[j]) continue;
    if (m->jnt_type[j] != UR3E_JNT_HINGE && m->jnt_type[j] != UR3E_JNT_SLIDE) continue;
    double q = d->qpos[m->jnt_qposadr[j]];
    for (int side = -1; side <= 1; side += 2) {
      double dist = side * (m->jnt_range[j][(side + 1) / 2] - q);
      if (dist < m->jnt_margin[j]) {
        int dof = m->jnt_dofadr[j];
        int r = add_row(d, UR3O_CNSTR_LIMIT_JOINT, j, dist, m->jnt_margin[j], 0, m->dof_invweight0[dof]);
        if (r < 0) return;
        for (int k = 0; k < nv; k++) d->efc_J[r][k] = 0;
        d->efc_J[r][dof] = -(double)side;
      }
    }
  }
  /* contacts (elliptic, condim 3) */
  for (int ci = 0; ci < d->ncon; ci++) {
    ur3o_contact* c = d->contact + ci;
    if (c->dim != 3) continue; /* only condim 3 is used by the UR3e models */
    int b1 = m->geom_bodyid[c->geom1], b2 = m->geom_bodyid[c->geom2];
    jac_point(m, d, b1, c->pos, jp1, 0);
    jac_point(m, d, b2, c->pos, jp2, 0);
    double diag = m->body_invweight0[b1][0] + m->body_invweight0[b2][0];
    if (d->nefc + 3 > UR3E_MAXEFC) { d->efc_overflow = 1; return; }
    c->efc_address = d->nefc;
    for (int k = 0; k < 3; k++) {
      int r = add_row(d, UR3O_CNSTR_CONTACT_ELLIPTIC, ci, c->dist, c->includemargin, 0, diag);
      if (r < 0) { c->efc_address = -1; return; }
      for (int v = 0; v < nv; v++) {
        double dj0 = jp2[0 * nv + v] - jp1[0 * nv + v];
        double dj1 = jp2[1 * nv + v] - jp1[1 * nv + v];
        double dj2 = jp2[2 * nv + v] - jp1[2 * nv + v];
        d->efc_J[r][v] = c->frame[3 * k] * dj0 + c->frame[3 * k + 1] * dj1 + c->frame[3 * k + 2] * dj2;
      }
    }
  }
}

static double get_impedance(const double* solimp, double pos, double margin) {
  double dmin = solimp[0], dmax = solimp[1], width = solimp[2], mid = solimp[3], power = solimp[4];
  if (dmin < MINIMP) dmin = MINIMP;
  if (dmin > MAXIMP) dmin = MAXIMP;
  if (dmax < MINIMP) dmax = MINIMP;
  if (dmax > MAXIMP) dmax = MAXIMP;
  if (dmin == dmax || width <= MINVAL) return 0.5 * (dmin + dmax);
  double x = (pos - margin) / width;
  if (x < 0) x = -x;
  if (x >= 1) return dmax;
  if (x <= 0) return dmin;
  double y;
  if (power == 1) {
    y = x;
  } else if (x <= mid) {
    /* integer power (the models use power = 2) */
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

static void make_impedance(const ur3e_model_t* m, ur3o_data* d) {
  for (int i = 0; i < d->nefc; i++) {
    const double *sref, *simp;
    int id = d->efc_id[i];
    switch (d->efc_type[i]) {
      case UR3O_CNSTR_EQUALITY: sref = m->eq_solref[id]; simp = m->eq_solimp[id]; break;
      case UR3O_CNSTR_FRICTION_DOF: sref = m->dof_solref[id]; simp = m->dof_solimp[id]; break;
      case UR3O_CNSTR_LIMIT_JOINT: sref = m->jnt_solref[id]; simp = m->jnt_solimp[id]; break;
      default: sref = d->contact[id].solref; simp = d->contact[id].solimp; break;
    }
    double imp = get_impedance(simp, d->efc_pos[i], d->efc_margin[i]);
    double dmax = simp[1];
    if (dmax < MINIMP) dmax = MINIMP;
    if (dmax > MAXIMP) dmax = MAXIMP;
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
    int friction_row = 0;
    if (d->efc_type[i] == UR3O_CNSTR_CONTACT_ELLIPTIC && i != d->contact[id].efc_address) friction_row = 1;
    if (d->efc_type[i] == UR3O_CNSTR_FRICTION_DOF) friction_row = 1;
    if (friction_row)
      d->efc_aref[i] = -B * d->efc_vel[i];
    else
      d->efc_aref[i] = -B * d->efc_vel[i] - K * imp * (d->efc_pos[i] - d->efc_margin[i]);
    double R = (1 - imp) * d->efc_diagApprox[i] / imp;
    d->efc_R[i] = R < MINVAL ? MINVAL : R;
  }
  /* elliptic friction regularisation */
  for (int ci = 0; ci < d->ncon; ci++) {
    ur3o_contact* c = d->contact + ci;
    int a = c->efc_address;
    if (a < 0) continue;
    d->efc_R[a + 1] = d->efc_R[a] / m->impratio;
    c->mu = c->friction[0] * sqrt(d->efc_R[a + 1] / d->efc_R[a]);
    for (int j = 1; j < c->dim - 1; j++)
      d->efc_R[a + j + 1] = d->efc_R[a + 1] * c->friction[0] * c->friction[0] / (c->friction[j] * c->friction[j]);
  }
  for (int i = 0; i < d->nefc; i++) d->efc_D[i] = 1.0 / d->efc_R[i];
}

/* ===================================================================== */
/* velocity stage: mj_comVel, mj_passive, mj_rne                          */
/* ===================================================================== */
static void com_vel(const ur3e_model_t* m, ur3o_data* d) {
  for (int k = 0; k < 6; k++) d->cvel[0][k] = 0;
  for (int i = 1; i < m->nbody; i++) {
    double cv[6];
    for (int k = 0; k < 6; k++) cv[k] = d->cvel[m->body_parentid[i]][k];
    int bda = m->body_dofadr[i];
    for (int j = 0; j < m->body_dofnum[i]; j++) {
      int dof = bda + j;
      int jt = m->jnt_type[m->dof_jntid[dof]];
      if (jt == UR3E_JNT_FREE) {
        /* translational: cdof_dot = 0, velocity += cdof*qvel for 3 dofs */
        for (int k = 0; k < 3; k++)
          for (int r = 0; r < 6; r++) d->cdof_dot[dof + k][r] = 0;
        double tmp[6] = {0, 0, 0, 0, 0, 0};
        for (int k = 0; k < 3; k++)
          for (int r = 0; r < 6; r++) tmp[r] += d->cdof[dof + k][r] * d->qvel[dof + k];
        for (int r = 0; r < 6; r++) cv[r] += tmp[r];
        /* rotational: all 3 cdof_dot with the same cvel */
        for (int k = 3; k < 6; k++) cross_motion(d->cdof_dot[dof + k], cv, d->cdof[dof + k]);
        for (int r = 0; r < 6; r++) tmp[r] = 0;
        for (int k = 3; k < 6; k++)
          for (int r = 0; r < 6; r++) tmp[r] += d->cdof[dof + k][r] * d->qvel[dof + k];
        for (int r = 0; r < 6; r++) cv[r] += tmp[r];
        j += 5;
      } else {
        cross_motion(d->cdof_dot[dof], cv, d->cdof[dof]);
        for (int r = 0; r < 6; r++) cv[r] += d->cdof[dof][r] * d->qvel[dof];
      }
    }
    for (int k = 0; k < 6; k++) d->cvel[i][k] = cv[k];
  }
}

static void rne(const ur3e_model_t* m, ur3o_data* d) {
  double cacc[UR3E_MAXBODY][6], cfrc[UR3E_MAXBODY][6];
  cacc[0][0] = cacc[0][1] = cacc[0][2] = 0;
  cacc[0][3] = -m->gravity[0]; cacc[0][4] = -m->gravity[1]; cacc[0][5] = -m->gravity[2];
  for (int k = 0; k < 6; k++) cfrc[0][k] = 0;
  for (int i = 1; i < m->nbody; i++) {
    double tmp[6] = {0, 0, 0, 0, 0, 0};
    int bda = m->body_dofadr[i];
    for (int j = 0; j < m->body_dofnum[i]; j++)
      for (int r = 0; r < 6; r++) tmp[r] += d->cdof_dot[bda + j][r] * d->qvel[bda + j];
    int p = m->body_parentid[i];
    for (int r = 0; r < 6; r++) cacc[i][r] = cacc[p][r] + tmp[r];
    double f1[6], f2[6], f3[6];
    mul_inert_vec(f1, d->cinert[i], cacc[i]);
    mul_inert_vec(f2, d->cinert[i], d->cvel[i]);
    cross_force(f3, d->cvel[i], f2);
    for (int r = 0; r < 6; r++) cfrc[i][r] = f1[r] + f3[r];
  }
  for (int i = m->nbody - 1; i > 0; i--) {
    int p = m->body_parentid[i];
    if (p > 0)
      for (int r = 0; r < 6; r++) cfrc[p][r] += cfrc[i][r];
  }
  for (int v = 0; v < m->nv; v++) d->qfrc_bias[v] = dot6(d->cdof[v], cfrc[m->dof_bodyid[v]]);
}

static void passive(const ur3e_model_t* m, ur3o_data* d) {
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

/* ===================================================================== */
/* actuation                                                              */
/* ===================================================================== */
static void actuation(const ur3e_model_t* m, ur3o_data* d) {
  for (int t = 0; t < m->ntendon; t++) {
    double v = 0;
    for (int k = 0; k < m->ten_num[t]; k++) v += m->ten_coef[t][k] * d->qvel[m->ten_dof[t][k]];
    d->ten_velocity[t] = v;
  }
  for (int v = 0; v < m->nv; v++) d->qfrc_actuator[v] = 0;
  for (int a = 0; a < m->nu; a++) {
    double vel = 0;
    for (int v = 0; v < m->nv; v++) vel += d->actuator_moment[a][v] * d->qvel[v];
    d->actuator_velocity[a] = vel;
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
    d->actuator_force[a] = f;
  }
  for (int v = 0; v < m->nv; v++) {
    double s = 0;
    for (int a = 0; a < m->nu; a++) s += d->actuator_moment[a][v] * d->actuator_force[a];
    d->qfrc_actuator[v] = s;
  }
}

/* ===================================================================== */
/* Newton solver (mj_solNewton semantics; elliptic cones)                  */
/* ===================================================================== */
typedef struct {
  const ur3e_model_t* m;
  ur3o_data* d;
  double jar[UR3E_MAXEFC];
  double Ma[UR3E_MAXNV];
  double grad[UR3E_MAXNV];
  double search[UR3E_MAXNV];
  double Mv[UR3E_MAXNV];
  double Jv[UR3E_MAXEFC];
  double H[UR3E_MAXNV][UR3E_MAXNV];
  double gauss, cost;
  double scale;
} solver_ctx;

/* forces, states and cost from jar (mj_constraintUpdate) */
static double constraint_update(const ur3e_model_t* m, ur3o_data* d, const double* jar) {
  double cost = 0;
  for (int i = 0; i < d->nefc; i++) {
    int t = d->efc_type[i];
    double D = d->efc_D[i], R = d->efc_R[i];
    if (t == UR3O_CNSTR_EQUALITY) {
      d->efc_force[i] = -D * jar[i];
      cost += 0.5 * D * jar[i] * jar[i];
      d->efc_state[i] = UR3O_STATE_QUADRATIC;
    } else if (t == UR3O_CNSTR_FRICTION_DOF) {
      double fl = d->efc_frictionloss[i];
      if (jar[i] <= -R * fl) {
        d->efc_force[i] = fl;
        cost += -0.5 * R * fl * fl - fl * jar[i];
        d->efc_state[i] = UR3O_STATE_LINEARNEG;
      } else if (jar[i] >= R * fl) {
        d->efc_force[i] = -fl;
        cost += -0.5 * R * fl * fl + fl * jar[i];
        d->efc_state[i] = UR3O_STATE_LINEARPOS;
      } else {
        d->efc_force[i] = -D * jar[i];
        cost += 0.5 * D * jar[i] * jar[i];
        d->efc_state[i] = UR3O_STATE_QUADRATIC;
      }
    } else if (t == UR3O_CNSTR_LIMIT_JOINT) {
      if (jar[i] >= 0) {
        d->efc_force[i] = 0;
        d->efc_state[i] = UR3O_STATE_SATISFIED;
      } else {
        d->efc_force[i] = -D * jar[i];
        cost += 0.5 * D * jar[i] * jar[i];
        d->efc_state[i] = UR3O_STATE_QUADRATIC;
      }
    } else { /* elliptic contact: handle the whole cone at its first row */
      ur3o_contact* c = d->contact + d->efc_id[i];
      int dim = c->dim;
      double mu = c->mu;
      double U[6];
      U[0] = jar[i] * mu;
      for (int j = 1; j < dim; j++) U[j] = jar[i + j] * c->friction[j - 1];
      double N = U[0];
      double T2 = 0;
      for (int j = 1; j < dim; j++) T2 += U[j] * U[j];
      double T = sqrt(T2);
      if (N >= mu * T || (T <= 0 && N >= 0)) {
        for (int j = 0; j < dim; j++) {
          d->efc_force[i + j] = 0;
          d->efc_state[i + j] = UR3O_STATE_SATISFIED;
        }
      } else if (mu * N + T <= 0 || (T <= 0 && N < 0)) {
        for (int j = 0; j < dim; j++) {
          d->efc_force[i + j] = -d->efc_D[i + j] * jar[i + j];
          cost += 0.5 * d->efc_D[i + j] * jar[i + j] * jar[i + j];
          d->efc_state[i + j] = UR3O_STATE_QUADRATIC;
        }
      } else {
        double Dm = d->efc_D[i] / (mu * mu * (1 + mu * mu));
        double NT = N - mu * T;
        cost += 0.5 * Dm * NT * NT;
        d->efc_force[i] = -Dm * NT * mu;
        for (int j = 1; j < dim; j++) d->efc_force[i + j] = Dm * NT * mu * U[j] / T * c->friction[j - 1];
        for (int j = 0; j < dim; j++) d->efc_state[i + j] = UR3O_STATE_CONE;
      }
      i += dim - 1;
    }
  }
  return cost;
}

static void eval_state(solver_ctx* s, const double* qacc) {
  const ur3e_model_t* m = s->m;
  ur3o_data* d = s->d;
  int nv = m->nv;
  mul_M(m, d, s->Ma, qacc);
  for (int i = 0; i < d->nefc; i++) {
    double v = 0;
    for (int k = 0; k < nv; k++) v += d->efc_J[i][k] * qacc[k];
    s->jar[i] = v - d->efc_aref[i];
  }
  double g = 0;
  for (int k = 0; k < nv; k++) g += (s->Ma[k] - d->qfrc_smooth[k]) * (qacc[k] - d->qacc_smooth[k]);
  s->gauss = 0.5 * g;
  s->cost = s->gauss + constraint_update(m, d, s->jar);
}

static void compute_grad(solver_ctx* s) {
  const ur3e_model_t* m = s->m;
  ur3o_data* d = s->d;
  int nv = m->nv;
  for (int k = 0; k < nv; k++) {
    double f = 0;
    for (int i = 0; i < d->nefc; i++) f += d->efc_J[i][k] * d->efc_force[i];
    d->qfrc_constraint[k] = f;
  }
  for (int k = 0; k < nv; k++) s->grad[k] = s->Ma[k] - d->qfrc_smooth[k] - d->qfrc_constraint[k];
}

/* H = M + J' D J (quadratic rows) + cone Hessians; dense Cholesky in place */
static void hessian_factor(solver_ctx* s) {
  const ur3e_model_t* m = s->m;
  ur3o_data* d = s->d;
  int nv = m->nv;
  for (int r = 0; r < nv; r++)
    for (int c = 0; c < nv; c++) s->H[r][c] = d->qM[r][c];
  for (int i = 0; i < d->nefc; i++) {
    int st = d->efc_state[i];
    if (st == UR3O_STATE_QUADRATIC) {
      double D = d->efc_D[i];
      for (int r = 0; r < nv; r++) {
        double jr = d->efc_J[i][r];
        if (jr == 0) continue;
        double djr = D * jr;
        for (int c = 0; c <= r; c++) s->H[r][c] += djr * d->efc_J[i][c];
      }
    } else if (st == UR3O_STATE_CONE && d->efc_type[i] == UR3O_CNSTR_CONTACT_ELLIPTIC) {
      ur3o_contact* c = d->contact + d->efc_id[i];
      int dim = c->dim;
      double mu = c->mu;
      double U[6], sc[6];
      sc[0] = mu;
      U[0] = s->jar[i] * mu;
      for (int j = 1; j < dim; j++) {
        sc[j] = c->friction[j - 1];
        U[j] = s->jar[i + j] * sc[j];
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
        for (int k = 1; k < dim; k++)
          Hc[j][k] = (j == k ? mu * mu - muNT : 0.0) + muNT * U[j] * U[k] / T2;
      for (int j = 0; j < dim; j++)
        for (int k = 0; k < dim; k++) Hc[j][k] = Hc[j][k] * Dm * sc[j] * sc[k];
      /* H += Jc' Hc Jc */
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
          s->H[r][cc] += acc;
        }
      }
      i += dim - 1;
    } else if (d->efc_type[i] == UR3O_CNSTR_CONTACT_ELLIPTIC) {
      i += d->contact[d->efc_id[i]].dim - 1;
    }
  }
  /* Cholesky, lower: H = L L' */
  for (int j = 0; j < nv; j++) {
    double sum = s->H[j][j];
    for (int k = 0; k < j; k++) sum -= s->H[j][k] * s->H[j][k];
    if (sum < MINVAL) sum = MINVAL;
    double ljj = sqrt(sum);
    s->H[j][j] = ljj;
    for (int i = j + 1; i < nv; i++) {
      double v = s->H[i][j];
      for (int k = 0; k < j; k++) v -= s->H[i][k] * s->H[j][k];
      s->H[i][j] = v / ljj;
    }
  }
}

static void hessian_solve(const solver_ctx* s, double* x, const double* b) {
  int nv = s->m->nv;
  for (int i = 0; i < nv; i++) {
    double v = b[i];
    for (int k = 0; k < i; k++) v -= s->H[i][k] * x[k];
    x[i] = v / s->H[i][i];
  }
  for (int i = nv - 1; i >= 0; i--) {
    double v = x[i];
    for (int k = nv - 1; k > i; k--) v -= s->H[k][i] * x[k];
    x[i] = v / s->H[i][i];
  }
}

/* 1-D cost, derivative and curvature along the search direction at step a */
static void ls_eval(const solver_ctx* s, double a, double* f, double* df, double* d2f) {
  const ur3o_data* d = s->d;
  int nv = s->m->nv;
  double g1 = 0, g2 = 0, g0 = s->gauss;
  for (int k = 0; k < nv; k++) {
    g1 += s->search[k] * (s->Ma[k] - d->qfrc_smooth[k]);
    g2 += s->search[k] * s->Mv[k];
  }
  double F = g0 + a * g1 + 0.5 * a * a * g2;
  double dF = g1 + a * g2;
  double d2F = g2;
  for (int i = 0; i < d->nefc; i++) {
    int t = d->efc_type[i];
    double D = d->efc_D[i], R = d->efc_R[i];
    double x = s->jar[i] + a * s->Jv[i];
    double v = s->Jv[i];
    if (t == UR3O_CNSTR_EQUALITY) {
      F += 0.5 * D * x * x; dF += D * x * v; d2F += D * v * v;
    } else if (t == UR3O_CNSTR_FRICTION_DOF) {
      double fl = d->efc_frictionloss[i];
      if (x <= -R * fl) { F += -0.5 * R * fl * fl - fl * x; dF += -fl * v; }
      else if (x >= R * fl) { F += -0.5 * R * fl * fl + fl * x; dF += fl * v; }
      else { F += 0.5 * D * x * x; dF += D * x * v; d2F += D * v * v; }
    } else if (t == UR3O_CNSTR_LIMIT_JOINT) {
      if (x < 0) { F += 0.5 * D * x * x; dF += D * x * v; d2F += D * v * v; }
    } else {
      const ur3o_contact* c = d->contact + d->efc_id[i];
      int dim = c->dim;
      double mu = c->mu;
      double U[6], V[6];
      U[0] = (s->jar[i] + a * s->Jv[i]) * mu;
      V[0] = s->Jv[i] * mu;
      for (int j = 1; j < dim; j++) {
        U[j] = (s->jar[i + j] + a * s->Jv[i + j]) * c->friction[j - 1];
        V[j] = s->Jv[i + j] * c->friction[j - 1];
      }
      double N = U[0];
      double T2 = 0;
      for (int j = 1; j < dim; j++) T2 += U[j] * U[j];
      double T = sqrt(T2);
      if (N >= mu * T || (T <= 0 && N >= 0)) {
        /* satisfied */
      } else if (mu * N + T <= 0 || (T <= 0 && N < 0)) {
        for (int j = 0; j < dim; j++) {
          double xj = s->jar[i + j] + a * s->Jv[i + j];
          double vj = s->Jv[i + j];
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

static double line_search(solver_ctx* s) {
  const ur3e_model_t* m = s->m;
  ur3o_data* d = s->d;
  int nv = m->nv;
  double snorm = 0;
  for (int k = 0; k < nv; k++) snorm += s->search[k] * s->search[k];
  snorm = sqrt(snorm);
  if (snorm < MINVAL) return 0;
  mul_M(m, d, s->Mv, s->search);
  for (int i = 0; i < d->nefc; i++) {
    double v = 0;
    for (int k = 0; k < nv; k++) v += d->efc_J[i][k] * s->search[k];
    s->Jv[i] = v;
  }
  double gtol = m->tolerance * m->ls_tolerance * snorm / s->scale;
  double f0, d0, h0;
  ls_eval(s, 0.0, &f0, &d0, &h0);
  if (d0 >= 0) return 0;
  double lo = 0.0, dlo = d0, hlo = h0;
  double hi = -1.0, dhi = 0, hhi = 0;
  double bestA = 0.0, bestF = f0;
  double a = -d0 / h0;
  for (int it = 0; it < m->ls_iterations; it++) {
    double f, df, d2f;
    ls_eval(s, a, &f, &df, &d2f);
    if (f < bestF) { bestF = f; bestA = a; }
    if (fabs(df) < gtol) return (f <= bestF) ? a : bestA;
    if (df < 0) { lo = a; dlo = df; hlo = d2f; }
    else { hi = a; dhi = df; hhi = d2f; }
    double na;
    if (hi < 0) {
      na = a - df / d2f; /* no upper bracket yet: Newton step forward */
      if (!(na > a)) na = 2 * a;
    } else {
      double c1 = lo - dlo / hlo; /* Newton from both ends, keep if inside */
      double c2 = hi - dhi / hhi;
      if (c1 > lo && c1 < hi) na = c1;
      else if (c2 > lo && c2 < hi) na = c2;
      else na = 0.5 * (lo + hi);
    }
    a = na;
  }
  return bestA;
}

static void solve_newton(const ur3e_model_t* m, ur3o_data* d) {
  int nv = m->nv;
  d->solver_niter = 0;
  if (d->nefc == 0) {
    for (int k = 0; k < nv; k++) d->qacc[k] = d->qacc_smooth[k];
    for (int k = 0; k < nv; k++) d->qfrc_constraint[k] = 0;
    return;
  }
  solver_ctx sctx;
  solver_ctx* s = &sctx;
  s->m = m; s->d = d;
  s->scale = 1.0 / (m->meaninertia * (nv > 1 ? nv : 1));
  /* warmstart: keep the cheaper of qacc_warmstart and qacc_smooth */
  double qacc[UR3E_MAXNV];
  for (int k = 0; k < nv; k++) qacc[k] = d->qacc_warmstart[k];
  eval_state(s, qacc);
  double cost_ws = s->cost;
  eval_state(s, d->qacc_smooth);
  double cost_sm = s->cost;
  if (cost_ws > cost_sm) {
    for (int k = 0; k < nv; k++) qacc[k] = d->qacc_smooth[k];
  } else {
    eval_state(s, qacc);
  }
  compute_grad(s);
  hessian_factor(s);
  double Mgrad[UR3E_MAXNV];
  hessian_solve(s, Mgrad, s->grad);
  for (int k = 0; k < nv; k++) s->search[k] = -Mgrad[k];
  for (int iter = 0; iter < m->iterations; iter++) {
    double alpha = line_search(s);
    d->solver_niter = iter + 1;
    if (alpha == 0) break;
    for (int k = 0; k < nv; k++) qacc[k] += alpha * s->search[k];
    double oldcost = s->cost;
    eval_state(s, qacc);
    compute_grad(s);
    double gn = 0;
    for (int k = 0; k < nv; k++) gn += s->grad[k] * s->grad[k];
    double improvement = s->scale * (oldcost - s->cost);
    double gradient = s->scale * sqrt(gn);
    if (improvement < m->tolerance || gradient < m->tolerance) break;
    hessian_factor(s);
    hessian_solve(s, Mgrad, s->grad);
    for (int k = 0; k < nv; k++) s->search[k] = -Mgrad[k];
  }
  for (int k = 0; k < nv; k++) d->qacc[k] = qacc[k];
}

/* ===================================================================== */
/* touch sensors (mj_sensorAcc, mjSENS_TOUCH)                             */
/* ===================================================================== */
static int ray_box_hit(const double sp[3], const double sm[9], const double ss[3], const double p[3],
                       const double dir[3]) {
  double lp[3], ld[3], dp[3] = {p[0] - sp[0], p[1] - sp[1], p[2] - sp[2]};
  mat_t_vec3(lp, sm, dp);
  mat_t_vec3(ld, sm, dir);
  double tmin = 0.0, tmax = 1e300;
  for (int k = 0; k < 3; k++) {
    if (fabs(ld[k]) < MINVAL) {
      if (lp[k] < -ss[k] || lp[k] > ss[k]) return 0;
    } else {
      double t1 = (-ss[k] - lp[k]) / ld[k], t2 = (ss[k] - lp[k]) / ld[k];
      if (t1 > t2) { double t = t1; t1 = t2; t2 = t; }
      if (t1 > tmin) tmin = t1;
      if (t2 < tmax) tmax = t2;
      if (tmin > tmax) return 0;
    }
  }
  return 1;
}

static void sensor_touch(const ur3e_model_t* m, ur3o_data* d) {
  for (int s = 0; s < m->ntouch; s++) {
    int site = m->touch_site[s];
    int body = m->site_bodyid[site];
    double sum = 0;
    for (int ci = 0; ci < d->ncon; ci++) {
      const ur3o_contact* c = d->contact + ci;
      if (c->efc_address < 0) continue;
      int b1 = m->geom_bodyid[c->geom1], b2 = m->geom_bodyid[c->geom2];
      if (body != b1 && body != b2) continue;
      double fn = d->efc_force[c->efc_address];
      if (fn <= 0) continue;
      double ray[3] = {c->frame[0], c->frame[1], c->frame[2]};
      if (body == b2) { ray[0] = -ray[0]; ray[1] = -ray[1]; ray[2] = -ray[2]; }
      if (ray_box_hit(d->site_xpos[site], d->site_xmat[site], m->site_size[site], c->pos, ray)) sum += fn;
    }
    d->touch[s] = sum;
  }
}

/* ===================================================================== */
/* mj_rnePostConstraint + mj_sensorAcc (actuatorfrc, torque)              */
/* ===================================================================== */
/* mju_mulDofVec: res = sum_j mat[j] * vec[j] over n dof rows (n == 1: a scaled copy; MuJoCo's
   mju_mulMatTVec skips zero multipliers) */
static void mul_dof_vec(double res[6], const double (*mat)[6], const double* vec, int n) {
  if (n == 1) {
    for (int k = 0; k < 6; k++) res[k] = mat[0][k] * vec[0];
    return;
  }
  for (int k = 0; k < 6; k++) res[k] = 0;
  for (int j = 0; j < n; j++) {
    double t = vec[j];
    if (t == 0) continue;
    for (int k = 0; k < 6; k++) res[k] += mat[j][k] * t;
  }
}

/* mju_transformSpatial for a force vector [torque; force]: move the torque's reference point from
   oldpos to newpos, then (rot != NULL) rotate both halves into the frame `rot` (new -> old) */
static void transform_force(double res[6], const double vec[6], const double newpos[3], const double oldpos[3],
                            const double* rot) {
  double dif[3] = {newpos[0] - oldpos[0], newpos[1] - oldpos[1], newpos[2] - oldpos[2]};
  double cros[3], tran[6];
  cross3(cros, dif, vec + 3);
  tran[0] = vec[0] - cros[0]; tran[1] = vec[1] - cros[1]; tran[2] = vec[2] - cros[2];
  tran[3] = vec[3]; tran[4] = vec[4]; tran[5] = vec[5];
  if (rot) {
    mat_t_vec3(res, rot, tran);
    mat_t_vec3(res + 3, rot, tran + 3);
  } else {
    for (int k = 0; k < 6; k++) res[k] = tran[k];
  }
}

/* MuJoCo 3.3.3 mj_rnePostConstraint: body accelerations and interaction forces after the
   constraint solve; external forces from contacts (elliptic: mj_contactForce = efc_force of the
   cone rows, no torque for condim 3) and connect equalities (force at the anchors) */
static void rne_post_constraint(const ur3e_model_t* m, ur3o_data* d) {
  int nb = m->nbody;
  for (int k = 0; k < 6; k++) d->cacc[0][k] = 0;
  d->cacc[0][3] = m->gravity[0] * -1; d->cacc[0][4] = m->gravity[1] * -1; d->cacc[0][5] = m->gravity[2] * -1;
  for (int i = 0; i < nb; i++)
    for (int k = 0; k < 6; k++) d->cfrc_ext[i][k] = 0;
  double cfrc[6], com[6];
  for (int ci = 0; ci < d->ncon; ci++) {
    const ur3o_contact* c = d->contact + ci;
    if (c->efc_address < 0) continue;
    double lfrc[3] = {d->efc_force[c->efc_address], d->efc_force[c->efc_address + 1],
                      d->efc_force[c->efc_address + 2]};
    double zero[3] = {0, 0, 0};
    mat_t_vec3(cfrc, c->frame, zero);
    mat_t_vec3(cfrc + 3, c->frame, lfrc);
    int k = m->geom_bodyid[c->geom1];
    if (k) {
      transform_force(com, cfrc, d->subtree_com[m->body_rootid[k]], c->pos, 0);
      for (int r = 0; r < 6; r++) d->cfrc_ext[k][r] -= com[r];
    }
    k = m->geom_bodyid[c->geom2];
    if (k) {
      transform_force(com, cfrc, d->subtree_com[m->body_rootid[k]], c->pos, 0);
      for (int r = 0; r < 6; r++) d->cfrc_ext[k][r] += com[r];
    }
  }
  /* equality rows lead the constraint list (make_constraint) */
  int i = 0;
  while (i < d->nefc && d->efc_type[i] == UR3O_CNSTR_EQUALITY) {
    int e = d->efc_id[i];
    if (m->eq_type[e] == UR3E_EQ_CONNECT) {
      cfrc[0] = cfrc[1] = cfrc[2] = 0;
      cfrc[3] = d->efc_force[i]; cfrc[4] = d->efc_force[i + 1]; cfrc[5] = d->efc_force[i + 2];
      for (int side = 0; side < 2; side++) {
        int k = side == 0 ? m->eq_obj1[e] : m->eq_obj2[e];
        if (!k) continue;
        double pos[3];
        mat_vec3(pos, d->xmat[k], m->eq_data[e] + 3 * side);
        pos[0] += d->xpos[k][0]; pos[1] += d->xpos[k][1]; pos[2] += d->xpos[k][2];
        transform_force(com, cfrc, d->subtree_com[m->body_rootid[k]], pos, 0);
        if (side == 0)
          for (int r = 0; r < 6; r++) d->cfrc_ext[k][r] += com[r];
        else
          for (int r = 0; r < 6; r++) d->cfrc_ext[k][r] -= com[r];
      }
      i += 3;
    } else {
      i++;
    }
  }
  for (int b = 1; b < nb; b++) {
    int bda = m->body_dofadr[b], n = m->body_dofnum[b];
    double tmp[6], tmp1[6];
    if (n > 0) mul_dof_vec(tmp, (const double(*)[6])d->cdof_dot[bda], d->qvel + bda, n);
    else for (int k = 0; k < 6; k++) tmp[k] = 0;
    int p = m->body_parentid[b];
    for (int k = 0; k < 6; k++) d->cacc[b][k] = d->cacc[p][k] + tmp[k];
    if (n > 0) mul_dof_vec(tmp, (const double(*)[6])d->cdof[bda], d->qacc + bda, n);
    else for (int k = 0; k < 6; k++) tmp[k] = 0;
    for (int k = 0; k < 6; k++) d->cacc[b][k] += tmp[k];
    mul_inert_vec(d->cfrc_int[b], d->cinert[b], d->cacc[b]);
    mul_inert_vec(tmp, d->cinert[b], d->cvel[b]);
    cross_force(tmp1, d->cvel[b], tmp);
    for (int k = 0; k < 6; k++) d->cfrc_int[b][k] += tmp1[k];
    for (int k = 0; k < 6; k++) d->cfrc_int[b][k] -= d->cfrc_ext[b][k];
  }
  for (int b = nb - 1; b > 0; b--) {
    int p = m->body_parentid[b];
    if (p)
      for (int k = 0; k < 6; k++) d->cfrc_int[p][k] += d->cfrc_int[b][k];
  }
}

/* mjData.sensordata in declaration order (touch from sensor_touch) */
static void sensors(const ur3e_model_t* m, ur3o_data* d) {
  int post = 0;
  for (int k = 0; k < m->nsensor; k++) post |= m->sensor_type[k] == UR3E_SENS_TORQUE;
  if (post) rne_post_constraint(m, d);
  int nt = 0;
  for (int k = 0; k < m->nsensor; k++) {
    double* out = d->sensordata + m->sensor_adr[k];
    int obj = m->sensor_objid[k];
    if (m->sensor_type[k] == UR3E_SENS_TOUCH) {
      out[0] = d->touch[nt++];
    } else if (m->sensor_type[k] == UR3E_SENS_ACTUATORFRC) {
      out[0] = d->actuator_force[obj];
    } else {
      int body = m->site_bodyid[obj];
      double res[6];
      transform_force(res, d->cfrc_int[body], d->site_xpos[obj], d->subtree_com[m->body_rootid[body]],
                      d->site_xmat[obj]);
      out[0] = res[0]; out[1] = res[1]; out[2] = res[2];
    }
  }
}

/* ===================================================================== */
/* forward / step                                                         */
/* ===================================================================== */
void ur3o_reset_data(const ur3e_model_t* m, ur3o_data* d) {
  memset(d, 0, sizeof(*d));
  for (int k = 0; k < m->nq; k++) d->qpos[k] = m->qpos0[k];
}

void ur3o_forward(const ur3e_model_t* m, ur3o_data* d) {
  int nv = m->nv;
  /* position */
  kinematics(m, d);
  com_pos(m, d);
  tendon_transmission(m, d);
  crb(m, d);
  memcpy(d->qLD, d->qM, sizeof(d->qM));
  factor_tree(m, d->qLD, d->qLDiagInv);
  collision(m, d);
  make_constraint(m, d);
  /* velocity */
  com_vel(m, d);
  passive(m, d);
  for (int i = 0; i < d->nefc; i++) {
    double v = 0;
    for (int k = 0; k < nv; k++) v += d->efc_J[i][k] * d->qvel[k];
    d->efc_vel[i] = v;
  }
  make_impedance(m, d);
  rne(m, d);
  /* actuation + smooth acceleration */
  actuation(m, d);
  for (int k = 0; k < nv; k++) d->qfrc_smooth[k] = d->qfrc_passive[k] - d->qfrc_bias[k] + d->qfrc_actuator[k];
  solve_tree(m, d->qLD, d->qLDiagInv, d->qacc_smooth, d->qfrc_smooth);
  /* constraint solve */
  solve_newton(m, d);
  sensor_touch(m, d);
  sensors(m, d);
}

static int is_bad(double x) { return x != x || x > MAXVAL || x < -MAXVAL; }

static void reset_bad(const ur3e_model_t* m, ur3o_data* d) {
  for (int k = 0; k < m->nq; k++) d->qpos[k] = m->qpos0[k];
  for (int k = 0; k < m->nv; k++) { d->qvel[k] = 0; d->qacc_warmstart[k] = 0; }
  d->time = 0;
  d->nwarning_bad++;
}

void ur3o_step(const ur3e_model_t* m, ur3o_data* d) {
  int nq = m->nq, nv = m->nv;
  int bad = 0;
  for (int k = 0; k < nq; k++) bad |= is_bad(d->qpos[k]);
  for (int k = 0; k < nv; k++) bad |= is_bad(d->qvel[k]);
  if (bad) reset_bad(m, d);
  ur3o_forward(m, d);
  bad = 0;
  for (int k = 0; k < nv; k++) bad |= is_bad(d->qacc[k]);
  if (bad) {
    reset_bad(m, d);
    ur3o_forward(m, d);
  }
  /* Euler with implicit dof damping (mj_Euler) */
  double qacc_int[UR3E_MAXNV];
  int damped = 0;
  for (int k = 0; k < nv; k++) damped |= m->dof_damping[k] > 0;
  if (damped) {
    double H[UR3E_MAXNV][UR3E_MAXNV];
    double hinv[UR3E_MAXNV], f[UR3E_MAXNV];
    memcpy(H, d->qM, sizeof(H));
    for (int k = 0; k < nv; k++) H[k][k] += m->timestep * m->dof_damping[k];
    factor_tree(m, H, hinv);
    for (int k = 0; k < nv; k++) f[k] = d->qfrc_smooth[k] + d->qfrc_constraint[k];
    solve_tree(m, H, hinv, qacc_int, f);
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
      double ang = h * normalize3(w);
      double qr[4];
      axis_angle_quat(qr, w, ang);
      double* q = d->qpos + a + 3;
      normalize4(q);
      mul_quat(q, q, qr);
    } else {
      d->qpos[a] += h * d->qvel[v];
    }
  }
  d->time += h;
  for (int k = 0; k < nv; k++) d->qacc_warmstart[k] = d->qacc[k];
}

/* ===================================================================== */
/* task predicates (utils/gym_utils.py)                                   */
/* ===================================================================== */
int ur3o_block_grasp_state(const ur3e_model_t* m, const ur3o_data* d) {
  /* gym_utils.py:108-128: number of distinct pads touching the fish */
  int lp = 0, rp = 0;
  for (int ci = 0; ci < d->ncon; ci++) {
    int b1 = m->geom_bodyid[d->contact[ci].geom1], b2 = m->geom_bodyid[d->contact[ci].geom2];
    int fish = (b1 == m->id_body_fish || b2 == m->id_body_fish);
    if (!fish) continue;
    if (b1 == m->id_body_lpad || b2 == m->id_body_lpad) lp = 1;
    if (b1 == m->id_body_rpad || b2 == m->id_body_rpad) rp = 1;
  }
  return lp + rp;
}

int ur3o_self_collision(const ur3e_model_t* m, const ur3o_data* d) {
  /* gym_utils.py:146-172 */
  for (int ci = 0; ci < d->ncon; ci++) {
    int b1 = m->geom_bodyid[d->contact[ci].geom1], b2 = m->geom_bodyid[d->contact[ci].geom2];
    int a1 = (m->mask_arm_bodies >> b1) & 1, a2 = (m->mask_arm_bodies >> b2) & 1;
    if (a1 && a2) {
      int g1 = (m->mask_gripper_bodies >> b1) & 1, g2 = (m->mask_gripper_bodies >> b2) & 1;
      if (g1 && g2) continue;
      return 1;
    }
  }
  return 0;
}

/* ===================================================================== */
/* scipy Rotation semantics (controller_func.get_rot_err)                  */
/* ===================================================================== */
void ur3o_quat_from_matrix(const double mt[9], double q[4]) {
  double dec[4] = {mt[0], mt[4], mt[8], mt[0] + mt[4] + mt[8]};
  int ch = 0;
  for (int k = 1; k < 4; k++)
    if (dec[k] > dec[ch]) ch = k;
  if (ch != 3) {
    int i = ch, j = (i + 1) % 3, k = (j + 1) % 3;
    q[i] = 1 - dec[3] + 2 * mt[3 * i + i];
    q[j] = mt[3 * j + i] + mt[3 * i + j];
    q[k] = mt[3 * k + i] + mt[3 * i + k];
    q[3] = mt[3 * k + j] - mt[3 * j + k];
  } else {
    q[0] = mt[7] - mt[5];
    q[1] = mt[2] - mt[6];
    q[2] = mt[3] - mt[1];
    q[3] = 1 + dec[3];
  }
  double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  q[0] /= n; q[1] /= n; q[2] /= n; q[3] /= n;
}

void ur3o_quat_from_rotvec(const double rv[3], double q[4]) {
  double ang = sqrt(rv[0] * rv[0] + rv[1] * rv[1] + rv[2] * rv[2]);
  double sc;
  if (ang <= 1e-3) {
    double a2 = ang * ang;
    sc = 0.5 - a2 / 48 + a2 * a2 / 3840;
  } else {
    sc = ur3e_sin(ang / 2) / ang;
  }
  q[0] = sc * rv[0]; q[1] = sc * rv[1]; q[2] = sc * rv[2];
  q[3] = ur3e_cos(ang / 2);
}

void ur3o_rotvec_from_quat(const double qin[4], double rv[3]) {
  double q[4] = {qin[0], qin[1], qin[2], qin[3]};
  if (q[3] < 0) { q[0] = -q[0]; q[1] = -q[1]; q[2] = -q[2]; q[3] = -q[3]; }
  double ang = 2 * ur3e_atan2(sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2]), q[3]);
  double sc;
  if (ang <= 1e-3) {
    double a2 = ang * ang;
    sc = 2 + a2 / 12 + 7 * a2 * a2 / 2880;
  } else {
    sc = ang / ur3e_sin(ang / 2);
  }
  rv[0] = sc * q[0]; rv[1] = sc * q[1]; rv[2] = sc * q[2];
}

/* utils/utils.py:158-162 get_site_xrotvec: R.from_matrix(xmat).as_rotvec() (scipy 1.15.3) */
void ur3o_rotvec_from_matrix(const double xmat[9], double rv[3]) {
  double q[4];
  ur3o_quat_from_matrix(xmat, q);
  ur3o_rotvec_from_quat(q, rv);
}

void ur3o_rot_err(const double xmat[9], const double target[3], double err[3]) {
  /* controller_func.py:30-48: q_err = R(target) * R(xmat)^-1 -> rotvec */
  double q[4], qd[4], qi[4], r[4];
  ur3o_quat_from_matrix(xmat, q);
  ur3o_quat_from_rotvec(target, qd);
  qi[0] = -q[0]; qi[1] = -q[1]; qi[2] = -q[2]; qi[3] = q[3];
  double cr[3];
  cross3(cr, qd, qi);
  r[0] = qd[3] * qi[0] + qi[3] * qd[0] + cr[0];
  r[1] = qd[3] * qi[1] + qi[3] * qd[1] + cr[1];
  r[2] = qd[3] * qi[2] + qi[3] * qd[2] + cr[2];
  r[3] = qd[3] * qi[3] - qd[0] * qi[0] - qd[1] * qi[1] - qd[2] * qi[2];
  ur3o_rotvec_from_quat(r, err);
}

/* ===================================================================== */
/* controllers                                                            */
/* ===================================================================== */
void ur3o_pid_task_ctrl_raw(const double traj[7], const double tcp_xpos[3], const double tcp_xmat[9],
                            const double J[36], const double qv[6], const double bias[6],
                            const ur3o_task_gains* g, double grip_scale, double ctrl[7]) {
  /* controller_func.py:68-117 (ki = 0; the np.clip result is discarded) */
  double ep[3] = {traj[0] - tcp_xpos[0], traj[1] - tcp_xpos[1], traj[2] - tcp_xpos[2]};
  double er[3];
  ur3o_rot_err(tcp_xmat, traj + 3, er);
  double jv[6];
  for (int r = 0; r < 6; r++) {
    double s = 0;
    for (int k = 0; k < 6; k++) s += J[6 * r + k] * qv[k];
    jv[r] = s;
  }
  double u[6];
  for (int r = 0; r < 3; r++) u[r] = g->kp_pos[r] * ep[r] - g->kd_pos[r] * jv[r];
  for (int r = 0; r < 3; r++) u[3 + r] = g->kp_rot[r] * er[r] - g->kd_rot[r] * jv[3 + r];
  for (int c = 0; c < 6; c++) {
    double s = 0;
    for (int r = 0; r < 6; r++) s += J[6 * r + c] * u[r];
    ctrl[c] = s + bias[c];
  }
  ctrl[6] = traj[6] * grip_scale;
}

void ur3o_pid_task_ctrl(const ur3e_model_t* m, const ur3o_data* d, const double traj[7],
                        const ur3o_task_gains* g, double* ctrl) {
  int nv = m->nv, s = m->id_site_tcp;
  double jp[3 * UR3E_MAXNV], jr[3 * UR3E_MAXNV], J[36];
  ur3o_jac_site(m, d, s, jp, jr);
  for (int c = 0; c < 6; c++) {
    for (int r = 0; r < 3; r++) {
      J[6 * r + c] = jp[r * nv + c];
      J[6 * (3 + r) + c] = jr[r * nv + c];
    }
  }
  double out[7];
  ur3o_pid_task_ctrl_raw(traj, d->site_xpos[s], d->site_xmat[s], J, d->qvel, d->qfrc_bias, g,
                         m->act_ctrlrange[m->nu - 1][1], out);
  for (int k = 0; k < 6; k++) ctrl[k] = out[k];
  if (m->nu > 6) ctrl[6] = out[6];
}

void ur3o_pd_joint_ctrl_raw(const double q[6], const double v[6], const double delta[6], const double jr[12],
                            const double cr[12], const ur3o_joint_gains* g, double u[6]) {
  /* controller_func.py:128-167 */
  for (int k = 0; k < 6; k++) {
    double t = q[k] + delta[k];
    if (t < jr[2 * k]) t = jr[2 * k];
    if (t > jr[2 * k + 1]) t = jr[2 * k + 1];
    double e = t - q[k];
    double uk = g->kp[k] * e + g->kd[k] * (-v[k]);
    if (uk < cr[2 * k]) uk = cr[2 * k];
    if (uk > cr[2 * k + 1]) uk = cr[2 * k + 1];
    u[k] = uk;
  }
}

static void arm_ranges(const ur3e_model_t* m, double jr[12], double cr[12]) {
  for (int k = 0; k < 6; k++) {
    jr[2 * k] = m->jnt_range[k][0]; jr[2 * k + 1] = m->jnt_range[k][1];
    cr[2 * k] = m->act_ctrlrange[k][0]; cr[2 * k + 1] = m->act_ctrlrange[k][1];
  }
}

void ur3o_move_j_ctrl(const ur3e_model_t* m, const ur3o_data* d, const double traj[7],
                      const ur3o_joint_gains* g, double* ctrl) {
  /* controller/move_j.py:14-38 */
  double delta[6], jr[12], cr[12], u[6];
  for (int k = 0; k < 6; k++) delta[k] = traj[k] - d->qpos[k];
  arm_ranges(m, jr, cr);
  ur3o_pd_joint_ctrl_raw(d->qpos, d->qvel, delta, jr, cr, g, u);
  for (int k = 0; k < 6; k++) ctrl[k] = u[k];
  if (m->nu > 6) ctrl[6] = traj[6] * m->act_ctrlrange[m->nu - 1][1];
}

void ur3o_pinv3x6(const double J[18], double P[18]) {
  /* pinv of a full-row-rank 3x6 matrix: J' (J J')^-1 */
  double A[9];
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) {
      double s = 0;
      for (int k = 0; k < 6; k++) s += J[6 * r + k] * J[6 * c + k];
      A[3 * r + c] = s;
    }
  double c00 = A[4] * A[8] - A[5] * A[7], c01 = A[5] * A[6] - A[3] * A[8], c02 = A[3] * A[7] - A[4] * A[6];
  double det = A[0] * c00 + A[1] * c01 + A[2] * c02;
  double inv[9];
  inv[0] = c00 / det;
  inv[3] = c01 / det;
  inv[6] = c02 / det;
  inv[1] = (A[2] * A[7] - A[1] * A[8]) / det;
  inv[4] = (A[0] * A[8] - A[2] * A[6]) / det;
  inv[7] = (A[1] * A[6] - A[0] * A[7]) / det;
  inv[2] = (A[1] * A[5] - A[2] * A[4]) / det;
  inv[5] = (A[2] * A[3] - A[0] * A[5]) / det;
  inv[8] = (A[0] * A[4] - A[1] * A[3]) / det;
  for (int k = 0; k < 6; k++)
    for (int c = 0; c < 3; c++) {
      double s = 0;
      for (int r = 0; r < 3; r++) s += J[6 * r + k] * inv[3 * r + c];
      P[3 * k + c] = s;
    }
}

void ur3o_move_l_ctrl_raw(const double traj[7], const double tcp_xpos[3], const double tcp_xmat[9],
                          const double Jp[18], const double Jr[18], const double q[6], const double v[6],
                          const double jr[12], const double cr[12], const ur3o_joint_gains* gpos,
                          const ur3o_joint_gains* grot, double grip_scale, double ctrl[7]) {
  /* controller/move_l.py:15-78: get_pos_joint_delta (:35-55) = pinv(jacp_arm) e_p,
     get_rot_joint_delta (:58-78) = pinv(jacr_arm) e_r, each through pd_joint_ctrl
     (controller_func.py:128-167) with its own gains, summed (:24-31); grip_ctrl on traj[6] */
  double Pp[18], Pr[18];
  ur3o_pinv3x6(Jp, Pp);
  ur3o_pinv3x6(Jr, Pr);
  double ep[3] = {traj[0] - tcp_xpos[0], traj[1] - tcp_xpos[1], traj[2] - tcp_xpos[2]};
  double er[3];
  ur3o_rot_err(tcp_xmat, traj + 3, er);
  double dp[6], dr[6], up[6], ur[6];
  for (int k = 0; k < 6; k++) {
    dp[k] = Pp[3 * k] * ep[0] + Pp[3 * k + 1] * ep[1] + Pp[3 * k + 2] * ep[2];
    dr[k] = Pr[3 * k] * er[0] + Pr[3 * k + 1] * er[1] + Pr[3 * k + 2] * er[2];
  }
  ur3o_pd_joint_ctrl_raw(q, v, dp, jr, cr, gpos, up);
  ur3o_pd_joint_ctrl_raw(q, v, dr, jr, cr, grot, ur);
  for (int k = 0; k < 6; k++) ctrl[k] = up[k] + ur[k];
  ctrl[6] = traj[6] * grip_scale;
}

void ur3o_move_l_ctrl(const ur3e_model_t* m, const ur3o_data* d, const double traj[7],
                      const ur3o_joint_gains* gpos, const ur3o_joint_gains* grot, double* ctrl) {
  /* mj_jacSite on the stale kinematics MjData holds after mj_step (move_l.py:47,70), fresh q / qdot */
  int nv = m->nv, s = m->id_site_tcp;
  double jp[3 * UR3E_MAXNV], jrr[3 * UR3E_MAXNV], Jp[18], Jr[18];
  ur3o_jac_site(m, d, s, jp, jrr);
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 6; c++) { Jp[6 * r + c] = jp[r * nv + c]; Jr[6 * r + c] = jrr[r * nv + c]; }
  double jr[12], cr[12], out[7];
  arm_ranges(m, jr, cr);
  ur3o_move_l_ctrl_raw(traj, d->site_xpos[s], d->site_xmat[s], Jp, Jr, d->qpos, d->qvel, jr, cr, gpos, grot,
                       m->act_ctrlrange[m->nu - 1][1], out);
  for (int k = 0; k < 6; k++) ctrl[k] = out[k];
  if (m->nu > 6) ctrl[6] = out[6];
}

/* ===================================================================== */
/* UR3eEnv2 epilogue                                                       */
/* ===================================================================== */
void ur3o_obs_v2(const ur3e_model_t* m, const ur3o_data* d, double obs[24]) {
  int st = m->id_site_tcp, sh = m->id_site_handle, gb = m->id_body_ghost;
  const double* tcp = d->site_xpos[st];
  const double* mug = d->site_xpos[sh];
  const double* gh = d->xpos[gb];
  double vt[6], vh[6];
  ur3o_site_velocity(m, d, st, vt);
  ur3o_site_velocity(m, d, sh, vh);
  for (int k = 0; k < 3; k++) {
    obs[k] = tcp[k];
    obs[3 + k] = mug[k];
    obs[6 + k] = gh[k];
    obs[9 + k] = tcp[k] - mug[k];
    obs[12 + k] = mug[k] - gh[k];
    obs[15 + k] = vt[3 + k];
    obs[18 + k] = vt[3 + k] - vh[3 + k];
  }
  obs[21] = d->qpos[6];
  obs[22] = d->qvel[6];
  /* get_robust_block_grasp_state (gym_utils.py:98-106) */
  int gs = ur3o_block_grasp_state(m, d);
  int robust = 0;
  if (gs == 2) {
    double dx = fabs(tcp[0] - mug[0]), dy = fabs(tcp[1] - mug[1]), dz = fabs(tcp[2] - mug[2]);
    robust = (dx < 0.01 && dy < 0.005 && dz < 0.05);
  }
  obs[23] = (double)robust;
}

double ur3o_reward_v2(const double obs[24], const double act[4]) {
  /* ur3e_env2.py:150-228 */
  double mug_z = obs[5];
  const double* g2m = obs + 9;
  const double* m2t = obs + 12;
  const double* gv = obs + 15;
  double grasped = obs[23];
  double grip = act[3];
  double xy = sqrt(g2m[0] * g2m[0] + g2m[1] * g2m[1]);
  double zerr = fabs(g2m[2] - 0.02);
  double place = sqrt(m2t[0] * m2t[0] + m2t[1] * m2t[1] + m2t[2] * m2t[2]);
  double ready = ur3e_exp(-10 * xy) * ur3e_exp(-20 * zerr);
  double align = 2.0 * ready;
  double grasp_act = 2.0 * grip * ready;
  double grasp_ach = 10.0 * grasped * ready;
  double lift = 8.0 * grasped * ur3e_tanh(8.0 * (mug_z > 0 ? mug_z : 0));
  double placement = grasped * (4.0 * ur3e_exp(-15 * place) - 1.5 * place);
  double success = 0.0;
  if (grasped != 0 && place < 0.05) success = 50.0;
  double pen = 0.0;
  pen += -1.0 * (-g2m[2] > 0 ? -g2m[2] : 0);
  pen += -0.01 * sqrt(gv[0] * gv[0] + gv[1] * gv[1] + gv[2] * gv[2]);
  return align + grasp_act + grasp_ach + lift + placement + success + pen;
}

int ur3o_termination_v2(const ur3e_model_t* m, const ur3o_data* d, const double obs[24]) {
  /* ur3e_env2.py:230-254 */
  double dx = obs[0] - obs[3], dy = obs[1] - obs[4], dz = obs[2] - obs[5];
  if (1.0 < sqrt(dx * dx + dy * dy + dz * dz)) return 1;
  if (ur3o_self_collision(m, d)) return 1;
  if (obs[5] <= m->fish_topple_z) return 1; /* get_mug_toppled, gym_utils.py:8-17 */
  return 0;
}

/* ===================================================================== */
/* UR3eEnv (ur3e-v0) and imitation-env epilogues                           */
/* ===================================================================== */
int ur3o_table_collision(const ur3e_model_t* m, const ur3o_data* d) {
  /* gym_utils.py:174-197: any gripper-tree body touching the table body */
  for (int ci = 0; ci < d->ncon; ci++) {
    int b1 = m->geom_bodyid[d->contact[ci].geom1], b2 = m->geom_bodyid[d->contact[ci].geom2];
    int g1 = (m->mask_gripper_bodies >> b1) & 1, g2 = (m->mask_gripper_bodies >> b2) & 1;
    if ((g1 && b2 == m->id_body_table) || (g2 && b1 == m->id_body_table)) return 1;
  }
  return 0;
}

void ur3o_obs_v0(const ur3e_model_t* m, const ur3o_data* d, double obs[13]) {
  /* ur3e_env.py _get_obs: tcp, handle_site, ghost, block grasp state, right_pad1_site */
  const double* tcp = d->site_xpos[m->id_site_tcp];
  const double* mug = d->site_xpos[m->id_site_handle];
  const double* gh = d->xpos[m->id_body_ghost];
  const double* pad = d->site_xpos[m->id_site_rpad];
  for (int k = 0; k < 3; k++) { obs[k] = tcp[k]; obs[3 + k] = mug[k]; obs[6 + k] = gh[k]; obs[10 + k] = pad[k]; }
  obs[9] = (double)ur3o_block_grasp_state(m, d);
}

void ur3o_obs_direct(const ur3e_model_t* m, const ur3o_data* d, double obs[13]) {
  /* imitation_env_direct.py _get_obs: tcp, handle_site, ghost, block grasp state, tcp linear velocity */
  const double* tcp = d->site_xpos[m->id_site_tcp];
  const double* mug = d->site_xpos[m->id_site_handle];
  const double* gh = d->xpos[m->id_body_ghost];
  double vt[6];
  ur3o_site_velocity(m, d, m->id_site_tcp, vt);
  for (int k = 0; k < 3; k++) { obs[k] = tcp[k]; obs[3 + k] = mug[k]; obs[6 + k] = gh[k]; obs[10 + k] = vt[3 + k]; }
  obs[9] = (double)ur3o_block_grasp_state(m, d);
}

static double sq(double x) { return x * x; }

double ur3o_reward_v0(const ur3e_model_t* m, const ur3o_data* d, const double obs[13], const double act[4]) {
  /* ur3e_env.py:compute_reward (the per-20-step print is dropped) */
  const double* gripper_pos = obs;
  const double* block_center = obs + 3;
  const double* target_pos = obs + 6;
  double grasp_state = obs[9];
  const double* pad_pos = obs + 10;
  double block_half_height = m->fish_half_z;
  double block_top_z = block_center[2] + block_half_height;
  double block_bottom_z = block_center[2] - block_half_height;
  double pad_to_block_top = pad_pos[2] - block_top_z;
  double gripper_to_block_center = gripper_pos[2] - block_center[2];
  double hx = gripper_pos[0] - block_center[0], hy = gripper_pos[1] - block_center[1];
  double horizontal_error = sqrt(hx * hx + hy * hy);
  int valid_grasp = grasp_state == 2 && fabs(pad_to_block_top) < 0.04 && horizontal_error < 0.03;
  double ideal_height_above = 0.5;
  double height_error = gripper_to_block_center - ideal_height_above;
  double z_tol = 0.1;
  double descent_reward = 1 * ((1 / z_tol) * (height_error + z_tol) * ur3e_exp(-(1 / z_tol) * height_error));
  double grasp_readiness = ur3e_exp(-sq(horizontal_error)) * ur3e_exp(-sq(pad_to_block_top)) *
                           ur3e_exp(-sq(height_error)) * 100 * ur3e_exp(-sq(act[3]));
  double alignment_reward = 4 * ur3e_exp(-60 * sq(horizontal_error));
  double grip_strength = act[3];
  double g2 = grasp_state == 2 ? 1.0 : 0.0, g1 = grasp_state >= 1 ? 1.0 : 0.0;
  double grasp_reward = 5.5 * g1 + 8.5 * g2 + 23.5 * grip_strength * grasp_readiness + 28.5 * g2 * grasp_readiness +
                        11.5 * g2 * grasp_readiness * ur3e_tanh(8 * grip_strength);
  double lift_reward = 12 * g2 * ur3e_tanh(4 * block_bottom_z);
  double px = block_center[0] - target_pos[0], py = block_center[1] - target_pos[1],
         pz = block_center[2] - target_pos[2];
  double d_place = sqrt(px * px + py * py + pz * pz);
  double placement_reward = -2 * d_place + 20 * ur3e_exp(-70 * sq(d_place));
  if (d_place < 0.05 && valid_grasp) placement_reward += 40;
  double hh = block_center[2] - gripper_pos[2] + 0.5;
  double dh = -100000000000.0 * (hh * hh * hh);
  double dangerous_height_penalty = dh < 0 ? dh : 0;
  double p2b = pad_to_block_top > 0 ? pad_to_block_top : 0;
  double penalties = -40 * ur3o_self_collision(m, d) + -25 * ur3o_table_collision(m, d) +
                     -8 * (block_center[2] <= m->fish_topple_z) + -4 * p2b + dangerous_height_penalty;
  double action_reward = 700.5 * grip_strength * grasp_readiness;
  double contact_achievement_bonus = 1700.5 * g2 * grasp_readiness * ur3e_tanh(10 * grip_strength);
  return descent_reward + alignment_reward + grasp_reward + lift_reward + placement_reward + action_reward +
         contact_achievement_bonus + penalties;
}

int ur3o_termination_v0(const ur3e_model_t* m, const ur3o_data* d, const double obs[13]) {
  /* ur3e_env.py:_check_termination */
  double dx = obs[0] - obs[3], dy = obs[1] - obs[4], dz = obs[2] - obs[5];
  double ex = obs[3] - obs[6], ey = obs[4] - obs[7], ez = obs[5] - obs[8];
  double d_pick = sqrt(dx * dx + dy * dy + dz * dz);
  double d_place = sqrt(ex * ex + ey * ey + ez * ez);
  if (d_place < 0.005) return 1;
  if (1 < d_pick) return 1;
  if (ur3o_self_collision(m, d)) return 1;
  if (obs[5] <= m->fish_topple_z) return 1;
  return 0;
}

/* ===================================================================== */
/* Philox4x32-10                                                           */
/* ===================================================================== */
void ur3o_philox4x32(const unsigned int ctr[4], const unsigned int key[2], unsigned int out[4]) {
  unsigned int c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
  unsigned int k0 = key[0], k1 = key[1];
  for (int r = 0; r < 10; r++) {
    unsigned long long p0 = (unsigned long long)0xD2511F53u * c0;
    unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c2;
    unsigned int hi0 = (unsigned int)(p0 >> 32), lo0 = (unsigned int)p0;
    unsigned int hi1 = (unsigned int)(p1 >> 32), lo1 = (unsigned int)p1;
    unsigned int n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

double ur3o_uniform01(unsigned long long seed, unsigned int env_id, unsigned int episode, unsigned int k) {
  unsigned int ctr[4] = {env_id, episode, k, 0x55523345u};
  unsigned int key[2] = {(unsigned int)seed, (unsigned int)(seed >> 32)};
  unsigned int o[4];
  ur3o_philox4x32(ctr, key, o);
  unsigned long long bits = ((unsigned long long)o[0] << 32) | o[1];
  return (double)(bits >> 11) * (1.0 / 9007199254740992.0);
}

/* ===================================================================== */
/* env API                                                                */
/* ===================================================================== */
void ur3o_env_init(const ur3e_model_t* m, ur3o_env* e, unsigned long long seed, unsigned int env_id) {
  memset(e, 0, sizeof(*e));
  e->seed = seed;
  e->env_id = env_id;
  ur3o_reset_data(m, &e->d);
}

void ur3o_env_reset(const ur3e_model_t* m, ur3o_env* e, double obs[24]) {
  /* MujocoEnv.reset -> mj_resetData -> UR3eEnv2.reset_model (ur3e_env2.py:101-109) */
  ur3o_data* d = &e->d;
  ur3o_reset_data(m, d);
  int key = m->id_key_down;
  for (int k = 0; k < m->nq; k++) d->qpos[k] = m->key_qpos[key][k];
  for (int k = 0; k < m->nv; k++) d->qvel[k] = m->key_qvel[key][k];
  /* get_mug_xpos_noise("high"), gym_utils.py:48-60: x += U[0,0.02], y += U[-0.25,0.2] */
  double u0 = ur3o_uniform01(e->seed, e->env_id, e->episode, 0);
  double u1 = ur3o_uniform01(e->seed, e->env_id, e->episode, 1);
  d->qpos[14] += 0.0 + (0.02 - 0.0) * u0;
  d->qpos[15] += -0.25 + (0.2 - -0.25) * u1;
  ur3o_forward(m, d);
  e->t = 0;
  e->ep_return = 0;
  e->ep_len = 0;
  e->episode++;
  ur3o_obs_v2(m, d, obs);
}

void ur3o_env_step_v2(const ur3e_model_t* m, ur3o_env* e, const ur3o_task_gains* g, const double a[4],
                      int frame_skip, double obs[24], double* reward, int* terminated, int* truncated) {
  /* ur3e_env2.py:72-99 */
  ur3o_data* d = &e->d;
  double traj[7] = {a[0], a[1], a[2], -1.209, -1.209, 1.209, a[3]};
  double ctrl[UR3E_MAXU];
  ur3o_pid_task_ctrl(m, d, traj, g, ctrl);
  for (int k = 0; k < m->nu; k++) d->ctrl[k] = ctrl[k];
  for (int s = 0; s < frame_skip; s++) ur3o_step(m, d);
  ur3o_obs_v2(m, d, obs);
  double r = ur3o_reward_v2(obs, a);
  e->t += 1;
  int term = ur3o_termination_v2(m, d, obs);
  int trunc = e->t >= 2500;
  double dx = obs[3] - obs[6], dy = obs[4] - obs[7], dz = obs[5] - obs[8];
  if (sqrt(dx * dx + dy * dy + dz * dz) < 0.05) {
    term = 1;
    r += 50.0;
  }
  e->ep_return += r;
  e->ep_len += 1;
  *reward = r;
  *terminated = term;
  *truncated = trunc;
}

int ur3o_sizeof_data(void) { return (int)sizeof(ur3o_data); }
int ur3o_sizeof_env(void) { return (int)sizeof(ur3o_env); }
