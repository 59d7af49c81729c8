/*
 * ur3e_batch.hip — MI355X (gfx950) batched UR3e environment: kernels + C ABI.
 *
 * One fused kernel per env-step (k_env_step): controller -> frame_skip physics
 * substeps -> observation / reward / termination -> in-kernel SB3 auto-reset.
 * One environment per wavefront lane; `envs_per_block` lanes of each 64-wide
 * wavefront are populated, trading lane packing for CU coverage (at 4096 envs
 * 16 envs/wave puts one wave on every one of the 256 CUs).
 *
 * Persistent per-env state lives in HBM structure-of-arrays ([field][env]) so
 * a wave's 64 lanes touch consecutive doubles: qpos[nq], qvel[nv],
 * qacc_warmstart[nv], the stale-kinematics carry[54] (tcp pose, arm Jacobian,
 * qfrc_bias[0:6] of the last forward pass — MuJoCo's post-mj_step mjData
 * semantics that the reference controller and observation read), and episode
 * counters.  User-facing tensors (actions, obs, get/set_state) are row-major.
 *
 * Reference behaviour restated (file:line in /root/reference):
 *   UR3eEnv2.step / reset_model / _get_obs / compute_reward / _check_termination
 *     gymnasium_env/envs/ur3e_env2.py:72-261
 *   pid_task_ctrl / pd_joint_ctrl     controller/controller_func.py:68-167
 *   move_j                            controller/move_j.py:14-38
 *   predicates                        utils/gym_utils.py:8-172
 *   mj_step (MuJoCo 3.3.3)            ur3e_engine.h
 */
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <chrono>

#include "../../include/ur3e_batch.h"
#include "ur3e_engine.h"
#include "ur3e_wave.h"


/* ================================================================== */
/* scipy Rotation semantics (controller_func.get_rot_err)              */
/* ================================================================== */
KD void k_quat_from_matrix(const double mt[9], double q[4]) {
  double dec[4] = {mt[0], mt[4], mt[8], mt[0] + mt[4] + mt[8]};
  int ch = 0;
  double dch = dec[0];
#pragma unroll
  for (int k = 1; k < 4; k++)
    if (dec[k] > dch) { ch = k; dch = dec[k]; }
  /* i = ch, j = (i + 1) % 3, k = (j + 1) % 3 spelt out per case (constant indices: no private
     array indexed at run time) */
  if (ch == 0) {
    q[0] = 1 - dec[3] + 2 * mt[0];
    q[1] = mt[3] + mt[1];
    q[2] = mt[6] + mt[2];
    q[3] = mt[7] - mt[5];
  } else if (ch == 1) {
    q[1] = 1 - dec[3] + 2 * mt[4];
    q[2] = mt[7] + mt[5];
    q[0] = mt[1] + mt[3];
    q[3] = mt[2] - mt[6];
  } else if (ch == 2) {
    q[2] = 1 - dec[3] + 2 * mt[8];
    q[0] = mt[2] + mt[6];
    q[1] = mt[5] + mt[7];
    q[3] = mt[3] - mt[1];
  } else {
    q[0] = mt[7] - mt[5];
    q[1] = mt[2] - mt[6];
    q[2] = mt[3] - mt[1];
    q[3] = 1 + dec[3];
  }
  double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  q[0] /= n; q[1] /= n; q[2] /= n; q[3] /= n;
}

__host__ __device__ static inline void k_quat_from_rotvec(const double rv[3], double q[4]) {
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

KD void k_rotvec_from_quat(const double qin[4], double rv[3]) {
  /* the sign flip as selects: a conditionally rewritten array would live in scratch */
  const bool neg = qin[3] < 0;
  double q[4] = {neg ? -qin[0] : qin[0], neg ? -qin[1] : qin[1], neg ? -qin[2] : qin[2], neg ? -qin[3] : qin[3]};
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

/* the rotation error against a target given as its quaternion qd (k_quat_from_rotvec of the target) */
KD void k_rot_err_q(const double xmat[9], const double qd[4], double err[3]) {
  double q[4], qi[4], r[4];
  k_quat_from_matrix(xmat, q);
  qi[0] = -q[0]; qi[1] = -q[1]; qi[2] = -q[2]; qi[3] = q[3];
  double cr[3];
  k_cross3(cr, qd, qi);
  r[0] = qd[3] * qi[0] + qi[3] * qd[0] + cr[0];
  r[1] = qd[3] * qi[1] + qi[3] * qd[1] + cr[1];
  r[2] = qd[3] * qi[2] + qi[3] * qd[2] + cr[2];
  r[3] = qd[3] * qi[3] - qd[0] * qi[0] - qd[1] * qi[1] - qd[2] * qi[2];
  k_rotvec_from_quat(r, err);
}

KD void k_rot_err(const double xmat[9], const double target[3], double err[3]) {
  double qd[4];
  k_quat_from_rotvec(target, qd);
  k_rot_err_q(xmat, qd, err);
}

/* ================================================================== */
/* controllers                                                         */
/* ================================================================== */
struct KGains {
  double task[12];
  double joint[12];
  double rot[12]; /* move_l rotation PD (config_l.yml "rot"); joint[] holds its "pos" gains */
};

/* pid_task_ctrl (controller_func.py:68-117): carry = [tcp_xpos 3, tcp_xmat 9, J 36, bias 6] */
KD void k_pid_task_ctrl(const double traj[7], const double* carry, const double qv[6], const KGains& g,
                        double grip_scale, double ctrl[7]) {
  const double* tcp_xpos = carry;
  const double* tcp_xmat = carry + 3;
  const double* J = carry + 12;
  const double* bias = carry + 48;
  double ep[3] = {traj[0] - tcp_xpos[0], traj[1] - tcp_xpos[1], traj[2] - tcp_xpos[2]};
  double er[3];
  k_rot_err(tcp_xmat, traj + 3, er);
  double jv[6];
  for (int r = 0; r < 6; r++) {
    double s = 0;
    for (int k = 0; k < 6; k++) s += J[6 * r + k] * qv[k];
    jv[r] = s;
  }
  double u[6];
  for (int r = 0; r < 3; r++) u[r] = g.task[r] * ep[r] - g.task[3 + r] * jv[r];
  for (int r = 0; r < 3; r++) u[3 + r] = g.task[6 + r] * er[r] - g.task[9 + r] * jv[3 + r];
  for (int c = 0; c < 6; c++) {
    double s = 0;
    for (int r = 0; r < 6; r++) s += J[6 * r + c] * u[r];
    ctrl[c] = s + bias[c];
  }
  ctrl[6] = traj[6] * grip_scale;
}

/* pinv of a full-row-rank 3x6 arm Jacobian block, J' (J J')^-1 with the 3x3 inverse by cofactors;
   np.linalg.pinv (SVD) in move_l.py:49,72 -- same operation order as oracle ur3o_pinv3x6 */
KD void k_pinv3x6(const double* J, double P[18]) {
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

/* pd_joint_ctrl (controller_func.py:128-167): target = clip(q + delta, jnt_range), u = kp e - kd qdot,
   clipped to the actuator ctrlrange */
KD void k_pd_joint(KModel m, const double* q, const double* v, const double delta[6], const double* g,
                   double u[6]) {
  for (int k = 0; k < 6; k++) {
    double t = q[k] + delta[k];
    if (t < m->jnt_range[k][0]) t = m->jnt_range[k][0];
    if (t > m->jnt_range[k][1]) t = m->jnt_range[k][1];
    double e = t - q[k];
    double uk = g[k] * e + g[6 + k] * (-v[k]);
    if (uk < m->act_ctrlrange[k][0]) uk = m->act_ctrlrange[k][0];
    if (uk > m->act_ctrlrange[k][1]) uk = m->act_ctrlrange[k][1];
    u[k] = uk;
  }
}

/* move_l.ctrl (controller/move_l.py:15-78): delta_p = pinv(Jp_arm) e_p (get_pos_joint_delta),
   delta_r = pinv(Jr_arm) e_r (get_rot_joint_delta), each through pd_joint_ctrl with its own gains,
   summed; grip_ctrl on traj[6].  Jacobian, tcp pose: the stale-kinematics carry, as mj_jacSite reads
   them after mj_step; q, qdot fresh */
KD void k_move_l_ctrl(KModel m, const double traj[7], const double* carry, const double* q, const double* v,
                      const KGains& g, double* ctrl) {
  const double* tcp_xpos = carry;
  const double* tcp_xmat = carry + 3;
  const double* J = carry + 12; /* [jacp; jacr] 6x6 row-major */
  double Pp[18], Pr[18];
  k_pinv3x6(J, Pp);
  k_pinv3x6(J + 18, Pr);
  double ep[3] = {traj[0] - tcp_xpos[0], traj[1] - tcp_xpos[1], traj[2] - tcp_xpos[2]};
  double er[3];
  k_rot_err(tcp_xmat, traj + 3, er);
  double dp[6], dr[6], up[6], ur[6];
  for (int k = 0; k < 6; k++) {
    dp[k] = Pp[3 * k] * ep[0] + Pp[3 * k + 1] * ep[1] + Pp[3 * k + 2] * ep[2];
    dr[k] = Pr[3 * k] * er[0] + Pr[3 * k + 1] * er[1] + Pr[3 * k + 2] * er[2];
  }
  k_pd_joint(m, q, v, dp, g.joint, up);
  k_pd_joint(m, q, v, dr, g.rot, ur);
  for (int k = 0; k < 6; k++) ctrl[k] = up[k] + ur[k];
  if (m->nu > 6) ctrl[6] = traj[6] * m->act_ctrlrange[m->nu - 1][1];
}

/* move_j = pd_joint_ctrl on delta = target - q (move_j.py:14-38, controller_func.py:128-167) */
KD void k_move_j_ctrl(KModel m, const KData* d, const double traj[7], const KGains& g, double* ctrl) {
  for (int k = 0; k < 6; k++) {
    double q = d->qpos[k];
    double delta = traj[k] - q;
    double t = q + delta;
    if (t < m->jnt_range[k][0]) t = m->jnt_range[k][0];
    if (t > m->jnt_range[k][1]) t = m->jnt_range[k][1];
    double e = t - q;
    double uk = g.joint[k] * e + g.joint[6 + k] * (-d->qvel[k]);
    if (uk < m->act_ctrlrange[k][0]) uk = m->act_ctrlrange[k][0];
    if (uk > m->act_ctrlrange[k][1]) uk = m->act_ctrlrange[k][1];
    ctrl[k] = uk;
  }
  if (m->nu > 6) ctrl[6] = traj[6] * m->act_ctrlrange[m->nu - 1][1];
}

/* ================================================================== */
/* stale-kinematics carry + UR3eEnv2 epilogue                          */
/* ================================================================== */
KD void k_make_carry(KModel m, const KData* d, double* carry) {
  int s = m->id_site_tcp;
  if (s < 0) {
    for (int k = 0; k < NCARRY; k++) carry[k] = 0;
    return;
  }
  for (int k = 0; k < 3; k++) carry[k] = d->site_xpos[s][k];
  for (int k = 0; k < 9; k++) carry[3 + k] = d->site_xmat[s][k];
  double jp[3][K_NV], jr[3][K_NV];
  k_jac_point(m, d, m->site_bodyid[s], d->site_xpos[s], jp, jr);
  for (int c = 0; c < 6; c++) {
    for (int r = 0; r < 3; r++) {
      carry[12 + 6 * r + c] = jp[r][c];
      carry[12 + 6 * (3 + r) + c] = jr[r][c];
    }
  }
  for (int k = 0; k < 6; k++) carry[48 + k] = d->qfrc_bias[k];
}

KD int k_block_grasp_state(KModel m, const KData* d) {
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

KD int k_self_collision(KModel m, const KData* d) {
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

KD void k_obs_v2(KModel m, const KData* d, double obs[24]) {
  int st = m->id_site_tcp, sh = m->id_site_handle, gb = m->id_body_ghost;
  const double* tcp = d->site_xpos[st];
  const double* mug = d->site_xpos[sh];
  const double* gh = d->xpos[gb];
  double vt[6], vh[6];
  k_site_velocity(m, d, st, vt);
  k_site_velocity(m, d, sh, vh);
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
  int gs = k_block_grasp_state(m, d);
  int robust = 0;
  if (gs == 2) {
    double dx = fabs(tcp[0] - mug[0]), dy = fabs(tcp[1] - mug[1]), dz = fabs(tcp[2] - mug[2]);
    robust = (dx < 0.01 && dy < 0.005 && dz < 0.05);
  }
  obs[23] = (double)robust;
}

KD double k_reward_v2(const double obs[24], const double act[4]) {
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

KD int k_termination_v2(KModel m, const KData* d, const double obs[24]) {
  double dx = obs[0] - obs[3], dy = obs[1] - obs[4], dz = obs[2] - obs[5];
  if (1.0 < sqrt(dx * dx + dy * dy + dz * dz)) return 1;
  if (k_self_collision(m, d)) return 1;
  if (obs[5] <= m->fish_topple_z) return 1;
  return 0;
}

/* ================================================================== */
/* Philox4x32-10 (counter = env id, episode, draw, tag; key = seed)    */
/* ================================================================== */
KD double k_uniform01(unsigned long long seed, unsigned int env_id, unsigned int episode, unsigned int k) {
  unsigned int c0 = env_id, c1 = episode, c2 = k, c3 = 0x55523345u;
  unsigned int k0 = (unsigned int)seed, k1 = (unsigned int)(seed >> 32);
  for (int r = 0; r < 10; r++) {
    unsigned long long p0 = (unsigned long long)0xD2511F53u * c0;
    unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c2;
    unsigned int hi0 = (unsigned int)(p0 >> 32), lo0 = (unsigned int)p0;
    unsigned int hi1 = (unsigned int)(p1 >> 32), lo1 = (unsigned int)p1;
    unsigned int n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  unsigned long long bits = ((unsigned long long)c0 << 32) | c1;
  return (double)(bits >> 11) * (1.0 / 9007199254740992.0);
}

/* ================================================================== */
/* device state                                                        */
/* ================================================================== */
struct KState {
  int n;
  /* element (field k, env e) at k*fs + e*es: lane-per-env mode uses [field][env] (fs = n, es = 1),
     workgroup-per-env mode uses [env][field] (fs = 1, es = width) so a workgroup's loads coalesce */
  int fs;
  int es_q, es_v, es_c;
  double* qpos;   /* nq fields */
  double* qvel;   /* nv fields */
  double* warm;   /* nv fields */
  double* carry;  /* NCARRY fields */
  int* t;
  unsigned int* episode;
  int* ep_len;
  double* ep_return;
  int* ncon;
  int* nwarn;
  double* touch; /* [env][UR3E_MAXTOUCH] touch sensors after the last forward */
  double* ctrl;  /* [env][UR3E_MAXU] d.ctrl after the last step (the controller output it applied) */
  double* sensordata; /* [env][UR3E_MAXSENSORDATA] mjData.sensordata of the last forward (sensors on) */
  double* actfrc; /* [env][UR3E_MAXU] mjData.actuator_force of the last forward (workgroup-per-env kernels) */
  /* tier routing (grasp tier on): hint[e] = the env's last committed forward had more than
     KConfig.route_ncon contacts (or route_nefc rows); route[e] = the snapshot of hint the current step routes by (written only
     between steps, by the last kernel of the step): routed envs skip the compact tier and run in the
     grasp tier concurrently with it.  Routing only picks the tier; every tier gives the same result. */
  unsigned char* hint;
  unsigned char* route;
  /* host-mapped word: the number of envs the last route snapshot routed (written by the snapshotting
     workgroup, read by the host without a sync to decide whether the next steps need the pre-pass) */
  int* routed_host;
};
/* an env whose last forward had more contacts or constraint rows than KConfig.route_ncon / route_nefc
   runs its next step in the grasp tier; the margin below the compact tier's capacity covers what one step
   can add: a contact or three joint-limit rows for the gym tier (KSS_NV), two contacts or eight rows for
   the scripted pick's wider tier (KSS_NV_W) */
/* host-side routing decision (ur3e_batch_step): run-ahead bound and how long routing stays on after
   the host last saw a routed env */
#define W_AHEAD 16
/* the run-ahead event is recorded every W_AHEAD_EVERY steps (a marker on the stream costs ~2-5 us of GPU
   time per record, profiles/r05_l): step k (k a multiple of it) waits for the marker of step k - W_AHEAD */
#ifndef W_AHEAD_EVERY
#define W_AHEAD_EVERY 8
#endif
static_assert(W_AHEAD % W_AHEAD_EVERY == 0, "run-ahead bound: a whole number of marker intervals");
#define W_AHEAD_NEV (W_AHEAD / W_AHEAD_EVERY + 1) /* marker ring: the waited slot is never the one re-recorded */
#define W_NTOTAL 6 /* device counters of ur3e_batch::d_ovf_total */
/* the compact tier's bails straight to the full-capacity tier while routing is on too (1) or to the grasp
   tier behind it (0, default): one serial launch fewer per routed step, but the scripted pick's compact bails
   then run at one env per 128-lane workgroup -- C3 box -1.5 %, the rest neutral (profiles/r06_ab A/B 6) */
#ifndef W_DIRECT_PRE
#define W_DIRECT_PRE 0
#endif
/* the mid tier (KSM_NV / KSM_NV_M) between the compact and the grasp tier (1, default) or none (0: A/B) */
#ifndef W_MID_TIER
#define W_MID_TIER 1
#endif
#define W_ROUTE_HOLD 64

struct KConfig {
  int task, frame_skip, max_episode_steps, auto_reset, reset_noise, reset_key;
  unsigned long long seed;
  int env_id_offset;
  int epb;
  int tier_con_cap;
  int np_lanes; /* survivor lanes per compact narrowphase chunk (1..W_NP_LANES) */
  int obs_sites; /* model has tcp / handle_site / ghost: the scripted tasks also emit the 24-d obs */
  int sensors;   /* compute and store mjData.sensordata every forward (full-capacity kernels) */
  unsigned int spin_limit; /* substep queue: flag polls before a waiting unit gives up (diagnostic knob) */
  int leave_static;        /* substep queue diagnostic: owners skip their static units (consumers claim them) */
  double gym_qd[4];        /* the gym tasks' fixed tcp rotation target (rotvec [-1.209, -1.209, 1.209]) as a
                              quaternion, k_quat_from_rotvec on the host (detmath: the same bits) */
  int split_from;          /* substep queue: envs of a queue from this index on run their last substep as two
                              half units (w_env_step_q); >= the envs per queue: no split */
  /* routing: an env whose committed forward had more contacts or rows than these runs its next step in
     the grasp tier (set at create from the handle's compact-tier capacity) */
  int route_ncon, route_nefc;
  /* an env routed past the compact tier whose committed forward had no more contacts / rows than these runs
     in the mid tier, else in the grasp tier (route2_ncon < 0: no mid tier) */
  int route2_ncon, route2_nefc;
  KGains gains;
};

/* gym_utils.get_mug_xpos_noise (gym_utils.py:48-60): x ~ U[0, 0.02] for every magnitude, y bounds by
   magnitude (reset_noise 1 = "high", 2 = "med", 3 = "low") */
KD void k_noise_ybounds(int mag, double* lo, double* hi) {
  if (mag == 2) { *lo = -0.2; *hi = 0.1; }
  else if (mag == 3) { *lo = -0.1; *hi = 0.01; }
  else { *lo = -0.25; *hi = 0.2; }
}

KD size_t SQ(const KState& s, int k, int e) { return (size_t)k * s.fs + (size_t)e * s.es_q; }
KD size_t SV(const KState& s, int k, int e) { return (size_t)k * s.fs + (size_t)e * s.es_v; }
KD size_t SC(const KState& s, int k, int e) { return (size_t)k * s.fs + (size_t)e * s.es_c; }

KD void k_load(KModel m, const KState& s, int e, KData* d) {
  for (int k = 0; k < m->nq; k++) d->qpos[k] = s.qpos[SQ(s, k, e)];
  for (int k = 0; k < m->nv; k++) d->qvel[k] = s.qvel[SV(s, k, e)];
  for (int k = 0; k < m->nv; k++) d->qacc_warmstart[k] = s.warm[SV(s, k, e)];
  d->nwarn = s.nwarn[e];
}

KD void k_store(KModel m, const KState& s, int e, const KData* d, const double* carry) {
  for (int k = 0; k < m->nq; k++) s.qpos[SQ(s, k, e)] = d->qpos[k];
  for (int k = 0; k < m->nv; k++) s.qvel[SV(s, k, e)] = d->qvel[k];
  for (int k = 0; k < m->nv; k++) s.warm[SV(s, k, e)] = d->qacc_warmstart[k];
  for (int k = 0; k < NCARRY; k++) s.carry[SC(s, k, e)] = carry[k];
  s.ncon[e] = d->ncon;
  s.nwarn[e] = d->nwarn;
  for (int k = 0; k < UR3E_MAXTOUCH; k++) s.touch[(size_t)e * UR3E_MAXTOUCH + k] = d->touch[k];
  for (int k = 0; k < m->nu; k++) s.ctrl[(size_t)e * UR3E_MAXU + k] = d->ctrl[k];
}

/* reset one env in registers/scratch: keyframe (+ mug noise), forward, obs, carry */
KD void k_reset_env(KModel m, const KConfig& c, const KState& s, int e, KData* d, double obs[24],
                    double carry[NCARRY]) {
  for (int k = 0; k < m->nq; k++) d->qpos[k] = m->qpos0[k];
  for (int k = 0; k < m->nv; k++) { d->qvel[k] = 0; d->qacc_warmstart[k] = 0; }
  for (int k = 0; k < m->nu; k++) d->ctrl[k] = 0;
  if (c.reset_key >= 0) {
    for (int k = 0; k < m->nq; k++) d->qpos[k] = m->key_qpos[c.reset_key][k];
    for (int k = 0; k < m->nv; k++) d->qvel[k] = m->key_qvel[c.reset_key][k];
  }
  unsigned int ep = s.episode[e];
  if (c.reset_noise && m->id_body_fish >= 0) {
    unsigned int gid = (unsigned int)(c.env_id_offset + e);
    double u0 = k_uniform01(c.seed, gid, ep, 0);
    double u1 = k_uniform01(c.seed, gid, ep, 1);
    double ylo, yhi;
    k_noise_ybounds(c.reset_noise, &ylo, &yhi);
    d->qpos[14] += 0.0 + (0.02 - 0.0) * u0;
    d->qpos[15] += ylo + (yhi - ylo) * u1;
  }
  d->nwarn = 0;
  k_forward(m, d);
  s.t[e] = 0;
  s.ep_len[e] = 0;
  s.ep_return[e] = 0;
  s.episode[e] = ep + 1;
  if (c.task == UR3E_TASK_GYM_V2 || c.obs_sites) k_obs_v2(m, d, obs);
  k_make_carry(m, d, carry);
}

KD int k_env_index(const KConfig& c, int n) {
  int lane = threadIdx.x;
  if (lane >= c.epb) return -1;
  int e = blockIdx.x * c.epb + lane;
  return e < n ? e : -1;
}

__global__ __launch_bounds__(64) void k_env_reset(const ur3e_model_t* __restrict__ m, KConfig c, KState s,
                                                  const unsigned char* __restrict__ mask,
                                                  double* __restrict__ obs_out) {
  int e = k_env_index(c, s.n);
  if (e < 0) return;
  if (mask && !mask[e]) return;
  KData d;
  double obs[24], carry[NCARRY];
  k_reset_env(m, c, s, e, &d, obs, carry);
  k_store(m, s, e, &d, carry);
  if (obs_out && (c.task == UR3E_TASK_GYM_V2 || c.obs_sites))
    for (int k = 0; k < 24; k++) obs_out[(size_t)e * 24 + k] = obs[k];
}

__global__ __launch_bounds__(64) void k_env_step(const ur3e_model_t* __restrict__ m, KConfig c, KState s,
                                                 const double* __restrict__ actions, int adim,
                                                 double* __restrict__ obs_out, double* __restrict__ rew_out,
                                                 unsigned char* __restrict__ term_out,
                                                 unsigned char* __restrict__ trunc_out,
                                                 double* __restrict__ tobs_out) {
  int e = k_env_index(c, s.n);
  if (e < 0) return;
  const int n = s.n;
  KData d;
  k_load(m, s, e, &d);
  double a[8];
  for (int k = 0; k < adim && k < 8; k++) a[k] = actions[(size_t)e * adim + k];
  double ctrl[K_NU];
  double carry[NCARRY];
  if (c.task == UR3E_TASK_MOVE_L) {
    for (int k = 0; k < NCARRY; k++) carry[k] = s.carry[SC(s, k, e)];
    k_move_l_ctrl(m, a, carry, d.qpos, d.qvel, c.gains, ctrl);
  } else if (c.task == UR3E_TASK_GYM_V2 || c.task == UR3E_TASK_TRAJ_L) {
    for (int k = 0; k < NCARRY; k++) carry[k] = s.carry[SC(s, k, e)];
    double traj[7];
    if (c.task == UR3E_TASK_GYM_V2) {
      traj[0] = a[0]; traj[1] = a[1]; traj[2] = a[2];
      traj[3] = -1.209; traj[4] = -1.209; traj[5] = 1.209;
      traj[6] = a[3];
    } else {
      for (int k = 0; k < 7; k++) traj[k] = a[k];
    }
    double out[7];
    k_pid_task_ctrl(traj, carry, d.qvel, c.gains, m->act_ctrlrange[m->nu - 1][1], out);
    for (int k = 0; k < 6; k++) ctrl[k] = out[k];
    if (m->nu > 6) ctrl[6] = out[6];
  } else if (c.task == UR3E_TASK_MOVE_J) {
    k_move_j_ctrl(m, &d, a, c.gains, ctrl);
  } else {
    for (int k = 0; k < m->nu; k++) ctrl[k] = a[k];
  }
  for (int k = 0; k < m->nu; k++) d.ctrl[k] = ctrl[k];
  int fs = (c.task == UR3E_TASK_GYM_V2 || c.task == UR3E_TASK_CTRL) ? c.frame_skip : 1;
  for (int sstep = 0; sstep < fs; sstep++) k_step(m, &d);
  k_make_carry(m, &d, carry);
  int t = s.t[e] + 1;
  s.t[e] = t;
  if (c.task != UR3E_TASK_GYM_V2) {
    s.ep_len[e] += 1;
    k_store(m, s, e, &d, carry);
    if (obs_out && c.obs_sites) {
      double ob[24];
      k_obs_v2(m, &d, ob);
      for (int k = 0; k < 24; k++) obs_out[(size_t)e * 24 + k] = ob[k];
    }
    return;
  }
  double obs[24];
  k_obs_v2(m, &d, obs);
  double r = k_reward_v2(obs, a);
  int term = k_termination_v2(m, &d, obs);
  int trunc = c.max_episode_steps > 0 ? (t >= c.max_episode_steps) : 0;
  double dx = obs[3] - obs[6], dy = obs[4] - obs[7], dz = obs[5] - obs[8];
  if (sqrt(dx * dx + dy * dy + dz * dz) < 0.05) {
    term = 1;
    r += 50.0;
  }
  s.ep_return[e] += r;
  s.ep_len[e] += 1;
  if (rew_out) rew_out[e] = r;
  if (term_out) term_out[e] = (unsigned char)term;
  if (trunc_out) trunc_out[e] = (unsigned char)trunc;
  if ((term || trunc) && c.auto_reset) {
    if (tobs_out)
      for (int k = 0; k < 24; k++) tobs_out[(size_t)e * 24 + k] = obs[k];
    k_reset_env(m, c, s, e, &d, obs, carry);
  }
  k_store(m, s, e, &d, carry);
  if (obs_out)
    for (int k = 0; k < 24; k++) obs_out[(size_t)e * 24 + k] = obs[k];
}

__global__ __launch_bounds__(64) void k_env_set_state(const ur3e_model_t* __restrict__ m, KConfig c, KState s,
                                                      const double* __restrict__ qpos,
                                                      const double* __restrict__ qvel,
                                                      const double* __restrict__ warm) {
  int e = k_env_index(c, s.n);
  if (e < 0) return;
  KData d;
  for (int k = 0; k < m->nq; k++) d.qpos[k] = qpos[(size_t)e * m->nq + k];
  for (int k = 0; k < m->nv; k++) d.qvel[k] = qvel[(size_t)e * m->nv + k];
  for (int k = 0; k < m->nv; k++) d.qacc_warmstart[k] = warm ? warm[(size_t)e * m->nv + k] : s.warm[SV(s, k, e)];
  d.nwarn = s.nwarn[e];
  for (int k = 0; k < m->nu; k++) d.ctrl[k] = 0;
  k_forward(m, &d);
  double carry[NCARRY];
  k_make_carry(m, &d, carry);
  k_store(m, s, e, &d, carry);
}


/* ================================================================== */
/* workgroup-per-env kernels (v2, default): see ur3e_wave.h            */
/* ================================================================== */
/* carry from the LDS working set: tcp pose, arm Jacobian (6x6), qfrc_bias[0:6] */
template <int NT, class KS>
WD void w_make_carry(KModel m, const KPlan* __restrict__ pl, const KS& s, double* carry) {
  const int tid = w_lane();
  int st = m->id_site_tcp;
  if (st < 0) {
    for (int k = tid; k < NCARRY; k += NT) carry[k] = 0;
    return;
  }
  int b = m->site_bodyid[st];
  const double* c = s.subtree_com[m->body_rootid[b]];
  const double* p = s.site_xpos[st];
  double off[3] = {p[0] - c[0], p[1] - c[1], p[2] - c[2]};
  for (int k = tid; k < NCARRY; k += NT) {
    double v;
    if (k < 3) {
      v = p[k];
    } else if (k < 12) {
      v = s.site_xmat[st][k - 3];
    } else if (k < 48) {
      int r = (k - 12) / 6, col = (k - 12) % 6;
      if (r < 3) {
        double jp[3];
        w_jacp_col(m, pl, s, b, off, col, jp);
        v = jp[r];
      } else {
        v = ((pl->body_dof_mask[b] >> col) & 1u) ? s.cdof[col][r - 3] : 0.0;
      }
    } else {
      v = s.qfrc_bias[k - 48];
    }
    carry[k] = v;
  }
}

/* mj_objectVelocity of a site (world frame, [w, v]); b, root: the site's body and its root (KPlan.sv_*
   resolves them on the host for the epilogue's two sites) */
template <class KS>
KD void w_site_velocity(KModel m, const KS& s, int site, double res[6], int b, int root) {
  const double* cv = s.cvel[b];
  const double* c = s.subtree_com[root];
  double dif[3] = {s.site_xpos[site][0] - c[0], s.site_xpos[site][1] - c[1], s.site_xpos[site][2] - c[2]};
  double cr[3];
  k_cross3(cr, dif, cv);
  res[0] = cv[0]; res[1] = cv[1]; res[2] = cv[2];
  res[3] = cv[3] - cr[0]; res[4] = cv[4] - cr[1]; res[5] = cv[5] - cr[2];
}
template <class KS>
KD void w_site_velocity(KModel m, const KS& s, int site, double res[6]) {
  const int b = m->site_bodyid[site];
  w_site_velocity(m, s, site, res, b, m->body_rootid[b]);
}

/* UR3eEnv2._get_obs (ur3e_env2.py:111-123), lane 0.  pads >= 0: the pad-contact scan below done
   beforehand by w_contact_flags (bit 0 left pad, bit 1 right pad) */
template <class KS>
KD void w_obs_v2(KModel m, const KS& s, double obs[24], int pads = -1) {
  int st = m->id_site_tcp, sh = m->id_site_handle, gb = m->id_body_ghost;
  const double* tcp = s.site_xpos[st];
  const double* mug = s.site_xpos[sh];
  const double* gh = s.xpos[gb];
  double vt[6], vh[6];
  if constexpr (KS::OVERLAY) {
    /* computed in w_forward while cvel was alive (same sites, same expression) */
    for (int k = 0; k < 6; k++) { vt[k] = s.site_vel[0][k]; vh[k] = s.site_vel[1][k]; }
  } else {
    w_site_velocity(m, s, st, vt);
    w_site_velocity(m, s, sh, vh);
  }
  for (int k = 0; k < 3; k++) {
    obs[k] = tcp[k];
    obs[3 + k] = mug[k];
    obs[6 + k] = gh[k];
    obs[9 + k] = tcp[k] - mug[k];
    obs[12 + k] = mug[k] - gh[k];
    obs[15 + k] = vt[3 + k];
    obs[18 + k] = vt[3 + k] - vh[3 + k];
  }
  obs[21] = s.qpos[6];
  obs[22] = s.qvel[6];
  int lp = 0, rp = 0;
  if (pads >= 0) {
    lp = pads & 1;
    rp = (pads >> 1) & 1;
  } else {
    for (int ci = 0; ci < s.ncon; ci++) {
      int b1 = m->geom_bodyid[s.con_geom1[ci]], b2 = m->geom_bodyid[s.con_geom2[ci]];
      if (!(b1 == m->id_body_fish || b2 == m->id_body_fish)) continue;
      if (b1 == m->id_body_lpad || b2 == m->id_body_lpad) lp = 1;
      if (b1 == m->id_body_rpad || b2 == m->id_body_rpad) rp = 1;
    }
  }
  int robust = 0;
  if (lp + rp == 2) {
    double dx = fabs(tcp[0] - mug[0]), dy = fabs(tcp[1] - mug[1]), dz = fabs(tcp[2] - mug[2]);
    robust = (dx < 0.01 && dy < 0.005 && dz < 0.05);
  }
  obs[23] = (double)robust;
}

/* armc >= 0: the arm self-contact scan below done beforehand by w_contact_flags (bit 2) */
template <class KS>
KD int w_termination_v2(KModel m, const KS& s, const double obs[24], int armc = -1) {
  double dx = obs[0] - obs[3], dy = obs[1] - obs[4], dz = obs[2] - obs[5];
  if (1.0 < sqrt(dx * dx + dy * dy + dz * dz)) return 1;
  if (armc >= 0) return (armc >> 2) & 1 ? 1 : obs[5] <= m->fish_topple_z;
  for (int ci = 0; ci < s.ncon; ci++) {
    int b1 = m->geom_bodyid[s.con_geom1[ci]], b2 = m->geom_bodyid[s.con_geom2[ci]];
    int a1 = (m->mask_arm_bodies >> b1) & 1, a2 = (m->mask_arm_bodies >> b2) & 1;
    if (a1 && a2) {
      int g1 = (m->mask_gripper_bodies >> b1) & 1, g2 = (m->mask_gripper_bodies >> b2) & 1;
      if (g1 && g2) continue;
      return 1;
    }
  }
  if (obs[5] <= m->fish_topple_z) return 1;
  return 0;
}

/* the contact-list scans of w_obs_v2 (gripper pads on the mug) and w_termination_v2 (arm self-contact)
   with one contact per lane: each scan is an OR over the list, so the order does not matter, and the
   per-contact body-id loads are issued together instead of one dependent pair per contact on lane 0.
   bit 0: fish-left pad, bit 1: fish-right pad, bit 2: arm-arm contact that is not gripper-gripper.
   Uniform result. */
template <int NT, class KS>
WD int w_contact_flags(KModel m, const KS& s) {
  int lp = 0, rp = 0, arm = 0;
  for (int ci = w_lane(); ci < s.ncon; ci += NT) {
    const int b1 = m->geom_bodyid[s.con_geom1[ci]], b2 = m->geom_bodyid[s.con_geom2[ci]];
    const bool fish = b1 == m->id_body_fish || b2 == m->id_body_fish;
    lp |= fish && (b1 == m->id_body_lpad || b2 == m->id_body_lpad);
    rp |= fish && (b1 == m->id_body_rpad || b2 == m->id_body_rpad);
    const int a1 = (m->mask_arm_bodies >> b1) & 1, a2 = (m->mask_arm_bodies >> b2) & 1;
    const int g1 = (m->mask_gripper_bodies >> b1) & 1, g2 = (m->mask_gripper_bodies >> b2) & 1;
    arm |= a1 && a2 && !(g1 && g2);
  }
  return w_any<NT>(lp) | (w_any<NT>(rp) << 1) | (w_any<NT>(arm) << 2);
}

/* gym_utils.get_self_collision / get_table_collision (gym_utils.py:146-197) on the LDS contact list */
template <class KS>
KD int w_self_collision(KModel m, const KS& s) {
  for (int ci = 0; ci < s.ncon; ci++) {
    int b1 = m->geom_bodyid[s.con_geom1[ci]], b2 = m->geom_bodyid[s.con_geom2[ci]];
    int a1 = (m->mask_arm_bodies >> b1) & 1, a2 = (m->mask_arm_bodies >> b2) & 1;
    if (a1 && a2) {
      int g1 = (m->mask_gripper_bodies >> b1) & 1, g2 = (m->mask_gripper_bodies >> b2) & 1;
      if (g1 && g2) continue;
      return 1;
    }
  }
  return 0;
}

template <class KS>
KD int w_table_collision(KModel m, const KS& s) {
  for (int ci = 0; ci < s.ncon; ci++) {
    int b1 = m->geom_bodyid[s.con_geom1[ci]], b2 = m->geom_bodyid[s.con_geom2[ci]];
    int g1 = (m->mask_gripper_bodies >> b1) & 1, g2 = (m->mask_gripper_bodies >> b2) & 1;
    if ((g1 && b2 == m->id_body_table) || (g2 && b1 == m->id_body_table)) return 1;
  }
  return 0;
}

template <class KS>
KD int w_block_grasp_state(KModel m, const KS& s) {
  int lp = 0, rp = 0;
  for (int ci = 0; ci < s.ncon; ci++) {
    int b1 = m->geom_bodyid[s.con_geom1[ci]], b2 = m->geom_bodyid[s.con_geom2[ci]];
    if (!(b1 == m->id_body_fish || b2 == m->id_body_fish)) continue;
    if (b1 == m->id_body_lpad || b2 == m->id_body_lpad) lp = 1;
    if (b1 == m->id_body_rpad || b2 == m->id_body_rpad) rp = 1;
  }
  return lp + rp;
}

/* UR3eEnv._get_obs (ur3e_env.py) / ImitationEnvDirect._get_obs (imitation_env_direct.py): 13-d */
template <class KS>
KD void w_obs13(KModel m, const KS& s, int direct, double obs[13]) {
  const double* tcp = s.site_xpos[m->id_site_tcp];
  const double* mug = s.site_xpos[m->id_site_handle];
  const double* gh = s.xpos[m->id_body_ghost];
  double tail[3];
  if (direct) {
    double vt[6];
    w_site_velocity(m, s, m->id_site_tcp, vt);
    tail[0] = vt[3]; tail[1] = vt[4]; tail[2] = vt[5];
  } else {
    const double* pad = s.site_xpos[m->id_site_rpad];
    tail[0] = pad[0]; tail[1] = pad[1]; tail[2] = pad[2];
  }
  for (int k = 0; k < 3; k++) { obs[k] = tcp[k]; obs[3 + k] = mug[k]; obs[6 + k] = gh[k]; obs[10 + k] = tail[k]; }
  obs[9] = (double)w_block_grasp_state(m, s);
}

KD double k_sq(double x) { return x * x; }

/* UR3eEnv.compute_reward (ur3e_env.py), same expressions as oracle ur3o_reward_v0 */
KD double k_reward_v0(KModel m, const double obs[13], const double act[4], int selfcol, int tablecol) {
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
  double grasp_readiness = ur3e_exp(-k_sq(horizontal_error)) * ur3e_exp(-k_sq(pad_to_block_top)) *
                           ur3e_exp(-k_sq(height_error)) * 100 * ur3e_exp(-k_sq(act[3]));
  double alignment_reward = 4 * ur3e_exp(-60 * k_sq(horizontal_error));
  double grip_strength = act[3];
  double g2 = grasp_state == 2 ? 1.0 : 0.0, g1 = grasp_state >= 1 ? 1.0 : 0.0;
  double grasp_reward = 5.5 * g1 + 8.5 * g2 + 23.5 * grip_strength * grasp_readiness + 28.5 * g2 * grasp_readiness +
                        11.5 * g2 * grasp_readiness * ur3e_tanh(8 * grip_strength);
  double lift_reward = 12 * g2 * ur3e_tanh(4 * block_bottom_z);
  double px = block_center[0] - target_pos[0], py = block_center[1] - target_pos[1],
         pz = block_center[2] - target_pos[2];
  double d_place = sqrt(px * px + py * py + pz * pz);
  double placement_reward = -2 * d_place + 20 * ur3e_exp(-70 * k_sq(d_place));
  if (d_place < 0.05 && valid_grasp) placement_reward += 40;
  double hh = block_center[2] - gripper_pos[2] + 0.5;
  double dh = -100000000000.0 * (hh * hh * hh);
  double dangerous_height_penalty = dh < 0 ? dh : 0;
  double p2b = pad_to_block_top > 0 ? pad_to_block_top : 0;
  double penalties = -40 * selfcol + -25 * tablecol + -8 * (block_center[2] <= m->fish_topple_z) + -4 * p2b +
                     dangerous_height_penalty;
  double action_reward = 700.5 * grip_strength * grasp_readiness;
  double contact_achievement_bonus = 1700.5 * g2 * grasp_readiness * ur3e_tanh(10 * grip_strength);
  return descent_reward + alignment_reward + grasp_reward + lift_reward + placement_reward + action_reward +
         contact_achievement_bonus + penalties;
}

KD int k_termination_v0(KModel m, const double obs[13], int selfcol) {
  double dx = obs[0] - obs[3], dy = obs[1] - obs[4], dz = obs[2] - obs[5];
  double ex = obs[3] - obs[6], ey = obs[4] - obs[7], ez = obs[5] - obs[8];
  double d_pick = sqrt(dx * dx + dy * dy + dz * dz);
  double d_place = sqrt(ex * ex + ey * ey + ez * ez);
  if (d_place < 0.005) return 1;
  if (1 < d_pick) return 1;
  if (selfcol) return 1;
  if (obs[5] <= m->fish_topple_z) return 1;
  return 0;
}

__host__ __device__ static inline int k_is_gym(int task) {
  return task == UR3E_TASK_GYM_V2 || (task >= UR3E_TASK_GYM_V0 && task <= UR3E_TASK_IMIT_DIRECT);
}
__host__ __device__ static inline int k_obs_dim(int task) { return (task == UR3E_TASK_GYM_V0 || task == UR3E_TASK_IMIT_DIRECT) ? 13 : 24; }

/* the task's observation into obs (lane 0) */
template <class KS>
KD void w_task_obs(KModel m, const KS& s, int task, double* obs) {
  if (task == UR3E_TASK_GYM_V0) w_obs13(m, s, 0, obs);
  else if (task == UR3E_TASK_IMIT_DIRECT) w_obs13(m, s, 1, obs);
  else w_obs_v2(m, s, obs);
}

/* per-env step results staged in LDS; nothing reaches global memory before w_commit, so a
   compact-tier env that overflows (s.ovf) can be recomputed from its untouched state */
struct WOut {
  double obs[24];
  double tobs[24];
  double a[8];
  double r, ep_return;
  int term, trunc, t, ep_len, did_reset;
  unsigned int episode;
  /* the env index, parked in LDS for the uses after the forward passes (auto-reset, queue hand-off,
     commit): kept in a register across the step it and the addresses derived from it were spilled */
  int e;
};

/* The compact tier's working set (the overlaid layout, with WOut behind it) lives in DYNAMIC LDS, sized
   at launch (w_dyn_lds): with static LDS the compiler derives the kernel's occupancy from it -- 16 KB
   allows 10 workgroups per CU, i.e. 2.5 waves per SIMD, which it rounds down to 2.  Out of its sight,
   the waves per SIMD the kernel is compiled for are W_COMPACT_WPE's alone (2, ~205 registers: eight envs
   per CU; 3 builds the measured-slower 168-register, ten-per-CU variant).  The other layouts keep
   static LDS. */
template <class KS>
constexpr size_t w_wout_off() { return (sizeof(KS) + 15) & ~(size_t)15; }
/* W_DYN_PAD: diagnostic builds only (A/B of the register budget at a fixed occupancy): extra dynamic
   LDS per compact workgroup */
#ifndef W_DYN_PAD
#define W_DYN_PAD 0
#endif
template <class KS>
constexpr size_t w_dyn_lds() { return KS::OVERLAY ? w_wout_off<KS>() + sizeof(WOut) + W_DYN_PAD : 0; }
template <class KS>
__device__ __forceinline__ KS& w_smem() {
  if constexpr (KS::OVERLAY) {
    extern __shared__ __align__(16) char w_dyn[];
    return *reinterpret_cast<KS*>(w_dyn);
  } else {
    __shared__ KS s;
    return s;
  }
}
template <class KS>
__device__ __forceinline__ WOut& w_wout() {
  if constexpr (KS::OVERLAY) {
    extern __shared__ __align__(16) char w_dyn[];
    return *reinterpret_cast<WOut*>(w_dyn + w_wout_off<KS>());
  } else {
    __shared__ WOut o;
    return o;
  }
}

template <int NT, class KS>
WD void w_load(KModel m, const KConfig& c, const KState& st, int e, KS& s, WOut& o) {
  const int tid = w_lane();
  for (int k = tid; k < m->nq; k += NT) s.qpos[k] = st.qpos[SQ(st, k, e)];
  for (int k = tid; k < m->nv; k += NT) { s.qvel[k] = st.qvel[SV(st, k, e)]; s.warm[k] = st.warm[SV(st, k, e)]; }
  if (tid == 0) {
    s.nwarn = st.nwarn[e];
    s.ovf = 0;
    /* diagnostic contact cap: > 0 caps the compact tier only (its envs then run in the grasp tier, which
       the step then always launches behind it), < 0 caps every bailing tier (compact and grasp: the envs
       reach the full-capacity tier) */
    const int cap = c.tier_con_cap, capv = cap > 0 ? cap : -cap;
    /* the compact tiers: the gym layout and the scripted pick's wider one (KSS_NV_W / KSS_NV_MW) */
    constexpr bool compact = KS::OVERLAY && KS::MAXCON <= W_WIDE_MAXCON;
    const bool capped = KS::BAIL && (cap < 0 || (cap > 0 && compact));
    s.cap_con = (capped && capv < KS::MAXCON) ? capv : KS::MAXCON;
    if constexpr (KS::OVERLAY) s.np_lanes = c.np_lanes;
    else s.sens = c.sensors;
    o.t = st.t[e]; o.ep_len = st.ep_len[e]; o.ep_return = st.ep_return[e]; o.episode = st.episode[e];
    o.did_reset = 0; o.term = 0; o.trunc = 0; o.r = 0; o.e = e;
  }
}

/* the single write-back point of every v2 kernel */
template <int NT, int TK = -1, class KS>
WD void w_commit(KModel m, const KConfig& c, const KState& st, int e, const KS& s, const WOut& o, double* obs_out,
                 double* rew_out, unsigned char* term_out, unsigned char* trunc_out, double* tobs_out, int stepped) {
  const int TASK = TK >= 0 ? TK : c.task; /* TK >= 0: kernel specialised for one task at compile time */
  const int tid = w_lane();
  for (int k = tid; k < m->nq; k += NT) st.qpos[SQ(st, k, e)] = s.qpos[k];
  for (int k = tid; k < m->nv; k += NT) { st.qvel[SV(st, k, e)] = s.qvel[k]; st.warm[SV(st, k, e)] = s.warm[k]; }
  for (int k = tid; k < NCARRY; k += NT) st.carry[SC(st, k, e)] = s.carry[k];
  for (int k = tid; k < UR3E_MAXTOUCH; k += NT) st.touch[(size_t)e * UR3E_MAXTOUCH + k] = s.touch[k];
  for (int k = tid; k < m->nu; k += NT) {
    st.ctrl[(size_t)e * UR3E_MAXU + k] = s.ctrl[k];
    st.actfrc[(size_t)e * UR3E_MAXU + k] = s.act_force[k];
  }
  if constexpr (!KS::OVERLAY) {
    if (c.sensors)
      for (int k = tid; k < m->nsensordata; k += NT)
        st.sensordata[(size_t)e * UR3E_MAXSENSORDATA + k] = s.sensordata[k];
  }
  const int od = k_obs_dim(TASK);
  if (tid == 0) {
    st.ncon[e] = s.ncon; st.nwarn[e] = s.nwarn;
    if (st.hint) {
      /* 0: the compact tier; 1: the mid tier; 2: the grasp tier */
      const bool over = s.ncon > c.route_ncon || s.nefc > c.route_nefc;
      const bool mid = c.route2_ncon >= 0 && s.ncon <= c.route2_ncon && s.nefc <= c.route2_nefc;
      st.hint[e] = (unsigned char)(over ? (mid ? 1 : 2) : 0);
    }
    st.t[e] = o.t; st.ep_len[e] = o.ep_len; st.ep_return[e] = o.ep_return; st.episode[e] = o.episode;
    if (stepped && k_is_gym(TASK)) {
      if (rew_out) rew_out[e] = o.r;
      if (term_out) term_out[e] = (unsigned char)o.term;
      if (trunc_out) trunc_out[e] = (unsigned char)o.trunc;
    }
  }
  if (k_is_gym(TASK)) {
    if (stepped && o.did_reset && tobs_out)
      for (int k = tid; k < od; k += NT) tobs_out[(size_t)e * od + k] = o.tobs[k];
  }
  if (obs_out && (k_is_gym(TASK) || c.obs_sites))
    for (int k = tid; k < od; k += NT) obs_out[(size_t)e * od + k] = o.obs[k];
}

/* reset the env held in LDS: keyframe (+ mug noise) -> forward -> obs, carry (all lanes) */
template <int NT, class KS>
WD void w_reset_prep(KModel m, const KConfig& c, int e, KS& s, WOut& o) {
  const int tid = w_lane();
  for (int k = tid; k < m->nq; k += NT) s.qpos[k] = c.reset_key >= 0 ? m->key_qpos[c.reset_key][k] : m->qpos0[k];
  for (int k = tid; k < m->nv; k += NT) { s.qvel[k] = c.reset_key >= 0 ? m->key_qvel[c.reset_key][k] : 0.0; s.warm[k] = 0; }
  for (int k = tid; k < m->nu; k += NT) s.ctrl[k] = 0;
  SYNC();
  if (tid == 0) {
    unsigned int ep = o.episode;
    if (c.reset_noise && m->id_body_fish >= 0) {
      unsigned int gid = (unsigned int)(c.env_id_offset + e);
      double u0 = k_uniform01(c.seed, gid, ep, 0);
      double u1 = k_uniform01(c.seed, gid, ep, 1);
      double ylo, yhi;
      k_noise_ybounds(c.reset_noise, &ylo, &yhi);
      s.qpos[14] += 0.0 + (0.02 - 0.0) * u0;
      s.qpos[15] += ylo + (yhi - ylo) * u1;
    }
    s.nwarn = 0;
    o.t = 0;
    o.ep_len = 0;
    o.ep_return = 0;
    o.episode = ep + 1;
  }
  SYNC();
}

template <int NT, int TK = -1, class KS>
WD void w_reset_finish(KModel m, const KPlan* __restrict__ pl, const KConfig& c, KS& s, WOut& o) {
  const int TASK = TK >= 0 ? TK : c.task; /* TK >= 0: kernel specialised for one task at compile time */
  const int tid = w_lane();
  if (tid == 0 && (k_is_gym(TASK) || c.obs_sites)) w_task_obs(m, s, TASK, o.obs);
  w_make_carry<NT>(m, pl, s, s.carry);
  SYNC();
}

template <int NT, int TK = -1, class KS>
WD void w_reset_env(KModel m, const KPlan* __restrict__ pl, const KConfig& c, int e, KS& s, WOut& o) {
  w_reset_prep<NT>(m, c, e, s, o);
  w_forward<NT>(m, pl, s);
  if (KS::BAIL && s.ovf) return;
  w_reset_finish<NT, TK>(m, pl, c, s, o);
}

/* mid-step state of an env between the substep units of the queued step kernel (w_env_step_q):
   qpos, qvel, qacc_warmstart after the unit's last Euler update, the applied ctrl and the warning
   count -- everything the next substep reads that is not in the env's committed state */
#define W_MID_QPOS 0
#define W_MID_QVEL K_NQ
#define W_MID_WARM (K_NQ + K_NV)
#define W_MID_CTRL (K_NQ + 2 * K_NV)
#define W_MID_NWARN (K_NQ + 2 * K_NV + K_NU)
/* records padded to whole 128-B lines (80 doubles): no line is shared by two envs, and one store
   instruction of the storing wave writes every line of the record whole */
#define W_MID (((W_MID_NWARN + 1) + 15) / 16 * 16)

/* hand-off words go write-through / L1-bypassing (sc1) at agent scope, so neither side needs a
   cache-maintenance fence (the MI355X publish/consume recipe R1: payload stores sc1 and drained
   before the flag; every payload load sc1) */
typedef __attribute__((address_space(1))) unsigned long long gu64_t;
KD void w_put_sc1(double* p, double v) {
  __hip_atomic_store((gu64_t*)p, __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

template <int NT, class KS>
WD void w_store_mid(KModel m, double* __restrict__ mid, int e, const KS& s) {
  const int tid = w_lane();
  double* p = mid + (size_t)e * W_MID;
  /* one 16-byte write-through store per lane (pairs of doubles): narrow sc1 stores each cost a
     separate partial-line write */
  if (tid < W_MID / 2) {
    double v[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int k = 2 * tid + h;
      double x = 0.0;
      if (k < W_MID_QVEL) x = k < m->nq ? s.qpos[k] : 0.0;
      else if (k < W_MID_WARM) x = k - W_MID_QVEL < m->nv ? s.qvel[k - W_MID_QVEL] : 0.0;
      else if (k < W_MID_CTRL) x = k - W_MID_WARM < m->nv ? s.warm[k - W_MID_WARM] : 0.0;
      else if (k < W_MID_NWARN) x = k - W_MID_CTRL < m->nu ? s.ctrl[k - W_MID_CTRL] : 0.0;
      else if (k == W_MID_NWARN) x = (double)s.nwarn;
      v[h] = x;
    }
    /* buffer descriptor over this env's mid record (wave-uniform base), aux 16 = sc1 */
    __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, W_MID * 8, 0x00020000);
    typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;
    const unsigned long long a = __builtin_bit_cast(unsigned long long, v[0]);
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v[1]);
    u32x4_t w = {(unsigned)a, (unsigned)(a >> 32), (unsigned)b, (unsigned)(b >> 32)};
    __builtin_amdgcn_raw_buffer_store_b128(w, rsrc, 16 * tid, 0, 16);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); /* every storing lane drained before the flag */
}

/* one env-step of env e into LDS (s, o), or the substeps [sub_begin, sub_end) of it.  Returns
   W_DONE (results staged for w_commit), W_BAIL (the compact tier overflowed: nothing was written)
   or W_PAUSED (sub_end < frame_skip: the state after substep sub_end - 1 is in LDS for
   w_store_mid).  sub_begin > 0 resumes from the mid-step state `mid`, skipping the controller. */
/* UR3eEnv2's epilogue (obs, compute_reward, termination, the success bonus; the lane-0 branch of
   w_env_step_body) with its five square roots on lanes 0-4 and its four exponentials (tanh's included)
   on lanes 0-3, one pass each instead of one after the other on lane 0: every operand and expression is
   k_reward_v2's / w_termination_v2's, so the bits are the same.  One wavefront (64 lanes). */
template <class KS>
WD void w_epilogue_v2_lanes(KModel m, const KConfig& c, const KS& s, WOut& o, int cfl) {
  constexpr int NT = 64;
  const int tid = w_lane();
  const int t = o.t + 1;
  if (tid == 0) {
    o.t = t;
    w_obs_v2(m, s, o.obs, cfl);
  }
  SYNC();
  const double* ob = o.obs;
  /* lane 0: |g2m.xy|, 1: |m2t|, 2: |gripper velocity|, 3: |tcp - mug| (termination), 4: |mug - target|
     (success); the two-term sum gets + 0 * 0, an exact no-op on a sum of squares */
  const int k = tid < 5 ? tid : 0;
  double v0, v1, v2;
  if (k == 0) { v0 = ob[9]; v1 = ob[10]; v2 = 0.0; }
  else if (k == 1) { v0 = ob[12]; v1 = ob[13]; v2 = ob[14]; }
  else if (k == 2) { v0 = ob[15]; v1 = ob[16]; v2 = ob[17]; }
  else if (k == 3) { v0 = ob[0] - ob[3]; v1 = ob[1] - ob[4]; v2 = ob[2] - ob[5]; }
  else { v0 = ob[3] - ob[6]; v1 = ob[4] - ob[7]; v2 = ob[5] - ob[8]; }
  const double nrm = sqrt(v0 * v0 + v1 * v1 + v2 * v2);
  const double xy = rl(nrm, 0), place = rl(nrm, 1), gvn = rl(nrm, 2), dterm = rl(nrm, 3), dsucc = rl(nrm, 4);
  const double mug_z = ob[5], zerr = fabs(ob[11] - 0.02);
  const double tx = 8.0 * (mug_z > 0 ? mug_z : 0); /* ur3e_tanh's argument; its |x| is x (>= 0 or NaN) */
  const double ax = tx < 0 ? -tx : tx;
  const int j = tid < 4 ? tid : 0;
  const double arg = j == 0 ? -10 * xy : (j == 1 ? -20 * zerr : (j == 2 ? -15 * place : 2.0 * ax));
  const double ex = ur3e_exp(arg);
  const double e_xy = rl(ex, 0), e_z = rl(ex, 1), e_pl = rl(ex, 2), e_th = rl(ex, 3);
  if (tid == 0) {
    const double grasped = ob[23], grip = o.a[3];
    const double ready = e_xy * e_z;
    const double align = 2.0 * ready;
    const double grasp_act = 2.0 * grip * ready;
    const double grasp_ach = 10.0 * grasped * ready;
    const double th_t = ax > 22.0 ? 1.0 : 1.0 - 2.0 / (e_th + 1.0);
    const double lift = 8.0 * grasped * (tx < 0 ? -th_t : th_t);
    const double placement = grasped * (4.0 * e_pl - 1.5 * place);
    double success = 0.0;
    if (grasped != 0 && place < 0.05) success = 50.0;
    double pen = 0.0;
    pen += -1.0 * (-ob[11] > 0 ? -ob[11] : 0);
    pen += -0.01 * gvn;
    double r = align + grasp_act + grasp_ach + lift + placement + success + pen;
    int term = 1.0 < dterm ? 1 : ((cfl >> 2) & 1 ? 1 : ob[5] <= m->fish_topple_z);
    const int trunc = c.max_episode_steps > 0 ? (t >= c.max_episode_steps) : 0;
    if (dsucc < 0.05) {
      term = 1;
      r += 50.0;
    }
    o.ep_return += r;
    o.ep_len += 1;
    o.r = r;
    o.term = term;
    o.trunc = trunc;
  }
}

/* workgroups of the full-capacity tier's launch (grid-stride over its list; it runs empty on most steps) */
#ifndef W_FULL_GRID
#define W_FULL_GRID 512
#endif
/* the resumed unit's mid-step record loaded together with the committed state (1) or after it (0) */
/* off: no measurable difference same-box (profiles/r04_ab A/B 8) */
#ifndef W_MID_EARLY
#define W_MID_EARLY 0
#endif
/* touch sensors only in the env-step's last forward pass (1, default) or in every pass (0: A/B) */
#ifndef W_TOUCH_LAST
#define W_TOUCH_LAST 1
#endif
/* the gym tasks' controller and epilogue spread over lanes (1, default) or on lane 0 (0: A/B) */
#ifndef W_EPI_LANES
#define W_EPI_LANES 1
#endif
#define W_BAIL 0
#define W_DONE 1
#define W_PAUSED 2
#define W_HALF 3
/* half (the queue's split last substep, compact tier): 0 = whole substeps; 1 = run until the first
   forward pass of the last substep has reached the constraint solver and return W_HALF (the working set
   in LDS is then handed on whole); 2 = resume there: the caller has restored that working set and WOut,
   so nothing is loaded and the step goes on with the solver, sub_begin = the last substep */
template <int NT, int TK = -1, class KS>
WD int w_env_step_body(KModel m, const KPlan* __restrict__ pl, const KConfig& c, const KState& st, int e,
                       const double* __restrict__ actions, int adim, KS& s, WOut& o, int sub_begin = 0,
                       int sub_end = 1 << 30, const double* __restrict__ mid = nullptr, int half = 0) {
  const int TASK = TK >= 0 ? TK : c.task; /* TK >= 0: kernel specialised for one task at compile time */
  const int tid = w_lane();
  WT_START();
  const int fs = (k_is_gym(TASK) || TASK == UR3E_TASK_CTRL) ? c.frame_skip : 1;
  if (half != 2) {
  /* resume (sub_begin > 0): the state after the previous unit's substeps and the ctrl it applied, one
     16-byte sc1 load per lane (the record's doubles 2 tid, 2 tid + 1).  It is issued before the
     committed-state loads, so the two round trips overlap, and scattered to LDS after them (it
     overwrites qpos, qvel, warm start and ctrl) */
  typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;
  u32x4_t wmid = {0u, 0u, 0u, 0u};
  const double* pmid = mid + (size_t)e * W_MID;
  if (W_MID_EARLY && sub_begin > 0 && tid < W_MID / 2) {
    __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)pmid, 0, W_MID * 8, 0x00020000);
    wmid = __builtin_amdgcn_raw_buffer_load_b128(rsrc, 16 * tid, 0, 16);
  }
  w_load<NT>(m, c, st, e, s, o);
  for (int k = tid; k < adim && k < 8; k += NT) o.a[k] = actions[(size_t)e * adim + k];
  for (int k = tid; k < NCARRY; k += NT) s.carry[k] = st.carry[SC(st, k, e)];
  SYNC();
  if (sub_begin > 0) {
    if (tid < W_MID / 2) {
      if (!W_MID_EARLY) {
        __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)pmid, 0, W_MID * 8, 0x00020000);
        wmid = __builtin_amdgcn_raw_buffer_load_b128(rsrc, 16 * tid, 0, 16);
      }
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int k = 2 * tid + h;
        const double x = __builtin_bit_cast(
            double, (unsigned long long)wmid[2 * h] | ((unsigned long long)wmid[2 * h + 1] << 32));
        if (k < W_MID_QVEL) {
          if (k < m->nq) s.qpos[k] = x;
        } else if (k < W_MID_WARM) {
          if (k - W_MID_QVEL < m->nv) s.qvel[k - W_MID_QVEL] = x;
        } else if (k < W_MID_CTRL) {
          if (k - W_MID_WARM < m->nv) s.warm[k - W_MID_WARM] = x;
        } else if (k < W_MID_NWARN) {
          if (k - W_MID_CTRL < m->nu) s.ctrl[k - W_MID_CTRL] = x;
        } else if (k == W_MID_NWARN) {
          s.nwarn = (int)x;
        }
      }
    }
    SYNC();
  }
  WT(24);
#if W_EPI_LANES
  /* the gym tasks' pid_task_ctrl across lanes: lane r < 6 forms row r of J qdot, of u and column r of
     J' u (the same sums in the same order as k_pid_task_ctrl); lane 0 alone the rotation error, against
     the fixed target's quaternion from the host (KConfig.gym_qd) or, for the scripted pick (TRAJ_L), the
     row's own rotvec target */
  constexpr bool CTRL_LANES = TK == UR3E_TASK_GYM_V2 || TK == UR3E_TASK_GYM_V0 || TK == UR3E_TASK_IMIT_INDIRECT ||
                              TK == UR3E_TASK_TRAJ_L;
#else
  constexpr bool CTRL_LANES = false;
#endif
  if constexpr (CTRL_LANES) {
    if (sub_begin == 0) {
      const double* J = s.carry + 12;
      double er = 0;
      if (tid == 0) {
        double e3[3];
        if constexpr (TK == UR3E_TASK_TRAJ_L) k_rot_err(s.carry + 3, o.a + 3, e3); /* the row's rotvec target */
        else k_rot_err_q(s.carry + 3, c.gym_qd, e3);
        er = e3[0];
        s.ctrl[0] = e3[1]; /* staged: the rotation error's y and z for lanes 4 and 5 (ctrl is rewritten below) */
        s.ctrl[1] = e3[2];
      }
      SYNC();
      const int r = tid < 6 ? tid : 0;
      double jv = 0;
#pragma unroll
      for (int k = 0; k < 6; k++) jv += J[6 * r + k] * s.qvel[k];
      const double er_r = r == 3 ? rl(er, 0) : (r == 4 ? s.ctrl[0] : s.ctrl[1]);
      const double ep_r = o.a[r < 3 ? r : 0] - s.carry[r < 3 ? r : 0];
      const double u = r < 3 ? c.gains.task[r] * ep_r - c.gains.task[3 + r] * jv
                             : c.gains.task[6 + r - 3] * er_r - c.gains.task[9 + r - 3] * jv;
      double su = 0;
#pragma unroll
      for (int k = 0; k < 6; k++) su += J[6 * k + r] * rl(u, k);
      const double cv = su + s.carry[48 + r];
      SYNC();
      if (tid < 6) s.ctrl[tid] = cv;
      if (tid == 6 && m->nu > 6) s.ctrl[6] = o.a[TK == UR3E_TASK_TRAJ_L ? 6 : 3] * m->act_ctrlrange[m->nu - 1][1];
    }
  } else if (tid == 0 && sub_begin == 0) {
    double ctrl[K_NU];
    if (TASK == UR3E_TASK_GYM_V2 || TASK == UR3E_TASK_TRAJ_L || TASK == UR3E_TASK_GYM_V0 ||
        TASK == UR3E_TASK_IMIT_INDIRECT) {
      double traj[7];
      if (TASK != UR3E_TASK_TRAJ_L) { /* [x, y, z] + fixed rotvec + grip */
        traj[0] = o.a[0]; traj[1] = o.a[1]; traj[2] = o.a[2];
        traj[3] = -1.209; traj[4] = -1.209; traj[5] = 1.209;
        traj[6] = o.a[3];
      } else {
        for (int k = 0; k < 7; k++) traj[k] = o.a[k];
      }
      double out[7];
      k_pid_task_ctrl(traj, s.carry, s.qvel, c.gains, m->act_ctrlrange[m->nu - 1][1], out);
      for (int k = 0; k < 6; k++) ctrl[k] = out[k];
      if (m->nu > 6) ctrl[6] = out[6];
    } else if (TASK == UR3E_TASK_MOVE_L) {
      k_move_l_ctrl(m, o.a, s.carry, s.qpos, s.qvel, c.gains, ctrl);
    } else if (TASK == UR3E_TASK_MOVE_J) {
      for (int k = 0; k < 6; k++) {
        double q = s.qpos[k];
        double delta = o.a[k] - q;
        double t = q + delta;
        if (t < m->jnt_range[k][0]) t = m->jnt_range[k][0];
        if (t > m->jnt_range[k][1]) t = m->jnt_range[k][1];
        double er = t - q;
        double uk = c.gains.joint[k] * er + c.gains.joint[6 + k] * (-s.qvel[k]);
        if (uk < m->act_ctrlrange[k][0]) uk = m->act_ctrlrange[k][0];
        if (uk > m->act_ctrlrange[k][1]) uk = m->act_ctrlrange[k][1];
        ctrl[k] = uk;
      }
      if (m->nu > 6) ctrl[6] = o.a[6] * m->act_ctrlrange[m->nu - 1][1];
    } else {
#pragma unroll
      for (int k = 0; k < K_NU; k++)
        if (k < m->nu) ctrl[k] = o.a[k];
    }
#pragma unroll
    for (int k = 0; k < K_NU; k++)
      if (k < m->nu) s.ctrl[k] = ctrl[k];
  }
  SYNC();
  WT(35);
  }
  /* substeps, the bad-qacc retry and the auto-reset all go through ONE w_forward site */
  int sub = sub_begin, retried = 0, resetting = 0;
  int part = half == 2 ? 2 : 0; /* the resumed unit's first forward pass starts at the solver */
  if (half != 2) w_step_pre<NT>(m, s);
  for (;;) {
    /* the model and plan are read-only kernel arguments, so their loads are invariant and LICM
       would hoist every model constant of the forward pass out of this loop, keeping them live
       (and spilled) across the whole substep; passing the pointers through an empty asm makes
       them loop-variant, so each stage loads its constants where it uses them */
    /* the pointers pass through the asm as constant-address-space pointers: laundered as generic
       pointers, the model/plan loads became FLAT loads, which count against lgkmcnt as well as
       vmcnt, so every wait for an LDS result also waited for the model constants in flight; as
       global pointers every uniform constant took a vector load and a VGPR, as constant ones the
       uniform loads are scalar (s_load, 5x fewer global_load in the queue kernel; +0.7 % same-box) */
    const __attribute__((address_space(4))) ur3e_model_t* mg =
        (const __attribute__((address_space(4))) ur3e_model_t*)m;
    const __attribute__((address_space(4))) KPlan* plg = (const __attribute__((address_space(4))) KPlan*)pl;
    asm volatile("" : "+s"(mg), "+s"(plg));
    const ur3e_model_t* mi = (const ur3e_model_t*)mg;
    const KPlan* pli = (const KPlan*)plg;
#define m mi
#define pl pli
    /* the split unit stops in the first forward pass of the last substep */
    const int p = (half == 1 && sub == fs - 1 && !retried && !resetting) ? 1 : part;
    part = 0;
    /* touch sensors: only the env-step's last forward pass (the last substep's, or the auto-reset's)
       reaches the commit */
    w_forward<NT>(m, pl, s, p, W_TOUCH_LAST ? (sub == fs - 1 || resetting) : true);
    if (KS::BAIL && s.ovf) return W_BAIL;
    if (p == 1) return W_HALF;
    if (resetting) {
      w_reset_finish<NT, TK>(m, pl, c, s, o);
      return W_DONE;
    }
    if (!retried && w_step_badacc<NT>(m, s)) {
      retried = 1;
      continue;
    }
    w_step_euler<NT>(m, pl, s);
    retried = 0;
    if (++sub < fs) {
      if (sub >= sub_end) return W_PAUSED;
      w_step_pre<NT>(m, s);
      continue;
    }
    w_make_carry<NT>(m, pl, s, s.carry);
    SYNC();
    WT(25);
    if (!k_is_gym(TASK)) {
      if (tid == 0) {
        o.t += 1; o.ep_len += 1;
        if (c.obs_sites) w_obs_v2(m, s, o.obs);
      }
      SYNC();
      return W_DONE;
    }
    if (tid == 0 && TASK != UR3E_TASK_GYM_V2) {
      /* ur3e-v0 / imitation envs: truncation tests t before the increment (ur3e_env.py:152-163,
         imitation_env_indirect.py:96-101, imitation_env_direct.py:98-103) */
      w_task_obs(m, s, TASK, o.obs);
      double r = -1.0;
      int term = 0;
      if (TASK == UR3E_TASK_GYM_V0) {
        const int sc = w_self_collision(m, s);
        r = k_reward_v0(m, o.obs, o.a, sc, w_table_collision(m, s));
        term = k_termination_v0(m, o.obs, sc);
      }
      const int trunc = c.max_episode_steps > 0 && o.t >= c.max_episode_steps;
      o.t += 1;
      o.ep_return += r;
      o.ep_len += 1;
      o.r = r;
      o.term = term;
      o.trunc = trunc;
    }
    const int cfl = TASK == UR3E_TASK_GYM_V2 ? w_contact_flags<NT>(m, s) : 0;
#if W_EPI_LANES
    constexpr bool EPI_LANES = TK == UR3E_TASK_GYM_V2 && NT == 64;
#else
    constexpr bool EPI_LANES = false;
#endif
    if constexpr (EPI_LANES) {
      w_epilogue_v2_lanes(m, c, s, o, cfl);
    } else if (tid == 0 && TASK == UR3E_TASK_GYM_V2) {
      int t = o.t + 1;
      o.t = t;
      w_obs_v2(m, s, o.obs, cfl);
      double r = k_reward_v2(o.obs, o.a);
      int term = w_termination_v2(m, s, o.obs, cfl);
      int trunc = c.max_episode_steps > 0 ? (t >= c.max_episode_steps) : 0;
      double dx = o.obs[3] - o.obs[6], dy = o.obs[4] - o.obs[7], dz = o.obs[5] - o.obs[8];
      if (sqrt(dx * dx + dy * dy + dz * dz) < 0.05) {
        term = 1;
        r += 50.0;
      }
      o.ep_return += r;
      o.ep_len += 1;
      o.r = r;
      o.term = term;
      o.trunc = trunc;
    }
    SYNC();
    WT(26);
    if ((o.term || o.trunc) && c.auto_reset) {
      for (int k = tid; k < k_obs_dim(TASK); k += NT) o.tobs[k] = o.obs[k];
      if (tid == 0) o.did_reset = 1;
      SYNC();
      w_reset_prep<NT>(m, c, __builtin_amdgcn_readfirstlane(o.e), s, o);
      resetting = 1;
      continue;
    }
    return W_DONE;
#undef m
#undef pl
  }
}

template <int NT, class KS = KSL>
__global__ __launch_bounds__(NT) void w_env_reset(const ur3e_model_t* __restrict__ m, const KPlan* __restrict__ pl,
                                                   KConfig c, KState st, const unsigned char* __restrict__ mask,
                                                   double* __restrict__ obs_out) {
  __shared__ KS s;
  __shared__ WOut o;
  const int e = blockIdx.x;
  if (e >= st.n) return;
  if (mask && !mask[e]) return;
  w_load<NT>(m, c, st, e, s, o);
  SYNC();
  w_reset_env<NT>(m, pl, c, e, s, o);
  w_commit<NT>(m, c, st, e, s, o, obs_out, nullptr, nullptr, nullptr, nullptr, 0);
}

/* one env per workgroup; a compact-tier (KS::BAIL) env that overflows is queued on ovf_list
   for w_env_step_list and writes nothing */
/* waves per SIMD the compact tier is compiled for: 2 caps it at 256 registers (arch + acc), so two envs
   share a SIMD.  The 16 KB working set would let a CU take ten (w_dyn_lds), and -DW_COMPACT_WPE=3 builds
   that (168 registers): measured slower, 7.22 M against 8.06 M env-steps/s, and 7.82 M with the same 168
   registers at eight per CU -- the third wave itself costs more than it hides (profiles/r04_ab) */
#ifndef W_COMPACT_WPE
#define W_COMPACT_WPE 2
#endif
/* the mesh-capable compact tier keeps two waves per SIMD: its GJK (simplex in private memory) does not
   fit 168 registers without spilling most of the forward pass */
#define W_WPE_OF(KS) (KS::MESHES ? 2 : W_COMPACT_WPE)
/* diagnostic build only (-DUR3E_WAVE_TRACE): per env of the last step launch, lane 0's
   s_memrealtime (100 MHz) at start and end, XCC_ID:HW_ID, and did_reset | ncon << 8 | blockIdx << 32 */
#ifdef UR3E_WAVE_TRACE
#define UR3E_WAVE_TRACE_MAX 16384
/* the queue kernel's rows: units at sub * n + e (the split units' second halves at frame_skip * n + e),
   then one row per workgroup from W_TRACE_WG_ROW */
#define W_TRACE_WG_ROW 12288
__device__ unsigned long long ur3e_wave_trace[UR3E_WAVE_TRACE_MAX][4];
/* which lanes store the queue kernel's unit stamps: every lane (same word, same value; default) or
   lane 0 alone (-DUR3E_TRACE_LANE0) */
#ifdef UR3E_TRACE_LANE0
#define W_TRACE_LANES (threadIdx.x == 0)
#else
#define W_TRACE_LANES true
#endif
#endif

/* XCD-aware env order: workgroups are dealt round-robin to the 8 XCDs (blockIdx % 8), so workgroup
   b runs env (b % 8) * (n / 8) + b / 8 -- each XCD steps one contiguous env range and neighbouring
   envs, whose per-env scalars and state rows share cache lines, meet in the same L2 instead of
   eight.  Envs are independent, so the order changes no result. */
KD int k_xcd_env(int b, int n) {
  if (n & 7) return b;
  return (b & 7) * (n >> 3) + (b >> 3);
}

/* a fresh view of the running kernel's arguments as the struct A that mirrors its parameter list: loads
   through it are not merged with earlier ones */
template <class A>
__device__ __forceinline__ const A& w_kargs() {
  const __attribute__((address_space(4))) A* p = (const __attribute__((address_space(4))) A*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return *(const A*)p;
}

/* w_env_step's arguments as they sit in the kernarg segment (see WQArgs): with W_KARG_STEP the kernel reads
   them through the kernarg view where they are used instead of all at entry */
struct WEArgs {
  const ur3e_model_t* m;
  const KPlan* pl;
  KConfig c;
  KState st;
  const double* actions;
  int adim;
  double* obs_out;
  double* rew_out;
  unsigned char* term_out;
  unsigned char* trunc_out;
  double* tobs_out;
  int* ovf_list;
  int* ovf_count;
};
static_assert(offsetof(WEArgs, c) == 16 && offsetof(WEArgs, st) == 16 + sizeof(KConfig) &&
                  offsetof(WEArgs, actions) == offsetof(WEArgs, st) + sizeof(KState),
              "WEArgs must mirror w_env_step's kernarg layout");
#ifndef W_KARG_STEP
#define W_KARG_STEP 1
#endif

template <int NT, class KS, int TK = -1>
__global__ __launch_bounds__(NT, (KS::OVERLAY ? W_WPE_OF(KS) : 1)) void w_env_step(const ur3e_model_t* __restrict__ m, const KPlan* __restrict__ pl,
                                                  KConfig c, KState st, const double* __restrict__ actions, int adim,
                                                  double* __restrict__ obs_out, double* __restrict__ rew_out,
                                                  unsigned char* __restrict__ term_out,
                                                  unsigned char* __restrict__ trunc_out,
                                                  double* __restrict__ tobs_out, int* __restrict__ ovf_list,
                                                  int* __restrict__ ovf_count) {
  KS& s = w_smem<KS>();
  WOut& o = w_wout<KS>();
#if W_KARG_STEP
  const WEArgs& U = w_kargs<WEArgs>();
#define EA(x) U.x
#else
#define EA(x) x
#endif
  if ((int)blockIdx.x >= EA(st).n) return;
  const int e = k_xcd_env((int)blockIdx.x, EA(st).n);
  if (EA(st).route && __builtin_amdgcn_readfirstlane(EA(st).route[e])) return; /* stepped by the grasp tier */
#ifdef UR3E_WAVE_TRACE
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
#endif
  WT_INIT();
  if (w_env_step_body<NT, TK>(EA(m), EA(pl), EA(c), EA(st), e, EA(actions), EA(adim), s, o) == W_BAIL) {
    if (threadIdx.x == 0) {
      /* each env is appended at most once per step and the fallback kernel re-zeroes the counter,
         so the slot is < n; the bound check keeps a corrupted counter from writing out of range */
      const WEArgs& V = w_kargs<WEArgs>();
      const int slot = atomicAdd(W_KARG_STEP ? V.ovf_count : ovf_count, 1);
      if (slot < EA(st).n) (W_KARG_STEP ? V.ovf_list : ovf_list)[slot] = e;
    }
    WT_FLUSH();
    return;
  }
#if W_KARG_STEP
  {
    const WEArgs& V = w_kargs<WEArgs>(); /* a fresh view: the commit's pointers are loaded here, not kept */
    w_commit<NT, TK>(V.m, V.c, V.st, e, s, o, V.obs_out, V.rew_out, V.term_out, V.trunc_out, V.tobs_out, 1);
  }
#else
  w_commit<NT, TK>(m, c, st, e, s, o, obs_out, rew_out, term_out, trunc_out, tobs_out, 1);
#endif
#undef EA
  WT(27);
  WT_FLUSH();
#ifdef UR3E_WAVE_TRACE
  if (threadIdx.x == 0 && e < UR3E_WAVE_TRACE_MAX) {
    ur3e_wave_trace[e][0] = t_start;
    ur3e_wave_trace[e][1] = __builtin_amdgcn_s_memrealtime();
    ur3e_wave_trace[e][2] = ((unsigned long long)(unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |
                            (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4); /* XCC_ID : HW_ID */
    ur3e_wave_trace[e][3] = (unsigned long long)o.did_reset | ((unsigned long long)s.ncon << 8) |
                            ((unsigned long long)blockIdx.x << 32);
  }
#endif
}

/* Queued compact-tier step (gym tasks, frame_skip > 1): a resident pool of workgroups pulls
   (substep, env) units from one device counter -- all envs' substep 0 first, then substep 1, ...
   A unit of substep k > 0 waits for env e's unit k - 1 (flag[e], released after its mid-step state
   is in HBM), resumes from that state, and the last substep runs the epilogue and commits.  Work is
   balanced at substep granularity, so the launch ends about half an env-step after the average
   instead of a whole slow env-step after it (a 4,096-env launch runs 2,048 envs at a time).
   Results are identical to w_env_step: every env runs the same substeps in the same order.
   qctl = {next unit per queue, workgroups done, epoch}: the last workgroup to finish re-zeroes the
   counters and advances the epoch, so the flags of this launch (epoch << 4 | substeps done,
   epoch << 4 | W_FLAG_CLAIMED while substep 0 runs, epoch << 4 | W_FLAG_BAILED once the env went to
   the fallback tiers) never match a later launch's.
   Forward progress.  Each workgroup's first unit is static (its rank in its queue, substep 0 only;
   the counters start past them), so a static unit may belong to a workgroup that is not resident
   yet -- e.g. while another queue launch or the grasp pre-pass holds the slots.  Static units are
   therefore claimed: the owner runs one only after moving its flag from an older epoch to CLAIMED
   (compare-and-swap), and a substep-1 unit that finds its producer static and unclaimed claims it
   the same way and runs substeps 0 and 1 itself.  Every other producer was pulled from a counter
   by a running workgroup, before its consumer, and does not wait on anything that is not also
   running; so every wait ends while only resident workgroups make progress.  The spin stays
   bounded (KConfig.spin_limit polls): a unit that gives up claims the env for the fallback tiers
   (atomic exchange: exactly one appender), which recompute the env-step from the committed state,
   and counts the give-up (queue_stats[0]).
   Split last substep (KConfig.split_from < envs per queue, half_buf set): the launch's last units are
   shortened.  For the envs of a queue from split_from on, the last substep's unit stops where its first
   forward pass reaches the constraint solver and hands the env's whole working set (the dynamic LDS
   block: KS and WOut) to half_buf (flag epoch << 4 | W_FLAG_HALF); a second-half unit, queued after
   every other unit, restores it and finishes the substep.  The units that end the launch are then about
   half a substep long, so the workgroups finish closer together; the hand-off is a copy of the LDS
   bytes, so the results are unchanged. */
#define W_FLAG_HALF 13
/* off: measured 4.3 % slower same-box (8.02-8.03 against 8.39-8.40 M env-steps/s, profiles/r04_ab A/B 8) --
   pulled-ahead units are no longer given to whichever workgroup frees first */
#ifndef W_CLAIM_AHEAD
#define W_CLAIM_AHEAD 0
#endif
/* off by default: measured same-box at 4,096 envs, 0 / 25 / 50 / 100 % split gave 7.95 / 7.65 / 7.86 /
   7.89 M env-steps/s (profiles/r04_e3) -- the hand-off and the second halves' waits on their first halves
   cost more than the shorter tail returns */
#ifndef W_SPLIT_PERCENT
#define W_SPLIT_PERCENT 0
#endif
#define W_FLAG_CLAIMED 14
#define W_FLAG_BAILED 15
#define W_SPIN_LIMIT (1u << 26)
#define W_NQUEUE 8 /* one unit queue per XCD (workgroup b serves queue b % 8: speed only) */
KD int w_flag_poll(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

/* the split unit's hand-off record: the dynamic LDS block (working set, then WOut) in 16-byte words */
template <class KS>
constexpr int w_half_words() { return (int)((w_wout_off<KS>() + sizeof(WOut) + 15) / 16); }
typedef __attribute__((ext_vector_type(4))) unsigned int w_u32x4_t;
/* write-through (sc1) 16-byte stores of the whole block, drained before the caller's flag release (the
   same publish recipe as w_store_mid) */
template <class KS>
WD void w_store_half(double* __restrict__ half_buf, int e) {
  extern __shared__ __align__(16) char w_dyn[];
  constexpr int HW = w_half_words<KS>();
  const int tid = w_lane();
  char* p = (char*)half_buf + (size_t)e * HW * 16;
  __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, HW * 16, 0x00020000);
  const w_u32x4_t* src = (const w_u32x4_t*)w_dyn;
#pragma unroll 4
  for (int i = tid; i < HW; i += 64) __builtin_amdgcn_raw_buffer_store_b128(src[i], rsrc, 16 * i, 0, 16);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
/* sc1 loads of the record back into the dynamic LDS block (after the flag was acquired) */
template <class KS>
WD void w_load_half(const double* __restrict__ half_buf, int e) {
  extern __shared__ __align__(16) char w_dyn[];
  constexpr int HW = w_half_words<KS>();
  const int tid = w_lane();
  const char* p = (const char*)half_buf + (size_t)e * HW * 16;
  __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, HW * 16, 0x00020000);
  w_u32x4_t* dst = (w_u32x4_t*)w_dyn;
#pragma unroll 4
  for (int i = tid; i < HW; i += 64) dst[i] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, 16 * i, 0, 16);
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

/* The queue kernel's arguments as they sit in the kernarg segment (the order and natural alignment of its
   parameter list; checked against the by-value copy at kernel start).  With W_KARG_PTR the kernel reads them
   through __builtin_amdgcn_kernarg_segment_ptr(), laundered through an empty asm at every unit, so each
   field is an s_load where it is used.  Read as by-value parameters, every field of KConfig / KState (560
   bytes) is loaded into SGPRs at kernel entry and kept live across the whole persistent loop: 256 SGPRs
   spilled to VGPR lanes, reloaded by v_readlane at ~800 sites (the unit's state load and commit, the queue
   protocol, the controller's gains). */
struct WQArgs {
  const ur3e_model_t* m;
  const KPlan* pl;
  KConfig c;
  KState st;
  const double* actions;
  int adim;
  double* obs_out;
  double* rew_out;
  unsigned char* term_out;
  unsigned char* trunc_out;
  double* tobs_out;
  int* ovf_list;
  int* ovf_ctl;
  int* qctl;
  int* flags;
  double* mid;
  unsigned long long* qstats;
  double* half_buf;
};
static_assert(offsetof(WQArgs, c) == 16 && offsetof(WQArgs, st) == 16 + sizeof(KConfig) &&
                  offsetof(WQArgs, actions) == offsetof(WQArgs, st) + sizeof(KState),
              "WQArgs must mirror w_env_step_q's kernarg layout");
#ifndef W_KARG_PTR
#define W_KARG_PTR 1
#endif
__device__ __forceinline__ const WQArgs& w_qargs() { return w_kargs<WQArgs>(); }

template <int NT, class KS, int TK = -1>
__global__ __launch_bounds__(NT, W_WPE_OF(KS)) void w_env_step_q(const ur3e_model_t* __restrict__ m,
                                                                  const KPlan* __restrict__ pl, KConfig c, KState st,
                                                                  const double* __restrict__ actions, int adim,
                                                                  double* __restrict__ obs_out,
                                                                  double* __restrict__ rew_out,
                                                                  unsigned char* __restrict__ term_out,
                                                                  unsigned char* __restrict__ trunc_out,
                                                                  double* __restrict__ tobs_out, int* __restrict__ ovf_list,
                                                                  int* ovf_ctl, int* qctl, int* flags,
                                                                  double* __restrict__ mid,
                                                                  unsigned long long* qstats,
                                                                  double* __restrict__ half_buf) {
  KS& s = w_smem<KS>();
  WOut& o = w_wout<KS>();
  __shared__ int s_u, s_epoch, s_flag, s_from;
  const int tid = threadIdx.x;
#if W_KARG_PTR
  /* the parameters are not read by name below (that would load them all at entry): QA(x) reads field x of
     the unit's fresh argument view U (w_qargs) */
#define QA(x) U.x
  const WQArgs& U0 = w_qargs();
  const int n = U0.st.n, fs = U0.c.frame_skip;
  const double* const half_buf_ = U0.half_buf;
  const int split_from_ = U0.c.split_from;
  const unsigned int spin_cfg_ = U0.c.spin_limit;
  int* const qctl_ = U0.qctl;
#else
#define QA(x) x
  const int n = st.n, fs = c.frame_skip;
  const double* const half_buf_ = half_buf;
  const int split_from_ = c.split_from;
  const unsigned int spin_cfg_ = c.spin_limit;
  int* const qctl_ = qctl;
#endif
  /* env partition: XCD-sized queues when n splits evenly, else one queue */
  const int nq = (n & 7) ? 1 : W_NQUEUE;
  const int q = (int)blockIdx.x % nq;
  const int nper = n / nq;
  /* split last substep for the queue's envs [k0, nper): their second halves are queued last */
  const int k0 = (half_buf_ && fs >= 2 && fs <= W_FLAG_HALF - 1 && split_from_ < nper)
                     ? (split_from_ > 0 ? split_from_ : 0) : nper;
  const int nfull = nper * fs;
  const int total = nfull + (nper - k0);
  /* static first units per queue: substep-0 units only */
  const int nstat = min((int)gridDim.x / nq, nper);
  const unsigned int spin_limit = spin_cfg_ ? spin_cfg_ : W_SPIN_LIMIT;
  if (tid == 0) s_epoch = __hip_atomic_load(qctl_ + W_NQUEUE + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  SYNC();
  /* wave-uniform values read from LDS pass through readfirstlane so they live in SGPRs: kept in
     VGPRs across the step they would be spilled (the kernel is at its 256-register budget) */
  const int E = __builtin_amdgcn_readfirstlane(s_epoch);
  const int bailed = (E << 4) | W_FLAG_BAILED;
#ifdef UR3E_WAVE_TRACE
  /* per workgroup (row W_TRACE_WG_ROW + blockIdx): started, exited */
  if (W_TRACE_WG_ROW + (int)blockIdx.x < UR3E_WAVE_TRACE_MAX) ur3e_wave_trace[W_TRACE_WG_ROW + blockIdx.x][0] = __builtin_amdgcn_s_memrealtime();
#endif
  /* the first unit of every workgroup is static (its rank in its queue; the counters start at the
     number of workgroups per queue): 2,048 workgroups contending for eight counters at once cost
     ~10 us of the launch */
  int first = (int)blockIdx.x / nq < nstat;
  /* the next unit, pulled while the current one runs (W_CLAIM_AHEAD, off by default): the pull's round trip overlaps the
     unit's own state loads instead of standing between two units.  Only while the queue is far from its
     end (two workgroup-rounds of units left), so the last units are still taken by whichever workgroup
     frees first.  A unit waits only on units of lower index, and a workgroup's pulled-ahead unit has a
     higher index than the one it runs, so every chain of waits ends at a running unit. */
  const int nslot = (int)gridDim.x / nq;
  int next = -1;
  for (;;) {
#if W_KARG_PTR
    const WQArgs& U = w_qargs();
#endif
    int u;
    const int is_static = first;
    if (first) {
      u = (int)blockIdx.x / nq;
      first = 0;
    } else if (next >= 0) {
      u = next;
      next = -1;
    } else {
      if (tid == 0) s_u = atomicAdd(QA(qctl) + q, 1);
      SYNC();
      u = __builtin_amdgcn_readfirstlane(s_u);
    }
    if (u >= total) break;
    /* kind: 0 = whole substep unit(s), 1 = first half of the last substep, 2 = its second half */
    int sub, loc, kind;
    if (u < nfull) {
      sub = u / nper;
      loc = u - sub * nper;
      kind = (sub == fs - 1 && loc >= k0) ? 1 : 0;
    } else {
      sub = fs;
      loc = k0 + (u - nfull);
      kind = 2;
    }
    const int e0 = q * nper + loc;
    if (QA(st).route && __builtin_amdgcn_readfirstlane(QA(st).route[e0])) continue; /* stepped by the grasp tier */
#ifdef UR3E_WAVE_TRACE
    if (W_TRACE_LANES && sub * n + e0 < UR3E_WAVE_TRACE_MAX) ur3e_wave_trace[sub * n + e0][0] = __builtin_amdgcn_s_memrealtime();
#endif
    int from = sub; /* first substep this unit runs */
    if (is_static) {
      /* claim the static unit; a consumer may have claimed it (and run it) already */
      if (tid == 0) {
        const int f = w_flag_poll(QA(flags) + e0);
        int ok = 0;
        if ((f >> 4) != E && !QA(c).leave_static) {
          int expect = f;
          ok = __hip_atomic_compare_exchange_strong(QA(flags) + e0, &expect, (E << 4) | W_FLAG_CLAIMED, __ATOMIC_RELAXED,
                                                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        s_flag = ok;
      }
      SYNC();
      if (!__builtin_amdgcn_readfirstlane(s_flag)) continue;
    } else if (sub > 0) {
      if (tid == 0) {
        const int want = (E << 4) | (kind == 2 ? W_FLAG_HALF : sub);
        int f = w_flag_poll(QA(flags) + e0);
        int fr = sub;
        /* producer is a static substep-0 unit not claimed yet: claim it and run both substeps */
        if (sub == 1 && u - nper < nstat && (f >> 4) != E) {
          int expect = f;
          if (__hip_atomic_compare_exchange_strong(QA(flags) + e0, &expect, (E << 4) | W_FLAG_CLAIMED, __ATOMIC_RELAXED,
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            fr = 0;
            f = want;
            atomicAdd(QA(qstats) + 1, 1ull);
          } else {
            f = expect; /* claimed (or finished) by its owner meanwhile: wait for it below */
          }
        }
        unsigned int spins = 0;
        while (f != want && f != bailed) {
          if (++spins > spin_limit) {
            const int old = atomicExch(QA(flags) + e0, bailed);
            if (old == want) {
              f = want; /* released while we gave up: keep going (and keep the flag final) */
              atomicExch(QA(flags) + e0, want);
            } else {
              f = bailed;
              if (old != bailed) {
                /* the env goes to the fallback tiers, which recompute its env-step (one appender) */
                atomicAdd(QA(qstats), 1ull);
                const int slot = atomicAdd(QA(ovf_ctl), 1);
                if (slot < n) QA(ovf_list)[slot] = e0;
              }
            }
            break;
          }
          __builtin_amdgcn_s_sleep(2);
          f = w_flag_poll(QA(flags) + e0);
        }
        s_flag = f;
        s_from = fr;
      }
      SYNC();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront"); /* payload loads are sc1: keep them below */
      if (__builtin_amdgcn_readfirstlane(s_flag) == bailed) continue;
      from = __builtin_amdgcn_readfirstlane(s_from);
    }
#ifdef UR3E_WAVE_TRACE
    if (W_TRACE_LANES && sub * n + e0 < UR3E_WAVE_TRACE_MAX) ur3e_wave_trace[sub * n + e0][1] = __builtin_amdgcn_s_memrealtime();
#endif
    if (kind == 2) {
      w_load_half<KS>(QA(half_buf), e0);
      SYNC();
    }
    const bool ahead = W_CLAIM_AHEAD && u + 2 * nslot < total;
    int nxt = 0;
    if (ahead && tid == 0) nxt = atomicAdd(QA(qctl) + q, 1);
    const int r0 = kind == 2 ? w_env_step_body<NT, TK>(QA(m), QA(pl), QA(c), QA(st), e0, QA(actions), QA(adim), s, o, fs - 1, 1 << 30,
                                                        nullptr, 2)
                             : w_env_step_body<NT, TK>(QA(m), QA(pl), QA(c), QA(st), e0, QA(actions), QA(adim), s, o, from,
                                                        kind ? fs : sub + 1, QA(mid), kind);
    const int r = __builtin_amdgcn_readfirstlane(r0);
    const int e = __builtin_amdgcn_readfirstlane(o.e); /* = e0, reloaded from LDS (see WOut::e) */
    if (r == W_BAIL) {
      if (tid == 0) {
        /* the full-capacity tier recomputes the whole env-step from the committed state */
        const int old = (sub + 1 < fs || kind == 1) ? atomicExch(QA(flags) + e, bailed) : 0;
        if (old != bailed) {
          const int slot = atomicAdd(QA(ovf_ctl), 1);
          if (slot < n) QA(ovf_list)[slot] = e;
        }
      }
    } else if (r == W_HALF) {
      w_store_half<KS>(QA(half_buf), e);
      SYNC();
      if (tid == 0) {
        const int old = atomicExch(QA(flags) + e, (E << 4) | W_FLAG_HALF);
        if (old == bailed) atomicExch(QA(flags) + e, bailed); /* a consumer gave up and claimed the env */
      }
    } else if (r == W_PAUSED) {
      w_store_mid<NT>(QA(m), QA(mid), e, s);
      SYNC();
      if (tid == 0) {
        const int old = atomicExch(QA(flags) + e, (E << 4) | (sub + 1));
        if (old == bailed) atomicExch(QA(flags) + e, bailed); /* a consumer gave up and claimed the env */
      }
    } else {
      w_commit<NT, TK>(QA(m), QA(c), QA(st), e, s, o, QA(obs_out), QA(rew_out), QA(term_out), QA(trunc_out), QA(tobs_out), 1);
    }
    if (ahead) {
      if (tid == 0) s_u = nxt;
      SYNC();
      next = __builtin_amdgcn_readfirstlane(s_u);
    }
    SYNC();
#ifdef UR3E_WAVE_TRACE
    /* per unit (sub * n + e): pulled, flag acquired, finished (s_memrealtime), workgroup | XCC << 32 */
    if (W_TRACE_LANES && sub * n + e < UR3E_WAVE_TRACE_MAX) {
      unsigned long long* tr = ur3e_wave_trace[sub * n + e];
      tr[2] = __builtin_amdgcn_s_memrealtime();
      tr[3] = (unsigned long long)blockIdx.x |
              ((unsigned long long)(unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32);
    }
#endif
  }
#ifdef UR3E_WAVE_TRACE
  if (W_TRACE_WG_ROW + (int)blockIdx.x < UR3E_WAVE_TRACE_MAX) ur3e_wave_trace[W_TRACE_WG_ROW + blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
#endif
  if (tid == 0) {
    __threadfence();
    if (atomicAdd(qctl_ + W_NQUEUE, 1) == (int)gridDim.x - 1) {
      for (int k = 0; k < W_NQUEUE; k++) atomicExch(qctl_ + k, k < nq ? nstat : 0);
      atomicExch(qctl_ + W_NQUEUE, 0);
      atomicExch(qctl_ + W_NQUEUE + 1, E >= 0x7ffffff ? 1 : E + 1); /* never 0: zeroed flags are unclaimed */
    }
  }
#undef QA
}

/* a fallback tier over the envs the tier before it queued (grid-stride over the list): the grasp
   tier (KSG_NV, 64 lanes) over the compact tier's list, the full-capacity tier (KSL, 128 lanes) over
   the grasp tier's list.  Each recomputes the whole env-step from the committed state.  A bailing
   tier (KS::BAIL) appends the envs it cannot hold to next_list for the tier after it.
   ovf_ctl = {count, blocks_done}: every workgroup reads the count, then the last workgroup to have
   read it re-zeroes both, so the next step's producer starts from an empty list.  The counters live
   and are reset entirely on the device, so a step captured into a HIP graph replays correctly any
   number of times (no host-side step parity baked into the graph). */
/* w_env_step_list's arguments as they sit in the kernarg segment (see WQArgs): with W_KARG_LIST the
   per-env loop reads them through a fresh kernarg view per env instead of keeping all of KConfig / KState
   in SGPRs across it (265-298 SGPRs spilled to VGPR lanes in the list tiers) */
struct WLArgs {
  const ur3e_model_t* m;
  const KPlan* pl;
  KConfig c;
  KState st;
  const double* actions;
  int adim;
  double* obs_out;
  double* rew_out;
  unsigned char* term_out;
  unsigned char* trunc_out;
  double* tobs_out;
  const int* ovf_list;
  int* ovf_ctl;
  unsigned long long* ovf_total;
  int* next_list;
  int* next_ctl;
  int* pred_list;
  int* pred_ctl;
  unsigned long long* ovf_total2;
  int* predm_list;
  int* predm_ctl;
};
static_assert(offsetof(WLArgs, c) == 16 && offsetof(WLArgs, st) == 16 + sizeof(KConfig) &&
                  offsetof(WLArgs, actions) == offsetof(WLArgs, st) + sizeof(KState),
              "WLArgs must mirror w_env_step_list's kernarg layout");
#ifndef W_KARG_LIST
#define W_KARG_LIST 1
#endif

/* waves per SIMD a list tier is compiled for: two (<= 256 registers) for a 64-lane overlaid layout small
   enough that more than four fit a CU's 160 KB of LDS (the mesh grasp tier, KSG_NV_M), else one */
template <int NT, class KS>
constexpr int w_list_wpe() {
  return (NT == 64 && KS::OVERLAY && sizeof(KS) + sizeof(WOut) <= 32768) ? 2 : 1;
}
template <int NT, class KS>
__global__ __launch_bounds__(NT, (w_list_wpe<NT, KS>())) void w_env_step_list(const ur3e_model_t* __restrict__ m,
                                                          const KPlan* __restrict__ pl, KConfig c, KState st,
                                                          const double* __restrict__ actions, int adim,
                                                          double* __restrict__ obs_out, double* __restrict__ rew_out,
                                                          unsigned char* __restrict__ term_out,
                                                          unsigned char* __restrict__ trunc_out,
                                                          double* __restrict__ tobs_out,
                                                          const int* __restrict__ ovf_list, int* ovf_ctl,
                                                          unsigned long long* __restrict__ ovf_total,
                                                          int* __restrict__ next_list, int* next_ctl,
                                                          int* __restrict__ pred_list, int* pred_ctl,
                                                          unsigned long long* __restrict__ ovf_total2,
                                                          int* __restrict__ predm_list, int* predm_ctl) {
  __shared__ KS s;
  __shared__ WOut o;
  __shared__ int s_cnt, s_cntm;
  if (pred_list && blockIdx.x == 0) {
    /* the last kernel of the step: snapshot the routing hints for the next step and list the routed
       envs for its pre-passes -- hint 1 the mid tier's list (predm, when there is one), hint 2 the grasp
       tier's (the order of a list does not matter: envs are independent) */
    if (threadIdx.x == 0) { s_cnt = 0; s_cntm = 0; }
    SYNC();
    auto put = [&](int e, unsigned int h) {
      if (h == 1u && predm_list) predm_list[atomicAdd(&s_cntm, 1)] = e;
      else pred_list[atomicAdd(&s_cnt, 1)] = e;
    };
    /* 16 envs per thread and load (4,096 envs: two passes of the workgroup instead of 32 dependent
       byte loads per thread) */
    const int n16 = st.n >> 4;
    for (int c = threadIdx.x; c < n16; c += NT) {
      const uint4 h = ((const uint4*)st.hint)[c];
      ((uint4*)st.route)[c] = h;
      if (h.x | h.y | h.z | h.w) {
        const unsigned int w[4] = {h.x, h.y, h.z, h.w};
        for (int k = 0; k < 16; k++) {
          const unsigned int hk = (w[k >> 2] >> (8 * (k & 3))) & 0xffu;
          if (hk) put(16 * c + k, hk);
        }
      }
    }
    for (int e = 16 * n16 + threadIdx.x; e < st.n; e += NT) {
      const unsigned char h = st.hint[e];
      st.route[e] = h;
      if (h) put(e, h);
    }
    SYNC();
    if (threadIdx.x == 0) {
      __hip_atomic_store(pred_ctl, s_cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (predm_ctl) __hip_atomic_store(predm_ctl, s_cntm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (st.routed_host)
        __hip_atomic_store(st.routed_host, s_cnt + s_cntm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    SYNC();
  }
  /* the producer launch has completed, so every workgroup reads the same final count: with an
     empty list (the common case) there is nothing to reset and each workgroup leaves at once,
     without the done-counter atomic (one contended atomic per workgroup costs ~10 us per launch) */
  if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(ovf_ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0)
    return;
  if (threadIdx.x == 0) {
    int cnt = __hip_atomic_load(ovf_ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    cnt = cnt < st.n ? cnt : st.n;
    s_cnt = cnt;
    if (atomicAdd(ovf_ctl + 1, 1) == (int)gridDim.x - 1) { /* every workgroup has read the count */
      atomicExch(ovf_ctl, 0);
      atomicExch(ovf_ctl + 1, 0);
      if (cnt) atomicAdd(ovf_total, (unsigned long long)cnt);
      if (cnt && ovf_total2) atomicAdd(ovf_total2, (unsigned long long)cnt); /* the list came from the compact tier */
    }
  }
  SYNC();
  const int cnt = s_cnt;
  for (int i = blockIdx.x; i < cnt; i += gridDim.x) {
#if W_KARG_LIST
    const WLArgs& U = w_kargs<WLArgs>();
#define LA(x) U.x
#else
#define LA(x) x
#endif
    const int e = LA(ovf_list)[i];
    WT_INIT();
    const int r = w_env_step_body<NT>(LA(m), LA(pl), LA(c), LA(st), e, LA(actions), LA(adim), s, o);
    WT_FLUSH();
    if (r == W_BAIL) {
      if constexpr (KS::BAIL) {
        if (threadIdx.x == 0) {
          const int slot = atomicAdd(LA(next_ctl), 1);
          if (slot < LA(st).n) LA(next_list)[slot] = e;
        }
      }
    } else {
      w_commit<NT>(LA(m), LA(c), LA(st), e, s, o, LA(obs_out), LA(rew_out), LA(term_out), LA(trunc_out), LA(tobs_out), 1);
    }
#undef LA
    SYNC();
  }
}

template <int NT, class KS = KSL>
__global__ __launch_bounds__(NT) void w_env_set_state(const ur3e_model_t* __restrict__ m,
                                                       const KPlan* __restrict__ pl, KConfig c, KState st,
                                                       const double* __restrict__ qpos,
                                                       const double* __restrict__ qvel,
                                                       const double* __restrict__ warm) {
  __shared__ KS s;
  __shared__ WOut o;
  const int e = blockIdx.x, tid = threadIdx.x;
  if (e >= st.n) return;
  w_load<NT>(m, c, st, e, s, o);
  SYNC();
  for (int k = tid; k < m->nq; k += NT) s.qpos[k] = qpos[(size_t)e * m->nq + k];
  for (int k = tid; k < m->nv; k += NT) {
    s.qvel[k] = qvel[(size_t)e * m->nv + k];
    if (warm) s.warm[k] = warm[(size_t)e * m->nv + k];
  }
  for (int k = tid; k < m->nu; k += NT) s.ctrl[k] = 0;
  SYNC();
  w_forward<NT>(m, pl, s);
  w_make_carry<NT>(m, pl, s, s.carry);
  SYNC();
  w_commit<NT>(m, c, st, e, s, o, nullptr, nullptr, nullptr, nullptr, nullptr, 0);
}

/* create(): qpos0 / zero velocities, episode 0; envs are valid after ur3e_batch_reset */
__global__ void k_env_init(const ur3e_model_t* __restrict__ m, KState s) {
  int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= s.n) return;
  for (int k = 0; k < m->nq; k++) s.qpos[SQ(s, k, e)] = m->qpos0[k];
  for (int k = 0; k < m->nv; k++) { s.qvel[SV(s, k, e)] = 0; s.warm[SV(s, k, e)] = 0; }
  for (int k = 0; k < NCARRY; k++) s.carry[SC(s, k, e)] = 0;
  s.t[e] = 0; s.episode[e] = 0; s.ep_len[e] = 0; s.ep_return[e] = 0; s.ncon[e] = 0; s.nwarn[e] = 0;
}

__global__ void k_env_get_state(int nq, int nv, KState s, double* __restrict__ qpos, double* __restrict__ qvel,
                                double* __restrict__ warm) {
  int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= s.n) return;
  if (qpos)
    for (int k = 0; k < nq; k++) qpos[(size_t)e * nq + k] = s.qpos[SQ(s, k, e)];
  if (qvel)
    for (int k = 0; k < nv; k++) qvel[(size_t)e * nv + k] = s.qvel[SV(s, k, e)];
  if (warm)
    for (int k = 0; k < nv; k++) warm[(size_t)e * nv + k] = s.warm[SV(s, k, e)];
}

__global__ void k_env_get_touch(KState s, int ntouch, double* __restrict__ out) {
  int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= s.n) return;
  for (int k = 0; k < ntouch; k++) out[(size_t)e * ntouch + k] = s.touch[(size_t)e * UR3E_MAXTOUCH + k];
}

__global__ void k_env_get_ctrl(KState s, int nu, double* __restrict__ out) {
  int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= s.n) return;
  for (int k = 0; k < nu; k++) out[(size_t)e * nu + k] = s.ctrl[(size_t)e * UR3E_MAXU + k];
}

__global__ void k_env_get_info(KState s, int* ncon, int* ep_len, double* ep_ret, int* nwarn) {
  int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= s.n) return;
  if (ncon) ncon[e] = s.ncon[e];
  if (ep_len) ep_len[e] = s.ep_len[e];
  if (ep_ret) ep_ret[e] = s.ep_return[e];
  if (nwarn) nwarn[e] = s.nwarn[e];
}

/* ================================================================== */
/* host side: C ABI                                                    */
/* ================================================================== */
struct ur3e_batch {
  int device;
  int n;
  int wave_nt; /* 0: lane-per-env kernels (v1); 64/128: workgroup-per-env kernels (v2) */
  int tiered;  /* 1: compact tier (KSS, 64 lanes) + full-capacity fallback over the overflow list */
  int main_tree; /* the model's dof tree equals gen_main_tree.h: use the specialised compact kernel */
  int wide;      /* the scripted pick's compact tier (KSS_NV_W: 10 contacts / 44 rows) */
  int mesh;      /* the mesh-capable tier set (KSS_NV_M / KSG_NV_M / KSL_M): main.xml's tree with convex
                    meshes, or a model beyond K_NG geoms / W_MAXCAND candidate pairs */
  int* d_ovf_list;
  int* d_ovf_ctl; /* {count, blocks_done}: device-resident, reset by w_env_step_list */
  unsigned long long* d_ovf_total; /* [0] env-steps the compact tier handed on, [1] the grasp tier,
                                      [2] routed to the grasp tier (with the mid tier's bails), [3] queue
                                      give-ups, [4] static queue units claimed by their consumer, [5] routed
                                      to the mid tier */
  int grasp;       /* the tiers are compact -> grasp (KSG_NV) -> full capacity (main.xml only) */
  int* h_routed;   /* host-mapped routed-env count of the last route snapshot (KState.routed_host) */
  int g_grid;      /* resident workgroups of the grasp-tier list kernel */
  int* d_ovf2_list; /* envs the grasp tier handed to the full-capacity tier */
  int* d_ovf2_ctl;
  int* d_pred_list; /* envs routed to the grasp tier for the next step (route snapshot) */
  int* d_pred_ctl;
  int midt;          /* the mid tier (KSM_NV / KSM_NV_M) between the compact and the grasp tier */
  int m_grid;        /* resident workgroups of the mid-tier list kernel */
  int* d_predm_list; /* envs routed to the mid tier for the next step (route snapshot); its bails join
                        d_pred_list for the grasp pre-pass after it */
  int* d_predm_ctl;
  hipStream_t side; /* the grasp-tier pre-pass runs here, concurrently with the compact tier */
  hipEvent_t ev_fork, ev_join;
  /* bounded run-ahead (grasp tier on): step k (a multiple of W_AHEAD_EVERY) waits for step k - W_AHEAD to
     finish before it enqueues, so the host-mapped routed count it reads is at most W_AHEAD + W_AHEAD_EVERY
     steps old */
  hipEvent_t ev_ahead[W_AHEAD_NEV];
  long long hstep;      /* steps enqueued outside graph capture */
  long long last_route; /* hstep at which the host last saw a nonzero routed count */
  int queued;      /* compact tier through the substep work queue (w_env_step_q) */
  int q_grid;      /* resident workgroups of w_env_step_q (occupancy x CUs) */
  int* d_qctl;     /* {next unit per queue [W_NQUEUE], workgroups done, epoch} */
  int* d_flags;    /* [n] per-env substep hand-off flags */
  double* d_mid;   /* [n][W_MID] mid-step state */
  double* d_half;  /* [n][w_half_words] the split units' working-set hand-off (queue; null while no split) */
  size_t half_bytes;
  ur3e_model_t host_model;
  ur3e_model_t* d_model;
  KPlan* d_plan;
  KConfig cfg;
  KState st;
  hipEvent_t ev0, ev1;
  int timing; /* record ev0/ev1 around each step (ur3e_batch_set_timing); off by default */
  int timed;
};

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

/* error path shared with the other translation units of the library (ur3e_vecnorm.hip) */
__attribute__((visibility("hidden"))) int ur3e_internal_fail(int code, const char* msg) { return fail(code, msg); }

#define HIPCHK(x)                                                                          \
  do {                                                                                     \
    hipError_t _e = (x);                                                                   \
    if (_e != hipSuccess) return fail(UR3E_EHIP, std::string(#x) + ": " + hipGetErrorString(_e)); \
  } while (0)

extern "C" int ur3e_abi_version(void) { return UR3E_ABI_VERSION; }
extern "C" const char* ur3e_last_error(void) { return g_err.c_str(); }

static int check_model(const ur3e_model_t* m) {
  if (m->version != UR3E_MODEL_VERSION) return fail(UR3E_EMODEL, "model image version mismatch");
  if (m->nq > K_NQ || m->nv > K_NV || m->nbody > K_NB || m->njnt > K_NJ || m->ngeom > K_NG_MESH ||
      m->nsite > K_NS || m->nu > K_NU)
    return fail(UR3E_EMODEL, "model exceeds kernel capacities (K_NQ/K_NV/K_NB/K_NJ/K_NG_MESH/K_NS/K_NU)");
  if (m->ncpair > UR3E_MAXCPAIR) return fail(UR3E_EMODEL, "too many collision candidates");
  return UR3E_OK;
}

static void build_plan(const ur3e_model_t* m, KPlan* pl) {
  memset(pl, 0, sizeof(*pl));
  for (int t = 0; t < m->ntendon; t++)
    for (int k = 0; k < m->ten_num[t]; k++) {
      const int dof = m->ten_dof[t][k], j = m->dof_jntid[dof];
      pl->ten_qadr[t][k] = m->jnt_qposadr[j] + (dof - m->jnt_dofadr[j]);
    }
  for (int a = 0; a < m->nu; a++) {
    const double g = m->act_gear[a];
    for (int v = 0; v < m->nv; v++) {
      double mom = 0;
      if (m->act_trntype[a] == UR3E_TRN_JOINT) {
        mom = (v == m->jnt_dofadr[m->act_trnid[a]]) ? g : 0.0;
      } else {
        const int t = m->act_trnid[a];
        for (int k = 0; k < m->ten_num[t]; k++)
          if (m->ten_dof[t][k] == v) mom = m->ten_coef[t][k] * g; /* same product as the oracle */
      }
      pl->act_moment[a][v] = mom;
    }
  }
  int nl = 0;
  for (int i = 1; i < m->nbody; i++) {
    pl->body_depth[i] = pl->body_depth[m->body_parentid[i]] + 1;
    if (pl->body_depth[i] > nl) nl = pl->body_depth[i];
  }
  pl->nlevel = nl;
  for (int i = 0; i < m->nv; i++) {
    int na = 0;
    unsigned int mask = 0;
    for (int j = m->dof_parentid[i]; j >= 0; j = m->dof_parentid[j]) {
      pl->dof_anc[i][na++] = j;
      mask |= 1u << j;
    }
    pl->dof_nanc[i] = na;
    pl->dof_anc_mask[i] = mask;
  }
  for (int b = 0; b < m->nbody; b++) {
    int dof = -1;
    for (int q = b; q > 0 && dof < 0; q = m->body_parentid[q])
      if (m->body_dofnum[q]) dof = m->body_dofadr[q] + m->body_dofnum[q] - 1;
    unsigned int mask = 0;
    for (int j = dof; j >= 0; j = m->dof_parentid[j]) mask |= 1u << j;
    pl->body_dof_mask[b] = mask;
  }
  for (int b = 0; b < m->nbody; b++) {
    const int jfc = m->body_jntnum[b] ? m->body_jntadr[b] : 0;
    pl->bj_type[b] = m->jnt_type[jfc];
    pl->bj_qadr[b] = m->jnt_qposadr[jfc];
    pl->bj_q0[b] = m->qpos0[pl->bj_qadr[b]];
    for (int c = 0; c < 3; c++) { pl->bj_axis[b][c] = m->jnt_axis[jfc][c]; pl->bj_pos[b][c] = m->jnt_pos[jfc][c]; }
  }
  for (int j = 0; j < m->njnt; j++) pl->jnt_root[j] = m->body_rootid[m->jnt_bodyid[j]];
  for (int v = 0; v < m->nv; v++)
    if (m->dof_frictionloss[v] > 0) pl->floss_dof[pl->nfloss++] = v;
  for (int b = 0; b < m->nbody; b++)
    if (m->body_jntnum[b] > pl->max_jntnum) pl->max_jntnum = m->body_jntnum[b];
  /* fixed row groups: equality constraints, then dof frictionloss (w_make_constraint's order) */
  int ng = 0, nr = 0;
  for (int e = 0; e < m->neq; e++) {
    pl->fix_type[ng] = m->eq_type[e] == UR3E_EQ_CONNECT ? G_CONNECT : G_JOINTEQ;
    pl->fix_id[ng] = e; pl->fix_row[ng] = nr; ng++;
    nr += m->eq_type[e] == UR3E_EQ_CONNECT ? 3 : 1;
  }
  for (int k = 0; k < pl->nfloss; k++) {
    pl->fix_type[ng] = G_FLOSS; pl->fix_id[ng] = pl->floss_dof[k]; pl->fix_row[ng] = nr; ng++; nr++;
  }
  pl->nfixgrp = ng;
  pl->nfixrow = nr;
  /* constraint sources (KPlan.cs_*): the row groups' constants with their index chains resolved; the sums
     are the device's own additions in its order, so the values are bit-identical */
  auto cs_sol = [&](int r, const double* ref, const double* imp) {
    for (int k = 0; k < 2; k++) pl->cs_d[r][k] = ref[k];
    for (int k = 0; k < 5; k++) pl->cs_d[r][2 + k] = imp[k];
  };
  for (int e = 0; e < m->neq; e++) {
    cs_sol(e, m->eq_solref[e], m->eq_solimp[e]);
    if (m->eq_type[e] == UR3E_EQ_CONNECT) {
      const int b1 = m->eq_obj1[e], b2 = m->eq_obj2[e];
      pl->cs_i[e][0] = m->body_rootid[b1]; pl->cs_i[e][1] = m->body_rootid[b2];
      pl->cs_i[e][2] = (int)pl->body_dof_mask[b1]; pl->cs_i[e][3] = (int)pl->body_dof_mask[b2];
      pl->cs_d[e][7] = m->body_invweight0[b1][0] + m->body_invweight0[b2][0];
    } else {
      const int j1 = m->eq_obj1[e], j2 = m->eq_obj2[e];
      const int d1 = m->jnt_dofadr[j1], a1 = m->jnt_qposadr[j1];
      pl->cs_i[e][0] = d1; pl->cs_i[e][2] = a1;
      pl->cs_d[e][9] = m->qpos0[a1];
      double diag = m->dof_invweight0[d1];
      if (j2 >= 0) {
        const int d2 = m->jnt_dofadr[j2], a2 = m->jnt_qposadr[j2];
        pl->cs_i[e][1] = d2; pl->cs_i[e][3] = a2;
        pl->cs_d[e][10] = m->qpos0[a2];
        diag += m->dof_invweight0[d2];
      } else {
        pl->cs_i[e][1] = -1; pl->cs_i[e][3] = 0;
      }
      pl->cs_d[e][7] = diag;
    }
  }
  for (int v = 0; v < m->nv; v++) {
    const int r = W_CS_DOF + v;
    cs_sol(r, m->dof_solref[v], m->dof_solimp[v]);
    pl->cs_d[r][7] = m->dof_invweight0[v];
  }
  for (int j = 0; j < m->njnt; j++) {
    const int r = W_CS_JNT + j;
    cs_sol(r, m->jnt_solref[j], m->jnt_solimp[j]);
    pl->cs_i[r][0] = m->jnt_dofadr[j]; pl->cs_i[r][2] = m->jnt_qposadr[j];
    pl->cs_i[r][1] = m->jnt_limited[j] && (m->jnt_type[j] == UR3E_JNT_HINGE || m->jnt_type[j] == UR3E_JNT_SLIDE);
    pl->cs_d[r][7] = m->dof_invweight0[m->jnt_dofadr[j]];
    pl->cs_d[r][8] = m->jnt_margin[j];
    pl->cs_d[r][9] = m->jnt_range[j][0]; pl->cs_d[r][10] = m->jnt_range[j][1];
  }
  for (int p = 0; p < m->ncpair; p++) {
    const int r = W_CS_PAIR + p;
    const int b1 = m->geom_bodyid[m->cpair_geom1[p]], b2 = m->geom_bodyid[m->cpair_geom2[p]];
    cs_sol(r, m->cpair_solref[p], m->cpair_solimp[p]);
    pl->cs_i[r][0] = m->body_rootid[b1]; pl->cs_i[r][1] = m->body_rootid[b2];
    pl->cs_i[r][2] = (int)pl->body_dof_mask[b1]; pl->cs_i[r][3] = (int)pl->body_dof_mask[b2];
    pl->cs_d[r][7] = m->body_invweight0[b1][0] + m->body_invweight0[b2][0];
    pl->cs_d[r][8] = m->cpair_margin[p] - m->cpair_gap[p];
  }
  for (int p = 0; p < m->ncpair; p++) {
    const int g1 = m->cpair_geom1[p], g2 = m->cpair_geom2[p];
    pl->pr_i[p][0] = g1; pl->pr_i[p][1] = g2; pl->pr_i[p][2] = m->geom_type[g1]; pl->pr_i[p][3] = m->geom_type[g2];
    pl->pr_d[p][0] = m->cpair_margin[p];
    pl->pr_d[p][1] = m->geom_rbound[g1]; pl->pr_d[p][2] = m->geom_rbound[g2];
    for (int k = 0; k < 3; k++) { pl->pr_d[p][3 + k] = m->geom_size[g1][k]; pl->pr_d[p][6 + k] = m->geom_size[g2][k]; }
  }
  for (int v = 0; v < m->nv; v++) {
    const int j = m->dof_jntid[v];
    const bool spring = m->jnt_stiffness[j] != 0 &&
                        (m->jnt_type[j] == UR3E_JNT_HINGE || m->jnt_type[j] == UR3E_JNT_SLIDE) && m->jnt_dofadr[j] == v;
    pl->pd_i[v][0] = m->dof_bodyid[v];
    pl->pd_i[v][1] = spring ? m->jnt_qposadr[j] : 0;
    pl->pd_d[v][0] = spring ? m->jnt_stiffness[j] : 0.0;
    pl->pd_d[v][1] = spring ? m->qpos_spring[m->jnt_qposadr[j]] : 0.0;
    pl->pd_d[v][2] = m->dof_damping[v];
  }
  for (int a = 0; a < m->nu; a++) {
    pl->pa_i[a][0] = m->act_ctrllimited[a] ? 1 : 0;
    pl->pa_i[a][1] = m->act_biastype[a] == UR3E_BIAS_AFFINE ? 1 : 0;
    pl->pa_i[a][2] = m->act_forcelimited[a] ? 1 : 0;
    pl->pa_i[a][3] = m->act_trntype[a] == UR3E_TRN_JOINT ? m->jnt_qposadr[m->act_trnid[a]] : -1;
    pl->pa_d[a][0] = m->act_ctrlrange[a][0]; pl->pa_d[a][1] = m->act_ctrlrange[a][1];
    pl->pa_d[a][2] = m->act_gainprm[a][0];
    for (int k = 0; k < 3; k++) pl->pa_d[a][3 + k] = m->act_biasprm[a][k];
    pl->pa_d[a][6] = m->act_forcerange[a][0]; pl->pa_d[a][7] = m->act_forcerange[a][1];
    pl->pa_d[a][8] = m->act_gear[a];
  }
  for (int e = 0; e < m->neq; e++) {
    pl->eqc_i[e][0] = m->eq_type[e] == UR3E_EQ_CONNECT ? 1 : 0;
    pl->eqc_i[e][1] = m->eq_obj1[e]; pl->eqc_i[e][2] = m->eq_obj2[e];
  }
  for (int f = 0; f < m->ngeom + m->nsite; f++) {
    const bool geom = f < m->ngeom;
    const int q = geom ? f : f - m->ngeom;
    pl->fr_b[f] = geom ? m->geom_bodyid[q] : m->site_bodyid[q];
    for (int c = 0; c < 3; c++) pl->fr_d[f][c] = geom ? m->geom_pos[q][c] : m->site_pos[q][c];
    for (int c = 0; c < 4; c++) pl->fr_d[f][3 + c] = geom ? m->geom_quat[q][c] : m->site_quat[q][c];
  }
  /* the Newton direction's element slots (r_direction's mapping, dense and block-diagonal) */
  for (int bdm = 0; bdm < 2; bdm++) {
    const int nv = m->nv, S = bdm ? UR3E_MAIN_SPLIT : 0;
    const bool bd = S > 0;
    const int nel = nv * (nv + 1) / 2, nel1 = S * (S + 1) / 2;
    const int nelb = bd ? nel1 + (nv - S) * (nv - S + 1) / 2 : nel;
    for (int lane = 0; lane < 64; lane++)
      for (int q = 0; q < W_HB_NQ; q++) {
        const int e = lane + 64 * q;
        const bool ev = e < nelb;
        const bool b2 = bd && e >= nel1;
        const int t = ev ? (b2 ? e - nel1 : e) : 0;
        int a = 0;
        while ((a + 1) * (a + 2) / 2 <= t) a++;
        const int off = b2 ? S : 0;
        const int k = off + a, c = off + t - a * (a + 1) / 2;
        /* an invalid slot aliases the lane's slot 0 element (r_direction stores slot 0 last) */
        const int ep0 = q > 0 ? (pl->hb_map[bdm][lane][0] >> 16) & 0xff : 0;
        const int ek = ev ? k : 0, ec = ev ? c : 0, ep = ev ? KTRI(k, c) : ep0;
        pl->hb_map[bdm][lane][q] = ek | (ec << 8) | (ep << 16) | ((ev ? 1 : 0) << 24);
      }
  }
  const int vsite[2] = {m->id_site_tcp, m->id_site_handle};
  for (int k = 0; k < 2; k++) {
    pl->sv_body[k] = vsite[k] >= 0 ? m->site_bodyid[vsite[k]] : -1;
    pl->sv_root[k] = vsite[k] >= 0 ? m->body_rootid[pl->sv_body[k]] : -1;
  }
}

extern "C" int ur3e_batch_create(const ur3e_model_t* model, const ur3e_config_t* cfg, int n_envs, int device,
                                 ur3e_batch_t** out) {
  if (!model || !cfg || !out || n_envs <= 0) return fail(UR3E_EINVAL, "null argument or n_envs <= 0");
  int rc = check_model(model);
  if (rc) return rc;
  if (cfg->task < 0 || cfg->task > UR3E_TASK_MOVE_L) return fail(UR3E_EINVAL, "unknown task");
  const int gym_other = cfg->task >= UR3E_TASK_GYM_V0 && cfg->task <= UR3E_TASK_IMIT_DIRECT;
  if (gym_other && cfg->envs_per_block > 0)
    return fail(UR3E_EINVAL, "ur3e-v0 / imitation tasks need a workgroup-per-env layout (envs_per_block <= 0)");
  if (gym_other && (model->id_site_tcp < 0 || model->id_site_handle < 0 ||
                                        model->id_body_ghost < 0 || model->id_body_fish < 0 ||
                                        model->id_site_rpad < 0))
    return fail(UR3E_EMODEL, "ur3e-v0 / imitation tasks need assets/main.xml");
  if (cfg->task == UR3E_TASK_GYM_V2 && (model->id_site_tcp < 0 || model->id_site_handle < 0 ||
                                        model->id_body_ghost < 0 || model->id_body_fish < 0))
    return fail(UR3E_EMODEL, "gym ur3e-v2 task needs tcp/handle_site/ghost/fish (assets/main.xml)");
  if ((cfg->task == UR3E_TASK_GYM_V2 || cfg->task == UR3E_TASK_TRAJ_L || cfg->task == UR3E_TASK_MOVE_L) &&
      model->id_site_tcp < 0)
    return fail(UR3E_EMODEL, "task-space control needs the tcp site");
  if (cfg->reset_key >= model->nkey) return fail(UR3E_EINVAL, "reset_key out of range");
  if (cfg->envs_per_block > 64) return fail(UR3E_EINVAL, "envs_per_block > 64");
  if (model->nmesh > 0 && cfg->envs_per_block > 0)
    return fail(UR3E_EINVAL, "convex mesh geoms need a workgroup-per-env layout (envs_per_block <= 0)");
  if (model->nmesh > UR3E_MAXMESH || model->nmeshvert > UR3E_MAXMESHVERT)
    return fail(UR3E_EMODEL, "convex meshes exceed the model image capacities");
  /* 0: two-tier (default); -64: full-capacity tier, 64 lanes; other negative: full-capacity tier,
     128 lanes; 1..64: v1 lane-per-env */
  if (cfg->sensors && cfg->envs_per_block > 0)
    return fail(UR3E_EINVAL, "sensors need a workgroup-per-env layout (envs_per_block <= 0)");
  if (cfg->sensors && model->nsensordata > UR3E_MAXSENSORDATA) return fail(UR3E_EMODEL, "too much sensordata");
  /* sensors: the torque sensors need mj_rnePostConstraint's body quantities after the solve, which
     only the full-capacity layout keeps, so a handle with sensors on runs the full-capacity tier */
  int tiered = cfg->envs_per_block == 0 && !cfg->sensors;
  int wave_nt = cfg->envs_per_block == 0 ? 128 : (cfg->envs_per_block == -64 ? 64 : (cfg->envs_per_block < 0 ? 128 : 0));
  KPlan plan;
  build_plan(model, &plan);
  int main_tree = model->nv == UR3E_MAIN_NV && plan.max_jntnum <= 1;
  for (int i = 0; i < model->nv && main_tree; i++)
    if (plan.dof_anc_mask[i] != ur3e_main_dof_anc_mask[i]) main_tree = 0;
  if (model->nbody != UR3E_MAIN_NB) main_tree = 0;
  for (int i = 0; i < model->nbody && main_tree; i++)
    if (model->body_parentid[i] != ur3e_main_body_parent[i] || model->body_dofnum[i] != ur3e_main_body_dofnum[i] ||
        model->body_jntadr[i] != ur3e_main_body_jntadr[i])
      main_tree = 0;
  /* the mesh-capable tier set: main.xml's tree with convex meshes (its compact and grasp tiers settle
     separated mesh pairs themselves), or any model beyond the default geom / candidate capacities (which
     then runs the full-capacity tier only, unless it has main.xml's tree) */
  int has_mesh = 0;
  for (int g = 0; g < model->ngeom; g++) has_mesh |= model->geom_type[g] == UR3E_GEOM_MESH;
  const int mesh = model->ngeom > K_NG || model->ncpair > W_MAXCAND || (main_tree && has_mesh);
  if (mesh) {
    if (model->ncpair > W_MAXCAND_MESH) return fail(UR3E_EMODEL, "too many collision candidates for v2 kernels");
    if (wave_nt == 64 || !wave_nt)
      return fail(UR3E_EINVAL, "this model runs in the mesh-capable layouts: envs_per_block 0 or -128");
    if (!main_tree) tiered = 0; /* the compact tiers are specialised for main.xml's tree */
  } else if (wave_nt && model->ncpair > W_MAXCAND) {
    return fail(UR3E_EMODEL, "too many collision candidates for v2 kernels");
  }
  HIPCHK(hipSetDevice(device));
  ur3e_batch* b = new ur3e_batch();
  b->device = device;
  b->n = n_envs;
  b->wave_nt = wave_nt;
  b->tiered = tiered;
  b->mesh = mesh;
  b->main_tree = main_tree;
  b->host_model = *model;
  b->timed = 0;
  b->timing = 0;
  KConfig& c = b->cfg;
  c.task = cfg->task;
  c.frame_skip = cfg->frame_skip > 0 ? cfg->frame_skip : 1;
  c.max_episode_steps = cfg->max_episode_steps;
  c.auto_reset = cfg->auto_reset;
  c.reset_noise = cfg->reset_noise;
  c.reset_key = cfg->reset_key;
  c.seed = cfg->seed;
  c.env_id_offset = cfg->env_id_offset;
  c.epb = cfg->envs_per_block > 0 && cfg->envs_per_block <= 64 ? cfg->envs_per_block : 16;
  c.tier_con_cap = cfg->tier_con_cap;
  c.np_lanes = cfg->np_chunk_lanes > 0 && cfg->np_chunk_lanes < W_NP_LANES ? cfg->np_chunk_lanes : W_NP_LANES;
  c.obs_sites = model->id_site_tcp >= 0 && model->id_site_handle >= 0 && model->id_body_ghost >= 0;
  c.sensors = cfg->sensors != 0;
  c.spin_limit = 0;
  c.leave_static = 0;
  c.split_from = 1 << 30;
  {
    const double rv[3] = {-1.209, -1.209, 1.209};
    k_quat_from_rotvec(rv, c.gym_qd);
  }
  /* the scripted pick (TRAJ_L) on main.xml runs the wider compact tier (KSS_NV_W; with meshes KSS_NV_MW) */
  b->wide = tiered && main_tree && cfg->task == UR3E_TASK_TRAJ_L;
  c.route_ncon = b->wide ? W_WIDE_MAXCON - 2 : W_SMALL_MAXCON - 1;
  c.route_nefc = b->wide ? W_WIDE_MAXEFC - 8 : W_SMALL_MAXEFC - 3;
  /* routed envs whose last forward fits the mid tier run there (no margin below its capacity: the states
     it serves -- a closed grasp, the carry -- hold their contact set from step to step; one that outgrows it
     bails to the grasp tier); set below once the handle's tiers are known */
  c.route2_ncon = -1;
  c.route2_nefc = -1;
  for (int k = 0; k < 12; k++) {
    c.gains.task[k] = cfg->task_gains[k];
    c.gains.joint[k] = cfg->joint_gains[k];
    c.gains.rot[k] = cfg->rot_joint_gains[k];
  }
  KState& s = b->st;
  s.n = n_envs;
  if (wave_nt) {
    s.fs = 1; s.es_q = model->nq; s.es_v = model->nv; s.es_c = NCARRY;
  } else {
    s.fs = n_envs; s.es_q = 1; s.es_v = 1; s.es_c = 1;
  }
  size_t nd = (size_t)n_envs;
  HIPCHK(hipMalloc(&b->d_model, sizeof(ur3e_model_t)));
  HIPCHK(hipMemcpy(b->d_model, model, sizeof(ur3e_model_t), hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&b->d_plan, sizeof(KPlan)));
  HIPCHK(hipMemcpy(b->d_plan, &plan, sizeof(KPlan), hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&s.qpos, sizeof(double) * nd * model->nq));
  HIPCHK(hipMalloc(&s.qvel, sizeof(double) * nd * model->nv));
  HIPCHK(hipMalloc(&s.warm, sizeof(double) * nd * model->nv));
  HIPCHK(hipMalloc(&s.carry, sizeof(double) * nd * NCARRY));
  HIPCHK(hipMalloc(&s.t, sizeof(int) * nd));
  HIPCHK(hipMalloc(&s.episode, sizeof(unsigned int) * nd));
  HIPCHK(hipMalloc(&s.ep_len, sizeof(int) * nd));
  HIPCHK(hipMalloc(&s.ep_return, sizeof(double) * nd));
  HIPCHK(hipMalloc(&s.ncon, sizeof(int) * nd));
  HIPCHK(hipMalloc(&s.nwarn, sizeof(int) * nd));
  HIPCHK(hipMalloc(&s.touch, sizeof(double) * nd * UR3E_MAXTOUCH));
  HIPCHK(hipMemset(s.touch, 0, sizeof(double) * nd * UR3E_MAXTOUCH));
  HIPCHK(hipMalloc(&s.ctrl, sizeof(double) * nd * UR3E_MAXU));
  HIPCHK(hipMemset(s.ctrl, 0, sizeof(double) * nd * UR3E_MAXU));
  HIPCHK(hipMalloc(&s.actfrc, sizeof(double) * nd * UR3E_MAXU));
  HIPCHK(hipMemset(s.actfrc, 0, sizeof(double) * nd * UR3E_MAXU));
  s.sensordata = nullptr;
  if (c.sensors) {
    HIPCHK(hipMalloc(&s.sensordata, sizeof(double) * nd * UR3E_MAXSENSORDATA));
    HIPCHK(hipMemset(s.sensordata, 0, sizeof(double) * nd * UR3E_MAXSENSORDATA));
  }
  HIPCHK(hipMemset(s.episode, 0, sizeof(unsigned int) * nd));
  HIPCHK(hipMemset(s.nwarn, 0, sizeof(int) * nd));
  HIPCHK(hipMalloc(&b->d_ovf_list, sizeof(int) * nd));
  HIPCHK(hipMalloc(&b->d_ovf_ctl, 2 * sizeof(int)));
  HIPCHK(hipMalloc(&b->d_ovf_total, W_NTOTAL * sizeof(unsigned long long)));
  HIPCHK(hipMemset(b->d_ovf_ctl, 0, 2 * sizeof(int)));
  /* grasp tier between the compact and the full-capacity tier (main.xml's specialised kernels) */
  b->grasp = tiered && b->main_tree;
  b->d_ovf2_list = nullptr; b->d_ovf2_ctl = nullptr; b->g_grid = 0;
  b->d_pred_list = nullptr; b->d_pred_ctl = nullptr; b->side = nullptr;
  b->midt = 0; b->m_grid = 0; b->d_predm_list = nullptr; b->d_predm_ctl = nullptr;
  s.hint = nullptr; s.route = nullptr; s.routed_host = nullptr; b->h_routed = nullptr;
  b->hstep = 0; b->last_route = -1;
  if (b->grasp) {
    int per_cu = 0, cus = 0;
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per_cu, b->mesh ? (const void*)w_env_step_list<64, KSG_NV_M> : (const void*)w_env_step_list<64, KSG_NV>, 64, 0));
    HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    b->g_grid = per_cu * cus;
    if (b->g_grid < 1) b->g_grid = 1;
    if (b->g_grid > n_envs) b->g_grid = n_envs;
    HIPCHK(hipMalloc(&b->d_ovf2_list, sizeof(int) * nd));
    HIPCHK(hipMalloc(&b->d_ovf2_ctl, 2 * sizeof(int)));
    HIPCHK(hipMemset(b->d_ovf2_ctl, 0, 2 * sizeof(int)));
    HIPCHK(hipMalloc(&b->d_pred_list, sizeof(int) * nd));
    HIPCHK(hipMalloc(&b->d_pred_ctl, 2 * sizeof(int)));
    HIPCHK(hipMemset(b->d_pred_ctl, 0, 2 * sizeof(int)));
    /* the mid tier (a positive diagnostic contact cap keeps the three-tier chain it tests) */
    b->midt = W_MID_TIER && cfg->tier_con_cap <= 0;
    if (b->midt) {
      int mper = 0;
      HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
          &mper, b->mesh ? (const void*)w_env_step_list<64, KSM_NV_M> : (const void*)w_env_step_list<64, KSM_NV>, 64, 0));
      b->m_grid = mper * cus;
      if (b->m_grid < 1) b->m_grid = 1;
      if (b->m_grid > n_envs) b->m_grid = n_envs;
      HIPCHK(hipMalloc(&b->d_predm_list, sizeof(int) * nd));
      HIPCHK(hipMalloc(&b->d_predm_ctl, 2 * sizeof(int)));
      HIPCHK(hipMemset(b->d_predm_ctl, 0, 2 * sizeof(int)));
      b->cfg.route2_ncon = W_MID_MAXCON;
      b->cfg.route2_nefc = W_MID_MAXEFC - 1;
    }
    HIPCHK(hipMalloc(&s.hint, nd));
    HIPCHK(hipMemset(s.hint, 0, nd));
    HIPCHK(hipMalloc(&s.route, nd));
    HIPCHK(hipMemset(s.route, 0, nd));
    HIPCHK(hipHostMalloc((void**)&b->h_routed, sizeof(int), hipHostMallocMapped));
    *(volatile int*)b->h_routed = 0;
    HIPCHK(hipHostGetDevicePointer((void**)&s.routed_host, b->h_routed, 0));
    /* high priority: the routed envs are the long ones, so their workgroups should be dispatched
       before the compact tier's fill the CUs */
    int prio_lo = 0, prio_hi = 0;
    HIPCHK(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
    HIPCHK(hipStreamCreateWithPriority(&b->side, hipStreamNonBlocking, prio_hi));
    HIPCHK(hipEventCreateWithFlags(&b->ev_fork, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&b->ev_join, hipEventDisableTiming));
    for (int k = 0; k < W_AHEAD_NEV; k++) HIPCHK(hipEventCreateWithFlags(&b->ev_ahead[k], hipEventDisableTiming));
  }
  /* substep work queue: gym tasks with several substeps per env-step on main.xml's compact tier
     (cfg->schedule 1 keeps one workgroup per env-step) */
  b->queued = tiered && b->main_tree && k_is_gym(cfg->task) && c.frame_skip > 1 &&
              c.frame_skip < W_FLAG_CLAIMED && cfg->schedule != 1; /* flag codes: substeps done < 14 */
  b->d_qctl = nullptr; b->d_flags = nullptr; b->d_mid = nullptr; b->d_half = nullptr; b->half_bytes = 0; b->q_grid = 0;
  if (b->queued) {
    int per_cu = 0, cus = 0;
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per_cu, b->mesh ? (const void*)w_env_step_q<64, KSS_NV_M, UR3E_TASK_GYM_V2> : (const void*)w_env_step_q<64, KSS_NV>,
        64, b->mesh ? w_dyn_lds<KSS_NV_M>() : w_dyn_lds<KSS_NV>()));
    HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    b->q_grid = per_cu * cus;
    if (b->q_grid < 1) b->q_grid = 1;
  }
  /* with no more envs than resident slots every env starts at once and the queue can only add
     hand-off waits (measured: 2,048 envs 4.5 M vs 4.1 M env-steps/s); above that it balances the
     second round at substep granularity (4,096 envs: 5.35 M -> 5.65 M) */
  if (b->queued && cfg->schedule == 0 && n_envs <= b->q_grid) b->queued = 0;
  if (b->queued) {
    const int units = n_envs * c.frame_skip;
    if (b->q_grid > units) b->q_grid = units;
    /* grid: a multiple of the queue count, so every queue has its share of workgroups */
    if (!(n_envs & 7)) b->q_grid = b->q_grid / W_NQUEUE * W_NQUEUE;
    if (b->q_grid < W_NQUEUE) b->q_grid = (n_envs & 7) ? (b->q_grid < 1 ? 1 : b->q_grid) : W_NQUEUE;
    int qinit[W_NQUEUE + 2] = {0};
    /* each queue's counter starts past the workgroups' static first units (w_env_step_q) */
    const int nq = (n_envs & 7) ? 1 : W_NQUEUE;
    const int nstat = b->q_grid / nq < n_envs / nq ? b->q_grid / nq : n_envs / nq; /* substep-0 units */
    for (int k = 0; k < nq; k++) qinit[k] = nstat;
    qinit[W_NQUEUE + 1] = 1; /* epoch */
    HIPCHK(hipMalloc(&b->d_qctl, sizeof(qinit)));
    HIPCHK(hipMemcpy(b->d_qctl, qinit, sizeof(qinit), hipMemcpyHostToDevice));
    HIPCHK(hipMalloc(&b->d_flags, sizeof(int) * nd));
    HIPCHK(hipMemset(b->d_flags, 0, sizeof(int) * nd));
    HIPCHK(hipMalloc(&b->d_mid, sizeof(double) * nd * W_MID));
    /* the split units' hand-off records (16.5 KB per env) only when a split is on: allocated here for a
       nonzero build default, else by ur3e_batch_set_queue_split (null disables the split in the kernel) */
    b->half_bytes = 16 * (size_t)(b->mesh ? w_half_words<KSS_NV_M>() : w_half_words<KSS_NV>()) * nd;
    if (W_SPLIT_PERCENT > 0) HIPCHK(hipMalloc(&b->d_half, b->half_bytes));
    /* the last W_SPLIT_PERCENT % of each queue's envs run their last substep as two half units (0: none) */
    const int nper = n_envs / nq;
    b->cfg.split_from = nper - nper * W_SPLIT_PERCENT / 100;
  }
  HIPCHK(hipMemset(b->d_ovf_total, 0, W_NTOTAL * sizeof(unsigned long long)));
  HIPCHK(hipEventCreate(&b->ev0));
  HIPCHK(hipEventCreate(&b->ev1));
  /* qpos0 / zero state; like a gymnasium Env, call ur3e_batch_reset before the first step */
  hipLaunchKernelGGL(k_env_init, dim3((n_envs + 255) / 256), dim3(256), 0, 0, b->d_model, s);
  HIPCHK(hipGetLastError());
  HIPCHK(hipDeviceSynchronize());
  *out = b;
  return UR3E_OK;
}

extern "C" int ur3e_batch_destroy(ur3e_batch_t* b) {
  if (!b) return UR3E_OK;
  (void)hipSetDevice(b->device);
  void* bufs[] = {b->d_model, b->d_plan, b->st.qpos, b->st.qvel, b->st.warm, b->st.carry, b->st.t, b->st.episode,
                  b->st.ep_len, b->st.ep_return, b->st.ncon, b->st.nwarn, b->st.touch, b->st.ctrl, b->st.actfrc,
                  b->d_ovf_list, b->d_ovf_ctl,
                  b->d_ovf_total};
  for (void* p : bufs) (void)hipFree(p);
  if (b->st.sensordata) (void)hipFree(b->st.sensordata);
  if (b->d_qctl) (void)hipFree(b->d_qctl);
  if (b->d_ovf2_list) (void)hipFree(b->d_ovf2_list);
  if (b->d_ovf2_ctl) (void)hipFree(b->d_ovf2_ctl);
  if (b->d_pred_list) (void)hipFree(b->d_pred_list);
  if (b->d_pred_ctl) (void)hipFree(b->d_pred_ctl);
  if (b->d_predm_list) (void)hipFree(b->d_predm_list);
  if (b->d_predm_ctl) (void)hipFree(b->d_predm_ctl);
  if (b->st.hint) (void)hipFree(b->st.hint);
  if (b->st.route) (void)hipFree(b->st.route);
  if (b->h_routed) (void)hipHostFree(b->h_routed);
  if (b->side) {
    (void)hipStreamDestroy(b->side);
    (void)hipEventDestroy(b->ev_fork);
    (void)hipEventDestroy(b->ev_join);
    for (int k = 0; k < W_AHEAD_NEV; k++) (void)hipEventDestroy(b->ev_ahead[k]);
  }
  if (b->d_flags) (void)hipFree(b->d_flags);
  if (b->d_mid) (void)hipFree(b->d_mid);
  if (b->d_half) (void)hipFree(b->d_half);
  (void)hipEventDestroy(b->ev0);
  (void)hipEventDestroy(b->ev1);
  delete b;
  return UR3E_OK;
}

static int grid_of(const ur3e_batch* b) { return (b->n + b->cfg.epb - 1) / b->cfg.epb; }

extern "C" int ur3e_batch_reset(ur3e_batch_t* b, const uint8_t* d_mask, double* d_obs, void* stream) {
  if (!b) return fail(UR3E_EINVAL, "null handle");
  HIPCHK(hipSetDevice(b->device));
  if (b->wave_nt == 128 && b->mesh)
    hipLaunchKernelGGL((w_env_reset<128, KSL_M>), dim3(b->n), dim3(128), 0, (hipStream_t)stream, b->d_model, b->d_plan,
                       b->cfg, b->st, d_mask, d_obs);
  else if (b->wave_nt == 128)
    hipLaunchKernelGGL(w_env_reset<128>, dim3(b->n), dim3(128), 0, (hipStream_t)stream, b->d_model, b->d_plan, b->cfg,
                       b->st, d_mask, d_obs);
  else if (b->wave_nt == 64)
    hipLaunchKernelGGL(w_env_reset<64>, dim3(b->n), dim3(64), 0, (hipStream_t)stream, b->d_model, b->d_plan, b->cfg,
                       b->st, d_mask, d_obs);
  else
    hipLaunchKernelGGL(k_env_reset, dim3(grid_of(b)), dim3(64), 0, (hipStream_t)stream, b->d_model, b->cfg, b->st,
                       d_mask, d_obs);
  HIPCHK(hipGetLastError());
  return UR3E_OK;
}

/* the tiered step's launches for one tier set (compact KSC, grasp KSG, full capacity KSF): the grasp
   pre-pass (pre), the compact tier, the grasp tier over the compact tier's bails, the full-capacity tier
   over the grasp tier's (or, without the grasp tier, the compact tier's) */
template <class KSC, class KSG, class KSF, class KSW, class KSM>
static int launch_tiers(ur3e_batch* b, hipStream_t st, const KState& kst, bool pre, const double* d_actions, int adim,
                        double* d_obs, double* d_reward, uint8_t* d_terminated, uint8_t* d_truncated,
                        double* d_terminal_obs) {
  const int task = b->cfg.task;
  /* routing off (no pre-pass): the grasp tier is not launched at all -- the compact tier's rare bails
     go straight to the full-capacity tier, which every env fits, and the step is two launches instead
     of three (an empty grasp-tier launch cost ~1.4 % of the step) */
  /* with routing on as well (W_DIRECT_PRE): the compact tier's bails -- a few per million env-steps once the
     routed envs run ahead of it -- go straight to the full-capacity tier too, and the serial (nearly always
     empty) grasp-tier launch behind the compact one is dropped; the full-capacity list then also takes the
     bails of the side stream's mid / grasp chain, which the step joins before it */
  const bool direct = b->grasp && (!pre || W_DIRECT_PRE) && b->cfg.tier_con_cap <= 0; /* a positive diagnostic
                                                                        cap keeps the grasp tier behind the compact one */
  int* const c_list = direct ? b->d_ovf2_list : b->d_ovf_list;
  int* const c_ctl = direct ? b->d_ovf2_ctl : b->d_ovf_ctl;
  if (pre) {
    /* fork: envs routed by the last step's hints run in the grasp tier on the side stream while
       the compact tier (which skips them) runs here */
    HIPCHK(hipEventRecord(b->ev_fork, st));
    HIPCHK(hipStreamWaitEvent(b->side, b->ev_fork, 0));
    /* the mid tier first: the envs it cannot hold join the grasp tier's list, which runs after it */
    if (b->midt)
      hipLaunchKernelGGL((w_env_step_list<64, KSM>), dim3(b->m_grid), dim3(64), 0, b->side, b->d_model, b->d_plan,
                         b->cfg, b->st, d_actions, adim, d_obs, d_reward, d_terminated, d_truncated, d_terminal_obs,
                         b->d_predm_list, b->d_predm_ctl, b->d_ovf_total + 5, b->d_pred_list, b->d_pred_ctl,
                         nullptr, nullptr, nullptr, nullptr, nullptr);
    hipLaunchKernelGGL((w_env_step_list<64, KSG>), dim3(b->g_grid), dim3(64), 0, b->side, b->d_model, b->d_plan,
                       b->cfg, b->st, d_actions, adim, d_obs, d_reward, d_terminated, d_truncated, d_terminal_obs,
                       b->d_pred_list, b->d_pred_ctl, b->d_ovf_total + 2, b->d_ovf2_list, b->d_ovf2_ctl,
                       nullptr, nullptr, nullptr, nullptr, nullptr);
    HIPCHK(hipEventRecord(b->ev_join, b->side));
  }
  /* main.xml: dof count and tree specialised at compile time; the gym ur3e-v2 and scripted
     move_l_mug tasks also get kernels specialised for their task (the other tasks' controller and
     epilogue code folds away, which keeps the register budget for the task that runs) */
  if constexpr (KSC::MESHES) { /* the mesh-capable set: generic kernels, plus the queue's ur3e-v2 one */
    if (b->queued && task == UR3E_TASK_GYM_V2)
      hipLaunchKernelGGL((w_env_step_q<64, KSC, UR3E_TASK_GYM_V2>), dim3(b->q_grid), dim3(64), w_dyn_lds<KSC>(), st,
                         b->d_model, b->d_plan, b->cfg, kst, d_actions, adim, d_obs, d_reward, d_terminated,
                         d_truncated, d_terminal_obs, c_list, c_ctl, b->d_qctl, b->d_flags,
                         b->d_mid, b->d_ovf_total + 3, b->d_half);
    else if (b->queued)
      hipLaunchKernelGGL((w_env_step_q<64, KSC>), dim3(b->q_grid), dim3(64), w_dyn_lds<KSC>(), st, b->d_model, b->d_plan,
                         b->cfg, kst, d_actions, adim, d_obs, d_reward, d_terminated, d_truncated,
                         d_terminal_obs, c_list, c_ctl, b->d_qctl, b->d_flags, b->d_mid,
                         b->d_ovf_total + 3, b->d_half);
    else if (b->wide)
      hipLaunchKernelGGL((w_env_step<64, KSW, UR3E_TASK_TRAJ_L>), dim3(b->n), dim3(64), w_dyn_lds<KSW>(), st, b->d_model,
                         b->d_plan, b->cfg, kst, d_actions, adim, d_obs, d_reward, d_terminated, d_truncated,
                         d_terminal_obs, c_list, c_ctl);
    else
      hipLaunchKernelGGL((w_env_step<64, KSC>), dim3(b->n), dim3(64), w_dyn_lds<KSC>(), st, b->d_model, b->d_plan, b->cfg,
                         kst, d_actions, adim, d_obs, d_reward, d_terminated, d_truncated, d_terminal_obs,
                         c_list, c_ctl);
  } else if (b->queued) { /* substep work queue (w_env_step_q) */
    if (task == UR3E_TASK_GYM_V2)
      hipLaunchKernelGGL((w_env_step_q<64, KSC, UR3E_TASK_GYM_V2>), dim3(b->q_grid), dim3(64), w_dyn_lds<KSC>(), st,
                         b->d_model, b->d_plan, b->cfg, kst, d_actions, adim, d_obs, d_reward, d_terminated,
                         d_truncated, d_terminal_obs, c_list, c_ctl, b->d_qctl, b->d_flags,
                         b->d_mid, b->d_ovf_total + 3, b->d_half);
    else
      hipLaunchKernelGGL((w_env_step_q<64, KSC>), dim3(b->q_grid), dim3(64), w_dyn_lds<KSC>(), st, b->d_model, b->d_plan,
                         b->cfg, kst, d_actions, adim, d_obs, d_reward, d_terminated, d_truncated,
                         d_terminal_obs, c_list, c_ctl, b->d_qctl, b->d_flags, b->d_mid,
                         b->d_ovf_total + 3, b->d_half);
  } else if (b->main_tree && task == UR3E_TASK_GYM_V2) {
    hipLaunchKernelGGL((w_env_step<64, KSC, UR3E_TASK_GYM_V2>), dim3(b->n), dim3(64), w_dyn_lds<KSC>(), st, b->d_model,
                       b->d_plan, b->cfg, kst, d_actions, adim, d_obs, d_reward, d_terminated, d_truncated,
                       d_terminal_obs, c_list, c_ctl);
  } else if (b->main_tree && task == UR3E_TASK_TRAJ_L) {
    hipLaunchKernelGGL((w_env_step<64, KSW, UR3E_TASK_TRAJ_L>), dim3(b->n), dim3(64), w_dyn_lds<KSW>(), st, b->d_model,
                       b->d_plan, b->cfg, kst, d_actions, adim, d_obs, d_reward, d_terminated, d_truncated,
                       d_terminal_obs, c_list, c_ctl);
  } else if (b->main_tree)
    hipLaunchKernelGGL((w_env_step<64, KSC>), dim3(b->n), dim3(64), w_dyn_lds<KSC>(), st, b->d_model, b->d_plan, b->cfg,
                       kst, d_actions, adim, d_obs, d_reward, d_terminated, d_truncated, d_terminal_obs,
                       c_list, c_ctl);
  else
    hipLaunchKernelGGL((w_env_step<64, KSS>), dim3(b->n), dim3(64), w_dyn_lds<KSS>(), st, b->d_model, b->d_plan, b->cfg, kst,
                       d_actions, adim, d_obs, d_reward, d_terminated, d_truncated, d_terminal_obs, c_list, c_ctl);
  int grid = b->n < W_FULL_GRID ? b->n : W_FULL_GRID;
  if (b->grasp) {
    /* join the pre-pass before anything reads its bails or hints: the grasp tier behind the compact one, or
       (direct) the full-capacity tier, whose list the side stream's chain appends to and whose workgroup 0
       snapshots the hints that chain commits */
    if (pre) HIPCHK(hipStreamWaitEvent(st, b->ev_join, 0));
    if (!direct) {
      /* compact-tier bails -> grasp tier; grasp-tier bails (both passes) -> full-capacity tier */
      hipLaunchKernelGGL((w_env_step_list<64, KSG>), dim3(b->g_grid), dim3(64), 0, st, b->d_model, b->d_plan,
                         b->cfg, b->st, d_actions, adim, d_obs, d_reward, d_terminated, d_truncated, d_terminal_obs,
                         b->d_ovf_list, b->d_ovf_ctl, b->d_ovf_total, b->d_ovf2_list, b->d_ovf2_ctl, nullptr,
                         nullptr, nullptr, nullptr, nullptr);
    }
    /* the full-capacity tier, whose workgroup 0 also snapshots the routing hints for the next step;
       fed by the compact tier directly (routing off), its count is the compact tier's hand-on too */
    hipLaunchKernelGGL((w_env_step_list<128, KSF>), dim3(grid), dim3(128), 0, st, b->d_model, b->d_plan, b->cfg,
                       b->st, d_actions, adim, d_obs, d_reward, d_terminated, d_truncated, d_terminal_obs,
                       b->d_ovf2_list, b->d_ovf2_ctl, b->d_ovf_total + 1, nullptr, nullptr, b->d_pred_list,
                       b->d_pred_ctl, (direct && !pre) ? b->d_ovf_total : nullptr, b->d_predm_list, b->d_predm_ctl);
  } else {
    hipLaunchKernelGGL((w_env_step_list<128, KSF>), dim3(grid), dim3(128), 0, st, b->d_model, b->d_plan, b->cfg,
                       b->st, d_actions, adim, d_obs, d_reward, d_terminated, d_truncated, d_terminal_obs,
                       b->d_ovf_list, b->d_ovf_ctl, b->d_ovf_total, nullptr, nullptr, nullptr, nullptr, nullptr,
                       nullptr, nullptr);
  }
  return UR3E_OK;
}

extern "C" int ur3e_batch_step(ur3e_batch_t* b, const double* d_actions, int adim, double* d_obs, double* d_reward,
                               uint8_t* d_terminated, uint8_t* d_truncated, double* d_terminal_obs, void* stream) {
  if (!b || !d_actions) return fail(UR3E_EINVAL, "null handle or actions");
  const int task = b->cfg.task;
  int need = (task == UR3E_TASK_GYM_V2 || task == UR3E_TASK_GYM_V0 || task == UR3E_TASK_IMIT_INDIRECT) ? 4
             : (task == UR3E_TASK_CTRL || task == UR3E_TASK_IMIT_DIRECT) ? b->host_model.nu : 7;
  if (adim != need) return fail(UR3E_EINVAL, "action dimension mismatch for task (expected " + std::to_string(need) + ")");
  HIPCHK(hipSetDevice(b->device));
  hipStream_t st = (hipStream_t)stream;
  /* the step only enqueues kernels whose control state is on the device, so it may be captured into
     a HIP graph; profiling events are recorded only when requested and never during a capture */
  int record = b->timing;
  if (record) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    HIPCHK(hipStreamIsCapturing(st, &cs));
    record = cs == hipStreamCaptureStatusNone;
  }
  bool capturing = false;
  if (record) HIPCHK(hipEventRecord(b->ev0, st));
  if (b->tiered) {
    /* the grasp-tier pre-pass runs only while routing is in use: the last route snapshot the host can
       see (host-mapped, read without a sync, possibly a step or two old) routed some env, or the step
       is being captured (a graph replays without the host).  Skipped, the compact tier steps every
       env (routing is off for this step: route = null), and the few that exceed it bail straight to the
       full-capacity tier after it -- the same results either way, routing only moves work between tiers. */
    KState kst = b->st;
    bool pre = false;
    if (b->grasp) {
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      HIPCHK(hipStreamIsCapturing(st, &cs));
      capturing = cs != hipStreamCaptureStatusNone;
      if (!capturing) {
        if (b->hstep >= W_AHEAD && b->hstep % W_AHEAD_EVERY == 0)
          HIPCHK(hipEventSynchronize(b->ev_ahead[((b->hstep - W_AHEAD) / W_AHEAD_EVERY) % W_AHEAD_NEV]));
        if (*(volatile int*)b->h_routed > 0) b->last_route = b->hstep;
      }
      /* routing stays on for W_ROUTE_HOLD steps after the last sighting (it comes in bursts: grasps) */
      pre = capturing || (b->last_route >= 0 && b->hstep - b->last_route < W_ROUTE_HOLD);
      if (!pre) kst.route = nullptr;
    }
    const int rc = b->mesh ? launch_tiers<KSS_NV_M, KSG_NV_M, KSL_M, KSS_NV_MW, KSM_NV_M>(b, st, kst, pre, d_actions, adim, d_obs, d_reward,
                                                                      d_terminated, d_truncated, d_terminal_obs)
                           : launch_tiers<KSS_NV, KSG_NV, KSL, KSS_NV_W, KSM_NV>(b, st, kst, pre, d_actions, adim, d_obs, d_reward,
                                                                d_terminated, d_truncated, d_terminal_obs);
    if (rc != UR3E_OK) return rc;
  } else if (b->wave_nt == 128 && b->mesh)
    hipLaunchKernelGGL((w_env_step<128, KSL_M>), dim3(b->n), dim3(128), 0, st, b->d_model, b->d_plan, b->cfg, b->st,
                       d_actions, adim, d_obs, d_reward, d_terminated, d_truncated, d_terminal_obs, b->d_ovf_list,
                       b->d_ovf_ctl);
  else if (b->wave_nt == 128)
    hipLaunchKernelGGL((w_env_step<128, KSL>), dim3(b->n), dim3(128), 0, st, b->d_model, b->d_plan, b->cfg, b->st,
                       d_actions, adim, d_obs, d_reward, d_terminated, d_truncated, d_terminal_obs, b->d_ovf_list,
                       b->d_ovf_ctl);
  else if (b->wave_nt == 64)
    hipLaunchKernelGGL((w_env_step<64, KSL>), dim3(b->n), dim3(64), 0, st, b->d_model, b->d_plan, b->cfg, b->st,
                       d_actions, adim, d_obs, d_reward, d_terminated, d_truncated, d_terminal_obs, b->d_ovf_list,
                       b->d_ovf_ctl);
  else
    hipLaunchKernelGGL(k_env_step, dim3(grid_of(b)), dim3(64), 0, st, b->d_model, b->cfg, b->st, d_actions, adim,
                       d_obs, d_reward, d_terminated, d_truncated, d_terminal_obs);
  HIPCHK(hipGetLastError());
  if (b->tiered && b->grasp && !capturing) {
    if (b->hstep % W_AHEAD_EVERY == 0) HIPCHK(hipEventRecord(b->ev_ahead[(b->hstep / W_AHEAD_EVERY) % W_AHEAD_NEV], st));
    b->hstep++;
  }
  if (record) {
    HIPCHK(hipEventRecord(b->ev1, st));
    b->timed = 1;
  }
  return UR3E_OK;
}

extern "C" int ur3e_batch_set_timing(ur3e_batch_t* b, int on) {
  if (!b) return fail(UR3E_EINVAL, "null handle");
  b->timing = on != 0;
  return UR3E_OK;
}

extern "C" int ur3e_batch_get_state(ur3e_batch_t* b, double* d_qpos, double* d_qvel, double* d_warm, void* stream) {
  if (!b) return fail(UR3E_EINVAL, "null handle");
  HIPCHK(hipSetDevice(b->device));
  hipLaunchKernelGGL(k_env_get_state, dim3((b->n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     b->host_model.nq, b->host_model.nv, b->st, d_qpos, d_qvel, d_warm);
  HIPCHK(hipGetLastError());
  return UR3E_OK;
}

extern "C" int ur3e_batch_set_state(ur3e_batch_t* b, const double* d_qpos, const double* d_qvel,
                                    const double* d_warm, void* stream) {
  if (!b || !d_qpos || !d_qvel) return fail(UR3E_EINVAL, "null handle or state");
  HIPCHK(hipSetDevice(b->device));
  if (b->wave_nt == 128 && b->mesh)
    hipLaunchKernelGGL((w_env_set_state<128, KSL_M>), dim3(b->n), dim3(128), 0, (hipStream_t)stream, b->d_model,
                       b->d_plan, b->cfg, b->st, d_qpos, d_qvel, d_warm);
  else if (b->wave_nt == 128)
    hipLaunchKernelGGL(w_env_set_state<128>, dim3(b->n), dim3(128), 0, (hipStream_t)stream, b->d_model, b->d_plan,
                       b->cfg, b->st, d_qpos, d_qvel, d_warm);
  else if (b->wave_nt == 64)
    hipLaunchKernelGGL(w_env_set_state<64>, dim3(b->n), dim3(64), 0, (hipStream_t)stream, b->d_model, b->d_plan,
                       b->cfg, b->st, d_qpos, d_qvel, d_warm);
  else
    hipLaunchKernelGGL(k_env_set_state, dim3(grid_of(b)), dim3(64), 0, (hipStream_t)stream, b->d_model, b->cfg,
                       b->st, d_qpos, d_qvel, d_warm);
  HIPCHK(hipGetLastError());
  return UR3E_OK;
}

extern "C" int ur3e_batch_get_info(ur3e_batch_t* b, int* d_ncon, int* d_ep_len, double* d_ep_return, int* d_nwarn,
                                   void* stream) {
  if (!b) return fail(UR3E_EINVAL, "null handle");
  HIPCHK(hipSetDevice(b->device));
  hipLaunchKernelGGL(k_env_get_info, dim3((b->n + 255) / 256), dim3(256), 0, (hipStream_t)stream, b->st, d_ncon,
                     d_ep_len, d_ep_return, d_nwarn);
  HIPCHK(hipGetLastError());
  return UR3E_OK;
}


__global__ void k_env_get_carry(KState s, double* __restrict__ out) {
  int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= s.n) return;
  for (int k = 0; k < NCARRY; k++) out[(size_t)e * NCARRY + k] = s.carry[SC(s, k, e)];
}

extern "C" int ur3e_batch_get_carry(ur3e_batch_t* b, double* d_carry, void* stream) {
  if (!b || !d_carry) return fail(UR3E_EINVAL, "null argument");
  HIPCHK(hipSetDevice(b->device));
  hipLaunchKernelGGL(k_env_get_carry, dim3((b->n + 255) / 256), dim3(256), 0, (hipStream_t)stream, b->st, d_carry);
  HIPCHK(hipGetLastError());
  return UR3E_OK;
}

extern "C" int ur3e_batch_get_touch(ur3e_batch_t* b, double* d_touch, void* stream) {
  if (!b || !d_touch) return fail(UR3E_EINVAL, "null argument");
  HIPCHK(hipSetDevice(b->device));
  if (b->host_model.ntouch > 0)
    hipLaunchKernelGGL(k_env_get_touch, dim3((b->n + 255) / 256), dim3(256), 0, (hipStream_t)stream, b->st,
                       b->host_model.ntouch, d_touch);
  HIPCHK(hipGetLastError());
  return UR3E_OK;
}

extern "C" int ur3e_batch_get_ctrl(ur3e_batch_t* b, double* d_ctrl, void* stream) {
  if (!b || !d_ctrl) return fail(UR3E_EINVAL, "null argument");
  HIPCHK(hipSetDevice(b->device));
  hipLaunchKernelGGL(k_env_get_ctrl, dim3((b->n + 255) / 256), dim3(256), 0, (hipStream_t)stream, b->st,
                     b->host_model.nu, d_ctrl);
  HIPCHK(hipGetLastError());
  return UR3E_OK;
}

/* controller/controller_func.py:191-200 get_task_space_state after mj_step: tcp site_xpos, tcp rotvec
   (scipy from_matrix(site_xmat).as_rotvec(), utils/utils.py:158-162) and get_boolean_grasp_contact
   ((left pad touch, right pad touch) > (0.1, 0.1) lexicographically, utils/utils.py:238-245), all of
   the step's last forward: the carry's tcp pose and the committed touch sensors */
__global__ void k_env_task_space_state(KState s, int tl, int tr, double* __restrict__ out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= s.n) return;
  double xm[9], q[4], rv[3];
  double* o = out + (size_t)e * 7;
  for (int k = 0; k < 3; k++) o[k] = s.carry[SC(s, k, e)];
  for (int k = 0; k < 9; k++) xm[k] = s.carry[SC(s, 3 + k, e)];
  k_quat_from_matrix(xm, q);
  k_rotvec_from_quat(q, rv);
  for (int k = 0; k < 3; k++) o[3 + k] = rv[k];
  const double l = s.touch[(size_t)e * UR3E_MAXTOUCH + tl], r = s.touch[(size_t)e * UR3E_MAXTOUCH + tr];
  o[6] = (l > 0.1 || (l == 0.1 && r > 0.1)) ? 1.0 : 0.0;
}

__global__ void k_env_get_actfrc(KState s, int nu, double* __restrict__ out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= s.n) return;
  for (int k = 0; k < nu; k++) out[(size_t)e * nu + k] = s.actfrc[(size_t)e * UR3E_MAXU + k];
}

/* the touch sensor (column of d_touch) whose site is on body `body`, or -1 */
static int touch_of_body(const ur3e_model_t* m, int body) {
  if (body < 0) return -1;
  for (int k = 0; k < m->ntouch; k++)
    if (m->site_bodyid[m->touch_site[k]] == body) return k;
  return -1;
}

extern "C" int ur3e_batch_get_task_space_state(ur3e_batch_t* b, double* d_out, void* stream) {
  if (!b || !d_out) return fail(UR3E_EINVAL, "null argument");
  const ur3e_model_t* m = &b->host_model;
  const int tl = touch_of_body(m, m->id_body_lpad), tr = touch_of_body(m, m->id_body_rpad);
  if (m->id_site_tcp < 0 || tl < 0 || tr < 0)
    return fail(UR3E_EMODEL, "task-space state needs the tcp site and the pad touch sensors (assets/main.xml)");
  HIPCHK(hipSetDevice(b->device));
  hipLaunchKernelGGL(k_env_task_space_state, dim3((b->n + 255) / 256), dim3(256), 0, (hipStream_t)stream, b->st,
                     tl, tr, d_out);
  HIPCHK(hipGetLastError());
  return UR3E_OK;
}

extern "C" int ur3e_batch_get_actuator_force(ur3e_batch_t* b, double* d_out, void* stream) {
  if (!b || !d_out) return fail(UR3E_EINVAL, "null argument");
  if (!b->tiered && !b->wave_nt) return fail(UR3E_EINVAL, "the v1 lane-per-env layout does not keep actuator forces");
  HIPCHK(hipSetDevice(b->device));
  hipLaunchKernelGGL(k_env_get_actfrc, dim3((b->n + 255) / 256), dim3(256), 0, (hipStream_t)stream, b->st,
                     b->host_model.nu, d_out);
  HIPCHK(hipGetLastError());
  return UR3E_OK;
}

__global__ void k_env_get_sensordata(KState s, int nsd, double* __restrict__ out) {
  int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= s.n) return;
  for (int k = 0; k < nsd; k++) out[(size_t)e * nsd + k] = s.sensordata[(size_t)e * UR3E_MAXSENSORDATA + k];
}

extern "C" int ur3e_batch_get_sensordata(ur3e_batch_t* b, double* d_sensordata, void* stream) {
  if (!b || !d_sensordata) return fail(UR3E_EINVAL, "null argument");
  if (!b->cfg.sensors) return fail(UR3E_EINVAL, "sensors are off (ur3e_config_t.sensors = 0)");
  HIPCHK(hipSetDevice(b->device));
  if (b->host_model.nsensordata > 0)
    hipLaunchKernelGGL(k_env_get_sensordata, dim3((b->n + 255) / 256), dim3(256), 0, (hipStream_t)stream, b->st,
                       b->host_model.nsensordata, d_sensordata);
  HIPCHK(hipGetLastError());
  return UR3E_OK;
}

/* The kernel a handle launches for one tier, picked by the same branches as launch_tiers and
   ur3e_batch_step (tier 0: the dominant step kernel -- the compact tier, or the only kernel of an
   untiered layout; 1: the grasp tier; 2: the full-capacity fallback tier).  fn = null: the handle has
   no such tier. */
struct KSel {
  const void* fn;
  int nt;
  size_t dyn; /* dynamic LDS bytes (the compact tiers' working set, w_dyn_lds) */
  const char* name;
};
#define K_SEL(F, NT, DYN, NAME) KSel{(const void*)(F), (NT), (size_t)(DYN), NAME}
static KSel step_kernel_sel(const ur3e_batch* b, int tier) {
  const int task = b->cfg.task;
  if (!b->tiered) {
    if (tier != 0) return KSel{nullptr, 0, 0, ""};
    if (b->wave_nt == 128 && b->mesh) return K_SEL((w_env_step<128, KSL_M>), 128, 0, "w_env_step<128,KSL_M> (full-capacity tier)");
    if (b->wave_nt == 128) return K_SEL((w_env_step<128, KSL>), 128, 0, "w_env_step<128,KSL> (full-capacity tier)");
    if (b->wave_nt == 64) return K_SEL((w_env_step<64, KSL>), 64, 0, "w_env_step<64,KSL> (full-capacity tier)");
    return K_SEL(k_env_step, 64, 0, "k_env_step (one env per lane)");
  }
  if (tier == 1) {
    if (!b->grasp) return KSel{nullptr, 0, 0, ""};
    return b->mesh ? K_SEL((w_env_step_list<64, KSG_NV_M>), 64, 0, "w_env_step_list<64,KSG_NV_M> (grasp tier)")
                   : K_SEL((w_env_step_list<64, KSG_NV>), 64, 0, "w_env_step_list<64,KSG_NV> (grasp tier)");
  }
  if (tier == 3) {
    if (!b->midt) return KSel{nullptr, 0, 0, ""};
    return b->mesh ? K_SEL((w_env_step_list<64, KSM_NV_M>), 64, 0, "w_env_step_list<64,KSM_NV_M> (mid tier)")
                   : K_SEL((w_env_step_list<64, KSM_NV>), 64, 0, "w_env_step_list<64,KSM_NV> (mid tier)");
  }
  if (tier == 2) {
    if (b->mesh) return K_SEL((w_env_step_list<128, KSL_M>), 128, 0, "w_env_step_list<128,KSL_M> (full-capacity tier)");
    return K_SEL((w_env_step_list<128, KSL>), 128, 0, "w_env_step_list<128,KSL> (full-capacity tier)");
  }
  if (b->mesh) {
    if (b->queued && task == UR3E_TASK_GYM_V2)
      return K_SEL((w_env_step_q<64, KSS_NV_M, UR3E_TASK_GYM_V2>), 64, w_dyn_lds<KSS_NV_M>(),
                   "w_env_step_q<64,KSS_NV_M,GYM_V2> (compact tier, substep work queue)");
    if (b->queued)
      return K_SEL((w_env_step_q<64, KSS_NV_M>), 64, w_dyn_lds<KSS_NV_M>(),
                   "w_env_step_q<64,KSS_NV_M> (compact tier, substep work queue)");
    if (b->wide)
      return K_SEL((w_env_step<64, KSS_NV_MW, UR3E_TASK_TRAJ_L>), 64, w_dyn_lds<KSS_NV_MW>(),
                   "w_env_step<64,KSS_NV_MW,TRAJ_L> (wide compact tier, one workgroup per env-step)");
    return K_SEL((w_env_step<64, KSS_NV_M>), 64, w_dyn_lds<KSS_NV_M>(),
                 "w_env_step<64,KSS_NV_M> (compact tier, one workgroup per env-step)");
  }
  if (b->queued && task == UR3E_TASK_GYM_V2)
    return K_SEL((w_env_step_q<64, KSS_NV, UR3E_TASK_GYM_V2>), 64, w_dyn_lds<KSS_NV>(),
                 "w_env_step_q<64,KSS_NV,GYM_V2> (compact tier, substep work queue)");
  if (b->queued)
    return K_SEL((w_env_step_q<64, KSS_NV>), 64, w_dyn_lds<KSS_NV>(),
                 "w_env_step_q<64,KSS_NV> (compact tier, substep work queue)");
  if (b->main_tree && task == UR3E_TASK_GYM_V2)
    return K_SEL((w_env_step<64, KSS_NV, UR3E_TASK_GYM_V2>), 64, w_dyn_lds<KSS_NV>(),
                 "w_env_step<64,KSS_NV,GYM_V2> (compact tier, one workgroup per env-step)");
  if (b->main_tree && task == UR3E_TASK_TRAJ_L)
    return K_SEL((w_env_step<64, KSS_NV_W, UR3E_TASK_TRAJ_L>), 64, w_dyn_lds<KSS_NV_W>(),
                 "w_env_step<64,KSS_NV_W,TRAJ_L> (wide compact tier, one workgroup per env-step)");
  if (b->main_tree)
    return K_SEL((w_env_step<64, KSS_NV>), 64, w_dyn_lds<KSS_NV>(),
                 "w_env_step<64,KSS_NV> (compact tier, one workgroup per env-step)");
  return K_SEL((w_env_step<64, KSS>), 64, w_dyn_lds<KSS>(), "w_env_step<64,KSS> (compact tier, one workgroup per env-step)");
}
#undef K_SEL

static void copy_cstr(char* dst, int len, const char* src) {
  if (!dst || len <= 0) return;
  int i = 0;
  for (; src && src[i] && i < len - 1; i++) dst[i] = src[i];
  dst[i] = 0;
}

extern "C" int ur3e_batch_tier_kernel(ur3e_batch_t* b, int tier, int* envs_per_cu, int* lds_bytes, int* regs,
                                      char* name, int name_len, char* symbol, int symbol_len) {
  if (!b) return fail(UR3E_EINVAL, "null handle");
  if (tier < 0 || tier > 3) return fail(UR3E_EINVAL, "tier must be 0 (step), 1 (grasp), 2 (full capacity) or 3 (mid)");
  const KSel k = step_kernel_sel(b, tier);
  if (!k.fn) return fail(UR3E_EINVAL, "the handle launches no kernel for this tier");
  HIPCHK(hipSetDevice(b->device));
  hipFuncAttributes attr;
  HIPCHK(hipFuncGetAttributes(&attr, k.fn));
  int blocks = 0;
  HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k.fn, k.nt, k.dyn));
  const bool lane_per_env = !b->tiered && !b->wave_nt; /* v1: one env per lane */
  if (envs_per_cu) *envs_per_cu = lane_per_env ? blocks * k.nt : blocks;
  if (lds_bytes) *lds_bytes = (int)(attr.sharedSizeBytes + k.dyn);
  if (regs) *regs = attr.numRegs;
  copy_cstr(name, name_len, k.name);
  if (symbol && symbol_len > 0) copy_cstr(symbol, symbol_len, hipKernelNameRefByPtr(k.fn, nullptr));
  return UR3E_OK;
}

/* resources and occupancy of the step kernel this handle launches (the dominant kernel) */
extern "C" int ur3e_batch_kernel_info(ur3e_batch_t* b, int* envs_per_cu, int* lds_bytes, int* regs) {
  return ur3e_batch_tier_kernel(b, 0, envs_per_cu, lds_bytes, regs, nullptr, 0, nullptr, 0);
}

/* diagnostics: per-stage cycle totals of the -DUR3E_STAGE_TIMING build (returns -1 otherwise) */
extern "C" int ur3e_debug_stage_cycles_tier(int tier, unsigned long long* cycles, unsigned long long* calls,
                                            int reset) {
#ifdef UR3E_STAGE_TIMING
  if (tier < 0 || tier > 2) return fail(UR3E_EINVAL, "tier must be 0 (compact), 1 (grasp) or 2 (full)");
  HIPCHK(hipDeviceSynchronize());
  unsigned long long c[3][W_NSTAGE_MARKS], k[3][W_NSTAGE_MARKS];
  HIPCHK(hipMemcpyFromSymbol(c, HIP_SYMBOL(ur3e_stage_cycles), sizeof(c)));
  HIPCHK(hipMemcpyFromSymbol(k, HIP_SYMBOL(ur3e_stage_calls), sizeof(k)));
  for (int i = 0; i < W_NSTAGE_MARKS; i++) { cycles[i] = c[tier][i]; calls[i] = k[tier][i]; }
  if (reset) {
    unsigned long long z[3][W_NSTAGE_MARKS] = {{0}};
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(ur3e_stage_cycles), z, sizeof(z)));
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(ur3e_stage_calls), z, sizeof(z)));
  }
  return UR3E_OK;
#else
  (void)tier; (void)cycles; (void)calls; (void)reset;
  return fail(UR3E_EINVAL, "library built without -DUR3E_STAGE_TIMING");
#endif
}

/* diagnostics: per-stage cycle totals of the compact tier (-DUR3E_STAGE_TIMING build) */
extern "C" int ur3e_debug_stage_cycles(unsigned long long* cycles, unsigned long long* calls, int reset) {
  return ur3e_debug_stage_cycles_tier(0, cycles, calls, reset);
}

/* diagnostic: copy the wave trace of the last step launch (UR3E_WAVE_TRACE builds only) */
extern "C" int ur3e_debug_wave_trace(unsigned long long* out, int n) {
#ifdef UR3E_WAVE_TRACE
  if (!out || n < 0 || n > UR3E_WAVE_TRACE_MAX) return fail(UR3E_EINVAL, "bad wave-trace request");
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(ur3e_wave_trace), sizeof(unsigned long long) * 4 * (size_t)n));
  return UR3E_OK;
#else
  (void)out; (void)n;
  return fail(UR3E_EINVAL, "library built without -DUR3E_WAVE_TRACE");
#endif
}

extern "C" int ur3e_batch_overflow_count(ur3e_batch_t* b, unsigned long long* total) {
  if (!b || !total) return fail(UR3E_EINVAL, "null argument");
  HIPCHK(hipSetDevice(b->device));
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(total, b->d_ovf_total, sizeof(unsigned long long), hipMemcpyDeviceToHost));
  return UR3E_OK;
}

extern "C" int ur3e_batch_tier_counts(ur3e_batch_t* b, unsigned long long* counts) {
  if (!b || !counts) return fail(UR3E_EINVAL, "null argument");
  HIPCHK(hipSetDevice(b->device));
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(counts, b->d_ovf_total, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  return UR3E_OK;
}

extern "C" int ur3e_batch_mid_count(ur3e_batch_t* b, unsigned long long* routed) {
  if (!b || !routed) return fail(UR3E_EINVAL, "null argument");
  HIPCHK(hipSetDevice(b->device));
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(routed, b->d_ovf_total + 5, sizeof(unsigned long long), hipMemcpyDeviceToHost));
  return UR3E_OK;
}

extern "C" int ur3e_batch_queue_stats(ur3e_batch_t* b, unsigned long long* stats) {
  if (!b || !stats) return fail(UR3E_EINVAL, "null argument");
  HIPCHK(hipSetDevice(b->device));
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(stats, b->d_ovf_total + 3, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  return UR3E_OK;
}

extern "C" int ur3e_batch_set_queue_debug(ur3e_batch_t* b, unsigned int spin_limit, int leave_static_units) {
  if (!b) return fail(UR3E_EINVAL, "null handle");
  b->cfg.spin_limit = spin_limit;
  b->cfg.leave_static = leave_static_units != 0;
  return UR3E_OK;
}

extern "C" int ur3e_batch_set_queue_split(ur3e_batch_t* b, int percent) {
  if (!b) return fail(UR3E_EINVAL, "null handle");
  if (percent < 0 || percent > 100) return fail(UR3E_EINVAL, "split percent outside [0, 100]");
  if (!b->queued) return percent ? fail(UR3E_EINVAL, "the handle does not run the substep work queue") : UR3E_OK;
  if (percent > 0 && !b->d_half) {
    HIPCHK(hipSetDevice(b->device));
    HIPCHK(hipMalloc(&b->d_half, b->half_bytes));
  }
  const int nper = b->n / ((b->n & 7) ? 1 : W_NQUEUE);
  b->cfg.split_from = nper - nper * percent / 100;
  return UR3E_OK;
}

/* Diagnostic for the queue's forward-progress test: workgroups that each hold 64 KB of LDS (two per CU
   fill 128 of the 160 KB, leaving room for one step workgroup) for hold_us microseconds of the constant
   100 MHz clock from their own start, then exit -- every wave reaches the exit.  Each sets its flag in
   host-mapped memory when it starts, so the host can wait until they are all resident before it
   launches the queue on another stream. */
#define W_HOLD_LDS_DOUBLES 8192
__global__ __launch_bounds__(64) void w_hold_slots(unsigned int* started, unsigned long long ticks, double* sink) {
  __shared__ double buf[W_HOLD_LDS_DOUBLES];
  const int l = threadIdx.x;
  for (int i = l; i < W_HOLD_LDS_DOUBLES; i += 64) buf[i] = (double)i;
  __syncthreads();
  /* a plain store per workgroup into host-mapped memory (no PCIe atomics needed) */
  if (l == 0) __hip_atomic_store(started + blockIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const unsigned long long t0 = wall_clock64();
  double acc = 0.0;
  int k = l;
  while (wall_clock64() - t0 < ticks) {
    acc += buf[k];
    k = (k + 64) & (W_HOLD_LDS_DOUBLES - 1);
    __builtin_amdgcn_s_sleep(8);
  }
  if (acc == -1.0) sink[l] = acc; /* never true: keeps the LDS reads */
}

extern "C" int ur3e_debug_hold_slots(int device, int workgroups, int hold_us, void* stream, int* started) {
  if (workgroups <= 0 || workgroups > 4096 || hold_us <= 0 || hold_us > 1000000)
    return fail(UR3E_EINVAL, "workgroups in [1, 4096], hold_us in [1, 1e6]");
  HIPCHK(hipSetDevice(device));
  /* one host-mapped counter and sink per process, kept for its lifetime: the call returns while the
     workgroups still hold their slots.  The counter is re-zeroed only after every workgroup of the
     previous call had started (they count only at their start). */
  static unsigned int* cnt = nullptr; /* one start flag per workgroup */
  static unsigned int* dcnt = nullptr;
  static double* sink = nullptr;
  if (!cnt) {
    HIPCHK(hipHostMalloc((void**)&cnt, 4096 * sizeof(unsigned int), hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(hipHostGetDevicePointer((void**)&dcnt, cnt, 0));
    HIPCHK(hipMalloc((void**)&sink, 64 * sizeof(double)));
  }
  for (int i = 0; i < workgroups; i++) ((volatile unsigned int*)cnt)[i] = 0;
  const unsigned long long ticks = 100ull * (unsigned long long)hold_us; /* wall_clock64: 100 MHz */
  hipLaunchKernelGGL(w_hold_slots, dim3(workgroups), dim3(64), 0, (hipStream_t)stream, dcnt, ticks, sink);
  HIPCHK(hipGetLastError());
  /* wait (bounded by twice the hold time) until every workgroup has started, then return: the caller
     launches the work that is to find its slots taken */
  const auto t0 = std::chrono::steady_clock::now();
  int seen = 0;
  for (;;) {
    seen = 0;
    for (int i = 0; i < workgroups; i++) seen += ((volatile unsigned int*)cnt)[i] != 0;
    if (seen >= workgroups || std::chrono::steady_clock::now() - t0 >= std::chrono::microseconds(2 * hold_us)) break;
  }
  if (started) *started = seen;
  return UR3E_OK;
}

extern "C" int ur3e_batch_obs_dim(const ur3e_batch_t* b) { return b ? k_obs_dim(b->cfg.task) : 0; }

/* which step kernel the handle launches: 0 compact tier, one workgroup per env-step (w_env_step);
   1 compact tier as a substep work queue (w_env_step_q); 2 full-capacity tier only; 3 lane per env */
extern "C" int ur3e_batch_schedule(const ur3e_batch_t* b) {
  if (!b) return -1;
  if (b->tiered) return b->queued ? 1 : 0;
  return b->wave_nt ? 2 : 3;
}

extern "C" int ur3e_batch_num_envs(const ur3e_batch_t* b) { return b ? b->n : 0; }
extern "C" int ur3e_batch_nq(const ur3e_batch_t* b) { return b ? b->host_model.nq : 0; }
extern "C" int ur3e_batch_nv(const ur3e_batch_t* b) { return b ? b->host_model.nv : 0; }
extern "C" int ur3e_batch_nu(const ur3e_batch_t* b) { return b ? b->host_model.nu : 0; }

extern "C" int ur3e_batch_last_step_ms(ur3e_batch_t* b, float* ms) {
  if (!b || !ms) return fail(UR3E_EINVAL, "null argument");
  if (!b->timed) return fail(UR3E_EINVAL, "no step recorded (enable with ur3e_batch_set_timing)");
  HIPCHK(hipEventSynchronize(b->ev1));
  HIPCHK(hipEventElapsedTime(ms, b->ev0, b->ev1));
  return UR3E_OK;
}
