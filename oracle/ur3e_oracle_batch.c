/*
 * ur3e_oracle_batch.c — batched drivers over the scalar CPU oracle (TEST
 * INFRASTRUCTURE ONLY).  These restate, env by env, exactly what one
 * ur3e_batch_step() launch of the MI355X library computes, so tests can compare
 * the two on the same inputs, and bench.py can time the oracle on the host
 * cores (OpenMP over envs, static schedule) as the `cpu_baseline`.
 *
 * Semantics per env-step (task ids mirror include/ur3e_batch.h):
 *   task 0 (gym ur3e-v2):  UR3eEnv2.step (gymnasium_env/envs/ur3e_env2.py:72-99)
 *                          + SB3 VecEnv auto-reset on terminated|truncated.
 *   task 1 (traj_l):       pid_task_ctrl on a [7] trajectory row + 1 mj_step
 *                          (controller/move_l_mug.py:67-81).
 *   task 2 (move_j):       pd_joint_ctrl on a [7] joint-target row + 1 mj_step
 *                          (controller/move_j.py:76-86).
 *   task 3 (ctrl):         raw ctrl row [nu] + frame_skip mj_step.
 *   task 7 (move_l):       move_l.ctrl on a [7] trajectory row (pinv joint deltas through two
 *                          pd_joint_ctrl calls) + 1 mj_step (controller/move_l.py:15-31,130-140).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "ur3e_oracle.h"
#ifdef _OPENMP
#include <omp.h>
#endif

/* OpenMP threads of the batch calls (bench.py's cpu_baseline times 1 thread and all threads) */
void ur3o_set_threads(int n) {
#ifdef _OPENMP
  if (n > 0) omp_set_num_threads(n);
#else
  (void)n;
#endif
}

typedef struct {
  int task;
  int frame_skip;
  int max_episode_steps;
  int auto_reset;
  int reset_noise;
  int reset_key;
  double task_gains[12];
  double joint_gains[12];
  unsigned long long seed;
  int env_id_offset;
  int envs_per_block;
  int tier_con_cap;
  double rot_joint_gains[12];
  int np_chunk_lanes; /* GPU-tier diagnostic, unused here (layout mirror of ur3e_config_t) */
  int sensors;        /* the oracle always computes sensordata (layout mirror) */
  int schedule;       /* GPU launch schedule, unused here (layout mirror) */
} ur3o_config;

/* the model has the sites the 24-d observation reads (main.xml) */
static int has_obs_sites(const ur3e_model_t* m) {
  return m->id_site_tcp >= 0 && m->id_site_handle >= 0 && m->id_body_ghost >= 0;
}

/* tasks (include/ur3e_batch.h): 0 gym v2, 1 traj_l, 2 move_j, 3 ctrl, 4 gym v0, 5 imitation
   indirect, 6 imitation direct */
static int is_gym(int task) { return task == 0 || (task >= 4 && task <= 6); }
int ur3o_obs_dim(int task) { return (task == 4 || task == 6) ? 13 : 24; }
static void task_obs(const ur3e_model_t* m, const ur3o_data* d, int task, double* obs) {
  if (task == 4) ur3o_obs_v0(m, d, obs);
  else if (task == 6) ur3o_obs_direct(m, d, obs);
  else ur3o_obs_v2(m, d, obs);
}

static void gains_from_cfg(const ur3o_config* c, ur3o_task_gains* tg, ur3o_joint_gains* jg) {
  for (int k = 0; k < 3; k++) {
    tg->kp_pos[k] = c->task_gains[k];
    tg->kd_pos[k] = c->task_gains[3 + k];
    tg->kp_rot[k] = c->task_gains[6 + k];
    tg->kd_rot[k] = c->task_gains[9 + k];
  }
  for (int k = 0; k < 6; k++) {
    jg->kp[k] = c->joint_gains[k];
    jg->kd[k] = c->joint_gains[6 + k];
  }
}

/* reset one env to the configured keyframe (+ optional "high" mug noise), forward */
static void env_reset(const ur3e_model_t* m, const ur3o_config* c, ur3o_env* e, double* obs) {
  ur3o_data* d = &e->d;
  ur3o_reset_data(m, d);
  int key = c->reset_key;
  if (key >= 0) {
    for (int k = 0; k < m->nq; k++) d->qpos[k] = m->key_qpos[key][k];
    for (int k = 0; k < m->nv; k++) d->qvel[k] = m->key_qvel[key][k];
  }
  if (c->reset_noise && m->id_body_fish >= 0) {
    double u0 = ur3o_uniform01(e->seed, e->env_id, e->episode, 0);
    double u1 = ur3o_uniform01(e->seed, e->env_id, e->episode, 1);
    /* gym_utils.get_mug_xpos_noise: 1 "high", 2 "med", 3 "low" */
    double ylo = -0.25, yhi = 0.2;
    if (c->reset_noise == 2) { ylo = -0.2; yhi = 0.1; }
    else if (c->reset_noise == 3) { ylo = -0.1; yhi = 0.01; }
    d->qpos[14] += 0.0 + (0.02 - 0.0) * u0;
    d->qpos[15] += ylo + (yhi - ylo) * u1;
  }
  ur3o_forward(m, d);
  e->t = 0;
  e->ep_return = 0;
  e->ep_len = 0;
  e->episode++;
  if (obs && (is_gym(c->task) || has_obs_sites(m))) task_obs(m, d, c->task, obs);
}

/* envs: array of n ur3o_env (opaque to python: allocate n*ur3o_sizeof_env()) */
void ur3o_batch_init(const ur3e_model_t* m, const ur3o_config* c, int n, ur3o_env* envs, double* obs) {
#pragma omp parallel for schedule(static)
  for (int i = 0; i < n; i++) {
    ur3o_env_init(m, &envs[i], c->seed, (unsigned int)(c->env_id_offset + i));
    env_reset(m, c, &envs[i], obs ? obs + (size_t)ur3o_obs_dim(c->task) * i : 0);
  }
}

void ur3o_batch_reset_one(const ur3e_model_t* m, const ur3o_config* c, ur3o_env* e, double* obs) {
  env_reset(m, c, e, obs);
}

/* one env-step for all envs.  actions: [n][adim].  Outputs may be NULL. */
void ur3o_batch_step(const ur3e_model_t* m, const ur3o_config* c, int n, ur3o_env* envs, const double* actions,
                     int adim, double* obs, double* reward, unsigned char* terminated, unsigned char* truncated,
                     double* terminal_obs) {
  ur3o_task_gains tg;
  ur3o_joint_gains jg;
  gains_from_cfg(c, &tg, &jg);
  ur3o_joint_gains rg;
  for (int k = 0; k < 6; k++) {
    rg.kp[k] = c->rot_joint_gains[k];
    rg.kd[k] = c->rot_joint_gains[6 + k];
  }
#pragma omp parallel for schedule(static)
  for (int i = 0; i < n; i++) {
    ur3o_env* e = &envs[i];
    ur3o_data* d = &e->d;
    const double* a = actions + (size_t)adim * i;
    double ctrl[UR3E_MAXU];
    const int od = ur3o_obs_dim(c->task);
    if (c->task == 0) {
      double o[24], r;
      int term, trunc;
      ur3o_env_step_v2(m, e, &tg, a, c->frame_skip, o, &r, &term, &trunc);
      if (c->max_episode_steps <= 0) trunc = 0;
      else trunc = e->t >= c->max_episode_steps;
      if (reward) reward[i] = r;
      if (terminated) terminated[i] = (unsigned char)term;
      if (truncated) truncated[i] = (unsigned char)trunc;
      if ((term || trunc) && c->auto_reset) {
        if (terminal_obs) memcpy(terminal_obs + 24 * (size_t)i, o, sizeof(o));
        env_reset(m, c, e, obs ? obs + 24 * (size_t)i : 0);
      } else if (obs) {
        memcpy(obs + 24 * (size_t)i, o, sizeof(o));
      }
      continue;
    }
    if (c->task >= 4 && c->task <= 6) {
      /* ur3e-v0 (ur3e_env.py:139-170), imitation indirect (imitation_env_indirect.py:73-106) and
         direct (imitation_env_direct.py:74-108): truncation tests t before the increment */
      if (c->task == 6) {
        for (int k = 0; k < m->nu; k++) ctrl[k] = a[k];
      } else {
        double traj[7] = {a[0], a[1], a[2], -1.209, -1.209, 1.209, a[3]};
        ur3o_pid_task_ctrl(m, d, traj, &tg, ctrl);
      }
      for (int k = 0; k < m->nu; k++) d->ctrl[k] = ctrl[k];
      for (int s = 0; s < c->frame_skip; s++) ur3o_step(m, d);
      double o[24];
      task_obs(m, d, c->task, o);
      double r = c->task == 4 ? ur3o_reward_v0(m, d, o, a) : -1.0;
      int term = c->task == 4 ? ur3o_termination_v0(m, d, o) : 0;
      int trunc = c->max_episode_steps > 0 && e->t >= c->max_episode_steps;
      e->t += 1;
      e->ep_return += r;
      e->ep_len += 1;
      if (reward) reward[i] = r;
      if (terminated) terminated[i] = (unsigned char)term;
      if (truncated) truncated[i] = (unsigned char)trunc;
      if ((term || trunc) && c->auto_reset) {
        if (terminal_obs) memcpy(terminal_obs + (size_t)od * i, o, sizeof(double) * od);
        env_reset(m, c, e, obs ? obs + (size_t)od * i : 0);
      } else if (obs) {
        memcpy(obs + (size_t)od * i, o, sizeof(double) * od);
      }
      continue;
    }
    if (c->task == 1) {
      ur3o_pid_task_ctrl(m, d, a, &tg, ctrl);
    } else if (c->task == 7) {
      ur3o_move_l_ctrl(m, d, a, &jg, &rg, ctrl);
    } else if (c->task == 2) {
      ur3o_move_j_ctrl(m, d, a, &jg, ctrl);
    } else {
      for (int k = 0; k < m->nu; k++) ctrl[k] = a[k];
    }
    for (int k = 0; k < m->nu; k++) d->ctrl[k] = ctrl[k];
    int fs = c->task == 3 ? c->frame_skip : 1;
    for (int s = 0; s < fs; s++) ur3o_step(m, d);
    e->t += 1;
    /* task-space observation for the scripted tasks (same 24-d layout as ur3e-v2) */
    if (obs && has_obs_sites(m)) ur3o_obs_v2(m, d, obs + 24 * (size_t)i);
  }
}

void ur3o_batch_get_state(const ur3e_model_t* m, int n, const ur3o_env* envs, double* qpos, double* qvel,
                          double* warm, int* ncon) {
  for (int i = 0; i < n; i++) {
    const ur3o_data* d = &envs[i].d;
    if (qpos) memcpy(qpos + (size_t)m->nq * i, d->qpos, sizeof(double) * m->nq);
    if (qvel) memcpy(qvel + (size_t)m->nv * i, d->qvel, sizeof(double) * m->nv);
    if (warm) memcpy(warm + (size_t)m->nv * i, d->qacc_warmstart, sizeof(double) * m->nv);
    if (ncon) ncon[i] = d->ncon;
  }
}

void ur3o_batch_set_state(const ur3e_model_t* m, int n, ur3o_env* envs, const double* qpos, const double* qvel,
                          const double* warm) {
#pragma omp parallel for schedule(static)
  for (int i = 0; i < n; i++) {
    ur3o_data* d = &envs[i].d;
    memcpy(d->qpos, qpos + (size_t)m->nq * i, sizeof(double) * m->nq);
    memcpy(d->qvel, qvel + (size_t)m->nv * i, sizeof(double) * m->nv);
    if (warm) memcpy(d->qacc_warmstart, warm + (size_t)m->nv * i, sizeof(double) * m->nv);
    ur3o_forward(m, d);
  }
}

/* diagnostics for tests */
void ur3o_env_diag(const ur3o_env* e, int* ncon, int* nefc, int* niter, double* touch) {
  *ncon = e->d.ncon;
  *nefc = e->d.nefc;
  *niter = e->d.solver_niter;
  for (int k = 0; k < UR3E_MAXTOUCH; k++) touch[k] = e->d.touch[k];
}

/* d.ctrl applied by the last step (UR3E_MAXU entries) */
void ur3o_env_sensordata(const ur3e_model_t* m, const ur3o_env* e, double* out) {
  for (int k = 0; k < m->nsensordata; k++) out[k] = e->d.sensordata[k];
}

/* controller/controller_func.py:191-200 get_task_space_state, read after mj_step (move_l_mug.py:80):
   tcp site_xpos (3), get_site_xrotvec = scipy from_matrix(site_xmat).as_rotvec() (3), and
   get_boolean_grasp_contact (utils/utils.py:238-245): the tuple (left pad touch, right pad touch) >
   (0.1, 0.1), compared lexicographically.  Positions and touch are those of the step's last forward. */
void ur3o_rotvec_from_matrix(const double xmat[9], double rv[3]);
void ur3o_env_task_space_state(const ur3e_model_t* m, const ur3o_env* e, int touch_left, int touch_right,
                               double out[7]) {
  const ur3o_data* d = &e->d;
  const int st = m->id_site_tcp;
  for (int k = 0; k < 3; k++) out[k] = d->site_xpos[st][k];
  ur3o_rotvec_from_matrix(d->site_xmat[st], out + 3);
  const double l = d->touch[touch_left], r = d->touch[touch_right];
  out[6] = (l > 0.1 || (l == 0.1 && r > 0.1)) ? 1.0 : 0.0;
}

/* utils/utils.py:201-211 get_jnt_torques: the actuatorfrc sensors, i.e. mjData.actuator_force of the
   last forward (actuators in declaration order: six arm motors, then the fingers) */
void ur3o_env_actuator_force(const ur3e_model_t* m, const ur3o_env* e, double* out) {
  for (int k = 0; k < m->nu; k++) out[k] = e->d.actuator_force[k];
}

void ur3o_env_ctrl(const ur3o_env* e, double* ctrl) {
  for (int k = 0; k < UR3E_MAXU; k++) ctrl[k] = e->d.ctrl[k];
}

/* single-env helpers for golden-vector tests */
void ur3o_forward_state(const ur3e_model_t* m, const double* qpos, const double* qvel, double* site_xpos,
                        double* site_xmat, double* qfrc_bias, double* qM, int* ncon) {
  ur3o_data* d = (ur3o_data*)malloc(sizeof(ur3o_data));
  ur3o_reset_data(m, d);
  memcpy(d->qpos, qpos, sizeof(double) * m->nq);
  memcpy(d->qvel, qvel, sizeof(double) * m->nv);
  ur3o_forward(m, d);
  if (site_xpos) memcpy(site_xpos, d->site_xpos, sizeof(double) * 3 * m->nsite);
  if (site_xmat) memcpy(site_xmat, d->site_xmat, sizeof(double) * 9 * m->nsite);
  if (qfrc_bias) memcpy(qfrc_bias, d->qfrc_bias, sizeof(double) * m->nv);
  if (qM)
    for (int i = 0; i < m->nv; i++)
      for (int j = 0; j < m->nv; j++) qM[i * m->nv + j] = d->qM[i][j];
  if (ncon) *ncon = d->ncon;
  free(d);
}

/* ur3e-v0 epilogue on a synthetic contact list (golden tests of ur3e_env.py compute_reward /
   _check_termination and gym_utils.get_table_collision): out_r = reward, out_i = {term, table} */
void ur3o_v0_epilogue(const ur3e_model_t* m, int ncon, const int* geom1, const int* geom2, const double* obs13,
                      const double* act4, double* out_r, int* out_i) {
  ur3o_data* d = (ur3o_data*)calloc(1, sizeof(ur3o_data));
  d->ncon = ncon;
  for (int k = 0; k < ncon; k++) { d->contact[k].geom1 = geom1[k]; d->contact[k].geom2 = geom2[k]; }
  *out_r = ur3o_reward_v0(m, d, obs13, act4);
  out_i[0] = ur3o_termination_v0(m, d, obs13);
  out_i[1] = ur3o_table_collision(m, d);
  free(d);
}

/* predicates on a synthetic contact list (golden tests of gym_utils.py:98-172, ur3e_env2.py:230-254) */
void ur3o_predicates(const ur3e_model_t* m, int ncon, const int* geom1, const int* geom2, const double* tcp,
                     const double* hnd, const double* obs, int* out) {
  ur3o_data* d = (ur3o_data*)calloc(1, sizeof(ur3o_data));
  d->ncon = ncon;
  for (int k = 0; k < ncon; k++) { d->contact[k].geom1 = geom1[k]; d->contact[k].geom2 = geom2[k]; }
  for (int k = 0; k < 3; k++) {
    d->site_xpos[m->id_site_tcp][k] = tcp[k];
    d->site_xpos[m->id_site_handle][k] = hnd[k];
  }
  double o[24];
  ur3o_obs_v2(m, d, o); /* obs[23] = robust grasp state (velocities are zero here) */
  out[0] = ur3o_block_grasp_state(m, d);
  out[1] = (int)o[23];
  out[2] = ur3o_self_collision(m, d);
  out[3] = hnd[2] <= m->fish_topple_z;
  out[4] = ur3o_termination_v2(m, d, obs);
  free(d);
}

/* deterministic-math probe for tests: fn 0 sin, 1 cos, 2 exp, 3 tanh, 4 atan, 5 atan2 */
#include "../ur3e_amd/csrc/detmath.h"
double ur3o_detmath(int fn, double x, double y) {
  switch (fn) {
    case 0: return ur3e_sin(x);
    case 1: return ur3e_cos(x);
    case 2: return ur3e_exp(x);
    case 3: return ur3e_tanh(x);
    case 4: return ur3e_atan(x);
    default: return ur3e_atan2(x, y);
  }
}
