/*
 * ur3e_oracle.h — CPU ORACLE for the MI355X UR3e step path.  TEST
 * INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
 * bench.py cpu_baseline leg as the checker; never linked into the product
 * (ur3e_amd/), which fails loudly without its HIP library.
 *
 * What it restates (scalar FP64, one env at a time, MuJoCo mjData-style
 * semantics including the post-step "stale kinematics"):
 *   - mj_step of MuJoCo 3.3.3 (reference requirements.txt:58; third-party,
 *     absent from /root/reference) as called by MujocoEnv.do_simulation
 *     (gymnasium_env/envs/ur3e_env2.py:83) and controller/move_l_mug.py:78:
 *     kinematics, com, fixed tendon, CRB + LDL', collision (plane-box,
 *     box-box), constraint rows (connect, joint equality, dof frictionloss,
 *     joint limits, elliptic contacts), RNE, passive, actuation, Newton
 *     solver, touch sensors, Euler with implicit damping, bad-value reset;
 *   - the controller layer: pid_task_ctrl (controller/controller_func.py:68-117),
 *     pd_joint_ctrl (:128-167), move_j (controller/move_j.py:14-38), move_l
 *     (controller/move_l.py:15-78), scipy Rotation conversions used there;
 *   - the UR3eEnv2 epilogue: _get_obs (ur3e_env2.py:111-123), compute_reward
 *     (:150-228), _check_termination (:230-254), truncation (:257-261),
 *     success override (:93-95), reset_model (:101-109).
 *
 * Parity status: MuJoCo itself is not importable and the MJCF meshes are
 * absent, so the physics restatement is "parity unpinned" against MuJoCo; the
 * controller / reward / predicate / trajectory layer is pinned by golden
 * vectors generated from the reference Python (tests/golden/).
 */
#ifndef UR3E_ORACLE_H
#define UR3E_ORACLE_H

#include "../include/ur3e_model.h"

#ifdef __cplusplus
extern "C" {
#endif

/* constraint types / states: MuJoCo numbering */
#define UR3O_CNSTR_EQUALITY 0
#define UR3O_CNSTR_FRICTION_DOF 1
#define UR3O_CNSTR_LIMIT_JOINT 3
#define UR3O_CNSTR_CONTACT_ELLIPTIC 7
#define UR3O_STATE_SATISFIED 0
#define UR3O_STATE_QUADRATIC 1
#define UR3O_STATE_LINEARNEG 2
#define UR3O_STATE_LINEARPOS 3
#define UR3O_STATE_CONE 4

typedef struct {
  double pos[3];
  double frame[9];
  double dist;
  double includemargin;
  double friction[5];
  double solref[2];
  double solimp[5];
  double mu;
  int dim;
  int geom1, geom2;
  int efc_address;
} ur3o_contact;

typedef struct {
  /* state */
  double time;
  double qpos[UR3E_MAXNQ];
  double qvel[UR3E_MAXNV];
  double qacc_warmstart[UR3E_MAXNV];
  double ctrl[UR3E_MAXU];
  /* position-dependent */
  double xpos[UR3E_MAXBODY][3];
  double xquat[UR3E_MAXBODY][4];
  double xmat[UR3E_MAXBODY][9];
  double xipos[UR3E_MAXBODY][3];
  double ximat[UR3E_MAXBODY][9];
  double xanchor[UR3E_MAXJNT][3];
  double xaxis[UR3E_MAXJNT][3];
  double geom_xpos[UR3E_MAXGEOM][3];
  double geom_xmat[UR3E_MAXGEOM][9];
  double site_xpos[UR3E_MAXSITE][3];
  double site_xmat[UR3E_MAXSITE][9];
  double subtree_com[UR3E_MAXBODY][3];
  double cinert[UR3E_MAXBODY][10];
  double cdof[UR3E_MAXNV][6];
  double ten_length[UR3E_MAXTEN];
  double actuator_length[UR3E_MAXU];
  double actuator_moment[UR3E_MAXU][UR3E_MAXNV];
  double crb[UR3E_MAXBODY][10];
  double qM[UR3E_MAXNV][UR3E_MAXNV];
  double qLD[UR3E_MAXNV][UR3E_MAXNV];
  double qLDiagInv[UR3E_MAXNV];
  /* contacts */
  int ncon;
  int con_overflow;
  ur3o_contact contact[UR3E_MAXCON];
  /* constraints */
  int nefc;
  int efc_overflow;
  int efc_type[UR3E_MAXEFC];
  int efc_id[UR3E_MAXEFC];
  double efc_J[UR3E_MAXEFC][UR3E_MAXNV];
  double efc_pos[UR3E_MAXEFC];
  double efc_margin[UR3E_MAXEFC];
  double efc_frictionloss[UR3E_MAXEFC];
  double efc_diagApprox[UR3E_MAXEFC];
  double efc_R[UR3E_MAXEFC];
  double efc_D[UR3E_MAXEFC];
  double efc_vel[UR3E_MAXEFC];
  double efc_aref[UR3E_MAXEFC];
  double efc_force[UR3E_MAXEFC];
  int efc_state[UR3E_MAXEFC];
  /* velocity-dependent */
  double cvel[UR3E_MAXBODY][6];
  double cdof_dot[UR3E_MAXNV][6];
  double qfrc_bias[UR3E_MAXNV];
  double qfrc_passive[UR3E_MAXNV];
  double ten_velocity[UR3E_MAXTEN];
  double actuator_velocity[UR3E_MAXU];
  /* actuation / acceleration */
  double actuator_force[UR3E_MAXU];
  double qfrc_actuator[UR3E_MAXNV];
  double qfrc_smooth[UR3E_MAXNV];
  double qacc_smooth[UR3E_MAXNV];
  double qfrc_constraint[UR3E_MAXNV];
  double qacc[UR3E_MAXNV];
  double touch[UR3E_MAXTOUCH];
  /* mj_rnePostConstraint (only when the model has torque sensors) and mjData.sensordata */
  double cacc[UR3E_MAXBODY][6], cfrc_int[UR3E_MAXBODY][6], cfrc_ext[UR3E_MAXBODY][6];
  double sensordata[UR3E_MAXSENSORDATA];
  int solver_niter;
  int nwarning_bad;
} ur3o_data;

/* gains for pid_task_ctrl (controller/config/config_l_mug.yml) and PD */
typedef struct {
  double kp_pos[3], kd_pos[3], kp_rot[3], kd_rot[3];
} ur3o_task_gains;
typedef struct {
  double kp[6], kd[6];
} ur3o_joint_gains;

/* gym env (UR3eEnv2) wrapper state */
typedef struct {
  ur3o_data d;
  int t;
  double ep_return;
  int ep_len;
  unsigned int episode;
  unsigned int env_id;
  unsigned long long seed;
} ur3o_env;

/* ---- physics ---- */
void ur3o_reset_data(const ur3e_model_t* m, ur3o_data* d);
void ur3o_forward(const ur3e_model_t* m, ur3o_data* d);
void ur3o_step(const ur3e_model_t* m, ur3o_data* d);
void ur3o_jac_site(const ur3e_model_t* m, const ur3o_data* d, int site, double* jacp, double* jacr);
void ur3o_site_velocity(const ur3e_model_t* m, const ur3o_data* d, int site, double res[6]);
int ur3o_block_grasp_state(const ur3e_model_t* m, const ur3o_data* d);
int ur3o_self_collision(const ur3e_model_t* m, const ur3o_data* d);

/* ---- rotations (scipy.spatial.transform.Rotation semantics) ---- */
void ur3o_quat_from_matrix(const double mat[9], double quat_xyzw[4]);
void ur3o_quat_from_rotvec(const double rv[3], double quat_xyzw[4]);
void ur3o_rotvec_from_quat(const double quat_xyzw[4], double rv[3]);
void ur3o_rot_err(const double xmat[9], const double target_rotvec[3], double err[3]);

/* ---- controllers ---- */
void ur3o_pid_task_ctrl_raw(const double traj7[7], const double tcp_xpos[3], const double tcp_xmat[9],
                            const double jac_arm[36], const double qvel6[6], const double bias6[6],
                            const ur3o_task_gains* g, double grip_scale, double ctrl7[7]);
void ur3o_pid_task_ctrl(const ur3e_model_t* m, const ur3o_data* d, const double traj7[7],
                        const ur3o_task_gains* g, double* ctrl);
void ur3o_pd_joint_ctrl_raw(const double q6[6], const double v6[6], const double delta6[6],
                            const double jnt_range[12], const double ctrl_range[12],
                            const ur3o_joint_gains* g, double u6[6]);
void ur3o_move_j_ctrl(const ur3e_model_t* m, const ur3o_data* d, const double traj7[7],
                      const ur3o_joint_gains* g, double* ctrl);
void ur3o_pinv3x6(const double J[18], double P[18]);
void ur3o_move_l_ctrl(const ur3e_model_t* m, const ur3o_data* d, const double traj7[7],
                      const ur3o_joint_gains* gpos, const ur3o_joint_gains* grot, double* ctrl);
void ur3o_move_l_ctrl_raw(const double traj[7], const double tcp_xpos[3], const double tcp_xmat[9],
                          const double Jp[18], const double Jr[18], const double q[6], const double v[6],
                          const double jr[12], const double cr[12], const ur3o_joint_gains* gpos,
                          const ur3o_joint_gains* grot, double grip_scale, double ctrl[7]);

/* ---- UR3eEnv2 epilogue ---- */
void ur3o_obs_v2(const ur3e_model_t* m, const ur3o_data* d, double obs[24]);
/* ur3e-v0 / imitation epilogues (gymnasium_env/envs/ur3e_env.py, imitation_env_direct.py) */
int ur3o_table_collision(const ur3e_model_t* m, const ur3o_data* d);
void ur3o_obs_v0(const ur3e_model_t* m, const ur3o_data* d, double obs[13]);
void ur3o_obs_direct(const ur3e_model_t* m, const ur3o_data* d, double obs[13]);
double ur3o_reward_v0(const ur3e_model_t* m, const ur3o_data* d, const double obs[13], const double act[4]);
int ur3o_termination_v0(const ur3e_model_t* m, const ur3o_data* d, const double obs[13]);
double ur3o_reward_v2(const double obs[24], const double act[4]);
int ur3o_termination_v2(const ur3e_model_t* m, const ur3o_data* d, const double obs[24]);

/* ---- counter-based RNG (Philox4x32-10) ---- */
void ur3o_philox4x32(const unsigned int ctr[4], const unsigned int key[2], unsigned int out[4]);
double ur3o_uniform01(unsigned long long seed, unsigned int env_id, unsigned int episode, unsigned int k);

/* ---- env API (gym ur3e-v2 semantics, SB3 auto-reset done by caller) ---- */
void ur3o_env_init(const ur3e_model_t* m, ur3o_env* e, unsigned long long seed, unsigned int env_id);
void ur3o_env_reset(const ur3e_model_t* m, ur3o_env* e, double obs[24]);
void ur3o_env_step_v2(const ur3e_model_t* m, ur3o_env* e, const ur3o_task_gains* g, const double action[4],
                      int frame_skip, double obs[24], double* reward, int* terminated, int* truncated);

/* ---- convenience for ctypes tests ---- */
int ur3o_sizeof_data(void);
int ur3o_sizeof_env(void);

#ifdef __cplusplus
}
#endif
#endif
