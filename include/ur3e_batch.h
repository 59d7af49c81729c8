/*
 * ur3e_batch.h — C ABI of the MI355X-native batched UR3e step library
 * (ur3e_amd/_lib/libur3e_amd.so, built from ur3e_amd/csrc/ur3e_batch.hip).
 *
 * One handle = N environments resident in HBM on one GPU.  Every pointer
 * argument named d_* is a DEVICE pointer (e.g. a torch tensor's data_ptr() on
 * the same device); `stream` is a hipStream_t (NULL = default stream).  All
 * calls only enqueue work on `stream` and return immediately (one exception:
 * on main.xml's tiered step, ur3e_batch_step waits for the step enqueued 16
 * calls earlier to finish, bounding how far the host runs ahead of the GPU;
 * never inside a graph capture).  Return value: 0
 * on success, a negative UR3E_E* code otherwise; ur3e_last_error() gives a
 * thread-local message.  A handle is not thread-safe.
 *
 * Graph capture: ur3e_batch_step, _reset, _set_state and the getters keep all of their control
 * state on the device (the overflow list of the two-tier step is reset by its own fallback kernel),
 * so a sequence of them can be captured into a HIP graph (hipStreamBeginCapture, or
 * torch.cuda.graph) and replayed any number of times.  ur3e_batch_overflow_count and
 * ur3e_batch_last_step_ms synchronise and must not be captured.
 *
 * Reference interfaces each entry point replaces (the reference's boundary is
 * Python — gymnasium Env + MuJoCo C API):
 *
 *   ur3e_batch_create   MujocoEnv.__init__ / UR3eEnv2.__init__
 *                       (gymnasium_env/envs/ur3e_env2.py:30-70) × N processes of
 *                       SubprocVecEnv (gymnasium_src/scripts/regular_rl/rl/train_rl.py:38-44)
 *   ur3e_batch_reset    MujocoEnv.reset -> mj_resetData -> UR3eEnv2.reset_model
 *                       (ur3e_env2.py:101-109; utils/gym_utils.py:63-79)
 *   ur3e_batch_step     UR3eEnv2.step (ur3e_env2.py:72-99) = pid_task_ctrl
 *                       (controller/controller_func.py:68-117) + do_simulation ->
 *                       mj_step × frame_skip + _get_obs + compute_reward +
 *                       termination/truncation, with SB3 VecEnv auto-reset; for the
 *                       scripted tasks: controller/move_l_mug.py:67-81 (traj_l),
 *                       controller/move_j.py:76-86 (move_j)
 *   ur3e_batch_get_state / ur3e_batch_set_state
 *                       MjData.qpos/qvel/qacc_warmstart read/write + mj_forward
 *                       (MujocoEnv.set_state; utils/utils.py:15-24)
 *   ur3e_batch_destroy  env.close()
 *   ur3e_batch_create_from_mjcf
 *                       gymnasium.make / init_mj.py:22-30 from the model file and gain YAML
 */
#ifndef UR3E_BATCH_H
#define UR3E_BATCH_H

#include <stdint.h>

#include "ur3e_model.h"

#ifdef __cplusplus
extern "C" {
#endif

#define UR3E_ABI_VERSION 9

/* tasks (what one env-step means) */
#define UR3E_TASK_GYM_V2 0  /* action [N,4] task-space (x,y,z,grip): gym ur3e-v2 */
#define UR3E_TASK_TRAJ_L 1  /* action [N,7] task-space trajectory row: pid_task_ctrl */
#define UR3E_TASK_MOVE_J 2  /* action [N,7] joint targets + grip: move_j PD */
#define UR3E_TASK_CTRL 3    /* action [N,nu] raw actuator controls */
/* the other registered gymnasium ids (gymnasium_env/register_envs.py:4-20); workgroup-per-env
   layouts only (envs_per_block <= 0) */
#define UR3E_TASK_GYM_V0 4          /* ur3e-v0 (ur3e_env.py): action [N,4], obs [N,13], T = 500 */
#define UR3E_TASK_IMIT_INDIRECT 5   /* imitation_indirect-v0: action [N,4], obs [N,24], reward -1 */
#define UR3E_TASK_IMIT_DIRECT 6     /* imitation_direct-v0: action [N,nu] ctrl, obs [N,13], reward -1 */
/* scripted move_l (controller/move_l.py:15-78): action [N,7] task-space trajectory row; joint deltas
   pinv(Jp_arm) e_p and pinv(Jr_arm) e_r through two pd_joint_ctrl calls (joint_gains = "pos",
   rot_joint_gains = "rot" of config_l.yml), summed; 1 physics step per env-step */
#define UR3E_TASK_MOVE_L 7

/* error codes */
#define UR3E_OK 0
#define UR3E_EINVAL -1
#define UR3E_EHIP -2
#define UR3E_ENOMEM -3
#define UR3E_EMODEL -4

typedef struct ur3e_config_t {
  int task;
  int frame_skip;        /* physics substeps per env-step (gym ur3e-v2: 2) */
  int max_episode_steps; /* truncation horizon (ur3e-v2: 2500); <= 0: never */
  int auto_reset;        /* SB3 VecEnv semantics on terminated|truncated */
  int reset_noise;       /* mug xy noise on reset, gym_utils.get_mug_xpos_noise: 0 none ("deterministic"),
                            1 "high" (ur3e-v2), 2 "med", 3 "low" */
  int reset_key;         /* keyframe index used by reset (-1: qpos0) */
  double task_gains[12]; /* kp_pos[3], kd_pos[3], kp_rot[3], kd_rot[3] (config_l_mug.yml) */
  double joint_gains[12];/* kp[6], kd[6] (config_j.yml; move_l: config_l.yml "pos") */
  unsigned long long seed; /* Philox key for reset noise */
  int env_id_offset;     /* global id of local env 0 (multi-GPU shards) */
  int envs_per_block;    /* kernel layout:
                            0 (default) = tiered: one 64-lane wavefront per env with a compact
                              LDS working set (<= W_SMALL_MAXCON contacts / W_SMALL_MAXEFC rows,
                              eight envs per CU); an env that exceeds it in any substep is
                              recomputed, same step, by the grasp tier (main.xml: the same code
                              path sized for W_GRASP_MAXCON contacts / W_GRASP_MAXEFC rows), and
                              one that exceeds that by the full-capacity tier;
                            -128 = full-capacity tier only, 128-lane workgroup per env;
                            -64 = full-capacity tier only, 64-lane wavefront per env;
                            1..64 = one env per lane, that many envs per wavefront (v1) */
  int tier_con_cap;      /* diagnostic (0 = off): > 0: the compact tier treats more than this many
                            contacts as overflow (its envs run in the grasp tier); < 0: the compact
                            and the grasp tier both treat more than -tier_con_cap contacts as
                            overflow (the envs reach the full-capacity tier) */
  double rot_joint_gains[12]; /* kp[6], kd[6] of the rotation PD in move_l (config_l.yml "rot") */
  int np_chunk_lanes;    /* diagnostic (0 = 16): survivor lanes per compact-tier narrowphase chunk;
                            smaller values exercise its multi-chunk path */
  int sensors;           /* 1: compute mjData.sensordata every forward (touch, actuatorfrc, torque via
                            mj_rnePostConstraint; assets/main.xml:384-405) for ur3e_batch_get_sensordata.
                            The torque sensors need the full-capacity layout, so the handle runs the
                            full-capacity tier (envs_per_block 0 -> 128 lanes per env; > 0 rejected) */
  int schedule;          /* two-tier step launch: 0 (default, auto) = gym tasks with frame_skip > 1 on
                            main.xml with more envs than resident workgroup slots run as a substep work
                            queue (a resident pool of workgroups pulls (substep, env) units, state handed
                            between substeps through HBM: balances the launch at substep granularity),
                            otherwise one workgroup per env-step; 1 = always one workgroup per env-step;
                            2 = always the queue (when applicable).  Same results either way. */
} ur3e_config_t;

typedef struct ur3e_batch ur3e_batch_t;

int ur3e_abi_version(void);
const char* ur3e_last_error(void);

/* The reference's files as the model and gains (ur3e_amd/csrc/ur3e_mjcf.cpp), for callers that are not
   Python.  The MJCF compiler and the YAML reader are the package's Python (ur3e_amd/model/compiler.py,
   ur3e_amd/gains.py), run through an embedded interpreter (libpython loaded on first use; in a Python
   process, the running one); nothing here touches the GPU.
     ur3e_model_from_mjcf: compile an MJCF file (assets/main.xml, ur3e_2f85.xml, ur3e_raw.xml: what
       MujocoEnv.__init__ / init_mj.py:22-30 load) into *out; meshes = "auto" (NULL), "mesh" or
       "surrogate" (ur3e_amd/model/compiler.py: real convex meshes when the files exist, else boxes).
     ur3e_config_gains_from_yaml: fill cfg's gains for cfg->task from a gain file as the reference reads
       it (task-space tasks: config_l_mug.yml, ur3e_env2.py:66-68; move_j: config_j.yml, move_j.py:46-52;
       move_l: config_l.yml, move_l.py:92-99); NULL: controller/config/<file> under the working
       directory, else the packaged copy of the reference's values.
     ur3e_batch_create_from_mjcf: both, then ur3e_batch_create (cfg's gains are replaced). */
int ur3e_model_from_mjcf(const char* mjcf_path, const char* meshes, ur3e_model_t* out);
int ur3e_config_gains_from_yaml(const char* config_yaml_path, ur3e_config_t* cfg);
int ur3e_batch_create_from_mjcf(const char* mjcf_path, const char* config_yaml_path, const ur3e_config_t* cfg,
                                int n_envs, int device, ur3e_batch_t** out);

/* allocates N envs at qpos0 / zero velocity; like gymnasium, call ur3e_batch_reset before stepping */
int ur3e_batch_create(const ur3e_model_t* model, const ur3e_config_t* cfg, int n_envs, int device,
                      ur3e_batch_t** out);
int ur3e_batch_destroy(ur3e_batch_t* b);

/* reset envs whose d_mask[i] != 0 (d_mask NULL: all); writes obs rows of reset envs */
int ur3e_batch_reset(ur3e_batch_t* b, const uint8_t* d_mask, double* d_obs, void* stream);

/* one env-step for all envs.  d_actions [N, adim] row-major.  Outputs may be NULL:
   d_obs [N,24], d_reward [N], d_terminated/d_truncated [N] u8, d_terminal_obs [N,24]
   (rows written only for envs that finished this step; d_obs then holds the reset obs).
   For the scripted tasks (TRAJ_L / MOVE_J / CTRL) d_obs, when given and the model has the
   tcp / handle_site / ghost frames, receives the same 24-d observation of the new state. */
int ur3e_batch_step(ur3e_batch_t* b, const double* d_actions, int adim, double* d_obs, double* d_reward,
                    uint8_t* d_terminated, uint8_t* d_truncated, double* d_terminal_obs, void* stream);

/* state in user layout: d_qpos [N,nq], d_qvel [N,nv], d_warm [N,nv] (any may be NULL) */
int ur3e_batch_get_state(ur3e_batch_t* b, double* d_qpos, double* d_qvel, double* d_warm, void* stream);
/* sets state then runs the forward pass (refreshes the stale-kinematics carry) */
int ur3e_batch_set_state(ur3e_batch_t* b, const double* d_qpos, const double* d_qvel, const double* d_warm,
                         void* stream);
/* diagnostics: d_ncon [N] contacts of the last forward, d_ep_len [N], d_ep_return [N],
   d_nwarn [N] bad-value auto-resets (each may be NULL) */
int ur3e_batch_get_info(ur3e_batch_t* b, int* d_ncon, int* d_ep_len, double* d_ep_return, int* d_nwarn,
                        void* stream);

/* stale-kinematics snapshot of the last forward, d_carry [N, 54]: tcp site_xpos (3), site_xmat (9),
   the arm columns of mj_jacSite(tcp) as [jacp; jacr] 6x6 row-major (36), qfrc_bias[0:6] (6) --
   what controller_func.py:68-117 reads from MjData before each pid_task_ctrl call */
int ur3e_batch_get_carry(ur3e_batch_t* b, double* d_carry, void* stream);

/* touch sensors of the last forward (main.xml: left/right pad sites, mjSENS_TOUCH semantics),
   d_touch [N, ntouch]; replaces d.sensordata reads in controller/move_l_mug.py:79 via
   utils/utils.py:238-240 (get_boolean_grasp_contact) */
int ur3e_batch_get_touch(ur3e_batch_t* b, double* d_touch, void* stream);

/* mjData.sensordata of the last forward, d_sensordata [N, model nsensordata] in the model's sensor
   declaration order (main.xml: 6 torque x3, 6 arm actuatorfrc, right/left pad touch, fingers
   actuatorfrc = 27 values); needs ur3e_config_t.sensors = 1.  Replaces d.sensor(name).data reads:
   get_jnt_torques (utils/utils.py:201-211, called at controller/move_l_mug.py:80) and
   get_grasp_contact (utils/utils.py:238-245) */
int ur3e_batch_get_sensordata(ur3e_batch_t* b, double* d_sensordata, void* stream);

/* controller/controller_func.py:191-200 get_task_space_state, as controller/move_l_mug.py:80 records it
   after every mj_step, d_out [N, 7]: tcp site_xpos (3), tcp rotvec = scipy Rotation.from_matrix(
   site_xmat).as_rotvec() (utils/utils.py:158-162; 3), and get_boolean_grasp_contact (utils/utils.py:
   238-245: (left pad touch, right pad touch) > (0.1, 0.1) compared as tuples; 1.0 / 0.0), all of the
   last step's final forward pass.  Needs main.xml's tcp site and pad touch sensors. */
int ur3e_batch_get_task_space_state(ur3e_batch_t* b, double* d_out, void* stream);

/* mjData.actuator_force of the last forward, d_out [N, nu]: the actuatorfrc sensors that
   utils/utils.py:201-211 get_jnt_torques reads (recorded at controller/move_l_mug.py:81), available
   in every tier (no sensors flag needed).  Not kept by the v1 lane-per-env layout (EINVAL). */
int ur3e_batch_get_actuator_force(ur3e_batch_t* b, double* d_out, void* stream);

/* d.ctrl after the last step, d_ctrl [N, nu]: the controller output the step applied (pid_task_ctrl
   torques + grip, PD torques, or the raw action); zero after a reset, like mj_resetData.  Replaces the
   `u` that gymnasium_src/scripts/imitation_rl/collect_demos.py:134-148 records as the direct action */
int ur3e_batch_get_ctrl(ur3e_batch_t* b, double* d_ctrl, void* stream);

/* env-steps the compact tier handed on to the fallback tiers since create (synchronises) */
int ur3e_batch_overflow_count(ur3e_batch_t* b, unsigned long long* total);

/* since create (synchronises): counts[0] env-steps the compact tier handed on (to the grasp tier while
   routing is in use, else straight to the full-capacity tier), counts[1] env-steps that reached the
   full-capacity tier, counts[2] env-steps routed to the grasp tier (the env's previous forward exceeded the
   compact tier's routing thresholds, 4 / 27 for the gym tasks and 8 / 36 for the scripted pick, and the mid
   tier's 16 / 63 -- or it bailed from the mid tier; it runs on an internal stream concurrently with the
   compact tier) */
int ur3e_batch_tier_counts(ur3e_batch_t* b, unsigned long long* counts);

/* since create (synchronises): env-steps routed to the mid tier (16 contacts / 64 rows), between the compact
   and the grasp tier -- a routed env whose previous forward fits it runs there, on the same internal stream
   as the grasp tier and ahead of it; the env-steps it hands on are counted again in tier_counts[2] */
int ur3e_batch_mid_count(ur3e_batch_t* b, unsigned long long* routed);

/* substep work queue (schedule 1), since create (synchronises): stats[0] units that gave up waiting
   for their producer (spin limit; the env-step then ran in the fallback tiers), stats[1] static
   first units that were claimed and run by their consumer because their own workgroup was not
   running yet.  Neither changes results. */
int ur3e_batch_queue_stats(ur3e_batch_t* b, unsigned long long* stats);

/* diagnostics of the substep work queue (results never change): spin_limit = flag polls before a
   waiting unit gives up (0 = the built-in bound, 2^26); leave_static_units = 1: workgroups skip their
   static first units, so every one of them is claimed and run by its consumer */
int ur3e_batch_set_queue_debug(ur3e_batch_t* b, unsigned int spin_limit, int leave_static_units);

/* substep work queue (schedule 1): the last `percent` % of each unit queue's envs run their last substep
   as two half units (the first stops where the forward pass reaches the constraint solver and hands the
   env's working set to the second, queued after every other unit), so the units that end the launch
   are shorter.  Results never change.  Default 0 (off: measured slower); non-queued
   handles accept only 0. */
int ur3e_batch_set_queue_split(ur3e_batch_t* b, int percent);

/* multi-GPU (north_star config C4), for hosts that hold their own RCCL communicator (ncclComm_t passed
   as void*; ur3e_amd/csrc/ur3e_gather.cpp, librccl loaded on first use): after a step, every rank sends
   its (obs [n, obs_dim], reward [n], terminated [n], truncated [n]) to `root`, which receives all ranks'
   in rank order into d_*_all ([nranks * n] rows; other ranks pass NULL).  Every rank's handle has the
   same n; the shards are contiguous global env ids (env_id_offset = rank * n).  Enqueued on `stream` as
   one point-to-point group, after the step that filled the buffers.  The env path itself has no
   collective.  PRECONDITION: every rank's handle has the same n and obs_dim (the same env id); the root
   posts receives of exactly its own sizes, so ranks that disagree leave the group's transfers unmatched
   (RCCL then hangs the streams) -- nothing here can detect it without a collective of its own.
   Replaces the reference's SubprocVecEnv gather of per-env step results (train_rl.py:38-44,
   stable_baselines3 make_vec_env), as north_star config C4 prescribes. */
int ur3e_batch_gather(ur3e_batch_t* b, void* rccl_comm, int root, const double* d_obs, const double* d_reward,
                      const uint8_t* d_terminated, const uint8_t* d_truncated, double* d_obs_all,
                      double* d_reward_all, uint8_t* d_terminated_all, uint8_t* d_truncated_all, void* stream);

/* ur3e_batch_gather with explicit sizes, for host-managed buffers (the handle only supplies n and
   obs_dim): the same point-to-point group, rank p's rows at [p * n, (p + 1) * n) of the root's buffers;
   the same precondition (equal n and obs_dim on every rank). */
int ur3e_gather_rows(void* rccl_comm, int root, int n, int obs_dim, const double* d_obs, const double* d_reward,
                     const uint8_t* d_terminated, const uint8_t* d_truncated, double* d_obs_all, double* d_reward_all,
                     uint8_t* d_terminated_all, uint8_t* d_truncated_all, void* stream);

/* diagnostic (the queue's forward-progress test): launch `workgroups` workgroups on `stream` that each
   hold 64 KB of LDS (two per CU leave room for one step workgroup) for hold_us microseconds, and
   return once they have all started (started = how many had, waited for at most 2 * hold_us), so
   that work launched next on another stream finds most of its workgroup slots taken.  Every
   workgroup exits after hold_us; results of other work never change. */
int ur3e_debug_hold_slots(int device, int workgroups, int hold_us, void* stream, int* started);

/* the step kernel this handle launches: 0 compact tier, one workgroup per env-step; 1 compact tier
   as a substep work queue; 2 full-capacity tier only; 3 one env per lane (v1) */
int ur3e_batch_schedule(const ur3e_batch_t* b);

/* observation width of the handle's task (24 or 13) */
int ur3e_batch_obs_dim(const ur3e_batch_t* b);

/* sizes */
int ur3e_batch_num_envs(const ur3e_batch_t* b);
int ur3e_batch_nq(const ur3e_batch_t* b);
int ur3e_batch_nv(const ur3e_batch_t* b);
int ur3e_batch_nu(const ur3e_batch_t* b);

/* the step kernel this handle launches: envs resident per CU (occupancy), static LDS bytes per
   workgroup, registers per lane */
int ur3e_batch_kernel_info(ur3e_batch_t* b, int* envs_per_cu, int* lds_bytes, int* regs);

/* the kernel the handle launches for `tier` (0: the step kernel -- the compact tier, or an untiered
   layout's only kernel; 1: the grasp tier; 2: the full-capacity fallback tier; 3: the mid tier), chosen by the same
   branches as ur3e_batch_step: envs resident per CU, LDS bytes per workgroup (static + dynamic),
   registers per lane, a readable name (name, NUL-terminated within name_len) and the code object's
   kernel symbol (symbol; empty when the runtime cannot name it).  UR3E_EINVAL for a tier the handle
   does not launch. */
int ur3e_batch_tier_kernel(ur3e_batch_t* b, int tier, int* envs_per_cu, int* lds_bytes, int* regs, char* name,
                           int name_len, char* symbol, int symbol_len);

/* profiling: with timing on (off by default), every ur3e_batch_step that is not being captured into
   a graph records a pair of HIP events around its kernels; last_step_ms reads the most recent pair */
int ur3e_batch_set_timing(ur3e_batch_t* b, int on);
int ur3e_batch_last_step_ms(ur3e_batch_t* b, float* ms);

#ifdef __cplusplus
}
#endif
#endif /* UR3E_BATCH_H */
