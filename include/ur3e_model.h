/*
 * ur3e_model.h — flat, fixed-capacity model image consumed by the MI355X step
 * kernels (ur3e_amd/csrc) and by the CPU oracle (oracle/).
 *
 * This is the boundary data format that replaces `mujoco.MjModel` on the hot
 * path (reference: MujocoEnv.__init__ → MjModel.from_xml_path,
 * gymnasium_env/envs/ur3e_env2.py:32,50-55; utils/utils.py:9-12).  It is produced
 * by ur3e_amd/model/compiler.py from the reference MJCF (assets/main.xml,
 * assets/ur3e_2f85.xml, assets/ur3e_raw.xml) plus the documented mesh surrogate
 * (ur3e_amd/model/surrogate.py): the MJCF meshes are absent everywhere.
 *
 * Layout rules: plain C, doubles and ints only, no pointers, so one image can be
 * memcpy'd to device memory and read with wave-uniform (scalar) loads.
 * Field meanings follow MuJoCo's mjModel of the same name.
 */
#ifndef UR3E_MODEL_H
#define UR3E_MODEL_H

#ifdef __cplusplus
extern "C" {
#endif

#define UR3E_MODEL_VERSION 6

#define UR3E_MAXBODY 28
#define UR3E_MAXJNT 16
#define UR3E_MAXNQ 24
#define UR3E_MAXNV 24
#define UR3E_MAXGEOM 32
#define UR3E_MAXSITE 20
#define UR3E_MAXCPAIR 320 /* collision candidate list after static filtering */
#define UR3E_MAXEQ 4
#define UR3E_MAXU 8
#define UR3E_MAXTEN 2
#define UR3E_MAXTENWRAP 4
#define UR3E_MAXKEY 2
#define UR3E_MAXTOUCH 4
#define UR3E_MAXSENSOR 16
#define UR3E_MAXSENSORDATA 48
#define UR3E_MAXMESH 16       /* convex mesh geoms' meshes */
#define UR3E_MAXMESHVERT 1024 /* hull vertices of all meshes */

/* per-env dynamic capacities (the kernels size scratch from these) */
#define UR3E_MAXCON 40                                   /* contacts per env (main.xml: nconmax 100) */
#define UR3E_MAXEFC (3 * UR3E_MAXCON + 40)               /* constraint rows per env; groups (connect,
                                                            contact) are reserved whole, first overflow stops */

/* joint types (MuJoCo numbering) */
#define UR3E_JNT_FREE 0
#define UR3E_JNT_BALL 1
#define UR3E_JNT_SLIDE 2
#define UR3E_JNT_HINGE 3

/* geom types (MuJoCo numbering for the ones used) */
#define UR3E_GEOM_PLANE 0
#define UR3E_GEOM_BOX 6
#define UR3E_GEOM_MESH 7 /* convex hull of a mesh asset (real meshes; see ur3e_amd/model/mesh.py) */

/* equality types */
#define UR3E_EQ_CONNECT 0
#define UR3E_EQ_JOINT 2

/* actuator transmission / gain / bias */
#define UR3E_TRN_JOINT 0
#define UR3E_TRN_TENDON 3
#define UR3E_GAIN_FIXED 0
#define UR3E_BIAS_NONE 0
#define UR3E_BIAS_AFFINE 1

/* sensor types (the subset main.xml declares, assets/main.xml:384-405) */
#define UR3E_SENS_TOUCH 0       /* 1 value: normal force of contacts in the site volume */
#define UR3E_SENS_ACTUATORFRC 1 /* 1 value: actuator_force */
#define UR3E_SENS_TORQUE 2      /* 3 values: cfrc_int torque at the site, site frame (mj_rnePostConstraint) */

/* cone */
#define UR3E_CONE_PYRAMIDAL 0
#define UR3E_CONE_ELLIPTIC 1

typedef struct ur3e_model_t {
  int version;
  int nq, nv, nu, nbody, njnt, ngeom, nsite, ncpair, neq, ntendon, nkey, ntouch;

  /* options (MuJoCo <option>) */
  double timestep;
  double gravity[3];
  int cone;
  double impratio;
  double tolerance;
  int iterations;
  int ls_iterations;
  double ls_tolerance;
  double meaninertia; /* mj_setConst: trace(M(qpos0))/nv */

  /* bodies, MuJoCo depth-first order, 0 = world */
  int body_parentid[UR3E_MAXBODY];
  int body_rootid[UR3E_MAXBODY];
  int body_weldid[UR3E_MAXBODY];
  int body_jntnum[UR3E_MAXBODY];
  int body_jntadr[UR3E_MAXBODY];
  int body_dofnum[UR3E_MAXBODY];
  int body_dofadr[UR3E_MAXBODY];
  double body_pos[UR3E_MAXBODY][3];
  double body_quat[UR3E_MAXBODY][4];
  double body_ipos[UR3E_MAXBODY][3];
  double body_iquat[UR3E_MAXBODY][4];
  double body_mass[UR3E_MAXBODY];
  double body_subtreemass[UR3E_MAXBODY];
  double body_inertia[UR3E_MAXBODY][3];
  double body_invweight0[UR3E_MAXBODY][2];

  /* joints */
  int jnt_type[UR3E_MAXJNT];
  int jnt_qposadr[UR3E_MAXJNT];
  int jnt_dofadr[UR3E_MAXJNT];
  int jnt_bodyid[UR3E_MAXJNT];
  int jnt_limited[UR3E_MAXJNT];
  double jnt_pos[UR3E_MAXJNT][3];
  double jnt_axis[UR3E_MAXJNT][3];
  double jnt_range[UR3E_MAXJNT][2];
  double jnt_stiffness[UR3E_MAXJNT];
  double jnt_margin[UR3E_MAXJNT];
  double jnt_solref[UR3E_MAXJNT][2]; /* solreflimit */
  double jnt_solimp[UR3E_MAXJNT][5]; /* solimplimit */

  /* dofs */
  int dof_bodyid[UR3E_MAXNV];
  int dof_jntid[UR3E_MAXNV];
  int dof_parentid[UR3E_MAXNV];
  double dof_armature[UR3E_MAXNV];
  double dof_damping[UR3E_MAXNV];
  double dof_frictionloss[UR3E_MAXNV];
  double dof_invweight0[UR3E_MAXNV];
  double dof_solref[UR3E_MAXNV][2]; /* solreffriction */
  double dof_solimp[UR3E_MAXNV][5]; /* solimpfriction */

  double qpos0[UR3E_MAXNQ];
  double qpos_spring[UR3E_MAXNQ];

  /* collision geoms (visual-only geoms are dropped after inertia compile) */
  int geom_type[UR3E_MAXGEOM];
  int geom_bodyid[UR3E_MAXGEOM];
  int geom_surrogate[UR3E_MAXGEOM]; /* 1: mesh replaced by documented box surrogate */
  double geom_pos[UR3E_MAXGEOM][3];
  double geom_quat[UR3E_MAXGEOM][4];
  double geom_size[UR3E_MAXGEOM][3];
  double geom_rbound[UR3E_MAXGEOM];

  /* sites */
  int site_bodyid[UR3E_MAXSITE];
  int site_type[UR3E_MAXSITE];
  double site_pos[UR3E_MAXSITE][3];
  double site_quat[UR3E_MAXSITE][4];
  double site_size[UR3E_MAXSITE][3];

  /* collision candidates in processing order (explicit <pair>s merged with
     statically-filtered dynamic geom pairs, sorted by body-pair signature).
     Parameters are final: explicit-pair values or MuJoCo geom mixing. */
  int cpair_geom1[UR3E_MAXCPAIR];
  int cpair_geom2[UR3E_MAXCPAIR];
  int cpair_explicit[UR3E_MAXCPAIR];
  int cpair_condim[UR3E_MAXCPAIR];
  double cpair_friction[UR3E_MAXCPAIR][5];
  double cpair_solref[UR3E_MAXCPAIR][2];
  double cpair_solimp[UR3E_MAXCPAIR][5];
  double cpair_margin[UR3E_MAXCPAIR];
  double cpair_gap[UR3E_MAXCPAIR];

  /* fixed tendons */
  int ten_num[UR3E_MAXTEN];
  int ten_dof[UR3E_MAXTEN][UR3E_MAXTENWRAP];
  double ten_coef[UR3E_MAXTEN][UR3E_MAXTENWRAP];

  /* equality constraints */
  int eq_type[UR3E_MAXEQ];
  int eq_obj1[UR3E_MAXEQ]; /* body (connect) or joint (joint) */
  int eq_obj2[UR3E_MAXEQ];
  double eq_data[UR3E_MAXEQ][11];
  double eq_solref[UR3E_MAXEQ][2];
  double eq_solimp[UR3E_MAXEQ][5];

  /* actuators */
  int act_trntype[UR3E_MAXU];
  int act_trnid[UR3E_MAXU];
  int act_gaintype[UR3E_MAXU];
  int act_biastype[UR3E_MAXU];
  int act_ctrllimited[UR3E_MAXU];
  int act_forcelimited[UR3E_MAXU];
  double act_ctrlrange[UR3E_MAXU][2];
  double act_forcerange[UR3E_MAXU][2];
  double act_gainprm[UR3E_MAXU][3];
  double act_biasprm[UR3E_MAXU][3];
  double act_gear[UR3E_MAXU];

  /* touch sensors (site ids), in sensor order */
  int touch_site[UR3E_MAXTOUCH];

  /* keyframes */
  double key_qpos[UR3E_MAXKEY][UR3E_MAXNQ];
  double key_qvel[UR3E_MAXKEY][UR3E_MAXNV];

  /* named ids used by controllers and env epilogues (-1 when absent) */
  int id_site_tcp, id_site_handle, id_site_lpad, id_site_rpad;
  int id_body_fish, id_body_ghost, id_body_lpad, id_body_rpad;
  int id_key_home, id_key_down;
  /* body-set masks (bit b = body b) for gym_utils.init_collision_cache */
  unsigned int mask_arm_bodies;     /* robot_base and descendants */
  unsigned int mask_gripper_bodies; /* robotiq_base_mount and descendants */
  /* get_mug_toppled threshold: max(dx, dy) of the first fish geom */
  double fish_topple_z;
  /* gym_utils.get_table_collision's table body (-1 when absent) */
  int id_body_table;
  /* get_body_size(m, "fish")[-1]: half height of the first fish geom (ur3e_env.py compute_reward) */
  double fish_half_z;
  /* all sensors in declaration order: mjData.sensordata[sensor_adr[k] ..] holds sensor k */
  int nsensor, nsensordata;
  int sensor_type[UR3E_MAXSENSOR];
  int sensor_objid[UR3E_MAXSENSOR]; /* site (touch, torque) or actuator (actuatorfrc) */
  int sensor_adr[UR3E_MAXSENSOR];
  /* convex mesh geoms (geom_type UR3E_GEOM_MESH, compiled when the MJCF's mesh files exist): each
     mesh's convex-hull vertices in its geom frame, which is the mesh's inertial frame (MuJoCo
     re-expresses a mesh about its centre of mass and principal axes); geom_dataid = mesh index */
  int nmesh, nmeshvert;
  int geom_dataid[UR3E_MAXGEOM];
  int mesh_vertadr[UR3E_MAXMESH];
  int mesh_vertnum[UR3E_MAXMESH];
  double mesh_vert[UR3E_MAXMESHVERT][3];
} ur3e_model_t;

#ifdef __cplusplus
}
#endif
#endif /* UR3E_MODEL_H */
