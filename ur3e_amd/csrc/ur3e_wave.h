/*
 * ur3e_wave.h — v2 step engine: ONE WORKGROUP (NT = 64 or 128 lanes) PER ENV,
 * the env's whole working set staged in LDS (KS, ~77 KB: two envs per CU).
 *
 * Why: the v1 layout (one env per lane, ~80 KB lane-private scratch) spills to
 * HBM — rocprofv3 measured ~330 KB of fetches per env-step and every dependent
 * access waiting on a miss (profiles/r01_v1_lane_per_env).  Here the same
 * arithmetic runs as cooperative lane-parallel stages over LDS:
 *   - tree passes (kinematics, com velocity, RNE forward) run level by level,
 *     one lane per body; subtree accumulations run one lane per component;
 *   - mass matrix rows, constraint row groups, collision candidates, Hessian
 *     elements, Newton vectors: one lane per output element;
 *   - the tree LDL' and both triangular solves run as column sweeps;
 *   - every serial reduction the oracle performs in a given order (costs,
 *     line-search sums, norms) is done by lane 0 over per-row contributions
 *     staged in LDS, in the oracle's order.
 * Parallelising over OUTPUT elements only, never splitting a sum, keeps every
 * result bit-identical to the CPU oracle (oracle/ur3e_oracle.c).
 *
 * Semantics: MuJoCo 3.3.3 mj_step (see ur3e_engine.h for the stage list) as
 * driven by gymnasium_env/envs/ur3e_env2.py:72-99.
 */
#ifndef UR3E_WAVE_H
#define UR3E_WAVE_H

#include "ur3e_engine.h"
#include "gen_main_tree.h"

#define W_MAXCAND 128 /* collision candidates handled per env (main.xml: 92) */
/* mesh-capable layouts (main.xml with its convex meshes: 24 colliding geoms, 234 candidate pairs) */
#define K_NG_MESH 24
#define W_MAXCAND_MESH 240
/* survivors of the bounding-sphere filter the overlaid (compact / grasp) layouts hold; an env-step with
   more hands on to the next tier */
#define W_MAXSURV 64
#define W_MAXGRP 96   /* constraint row groups */
/* the overlaid layouts' row groups beyond their contacts (equality and frictionloss groups of the plan, active
   joint limits): with W_ROWS_IN_HL, an env-step with more groups than MAXCON + this hands on to the next tier
   (r_mc_layout) */
#ifndef W_GRP_EXTRA
#define W_GRP_EXTRA 24
#endif
/* the 64+-row overlaid layouts keep the rows' R / D / aref, the Newton Hessian and the solved forces in one
   union of the constraint area, and their group arrays sized by contacts (1), or side by side (0, default).
   1 takes the mid tier from 25.2 to 22.9 KB of LDS, seven envs per CU instead of six, bit-exact, and measured
   0.6-1.2 % slower on the scripted pick (profiles/r06_ab A/B 7): its envs fit the chip at six per CU already */
/* the Newton Hessian build's first-tree slot skip (ur3e_wave_r.h; 0, default: A/B 9) */
#ifndef W_T2_SKIP
#define W_T2_SKIP 0
#endif
#ifndef W_ROWS_IN_HL
#define W_ROWS_IN_HL 0
#endif
/* compact-tier narrowphase: survivor lanes per chunk (their clip polygons live in LDS) and staged
   raw contacts per chunk (>= the compact tier's MAXCON: a chunk staging more has overflowed) */
#define W_NP_LANES 8
#define W_NP_STAGE 16

/* host-precomputed tree bookkeeping for the cooperative stages */
/* stage-timing marks of the -DUR3E_STAGE_TIMING build (tools/stage_timing.py) */
#define W_NSTAGE_MARKS 50

#define W_HB_NQ ((K_NV * (K_NV + 1) / 2 + 63) / 64)
/* the Newton direction's element slots from the plan (1, default) or solved per call (0: A/B) */
#ifndef W_HB_MAP
#define W_HB_MAP 1
#endif
#define W_CS_DOF UR3E_MAXEQ
#define W_CS_JNT (UR3E_MAXEQ + K_NV)
#define W_CS_PAIR (UR3E_MAXEQ + K_NV + K_NJ)
#define W_NCS (W_CS_PAIR + UR3E_MAXCPAIR)

struct KPlan {
  int nlevel;
  int body_depth[K_NB];
  unsigned int dof_anc_mask[K_NV]; /* bit j: j is a proper ancestor of dof i */
  int dof_nanc[K_NV];
  int dof_anc[K_NV][K_NV];         /* proper ancestors, nearest first */
  unsigned int body_dof_mask[K_NB];
  int nfloss;
  int floss_dof[K_NV];
  int neq_rows;
  int max_jntnum; /* joints on the busiest body (the compact tier's body passes need <= 1) */
  /* row groups that exist every step (equality, then frictionloss), in oracle order */
  int nfixgrp, nfixrow;
  int fix_type[UR3E_MAXEQ + K_NV], fix_id[UR3E_MAXEQ + K_NV], fix_row[UR3E_MAXEQ + K_NV];
  /* actuator moment arm per dof (mj_transmission: gear for a joint transmission, coef * gear for
     each dof of a fixed tendon, 0 elsewhere); model constants, so computed once on the host */
  double act_moment[K_NU][K_NV];
  int ten_qadr[UR3E_MAXTEN][UR3E_MAXTENWRAP]; /* qpos address of each fixed-tendon dof */
  /* per body, its first joint's constants (joint 0's for a body without joints, as the passes
     index it), and per joint its body's root: the compact tier's body passes then load every model
     constant one level deep instead of through body -> joint -> qpos index chains */
  int bj_type[K_NB], bj_qadr[K_NB];
  double bj_q0[K_NB], bj_axis[K_NB][3], bj_pos[K_NB][3];
  int jnt_root[K_NJ];
  /* constraint sources of the compact tier's row groups (r_mc_rows), one row per source -- equality e,
     frictionloss dof W_CS_DOF + v, joint limit W_CS_JNT + j, contact pair W_CS_PAIR + p -- with every
     index chain of the group data resolved on the host, so a group loads its constants one level deep:
       cs_i: connect / contact: body roots 1, 2 and body dof masks 1, 2; joint equality: dof 1, dof 2
             (-1: none), qpos address 1, 2; limit: dof, limited hinge / slide (1 / 0), qpos address, -;
       cs_d: solref[2], solimp[5], diag (the sum of the two invweights where there are two, in the
             device's order), margin (contact: margin - gap), qpos0 at address 1 | range low,
             qpos0 at address 2 | range high */
  int cs_i[W_NCS][4];
  double cs_d[W_NCS][11];
  /* collision candidates (the overlaid layouts' broadphase and narrowphase), one row per pair with its
     geoms' constants: pr_i = geom 1, geom 2, type 1, type 2; pr_d = margin, rbound 1, rbound 2, size 1[3],
     size 2[3] */
  int pr_i[UR3E_MAXCPAIR][4];
  double pr_d[UR3E_MAXCPAIR][9];
  /* the epilogue's velocity sites (tcp, handle): body and its root (-1: no such site) */
  int sv_body[2], sv_root[2];
  /* per dof, the passive forces' constants: pd_i = body, spring qpos address; pd_d = stiffness where
     the dof's joint has a spring term (hinge or slide, its first dof; else 0), qpos_spring there, damping */
  int pd_i[K_NV][2];
  double pd_d[K_NV][3];
  /* per actuator: pa_i = ctrllimited, affine bias, forcelimited, qpos address of a joint transmission
     (-1: tendon); pa_d = ctrlrange[2], gainprm[0], biasprm[0..2], forcerange[2], gear */
  int pa_i[K_NU][4];
  double pa_d[K_NU][9];
  /* per equality: connect (1 / 0), body 1, body 2 */
  int eqc_i[UR3E_MAXEQ][3];
  /* the kinematics' frames, geoms then sites: body, pos[3], quat[4] */
  int fr_b[UR3E_MAXGEOM + UR3E_MAXSITE];
  double fr_d[UR3E_MAXGEOM + UR3E_MAXSITE][7];
  /* the Newton direction's element slots (r_direction): lane l, slot q holds lower-triangle element
     (k, c) at packed index p, for the dense [0] and the block-diagonal [1] Hessian (UR3E_MAIN_SPLIT):
     k | c << 8 | p << 16 | valid << 24; an invalid slot's p is the lane's slot-0 element */
  int hb_map[2][64][W_HB_NQ];
};
/* the per-dof / per-actuator / per-equality plan rows of com_pos and the passive and actuator forces
   (1, default) or the model's index chains (0: A/B) */
#ifndef W_FLAT_DYN
#define W_FLAT_DYN 1
#endif

/* constraint row groups (one lane builds one group) */
#define G_CONNECT 0
#define G_JOINTEQ 1
#define G_FLOSS 2
#define G_LIMIT 3
#define G_CONTACT 4

/* ---- the overlaid layouts' narrowphase area (KN) ---- */
/* convex meshes in the overlaid layouts (ur3e_cvx_wave.h): one wave settles one mesh pair at a time, its
   GJK simplex and EPA polytope in this LDS work area (wave-uniform state) */
#define WC_MAXV UR3E_EPA_MAXV
#define WC_MAXF UR3E_EPA_MAXF
#define WC_MAXE 64 /* horizon edges of one EPA step held in LDS (convex.h: 3 * UR3E_EPA_MAXF) */
#define WC_FSLOT ((WC_MAXF + 63) / 64)

/* LDS work area of one mesh pair (wave-uniform state) */
struct WCvxWork {
  /* GJK simplex: support points of A - B, A and B, and the closest point's barycentric weights */
  double sw[4][3], sa[4][3], sb[4][3], slam[4];
  int sn;
  /* EPA polytope: vertices (w = a - b, recomputed with convex.h's operation), faces */
  double pa[WC_MAXV][3], pb[WC_MAXV][3];
  double fn[WC_MAXF][3], fd[WC_MAXF];
  int fv[WC_MAXF]; /* i | j << 8 | k << 16, bit 24: alive */
  int edge[WC_MAXE]; /* horizon edge i | j << 8 */
  int pnv, pnf, ne;
  /* plane–convex selection */
  double psd[UR3E_CVX_PLANE_MAX];
  int psel[UR3E_CVX_PLANE_MAX];
};

/* one mesh pair's raw contacts, per survivor slot (filled by the mesh pass before the chunked
   narrowphase, which emits them at the pair's place in candidate order) */
template <int MC>
struct WMeshRes {
  double raw[MC][7]; /* pos[3], n[3], dist */
  signed char cnt[W_MAXSURV];
  unsigned char at[W_MAXSURV];
  int nraw;
};

/* the chunked narrowphase's clip polygons of one chunk of survivor lanes ([buf][vertex][coord][lane],
   conflict-free across lanes) and that chunk's staged raw contacts; the mesh-capable layouts also hold
   the mesh pass's results (alive through the chunks) and its work area (dead by then, so it shares the
   chunk buffers' bytes) */
template <int NPST>
struct KNChunk {
  double np_clip[2][8][3][W_NP_LANES];
  double np_stage[7][NPST]; /* pos[3], n[3], dist */
  int np_key[NPST];         /* survivor lane * 8 + contact index within the lane */
  int np_nstage;
};
template <int NPST, int MC, bool MESH>
struct KNArea : KNChunk<NPST> {
  __device__ __forceinline__ KNChunk<NPST>& chunk() { return *this; }
};
template <int NPST, int MC>
struct KNArea<NPST, MC, true> {
  union {
    KNChunk<NPST> ch;
    WCvxWork cw;
  };
  WMeshRes<MC> mres;
  __device__ __forceinline__ KNChunk<NPST>& chunk() { return ch; }
};

/* Two LDS layouts.  The full-capacity tier (rows > 64, KSL) keeps every array side by side.  The
   compact tier (rows <= 64: one 64-lane wavefront, register-resident solver) overlays the arrays
   of the position/velocity stages with those of the constraint stages, see the specialisation
   below. */
template <int MC, int ME, int NVC = 0, int TREE = 0, bool OVERLAY = (ME <= 64), int NGC = K_NG>
struct KSX;

template <int MC, int ME, int NVC, int TREE, int NGC>
struct KSX<MC, ME, NVC, TREE, false, NGC> {
  static constexpr bool OVERLAY = false;
  static constexpr bool RHL = false; /* separate row arrays (see the overlaid layout) */
  /* geoms this layout holds; NGC = K_NG_MESH: the mesh-capable variant (main.xml with real meshes) */
  static constexpr int NG = NGC;
  static constexpr bool MESHES = NGC == K_NG_MESH;
  static constexpr int NCAND = MESHES ? W_MAXCAND_MESH : W_MAXCAND;
  static constexpr int NV = NVC;    /* > 0: kernel specialised for a model with exactly NVC dofs */
  static constexpr int STATIC_TREE = TREE; /* 1: main.xml's dof tree as compile-time tables */
  static constexpr int MAXCON = MC; /* contacts this tier holds */
  static constexpr int MAXEFC = ME; /* constraint rows this tier holds */
  static constexpr int MAXGRP = ME < W_MAXGRP ? ME : W_MAXGRP;
  /* a tier smaller than the oracle's capacity never clamps: it flags the env
     (ovf) and the env-step is recomputed by the full-capacity tier */
  static constexpr bool BAIL = (MC < K_MAXCON) || (ME < K_MAXEFC);
  /* state */
  double qpos[K_NQ], qvel[K_NV], warm[K_NV], ctrl[K_NU];
  /* position stage */
  double xpos[K_NB][3], xquat[K_NB][4], xmat[K_NB][9];
  double xanchor[K_NJ][3], xaxis[K_NJ][3];
  double geom_xpos[NGC][3], geom_xmat[NGC][9];
  double site_xpos[K_NS][3], site_xmat[K_NS][9];
  double subtree_com[K_NB][3], cinert[K_NB][10], cdof[K_NV][6];
  double cvel[K_NB][6], cdof_dot[K_NV][6];
  double actuator_length[K_NU], act_force[K_NU];
  double qM[K_NV][K_NV], LDinv[K_NV];
  double H[K_NV][K_NV]; /* Newton Hessian; also holds the tree factor of M before Newton (qLD) */
  double qloc[K_NJ][4];
  /* vectors */
  double qfrc_bias[K_NV], qfrc_passive[K_NV], qfrc_smooth[K_NV], qacc_smooth[K_NV], qacc[K_NV];
  double qfrc_constraint[K_NV], Ma[K_NV], grad[K_NV], search[K_NV], Mv[K_NV], xv[K_NV], fv[K_NV];
  double tmpv[K_NV];
  /* body temporaries (crb / cacc / cfrc) aliased with per-row Newton temporaries */
  union {
    struct {
      double b10[K_NB][10];
      double b6[K_NB][6];
    } body;
    struct {
      double F[ME], dF[ME], d2F[ME];
    } row;
  } u;
  /* contacts */
  double con_pos[MC][3], con_frame[MC][9], con_dist[MC], con_mu[MC];
  double con_Hc[MC][9];
  int con_geom1[MC], con_geom2[MC], con_cpair[MC], con_efc[MC];
  int cand_count[NCAND], cand_off[NCAND];
  /* constraint rows */
  double efc_J[ME][K_NV];
  double efc_R[ME], efc_D[ME], efc_aref[ME], efc_floss[ME];
  double efc_force[ME], jar[ME], Jv[ME];
  int efc_type[ME], efc_id[ME], efc_state[ME], rowflag[ME], efc_grp[ME];
  int grp_type[MAXGRP], grp_id[MAXGRP], grp_row[MAXGRP];
  double touch[UR3E_MAXTOUCH];
  /* sensors (ur3e_config_t.sensors): mjData.sensordata and mj_rnePostConstraint's body quantities */
  double sensordata[UR3E_MAXSENSORDATA];
  double cacc[K_NB][6], cfrc_int[K_NB][6], cfrc_ext[K_NB][6];
  int sens;
  double carry[NCARRY]; /* the stale-kinematics carry: read by the controller, rebuilt after the last forward */
  /* scalars */
  double gauss, cost, scale, g1, g2, lsF, lsdF, lsd2F, sred;
  int ncon, nefc, ngrp, nwarn, flag, ovf, cap_con;
  unsigned long long tlast;
#ifdef UR3E_STAGE_TIMING
  unsigned long long tacc[W_NSTAGE_MARKS];
  unsigned int tcnt[W_NSTAGE_MARKS];
#endif
};

/* Compact-tier layout (one 64-lane wavefront per env), sized so that EIGHT envs fit the 160 KB
   of LDS of a CU (<= 20 KB each, two wavefronts per SIMD).  w_forward runs its stages in the order
     kinematics -> com_pos -> crb -> com_vel/RNE/passive/actuation -> collision -> constraint rows
     -> M^-1 qfrc_smooth -> Newton -> touch -> Euler,
   and the arrays are grouped by lifetime:
     - outside the union: what survives a substep or is read by the epilogue / carry (state, body
       and site positions, com quantities, packed qM, contacts, dof vectors) plus three small
       values precomputed so that their inputs can die early: the connect-constraint anchors
       (eq_p, from xmat), the tcp/handle site velocities (site_vel, from cvel) and the unit
       contact normals (con_n; the rest of the contact frame is rebuilt from it, bit for bit);
     - KC, kinematics .. collision: geom poses, collision candidates;
     - KA, kinematics .. com_pos: body orientations, joint axes/anchors (overlaid with KB);
     - KB, com_pos .. RNE: cinert, cvel, cdof_dot, crb/cacc/cfrc, actuation;
     - N, constraint rows .. Euler: Jacobian and row data, cone Hessians, the packed Newton
       Hessian / tree-factor scratch (the register solver only touches j <= i).
   Only the fields the compact code path touches exist here. */
#define KTRI(i, j) ((i) * ((i) + 1) / 2 + (j))
template <int MC, int ME, int NVC, int TREE, int NGC>
struct KSX<MC, ME, NVC, TREE, true, NGC> {
  static constexpr bool OVERLAY = true;
  static constexpr int NG = NGC;
  static constexpr bool MESHES = NGC == K_NG_MESH;
  /* candidate pairs: only the bounding-sphere survivors are listed (W_MAXSURV; more bail) */
  static constexpr int NCAND = MESHES ? W_MAXCAND_MESH : W_MAXCAND;
  static constexpr int NV = NVC;
  static constexpr int STATIC_TREE = TREE;
  static constexpr int MAXCON = MC;
  static constexpr int MAXEFC = ME;
  /* each group holds a row, so ME bounds the groups; with W_ROWS_IN_HL, in the layouts of 64+ rows, so do the
     contacts plus W_GRP_EXTRA (r_mc_layout bails beyond it) */
  static constexpr int MAXGRP0 = ME < W_MAXGRP ? ME : W_MAXGRP;
  static constexpr int MAXGRP = (W_ROWS_IN_HL && ME >= 64 && MC + W_GRP_EXTRA < MAXGRP0) ? MC + W_GRP_EXTRA : MAXGRP0;
  static constexpr bool BAIL = (MC < K_MAXCON) || (ME < K_MAXEFC);
  /* constraint rows per lane of the register solver: row r lives on lane r % 64, slot r / 64 */
  static constexpr int RPL = (ME + 63) / 64;
  /* the rows' R / D / aref, Hl and the solved forces share bytes (W_ROWS_IN_HL) in the layouts whose envs
     per CU their LDS bounds (the mid and grasp tiers, 64+ rows); the compact tiers are bound by registers */
  static constexpr bool RHL = W_ROWS_IN_HL && ME >= 64;
  /* raw contacts one narrowphase chunk may stage (a chunk staging more has overflowed MAXCON) */
  static constexpr int NPST = MC > W_NP_STAGE ? MC : W_NP_STAGE;
  static_assert(RPL <= 2 && MC <= 64, "the register solver holds at most two rows per lane");
  /* ---- live for the whole env-step ---- */
  double qpos[K_NQ], qvel[K_NV], warm[K_NV], ctrl[K_NU];
  double xpos[K_NB][3];
  double site_xpos[K_NS][3], site_xmat[K_NS][9];
  double subtree_com[K_NB][3], cdof[K_NV][6];
  double qMp[K_NV * (K_NV + 1) / 2]; /* mass matrix, packed lower triangle */
  double qfrc_bias[K_NV], qfrc_smooth[K_NV], qacc_smooth[K_NV], qacc[K_NV], qfrc_constraint[K_NV];
  double con_pos[MC][3], con_n[MC][3], con_dist[MC], con_mu[MC];
  int con_geom1[MC], con_geom2[MC], con_cpair[MC], con_efc[MC];
  double touch[UR3E_MAXTOUCH];
  double eq_p[UR3E_MAXEQ][6];  /* connect anchors p1, p2 in world coordinates */
  double act_force[K_NU];      /* mjData.actuator_force of the last forward (committed: get_jnt_torques) */
  double site_vel[2][6];       /* [tcp, handle] mj_objectVelocity (world, [w, v]) */
  int ncon, nefc, ngrp, nwarn, flag, ovf, cap_con;
  int bdiag; /* static tree: no constraint row couples the two dof trees (set by r_mc_rows) */
  int np_lanes; /* survivor lanes per narrowphase chunk (KConfig.np_lanes, <= W_NP_LANES) */
  unsigned long long tlast;
#ifdef UR3E_STAGE_TIMING
  unsigned int tacc[W_NSTAGE_MARKS]; /* 32-bit: keeps the timing build's layout near 20 KB (with MAXCON 9) */
  unsigned int tcnt[W_NSTAGE_MARKS];
#endif
  union {
    struct {
      /* KC */
      double geom_xpos[NGC][3], geom_xmat[NGC][9];
      int cand_off[W_MAXSURV]; /* bounding-sphere survivors, in candidate order */
      union {
        struct { /* KA */
          double xquat[K_NB][4], xmat[K_NB][9];
          double xanchor[K_NJ][3], xaxis[K_NJ][3], qloc[K_NJ][4];
        };
        struct { /* KB */
          double cinert[K_NB][10], cvel[K_NB][6];
          double actuator_length[K_NU], qfrc_passive[K_NV];
          /* body temporaries by lifetime: the composite inertia (crb) for the mass matrix; then cacc and
             cdof_dot in the velocity / acceleration pass; then cacc and cfrc in RNE, cfrc over the dead
             cdof_dot (w_crb, w_cacc, w_cdof_dot, w_cfrc pick the arrays in either layout) */
          union {
            struct { double b10[K_NB][10]; } crb;
            struct { double cacc[K_NB][6]; double cdof_dot[K_NV][6]; } va;
            struct { double cacc[K_NB][6]; double cfrc[K_NB][6]; } rne;
          } u;
        };
        KNArea<NPST, MC, MESHES> kn; /* KN, collision (above) */
      };
    };
    struct { /* CR: the stale-kinematics carry, alive only before the first forward (the controller reads it)
                and after the last (rebuilt for the commit), when nothing else in the union is */
      double carry[NCARRY];
    };
    struct { /* N */
      double efc_J[ME][K_NV];
      int efc_type[ME], efc_id[ME], efc_grp[ME];
      int grp_type[MAXGRP], grp_id[MAXGRP], grp_row[MAXGRP];
#if W_T2_SKIP
      /* static tree: per row slot, the rows with no nonzero in the first dof tree (r_mc_rows, for the Hessian
         build's slot skip) */
      unsigned long long t2rows[RPL];
#endif
      double con_Hc[MC][9];
      /* RHL: by lifetime, the rows' regulariser, its inverse and reference acceleration from
         w_make_constraint until r_load_rows copies them into the solver's registers; then the Newton
         Hessian, its factor and (RPL 1) the ordered-sum slots; then the solved forces, which only the touch
         sensors read before the implicit-damping tree solve reuses the bytes.  The smooth acceleration's
         tree solve, which uses Hl too, then runs before the rows are made (w_forward).  Without RHL the
         three lie side by side (the pads are empty with it) */
      union {
        struct { double efc_R[ME], efc_D[ME], efc_aref[ME]; };
        struct { double rhl_pad0_[RHL ? 0 : 3 * ME]; double Hl[K_NV * (K_NV + 1) / 2]; };
        struct { double rhl_pad1_[RHL ? 0 : 3 * ME + K_NV * (K_NV + 1) / 2]; double efc_force[ME]; };
      };
      /* ordered-sum slots of the register solver when rows span two lanes' slots (RPL 2); with
         RPL 1 the three 64-double slots live in Hl (see R_SLOT) */
      double rslot[RPL > 1 ? 3 * 64 * RPL : 1];
    };
  };
};

/* the body temporaries in either layout (the overlaid one packs them by lifetime) */
template <class S>
__device__ __forceinline__ auto w_crb(S& s) {
  if constexpr (std::remove_const_t<S>::OVERLAY) return s.u.crb.b10;
  else return s.u.body.b10;
}
template <class S>
__device__ __forceinline__ auto w_cacc(S& s) {
  if constexpr (std::remove_const_t<S>::OVERLAY) return s.u.va.cacc;
  else return s.u.body.b10;
}
template <class S>
__device__ __forceinline__ auto w_cdof_dot(S& s) {
  if constexpr (std::remove_const_t<S>::OVERLAY) return s.u.va.cdof_dot;
  else return s.cdof_dot;
}
template <class S>
__device__ __forceinline__ auto w_cfrc(S& s) {
  if constexpr (std::remove_const_t<S>::OVERLAY) return s.u.rne.cfrc;
  else return s.u.body.b6;
}

/* mass-matrix element (i, j) in either layout */
template <class KS>
__device__ __forceinline__ double qm_get(const KS& s, int i, int j) {
  if constexpr (KS::OVERLAY) return s.qMp[i >= j ? KTRI(i, j) : KTRI(j, i)];
  else return s.qM[i][j];
}
/* the overlaid layouts' packed mass-matrix element (row, j) for loops over a compile-time j: the byte
   offset is a per-row base plus a constant either side of the diagonal (rb + 8 j for j <= row, by symmetry
   8 row + 8 KTRI(j, 0) for j > row), and the right one is always the larger (T(row) + j >= T(j) + row
   exactly when j <= row, T(n) = n (n + 1) / 2; equal offsets are the same element): two adds and a max per
   element instead of the max / min / multiply of KTRI(max, min), and no per-element compare mask; the same
   element as qm_get(s, row, j) */
struct QmIx {
  int rb, rc, row;
};
__device__ __forceinline__ QmIx qm_ix(int row) { return QmIx{8 * KTRI(row, 0), 8 * row, row}; }
template <class KS>
__device__ __forceinline__ double qm_at(const KS& s, const QmIx& q, int j) {
  const int a = q.rb + 8 * j, b = q.rc + 8 * KTRI(j, 0);
  const int off = a > b ? a : b;
  return *reinterpret_cast<const double*>(reinterpret_cast<const char*>(s.qMp) + off);
}
/* full-capacity tier: the oracle's limits (UR3E_MAXCON contacts, UR3E_MAXEFC rows) */
typedef KSX<K_MAXCON, K_MAXEFC> KSL;
/* compact tier: sized for the gym workload on main.xml -- the mug resting on the table (4 contacts,
   13 fixed rows + 3 per contact = 25) plus joint-limit rows (25-27 rows over random-action rollouts,
   tools/contact_hist.py) -- with room for one more contact, so that the working set stays under
   16 KB: ten envs per CU.  Env-steps beyond it (grasps, arm contacts) run in the grasp tier. */
#ifndef W_SMALL_MAXCON
#define W_SMALL_MAXCON 5
#endif
#ifndef W_SMALL_MAXEFC
#define W_SMALL_MAXEFC 30
#endif
typedef KSX<W_SMALL_MAXCON, W_SMALL_MAXEFC> KSS;
/* compact tier specialised for main.xml: compile-time dof count and dof tree (gen_main_tree.h),
   so dof loops have constant trip counts and tree tests fold away */
typedef KSX<W_SMALL_MAXCON, W_SMALL_MAXEFC, UR3E_MAIN_NV, 1> KSS_NV;
/* the compact tier of the scripted pick (move_l_mug, TRAJ_L): its approach and release rows see 5-8
   contacts, which the gym tier would route to the grasp tier (measured: C3 5.9 M env-steps/s at 5/30
   against 8.0 M at 10/44; the gym workload the other way round, 8.07 M against 7.84 M) */
#ifndef W_WIDE_MAXCON
#define W_WIDE_MAXCON 10
#endif
#ifndef W_WIDE_MAXEFC
#define W_WIDE_MAXEFC 44
#endif
typedef KSX<W_WIDE_MAXCON, W_WIDE_MAXEFC, UR3E_MAIN_NV, 1> KSS_NV_W;
static_assert(UR3E_MAIN_NV <= K_NV, "main.xml dofs exceed K_NV");
/* grasp tier, between the compact and the full-capacity tier: the compact tier's code path (overlaid
   LDS layout, register-resident solver with two rows per lane) sized for a firm grasp of the
   box-surrogate pads, where main.xml reaches 12-20 contacts (C3 grasp and carry rows,
   tools/contact_hist.py); its bails go on to the full-capacity tier */
#ifndef W_GRASP_MAXCON
#define W_GRASP_MAXCON 24
#endif
#ifndef W_GRASP_MAXEFC
#define W_GRASP_MAXEFC 96
#endif
typedef KSX<W_GRASP_MAXCON, W_GRASP_MAXEFC, UR3E_MAIN_NV, 1, true> KSG_NV;
/* the same three tiers for main.xml with its convex meshes (K_NG_MESH geoms, W_MAXCAND_MESH candidate
   pairs): the compact and grasp tiers settle a mesh pair whose hulls GJK finds separated beyond the
   margin themselves (no contact, the oracle's decision with the same code) and hand on an env-step whose
   mesh pair touches; the full-capacity tier runs GJK + EPA */
typedef KSX<W_SMALL_MAXCON, W_SMALL_MAXEFC, UR3E_MAIN_NV, 1, true, K_NG_MESH> KSS_NV_M;
/* the mesh model's grasp tier.  18 contacts / 72 rows (30.3 KB, built for two waves per SIMD: five envs per CU
   instead of four) was measured +2.7 % on the C3 mesh pick without the mid tier (profiles/r06_ab A/B 1), but
   the scripted pick's grasp rows reach beyond it in a few envs (the full-capacity tier took 0.1 % of rows
   2,100-2,600, which cost that window 12 %); with the mid tier taking the carry's 16-contact states, the grasp
   tier only serves the rarer larger ones, so it keeps the box model's 24 / 96 (A/B 3) */
#ifndef W_GRASP_MESH_MAXCON
#define W_GRASP_MESH_MAXCON W_GRASP_MAXCON
#endif
#ifndef W_GRASP_MESH_MAXEFC
#define W_GRASP_MESH_MAXEFC W_GRASP_MAXEFC
#endif
typedef KSX<W_GRASP_MESH_MAXCON, W_GRASP_MESH_MAXEFC, UR3E_MAIN_NV, 1, true, K_NG_MESH> KSG_NV_M;
/* mid tier, between the compact and the grasp tier: 16 contacts / 64 rows -- one constraint row per lane, so
   the register solver of the compact tier (RPL 1) instead of the grasp tier's two rows per lane -- in a 25.2 KB
   layout built for two waves per SIMD: six envs per CU.  It takes the routed env-steps that fit it, which on
   the scripted pick are the closed gripper's carry states (16 contacts, 62-63 rows, 28 % of the envs; the
   grasp tier's 18/72 and 24/96 run them at five and four per CU with twice the row work per lane); its bails
   join the grasp tier's pre-pass list. */
#ifndef W_MID_MAXCON
#define W_MID_MAXCON 16
#endif
#ifndef W_MID_MAXEFC
#define W_MID_MAXEFC 64
#endif
typedef KSX<W_MID_MAXCON, W_MID_MAXEFC, UR3E_MAIN_NV, 1, true> KSM_NV;
typedef KSX<W_MID_MAXCON, W_MID_MAXEFC, UR3E_MAIN_NV, 1, true, K_NG_MESH> KSM_NV_M;
typedef KSX<K_MAXCON, K_MAXEFC, 0, 0, false, K_NG_MESH> KSL_M;
/* the scripted pick's wider compact tier (10 contacts / 44 rows) with the mesh geoms: its carry rows hold the
   mug on the table, the pads and the closed fingers' linkage meshes (7-8 contacts) */
typedef KSX<W_WIDE_MAXCON, W_WIDE_MAXEFC, UR3E_MAIN_NV, 1, true, K_NG_MESH> KSS_NV_MW;
#define NVOF(KS, m) ((KS::NV) ? (KS::NV) : (m)->nv)

/* Barrier between cooperative phases.  With one 64-lane wavefront per env (NT == 64) the
   wave's LDS instructions issue and complete in program order, so cross-lane LDS hand-offs only
   need a compiler fence (no s_barrier, no workgroup fence); with NT == 128 the two waves need a
   real workgroup barrier. */
template <int NT>
__device__ __forceinline__ void wsync() {
  if constexpr (NT == 64) {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  } else {
    __syncthreads();
  }
}
#define SYNC() wsync<NT>()
#define SYNC64() wsync<64>()

/* any lane of the workgroup has pred set (uniform result) */
template <int NT>
__device__ __forceinline__ int w_any(int pred) {
  if constexpr (NT == 64) {
    return __ballot(pred) != 0;
  } else {
    return __syncthreads_or(pred);
  }
}
#define WD __device__ static __forceinline__

/* diagnostic build only (-DUR3E_STAGE_TIMING): per-stage shader-clock cycles, lane 0 of every env */
#ifdef UR3E_STAGE_TIMING
/* [tier][stage]: tier 0 compact (KS::MAXCON <= W_SMALL_MAXCON), 1 grasp (other overlaid layouts),
   2 full capacity */
__device__ unsigned long long ur3e_stage_cycles[3][W_NSTAGE_MARKS];
__device__ unsigned long long ur3e_stage_calls[3][W_NSTAGE_MARKS];
#define W_TIER_OF(s)                                                                          \
  (std::remove_reference_t<decltype(s)>::MAXCON <= W_SMALL_MAXCON                           \
       ? 0                                                                                   \
       : (std::remove_reference_t<decltype(s)>::OVERLAY ? 1 : 2))
/* accumulated per wave in LDS and flushed once at kernel end: a global atomic per mark would sit in
   the wave's vmcnt queue and bill its (contended) latency to the next stage that loads from memory */
#define WT(k)                                                           \
  do {                                                                  \
    if (w_lane() == 0) {                                             \
      unsigned long long _t = __builtin_amdgcn_s_memtime();            \
      s.tacc[k] += _t - s.tlast;                                        \
      s.tcnt[k] += 1;                                                   \
      s.tlast = _t;                                                     \
    }                                                                   \
  } while (0)
#define WT_START()                                                      \
  do {                                                                  \
    if (w_lane() == 0) s.tlast = __builtin_amdgcn_s_memtime();       \
  } while (0)
#define WT_INIT()                                                       \
  do {                                                                  \
    if (w_lane() < W_NSTAGE_MARKS) { s.tacc[w_lane()] = 0; s.tcnt[w_lane()] = 0; } \
  } while (0)
#define WT_FLUSH()                                                      \
  do {                                                                  \
    __builtin_amdgcn_wave_barrier();                                    \
    if (w_lane() < W_NSTAGE_MARKS && s.tcnt[w_lane()]) {          \
      atomicAdd(&ur3e_stage_cycles[W_TIER_OF(s)][w_lane()], (unsigned long long)s.tacc[w_lane()]);  \
      atomicAdd(&ur3e_stage_calls[W_TIER_OF(s)][w_lane()], (unsigned long long)s.tcnt[w_lane()]); \
    }                                                                   \
  } while (0)
#else
#define WT(k) \
  do {        \
  } while (0)
#define WT_START() \
  do {             \
  } while (0)
#define WT_INIT() \
  do {            \
  } while (0)
#define WT_FLUSH() \
  do {             \
  } while (0)
#endif

#include "ur3e_wave_r.h"
#include "ur3e_cvx_wave.h"

/* ================================================================== */
/* kinematics (level-parallel over bodies)                             */
/* ================================================================== */
template <int NT, class KS>
WD void w_kinematics(KModel m, const KPlan* __restrict__ pl, KS& s) {
  const int tid = w_lane();
  if (tid == 0) {
    s.xpos[0][0] = s.xpos[0][1] = s.xpos[0][2] = 0;
    s.xquat[0][0] = 1; s.xquat[0][1] = s.xquat[0][2] = s.xquat[0][3] = 0;
    k_quat2mat(s.xmat[0], s.xquat[0]);
  }
  /* hinge rotations do not depend on the parent: all joints at once */
  for (int j = tid; j < m->njnt; j += NT) {
    if (m->jnt_type[j] == UR3E_JNT_FREE) continue;
    int a = m->jnt_qposadr[j];
    k_axis_angle_quat(s.qloc[j], m->jnt_axis[j], s.qpos[a] - m->qpos0[a]);
  }
  SYNC();
  const int nb = m->nbody;
  for (int lvl = 1; lvl <= pl->nlevel; lvl++) {
    for (int i = tid; i < nb; i += NT) {
      if (i == 0 || pl->body_depth[i] != lvl) continue;
      int pid = m->body_parentid[i];
      double xpos[3], xquat[4];
      int jfirst = m->body_jntadr[i];
      if (m->body_jntnum[i] == 1 && m->jnt_type[jfirst] == UR3E_JNT_FREE) {
        int a = m->jnt_qposadr[jfirst];
        xpos[0] = s.qpos[a]; xpos[1] = s.qpos[a + 1]; xpos[2] = s.qpos[a + 2];
        xquat[0] = s.qpos[a + 3]; xquat[1] = s.qpos[a + 4]; xquat[2] = s.qpos[a + 5]; xquat[3] = s.qpos[a + 6];
        k_normalize4(xquat);
        s.xanchor[jfirst][0] = xpos[0]; s.xanchor[jfirst][1] = xpos[1]; s.xanchor[jfirst][2] = xpos[2];
        s.xaxis[jfirst][0] = 0; s.xaxis[jfirst][1] = 0; s.xaxis[jfirst][2] = 1;
      } else {
        double t[3];
        k_mat_vec3(t, s.xmat[pid], m->body_pos[i]);
        xpos[0] = s.xpos[pid][0] + t[0]; xpos[1] = s.xpos[pid][1] + t[1]; xpos[2] = s.xpos[pid][2] + t[2];
        k_mul_quat(xquat, s.xquat[pid], m->body_quat[i]);
        for (int k = 0; k < m->body_jntnum[i]; k++) {
          int j = jfirst + k;
          double xaxis[3], xanchor[3], vec[3];
          k_rot_vec_quat(xaxis, m->jnt_axis[j], xquat);
          k_rot_vec_quat(xanchor, m->jnt_pos[j], xquat);
          xanchor[0] += xpos[0]; xanchor[1] += xpos[1]; xanchor[2] += xpos[2];
          k_mul_quat(xquat, xquat, s.qloc[j]);
          k_rot_vec_quat(vec, m->jnt_pos[j], xquat);
          xpos[0] = xanchor[0] - vec[0]; xpos[1] = xanchor[1] - vec[1]; xpos[2] = xanchor[2] - vec[2];
          for (int c = 0; c < 3; c++) { s.xanchor[j][c] = xanchor[c]; s.xaxis[j][c] = xaxis[c]; }
        }
      }
      k_normalize4(xquat);
      for (int c = 0; c < 3; c++) s.xpos[i][c] = xpos[c];
      for (int c = 0; c < 4; c++) s.xquat[i][c] = xquat[c];
      k_quat2mat(s.xmat[i], xquat);
    }
    SYNC();
  }
  for (int g = tid; g < m->ngeom + m->nsite; g += NT) {
    if (g < m->ngeom) {
      int b = m->geom_bodyid[g];
      k_local2global(s.geom_xpos[g], s.geom_xmat[g], s.xpos[b], s.xquat[b], s.xmat[b], m->geom_pos[g],
                     m->geom_quat[g]);
    } else {
      int q = g - m->ngeom;
      int b = m->site_bodyid[q];
      k_local2global(s.site_xpos[q], s.site_xmat[q], s.xpos[b], s.xquat[b], s.xmat[b], m->site_pos[q],
                     m->site_quat[q]);
    }
  }
  SYNC();
}

/* ================================================================== */
/* com_pos: subtree com, cinert, cdof                                  */
/* ================================================================== */
template <int NT, class KS>
WD void w_com_pos(KModel m, const KPlan* __restrict__ pl, KS& s) {
  const int tid = w_lane();
  const int nb = m->nbody;
  double xipos[3] = {0, 0, 0}, ximat[9];
  if (tid < nb) {
    int i = tid;
    if (i == 0) {
      k_quat2mat(ximat, s.xquat[0]);
    } else {
      k_local2global(xipos, ximat, s.xpos[i], s.xquat[i], s.xmat[i], m->body_ipos[i], m->body_iquat[i]);
    }
  }
  if constexpr (NT == 64) {
    /* mass-weighted positions summed up the tree in registers (r_subtree_sum) */
    double sm[3] = {0, 0, 0};
    if (tid < nb) {
      const double mass = m->body_mass[tid];
      sm[0] = xipos[0] * mass; sm[1] = xipos[1] * mass; sm[2] = xipos[2] * mass;
    }
    if constexpr (KS::STATIC_TREE) {
      /* the sums go through subtree_com's rows, components across lanes */
      if (tid < nb)
        for (int k = 0; k < 3; k++) s.subtree_com[tid][k] = sm[k];
      SYNC();
      r_subtree_sum_cols<3, false>(s.subtree_com, s.subtree_com);
      if (tid < nb)
        for (int k = 0; k < 3; k++) sm[k] = s.subtree_com[tid][k];
      SYNC();
    } else {
      r_subtree_sum<3, false>(m, sm);
    }
    if (tid < nb) {
      const int i = tid;
      if (m->body_subtreemass[i] < K_MINVAL) {
        s.subtree_com[i][0] = xipos[0]; s.subtree_com[i][1] = xipos[1]; s.subtree_com[i][2] = xipos[2];
      } else {
        double sc = 1.0 / m->body_subtreemass[i];
        s.subtree_com[i][0] = sm[0] * sc; s.subtree_com[i][1] = sm[1] * sc; s.subtree_com[i][2] = sm[2] * sc;
      }
    }
    SYNC();
    WT(32);
  } else {
    if (tid < nb) {
      int i = tid;
      s.subtree_com[i][0] = xipos[0] * m->body_mass[i];
      s.subtree_com[i][1] = xipos[1] * m->body_mass[i];
      s.subtree_com[i][2] = xipos[2] * m->body_mass[i];
    }
    SYNC();
    if (tid < 3) {
      for (int i = nb - 1; i > 0; i--) s.subtree_com[m->body_parentid[i]][tid] += s.subtree_com[i][tid];
    }
    SYNC();
    if (tid < nb) {
      int i = tid;
      if (m->body_subtreemass[i] < K_MINVAL) {
        s.subtree_com[i][0] = xipos[0]; s.subtree_com[i][1] = xipos[1]; s.subtree_com[i][2] = xipos[2];
      } else {
        double sc = 1.0 / m->body_subtreemass[i];
        s.subtree_com[i][0] *= sc; s.subtree_com[i][1] *= sc; s.subtree_com[i][2] *= sc;
      }
    }
    SYNC();
  }
  for (int j = tid; j < m->njnt; j += NT) {
    int b = m->jnt_bodyid[j];
    int da = m->jnt_dofadr[j];
    const double* c = s.subtree_com[pl->jnt_root[j]];
    double off[3] = {c[0] - s.xanchor[j][0], c[1] - s.xanchor[j][1], c[2] - s.xanchor[j][2]};
    if (m->jnt_type[j] == UR3E_JNT_FREE) {
      for (int k = 0; k < 3; k++) {
        for (int r = 0; r < 6; r++) s.cdof[da + k][r] = 0;
        s.cdof[da + k][3 + k] = 1;
      }
      for (int k = 0; k < 3; k++) {
        double ax[3] = {s.xmat[b][k], s.xmat[b][3 + k], s.xmat[b][6 + k]};
        double cr[3];
        k_cross3(cr, ax, off);
        s.cdof[da + 3 + k][0] = ax[0]; s.cdof[da + 3 + k][1] = ax[1]; s.cdof[da + 3 + k][2] = ax[2];
        s.cdof[da + 3 + k][3] = cr[0]; s.cdof[da + 3 + k][4] = cr[1]; s.cdof[da + 3 + k][5] = cr[2];
      }
    } else {
      double cr[3];
      k_cross3(cr, s.xaxis[j], off);
      s.cdof[da][0] = s.xaxis[j][0]; s.cdof[da][1] = s.xaxis[j][1]; s.cdof[da][2] = s.xaxis[j][2];
      s.cdof[da][3] = cr[0]; s.cdof[da][4] = cr[1]; s.cdof[da][5] = cr[2];
    }
  }
  WT(33);
  if constexpr (KS::OVERLAY) {
    /* connect anchors for the constraint rows (r_mc_rows), while xmat is still alive */
    for (int e = tid; e < m->neq; e += NT) {
      int isc, b1, b2;
      if (W_FLAT_DYN) { isc = pl->eqc_i[e][0]; b1 = pl->eqc_i[e][1]; b2 = pl->eqc_i[e][2]; }
      else { isc = m->eq_type[e] == UR3E_EQ_CONNECT; b1 = m->eq_obj1[e]; b2 = m->eq_obj2[e]; }
      if (!isc) continue;
      double p1[3], p2[3];
      k_mat_vec3(p1, s.xmat[b1], m->eq_data[e]);
      p1[0] += s.xpos[b1][0]; p1[1] += s.xpos[b1][1]; p1[2] += s.xpos[b1][2];
      k_mat_vec3(p2, s.xmat[b2], m->eq_data[e] + 3);
      p2[0] += s.xpos[b2][0]; p2[1] += s.xpos[b2][1]; p2[2] += s.xpos[b2][2];
      for (int k = 0; k < 3; k++) { s.eq_p[e][k] = p1[k]; s.eq_p[e][3 + k] = p2[k]; }
    }
    /* xquat/xmat/xanchor/xaxis (KA) are dead from here; cinert and actuator_length (KB) reuse
       their bytes, so every KA read above must have issued first */
    SYNC();
  }
  if (tid < nb) {
    int i = tid;
    double* r = s.cinert[i];
    if (i == 0) {
      for (int k = 0; k < 10; k++) r[k] = 0;
    } else {
      const double* mat = ximat;
      const double* in = m->body_inertia[i];
      const double* c = s.subtree_com[m->body_rootid[i]];
      double dif[3] = {xipos[0] - c[0], xipos[1] - c[1], xipos[2] - c[2]};
      double mass = m->body_mass[i];
      double tmp[9] = {mat[0] * in[0], mat[3] * in[0], mat[6] * in[0], mat[1] * in[1], mat[4] * in[1],
                       mat[7] * in[1], mat[2] * in[2], mat[5] * in[2], mat[8] * in[2]};
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
  }
  for (int a = tid; a < m->nu; a += NT) {
    double g;
    int qa;
    if (W_FLAT_DYN) { g = pl->pa_d[a][8]; qa = pl->pa_i[a][3]; }
    else { g = m->act_gear[a]; qa = m->act_trntype[a] == UR3E_TRN_JOINT ? m->jnt_qposadr[m->act_trnid[a]] : -1; }
    if (qa >= 0) {
      s.actuator_length[a] = s.qpos[qa] * g;
    } else {
      int t = m->act_trnid[a];
      double len = 0;
      for (int k = 0; k < m->ten_num[t]; k++) len += m->ten_coef[t][k] * s.qpos[pl->ten_qadr[t][k]];
      s.actuator_length[a] = len * g;
    }
  }
  SYNC();
}

/* ================================================================== */
/* CRB mass matrix + tree LDL'                                         */
/* ================================================================== */
template <int NT, class KS>
WD void w_crb(KModel m, const KPlan* __restrict__ pl, KS& s) {
  const int tid = w_lane();
  const int nb = m->nbody, nv = NVOF(KS, m);
  if constexpr (NT == 64) {
    /* composite inertias summed up the tree in registers (lane = body) */
    if constexpr (KS::STATIC_TREE) {
      /* components across lanes: cinert rows in, crb rows out */
      r_subtree_sum_cols<10, true>(s.cinert, w_crb(s));
    } else {
      double crb[10];
      for (int k = 0; k < 10; k++) crb[k] = tid < nb ? s.cinert[tid][k] : 0.0;
      r_subtree_sum<10, true>(m, crb);
      if (tid < nb)
        for (int k = 0; k < 10; k++) w_crb(s)[tid][k] = crb[k];
    }
    WT(34);
  } else {
    for (int e = tid; e < nb * 10; e += NT) w_crb(s)[e / 10][e % 10] = s.cinert[e / 10][e % 10];
  }
  if constexpr (KS::OVERLAY) {
    for (int e = tid; e < nv * (nv + 1) / 2; e += NT) s.qMp[e] = 0;
  } else {
    for (int e = tid; e < nv * nv; e += NT) s.qM[e / nv][e % nv] = 0;
  }
  SYNC();
  if constexpr (NT != 64) {
    if (tid < 10) {
      for (int i = nb - 1; i > 0; i--) {
        int p = m->body_parentid[i];
        if (p > 0) w_crb(s)[p][tid] += w_crb(s)[i][tid];
      }
    }
    SYNC();
  }
  if (tid < nv) {
    int i = tid;
    double buf[6];
    k_mul_inert_vec(buf, w_crb(s)[m->dof_bodyid[i]], s.cdof[i]);
    double mii = m->dof_armature[i];
    mii += k_dot6(s.cdof[i], buf);
    if constexpr (KS::OVERLAY) s.qMp[KTRI(i, i)] = mii;
    else s.qM[i][i] = mii;
    /* ancestors nearest first, from the plan (independent loads instead of a parent-pointer chase) */
    const int na = pl->dof_nanc[i];
    for (int k = 0; k < na; k++) {
      const int j = pl->dof_anc[i][k];
      double v = 0.0;
      v += k_dot6(s.cdof[j], buf);
      if constexpr (KS::OVERLAY) {
        s.qMp[KTRI(i, j)] = v; /* ancestors have lower indices */
      } else {
        s.qM[i][j] = v;
        s.qM[j][i] = v;
      }
    }
  }
  SYNC();
}

/* A (K_NV x K_NV in LDS) -> reverse tree LDL' in place, diaginv */
template <int NT>
WD void w_factor_tree(KModel m, const KPlan* __restrict__ pl, double (*A)[K_NV], double* diaginv,
                                     double* tmp) {
  const int tid = w_lane();
  const int nv = m->nv;
  for (int k = nv - 1; k >= 0; k--) {
    const int na = pl->dof_nanc[k];
    if (na == 0) {
      if (tid == 0 && A[k][k] < K_MINVAL) A[k][k] = K_MINVAL;
      continue;
    }
    if (tid == 0 && A[k][k] < K_MINVAL) A[k][k] = K_MINVAL;
    SYNC();
    if (tid < na) tmp[tid] = A[k][pl->dof_anc[k][tid]] / A[k][k];
    SYNC();
    const int npair = na * (na + 1) / 2;
    for (int e = tid; e < npair; e += NT) {
      int p = 0, rem = e;
      while (rem >= na - p) { rem -= na - p; p++; }
      int q = p + rem;
      int i = pl->dof_anc[k][p], j = pl->dof_anc[k][q];
      A[i][j] -= A[k][j] * tmp[p];
    }
    SYNC();
    if (tid < na) A[k][pl->dof_anc[k][tid]] = tmp[tid];
    SYNC();
  }
  SYNC();
  for (int i = tid; i < nv; i += NT) diaginv[i] = 1.0 / A[i][i];
  SYNC();
}

/* x = A^-1 b with the tree factor; x, b in LDS (may alias) */
template <int NT>
WD void w_solve_tree(KModel m, const KPlan* __restrict__ pl, const double (*A)[K_NV],
                                    const double* diaginv, double* x, const double* b) {
  const int tid = w_lane();
  const int nv = m->nv;
  if (tid < nv) x[tid] = b[tid];
  SYNC();
  for (int i = nv - 1; i >= 0; i--) {
    if (pl->dof_nanc[i] == 0) continue;
    if (tid < nv && ((pl->dof_anc_mask[i] >> tid) & 1u)) x[tid] -= A[i][tid] * x[i];
    SYNC();
  }
  if (tid < nv) x[tid] *= diaginv[tid];
  SYNC();
  for (int j = 0; j < nv; j++) {
    if (tid < nv && ((pl->dof_anc_mask[tid] >> j) & 1u)) x[tid] -= A[tid][j] * x[j];
    SYNC();
  }
}

/* ================================================================== */
/* collision: per-candidate lanes, prefix offsets, deterministic order */
/* ================================================================== */
/* a candidate pair's constants: from the plan's pair rows (one load level, the overlaid layouts) or
   through the model's pair -> geom chain (the full-capacity layouts); the same values either way */
struct WPairRow {
  int g1, g2, t1, t2;
  double margin, rb1, rb2;
  const double* s1; /* the geoms' sizes, in memory: the narrowphase indexes them at run time */
  const double* s2;
};
/* the overlaid box layouts read the plan rows (1, default) or the model's chains (0: A/B) */
#ifndef W_FLAT_PAIRS
#define W_FLAT_PAIRS 1
#endif
WD WPairRow w_pair_row_m(KModel m, int p) {
  WPairRow P;
  P.g1 = m->cpair_geom1[p]; P.g2 = m->cpair_geom2[p];
  P.t1 = m->geom_type[P.g1]; P.t2 = m->geom_type[P.g2];
  P.margin = m->cpair_margin[p];
  P.rb1 = m->geom_rbound[P.g1]; P.rb2 = m->geom_rbound[P.g2];
  P.s1 = m->geom_size[P.g1]; P.s2 = m->geom_size[P.g2];
  return P;
}
template <class KS>
WD WPairRow w_pair_row(KModel m, const KPlan* __restrict__ pl, int p) {
  /* the mesh-capable layouts keep the model's chains: measured 0.3 % slower with the rows (A/B 5) */
  if (!W_FLAT_PAIRS || KS::MESHES) return w_pair_row_m(m, p);
  WPairRow P;
  P.g1 = pl->pr_i[p][0]; P.g2 = pl->pr_i[p][1]; P.t1 = pl->pr_i[p][2]; P.t2 = pl->pr_i[p][3];
  P.margin = pl->pr_d[p][0]; P.rb1 = pl->pr_d[p][1]; P.rb2 = pl->pr_d[p][2];
  P.s1 = &pl->pr_d[p][3]; P.s2 = &pl->pr_d[p][6];
  return P;
}

/* bounding-sphere test of candidate pair p (mj_collideGeoms' rbound early-out) */
template <class KS>
WD bool w_pair_near(const KS& s, const WPairRow& P) {
  const int g1 = P.g1, g2 = P.g2;
  const double margin = P.margin;
  const double rb1 = P.rb1, rb2 = P.rb2;
  if (rb1 > 0 && rb2 > 0) {
    double dx = s.geom_xpos[g1][0] - s.geom_xpos[g2][0];
    double dy = s.geom_xpos[g1][1] - s.geom_xpos[g2][1];
    double dz = s.geom_xpos[g1][2] - s.geom_xpos[g2][2];
    double lim = rb1 + rb2 + margin;
    if (dx * dx + dy * dy + dz * dz > lim * lim) return false;
  }
  return true;
}

/* The pair is certain to give no contact, decided before the narrowphase (bounding spheres alone keep every
   plane pair and the always-overlapping neighbours: 27 of main.xml's 92 candidates survive them in every
   gym state, 24 of them plane-box).  Plane-box: the box's lowest corner, n.(c - p) - sum_i h_i |n.a_i|,
   lies beyond the margin by more than 1e-9 -- every corner's computed distance then exceeds the margin
   too (their rounding error is ~1e-15 of the ~1 m scale), so k_plane_box_t would emit none.  Box-box:
   the six face axes of k_box_box_t's separating-axis test, computed with the same expressions in the
   same order, and one of them separates beyond the margin -- the routine returns 0 there.  Plane-mesh:
   the hull's bounding radius; box-mesh and mesh-mesh: the hulls' boxes (below).  Either way
   the pair's result (no contact) is unchanged, and only its narrowphase is skipped. */
template <class KS>
WD bool w_pair_apart(const KS& s, const WPairRow& P) {
  const int g1 = P.g1, g2 = P.g2;
  const int t1 = P.t1, t2 = P.t2;
  const double margin = P.margin;
  if (t1 == UR3E_GEOM_PLANE && t2 == UR3E_GEOM_MESH) {
    /* every hull vertex lies within geom_rbound of the geom's origin (the compiler's bound over the
       same vertices), so the centre beyond the margin by more than rbound + 1e-9 keeps every vertex
       distance of ur3e_plane_convex above the margin: the pair gives no contact */
    const double* pm = s.geom_xmat[g1];
    const double n[3] = {pm[2], pm[5], pm[8]};
    const double dif[3] = {s.geom_xpos[g2][0] - s.geom_xpos[g1][0], s.geom_xpos[g2][1] - s.geom_xpos[g1][1],
                           s.geom_xpos[g2][2] - s.geom_xpos[g1][2]};
    return k_dot3(n, dif) - P.rb2 > margin + 1e-9;
  }
  const bool mesh2 = t2 == UR3E_GEOM_MESH, mesh1 = t1 == UR3E_GEOM_MESH;
  if (t2 != UR3E_GEOM_BOX && !mesh2) return false;
  if (t1 == UR3E_GEOM_PLANE) {
    if (mesh2) return false;
    const double* pm = s.geom_xmat[g1];
    const double* bm = s.geom_xmat[g2];
    const double n[3] = {pm[2], pm[5], pm[8]};
    const double dif[3] = {s.geom_xpos[g2][0] - s.geom_xpos[g1][0], s.geom_xpos[g2][1] - s.geom_xpos[g1][1],
                           s.geom_xpos[g2][2] - s.geom_xpos[g1][2]};
    const double dist = k_dot3(n, dif);
    double ext = 0;
#pragma unroll
    for (int c = 0; c < 3; c++) ext += P.s2[c] * fabs(n[0] * bm[c] + n[1] * bm[3 + c] + n[2] * bm[6 + c]);
    return dist - ext > margin + 1e-9;
  }
  if (t1 != UR3E_GEOM_BOX && !mesh1) return false;
  /* box-box: k_box_box_t's own decision (> margin).  A convex mesh lies inside its geom_size box (the
     compiler's half extents of the same hull vertices), so two shapes whose boxes separate by more than
     the margin + 1e-6 along a face axis are apart beyond the margin: GJK (the wavefront's or the full
     tier's) finds no contact for them, to well within that 1e-6 */
  const double lim = (mesh1 || mesh2) ? margin + 1e-6 : margin;
  const double* R1 = s.geom_xmat[g1];
  const double* R2 = s.geom_xmat[g2];
  const double* s1 = P.s1;
  const double* s2 = P.s2;
  double a[3][3], b[3][3];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    a[k][0] = R1[k]; a[k][1] = R1[3 + k]; a[k][2] = R1[6 + k];
    b[k][0] = R2[k]; b[k][1] = R2[3 + k]; b[k][2] = R2[6 + k];
  }
  const double pp[3] = {s.geom_xpos[g2][0] - s.geom_xpos[g1][0], s.geom_xpos[g2][1] - s.geom_xpos[g1][1],
                        s.geom_xpos[g2][2] - s.geom_xpos[g1][2]};
  bool apart = false;
#pragma unroll
  for (int code = 0; code < 6; code++) {
    const double* ax = code < 3 ? a[code] : b[code - 3];
    double ext = 0;
#pragma unroll
    for (int k = 0; k < 3; k++) ext += s1[k] * fabs(k_dot3(a[k], ax));
#pragma unroll
    for (int k = 0; k < 3; k++) ext += s2[k] * fabs(k_dot3(b[k], ax));
    const double sep = fabs(k_dot3(pp, ax)) - ext;
    apart |= sep > lim;
  }
  return apart;
}

/* geom g as a convex shape (convex.h): box half sizes, or its mesh's hull vertices (model image) */
template <class KS>
__device__ __forceinline__ void w_geom_convex(KModel m, const KS& s, int g, ur3e_cvx* c) {
  if (m->geom_type[g] == UR3E_GEOM_MESH) {
    const int id = m->geom_dataid[g];
    c->v = &m->mesh_vert[m->mesh_vertadr[id]][0];
    c->nv = m->mesh_vertnum[id];
  } else {
    c->v = nullptr;
    c->nv = 0;
  }
  for (int k = 0; k < 3; k++) { c->size[k] = m->geom_size[g][k]; c->pos[k] = s.geom_xpos[g][k]; }
  for (int k = 0; k < 9; k++) c->mat[k] = s.geom_xmat[g][k];
}

/* convex mesh pairs, full-capacity tier only: plane-mesh (<= UR3E_CVX_PLANE_MAX contacts), box-mesh
   and mesh-mesh (GJK + EPA, one contact); the same convex.h code as the oracle's mesh_collide.  Inlined:
   the narrowphase runs in a divergent region (one candidate per lane), where an out-of-line call was
   once miscompiled (r_collision) */
template <class KS>
__device__ __forceinline__ int w_mesh_collide(KModel m, const KS& s, int g1, int g2, double margin, KRaw* raw) {
  ur3e_cvx b;
  w_geom_convex(m, s, g2, &b);
  if (m->geom_type[g1] == UR3E_GEOM_PLANE) {
    double pos[UR3E_CVX_PLANE_MAX][3], nrm[UR3E_CVX_PLANE_MAX][3], dist[UR3E_CVX_PLANE_MAX];
    const int n = ur3e_plane_convex(s.geom_xpos[g1], s.geom_xmat[g1], &b, margin, pos, nrm, dist);
    for (int k = 0; k < n; k++) {
      for (int c = 0; c < 3; c++) { raw[k].pos[c] = pos[k][c]; raw[k].n[c] = nrm[k][c]; }
      raw[k].dist = dist[k];
    }
    return n;
  }
  ur3e_cvx a;
  w_geom_convex(m, s, g1, &a);
  ur3e_epa scratch;
  return ur3e_convex_convex(&a, &b, margin, &scratch, raw[0].pos, raw[0].n, &raw[0].dist);
}

/* narrowphase of candidate pair p (after w_pair_near): raw contacts, returns their count */
template <class KS, bool INL = false>
WD int w_narrow_core(KModel m, const KS& s, int p, KRaw* raw) {
  int g1 = m->cpair_geom1[p], g2 = m->cpair_geom2[p];
  double margin = m->cpair_margin[p];
  int t1 = m->geom_type[g1], t2 = m->geom_type[g2];
  if constexpr (!KS::OVERLAY) {
    if (t2 == UR3E_GEOM_MESH) return w_mesh_collide(m, s, g1, g2, margin, raw);
  }
  if (t1 == UR3E_GEOM_PLANE && t2 == UR3E_GEOM_BOX)
    return k_plane_box(s.geom_xpos[g1], s.geom_xmat[g1], s.geom_xpos[g2], s.geom_xmat[g2], m->geom_size[g2], margin,
                       raw);
  if (t1 == UR3E_GEOM_BOX && t2 == UR3E_GEOM_BOX) {
    if constexpr (INL)
      return k_box_box_inl(s.geom_xpos[g1], s.geom_xmat[g1], m->geom_size[g1], s.geom_xpos[g2], s.geom_xmat[g2],
                           m->geom_size[g2], margin, raw);
    else
      return k_box_box(s.geom_xpos[g1], s.geom_xmat[g1], m->geom_size[g1], s.geom_xpos[g2], s.geom_xmat[g2],
                       m->geom_size[g2], margin, raw);
  }
  return 0;
}

/* compact tier: clip polygons in LDS (lane ln of the chunk) and contacts staged in LDS through an
   LDS counter, keyed by (lane, index) so that the copy pass can place them in candidate order */
struct KLdsClip {
  double* base;
  int ln;
  __device__ __forceinline__ double get(int buf, int v, int c) const {
    return base[((buf * 8 + v) * 3 + c) * W_NP_LANES + ln];
  }
  __device__ __forceinline__ void set(int buf, int v, int c, double x) {
    base[((buf * 8 + v) * 3 + c) * W_NP_LANES + ln] = x;
  }
};
template <int NST>
struct KStageEmit {
  double* st;
  int* key;
  int* nst;
  int ln;
  __device__ __forceinline__ void operator()(int k, const double pos[3], const double n[3], double dist) const {
    const int slot = atomicAdd(nst, 1);
    if (slot < NST) {
      st[0 * NST + slot] = pos[0]; st[1 * NST + slot] = pos[1]; st[2 * NST + slot] = pos[2];
      st[3 * NST + slot] = n[0]; st[4 * NST + slot] = n[1]; st[5 * NST + slot] = n[2];
      st[6 * NST + slot] = dist;
      key[slot] = ln * 8 + k;
    }
  }
};

/* w_narrow_core with the compact tier's LDS clip buffers and contact stage (lane ln < W_NP_LANES) */
template <class KS>
WD int w_narrow_lds(KS& s, const WPairRow& P, int ln, int slot) {
  const int g1 = P.g1, g2 = P.g2;
  const double margin = P.margin;
  const int t1 = P.t1, t2 = P.t2;
  auto& ch = s.kn.chunk();
  const KStageEmit<KS::NPST> emit{&ch.np_stage[0][0], ch.np_key, &ch.np_nstage, ln};
  /* convex meshes: in the mesh-capable layouts (compact and grasp tiers) w_mesh_pass (ur3e_cvx_wave.h)
     has already settled every mesh pair -- GJK, EPA and plane-convex in the wavefront -- and left its raw
     contacts in s.kn.mres; they are emitted here at the pair's place in candidate order.  The only hand-offs
     are an EPA horizon beyond WC_MAXE or more contacts than the layout holds (ovf).  Layouts without
     meshes never see a mesh pair (the model selects the mesh-capable set) */
  if (t2 == UR3E_GEOM_MESH) {
    if constexpr (KS::MESHES) {
      /* settled by the wave in w_mesh_pass: emit its contacts at the pair's place */
      const int c = s.kn.mres.cnt[slot];
      const int at = s.kn.mres.at[slot];
      for (int k = 0; k < c; k++) {
        const double* r = s.kn.mres.raw[at + k];
        const double pos[3] = {r[0], r[1], r[2]}, nn[3] = {r[3], r[4], r[5]};
        emit(k, pos, nn, r[6]);
      }
      return c;
    } else {
      s.ovf = 1; /* hand the env-step on to the tier that runs the mesh narrowphase */
      return 0;
    }
  }
  if (t1 == UR3E_GEOM_PLANE && t2 == UR3E_GEOM_BOX)
    return k_plane_box_t(s.geom_xpos[g1], s.geom_xmat[g1], s.geom_xpos[g2], s.geom_xmat[g2], P.s2, margin, emit);
  if (t1 == UR3E_GEOM_BOX && t2 == UR3E_GEOM_BOX) {
    KLdsClip clip{&ch.np_clip[0][0][0][0], ln};
    return k_box_box_t(s.geom_xpos[g1], s.geom_xmat[g1], P.s1, s.geom_xpos[g2], s.geom_xmat[g2], P.s2, margin, clip,
                       emit);
  }
  return 0;
}

template <class KS>
WD int w_narrow(KModel m, const KS& s, int p, KRaw* raw) {
  return w_pair_near(s, w_pair_row_m(m, p)) ? w_narrow_core(m, s, p, raw) : 0;
}

/* mesh-capable overlaid layouts: every survivor pair with a convex mesh (plane-mesh, box-mesh, mesh-mesh)
   settled by the whole wave, one pair at a time in candidate order (ur3e_cvx_wave.h: convex.h's results,
   bit for bit); its raw contacts wait in s.kn.mres until the chunked narrowphase emits them at the pair's
   place.  More raw contacts than the layout holds, or an EPA horizon beyond WC_MAXE, hand the env-step on. */
template <class KS>
WD void w_mesh_pass(KModel m, const KPlan* __restrict__ pl, KS& s, int nsurv) {
  const int lane = w_lane();
  auto& R = s.kn.mres;
  auto& W = s.kn.cw;
  constexpr int MC = KS::MAXCON;
  R.cnt[lane] = 0;
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  const int slot = lane;
  const int p = slot < nsurv ? s.cand_off[slot] : 0;
  const bool mesh = slot < nsurv && m->geom_type[m->cpair_geom2[p]] == UR3E_GEOM_MESH;
  unsigned long long bm = __ballot(mesh);
  int nraw = 0;
  while (bm) {
    const int q = __builtin_ctzll(bm);
    bm &= bm - 1;
    const int pq = rli(p, q);
#ifdef UR3E_STAGE_TIMING
    if (lane == 0) s.tcnt[49] += 1; /* diagnostic: mesh pairs settled by the wave */
#endif
    const int g1 = m->cpair_geom1[pq], g2 = m->cpair_geom2[pq];
    const double margin = m->cpair_margin[pq];
    WCvxShape B;
    WCvxLane lb;
    wc_shape(m, s, g2, B, lb);
    int c;
    if (m->geom_type[g1] == UR3E_GEOM_PLANE) {
      c = wc_plane_convex(s.geom_xpos[g1], s.geom_xmat[g1], B, lb, margin, W, &R.raw[nraw], MC - nraw);
    } else {
      WCvxShape A;
      WCvxLane la;
      wc_shape(m, s, g1, A, la);
      double res[7];
      c = wc_convex_convex(A, la, B, lb, W, margin, res);
      if (c == 1 && nraw < MC) {
        if (lane < 7) R.raw[nraw][lane] = lane == 0 ? res[0] : lane == 1 ? res[1] : lane == 2 ? res[2] : lane == 3 ? res[3]
                                          : lane == 4 ? res[4] : lane == 5 ? res[5] : res[6];
      }
    }
    if (c < 0 || nraw + c > MC) { /* beyond this layout: the next tier settles the env-step */
      if (lane == 0) s.ovf = 1;
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
      return;
    }
    if (lane == 0) {
      R.cnt[q] = (signed char)c;
      R.at[q] = (unsigned char)nraw;
    }
    nraw += c;
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }
}

/* contact c of the env from raw contact r of candidate pair p */
template <class KS>
WD void w_store_contact(KModel m, KS& s, int c, int p, const KRaw& r) {
  s.con_pos[c][0] = r.pos[0]; s.con_pos[c][1] = r.pos[1]; s.con_pos[c][2] = r.pos[2];
  if constexpr (KS::OVERLAY) {
    double u[3] = {r.n[0], r.n[1], r.n[2]};
    k_normalize3(u); /* = frame row 0 of k_make_frame */
    s.con_n[c][0] = u[0]; s.con_n[c][1] = u[1]; s.con_n[c][2] = u[2];
  } else {
    k_make_frame(s.con_frame[c], r.n);
  }
  s.con_dist[c] = r.dist;
  s.con_geom1[c] = m->cpair_geom1[p];
  s.con_geom2[c] = m->cpair_geom2[p];
  s.con_cpair[c] = p;
  s.con_mu[c] = 0;
  s.con_efc[c] = -1;
}

/* one 64-lane wavefront: bounding-sphere filter over all candidates, survivors compacted in
   candidate order (ballot + mbcnt), ONE narrowphase per survivor (lane = survivor), contact
   offsets by a wave prefix scan of the counts, contacts written from the lane's own results.
   Same contacts in the same order as the count / prefix / write passes of w_collision. */
/* the bounding-sphere survivors' list of the overlaid layouts' two-pass broadphase (r_collision): the
   narrowphase area's clip buffers, which are dead until the narrowphase (KS::NCAND ints <= 1 KB) */
template <class KS>
__device__ __forceinline__ int* w_near_list(KS& s) {
  static_assert(sizeof(s.kn.chunk().np_clip) >= KS::NCAND * sizeof(int), "near list exceeds the clip buffers");
  return reinterpret_cast<int*>(&s.kn.chunk().np_clip[0][0][0][0]);
}
/* the exact pre-narrowphase cull (w_pair_apart) on (1, default) or off (0: A/B) */
#ifndef W_PAIR_CULL
#define W_PAIR_CULL 1
#endif
/* the mesh-capable overlaid layouts' two-pass broadphase (1, default) or the single fused pass (0: A/B).
   Measured (profiles/r05_ab, A/B 2): +0.5 % on the mesh model (234 candidates, four sphere passes), -1 % on
   the box surrogate (92 candidates, two passes), which keeps the fused pass */
#ifndef W_BROAD_2PASS
#define W_BROAD_2PASS 1
#endif
/* the mesh-capable broadphase's pair constants for all its passes loaded ahead of the sphere tests (1: A/B) or
   per pass (0, default).  Dropped: same-box A/B 8.806 against 8.815 M env-steps/s (profiles/r06_ab A/B 2) --
   the model constants' load latency is not on the wave's critical path here */
#ifndef W_BROAD_AHEAD
#define W_BROAD_AHEAD 0
#endif
template <class KS>
WD void r_collision(KModel m, const KPlan* __restrict__ pl, KS& s) {
  const int lane = w_lane();
  const int np = m->ncpair;
  int nsurv = 0;
  /* the overlaid layouts list W_MAXSURV survivors (an env-step with more hands on); the full-capacity
     layout every candidate */
  constexpr int CAP = KS::OVERLAY ? W_MAXSURV : KS::NCAND;
  if constexpr (KS::OVERLAY && KS::MESHES && W_PAIR_CULL && W_BROAD_2PASS) {
    /* two compacted passes: the bounding-sphere test over every candidate (64 per pass), its survivors
       listed in candidate order in the narrowphase area (dead until the narrowphase); then the exact cull
       over that list only -- one pass for the sphere survivors instead of one per 64 candidates, whose
       few surviving lanes would run the separating-axis test in every pass */
    int* near = w_near_list(s);
    constexpr int NCAP = KS::NCAND;
    int nnear = 0;
#if W_BROAD_AHEAD
    /* every pass's pair constants (the model's pair -> geom chains) issued before the first sphere test, so
       the passes wait for one round of global loads instead of one per pass */
    constexpr int NB = (KS::NCAND + 63) / 64;
    WPairRow PR[NB];
#pragma unroll
    for (int b = 0; b < NB; b++) {
      const int p = 64 * b + lane;
      PR[b] = w_pair_row<KS>(m, pl, p < np ? p : 0);
    }
#pragma unroll
    for (int b = 0; b < NB; b++) {
      const int p = 64 * b + lane;
      if (64 * b >= np) break;
      const bool ok = p < np && w_pair_near(s, PR[b]);
      const unsigned long long bm = __ballot(ok);
      const int at = nnear + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u));
      if (ok && at < NCAP) near[at] = p;
      nnear += __popcll(bm);
    }
#else
    for (int base = 0; base < np; base += 64) {
      const int p = base + lane;
      const bool ok = p < np && w_pair_near(s, w_pair_row<KS>(m, pl, p));
      const unsigned long long bm = __ballot(ok);
      const int at = nnear + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u));
      if (ok && at < NCAP) near[at] = p;
      nnear += __popcll(bm);
    }
#endif
    if (nnear > NCAP) nnear = NCAP; /* np <= KS::NCAND (the host checks ncpair): never taken */
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    for (int base = 0; base < nnear; base += 64) {
      const int k = base + lane;
      const int p = k < nnear ? near[k] : 0;
      const bool ok = k < nnear && !w_pair_apart(s, w_pair_row<KS>(m, pl, p));
      const unsigned long long bm = __ballot(ok);
      const int at = nsurv + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u));
      if (ok && at < CAP) s.cand_off[at] = p;
      nsurv += __popcll(bm);
    }
  } else {
    for (int base = 0; base < np; base += 64) {
      const int p = base + lane;
      bool ok = false;
      if (p < np) {
        const WPairRow P = w_pair_row<KS>(m, pl, p);
        ok = w_pair_near(s, P) && !(W_PAIR_CULL && w_pair_apart(s, P));
      }
      const unsigned long long bm = __ballot(ok);
      const int at = nsurv + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u));
      if (ok && at < CAP) s.cand_off[at] = p;
      nsurv += __popcll(bm);
    }
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  if constexpr (KS::OVERLAY) {
    if (nsurv > CAP) {
      if (lane == 0) s.ovf = 1;
      nsurv = CAP;
    }
  }
  WT(39);
  int total = 0;
  if constexpr (KS::OVERLAY) {
    /* survivors in chunks of W_NP_LANES lanes: narrowphase with its clip polygons in LDS, raw
       contacts staged in LDS, then one lane per staged contact writes it at (prefix of its
       survivor lane) + (its index), the order of the pass below -- no private (scratch) arrays */
    constexpr int NST = KS::NPST;
    static_assert(KS::BAIL && KS::MAXCON <= NST && NST <= 64, "compact narrowphase stage must hold MAXCON");
    if constexpr (KS::MESHES) {
      w_mesh_pass(m, pl, s, nsurv);
      WT(48);
    }
    auto& ch = s.kn.chunk();
    if (lane == 0) ch.np_nstage = 0;
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    const int npl = s.np_lanes;
    for (int base = 0; base < nsurv; base += npl) {
      const int slot = base + lane;
      const bool act = lane < npl && slot < nsurv;
      const int p = s.cand_off[act ? slot : 0];
      int cnt = 0;
      if (act) cnt = w_narrow_lds(s, w_pair_row<KS>(m, pl, p), lane, slot);
      int incl = cnt;
#pragma unroll
      for (int d = 1; d < W_NP_LANES; d <<= 1) {
        const int y = __shfl_up(incl, d);
        if (lane >= d) incl += y;
      }
      const int off = total + incl - cnt;
      total += rli(incl, W_NP_LANES - 1);
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
      const int nall = ch.np_nstage;
      const int nst = nall < NST ? nall : NST;
      const int key = lane < nst ? ch.np_key[lane] : 0;
      const int src = key >> 3, kk = key & 7;
      const int offs = shfi(off, src), ps = shfi(p, src);
      if (lane < nst && offs + kk < KS::MAXCON) {
        KRaw r;
        r.pos[0] = ch.np_stage[0][lane]; r.pos[1] = ch.np_stage[1][lane]; r.pos[2] = ch.np_stage[2][lane];
        r.n[0] = ch.np_stage[3][lane]; r.n[1] = ch.np_stage[4][lane]; r.n[2] = ch.np_stage[5][lane];
        r.dist = ch.np_stage[6][lane];
        w_store_contact(m, s, offs + kk, ps, r);
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
      if (lane == 0) {
        if (nall > NST) s.ovf = 1; /* contacts were dropped from the stage: > MAXCON anyway */
        ch.np_nstage = 0;
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
    }
    if (lane == 0) {
      s.ncon = total < KS::MAXCON ? total : KS::MAXCON;
      if (total > s.cap_con) s.ovf = 1;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    return;
  }
  for (int base = 0; base < nsurv; base += 64) {
    const int slot = base + lane;
    /* the box-box routine is inlined here: an out-of-line call from this divergent region was
       miscompiled in an earlier, register-saturated build (state read after the forward pass came
       back corrupted), while the inlined form is bit-exact */
    const bool act = slot < nsurv;
    const int p = s.cand_off[act ? slot : 0];
    KRaw raw[8];
    /* lanes without a survivor stay masked off, so their private-segment (scratch) stores of
       the clip polygons and raw contacts never reach memory */
    int cnt = 0;
    if (act) cnt = w_narrow_core<KS, true>(m, s, p, raw);
    int incl = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int y = __shfl_up(incl, d);
      if (lane >= d) incl += y;
    }
    const int off = total + incl - cnt;
    total += rli(incl, 63);
    for (int k = 0; k < cnt && off + k < KS::MAXCON; k++) w_store_contact(m, s, off + k, p, raw[k]);
  }
  if (lane == 0) {
    s.ncon = total < KS::MAXCON ? total : KS::MAXCON;
    if (KS::BAIL && total > s.cap_con) s.ovf = 1;
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

/* the 128-lane full-capacity layout: counts of every candidate, prefix offsets, contacts */
template <int NT, class KS>
WD void w_collision_all(KModel m, KS& s) {
  const int tid = w_lane();
  const int np = m->ncpair;
  KRaw raw[8];
  for (int p = tid; p < np; p += NT) s.cand_count[p] = w_narrow(m, s, p, raw);
  SYNC();
  if (tid == 0) {
    int off = 0;
    for (int p = 0; p < np; p++) {
      s.cand_off[p] = off;
      off += s.cand_count[p];
    }
    s.ncon = off < KS::MAXCON ? off : KS::MAXCON;
    if (KS::BAIL && off > s.cap_con) s.ovf = 1;
  }
  SYNC();
  if (KS::BAIL && s.ovf) return;
  for (int p = tid; p < np; p += NT) {
    int cnt = s.cand_count[p];
    int off = s.cand_off[p];
    if (cnt == 0 || off >= KS::MAXCON) continue;
    int n = w_narrow(m, s, p, raw);
    for (int k = 0; k < n && off + k < KS::MAXCON; k++) w_store_contact(m, s, off + k, p, raw[k]);
  }
  SYNC();
}

template <int NT, class KS>
WD void w_collision(KModel m, const KPlan* __restrict__ pl, KS& s) {
  if constexpr (NT == 64) {
    r_collision<KS>(m, pl, s);
  } else {
    w_collision_all<NT>(m, s);
  }
}

/* ================================================================== */
/* constraint rows                                                     */
/* ================================================================== */
/* translational point-Jacobian column v of `body` at p (zero outside the chain) */
template <class KS>
KD void w_jacp_col(KModel m, const KPlan* __restrict__ pl, const KS& s, int body, const double off[3], int v,
                   double out[3]) {
  if ((pl->body_dof_mask[body] >> v) & 1u) {
    const double* cd = s.cdof[v];
    double cr[3];
    k_cross3(cr, cd, off);
    out[0] = cd[3] + cr[0];
    out[1] = cd[4] + cr[1];
    out[2] = cd[5] + cr[2];
  } else {
    out[0] = 0; out[1] = 0; out[2] = 0;
  }
}

template <class KS>
KD void w_row_impedance(KModel m, KS& s, int r, const double* sref, const double* simp, double pos, double margin,
                        double diag, int friction_row) {
  const int nv = NVOF(KS, m);
  double vel = 0;
  for (int k = 0; k < nv; k++) vel += s.efc_J[r][k] * s.qvel[k];
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
    s.efc_aref[r] = -B * vel;
  else
    s.efc_aref[r] = -B * vel - K * imp * (pos - margin);
  double R = (1 - imp) * diag / imp;
  s.efc_R[r] = R < K_MINVAL ? K_MINVAL : R;
}

template <int NT, class KS>
WD void w_make_constraint(KModel m, const KPlan* __restrict__ pl, KS& s) {
  const int tid = w_lane();
  const int nv = NVOF(KS, m);
  constexpr bool REG = (NT == 64 && KS::OVERLAY);
  if constexpr (REG) {
    r_mc_layout(m, pl, s);
    WT(36);
    if (s.ovf) return;
      r_mc_rows(m, pl, s);
  } else {
  /* lane 0 lays out the row groups in oracle order; a group that does not fit stops the layout */
  if (tid == 0) {
    int nrow = 0, ng = 0, stop = 0;
    for (int e = 0; e < m->neq && !stop; e++) {
      int need = m->eq_type[e] == UR3E_EQ_CONNECT ? 3 : 1;
      if (nrow + need > KS::MAXEFC) { stop = 1; break; }
      s.grp_type[ng] = m->eq_type[e] == UR3E_EQ_CONNECT ? G_CONNECT : G_JOINTEQ;
      s.grp_id[ng] = e; s.grp_row[ng] = nrow; ng++; nrow += need;
    }
    for (int k = 0; k < pl->nfloss && !stop; k++) {
      if (nrow + 1 > KS::MAXEFC) { stop = 1; break; }
      s.grp_type[ng] = G_FLOSS; s.grp_id[ng] = pl->floss_dof[k]; s.grp_row[ng] = nrow; ng++; nrow++;
    }
    for (int j = 0; j < m->njnt && !stop; j++) {
      if (!m->jnt_limited[j]) continue;
      if (m->jnt_type[j] != UR3E_JNT_HINGE && m->jnt_type[j] != UR3E_JNT_SLIDE) continue;
      double q = s.qpos[m->jnt_qposadr[j]];
      for (int side = -1; side <= 1; side += 2) {
        double dist = side * (m->jnt_range[j][(side + 1) / 2] - q);
        if (dist < m->jnt_margin[j]) {
          if (nrow + 1 > KS::MAXEFC) { stop = 1; break; }
          s.grp_type[ng] = G_LIMIT; s.grp_id[ng] = 2 * j + (side + 1) / 2; s.grp_row[ng] = nrow; ng++; nrow++;
        }
      }
    }
    for (int c = 0; c < s.ncon && !stop; c++) {
      if (m->cpair_condim[s.con_cpair[c]] != 3) continue;
      if (nrow + 3 > KS::MAXEFC) { stop = 1; break; }
      s.grp_type[ng] = G_CONTACT; s.grp_id[ng] = c; s.grp_row[ng] = nrow; ng++; nrow += 3;
    }
    s.ngrp = ng;
    s.nefc = nrow;
    if (KS::BAIL && stop) s.ovf = 1;
  }
  SYNC();
  if (KS::BAIL && s.ovf) return;
  /* phase A: Jacobian entries, one lane per (group, dof) */
  const int nitem = s.ngrp * nv;
  for (int it = tid; it < nitem; it += NT) {
    int g = it / nv, v = it % nv;
    int type = s.grp_type[g], id = s.grp_id[g], r = s.grp_row[g];
    int nrow = (type == G_CONNECT || type == G_CONTACT) ? 3 : 1;
    if (v == 0) {
      int ct = type == G_CONNECT || type == G_JOINTEQ ? CN_EQUALITY
             : type == G_FLOSS ? CN_FRICTION_DOF : type == G_LIMIT ? CN_LIMIT_JOINT : CN_CONTACT_ELLIPTIC;
      int cid = type == G_LIMIT ? (id >> 1) : id;
      for (int k = 0; k < nrow; k++) {
        s.efc_type[r + k] = ct; s.efc_id[r + k] = cid; s.efc_grp[r + k] = g;
        s.efc_floss[r + k] = type == G_FLOSS ? m->dof_frictionloss[id] : 0.0;
      }
      if (type == G_CONTACT) s.con_efc[id] = r;
    }
    if (type == G_CONNECT) {
      int e = id;
      int b1 = m->eq_obj1[e], b2 = m->eq_obj2[e];
      double p1[3], p2[3];
      k_mat_vec3(p1, s.xmat[b1], m->eq_data[e]);
      p1[0] += s.xpos[b1][0]; p1[1] += s.xpos[b1][1]; p1[2] += s.xpos[b1][2];
      k_mat_vec3(p2, s.xmat[b2], m->eq_data[e] + 3);
      p2[0] += s.xpos[b2][0]; p2[1] += s.xpos[b2][1]; p2[2] += s.xpos[b2][2];
      const double* c1 = s.subtree_com[m->body_rootid[b1]];
      const double* c2 = s.subtree_com[m->body_rootid[b2]];
      double o1[3] = {p1[0] - c1[0], p1[1] - c1[1], p1[2] - c1[2]};
      double o2[3] = {p2[0] - c2[0], p2[1] - c2[1], p2[2] - c2[2]};
      double j1[3], j2[3];
      w_jacp_col(m, pl, s, b1, o1, v, j1);
      w_jacp_col(m, pl, s, b2, o2, v, j2);
      for (int k = 0; k < 3; k++) s.efc_J[r + k][v] = j1[k] - j2[k];
    } else if (type == G_JOINTEQ) {
      int e = id;
      int j1 = m->eq_obj1[e], j2 = m->eq_obj2[e];
      double val = 0;
      if (v == m->jnt_dofadr[j1]) val = 1;
      if (j2 >= 0 && v == m->jnt_dofadr[j2]) {
        const double* c = m->eq_data[e];
        int a2 = m->jnt_qposadr[j2];
        double q2 = s.qpos[a2] - m->qpos0[a2];
        double dpoly = c[1] + q2 * (2 * c[2] + q2 * (3 * c[3] + q2 * 4 * c[4]));
        val = -dpoly;
      }
      s.efc_J[r][v] = val;
    } else if (type == G_FLOSS) {
      s.efc_J[r][v] = v == id ? 1.0 : 0.0;
    } else if (type == G_LIMIT) {
      int j = id >> 1;
      int side = (id & 1) ? 1 : -1;
      s.efc_J[r][v] = v == m->jnt_dofadr[j] ? -(double)side : 0.0;
    } else {
      int c = id;
      int b1 = m->geom_bodyid[s.con_geom1[c]], b2 = m->geom_bodyid[s.con_geom2[c]];
      const double* pos = s.con_pos[c];
      const double* c1 = s.subtree_com[m->body_rootid[b1]];
      const double* c2 = s.subtree_com[m->body_rootid[b2]];
      double o1[3] = {pos[0] - c1[0], pos[1] - c1[1], pos[2] - c1[2]};
      double o2[3] = {pos[0] - c2[0], pos[1] - c2[1], pos[2] - c2[2]};
      const double* fr = s.con_frame[c];
      double j1[3], j2[3];
      w_jacp_col(m, pl, s, b1, o1, v, j1);
      w_jacp_col(m, pl, s, b2, o2, v, j2);
      double dj0 = j2[0] - j1[0], dj1 = j2[1] - j1[1], dj2 = j2[2] - j1[2];
      for (int k = 0; k < 3; k++) s.efc_J[r + k][v] = fr[3 * k] * dj0 + fr[3 * k + 1] * dj1 + fr[3 * k + 2] * dj2;
    }
  }
  SYNC();
  }
  /* phase B: reference acceleration and regulariser, one lane per row */
  if constexpr (!REG)
  for (int r = tid; r < s.nefc; r += NT) {
    int g = s.efc_grp[r];
    int type = s.grp_type[g], id = s.grp_id[g];
    int k = r - s.grp_row[g];
    if (type == G_CONNECT) {
      int e = id;
      int b1 = m->eq_obj1[e], b2 = m->eq_obj2[e];
      double p1[3], p2[3];
      k_mat_vec3(p1, s.xmat[b1], m->eq_data[e]);
      p1[0] += s.xpos[b1][0]; p1[1] += s.xpos[b1][1]; p1[2] += s.xpos[b1][2];
      k_mat_vec3(p2, s.xmat[b2], m->eq_data[e] + 3);
      p2[0] += s.xpos[b2][0]; p2[1] += s.xpos[b2][1]; p2[2] += s.xpos[b2][2];
      double diag = m->body_invweight0[b1][0] + m->body_invweight0[b2][0];
      w_row_impedance(m, s, r, m->eq_solref[e], m->eq_solimp[e], p1[k] - p2[k], 0, diag, 0);
    } else if (type == G_JOINTEQ) {
      int e = id;
      int j1 = m->eq_obj1[e], j2 = m->eq_obj2[e];
      const double* c = m->eq_data[e];
      int a1 = m->jnt_qposadr[j1];
      double q1 = s.qpos[a1] - m->qpos0[a1];
      double pos;
      double diag = m->dof_invweight0[m->jnt_dofadr[j1]];
      if (j2 >= 0) {
        int a2 = m->jnt_qposadr[j2];
        double q2 = s.qpos[a2] - m->qpos0[a2];
        pos = q1 - (c[0] + q2 * (c[1] + q2 * (c[2] + q2 * (c[3] + q2 * c[4]))));
        diag += m->dof_invweight0[m->jnt_dofadr[j2]];
      } else {
        pos = q1 - c[0];
      }
      w_row_impedance(m, s, r, m->eq_solref[e], m->eq_solimp[e], pos, 0, diag, 0);
    } else if (type == G_FLOSS) {
      w_row_impedance(m, s, r, m->dof_solref[id], m->dof_solimp[id], 0, 0, m->dof_invweight0[id], 1);
    } else if (type == G_LIMIT) {
      int j = id >> 1;
      int side = (id & 1) ? 1 : -1;
      double q = s.qpos[m->jnt_qposadr[j]];
      double dist = side * (m->jnt_range[j][(side + 1) / 2] - q);
      w_row_impedance(m, s, r, m->jnt_solref[j], m->jnt_solimp[j], dist, m->jnt_margin[j],
                      m->dof_invweight0[m->jnt_dofadr[j]], 0);
    } else {
      int c = id;
      int p = s.con_cpair[c];
      int b1 = m->geom_bodyid[s.con_geom1[c]], b2 = m->geom_bodyid[s.con_geom2[c]];
      double diag = m->body_invweight0[b1][0] + m->body_invweight0[b2][0];
      double incl = m->cpair_margin[p] - m->cpair_gap[p];
      w_row_impedance(m, s, r, m->cpair_solref[p], m->cpair_solimp[p], s.con_dist[c], incl, diag, k > 0);
    }
  }
  SYNC();
  /* phase C: elliptic regularisation per contact */
  for (int g = tid; g < s.ngrp; g += NT) {
    if (s.grp_type[g] != G_CONTACT) continue;
    int c = s.grp_id[g], r = s.grp_row[g];
    int p = s.con_cpair[c];
    double fr0 = m->cpair_friction[p][0];
    s.efc_R[r + 1] = s.efc_R[r] / m->impratio;
    s.con_mu[c] = fr0 * sqrt(s.efc_R[r + 1] / s.efc_R[r]);
    s.efc_R[r + 2] = s.efc_R[r + 1] * fr0 * fr0 / (m->cpair_friction[p][1] * m->cpair_friction[p][1]);
  }
  SYNC();
  for (int i = tid; i < s.nefc; i += NT) s.efc_D[i] = 1.0 / s.efc_R[i];
  SYNC();
}

/* ================================================================== */
/* velocity stage                                                      */
/* ================================================================== */
template <int NT, class KS>
WD void w_com_vel(KModel m, const KPlan* __restrict__ pl, KS& s) {
  const int tid = w_lane();
  const int nb = m->nbody;
  if (tid < 6) s.cvel[0][tid] = 0;
  SYNC();
  for (int lvl = 1; lvl <= pl->nlevel; lvl++) {
    for (int i = tid; i < nb; i += NT) {
      if (i == 0 || pl->body_depth[i] != lvl) continue;
      double cv[6];
      for (int k = 0; k < 6; k++) cv[k] = s.cvel[m->body_parentid[i]][k];
      int bda = m->body_dofadr[i];
      for (int j = 0; j < m->body_dofnum[i]; j++) {
        int dof = bda + j;
        int jt = m->jnt_type[m->dof_jntid[dof]];
        if (jt == UR3E_JNT_FREE) {
          for (int k = 0; k < 3; k++)
            for (int r = 0; r < 6; r++) w_cdof_dot(s)[dof + k][r] = 0;
          double tmp[6] = {0, 0, 0, 0, 0, 0};
          for (int k = 0; k < 3; k++)
            for (int r = 0; r < 6; r++) tmp[r] += s.cdof[dof + k][r] * s.qvel[dof + k];
          for (int r = 0; r < 6; r++) cv[r] += tmp[r];
          for (int k = 3; k < 6; k++) k_cross_motion(w_cdof_dot(s)[dof + k], cv, s.cdof[dof + k]);
          for (int r = 0; r < 6; r++) tmp[r] = 0;
          for (int k = 3; k < 6; k++)
            for (int r = 0; r < 6; r++) tmp[r] += s.cdof[dof + k][r] * s.qvel[dof + k];
          for (int r = 0; r < 6; r++) cv[r] += tmp[r];
          j += 5;
        } else {
          k_cross_motion(w_cdof_dot(s)[dof], cv, s.cdof[dof]);
          for (int r = 0; r < 6; r++) cv[r] += s.cdof[dof][r] * s.qvel[dof];
        }
      }
      for (int k = 0; k < 6; k++) s.cvel[i][k] = cv[k];
    }
    SYNC();
  }
}

template <int NT, class KS>
WD void w_rne_passive(KModel m, const KPlan* __restrict__ pl, KS& s) {
  const int tid = w_lane();
  const int nb = m->nbody, nv = NVOF(KS, m);
  auto cacc = w_cacc(s);
  auto cfrc = w_cfrc(s);
  constexpr bool REG = (NT == 64 && KS::OVERLAY);
  if constexpr (REG) {
    r_cfrc(m, s); /* cacc came from r_vel_acc */
  } else {
  if (tid == 0) {
    cacc[0][0] = cacc[0][1] = cacc[0][2] = 0;
    cacc[0][3] = -m->gravity[0]; cacc[0][4] = -m->gravity[1]; cacc[0][5] = -m->gravity[2];
    for (int k = 0; k < 6; k++) cfrc[0][k] = 0;
  }
  SYNC();
  for (int lvl = 1; lvl <= pl->nlevel; lvl++) {
    for (int i = tid; i < nb; i += NT) {
      if (i == 0 || pl->body_depth[i] != lvl) continue;
      double tmp[6] = {0, 0, 0, 0, 0, 0};
      int bda = m->body_dofadr[i];
      for (int j = 0; j < m->body_dofnum[i]; j++)
        for (int r = 0; r < 6; r++) tmp[r] += w_cdof_dot(s)[bda + j][r] * s.qvel[bda + j];
      int p = m->body_parentid[i];
      for (int r = 0; r < 6; r++) cacc[i][r] = cacc[p][r] + tmp[r];
    }
    SYNC();
  }
  if (tid >= 1 && tid < nb) {
    int i = tid;
    double f1[6], f2[6], f3[6];
    k_mul_inert_vec(f1, s.cinert[i], cacc[i]);
    k_mul_inert_vec(f2, s.cinert[i], s.cvel[i]);
    k_cross_force(f3, s.cvel[i], f2);
    for (int r = 0; r < 6; r++) cfrc[i][r] = f1[r] + f3[r];
  }
  SYNC();
  if (tid < 6) {
    for (int i = nb - 1; i > 0; i--) {
      int p = m->body_parentid[i];
      if (p > 0) cfrc[p][tid] += cfrc[i][tid];
    }
  }
  SYNC();
  }
  if constexpr (W_FLAT_DYN) {
    /* the same terms from the plan's per-dof and per-actuator rows (one load level) */
    if (tid < nv) {
      const int v = tid;
      const int bv = pl->pd_i[v][0], qa = pl->pd_i[v][1];
      const double k = pl->pd_d[v][0], spring = pl->pd_d[v][1], b = pl->pd_d[v][2];
      s.qfrc_bias[v] = k_dot6(s.cdof[v], cfrc[bv]);
      double pf = 0;
      if (k != 0) pf = -k * (s.qpos[qa] - spring);
      if (b != 0) pf -= b * s.qvel[v];
      s.qfrc_passive[v] = pf;
    }
    for (int a = tid; a < m->nu; a += NT) {
      int ai[4];
      double ad[9];
      for (int q = 0; q < 4; q++) ai[q] = pl->pa_i[a][q];
      for (int q = 0; q < 8; q++) ad[q] = pl->pa_d[a][q];
      double vel = 0;
      for (int v = 0; v < nv; v++) vel += pl->act_moment[a][v] * s.qvel[v];
      double ctrl = s.ctrl[a];
      if (ai[0]) {
        if (ctrl < ad[0]) ctrl = ad[0];
        if (ctrl > ad[1]) ctrl = ad[1];
      }
      double f = ad[2] * ctrl;
      if (ai[1]) f += ad[3] + ad[4] * s.actuator_length[a] + ad[5] * vel;
      if (ai[2]) {
        if (f < ad[6]) f = ad[6];
        if (f > ad[7]) f = ad[7];
      }
      s.act_force[a] = f;
    }
  } else {
  if (tid < nv) {
    int v = tid;
    s.qfrc_bias[v] = k_dot6(s.cdof[v], cfrc[m->dof_bodyid[v]]);
    /* passive: spring (per joint, one dof here) then damping */
    double pf = 0;
    int j = m->dof_jntid[v];
    double k = m->jnt_stiffness[j];
    if (k != 0 && (m->jnt_type[j] == UR3E_JNT_HINGE || m->jnt_type[j] == UR3E_JNT_SLIDE) && m->jnt_dofadr[j] == v) {
      int a = m->jnt_qposadr[j];
      pf = -k * (s.qpos[a] - m->qpos_spring[a]);
    }
    double b = m->dof_damping[v];
    if (b != 0) pf -= b * s.qvel[v];
    s.qfrc_passive[v] = pf;
  }
  for (int a = tid; a < m->nu; a += NT) {
    double vel = 0;
    for (int v = 0; v < nv; v++) vel += pl->act_moment[a][v] * s.qvel[v];
    double ctrl = s.ctrl[a];
    if (m->act_ctrllimited[a]) {
      if (ctrl < m->act_ctrlrange[a][0]) ctrl = m->act_ctrlrange[a][0];
      if (ctrl > m->act_ctrlrange[a][1]) ctrl = m->act_ctrlrange[a][1];
    }
    double f = m->act_gainprm[a][0] * ctrl;
    if (m->act_biastype[a] == UR3E_BIAS_AFFINE)
      f += m->act_biasprm[a][0] + m->act_biasprm[a][1] * s.actuator_length[a] + m->act_biasprm[a][2] * vel;
    if (m->act_forcelimited[a]) {
      if (f < m->act_forcerange[a][0]) f = m->act_forcerange[a][0];
      if (f > m->act_forcerange[a][1]) f = m->act_forcerange[a][1];
    }
    s.act_force[a] = f;
  }
  }
  SYNC();
  if (tid < nv) {
    int v = tid;
    double sa = 0;
    for (int a = 0; a < m->nu; a++) sa += pl->act_moment[a][v] * s.act_force[a];
    s.qfrc_smooth[v] = s.qfrc_passive[v] - s.qfrc_bias[v] + sa;
  }
  SYNC();
}

/* ================================================================== */
/* Newton solver                                                       */
/* ================================================================== */
/* per-row force/state and cost contribution (rowflag: adds to the cost) */
template <int NT, class KS>
WD void w_constraint_update(KModel m, KS& s) {
  const int tid = w_lane();
  const int nefc = s.nefc;
  for (int i = tid; i < nefc; i += NT) {
    int t = s.efc_type[i];
    double D = s.efc_D[i], R = s.efc_R[i];
    double jar = s.jar[i];
    if (t == CN_EQUALITY) {
      s.efc_force[i] = -D * jar;
      s.u.row.F[i] = 0.5 * D * jar * jar; s.rowflag[i] = 1;
      s.efc_state[i] = ST_QUADRATIC;
    } else if (t == CN_FRICTION_DOF) {
      double fl = s.efc_floss[i];
      if (jar <= -R * fl) {
        s.efc_force[i] = fl;
        s.u.row.F[i] = -0.5 * R * fl * fl - fl * jar;
        s.efc_state[i] = ST_LINEARNEG;
      } else if (jar >= R * fl) {
        s.efc_force[i] = -fl;
        s.u.row.F[i] = -0.5 * R * fl * fl + fl * jar;
        s.efc_state[i] = ST_LINEARPOS;
      } else {
        s.efc_force[i] = -D * jar;
        s.u.row.F[i] = 0.5 * D * jar * jar;
        s.efc_state[i] = ST_QUADRATIC;
      }
      s.rowflag[i] = 1;
    } else if (t == CN_LIMIT_JOINT) {
      if (jar >= 0) {
        s.efc_force[i] = 0;
        s.efc_state[i] = ST_SATISFIED;
        s.rowflag[i] = 0;
      } else {
        s.efc_force[i] = -D * jar;
        s.u.row.F[i] = 0.5 * D * jar * jar; s.rowflag[i] = 1;
        s.efc_state[i] = ST_QUADRATIC;
      }
    } else {
      int c = s.efc_id[i];
      if (s.con_efc[c] != i) continue; /* cone handled at its first row */
      int p = s.con_cpair[c];
      const int dim = 3;
      double mu = s.con_mu[c];
      double U[3];
      U[0] = s.jar[i] * mu;
      for (int j = 1; j < dim; j++) U[j] = s.jar[i + j] * m->cpair_friction[p][j - 1];
      double N = U[0];
      double T2 = 0;
      for (int j = 1; j < dim; j++) T2 += U[j] * U[j];
      double T = sqrt(T2);
      if (N >= mu * T || (T <= 0 && N >= 0)) {
        for (int j = 0; j < dim; j++) {
          s.efc_force[i + j] = 0;
          s.efc_state[i + j] = ST_SATISFIED;
          s.rowflag[i + j] = 0;
        }
      } else if (mu * N + T <= 0 || (T <= 0 && N < 0)) {
        for (int j = 0; j < dim; j++) {
          s.efc_force[i + j] = -s.efc_D[i + j] * s.jar[i + j];
          s.u.row.F[i + j] = 0.5 * s.efc_D[i + j] * s.jar[i + j] * s.jar[i + j];
          s.rowflag[i + j] = 1;
          s.efc_state[i + j] = ST_QUADRATIC;
        }
      } else {
        double Dm = s.efc_D[i] / (mu * mu * (1 + mu * mu));
        double NT_ = N - mu * T;
        s.u.row.F[i] = 0.5 * Dm * NT_ * NT_;
        s.rowflag[i] = 1;
        s.rowflag[i + 1] = 0;
        s.rowflag[i + 2] = 0;
        s.efc_force[i] = -Dm * NT_ * mu;
        for (int j = 1; j < dim; j++) s.efc_force[i + j] = Dm * NT_ * mu * U[j] / T * m->cpair_friction[p][j - 1];
        for (int j = 0; j < dim; j++) s.efc_state[i + j] = ST_CONE;
      }
    }
  }
  SYNC();
}

template <int NT, class KS>
WD void w_eval_state(KModel m, KS& s, const double* qacc) {
  const int tid = w_lane();
  const int nv = NVOF(KS, m);
  for (int i = tid; i < nv + s.nefc; i += NT) {
    if (i < nv) {
      double v = 0;
      for (int j = 0; j < nv; j++) v += s.qM[i][j] * qacc[j];
      s.Ma[i] = v;
    } else {
      int r = i - nv;
      double v = 0;
      for (int k = 0; k < nv; k++) v += s.efc_J[r][k] * qacc[k];
      s.jar[r] = v - s.efc_aref[r];
    }
  }
  SYNC();
  w_constraint_update<NT>(m, s);
  /* lane 0: Gauss term (k order), lane 1: constraint cost (row order) -- one loop, two data streams */
  if (tid < 2) {
    double acc = 0;
    int len = tid == 0 ? nv : s.nefc;
    for (int i = 0; i < len; i++) {
      double term = tid == 0 ? (s.Ma[i] - s.qfrc_smooth[i]) * (qacc[i] - s.qacc_smooth[i])
                             : (s.rowflag[i] ? s.u.row.F[i] : 0.0);
      if (tid == 0 || s.rowflag[i]) acc += term;
    }
    s.tmpv[tid] = acc;
  }
  SYNC();
  if (tid == 0) {
    s.gauss = 0.5 * s.tmpv[0];
    s.cost = s.gauss + s.tmpv[1];
  }
  SYNC();
}

template <int NT, class KS>
WD void w_compute_grad(KModel m, KS& s) {
  const int tid = w_lane();
  const int nv = NVOF(KS, m);
  if (tid < nv) {
    int k = tid;
    double f = 0;
    for (int i = 0; i < s.nefc; i++) f += s.efc_J[i][k] * s.efc_force[i];
    s.qfrc_constraint[k] = f;
    s.grad[k] = s.Ma[k] - s.qfrc_smooth[k] - f;
  }
  SYNC();
}

template <int NT, class KS>
WD void w_hessian_factor(KModel m, KS& s) {
  const int tid = w_lane();
  const int nv = NVOF(KS, m);
  /* cone Hessians (middle zone), one lane per contact */
  for (int c = tid; c < s.ncon; c += NT) {
    int i = s.con_efc[c];
    if (i < 0 || s.efc_state[i] != ST_CONE) continue;
    int p = s.con_cpair[c];
    const int dim = 3;
    double mu = s.con_mu[c];
    double U[3], sc[3];
    sc[0] = mu;
    U[0] = s.jar[i] * mu;
    for (int j = 1; j < dim; j++) {
      sc[j] = m->cpair_friction[p][j - 1];
      U[j] = s.jar[i + j] * sc[j];
    }
    double T2 = 0;
    for (int j = 1; j < dim; j++) T2 += U[j] * U[j];
    double T = sqrt(T2);
    double N = U[0];
    double Dm = s.efc_D[i] / (mu * mu * (1 + mu * mu));
    double Hc[3][3];
    Hc[0][0] = 1;
    for (int j = 1; j < dim; j++) {
      Hc[0][j] = -mu * U[j] / T;
      Hc[j][0] = Hc[0][j];
    }
    double muNT = mu * N / T;
    for (int j = 1; j < dim; j++)
      for (int k = 1; k < dim; k++) Hc[j][k] = (j == k ? mu * mu - muNT : 0.0) + muNT * U[j] * U[k] / T2;
    for (int j = 0; j < dim; j++)
      for (int k = 0; k < dim; k++) s.con_Hc[c][3 * j + k] = Hc[j][k] * Dm * sc[j] * sc[k];
  }
  SYNC();
  /* H = M + J' D J + cone blocks, lower triangle, one lane per element, rows in oracle order */
  const int nel = nv * (nv + 1) / 2;
  for (int e = tid; e < nel; e += NT) {
    int r = 0, rem = e;
    while (rem > r) { rem -= r + 1; r++; }
    int c = rem;
    double h = s.qM[r][c];
    for (int i = 0; i < s.nefc; i++) {
      int st = s.efc_state[i];
      if (st == ST_QUADRATIC) {
        double jr = s.efc_J[i][r];
        if (jr == 0) continue;
        double djr = s.efc_D[i] * jr;
        h += djr * s.efc_J[i][c];
      } else if (st == ST_CONE && s.efc_type[i] == CN_CONTACT_ELLIPTIC) {
        int ci = s.efc_id[i];
        if (s.con_efc[ci] != i) continue;
        const double* Hc = s.con_Hc[ci];
        double t[3];
        for (int j = 0; j < 3; j++) {
          double acc = 0;
          for (int k = 0; k < 3; k++) acc += Hc[3 * j + k] * s.efc_J[i + k][r];
          t[j] = acc;
        }
        double acc = 0;
        for (int j = 0; j < 3; j++) acc += s.efc_J[i + j][c] * t[j];
        h += acc;
      }
    }
    s.H[r][c] = h;
  }
  SYNC();
  WT(10);
  /* Cholesky H = L L' (lower), right-looking: element (i,k) receives the updates
     -= L[i][j]*L[k][j] for j = 0,1,... in the same order as the oracle's left-looking loop */
  for (int j = 0; j < nv; j++) {
    if (tid == 0) {
      double sum = s.H[j][j];
      if (sum < K_MINVAL) sum = K_MINVAL;
      s.H[j][j] = sqrt(sum);
    }
    SYNC();
    double ljj = s.H[j][j];
    for (int i = j + 1 + tid; i < nv; i += NT) s.H[i][j] = s.H[i][j] / ljj;
    SYNC();
    const int nt = nv - j - 1; /* trailing block (j+1..nv-1), lower triangle incl. diagonal */
    const int nel2 = nt * (nt + 1) / 2;
    for (int e = tid; e < nel2; e += NT) {
      int a = 0, rem = e;
      while (rem > a) { rem -= a + 1; a++; }
      int i = j + 1 + a, k = j + 1 + rem;
      s.H[i][k] -= s.H[i][j] * s.H[k][j];
    }
    SYNC();
  }
}

/* x = H^-1 b by column sweeps (oracle order: forward k ascending, back k descending) */
template <int NT, class KS>
WD void w_hessian_solve(KModel m, KS& s, double* x, const double* b) {
  const int tid = w_lane();
  const int nv = NVOF(KS, m);
  if (tid < nv) s.tmpv[tid] = b[tid];
  SYNC();
  for (int k = 0; k < nv; k++) {
    if (tid == 0) x[k] = s.tmpv[k] / s.H[k][k];
    SYNC();
    if (tid > k && tid < nv) s.tmpv[tid] -= s.H[tid][k] * x[k];
    SYNC();
  }
  if (tid < nv) s.tmpv[tid] = x[tid];
  SYNC();
  for (int i = nv - 1; i >= 0; i--) {
    if (tid == 0) x[i] = s.tmpv[i] / s.H[i][i];
    SYNC();
    if (tid < i) s.tmpv[tid] -= s.H[i][tid] * x[i];
    SYNC();
  }
}

/* line-search 1-D evaluation at step a: per-row contributions + ordered sums on lane 0 */
template <int NT, class KS>
WD void w_ls_eval(KModel m, KS& s, double a) {
  const int tid = w_lane();
  const int nefc = s.nefc;
  for (int i = tid; i < nefc; i += NT) {
    int t = s.efc_type[i];
    double D = s.efc_D[i], R = s.efc_R[i];
    double x = s.jar[i] + a * s.Jv[i];
    double v = s.Jv[i];
    double F = 0, dF = 0, d2F = 0;
    int flag = 0; /* 1: F,dF,d2F; 2: F,dF only */
    if (t == CN_EQUALITY) {
      F = 0.5 * D * x * x; dF = D * x * v; d2F = D * v * v; flag = 1;
    } else if (t == CN_FRICTION_DOF) {
      double fl = s.efc_floss[i];
      if (x <= -R * fl) { F = -0.5 * R * fl * fl - fl * x; dF = -fl * v; flag = 2; }
      else if (x >= R * fl) { F = -0.5 * R * fl * fl + fl * x; dF = fl * v; flag = 2; }
      else { F = 0.5 * D * x * x; dF = D * x * v; d2F = D * v * v; flag = 1; }
    } else if (t == CN_LIMIT_JOINT) {
      if (x < 0) { F = 0.5 * D * x * x; dF = D * x * v; d2F = D * v * v; flag = 1; }
    } else {
      int c = s.efc_id[i];
      if (s.con_efc[c] != i) continue;
      int p = s.con_cpair[c];
      const int dim = 3;
      double mu = s.con_mu[c];
      double U[3], V[3];
      U[0] = (s.jar[i] + a * s.Jv[i]) * mu;
      V[0] = s.Jv[i] * mu;
      for (int j = 1; j < dim; j++) {
        U[j] = (s.jar[i + j] + a * s.Jv[i + j]) * m->cpair_friction[p][j - 1];
        V[j] = s.Jv[i + j] * m->cpair_friction[p][j - 1];
      }
      double N = U[0];
      double T2 = 0;
      for (int j = 1; j < dim; j++) T2 += U[j] * U[j];
      double T = sqrt(T2);
      s.rowflag[i + 1] = 0;
      s.rowflag[i + 2] = 0;
      if (N >= mu * T || (T <= 0 && N >= 0)) {
      } else if (mu * N + T <= 0 || (T <= 0 && N < 0)) {
        for (int j = 0; j < dim; j++) {
          double xj = s.jar[i + j] + a * s.Jv[i + j];
          double vj = s.Jv[i + j];
          double Dj = s.efc_D[i + j];
          s.u.row.F[i + j] = 0.5 * Dj * xj * xj;
          s.u.row.dF[i + j] = Dj * xj * vj;
          s.u.row.d2F[i + j] = Dj * vj * vj;
          s.rowflag[i + j] = 1;
        }
        continue;
      } else {
        double Dm = s.efc_D[i] / (mu * mu * (1 + mu * mu));
        double UV = 0, VV = 0;
        for (int j = 1; j < dim; j++) { UV += U[j] * V[j]; VV += V[j] * V[j]; }
        double NT_ = N - mu * T;
        double dNT = V[0] - mu * UV / T;
        double d2NT = -mu * (VV * T2 - UV * UV) / (T2 * T);
        F = 0.5 * Dm * NT_ * NT_;
        dF = Dm * NT_ * dNT;
        d2F = Dm * (dNT * dNT + NT_ * d2NT);
        flag = 1;
      }
    }
    s.u.row.F[i] = F; s.u.row.dF[i] = dF; s.u.row.d2F[i] = d2F;
    s.rowflag[i] = flag;
  }
  SYNC();
  /* lanes 0/1/2 accumulate F / dF / d2F in row order (same sequence as the oracle, run side by side) */
  if (tid < 3) {
    double acc = tid == 0 ? s.gauss + a * s.g1 + 0.5 * a * a * s.g2 : (tid == 1 ? s.g1 + a * s.g2 : s.g2);
    const double* arr = tid == 0 ? s.u.row.F : (tid == 1 ? s.u.row.dF : s.u.row.d2F);
    for (int i = 0; i < nefc; i++) {
      int f = s.rowflag[i];
      if (f && (tid < 2 || f == 1)) acc += arr[i];
    }
    s.tmpv[tid] = acc;
  }
  SYNC();
  s.lsF = s.tmpv[0]; s.lsdF = s.tmpv[1]; s.lsd2F = s.tmpv[2];
}

template <int NT, class KS>
WD double w_line_search(KModel m, KS& s) {
  const int tid = w_lane();
  const int nv = NVOF(KS, m);
  if (tid == 0) {
    double sn = 0;
    for (int k = 0; k < nv; k++) sn += s.search[k] * s.search[k];
    s.sred = sqrt(sn);
  }
  for (int i = tid; i < nv + s.nefc; i += NT) {
    if (i < nv) {
      double v = 0;
      for (int j = 0; j < nv; j++) v += s.qM[i][j] * s.search[j];
      s.Mv[i] = v;
    } else {
      int r = i - nv;
      double v = 0;
      for (int k = 0; k < nv; k++) v += s.efc_J[r][k] * s.search[k];
      s.Jv[r] = v;
    }
  }
  SYNC();
  double snorm = s.sred;
  if (snorm < K_MINVAL) return 0;
  if (tid < 2) {
    double acc = 0;
    for (int k = 0; k < nv; k++) acc += s.search[k] * (tid == 0 ? (s.Ma[k] - s.qfrc_smooth[k]) : s.Mv[k]);
    if (tid == 0) s.g1 = acc;
    else s.g2 = acc;
  }
  SYNC();
  double gtol = m->tolerance * m->ls_tolerance * snorm / s.scale;
  w_ls_eval<NT>(m, s, 0.0);
  double f0 = s.lsF, d0 = s.lsdF, h0 = s.lsd2F;
  if (d0 >= 0) return 0;
  double lo = 0.0, dlo = d0, hlo = h0;
  double hi = -1.0, dhi = 0, hhi = 0;
  double bestA = 0.0, bestF = f0;
  double a = -d0 / h0;
  for (int it = 0; it < m->ls_iterations; it++) {
    w_ls_eval<NT>(m, s, a);
    double f = s.lsF, df = s.lsdF, d2f = s.lsd2F;
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

template <int NT, class KS>
WD void w_solve_newton(KModel m, KS& s) {
  const int tid = w_lane();
  const int nv = NVOF(KS, m);
  if (s.nefc == 0) {
    if (tid < nv) { s.qacc[tid] = s.qacc_smooth[tid]; s.qfrc_constraint[tid] = 0; }
    SYNC();
    return;
  }
  if (tid == 0) s.scale = 1.0 / (m->meaninertia * (nv > 1 ? nv : 1));
  if (tid < nv) s.qacc[tid] = s.warm[tid];
  SYNC();
  w_eval_state<NT>(m, s, s.qacc);
  double cost_ws = s.cost;
  w_eval_state<NT>(m, s, s.qacc_smooth);
  double cost_sm = s.cost;
  if (cost_ws > cost_sm) {
    if (tid < nv) s.qacc[tid] = s.qacc_smooth[tid];
    SYNC();
  } else {
    w_eval_state<NT>(m, s, s.qacc);
  }
  w_compute_grad<NT>(m, s);
  WT(9);
  w_hessian_factor<NT>(m, s);
  WT(11);
  w_hessian_solve<NT>(m, s, s.xv, s.grad);
  if (tid < nv) s.search[tid] = -s.xv[tid];
  SYNC();
  WT(12);
  for (int iter = 0; iter < m->iterations; iter++) {
    double alpha = w_line_search<NT>(m, s);
    WT(13);
    if (alpha == 0) break;
    if (tid < nv) s.qacc[tid] += alpha * s.search[tid];
    SYNC();
    double oldcost = s.cost;
    w_eval_state<NT>(m, s, s.qacc);
    w_compute_grad<NT>(m, s);
    WT(14);
    if (tid == 0) {
      double gn = 0;
      for (int k = 0; k < nv; k++) gn += s.grad[k] * s.grad[k];
      s.sred = gn;
    }
    SYNC();
    double improvement = s.scale * (oldcost - s.cost);
    double gradient = s.scale * sqrt(s.sred);
    if (improvement < m->tolerance || gradient < m->tolerance) break;
    w_hessian_factor<NT>(m, s);
    WT(11);
    w_hessian_solve<NT>(m, s, s.xv, s.grad);
    if (tid < nv) s.search[tid] = -s.xv[tid];
    SYNC();
    WT(12);
  }
}

/* ================================================================== */
/* forward / step                                                      */
/* ================================================================== */
/* sensors: mj_rnePostConstraint + mjData.sensordata (oracle rne_post_constraint / sensors), the   */
/* full-capacity layout only -- the compact tier's overlaid LDS has no room for cinert/cvel/cdof_dot */
/* after the solve, so a handle with sensors on runs the full-capacity kernels (ur3e_batch_create)  */
/* ================================================================== */
/* oracle transform_force: torque reference point oldpos -> newpos, then optionally into frame rot */
KD void w_transform_force(double res[6], const double vec[6], const double newpos[3], const double oldpos[3],
                          const double* rot) {
  double dif[3] = {newpos[0] - oldpos[0], newpos[1] - oldpos[1], newpos[2] - oldpos[2]};
  double cros[3], tran[6];
  k_cross3(cros, dif, vec + 3);
  tran[0] = vec[0] - cros[0]; tran[1] = vec[1] - cros[1]; tran[2] = vec[2] - cros[2];
  tran[3] = vec[3]; tran[4] = vec[4]; tran[5] = vec[5];
  if (rot) {
    k_mat_t_vec3(res, rot, tran);
    k_mat_t_vec3(res + 3, rot, tran + 3);
  } else {
    for (int k = 0; k < 6; k++) res[k] = tran[k];
  }
}

template <int NT, class KS>
WD void w_sensors(KModel m, const KPlan* __restrict__ pl, KS& s) {
  if constexpr (!KS::OVERLAY) {
    const int tid = w_lane();
    const int nb = m->nbody;
    int post = 0;
    for (int k = 0; k < m->nsensor; k++) post |= m->sensor_type[k] == UR3E_SENS_TORQUE;
    if (post) {
      /* cfrc_ext, lane = body: every body sums its contributions in the oracle's order (contacts,
         then the connect rows that lead the constraint list) */
      for (int b = tid; b < nb; b += NT) {
        double ext[6] = {0, 0, 0, 0, 0, 0};
        if (b > 0) {
          for (int ci = 0; ci < s.ncon; ci++) {
            const int adr = s.con_efc[ci];
            if (adr < 0) continue;
            const int b1 = m->geom_bodyid[s.con_geom1[ci]], b2 = m->geom_bodyid[s.con_geom2[ci]];
            if (b != b1 && b != b2) continue;
            double lfrc[3] = {s.efc_force[adr], s.efc_force[adr + 1], s.efc_force[adr + 2]};
            double zero[3] = {0, 0, 0};
            double cfrc[6], com[6];
            k_mat_t_vec3(cfrc, s.con_frame[ci], zero);
            k_mat_t_vec3(cfrc + 3, s.con_frame[ci], lfrc);
            if (b == b1) {
              w_transform_force(com, cfrc, s.subtree_com[m->body_rootid[b]], s.con_pos[ci], 0);
              for (int r = 0; r < 6; r++) ext[r] -= com[r];
            }
            if (b == b2) {
              w_transform_force(com, cfrc, s.subtree_com[m->body_rootid[b]], s.con_pos[ci], 0);
              for (int r = 0; r < 6; r++) ext[r] += com[r];
            }
          }
          int i = 0;
          while (i < s.nefc && s.efc_type[i] == CN_EQUALITY) {
            const int e = s.efc_id[i];
            if (m->eq_type[e] == UR3E_EQ_CONNECT) {
              double cfrc[6] = {0, 0, 0, s.efc_force[i], s.efc_force[i + 1], s.efc_force[i + 2]};
              for (int side = 0; side < 2; side++) {
                const int k = side == 0 ? m->eq_obj1[e] : m->eq_obj2[e];
                if (k != b) continue;
                double pos[3], com[6];
                k_mat_vec3(pos, s.xmat[k], m->eq_data[e] + 3 * side);
                pos[0] += s.xpos[k][0]; pos[1] += s.xpos[k][1]; pos[2] += s.xpos[k][2];
                w_transform_force(com, cfrc, s.subtree_com[m->body_rootid[k]], pos, 0);
                if (side == 0)
                  for (int r = 0; r < 6; r++) ext[r] += com[r];
                else
                  for (int r = 0; r < 6; r++) ext[r] -= com[r];
              }
              i += 3;
            } else {
              i++;
            }
          }
        }
        for (int r = 0; r < 6; r++) s.cfrc_ext[b][r] = ext[r];
      }
      /* cacc, lane = component: each component's tree sweep is serial in body order */
      if (tid < 6) {
        const int k = tid;
        s.cacc[0][k] = k < 3 ? 0.0 : m->gravity[k - 3] * -1;
        for (int b = 1; b < nb; b++) {
          const int bda = m->body_dofadr[b], n = m->body_dofnum[b];
          double t = 0;
          if (n == 1) {
            t = w_cdof_dot(s)[bda][k] * s.qvel[bda];
          } else if (n > 1) {
            for (int j = 0; j < n; j++) {
              const double v = s.qvel[bda + j];
              if (v == 0) continue;
              t += w_cdof_dot(s)[bda + j][k] * v;
            }
          }
          double c = s.cacc[m->body_parentid[b]][k] + t;
          t = 0;
          if (n == 1) {
            t = s.cdof[bda][k] * s.qacc[bda];
          } else if (n > 1) {
            for (int j = 0; j < n; j++) {
              const double a = s.qacc[bda + j];
              if (a == 0) continue;
              t += s.cdof[bda + j][k] * a;
            }
          }
          s.cacc[b][k] = c + t;
        }
      }
      SYNC();
      /* cfrc_int before accumulation, lane = body */
      for (int b = 1 + tid; b < nb; b += NT) {
        double f[6], tmp[6], tmp1[6];
        k_mul_inert_vec(f, s.cinert[b], s.cacc[b]);
        k_mul_inert_vec(tmp, s.cinert[b], s.cvel[b]);
        k_cross_force(tmp1, s.cvel[b], tmp);
        for (int r = 0; r < 6; r++) f[r] += tmp1[r];
        for (int r = 0; r < 6; r++) s.cfrc_int[b][r] = f[r] - s.cfrc_ext[b][r];
      }
      SYNC();
      /* accumulate children into parents, lane = component, reverse body order */
      if (tid < 6)
        for (int b = nb - 1; b > 0; b--) {
          const int p = m->body_parentid[b];
          if (p) s.cfrc_int[p][tid] += s.cfrc_int[b][tid];
        }
      SYNC();
    }
    /* sensordata in declaration order, lane = sensor */
    for (int k = tid; k < m->nsensor; k += NT) {
      double* out = s.sensordata + m->sensor_adr[k];
      const int obj = m->sensor_objid[k];
      const int type = m->sensor_type[k];
      if (type == UR3E_SENS_TOUCH) {
        int nt = 0;
        for (int j = 0; j < k; j++) nt += m->sensor_type[j] == UR3E_SENS_TOUCH;
        out[0] = s.touch[nt];
      } else if (type == UR3E_SENS_ACTUATORFRC) {
        out[0] = s.act_force[obj];
      } else {
        const int body = m->site_bodyid[obj];
        double res[6];
        w_transform_force(res, s.cfrc_int[body], s.site_xpos[obj], s.subtree_com[m->body_rootid[body]],
                          s.site_xmat[obj]);
        out[0] = res[0]; out[1] = res[1]; out[2] = res[2];
      }
    }
    SYNC();
  }
}

/* ================================================================== */
/* part (compact tier, the queue's split units): 0 = the whole forward pass; 1 = up to the smooth
   acceleration (everything before the constraint solver), 2 = the rest, from the state part 1 left in
   LDS.  Part 1's last stage and part 2's first read and write only the working set, so a part-1 unit
   can hand the working set to another workgroup, which runs part 2 with the same bits. */
/* touch = false (compact tier): skip the touch sensors -- the caller's later forward pass of the same
   env-step recomputes them before anything reads them (w_commit reads the last pass's) */
template <int NT, class KS>
WD void w_forward(KModel m, const KPlan* __restrict__ pl, KS& s, int part = 0, bool touch = true) {
  const int tid = w_lane();
  const int nv = NVOF(KS, m);
  constexpr bool REG = (NT == 64 && KS::OVERLAY); /* compact tier: ur3e_wave_r.h */
  if (REG && part == 2) goto solve;
  {
  /* diagnostic builds only (-DUR3E_DOUBLE_STAGE=k): the compact tier runs idempotent stage k twice, so
     the difference of SQ_INSTS_VALU against the normal build is that stage's instruction count
     (tools/stage_insts.py); results are unchanged */
#ifndef UR3E_DOUBLE_STAGE
#define UR3E_DOUBLE_STAGE -1
#endif
#define W_DBL(k, stmt) do { stmt; if (REG && UR3E_DOUBLE_STAGE == (k)) { stmt; } } while (0)
  static_assert(!KS::OVERLAY || REG, "the overlaid layout is only valid for the 64-lane register path");
  WT(23);
  if constexpr (REG) {
    /* the main.xml-specialised kernels only run on models with <= 1 joint per body (host check), so
       the general per-level pass is not compiled into them */
    if constexpr (KS::STATIC_TREE) W_DBL(0, r_kinematics(m, pl, s));
    else if (pl->max_jntnum <= 1) r_kinematics(m, pl, s);
    else w_kinematics<NT>(m, pl, s);
  } else {
    w_kinematics<NT>(m, pl, s);
  }
  WT(0);
  w_com_pos<NT>(m, pl, s);
  WT(1);
  w_crb<NT>(m, pl, s);
  if constexpr (!REG) {
    for (int e = tid; e < nv * nv; e += NT) s.H[e / nv][e % nv] = s.qM[e / nv][e % nv];
    SYNC();
    WT(2);
    w_factor_tree<NT>(m, pl, s.H, s.LDinv, s.tmpv);
  }
  WT(3);
  if constexpr (KS::OVERLAY) {
    /* velocity-dependent forces first: their scratch shares bytes with the constraint rows */
    W_DBL(6, r_vel_acc(m, pl, s));
    /* the epilogue's site velocities (w_obs_v2), while cvel (KB) is alive */
    if (tid < 2) {
      const int site = tid == 0 ? m->id_site_tcp : m->id_site_handle;
      double v[6] = {0, 0, 0, 0, 0, 0};
      if (site >= 0) {
        if (W_FLAT_PAIRS) w_site_velocity(m, s, site, v, pl->sv_body[tid], pl->sv_root[tid]);
        else w_site_velocity(m, s, site, v);
      }
      for (int k = 0; k < 6; k++) s.site_vel[tid][k] = v[k];
    }
    WT(6);
    W_DBL(7, w_rne_passive<NT>(m, pl, s));
    WT(7);
  }
  W_DBL(4, w_collision<NT>(m, pl, s));
  WT(4);
  if (KS::BAIL && s.ovf) return;
  if constexpr (REG && KS::RHL) {
    /* the smooth acceleration before the constraint rows (it reads neither): its tree solve's LDS transpose
       shares bytes with the rows' R / D / aref (KSX::RHL) */
    double x;
    W_DBL(8, x = r_tree_solve(m, pl, s, false, tid < nv ? s.qfrc_smooth[tid] : 0.0));
    if (tid < nv) s.qacc_smooth[tid] = x;
    SYNC();
    WT(8);
  }
  W_DBL(5, w_make_constraint<NT>(m, pl, s));
  WT(5);
  if (KS::BAIL && s.ovf) return;
  if constexpr (!KS::OVERLAY) {
    if constexpr (REG) r_vel_acc(m, pl, s);
    else w_com_vel<NT>(m, pl, s);
    WT(6);
    w_rne_passive<NT>(m, pl, s);
    WT(7);
  }
  if constexpr (REG && !KS::RHL) {
    double x;
    W_DBL(8, x = r_tree_solve(m, pl, s, false, tid < nv ? s.qfrc_smooth[tid] : 0.0));
    if (tid < nv) s.qacc_smooth[tid] = x;
    SYNC();
    WT(8);
  } else if constexpr (!REG) {
    w_solve_tree<NT>(m, pl, s.H, s.LDinv, s.qacc_smooth, s.qfrc_smooth);
    WT(8);
  }
  if (REG && part == 1) return;
  }
solve:
  if constexpr (REG)
    W_DBL(15, r_solve_newton(m, pl, s));
  else
    w_solve_newton<NT>(m, s);
  WT(15);
  /* touch sensors, oracle sensor_touch: sum over contacts (in contact order) of the normal force
     of contacts on the sensor's body whose ray hits the site box */
  if constexpr (NT == 64 && KS::MAXCON <= 16) {
    if (touch) {
    /* lane = (sensor, contact): every contact tested at once, then an ordered per-sensor sum with
       -0.0 (the exact additive identity) for contacts that do not count */
    const int ts = tid >> 4, ci = tid & 15;
    double val = -0.0;
    if (ts < m->ntouch && ci < s.ncon) {
      const int site = m->touch_site[ts];
      const int body = m->site_bodyid[site];
      const int adr = s.con_efc[ci];
      const int b1 = m->geom_bodyid[s.con_geom1[ci]], b2 = m->geom_bodyid[s.con_geom2[ci]];
      if (adr >= 0 && (body == b1 || body == b2)) {
        const double fn = s.efc_force[adr];
        if (fn > 0) {
          double sp[3], sm[9], ss[3];
          for (int k = 0; k < 3; k++) { sp[k] = s.site_xpos[site][k]; ss[k] = m->site_size[site][k]; }
          for (int k = 0; k < 9; k++) sm[k] = s.site_xmat[site][k];
          double ray[3];
          if constexpr (KS::OVERLAY) { ray[0] = s.con_n[ci][0]; ray[1] = s.con_n[ci][1]; ray[2] = s.con_n[ci][2]; }
          else { ray[0] = s.con_frame[ci][0]; ray[1] = s.con_frame[ci][1]; ray[2] = s.con_frame[ci][2]; }
          if (body == b2) { ray[0] = -ray[0]; ray[1] = -ray[1]; ray[2] = -ray[2]; }
          double cp[3] = {s.con_pos[ci][0], s.con_pos[ci][1], s.con_pos[ci][2]};
          if (k_ray_box_hit(sp, sm, ss, cp, ray)) val = fn;
        }
      }
    }
    const int nt = m->ntouch, nc = s.ncon;
    double mine = 0;
    for (int k = 0; k < nt; k++) {
      double sum = 0;
      for (int c = 0; c < nc; c++) sum += rl(val, (k << 4) + c);
      if (tid == k) mine = sum;
    }
    if (tid < nt) s.touch[tid] = mine;
    }
    WT(21);
  } else if (tid < m->ntouch) {
    const int site = m->touch_site[tid];
    const int body = m->site_bodyid[site];
    double sp[3], sm[9], ss[3];
    for (int k = 0; k < 3; k++) { sp[k] = s.site_xpos[site][k]; ss[k] = m->site_size[site][k]; }
    for (int k = 0; k < 9; k++) sm[k] = s.site_xmat[site][k];
    double sum = 0;
    for (int ci = 0; ci < s.ncon; ci++) {
      const int adr = s.con_efc[ci];
      if (adr < 0) continue;
      const int b1 = m->geom_bodyid[s.con_geom1[ci]], b2 = m->geom_bodyid[s.con_geom2[ci]];
      if (body != b1 && body != b2) continue;
      const double fn = s.efc_force[adr];
      if (fn <= 0) continue;
      double ray[3];
      if constexpr (KS::OVERLAY) { ray[0] = s.con_n[ci][0]; ray[1] = s.con_n[ci][1]; ray[2] = s.con_n[ci][2]; }
      else { ray[0] = s.con_frame[ci][0]; ray[1] = s.con_frame[ci][1]; ray[2] = s.con_frame[ci][2]; }
      if (body == b2) { ray[0] = -ray[0]; ray[1] = -ray[1]; ray[2] = -ray[2]; }
      double cp[3] = {s.con_pos[ci][0], s.con_pos[ci][1], s.con_pos[ci][2]};
      if (k_ray_box_hit(sp, sm, ss, cp, ray)) sum += fn;
    }
    s.touch[tid] = sum;
  }
  SYNC();
  if constexpr (!KS::OVERLAY) {
    if (s.sens) w_sensors<NT>(m, pl, s);
  }
}

/* mj_step pieces around the forward pass, so a caller can keep ONE inlined copy of w_forward
   (the kernel is large; a single copy keeps its instruction footprint down) */
template <int NT, class KS>
WD void w_step_pre(KModel m, KS& s) {
  const int tid = w_lane();
  const int nq = m->nq, nv = NVOF(KS, m);
  int bad = 0;
  for (int k = tid; k < nq; k += NT) bad |= k_is_bad(s.qpos[k]);
  for (int k = tid; k < nv; k += NT) bad |= k_is_bad(s.qvel[k]);
  if (w_any<NT>(bad)) {
    if (tid < nq) s.qpos[tid] = m->qpos0[tid];
    if (tid < nv) { s.qvel[tid] = 0; s.warm[tid] = 0; }
    if (tid == 0) s.nwarn++;
    SYNC();
  }
}

/* after the first forward of a substep: bad qacc -> reset state, returns 1 (forward again) */
template <int NT, class KS>
WD int w_step_badacc(KModel m, KS& s) {
  const int tid = w_lane();
  const int nq = m->nq, nv = NVOF(KS, m);
  int bad = 0;
  for (int k = tid; k < nv; k += NT) bad |= k_is_bad(s.qacc[k]);
  if (w_any<NT>(bad)) {
    if (tid < nq) s.qpos[tid] = m->qpos0[tid];
    if (tid < nv) { s.qvel[tid] = 0; s.warm[tid] = 0; }
    if (tid == 0) s.nwarn++;
    SYNC();
    return 1;
  }
  return 0;
}

/* mj_Euler's position update (free joints: quaternion integration) */
template <int NT, class KS>
WD void w_integrate_pos(KModel m, KS& s, double h) {
  const int tid = w_lane();
  for (int j = tid; j < m->njnt; j += NT) {
    int a = m->jnt_qposadr[j], v = m->jnt_dofadr[j];
    if (m->jnt_type[j] == UR3E_JNT_FREE) {
      s.qpos[a] += h * s.qvel[v];
      s.qpos[a + 1] += h * s.qvel[v + 1];
      s.qpos[a + 2] += h * s.qvel[v + 2];
      double w[3] = {s.qvel[v + 3], s.qvel[v + 4], s.qvel[v + 5]};
      double ang = h * k_normalize3(w);
      double qr[4];
      k_axis_angle_quat(qr, w, ang);
      double q[4] = {s.qpos[a + 3], s.qpos[a + 4], s.qpos[a + 5], s.qpos[a + 6]};
      k_normalize4(q);
      k_mul_quat(q, q, qr);
      s.qpos[a + 3] = q[0]; s.qpos[a + 4] = q[1]; s.qpos[a + 5] = q[2]; s.qpos[a + 6] = q[3];
    } else {
      s.qpos[a] += h * s.qvel[v];
    }
  }
}

template <int NT, class KS>
WD void w_step_euler(KModel m, const KPlan* __restrict__ pl, KS& s) {
  const int tid = w_lane();
  const int nv = NVOF(KS, m);
  /* Euler with implicit damping: (M + h D) qacc_int = qfrc_smooth + qfrc_constraint */
  WT(22);
  int damped = 0;
  for (int k = 0; k < nv; k++) damped |= m->dof_damping[k] > 0;
  double x = 0; /* qacc used for the velocity update, lane = dof */
  if constexpr (KS::OVERLAY) {
    /* the solve's result stays in the lane's register (no LDS vector) */
    if (!damped) x = tid < nv ? s.qacc[tid] : 0.0;
    else x = r_tree_solve(m, pl, s, true, tid < nv ? s.qfrc_smooth[tid] + s.qfrc_constraint[tid] : 0.0);
  } else {
    if (!damped) {
      if (tid < nv) s.xv[tid] = s.qacc[tid];
      SYNC();
    } else if constexpr (NT == 64 && KS::MAXEFC <= 64) {
      double y = r_tree_solve(m, pl, s, true, tid < nv ? s.qfrc_smooth[tid] + s.qfrc_constraint[tid] : 0.0);
      if (tid < nv) s.xv[tid] = y;
      SYNC();
    } else {
      for (int e = tid; e < nv * nv; e += NT) s.H[e / nv][e % nv] = s.qM[e / nv][e % nv];
      SYNC();
      if (tid < nv) {
        s.H[tid][tid] += m->timestep * m->dof_damping[tid];
        s.fv[tid] = s.qfrc_smooth[tid] + s.qfrc_constraint[tid];
      }
      SYNC();
      w_factor_tree<NT>(m, pl, s.H, s.grad, s.tmpv);
      w_solve_tree<NT>(m, pl, s.H, s.grad, s.xv, s.fv);
    }
    if (tid < nv) x = s.xv[tid];
  }
  WT(16);
  double h = m->timestep;
  if (tid < nv) s.qvel[tid] += h * x;
  SYNC();
  w_integrate_pos<NT>(m, s, h);
  if (tid < nv) s.warm[tid] = s.qacc[tid];
  SYNC();
  WT(17);
}

template <int NT, class KS>
WD void w_step(KModel m, const KPlan* __restrict__ pl, KS& s) {
  w_step_pre<NT>(m, s);
  w_forward<NT>(m, pl, s);
  if (KS::BAIL && s.ovf) return;
  if (w_step_badacc<NT>(m, s)) {
    w_forward<NT>(m, pl, s);
    if (KS::BAIL && s.ovf) return;
  }
  w_step_euler<NT>(m, pl, s);
}

#endif /* UR3E_WAVE_H */
