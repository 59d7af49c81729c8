/*
 * ur3e_oracle_probe.c — TEST INFRASTRUCTURE ONLY: accessors over one oracle
 * mjData-like record (ur3o_data) for the physics known-answer tests
 * (tests/test_physics_kat.py) and the independent constraint-solver check
 * (tests/test_solver_independent.py).  They copy the oracle's state, contacts
 * and constraint problem out to plain arrays; none of them computes physics.
 */
#include <string.h>

#include "ur3e_oracle.h"

int ur3o_data_init(const ur3e_model_t* m, ur3o_data* d) {
  ur3o_reset_data(m, d);
  return 0;
}

void ur3o_data_set(const ur3e_model_t* m, ur3o_data* d, const double* qpos, const double* qvel,
                   const double* ctrl) {
  if (qpos) memcpy(d->qpos, qpos, sizeof(double) * m->nq);
  if (qvel) memcpy(d->qvel, qvel, sizeof(double) * m->nv);
  if (ctrl) memcpy(d->ctrl, ctrl, sizeof(double) * m->nu);
}

void ur3o_data_set_warmstart(const ur3e_model_t* m, ur3o_data* d, const double* warm) {
  memcpy(d->qacc_warmstart, warm, sizeof(double) * m->nv);
}

void ur3o_data_get(const ur3e_model_t* m, const ur3o_data* d, double* qpos, double* qvel, double* qacc,
                   double* qacc_smooth, double* qfrc_smooth, double* qM) {
  int nv = m->nv;
  if (qpos) memcpy(qpos, d->qpos, sizeof(double) * m->nq);
  if (qvel) memcpy(qvel, d->qvel, sizeof(double) * nv);
  if (qacc) memcpy(qacc, d->qacc, sizeof(double) * nv);
  if (qacc_smooth) memcpy(qacc_smooth, d->qacc_smooth, sizeof(double) * nv);
  if (qfrc_smooth) memcpy(qfrc_smooth, d->qfrc_smooth, sizeof(double) * nv);
  if (qM)
    for (int r = 0; r < nv; r++)
      for (int c = 0; c < nv; c++) qM[r * nv + c] = d->qM[r][c];
}

/* contacts of the last forward: pos [n,3], frame [n,9], dist [n], geoms [n,2], friction [n,5],
   mu [n], efc_address [n]; returns ncon (at most maxc rows copied) */
int ur3o_data_contacts(const ur3o_data* d, int maxc, double* pos, double* frame, double* dist, int* geoms,
                       double* friction, double* mu, int* efc_address) {
  int n = d->ncon < maxc ? d->ncon : maxc;
  for (int i = 0; i < n; i++) {
    const ur3o_contact* c = d->contact + i;
    memcpy(pos + 3 * i, c->pos, sizeof(double) * 3);
    memcpy(frame + 9 * i, c->frame, sizeof(double) * 9);
    dist[i] = c->dist;
    geoms[2 * i] = c->geom1;
    geoms[2 * i + 1] = c->geom2;
    memcpy(friction + 5 * i, c->friction, sizeof(double) * 5);
    mu[i] = c->mu;
    efc_address[i] = c->efc_address;
  }
  return d->ncon;
}

/* constraint rows of the last forward: type, id, state [n]; J [n, nv]; pos, margin, frictionloss,
   diagApprox, R, D, vel, aref, force [n]; returns nefc (at most maxr rows copied) */
int ur3o_data_efc(const ur3e_model_t* m, const ur3o_data* d, int maxr, int* type, int* id, int* state,
                  double* J, double* pos, double* margin, double* floss, double* diag, double* R, double* D,
                  double* vel, double* aref, double* force) {
  int nv = m->nv;
  int n = d->nefc < maxr ? d->nefc : maxr;
  for (int i = 0; i < n; i++) {
    type[i] = d->efc_type[i];
    id[i] = d->efc_id[i];
    state[i] = d->efc_state[i];
    for (int k = 0; k < nv; k++) J[i * nv + k] = d->efc_J[i][k];
    pos[i] = d->efc_pos[i];
    margin[i] = d->efc_margin[i];
    floss[i] = d->efc_frictionloss[i];
    diag[i] = d->efc_diagApprox[i];
    R[i] = d->efc_R[i];
    D[i] = d->efc_D[i];
    vel[i] = d->efc_vel[i];
    aref[i] = d->efc_aref[i];
    force[i] = d->efc_force[i];
  }
  return d->nefc;
}

int ur3o_data_niter(const ur3o_data* d) { return d->solver_niter; }

void ur3o_data_sensordata(const ur3e_model_t* m, const ur3o_data* d, double* out) {
  memcpy(out, d->sensordata, sizeof(double) * m->nsensordata);
}

/* cfrc_int / cfrc_ext / cacc of the last forward's mj_rnePostConstraint, [nbody, 6] each */
void ur3o_data_rnepost(const ur3e_model_t* m, const ur3o_data* d, double* cacc, double* cfrc_int,
                       double* cfrc_ext) {
  memcpy(cacc, d->cacc, sizeof(double) * 6 * m->nbody);
  memcpy(cfrc_int, d->cfrc_int, sizeof(double) * 6 * m->nbody);
  memcpy(cfrc_ext, d->cfrc_ext, sizeof(double) * 6 * m->nbody);
}

/* geom poses of the last forward: xpos [ngeom, 3], xmat [ngeom, 9] (tier-routing diagnostics) */
void ur3o_data_geom_pose(const ur3e_model_t* m, const ur3o_data* d, double* xpos, double* xmat) {
  for (int g = 0; g < m->ngeom; g++) {
    memcpy(xpos + 3 * g, d->geom_xpos[g], sizeof(double) * 3);
    memcpy(xmat + 9 * g, d->geom_xmat[g], sizeof(double) * 9);
  }
}
