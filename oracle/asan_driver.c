/* Sanitizer driver for the CPU oracle (test infrastructure only): runs the oracle's batch step under
   AddressSanitizer + UndefinedBehaviorSanitizer (make -C oracle asan).  Inputs are raw images written
   by tests/test_oracle_asan.py: the ur3e_model_t, the ur3e_config_t (ur3o_config mirrors its layout),
   and an actions file [steps][n][adim] f64.  Output: final obs [n][od], qpos [n][nq], qvel [n][nv]
   and the per-step rewards [steps][n], f64, for the test to compare with the normal build.
   usage: ur3e_oracle_asan MODEL CFG ACTIONS N STEPS ADIM OUT */
#include <stdio.h>
#include <stdlib.h>

#include "../include/ur3e_batch.h"

int ur3o_sizeof_env(void);
int ur3o_obs_dim(int task);
void ur3o_batch_init(const ur3e_model_t* m, const ur3e_config_t* c, int n, void* envs, double* obs);
void ur3o_batch_step(const ur3e_model_t* m, const ur3e_config_t* c, int n, void* envs, const double* actions,
                     int adim, double* obs, double* reward, unsigned char* terminated, unsigned char* truncated,
                     double* terminal_obs);
void ur3o_batch_get_state(const ur3e_model_t* m, int n, const void* envs, double* qpos, double* qvel, double* warm,
                          int* ncon);

static void* slurp(const char* path, size_t want) {
  FILE* f = fopen(path, "rb");
  if (!f) { perror(path); exit(2); }
  void* p = malloc(want);
  if (fread(p, 1, want, f) != want) { fprintf(stderr, "%s: short read\n", path); exit(2); }
  fclose(f);
  return p;
}

int main(int argc, char** argv) {
  if (argc != 8) { fprintf(stderr, "usage: %s MODEL CFG ACTIONS N STEPS ADIM OUT\n", argv[0]); return 2; }
  const int n = atoi(argv[4]), steps = atoi(argv[5]), adim = atoi(argv[6]);
  ur3e_model_t* m = (ur3e_model_t*)slurp(argv[1], sizeof(ur3e_model_t));
  ur3e_config_t* c = (ur3e_config_t*)slurp(argv[2], sizeof(ur3e_config_t));
  double* act = (double*)slurp(argv[3], sizeof(double) * (size_t)steps * n * adim);
  const int od = ur3o_obs_dim(c->task);
  void* envs = calloc((size_t)n, (size_t)ur3o_sizeof_env());
  double* obs = (double*)calloc((size_t)n * od, sizeof(double));
  double* tobs = (double*)calloc((size_t)n * od, sizeof(double));
  double* rew = (double*)calloc((size_t)steps * n, sizeof(double));
  unsigned char* term = (unsigned char*)calloc((size_t)n, 1);
  unsigned char* trunc = (unsigned char*)calloc((size_t)n, 1);
  ur3o_batch_init(m, c, n, envs, obs);
  for (int t = 0; t < steps; t++)
    ur3o_batch_step(m, c, n, envs, act + (size_t)t * n * adim, adim, obs, rew + (size_t)t * n, term, trunc, tobs);
  double* qp = (double*)calloc((size_t)n * m->nq, sizeof(double));
  double* qv = (double*)calloc((size_t)n * m->nv, sizeof(double));
  double* wa = (double*)calloc((size_t)n * m->nv, sizeof(double));
  int* nc = (int*)calloc((size_t)n, sizeof(int));
  ur3o_batch_get_state(m, n, envs, qp, qv, wa, nc);
  FILE* f = fopen(argv[7], "wb");
  if (!f) { perror(argv[7]); return 2; }
  fwrite(obs, sizeof(double), (size_t)n * od, f);
  fwrite(qp, sizeof(double), (size_t)n * m->nq, f);
  fwrite(qv, sizeof(double), (size_t)n * m->nv, f);
  fwrite(rew, sizeof(double), (size_t)steps * n, f);
  fclose(f);
  free(m); free(c); free(act); free(envs); free(obs); free(tobs); free(rew); free(term); free(trunc);
  free(qp); free(qv); free(wa); free(nc);
  return 0;
}
