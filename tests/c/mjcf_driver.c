/* A non-Python caller of the C ABI (tests/test_abi_mjcf.py, tests/test_gpu_abi_mjcf.py): what a cgo / JNI /
   plain C host of the library does to get from the reference's files to a stepping handle.

     mjcf_driver image  MJCF OUT              ur3e_model_from_mjcf -> OUT (raw ur3e_model_t)
     mjcf_driver gains  YAML|- TASK OUT       ur3e_config_gains_from_yaml -> OUT (36 doubles)
     mjcf_driver step   MJCF YAML|- N STEPS ACTIONS OUT
                        ur3e_batch_create_from_mjcf (task CTRL, no auto-reset, no reset noise), reset,
                        ur3e_batch_set_state from the first N*(nq+nv) doubles of ACTIONS' header file
                        ACTIONS.state, STEPS steps of the [STEPS][N][nu] actions in ACTIONS, then
                        OUT = qpos [N][nq], qvel [N][nv], ncon [N] (as doubles)

   Built by the tests with gcc against include/ and ur3e_amd/_lib/libur3e_amd.so (+ libamdhip64 for the
   device buffers).  No Python in this process until the library embeds it for the MJCF compiler. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "ur3e_batch.h"

static int die(const char* what, int rc) {
  fprintf(stderr, "%s failed (%d): %s\n", what, rc, ur3e_last_error());
  return 1;
}

static double* read_doubles(const char* path, size_t* n) {
  FILE* f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  long sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  double* d = (double*)malloc((size_t)sz);
  *n = fread(d, sizeof(double), (size_t)sz / sizeof(double), f);
  fclose(f);
  return d;
}

int main(int argc, char** argv) {
  if (argc >= 4 && !strcmp(argv[1], "image")) {
    ur3e_model_t* m = (ur3e_model_t*)malloc(sizeof(ur3e_model_t));
    int rc = ur3e_model_from_mjcf(argv[2], NULL, m);
    if (rc) return die("ur3e_model_from_mjcf", rc);
    FILE* f = fopen(argv[3], "wb");
    fwrite(m, sizeof(ur3e_model_t), 1, f);
    fclose(f);
    printf("nq=%d nv=%d nu=%d nbody=%d ngeom=%d\n", m->nq, m->nv, m->nu, m->nbody, m->ngeom);
    return 0;
  }
  if (argc >= 5 && !strcmp(argv[1], "gains")) {
    ur3e_config_t c;
    memset(&c, 0, sizeof c);
    c.task = atoi(argv[3]);
    int rc = ur3e_config_gains_from_yaml(strcmp(argv[2], "-") ? argv[2] : NULL, &c);
    if (rc) return die("ur3e_config_gains_from_yaml", rc);
    FILE* f = fopen(argv[4], "wb");
    fwrite(c.task_gains, sizeof(double), 12, f);
    fwrite(c.joint_gains, sizeof(double), 12, f);
    fwrite(c.rot_joint_gains, sizeof(double), 12, f);
    fclose(f);
    return 0;
  }
  if (argc >= 8 && !strcmp(argv[1], "step")) {
    const int n = atoi(argv[4]), steps = atoi(argv[5]);
    ur3e_config_t c;
    memset(&c, 0, sizeof c);
    c.task = UR3E_TASK_CTRL;
    c.frame_skip = 1;
    c.max_episode_steps = 0;
    c.auto_reset = 0;
    c.reset_noise = 0;
    c.reset_key = -1;
    ur3e_batch_t* b = NULL;
    int rc = ur3e_batch_create_from_mjcf(argv[2], strcmp(argv[3], "-") ? argv[3] : NULL, &c, n, 0, &b);
    if (rc) return die("ur3e_batch_create_from_mjcf", rc);
    const int nq = ur3e_batch_nq(b), nv = ur3e_batch_nv(b), nu = ur3e_batch_nu(b), od = ur3e_batch_obs_dim(b);
    size_t na = 0, ns = 0;
    double* act = read_doubles(argv[6], &na);
    char sp[4096];
    snprintf(sp, sizeof sp, "%s.state", argv[6]);
    double* st = read_doubles(sp, &ns);
    if (!act || na != (size_t)steps * n * nu || !st || ns != (size_t)n * (nq + nv)) {
      fprintf(stderr, "input sizes: actions %zu (want %d), state %zu (want %d)\n", na, steps * n * nu, ns,
              n * (nq + nv));
      return 1;
    }
    double *d_obs, *d_rew, *d_tobs, *d_act, *d_qp, *d_qv;
    unsigned char *d_term, *d_trunc;
    int* d_ncon;
    if (hipMalloc((void**)&d_obs, sizeof(double) * n * od) || hipMalloc((void**)&d_tobs, sizeof(double) * n * od) ||
        hipMalloc((void**)&d_rew, sizeof(double) * n) || hipMalloc((void**)&d_act, sizeof(double) * n * nu) ||
        hipMalloc((void**)&d_qp, sizeof(double) * n * nq) || hipMalloc((void**)&d_qv, sizeof(double) * n * nv) ||
        hipMalloc((void**)&d_term, n) || hipMalloc((void**)&d_trunc, n) || hipMalloc((void**)&d_ncon, sizeof(int) * n))
      return die("hipMalloc", -2);
    if ((rc = ur3e_batch_reset(b, NULL, d_obs, NULL))) return die("ur3e_batch_reset", rc);
    hipMemcpy(d_qp, st, sizeof(double) * n * nq, hipMemcpyHostToDevice);
    hipMemcpy(d_qv, st + (size_t)n * nq, sizeof(double) * n * nv, hipMemcpyHostToDevice);
    if ((rc = ur3e_batch_set_state(b, d_qp, d_qv, NULL, NULL))) return die("ur3e_batch_set_state", rc);
    for (int t = 0; t < steps; t++) {
      hipMemcpy(d_act, act + (size_t)t * n * nu, sizeof(double) * n * nu, hipMemcpyHostToDevice);
      if ((rc = ur3e_batch_step(b, d_act, nu, d_obs, d_rew, d_term, d_trunc, d_tobs, NULL)))
        return die("ur3e_batch_step", rc);
    }
    if ((rc = ur3e_batch_get_state(b, d_qp, d_qv, NULL, NULL))) return die("ur3e_batch_get_state", rc);
    if ((rc = ur3e_batch_get_info(b, d_ncon, NULL, NULL, NULL, NULL))) return die("ur3e_batch_get_info", rc);
    if (hipDeviceSynchronize()) return die("hipDeviceSynchronize", -2);
    double* out = (double*)malloc(sizeof(double) * n * (nq + nv + 1));
    int* nc = (int*)malloc(sizeof(int) * n);
    hipMemcpy(out, d_qp, sizeof(double) * n * nq, hipMemcpyDeviceToHost);
    hipMemcpy(out + (size_t)n * nq, d_qv, sizeof(double) * n * nv, hipMemcpyDeviceToHost);
    hipMemcpy(nc, d_ncon, sizeof(int) * n, hipMemcpyDeviceToHost);
    for (int i = 0; i < n; i++) out[(size_t)n * (nq + nv) + i] = nc[i];
    FILE* f = fopen(argv[7], "wb");
    fwrite(out, sizeof(double), (size_t)n * (nq + nv + 1), f);
    fclose(f);
    ur3e_batch_destroy(b);
    printf("stepped %d envs x %d steps (nq=%d nv=%d nu=%d)\n", n, steps, nq, nv, nu);
    return 0;
  }
  fprintf(stderr, "usage: see the header comment\n");
  return 2;
}
