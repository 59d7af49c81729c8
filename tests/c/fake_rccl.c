/* Test infrastructure: a stand-in for librccl's point-to-point API (ncclGroupStart/End, ncclSend/Recv,
 * ncclCommCount/UserRank, ncclGetErrorString) between CPU processes, so that the C ABI's gather
 * (ur3e_gather_rows, ur3e_amd/csrc/ur3e_gather.cpp) runs with several ranks and no GPU.  Loaded by the
 * library through UR3E_RCCL_LIB.  "Device" buffers are host memory; the stream is ignored.  A send
 * writes its bytes to <dir>/<src>_<dst>_<seq> (seq counts the messages of that rank pair, so the
 * receive order must match the send order, as in RCCL); a receive waits for that file and checks its
 * size against its own count (a mismatch returns an error instead of hanging). */
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#define MAXR 64
typedef struct {
  int rank, nranks;
  char dir[512];
  int sseq[MAXR], rseq[MAXR];
} fake_comm;

static size_t type_size(int t) { return t == 8 ? 8 : t == 1 ? 1 : 0; } /* ncclDouble, ncclUint8 */

void* fake_comm_init(int rank, int nranks, const char* dir) {
  if (nranks < 1 || nranks > MAXR || rank < 0 || rank >= nranks) return NULL;
  fake_comm* c = (fake_comm*)calloc(1, sizeof(fake_comm));
  c->rank = rank;
  c->nranks = nranks;
  snprintf(c->dir, sizeof c->dir, "%s", dir);
  return c;
}
void fake_comm_free(void* c) { free(c); }

int ncclGroupStart(void) { return 0; }
int ncclGroupEnd(void) { return 0; }
int ncclCommCount(void* comm, int* n) {
  *n = ((fake_comm*)comm)->nranks;
  return 0;
}
int ncclCommUserRank(void* comm, int* r) {
  *r = ((fake_comm*)comm)->rank;
  return 0;
}
const char* ncclGetErrorString(int rc) { return rc == 5 ? "fake: size mismatch" : "fake: error"; }

int ncclSend(const void* buf, size_t count, int type, int peer, void* comm, void* stream) {
  (void)stream;
  fake_comm* c = (fake_comm*)comm;
  if (peer < 0 || peer >= c->nranks) return 4;
  char tmp[600], fin[600];
  snprintf(fin, sizeof fin, "%s/%d_%d_%d", c->dir, c->rank, peer, c->sseq[peer]);
  snprintf(tmp, sizeof tmp, "%s.tmp", fin);
  c->sseq[peer]++;
  FILE* f = fopen(tmp, "wb");
  if (!f) return 3;
  const size_t nb = count * type_size(type);
  if (nb && fwrite(buf, 1, nb, f) != nb) { fclose(f); return 3; }
  fclose(f);
  return rename(tmp, fin) ? 3 : 0; /* the receiver sees whole messages only */
}

int ncclRecv(void* buf, size_t count, int type, int peer, void* comm, void* stream) {
  (void)stream;
  fake_comm* c = (fake_comm*)comm;
  if (peer < 0 || peer >= c->nranks) return 4;
  char fin[600];
  snprintf(fin, sizeof fin, "%s/%d_%d_%d", c->dir, peer, c->rank, c->rseq[peer]);
  c->rseq[peer]++;
  struct stat st;
  for (int k = 0; stat(fin, &st) != 0; k++) {
    if (k > 20000) return 3; /* 20 s */
    struct timespec ts = {0, 1000000};
    nanosleep(&ts, NULL);
  }
  const size_t nb = count * type_size(type);
  if ((size_t)st.st_size != nb) return 5;
  FILE* f = fopen(fin, "rb");
  if (!f) return 3;
  const size_t got = nb ? fread(buf, 1, nb, f) : 0;
  fclose(f);
  return got == nb ? 0 : 3;
}
