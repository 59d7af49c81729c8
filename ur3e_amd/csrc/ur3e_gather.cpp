/*
 * ur3e_gather.cpp — the C ABI's multi-GPU gather (include/ur3e_batch.h: ur3e_batch_gather) for hosts
 * that are not Python and hold their own RCCL communicator (the Python path gathers with
 * torch.distributed, ur3e_amd/envs/sharded.py).  One process per GPU, one handle per process, the same
 * env count on every rank (contiguous global env ids, env_id_offset = rank * n): the policy rank `root`
 * receives every rank's (obs, reward, terminated, truncated) after a step, ranks in order -- north_star
 * config C4's "RCCL gather of (obs, reward, done)".  The env path itself has no collective; this is a
 * point-to-point group (ncclSend from every rank, ncclRecv on the root, itself included) enqueued on the
 * caller's stream, so it orders after the step that produced the buffers.  librccl is loaded with dlopen
 * on first use: the library has no link-time RCCL dependency, and a communicator is the caller's
 * (ncclComm_t passed as void*).
 */
#include <dlfcn.h>
#include <stdlib.h>

#include <string>

#include "../../include/ur3e_batch.h"

__attribute__((visibility("hidden"))) int ur3e_internal_fail(int code, const char* msg);

namespace {

/* the RCCL entry points used here (rccl.h: ncclResult_t is an enum, ncclComm_t a pointer) */
struct Rccl {
  int (*GroupStart)(void) = nullptr;
  int (*GroupEnd)(void) = nullptr;
  int (*Send)(const void*, size_t, int, int, void*, void*) = nullptr;
  int (*Recv)(void*, size_t, int, int, void*, void*) = nullptr;
  int (*CommCount)(void*, int*) = nullptr;
  int (*CommUserRank)(void*, int*) = nullptr;
  const char* (*GetErrorString)(int) = nullptr;
  bool ok = false;
};
constexpr int kUint8 = 1, kFloat64 = 8; /* ncclUint8, ncclDouble */

int fail(int code, const std::string& msg) { return ur3e_internal_fail(code, msg.c_str()); }

bool load_rccl(Rccl& r, std::string& err) {
  static Rccl cached;
  if (cached.ok) {
    r = cached;
    return true;
  }
  void* h = nullptr;
  /* UR3E_RCCL_LIB: another library with RCCL's point-to-point API (the CPU test's in-process fake,
     tests/c/fake_rccl.c, drives the rank-offset arithmetic below with several ranks and no GPU) */
  const char* over = getenv("UR3E_RCCL_LIB");
  if (over && *over) {
    h = dlopen(over, RTLD_NOW | RTLD_LOCAL);
  } else {
    for (const char* n : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
      if (!h) h = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
  }
  if (!h) {
    err = "librccl not found";
    return false;
  }
  Rccl q;
  q.GroupStart = (int (*)(void))dlsym(h, "ncclGroupStart");
  q.GroupEnd = (int (*)(void))dlsym(h, "ncclGroupEnd");
  q.Send = (int (*)(const void*, size_t, int, int, void*, void*))dlsym(h, "ncclSend");
  q.Recv = (int (*)(void*, size_t, int, int, void*, void*))dlsym(h, "ncclRecv");
  q.CommCount = (int (*)(void*, int*))dlsym(h, "ncclCommCount");
  q.CommUserRank = (int (*)(void*, int*))dlsym(h, "ncclCommUserRank");
  q.GetErrorString = (const char* (*)(int))dlsym(h, "ncclGetErrorString");
  if (!q.GroupStart || !q.GroupEnd || !q.Send || !q.Recv || !q.CommCount || !q.CommUserRank || !q.GetErrorString) {
    err = "librccl lacks the point-to-point API";
    return false;
  }
  q.ok = true;
  cached = q;
  r = q;
  return true;
}

}  // namespace

extern "C" int ur3e_gather_rows(void* rccl_comm, int root, int n, int obs_dim, const double* d_obs,
                                const double* d_reward, const uint8_t* d_terminated, const uint8_t* d_truncated,
                                double* d_obs_all, double* d_reward_all, uint8_t* d_terminated_all,
                                uint8_t* d_truncated_all, void* stream) {
  if (!rccl_comm || !d_obs || !d_reward || !d_terminated || !d_truncated)
    return fail(UR3E_EINVAL, "null communicator or buffer");
  if (n <= 0 || obs_dim <= 0) return fail(UR3E_EINVAL, "n and obs_dim must be positive");
  Rccl r;
  std::string err;
  if (!load_rccl(r, err)) return fail(UR3E_EINVAL, err);
  int nranks = 0, rank = 0;
  if (r.CommCount(rccl_comm, &nranks) || r.CommUserRank(rccl_comm, &rank))
    return fail(UR3E_EINVAL, "not an RCCL communicator");
  if (root < 0 || root >= nranks) return fail(UR3E_EINVAL, "root outside the communicator");
  if (rank == root && (!d_obs_all || !d_reward_all || !d_terminated_all || !d_truncated_all))
    return fail(UR3E_EINVAL, "the root needs the gathered buffers");
  /* rank p's rows land at rows [p * n, (p + 1) * n) of the root's buffers: every rank must pass the same
     n and obs_dim (a precondition, include/ur3e_batch.h), or the send and receive counts disagree */
  const size_t nn = (size_t)n, od = (size_t)obs_dim;
  int rc = r.GroupStart();
  if (!rc) rc = r.Send(d_obs, nn * od, kFloat64, root, rccl_comm, stream);
  if (!rc) rc = r.Send(d_reward, nn, kFloat64, root, rccl_comm, stream);
  if (!rc) rc = r.Send(d_terminated, nn, kUint8, root, rccl_comm, stream);
  if (!rc) rc = r.Send(d_truncated, nn, kUint8, root, rccl_comm, stream);
  if (rank == root)
    for (int p = 0; p < nranks && !rc; p++) {
      rc = r.Recv(d_obs_all + (size_t)p * nn * od, nn * od, kFloat64, p, rccl_comm, stream);
      if (!rc) rc = r.Recv(d_reward_all + (size_t)p * nn, nn, kFloat64, p, rccl_comm, stream);
      if (!rc) rc = r.Recv(d_terminated_all + (size_t)p * nn, nn, kUint8, p, rccl_comm, stream);
      if (!rc) rc = r.Recv(d_truncated_all + (size_t)p * nn, nn, kUint8, p, rccl_comm, stream);
    }
  const int rc2 = r.GroupEnd();
  if (rc || rc2) return fail(UR3E_EHIP, std::string("RCCL: ") + r.GetErrorString(rc ? rc : rc2));
  return UR3E_OK;
}

extern "C" int ur3e_batch_gather(ur3e_batch_t* b, void* rccl_comm, int root, const double* d_obs,
                                 const double* d_reward, const uint8_t* d_terminated, const uint8_t* d_truncated,
                                 double* d_obs_all, double* d_reward_all, uint8_t* d_terminated_all,
                                 uint8_t* d_truncated_all, void* stream) {
  if (!b) return fail(UR3E_EINVAL, "null handle");
  return ur3e_gather_rows(rccl_comm, root, ur3e_batch_num_envs(b), ur3e_batch_obs_dim(b), d_obs, d_reward,
                          d_terminated, d_truncated, d_obs_all, d_reward_all, d_terminated_all, d_truncated_all,
                          stream);
}
