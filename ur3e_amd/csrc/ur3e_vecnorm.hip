/* On-device SB3 VecNormalize (include/ur3e_vecnorm.h): running observation / return statistics in
 * numpy's exact reduction order, then normalisation.
 *
 * k_vn_stats (two workgroups of 1024 threads on two CUs, rows staged through LDS):
 *   block 1: returns = returns * gamma + reward (all threads), then thread 0 runs numpy's pairwise
 *     summation (8 accumulators per <=128 block, halves rounded down to multiples of 8) over each
 *     8192-element buffer, the buffer sums added in order, for the 1-D mean and var of the returns;
 *   block 0, thread j < dim: column j of obs [n, dim]: mean = (((x0 + x1) + x2) + ...) / n and
 *     var = sum((x - mean)^2) / n in the same row-sequential order numpy uses for an axis-0
 *     reduction of a C-contiguous array, then RunningMeanStd.update_from_moments.
 * k_vn_apply (n x dim threads): obs / terminal-obs normalisation to f32, reward normalisation,
 *   returns[done] = 0.
 * The bound is the serial order SB3 fixes (~8k dependent FP64 adds per column at n = 4096), so the
 * loads are staged into LDS by the whole workgroup and kept off the add chains. */
#include <hip/hip_runtime.h>

#include "../../include/ur3e_batch.h"
#include "../../include/ur3e_vecnorm.h"

int ur3e_internal_fail(int code, const char* msg);

#define VN_CHK(x)                                                       \
  do {                                                                  \
    hipError_t _e = (x);                                                \
    if (_e != hipSuccess) return ur3e_internal_fail(UR3E_EHIP, hipGetErrorString(_e)); \
  } while (0)

/* numpy pairwise_sum over a contiguous double array (numpy/_core/src/umath/loops_utils.h.src), of
   the values f(a[i]): blocks < 8 sum sequentially from 0.0, blocks <= 128 use 8 strided accumulators
   combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) plus a sequential tail, larger blocks split at
   n/2 rounded down to a multiple of 8.  The recursion runs on an explicit stack.  P is an LDS- or
   global-address-space pointer: through a generic pointer every load of this serial chain would be
   a FLAT load (LDS data at FLAT latency, and every wait counting both memory counters). */
typedef const __attribute__((address_space(3))) double* VnLds;
typedef const __attribute__((address_space(1))) double* VnGlobal;
template <class P, class F>
__device__ static double vn_pairwise(P a, int n, F f) {
  struct Fr { int off, len, stage; double left; };
  Fr stk[32];
  int sp = 0;
  stk[0] = {0, n, 0, 0.0};
  double ret = 0.0;
  for (;;) {
    Fr& fr = stk[sp];
    if (fr.stage == 0) {
      if (fr.len < 8) {
        double res = 0.0;
        for (int i = 0; i < fr.len; i++) res += f(a[fr.off + i]);
        ret = res;
      } else if (fr.len <= 128) {
        double r[8];
        for (int j = 0; j < 8; j++) r[j] = f(a[fr.off + j]);
        int i;
        for (i = 8; i < fr.len - (fr.len % 8); i += 8)
          for (int j = 0; j < 8; j++) r[j] += f(a[fr.off + i + j]);
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < fr.len; i++) res += f(a[fr.off + i]);
        ret = res;
      } else {
        int n2 = fr.len / 2;
        n2 -= n2 % 8;
        fr.stage = 1;
        stk[sp + 1] = {fr.off, n2, 0, 0.0};
        sp++;
        continue;
      }
    } else if (fr.stage == 1) {
      /* left half is in ret: descend into the right half */
      int n2 = fr.len / 2;
      n2 -= n2 % 8;
      fr.left = ret;
      fr.stage = 2;
      stk[sp + 1] = {fr.off + n2, fr.len - n2, 0, 0.0};
      sp++;
      continue;
    } else {
      ret = fr.left + ret;
    }
    if (sp == 0) return ret;
    sp--;
  }
}

/* a 1-D np.sum / np.mean of a contiguous double array: numpy's reduction iterator hands the add loop
   buffers of at most NPY_BUFSIZE = 8192 elements and accumulates the per-buffer pairwise sums in
   order, starting from the additive identity -- for n > 8192 a single whole-array pairwise sum would
   round differently */
#define VN_NP_BUFSIZE 8192
template <class P, class F>
__device__ static double vn_sum(P a, int n, F f) {
  double res = 0.0;
  for (int b = 0; b < n; b += VN_NP_BUFSIZE) res = res + vn_pairwise(a + b, n - b < VN_NP_BUFSIZE ? n - b : VN_NP_BUFSIZE, f);
  return res;
}

/* RunningMeanStd.update_from_moments in the operation order of common/running_mean_std.py; the
   caller stores the new count (shared by all columns) once */
__device__ static void vn_moments(double* mean, double* var, double c, double bmean, double bvar, double bcount) {
  const double m = *mean, v = *var;
  const double delta = bmean - m;
  const double tot = c + bcount;
  const double new_mean = m + delta * bcount / tot;
  const double m_a = v * c;
  const double m_b = bvar * bcount;
  const double m_2 = m_a + m_b + delta * delta * c * bcount / (c + bcount);
  const double new_var = m_2 / (c + bcount);
  *mean = new_mean;
  *var = new_var;
}

/* One workgroup of VN_NT threads.  The serial orders are fixed by numpy, so the work here is keeping
   the loads off the dependent add chains: the whole workgroup stages row chunks of obs (and the
   returns) into LDS with coalesced loads, then the lanes that own a column (obs) or lane 0
   (returns, pairwise) walk LDS in numpy's order. */
#define VN_NT 1024
#define VN_LDS_DOUBLES 12288 /* 96 KB of obs rows per chunk */
#define VN_RET_LDS 4096      /* returns staged in LDS when n <= this (32 KB) */
__global__ __launch_bounds__(VN_NT) void k_vn_stats(ur3e_vecnorm_stats_t st, int n, int dim,
                                                    const double* __restrict__ obs, const double* __restrict__ rew,
                                                    int upd_obs, int upd_ret, double gamma, int reset) {
  __shared__ double buf[VN_LDS_DOUBLES];
  __shared__ double rbuf[VN_RET_LDS];
  const int tid = threadIdx.x;
  const double bn = (double)n;
  /* block 1: discounted returns and their statistics (1-D: numpy pairwise summation); block 0: the
     observation columns -- independent, so they run on two CUs at once */
  if (blockIdx.x == 1) {
  if (reset) {
    for (int i = tid; i < n; i += VN_NT) st.returns[i] = 0.0;
  } else if (upd_ret) {
    const bool in_lds = n <= VN_RET_LDS;
    for (int i = tid; i < n; i += VN_NT) {
      const double r = st.returns[i] * gamma + rew[i];
      st.returns[i] = r;
      if (in_lds) rbuf[i] = r;
    }
    __threadfence_block();
    __syncthreads();
    if (tid == 0) {
      double bm, q;
      if (in_lds) {
        const VnLds a = (VnLds)rbuf;
        bm = vn_sum(a, n, [](double x) { return x; }) / bn;
        q = vn_sum(a, n, [bm](double x) { const double d = x - bm; return d * d; });
      } else {
        const VnGlobal a = (VnGlobal)st.returns;
        bm = vn_sum(a, n, [](double x) { return x; }) / bn;
        q = vn_sum(a, n, [bm](double x) { const double d = x - bm; return d * d; });
      }
      const double c = *st.ret_count;
      vn_moments(st.ret_mean, st.ret_var, c, bm, q / bn, bn);
      *st.ret_count = bn + c;
    }
  }
  return;
  }
  if (!upd_obs) return;
  /* ---- observation columns: np.mean / np.var over axis 0 of a C-contiguous [n, dim], row-sequential
     per column; two sweeps (sum, then squared deviations from the batch mean) ---- */
  const int rows = VN_LDS_DOUBLES / dim;
  const int j = tid;
  double s = 0.0, bm = 0.0, q = 0.0;
  for (int pass = 0; pass < 2; pass++) {
    for (int base = 0; base < n; base += rows) {
      const int nr = n - base < rows ? n - base : rows;
      __syncthreads();
      const size_t off = (size_t)base * dim;
      for (int k = tid; k < nr * dim; k += VN_NT) buf[k] = obs[off + k];
      __syncthreads();
      if (j < dim) {
        int i0 = 0;
        if (base == 0) { /* numpy starts each column from its first element */
          if (pass == 0) {
            s = buf[j];
          } else {
            const double d0 = buf[j] - bm;
            q = d0 * d0;
          }
          i0 = 1;
        }
        if (pass == 0) {
#pragma unroll 8
          for (int i = i0; i < nr; i++) s = s + buf[i * dim + j];
        } else {
#pragma unroll 8
          for (int i = i0; i < nr; i++) {
            const double d = buf[i * dim + j] - bm;
            q = q + d * d;
          }
        }
      }
    }
    if (pass == 0) bm = s / bn;
  }
  if (j < dim) vn_moments(st.obs_mean + j, st.obs_var + j, *st.obs_count, bm, q / bn, bn);
  __syncthreads(); /* every column read the old count before it is replaced */
  if (tid == 0) *st.obs_count = bn + *st.obs_count;
}

__device__ static inline float vn_norm(double x, double mean, double var, double eps, double clip) {
  double v = (x - mean) / sqrt(var + eps);
  v = v < -clip ? -clip : v;
  v = v > clip ? clip : v;
  return (float)v;
}

__global__ void k_vn_apply(ur3e_vecnorm_stats_t st, int n, int dim, const double* __restrict__ obs,
                           const double* __restrict__ rew, const unsigned char* __restrict__ term,
                           const unsigned char* __restrict__ trunc, const double* __restrict__ tobs, int norm_obs,
                           int norm_reward, double clip_obs, double clip_reward, double eps, float* __restrict__ obs_out,
                           double* __restrict__ rew_out, float* __restrict__ tobs_out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n * dim) return;
  const int i = k / dim, j = k - i * dim;
  const bool done = term && trunc && (term[i] || trunc[i]);
  if (norm_obs && obs_out) {
    const double m = st.obs_mean[j], v = st.obs_var[j];
    obs_out[k] = vn_norm(obs[k], m, v, eps, clip_obs);
    if (done && tobs && tobs_out) tobs_out[k] = vn_norm(tobs[k], m, v, eps, clip_obs);
  }
  if (j == 0) {
    if (rew && rew_out) {
      double r = rew[i];
      if (norm_reward) {
        r = r / sqrt(st.ret_var[0] + eps);
        r = r < -clip_reward ? -clip_reward : r;
        r = r > clip_reward ? clip_reward : r;
      }
      rew_out[i] = r;
    }
    if (done) st.returns[i] = 0.0;
  }
}

static int vn_check(const ur3e_vecnorm_stats_t* st, const ur3e_vecnorm_cfg_t* cfg, int n, int dim, const double* obs) {
  if (!st || !cfg || !obs) return ur3e_internal_fail(UR3E_EINVAL, "null argument");
  if (n <= 0 || dim <= 0 || dim > 64) return ur3e_internal_fail(UR3E_EINVAL, "need n > 0 and 0 < dim <= 64");
  if (!st->obs_mean || !st->obs_var || !st->obs_count || !st->ret_mean || !st->ret_var || !st->ret_count ||
      !st->returns)
    return ur3e_internal_fail(UR3E_EINVAL, "null statistics buffer");
  return UR3E_OK;
}

extern "C" int ur3e_vecnorm_step(const ur3e_vecnorm_stats_t* st, const ur3e_vecnorm_cfg_t* cfg, int n, int dim,
                                 const double* d_obs, const double* d_rew, const unsigned char* d_term,
                                 const unsigned char* d_trunc, const double* d_tobs, float* d_obs_out,
                                 double* d_rew_out, float* d_tobs_out, void* stream) {
  int rc = vn_check(st, cfg, n, dim, d_obs);
  if (rc) return rc;
  if (!d_rew || !d_term || !d_trunc) return ur3e_internal_fail(UR3E_EINVAL, "null reward / done buffer");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_vn_stats, dim3(2), dim3(VN_NT), 0, s, *st, n, dim, d_obs, d_rew, cfg->training && cfg->norm_obs,
                     cfg->training, cfg->gamma, 0);
  VN_CHK(hipGetLastError());
  hipLaunchKernelGGL(k_vn_apply, dim3((n * dim + 255) / 256), dim3(256), 0, s, *st, n, dim, d_obs, d_rew, d_term,
                     d_trunc, d_tobs, cfg->norm_obs, cfg->norm_reward, cfg->clip_obs, cfg->clip_reward, cfg->epsilon,
                     d_obs_out, d_rew_out, d_tobs_out);
  VN_CHK(hipGetLastError());
  return UR3E_OK;
}

extern "C" int ur3e_vecnorm_reset(const ur3e_vecnorm_stats_t* st, const ur3e_vecnorm_cfg_t* cfg, int n, int dim,
                                  const double* d_obs, float* d_obs_out, void* stream) {
  int rc = vn_check(st, cfg, n, dim, d_obs);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_vn_stats, dim3(2), dim3(VN_NT), 0, s, *st, n, dim, d_obs, nullptr, cfg->training && cfg->norm_obs,
                     0, cfg->gamma, 1);
  VN_CHK(hipGetLastError());
  hipLaunchKernelGGL(k_vn_apply, dim3((n * dim + 255) / 256), dim3(256), 0, s, *st, n, dim, d_obs, nullptr, nullptr,
                     nullptr, nullptr, cfg->norm_obs, 0, cfg->clip_obs, 0.0, cfg->epsilon, d_obs_out, nullptr, nullptr);
  VN_CHK(hipGetLastError());
  return UR3E_OK;
}

extern "C" int ur3e_vecnorm_normalize_obs(const ur3e_vecnorm_stats_t* st, const ur3e_vecnorm_cfg_t* cfg, int n,
                                          int dim, const double* d_obs, float* d_obs_out, void* stream) {
  int rc = vn_check(st, cfg, n, dim, d_obs);
  if (rc) return rc;
  if (!d_obs_out) return ur3e_internal_fail(UR3E_EINVAL, "null output");
  hipLaunchKernelGGL(k_vn_apply, dim3((n * dim + 255) / 256), dim3(256), 0, (hipStream_t)stream, *st, n, dim, d_obs,
                     nullptr, nullptr, nullptr, nullptr, 1, 0, cfg->clip_obs, 0.0, cfg->epsilon, d_obs_out, nullptr,
                     nullptr);
  VN_CHK(hipGetLastError());
  return UR3E_OK;
}
