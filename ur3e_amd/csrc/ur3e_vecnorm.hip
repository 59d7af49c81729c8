/* On-device SB3 VecNormalize (include/ur3e_vecnorm.h): running observation / return statistics in
 * numpy's exact reduction order, then normalisation.
 *
 * k_vn_stats (dim + 1 workgroups of 1024 threads, one per observation column and one for the returns):
 *   workgroup dim: returns = returns * gamma + reward (all threads), then numpy's pairwise summation
 *     (8 accumulators per <=128 block, halves rounded down to multiples of 8) over each 8192-element
 *     buffer, leaves on separate threads, the tree and the buffer sums added in numpy's order, for the
 *     1-D mean and var of the returns;
 *   workgroup j < dim: column j of obs [n, dim]: mean = (((x0 + x1) + x2) + ...) / n and
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

/* numpy pairwise_sum (numpy/_core/src/umath/loops_utils.h.src) over a contiguous double array, of the
   values f(a[i]): blocks < 8 sum sequentially from 0.0, blocks <= 128 use 8 strided accumulators
   combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) plus a sequential tail, larger blocks split at n/2 rounded
   down to a multiple of 8.  vn_leaf is a block of <= 128; vn_sum_par below lays out the splits.  P is an
   LDS- or global-address-space pointer: through a generic pointer every load of these serial chains
   would be a FLAT load (LDS data at FLAT latency, and every wait counting both memory counters). */
typedef const __attribute__((address_space(3))) double* VnLds;
typedef const __attribute__((address_space(1))) double* VnGlobal;
template <class P, class F>
__device__ static double vn_leaf(P a, int len, F f) {
  if (len < 8) {
    double res = 0.0;
    for (int i = 0; i < len; i++) res += f(a[i]);
    return res;
  }
  double r[8];
#pragma unroll
  for (int j = 0; j < 8; j++) r[j] = f(a[j]);
  int i;
  for (i = 8; i < len - (len % 8); i += 8)
#pragma unroll
    for (int j = 0; j < 8; j++) r[j] += f(a[i + j]);
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < len; i++) res += f(a[i]);
  return res;
}

/* a 1-D np.sum / np.mean of a contiguous double array: numpy's reduction iterator hands the add loop
   buffers of at most NPY_BUFSIZE = 8192 elements and accumulates the per-buffer pairwise sums in
   order, starting from the additive identity -- for n > 8192 a single whole-array pairwise sum would
   round differently */
#define VN_NP_BUFSIZE 8192

/* The same 1-D sum with the whole workgroup: numpy's pairwise recursion over each 8192-element buffer is laid
   out as a node list (thread 0, children after their parent: a node longer than 128 splits at half its
   length rounded down to a multiple of 8), every leaf (<= 128 elements) is summed by its own thread with
   numpy's leaf code (vn_leaf), and thread 0 adds each internal node's
   children left + right, children first -- the same additions in the same tree as the serial recursion,
   without its frame stack in private memory (round 5: 174 us of the 180 us statistics kernel at 4,096
   envs were that stack's walk on one thread). */
#define VN_MAXNODE 256 /* a tree over <= 8192 elements has <= 255 nodes (leaves hold >= 64) */
struct VnTree {
  int off[VN_MAXNODE], len[VN_MAXNODE], left[VN_MAXNODE];
  double val[VN_MAXNODE];
  int nn;
};
template <class P, class F>
__device__ static double vn_sum_par(VnTree& t, P a, int n, F f) {
  const int tid = threadIdx.x;
  double res = 0.0;
  for (int b = 0; b < n; b += VN_NP_BUFSIZE) {
    const int len = n - b < VN_NP_BUFSIZE ? n - b : VN_NP_BUFSIZE;
    __syncthreads();
    if (tid == 0) {
      t.off[0] = b;
      t.len[0] = len;
      int nn = 1;
      for (int k = 0; k < nn; k++) {
        const int l = t.len[k];
        if (l <= 128) {
          t.left[k] = -1;
          continue;
        }
        int n2 = l / 2;
        n2 -= n2 % 8;
        t.left[k] = nn;
        t.off[nn] = t.off[k]; t.len[nn] = n2;
        t.off[nn + 1] = t.off[k] + n2; t.len[nn + 1] = l - n2;
        nn += 2;
      }
      t.nn = nn;
    }
    __syncthreads();
    const int nn = t.nn;
    for (int k = tid; k < nn; k += blockDim.x)
      if (t.left[k] < 0) t.val[k] = vn_leaf(a + t.off[k], t.len[k], f);
    __syncthreads();
    if (tid == 0) {
      for (int k = nn - 1; k >= 0; k--)
        if (t.left[k] >= 0) t.val[k] = t.val[t.left[k]] + t.val[t.left[k] + 1];
      t.val[0] = res + t.val[0];
    }
    __syncthreads();
    res = t.val[0];
  }
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

/* dim + 1 workgroups of VN_NT threads.  The serial orders are fixed by numpy, so the work is keeping
   everything but the dependent additions off the chains.  Workgroup j < dim owns observation column j
   and runs it on its first wave with the column in REGISTERS: lane k holds VN_RPL consecutive rows of
   each 64 * VN_RPL-row round, and the chain visits the lanes in order -- lane k adds its rows (a run of
   dependent adds with register operands, no memory access on the chain) and hands the running sum to
   lane k + 1 by readlane.  Both sweeps (sum; then the squared deviations from the batch mean, formed on
   all lanes at once before the chain) load the column once each.  Workgroup dim owns the returns (1-D,
   numpy's pairwise tree, vn_sum_par).  The columns run on separate CUs at once; the new observation
   count (shared by every column) is stored by k_vn_apply, after every column has read the old one.
   Round 5: one workgroup walking all 24 columns through restaged LDS chunks took 126 us at 4,096 envs;
   chains over LDS, 81 us (bound by the reads' latency); in registers, see DESIGN.md section 7. */
#define VN_NT 1024
#define VN_RPL 32            /* rows per lane per round (64 VGPRs: the 1,024-thread bound allows 128) */
#define VN_RET_LDS 4096      /* returns staged in LDS when n <= this (32 KB) */

__device__ __forceinline__ double vn_rl(double v, int lane) {
  long long b = __builtin_bit_cast(long long, v);
  int lo = __builtin_amdgcn_readlane((int)(unsigned)(b & 0xffffffffll), lane);
  int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __builtin_bit_cast(double, (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

/* one sweep of column j (wave 0): PASS 0 returns x0 + x1 + ... (row order), PASS 1 d0^2 + d1^2 + ...
   with d = x - bm; the first term starts the sum (numpy's reduction has no identity there) */
template <int PASS>
__device__ static double vn_column(const double* __restrict__ obs, int n, int dim, int j, double bm) {
  const int lane = threadIdx.x;
  double s = 0.0;
  for (int base = 0; base < n; base += 64 * VN_RPL) {
    double v[VN_RPL];
#pragma unroll
    for (int r = 0; r < VN_RPL; r++) {
      const int row = base + lane * VN_RPL + r;
      const double x = row < n ? obs[(size_t)row * dim + j] : 0.0;
      if (PASS == 0) {
        v[r] = x;
      } else {
        const double d = x - bm;
        v[r] = d * d;
      }
    }
    for (int t = 0; t < 64; t++) {
      const int row0 = base + t * VN_RPL;
      if (row0 >= n) break;
      const int cnt = n - row0 < VN_RPL ? n - row0 : VN_RPL;
      if (lane == t) {
        double acc = row0 == 0 ? v[0] : s + v[0];
        if (cnt == VN_RPL) {
#pragma unroll
          for (int r = 1; r < VN_RPL; r++) acc = acc + v[r];
        } else {
#pragma unroll
          for (int r = 1; r < VN_RPL; r++)
            if (r < cnt) acc = acc + v[r];
        }
        s = acc;
      }
      s = vn_rl(s, t);
    }
  }
  return s;
}

__global__ __launch_bounds__(VN_NT) void k_vn_stats(ur3e_vecnorm_stats_t st, int n, int dim,
                                                    const double* __restrict__ obs, const double* __restrict__ rew,
                                                    int upd_obs, int upd_ret, double gamma, int reset) {
  __shared__ double rbuf[VN_RET_LDS];
  __shared__ VnTree tree;
  const int tid = threadIdx.x;
  const double bn = (double)n;
  if ((int)blockIdx.x == dim) {
    /* the discounted returns and their statistics (1-D: numpy pairwise summation) */
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
      double bm, q;
      if (in_lds) {
        const VnLds a = (VnLds)rbuf;
        bm = vn_sum_par(tree, a, n, [](double x) { return x; }) / bn;
        q = vn_sum_par(tree, a, n, [bm](double x) { const double d = x - bm; return d * d; });
      } else {
        const VnGlobal a = (VnGlobal)st.returns;
        bm = vn_sum_par(tree, a, n, [](double x) { return x; }) / bn;
        q = vn_sum_par(tree, a, n, [bm](double x) { const double d = x - bm; return d * d; });
      }
      if (tid == 0) {
        const double c = *st.ret_count;
        vn_moments(st.ret_mean, st.ret_var, c, bm, q / bn, bn);
        *st.ret_count = bn + c;
      }
    }
    return;
  }
  if (!upd_obs) return;
  /* ---- observation column j: np.mean / np.var over axis 0 of a C-contiguous [n, dim], row-sequential ---- */
  if (tid >= 64) return;
  const int j = blockIdx.x;
  const double bm = vn_column<0>(obs, n, dim, j, 0.0) / bn;
  const double q = vn_column<1>(obs, n, dim, j, bm);
  if (tid == 0) vn_moments(st.obs_mean + j, st.obs_var + j, *st.obs_count, bm, q / bn, bn);
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
                           double* __restrict__ rew_out, float* __restrict__ tobs_out, int upd_count) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n * dim) return;
  /* the observation count of the statistics k_vn_stats just updated (every column read the old one) */
  if (upd_count && k == 0) *st.obs_count = (double)n + *st.obs_count;
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
  const int upd_obs = cfg->training && cfg->norm_obs;
  hipLaunchKernelGGL(k_vn_stats, dim3(dim + 1), dim3(VN_NT), 0, s, *st, n, dim, d_obs, d_rew, upd_obs, cfg->training,
                     cfg->gamma, 0);
  VN_CHK(hipGetLastError());
  hipLaunchKernelGGL(k_vn_apply, dim3((n * dim + 255) / 256), dim3(256), 0, s, *st, n, dim, d_obs, d_rew, d_term,
                     d_trunc, d_tobs, cfg->norm_obs, cfg->norm_reward, cfg->clip_obs, cfg->clip_reward, cfg->epsilon,
                     d_obs_out, d_rew_out, d_tobs_out, upd_obs);
  VN_CHK(hipGetLastError());
  return UR3E_OK;
}

extern "C" int ur3e_vecnorm_reset(const ur3e_vecnorm_stats_t* st, const ur3e_vecnorm_cfg_t* cfg, int n, int dim,
                                  const double* d_obs, float* d_obs_out, void* stream) {
  int rc = vn_check(st, cfg, n, dim, d_obs);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  const int upd_obs = cfg->training && cfg->norm_obs;
  hipLaunchKernelGGL(k_vn_stats, dim3(dim + 1), dim3(VN_NT), 0, s, *st, n, dim, d_obs, nullptr, upd_obs, 0, cfg->gamma, 1);
  VN_CHK(hipGetLastError());
  hipLaunchKernelGGL(k_vn_apply, dim3((n * dim + 255) / 256), dim3(256), 0, s, *st, n, dim, d_obs, nullptr, nullptr,
                     nullptr, nullptr, cfg->norm_obs, 0, cfg->clip_obs, 0.0, cfg->epsilon, d_obs_out, nullptr, nullptr,
                     upd_obs);
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
                     nullptr, 0);
  VN_CHK(hipGetLastError());
  return UR3E_OK;
}
