// Round-5 A/B (profiles/r05_ab/): does a 64-lane wave holding TWO envs (lanes 0-31 and 32-63, one per half)
// beat one env per wave on the Newton solver's direction stage?  The stage is rebuilt here in the compact
// tier's register-resident style (ur3e_wave_r.h r_direction): the Hessian H = M + sum_r D_r J_r J_r' built
// element-parallel (lane = lower-triangle element, rows in order), handed to row layout through LDS, a
// right-looking Cholesky with lane k holding row k (column entries broadcast), the forward sweep in
// registers and the backward sweep through L' in LDS -- nv = 20 dofs, 26 constraint rows (the gym step's).
//   mode 0: one env per wave (broadcast = v_readlane), LDS padded to the product's 16,208 B per env:
//           8 waves (8 envs) per CU, two waves per SIMD;
//   mode 1: two envs per wave, broadcast within each half by two v_readlane pairs and a select;
//   mode 2: two envs per wave, broadcast within each half by ds_bpermute;
//   modes 1 and 2 take 2 x 16,208 B of LDS per wave: 4 waves (8 envs) per CU, one wave per SIMD.
// Every mode computes the same numbers (checked bitwise); the figure of merit is ns per env-direction at
// equal envs per CU.  usage: ubench_halfwave [envs] [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define NV 20
#define NR 26
#define NEL (NV * (NV + 1) / 2)
#define LDS_ENV 16208 /* the compact tier's working set per env (w_dyn_lds<KSS_NV>) */

#define CHK(x)                                                                     \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

__device__ __forceinline__ int lane_id() {
  int l = (int)threadIdx.x;
  asm volatile("" : "+v"(l));
  return l;
}
__device__ __forceinline__ double rl(double v, int lane) {
  long long b = __builtin_bit_cast(long long, v);
  int lo = __builtin_amdgcn_readlane((int)(unsigned)(b & 0xffffffffll), lane);
  int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __builtin_bit_cast(double, (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ double bp(double v, int src) {
  long long b = __builtin_bit_cast(long long, v);
  int lo = __builtin_amdgcn_ds_bpermute(src << 2, (int)(unsigned)(b & 0xffffffffll));
  int hi = __builtin_amdgcn_ds_bpermute(src << 2, (int)(b >> 32));
  return __builtin_bit_cast(double, (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
/* value of v on the env's lane k (k uniform) */
template <int MODE>
__device__ __forceinline__ double bc(double v, int k, int lane) {
  if constexpr (MODE == 0) return rl(v, k);
  else if constexpr (MODE == 1) {
    const double a = rl(v, k), b = rl(v, 32 + k);
    return lane < 32 ? a : b;
  } else {
    return bp(v, (lane & 32) | k);
  }
}
__device__ __forceinline__ void wbar() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

extern __shared__ double lds[];

template <int MODE>
__global__ __launch_bounds__(64) void k_direction(const double* __restrict__ Mp, const double* __restrict__ Jg,
                                                  const double* __restrict__ Dg, const double* __restrict__ bg,
                                                  double* __restrict__ xg, int n, int reps) {
  constexpr bool HALF = MODE != 0;
  constexpr int L = HALF ? 32 : 64;                /* lanes per env */
  constexpr int NQ = (NEL + L - 1) / L;            /* element slots per lane */
  const int lane = lane_id();
  const int li = lane & (L - 1);
  const int e = HALF ? 2 * blockIdx.x + (lane >> 5) : blockIdx.x;
  if (e >= n) return; /* n is even in HALF mode: both halves of a wave are live */
  double* my = lds + (HALF ? (lane >> 5) * (LDS_ENV / 8) : 0);
  double* J = my;                 /* [NR][NV] */
  double* Hl = my + NR * NV;      /* packed lower triangle */
  double* Lt = Hl + NEL;          /* [NV][NV] rows of L */
  for (int k = li; k < NR * NV; k += L) J[k] = Jg[(size_t)e * NR * NV + k];
  double D[NR];
#pragma unroll
  for (int r = 0; r < NR; r++) D[r] = Dg[(size_t)e * NR + r];
  /* element slots: lane li owns elements li + L q, with (row, col) of each */
  int er[NQ], ecl[NQ];
  double m0[NQ];
#pragma unroll
  for (int q = 0; q < NQ; q++) {
    const int el = li + L * q;
    int k = 0;
    while ((k + 1) * (k + 2) / 2 <= el) k++;
    er[q] = el < NEL ? k : 0;
    ecl[q] = el < NEL ? el - k * (k + 1) / 2 : 0;
    m0[q] = el < NEL ? Mp[(size_t)e * NEL + el] : 0.0;
  }
  double b = li < NV ? bg[(size_t)e * NV + li] : 0.0;
  wbar();
  double x = 0;
  for (int rep = 0; rep < reps; rep++) {
    /* H build, rows in order */
    double hv[NQ];
#pragma unroll
    for (int q = 0; q < NQ; q++) hv[q] = m0[q];
#pragma unroll 2
    for (int r = 0; r < NR; r++) {
#pragma unroll
      for (int q = 0; q < NQ; q++) hv[q] = hv[q] + D[r] * J[r * NV + er[q]] * J[r * NV + ecl[q]];
    }
#pragma unroll
    for (int q = 0; q < NQ; q++)
      if (li + L * q < NEL) Hl[li + L * q] = hv[q];
    wbar();
    /* row layout: lane k holds row k */
    double h[NV];
    const int row = li < NV ? li : 0;
#pragma unroll
    for (int j = 0; j < NV; j++) h[j] = j <= row ? Hl[row * (row + 1) / 2 + j] : 0.0;
    wbar();
    /* right-looking Cholesky */
#pragma unroll
    for (int j = 0; j < NV; j++) {
      const double dj = bc<MODE>(h[j], j, lane);
      const double pj = sqrt(dj);
      const double lj = li == j ? pj : h[j] / pj;
      h[j] = lj;
#pragma unroll
      for (int k = j + 1; k < NV; k++) {
        const double lk = bc<MODE>(lj, k, lane);
        h[k] = h[k] - lj * lk;
      }
    }
    /* forward sweep in registers */
    double y = b;
#pragma unroll
    for (int k = 0; k < NV; k++) {
      if (li == k) y = y / h[k];
      const double yk = bc<MODE>(y, k, lane);
      if (li > k) y = y - h[k] * yk;
    }
    /* backward sweep through L' in LDS */
    if (li < NV) {
#pragma unroll
      for (int j = 0; j < NV; j++) Lt[li * NV + j] = h[j];
    }
    wbar();
    x = y;
#pragma unroll
    for (int k = NV - 1; k >= 0; k--) {
      if (li == k) x = x / h[k];
      const double xk = bc<MODE>(x, k, lane);
      if (li < k) x = x - Lt[k * NV + row] * xk;
    }
    wbar();
    b = b + 1e-3 * x; /* the next repetition depends on this one */
  }
  if (li < NV) xg[(size_t)e * NV + li] = x;
}

template <int MODE>
static float run(int n, int reps, const double* Mp, const double* J, const double* D, const double* b, double* x,
                 int iters) {
  const int blocks = MODE == 0 ? n : n / 2;
  const size_t dyn = MODE == 0 ? LDS_ENV : 2 * LDS_ENV;
  hipEvent_t a, c;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&c));
  hipLaunchKernelGGL(k_direction<MODE>, dim3(blocks), dim3(64), dyn, 0, Mp, J, D, b, x, n, reps); /* warm */
  CHK(hipGetLastError());
  CHK(hipDeviceSynchronize());
  std::vector<float> t;
  for (int i = 0; i < iters; i++) {
    CHK(hipEventRecord(a, 0));
    hipLaunchKernelGGL(k_direction<MODE>, dim3(blocks), dim3(64), dyn, 0, Mp, J, D, b, x, n, reps);
    CHK(hipEventRecord(c, 0));
    CHK(hipEventSynchronize(c));
    float ms;
    CHK(hipEventElapsedTime(&ms, a, c));
    t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  int occ = 0;
  CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_direction<MODE>, 64, dyn));
  hipFuncAttributes attr;
  CHK(hipFuncGetAttributes(&attr, (const void*)k_direction<MODE>));
  const float med = t[t.size() / 2];
  printf("{\"mode\": %d, \"envs\": %d, \"reps\": %d, \"ms_median\": %.4f, \"ns_per_env_direction\": %.2f, "
         "\"waves_per_cu\": %d, \"envs_per_cu\": %d, \"vgpr\": %d, \"scratch\": %d}\n",
         MODE, n, reps, med, 1e6 * med / ((double)n * reps), occ, occ * (MODE == 0 ? 1 : 2), attr.numRegs,
         (int)attr.localSizeBytes);
  CHK(hipEventDestroy(a));
  CHK(hipEventDestroy(c));
  return med;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4096;
  const int reps = argc > 2 ? atoi(argv[2]) : 16;
  if (n <= 0 || (n & 1)) { fprintf(stderr, "envs must be positive and even\n"); return 2; }
  std::vector<double> Mp((size_t)n * NEL), J((size_t)n * NR * NV), D((size_t)n * NR), b((size_t)n * NV);
  srand(7);
  auto u = [] { return (double)rand() / RAND_MAX - 0.5; };
  for (int e = 0; e < n; e++) {
    /* SPD M: A A' + 20 I (packed lower) */
    double A[NV][NV];
    for (int i = 0; i < NV; i++)
      for (int j = 0; j < NV; j++) A[i][j] = u();
    for (int i = 0; i < NV; i++)
      for (int j = 0; j <= i; j++) {
        double s = i == j ? 20.0 : 0.0;
        for (int k = 0; k < NV; k++) s += A[i][k] * A[j][k];
        Mp[(size_t)e * NEL + i * (i + 1) / 2 + j] = s;
      }
    for (int k = 0; k < NR * NV; k++) J[(size_t)e * NR * NV + k] = u();
    for (int r = 0; r < NR; r++) D[(size_t)e * NR + r] = 1.0 + u();
    for (int k = 0; k < NV; k++) b[(size_t)e * NV + k] = u();
  }
  double *dM, *dJ, *dD, *db, *dx[3];
  CHK(hipMalloc(&dM, Mp.size() * 8));
  CHK(hipMalloc(&dJ, J.size() * 8));
  CHK(hipMalloc(&dD, D.size() * 8));
  CHK(hipMalloc(&db, b.size() * 8));
  for (int k = 0; k < 3; k++) CHK(hipMalloc(&dx[k], (size_t)n * NV * 8));
  CHK(hipMemcpy(dM, Mp.data(), Mp.size() * 8, hipMemcpyHostToDevice));
  CHK(hipMemcpy(dJ, J.data(), J.size() * 8, hipMemcpyHostToDevice));
  CHK(hipMemcpy(dD, D.data(), D.size() * 8, hipMemcpyHostToDevice));
  CHK(hipMemcpy(db, b.data(), b.size() * 8, hipMemcpyHostToDevice));
  for (int round = 0; round < 3; round++) {
    run<0>(n, reps, dM, dJ, dD, db, dx[0], 7);
    run<1>(n, reps, dM, dJ, dD, db, dx[1], 7);
    run<2>(n, reps, dM, dJ, dD, db, dx[2], 7);
  }
  std::vector<double> x0((size_t)n * NV), x1((size_t)n * NV), x2((size_t)n * NV);
  CHK(hipMemcpy(x0.data(), dx[0], x0.size() * 8, hipMemcpyDeviceToHost));
  CHK(hipMemcpy(x1.data(), dx[1], x1.size() * 8, hipMemcpyDeviceToHost));
  CHK(hipMemcpy(x2.data(), dx[2], x2.size() * 8, hipMemcpyDeviceToHost));
  const bool same = !memcmp(x0.data(), x1.data(), x0.size() * 8) && !memcmp(x0.data(), x2.data(), x0.size() * 8);
  double mx = 0;
  for (double v : x0) mx = std::max(mx, std::fabs(v));
  printf("{\"bitwise_equal_across_modes\": %s, \"max_abs_x\": %.6g}\n", same ? "true" : "false", mx);
  return same ? 0 : 1;
}
