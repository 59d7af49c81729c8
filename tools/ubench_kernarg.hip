// Diagnostic microbenchmark (round 5): the cost of a large by-value kernel argument.  Two kernels with the
// same body (a dependent FP64 chain, 2048 one-wave workgroups, 16 KB dynamic LDS), one with a ~900 B
// by-value struct argument (the queue kernel's KConfig + KState are 944 B of kernarg), one without; each
// alone back to back and alternating with a short 512 x 128 kernel.
#include <hip/hip_runtime.h>
#include <cstdio>

struct BigArg { double v[112]; };

__device__ __forceinline__ double body(int iters) {
  double x = threadIdx.x * 1e-3 + blockIdx.x;
  for (int i = 0; i < iters; i++) x = x * 0.999999 + 1e-9;
  return x;
}
__global__ void __launch_bounds__(64, 2) k_small_arg(double* out, int iters) {
  extern __shared__ double lds[];
  const double x = body(iters);
  lds[threadIdx.x] = x;
  __builtin_amdgcn_wave_barrier();
  if (x == 12345.0) out[blockIdx.x] = lds[(threadIdx.x + 1) & 63];
}
__global__ void __launch_bounds__(64, 2) k_big_arg(double* out, int iters, BigArg ba) {
  extern __shared__ double lds[];
  const double x = body(iters);
  lds[threadIdx.x] = x;
  __builtin_amdgcn_wave_barrier();
  if (x == 12345.0) out[blockIdx.x] = lds[(threadIdx.x + 1) & 63] + ba.v[111];
}
__global__ void __launch_bounds__(64, 2) k_ptr_arg(double* out, int iters, const BigArg* __restrict__ pa) {
  extern __shared__ double lds[];
  const double x = body(iters);
  lds[threadIdx.x] = x;
  __builtin_amdgcn_wave_barrier();
  if (x == 12345.0) out[blockIdx.x] = lds[(threadIdx.x + 1) & 63] + pa->v[111];
}
__global__ void __launch_bounds__(128) k_short(double* out, int n) {
  if (blockIdx.x * 128 + threadIdx.x == n) out[0] = 1.0;
}
__global__ void __launch_bounds__(128) k_short_big(double* out, int n, BigArg ba) {
  /* 80 KB of static LDS per workgroup, like the full-capacity tier's list kernel */
  __shared__ double big_lds[10240];
  if (blockIdx.x * 128 + threadIdx.x == n) {
    big_lds[threadIdx.x] = ba.v[3];
    out[0] = big_lds[(threadIdx.x + 1) & 127];
  }
}

int main() {
  double* d;
  BigArg* dpa;
  hipMalloc(&d, 1 << 20);
  hipMalloc(&dpa, sizeof(BigArg));
  hipMemset(dpa, 0, sizeof(BigArg));
  hipStream_t s;
  hipStreamCreate(&s);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  BigArg ba;
  for (int k = 0; k < 112; k++) ba.v[k] = 0.0;
  const int iters = 20000, reps = 200;
  auto run = [&](int kind, int with_short) {
    for (int r = -5; r < reps; r++) {
      if (r == 0) hipEventRecord(a, s);
      if (kind == 0) hipLaunchKernelGGL(k_small_arg, dim3(2048), dim3(64), 16384, s, d, iters);
      if (kind == 1) hipLaunchKernelGGL(k_big_arg, dim3(2048), dim3(64), 16384, s, d, iters, ba);
      if (kind == 2) hipLaunchKernelGGL(k_ptr_arg, dim3(2048), dim3(64), 16384, s, d, iters, dpa);
      if (with_short == 1) hipLaunchKernelGGL(k_short, dim3(512), dim3(128), 0, s, d, -1);
      if (with_short == 2) hipLaunchKernelGGL(k_short_big, dim3(512), dim3(128), 0, s, d, -1, ba);
    }
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms * 1e3 / reps;
  };
  const char* kn[3] = {"small kernarg", "900 B by value", "pointer to it"};
  for (int round = 0; round < 3; round++)
    for (int kind = 0; kind < 3; kind++) {
      const float t0 = run(kind, 0), t1 = run(kind, 1), t2 = run(kind, 2);
      printf("round %d, %-15s: alone %.2f us; + short kernel %.2f (+%.2f); + short kernel with 900 B arg and 80 KB LDS %.2f (+%.2f)\n",
             round, kn[kind], t0, t1, t1 - t0, t2, t2 - t0);
    }
  return 0;
}
