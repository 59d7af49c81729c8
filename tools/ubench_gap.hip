// Diagnostic microbenchmark (round 5): what sets the ~5.5 us gap before each step's queue kernel?
// A long kernel shaped like the queue kernel (2048 one-wave workgroups, 16 KB dynamic LDS) alternates with
// a short one shaped like the full-tier list kernel (512 x 128 threads).  Variables: a private segment in the
// short kernel, and the long kernel writing ~13 MB per launch (the step's state write-back) with plain,
// nontemporal or write-through (sc1) stores.  Reports the per-iteration time.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __attribute__((address_space(1))) unsigned long long gu64_t;

struct BigArg { double v[112]; };  /* a ~900 B by-value argument, like the queue kernel's KConfig + KState */

template <int WR>
__global__ void __launch_bounds__(64, 2) k_long(double* out, double* big, int iters, BigArg ba) {
  extern __shared__ double lds[];
  double x = threadIdx.x * 1e-3 + blockIdx.x + ba.v[(blockIdx.x & 7) * 13] + ba.v[111]; /* uniform reads */
  for (int i = 0; i < iters; i++) x = x * 0.999999 + 1e-9;
  lds[threadIdx.x] = x;
  __builtin_amdgcn_wave_barrier();
  if (WR) {
    /* 2 envs per workgroup-slot: 4096 x 400 doubles = 13.1 MB, each wave its own contiguous rows */
    double* p = big + (size_t)blockIdx.x * 800;
    for (int k = threadIdx.x; k < 800; k += 64) {
      if (WR == 1) p[k] = x + k;
      else if (WR == 2) __builtin_nontemporal_store(x + k, p + k);
      else __hip_atomic_store((gu64_t*)(p + k), __builtin_bit_cast(unsigned long long, x + k), __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (x == 12345.0) out[blockIdx.x] = lds[(threadIdx.x + 1) & 63];
}

__global__ void __launch_bounds__(128) k_short(double* out, int n) {
  if (blockIdx.x * 128 + threadIdx.x == n) out[0] = 1.0;
}

__global__ void __launch_bounds__(128) k_short_scratch(double* out, int n, int k) {
  volatile double priv[1536];  // 12 KB of private segment per lane, like the full tier's
  const int t = blockIdx.x * 128 + threadIdx.x;
  if (t == n) {
    for (int i = 0; i < 1536; i++) priv[i] = i * 0.5;
    out[0] = priv[k % 1536];
  }
}

int main() {
  double *d, *big;
  hipMalloc(&d, 1 << 20);
  hipMalloc(&big, (size_t)2048 * 800 * 8);
  hipStream_t s;
  hipStreamCreate(&s);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int iters = 20000, reps = 200;
  BigArg ba;
  for (int k = 0; k < 112; k++) ba.v[k] = 0.0;
  auto launch_long = [&](int wr) {
    if (wr == 0) hipLaunchKernelGGL(k_long<0>, dim3(2048), dim3(64), 16384, s, d, big, iters, ba);
    if (wr == 1) hipLaunchKernelGGL(k_long<1>, dim3(2048), dim3(64), 16384, s, d, big, iters, ba);
    if (wr == 2) hipLaunchKernelGGL(k_long<2>, dim3(2048), dim3(64), 16384, s, d, big, iters, ba);
    if (wr == 3) hipLaunchKernelGGL(k_long<3>, dim3(2048), dim3(64), 16384, s, d, big, iters, ba);
  };
  hipEvent_t evn[16];
  for (int k = 0; k < 16; k++) hipEventCreateWithFlags(&evn[k], hipEventDisableTiming);
  auto run = [&](int mode, int wr) {
    for (int r = -5; r < reps; r++) {
      if (r == 0) hipEventRecord(a, s);
      launch_long(wr);
      if (mode >= 1) hipLaunchKernelGGL(k_short, dim3(512), dim3(128), 0, s, d, -1);
      if (mode == 2) hipEventRecord(evn[(r + 16) % 16], s);  /* a no-timing event per iteration */
    }
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms * 1e3 / reps;
  };
  const char* wn[4] = {"no writes", "plain stores", "nontemporal", "write-through sc1"};
  for (int round = 0; round < 2; round++)
    for (int wr = 0; wr < 4; wr++) {
      float t0 = run(0, wr), t1 = run(1, wr), t2 = run(2, wr);
      printf("round %d, long kernel %-18s: alone %.2f us/iter; + short %.2f (+%.2f); + short + event record %.2f (+%.2f)\n",
             round, wn[wr], t0, t1, t1 - t0, t2, t2 - t0);
    }
  return 0;
}
