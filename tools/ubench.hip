// Micro-benchmarks of the cross-lane primitives used by the compact-tier solver (diagnostic only).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/ubench tools/ubench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>

#define NV 20
__device__ __forceinline__ double rl(double v, int lane) {
  long long b = __builtin_bit_cast(long long, v);
  int lo = __builtin_amdgcn_readlane((int)(unsigned int)(b & 0xffffffffll), lane);
  int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __builtin_bit_cast(double, (long long)(((unsigned long long)(unsigned int)hi << 32) | (unsigned int)lo));
}

// 0: dependent fp64 add chain (1000)
// 1: dependent rl-sum over 20 lanes (x50)
// 2: sqrt chain (100), 3: div chain (100)
// 4: cholesky readlane, 5: cholesky LDS broadcast
__global__ void kb(int which, double* out, unsigned long long* cyc, int reps) {
  __shared__ double sh[64 * 16 + NV * NV + 64];
  const int lane = threadIdx.x;
  double v = 1.0 + lane * 1e-3;
  double h[NV];
  for (int c = 0; c < NV; c++) h[c] = (lane == c ? 40.0 : 0.0) + 1.0 / (1 + lane + c);
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; r++) {
    if (which == 0) {
      for (int i = 0; i < 1000; i++) v = v + 1e-9 * i;
    } else if (which == 1) {
      for (int it = 0; it < 50; it++) {
        double acc = 0;
        for (int i = 0; i < NV; i++) acc += rl(v, i);
        v = acc * 1e-3;
      }
    } else if (which == 2) {
      for (int i = 0; i < 100; i++) v = sqrt(v + 1.0);
    } else if (which == 3) {
      for (int i = 0; i < 100; i++) v = 3.0 / (v + 1.0);
    } else if (which == 6) {
      double a0 = v, a1 = v + 1, a2 = v + 2, a3 = v + 3, a4 = v + 4, a5 = v + 5, a6 = v + 6, a7 = v + 7;
      for (int i = 0; i < 125; i++) {
        a0 = a0 * 1.0000001; a1 = a1 * 1.0000001; a2 = a2 * 1.0000001; a3 = a3 * 1.0000001;
        a4 = a4 * 1.0000001; a5 = a5 * 1.0000001; a6 = a6 * 1.0000001; a7 = a7 * 1.0000001;
      }
      v = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    } else if (which == 7) {
      for (int i = 0; i < 1000; i++) v = v * 1.0000001;
    } else if (which == 8) {
      float f0 = v, f1 = v + 1, f2 = v + 2, f3 = v + 3, f4 = v + 4, f5 = v + 5, f6 = v + 6, f7 = v + 7;
      for (int i = 0; i < 125; i++) {
        f0 = f0 * 1.0000001f; f1 = f1 * 1.0000001f; f2 = f2 * 1.0000001f; f3 = f3 * 1.0000001f;
        f4 = f4 * 1.0000001f; f5 = f5 * 1.0000001f; f6 = f6 * 1.0000001f; f7 = f7 * 1.0000001f;
      }
      v = f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7;
    } else if (which == 9) {
      /* dependent LDS pointer chase (ds_read_b32 -> address of the next read), x100 */
      int* ish = (int*)sh;
      ish[lane] = (lane + 1) & 63;
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
      int idx = lane;
      for (int i = 0; i < 100; i++) { idx = ish[idx]; asm volatile("" : "+v"(idx)); }
      v += idx;
    } else if (which == 10) {
      /* LDS write -> read-back round trip of a double through a neighbour lane, x100 */
      for (int i = 0; i < 100; i++) {
        sh[lane] = v;
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        v = sh[(lane + 1) & 63] * 1.0000001;
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
      }
    } else if (which == 11) {
      /* 16 doubles copied parent -> child per "level" (kinematics level loop shape), x20 levels */
      int pid = lane > 0 ? lane - 1 : 0;
      for (int l = 1; l <= 20; l++) {
        if (lane == l) {
          for (int c = 0; c < 16; c++) sh[lane * 16 + c] = sh[pid * 16 + c] + 1e-9;
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
      }
      v += sh[lane];
    } else if (which == 4) {
#pragma unroll
      for (int j = 0; j < NV; j++) {
        double sum = rl(h[j], j);
        if (sum < 1e-15) sum = 1e-15;
        double ljj = sqrt(sum);
        if (lane > j) h[j] = h[j] / ljj;
        if (lane == j) h[j] = ljj;
#pragma unroll
        for (int k = j + 1; k < NV; k++) {
          double lkj = rl(h[j], k);
          if (lane >= k) h[k] -= h[j] * lkj;
        }
      }
      v += h[NV - 1];
    } else if (which == 5) {
#pragma unroll
      for (int j = 0; j < NV; j++) {
        double sum = rl(h[j], j);
        if (sum < 1e-15) sum = 1e-15;
        double ljj = sqrt(sum);
        if (lane > j) h[j] = h[j] / ljj;
        if (lane == j) h[j] = ljj;
        sh[lane] = h[j];
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        double col[NV];
#pragma unroll
        for (int k = j + 1; k < NV; k++) col[k] = sh[k];
#pragma unroll
        for (int k = j + 1; k < NV; k++)
          if (lane >= k) h[k] -= h[j] * col[k];
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
      }
      v += h[NV - 1];
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + lane] = v;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  double* out;
  unsigned long long* cyc;
  hipMalloc(&out, sizeof(double) * 64 * 4096);
  hipMalloc(&cyc, sizeof(unsigned long long) * 4096);
  const char* names[] = {"fp64 add chain x1000", "rl-sum 20 lanes x50", "sqrt chain x100", "div chain x100",
                         "cholesky20 readlane", "cholesky20 lds-bcast", "fp64 mul 8 indep x125", "fp64 mul dep x1000",
                         "fp32 mul 8 indep x125", "lds ptr-chase x100", "lds wr->rd trip x100",
                         "lds level copy x20"};
  for (int which = 0; which < 12; which++) {
    for (int grid : {1, 1024}) {
      int reps = 4;
      hipLaunchKernelGGL(kb, dim3(grid), dim3(64), 0, 0, which, out, cyc, 1);
      hipLaunchKernelGGL(kb, dim3(grid), dim3(64), 0, 0, which, out, cyc, reps);
      hipDeviceSynchronize();
      unsigned long long h[1024];
      hipMemcpy(h, cyc, sizeof(unsigned long long) * grid, hipMemcpyDeviceToHost);
      double avg = 0;
      for (int i = 0; i < grid; i++) avg += h[i];
      avg /= grid * reps;
      printf("%-26s grid %5d : %10.0f cycles per rep\n", names[which], grid, avg);
    }
  }
  return 0;
}
