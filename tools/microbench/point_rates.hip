// Throughput of the field and group operations the batch verifier is built from, on gfx950:
// every lane runs an independent dependent chain of one operation (all CUs busy, 4 waves/SIMD
// launch bound as the production kernels). Prints lane-operations per second and the implied
// v_mad_u64_u32 issue rate.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "edc_common.h"
using namespace edc;

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 256;

__device__ fe seed_fe(uint32_t s) {
  fe a;
  for (int i = 0; i < 9; ++i) a.v[i] = (s * 2654435761u + i * 40503u) & M29;
  return a;
}

__global__ void __launch_bounds__(256, 4) k_sqr(uint32_t* out, uint32_t s) {
  fe a = seed_fe(s + blockIdx.x * 256 + threadIdx.x);
  for (int i = 0; i < ITERS; ++i) a = fe_sqr(a);
  out[blockIdx.x * 256 + threadIdx.x] = a.v[0] ^ a.v[8];
}
__global__ void __launch_bounds__(256, 4) k_mul(uint32_t* out, uint32_t s) {
  fe a = seed_fe(s + blockIdx.x * 256 + threadIdx.x), b = seed_fe(s * 7 + threadIdx.x);
  for (int i = 0; i < ITERS; ++i) a = fe_mul(a, b);
  out[blockIdx.x * 256 + threadIdx.x] = a.v[0] ^ a.v[8];
}
__global__ void __launch_bounds__(256, 4) k_madd(uint32_t* out, uint32_t s) {
  ge_p3 P;
  P.X = seed_fe(s + threadIdx.x); P.Y = seed_fe(s + 1 + threadIdx.x); P.Z = fe_one(); P.T = seed_fe(s + 3);
  ge_niels q;
  q.ypx = seed_fe(s ^ blockIdx.x); q.ymx = seed_fe(s + 5); q.xy2d = seed_fe(s + 9);
  for (int i = 0; i < ITERS / 8; ++i) P = ge_madd(P, q);
  out[blockIdx.x * 256 + threadIdx.x] = P.X.v[0] ^ P.Z.v[8];
}
__global__ void __launch_bounds__(256, 4) k_madd_sgn(uint32_t* out, uint32_t s) {
  ge_p3 P;
  P.X = seed_fe(s + threadIdx.x); P.Y = seed_fe(s + 1 + threadIdx.x); P.Z = fe_one(); P.T = seed_fe(s + 3);
  ge_niels q;
  q.ypx = seed_fe(s ^ blockIdx.x); q.ymx = seed_fe(s + 5); q.xy2d = seed_fe(s + 9);
  uint32_t bits = s * 2654435761u + threadIdx.x;
  for (int i = 0; i < ITERS / 8; ++i) P = ge_madd_sgn(P, q, (bits >> (i & 31)) & 1u);
  out[blockIdx.x * 256 + threadIdx.x] = P.X.v[0] ^ P.Z.v[8];
}
__global__ void __launch_bounds__(256, 4) k_dbl(uint32_t* out, uint32_t s) {
  ge_p3 P;
  P.X = seed_fe(s + threadIdx.x); P.Y = seed_fe(s + 1 + threadIdx.x); P.Z = fe_one(); P.T = seed_fe(s + 3);
  for (int i = 0; i < ITERS / 8; ++i) P = ge_dbl(P);
  out[blockIdx.x * 256 + threadIdx.x] = P.X.v[0] ^ P.Z.v[8];
}

typedef void (*kfn)(uint32_t*, uint32_t);

int run(const char* name, kfn f, int ops_per_lane, double mads_per_op, uint32_t* d, int blocks) {
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, d, 1u);
  CHK(hipDeviceSynchronize());
  const int reps = 5;
  CHK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, d, 2u + r);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
  double ops = (double)blocks * 256 * ops_per_lane * reps;
  double rate = ops / (ms * 1e-3);
  // cycles per wave-operation per SIMD at the nominal 2.4 GHz (1024 SIMDs)
  const double cyc = 1024.0 * 2.4e9 / (rate / 64.0);
  printf("%-10s %9.3f G lane-ops/s  %8.2f T v_mad_u64_u32/s issued (%.0f per op)  %7.0f cyc/wave-op/SIMD\n", name,
         rate / 1e9, rate * mads_per_op / 1e12, mads_per_op, cyc);
  return 0;
}

int main() {
  const int blocks = 256 * 4 * 8;
  uint32_t* d;
  CHK(hipMalloc(&d, (size_t)blocks * 256 * 4));
  run("fe_sqr", k_sqr, ITERS, 63, d, blocks);
  run("fe_mul", k_mul, ITERS, 99, d, blocks);
  run("ge_madd", k_madd, ITERS / 8, 7 * 99, d, blocks);
  run("ge_madd_sgn", k_madd_sgn, ITERS / 8, 7 * 99, d, blocks);
  run("ge_dbl", k_dbl, ITERS / 8, 4 * 63 + 4 * 99, d, blocks);
  CHK(hipFree(d));
  return 0;
}
