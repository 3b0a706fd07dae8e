// Single-wave latency of the field and quad point operations on gfx950: the serial tails of the
// MSM (Horner pass, window combines) run one dependent chain on one wave. Compares the
// throughput-shaped fe_mul / fe_sqr (one long carry chain through the mad addends) with the
// latency-shaped fe_mul_lat / fe_sqr_lat (fe_lat.h here: independent column chains, parallel
// carries) in real shader cycles (s_memtime) per operation, with the quad point operations
// beside them, and checks that both field shapes give the same values.
// Result (profiles/r02_lat_probe.txt): the latency shape is slower (a lone wave is issue-bound).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I. -I../../ed25519-consensus_amd/csrc lat_probe.hip -o lat_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include "ge_quad.h"
#include "fe_lat.h"
using namespace edc;

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 512;

__device__ fe seed_fe(uint32_t s) {
  fe a;
  for (int i = 0; i < 9; ++i) a.v[i] = (s * 2654435761u + i * 40503u) & M29;
  return a;
}

__device__ ge_p3 seed_pt(uint32_t s) {
  ge_p3 P;
  P.X = seed_fe(s); P.Y = seed_fe(s + 1); P.Z = seed_fe(s + 2); P.T = seed_fe(s + 3);
  return P;
}

template <int OP>
__global__ void k_chain(uint32_t* out, unsigned long long* clk, uint32_t s) {
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  uint32_t h = 0;
  if (OP < 4) {
    fe a = seed_fe(s + threadIdx.x), b = seed_fe(s * 7 + threadIdx.x);
    for (int i = 0; i < ITERS; ++i) {
      if (OP == 0) a = fe_mul(a, b);
      if (OP == 1) a = fe_mul_lat(a, b);
      if (OP == 2) a = fe_sqr(a);
      if (OP == 3) a = fe_sqr_lat(a);
    }
    h = a.v[0] ^ a.v[8];
  } else {
    ge_p3 P = seed_pt(s + threadIdx.x / 4), Q = seed_pt(s * 5 + threadIdx.x / 4);
    for (int i = 0; i < ITERS; ++i) {
      if (OP == 4) P = quad_dbl(P);
      if (OP == 5) P = quad_add(P, Q);
    }
    h = P.X.v[0] ^ P.T.v[8];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = h;
  if (threadIdx.x == 0) clk[blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
}

// both shapes give the same canonical values
__global__ void k_check(uint32_t* bad, uint32_t s) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  fe a = seed_fe(s + t), b = seed_fe(s * 3 + t), x = a, y = a;
  for (int i = 0; i < 64; ++i) {
    x = fe_mul(fe_sqr(x), fe_add(b, x));
    y = fe_mul_lat(fe_sqr_lat(y), fe_add(b, y));
  }
  if (!fe_eq(x, y)) atomicOr(bad, 1u);
}

typedef void (*kfn)(uint32_t*, unsigned long long*, uint32_t);

int main() {
  uint32_t *out, *bad;
  unsigned long long* clk;
  CHK(hipMalloc(&out, 1 << 20));
  CHK(hipMalloc(&bad, 4));
  CHK(hipMalloc(&clk, 4096));
  CHK(hipMemset(bad, 0, 4));
  hipLaunchKernelGGL(k_check, dim3(64), dim3(256), 0, 0, bad, 12345u);
  CHK(hipDeviceSynchronize());
  uint32_t hb = 0;
  CHK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
  printf("check (0 = throughput and latency shapes agree): %u\n", hb);
  struct { kfn f; const char* name; } ks[] = {
      {k_chain<0>, "fe_mul"},  {k_chain<1>, "fe_mul_lat"},   {k_chain<2>, "fe_sqr"},   {k_chain<3>, "fe_sqr_lat"},
      {k_chain<4>, "quad_dbl"}, {k_chain<5>, "quad_add"}};
  for (int waves : {1, 4}) {
    for (auto& k : ks) {
      unsigned long long c[4] = {0, 0, 0, 0};
      for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k.f, dim3(1), dim3(64 * waves), 0, 0, out, clk, 7u + rep);
        CHK(hipDeviceSynchronize());
      }
      CHK(hipMemcpy(c, clk, 8, hipMemcpyDeviceToHost));
      printf("%-13s waves/CU %d: %7.1f cycles per op\n", k.name, waves, (double)c[0] / ITERS);
    }
  }
  return hb ? 2 : 0;
}
