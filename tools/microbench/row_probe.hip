// Row (limb-sliced) point arithmetic (csrc/ge_row.h) against the quad layout (ge_quad.h) on gfx950:
//  1. equality: a chain of doublings and additions of random points in both layouts, every
//     coordinate compared as a field element (canonical form);
//  2. single-wave latency (s_memtime cycles) of a doubling and an addition in each layout.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../ed25519-consensus_amd/csrc row_probe.hip -o row_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include "ge_quad.h"
#include "ge_row.h"
#include "edc_common.h"
using namespace edc;

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ fe seed_fe(uint32_t s) {
  fe a;
  uint32_t x = s * 2654435761u + 12345u;
  for (int i = 0; i < 9; ++i) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    a.v[i] = x & M29;
  }
  return a;
}
__device__ ge_p3 seed_pt(uint32_t s) {
  ge_p3 P;
  P.X = seed_fe(4 * s); P.Y = seed_fe(4 * s + 1); P.Z = seed_fe(4 * s + 2); P.T = seed_fe(4 * s + 3);
  return P;
}

// one workgroup of 64 lanes per test case: the quad version on lanes 0..3, the row version on
// the whole wave; both write canonical words of X, Y, Z, T
__global__ void k_check(uint32_t* bad, uint32_t* dump, int nd, int every) {
  __shared__ uint32_t pq[36], pr[36], qs[36];
  const uint32_t s = blockIdx.x;
  const ge_p3 P0 = seed_pt(7 * s + 1), Q = seed_pt(7 * s + 3);
  if (threadIdx.x == 0) st_fe(qs, Q.X), st_fe(qs + 9, Q.Y), st_fe(qs + 18, Q.Z), st_fe(qs + 27, Q.T);
  __syncthreads();
  if (threadIdx.x < 4) {
    quad_pt a = quad_distribute(P0);
    for (int i = 1; i <= nd; ++i) {
      a = quad_dbl_d(a);
      if (i % every == 0) a = quad_add_d(a, Q);
    }
    ge_p3 r = quad_collect(a);
    if (threadIdx.x == 0) {
      st_fe(pq, fe_canon(r.X)); st_fe(pq + 9, fe_canon(r.Y)); st_fe(pq + 18, fe_canon(r.Z)); st_fe(pq + 27, fe_canon(r.T));
    }
  }
  __syncthreads();
  {
    const RowCtx c = row_ctx();
    const uint32_t d2 = row_d2(c);
    __shared__ uint32_t p0s[36];
    if (threadIdx.x == 0) st_fe(p0s, P0.X), st_fe(p0s + 9, P0.Y), st_fe(p0s + 18, P0.Z), st_fe(p0s + 27, P0.T);
    __syncthreads();
    uint32_t a = row_ld_ext(c, p0s);
    const uint32_t bq = row_cached(c, qs, d2);
    for (int i = 1; i <= nd; ++i) {
      a = row_dbl(c, a);
      if (i % every == 0) a = row_add(c, a, bq);
    }
    __shared__ uint32_t raw[36];
    row_st_ext(c, raw, a);
    __syncthreads();
    if (threadIdx.x == 0) {
      ge_p3 r = ld_ext(raw);
      st_fe(pr, fe_canon(r.X)); st_fe(pr + 9, fe_canon(r.Y)); st_fe(pr + 18, fe_canon(r.Z)); st_fe(pr + 27, fe_canon(r.T));
    }
  }
  __syncthreads();
  if (threadIdx.x < 36 && pq[threadIdx.x] != pr[threadIdx.x]) atomicAdd(bad, 1u);
  if (s == 0 && threadIdx.x < 36) { dump[threadIdx.x] = pq[threadIdx.x]; dump[36 + threadIdx.x] = pr[threadIdx.x]; }
}

// field-level check of rf_mul against fe_mul on random inputs (including max-bound limbs)
__global__ void k_check_mul(uint32_t* bad) {
  __shared__ uint32_t A[9], B[9], R[9];
  const uint32_t s = blockIdx.x;
  fe a = seed_fe(3 * s + 5), b = seed_fe(3 * s + 6);
  if (s % 4 == 1) for (int i = 0; i < 9; ++i) { a.v[i] = (1u << 30) + (1u << 29) + (a.v[i] & 0xFFFFF); }   // < 2^30.41
  if (s % 4 == 2) for (int i = 0; i < 9; ++i) { a.v[i] = 0x59000000u; b.v[i] = 0x59000000u; }
  if (threadIdx.x == 0) { st_fe(A, a); st_fe(B, b); }
  __syncthreads();
  const RowCtx c = row_ctx();
  const uint32_t ra = c.live ? A[c.j] : 0u, rb = c.live ? B[c.j] : 0u;
  const uint32_t r = rf_mul(c, ra, rb);
  if (threadIdx.x < 9) R[threadIdx.x] = r;
  __syncthreads();
  if (threadIdx.x == 0) {
    fe rr = ld_fe(R);
    for (int i = 0; i < 9; ++i) if (rr.v[i] >= (1u << 29) + (1u << 19)) atomicAdd(bad, 1000u);
    if (!fe_eq(rr, fe_mul(a, b))) atomicAdd(bad, 1u);
  }
  if (threadIdx.x >= 9 && threadIdx.x < 16 && r != 0) atomicAdd(bad, 100000u);
}

constexpr int ITERS = 256;
template <int OP>
__global__ void k_time(uint32_t* out, unsigned long long* clk) {
  __shared__ uint32_t qs[36];
  const ge_p3 P = seed_pt(threadIdx.x / 4 + 11), Q = seed_pt(5);
  if (threadIdx.x == 0) st_fe(qs, Q.X), st_fe(qs + 9, Q.Y), st_fe(qs + 18, Q.Z), st_fe(qs + 27, Q.T);
  __syncthreads();
  uint32_t h = 0;
  uint64_t t0 = 0, t1 = 0;
  if (OP < 2) {
    quad_pt a = quad_distribute(P);
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) a = OP == 0 ? quad_dbl_d(a) : quad_add_d(a, Q);
    t1 = __builtin_amdgcn_s_memtime();
    h = a.c.v[0];
  } else {
    const RowCtx c = row_ctx();
    const uint32_t d2 = row_d2(c);
    uint32_t a = row_ld_ext(c, qs);
    const uint32_t bq = row_cached(c, qs, d2);
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) a = OP == 2 ? row_dbl(c, a) : row_add(c, a, bq);
    t1 = __builtin_amdgcn_s_memtime();
    h = a;
  }
  out[threadIdx.x] = h;
  if (threadIdx.x == 0) clk[0] = t1 - t0;
}

int main() {
  uint32_t *bad, *dump, *out;
  unsigned long long* clk;
  CHK(hipMalloc(&bad, 8));
  CHK(hipMalloc(&dump, 1024));
  CHK(hipMalloc(&out, 4096));
  CHK(hipMalloc(&clk, 64));
  CHK(hipMemset(bad, 0, 8));
  hipLaunchKernelGGL(k_check_mul, dim3(4096), dim3(64), 0, 0, bad);
  CHK(hipDeviceSynchronize());
  uint32_t hb = 0;
  CHK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
  printf("rf_mul vs fe_mul mismatches (0 = equal): %u\n", hb);
  uint32_t tot = hb;
  CHK(hipMemset(bad, 0, 8));
  hipLaunchKernelGGL(k_check, dim3(512), dim3(64), 0, 0, bad, dump, 260, 9);
  CHK(hipDeviceSynchronize());
  CHK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
  printf("row vs quad chain (260 doublings, an addition every 9th) mismatching words: %u\n", hb);
  tot += hb;
  if (hb) {
    uint32_t d[72];
    CHK(hipMemcpy(d, dump, sizeof(d), hipMemcpyDeviceToHost));
    for (int i = 0; i < 36; ++i) printf("%2d %08x %08x\n", i, d[i], d[36 + i]);
  }
  typedef void (*kfn)(uint32_t*, unsigned long long*);
  struct { kfn f; const char* name; } ks[] = {{k_time<0>, "quad_dbl_d"}, {k_time<1>, "quad_add_d"},
                                              {k_time<2>, "row_dbl"}, {k_time<3>, "row_add"}};
  for (auto& k : ks) {
    unsigned long long c = 0;
    for (int rep = 0; rep < 3; ++rep) {
      hipLaunchKernelGGL(k.f, dim3(1), dim3(64), 0, 0, out, clk);
      CHK(hipDeviceSynchronize());
    }
    CHK(hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost));
    printf("%-12s %8.1f cycles per op (one wave)\n", k.name, (double)c / ITERS);
  }
  return tot ? 2 : 0;
}
