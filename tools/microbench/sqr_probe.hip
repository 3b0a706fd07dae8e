// Where does a field squaring's time go on gfx950? Runs the production fe_sqr as dependent
// chains under several occupancy / ILP shapes and stamps the in-kernel clock
// (s_memtime / s_memrealtime, MI355X_MICROARCH.md DVFS item 6), so the cost can be stated in
// real shader cycles per wave-squaring per SIMD and compared with the instruction-issue sum.
// Result (profiles/r01_sqr_probe.txt, r02_sqr_probe_radix.txt, r02_sqr_probe_r25.txt): ~380 cycles per wave-squaring at every occupancy (2-8
// waves/SIMD) and with two independent chains per lane, so the squaring is VALU-issue-bound;
// 16 extra `s_nop 0` per squaring cost nothing (the hazard pads LLVM puts after inline asm are
// free), and a hazard-aware hand schedule of every instruction (tried, not kept) ran the same.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../ed25519-consensus_amd/csrc sqr_probe.hip -o sqr_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include "fe25519.h"
using namespace edc;

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 1024;

__device__ fe seed_fe(uint32_t s) {
  fe a;
  for (int i = 0; i < 9; ++i) a.v[i] = (s * 2654435761u + i * 40503u) & M29;
  return a;
}

__device__ __forceinline__ void stamp(unsigned long long* clk, uint64_t t0, uint64_t r0) {
  if (threadIdx.x == 0) {
    uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

template <int W>
__global__ void __launch_bounds__(256, W) k_sqr(uint32_t* out, unsigned long long* clk, uint32_t s) {
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  fe a = seed_fe(s + blockIdx.x * 256 + threadIdx.x);
  for (int i = 0; i < ITERS; ++i) a = fe_sqr(a);
  out[blockIdx.x * 256 + threadIdx.x] = a.v[0] ^ a.v[8];
  stamp(clk, t0, r0);
}

template <int W>
__global__ void __launch_bounds__(256, W) k_sqr2(uint32_t* out, unsigned long long* clk, uint32_t s) {
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  fe a = seed_fe(s + blockIdx.x * 256 + threadIdx.x), b = seed_fe(s * 3 + blockIdx.x * 256 + threadIdx.x);
  for (int i = 0; i < ITERS / 2; ++i) { a = fe_sqr(a); b = fe_sqr(b); }
  out[blockIdx.x * 256 + threadIdx.x] = a.v[0] ^ a.v[8] ^ b.v[1];
  stamp(clk, t0, r0);
}

template <int W>
__global__ void __launch_bounds__(256, W) k_mul(uint32_t* out, unsigned long long* clk, uint32_t s) {
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  fe a = seed_fe(s + blockIdx.x * 256 + threadIdx.x), b = seed_fe(s * 7 + threadIdx.x);
  for (int i = 0; i < ITERS; ++i) a = fe_mul(a, b);
  out[blockIdx.x * 256 + threadIdx.x] = a.v[0] ^ a.v[8];
  stamp(clk, t0, r0);
}

// pure issue rate of independent v_mad_u64_u32 (8 chains), for the cycle calibration
template <int W>
__global__ void __launch_bounds__(256, W) k_mad(uint32_t* out, unsigned long long* clk, uint32_t s) {
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  uint64_t acc[8];
  uint32_t x = s + threadIdx.x, y = s ^ blockIdx.x;
  for (int j = 0; j < 8; ++j) acc[j] = j;
  for (int i = 0; i < ITERS * 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = mad64(x + j, y, acc[j]);
  uint64_t r = 0;
  for (int j = 0; j < 8; ++j) r ^= acc[j];
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)r ^ (uint32_t)(r >> 32);
  stamp(clk, t0, r0);
}

// price of s_nop 0: the production squaring plus 16 explicit pads
template <int W>
__global__ void __launch_bounds__(256, W) k_sqr_nop(uint32_t* out, unsigned long long* clk, uint32_t s) {
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  fe a = seed_fe(s + blockIdx.x * 256 + threadIdx.x);
  for (int i = 0; i < ITERS; ++i) {
    a = fe_sqr(a);
    asm volatile("s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n"
                 "s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0");
  }
  out[blockIdx.x * 256 + threadIdx.x] = a.v[0] ^ a.v[8];
  stamp(clk, t0, r0);
}

// ---- full-radix alternative (north star: "64-bit-limb arithmetic"): 4 x 64-bit limbs held as
// 8 x 32-bit words, value < 2^256, mod p via 2^256 == 38. Comba columns of the 28 cross products
// accumulate in 64 bits with the carry-out of every v_mad_u64_u32 counted by a v_addc_co_u32
// (the carry-in-mad trick of radix 2^29 is impossible: full 32-bit limbs overflow a 64-bit
// column), then doubling, the 8 squares and the 38-fold.
__device__ __forceinline__ uint64_t mad_cc(uint32_t a, uint32_t b, uint64_t c, uint32_t& cnt) {
  uint64_t d;
  asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %4\n\tv_addc_co_u32 %1, vcc, 0, %1, vcc"
               : "=&v"(d), "+v"(cnt) : "v"(a), "v"(b), "v"(c) : "vcc");
  return d;
}

struct fe32 { uint32_t w[8]; };

__device__ __forceinline__ fe32 sqr_r32(const fe32& x) {
  const uint32_t* a = x.w;
  uint32_t t[16];
  // cross products sum_{i<j} a_i a_j, column by column (96-bit running value cnt:acc)
  uint64_t acc = 0;
  uint32_t cnt = 0;
#pragma unroll
  for (int k = 1; k < 14; ++k) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int j = k - i;
      if (j > i && j < 8) acc = mad_cc(a[i], a[j], acc, cnt);
    }
    t[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)cnt << 32);
    cnt = 0;
  }
  t[0] = 0;
  t[14] = (uint32_t)acc;
  t[15] = (uint32_t)(acc >> 32);
  // double, then add the squares a_i^2 at columns 2i, 2i+1
  uint32_t top = 0;
#pragma unroll
  for (int k = 15; k >= 1; --k) t[k] = (t[k] << 1) | (t[k - 1] >> 31);
  t[0] = 0;
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t p = (uint64_t)a[i] * a[i];
    uint64_t lo = (uint64_t)t[2 * i] + (uint32_t)p + (c & 0xFFFFFFFFull);
    t[2 * i] = (uint32_t)lo;
    uint64_t hi = (uint64_t)t[2 * i + 1] + (p >> 32) + (lo >> 32) + (c >> 32);
    t[2 * i + 1] = (uint32_t)hi;
    c = hi >> 32;
  }
  top = (uint32_t)c;
  (void)top;
  // fold: t_lo + 38 t_hi (each mad's addend t_lo + carry < 2^33, result < 2^39)
  fe32 r;
  uint64_t f = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    f = mad64(t[8 + i], 38u, (uint64_t)t[i] + (f >> 32));
    r.w[i] = (uint32_t)f;
  }
  // the last carry (< 2^6) once more: 2^256 == 38; a carry out of this pass is folded again
  uint64_t g = (uint64_t)r.w[0] + (f >> 32) * 38u;
  r.w[0] = (uint32_t)g;
#pragma unroll
  for (int i = 1; i < 8; ++i) {
    g = (uint64_t)r.w[i] + (g >> 32);
    r.w[i] = (uint32_t)g;
  }
  r.w[0] += (uint32_t)(g >> 32) * 38u;
  return r;
}

__device__ fe32 seed_fe32(uint32_t s) {
  fe32 a;
  for (int i = 0; i < 8; ++i) a.w[i] = s * 2654435761u + i * 40503u;
  return a;
}

template <int W>
__global__ void __launch_bounds__(256, W) k_sqr_r32(uint32_t* out, unsigned long long* clk, uint32_t s) {
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  fe32 a = seed_fe32(s + blockIdx.x * 256 + threadIdx.x);
  for (int i = 0; i < ITERS; ++i) a = sqr_r32(a);
  out[blockIdx.x * 256 + threadIdx.x] = a.w[0] ^ a.w[7];
  stamp(clk, t0, r0);
}

// correctness of sqr_r32 against the production radix-2^29 fe_sqr (canonical results compared)
__global__ void k_check_r32(uint32_t* bad, uint32_t s) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  fe32 a = seed_fe32(s + t);
  a.w[7] &= 0x7FFFFFFFu;                 // < 2^255: the same value in both representations
  fe x = fe_from_words(a.w);
  for (int i = 0; i < 16; ++i) { a = sqr_r32(a); x = fe_sqr(x); }
  // canonical form of the full-radix value: < 2^256, reduce through radix 2^29 (bit 255 folded as 19)
  uint32_t w[8], y[8];
  for (int i = 0; i < 8; ++i) w[i] = a.w[i];
  const uint32_t b255 = w[7] >> 31;
  w[7] &= 0x7FFFFFFFu;
  fe z = fe_from_words(w);
  z.v[0] += 19u * b255;
  fe_to_words(z, w);
  fe_to_words(x, y);
  uint32_t diff = 0;
  for (int i = 0; i < 8; ++i) diff |= w[i] ^ y[i];
  if (diff) atomicAdd(bad, 1u);
}

// ---- 5 x 51-bit limbs ("64-bit limbs" of the dalek u64 backend) on 32-bit multipliers: each
// 51-bit limb is two 25.5-bit halves, i.e. ten limbs of 26 / 25 bits (weights 2^ceil(25.5 i)),
// 2^255 == 19. A product f_i f_j lands in column i + j (mod 10) with factor 2 when i and j are
// both odd and 19 when it wraps, so the squaring is 55 v_mad_u64_u32 over pre-doubled / x19 / x38
// operands (all < 2^32), chained columns (carry of column k = addend of column k+1) and one
// x19 fold of the top carry: 8 fewer products than radix 2^29 (63), two more column carries,
// ~13 operand pre-multiplications.
struct fe10 { uint32_t v[10]; };

__device__ __forceinline__ uint32_t mul19(uint32_t x) { return (x << 4) + (x << 1) + x; }

__device__ __forceinline__ fe10 sqr_r25(const fe10& a) {
  const uint32_t* f = a.v;
  const uint32_t f0_2 = f[0] << 1, f1_2 = f[1] << 1, f2_2 = f[2] << 1, f3_2 = f[3] << 1, f4_2 = f[4] << 1,
                 f5_2 = f[5] << 1, f6_2 = f[6] << 1, f7_2 = f[7] << 1;
  const uint32_t f6_19 = mul19(f[6]), f8_19 = mul19(f[8]);
  const uint32_t f5_38 = mul19(f[5]) << 1, f7_38 = mul19(f[7]) << 1, f9_38 = mul19(f[9]) << 1;
  fe10 r;
  uint64_t acc;
  acc = mad64(f[0], f[0], 0);
  acc = mad64(f1_2, f9_38, acc); acc = mad64(f2_2, f8_19, acc); acc = mad64(f3_2, f7_38, acc);
  acc = mad64(f4_2, f6_19, acc); acc = mad64(f[5], f5_38, acc);
  r.v[0] = (uint32_t)acc & 0x3FFFFFFu; acc >>= 26;
  acc = mad64(f0_2, f[1], acc); acc = mad64(f[2], f9_38, acc); acc = mad64(f3_2, f8_19, acc);
  acc = mad64(f[4], f7_38, acc); acc = mad64(f5_2, f6_19, acc);
  r.v[1] = (uint32_t)acc & 0x1FFFFFFu; acc >>= 25;
  acc = mad64(f0_2, f[2], acc); acc = mad64(f1_2, f[1], acc); acc = mad64(f3_2, f9_38, acc);
  acc = mad64(f4_2, f8_19, acc); acc = mad64(f5_2, f7_38, acc); acc = mad64(f[6], f6_19, acc);
  r.v[2] = (uint32_t)acc & 0x3FFFFFFu; acc >>= 26;
  acc = mad64(f0_2, f[3], acc); acc = mad64(f1_2, f[2], acc); acc = mad64(f[4], f9_38, acc);
  acc = mad64(f5_2, f8_19, acc); acc = mad64(f[6], f7_38, acc);
  r.v[3] = (uint32_t)acc & 0x1FFFFFFu; acc >>= 25;
  acc = mad64(f0_2, f[4], acc); acc = mad64(f1_2, f3_2, acc); acc = mad64(f[2], f[2], acc);
  acc = mad64(f5_2, f9_38, acc); acc = mad64(f6_2, f8_19, acc); acc = mad64(f[7], f7_38, acc);
  r.v[4] = (uint32_t)acc & 0x3FFFFFFu; acc >>= 26;
  acc = mad64(f0_2, f[5], acc); acc = mad64(f1_2, f[4], acc); acc = mad64(f2_2, f[3], acc);
  acc = mad64(f[6], f9_38, acc); acc = mad64(f7_2, f8_19, acc);
  r.v[5] = (uint32_t)acc & 0x1FFFFFFu; acc >>= 25;
  acc = mad64(f0_2, f[6], acc); acc = mad64(f1_2, f5_2, acc); acc = mad64(f2_2, f[4], acc);
  acc = mad64(f3_2, f[3], acc); acc = mad64(f7_2, f9_38, acc); acc = mad64(f[8], f8_19, acc);
  r.v[6] = (uint32_t)acc & 0x3FFFFFFu; acc >>= 26;
  acc = mad64(f0_2, f[7], acc); acc = mad64(f1_2, f[6], acc); acc = mad64(f2_2, f[5], acc);
  acc = mad64(f3_2, f[4], acc); acc = mad64(f[8], f9_38, acc);
  r.v[7] = (uint32_t)acc & 0x1FFFFFFu; acc >>= 25;
  acc = mad64(f0_2, f[8], acc); acc = mad64(f1_2, f7_2, acc); acc = mad64(f2_2, f[6], acc);
  acc = mad64(f3_2, f5_2, acc); acc = mad64(f[4], f[4], acc); acc = mad64(f[9], f9_38, acc);
  r.v[8] = (uint32_t)acc & 0x3FFFFFFu; acc >>= 26;
  acc = mad64(f0_2, f[9], acc); acc = mad64(f1_2, f[8], acc); acc = mad64(f2_2, f[7], acc);
  acc = mad64(f3_2, f[6], acc); acc = mad64(f4_2, f[5], acc);
  r.v[9] = (uint32_t)acc & 0x1FFFFFFu; acc >>= 25;
  // top carry (weight 2^255 == 19) into limb 0, its overflow into limb 1
  const uint64_t t = mad64((uint32_t)acc, 19u, (uint64_t)r.v[0]) + ((uint64_t)(uint32_t)(acc >> 32) * 19u << 32);
  r.v[0] = (uint32_t)t & 0x3FFFFFFu;
  r.v[1] += (uint32_t)(t >> 26);
  return r;
}

__device__ __forceinline__ uint32_t bits_at(const uint32_t w[8], int start, int len) {
  const int k = start >> 5, sh = start & 31;
  const uint64_t two = (uint64_t)w[k] | ((uint64_t)(k < 7 ? w[k + 1] : 0u) << 32);
  return (uint32_t)(two >> sh) & ((1u << len) - 1u);
}
__device__ const int R25_OFF[11] = {0, 26, 51, 77, 102, 128, 153, 179, 204, 230, 255};

__device__ fe10 fe10_from_words(const uint32_t w[8]) {
  fe10 a;
  for (int i = 0; i < 10; ++i) a.v[i] = bits_at(w, R25_OFF[i], R25_OFF[i + 1] - R25_OFF[i]);
  return a;
}
// canonical 8 words of a lazy fe10 (serial carries, 2^255 == 19, then radix 2^29 canonicalisation)
__device__ void fe10_to_words(fe10 a, uint32_t out[8]) {
  for (int pass = 0; pass < 3; ++pass) {
    uint32_t c = 0;
    for (int i = 0; i < 10; ++i) {
      const int len = R25_OFF[i + 1] - R25_OFF[i];
      const uint64_t x = (uint64_t)a.v[i] + c;
      a.v[i] = (uint32_t)x & ((1u << len) - 1u);
      c = (uint32_t)(x >> len);
    }
    a.v[0] += 19u * c;
  }
  uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 10; ++i) {
    const int st = R25_OFF[i], k = st >> 5, sh = st & 31;
    w[k] |= a.v[i] << sh;
    if (sh && k < 7) w[k + 1] |= (uint32_t)((uint64_t)a.v[i] >> (32 - sh));
  }
  fe z = fe_from_words(w);   // < 2^255
  fe_to_words(z, out);
}

template <int W>
__global__ void __launch_bounds__(256, W) k_sqr_r25(uint32_t* out, unsigned long long* clk, uint32_t s) {
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  fe10 a;
  for (int i = 0; i < 10; ++i) a.v[i] = ((s + blockIdx.x * 256 + threadIdx.x) * 2654435761u + i * 40503u) & 0x1FFFFFFu;
  for (int i = 0; i < ITERS; ++i) a = sqr_r25(a);
  out[blockIdx.x * 256 + threadIdx.x] = a.v[0] ^ a.v[9];
  stamp(clk, t0, r0);
}

__global__ void k_check_r25(uint32_t* bad, uint32_t s) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  fe32 a = seed_fe32(s + t);
  a.w[7] &= 0x7FFFFFFFu;
  fe x = fe_from_words(a.w);
  fe10 y = fe10_from_words(a.w);
  for (int i = 0; i < 16; ++i) { y = sqr_r25(y); x = fe_sqr(x); }
  uint32_t w[8], v[8];
  fe10_to_words(y, w);
  fe_to_words(x, v);
  uint32_t diff = 0;
  for (int i = 0; i < 8; ++i) diff |= w[i] ^ v[i];
  if (diff) atomicAdd(bad, 1u);
}

typedef void (*kfn)(uint32_t*, unsigned long long*, uint32_t);

// occupancy is pinned with dynamic LDS: w blocks of 256 lanes (one wave per SIMD each) per CU
int run(const char* name, kfn f, int w, double ops_per_lane, double issue_est, uint32_t* d, unsigned long long* clk, int blocks) {
  const size_t lds = (160 * 1024) / w - 1024;
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(f, dim3(blocks), dim3(256), lds, 0, d, clk, 1u + r);  // warm the clock state
  CHK(hipDeviceSynchronize());
  const int reps = 10;
  CHK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(f, dim3(blocks), dim3(256), lds, 0, d, clk, 100u + r);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> h(2 * blocks);
  CHK(hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost));
  std::vector<double> ghz;
  for (int b = 0; b < blocks; ++b) if (h[2 * b + 1]) ghz.push_back((double)h[2 * b] / h[2 * b + 1] * 0.1);
  std::sort(ghz.begin(), ghz.end());
  double clk_ghz = ghz[ghz.size() / 2];
  double lane_ops = (double)blocks * 256 * ops_per_lane * reps;
  double wave_ops_per_simd = lane_ops / 64 / 1024;
  double cyc = ms * 1e-3 * clk_ghz * 1e9 / wave_ops_per_simd;
  printf("%-14s %8.3f ms  %7.2f G lane-ops/s  clock %.3f GHz  %7.1f cyc/wave-op/SIMD  (issue estimate %.0f)\n", name,
         ms / reps, lane_ops / (ms * 1e-3) / 1e9, clk_ghz, cyc, issue_est);
  return 0;
}

int main() {
  const int blocks = 256 * 8 * 4;
  uint32_t* d;
  unsigned long long* clk;
  CHK(hipMalloc(&d, (size_t)blocks * 256 * 4));
  CHK(hipMalloc(&clk, (size_t)blocks * 16));
  run("mad x8 w4", k_mad<4>, 4, ITERS * 8 * 8, 4, d, clk, blocks);
  run("mad x8 w8", k_mad<8>, 8, ITERS * 8 * 8, 4, d, clk, blocks);
  run("sqr w4", k_sqr<4>, 4, ITERS, 336, d, clk, blocks);
  run("sqr w8", k_sqr<8>, 8, ITERS, 336, d, clk, blocks);
  run("sqr ilp2 w4", k_sqr2<4>, 4, ITERS, 336, d, clk, blocks);
  run("sqr ilp2 w2", k_sqr2<2>, 2, ITERS, 336, d, clk, blocks);
  run("sqr+16nop w4", k_sqr_nop<4>, 4, ITERS, 336, d, clk, blocks);
  {
    uint32_t* bad;
    CHK(hipMalloc(&bad, 4));
    CHK(hipMemset(bad, 0, 4));
    hipLaunchKernelGGL(k_check_r32, dim3(1024), dim3(256), 0, 0, bad, 12345u);
    uint32_t hb = 0;
    CHK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
    printf("sqr_r32 vs fe_sqr: %u mismatches of %d (16 chained squarings each)\n", hb, 1024 * 256);
    CHK(hipFree(bad));
  }
  {
    uint32_t* bad;
    CHK(hipMalloc(&bad, 4));
    CHK(hipMemset(bad, 0, 4));
    hipLaunchKernelGGL(k_check_r25, dim3(1024), dim3(256), 0, 0, bad, 777u);
    uint32_t hb = 0;
    CHK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
    printf("sqr_r25 vs fe_sqr: %u mismatches of %d (16 chained squarings each)\n", hb, 1024 * 256);
    CHK(hipFree(bad));
  }
  run("sqr_r25 w4", k_sqr_r25<4>, 4, ITERS, 0, d, clk, blocks);
  run("sqr_r25 w8", k_sqr_r25<8>, 8, ITERS, 0, d, clk, blocks);
  run("sqr_r32 w4", k_sqr_r32<4>, 4, ITERS, 0, d, clk, blocks);
  run("sqr_r32 w8", k_sqr_r32<8>, 8, ITERS, 0, d, clk, blocks);
  run("mul w4", k_mul<4>, 4, ITERS, 456, d, clk, blocks);
  run("mul w8", k_mul<8>, 8, ITERS, 456, d, clk, blocks);
  CHK(hipFree(d));
  return 0;
}
