// Shared device-side storage helpers and the workspace layout used by every kernel.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "fe25519.h"
#include "ge25519.h"
#include "sc25519.h"
#include "sha512.h"
#include "chacha20.h"
#include "keycache.h"

namespace edc {

// ---- HBM record layouts ----
// affine Niels point: ypx | ymx | xy2d as 9 radix-2^29 limbs each (27 words), padded to 32 words
// so that every record is exactly one 128-byte cache line: the MSM gathers points in random
// order, and a 112-byte record straddled two lines most of the time.
constexpr int NIELS_WORDS = 32;
// extended point: X | Y | Z | T, 36 words (144 B)
constexpr int EXT_WORDS = 36;

__device__ __forceinline__ fe ld_fe(const uint32_t* p) {
  fe r;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = p[i];
  return r;
}
__device__ __forceinline__ void st_fe(uint32_t* p, const fe& a) {
#pragma unroll
  for (int i = 0; i < 9; ++i) p[i] = a.v[i];
}

__device__ __forceinline__ ge_niels ld_niels(const uint32_t* base, uint32_t idx) {
  const uint4* q = reinterpret_cast<const uint4*>(base + (size_t)idx * NIELS_WORDS);
  uint32_t w[28];
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    uint4 t = q[i];
    w[4 * i] = t.x; w[4 * i + 1] = t.y; w[4 * i + 2] = t.z; w[4 * i + 3] = t.w;
  }
  ge_niels n;
#pragma unroll
  for (int i = 0; i < 9; ++i) { n.ypx.v[i] = w[i]; n.ymx.v[i] = w[9 + i]; n.xy2d.v[i] = w[18 + i]; }
  return n;
}
__device__ __forceinline__ void st_niels(uint32_t* base, uint32_t idx, const ge_niels& n) {
  uint32_t w[28];
#pragma unroll
  for (int i = 0; i < 9; ++i) { w[i] = n.ypx.v[i]; w[9 + i] = n.ymx.v[i]; w[18 + i] = n.xy2d.v[i]; }
  w[27] = 0;
  uint4* q = reinterpret_cast<uint4*>(base + (size_t)idx * NIELS_WORDS);
#pragma unroll
  for (int i = 0; i < 7; ++i) q[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
}

__device__ __forceinline__ ge_p3 ld_ext(const uint32_t* p) {
  ge_p3 r;
  r.X = ld_fe(p); r.Y = ld_fe(p + 9); r.Z = ld_fe(p + 18); r.T = ld_fe(p + 27);
  return r;
}
__device__ __forceinline__ void st_ext(uint32_t* p, const ge_p3& a) {
  st_fe(p, a.X); st_fe(p + 9, a.Y); st_fe(p + 18, a.Z); st_fe(p + 27, a.T);
}

__device__ __forceinline__ void ld_words8(const uint8_t* p, uint32_t w[8]) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  uint4 a = q[0], b = q[1];
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}

// ---- scalar windows (Pippenger) ----
constexpr int WIN_BITS = 16;
constexpr int NWIN_FULL = 16;      // 253-bit coefficients (B, A keys)
constexpr int NWIN_Z = 8;          // 128-bit z (R points), top window unsigned
constexpr int SLICE_BITS = 8;      // 256 buckets per slice (one workgroup)
constexpr int NSLICE = 256;        // slices per window (window 7 needs buckets up to 2^16)
constexpr int NBIN = NWIN_FULL * NSLICE;

// signed radix-2^16 recoding. For z scalars (nwin = 8) the last digit is left unsigned and
// may reach 2^16 (no carry out of bit 128); for 253-bit scalars no carry leaves window 15.
__device__ __forceinline__ int scalar_digit(const uint32_t s[8], int w, int& carry, bool top_unsigned) {
  uint32_t raw = ((s[w >> 1] >> ((w & 1) * 16)) & 0xFFFFu) + (uint32_t)carry;
  if (top_unsigned) { carry = 0; return (int)raw; }
  if (raw >= 0x8000u) { carry = 1; return (int)raw - 0x10000; }
  carry = 0;
  return (int)raw;
}

// 64-bit limb-sum accumulators per distinct key (12 limbs of a 128 x 256-bit product)
constexpr int KEY_ACC_LIMBS = 12;

// flags slot indices (FLAG_WINMASK: bit w set when MSM window w has at least one entry)
enum { FLAG_BAD = 0, FLAG_NKEYS = 1, FLAG_VERDICT = 2, FLAG_WINMASK = 3, FLAG_COUNT = 8 };

// Few-key batches (consensus votes: m validators << n votes). Every full-width coefficient
// (B and each distinct key) is split as c = c_lo + 2^128 c_hi over the points P and
// [2^128]P, so EVERY scalar of the MSM is < 2^128 and only the 8 low windows exist: half the
// bucket reductions and half the Horner doublings. The shifted key points cost 128 doublings
// per key, computed on a side stream under the R decompression; [2^128]B is a context
// constant. Point layout in few-key mode:
//   0 = B, 1..n = R_i, n+1..n+m = A_j, n+m+1..n+2m = [2^128]A_j, n+2m+1 = [2^128]B.
constexpr uint32_t FEW_KEY_MIN_N = 4096;
constexpr int BTAB_BSHIFT = 8;     // context table entry holding [2^128]B
constexpr int BTAB_ENTRIES = 9;
constexpr uint32_t FEW_KEY_RATIO = 16;
__host__ __device__ __forceinline__ bool few_key_mode(uint32_t n, uint32_t m) {
  return n >= FEW_KEY_MIN_N && (uint64_t)m * FEW_KEY_RATIO <= n;
}
__host__ __device__ __forceinline__ uint32_t msm_num_points(uint32_t n, uint32_t m) {
  return few_key_mode(n, m) ? n + 2 * m + 2 : 1 + n + m;
}
// point p of the MSM carries a scalar < 2^128 (8 windows, top digit unsigned)?
__device__ __forceinline__ bool msm_short_scalar(uint32_t p, uint32_t n, bool few) {
  return few || (p >= 1 && p <= n);
}

}  // namespace edc
