// Limb-sliced ("row") point arithmetic for the serial chains of the MSM tail (Horner pass, window
// combines). One wave holds ONE point: row q of the wave (lanes 16q..16q+15) holds coordinate q
// (0: X, 1: Y, 2: Z, 3: T) and lane j < 9 of a row holds limb j of it (radix 2^29, the limbs of
// fe25519.h); lanes 9..15 of every row hold 0. A field multiplication then costs every lane 9
// v_mad_u64_u32 (lane k sums the product column k) instead of the 99 of a whole product on one
// lane: operands reach the lanes by DPP (row_newbcast:i broadcasts a_i, row_shr:i shifts b), the
// four rows exchange coordinates with v_permlane16/32_swap, and the carries are two parallel
// rounds with DPP shifts. A lone wave issues about one VALU instruction per 5.5 cycles whether
// or not it depends on the previous one (profiles/r02_lat_probe.txt), so the serial chain's time
// is its instruction count: a doubling is ~160 instructions here against ~420 in the quad layout
// of ge_quad.h.
//
// The formulas are those of quad_dbl_d / quad_add_d (ge_quad.h), so every coordinate is the same
// field element as in the quad layout (canonical bytes unchanged). Bounds are fe25519.h's: the
// multiplication takes limbs < 2^30.41 and returns reduced limbs (< 2^29 + 2^19).
#pragma once
#include <hip/hip_runtime.h>
#include "fe25519.h"

namespace edc {

// lane geometry of the row layout
__device__ __forceinline__ uint32_t row_limb() { return threadIdx.x & 15u; }
__device__ __forceinline__ uint32_t row_id() { return (threadIdx.x >> 4) & 3u; }

// DPP moves inside a 16-lane row; lanes whose source lies outside the row read 0 (bound_ctrl)
template <int CTRL>
__device__ __forceinline__ uint32_t row_dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
template <int N> __device__ __forceinline__ uint32_t row_shr(uint32_t v) { return row_dpp<0x110 + N>(v); }   // lane j <- j-N
template <int N> __device__ __forceinline__ uint32_t row_shl(uint32_t v) { return row_dpp<0x100 + N>(v); }   // lane j <- j+N
template <int N> __device__ __forceinline__ uint32_t row_bc(uint32_t v) { return row_dpp<0x150 + N>(v); }    // lane j <- N

// the four rows of v as four values replicated over every row (3 permlane swaps):
// r0 = row 0 everywhere, ..., r3 = row 3 everywhere
__device__ __forceinline__ void row_spread4(uint32_t v, uint32_t& r0, uint32_t& r1, uint32_t& r2, uint32_t& r3) {
  const auto h = __builtin_amdgcn_permlane32_swap(v, v, false, false);   // [v0 v1 v0 v1], [v2 v3 v2 v3]
  const auto a = __builtin_amdgcn_permlane16_swap(h[0], h[0], false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(h[1], h[1], false, false);
  r0 = a[0]; r1 = a[1]; r2 = b[0]; r3 = b[1];
}
// rows 0 and 1 of v replicated over every row (2 swaps)
__device__ __forceinline__ void row_spread01(uint32_t v, uint32_t& r0, uint32_t& r1) {
  const auto h = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  const auto a = __builtin_amdgcn_permlane16_swap(h[0], h[0], false, false);
  r0 = a[0]; r1 = a[1];
}

// per-lane constants of one row layout, computed once per kernel
struct RowCtx {
  uint32_t j;        // limb index (lane & 15)
  uint32_t subk;     // fe_sub bias limb (EDC_SUB_K*), 0 on the padding lanes
  bool live;         // j < 9
  bool l0, l1, l7, l8;
};

__device__ __forceinline__ RowCtx row_ctx() {
  RowCtx c;
  c.j = row_limb();
  c.live = c.j < 9;
  c.l0 = c.j == 0; c.l1 = c.j == 1; c.l7 = c.j == 7; c.l8 = c.j == 8;
  c.subk = c.j == 0 ? EDC_SUB_K0 : (c.j == 8 ? EDC_SUB_K8 : (c.live ? EDC_SUB_K1 : 0u));
  return c;
}

// one parallel carry round (fe_carry): limbs < 2^32 in, reduced out
__device__ __forceinline__ uint32_t rf_carry(const RowCtx& c, uint32_t t) {
  const uint32_t sh = t >> 29;
  uint32_t r = (t & M29) + row_shr<1>(sh);       // lane 0 reads 0
  const uint32_t top = row_shl<8>(sh);            // lane 0 <- carry out of limb 8
  r += (c.l0 ? top : 0u) * 1216u;
  return c.live ? r : 0u;
}

__device__ __forceinline__ uint32_t rf_add(uint32_t a, uint32_t b) { return a + b; }   // lazy (fe_add)
__device__ __forceinline__ uint32_t rf_add_c(const RowCtx& c, uint32_t a, uint32_t b) { return rf_carry(c, a + b); }
__device__ __forceinline__ uint32_t rf_sub(const RowCtx& c, uint32_t a, uint32_t b) {   // fe_sub
  return rf_carry(c, a + c.subk - b);
}

// a * b: lane k (0..15) accumulates product column k = sum_i a_i b_(k-i) in one 64-bit register
// (b's padding lanes and the row bound supply the zeros); column 16 = a_8 b_8 on every lane.
// Columns 9..16 fold into 0..8 as in fe_mul: column k takes lo32(col k+9) * 1216 and
// hi32(col k+8) * 9728. Then the 64-bit columns (< 2^64) are cut in 29-bit pieces p0 + p1 2^29 +
// p2 2^58, limb k = p0_k + p1_(k-1) + p2_(k-2) (wrapping pieces times 1216), and one carry round.
__device__ __forceinline__ uint32_t rf_mul(const RowCtx& c, uint32_t a, uint32_t b) {
  const uint32_t a8 = row_bc<8>(a);
  uint64_t acc = mad64(row_bc<0>(a), b, 0);
  acc = mad64(row_bc<1>(a), row_shr<1>(b), acc);
  acc = mad64(row_bc<2>(a), row_shr<2>(b), acc);
  acc = mad64(row_bc<3>(a), row_shr<3>(b), acc);
  acc = mad64(row_bc<4>(a), row_shr<4>(b), acc);
  acc = mad64(row_bc<5>(a), row_shr<5>(b), acc);
  acc = mad64(row_bc<6>(a), row_shr<6>(b), acc);
  acc = mad64(row_bc<7>(a), row_shr<7>(b), acc);
  acc = mad64(a8, row_shr<8>(b), acc);
  const uint64_t c16 = mad64(a8, row_bc<8>(b), 0);
  // fold columns 9..16
  uint32_t x = row_shl<9>((uint32_t)acc);          // lo32(col k+9); lanes 7.. read 0
  uint32_t y = row_shl<8>((uint32_t)(acc >> 32));  // hi32(col k+8)
  x = c.l7 ? (uint32_t)c16 : x;
  y = c.l8 ? (uint32_t)(c16 >> 32) : (c.l0 ? 0u : y);
  acc = mad64(x, 1216u, acc);
  acc = mad64(y, 9728u, acc);
  // columns (< 2^64) -> limbs
  const uint32_t lo = (uint32_t)acc, hi = (uint32_t)(acc >> 32);
  const uint32_t p0 = lo & M29;
  const uint32_t p1 = __builtin_amdgcn_alignbit(hi, lo, 29) & M29;
  const uint32_t p2 = hi >> 26;
  // pieces past limb 8 wrap to limbs 0 / 1 times 1216: lane 0 takes p1_8 + p2_7, lane 1 p2_8
  const uint32_t w1 = row_shl<8>(p1), w2 = row_shl<7>(p2);
  const uint32_t u = (c.l0 ? w1 : 0u) + (c.j <= 1 ? w2 : 0u);
  const uint64_t q = mad64(u, 1216u, 0);           // < 2^39.3 on lane 0, < 2^16.3 on lane 1, else 0
  const uint32_t qlo = (uint32_t)q;
  const uint32_t qsh = __builtin_amdgcn_alignbit((uint32_t)(q >> 32), qlo, 29);   // q >> 29
  uint32_t t = p0 + row_shr<1>(p1) + row_shr<2>(p2) + (c.l0 ? (qlo & M29) : qlo) + row_shr<1>(qsh);
  t = c.live ? t : 0u;                             // < 2^30.01
  return rf_carry(c, t);
}

__device__ __forceinline__ uint32_t rf_sqr(const RowCtx& c, uint32_t a) { return rf_mul(c, a, a); }

// ---- points: row q = coordinate q ----
// load an extended point stored as X | Y | Z | T (36 words, ge_p3 / EXT_WORDS layout)
__device__ __forceinline__ uint32_t row_ld_ext(const RowCtx& c, const uint32_t* p) {
  return c.live ? p[9 * row_id() + c.j] : 0u;
}
__device__ __forceinline__ void row_st_ext(const RowCtx& c, uint32_t* p, uint32_t v) {
  if (c.live) p[9 * row_id() + c.j] = v;
}

// limbs of 2d on the live lanes (fe_d2)
__device__ __forceinline__ uint32_t row_d2(const RowCtx& c) {
  const fe d = fe_d2();
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) r = c.j == (uint32_t)i ? d.v[i] : r;
  return r;
}

// second operand of an addition of Q (extended, at p): (Y - X, Y + X carried, Z, 2d T), the
// projective Niels form of quad_add_d's first round; d2 = row_d2(c)
__device__ __forceinline__ uint32_t row_cached(const RowCtx& c, const uint32_t* p, uint32_t d2) {
  const uint32_t q = row_id();
  const uint32_t y = c.live ? p[(q <= 1 ? 9 : 9 * q) + c.j] : 0u;
  const uint32_t x = c.live ? p[c.j] : 0u;
  const uint32_t s = rf_sub(c, y, x), a = rf_add_c(c, y, x);
  const uint32_t t = rf_mul(c, y, d2);
  return q == 0 ? s : (q == 1 ? a : (q == 2 ? y : t));
}

// 2P (quad_dbl_d's formulas): squares of X, Y, Z, X+Y, then X3 = Xc Tc, Y3 = Yc Zc, Z3 = Zc Tc,
// T3 = Xc Yc
__device__ __forceinline__ uint32_t row_dbl(const RowCtx& c, uint32_t p) {
  const uint32_t q = row_id();
  uint32_t X, Y;
  row_spread01(p, X, Y);
  const uint32_t s = rf_sqr(c, q == 3 ? rf_add(X, Y) : p);
  uint32_t XX, YY, ZZ, U;
  row_spread4(s, XX, YY, ZZ, U);
  const bool mid = q == 1 || q == 2, odd = (q & 1) != 0;
  const uint32_t a = rf_sub(c, mid ? YY : U, mid ? XX : rf_add(YY, XX));
  const uint32_t b = rf_add(XX, odd ? YY : rf_sub(c, rf_add(ZZ, ZZ), YY));
  return rf_mul(c, a, b);
}

// P + Q with Q's second-operand form bq = row_cached(...) (quad_add_d's formulas)
__device__ __forceinline__ uint32_t row_add(const RowCtx& c, uint32_t p, uint32_t bq) {
  const uint32_t q = row_id();
  uint32_t X, Y;
  row_spread01(p, X, Y);
  const uint32_t a = q == 0 ? rf_sub(c, Y, X) : (q == 1 ? rf_add(Y, X) : p);
  const uint32_t m = rf_mul(c, a, bq);
  uint32_t A, B, ZZ, C;
  row_spread4(m, A, B, ZZ, C);
  const uint32_t D = rf_add_c(c, ZZ, ZZ);
  const bool mid = q == 1 || q == 2, odd = (q & 1) != 0;
  const uint32_t a2 = mid ? rf_add(D, C) : rf_sub(c, B, A);
  const uint32_t b2 = odd ? rf_add(B, A) : rf_sub(c, D, C);
  return rf_mul(c, a2, b2);
}

}  // namespace edc
