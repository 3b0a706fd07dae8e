// Scalars mod l = 2^252 + 27742317777372353535851937790883648493, 8 x 32-bit LE limbs.
// Restates curve25519-dalek-ng 4.1 Scalar (not vendored; reference call sites):
//   Scalar::from_hash            -> sc_reduce_wide    (src/batch.rs:86-91)
//   Scalar::from_canonical_bytes -> sc_is_canonical   (src/batch.rs:193, verification_key.rs:240)
//   z * s, z * k, +=, -=          -> sc_mul / sc_add / sc_sub (src/batch.rs:195-198)
// Wide reduction by folding 2^252 == -(l - 2^252) in signed radix 2^29 (sc_reduce_wide); the
// word-radix Barrett form (HAC 14.42, b = 2^32) stays as a second opinion for the host tests. Every
// loop is fully unrolled: a runtime index into a limb array lowers to s_set_gpr_idx indexing.
#pragma once
#include <stdint.h>
#include "fe25519.h"  // EDC_HD

namespace edc {

struct sc { uint32_t v[8]; };

EDC_HD sc sc_l() {
  sc r;
  const uint32_t L[8] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu,
                         0u, 0u, 0u, 0x10000000u};
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = L[i];
  return r;
}

EDC_HD void sc_mu(uint32_t m[9]) {
  const uint32_t MU[9] = {0x0a2c131bu, 0xed9ce5a3u, 0x086329a7u, 0x2106215du,
                          0xffffffebu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xfu};
#pragma unroll
  for (int i = 0; i < 9; ++i) m[i] = MU[i];
}

EDC_HD sc sc_zero() { sc r; for (int i = 0; i < 8; ++i) r.v[i] = 0; return r; }

// a >= b (8 limbs)
EDC_HD bool sc_geq(const uint32_t* a, const uint32_t* b, int n) {
#pragma unroll
  for (int i = n - 1; i >= 0; --i) {
    if (a[i] != b[i]) return a[i] > b[i];
  }
  return true;
}

// r = a - b over n limbs, returns borrow
EDC_HD uint32_t mp_sub(uint32_t* r, const uint32_t* a, const uint32_t* b, int n) {
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < n; ++i) {
    uint64_t t = (uint64_t)a[i] - b[i] - br;
    r[i] = (uint32_t)t;
    br = (t >> 63) & 1;
  }
  return (uint32_t)br;
}

// Scalar::from_canonical_bytes accepts iff the 256-bit LE integer is < l.
EDC_HD bool sc_is_canonical(const uint32_t s[8]) {
  sc L = sc_l();
  return !sc_geq(s, L.v, 8);
}

// ---- x mod l by folding 2^252 == -c (mod l), c = l - 2^252 < 2^125, in signed radix 2^29 ----
// Columns accumulate in one signed 64-bit register through v_mad_i64_i32 (|product| < 2^58, at
// most 5 per column), so there are no 32-bit carry chains and no register-pair shuffling (the
// word-radix Barrett below spends two thirds of its instructions on moves). Three folds bring a
// 512-bit x into (-2^131, 2^252); adding l when negative finishes (2^252 < l).
//   fold 1: x = H1 2^252 + L1, 0 <= H1 < 2^260     -> y = L1 - H1 c in (-2^385, 2^252)
//   fold 2: y = H2 2^252 + L2, -2^133 <= H2 <= 0   -> z = L2 - H2 c in [0, 2^258)
//   fold 3: z = H3 2^252 + L3, 0 <= H3 < 2^6       -> r = L3 - H3 c in (-2^131, 2^252)
// c's radix-2^29 limbs (c = 0x14def9dea2f79cd65812631a5cf5d3ed)
#define EDC_SC_C0 0x1cf5d3edu
#define EDC_SC_C1 0x009318d2u
#define EDC_SC_C2 0x1de73596u
#define EDC_SC_C3 0x1df3bd45u
#define EDC_SC_C4 0x0000014du

EDC_HD int64_t smad64(int32_t a, int32_t b, int64_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  int64_t d;
  asm("v_mad_i64_i32 %0, vcc, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c) : "vcc");
  return d;
#else
  return (int64_t)a * b + c;
#endif
}

// bits [b, b + 29) of a 512-bit LE word array (b + 29 <= 512 or the missing bits read as 0)
EDC_HD uint32_t sc_bits29(const uint32_t x[16], int b) {
  const int w = b >> 5, s = b & 31;
  const uint32_t hi = w + 1 < 16 ? x[w + 1] : 0u;
#if defined(__HIP_DEVICE_COMPILE__)
  // one v_alignbit_b32 on the two words (a 64-bit shift of the pair lowers to an unaligned 8-byte
  // load of the array from scratch)
  return __builtin_amdgcn_alignbit(hi, x[w], s) & ((1u << 29) - 1u);
#else
  return (uint32_t)((((uint64_t)hi << 32) | x[w]) >> s) & ((1u << 29) - 1u);
#endif
}

// One column pass: acc_k = lo[k] + carry - sum_{i+j=k} h[i] c[j]; out[k] = acc_k mod 2^29, carry
// = acc_k >> 29 (arithmetic). nh limbs of h, nlo limbs of lo, ncol columns; returns the carry out.
template <int NH, int NLO, int NCOL>
EDC_HD int64_t sc_fold_cols(const int32_t h[NH], const int32_t lo[NLO], int32_t out[NCOL]) {
  const int32_t nc[5] = {-(int32_t)EDC_SC_C0, -(int32_t)EDC_SC_C1, -(int32_t)EDC_SC_C2, -(int32_t)EDC_SC_C3,
                         -(int32_t)EDC_SC_C4};
  int64_t acc = 0;
#pragma unroll
  for (int k = 0; k < NCOL; ++k) {
    if (k < NLO) acc = smad64(lo[k], 1, acc);
#pragma unroll
    for (int i = 0; i < NH; ++i)
      if (k - i >= 0 && k - i < 5) acc = smad64(h[i], nc[k - i], acc);
    out[k] = (int32_t)((uint32_t)acc & ((1u << 29) - 1u));
    acc >>= 29;
  }
  return acc;
}

// x: 16 limbs (512-bit LE) -> x mod l
EDC_HD sc sc_reduce_wide(const uint32_t x[16]) {
  constexpr uint32_t M = (1u << 29) - 1u, M20 = (1u << 20) - 1u;
  int32_t lo[9], h1[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    lo[k] = (int32_t)(k < 8 ? sc_bits29(x, 29 * k) : sc_bits29(x, 232) & M20);
    h1[k] = (int32_t)sc_bits29(x, 252 + 29 * k);
  }
  // fold 1: 13 columns, limb 13 = the carry out
  int32_t y[13];
  const int64_t y13 = sc_fold_cols<9, 9, 13>(h1, lo, y);
  // fold 2: H2 = y >> 252 as 5 limbs (the top one signed), L2 = y mod 2^252
  int32_t h2[5];
#pragma unroll
  for (int k = 0; k < 4; ++k) h2[k] = (int32_t)((((uint32_t)y[8 + k] >> 20) | ((uint32_t)y[9 + k] << 9)) & M);
  h2[4] = (int32_t)((uint32_t)y[12] >> 20) + (int32_t)y13 * 512;
  y[8] &= (int32_t)M20;
  int32_t z[9];
  const int64_t z9 = sc_fold_cols<5, 9, 9>(h2, y, z);
  // fold 3: H3 = z >> 252 (small, signed)
  int32_t h3[1] = {(int32_t)((uint32_t)z[8] >> 20) + (int32_t)z9 * 512};
  z[8] &= (int32_t)M20;
  int32_t r[9];
  const int64_t r9 = sc_fold_cols<1, 9, 9>(h3, z, r);
  // r = r[0..7] + top 2^232 with top = r[8] + r9 2^29 in [-1, 2^20): add l = c + 2^20 2^232 if
  // negative (the sum is then in [0, l))
  const int32_t top = r[8] + (int32_t)r9 * (1 << 29);
  const bool neg = top < 0;
  const int32_t lv[5] = {(int32_t)EDC_SC_C0, (int32_t)EDC_SC_C1, (int32_t)EDC_SC_C2, (int32_t)EDC_SC_C3,
                         (int32_t)EDC_SC_C4};
  uint32_t f[9];
  int64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    acc = smad64(r[k], 1, acc);
    if (k < 5) acc = smad64(lv[k], (int32_t)neg, acc);
    f[k] = (uint32_t)acc & M;
    acc >>= 29;
  }
  f[8] = (uint32_t)((int32_t)acc + top + (neg ? (1 << 20) : 0));
  sc out;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int b = 32 * j, k = b / 29, s = b % 29;      // word j = limbs k, k+1 (and k+2) shifted
    uint32_t w = f[k] >> s;
    if (k + 1 < 9) w |= f[k + 1] << (29 - s);
    if (29 - s + 29 < 32 && k + 2 < 9) w |= f[k + 2] << (58 - s);
    out.v[j] = w;
  }
  return out;
}

// The word-radix Barrett form (kept as the host tests' second opinion)
EDC_HD sc sc_reduce_wide_barrett(const uint32_t x[16]) {
  uint32_t mu[9];
  sc_mu(mu);
  // q1 = x >> 224 : limbs 7..15 (9 limbs)
  const uint32_t* q1 = x + 7;
  // q3 = (q1 * mu) >> 288 : we need product limbs 9..17
  uint32_t q2[18];
#pragma unroll
  for (int i = 0; i < 18; ++i) q2[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      uint64_t t = (uint64_t)q1[i] * mu[j] + q2[i + j] + carry;
      q2[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    q2[i + 9] = (uint32_t)carry;
  }
  const uint32_t* q3 = q2 + 9;  // 9 limbs
  // r2 = (q3 * l) mod b^9
  sc L = sc_l();
  uint32_t r2[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) r2[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    uint64_t carry = 0;
    int j = 0;
#pragma unroll
    for (; j + i < 9 && j < 8; ++j) {
      uint64_t t = (uint64_t)q3[i] * L.v[j] + r2[i + j] + carry;
      r2[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    if (i + j < 9) r2[i + j] = (uint32_t)carry;  // only i == 0 lands here (position 8)
  }
  uint32_t r[9];
  mp_sub(r, x, r2, 9);  // mod b^9 (borrow discarded)
  uint32_t L9[9];
#pragma unroll
  for (int i = 0; i < 8; ++i) L9[i] = L.v[i];
  L9[8] = 0;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    uint32_t t[9];
    uint32_t br = mp_sub(t, r, L9, 9);
#pragma unroll
    for (int i = 0; i < 9; ++i) r[i] = br ? r[i] : t[i];
  }
  sc out;
#pragma unroll
  for (int i = 0; i < 8; ++i) out.v[i] = r[i];
  return out;
}

// Scalar::from_hash: 64-byte digest as a 512-bit LE integer mod l
EDC_HD sc sc_from_digest(const uint8_t d[64]) {
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i)
    x[i] = (uint32_t)d[4 * i] | ((uint32_t)d[4 * i + 1] << 8) | ((uint32_t)d[4 * i + 2] << 16) |
           ((uint32_t)d[4 * i + 3] << 24);
  return sc_reduce_wide(x);
}

// a * b mod l for a, b < 2^256
EDC_HD sc sc_mul(const sc& a, const sc& b) {
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint64_t t = (uint64_t)a.v[i] * b.v[j] + x[i + j] + carry;
      x[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    x[i + 8] = (uint32_t)carry;
  }
  return sc_reduce_wide(x);
}

// (a < 2^128 as 4 limbs) * b mod l
EDC_HD sc sc_mul128(const uint32_t a[4], const sc& b) {
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint64_t t = (uint64_t)a[i] * b.v[j] + x[i + j] + carry;
      x[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    x[i + 8] = (uint32_t)carry;
  }
  return sc_reduce_wide(x);
}

// a + b mod l for a, b < l
EDC_HD sc sc_add(const sc& a, const sc& b) {
  uint32_t t[9];
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c += (uint64_t)a.v[i] + b.v[i];
    t[i] = (uint32_t)c;
    c >>= 32;
  }
  t[8] = (uint32_t)c;
  sc L = sc_l();
  uint32_t L9[9];
#pragma unroll
  for (int i = 0; i < 8; ++i) L9[i] = L.v[i];
  L9[8] = 0;
  uint32_t u[9];
  uint32_t br = mp_sub(u, t, L9, 9);
  sc r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = br ? t[i] : u[i];
  return r;
}

// a - b mod l for a, b < l
EDC_HD sc sc_sub(const sc& a, const sc& b) {
  uint32_t t[8];
  uint32_t br = mp_sub(t, a.v, b.v, 8);
  sc r;
  if (br) {
    sc L = sc_l();
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      c += (uint64_t)t[i] + L.v[i];
      r.v[i] = (uint32_t)c;
      c >>= 32;
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = t[i];
  }
  return r;
}

}  // namespace edc
