// Scalars mod l = 2^252 + 27742317777372353535851937790883648493, 8 x 32-bit LE limbs.
// Restates curve25519-dalek-ng 4.1 Scalar (not vendored; reference call sites):
//   Scalar::from_hash            -> sc_reduce_wide    (src/batch.rs:86-91)
//   Scalar::from_canonical_bytes -> sc_is_canonical   (src/batch.rs:193, verification_key.rs:240)
//   z * s, z * k, +=, -=          -> sc_mul / sc_add / sc_sub (src/batch.rs:195-198)
// Barrett reduction (HAC 14.42, b = 2^32, k = 8) with mu = floor(2^512 / l). Every loop is
// fully unrolled: a runtime index into a limb array lowers to s_set_gpr_idx register indexing.
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

// x: 16 limbs (512-bit LE) -> x mod l
EDC_HD sc sc_reduce_wide(const uint32_t x[16]) {
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
