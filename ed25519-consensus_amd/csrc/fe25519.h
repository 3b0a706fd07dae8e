// GF(2^255-19) arithmetic for gfx950, radix 2^29 x 9 limbs, products on v_mad_u64_u32.
//
// Why radix 2^29: a 9x9 schoolbook column holds at most 9 products of <=2^60.8 bits, so every
// column accumulates in ONE 64-bit register through a chain of v_mad_u64_u32 (32x32+64 -> 64)
// with no carry instructions at all (the 2^32 radix needs a v_addc per product plus hazard
// nops). Limbs are allowed to run slightly over 29 bits ("lazy" form) and the element is only
// canonicalised when bytes are needed (compress / equality / sign).
//
// Invariants (checked in tests/test_native_math.py against the Python oracle):
//   reduced  : every limb < 2^29 + 2^19          (output of mul / sqr / sub / carry)
//   mul input: every limb < 2^30.41               (reduced, or lazy sum of two reduced)
//   value    : < 2^261; 2^261 == 1216 (mod p) is the top fold constant.
//
// Reference semantics restated (curve25519-dalek-ng 4.1 FieldElement, not vendored):
//   from_bytes masks bit 255 and does NOT reduce; to_bytes is the canonical encoding;
//   is_negative is the low bit of the canonical encoding.
#pragma once
#include <stdint.h>

#ifndef EDC_HD
#if defined(__HIPCC__)
#define EDC_HD __host__ __device__ __forceinline__
#else
#define EDC_HD static inline
#endif
#endif

namespace edc {

constexpr uint32_t M29 = (1u << 29) - 1;

struct fe {
  uint32_t v[9];
};

EDC_HD uint64_t mul64(uint32_t a, uint32_t b) { return (uint64_t)a * b; }

// a * b + c as ONE v_mad_u64_u32 on the device. Spelled as inline asm so that LLVM cannot
// reassociate a chain of them (it would pull the carry addend out into a separate 64-bit add).
EDC_HD uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint64_t d;
  asm("v_mad_u64_u32 %0, vcc, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c) : "vcc");
  return d;
#else
  return (uint64_t)a * b + c;
#endif
}

// One product of a carried column: the chain alternates the asm form (even steps) with LLVM's own
// mul + add (odd steps, which it forms into v_mad_u64_u32 with the running sum as addend). A single
// plain step between two asm statements cannot be reassociated, and it separates the asm
// statements: two back-to-back dependent asm statements cost a hazard wait state (s_nop) on
// gfx950, since the compiler cannot see what the first one was.
EDC_HD void mad_step(uint64_t& acc, int j, uint32_t x, uint32_t y) {
  if (j & 1) acc += mul64(x, y);
  else acc = mad64(x, y, acc);
}

EDC_HD fe fe_zero() { fe r; for (int i = 0; i < 9; ++i) r.v[i] = 0; return r; }
EDC_HD fe fe_one() { fe r = fe_zero(); r.v[0] = 1; return r; }

// 32 little-endian bytes given as 8 LE words; bit 255 is masked (dalek from_bytes).
EDC_HD fe fe_from_words(const uint32_t w[8]) {
  fe r;
  r.v[0] = w[0] & M29;
  r.v[1] = ((w[0] >> 29) | (w[1] << 3)) & M29;
  r.v[2] = ((w[1] >> 26) | (w[2] << 6)) & M29;
  r.v[3] = ((w[2] >> 23) | (w[3] << 9)) & M29;
  r.v[4] = ((w[3] >> 20) | (w[4] << 12)) & M29;
  r.v[5] = ((w[4] >> 17) | (w[5] << 15)) & M29;
  r.v[6] = ((w[5] >> 14) | (w[6] << 18)) & M29;
  r.v[7] = ((w[6] >> 11) | (w[7] << 21)) & M29;
  r.v[8] = (w[7] >> 8) & 0x7FFFFFu;
  return r;
}

// lazy add: both inputs reduced -> output is a valid mul input (NOT a valid add input)
EDC_HD fe fe_add(const fe& a, const fe& b) {
  fe r;
  for (int i = 0; i < 9; ++i) r.v[i] = a.v[i] + b.v[i];
  return r;
}

// one parallel carry round: limbs < 2^32 in -> reduced out
EDC_HD fe fe_carry(const fe& a) {
  fe r;
  uint32_t top = a.v[8] >> 29;
  r.v[0] = (a.v[0] & M29) + top * 1216u;
  for (int i = 1; i < 9; ++i) r.v[i] = (a.v[i] & M29) + (a.v[i - 1] >> 29);
  return r;
}

// carried add: reduced + reduced -> reduced
EDC_HD fe fe_add_c(const fe& a, const fe& b) { return fe_carry(fe_add(a, b)); }

// 16p-free bias K == 0 (mod p) with every limb >= 2^30.41, so a + K - b never underflows a limb:
// K = 4p + 2^263 - 4864 (2^263 == 4*1216 = 4864 mod p).
#define EDC_SUB_K0 (0x80000000u - 76u - 4864u)
#define EDC_SUB_K1 (0x80000000u - 4u)
#define EDC_SUB_K8 (0x80000000u + 0x2000000u - 4u)

// a: mul-input bound (limbs < 2^30.41), b: limbs <= K_i -> reduced output
EDC_HD fe fe_sub(const fe& a, const fe& b) {
  fe t;
  t.v[0] = a.v[0] + EDC_SUB_K0 - b.v[0];
  for (int i = 1; i < 8; ++i) t.v[i] = a.v[i] + EDC_SUB_K1 - b.v[i];
  t.v[8] = a.v[8] + EDC_SUB_K8 - b.v[8];
  return fe_carry(t);
}

EDC_HD fe fe_neg(const fe& a) { return fe_sub(fe_zero(), a); }

// Lazy subtraction, no carry pass: a limbs < 2^30 + 2^20 (reduced, or a lazy sum of two reduced),
// b limbs <= K_i -> limbs < 2^31.61. Such an element is a valid fe_mul operand ONLY against a
// REDUCED partner (limbs < 2^29 + 2^19): a column then holds at most 9 products
// < 2^31.61 * 2^29.002 = 2^60.61, i.e. < 2^63.78 with the fold terms, inside the 64-bit
// accumulator (fe_mul's symmetric bound, 2^30.41 per operand, is the other admissible case).
// Point formulas use it on one side of every product whose other side is carried.
EDC_HD fe fe_sub_lazy(const fe& a, const fe& b) {
  fe t;
  t.v[0] = a.v[0] + EDC_SUB_K0 - b.v[0];
  for (int i = 1; i < 8; ++i) t.v[i] = a.v[i] + EDC_SUB_K1 - b.v[i];
  t.v[8] = a.v[8] + EDC_SUB_K8 - b.v[8];
  return t;
}

// Top-column fold shared by mul and sqr: acc = the carry out of column 8 (< 2^35), i.e. the
// value acc * 2^261 == acc * 1216 still to be added at limb 0.
EDC_HD fe fe_fold_top(fe r, uint64_t top) {
  uint64_t t = (uint64_t)r.v[0] + mul64((uint32_t)top, 1216u) + (mul64((uint32_t)(top >> 32), 1216u) << 32);
  r.v[0] = (uint32_t)t & M29;
  r.v[1] += (uint32_t)(t >> 29);                  // < 2^17 extra
  return r;
}

// Products are accumulated column by column in ONE 64-bit register per column through chains of
// v_mad_u64_u32 (32x32+64). Columns 9..16 (weight 2^(29k) = 2^(29(k-9)) * 2^261, 2^261 == 1216
// mod p) are summed first; low column k then starts from the carry out of column k-1, so the
// carry rides in a mad addend instead of a separate 64-bit add, and it absorbs the fold terms
// lo32(col k+9) * 1216 and hi32(col k+8) * 2^32 * 1216 = hi * 9728 as two more products.
// Column bound: 9 products < 2^60.82 (inputs < 2^30.41) + fold < 2^45.3 + carry < 2^35 < 2^64;
// or one input reduced (< 2^29.002) and the other < 2^31.83 (fe_sub_lazy outputs: < 2^31.61).
EDC_HD fe fe_mul(const fe& a, const fe& b) {
  uint64_t h[8];
#pragma unroll
  for (int k = 9; k < 17; ++k) {
    uint64_t s = 0;
#pragma unroll
    for (int i = k - 8; i <= 8; ++i) s += mul64(a.v[i], b.v[k - i]);
    h[k - 9] = s;
  }
  fe r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    int j = 0;
    if (k < 8) mad_step(acc, j++, (uint32_t)h[k], 1216u);
    if (k >= 1) mad_step(acc, j++, (uint32_t)(h[k - 1] >> 32), 9728u);
#pragma unroll
    for (int i = 0; i <= k; ++i) mad_step(acc, j++, a.v[i], b.v[k - i]);
    r.v[k] = (uint32_t)acc & M29;
    acc >>= 29;
  }
  return fe_fold_top(r, acc);
}

EDC_HD fe fe_sqr(const fe& a) {
  uint32_t d[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) d[i] = a.v[i] << 1;
  uint64_t h[8];
#pragma unroll
  for (int k = 9; k < 17; ++k) {
    uint64_t s = 0;
#pragma unroll
    for (int i = k - 8; 2 * i < k; ++i) s += mul64(a.v[i], d[k - i]);
    if ((k & 1) == 0) s += mul64(a.v[k / 2], a.v[k / 2]);
    h[k - 9] = s;
  }
  fe r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    int j = 0;
    if (k < 8) mad_step(acc, j++, (uint32_t)h[k], 1216u);
    if (k >= 1) mad_step(acc, j++, (uint32_t)(h[k - 1] >> 32), 9728u);
#pragma unroll
    for (int i = 0; 2 * i < k; ++i) mad_step(acc, j++, a.v[i], d[k - i]);
    if ((k & 1) == 0) mad_step(acc, j++, a.v[k / 2], a.v[k / 2]);
    r.v[k] = (uint32_t)acc & M29;
    acc >>= 29;
  }
  return fe_fold_top(r, acc);
}

EDC_HD fe fe_sqr_n(fe a, int n) {
  for (int i = 0; i < n; ++i) a = fe_sqr(a);
  return a;
}

// multiply by a small constant (< 2^13)
EDC_HD fe fe_mul_small(const fe& a, uint32_t c) {
  fe r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    acc += mul64(a.v[k], c);
    r.v[k] = (uint32_t)acc & M29;
    acc >>= 29;
  }
  return fe_fold_top(r, acc);
}

// canonical value (< p) as 9 limbs with limb 8 < 2^23
EDC_HD fe fe_canon(const fe& a) {
  fe r;
  uint32_t c = 0;
  // full serial carry
  for (int i = 0; i < 8; ++i) {
    uint32_t t = a.v[i] + c;                       // a.v[i] < 2^30.41, c < 2^4 -> no overflow
    r.v[i] = t & M29;
    c = t >> 29;
  }
  uint32_t t8 = a.v[8] + c;
  // value = sum + t8 * 2^232; fold bits >= 255 with 2^255 == 19
  uint32_t q = t8 >> 23;
  r.v[8] = t8 & 0x7FFFFFu;
  uint32_t add = q * 19u;
  for (int pass = 0; pass < 2; ++pass) {
    c = add;
    for (int i = 0; i < 8; ++i) {
      uint32_t t = r.v[i] + c;
      r.v[i] = t & M29;
      c = t >> 29;
    }
    t8 = r.v[8] + c;
    q = t8 >> 23;
    r.v[8] = t8 & 0x7FFFFFu;
    add = q * 19u;
  }
  // now value < 2^255; subtract p if value >= p  <=>  value + 19 >= 2^255
  fe s;
  c = 19;
  for (int i = 0; i < 8; ++i) {
    uint32_t t = r.v[i] + c;
    s.v[i] = t & M29;
    c = t >> 29;
  }
  uint32_t s8 = r.v[8] + c;
  uint32_t ge = s8 >> 23;                          // 1 iff value >= p
  s.v[8] = s8 & 0x7FFFFFu;
  uint32_t mask = 0u - ge;
  for (int i = 0; i < 9; ++i) r.v[i] = (s.v[i] & mask) | (r.v[i] & ~mask);
  return r;
}

// canonical 32-byte encoding as 8 LE words
EDC_HD void fe_to_words(const fe& a, uint32_t w[8]) {
  fe c = fe_canon(a);
  w[0] = c.v[0] | (c.v[1] << 29);
  w[1] = (c.v[1] >> 3) | (c.v[2] << 26);
  w[2] = (c.v[2] >> 6) | (c.v[3] << 23);
  w[3] = (c.v[3] >> 9) | (c.v[4] << 20);
  w[4] = (c.v[4] >> 12) | (c.v[5] << 17);
  w[5] = (c.v[5] >> 15) | (c.v[6] << 14);
  w[6] = (c.v[6] >> 18) | (c.v[7] << 11);
  w[7] = (c.v[7] >> 21) | (c.v[8] << 8);
}

EDC_HD bool fe_is_negative(const fe& a) { return fe_canon(a).v[0] & 1u; }

// a == 0 (mod p) without the full canonical form: one serial carry, one fold of the bits >= 255
// (2^255 == 19) and a second carry give a value V < 2^255 + 2^13 < 2p in 29-bit limbs, so
// a == 0 iff V is 0 or p.
EDC_HD bool fe_is_zero(const fe& a) {
  uint32_t r[9], c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t t = a.v[i] + c;                 // a.v[i] < 2^30.41, c < 2^4
    r[i] = t & M29;
    c = t >> 29;
  }
  uint32_t t8 = a.v[8] + c;
  c = (t8 >> 23) * 19u;
  r[8] = t8 & 0x7FFFFFu;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t t = r[i] + c;
    r[i] = t & M29;
    c = t >> 29;
  }
  r[8] += c;
  uint32_t z = 0, q = (r[0] ^ (M29 - 18u)) | (r[8] ^ 0x7FFFFFu);
#pragma unroll
  for (int i = 0; i < 9; ++i) z |= r[i];
#pragma unroll
  for (int i = 1; i < 8; ++i) q |= r[i] ^ M29;
  return z == 0 || q == 0;
}

EDC_HD bool fe_eq(const fe& a, const fe& b) {
  fe x = fe_canon(a), y = fe_canon(b);
  uint32_t o = 0;
  for (int i = 0; i < 9; ++i) o |= x.v[i] ^ y.v[i];
  return o == 0;
}

EDC_HD fe fe_select(const fe& a, const fe& b, bool pick_b) {
  uint32_t m = 0u - (uint32_t)pick_b;
  fe r;
  for (int i = 0; i < 9; ++i) r.v[i] = (b.v[i] & m) | (a.v[i] & ~m);
  return r;
}

// z^(2^250 - 1) and z^11 (shared prefix of the inversion and (p-5)/8 chains)
EDC_HD void fe_pow22501(const fe& z, fe& t19, fe& t3) {
  fe t0 = fe_sqr(z);                 // 2
  fe t1 = fe_sqr_n(t0, 2);           // 8
  t1 = fe_mul(z, t1);                // 9
  t0 = fe_mul(t0, t1);               // 11
  t3 = t0;
  fe t2 = fe_sqr(t0);                // 22
  t1 = fe_mul(t1, t2);               // 2^5 - 1
  t2 = fe_sqr_n(t1, 5);
  t1 = fe_mul(t2, t1);               // 2^10 - 1
  t2 = fe_sqr_n(t1, 10);
  t2 = fe_mul(t2, t1);               // 2^20 - 1
  fe t4 = fe_sqr_n(t2, 20);
  t2 = fe_mul(t4, t2);               // 2^40 - 1
  t2 = fe_sqr_n(t2, 10);
  t1 = fe_mul(t2, t1);               // 2^50 - 1
  t2 = fe_sqr_n(t1, 50);
  t2 = fe_mul(t2, t1);               // 2^100 - 1
  t4 = fe_sqr_n(t2, 100);
  t2 = fe_mul(t4, t2);               // 2^200 - 1
  t2 = fe_sqr_n(t2, 50);
  t19 = fe_mul(t2, t1);              // 2^250 - 1
}

// z^((p-5)/8) = z^(2^252 - 3)
EDC_HD fe fe_pow_p58(const fe& z) {
  fe t19, t3;
  fe_pow22501(z, t19, t3);
  fe t = fe_sqr_n(t19, 2);
  return fe_mul(t, z);
}

// z^(p-2) = z^(2^255 - 21)
EDC_HD fe fe_invert(const fe& z) {
  fe t19, t3;
  fe_pow22501(z, t19, t3);
  fe t = fe_sqr_n(t19, 5);
  return fe_mul(t, t3);
}

// ---- constants (radix 2^29 limbs, canonical) ----
EDC_HD fe fe_const(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t w4,
                   uint32_t w5, uint32_t w6, uint32_t w7) {
  uint32_t w[8] = {w0, w1, w2, w3, w4, w5, w6, w7};
  return fe_from_words(w);
}
// d = -121665/121666
EDC_HD fe fe_d() {
  return fe_const(0x135978a3u, 0x75eb4dcau, 0x4141d8abu, 0x00700a4du, 0x7779e898u, 0x8cc74079u,
                  0x2b6ffe73u, 0x52036ceeu);
}
// 2d
EDC_HD fe fe_d2() {
  return fe_const(0x26b2f159u, 0xebd69b94u, 0x8283b156u, 0x00e0149au, 0xeef3d130u, 0x198e80f2u,
                  0x56dffce7u, 0x2406d9dcu);
}
// sqrt(-1)
EDC_HD fe fe_sqrtm1() {
  return fe_const(0x4a0ea0b0u, 0xc4ee1b27u, 0xad2fe478u, 0x2f431806u, 0x3dfbd7a7u, 0x2b4d0099u,
                  0x4fc1df0bu, 0x2b832480u);
}

}  // namespace edc
