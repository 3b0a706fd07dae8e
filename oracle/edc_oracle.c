/*
 * CPU ORACLE / BASELINE (TEST INFRASTRUCTURE ONLY): plain-C restatement of the verification
 * path of ed25519-consensus 2.1.0 following the published algorithms of its arithmetic crate
 * curve25519-dalek-ng ^4.1, u64_backend (NOT vendored under /root/reference; Cargo.toml:18):
 *   - FieldElement51: 5 x 51-bit limbs, u128 products, lazy adds, to_bytes canonical;
 *   - CompressedEdwardsY::decompress via sqrt_ratio_i (ZIP215: y not reduce-checked, sign bit on
 *     x = 0 accepted);
 *   - vartime_multiscalar_mul: Straus with width-5 NAF tables below 190 terms, Pippenger with
 *     signed radix-2^w digits (w = 6 / 7 / 8 for < 500 / < 800 / larger) above;
 *   - vartime_double_scalar_mul_basepoint: width-5 NAF for A, width-8 NAF with an odd-multiples
 *     table for B;
 *   - Scalar: from_hash (wide reduction), from_canonical_bytes (s < l), mod-l products.
 * The verification logic restates reference src/batch.rs:82-217 (queue: k = H(R||A||M),
 * HashMap by raw key bytes; verify: decode, z, coalesced MSM, [8]check == 0) and
 * src/verification_key.rs:160-258 (try_from / verify_prehashed, error order).
 * z_j = ChaCha20Rng(seed) keystream bytes [16j, 16j+16) in QUEUE order.
 *
 * Used by tests/ (parity checker at sizes the Python oracle cannot reach) and by bench.py's
 * cpu_baseline leg (kind "port"). Never linked into the product library.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef unsigned __int128 u128;

/* ============================================================ field: 5 x 51 bits */
typedef struct { uint64_t v[5]; } fe;
#define M51 ((1ULL << 51) - 1)

static inline uint64_t ld64(const uint8_t* p) {
  uint64_t r = 0;
  for (int i = 7; i >= 0; --i) r = (r << 8) | p[i];
  return r;
}

static fe fe_frombytes(const uint8_t s[32]) { /* masks bit 255, no reduction */
  uint64_t w0 = ld64(s), w1 = ld64(s + 8), w2 = ld64(s + 16), w3 = ld64(s + 24);
  fe h;
  h.v[0] = w0 & M51;
  h.v[1] = ((w0 >> 51) | (w1 << 13)) & M51;
  h.v[2] = ((w1 >> 38) | (w2 << 26)) & M51;
  h.v[3] = ((w2 >> 25) | (w3 << 39)) & M51;
  h.v[4] = (w3 >> 12) & M51;
  return h;
}

static inline fe fe_weak(fe a) { /* carry: limbs < 2^51 + 2^13ish */
  uint64_t c;
  c = a.v[0] >> 51; a.v[0] &= M51; a.v[1] += c;
  c = a.v[1] >> 51; a.v[1] &= M51; a.v[2] += c;
  c = a.v[2] >> 51; a.v[2] &= M51; a.v[3] += c;
  c = a.v[3] >> 51; a.v[3] &= M51; a.v[4] += c;
  c = a.v[4] >> 51; a.v[4] &= M51; a.v[0] += c * 19;
  return a;
}

static void fe_tobytes(uint8_t s[32], fe a) {
  a = fe_weak(a);
  uint64_t q = (a.v[0] + 19) >> 51;
  q = (a.v[1] + q) >> 51;
  q = (a.v[2] + q) >> 51;
  q = (a.v[3] + q) >> 51;
  q = (a.v[4] + q) >> 51;
  a.v[0] += 19 * q;
  a.v[1] += a.v[0] >> 51; a.v[0] &= M51;
  a.v[2] += a.v[1] >> 51; a.v[1] &= M51;
  a.v[3] += a.v[2] >> 51; a.v[2] &= M51;
  a.v[4] += a.v[3] >> 51; a.v[3] &= M51;
  a.v[4] &= M51;
  uint64_t w[4];
  w[0] = a.v[0] | (a.v[1] << 51);
  w[1] = (a.v[1] >> 13) | (a.v[2] << 38);
  w[2] = (a.v[2] >> 26) | (a.v[3] << 25);
  w[3] = (a.v[3] >> 39) | (a.v[4] << 12);
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) s[8 * i + j] = (uint8_t)(w[i] >> (8 * j));
}

static inline fe fe_add(fe a, fe b) {
  fe r;
  for (int i = 0; i < 5; ++i) r.v[i] = a.v[i] + b.v[i];
  return r;
}
/* a - b + 16p, then carry (dalek Sub for FieldElement51) */
static inline fe fe_sub(fe a, fe b) {
  fe r;
  r.v[0] = (a.v[0] + 36028797018963664ULL) - b.v[0];
  r.v[1] = (a.v[1] + 36028797018963952ULL) - b.v[1];
  r.v[2] = (a.v[2] + 36028797018963952ULL) - b.v[2];
  r.v[3] = (a.v[3] + 36028797018963952ULL) - b.v[3];
  r.v[4] = (a.v[4] + 36028797018963952ULL) - b.v[4];
  return fe_weak(r);
}
static inline fe fe_neg(fe a) { fe z = {{0, 0, 0, 0, 0}}; return fe_sub(z, a); }

static inline fe fe_mul(fe a, fe b) {
  uint64_t b1 = b.v[1] * 19, b2 = b.v[2] * 19, b3 = b.v[3] * 19, b4 = b.v[4] * 19;
  u128 c0 = (u128)a.v[0] * b.v[0] + (u128)a.v[4] * b1 + (u128)a.v[3] * b2 + (u128)a.v[2] * b3 + (u128)a.v[1] * b4;
  u128 c1 = (u128)a.v[1] * b.v[0] + (u128)a.v[0] * b.v[1] + (u128)a.v[4] * b2 + (u128)a.v[3] * b3 + (u128)a.v[2] * b4;
  u128 c2 = (u128)a.v[2] * b.v[0] + (u128)a.v[1] * b.v[1] + (u128)a.v[0] * b.v[2] + (u128)a.v[4] * b3 + (u128)a.v[3] * b4;
  u128 c3 = (u128)a.v[3] * b.v[0] + (u128)a.v[2] * b.v[1] + (u128)a.v[1] * b.v[2] + (u128)a.v[0] * b.v[3] + (u128)a.v[4] * b4;
  u128 c4 = (u128)a.v[4] * b.v[0] + (u128)a.v[3] * b.v[1] + (u128)a.v[2] * b.v[2] + (u128)a.v[1] * b.v[3] + (u128)a.v[0] * b.v[4];
  fe r;
  c1 += (uint64_t)(c0 >> 51); r.v[0] = (uint64_t)c0 & M51;
  c2 += (uint64_t)(c1 >> 51); r.v[1] = (uint64_t)c1 & M51;
  c3 += (uint64_t)(c2 >> 51); r.v[2] = (uint64_t)c2 & M51;
  c4 += (uint64_t)(c3 >> 51); r.v[3] = (uint64_t)c3 & M51;
  uint64_t carry = (uint64_t)(c4 >> 51); r.v[4] = (uint64_t)c4 & M51;
  r.v[0] += carry * 19;
  r.v[1] += r.v[0] >> 51; r.v[0] &= M51;
  return r;
}

static inline fe fe_sq(fe a) {
  uint64_t d0 = a.v[0] * 2, d1 = a.v[1] * 2, a3_19 = a.v[3] * 19, a4_19 = a.v[4] * 19;
  u128 c0 = (u128)a.v[0] * a.v[0] + (u128)d1 * a4_19 + (u128)(a.v[2] * 2) * a3_19;
  u128 c1 = (u128)a.v[3] * a3_19 + (u128)d0 * a.v[1] + (u128)(a.v[2] * 2) * a4_19;
  u128 c2 = (u128)a.v[1] * a.v[1] + (u128)d0 * a.v[2] + (u128)(a.v[4] * 2) * a3_19;
  u128 c3 = (u128)a.v[4] * a4_19 + (u128)d0 * a.v[3] + (u128)d1 * a.v[2];
  u128 c4 = (u128)a.v[2] * a.v[2] + (u128)d0 * a.v[4] + (u128)d1 * a.v[3];
  fe r;
  c1 += (uint64_t)(c0 >> 51); r.v[0] = (uint64_t)c0 & M51;
  c2 += (uint64_t)(c1 >> 51); r.v[1] = (uint64_t)c1 & M51;
  c3 += (uint64_t)(c2 >> 51); r.v[2] = (uint64_t)c2 & M51;
  c4 += (uint64_t)(c3 >> 51); r.v[3] = (uint64_t)c3 & M51;
  uint64_t carry = (uint64_t)(c4 >> 51); r.v[4] = (uint64_t)c4 & M51;
  r.v[0] += carry * 19;
  r.v[1] += r.v[0] >> 51; r.v[0] &= M51;
  return r;
}

static inline fe fe_pow2k(fe a, int k) {
  for (int i = 0; i < k; ++i) a = fe_sq(a);
  return a;
}

static void fe_pow22501(fe z, fe* t19, fe* t3) {
  fe t0 = fe_sq(z);
  fe t1 = fe_pow2k(t0, 2);
  fe t2 = fe_mul(z, t1);
  *t3 = fe_mul(t0, t2);
  fe t4 = fe_sq(*t3);
  fe t5 = fe_mul(t2, t4);
  fe t6 = fe_pow2k(t5, 5);
  fe t7 = fe_mul(t6, t5);
  fe t8 = fe_pow2k(t7, 10);
  fe t9 = fe_mul(t8, t7);
  fe t10 = fe_pow2k(t9, 20);
  fe t11 = fe_mul(t10, t9);
  fe t12 = fe_pow2k(t11, 10);
  fe t13 = fe_mul(t12, t7);
  fe t14 = fe_pow2k(t13, 50);
  fe t15 = fe_mul(t14, t13);
  fe t16 = fe_pow2k(t15, 100);
  fe t17 = fe_mul(t16, t15);
  fe t18 = fe_pow2k(t17, 50);
  *t19 = fe_mul(t18, t13);
}
static fe fe_invert(fe z) {
  fe t19, t3;
  fe_pow22501(z, &t19, &t3);
  return fe_mul(fe_pow2k(t19, 5), t3);
}
static fe fe_pow_p58(fe z) {
  fe t19, t3;
  fe_pow22501(z, &t19, &t3);
  return fe_mul(fe_pow2k(t19, 2), z);
}

static int fe_eq(fe a, fe b) {
  uint8_t x[32], y[32];
  fe_tobytes(x, a);
  fe_tobytes(y, b);
  return memcmp(x, y, 32) == 0;
}
static int fe_is_negative(fe a) {
  uint8_t x[32];
  fe_tobytes(x, a);
  return x[0] & 1;
}
static int fe_is_zero(fe a) {
  uint8_t x[32], z[32] = {0};
  fe_tobytes(x, a);
  return memcmp(x, z, 32) == 0;
}

static fe FE_ONE, FE_D, FE_D2, FE_SQRTM1;

static fe fe_from_hex_le(const char* hex) {
  uint8_t b[32];
  for (int i = 0; i < 32; ++i) {
    unsigned v;
    char t[3] = {hex[2 * i], hex[2 * i + 1], 0};
    v = (unsigned)strtoul(t, NULL, 16);
    b[i] = (uint8_t)v;
  }
  return fe_frombytes(b);
}

/* dalek FieldElement::sqrt_ratio_i */
static int fe_sqrt_ratio_i(fe u, fe v, fe* out) {
  fe v3 = fe_mul(fe_sq(v), v);
  fe v7 = fe_mul(fe_sq(v3), v);
  fe r = fe_mul(fe_mul(u, v3), fe_pow_p58(fe_mul(u, v7)));
  fe check = fe_mul(v, fe_sq(r));
  fe nu = fe_neg(u);
  int correct = fe_eq(check, u);
  int flipped = fe_eq(check, nu);
  int flipped_i = fe_eq(check, fe_mul(nu, FE_SQRTM1));
  if (flipped || flipped_i) r = fe_mul(FE_SQRTM1, r);
  if (fe_is_negative(r)) r = fe_neg(r);
  *out = r;
  return correct || flipped;
}

/* ============================================================ points */
typedef struct { fe X, Y, Z, T; } ge;             /* EdwardsPoint */
typedef struct { fe X, Y, Z; } gp;                /* ProjectivePoint */
typedef struct { fe X, Y, Z, T; } gc;             /* CompletedPoint */
typedef struct { fe YpX, YmX, Z, T2d; } gpn;      /* ProjectiveNielsPoint */
typedef struct { fe ypx, ymx, xy2d; } gan;        /* AffineNielsPoint */

static ge ge_identity(void) {
  ge r;
  memset(&r, 0, sizeof r);
  r.Y = FE_ONE; r.Z = FE_ONE;
  return r;
}
static int ge_decompress(const uint8_t s[32], ge* P) {
  fe Y = fe_frombytes(s);
  fe YY = fe_sq(Y);
  fe u = fe_sub(YY, FE_ONE);
  fe v = fe_add(fe_mul(YY, FE_D), FE_ONE);
  fe X;
  int ok = fe_sqrt_ratio_i(u, v, &X);
  if (!ok) return 0;
  if (s[31] >> 7) X = fe_neg(X);
  P->X = X; P->Y = Y; P->Z = FE_ONE; P->T = fe_mul(X, Y);
  return 1;
}
static void ge_compress(uint8_t s[32], ge P) {
  fe zi = fe_invert(P.Z);
  fe x = fe_mul(P.X, zi), y = fe_mul(P.Y, zi);
  fe_tobytes(s, y);
  s[31] ^= (uint8_t)(fe_is_negative(x) << 7);
}
static gpn ge_to_pniels(ge P) {
  gpn n;
  n.YpX = fe_add(P.Y, P.X); n.YmX = fe_sub(P.Y, P.X); n.Z = P.Z; n.T2d = fe_mul(P.T, FE_D2);
  return n;
}
static ge gc_to_ge(gc c) {
  ge r;
  r.X = fe_mul(c.X, c.T); r.Y = fe_mul(c.Y, c.Z); r.Z = fe_mul(c.Z, c.T); r.T = fe_mul(c.X, c.Y);
  return r;
}
static gp gc_to_gp(gc c) {
  gp r;
  r.X = fe_mul(c.X, c.T); r.Y = fe_mul(c.Y, c.Z); r.Z = fe_mul(c.Z, c.T);
  return r;
}
static ge gp_to_ge(gp p) {
  ge r;
  r.X = fe_mul(p.X, p.Z); r.Y = fe_mul(p.Y, p.Z); r.Z = fe_sq(p.Z); r.T = fe_mul(p.X, p.Y);
  return r;
}
static gc gp_double(gp p) {
  fe XX = fe_sq(p.X), YY = fe_sq(p.Y), ZZ = fe_sq(p.Z);
  fe ZZ2 = fe_add(ZZ, ZZ);
  fe XpY2 = fe_sq(fe_add(p.X, p.Y));
  fe YYpXX = fe_add(YY, XX), YYmXX = fe_sub(YY, XX);
  gc c;
  c.X = fe_sub(XpY2, YYpXX); c.Y = YYpXX; c.Z = YYmXX; c.T = fe_sub(ZZ2, YYmXX);
  return c;
}
static gc ge_add_pn(ge P, gpn q) {
  fe PP = fe_mul(fe_add(P.Y, P.X), q.YpX), MM = fe_mul(fe_sub(P.Y, P.X), q.YmX);
  fe TT2d = fe_mul(P.T, q.T2d), ZZ = fe_mul(P.Z, q.Z), ZZ2 = fe_add(ZZ, ZZ);
  gc c;
  c.X = fe_sub(PP, MM); c.Y = fe_add(PP, MM); c.Z = fe_add(ZZ2, TT2d); c.T = fe_sub(ZZ2, TT2d);
  return c;
}
static gc ge_sub_pn(ge P, gpn q) {
  fe PM = fe_mul(fe_add(P.Y, P.X), q.YmX), MP = fe_mul(fe_sub(P.Y, P.X), q.YpX);
  fe TT2d = fe_mul(P.T, q.T2d), ZZ = fe_mul(P.Z, q.Z), ZZ2 = fe_add(ZZ, ZZ);
  gc c;
  c.X = fe_sub(PM, MP); c.Y = fe_add(PM, MP); c.Z = fe_sub(ZZ2, TT2d); c.T = fe_add(ZZ2, TT2d);
  return c;
}
static gc ge_add_an(ge P, gan q) {
  fe PP = fe_mul(fe_add(P.Y, P.X), q.ypx), MM = fe_mul(fe_sub(P.Y, P.X), q.ymx);
  fe Txy2d = fe_mul(P.T, q.xy2d), Z2 = fe_add(P.Z, P.Z);
  gc c;
  c.X = fe_sub(PP, MM); c.Y = fe_add(PP, MM); c.Z = fe_add(Z2, Txy2d); c.T = fe_sub(Z2, Txy2d);
  return c;
}
static gc ge_sub_an(ge P, gan q) {
  fe PM = fe_mul(fe_add(P.Y, P.X), q.ymx), MP = fe_mul(fe_sub(P.Y, P.X), q.ypx);
  fe Txy2d = fe_mul(P.T, q.xy2d), Z2 = fe_add(P.Z, P.Z);
  gc c;
  c.X = fe_sub(PM, MP); c.Y = fe_add(PM, MP); c.Z = fe_sub(Z2, Txy2d); c.T = fe_add(Z2, Txy2d);
  return c;
}
static ge ge_add(ge P, ge Q) { return gc_to_ge(ge_add_pn(P, ge_to_pniels(Q))); }
static ge ge_neg(ge P) { P.X = fe_neg(P.X); P.T = fe_neg(P.T); return P; }
static ge ge_dbl(ge P) { gp p = {P.X, P.Y, P.Z}; return gc_to_ge(gp_double(p)); }
static ge ge_mul_pow2(ge P, int k) {
  gp p = {P.X, P.Y, P.Z};
  gc c;
  for (int i = 0; i < k - 1; ++i) { c = gp_double(p); p = gc_to_gp(c); }
  return gc_to_ge(gp_double(p));
}
static ge ge_mul_by_cofactor(ge P) { return ge_mul_pow2(P, 3); }
static int ge_is_identity(ge P) { return fe_is_zero(P.X) && fe_eq(P.Y, P.Z); }

static ge GE_B;
static gan B_ODD[64];   /* [1,3,...,127]B, affine Niels (NAF-8 table) */

/* ============================================================ scalars mod l (4 x 64) */
static const uint64_t L64[4] = {0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0ULL, 0x1000000000000000ULL};
static const uint64_t MU64[5] = {0xed9ce5a30a2c131bULL, 0x2106215d086329a7ULL, 0xffffffffffffffebULL,
                                 0xffffffffffffffffULL, 0xfULL};

static int geq_n(const uint64_t* a, const uint64_t* b, int n) {
  for (int i = n - 1; i >= 0; --i)
    if (a[i] != b[i]) return a[i] > b[i];
  return 1;
}
static uint64_t sub_n(uint64_t* r, const uint64_t* a, const uint64_t* b, int n) {
  uint64_t br = 0;
  for (int i = 0; i < n; ++i) {
    u128 t = (u128)a[i] - b[i] - br;
    r[i] = (uint64_t)t;
    br = (uint64_t)(t >> 64) & 1;
  }
  return br;
}
/* x (8 limbs) mod l -> r (4 limbs), Barrett b = 2^64, k = 4 */
static void sc_reduce512(const uint64_t x[8], uint64_t r[4]) {
  const uint64_t* q1 = x + 3;             /* 5 limbs */
  uint64_t q2[10] = {0};
  for (int i = 0; i < 5; ++i) {
    uint64_t c = 0;
    for (int j = 0; j < 5; ++j) {
      u128 t = (u128)q1[i] * MU64[j] + q2[i + j] + c;
      q2[i + j] = (uint64_t)t;
      c = (uint64_t)(t >> 64);
    }
    q2[i + 5] = c;
  }
  const uint64_t* q3 = q2 + 5;            /* 5 limbs */
  uint64_t r2[5] = {0};
  for (int i = 0; i < 5; ++i) {
    uint64_t c = 0;
    int j = 0;
    for (; j < 4 && i + j < 5; ++j) {
      u128 t = (u128)q3[i] * L64[j] + r2[i + j] + c;
      r2[i + j] = (uint64_t)t;
      c = (uint64_t)(t >> 64);
    }
    if (i + j < 5) r2[i + j] = c;
  }
  uint64_t rr[5];
  sub_n(rr, x, r2, 5);
  uint64_t L5[5] = {L64[0], L64[1], L64[2], L64[3], 0};
  for (int it = 0; it < 3; ++it) {
    uint64_t t[5];
    if (!sub_n(t, rr, L5, 5)) memcpy(rr, t, sizeof t);
  }
  memcpy(r, rr, 32);
}
static void sc_from_bytes64(const uint8_t d[64], uint64_t r[4]) {
  uint64_t x[8];
  for (int i = 0; i < 8; ++i) x[i] = ld64(d + 8 * i);
  sc_reduce512(x, r);
}
static void sc_mul(const uint64_t a[4], const uint64_t b[4], uint64_t r[4]) {
  uint64_t x[8] = {0};
  for (int i = 0; i < 4; ++i) {
    uint64_t c = 0;
    for (int j = 0; j < 4; ++j) {
      u128 t = (u128)a[i] * b[j] + x[i + j] + c;
      x[i + j] = (uint64_t)t;
      c = (uint64_t)(t >> 64);
    }
    x[i + 4] = c;
  }
  sc_reduce512(x, r);
}
static void sc_add(const uint64_t a[4], const uint64_t b[4], uint64_t r[4]) {
  uint64_t x[8] = {0};
  u128 c = 0;
  for (int i = 0; i < 4; ++i) { c += (u128)a[i] + b[i]; x[i] = (uint64_t)c; c >>= 64; }
  x[4] = (uint64_t)c;
  sc_reduce512(x, r);
}
static void sc_sub(const uint64_t a[4], const uint64_t b[4], uint64_t r[4]) {
  uint64_t t[4];
  if (sub_n(t, a, b, 4)) {
    u128 c = 0;
    for (int i = 0; i < 4; ++i) { c += (u128)t[i] + L64[i]; t[i] = (uint64_t)c; c >>= 64; }
  }
  memcpy(r, t, 32);
}
static int sc_canonical(const uint8_t s[32]) {
  uint64_t x[4] = {ld64(s), ld64(s + 8), ld64(s + 16), ld64(s + 24)};
  if (s[31] >> 7) return 0;
  return !geq_n(x, L64, 4);
}

/* width-w NAF of a scalar < 2^255 (dalek Scalar::non_adjacent_form) */
static void naf(const uint64_t s[4], int w, int8_t out[256]) {
  memset(out, 0, 256);
  uint64_t x[5] = {s[0], s[1], s[2], s[3], 0};
  int width = 1 << w, wmask = width - 1;
  int pos = 0, carry = 0;
  while (pos < 256) {
    int idx = pos / 64, bit = pos % 64;
    uint64_t bits = (bit < 64 - w) ? (x[idx] >> bit) : ((x[idx] >> bit) | (x[idx + 1] << (64 - bit)));
    int window = carry + (int)(bits & (uint64_t)wmask);
    if ((window & 1) == 0) { pos += 1; continue; }
    if (window < width / 2) { carry = 0; out[pos] = (int8_t)window; }
    else { carry = 1; out[pos] = (int8_t)(window - width); }
    pos += w;
  }
}

/* signed radix-2^w digits (dalek Scalar::to_radix_2w), returns digit count */
static int radix_2w(const uint64_t s[4], int w, int8_t* d) {
  int count = (256 + w - 1) / w;
  uint64_t radix = 1ULL << w, mask = radix - 1;
  int64_t carry = 0;
  for (int i = 0; i < count; ++i) {
    int bitpos = i * w, li = bitpos / 64, bi = bitpos % 64;
    uint64_t bits = s[li] >> bi;
    if (bi + w > 64 && li + 1 < 4) bits |= s[li + 1] << (64 - bi);
    int64_t coef = carry + (int64_t)(bits & mask);
    carry = (coef + (int64_t)(radix / 2)) >> w;
    d[i] = (int8_t)(coef - (carry << w));
  }
  if (carry) { d[count] = (int8_t)carry; return count + 1; }
  d[count] = 0;
  return count + 1;
}

/* ============================================================ MSM */
static ge msm_straus(size_t n, const uint64_t (*sc)[4], const ge* pts) {
  gpn* tab = (gpn*)malloc(n * 8 * sizeof(gpn));
  int8_t* nafs = (int8_t*)malloc(n * 256);
  for (size_t i = 0; i < n; ++i) {
    ge A = pts[i], A2 = ge_dbl(A);
    tab[i * 8] = ge_to_pniels(A);
    for (int j = 1; j < 8; ++j) { A = gc_to_ge(ge_add_pn(A2, tab[i * 8 + j - 1])); tab[i * 8 + j] = ge_to_pniels(A); }
    naf(sc[i], 5, nafs + i * 256);
  }
  gp r = {fe_from_hex_le("0000000000000000000000000000000000000000000000000000000000000000"), FE_ONE, FE_ONE};
  for (int k = 255; k >= 0; --k) {
    gc t = gp_double(r);
    for (size_t i = 0; i < n; ++i) {
      int d = nafs[i * 256 + k];
      if (d > 0) t = ge_add_pn(gc_to_ge(t), tab[i * 8 + d / 2]);
      else if (d < 0) t = ge_sub_pn(gc_to_ge(t), tab[i * 8 + (-d) / 2]);
    }
    r = gc_to_gp(t);
  }
  free(tab);
  free(nafs);
  return gp_to_ge(r);
}

static ge msm_pippenger(size_t n, const uint64_t (*sc)[4], const ge* pts) {
  int w = n < 500 ? 6 : (n < 800 ? 7 : 8);
  int nb = 1 << (w - 1);
  int maxd = (256 + w - 1) / w + 1;
  int8_t* digits = (int8_t*)malloc(n * (size_t)maxd);
  gpn* pn = (gpn*)malloc(n * sizeof(gpn));
  int cnt = 0;
  for (size_t i = 0; i < n; ++i) {
    cnt = radix_2w(sc[i], w, digits + i * maxd);
    pn[i] = ge_to_pniels(pts[i]);
  }
  ge* buckets = (ge*)malloc(nb * sizeof(ge));
  ge total = ge_identity();
  for (int win = cnt - 1; win >= 0; --win) {
    for (int b = 0; b < nb; ++b) buckets[b] = ge_identity();
    for (size_t i = 0; i < n; ++i) {
      int d = digits[i * maxd + win];
      if (d > 0) buckets[d - 1] = gc_to_ge(ge_add_pn(buckets[d - 1], pn[i]));
      else if (d < 0) buckets[-d - 1] = gc_to_ge(ge_sub_pn(buckets[-d - 1], pn[i]));
    }
    ge inter = buckets[nb - 1], sum = buckets[nb - 1];
    for (int b = nb - 2; b >= 0; --b) {
      inter = ge_add(inter, buckets[b]);
      sum = ge_add(sum, inter);
    }
    total = (win == cnt - 1) ? sum : ge_add(ge_mul_pow2(total, w), sum);
  }
  free(digits);
  free(pn);
  free(buckets);
  return total;
}

static ge msm(size_t n, const uint64_t (*sc)[4], const ge* pts) {
  if (n == 0) return ge_identity();
  return n < 190 ? msm_straus(n, sc, pts) : msm_pippenger(n, sc, pts);
}

/* [a]A + [b]B, NAF-5 for A, NAF-8 with the B odd-multiples table */
static ge double_scalar_mul_basepoint(const uint64_t a[4], ge A, const uint64_t b[4]) {
  int8_t an[256], bn[256];
  naf(a, 5, an);
  naf(b, 8, bn);
  gpn tab[8];
  ge P = A, A2 = ge_dbl(A);
  tab[0] = ge_to_pniels(P);
  for (int j = 1; j < 8; ++j) { P = gc_to_ge(ge_add_pn(A2, tab[j - 1])); tab[j] = ge_to_pniels(P); }
  int i = 255;
  while (i >= 0 && an[i] == 0 && bn[i] == 0) --i;
  gp r = {fe_from_hex_le("0000000000000000000000000000000000000000000000000000000000000000"), FE_ONE, FE_ONE};
  for (; i >= 0; --i) {
    gc t = gp_double(r);
    if (an[i] > 0) t = ge_add_pn(gc_to_ge(t), tab[an[i] / 2]);
    else if (an[i] < 0) t = ge_sub_pn(gc_to_ge(t), tab[(-an[i]) / 2]);
    if (bn[i] > 0) t = ge_add_an(gc_to_ge(t), B_ODD[bn[i] / 2]);
    else if (bn[i] < 0) t = ge_sub_an(gc_to_ge(t), B_ODD[(-bn[i]) / 2]);
    r = gc_to_gp(t);
  }
  return gp_to_ge(r);
}

/* ============================================================ SHA-512 */
static const uint64_t K512[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL, 0x3956c25bf348b538ULL,
    0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL, 0xd807aa98a3030242ULL, 0x12835b0145706fbeULL,
    0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL, 0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL,
    0xc19bf174cf692694ULL, 0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL, 0x983e5152ee66dfabULL,
    0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL, 0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL,
    0x06ca6351e003826fULL, 0x142929670a0e6e70ULL, 0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL,
    0x53380d139d95b3dfULL, 0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL, 0xd192e819d6ef5218ULL,
    0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL, 0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL,
    0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL, 0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL,
    0x682e6ff3d6b2b8a3ULL, 0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL, 0xca273eceea26619cULL,
    0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL, 0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL,
    0x113f9804bef90daeULL, 0x1b710b35131c471bULL, 0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL,
    0x431d67c49c100d4cULL, 0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

typedef struct { uint64_t h[8]; uint8_t buf[128]; size_t len; uint64_t total; } sha512_ctx;
#define ROR(x, n) (((x) >> (n)) | ((x) << (64 - (n))))
static void sha512_block(uint64_t h[8], const uint8_t* p) {
  uint64_t w[80];
  for (int t = 0; t < 16; ++t) {
    uint64_t v = 0;
    for (int b = 0; b < 8; ++b) v = (v << 8) | p[8 * t + b];
    w[t] = v;
  }
  for (int t = 16; t < 80; ++t) {
    uint64_t s0 = ROR(w[t - 15], 1) ^ ROR(w[t - 15], 8) ^ (w[t - 15] >> 7);
    uint64_t s1 = ROR(w[t - 2], 19) ^ ROR(w[t - 2], 61) ^ (w[t - 2] >> 6);
    w[t] = w[t - 16] + s0 + w[t - 7] + s1;
  }
  uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int t = 0; t < 80; ++t) {
    uint64_t t1 = hh + (ROR(e, 14) ^ ROR(e, 18) ^ ROR(e, 41)) + ((e & f) ^ (~e & g)) + K512[t] + w[t];
    uint64_t t2 = (ROR(a, 28) ^ ROR(a, 34) ^ ROR(a, 39)) + ((a & b) ^ (a & c) ^ (b & c));
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}
static void sha512_init(sha512_ctx* c) {
  static const uint64_t iv[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                                 0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
  memcpy(c->h, iv, sizeof iv);
  c->len = 0;
  c->total = 0;
}
static void sha512_update(sha512_ctx* c, const uint8_t* p, size_t n) {
  c->total += n;
  while (n) {
    size_t take = 128 - c->len;
    if (take > n) take = n;
    memcpy(c->buf + c->len, p, take);
    c->len += take; p += take; n -= take;
    if (c->len == 128) { sha512_block(c->h, c->buf); c->len = 0; }
  }
}
static void sha512_final(sha512_ctx* c, uint8_t out[64]) {
  uint64_t bits = c->total * 8;
  uint8_t pad = 0x80;
  sha512_update(c, &pad, 1);
  uint8_t z = 0;
  while (c->len != 112) sha512_update(c, &z, 1);
  uint8_t lenb[16] = {0};
  for (int i = 0; i < 8; ++i) lenb[15 - i] = (uint8_t)(bits >> (8 * i));
  sha512_update(c, lenb, 16);
  for (int i = 0; i < 8; ++i)
    for (int b = 0; b < 8; ++b) out[8 * i + b] = (uint8_t)(c->h[i] >> (56 - 8 * b));
}

static void challenge(const uint8_t* R, const uint8_t* A, const uint8_t* m, size_t mlen, uint64_t k[4]) {
  sha512_ctx c;
  uint8_t d[64];
  sha512_init(&c);
  sha512_update(&c, R, 32);
  sha512_update(&c, A, 32);
  sha512_update(&c, m, mlen);
  sha512_final(&c, d);
  sc_from_bytes64(d, k);
}

/* ============================================================ ChaCha20 z stream */
static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static void chacha_block(const uint32_t key[8], uint64_t ctr, uint32_t out[16]) {
  uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1], key[2], key[3],
                    key[4], key[5], key[6], key[7], (uint32_t)ctr, (uint32_t)(ctr >> 32), 0, 0};
  uint32_t x[16];
  memcpy(x, s, sizeof x);
#define QR(a, b, c, d) x[a] += x[b]; x[d] = rotl32(x[d] ^ x[a], 16); x[c] += x[d]; x[b] = rotl32(x[b] ^ x[c], 12); \
  x[a] += x[b]; x[d] = rotl32(x[d] ^ x[a], 8); x[c] += x[d]; x[b] = rotl32(x[b] ^ x[c], 7);
  for (int i = 0; i < 10; ++i) {
    QR(0, 4, 8, 12) QR(1, 5, 9, 13) QR(2, 6, 10, 14) QR(3, 7, 11, 15)
    QR(0, 5, 10, 15) QR(1, 6, 11, 12) QR(2, 7, 8, 13) QR(3, 4, 9, 14)
  }
#undef QR
  for (int i = 0; i < 16; ++i) out[i] = x[i] + s[i];
}
static void draw_z(const uint8_t seed[32], uint64_t j, uint64_t z[4]) {
  uint32_t key[8], blk[16];
  for (int i = 0; i < 8; ++i)
    key[i] = (uint32_t)seed[4 * i] | ((uint32_t)seed[4 * i + 1] << 8) | ((uint32_t)seed[4 * i + 2] << 16) |
             ((uint32_t)seed[4 * i + 3] << 24);
  chacha_block(key, j >> 2, blk);
  int q = (int)(j & 3);
  z[0] = (uint64_t)blk[4 * q] | ((uint64_t)blk[4 * q + 1] << 32);
  z[1] = (uint64_t)blk[4 * q + 2] | ((uint64_t)blk[4 * q + 3] << 32);
  z[2] = z[3] = 0;
}

/* ============================================================ init */
static int g_init = 0;
static pthread_mutex_t g_init_mu = PTHREAD_MUTEX_INITIALIZER;
static void oc_init_once(void) {
  pthread_mutex_lock(&g_init_mu);
  if (!g_init) {
    memset(&FE_ONE, 0, sizeof FE_ONE);
    FE_ONE.v[0] = 1;
    FE_D = fe_from_hex_le("a3785913ca4deb75abd841414d0a700098e879777940c78c73fe6f2bee6c0352");
    FE_D2 = fe_from_hex_le("59f1b226949bd6eb56b183829a14e00030d1f3eef2808e19e7fcdf56dcd90624");
    FE_SQRTM1 = fe_from_hex_le("b0a00e4a271beec478e42fad0618432fa7d7fb3d99004d2b0bdfc14f8024832b");
    uint8_t bb[32];
    memset(bb, 0x66, 32);
    bb[0] = 0x58;
    ge_decompress(bb, &GE_B);
    ge P = GE_B, B2 = ge_dbl(GE_B);
    for (int j = 0; j < 64; ++j) {
      fe zi = fe_invert(P.Z);
      fe x = fe_mul(P.X, zi), y = fe_mul(P.Y, zi);
      B_ODD[j].ypx = fe_add(y, x);
      B_ODD[j].ymx = fe_sub(y, x);
      B_ODD[j].xy2d = fe_mul(fe_mul(x, y), FE_D2);
      P = ge_add(P, B2);
    }
    g_init = 1;
  }
  pthread_mutex_unlock(&g_init_mu);
}

/* ============================================================ verification */
enum { OC_OK = 0, OC_INVALID_SIGNATURE = 1, OC_MALFORMED_PUBLIC_KEY = 2 };

static int verify_prehashed(const uint8_t* A_bytes, const uint8_t* sig, const uint64_t k[4]) {
  ge A;
  if (!ge_decompress(A_bytes, &A)) return OC_MALFORMED_PUBLIC_KEY;   /* try_from */
  if (!sc_canonical(sig + 32)) return OC_INVALID_SIGNATURE;           /* s before R */
  ge R;
  if (!ge_decompress(sig, &R)) return OC_INVALID_SIGNATURE;
  uint64_t s[4] = {ld64(sig + 32), ld64(sig + 40), ld64(sig + 48), ld64(sig + 56)};
  ge Rp = double_scalar_mul_basepoint(k, ge_neg(A), s);
  ge d = ge_add(R, ge_neg(Rp));
  return ge_is_identity(ge_mul_by_cofactor(d)) ? OC_OK : OC_INVALID_SIGNATURE;
}

/* HashMap<VerificationKeyBytes, Vec<(k, sig, j)>>: open addressing on the raw key bytes */
typedef struct { uint32_t first; uint32_t count; uint32_t head; } group;

static uint64_t key_hash(const uint8_t* k) {
  uint64_t h = 0x9e3779b97f4a7c15ULL;
  for (int i = 0; i < 4; ++i) { h ^= ld64(k + 8 * i); h *= 0xff51afd7ed558ccdULL; h ^= h >> 33; }
  return h;
}

int oc_batch_verify_range(size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg,
                          const uint64_t* off, const uint8_t z_seed[32], const uint8_t* zexp, uint64_t z_base,
                          uint8_t check8[32], uint8_t partial_affine[64]) {
  oc_init_once();
  /* queue: k at queue time + grouping by raw key bytes */
  uint64_t (*k)[4] = (uint64_t (*)[4])malloc((n ? n : 1) * 32);
  size_t T = 16;
  while (T < 2 * n + 2) T <<= 1;
  int32_t* tab = (int32_t*)malloc(T * sizeof(int32_t));
  for (size_t i = 0; i < T; ++i) tab[i] = -1;
  uint32_t* grp = (uint32_t*)malloc((n ? n : 1) * sizeof(uint32_t));  /* group id per item */
  uint32_t* rep = (uint32_t*)malloc((n ? n : 1) * sizeof(uint32_t));  /* first item per group */
  uint32_t m = 0;
  for (size_t i = 0; i < n; ++i) {
    challenge(sig + 64 * i, vk + 32 * i, msg + off[i], off[i + 1] - off[i], k[i]);
    size_t h = key_hash(vk + 32 * i) & (T - 1);
    for (;;) {
      if (tab[h] < 0) { tab[h] = (int32_t)m; rep[m] = (uint32_t)i; grp[i] = m++; break; }
      if (memcmp(vk + 32 * rep[tab[h]], vk + 32 * i, 32) == 0) { grp[i] = (uint32_t)tab[h]; break; }
      h = (h + 1) & (T - 1);
    }
  }
  /* verify */
  size_t nterms = 1 + m + n;
  uint64_t (*sc)[4] = (uint64_t (*)[4])calloc(nterms, 32);
  ge* pts = (ge*)malloc(nterms * sizeof(ge));
  int rc = OC_OK;
  pts[0] = GE_B;
  for (uint32_t g = 0; g < m; ++g) {
    if (!ge_decompress(vk + 32 * rep[g], &pts[1 + g])) { rc = OC_INVALID_SIGNATURE; goto done; }
  }
  uint64_t Bc[4] = {0, 0, 0, 0};
  for (size_t i = 0; i < n; ++i) {
    if (!ge_decompress(sig + 64 * i, &pts[1 + m + i])) { rc = OC_INVALID_SIGNATURE; goto done; }
    if (!sc_canonical(sig + 64 * i + 32)) { rc = OC_INVALID_SIGNATURE; goto done; }
    uint64_t s[4] = {ld64(sig + 64 * i + 32), ld64(sig + 64 * i + 40), ld64(sig + 64 * i + 48), ld64(sig + 64 * i + 56)};
    uint64_t z[4];
    if (zexp) { z[0] = ld64(zexp + 16 * i); z[1] = ld64(zexp + 16 * i + 8); z[2] = z[3] = 0; }
    else draw_z(z_seed, z_base + i, z);
    uint64_t zs[4], zk[4];
    sc_mul(z, s, zs);
    sc_sub(Bc, zs, Bc);
    memcpy(sc[1 + m + i], z, 32);
    sc_mul(z, k[i], zk);
    sc_add(sc[1 + grp[i]], zk, sc[1 + grp[i]]);
  }
  memcpy(sc[0], Bc, 32);
  {
    ge check = msm(nterms, (const uint64_t (*)[4])sc, pts);
    if (partial_affine) {
      fe zi = fe_invert(check.Z);
      fe_tobytes(partial_affine, fe_mul(check.X, zi));
      fe_tobytes(partial_affine + 32, fe_mul(check.Y, zi));
    }
    ge c8 = ge_mul_by_cofactor(check);
    rc = ge_is_identity(c8) ? OC_OK : OC_INVALID_SIGNATURE;
    if (check8) ge_compress(check8, c8);
  }
done:
  free(k); free(tab); free(grp); free(rep); free(sc); free(pts);
  return rc;
}

int oc_batch_verify(size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg, const uint64_t* off,
                    const uint8_t z_seed[32], uint8_t check8[32], int* evaluated) {
  uint8_t c8[32];
  memset(c8, 0, 32);
  int rc = oc_batch_verify_range(n, vk, sig, msg, off, z_seed, NULL, 0, c8, NULL);
  if (check8) memcpy(check8, c8, 32);
  if (evaluated) {
    static const uint8_t zero[32] = {0};
    *evaluated = memcmp(c8, zero, 32) != 0;
  }
  return rc;
}

int oc_verify(const uint8_t* vk, const uint8_t* sig, const uint8_t* msg, size_t mlen) {
  oc_init_once();
  uint64_t k[4];
  challenge(sig, vk, msg, mlen, k);
  return verify_prehashed(vk, sig, k);
}

/* shard partial (affine x || y of the shard's check point) and combination, for the
   multi-rank tests: combine = sum of partials, [8], identity */
int oc_combine_affine(size_t g, const uint8_t* parts, uint8_t check8[32]) {
  oc_init_once();
  ge acc = ge_identity();
  for (size_t i = 0; i < g; ++i) {
    ge P;
    P.X = fe_frombytes(parts + 64 * i);
    P.Y = fe_frombytes(parts + 64 * i + 32);
    P.Z = FE_ONE;
    P.T = fe_mul(P.X, P.Y);
    acc = ge_add(acc, P);
  }
  ge c8 = ge_mul_by_cofactor(acc);
  if (check8) ge_compress(check8, c8);
  return ge_is_identity(c8) ? OC_OK : OC_INVALID_SIGNATURE;
}

/* Full-size oracle check of a GPU batch (tests only): the batch equation is linear and z is drawn
   at global queue indices, so `parts` contiguous ranges, each one oc_batch_verify_range at
   z_base + its start (one thread each), give partial points whose sum is the whole batch's check
   point. partials: parts x 64 bytes (affine x || y); rcs[g] = OC_OK / OC_INVALID_SIGNATURE of the
   range alone, evaluated[g] = 0 when the range was rejected before its MSM (undecodable / s >= l). */
typedef struct {
  size_t lo, hi;
  const uint8_t *vk, *sig, *msg, *seed;
  const uint64_t* off;
  uint64_t z_base;
  uint8_t* partial;
  int rc, evaluated;
} pjob;

static void* pworker(void* p) {
  pjob* j = (pjob*)p;
  size_t n = j->hi - j->lo;
  uint64_t* o = (uint64_t*)malloc((n + 1) * sizeof(uint64_t));
  for (size_t i = 0; i <= n; ++i) o[i] = j->off[j->lo + i] - j->off[j->lo];
  uint8_t c8[32];
  memset(c8, 0, 32);
  j->rc = oc_batch_verify_range(n, j->vk + 32 * j->lo, j->sig + 64 * j->lo, j->msg + j->off[j->lo], o, j->seed, NULL,
                                j->z_base + j->lo, c8, j->partial);
  static const uint8_t zero[32] = {0};
  j->evaluated = memcmp(c8, zero, 32) != 0;
  free(o);
  return NULL;
}

int oc_partials_parallel(size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg, const uint64_t* off,
                         const uint8_t z_seed[32], int parts, uint64_t z_base, uint8_t* partials, int* rcs,
                         int* evaluated) {
  oc_init_once();
  if (parts < 1) return -1;
  pjob* jobs = (pjob*)calloc((size_t)parts, sizeof(pjob));
  pthread_t* th = (pthread_t*)malloc((size_t)parts * sizeof(pthread_t));
  for (int g = 0; g < parts; ++g) {
    jobs[g].lo = n * (size_t)g / (size_t)parts;
    jobs[g].hi = n * (size_t)(g + 1) / (size_t)parts;
    jobs[g].vk = vk; jobs[g].sig = sig; jobs[g].msg = msg; jobs[g].off = off; jobs[g].seed = z_seed;
    jobs[g].z_base = z_base;
    jobs[g].partial = partials + 64 * (size_t)g;
    memset(jobs[g].partial, 0, 64);
    pthread_create(&th[g], NULL, pworker, &jobs[g]);
  }
  for (int g = 0; g < parts; ++g) {
    pthread_join(th[g], NULL);
    rcs[g] = jobs[g].rc;
    evaluated[g] = jobs[g].evaluated;
  }
  free(jobs);
  free(th);
  return 0;
}

/* ============================================================ all-core CPU baseline */
typedef struct {
  size_t lo, hi;
  const uint8_t *vk, *sig, *msg;
  const uint64_t* off;
  int rc;
} job;

static void* worker(void* p) {
  job* j = (job*)p;
  size_t n = j->hi - j->lo;
  uint64_t* o = (uint64_t*)malloc((n + 1) * sizeof(uint64_t));
  for (size_t i = 0; i <= n; ++i) o[i] = j->off[j->lo + i] - j->off[j->lo];
  uint8_t seed[32];
  for (int i = 0; i < 32; ++i) seed[i] = (uint8_t)(0x33 + j->lo + i);
  j->rc = oc_batch_verify_range(n, j->vk + 32 * j->lo, j->sig + 64 * j->lo, j->msg + j->off[j->lo], o, seed, NULL,
                                0, NULL, NULL);
  free(o);
  return NULL;
}

/* One Verifier per thread over equal contiguous chunks (queue incl. SHA-512 + verify),
   wall time in seconds; *all_ok = every chunk verified. */
double oc_baseline(size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg, const uint64_t* off,
                   int threads, size_t chunk, int* all_ok) {
  oc_init_once();
  if (chunk == 0) chunk = (n + threads - 1) / threads;
  size_t nj = (n + chunk - 1) / chunk;
  job* jobs = (job*)calloc(nj, sizeof(job));
  for (size_t i = 0; i < nj; ++i) {
    jobs[i].lo = i * chunk;
    jobs[i].hi = (i + 1) * chunk < n ? (i + 1) * chunk : n;
    jobs[i].vk = vk; jobs[i].sig = sig; jobs[i].msg = msg; jobs[i].off = off;
  }
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  pthread_t* th = (pthread_t*)malloc(threads * sizeof(pthread_t));
  size_t next = 0;
  while (next < nj) {
    int k = 0;
    for (; k < threads && next < nj; ++k, ++next) pthread_create(&th[k], NULL, worker, &jobs[next]);
    for (int q = 0; q < k; ++q) pthread_join(th[q], NULL);
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  int ok = 1;
  for (size_t i = 0; i < nj; ++i) ok &= jobs[i].rc == OC_OK;
  if (all_ok) *all_ok = ok;
  free(jobs);
  free(th);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* Small-batch timing on the calling thread (the shape of reference benches/bench.rs:25-71): reps x
   (queue + verify) of one n-item batch, or reps x (VerificationKey::try_from + verify) of every item
   ("Unbatched verification"). Seconds; *all_ok = every run accepted. CPU baseline only. */
static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

double oc_bench_batch(size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg, const uint64_t* off,
                      int reps, int* all_ok) {
  oc_init_once();
  uint8_t seed[32];
  int ok = 1;
  const double t0 = now_s();
  for (int r = 0; r < reps; ++r) {
    for (int i = 0; i < 32; ++i) seed[i] = (uint8_t)(r * 7 + i);
    ok &= oc_batch_verify_range(n, vk, sig, msg, off, seed, NULL, 0, NULL, NULL) == OC_OK;
  }
  const double t = now_s() - t0;
  if (all_ok) *all_ok = ok;
  return t;
}

double oc_bench_single(size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg, const uint64_t* off,
                       int reps, int* all_ok) {
  oc_init_once();
  int ok = 1;
  const double t0 = now_s();
  for (int r = 0; r < reps; ++r)
    for (size_t i = 0; i < n; ++i)
      ok &= oc_verify(vk + 32 * i, sig + 64 * i, msg + off[i], (size_t)(off[i + 1] - off[i])) == OC_OK;
  const double t = now_s() - t0;
  if (all_ok) *all_ok = ok;
  return t;
}
