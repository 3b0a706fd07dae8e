// Test-only host build of the SAME device math headers (csrc/*.h compiled by g++), so the
// radix-2^29 field, curve, scalar, SHA-512 and ChaCha20 logic is checked against the Python
// oracle on CPU without a GPU. Never linked into the product library.
#include <stdint.h>
#include <string.h>
#include "fe25519.h"
#include "ge25519.h"
#include "sc25519.h"
#include "sha512.h"
#include "chacha20.h"

using namespace edc;

static void bytes_to_words(const uint8_t* b, uint32_t w[8]) {
  for (int i = 0; i < 8; ++i)
    w[i] = (uint32_t)b[4 * i] | ((uint32_t)b[4 * i + 1] << 8) | ((uint32_t)b[4 * i + 2] << 16) |
           ((uint32_t)b[4 * i + 3] << 24);
}
static void words_to_bytes(const uint32_t w[8], uint8_t* b) {
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 4; ++j) b[4 * i + j] = (uint8_t)(w[i] >> (8 * j));
}

extern "C" {

// field: op 0 mul, 1 sqr, 2 add_c, 3 sub, 4 invert, 5 pow_p58, 6 neg ; canonical bytes out
void hc_fe_op(int op, const uint8_t* a, const uint8_t* b, uint8_t* out) {
  uint32_t wa[8], wb[8], wo[8];
  bytes_to_words(a, wa);
  bytes_to_words(b, wb);
  fe x = fe_from_words(wa), y = fe_from_words(wb), r;
  switch (op) {
    case 0: r = fe_mul(x, y); break;
    case 1: r = fe_sqr(x); break;
    case 2: r = fe_add_c(x, y); break;
    case 3: r = fe_sub(x, y); break;
    case 4: r = fe_invert(x); break;
    case 5: r = fe_pow_p58(x); break;
    default: r = fe_neg(x); break;
  }
  fe_to_words(r, wo);
  words_to_bytes(wo, out);
}

// raw limbs in (any lazy form the caller picks, e.g. every limb at the mul-input bound):
// op 0 mul, 1 sqr; out = canonical bytes, lim = the output limbs
void hc_fe_limbs(int op, const uint32_t* a, const uint32_t* b, uint8_t* out, uint32_t* lim) {
  fe x, y, r;
  for (int i = 0; i < 9; ++i) { x.v[i] = a[i]; y.v[i] = b[i]; }
  switch (op) {
    case 0: r = fe_mul(x, y); break;
    default: r = fe_sqr(x); break;
  }
  for (int i = 0; i < 9; ++i) lim[i] = r.v[i];
  uint32_t wo[8];
  fe_to_words(r, wo);
  words_to_bytes(wo, out);
}

// fe_is_zero on raw limbs (any form with limbs < 2^30.41)
int hc_fe_is_zero_limbs(const uint32_t* a) {
  fe x;
  for (int i = 0; i < 9; ++i) x.v[i] = a[i];
  return fe_is_zero(x) ? 1 : 0;
}

// stress the lazy bounds: r = ((a+b)*(c+d) - (a*b)) chained k times
void hc_fe_chain(const uint8_t* a, const uint8_t* b, int k, uint8_t* out) {
  uint32_t wa[8], wb[8], wo[8];
  bytes_to_words(a, wa);
  bytes_to_words(b, wb);
  fe x = fe_from_words(wa), y = fe_from_words(wb);
  for (int i = 0; i < k; ++i) {
    fe s = fe_mul(fe_add(x, y), fe_add(y, x));
    fe t = fe_sub(s, fe_add(x, x));
    x = y;
    y = fe_sqr(fe_sub(t, y));
  }
  fe_to_words(y, wo);
  words_to_bytes(wo, out);
}

// decompress: returns ok; out = canonical x || y
int hc_decompress(const uint8_t* enc, uint8_t* out) {
  uint32_t w[8], wx[8], wy[8];
  bytes_to_words(enc, w);
  ge_p3 P;
  bool ok = ge_decompress(w, P);
  fe_to_words(P.X, wx);
  fe_to_words(P.Y, wy);
  words_to_bytes(wx, out);
  words_to_bytes(wy, out + 32);
  return ok ? 1 : 0;
}

// out = compress(8 * (decompress(a) + decompress(b))) and compress(a + b), compress(2a)
int hc_point_ops(const uint8_t* a, const uint8_t* b, uint8_t* sum, uint8_t* dbl, uint8_t* madd,
                 uint8_t* cof) {
  uint32_t wa[8], wb[8], w[8];
  bytes_to_words(a, wa);
  bytes_to_words(b, wb);
  ge_p3 P, Q;
  if (!ge_decompress(wa, P) || !ge_decompress(wb, Q)) return 0;
  ge_compress(ge_add(P, Q), w); words_to_bytes(w, sum);
  ge_compress(ge_dbl(P), w); words_to_bytes(w, dbl);
  ge_compress(ge_madd(P, ge_to_niels_affine(Q)), w); words_to_bytes(w, madd);
  ge_compress(ge_mul_by_cofactor(P), w); words_to_bytes(w, cof);
  return 1;
}

// out = compress(a + b) or compress(a - b) through ge_madd_sgn (the accumulation's signed
// mixed addition), after `pre` doublings of a (so the accumulator is a projective point)
int hc_point_madd_sgn(const uint8_t* a, const uint8_t* b, int neg, int pre, uint8_t* out) {
  uint32_t wa[8], wb[8], w[8];
  bytes_to_words(a, wa);
  bytes_to_words(b, wb);
  ge_p3 P, Q;
  if (!ge_decompress(wa, P) || !ge_decompress(wb, Q)) return 0;
  for (int i = 0; i < pre; ++i) P = ge_dbl(P);
  ge_compress(ge_madd_sgn(P, ge_to_niels_affine(Q), neg != 0), w);
  words_to_bytes(w, out);
  return 1;
}

// fe_sub_lazy(a, b) limbs (a, b raw limbs)
void hc_fe_sub_lazy(const uint32_t* a, const uint32_t* b, uint32_t* out) {
  fe x, y;
  for (int i = 0; i < 9; ++i) { x.v[i] = a[i]; y.v[i] = b[i]; }
  fe r = fe_sub_lazy(x, y);
  for (int i = 0; i < 9; ++i) out[i] = r.v[i];
}

void hc_sha512(const uint8_t* head0, const uint8_t* head1, const uint8_t* msg, uint64_t mlen,
               uint8_t* out) {
  sha_src s{head0, head1, msg, mlen};
  sha512_src(s, out);
}

void hc_challenge(const uint8_t* R, const uint8_t* A, const uint8_t* msg, uint64_t mlen,
                  uint8_t* k_out) {
  uint8_t d[64];
  sha_src s{R, A, msg, mlen};
  sha512_src(s, d);
  sc k = sc_from_digest(d);
  words_to_bytes(k.v, k_out);
}

void hc_sc_reduce_wide(const uint8_t* x64, uint8_t* out) {
  sc k = sc_from_digest(x64);
  words_to_bytes(k.v, out);
}

// op 0 mul, 1 add, 2 sub, 3 mul128 (a's low 16 bytes)
void hc_sc_op(int op, const uint8_t* a, const uint8_t* b, uint8_t* out) {
  sc x, y, r;
  bytes_to_words(a, x.v);
  bytes_to_words(b, y.v);
  switch (op) {
    case 0: r = sc_mul(x, y); break;
    case 1: r = sc_add(x, y); break;
    case 2: r = sc_sub(x, y); break;
    default: r = sc_mul128(x.v, y); break;
  }
  words_to_bytes(r.v, out);
}

int hc_sc_is_canonical(const uint8_t* s) {
  uint32_t w[8];
  bytes_to_words(s, w);
  return sc_is_canonical(w) ? 1 : 0;
}

void hc_chacha_block(const uint8_t* key, uint64_t counter, uint8_t* out) {
  uint32_t k[8], o[16];
  bytes_to_words(key, k);
  chacha20_block(k, counter, o);
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 4; ++j) out[4 * i + j] = (uint8_t)(o[i] >> (8 * j));
}

}  // extern "C"
