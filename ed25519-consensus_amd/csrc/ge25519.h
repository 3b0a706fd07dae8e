// Edwards25519 group arithmetic (twisted Edwards, a = -1) in extended coordinates on top of
// fe25519.h. All formulas are complete (no exceptional cases), so one lane = one point with no
// data-dependent branches except the ZIP215 decode verdict.
//
// Restates, for the verification path of ed25519-consensus 2.1.0:
//   CompressedEdwardsY::decompress  (reference src/batch.rs:183-185, :190-192,
//                                    src/verification_key.rs:166-168, :242-244)
//   EdwardsPoint::compress / mul_by_cofactor / is_identity (src/batch.rs:212,
//                                    src/verification_key.rs:253)
#pragma once
#include "fe25519.h"

namespace edc {

struct ge_p3 { fe X, Y, Z, T; };          // extended: x = X/Z, y = Y/Z, xy = T/Z
struct ge_niels { fe ypx, ymx, xy2d; };   // affine Niels: (y+x, y-x, 2dxy), Z = 1
struct ge_cached { fe ypx, ymx, Z, T2d; };// projective Niels

EDC_HD ge_p3 ge_identity() {
  ge_p3 r; r.X = fe_zero(); r.Y = fe_one(); r.Z = fe_one(); r.T = fe_zero(); return r;
}

EDC_HD ge_niels ge_niels_identity() {
  ge_niels r; r.ypx = fe_one(); r.ymx = fe_one(); r.xy2d = fe_zero(); return r;
}

// dalek FieldElement::sqrt_ratio_i as decoding uses it. Returns was_nonzero_square (or u == 0);
// when it holds, r is a root of u/v of either sign (ge_decompress fixes the sign in the same
// select that applies the encoding's sign bit). dalek's third test (check == -u sqrt(-1)) only
// changes r when the result is rejected, so it is not computed.
EDC_HD bool fe_sqrt_ratio_i(const fe& u, const fe& v, fe& r) {
  const fe v2 = fe_sqr(v);
  const fe uv3 = fe_mul(u, fe_mul(v2, v));
  const fe uv7 = fe_mul(uv3, fe_sqr(v2));             // u v^3 * v^4: one multiplication fewer than u * v^7
  r = fe_mul(uv3, fe_pow_p58(uv7));
  fe check = fe_mul(v, fe_sqr(r));
  // a == b (mod p) tested as canon(a - b) == 0: one canonicalisation per test instead of two
  bool correct = fe_is_zero(fe_sub(check, u));                        // check == u
  bool flipped = fe_is_zero(fe_add(check, u));                        // check == -u
  r = fe_select(r, fe_mul(fe_sqrtm1(), r), flipped);
  return correct || flipped;
}

// ZIP215 decode: y = bytes & (2^255-1) (NOT reduced), x from sqrt_ratio_i, negative iff bit 255.
// Returns false iff the y coordinate is not on the curve.
EDC_HD bool ge_decompress(const uint32_t w[8], ge_p3& P) {
  fe Y = fe_from_words(w);
  fe one = fe_one();
  fe YY = fe_sqr(Y);
  fe u = fe_sub(YY, one);
  fe v = fe_add_c(fe_mul(YY, fe_d()), one);
  fe X;
  bool ok = fe_sqrt_ratio_i(u, v, X);
  const bool sign = (w[7] >> 31) != 0;
  X = fe_select(X, fe_neg(X), fe_is_negative(X) != sign);   // |x|, then negated iff the sign bit
  P.X = X;
  P.Y = fe_carry(Y);
  P.Z = one;
  P.T = fe_mul(X, Y);
  return ok;
}

EDC_HD ge_niels ge_to_niels_affine(const ge_p3& P) {  // requires Z == 1
  ge_niels n;
  n.ypx = fe_add_c(P.Y, P.X);
  n.ymx = fe_sub(P.Y, P.X);
  n.xy2d = fe_mul(P.T, fe_d2());
  return n;
}

EDC_HD ge_cached ge_to_cached(const ge_p3& P) {
  ge_cached c;
  c.ypx = fe_add_c(P.Y, P.X);
  c.ymx = fe_sub(P.Y, P.X);
  c.Z = P.Z;
  c.T2d = fe_mul(P.T, fe_d2());
  return c;
}

EDC_HD ge_niels ge_niels_neg(const ge_niels& n) {
  ge_niels r; r.ypx = n.ymx; r.ymx = n.ypx; r.xy2d = fe_neg(n.xy2d); return r;
}

EDC_HD ge_cached ge_cached_neg(const ge_cached& n) {
  ge_cached r; r.ypx = n.ymx; r.ymx = n.ypx; r.Z = n.Z; r.T2d = fe_neg(n.T2d); return r;
}

EDC_HD ge_p3 ge_neg(const ge_p3& P) {
  ge_p3 r; r.X = fe_neg(P.X); r.Y = P.Y; r.Z = P.Z; r.T = fe_neg(P.T); return r;
}

// Scheduling fence between the multiplications of a point formula on the device: the seven
// products of a mixed addition are independent, and interleaving them lets the scheduler keep
// several 17-column accumulators live at once, which spills at 4 waves/SIMD (128 VGPRs).
#if defined(__HIP_DEVICE_COMPILE__)
#define EDC_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define EDC_SCHED_FENCE() ((void)0)
#endif

// Carry passes in the addition formulas. E, F, G, H each meet two others in X3 = EF, Y3 = GH,
// T3 = EH, Z3 = FG (a 4-cycle), so carrying F and H alone puts a reduced operand in every
// product; E = B - A and G = D +- C stay lazy (fe_sub_lazy bound), as does Y1 - X1 against the
// reduced record half and D = 2 Z1. Two carry passes per addition instead of four. Inputs: P's
// coordinates and the record's fields reduced (every producer ends in fe_mul / fe_sub / fe_add_c).
// P + Q, Q affine Niels: 7M
EDC_HD ge_p3 ge_madd(const ge_p3& P, const ge_niels& q) {
  fe A = fe_mul(fe_sub_lazy(P.Y, P.X), q.ymx);
  EDC_SCHED_FENCE();
  fe B = fe_mul(fe_add(P.Y, P.X), q.ypx);
  EDC_SCHED_FENCE();
  fe C = fe_mul(P.T, q.xy2d);
  EDC_SCHED_FENCE();
  fe D = fe_add(P.Z, P.Z);
  fe E = fe_sub_lazy(B, A), F = fe_sub(D, C), G = fe_add(D, C), H = fe_add_c(B, A);
  ge_p3 r;
  r.X = fe_mul(E, F);
  EDC_SCHED_FENCE();
  r.Y = fe_mul(G, H);
  EDC_SCHED_FENCE();
  r.T = fe_mul(E, H);
  EDC_SCHED_FENCE();
  r.Z = fe_mul(F, G);
  return r;
}

// P + Q, Q projective Niels: 8M
EDC_HD ge_p3 ge_add_cached(const ge_p3& P, const ge_cached& q) {
  fe A = fe_mul(fe_sub_lazy(P.Y, P.X), q.ymx);
  EDC_SCHED_FENCE();
  fe B = fe_mul(fe_add(P.Y, P.X), q.ypx);
  EDC_SCHED_FENCE();
  fe C = fe_mul(P.T, q.T2d);
  EDC_SCHED_FENCE();
  fe ZZ = fe_mul(P.Z, q.Z);
  fe D = fe_add(ZZ, ZZ);
  fe E = fe_sub_lazy(B, A), F = fe_sub(D, C), G = fe_add(D, C), H = fe_add_c(B, A);
  ge_p3 r;
  r.X = fe_mul(E, F);
  EDC_SCHED_FENCE();
  r.Y = fe_mul(G, H);
  EDC_SCHED_FENCE();
  r.T = fe_mul(E, H);
  EDC_SCHED_FENCE();
  r.Z = fe_mul(F, G);
  return r;
}

// P + Q (neg = false) or P - Q (neg = true), Q affine Niels: 7M. -Q is (y-x, y+x, -2dxy), so
// the sign only swaps which of Y-X, Y+X meets which record half, and F / G (C changes sign):
// 36 selects instead of ge_niels_neg's swap, negation and select of the whole record.
EDC_HD ge_p3 ge_madd_sgn(const ge_p3& P, const ge_niels& q, bool neg) {
  const fe ym = fe_select(q.ymx, q.ypx, neg), yp = fe_select(q.ypx, q.ymx, neg);
  fe A = fe_mul(fe_sub_lazy(P.Y, P.X), ym);
  EDC_SCHED_FENCE();
  fe B = fe_mul(fe_add(P.Y, P.X), yp);
  EDC_SCHED_FENCE();
  fe C = fe_mul(P.T, q.xy2d);
  EDC_SCHED_FENCE();
  fe D = fe_add(P.Z, P.Z);
  fe E = fe_sub_lazy(B, A), H = fe_add_c(B, A);
  const fe dmc = fe_sub_lazy(D, C), dpc = fe_add(D, C);
  // F (carried) is D - C, or D + C for -Q; G keeps the other one lazy
  fe F = fe_carry(fe_select(dmc, dpc, neg)), G = fe_select(dpc, dmc, neg);
  ge_p3 r;
  r.X = fe_mul(E, F);
  EDC_SCHED_FENCE();
  r.Y = fe_mul(G, H);
  EDC_SCHED_FENCE();
  r.T = fe_mul(E, H);
  EDC_SCHED_FENCE();
  r.Z = fe_mul(F, G);
  return r;
}

// P + Q both extended: 9M
EDC_HD ge_p3 ge_add(const ge_p3& P, const ge_p3& Q) { return ge_add_cached(P, ge_to_cached(Q)); }

// 2P: 4S + 4M (dalek ProjectivePoint::double through the completed form). with_t=false
// skips T3 for chains of doublings whose T is never read.
EDC_HD ge_p3 ge_dbl(const ge_p3& P, bool with_t = true) {
  fe XX = fe_sqr(P.X);
  EDC_SCHED_FENCE();
  fe YY = fe_sqr(P.Y);
  EDC_SCHED_FENCE();
  fe ZZ = fe_sqr(P.Z);
  EDC_SCHED_FENCE();
  fe ZZ2 = fe_add(ZZ, ZZ);
  fe XpY2 = fe_sqr(fe_add(P.X, P.Y));
  fe Yc = fe_add(YY, XX);
  fe Zc = fe_sub(YY, XX);
  fe Xc = fe_sub(XpY2, Yc);
  fe Tc = fe_sub_lazy(ZZ2, Zc);     // lazy: meets only Xc and Zc (both carried)
  ge_p3 r;
  r.X = fe_mul(Xc, Tc);
  EDC_SCHED_FENCE();
  r.Y = fe_mul(Yc, Zc);
  EDC_SCHED_FENCE();
  r.Z = fe_mul(Zc, Tc);
  r.T = with_t ? fe_mul(Xc, Yc) : fe_zero();
  return r;
}

EDC_HD ge_p3 ge_mul_by_cofactor(const ge_p3& P) {
  return ge_dbl(ge_dbl(ge_dbl(P, false), false), true);
}

// dalek IsIdentity on EdwardsPoint: X == 0 and Y == Z (projective). Z != 0 is also required:
// every point the complete formulas produce from curve points has Z != 0, so the degenerate
// (0 : 0 : 0 : 0) can only come from a fault and must never read as the identity.
EDC_HD bool ge_is_identity(const ge_p3& P) {
  return fe_is_zero(P.X) && fe_eq(P.Y, P.Z) && !fe_is_zero(P.Z);
}

EDC_HD void ge_compress(const ge_p3& P, uint32_t w[8]) {
  fe zi = fe_invert(P.Z);
  fe x = fe_mul(P.X, zi);
  fe y = fe_mul(P.Y, zi);
  fe_to_words(y, w);
  w[7] |= (uint32_t)fe_is_negative(x) << 31;
}

// ed25519 basepoint B (y = 4/5, x positive)
EDC_HD ge_p3 ge_basepoint() {
  ge_p3 B;
  B.X = fe_const(0x8f25d51au, 0xc9562d60u, 0x9525a7b2u, 0x692cc760u, 0xfdd6dc5cu, 0xc0a4e231u,
                 0xcd6e53feu, 0x216936d3u);
  B.Y = fe_const(0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u,
                 0x66666666u, 0x66666666u);
  B.Z = fe_one();
  B.T = fe_mul(B.X, B.Y);
  return B;
}

}  // namespace edc
