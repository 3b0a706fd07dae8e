// 4-lane cooperative point arithmetic for the latency-bound parts of the MSM (bucket / slice /
// window reductions and the final Horner pass). The 4 lanes of a quad (lane & 3) hold the same
// point; in each of the two multiplication rounds of a formula every lane computes ONE of the
// four independent field multiplications, and DPP quad_perm broadcasts (v_mov_b32 dpp, no LDS)
// hand the four products to all lanes. Serial depth per doubling / addition drops from 8-9
// multiplications to 2 (+1 for the cached-form conversion of a general addition).
#pragma once
#include <hip/hip_runtime.h>
#include "ge25519.h"

namespace edc {

__device__ __forceinline__ int quad_lane() { return (int)(threadIdx.x & 3u); }

template <int J>
__device__ __forceinline__ uint32_t quad_bcast(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, J * 0x55, 0xF, 0xF, true);
}

__device__ __forceinline__ void quad_gather(const fe& mine, fe& r0, fe& r1, fe& r2, fe& r3) {
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    r0.v[i] = quad_bcast<0>(mine.v[i]);
    r1.v[i] = quad_bcast<1>(mine.v[i]);
    r2.v[i] = quad_bcast<2>(mine.v[i]);
    r3.v[i] = quad_bcast<3>(mine.v[i]);
  }
}

__device__ __forceinline__ fe quad_pick(int q, const fe& a0, const fe& a1, const fe& a2, const fe& a3) {
  fe r;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    uint32_t x = q == 0 ? a0.v[i] : a1.v[i];
    uint32_t y = q == 2 ? a2.v[i] : a3.v[i];
    r.v[i] = q < 2 ? x : y;
  }
  return r;
}

// 2P (dalek double through the completed form), T3 always produced
__device__ __forceinline__ ge_p3 quad_dbl(const ge_p3& P) {
  const int q = quad_lane();
  fe in = quad_pick(q, P.X, P.Y, P.Z, fe_add(P.X, P.Y));
  fe s = fe_sqr(in);
  fe XX, YY, ZZ, XpY2;
  quad_gather(s, XX, YY, ZZ, XpY2);
  fe ZZ2 = fe_add(ZZ, ZZ);
  fe Yc = fe_add(YY, XX);
  fe Zc = fe_sub(YY, XX);
  fe Xc = fe_sub(XpY2, Yc);
  fe Tc = fe_sub(ZZ2, Zc);
  // X3 = Xc Tc, Y3 = Yc Zc, Z3 = Zc Tc, T3 = Xc Yc
  fe a = quad_pick(q, Xc, Yc, Zc, Xc);
  fe b = quad_pick(q, Tc, Zc, Tc, Yc);
  fe m = fe_mul(a, b);
  ge_p3 r;
  quad_gather(m, r.X, r.Y, r.Z, r.T);
  return r;
}

// P + Q, Q in projective Niels (cached) form
__device__ __forceinline__ ge_p3 quad_add_cached(const ge_p3& P, const ge_cached& Q) {
  const int q = quad_lane();
  fe a = quad_pick(q, fe_sub(P.Y, P.X), fe_add(P.Y, P.X), P.T, P.Z);
  fe b = quad_pick(q, Q.ymx, Q.ypx, Q.T2d, Q.Z);
  fe m = fe_mul(a, b);
  fe A, B, C, ZZ;
  quad_gather(m, A, B, C, ZZ);
  fe D = fe_add_c(ZZ, ZZ);
  fe E = fe_sub(B, A), F = fe_sub(D, C), G = fe_add(D, C), H = fe_add(B, A);
  // X3 = E F, Y3 = G H, Z3 = F G, T3 = E H
  fe a2 = quad_pick(q, E, G, F, E);
  fe b2 = quad_pick(q, F, H, G, H);
  fe m2 = fe_mul(a2, b2);
  ge_p3 r;
  quad_gather(m2, r.X, r.Y, r.Z, r.T);
  return r;
}

// P + Q, Q affine Niels (Z2 = 1): three products in the first round (lane 3 repeats lane 2's)
__device__ __forceinline__ ge_p3 quad_madd(const ge_p3& P, const ge_niels& Q) {
  const int q = quad_lane();
  fe a = quad_pick(q, fe_sub(P.Y, P.X), fe_add(P.Y, P.X), P.T, P.T);
  fe b = quad_pick(q, Q.ymx, Q.ypx, Q.xy2d, Q.xy2d);
  fe m = fe_mul(a, b);
  fe A, B, C, C2;
  quad_gather(m, A, B, C, C2);
  fe D = fe_add_c(P.Z, P.Z);
  fe E = fe_sub(B, A), F = fe_sub(D, C), G = fe_add(D, C), H = fe_add(B, A);
  fe a2 = quad_pick(q, E, G, F, E);
  fe b2 = quad_pick(q, F, H, G, H);
  fe m2 = fe_mul(a2, b2);
  ge_p3 r;
  quad_gather(m2, r.X, r.Y, r.Z, r.T);
  return r;
}

// the point held by lane J of each quad, on every lane of the quad
template <int J>
__device__ __forceinline__ ge_p3 quad_bcast_point(const ge_p3& P) {
  ge_p3 r;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    r.X.v[i] = quad_bcast<J>(P.X.v[i]);
    r.Y.v[i] = quad_bcast<J>(P.Y.v[i]);
    r.Z.v[i] = quad_bcast<J>(P.Z.v[i]);
    r.T.v[i] = quad_bcast<J>(P.T.v[i]);
  }
  return r;
}

// P + Q, both extended (one extra multiplication round for T2 * 2d)
__device__ __forceinline__ ge_p3 quad_add(const ge_p3& P, const ge_p3& Q) {
  ge_cached c;
  c.ypx = fe_add_c(Q.Y, Q.X);
  c.ymx = fe_sub(Q.Y, Q.X);
  c.Z = Q.Z;
  c.T2d = fe_mul(Q.T, fe_d2());
  return quad_add_cached(P, c);
}

// ---- distributed layout, for long serial chains (Horner, window combines) ----
// Lane q of the quad holds ONE coordinate of the point (0: X, 1: Y, 2: Z, 3: T). The second
// multiplication round of a doubling or addition then leaves each lane with exactly its own new
// coordinate, so the final four-way broadcast of the replicated form (36 DPP moves) and the
// four-way operand selects (27 v_cndmask each) disappear: every lane picks its operands from two
// candidates under a fixed lane mask. Same formulas as quad_dbl / quad_add_cached, so every
// coordinate is the same field element (the canonical bytes of a result are unchanged).
struct quad_pt {
  fe c;
};

__device__ __forceinline__ quad_pt quad_distribute(const ge_p3& P) {
  return {quad_pick(quad_lane(), P.X, P.Y, P.Z, P.T)};
}

__device__ __forceinline__ ge_p3 quad_collect(const quad_pt& p) {
  ge_p3 r;
  quad_gather(p.c, r.X, r.Y, r.Z, r.T);
  return r;
}

__device__ __forceinline__ fe fe_sel(bool c, const fe& a, const fe& b) {
  fe r;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = c ? a.v[i] : b.v[i];
  return r;
}

// 2P: lanes square X, Y, Z, (X+Y) (lane 3 drops T), then X3 = Xc Tc, Y3 = Yc Zc, Z3 = Zc Tc,
// T3 = Xc Yc (quad_dbl's completed-form values) with a = (lane 1, 2 ? Zc : Xc) and
// b = (odd lane ? Yc : Tc)
__device__ __forceinline__ quad_pt quad_dbl_d(const quad_pt& p) {
  const int q = quad_lane();
  fe x, y;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    x.v[i] = quad_bcast<0>(p.c.v[i]);
    y.v[i] = quad_bcast<1>(p.c.v[i]);
  }
  const fe s = fe_sqr(fe_sel(q == 3, fe_add(x, y), p.c));
  // each lane forms only its two operands: a = u - v with u = (X+Y)^2 on lanes 0, 3 and Y^2 on
  // lanes 1, 2 (one quad_perm [3,1,1,3] move per limb), v = Yc = Y^2 + X^2 or X^2, so a = Xc or
  // Zc; b = X^2 + (odd lane ? Y^2 : 2Z^2 - Y^2), i.e. Yc or Tc = 2Z^2 - Zc
  fe XX, YY, ZZ, u;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    XX.v[i] = quad_bcast<0>(s.v[i]);
    YY.v[i] = quad_bcast<1>(s.v[i]);
    ZZ.v[i] = quad_bcast<2>(s.v[i]);
    u.v[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)s.v[i], 3 | (1 << 2) | (1 << 4) | (3 << 6), 0xF, 0xF, true);
  }
  const bool mid = q == 1 || q == 2, odd = (q & 1) != 0;
  const fe a = fe_sub(u, fe_sel(mid, XX, fe_add(YY, XX)));
  const fe b = fe_add(XX, fe_sel(odd, YY, fe_sub(fe_add(ZZ, ZZ), YY)));
  return {fe_mul(a, b)};
}

// P + Q, Q extended and replicated on the quad's lanes: first round A = (Y1-X1)(Y2-X2),
// B = (Y1+X1)(Y2+X2), lane 2 Z1 Z2, lane 3 T1 (2d T2); then X3 = E F, Y3 = G H, Z3 = F G,
// T3 = E H with a = (lane 1, 2 ? G : E) and b = (odd lane ? H : F)
__device__ __forceinline__ quad_pt quad_add_d(const quad_pt& p, const ge_p3& Q) {
  const int q = quad_lane();
  fe x, y;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    x.v[i] = quad_bcast<0>(p.c.v[i]);
    y.v[i] = quad_bcast<1>(p.c.v[i]);
  }
  const fe qymx = fe_sub(Q.Y, Q.X), qypx = fe_add_c(Q.Y, Q.X);
  const fe qt2d = fe_mul(Q.T, fe_d2());
  const fe a = fe_sel(q == 0, fe_sub(y, x), fe_sel(q == 1, fe_add(y, x), p.c));
  const fe b = fe_sel(q == 0, qymx, fe_sel(q == 1, qypx, fe_sel(q == 2, Q.Z, qt2d)));
  const fe m = fe_mul(a, b);
  fe A, B, ZZ, C;
  quad_gather(m, A, B, ZZ, C);
  const fe D = fe_add_c(ZZ, ZZ);
  const fe E = fe_sub(B, A), F = fe_sub(D, C), G = fe_add(D, C), H = fe_add(B, A);
  const bool mid = q == 1 || q == 2, odd = (q & 1) != 0;
  return {fe_mul(fe_sel(mid, G, E), fe_sel(odd, H, F))};
}

}  // namespace edc
