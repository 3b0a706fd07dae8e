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
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, J * 0x55, 0xF, 0xF, false);
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

}  // namespace edc
