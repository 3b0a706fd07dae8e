// Latency-shaped GF(2^255-19) multiplication and squaring, an experiment for the serial tails of
// the MSM (the Horner pass, window combines): one wave runs a long chain of dependent point
// operations there. MEASURED SLOWER than the product's fe_mul / fe_sqr even on one wave
// (profiles/r02_lat_probe.txt: 993 vs 777 cycles per product, 769 vs 601 per square): a lone
// wave64 is issue-bound on gfx950 (a v_mad_u64_u32 costs its issue slots whether or not the next
// one depends on it), so the extra instructions cost more than the shorter chains save. Kept
// with tools/microbench/lat_probe.hip as the record; not used by the library.
//
// fe_mul / fe_sqr (fe25519.h) are shaped for throughput: the low columns run as ONE chain of
// ~61 v_mad_u64_u32 through the carry addend (no carry instructions at all), which is ideal with
// many waves per SIMD and slow with one. Here every column is its own chain (depth <= 9 for a
// product, <= 5 for a square), the high columns are folded into the low ones by two mads each
// (2^261 == 1216 mod p), and the carries run in two parallel rounds: each 64-bit column splits
// into 29-bit digits x + y 2^29 + z 2^58 that are added three at a time into the limbs, then one
// more round of (limb & M29) + (previous limb >> 29). About 30 more instructions per operation,
// roughly a third of the dependency depth.
//
// Same contract as fe_mul / fe_sqr: inputs are mul inputs (limbs < 2^30.41), outputs reduced
// (limbs < 2^29 + 2^19), value congruent mod p (lat_probe's k_check compares them on the GPU).
#pragma once
#include "fe25519.h"

namespace edc {

// 9 low columns c[0..8] (< 2^64 each, high columns already folded) -> reduced limbs
EDC_HD fe fe_carry_cols(const uint64_t c[9]) {
  uint32_t x[9], y[9], z[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    x[k] = (uint32_t)c[k] & M29;
    y[k] = (uint32_t)(c[k] >> 29) & M29;
    z[k] = (uint32_t)(c[k] >> 58);
  }
  // r_k = x_k + y_{k-1} + z_{k-2} (< 2^30.01); r_9 = y_8 + z_7 and r_10 = z_8 sit at 2^261, 2^290
  uint32_t r[9];
  r[0] = x[0];
  r[1] = x[1] + y[0];
#pragma unroll
  for (int k = 2; k < 9; ++k) r[k] = x[k] + y[k - 1] + z[k - 2];
  const uint32_t r9 = y[8] + z[7], r10 = z[8];
  const uint64_t t0 = mad64(r9, 1216u, (uint64_t)r[0]);          // < 2^39.3
  r[0] = (uint32_t)t0 & M29;
  r[1] += (uint32_t)(t0 >> 29) + r10 * 1216u;                   // + < 2^10.3 + < 2^16.3
  // one parallel carry round: limbs < 2^30.02 -> < 2^29 + 2 (limb 0: + 2 * 1216)
  fe o;
  o.v[0] = r[0] + (r[8] >> 29) * 1216u;
#pragma unroll
  for (int k = 1; k < 9; ++k) o.v[k] = (r[k] & M29) + (r[k - 1] >> 29);
  return o;
}

// high columns 9..16 folded into the low ones: lo32(c_{k+9}) * 1216 at k, hi32(c_{k+8}) * 9728
// (= 2^32 * 1216 / 2^29) at k; both mads go last in a column so its products do not wait for them
EDC_HD void fe_fold_cols(uint64_t c[17]) {
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    if (k < 8) c[k] = mad64((uint32_t)c[k + 9], 1216u, c[k]);
    if (k >= 1) c[k] = mad64((uint32_t)(c[k + 8] >> 32), 9728u, c[k]);
  }
}

// a * b; column k = sum_{i+j=k} a_i b_j (<= 9 products < 2^60.82 each, + folds < 2^45.3: < 2^64)
EDC_HD fe fe_mul_lat(const fe& a, const fe& b) {
  uint64_t c[17];
#pragma unroll
  for (int k = 0; k < 17; ++k) {
    const int i0 = k < 9 ? 0 : k - 8, i1 = k < 9 ? k : 8;
    uint64_t s = mul64(a.v[i0], b.v[k - i0]);
#pragma unroll
    for (int i = i0 + 1; i <= i1; ++i) s = mad64(a.v[i], b.v[k - i], s);
    c[k] = s;
  }
  fe_fold_cols(c);
  return fe_carry_cols(c);
}

// a^2; column k = sum_{i<j, i+j=k} a_i (2 a_j) + a_{k/2}^2 (<= 4 products < 2^61.82 + one < 2^60.82)
EDC_HD fe fe_sqr_lat(const fe& a) {
  uint32_t d[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) d[i] = a.v[i] << 1;
  uint64_t c[17];
#pragma unroll
  for (int k = 0; k < 17; ++k) {
    const int i0 = k < 9 ? 0 : k - 8;
    uint64_t s = (k & 1) ? 0ull : mul64(a.v[k / 2], a.v[k / 2]);
#pragma unroll
    for (int i = i0; 2 * i < k; ++i) s = mad64(a.v[i], d[k - i], s);
    c[k] = s;
  }
  fe_fold_cols(c);
  return fe_carry_cols(c);
}

}  // namespace edc
