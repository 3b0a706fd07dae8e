// Per-signature kernels:
//   k_verify_single  VerificationKey::try_from + verify_prehashed, one lane per item (K5):
//                    the fallback after a failed batch (reference src/batch.rs:104-107,
//                    src/verification_key.rs:160-175, :237-258)
//   k_sign           SigningKey::from(seed) + sign (test-data source only; reference
//                    src/signing_key.rs) -- synthetic batches are generated on the GPU
//   k_decode         CompressedEdwardsY::decompress for the API (canonical x||y + verdict)
#include "edc_common.h"
#include "edc_launch.h"
#include "ge_quad.h"

namespace edc {

__device__ __forceinline__ ge_niels to_niels(const ge_p3& P) {  // x = X/Z, y = Y/Z
  fe zi = fe_invert(P.Z);
  ge_p3 a;
  a.X = fe_mul(P.X, zi); a.Y = fe_mul(P.Y, zi); a.Z = fe_one(); a.T = fe_mul(a.X, a.Y);
  return ge_to_niels_affine(a);
}

// context constants as affine Niels: [i]B for i = 1..8 (entries 0..7)
__global__ void k_init_btable(uint32_t* btab) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  ge_p3 B = ge_basepoint();
  ge_p3 acc = B;
  for (int i = 0; i < BTAB_ENTRIES; ++i) {
    st_niels(btab, i, to_niels(acc));
    acc = ge_add(acc, B);
  }
}

// signed radix-16 digits of a scalar < 2^255, 64 digits in [-7, 8]
__device__ __forceinline__ void radix16(const uint32_t s[8], int8_t d[64]) {
  int carry = 0;
  for (int j = 0; j < 64; ++j) {
    int v = (int)((s[j >> 3] >> (4 * (j & 7))) & 15u) + carry;
    if (j < 63 && v > 8) { v -= 16; carry = 1; } else { carry = 0; }
    d[j] = (int8_t)v;
  }
}

// the same recoding without a digit array: bit j of the mask is the carry out of position j
// (digit j was lowered by 16); digit j = nibble j + carry in - 16 carry out
__device__ __forceinline__ uint64_t radix16_carries(const uint32_t s[8]) {
  uint64_t m = 0;
  uint32_t carry = 0;
  for (int j = 0; j < 63; ++j) {
    const uint32_t v = ((s[j >> 3] >> (4 * (j & 7))) & 15u) + carry;
    carry = v > 8;
    m |= (uint64_t)carry << j;
  }
  return m;
}
// s[w] for a runtime w as a select chain (a runtime-indexed register array goes to scratch)
__device__ __forceinline__ uint32_t word_at(const uint32_t s[8], int w) {
  uint32_t r = s[0];
#pragma unroll
  for (int q = 1; q < 8; ++q) r = w == q ? s[q] : r;
  return r;
}
__device__ __forceinline__ int radix16_digit(const uint32_t s[8], uint64_t carries, int j) {
  const int nib = (int)((word_at(s, j >> 3) >> (4 * (j & 7))) & 15u);
  const int cin = j ? (int)((carries >> (j - 1)) & 1) : 0;
  return nib + cin - 16 * (int)((carries >> j) & 1);
}

// signed radix-256 digits of a scalar whose top byte is <= 127 (s < l; a clamped secret scalar,
// bit 255 clear): 32 digits in [-127, 128], no carry out of byte 31; bit j of the
// mask is the carry out of byte j (the digit was lowered by 256)
__device__ __forceinline__ uint32_t radix256_carries(const uint32_t s[8]) {
  uint32_t m = 0, carry = 0;
  for (int j = 0; j < 31; ++j) {
    const uint32_t v = ((s[j >> 2] >> (8 * (j & 3))) & 255u) + carry;
    carry = v > 128;
    m |= carry << j;
  }
  return m;
}
__device__ __forceinline__ int radix256_digit(const uint32_t s[8], uint32_t carries, int j) {
  const int byte = (int)((word_at(s, j >> 2) >> (8 * (j & 3))) & 255u);
  const int cin = j ? (int)((carries >> (j - 1)) & 1u) : 0;
  return byte + cin - 256 * (int)((carries >> j) & 1u);
}
// acc + [s]B from the radix-256 comb (btab entries BTAB_ENTRIES..): 32 signed additions
__device__ __forceinline__ ge_p3 add_base_comb(ge_p3 acc, const uint32_t s[8], const uint32_t* __restrict__ btab) {
  const uint32_t sc = radix256_carries(s);
  const uint32_t* comb = btab + (size_t)BTAB_ENTRIES * NIELS_WORDS;
  for (int j = 0; j < B256_POS; ++j) {
    const int b = radix256_digit(s, sc, j);
    const int bi = b < 0 ? -b : b;
    const ge_niels nb = bi ? ld_niels(comb, j * B256_MULT + bi - 1) : ge_niels_identity();
    acc = ge_madd_sgn(acc, nb, b < 0);
  }
  return acc;
}

__device__ __forceinline__ ge_cached cached_identity() {
  ge_cached c; c.ypx = fe_one(); c.ymx = fe_one(); c.Z = fe_one(); c.T2d = fe_zero(); return c;
}

__device__ __forceinline__ void st_cached(uint32_t* p, const ge_cached& c) {
  st_fe(p, c.ypx); st_fe(p + 9, c.ymx); st_fe(p + 18, c.Z); st_fe(p + 27, c.T2d);
}
__device__ __forceinline__ ge_cached ld_cached(const uint32_t* p) {
  ge_cached c; c.ypx = ld_fe(p); c.ymx = ld_fe(p + 9); c.Z = ld_fe(p + 18); c.T2d = ld_fe(p + 27); return c;
}

constexpr int SV_THREADS = 256;
constexpr int SV_TAB_WORDS = 9 * EXT_WORDS;   // per-item [1..8]P (projective Niels) + R parked

// R' = [k]P + [s]B, signed radix-16 windows. P's table of 8 cached multiples lives in the
// item's global scratch record (LDS for 8 x 144 bytes per lane held 0.5 waves per SIMD); B's
// affine Niels multiples come from the context table.
__device__ ge_p3 double_scalar_mul(const uint32_t k[8], const ge_p3& P, const uint32_t s[8],
                                   const uint32_t* btab, uint32_t* tab) {
  ge_cached c = ge_to_cached(P);
  ge_p3 acc = P;
  st_cached(tab, c);
  for (int i = 1; i < 8; ++i) {
    acc = ge_add_cached(acc, c);
    st_cached(tab + i * EXT_WORDS, ge_to_cached(acc));
  }
  const uint64_t kc = radix16_carries(k);
  acc = ge_identity();
  for (int j = 63; j >= 0; --j) {
    if (j != 63) {
      acc = ge_dbl(acc, false);
      acc = ge_dbl(acc, false);
      acc = ge_dbl(acc, false);
      acc = ge_dbl(acc, true);
    }
    int a = radix16_digit(k, kc, j);
    int ai = a < 0 ? -a : a;
    ge_cached q = ai ? ld_cached(tab + (ai - 1) * EXT_WORDS) : cached_identity();
    if (a < 0) q = ge_cached_neg(q);
    acc = ge_add_cached(acc, q);
  }
  return add_base_comb(acc, s, btab);                // [s]B: 32 comb additions, no doublings
}

// verdict codes: 0 Ok, 1 InvalidSignature, 2 MalformedPublicKey
// Cached key (keycache.h): [s]B - [k]A from comb tables and NO doublings (the joint windowed
// loop below needs 252): -[k]A over the key's 64 radix-16 positions, [s]B over B's 32 radix-256
// positions (btab). One affine Niels record per digit; zero digits add the identity
// (branch-free across the wave).
__device__ ge_p3 comb_double_base(const uint32_t k[8], const uint32_t s[8], const uint32_t* __restrict__ acomb,
                                  const uint32_t* __restrict__ btab) {
  const uint64_t kc = radix16_carries(k);
  ge_p3 acc = ge_identity();
  for (int j = 0; j < COMB_POS; ++j) {
    const int a = radix16_digit(k, kc, j);
    const int ai = a < 0 ? -a : a;
    ge_niels q = ai ? ld_niels(acomb, j * COMB_MULT + ai - 1) : ge_niels_identity();
    acc = ge_madd_sgn(acc, q, a > 0);          // -[k]A
  }
  return add_base_comb(acc, s, btab);
}

// Per-item verification of the items whose key is registered in the context's cache (the
// other lanes exit; k_verify_single skips these items). Its own kernel, so that neither path
// inherits the other's register allocation.
__global__ void __launch_bounds__(SV_THREADS, 3) k_verify_comb(uint32_t n, const uint8_t* __restrict__ vk,
                                                               const uint8_t* __restrict__ sig,
                                                               const uint32_t* __restrict__ kscal,
                                                               uint8_t* __restrict__ verdict, KeyCacheView kcache,
                                                               const uint32_t* __restrict__ btab) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[8];
  ld_words8(vk + (size_t)i * 32, w);
  const int ci = kc_lookup(kcache, w);
  if (ci < 0) return;
  if (!kcache.ok[ci]) { verdict[i] = 2; return; }                 // try_from: MalformedPublicKey
  uint32_t sw[8];
  ld_words8(sig + (size_t)i * 64 + 32, sw);
  if (!sc_is_canonical(sw)) { verdict[i] = 1; return; }          // s checked before R
  uint32_t rw[8];
  ld_words8(sig + (size_t)i * 64, rw);
  ge_p3 R;
  if (!ge_decompress(rw, R)) { verdict[i] = 1; return; }
  uint32_t k[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) k[j] = kscal[(size_t)i * 8 + j];
  if (!sc_is_canonical(k)) { verdict[i] = 1; return; }           // k >= l: its digits exceed the comb
  const ge_p3 Rp = comb_double_base(k, sw, kcache.comb + (size_t)ci * COMB_ENTRIES * NIELS_WORDS, btab);
  verdict[i] = ge_is_identity(ge_mul_by_cofactor(ge_add(R, ge_neg(Rp)))) ? 0 : 1;
}

__global__ void __launch_bounds__(SV_THREADS, 3) k_verify_single(uint32_t n, const uint8_t* __restrict__ vk,
                                                                 const uint8_t* __restrict__ sig,
                                                                 const uint32_t* __restrict__ kscal,
                                                                 const uint32_t* __restrict__ btab,
                                                                 uint32_t* __restrict__ vtab,
                                                                 uint8_t* __restrict__ verdict,
                                                                 KeyCacheView kcache) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[8];
  ld_words8(vk + (size_t)i * 32, w);
  if (kc_lookup(kcache, w) >= 0) return;                          // done by k_verify_comb
  ge_p3 A;
  if (!ge_decompress(w, A)) { verdict[i] = 2; return; }          // try_from: MalformedPublicKey
  uint32_t sw[8];
  ld_words8(sig + (size_t)i * 64 + 32, sw);
  if (!sc_is_canonical(sw)) { verdict[i] = 1; return; }          // s checked before R
  uint32_t rw[8];
  ld_words8(sig + (size_t)i * 64, rw);
  uint32_t* tab = vtab + (size_t)i * SV_TAB_WORDS;
  {
    ge_p3 R;
    if (!ge_decompress(rw, R)) { verdict[i] = 1; return; }
    st_ext(tab + 8 * EXT_WORDS, R);    // parked in the scratch record: not live across the loop
  }
  uint32_t k[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) k[j] = kscal[(size_t)i * 8 + j];
  if (!sc_is_canonical(k)) { verdict[i] = 1; return; }           // k >= l: its digits exceed the table
  ge_p3 Rp = double_scalar_mul(k, ge_neg(A), sw, btab, tab);
  ge_p3 d = ge_add(ld_ext(tab + 8 * EXT_WORDS), ge_neg(Rp));
  verdict[i] = ge_is_identity(ge_mul_by_cofactor(d)) ? 0 : 1;
}

// Latency form of k_verify_single for small item lists (the grouped fallback's failing ranges):
// one QUAD of lanes per item (ge_quad.h), so every point operation of the 252-doubling chain is
// two rounds of one field multiplication per lane instead of eight serial ones. A and R are
// decoded at once on different lanes of the quad; the table of [1..8](-A) and the parked R live
// in LDS. Same verdict codes as k_verify_single; items with a cached key are left to
// k_verify_comb.
constexpr int VQ_ITEMS = 16;                       // items per 64-lane workgroup
__global__ void __launch_bounds__(64) k_verify_quad(uint32_t n, const uint8_t* __restrict__ vk,
                                                    const uint8_t* __restrict__ sig,
                                                    const uint32_t* __restrict__ kscal,
                                                    const uint32_t* __restrict__ btab,
                                                    uint8_t* __restrict__ verdict, KeyCacheView kcache) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[VQ_ITEMS][9 * EXT_WORDS];
  const uint32_t i = (blockIdx.x * 64 + threadIdx.x) >> 2;
  const int q = (int)(threadIdx.x & 3);
  uint32_t* tab = lds[threadIdx.x >> 2];
  if (i >= n) return;                              // whole quads leave together
  uint32_t aw[8], rw[8], sw[8];
  ld_words8(vk + (size_t)i * 32, aw);
  if (kc_lookup(kcache, aw) >= 0) return;          // done by k_verify_comb
  ld_words8(sig + (size_t)i * 64, rw);
  ld_words8(sig + (size_t)i * 64 + 32, sw);
  uint32_t w[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) w[j] = q == 1 ? rw[j] : aw[j];
  ge_p3 D;
  const bool ok = ge_decompress(w, D);             // lane 1: R, the others: A
  const uint32_t okA = quad_bcast<0>(ok ? 1u : 0u), okR = quad_bcast<1>(ok ? 1u : 0u);
  if (!okA) { if (q == 0) verdict[i] = 2; return; }          // try_from: MalformedPublicKey
  if (!sc_is_canonical(sw)) { if (q == 0) verdict[i] = 1; return; }   // s checked before R
  if (!okR) { if (q == 0) verdict[i] = 1; return; }
  const ge_p3 R = quad_bcast_point<1>(D);
  if (q == 0) st_ext(tab + 8 * EXT_WORDS, R);      // parked: not live across the loop
  const ge_p3 nA = ge_neg(quad_bcast_point<0>(D));
  const ge_cached c1 = ge_to_cached(nA);
  ge_p3 acc = nA;
  if (q == 0) st_cached(tab, c1);
  for (int d = 1; d < 8; ++d) {
    acc = quad_add_cached(acc, c1);
    const ge_cached cd = ge_to_cached(acc);
    if (q == 0) st_cached(tab + d * EXT_WORDS, cd);
  }
  uint32_t k[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) k[j] = kscal[(size_t)i * 8 + j];
  if (!sc_is_canonical(k)) { if (q == 0) verdict[i] = 1; return; }   // k >= l (whole quad leaves)
  const uint64_t kc = radix16_carries(k);
  acc = ge_identity();
  for (int j = 63; j >= 0; --j) {                  // R' = [k](-A) + [s]B: [k](-A) here
    if (j != 63) {
      acc = quad_dbl(acc);
      acc = quad_dbl(acc);
      acc = quad_dbl(acc);
      acc = quad_dbl(acc);
    }
    const int a = radix16_digit(k, kc, j);
    const int ai = a < 0 ? -a : a;
    ge_cached qa = ai ? ld_cached(tab + (ai - 1) * EXT_WORDS) : cached_identity();
    if (a < 0) qa = ge_cached_neg(qa);
    acc = quad_add_cached(acc, qa);
  }
  {                                                // + [s]B: 32 radix-256 comb additions
    const uint32_t sc = radix256_carries(sw);
    const uint32_t* comb = btab + (size_t)BTAB_ENTRIES * NIELS_WORDS;
    for (int j = 0; j < B256_POS; ++j) {
      const int b = radix256_digit(sw, sc, j);
      const int bi = b < 0 ? -b : b;
      ge_niels nb = bi ? ld_niels(comb, j * B256_MULT + bi - 1) : ge_niels_identity();
      if (b < 0) nb = ge_niels_neg(nb);
      acc = quad_madd(acc, nb);
    }
  }
  ge_p3 d = quad_add(ld_ext(tab + 8 * EXT_WORDS), ge_neg(acc));
  d = quad_dbl(quad_dbl(quad_dbl(d)));
  if (q == 0) verdict[i] = ge_is_identity(d) ? 0 : 1;
}

// [x]B, x < 2^256
__device__ ge_p3 base_mul(const uint32_t x[8], const uint32_t* btab) {
  int8_t d[64];
  radix16(x, d);
  ge_p3 acc = ge_identity();
  for (int j = 63; j >= 0; --j) {
    if (j != 63) {
      acc = ge_dbl(acc, false);
      acc = ge_dbl(acc, false);
      acc = ge_dbl(acc, false);
      acc = ge_dbl(acc, true);
    }
    int b = d[j];
    int bi = b < 0 ? -b : b;
    ge_niels nb = bi ? ld_niels(btab, bi - 1) : ge_niels_identity();
    acc = ge_madd_sgn(acc, nb, b < 0);
  }
  return acc;
}

// the radix-256 comb of B (btab entries BTAB_ENTRIES..): lane j*128 + d-1 -> [d 256^j]B,
// computed from the 8 multiples already in btab; a context builds it once
__global__ void __launch_bounds__(256) k_init_b256(uint32_t* btab) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (uint32_t)B256_ENTRIES) return;
  const uint32_t j = i / B256_MULT, d = i % B256_MULT + 1;
  uint32_t x[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  x[j >> 2] = d << (8 * (j & 3));                  // d <= 128 fits byte j
  st_niels(btab + (size_t)BTAB_ENTRIES * NIELS_WORDS, i, to_niels(base_mul(x, btab)));
}

__device__ __forceinline__ void words_to_bytes32(const uint32_t w[8], uint8_t* out) {
  for (int j = 0; j < 8; ++j)
    for (int b = 0; b < 4; ++b) out[4 * j + b] = (uint8_t)(w[j] >> (8 * b));
}

// SigningKey::from(seed) then sign(msg): a = clamp(H(seed)[0..32]), prefix = H(seed)[32..64],
// r = H(prefix || M), R = [r]B, k = H(R || A || M), s = r + k a. vk_out/sig_out per item.
// When shared_key != 0 every item is signed by seed 0 (no per-item key derivation repeated).
__global__ void __launch_bounds__(64) k_sign(uint32_t n, const uint8_t* __restrict__ seeds,
                                             const uint32_t* __restrict__ seed_index,
                                             const uint8_t* __restrict__ msg,
                                             const uint64_t* __restrict__ off,
                                             const uint32_t* __restrict__ btab,
                                             uint8_t* __restrict__ vk_out, uint8_t* __restrict__ sig_out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t si = seed_index ? seed_index[i] : i;
  const uint8_t* seed = seeds + (size_t)si * 32;
  uint8_t h[64];
  sha_src hs{seed, nullptr, nullptr, 0};
  sha512_src(hs, h);
  uint8_t ab[32];
  for (int j = 0; j < 32; ++j) ab[j] = h[j];
  ab[0] &= 248; ab[31] &= 127; ab[31] |= 64;
  uint32_t a[8];
  for (int j = 0; j < 8; ++j)
    a[j] = (uint32_t)ab[4 * j] | ((uint32_t)ab[4 * j + 1] << 8) | ((uint32_t)ab[4 * j + 2] << 16) |
           ((uint32_t)ab[4 * j + 3] << 24);
  uint32_t Aw[8];
  ge_compress(add_base_comb(ge_identity(), a, btab), Aw);   // [a]B: clamped a < 2^255, top digit <= 128
  uint8_t Ab[32];
  words_to_bytes32(Aw, Ab);
  const uint64_t o0 = off[i], o1 = off[i + 1];
  uint8_t rd[64];
  sha_src rs{h + 32, nullptr, msg + o0, o1 - o0};
  sha512_src(rs, rd);
  sc r = sc_from_digest(rd);
  uint32_t Rw[8];
  ge_compress(add_base_comb(ge_identity(), r.v, btab), Rw);  // [r]B from the radix-256 comb
  uint8_t Rb[32];
  words_to_bytes32(Rw, Rb);
  uint8_t kd[64];
  sha_src ks{Rb, Ab, msg + o0, o1 - o0};
  sha512_src(ks, kd);
  sc k = sc_from_digest(kd);
  sc as;
  for (int j = 0; j < 8; ++j) as.v[j] = a[j];
  sc s = sc_add(r, sc_mul(k, as));
  for (int j = 0; j < 32; ++j) {
    vk_out[(size_t)i * 32 + j] = Ab[j];
    sig_out[(size_t)i * 64 + j] = Rb[j];
  }
  words_to_bytes32(s.v, sig_out + (size_t)i * 64 + 32);
}

// CompressedEdwardsY::decompress: ok[i] = 1 and canonical x || y, or ok[i] = 0
__global__ void __launch_bounds__(256) k_decode(uint32_t n, const uint8_t* __restrict__ enc,
                                                uint8_t* __restrict__ xy, uint8_t* __restrict__ ok) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[8], wx[8], wy[8];
  ld_words8(enc + (size_t)i * 32, w);
  ge_p3 P;
  ok[i] = ge_decompress(w, P) ? 1 : 0;
  fe_to_words(P.X, wx);
  fe_to_words(P.Y, wy);
  words_to_bytes32(wx, xy + (size_t)i * 64);
  words_to_bytes32(wy, xy + (size_t)i * 64 + 32);
}

// ---- validator-key cache (keycache.h) ----
__global__ void __launch_bounds__(256) k_kc_decode(uint32_t m, const uint32_t* __restrict__ keys,
                                                   uint32_t* __restrict__ ext, uint8_t* __restrict__ ok) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  uint32_t w[8];
  ld_words8(reinterpret_cast<const uint8_t*>(keys + (size_t)i * 8), w);
  ge_p3 P;
  ok[i] = ge_decompress(w, P) ? 1 : 0;
  st_ext(ext + (size_t)i * EXT_WORDS, P);
}

__global__ void k_kc_basepoint(uint32_t* ext) {
  if (threadIdx.x == 0 && blockIdx.x == 0) st_ext(ext, ge_basepoint());
}

// comb[c][j][d-1] = [d 16^j] P_c: one lane per (point, position, multiple), one-off per cache load
__global__ void __launch_bounds__(256) k_kc_comb(uint32_t m, const uint32_t* __restrict__ ext,
                                                 uint32_t* __restrict__ comb) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t c = (uint32_t)(t / COMB_ENTRIES);
  if (c >= m) return;
  const uint32_t r = (uint32_t)(t % COMB_ENTRIES);
  const int j = (int)(r / COMB_MULT), d = (int)(r % COMB_MULT) + 1;
  ge_p3 P = ld_ext(ext + (size_t)c * EXT_WORDS);
  for (int q = 0; q < 4 * j; ++q) P = ge_dbl(P);
  ge_p3 Q = P;
  for (int q = 1; q < d; ++q) Q = ge_add(Q, P);
  st_niels(comb + (size_t)c * COMB_ENTRIES * NIELS_WORDS, r, to_niels(Q));
}

// VerificationKey::try_from (src/verification_key.rs:160-175): 0 Ok, 2 MalformedPublicKey
__global__ void __launch_bounds__(256) k_vk_validate(uint32_t n, const uint8_t* __restrict__ enc,
                                                     uint8_t* __restrict__ code) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[8];
  ld_words8(enc + (size_t)i * 32, w);
  ge_p3 P;
  code[i] = ge_decompress(w, P) ? 0 : 2;
}

// ChaCha20 keystream bytes [byte_off, byte_off + len) for synthetic data (64-byte aligned start)
__global__ void __launch_bounds__(256) k_chacha_fill(uint64_t nblocks, uint64_t blk0, uint32_t k0,
                                                     uint32_t k1, uint32_t k2, uint32_t k3, uint32_t k4,
                                                     uint32_t k5, uint32_t k6, uint32_t k7,
                                                     uint32_t* __restrict__ out) {
  uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblocks) return;
  uint32_t key[8] = {k0, k1, k2, k3, k4, k5, k6, k7};
  uint32_t o[16];
  chacha20_block(key, blk0 + b, o);
  for (int j = 0; j < 16; ++j) out[b * 16 + j] = o[j];
}

// ---------------------------------------------------------------- launchers
static inline uint32_t cdiv(uint64_t a, uint32_t b) { return (uint32_t)((a + b - 1) / b); }

void launch_init_btable(hipStream_t st, uint32_t* btab) {
  hipLaunchKernelGGL(k_init_btable, dim3(1), dim3(64), 0, st, btab);
  hipLaunchKernelGGL(k_init_b256, dim3(cdiv(B256_ENTRIES, 256)), dim3(256), 0, st, btab);
}
void launch_verify_single(hipStream_t st, uint32_t n, const uint8_t* vk, const uint8_t* sig,
                          const uint32_t* k, const uint32_t* btab, uint32_t* vtab, uint8_t* verdict,
                          const KeyCacheView& kc, const uint32_t* bcomb) {
  if (!n) return;
  if (kc.table)
    hipLaunchKernelGGL(k_verify_comb, dim3(cdiv(n, SV_THREADS)), dim3(SV_THREADS), 0, st, n, vk, sig, k, verdict, kc,
                       btab);
  hipLaunchKernelGGL(k_verify_single, dim3(cdiv(n, SV_THREADS)), dim3(SV_THREADS), 0, st, n, vk, sig, k, btab,
                     vtab, verdict, kc);
}
void launch_verify_quad(hipStream_t st, uint32_t n, const uint8_t* vk, const uint8_t* sig, const uint32_t* k,
                        const uint32_t* btab, uint8_t* verdict, const KeyCacheView& kc, const uint32_t* bcomb) {
  if (!n) return;
  if (kc.table)
    hipLaunchKernelGGL(k_verify_comb, dim3(cdiv(n, SV_THREADS)), dim3(SV_THREADS), 0, st, n, vk, sig, k, verdict, kc,
                       btab);
  hipLaunchKernelGGL(k_verify_quad, dim3(cdiv(4ull * n, 64)), dim3(64), 0, st, n, vk, sig, k, btab, verdict, kc);
}
void launch_kc_decode(hipStream_t st, uint32_t m, const uint32_t* keys, uint32_t* ext, uint8_t* ok) {
  if (m) hipLaunchKernelGGL(k_kc_decode, dim3(cdiv(m, 256)), dim3(256), 0, st, m, keys, ext, ok);
}
void launch_kc_basepoint(hipStream_t st, uint32_t* ext) {
  hipLaunchKernelGGL(k_kc_basepoint, dim3(1), dim3(64), 0, st, ext);
}
void launch_kc_comb(hipStream_t st, uint32_t m, const uint32_t* ext, uint32_t* comb) {
  if (m) hipLaunchKernelGGL(k_kc_comb, dim3(cdiv((uint64_t)m * COMB_ENTRIES, 256)), dim3(256), 0, st, m, ext, comb);
}
void launch_vk_validate(hipStream_t st, uint32_t n, const uint8_t* enc, uint8_t* code) {
  if (n) hipLaunchKernelGGL(k_vk_validate, dim3(cdiv(n, 256)), dim3(256), 0, st, n, enc, code);
}
size_t verify_single_scratch_words(size_t n) { return n * SV_TAB_WORDS; }
void launch_sign(hipStream_t st, uint32_t n, const uint8_t* seeds, const uint32_t* seed_index,
                 const uint8_t* msg, const uint64_t* off, const uint32_t* btab, uint8_t* vk_out,
                 uint8_t* sig_out) {
  if (n) hipLaunchKernelGGL(k_sign, dim3(cdiv(n, 64)), dim3(64), 0, st, n, seeds, seed_index, msg, off, btab,
                            vk_out, sig_out);
}
void launch_decode(hipStream_t st, uint32_t n, const uint8_t* enc, uint8_t* xy, uint8_t* ok) {
  if (n) hipLaunchKernelGGL(k_decode, dim3(cdiv(n, 256)), dim3(256), 0, st, n, enc, xy, ok);
}
void launch_chacha_fill(hipStream_t st, const uint32_t key[8], uint64_t blk0, uint64_t nblocks,
                        uint32_t* out) {
  if (nblocks)
    hipLaunchKernelGGL(k_chacha_fill, dim3(cdiv(nblocks, 256)), dim3(256), 0, st, nblocks, blk0,
                       key[0], key[1], key[2], key[3], key[4], key[5], key[6], key[7], out);
}

}  // namespace edc
