// SHA-512 (FIPS 180-4) for one message per lane. The message is the concatenation of up to
// three byte segments -- R || A || M for the challenge k = H(R||A||M) (reference
// src/batch.rs:86-91, src/verification_key.rs:226-231; sha2 0.9 Sha512::chain) -- streamed
// straight from global memory into 128-byte blocks, so the hash needs no staging buffer.
// 64-bit words are native uint64_t; hipcc lowers rotates to v_alignbit_b32 pairs.
#pragma once
#include <stdint.h>
#include "fe25519.h"  // EDC_HD

namespace edc {

// round constants: __constant__ on the device (wave-uniform scalar loads), const on the host
#if defined(__HIP_DEVICE_COMPILE__)
__constant__ uint64_t SHA512_K[80] = {
#else
static const uint64_t SHA512_K[80] = {
#endif
    0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull,
    0x3956c25bf348b538ull, 0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull,
    0xd807aa98a3030242ull, 0x12835b0145706fbeull, 0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull,
    0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull, 0xc19bf174cf692694ull,
    0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
    0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull,
    0x983e5152ee66dfabull, 0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull,
    0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull, 0x06ca6351e003826full, 0x142929670a0e6e70ull,
    0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull, 0x53380d139d95b3dfull,
    0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
    0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull,
    0xd192e819d6ef5218ull, 0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull,
    0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull, 0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull,
    0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull, 0x682e6ff3d6b2b8a3ull,
    0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
    0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull,
    0xca273eceea26619cull, 0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull,
    0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull, 0x113f9804bef90daeull, 0x1b710b35131c471bull,
    0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull, 0x431d67c49c100d4cull,
    0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull};

// Native 64-bit words: LLVM lowers a 64-bit rotate to two v_alignbit_b32, a three-way xor / ch /
// maj to one v_bitop3_b32 per half and an add to one v_lshl_add_u64 (64-bit values kept in
// register pairs; a 32-bit-halves formulation costs v_mov shuffles to rebuild the pairs).
EDC_HD uint32_t lo32(uint64_t x) { return (uint32_t)x; }
EDC_HD uint32_t hi32(uint64_t x) { return (uint32_t)(x >> 32); }
// On the device the pair is built as a bit cast of a 2 x u32 vector: the halves land in one
// register pair and the 64-bit adds take it whole. Written as (hi << 32) | lo, LLVM instead
// re-associated every sum into separate zero-extended lo / hi contributions: per round three more
// v_lshl_add_u64 and four v_mov_b32 (34 instead of 27 VALU instructions per round).
#if defined(__HIP_DEVICE_COMPILE__)
typedef uint32_t edc_u32x2 __attribute__((ext_vector_type(2)));
EDC_HD uint64_t mk64(uint32_t lo, uint32_t hi) { return __builtin_bit_cast(uint64_t, edc_u32x2{lo, hi}); }
#else
EDC_HD uint64_t mk64(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }
#endif
// funnel shift right of hi:lo by n (0 < n < 32)
EDC_HD uint32_t fshr32(uint32_t hi, uint32_t lo, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbit(hi, lo, n);
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> n);
#endif
}
EDC_HD uint32_t xor3_32(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}
// halves of rotr(x, n) for a compile-time n (one v_alignbit_b32 each)
template <int N> EDC_HD uint32_t rotr_lo(uint32_t l, uint32_t h) { return N < 32 ? fshr32(h, l, N) : fshr32(l, h, N - 32); }
template <int N> EDC_HD uint32_t rotr_hi(uint32_t l, uint32_t h) { return N < 32 ? fshr32(l, h, N) : fshr32(h, l, N - 32); }
// rotr(x, n1) ^ rotr(x, n2) ^ rotr(x, n3): six v_alignbit_b32 + two v_bitop3_b32
template <int N1, int N2, int N3>
EDC_HD uint64_t rot3(uint64_t x) {
  const uint32_t l = lo32(x), h = hi32(x);
  return mk64(xor3_32(rotr_lo<N1>(l, h), rotr_lo<N2>(l, h), rotr_lo<N3>(l, h)),
              xor3_32(rotr_hi<N1>(l, h), rotr_hi<N2>(l, h), rotr_hi<N3>(l, h)));
}
// rotr(x, n1) ^ rotr(x, n2) ^ (x >> n3), n3 < 32
template <int N1, int N2, int N3>
EDC_HD uint64_t sig_small(uint64_t x) {
  const uint32_t l = lo32(x), h = hi32(x);
  return mk64(xor3_32(rotr_lo<N1>(l, h), rotr_lo<N2>(l, h), fshr32(h, l, N3)),
              xor3_32(rotr_hi<N1>(l, h), rotr_hi<N2>(l, h), h >> N3));
}

// ch and maj as one v_bitop3_b32 per half (truth tables 0xCA and 0xE8 over (S0, S1, S2));
// LLVM otherwise emits bfi + and / four ands and xors
EDC_HD uint64_t ch64(uint64_t e, uint64_t f, uint64_t g) {
#if defined(__HIP_DEVICE_COMPILE__)
  return mk64(__builtin_amdgcn_bitop3_b32(lo32(e), lo32(f), lo32(g), 0xCA),
              __builtin_amdgcn_bitop3_b32(hi32(e), hi32(f), hi32(g), 0xCA));
#else
  return (e & f) ^ (~e & g);
#endif
}
EDC_HD uint64_t maj64(uint64_t a, uint64_t b, uint64_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return mk64(__builtin_amdgcn_bitop3_b32(lo32(a), lo32(b), lo32(c), 0xE8),
              __builtin_amdgcn_bitop3_b32(hi32(a), hi32(b), hi32(c), 0xE8));
#else
  return (a & b) ^ (a & c) ^ (b & c);
#endif
}

#define EDC_SHA_ROUND(a, b, c, d, e, f, g, h, k, wt)                                              \
  {                                                                                              \
    const uint64_t t1 = h + rot3<14, 18, 41>(e) + ch64(e, f, g) + (k) + (wt);                     \
    const uint64_t t2 = rot3<28, 34, 39>(a) + maj64(a, b, c);                                     \
    d += t1;                                                                                     \
    h = t1 + t2;                                                                                 \
  }

// 80 rounds as 5 x 16: the 16-round body is unrolled (message words in registers, the eight
// working variables renamed instead of moved), the 5 passes are a loop.
EDC_HD void sha512_compress(uint64_t hs[8], const uint64_t win[16]) {
  uint64_t w[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) w[t] = win[t];
  uint64_t a = hs[0], b = hs[1], c = hs[2], d = hs[3], e = hs[4], f = hs[5], g = hs[6], h = hs[7];
#pragma unroll 1
  for (int r = 0; r < 5; ++r) {
    if (r) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const uint64_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
        const uint64_t s0 = sig_small<1, 8, 7>(w15);
        const uint64_t s1 = sig_small<19, 61, 6>(w2);
        w[j] = w[j] + s0 + w[(j + 9) & 15] + s1;
      }
    }
    const uint64_t* K = SHA512_K + 16 * r;
#pragma unroll
    for (int j = 0; j < 16; j += 8) {
      EDC_SHA_ROUND(a, b, c, d, e, f, g, h, K[j + 0], w[j + 0]);
      EDC_SHA_ROUND(h, a, b, c, d, e, f, g, K[j + 1], w[j + 1]);
      EDC_SHA_ROUND(g, h, a, b, c, d, e, f, K[j + 2], w[j + 2]);
      EDC_SHA_ROUND(f, g, h, a, b, c, d, e, K[j + 3], w[j + 3]);
      EDC_SHA_ROUND(e, f, g, h, a, b, c, d, K[j + 4], w[j + 4]);
      EDC_SHA_ROUND(d, e, f, g, h, a, b, c, K[j + 5], w[j + 5]);
      EDC_SHA_ROUND(c, d, e, f, g, h, a, b, K[j + 6], w[j + 6]);
      EDC_SHA_ROUND(b, c, d, e, f, g, h, a, K[j + 7], w[j + 7]);
    }
  }
  hs[0] += a; hs[1] += b; hs[2] += c; hs[3] += d;
  hs[4] += e; hs[5] += f; hs[6] += g; hs[7] += h;
}
#undef EDC_SHA_ROUND

EDC_HD void sha512_init(uint64_t h[8]) {
  h[0] = 0x6a09e667f3bcc908ull; h[1] = 0xbb67ae8584caa73bull; h[2] = 0x3c6ef372fe94f82bull;
  h[3] = 0xa54ff53a5f1d36f1ull; h[4] = 0x510e527fade682d1ull; h[5] = 0x9b05688c2b3e6c1full;
  h[6] = 0x1f83d9abfb41bd6bull; h[7] = 0x5be0cd19137e2179ull;
}

// Byte source: a fixed 64-byte head (two 32-byte pieces, e.g. R and A) followed by a variable
// message. Pass head1 = nullptr for a 32-byte head (signing: prefix || M).
struct sha_src {
  const uint8_t* head0;
  const uint8_t* head1;
  const uint8_t* msg;
  uint64_t mlen;
};

EDC_HD uint32_t bswap32(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xFF00u) | ((x << 8) & 0xFF0000u) | (x << 24);
}

// big-endian 64-bit word from an 8-byte-aligned pointer (R / A / seed heads)
EDC_HD uint64_t load_be64(const uint8_t* p) {
  const uint32_t* q = reinterpret_cast<const uint32_t*>(p);
  return ((uint64_t)bswap32(q[0]) << 32) | bswap32(q[1]);
}

// 4-byte-aligned dword containing byte p. Reading it never leaves the page of p, so it is safe
// for any p inside the message arena.
EDC_HD uint32_t ld_dword_at(uintptr_t a) { return *reinterpret_cast<const uint32_t*>(a); }

// Big-endian word of the padded message tail starting at message byte j (j may exceed mlen).
// Every word inside the message, the last partial one included, is assembled the same way from
// three aligned dwords (funnel shifts, v_alignbyte on gfx950; dword addresses clamped to the one
// holding the message's last byte, so nothing past the message is read beyond that dword), then
// the bytes past the end are masked and the 0x80 marker inserted. Lanes hashing messages of
// different lengths thus take one path per word (a byte-by-byte tail was a divergent branch
// that every wave of a variable-length batch executed for every word of its last block).
EDC_HD uint64_t msg_word(const uint8_t* m, uint64_t mlen, uint64_t j) {
  if (j >= mlen) return j == mlen ? (0x80ull << 56) : 0ull;   // padding only: marker or zeros
  const uintptr_t p = (uintptr_t)(m + j);
  const uintptr_t last = (uintptr_t)(m + mlen - 1) & ~(uintptr_t)3;
  const uintptr_t a = p & ~(uintptr_t)3;
  const uintptr_t a1 = a + 4 < last ? a + 4 : last, a2 = ((p + 7) & ~(uintptr_t)3) < last ? ((p + 7) & ~(uintptr_t)3) : last;
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t d0 = ld_dword_at(a), d1 = ld_dword_at(a1), d2 = ld_dword_at(a2);
#else   // host build (tests/native): the same dwords, without touching bytes past the message
  const uintptr_t end = (uintptr_t)(m + mlen);
  auto ld = [end](uintptr_t q) {
    uint32_t v = 0;
    for (int b = 0; b < 4; ++b)
      if (q + b < end) v |= (uint32_t)*reinterpret_cast<const uint8_t*>(q + b) << (8 * b);
    return v;
  };
  const uint32_t d0 = ld(a), d1 = ld(a1), d2 = ld(a2);
#endif
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t sh = (uint32_t)(p & 3);                       // funnel shifts by bytes, no branch
  const uint32_t lo = __builtin_amdgcn_alignbyte(d1, d0, sh), hi = __builtin_amdgcn_alignbyte(d2, d1, sh);
#else
  const uint32_t sh = (uint32_t)(p & 3) * 8;
  const uint32_t lo = sh ? (d0 >> sh) | (d1 << (32 - sh)) : d0;
  const uint32_t hi = sh ? (d1 >> sh) | (d2 << (32 - sh)) : d1;
#endif
  uint64_t w = ((uint64_t)bswap32(lo) << 32) | bswap32(hi);
  const uint64_t rem = mlen - j;                               // >= 1
  if (rem < 8) {                                               // keep rem bytes, then the marker
    const uint32_t kb = 8 * (uint32_t)rem;
    w = (w & (~0ull << (64 - kb))) | (0x80ull << (56 - kb));
  }
  return w;
}

// SHA-512(head0[0..32) || head1[0..32) || msg[0..mlen)) as the 8 big-endian state words.
EDC_HD void sha512_src_state(const sha_src& s, uint64_t h[8]) {
  sha512_init(h);
  const uint64_t hlen = s.head1 ? 64 : 32;
  const uint64_t total = hlen + s.mlen;
  const uint64_t nblocks = (total + 17 + 127) / 128;
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t pf0 = 0, pf1 = 0;
#endif
#pragma unroll 1
  for (uint64_t blk = 0; blk < nblocks; ++blk) {
    uint64_t w[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      uint64_t off = blk * 128 + 8 * (uint64_t)t;
      if (off < 32) w[t] = load_be64(s.head0 + off);
      else if (off < hlen) w[t] = load_be64(s.head1 + (off - 32));
      else w[t] = msg_word(s.msg, s.mlen, off - hlen);
    }
    if (blk == nblocks - 1) {
      w[14] = 0;                 // bit-length high word (messages < 2^61 bytes)
      w[15] = total << 3;
    }
#if defined(__HIP_DEVICE_COMPILE__)
    // touch the next block's message lines (both 64-byte halves) so that they are on their way
    // to the caches while this block compresses; the loaded values are never used
    if (blk + 1 < nblocks && s.mlen) {
      const uint64_t j0 = (blk + 1) * 128 - hlen;
      const uintptr_t lo = (uintptr_t)s.msg, hi = ((uintptr_t)(s.msg + s.mlen - 1)) & ~(uintptr_t)3;
      uintptr_t q0 = (lo + j0) & ~(uintptr_t)3, q1 = (lo + j0 + 124) & ~(uintptr_t)3;
      q0 = q0 < hi ? q0 : hi;
      q1 = q1 < hi ? q1 : hi;
      pf0 = *reinterpret_cast<const uint32_t*>(q0);
      pf1 = *reinterpret_cast<const uint32_t*>(q1);
    }
#endif
    sha512_compress(h, w);
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" ::"v"(pf0), "v"(pf1));   // consumed after the compression: the loads stay in flight over it
#endif
  }
}

// digest bytes in out[0..64)
EDC_HD void sha512_src(const sha_src& s, uint8_t out[64]) {
  uint64_t h[8];
  sha512_src_state(s, h);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int b = 0; b < 8; ++b) out[8 * i + b] = (uint8_t)(h[i] >> (56 - 8 * b));
}

// digest as 16 little-endian 32-bit words (the 512-bit LE integer Scalar::from_hash reduces)
EDC_HD void sha512_src_le_words(const sha_src& s, uint32_t x[16]) {
  uint64_t h[8];
  sha512_src_state(s, h);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    x[2 * i] = bswap32((uint32_t)(h[i] >> 32));
    x[2 * i + 1] = bswap32((uint32_t)h[i]);
  }
}

}  // namespace edc
