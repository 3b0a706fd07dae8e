// Persistent validator-key cache.
//
// Consensus re-verifies votes from the same few hundred validator keys block after block. The
// reference decodes A once per VerificationKey and keeps it (src/verification_key.rs:106-114,
// :160-175), but a batch::Verifier re-decodes every distinct key on every verify
// (src/batch.rs:183-185). The cache decodes each registered key ONCE per context and keeps, per
// key, a fixed-base comb table
//     comb[j][d-1] = [d * 16^j] A    (j = 0..63, d = 1..8), affine Niels, 512 records = 64 KB
// so that
//   - a batch takes A (= comb[0][0]) and, with split coefficients (edc_common.h), [2^128]A
//     (= comb[32][0]) from the cache instead of decoding / doubling them;
//   - the per-item fallback computes [s]B - [k]A as 128 mixed additions and NO doublings
//     (signed radix-16 digits, one comb record each for k and s), against 252 doublings + 128
//     additions + one A decode + 7 table additions per item without the cache.
// Verdicts are unchanged: group arithmetic is exact, and an undecodable cached key keeps
// ok = 0 (MalformedPublicKey for single verification, a failed batch otherwise).
#pragma once
#include <stdint.h>

namespace edc {

constexpr int COMB_POS = 64;                      // radix-16 positions
constexpr int COMB_MULT = 8;                      // |digit| in 1..8
constexpr int COMB_ENTRIES = COMB_POS * COMB_MULT;
constexpr int COMB_SHIFT128 = 32 * COMB_MULT;     // [16^32]A = [2^128]A
constexpr uint32_t KC_EMPTY = 0xFFFFFFFFu;
constexpr uint32_t KC_MAX_KEYS = 1u << 16;        // 4 GB of comb tables

// Read-only device view of a context's cache (all pointers null = no cache).
struct KeyCacheView {
  const uint32_t* table;   // tmask+1 slots: cache index or KC_EMPTY (open addressing)
  const uint32_t* keys;    // m x 8 words: raw key bytes
  const uint8_t* ok;       // m: 1 iff the key decodes (VerificationKey::try_from succeeds)
  const uint32_t* comb;    // m x COMB_ENTRIES affine Niels records
  uint32_t tmask;
  uint32_t m;
  const uint32_t* bcomb;   // COMB_ENTRIES records of B (built with the first cache)
  uint32_t s0, s1;         // hash key (per-context secret: keys added from untrusted input cannot
                           // be chosen to collide in the table)
};

__host__ __device__ inline uint32_t kc_hash(const uint32_t w[8], uint32_t s0, uint32_t s1) {
  uint32_t h = 0x2545F491u ^ s0;
  for (int j = 0; j < 8; ++j) {
    h ^= w[j];
    h *= 0x9E3779B1u;
    h ^= h >> 15;
  }
  h ^= s1;
  h *= 0x85EBCA77u;
  h ^= h >> 13;
  return h;
}

#if defined(__HIPCC__)
// cache index of the raw key bytes w, or -1
__device__ __forceinline__ int kc_lookup(const KeyCacheView& kc, const uint32_t w[8]) {
  if (!kc.table) return -1;
  uint32_t h = kc_hash(w, kc.s0, kc.s1) & kc.tmask;
  for (uint32_t probe = 0; probe <= kc.tmask; ++probe) {
    const uint32_t c = kc.table[h];
    if (c == KC_EMPTY) return -1;
    const uint4* q = reinterpret_cast<const uint4*>(kc.keys + (size_t)c * 8);
    const uint4 a = q[0], b = q[1];
    if (a.x == w[0] && a.y == w[1] && a.z == w[2] && a.w == w[3] && b.x == w[4] && b.y == w[5] &&
        b.z == w[6] && b.w == w[7])
      return (int)c;
    h = (h + 1) & kc.tmask;
  }
  return -1;
}
#endif

}  // namespace edc
