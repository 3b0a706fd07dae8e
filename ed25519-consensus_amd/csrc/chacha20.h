// ChaCha20 keystream block (djb layout: 64-bit block counter in words 12-13, stream id 0 in
// words 14-15), bit-exact with rand_chacha::ChaCha20Rng::from_seed(seed). The batch verifier's
// z_i = u128::from_le_bytes(keystream[16i..16i+16]) (gen_u128, reference src/batch.rs:64-68),
// so block b yields z_{4b} .. z_{4b+3} and any shard can generate its own z from the global index.
#pragma once
#include <stdint.h>
#include "fe25519.h"  // EDC_HD

namespace edc {

EDC_HD uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

#define EDC_QR(a, b, c, d)                      \
  x[a] += x[b]; x[d] = rotl32(x[d] ^ x[a], 16); \
  x[c] += x[d]; x[b] = rotl32(x[b] ^ x[c], 12); \
  x[a] += x[b]; x[d] = rotl32(x[d] ^ x[a], 8);  \
  x[c] += x[d]; x[b] = rotl32(x[b] ^ x[c], 7);

EDC_HD void chacha20_block(const uint32_t key[8], uint64_t counter, uint32_t out[16]) {
  uint32_t st[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                     key[0], key[1], key[2], key[3], key[4], key[5], key[6], key[7],
                     (uint32_t)counter, (uint32_t)(counter >> 32), 0u, 0u};
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = st[i];
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    EDC_QR(0, 4, 8, 12) EDC_QR(1, 5, 9, 13) EDC_QR(2, 6, 10, 14) EDC_QR(3, 7, 11, 15)
    EDC_QR(0, 5, 10, 15) EDC_QR(1, 6, 11, 12) EDC_QR(2, 7, 8, 13) EDC_QR(3, 4, 9, 14)
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) out[i] = x[i] + st[i];
}
#undef EDC_QR

}  // namespace edc
