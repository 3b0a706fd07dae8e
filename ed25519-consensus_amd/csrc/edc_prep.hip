// Per-signature and per-key preparation kernels for batch verification
// (reference src/batch.rs:82-94 queue-time hashing, :174-203 the decode/coefficient loop).
//
//   k_challenge     k_i = SHA-512(R_i || A_i || M_i) mod l                (K1)
//   k_decompress_R  ZIP215 decode of R_i -> affine Niels point             (K2)
//   k_key_insert    group signatures by raw key bytes (HashMap<VerificationKeyBytes,..>)
//   k_key_index     dense key index per signature
//   k_decompress_A  ZIP215 decode of each distinct key                      (K2)
//   k_coef          z_i (ChaCha20), s_i < l check, u_i = z_i s_i, v_i = z_i k_i,
//                   per-key and global 64-bit limb sums                      (K3)
//   k_key_final     A_coeff = sum v_i mod l per key; B_coeff = -sum u_i mod l
#include "edc_common.h"
#include "edc_launch.h"

namespace edc {

__global__ void __launch_bounds__(256) k_challenge(uint32_t n, const uint8_t* __restrict__ vk,
                                                   const uint8_t* __restrict__ sig,
                                                   const uint8_t* __restrict__ msg,
                                                   const uint64_t* __restrict__ off,
                                                   uint32_t* __restrict__ k_out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t o0 = off[i], o1 = off[i + 1];
  sha_src s{sig + (size_t)i * 64, vk + (size_t)i * 32, msg + o0, o1 - o0};
  uint8_t d[64];
  sha512_src(s, d);
  sc k = sc_from_digest(d);
#pragma unroll
  for (int j = 0; j < 8; ++j) k_out[(size_t)i * 8 + j] = k.v[j];
}

// R_i -> points[1 + i]
__global__ void __launch_bounds__(256) k_decompress_R(uint32_t n, const uint8_t* __restrict__ sig,
                                                      uint32_t* __restrict__ pts,
                                                      int* __restrict__ flags) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[8];
  ld_words8(sig + (size_t)i * 64, w);
  ge_p3 P;
  bool ok = ge_decompress(w, P);
  st_niels(pts, 1 + i, ge_to_niels_affine(P));
  if (!ok) atomicOr(&flags[FLAG_BAD], 1);
}

__device__ __forceinline__ uint32_t key_hash(const uint32_t w[8], uint32_t salt) {
  uint32_t h = salt ^ 0x9E3779B9u;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    h ^= w[j];
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
  }
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

// Open-addressing insert keyed by the raw 32 key bytes. table[] holds the index of the first
// signature that claimed the slot (0xFFFFFFFF = empty; a slot never changes once claimed, so a
// stale relaxed read is safe). The claimer also draws the dense key index.
__global__ void __launch_bounds__(256) k_key_insert(uint32_t n, const uint8_t* __restrict__ vk,
                                                    uint32_t* __restrict__ table, uint32_t tmask,
                                                    uint32_t salt, uint32_t* __restrict__ slot_key,
                                                    uint32_t* __restrict__ key_slot_of_sig,
                                                    uint32_t* __restrict__ key_rep,
                                                    int* __restrict__ flags) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[8];
  ld_words8(vk + (size_t)i * 32, w);
  uint32_t h = key_hash(w, salt) & tmask;
  for (uint32_t probe = 0; probe <= tmask; ++probe) {
    uint32_t cur = __hip_atomic_load(&table[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == 0xFFFFFFFFu) {
      uint32_t prev = atomicCAS(&table[h], 0xFFFFFFFFu, i);
      if (prev == 0xFFFFFFFFu) {
        uint32_t kidx = (uint32_t)atomicAdd(&flags[FLAG_NKEYS], 1);
        slot_key[h] = kidx;
        key_rep[kidx] = i;
        key_slot_of_sig[i] = h;
        return;
      }
      cur = prev;
    }
    uint32_t o[8];
    ld_words8(vk + (size_t)cur * 32, o);
    bool eq = true;
#pragma unroll
    for (int j = 0; j < 8; ++j) eq &= (o[j] == w[j]);
    if (eq) {
      key_slot_of_sig[i] = h;
      return;
    }
    h = (h + 1) & tmask;
  }
}

__global__ void __launch_bounds__(256) k_key_index(uint32_t n, const uint32_t* __restrict__ key_slot_of_sig,
                                                   const uint32_t* __restrict__ slot_key,
                                                   uint32_t* __restrict__ key_index) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  key_index[i] = slot_key[key_slot_of_sig[i]];
}

// distinct key j -> points[1 + n + j]
__global__ void __launch_bounds__(256) k_decompress_A(uint32_t n, const uint8_t* __restrict__ vk,
                                                      const uint32_t* __restrict__ key_rep,
                                                      uint32_t* __restrict__ pts,
                                                      int* __restrict__ flags) {
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t m = (uint32_t)flags[FLAG_NKEYS];
  if (j >= m) return;
  uint32_t w[8];
  ld_words8(vk + (size_t)key_rep[j] * 32, w);
  ge_p3 P;
  bool ok = ge_decompress(w, P);
  st_niels(pts, 1 + n + j, ge_to_niels_affine(P));
  if (!ok) atomicOr(&flags[FLAG_BAD], 1);
}

// z_i as 4 LE words of the ChaCha20 keystream at global index zi
__device__ __forceinline__ void draw_z(const uint32_t seed[8], uint64_t zi, uint32_t z[4]) {
  uint32_t blk[16];
  chacha20_block(seed, zi >> 2, blk);
  int q = (int)(zi & 3);
#pragma unroll
  for (int j = 0; j < 4; ++j) z[j] = blk[4 * q + j];
}

struct seed8 { uint32_t w[8]; };

constexpr int COEF_CHUNK = 2048;   // signatures per workgroup
constexpr int COEF_SLOTS = 256;    // LDS key-accumulator slots

// Coefficients of the batch equation (reference src/batch.rs:193-198):
//   B_coeff -= z*s ; A_coeff[key] += z*k ; R coefficient = z.
// Integer limb sums are order-independent, so the LDS pre-aggregation + 64-bit atomics give
// bit-identical coefficients for any schedule.
__global__ void __launch_bounds__(256) k_coef(uint32_t n, const uint8_t* __restrict__ sig,
                                              const uint32_t* __restrict__ kscal,
                                              const uint8_t* __restrict__ zexp, seed8 seed,
                                              uint64_t zbase, const uint32_t* __restrict__ key_index,
                                              uint32_t* __restrict__ scal,
                                              unsigned long long* __restrict__ key_acc,
                                              unsigned long long* __restrict__ u_acc,
                                              int* __restrict__ flags) {
  __shared__ uint32_t tag[COEF_SLOTS];
  __shared__ unsigned long long acc[COEF_SLOTS][8];
  __shared__ unsigned long long uacc[8];
  for (int s = threadIdx.x; s < COEF_SLOTS; s += blockDim.x) {
    tag[s] = 0xFFFFFFFFu;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[s][j] = 0;
  }
  if (threadIdx.x < 8) uacc[threadIdx.x] = 0;
  __syncthreads();
  bool bad = false;
  uint32_t base = blockIdx.x * COEF_CHUNK;
  for (uint32_t t = threadIdx.x; t < COEF_CHUNK; t += blockDim.x) {
    uint32_t i = base + t;
    if (i >= n) break;
    uint32_t z[4];
    if (zexp) {
      const uint32_t* zp = reinterpret_cast<const uint32_t*>(zexp + (size_t)i * 16);
#pragma unroll
      for (int j = 0; j < 4; ++j) z[j] = zp[j];
    } else {
      draw_z(seed.w, zbase + i, z);
    }
    uint32_t sw[8];
    ld_words8(sig + (size_t)i * 64 + 32, sw);
    bad |= !sc_is_canonical(sw);
    sc s, k;
#pragma unroll
    for (int j = 0; j < 8; ++j) { s.v[j] = sw[j]; k.v[j] = kscal[(size_t)i * 8 + j]; }
    sc u = sc_mul128(z, s);
    sc v = sc_mul128(z, k);
    // R coefficient = z (point 1 + i)
    uint32_t* sp = scal + (size_t)(1 + i) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) sp[j] = j < 4 ? z[j] : 0u;
#pragma unroll
    for (int j = 0; j < 8; ++j) atomicAdd(&uacc[j], (unsigned long long)u.v[j]);
    uint32_t key = key_index[i];
    uint32_t slot = key & (COEF_SLOTS - 1);
    uint32_t prev = atomicCAS(&tag[slot], 0xFFFFFFFFu, key);
    if (prev == 0xFFFFFFFFu || prev == key) {
#pragma unroll
      for (int j = 0; j < 8; ++j) atomicAdd(&acc[slot][j], (unsigned long long)v.v[j]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) atomicAdd(&key_acc[(size_t)key * 8 + j], (unsigned long long)v.v[j]);
    }
  }
  if (bad) atomicOr(&flags[FLAG_BAD], 1);
  __syncthreads();
  for (int s = threadIdx.x; s < COEF_SLOTS; s += blockDim.x) {
    uint32_t key = tag[s];
    if (key != 0xFFFFFFFFu) {
#pragma unroll
      for (int j = 0; j < 8; ++j) atomicAdd(&key_acc[(size_t)key * 8 + j], acc[s][j]);
    }
  }
  if (threadIdx.x < 8) atomicAdd(&u_acc[threadIdx.x], uacc[threadIdx.x]);
}

// sum_j L[j] * 2^(32 j) mod l, L[j] < 2^64
__device__ __forceinline__ sc reduce_limb_sums(const unsigned long long* L) {
  uint32_t x[16];
  unsigned long long carry = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    unsigned long long lo = j < 8 ? (L[j] & 0xFFFFFFFFull) : 0ull;
    unsigned long long hi = (j >= 1 && j <= 8) ? (L[j - 1] >> 32) : 0ull;
    unsigned long long t = lo + hi + carry;
    x[j] = (uint32_t)t;
    carry = t >> 32;
  }
  return sc_reduce_wide(x);
}

__global__ void __launch_bounds__(256) k_key_final(uint32_t n, const unsigned long long* __restrict__ key_acc,
                                                   const unsigned long long* __restrict__ u_acc,
                                                   uint32_t* __restrict__ scal,
                                                   const int* __restrict__ flags) {
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t m = (uint32_t)flags[FLAG_NKEYS];
  if (j < m) {
    sc a = reduce_limb_sums(key_acc + (size_t)j * 8);
#pragma unroll
    for (int q = 0; q < 8; ++q) scal[(size_t)(1 + n + j) * 8 + q] = a.v[q];
  }
  if (j == 0) {
    sc u = reduce_limb_sums(u_acc);
    sc b = sc_sub(sc_zero(), u);
#pragma unroll
    for (int q = 0; q < 8; ++q) scal[q] = b.v[q];
  }
}

__global__ void k_init_basepoint(uint32_t* pts) {
  if (threadIdx.x == 0 && blockIdx.x == 0) st_niels(pts, 0, ge_to_niels_affine(ge_basepoint()));
}

// ---------------------------------------------------------------- launchers
static inline uint32_t cdiv(uint64_t a, uint32_t b) { return (uint32_t)((a + b - 1) / b); }

void launch_challenge(hipStream_t st, uint32_t n, const uint8_t* vk, const uint8_t* sig,
                      const uint8_t* msg, const uint64_t* off, uint32_t* k) {
  if (n) hipLaunchKernelGGL(k_challenge, dim3(cdiv(n, 256)), dim3(256), 0, st, n, vk, sig, msg, off, k);
}
void launch_decompress_R(hipStream_t st, uint32_t n, const uint8_t* sig, uint32_t* pts, int* flags) {
  if (n) hipLaunchKernelGGL(k_decompress_R, dim3(cdiv(n, 256)), dim3(256), 0, st, n, sig, pts, flags);
}
void launch_keys(hipStream_t st, uint32_t n, const uint8_t* vk, uint32_t* table, uint32_t tmask,
                 uint32_t salt, uint32_t* slot_key, uint32_t* key_slot_of_sig, uint32_t* key_rep,
                 uint32_t* key_index, uint32_t* pts, int* flags) {
  if (!n) return;
  hipLaunchKernelGGL(k_key_insert, dim3(cdiv(n, 256)), dim3(256), 0, st, n, vk, table, tmask, salt,
                     slot_key, key_slot_of_sig, key_rep, flags);
  hipLaunchKernelGGL(k_key_index, dim3(cdiv(n, 256)), dim3(256), 0, st, n, key_slot_of_sig, slot_key,
                     key_index);
  hipLaunchKernelGGL(k_decompress_A, dim3(cdiv(n, 256)), dim3(256), 0, st, n, vk, key_rep, pts, flags);
}
void launch_coef(hipStream_t st, uint32_t n, const uint8_t* sig, const uint32_t* k, const uint8_t* zexp,
                 const uint32_t seed[8], uint64_t zbase, const uint32_t* key_index, uint32_t* scal,
                 unsigned long long* key_acc, unsigned long long* u_acc, int* flags) {
  seed8 s;
  for (int j = 0; j < 8; ++j) s.w[j] = seed[j];
  if (n)
    hipLaunchKernelGGL(k_coef, dim3(cdiv(n, COEF_CHUNK)), dim3(256), 0, st, n, sig, k, zexp, s, zbase,
                       key_index, scal, key_acc, u_acc, flags);
  hipLaunchKernelGGL(k_key_final, dim3(cdiv(n > 0 ? n : 1, 256)), dim3(256), 0, st, n, key_acc, u_acc,
                     scal, flags);
}
void launch_init_basepoint(hipStream_t st, uint32_t* pts) {
  hipLaunchKernelGGL(k_init_basepoint, dim3(1), dim3(64), 0, st, pts);
}

}  // namespace edc
