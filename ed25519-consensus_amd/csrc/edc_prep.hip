// Per-signature and per-key preparation kernels for batch verification
// (reference src/batch.rs:82-94 queue-time hashing, :174-203 the decode/coefficient loop).
//
//   k_challenge     k_i = SHA-512(R_i || A_i || M_i) mod l                (K1)
//   k_key_insert    group signatures by raw key bytes (HashMap<VerificationKeyBytes,..>)
//   k_key_index     dense key index per signature
//   k_decompress    ZIP215 decode of every R_i and every distinct key -> affine Niels (K2)
//   k_coef          z_i (ChaCha20), s_i < l check, u_i = z_i s_i, v_i = z_i k_i,
//                   per-key and global 64-bit limb sums                      (K3)
//   k_key_final     A_coeff = sum v_i mod l per key; B_coeff = -sum u_i mod l
#include "edc_common.h"
#include "edc_launch.h"
#include "ge_quad.h"

namespace edc {

constexpr int SHA_CLASSES = 16;   // block counts 1..14, 15+, and out-of-range lanes
constexpr int SHA_THREADS = 256;  // items regrouped per workgroup
#ifndef EDC_SHA_OCC
#define EDC_SHA_OCC 4
#endif
#ifndef EDC_SHA_STAGED
#define EDC_SHA_STAGED 1
#endif

// ---- SHA-512 over R || A || M with the message staged through LDS (k_challenge) ----
// Each block's message bytes (a 128-byte window; 64 bytes in block 0, after R || A) are fetched
// for the whole wave by LDS-DMA (global_load_lds_dwordx4) before they are needed: instruction c
// moves every lane's c-th 16-byte chunk of its window (16-byte aligned, 9 chunks cover 128 bytes
// at any alignment) into column `lane` of row c of the wave's buffer, so no VGPR holds the
// loads and the next block's chunks travel while the current block compresses. Chunks past the
// message's last 16-byte chunk come from a zero line, so the window already holds the padding's
// zeros; the lane whose message ends in the window fixes the one chunk that straddles the end
// (marker 0x80, zeros after it) in its own column. The words are then assembled from LDS dwords
// with one funnel shift (v_alignbyte) and one byte swap (v_perm) per half: ~5 VALU per word,
// where the per-lane global walk (three clamped dword loads per word, each waited on at once)
// cost ~45 and serialized the memory latency word by word.
constexpr int SHA_WIN_CHUNKS = 9;
__device__ __attribute__((aligned(16))) uint32_t g_sha_zero[4];

__device__ __forceinline__ void sha_dma16(const void* gsrc, uint32_t* lds_row) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gsrc,
                                   (__attribute__((address_space(3))) void*)lds_row, 16, 0, 0);
}

// dword x of lane's window column (row = 16-byte chunk, 256 dwords per row)
__device__ __forceinline__ uint32_t* sha_col(uint32_t* wbuf, uint32_t lane, uint32_t x) {
  return wbuf + (x >> 2) * 256 + lane * 4 + (x & 3);
}

// Issue the DMA of block blk's window (every lane of the wave takes part, live or not).
__device__ __forceinline__ void sha_stage(uint32_t* wbuf, uintptr_t mbase, uint64_t mlen, uint32_t blk) {
  const uint64_t w0 = blk ? (uint64_t)blk * 128 - 64 : 0;
  const uintptr_t S = (mbase + w0) & ~(uintptr_t)15;
  const uintptr_t last = mlen ? ((mbase + mlen - 1) & ~(uintptr_t)15) : 0;
  // a window that starts at or past the message's end is all padding: every chunk zero (its first
  // chunk may still be the message's last one, whose bytes past the end are not zero)
  const bool inside = mlen > w0;
#pragma unroll
  for (int c = 0; c < SHA_WIN_CHUNKS; ++c) {
    if (blk == 0 && c >= 5) break;                 // block 0: 64 message bytes, 5 chunks
    const uintptr_t g = S + 16u * c;
    const void* src = (inside && g <= last) ? (const void*)g : (const void*)g_sha_zero;
    sha_dma16(src, wbuf + c * 256);
  }
}

// SHA-512(R || A || M) state of item i (lane of a wave whose every lane calls this, live or not).
__device__ __forceinline__ bool sha_staged_state(uint32_t i, uint32_t n, const uint8_t* __restrict__ vk,
                                                 const uint8_t* __restrict__ sig, const uint8_t* __restrict__ msg,
                                                 const uint64_t* __restrict__ off, uint32_t* wbuf, uint64_t h[8]) {
  const uint32_t lane = threadIdx.x & 63;
  const bool live = i < n;
  const uint64_t o0 = live ? off[i] : 0, mlen = live ? off[i + 1] - o0 : 0;
  const uint64_t total = 64 + mlen;
  const uint32_t nblocks = live ? (uint32_t)((total + 17 + 127) / 128) : 0u;
  uint32_t nb_max = nblocks;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) nb_max = max(nb_max, (uint32_t)__shfl_xor((int)nb_max, d, 64));
  nb_max = __builtin_amdgcn_readfirstlane(nb_max);
  const uintptr_t mbase = (uintptr_t)msg + o0;
  sha512_init(h);
  sha_stage(wbuf, mbase, mlen, 0);
#pragma unroll 1
  for (uint32_t blk = 0; blk < nb_max; ++blk) {
    const uint64_t w0 = blk ? (uint64_t)blk * 128 - 64 : 0;
    const uint32_t wlen = blk ? 128u : 64u;
    const uint32_t q0b = (uint32_t)((mbase + w0) & 15);
    uint64_t w[16];
    if (blk == 0 && blk < nblocks) {               // R || A: words 0..7, 16-byte aligned rows
#pragma unroll
      for (int t = 0; t < 4; ++t) w[t] = load_be64(sig + (size_t)i * 64 + 8 * t);
#pragma unroll
      for (int t = 0; t < 4; ++t) w[4 + t] = load_be64(vk + (size_t)i * 32 + 8 * t);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);            // vmcnt(0): this block's chunks are in LDS
    asm volatile("" ::: "memory");
    // the message ends in this window: marker 0x80 at its end, zeros to the end of that chunk
    const int64_t e_rel = (int64_t)mlen - (int64_t)w0;
    if (live && e_rel >= 0 && e_rel < (int64_t)wlen) {
      const uint32_t pos = q0b + (uint32_t)e_rel, di = pos >> 2, sb = 8 * (pos & 3);
      uint32_t* p = sha_col(wbuf, lane, di);
      *p = (*p & ((1u << sb) - 1u)) | (0x80u << sb);
      const uint32_t rest = 3u - (di & 3u);        // dwords after di in its 16-byte chunk
      if (rest >= 1) p[1] = 0u;
      if (rest >= 2) p[2] = 0u;
      if (rest >= 3) p[3] = 0u;
    }
    // window dwords from the one holding byte q0b: four base pointers (x = b0 + 4j + r)
    const uint32_t b0 = q0b >> 2, sh = q0b & 3;
    uint32_t* P0 = sha_col(wbuf, lane, b0), *P1 = sha_col(wbuf, lane, b0 + 1);
    uint32_t* P2 = sha_col(wbuf, lane, b0 + 2), *P3 = sha_col(wbuf, lane, b0 + 3);
    auto dw = [&](int k) -> uint32_t {
      const int j = k >> 2, r = k & 3;
      return (r == 0 ? P0 : r == 1 ? P1 : r == 2 ? P2 : P3)[j * 256];
    };
    const int t0 = blk ? 0 : 8;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      if (t < t0) continue;
      const int k = 2 * (t - t0);
      const uint32_t d0 = dw(k), d1 = dw(k + 1), d2 = dw(k + 2);
      const uint32_t lo = __builtin_amdgcn_alignbyte(d1, d0, sh), hi = __builtin_amdgcn_alignbyte(d2, d1, sh);
      w[t] = mk64(bswap32(hi), bswap32(lo));
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);            // lgkmcnt(0): the window is read before it is refilled
    asm volatile("" ::: "memory");
    if (blk + 1 < nb_max) sha_stage(wbuf, mbase, mlen, blk + 1);
    if (blk < nblocks) {
      if (blk == nblocks - 1) {
        w[14] = 0;                                  // bit-length high word (messages < 2^61 bytes)
        w[15] = total << 3;
      }
      sha512_compress(h, w);
    }
  }
  return live;
}
__global__ void __launch_bounds__(SHA_THREADS, EDC_SHA_OCC) k_challenge(uint32_t n, const uint8_t* __restrict__ vk,
                                                   const uint8_t* __restrict__ sig,
                                                   const uint8_t* __restrict__ msg,
                                                   const uint64_t* __restrict__ off,
                                                   uint32_t* __restrict__ k_out) {
  // Variable-length messages: a wave runs as many SHA-512 blocks as its longest message, so the
  // workgroup's 256 items are first regrouped by block count (LDS counting sort) and each lane
  // hashes the item at its sorted position; waves then hold messages of similar length.
  // Equal-length batches keep the identity order.
  __shared__ uint32_t cls_cnt[SHA_CLASSES], cls_base[SHA_CLASSES];
  __shared__ uint32_t order[SHA_THREADS];
  const uint32_t t = threadIdx.x;
  const uint32_t i0 = blockIdx.x * blockDim.x + t;
  uint32_t cls = SHA_CLASSES - 1;                     // out-of-range lanes sort last
  if (i0 < n) {
    const uint64_t nb = (64 + (off[i0 + 1] - off[i0]) + 17 + 127) / 128;
    cls = nb < SHA_CLASSES - 1 ? (uint32_t)nb - 1 : SHA_CLASSES - 2;
  }
  if (t < SHA_CLASSES) cls_cnt[t] = 0;
  __syncthreads();
  const uint32_t rank = atomicAdd(&cls_cnt[cls], 1u);
  __syncthreads();
  if (t == 0) {
    uint32_t run = 0;
    for (int c = 0; c < SHA_CLASSES; ++c) { cls_base[c] = run; run += cls_cnt[c]; }
  }
  __syncthreads();
  order[cls_base[cls] + rank] = i0;
  __syncthreads();
  const uint32_t i = order[t];
#if EDC_SHA_STAGED
  __shared__ __attribute__((aligned(16))) uint32_t win[SHA_THREADS / 64][SHA_WIN_CHUNKS * 256];
  uint64_t h[8];
  const bool live = sha_staged_state(i, n, vk, sig, msg, off, win[t >> 6], h);
  if (!live) return;
  uint32_t x[16];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    x[2 * j] = bswap32((uint32_t)(h[j] >> 32));
    x[2 * j + 1] = bswap32((uint32_t)h[j]);
  }
#else
  if (i >= n) return;
  uint64_t o0 = off[i], o1 = off[i + 1];
  sha_src s{sig + (size_t)i * 64, vk + (size_t)i * 32, msg + o0, o1 - o0};
  uint32_t x[16];
  sha512_src_le_words(s, x);
#endif
  sc k = sc_reduce_wide(x);
  uint4* kp = reinterpret_cast<uint4*>(k_out + (size_t)i * 8);
  kp[0] = make_uint4(k.v[0], k.v[1], k.v[2], k.v[3]);
  kp[1] = make_uint4(k.v[4], k.v[5], k.v[6], k.v[7]);
}

// ZIP215 decode (K2) of every signature's R_i -> points[1 + i] and of every distinct key j (its
// first signature's raw bytes, src/batch.rs:183-185) -> points[1 + n + j], in ONE launch: lanes
// [0, n) decode R_i, lanes [n, n + m) decode the keys (m is read on the device; surplus lanes
// exit). Keys registered in the context's cache copy their decoded record instead. Per-item and
// per-key failure bits are kept for the grouped fallback.
__device__ __forceinline__ void copy_record(uint32_t* __restrict__ pts, uint32_t idx, const uint32_t* __restrict__ src) {
  const uint4* q = reinterpret_cast<const uint4*>(src);
  uint4* d = reinterpret_cast<uint4*>(pts + (size_t)idx * NIELS_WORDS);
#pragma unroll
  for (int i = 0; i < NIELS_WORDS / 4; ++i) d[i] = q[i];
}

// [2^128]P as affine Niels (split coefficients, a key missing from the cache: the slow path; the
// host stops planning split coefficients after such a batch)
__device__ __noinline__ ge_niels shift128_niels(ge_p3 P) {
  for (int k = 0; k < 128; ++k) P = ge_dbl(P, k == 127);
  const fe zi = fe_invert(P.Z);
  ge_p3 A;
  A.X = fe_mul(P.X, zi);
  A.Y = fe_mul(P.Y, zi);
  A.Z = fe_one();
  A.T = fe_mul(A.X, A.Y);
  return ge_to_niels_affine(A);
}

// n: the batch's items (key points sit at 1 + n + j); this launch decodes R of items
// [r0, r0 + rcnt) and, on `klanes` key lanes (0: none), the distinct keys (a chunked host-buffer
// call decodes each chunk's R as it lands and the keys once the key grouping is done). The key
// count m is only known on the device: the host sizes klanes from the previous grouped batch, and
// a lane decodes keys j, j + klanes, ... when m is larger.
#ifndef EDC_DEC_LDS_PAD
#define EDC_DEC_LDS_PAD 0
#endif
#ifndef EDC_DEC_OCC
#define EDC_DEC_OCC 4   // waves per SIMD the decode is compiled for (128 VGPRs; 5 -> 96 with spills outside the squaring loops)
#endif
__global__ void __launch_bounds__(256, EDC_DEC_OCC) k_decompress(uint32_t n, uint32_t r0, uint32_t rcnt, uint32_t klanes,
                                                       const uint8_t* __restrict__ sig,
                                                       const uint8_t* __restrict__ vk,
                                                       const uint32_t* __restrict__ key_rep, int per_sig_host,
                                                       uint32_t* __restrict__ pts, uint8_t* __restrict__ itembad_r,
                                                       uint8_t* __restrict__ keybad, int* __restrict__ flags,
                                                       KeyCacheView kcache, int split) {
  const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
  BATCH_STAMP(flags, BST_DECODE);
#if EDC_DEC_LDS_PAD
  // measurement knob: LDS the decode never reads, so that at most 160 KB / pad decode workgroups
  // share a CU and the rest of its VGPRs stay free for the other batches' kernels
  __shared__ uint32_t dec_pad[EDC_DEC_LDS_PAD / 4];
  asm volatile("" :: "v"(dec_pad));
#endif
  uint32_t w[8];
  if (lane < rcnt) {
    const uint32_t i = r0 + lane;
    ld_words8(sig + (size_t)i * 64, w);
    ge_p3 P;
    const bool ok = ge_decompress(w, P);
    st_niels(pts, 1 + i, ge_to_niels_affine(P));
    itembad_r[i] = ok ? 0 : ITEM_BAD_R;   // its own array: k_coef writes the s bits concurrently
    if (!ok) atomicOr(&flags[FLAG_BAD], 1);
    return;
  }
  const uint32_t kbase = (rcnt + 63u) & ~63u;   // key lanes start on a wave boundary (no R/key divergence)
  if (lane < kbase || lane - kbase >= klanes) return;
  const uint32_t m = (uint32_t)flags[FLAG_NKEYS];
  const bool per_sig = per_sig_host || flags[FLAG_OVF];
  for (uint32_t j = lane - kbase; j < m; j += klanes) {
  ld_words8(vk + (size_t)(per_sig ? j : key_rep[j]) * 32, w);
  const int ci = kc_lookup(kcache, w);
  bool ok;
  if (ci >= 0) {                    // registered key: A = comb[0][0], decoded once per context
    const uint32_t* comb = kcache.comb + (size_t)ci * COMB_ENTRIES * NIELS_WORDS;
    copy_record(pts, 1 + n + j, comb);
    if (split) copy_record(pts, split_hi_point(n, m, j), comb + (size_t)COMB_SHIFT128 * NIELS_WORDS);
    ok = kcache.ok[ci] != 0;
  } else {
    ge_p3 P;
    ok = ge_decompress(w, P);
    st_niels(pts, 1 + n + j, ge_to_niels_affine(P));
    if (kcache.table) atomicAdd(&flags[FLAG_UNCACHED], 1);
    if (split) st_niels(pts, split_hi_point(n, m, j), shift128_niels(P));
  }
  if (split && j == 0) copy_record(pts, split_b_hi_point(n, m), kcache.bcomb + (size_t)COMB_SHIFT128 * NIELS_WORDS);
  keybad[j] = ok ? 0 : 1;
  if (!ok) atomicOr(&flags[FLAG_BAD], 1);
  }
}

// Slot hash of the raw key bytes under a 64-bit per-context secret (drawn from OS randomness
// when the context is created, re-mixed per batch): callers cannot aim chosen keys at one slot
// without it. Probing is additionally capped (KEY_PROBE_CAP): a batch whose keys still collide
// switches to one key term per signature (FLAG_OVF), which is the same group element, so
// adversarial keys cost at most the distinct-key path.
constexpr uint32_t KEY_PROBE_CAP = 64;
__device__ __forceinline__ uint32_t key_hash(const uint32_t w[8], uint32_t s0, uint32_t s1) {
  uint32_t h = s0 ^ 0x9E3779B9u, g = s1 ^ 0x7F4A7C15u;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    h ^= w[j];
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    g += w[j] ^ h;
    g *= 0xC2B2AE35u;
    g ^= g >> 16;
  }
  h ^= (g << 11) | (g >> 21);
  h *= 0x27D4EB2Fu;
  h ^= h >> 15;
  return h;
}

// Open-addressing insert keyed by the raw 32 key bytes. table[] holds the index of the first
// signature that claimed the slot (0xFFFFFFFF = empty; a slot never changes once claimed, so a
// stale relaxed read is safe). The claimer also draws the dense key index.
__device__ __forceinline__ void key_insert_one(uint32_t i, const uint8_t* __restrict__ vk,
                                               uint32_t* __restrict__ table, uint32_t tmask, uint32_t salt0,
                                               uint32_t salt1, uint32_t probe_cap, uint32_t* __restrict__ slot_key,
                                               uint32_t* __restrict__ key_slot_of_sig, uint32_t* __restrict__ key_rep,
                                               unsigned long long* __restrict__ key_acc, int* __restrict__ flags) {
  uint32_t w[8];
  ld_words8(vk + (size_t)i * 32, w);
  uint32_t h = key_hash(w, salt0, salt1) & tmask;
  for (uint32_t probe = 0; probe < probe_cap; ++probe) {
    // plain (L1-cached) first probe: a slot never changes once claimed, and a stale EMPTY is
    // resolved by the CAS below, so the hot validator slots are served from L1
    uint32_t cur = __hip_atomic_load(&table[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (cur == 0xFFFFFFFFu) {
      uint32_t prev = atomicCAS(&table[h], 0xFFFFFFFFu, i);
      if (prev == 0xFFFFFFFFu) {
        // dense key index: one counter atomic per wave for all lanes claiming in this round
        // (distinct-key batches claim on every lane; a per-lane atomic on one address serializes)
        const uint64_t act = __ballot(1);
        const int leader = __ffsll((unsigned long long)act) - 1;
        const uint32_t lane = __lane_id();
        const uint32_t rank = (uint32_t)__popcll(act & ((1ull << lane) - 1));
        uint32_t base = 0;
        if ((int)lane == leader) base = (uint32_t)atomicAdd(&flags[FLAG_NKEYS], __popcll(act));
        base = __shfl(base, leader);
        uint32_t kidx = base + rank;
        slot_key[h] = kidx;
        key_rep[kidx] = i;
        key_slot_of_sig[i] = h;
#pragma unroll
        for (int j = 0; j < KEY_ACC_LIMBS; ++j) key_acc[(size_t)kidx * KEY_ACC_LIMBS + j] = 0;
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
  atomicOr(&flags[FLAG_OVF], 1);    // give up grouping for this batch (see KEY_PROBE_CAP)
}

__global__ void __launch_bounds__(256) k_key_insert(uint32_t n, const uint8_t* __restrict__ vk,
                                                    uint32_t* __restrict__ table, uint32_t tmask,
                                                    uint32_t salt0, uint32_t salt1, uint32_t probe_cap,
                                                    uint32_t* __restrict__ slot_key,
                                                    uint32_t* __restrict__ key_slot_of_sig,
                                                    uint32_t* __restrict__ key_rep,
                                                    unsigned long long* __restrict__ key_acc,
                                                    int* __restrict__ flags) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) key_insert_one(i, vk, table, tmask, salt0, salt1, probe_cap, slot_key, key_slot_of_sig, key_rep,
                            key_acc, flags);
}

// Seeding pass over a sample of KEY_SEED_SAMPLE signatures (multiplicative hashing of the sample
// index, so that no period in the key order -- e.g. round-robin validators -- aliases): the table is empty
// at the start of a batch, and without it every concurrently resident lane of k_key_insert sees
// its validator's slot still empty and CASes it -- a million CAS on ~150 words, serialized in
// L2 (0.1 ms at 2^20). With the validators claimed here, the full pass finds them with plain loads.
constexpr uint32_t KEY_SEED_SAMPLE = 4096;
__global__ void __launch_bounds__(256) k_key_seed(uint32_t n, const uint8_t* __restrict__ vk,
                                                  uint32_t* __restrict__ table, uint32_t tmask,
                                                  uint32_t salt0, uint32_t salt1, uint32_t probe_cap,
                                                  uint32_t* __restrict__ slot_key,
                                                  uint32_t* __restrict__ key_slot_of_sig,
                                                  uint32_t* __restrict__ key_rep,
                                                  unsigned long long* __restrict__ key_acc,
                                                  int* __restrict__ flags) {
  const uint32_t i = (uint32_t)(((uint64_t)(blockIdx.x * blockDim.x + threadIdx.x) * 2654435761u) % n);
  key_insert_one(i, vk, table, tmask, salt0, salt1, probe_cap, slot_key, key_slot_of_sig, key_rep, key_acc, flags);
}

// dense key index per signature; after a probe overflow the batch falls back to one key term
// per signature (m = n), decided here on the device. kcap: the most distinct keys the caller's
// per-(range, key) sums have room for (several batches in one launch); more also fall back.
__global__ void __launch_bounds__(256) k_key_index(uint32_t n, const uint32_t* __restrict__ key_slot_of_sig,
                                                   const uint32_t* __restrict__ slot_key,
                                                   uint32_t* __restrict__ key_index, int* __restrict__ flags,
                                                   uint32_t kcap) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // every lane decides from the values k_key_insert left: FLAG_NKEYS is only rewritten to n,
  // which is > kcap whenever the original count was
  const bool over = (uint32_t)flags[FLAG_NKEYS] > kcap;
  if (flags[FLAG_OVF] || over) {
    if (i == 0) {
      flags[FLAG_OVF] = 1;
      flags[FLAG_NKEYS] = (int)n;
    }
    return;
  }
  key_index[i] = slot_key[key_slot_of_sig[i]];
}

struct seed8 { uint32_t w[8]; };

constexpr int COEF_SIGS_PER_THREAD = 8;             // two ChaCha blocks -> z for 8 signatures
constexpr int COEF_SLOTS = 256;                     // LDS key-accumulator slots
constexpr int PL = 12;                              // limbs of a 128 x 256-bit product
static_assert(PL == KEY_ACC_LIMBS, "limb sums");
// k_coef's per-workgroup slot dump (batch mode): nwg x COEF_SLOTS tags, then the 64-bit sums
__device__ __forceinline__ unsigned long long* coef_part_sums(uint32_t* part, uint32_t nwg) {
  return reinterpret_cast<unsigned long long*>(part + (((size_t)nwg * COEF_SLOTS + 1) & ~(size_t)1));
}
static_assert(COEF_CHUNK == 256 * COEF_SIGS_PER_THREAD, "k_coef chunk (edc_common.h)");

// r[0..11] = z (4 limbs) * s (8 limbs), exact
__device__ __forceinline__ void mul_128x256(const uint32_t z[4], const uint32_t s[8], uint32_t r[PL]) {
#pragma unroll
  for (int i = 0; i < PL; ++i) r[i] = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint64_t t = (uint64_t)z[i] * s[j] + r[i + j] + c;
      r[i + j] = (uint32_t)t;
      c = t >> 32;
    }
    r[i + 8] = (uint32_t)c;
  }
}

// Coefficients of the batch equation (reference src/batch.rs:193-198):
//   B_coeff -= z*s ; A_coeff[key] += z*k ; R coefficient = z.
// The 381-bit products are NOT reduced per signature: their 32-bit limbs are summed exactly in
// 64-bit accumulators (per thread in registers for sum z*s, per key through LDS slots / global
// 64-bit atomics for sum z*k) and reduced mod l once (k_key_final). Integer sums are
// order-independent, so any schedule gives bit-identical coefficients.
// Range mode (rsize > 0, grouped fallback): the sums are kept per (range, key) pair, index
// (i / rsize) * m + key, and per range for z*s (rsize is a multiple of COEF_CHUNK, so a workgroup
// never straddles two ranges).
__global__ void __launch_bounds__(256) k_coef(uint32_t n, const uint8_t* __restrict__ sig,
                                              const uint32_t* __restrict__ kscal,
                                              const uint8_t* __restrict__ zexp, seed8 seed,
                                              uint64_t zbase, const uint32_t* __restrict__ key_index,
                                              uint32_t* __restrict__ scal,
                                              unsigned long long* __restrict__ key_acc,
                                              unsigned long long* __restrict__ u_acc,
                                              uint8_t* __restrict__ itembad,
                                              int* __restrict__ flags, int per_sig_host, uint32_t rsize, uint32_t m,
                                              uint32_t* __restrict__ coef_part, int split, uint32_t item0,
                                              uint32_t iend) {
  __shared__ uint32_t tag[COEF_SLOTS];
  __shared__ unsigned long long acc[COEF_SLOTS][PL];
  __shared__ unsigned long long red[4][PL];
  BATCH_STAMP(flags, BST_COEF);
  const bool per_sig = per_sig_host || flags[FLAG_OVF];
  for (int s = threadIdx.x; s < COEF_SLOTS; s += blockDim.x) {
    tag[s] = 0xFFFFFFFFu;
#pragma unroll
    for (int j = 0; j < PL; ++j) acc[s][j] = 0;
  }
  __syncthreads();
  unsigned long long ua[PL];
#pragma unroll
  for (int j = 0; j < PL; ++j) ua[j] = 0;
  bool bad = false, karg = false;
  // items [item0, iend) of the n-item batch (item0 a multiple of COEF_CHUNK: a chunked host-buffer
  // call launches one range per chunk as it lands; workgroup wg's slot dump sits at its place in
  // the whole batch's layout)
  const uint32_t wg = item0 / COEF_CHUNK + blockIdx.x, nwg = (n + COEF_CHUNK - 1) / COEF_CHUNK;
  const uint32_t base = wg * COEF_CHUNK;
  const uint32_t pair0 = rsize ? (base / rsize) * m : 0u;
  for (int grp = 0; grp < COEF_SIGS_PER_THREAD / 4; ++grp) {
    const uint32_t i0 = base + 4 * (threadIdx.x + 256 * grp);
    if (i0 >= iend) break;
    uint32_t blk[16];
    const bool aligned = ((zbase + i0) & 3) == 0;
    if (!zexp && aligned) chacha20_block(seed.w, (zbase + i0) >> 2, blk);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t i = i0 + q;
      if (i >= iend) break;
      uint32_t z[4];
      if (zexp) {
        const uint4 zz = *reinterpret_cast<const uint4*>(zexp + (size_t)i * 16);
        z[0] = zz.x; z[1] = zz.y; z[2] = zz.z; z[3] = zz.w;
      } else if (aligned) {
#pragma unroll
        for (int j = 0; j < 4; ++j) z[j] = blk[4 * q + j];
      } else {
        uint32_t b2[16];
        chacha20_block(seed.w, (zbase + i) >> 2, b2);
        const int o = (int)((zbase + i) & 3);
#pragma unroll
        for (int j = 0; j < 4; ++j) z[j] = b2[4 * o + j];
      }
      uint32_t sw[8], kw[8];
      ld_words8(sig + (size_t)i * 64 + 32, sw);
      const uint4* kp = reinterpret_cast<const uint4*>(kscal + (size_t)i * 8);
      uint4 k0 = kp[0], k1 = kp[1];
      kw[0] = k0.x; kw[1] = k0.y; kw[2] = k0.z; kw[3] = k0.w; kw[4] = k1.x; kw[5] = k1.y; kw[6] = k1.z; kw[7] = k1.w;
      const bool s_bad = !sc_is_canonical(sw);
      bad |= s_bad;
      karg |= !sc_is_canonical(kw);   // k from Scalar::from_hash is < l; only a prehashed caller can break it
      if (itembad) itembad[i] = s_bad ? ITEM_BAD_S : 0;   // first writer of the batch's per-item bits
      uint32_t u[PL], v[PL];
      mul_128x256(z, sw, u);
      mul_128x256(z, kw, v);
#pragma unroll
      for (int j = 0; j < PL; ++j) ua[j] += u[j];
      uint4* sp = reinterpret_cast<uint4*>(scal + (size_t)(1 + i) * 8);
      sp[0] = make_uint4(z[0], z[1], z[2], z[3]);
      sp[1] = make_uint4(0, 0, 0, 0);
      if (per_sig) {               // ungrouped keys: A_i's coefficient is z_i k_i mod l itself
        uint32_t x[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) x[j] = j < PL ? v[j] : 0u;
        const sc a = sc_reduce_wide(x);
        uint4* ap = reinterpret_cast<uint4*>(scal + (size_t)(1 + n + i) * 8);
        ap[0] = make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]);
        if (split) {                 // lo on A_i, hi on [2^128]A_i (key layout m = n)
          ap[1] = make_uint4(0, 0, 0, 0);
          uint4* hp = reinterpret_cast<uint4*>(scal + (size_t)split_hi_point(n, n, i) * 8);
          hp[0] = make_uint4(a.v[4], a.v[5], a.v[6], a.v[7]);
          hp[1] = make_uint4(0, 0, 0, 0);
        } else {
          ap[1] = make_uint4(a.v[4], a.v[5], a.v[6], a.v[7]);
        }
        continue;
      }
      const uint32_t key = pair0 + key_index[i];
      const uint32_t slot = key & (COEF_SLOTS - 1);
      const uint32_t prev = atomicCAS(&tag[slot], 0xFFFFFFFFu, key);
      if (prev == 0xFFFFFFFFu || prev == key) {
#pragma unroll
        for (int j = 0; j < PL; ++j) atomicAdd(&acc[slot][j], (unsigned long long)v[j]);
      } else {
#pragma unroll
        for (int j = 0; j < PL; ++j) atomicAdd(&key_acc[(size_t)key * PL + j], (unsigned long long)v[j]);
      }
    }
  }
  if (bad) atomicOr(&flags[FLAG_BAD], 1);
  if (karg) atomicOr(&flags[FLAG_KARG], 1);
  // workgroup reduction of the per-thread z*s limb sums (64-bit shuffles, then LDS)
#pragma unroll
  for (int j = 0; j < PL; ++j) {
    unsigned long long x = ua[j];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_down(x, d, 64);
    ua[j] = x;
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < PL; ++j) red[wv][j] = ua[j];
  }
  __syncthreads();
  if (threadIdx.x < PL) {
    unsigned long long x = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    atomicAdd(&u_acc[(rsize ? (size_t)(base / rsize) * PL : 0) + threadIdx.x], x);
  }
  if (coef_part) {
    // batch mode: this workgroup's key slots go out as plain stores, merged per slot by
    // k_coef_merge (a few validators' sums hit by every workgroup made the global atomics
    // serialize: 0.09 of the 0.17 ms of this phase at 2^20 votes from 150 keys)
    uint32_t* ptag = coef_part + (size_t)wg * COEF_SLOTS;
    unsigned long long* psum = coef_part_sums(coef_part, nwg) + (size_t)wg * COEF_SLOTS * PL;
    for (int s = threadIdx.x; s < COEF_SLOTS; s += blockDim.x) {
      ptag[s] = tag[s];
      if (tag[s] != 0xFFFFFFFFu) {
#pragma unroll
        for (int j = 0; j < PL; ++j) psum[(size_t)s * PL + j] = acc[s][j];
      }
    }
    return;
  }
  for (int s = threadIdx.x; s < COEF_SLOTS; s += blockDim.x) {
    const uint32_t key = tag[s];
    if (key != 0xFFFFFFFFu) {
#pragma unroll
      for (int j = 0; j < PL; ++j) atomicAdd(&key_acc[(size_t)key * PL + j], acc[s][j]);
    }
  }
}

// Per LDS slot s: the sums the k_coef workgroups left for s. The slot's usual key (the first
// non-empty tag seen) is summed in registers and added once; other keys sharing the slot (more
// than COEF_SLOTS distinct keys) go to key_acc by atomics, which are then rarely contended.
__global__ void __launch_bounds__(256) k_coef_merge(uint32_t nwg, const uint32_t* __restrict__ coef_part,
                                                    unsigned long long* __restrict__ key_acc) {
  __shared__ uint32_t lead;
  __shared__ unsigned long long red[4][PL];
  const uint32_t s = blockIdx.x, t = threadIdx.x;
  const unsigned long long* psum = coef_part_sums(const_cast<uint32_t*>(coef_part), nwg);
  if (t == 0) lead = 0xFFFFFFFFu;
  __syncthreads();
  for (uint32_t w = t; w < nwg; w += blockDim.x) {
    const uint32_t tg = coef_part[(size_t)w * COEF_SLOTS + s];
    if (tg != 0xFFFFFFFFu) atomicCAS(&lead, 0xFFFFFFFFu, tg);
  }
  __syncthreads();
  const uint32_t L = lead;
  if (L == 0xFFFFFFFFu) return;                 // uniform: no workgroup used this slot
  unsigned long long mine[PL];
#pragma unroll
  for (int j = 0; j < PL; ++j) mine[j] = 0;
  for (uint32_t w = t; w < nwg; w += blockDim.x) {
    const uint32_t tg = coef_part[(size_t)w * COEF_SLOTS + s];
    if (tg == 0xFFFFFFFFu) continue;
    const unsigned long long* src = psum + ((size_t)w * COEF_SLOTS + s) * PL;
    if (tg == L) {
#pragma unroll
      for (int j = 0; j < PL; ++j) mine[j] += src[j];
    } else {
#pragma unroll
      for (int j = 0; j < PL; ++j) atomicAdd(&key_acc[(size_t)tg * PL + j], src[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < PL; ++j) {
    unsigned long long x = mine[j];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_down(x, d, 64);
    mine[j] = x;
  }
  if ((t & 63) == 0) {
#pragma unroll
    for (int j = 0; j < PL; ++j) red[t >> 6][j] = mine[j];
  }
  __syncthreads();
  if (t < PL) atomicAdd(&key_acc[(size_t)L * PL + t], red[0][t] + red[1][t] + red[2][t] + red[3][t]);
}

// sum_j L[j] * 2^(32 j) mod l for PL limb sums L[j] < 2^64 (value < 2^448)
__device__ __forceinline__ sc reduce_limb_sums(const unsigned long long* L) {
  uint32_t x[16];
  unsigned long long carry = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    unsigned long long lo = j < PL ? (L[j] & 0xFFFFFFFFull) : 0ull;
    unsigned long long hi = (j >= 1 && j <= PL) ? (L[j - 1] >> 32) : 0ull;
    unsigned long long t = lo + hi + carry;
    x[j] = (uint32_t)t;
    carry = t >> 32;
  }
  return sc_reduce_wide(x);
}

__device__ __forceinline__ void store_scalar(uint32_t* scal, size_t idx, const sc& c) {
  uint4* d = reinterpret_cast<uint4*>(scal + idx * 8);
  d[0] = make_uint4(c.v[0], c.v[1], c.v[2], c.v[3]);
  d[1] = make_uint4(c.v[4], c.v[5], c.v[6], c.v[7]);
}

// c = lo + 2^128 hi: lo -> scalar lo_idx, hi -> scalar hi_idx (split coefficients, edc_common.h)
__device__ __forceinline__ void store_split(uint32_t* scal, size_t lo_idx, size_t hi_idx, const sc& c) {
  uint4* l = reinterpret_cast<uint4*>(scal + lo_idx * 8);
  uint4* h = reinterpret_cast<uint4*>(scal + hi_idx * 8);
  l[0] = make_uint4(c.v[0], c.v[1], c.v[2], c.v[3]);
  l[1] = make_uint4(0, 0, 0, 0);
  h[0] = make_uint4(c.v[4], c.v[5], c.v[6], c.v[7]);
  h[1] = make_uint4(0, 0, 0, 0);
}

// Batch: A_coeff of key j = sum z k mod l -> scalar of point n+1+j; B_coeff = -sum z s -> point 0
// (split: the high halves go to the [2^128] points).
__global__ void __launch_bounds__(256) k_key_final(uint32_t n, const unsigned long long* __restrict__ key_acc,
                                                   const unsigned long long* __restrict__ u_acc,
                                                   uint32_t* __restrict__ scal,
                                                   const int* __restrict__ flags, int per_sig_host, int split) {
  const uint32_t j0 = blockIdx.x * blockDim.x + threadIdx.x;
  const bool per_sig = per_sig_host || flags[FLAG_OVF];
  const uint32_t mk = (uint32_t)flags[FLAG_NKEYS];          // key points of the layout
  const uint32_t m = per_sig ? 0u : mk;                     // keys whose sums are reduced here
  for (uint32_t j = j0; j < m; j += gridDim.x * blockDim.x) {
    const sc c = reduce_limb_sums(key_acc + (size_t)j * PL);
    if (split) store_split(scal, 1 + n + j, split_hi_point(n, mk, j), c);
    else store_scalar(scal, 1 + n + j, c);
  }
  if (j0 == 0) {
    const sc b = sc_sub(sc_zero(), reduce_limb_sums(u_acc));
    if (split) store_split(scal, 0, split_b_hi_point(n, mk), b);
    else store_scalar(scal, 0, b);
  }
}

// Range mode (grouped fallback): listed MSM terms (point, range, scalar). Pairs q = g m + j
// (grouped keys) -> (n+1+j, g, sum z k of key j in range g); then one B term per range g ->
// (0, g, -sum z s of range g). Absent pairs have scalar 0 and produce no digits.
__global__ void __launch_bounds__(256) k_range_terms(uint32_t n, uint32_t nranges, uint32_t m,
                                                     const unsigned long long* __restrict__ key_acc,
                                                     const unsigned long long* __restrict__ u_acc,
                                                     uint32_t* __restrict__ xpt, uint32_t* __restrict__ xrg,
                                                     uint32_t* __restrict__ xscal) {
  const uint32_t npair = nranges * m;
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < npair + nranges; q += gridDim.x * blockDim.x) {
    if (q < npair) {
      xpt[q] = 1 + n + q % m;
      xrg[q] = q / m;
      store_scalar(xscal, q, reduce_limb_sums(key_acc + (size_t)q * PL));
    } else {
      const uint32_t g = q - npair;
      xpt[q] = 0;
      xrg[q] = g;
      store_scalar(xscal, q, sc_sub(sc_zero(), reduce_limb_sums(u_acc + (size_t)g * PL)));
    }
  }
}

// Several batches in one launch (nr equal ranges of n / nr items): listed MSM terms from the
// per-(range, key) sums, laid out key-major per range (sum of key j in range g at g * kstride + j,
// so the host needs no key count): q < nr m -> (n+1+j, g, sum z k), then one B term per range.
// m comes from the batch's key grouping (0 with one key term per signature: those terms are
// point terms, k_coef wrote their scalars).
__global__ void __launch_bounds__(256) k_multi_terms(uint32_t n, uint32_t nr, uint32_t kstride,
                                                     const unsigned long long* __restrict__ key_acc,
                                                     const unsigned long long* __restrict__ u_acc,
                                                     const int* __restrict__ flags, int per_sig_host,
                                                     uint32_t* __restrict__ xpt, uint32_t* __restrict__ xrg,
                                                     uint32_t* __restrict__ xscal) {
  const bool per_sig = per_sig_host || flags[FLAG_OVF];
  const uint32_t m = per_sig ? 0u : (uint32_t)flags[FLAG_NKEYS];
  const uint32_t npair = nr * m;
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < npair + nr; q += gridDim.x * blockDim.x) {
    if (q < npair) {
      const uint32_t g = q / m, j = q - g * m;
      xpt[q] = 1 + n + j;
      xrg[q] = g;
      store_scalar(xscal, q, reduce_limb_sums(key_acc + ((size_t)g * kstride + j) * PL));
    } else {
      const uint32_t g = q - npair;
      xpt[q] = 0;
      xrg[q] = g;
      store_scalar(xscal, q, sc_sub(sc_zero(), reduce_limb_sums(u_acc + (size_t)g * PL)));
    }
  }
}

// Range mode: rbad[g] = 1 iff range g holds an item whose R or s failed, or whose key failed to
// decode (such ranges are verified item by item whatever their partial point).
__global__ void __launch_bounds__(256) k_range_prebad(uint32_t n, uint32_t rsize, const uint8_t* __restrict__ itembad,
                                                      const uint8_t* __restrict__ itembad_r,
                                                      const uint8_t* __restrict__ keybad,
                                                      const uint32_t* __restrict__ key_index, int per_sig_host,
                                                      const int* __restrict__ flags, uint8_t* __restrict__ rbad) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bool per_sig = per_sig_host || (flags && flags[FLAG_OVF]);
  if (itembad[i] || itembad_r[i] || keybad[per_sig ? i : key_index[i]]) rbad[i / rsize] = 1;
}

__global__ void k_init_basepoint(uint32_t* pts) {
  if (threadIdx.x == 0 && blockIdx.x == 0) st_niels(pts, 0, ge_to_niels_affine(ge_basepoint()));
}

// ---------------------------------------------------------------- launchers
static inline uint32_t cdiv(uint64_t a, uint32_t b) { return (uint32_t)((a + b - 1) / b); }
static inline uint32_t grid_cap(uint32_t g, uint32_t cap) { return g < cap ? g : cap; }

void launch_challenge(hipStream_t st, uint32_t n, const uint8_t* vk, const uint8_t* sig,
                      const uint8_t* msg, const uint64_t* off, uint32_t* k) {
  if (n)
    hipLaunchKernelGGL(k_challenge, dim3(cdiv(n, SHA_THREADS)), dim3(SHA_THREADS), 0, st, n, vk, sig, msg, off, k);
}
void launch_decompress_range(hipStream_t st, uint32_t n, uint32_t r0, uint32_t rcnt, uint32_t klanes, const uint8_t* sig,
                             const uint8_t* vk, const uint32_t* key_rep, bool per_sig, uint32_t* pts, uint8_t* itembad,
                             uint8_t* keybad, int* flags, const KeyCacheView& kc, bool split) {
  // lanes [0, rcnt) decode R; the key lanes start at the next wave boundary. A wave holding both
  // would run both decodes one after the other, which doubles a small batch's decode latency.
  // Small launches use one wave per workgroup so that the waves spread over CUs instead of sharing
  // SIMDs.
  if (klanes > n) klanes = n;
  const uint64_t lanes = ((rcnt + 63ull) & ~63ull) + klanes;
  if (!n || !lanes) return;
  const uint32_t block = lanes <= 16384 ? 64 : 256;
  hipLaunchKernelGGL(k_decompress, dim3(cdiv(lanes, block)), dim3(block), 0, st, n, r0, rcnt, klanes, sig, vk,
                     key_rep, per_sig ? 1 : 0, pts, itembad, keybad, flags, kc, split ? 1 : 0);
}
void launch_decompress(hipStream_t st, uint32_t n, const uint8_t* sig, const uint8_t* vk, const uint32_t* key_rep,
                       bool per_sig, uint32_t* pts, uint8_t* itembad, uint8_t* keybad, int* flags,
                       const KeyCacheView& kc, bool split, uint32_t klanes) {
  launch_decompress_range(st, n, 0, n, klanes ? klanes : n, sig, vk, key_rep, per_sig, pts, itembad, keybad, flags, kc,
                          split);
}
void launch_keys(hipStream_t st, uint32_t n, const uint8_t* vk, uint32_t* table, uint32_t tmask,
                 const uint32_t salt[2], bool force_overflow, uint32_t* slot_key, uint32_t* key_slot_of_sig,
                 uint32_t* key_rep, uint32_t* key_index, unsigned long long* key_acc, int* flags, uint32_t kcap) {
  if (!n) return;
  const uint32_t cap = force_overflow ? 0u : KEY_PROBE_CAP;
  if (n > 4 * KEY_SEED_SAMPLE) {
    hipLaunchKernelGGL(k_key_seed, dim3(KEY_SEED_SAMPLE / 256), dim3(256), 0, st, n, vk, table, tmask,
                       salt[0], salt[1], cap, slot_key, key_slot_of_sig, key_rep, key_acc, flags);
  }
  hipLaunchKernelGGL(k_key_insert, dim3(cdiv(n, 256)), dim3(256), 0, st, n, vk, table, tmask, salt[0], salt[1], cap,
                     slot_key, key_slot_of_sig, key_rep, key_acc, flags);
  hipLaunchKernelGGL(k_key_index, dim3(cdiv(n, 256)), dim3(256), 0, st, n, key_slot_of_sig, slot_key,
                     key_index, flags, kcap);
}
// One launch for the per-batch resets (flags, global coefficient sums, result block, key table,
// MSM bin counts) instead of five runtime fills: each fill is a launch of its own, ~8 us apiece in
// the latency of a small batch.
__global__ void __launch_bounds__(256) k_init_batch(int* __restrict__ flags, int nkeys, unsigned long long* __restrict__ u_acc,
                                                    uint32_t* __restrict__ d_out, uint32_t* __restrict__ table, uint32_t T,
                                                    uint32_t* __restrict__ counts, uint32_t nbin) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x, stride = gridDim.x * blockDim.x;
  BATCH_STAMP(flags, BST_INIT);
  if (i < FLAG_COUNT) flags[i] = (i == FLAG_NKEYS && nkeys >= 0) ? nkeys : 0;
  if (i < KEY_ACC_LIMBS) u_acc[i] = 0;
  if (i < 64) d_out[i] = 0;
  for (uint32_t j = i; j < T; j += stride) table[j] = 0xFFFFFFFFu;
  for (uint32_t j = i; j < nbin; j += stride) counts[j] = 0;
}

void launch_init_batch(hipStream_t st, int* flags, int nkeys, unsigned long long* u_acc, uint8_t* d_out, uint32_t* table,
                       uint32_t T, uint32_t* counts, uint32_t nbin) {
  const uint32_t work = T > nbin ? T : nbin;
  uint32_t grid = cdiv(work > 256 ? work : 256, 256);
  if (grid > 4096) grid = 4096;
  hipLaunchKernelGGL(k_init_batch, dim3(grid), dim3(256), 0, st, flags, nkeys, u_acc, reinterpret_cast<uint32_t*>(d_out),
                     table, T, counts, nbin);
}

void launch_coef(hipStream_t st, uint32_t n, const uint8_t* sig, const uint32_t* k, const uint8_t* zexp,
                 const uint32_t seed[8], uint64_t zbase, const uint32_t* key_index, uint32_t* scal,
                 unsigned long long* key_acc, unsigned long long* u_acc, uint8_t* itembad, int* flags,
                 bool per_sig, uint32_t* coef_part, bool split) {
  seed8 s;
  for (int j = 0; j < 8; ++j) s.w[j] = seed[j];
  if (n) {
    const uint32_t nwg = cdiv(n, COEF_CHUNK);
    uint32_t* part = per_sig ? nullptr : coef_part;
    hipLaunchKernelGGL(k_coef, dim3(nwg), dim3(256), 0, st, n, sig, k, zexp, s, zbase, key_index, scal, key_acc,
                       u_acc, itembad, flags, per_sig ? 1 : 0, 0u, 0u, part, split ? 1 : 0, 0u, n);
  }
  launch_coef_finish(st, n, key_acc, u_acc, scal, flags, per_sig, coef_part, split);
}
void launch_coef_range(hipStream_t st, uint32_t n, uint32_t item0, uint32_t cnt, const uint8_t* sig, const uint32_t* k,
                       const uint8_t* zexp, const uint32_t seed[8], uint64_t zbase, const uint32_t* key_index,
                       uint32_t* scal, unsigned long long* key_acc, unsigned long long* u_acc, uint8_t* itembad,
                       int* flags, bool per_sig, uint32_t* coef_part, bool split) {
  seed8 s;
  for (int j = 0; j < 8; ++j) s.w[j] = seed[j];
  if (cnt)
    hipLaunchKernelGGL(k_coef, dim3(cdiv(cnt, COEF_CHUNK)), dim3(256), 0, st, n, sig, k, zexp, s, zbase, key_index,
                       scal, key_acc, u_acc, itembad, flags, per_sig ? 1 : 0, 0u, 0u, per_sig ? nullptr : coef_part,
                       split ? 1 : 0, item0, item0 + cnt);
}
void launch_coef_finish(hipStream_t st, uint32_t n, unsigned long long* key_acc, unsigned long long* u_acc,
                        uint32_t* scal, int* flags, bool per_sig, uint32_t* coef_part, bool split) {
  if (n && !per_sig)
    hipLaunchKernelGGL(k_coef_merge, dim3(COEF_SLOTS), dim3(256), 0, st, cdiv(n, COEF_CHUNK), coef_part, key_acc);
  hipLaunchKernelGGL(k_key_final, dim3(grid_cap(cdiv(n > 0 ? n : 1, 256), 1024)), dim3(256), 0, st, n, key_acc,
                     u_acc, scal, flags, per_sig ? 1 : 0, split ? 1 : 0);
}
size_t coef_part_words(size_t cap_n) {
  const size_t nwg = (cap_n + COEF_CHUNK - 1) / COEF_CHUNK;
  return ((nwg * COEF_SLOTS + 1) & ~(size_t)1) + nwg * COEF_SLOTS * PL * 2;
}

void launch_range_coef(hipStream_t st, uint32_t n, uint32_t rsize, uint32_t nranges, uint32_t m, bool per_sig,
                       const uint8_t* sig, const uint32_t* k, const uint8_t* zexp, const uint32_t seed[8],
                       uint64_t zbase, const uint32_t* key_index, uint32_t* scal, unsigned long long* key_acc,
                       unsigned long long* u_acc, int* flags, uint32_t* xpt, uint32_t* xrg, uint32_t* xscal) {
  seed8 s;
  for (int j = 0; j < 8; ++j) s.w[j] = seed[j];
  const uint32_t mm = per_sig ? 0u : m;
  (void)hipMemsetAsync(key_acc, 0, (size_t)nranges * mm * PL * sizeof(unsigned long long), st);
  (void)hipMemsetAsync(u_acc, 0, (size_t)nranges * PL * sizeof(unsigned long long), st);
  if (n)
    hipLaunchKernelGGL(k_coef, dim3(cdiv(n, COEF_CHUNK)), dim3(256), 0, st, n, sig, k, zexp, s, zbase,
                       key_index, scal, key_acc, u_acc, (uint8_t*)nullptr, flags, per_sig ? 1 : 0, rsize, mm,
                       (uint32_t*)nullptr, 0, 0u, n);
  hipLaunchKernelGGL(k_range_terms, dim3(grid_cap(cdiv((uint64_t)nranges * (mm + 1), 256), 1024)), dim3(256), 0, st,
                     n, nranges, mm, key_acc, u_acc, xpt, xrg, xscal);
}
void launch_multi_coef(hipStream_t st, uint32_t n, uint32_t nr, uint32_t kstride, bool per_sig, const uint8_t* sig,
                       const uint32_t* k, const uint32_t seed[8], uint64_t zbase, const uint32_t* key_index,
                       uint32_t* scal, unsigned long long* key_acc, unsigned long long* u_acc, uint8_t* itembad,
                       int* flags, uint32_t* xpt, uint32_t* xrg, uint32_t* xscal) {
  seed8 s;
  for (int j = 0; j < 8; ++j) s.w[j] = seed[j];
  if (!per_sig) (void)hipMemsetAsync(key_acc, 0, (size_t)nr * kstride * PL * sizeof(unsigned long long), st);
  (void)hipMemsetAsync(u_acc, 0, (size_t)nr * PL * sizeof(unsigned long long), st);
  if (n)
    hipLaunchKernelGGL(k_coef, dim3(cdiv(n, COEF_CHUNK)), dim3(256), 0, st, n, sig, k, (const uint8_t*)nullptr, s, zbase,
                       key_index, scal, key_acc, u_acc, itembad, flags, per_sig ? 1 : 0, n / nr, kstride,
                       (uint32_t*)nullptr, 0, 0u, n);
  hipLaunchKernelGGL(k_multi_terms, dim3(grid_cap(cdiv((uint64_t)nr * (per_sig ? 1 : kstride + 1), 256), 1024)),
                     dim3(256), 0, st, n, nr, kstride, key_acc, u_acc, flags, per_sig ? 1 : 0, xpt, xrg, xscal);
}
void launch_range_prebad(hipStream_t st, uint32_t n, uint32_t rsize, const uint8_t* itembad, const uint8_t* itembad_r,
                         const uint8_t* keybad,
                         const uint32_t* key_index, bool per_sig, uint8_t* rbad, const int* flags) {
  if (n)
    hipLaunchKernelGGL(k_range_prebad, dim3(cdiv(n, 256)), dim3(256), 0, st, n, rsize, itembad, itembad_r, keybad,
                       key_index, per_sig ? 1 : 0, flags, rbad);
}
// Key-indexed host submissions (edc_batch_submit_indexed): item i's raw key bytes from the key
// cache, vk_out[i] = keys[reg[key_idx[i]]] (indices were range-checked on the host), so the
// batch pipeline downstream sees the same 32-byte keys a per-item submission would carry.
__global__ void __launch_bounds__(256) k_expand_keys(uint32_t n, const uint32_t* __restrict__ key_idx,
                                                     const uint32_t* __restrict__ reg,
                                                     const uint32_t* __restrict__ keys, uint32_t* __restrict__ vk_out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4* src = reinterpret_cast<const uint4*>(keys + (size_t)reg[key_idx[i]] * 8);
  uint4* dst = reinterpret_cast<uint4*>(vk_out + (size_t)i * 8);
  dst[0] = src[0];
  dst[1] = src[1];
}
void launch_expand_keys(hipStream_t st, uint32_t n, const uint32_t* key_idx, const uint32_t* reg,
                        const uint32_t* keys, uint8_t* vk_out) {
  if (n) hipLaunchKernelGGL(k_expand_keys, dim3(cdiv(n, 256)), dim3(256), 0, st, n, key_idx, reg, keys,
                            reinterpret_cast<uint32_t*>(vk_out));
}
// grouped fallback: the items to verify one by one, gathered into contiguous staging buffers
__global__ void __launch_bounds__(256) k_gather_items(uint32_t c, const uint32_t* __restrict__ idx,
                                                      const uint8_t* __restrict__ vk, const uint8_t* __restrict__ sig,
                                                      const uint32_t* __restrict__ k, uint8_t* __restrict__ out_vk,
                                                      uint8_t* __restrict__ out_sig, uint32_t* __restrict__ out_k) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= c) return;
  const size_t i = idx[j];
  const uint4* a = reinterpret_cast<const uint4*>(vk + i * 32);
  uint4* da = reinterpret_cast<uint4*>(out_vk + (size_t)j * 32);
  da[0] = a[0]; da[1] = a[1];
  const uint4* b = reinterpret_cast<const uint4*>(sig + i * 64);
  uint4* db = reinterpret_cast<uint4*>(out_sig + (size_t)j * 64);
  db[0] = b[0]; db[1] = b[1]; db[2] = b[2]; db[3] = b[3];
  const uint4* q = reinterpret_cast<const uint4*>(k + i * 8);
  uint4* dq = reinterpret_cast<uint4*>(out_k + (size_t)j * 8);
  dq[0] = q[0]; dq[1] = q[1];
}
void launch_gather_items(hipStream_t st, uint32_t c, const uint32_t* idx, const uint8_t* vk, const uint8_t* sig,
                         const uint32_t* k, uint8_t* out_vk, uint8_t* out_sig, uint32_t* out_k) {
  if (c) hipLaunchKernelGGL(k_gather_items, dim3(cdiv(c, 256)), dim3(256), 0, st, c, idx, vk, sig, k, out_vk, out_sig, out_k);
}
void launch_init_basepoint(hipStream_t st, uint32_t* pts) {
  hipLaunchKernelGGL(k_init_basepoint, dim3(1), dim3(64), 0, st, pts);
}

// test hook: n 64-byte LE integers -> n 32-byte canonical residues mod l (sc_reduce_wide, the
// reduction of Scalar::from_hash), so the device build of the folds meets chosen edge values
__global__ void __launch_bounds__(256) k_sc_reduce_wide(uint32_t n, const uint32_t* __restrict__ in,
                                                        uint32_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t x[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) x[j] = in[(size_t)i * 16 + j];
  const sc r = sc_reduce_wide(x);
#pragma unroll
  for (int j = 0; j < 8; ++j) out[(size_t)i * 8 + j] = r.v[j];
}
void launch_sc_reduce_wide(hipStream_t st, uint32_t n, const uint32_t* in, uint32_t* out) {
  if (n) hipLaunchKernelGGL(k_sc_reduce_wide, dim3(cdiv(n, 256)), dim3(256), 0, st, n, in, out);
}

}  // namespace edc
