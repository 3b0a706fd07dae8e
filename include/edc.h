/*
 * edc.h -- C ABI of the MI355X (gfx950) ed25519-consensus batch-verification engine.
 *
 * This is the drop-in boundary for ONE hot path of informalsystems/ed25519-consensus 2.1.0:
 * ZIP215 batch verification and its per-signature fallback. Every entry point below replaces a
 * named Rust API of the reference (file:line into the reference tree) and keeps its exact
 * semantics: non-canonical A/R encodings accepted, s must be < l, cofactored equation, batch
 * and single verification agree. A Rust shim binds these symbols.
 *
 * Conventions
 *  - Host buffers are borrowed for the duration of the call; all calls are synchronous.
 *  - Items are in QUEUE order. vk: n*32 bytes, sig: n*64 bytes (R || s), messages are one
 *    arena `msg` with n+1 offsets (message i = msg[msg_off[i] .. msg_off[i+1])).
 *  - Device-resident inputs (the *_device entries): vk / sig / k arrays 16-byte aligned; the
 *    message arena is read in whole aligned 16-byte chunks (the SHA-512 kernel stages each
 *    message through LDS by DMA), i.e. from the 16-byte boundary at or before a message's first
 *    byte to the one after its last byte; those bytes must be mapped (they are never used).
 *    Device allocations (hipMalloc, torch tensors) always satisfy both, as such chunks never cross
 *    a page; host buffers have no such rule (they are staged into the context's own buffers).
 *  - z_i = u128::from_le_bytes(ChaCha20Rng::from_seed(z_seed) keystream[16(z_base+i) ..]),
 *    i.e. gen_u128 (reference src/batch.rs:64-68) drawn in queue order. Batch verification is
 *    sound only when z is unpredictable to the signers: z_seed must come from a CSPRNG, fresh for
 *    every verification (the reference takes `impl RngCore + CryptoRng`). Fixed seeds are for
 *    reproducible tests and benchmarks only.
 *  - Return codes: EDC_OK / EDC_INVALID_SIGNATURE / EDC_MALFORMED_PUBLIC_KEY mirror
 *    ed25519_consensus::Error (reference src/error.rs:7-20); negative = runtime failure
 *    (never mapped to Ok by callers).
 *  - One context = one GPU = one HIP stream. A context must not be used from two threads at
 *    once; use one context per thread (or per GPU / process).
 */
#ifndef EDC_H
#define EDC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EDC_OK 0
#define EDC_INVALID_SIGNATURE 1      /* Error::InvalidSignature  (src/error.rs:17) */
#define EDC_MALFORMED_PUBLIC_KEY 2   /* Error::MalformedPublicKey (src/error.rs:14) */
#define EDC_ERR_HIP (-1)
#define EDC_ERR_ARG (-2)
#define EDC_ERR_NOMEM (-3)

typedef struct edc_ctx edc_ctx;

/* Number of visible GPUs (hipGetDeviceCount), or a negative error. */
int edc_device_count(void);

/* Create a context bound to one GPU (its own stream, constant tables, grow-only workspace). */
edc_ctx* edc_create(int device);
void edc_destroy(edc_ctx* ctx);
/* Text of the last runtime error on this context ("" if none). */
const char* edc_last_error(const edc_ctx* ctx);

/*
 * batch::Verifier::queue (x n) + Verifier::verify(rng)
 *   reference src/batch.rs:127-137 (queue: k = H(R||A||M), group by raw key bytes)
 *             src/batch.rs:149-217 (verify: decode, z, coalesced MSM, [8]check == 0)
 * Returns EDC_OK if the batch equation holds, EDC_INVALID_SIGNATURE otherwise (including any
 * undecodable A/R or non-canonical s, as the reference). check8 (nullable) receives the
 * compressed [8]*check point when the equation was evaluated (zeros when the batch was
 * rejected before the MSM).
 * Host-buffer synchronous calls (this one, edc_batch_verify_z, edc_batch_verify_prehashed) from
 * 2^16 items copy their inputs in chunks and start each chunk's work as it lands; for the call's
 * duration the engine runs two helper threads of its own on ctx (joined before it returns), so
 * the one-context-per-thread rule below is unchanged. Results equal the one-piece path's.
 */
int edc_batch_verify(edc_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig,
                     const uint8_t* msg, const uint64_t* msg_off, const uint8_t z_seed[32],
                     uint8_t check8[32]);

/* Same, with caller-drawn z (n*16 bytes, LE u128 per item) for RNGs other than ChaCha20. */
int edc_batch_verify_z(edc_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig,
                       const uint8_t* msg, const uint64_t* msg_off, const uint8_t* z,
                       uint8_t check8[32]);

/*
 * Device-resident variant (inputs already in this GPU's HBM, e.g. torch tensors). d_z may be
 * NULL (then z comes from z_seed at global indices z_base + i).
 */
int edc_batch_verify_device(edc_ctx* ctx, size_t n, const uint8_t* d_vk, const uint8_t* d_sig,
                            const uint8_t* d_msg, const uint64_t* d_msg_off,
                            const uint8_t z_seed[32], uint64_t z_base, const uint8_t* d_z,
                            uint8_t check8[32]);

/*
 * Asynchronous form of edc_batch_verify_device for streams of batches (a consensus node
 * verifying block after block): edc_batch_submit_device enqueues the whole pipeline on one of the
 * context's in-flight slots (16) and returns a ticket >= 0 (or <0); edc_batch_wait blocks for that
 * ticket and returns its verdict (EDC_OK / EDC_INVALID_SIGNATURE, <0 on runtime failure), with
 * optional check8 (needs want_check8), partial point and bad flag. Tickets must be waited in
 * submission order before their slot is reused; inputs must stay valid until the wait.
 * Whenever *bad is set (an undecodable R or key, or s >= l in the batch) the partial is the
 * IDENTITY, not the shard's check point: a caller combining partials must OR the bad flags and
 * treat a set flag as a rejection (edc_combine_partials' bad_any), never test [8]*partial alone.
 */
int64_t edc_batch_submit_device(edc_ctx* ctx, size_t n, const uint8_t* d_vk, const uint8_t* d_sig,
                                const uint8_t* d_msg, const uint64_t* d_msg_off,
                                const uint8_t z_seed[32], uint64_t z_base, const uint8_t* d_z,
                                int want_check8);
int edc_batch_wait(edc_ctx* ctx, int64_t ticket, uint8_t check8[32], uint8_t partial[128], int* bad);

/*
 * Several consecutive batches in ONE launch sequence (a node verifying several blocks' votes at
 * once, or one GPU's shards of consecutive blocks; reference src/batch.rs:149-217 once per batch):
 * nb (1..16) batches of n_per items each (n_per a multiple of 2048), back to back in device
 * memory -- batch b is items [b n_per, (b+1) n_per) of d_vk / d_sig and of the message arena's
 * nb n_per + 1 offsets (or of d_k: nb n_per prehashed challenges, messages unused, d_msg /
 * d_msg_off may be NULL). Batch b's z are drawn at global indices z_base + b n_per + i, so batch
 * by batch its verdict, bad flag, check8 and partial equal edc_batch_verify_device /
 * edc_batch_partial_device of batch b alone at z_base + b n_per (see "Union first" below). Every per-item kernel runs once over all nb n_per items
 * and the MSM is range-tagged (one range per batch), so small batches fill the GPU like one
 * large batch. Waited with edc_batch_wait_multi (same ticket rules as edc_batch_submit_device):
 * verdicts[b] (EDC_OK / EDC_INVALID_SIGNATURE), optional check8 (nb x 32; a launch run batch by
 * batch from the start, edc_set_multi_union(ctx, 0), computes it only with want_check8),
 * partials (nb x 128) and bad flags (nb); returns EDC_INVALID_SIGNATURE if any batch failed.
 *
 * Union first (default; edc_set_multi_union): the launch runs as ONE batch over all nb n_per items
 * (same z). Its equation is the sum of the batches' equations, so when it holds every batch holds
 * -- with the probability batch verification itself gives, as Verifier::verify accepting a batch
 * accepts each of its items -- and every batch reports EDC_OK, bad 0 and the identity as check8.
 * When it fails (or partials are asked for at the wait), the wait reruns the launch batch by batch
 * as above before returning, so failing batches get exactly their own verdict, bad flag and
 * check8. edc_set_multi_union(ctx, 0) always runs batch by batch; edc_multi_union_stats counts the
 * union launches that passed and those rerun.
 */
int64_t edc_batch_submit_multi_device(edc_ctx* ctx, size_t nb, size_t n_per, const uint8_t* d_vk, const uint8_t* d_sig,
                                      const uint8_t* d_msg, const uint64_t* d_msg_off, const uint8_t* d_k,
                                      const uint8_t z_seed[32], uint64_t z_base, int want_check8);
int edc_batch_wait_multi(edc_ctx* ctx, int64_t ticket, size_t nb, int* verdicts, uint8_t* check8, uint8_t* partials,
                         int* bad);
int edc_set_multi_union(edc_ctx* ctx, int on);
int edc_multi_union_stats(const edc_ctx* ctx, uint64_t* passed, uint64_t* rerun);

/*
 * Host-buffer form of edc_batch_submit_device (replaces src/batch.rs:149 `Verifier::verify` for a
 * caller streaming consecutive batches from host memory): the inputs are copied into the slot's
 * own device buffers on the slot's stream, so the PCIe transfer of this batch overlaps the kernels
 * of the batches already in flight. Host buffers are borrowed until edc_batch_wait(ticket)
 * returns. Waited with edc_batch_wait; same ticket rules.
 */
int64_t edc_batch_submit(edc_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg,
                         const uint64_t* msg_off, const uint8_t z_seed[32], uint64_t z_base, int want_check8);

/*
 * edc_batch_submit for a node whose votes come from its registered validator set: item i's key
 * is key_idx[i], a position in the list last given to edc_keycache_load (4 bytes over PCIe per
 * item instead of 32). The device expands the indices to the raw 32-byte keys, so verdicts and
 * [8]*check equal edc_batch_submit with those keys. An index outside the list -> EDC_ERR_ARG.
 */
int64_t edc_batch_submit_indexed(edc_ctx* ctx, size_t n, const uint32_t* key_idx, const uint8_t* sig,
                                 const uint8_t* msg, const uint64_t* msg_off, const uint8_t z_seed[32],
                                 uint64_t z_base, int want_check8);

/*
 * Multi-GPU shard: evaluate this shard's part of the batch equation WITHOUT the cofactor /
 * identity step. partial (128 bytes) = canonical X||Y||Z||T of the shard's check point;
 * *bad = 1 if any item of the shard failed decoding / canonicity, and then the partial is the
 * IDENTITY (deterministic whatever the addition order; the off-curve sum is not): callers must
 * check *bad and pass the OR of the shards' flags to edc_combine_partials, whose verdict is then a
 * rejection. Items are the shard's slice of the global queue starting at global index z_base
 * (device pointers).
 */
int edc_batch_partial_device(edc_ctx* ctx, size_t n, const uint8_t* d_vk, const uint8_t* d_sig,
                             const uint8_t* d_msg, const uint64_t* d_msg_off,
                             const uint8_t z_seed[32], uint64_t z_base, const uint8_t* d_z,
                             uint8_t partial[128], int* bad);

/*
 * Combine g shard partials (g*128 bytes, any order) and the OR of their bad flags into the
 * batch verdict (src/batch.rs:212-216). check8 nullable.
 */
int edc_combine_partials(edc_ctx* ctx, size_t g, const uint8_t* partials, int bad_any,
                         uint8_t check8[32]);

/*
 * Device-side combine of g gathered exchange records (the multi-rank path's all-gather output,
 * already in this GPU's memory): record r at d_records + r*stride holds a shard's canonical
 * 128-byte partial point followed by its bad byte. The sum, x8 and the identity test (reference
 * src/batch.rs:212-216) run as one small kernel ENQUEUED on the caller's HIP stream `stream`
 * (the stream the all-gather ran on, so no host round trip and no synchronization; it must belong
 * to ctx's device, else EDC_ERR_ARG; the calling thread's current device is left unchanged); the 256-byte
 * result block lands in d_out (device, 16-byte aligned): int[0] = 0 Ok / 1 reject, int[1] = bad.
 */
int edc_combine_records_device(edc_ctx* ctx, void* stream, size_t g, const uint8_t* d_records, size_t stride,
                               uint8_t* d_out);

/*
 * VerificationKey::try_from(vk) + VerificationKey::verify(sig, msg) for each item
 *   reference src/verification_key.rs:160-175 (try_from -> MalformedPublicKey)
 *             src/verification_key.rs:225-258 (verify / verify_prehashed)
 * verdicts[i] in {EDC_OK, EDC_INVALID_SIGNATURE, EDC_MALFORMED_PUBLIC_KEY}. Returns 0 or <0.
 */
int edc_verify_each(edc_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig,
                    const uint8_t* msg, const uint64_t* msg_off, uint8_t* verdicts);

/* Device-resident edc_verify_each: verdicts into d_verdicts (n bytes of this GPU's memory). */
int edc_verify_each_device(edc_ctx* ctx, size_t n, const uint8_t* d_vk, const uint8_t* d_sig,
                           const uint8_t* d_msg, const uint64_t* d_msg_off, uint8_t* d_verdicts);

/*
 * Grouped fallback after a failed batch (the caller-driven Item::verify_single loop of
 * reference tests/batch.rs:37-43, src/batch.rs:104-107). The batch equation is linear, so it
 * restricts to any subset of the items: ONE range-tagged MSM pass evaluates it over about 128
 * contiguous ranges by default (edc_set_fallback_shape; same z, same k, the decoded points of the
 * batch prefix); ranges whose
 * [8]*check is not the identity, or that hold an item with an undecodable R / key or a
 * non-canonical s, are verified item by item. verdicts (host, n bytes) receive
 * Item::verify_single's code for every item. Returns the number of invalid items, or <0.
 * `leaf` is ignored (kept for ABI compatibility): range sizes are chosen by the library.
 *
 * Soundness: an item of a passing range is reported valid because its range's batch equation
 * holds, exactly as Verifier::verify accepts a batch (ZIP215: batch == single). Like the
 * reference's batch verification this is probabilistic: it relies on z being unpredictable to
 * whoever made the signatures. z_seed MUST be fresh and secret for every call (e.g. 32 bytes
 * of OS randomness); a known or reused seed lets crafted invalid signatures cancel inside a
 * range and be reported valid.
 */
int edc_find_invalid_device(edc_ctx* ctx, size_t n, const uint8_t* d_vk, const uint8_t* d_sig,
                            const uint8_t* d_msg, const uint64_t* d_msg_off, const uint8_t z_seed[32],
                            size_t leaf, uint8_t* verdicts);

/*
 * Verifier::verify(rng) and, if it fails, the per-item fallback in one call (the flow of
 * reference tests/batch.rs:18-44): the batch runs once; on failure the grouped fallback above
 * reuses that batch's k, points and grouping instead of recomputing them. Returns EDC_OK
 * (verdicts all 0) or EDC_INVALID_SIGNATURE with verdicts[i] = Item::verify_single's code and
 * *n_invalid (nullable) their count; <0 on runtime failure. check8 (nullable) as
 * edc_batch_verify. Same z_seed requirement as edc_find_invalid_device.
 */
int edc_batch_verify_fallback_device(edc_ctx* ctx, size_t n, const uint8_t* d_vk, const uint8_t* d_sig,
                                     const uint8_t* d_msg, const uint64_t* d_msg_off, const uint8_t z_seed[32],
                                     uint8_t* verdicts, int* n_invalid, uint8_t check8[32]);

/*
 * Prehashed batches: the reference's batch::Item is {vk_bytes, sig, k} (src/batch.rs:76-80) --
 * k = H(R||A||M) mod l is computed once, at Item::from (src/batch.rs:82-94), and
 * Verifier::queue / verify (src/batch.rs:127-137, :149-217) never see the message again. These
 * entries take that k (n*32 bytes, queue order, canonical little-endian scalars < l, as
 * Scalar::from_hash returns) instead of the message arena: SHA-512 is skipped and only
 * 32 + 64 + 32 bytes per item are read. Everything downstream is the message path's pipeline, so
 * verdicts and check8 are bit-identical to edc_batch_verify on the messages those k came from.
 * A k >= l is a broken caller contract: the call returns EDC_ERR_ARG (never a verdict).
 *  - edc_batch_verify_prehashed: host buffers, synchronous; z from z_seed (ChaCha20, as
 *    edc_batch_verify) or, when z_seed is NULL, caller-drawn z (n*16 bytes, LE u128 per item).
 *  - edc_batch_verify_prehashed_device: device buffers; z as edc_batch_verify_device.
 *  - edc_batch_submit_prehashed / _device: asynchronous forms (edc_batch_submit /
 *    edc_batch_submit_device rules; waited with edc_batch_wait). Inputs are borrowed until the wait.
 *  - edc_batch_verify_prehashed_fallback[_device]: the batch and, if it fails, the grouped fallback
 *    of edc_batch_verify_fallback_device (verdicts[i] = Item::verify_single's code, src/batch.rs:104-107).
 * Device k / z arrays must be 16-byte aligned (EDC_ERR_ARG otherwise).
 */
int edc_batch_verify_prehashed(edc_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* k,
                               const uint8_t z_seed[32], const uint8_t* z, uint8_t check8[32]);
int edc_batch_verify_prehashed_device(edc_ctx* ctx, size_t n, const uint8_t* d_vk, const uint8_t* d_sig,
                                      const uint8_t* d_k, const uint8_t z_seed[32], uint64_t z_base,
                                      const uint8_t* d_z, uint8_t check8[32]);
int64_t edc_batch_submit_prehashed(edc_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* k,
                                   const uint8_t z_seed[32], uint64_t z_base, int want_check8);
int64_t edc_batch_submit_prehashed_device(edc_ctx* ctx, size_t n, const uint8_t* d_vk, const uint8_t* d_sig,
                                          const uint8_t* d_k, const uint8_t z_seed[32], uint64_t z_base,
                                          const uint8_t* d_z, int want_check8);
/*
 * edc_batch_submit_prehashed with the keys given as positions in the list last given to
 * edc_keycache_load (as edc_batch_submit_indexed): 4 + 64 + 32 = 100 bytes per item over PCIe, for
 * a node whose votes come from its registered validator set. Verdicts and check8 equal
 * edc_batch_submit_prehashed with those keys. An index outside the list -> EDC_ERR_ARG.
 */
int64_t edc_batch_submit_prehashed_indexed(edc_ctx* ctx, size_t n, const uint32_t* key_idx, const uint8_t* sig,
                                           const uint8_t* k, const uint8_t z_seed[32], uint64_t z_base,
                                           int want_check8);
int edc_batch_verify_prehashed_fallback(edc_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig,
                                        const uint8_t* k, const uint8_t z_seed[32], uint8_t* verdicts,
                                        int* n_invalid, uint8_t check8[32]);
int edc_batch_verify_prehashed_fallback_device(edc_ctx* ctx, size_t n, const uint8_t* d_vk, const uint8_t* d_sig,
                                               const uint8_t* d_k, const uint8_t z_seed[32], uint8_t* verdicts,
                                               int* n_invalid, uint8_t check8[32]);

/*
 * batch::Item::verify_single (reference src/batch.rs:104-107): as edc_verify_each but with the
 * queue-time challenge k (n*32 bytes, canonical scalars) instead of the message. Any k >= l
 * (which Scalar::from_hash never returns) makes the call EDC_ERR_ARG, checked on the host before
 * anything is launched.
 */
int edc_verify_prehashed_each(edc_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig,
                              const uint8_t* k, uint8_t* verdicts);

/*
 * impl From<(VerificationKeyBytes, Signature, &M)> for batch::Item (reference src/batch.rs:82-94):
 * k_i = Scalar::from_hash(Sha512(R_i || A_i || M_i)) as 32 canonical LE bytes per item.
 */
int edc_challenge(edc_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig,
                  const uint8_t* msg, const uint64_t* msg_off, uint8_t* k_out);

/*
 * CompressedEdwardsY::decompress as used by VerificationKey::try_from
 * (reference src/verification_key.rs:166-168): ok[i] = 1 and xy[i] = canonical x || y, or
 * ok[i] = 0 when the encoding is not a curve point. Returns 0 or <0.
 */
int edc_decompress(edc_ctx* ctx, size_t n, const uint8_t* enc, uint8_t* xy, uint8_t* ok);

/*
 * VerificationKey::try_from(VerificationKeyBytes) for n keys at once -- key ingestion, e.g. a
 * validator set or serde-deserialized keys (reference src/verification_key.rs:160-175, :106-109;
 * tests/unit_tests.rs:32-40). codes[i] = EDC_OK or EDC_MALFORMED_PUBLIC_KEY. Returns 0 or <0.
 */
int edc_vk_validate(edc_ctx* ctx, size_t n, const uint8_t* vk, uint8_t* codes);

/*
 * Persistent validator-key cache: the reference's VerificationKey keeps its decoded point
 * (src/verification_key.rs:106-114, :160-175) while batch::Verifier re-decodes every distinct
 * key per verify (src/batch.rs:183-185). edc_keycache_load decodes the m keys (n*32 bytes,
 * duplicates allowed) ONCE and keeps a 64 KB fixed-base table per distinct key in this
 * context, replacing any previous cache. Every later batch / per-item call on the context
 * takes A and [2^128]A of a registered key from the cache, and the per-item fallback computes
 * [s]B - [k]A for it without doublings. Verdicts are identical with and without the cache
 * (an undecodable registered key stays MalformedPublicKey / fails the batch). ok (nullable,
 * m bytes) receives 1 where the key decodes. Returns the number of distinct keys cached
 * (<= 65536) or <0; refused while submitted batches are in flight.
 */
int64_t edc_keycache_load(edc_ctx* ctx, size_t m, const uint8_t* vk, uint8_t* ok);
int edc_keycache_clear(edc_ctx* ctx);
size_t edc_keycache_size(const edc_ctx* ctx);

/*
 * Per-object decoded key (reference src/verification_key.rs:106-114, :160-175: VerificationKey
 * decodes A once at try_from and keeps minus_A for every later verify): adds the keys of vk (m x 32
 * bytes) that are not cached yet to this context's cache WITHOUT replacing it. Cached keys keep
 * their places, so the list last given to edc_keycache_load stays valid for
 * edc_batch_submit_indexed (this call does not change that list). Every later batch or per-item
 * call finds a key added here exactly as one loaded by edc_keycache_load. ok (nullable, m bytes)
 * as edc_keycache_load. The table's hash is keyed by a per-context secret, so keys taken from
 * untrusted input cannot be chosen to collide. Keys that do not decode (try_from's
 * MalformedPublicKey) are NOT added (ok = 0 for them), so untrusted malformed keys cannot pin comb
 * tables. Returns the number of distinct keys now cached or <0; refused while submitted batches
 * are in flight.
 */
int64_t edc_keycache_add(edc_ctx* ctx, size_t m, const uint8_t* vk, uint8_t* ok);

/*
 * SigningKey::from([u8;32]) + SigningKey::sign (reference src/signing_key.rs:118-150,
 * :186-205) -- test/benchmark data source. seed_index (nullable) maps item i to seed
 * seed_index[i] (shared validator keys); vk_out n*32, sig_out n*64.
 */
int edc_sign(edc_ctx* ctx, size_t n, const uint8_t* seeds, size_t nseeds, const uint32_t* seed_index,
             const uint8_t* msg, const uint64_t* msg_off, uint8_t* vk_out, uint8_t* sig_out);
/* Device-pointer variant of edc_sign (all pointers in this GPU's memory). */
int edc_sign_device(edc_ctx* ctx, size_t n, const uint8_t* d_seeds, const uint32_t* d_seed_index,
                    const uint8_t* d_msg, const uint64_t* d_msg_off, uint8_t* d_vk_out,
                    uint8_t* d_sig_out);

/* ChaCha20 keystream blocks [blk0, blk0+nblocks) of key into d_out (64 bytes each), on device. */
int edc_chacha_fill_device(edc_ctx* ctx, const uint8_t key[32], uint64_t blk0, uint64_t nblocks,
                           uint8_t* d_out);

/*
 * Key grouping policy. The reference coalesces signatures by raw key bytes (HashMap,
 * src/batch.rs:114-137) so each distinct key is one MSM term; this only saves work when keys
 * repeat. mode 0 (default, auto): group, unless the last grouped batch on this context had more
 * distinct keys than half its signatures, in which case the next batches (regrouping every 8th)
 * keep one A_i term per signature with coefficient z_i k_i. mode 1: always group. mode 2: never.
 * mode 3 (tests): group, but with a zero probe budget, so every batch takes the on-device
 * overflow path that an adversarial key set would trigger (grouping abandoned mid-batch, one key
 * term per signature). Grouping hashes the raw key bytes under a per-context secret from OS
 * randomness and caps its probes, so chosen keys cannot make it quadratic.
 * Every mode gives the same group element, hence identical verdicts and [8]*check.
 */
int edc_set_key_grouping(edc_ctx* ctx, int mode);

/*
 * Split coefficients with the validator-key cache (edc_keycache_load). While the last batch found
 * every key in the cache, mode 0 (default, auto) writes each 253-bit B / key coefficient as
 * lo + 2^128 hi with hi on the cached [2^128]A (and [2^128]B), so every MSM term is 128 bits and
 * the final Horner chain is ~128 doublings instead of ~250 (lower per-batch latency). A key
 * missing from the cache still verifies exactly (it is doubled on the device) and turns the split
 * off until a batch finds all its keys again. mode 1: never split. Same group element in every
 * mode: identical verdicts and [8]*check. Replaces nothing in the reference (an MSM evaluation
 * order, src/batch.rs:205-210).
 */
int edc_set_key_split(edc_ctx* ctx, int mode);

/*
 * Pippenger shape for this context's batches (tuning / measurement): window width `bits` (8..16)
 * and number of parts a batch's terms are split into (1..64; parts are summed per window). 0 for
 * either picks it from the batch size (default). Results never depend on it.
 */
int edc_set_msm_shape(edc_ctx* ctx, int bits, int parts);

/*
 * Target MSM entries per bin (tuning / measurement; >= 256, 0 = from the batch size, default):
 * with automatic parts, the slices of the densest windows are split into sub-bins of about this
 * many digits each, one workgroup per bin. Results never depend on it.
 */
int edc_set_msm_bin_entries(edc_ctx* ctx, int entries);

/*
 * Test knob (process-wide): at most `max_entries` (0..16384, default 16384) MSM entries per
 * workgroup go through the binning scatter's LDS stage; workgroups with more store each entry
 * directly. 0 forces the direct stores everywhere. Results never depend on it.
 */
int edc_debug_set_scatter_stage(uint32_t max_entries);

/*
 * Test hook: the device's wide scalar reduction (Scalar::from_hash after SHA-512, reference
 * src/batch.rs:86-91) on n caller-chosen 64-byte little-endian integers d_in (device, 16-byte
 * aligned) -> n canonical 32-byte residues mod l in d_out (device, 16-byte aligned), synchronous.
 * Lets tests drive the reduction's fold boundaries, which SHA-512 outputs practically never hit.
 */
int edc_debug_sc_reduce_wide(edc_ctx* ctx, size_t n, const uint8_t* d_in, uint8_t* d_out);

/*
 * Shape of the grouped fallback's range MSM (tuning / measurement): about `ranges` contiguous
 * ranges (1..1024, default 32) with `bits`-bit windows (8..13, default 10). The range count is
 * capped so that ranges x bins per range stays within the MSM's 8192 bins (e.g. at most 24 ranges
 * with 13-bit windows). Results never depend on it.
 */
int edc_set_fallback_shape(edc_ctx* ctx, int ranges, int bits);

/*
 * Number of in-flight slots (1..16, default 16) this context's submissions rotate over; each slot
 * holds its own workspace and hardware queue. Contexts that share one GPU (edc_create_multi with
 * a repeated device) get 16 / (contexts on that GPU). Refused while batches are in flight.
 */
int edc_set_slots(edc_ctx* ctx, int k);

/*
 * Pre-allocate the workspaces of every in-flight slot for batches of up to n items (otherwise
 * they grow on first use). Not a reference API: a setup call for streaming callers.
 */
int edc_reserve(edc_ctx* ctx, size_t n);

/*
 * Per-phase device timings of the last batch call (HIP events on the context stream), enabled
 * by edc_set_timing(ctx, 1). Returns the number of phases written (<= cap); names via
 * edc_timing_name(i).
 */
void edc_set_timing(edc_ctx* ctx, int enable);
int edc_last_timings(const edc_ctx* ctx, float* ms, int cap);
const char* edc_timing_name(int i);
/* The last timed batch's accumulation kernel alone (k_msm_accum_dma, between HIP events on its
 * stream): duration in ms and the number of digit entries it added (one signed mixed addition
 * each), for the accumulation's own roofline in bench.py. EDC_ERR_ARG before any timed batch. */
int edc_last_msm_accum(const edc_ctx* ctx, float* ms, uint64_t* entries);

/* Synchronize the context stream (for callers that time around device calls). */
int edc_synchronize(edc_ctx* ctx);

/*
 * Several GPUs in one process (a node verifying each block's votes across all of its MI355X):
 * one batch::Verifier::verify (reference src/batch.rs:149-217) split into contiguous shards, one
 * per listed device (a device may be listed more than once: several contexts on one GPU). Shard g
 * draws its z at its global queue indices, evaluates its part of the batch equation to one
 * partial point (128 bytes); the partials are gathered through the host and combined on the
 * first device (x8, identity). Verdicts and check8 are bit-identical to edc_batch_verify on one
 * device for any device list. Host buffers as edc_batch_verify; synchronous (the pipelined,
 * device-to-device form is edc_multi_submit / edc_multi_wait below).
 */
typedef struct edc_multi edc_multi;
edc_multi* edc_create_multi(const int* devices, int ndev);
void edc_destroy_multi(edc_multi* m);
int edc_multi_size(const edc_multi* m);
/* per-device context i (e.g. to load the validator-key cache on every device) */
edc_ctx* edc_multi_context(edc_multi* m, int i);
const char* edc_multi_last_error(const edc_multi* m);
int edc_multi_batch_verify(edc_multi* m, size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg,
                           const uint64_t* msg_off, const uint8_t z_seed[32], uint8_t check8[32]);
/*
 * Pipelined form of edc_multi_batch_verify for a node verifying block after block across its
 * GPUs (reference src/batch.rs:149-217, one Verifier::verify per block): edc_multi_submit splits
 * the batch into contiguous shards, enqueues each on its device's next in-flight slot (host
 * inputs copied on that slot's stream, as edc_batch_submit) and returns a ticket >= 0 without
 * waiting. Each shard's 128-byte partial point (with its bad flag) reaches the first device, where
 * a combine on its own stream sums the partials (x8, identity) as soon as the last shard lands:
 * by a peer store over xGMI when peer access from the shard's device to the first device could be
 * enabled at edc_create_multi, otherwise through the shard slot's pinned host mirror (a 256-byte
 * host-to-device copy on the combine stream); edc_create_multi fails (NULL) if enabling a
 * possible peer access fails. edc_multi_wait blocks for the ticket and returns EDC_OK /
 * EDC_INVALID_SIGNATURE / <0 with optional check8 (needs want_check8). Up to R batches in flight,
 * R = 16 / (contexts sharing the busiest listed GPU), e.g. 16 for distinct devices, 8 for [0, 0];
 * tickets are waited in submission order; host buffers are borrowed until the
 * wait. edc_multi_submit_device takes per-device slices already resident in each device's HBM:
 * n[g] items at d_vk[g], d_sig[g], d_msg[g], d_msg_off[g] form shard g, with global queue indices
 * (for z) starting at n[0] + ... + n[g-1]. Verdicts and check8 equal edc_batch_verify of the
 * concatenated batch on one device.
 */
int64_t edc_multi_submit(edc_multi* m, size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg,
                         const uint64_t* msg_off, const uint8_t z_seed[32], int want_check8);
int64_t edc_multi_submit_device(edc_multi* m, const size_t* n, const uint8_t* const* d_vk,
                                const uint8_t* const* d_sig, const uint8_t* const* d_msg,
                                const uint64_t* const* d_msg_off, const uint8_t z_seed[32], int want_check8);
int edc_multi_wait(edc_multi* m, int64_t ticket, uint8_t check8[32]);
/*
 * How shard i's result block reaches the first device: 0 = same GPU (local copy), 1 = peer store
 * over xGMI (peer access enabled), 2 = staged through pinned host memory. <0 for a bad index.
 * Test knob: edc_multi_debug_force_staged(m, 1) routes every shard through host memory (the
 * fallback a device pair without peer access takes); 0 restores the routes edc_create_multi found.
 * Refused while batches are in flight. Status: distinct-device lists have not run on hardware in
 * this repository's tests (the pool's boxes hold one GPU); the staged and local routes have.
 */
int edc_multi_route(const edc_multi* m, int i);
int edc_multi_debug_force_staged(edc_multi* m, int on);
/*
 * edc_multi_batch_verify and, on failure, the grouped fallback on every shard whose own partial
 * fails (edc_batch_verify_fallback_device semantics): verdicts (host, n bytes) = Item::verify_single
 * codes, *n_invalid their count. Returns EDC_OK / EDC_INVALID_SIGNATURE / <0.
 */
int edc_multi_batch_verify_fallback(edc_multi* m, size_t n, const uint8_t* vk, const uint8_t* sig,
                                    const uint8_t* msg, const uint64_t* msg_off, const uint8_t z_seed[32],
                                    uint8_t* verdicts, int* n_invalid, uint8_t check8[32]);

#ifdef __cplusplus
}
#endif

#endif /* EDC_H */
