// Host-side launchers for every kernel (one translation unit per kernel family).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "keycache.h"
#include "edc_common.h"

namespace edc {
// edc_prep.hip
void launch_challenge(hipStream_t st, uint32_t n, const uint8_t* vk, const uint8_t* sig,
                      const uint8_t* msg, const uint64_t* off, uint32_t* k);
void launch_decompress(hipStream_t st, uint32_t n, const uint8_t* sig, const uint8_t* vk, const uint32_t* key_rep,
                       bool per_sig, uint32_t* pts, uint8_t* itembad, uint8_t* keybad, int* flags,
                       const KeyCacheView& kc, bool split = false, uint32_t klanes = 0);
// R of items [r0, r0 + rcnt) of an n-item batch, and the distinct keys on klanes lanes (0: none;
// launch_decompress: 0 = n, one lane per possible key)
void launch_decompress_range(hipStream_t st, uint32_t n, uint32_t r0, uint32_t rcnt, uint32_t klanes, const uint8_t* sig,
                             const uint8_t* vk, const uint32_t* key_rep, bool per_sig, uint32_t* pts, uint8_t* itembad,
                             uint8_t* keybad, int* flags, const KeyCacheView& kc, bool split = false);
void launch_keys(hipStream_t st, uint32_t n, const uint8_t* vk, uint32_t* table, uint32_t tmask,
                 const uint32_t salt[2], bool force_overflow, uint32_t* slot_key, uint32_t* key_slot_of_sig,
                 uint32_t* key_rep, uint32_t* key_index, unsigned long long* key_acc, int* flags,
                 uint32_t kcap = 0xFFFFFFFFu);
// per-signature key terms (no grouping): m = n, key j is signature j's own key (key_rep = null)
void launch_coef(hipStream_t st, uint32_t n, const uint8_t* sig, const uint32_t* k, const uint8_t* zexp,
                 const uint32_t seed[8], uint64_t zbase, const uint32_t* key_index, uint32_t* scal,
                 unsigned long long* key_acc, unsigned long long* u_acc, uint8_t* itembad, int* flags,
                 bool per_sig, uint32_t* coef_part, bool split = false);
// launch_coef in pieces (chunked host-buffer calls): the per-item pass over items
// [item0, item0 + cnt) (item0 a multiple of COEF_CHUNK) as each chunk lands, then once the
// per-key merge and the coefficient reduction
void launch_coef_range(hipStream_t st, uint32_t n, uint32_t item0, uint32_t cnt, const uint8_t* sig, const uint32_t* k,
                       const uint8_t* zexp, const uint32_t seed[8], uint64_t zbase, const uint32_t* key_index,
                       uint32_t* scal, unsigned long long* key_acc, unsigned long long* u_acc, uint8_t* itembad,
                       int* flags, bool per_sig, uint32_t* coef_part, bool split = false);
void launch_coef_finish(hipStream_t st, uint32_t n, unsigned long long* key_acc, unsigned long long* u_acc,
                        uint32_t* scal, int* flags, bool per_sig, uint32_t* coef_part, bool split = false);
// words of k_coef's per-workgroup key-slot dump for batches of up to cap_n signatures
size_t coef_part_words(size_t cap_n);
// grouped fallback: per-(range, key) / per-range coefficients as listed MSM terms
void launch_range_coef(hipStream_t st, uint32_t n, uint32_t rsize, uint32_t nranges, uint32_t m, bool per_sig,
                       const uint8_t* sig, const uint32_t* k, const uint8_t* zexp, const uint32_t seed[8],
                       uint64_t zbase, const uint32_t* key_index, uint32_t* scal, unsigned long long* key_acc,
                       unsigned long long* u_acc, int* flags, uint32_t* xpt, uint32_t* xrg, uint32_t* xscal);
// several batches in one launch (nr equal ranges of n / nr items, n / nr a multiple of COEF_CHUNK):
// per-item z and s checks, per-(range, key) sums at g * kstride + key (grouped keys; more than
// kstride distinct keys must have set FLAG_OVF: launch_keys' kcap), listed key / B terms
void launch_multi_coef(hipStream_t st, uint32_t n, uint32_t nr, uint32_t kstride, bool per_sig, const uint8_t* sig,
                       const uint32_t* k, const uint32_t seed[8], uint64_t zbase, const uint32_t* key_index,
                       uint32_t* scal, unsigned long long* key_acc, unsigned long long* u_acc, uint8_t* itembad,
                       int* flags, uint32_t* xpt, uint32_t* xrg, uint32_t* xscal);
void launch_range_prebad(hipStream_t st, uint32_t n, uint32_t rsize, const uint8_t* itembad, const uint8_t* itembad_r,
                         const uint8_t* keybad,
                         const uint32_t* key_index, bool per_sig, uint8_t* rbad, const int* flags = nullptr);
void launch_init_basepoint(hipStream_t st, uint32_t* pts);
void launch_sc_reduce_wide(hipStream_t st, uint32_t n, const uint32_t* in, uint32_t* out);
void launch_gather_items(hipStream_t st, uint32_t c, const uint32_t* idx, const uint8_t* vk, const uint8_t* sig,
                         const uint32_t* k, uint8_t* out_vk, uint8_t* out_sig, uint32_t* out_k);
// vk_out[i] = keys[reg[key_idx[i]]] (32 bytes each; key-indexed host submissions)
void launch_expand_keys(hipStream_t st, uint32_t n, const uint32_t* key_idx, const uint32_t* reg,
                        const uint32_t* keys, uint8_t* vk_out);
// per-batch resets in one launch: flags (FLAG_NKEYS = nkeys if >= 0), u_acc, the 256-byte result
// block, table[0..T) = 0xFFFFFFFF, counts[0..nbin) = 0 (T / nbin may be 0)
void launch_init_batch(hipStream_t st, int* flags, int nkeys, unsigned long long* u_acc, uint8_t* d_out, uint32_t* table,
                       uint32_t T, uint32_t* counts, uint32_t nbin);
// edc_msm.hip: per-device kernel attributes (the scatter's dynamic LDS beyond 64 KB); call on
// every device a context uses, after hipSetDevice
hipError_t msm_init_device();
// edc_msm.hip (counts_zeroed: the caller already cleared counts, e.g. launch_init_batch)
void launch_msm_bin(hipStream_t st, const MsmPlan& P, const MsmTerms& T, uint32_t max_terms, uint32_t* counts,
                    uint32_t* offsets, uint32_t* cursor, uint2* entries, const int* flags, bool counts_zeroed = false);
// per-bin counting sort of the binned entries by bucket (needs only the binning: enqueued right
// after launch_msm_bin, so on a dual-stream slot it overlaps the decode)
void launch_msm_sort(hipStream_t st, const MsmPlan& P, const uint32_t* counts, const uint32_t* offsets,
                     const uint2* entries, uint32_t* sorted, uint32_t* bucket_end, uint32_t* buckets);
// accumulation (+ bin reduction) of the sorted entries; launch_msm_sort must have run
void launch_msm_bucket(hipStream_t st, const MsmPlan& P, const uint32_t* counts, const uint32_t* offsets,
                       const uint2* entries, uint32_t* sorted, uint32_t* bucket_end, const uint32_t* pts,
                       uint32_t* buckets, uint32_t* heads, uint32_t* slice_W, uint32_t* slice_T, int probe_skip = 0,
                       hipEvent_t acc_begin = nullptr, hipEvent_t acc_end = nullptr, bool latency = false,
                       int* stamp_flags = nullptr);   // EDC_BATCH_STAMPS builds: the batch's flags
size_t msm_bucket_words(uint32_t nbin);
void launch_msm_tail(hipStream_t st, const MsmPlan& P, const uint32_t* slice_W, const uint32_t* slice_T,
                     uint32_t* win, int* flags, int want_compress, uint8_t* out, uint8_t* hout = nullptr);
void launch_msm_range_tail(hipStream_t st, const MsmPlan& P, const uint32_t* slice_W, const uint32_t* slice_T,
                           uint32_t* win, uint8_t* rverdict);
// several batches in one launch: per range the window combine, Horner, x8 and identity, one
// 256-byte result block per range at out + 256 g (and hout + 256 g)
void launch_msm_multi_tail(hipStream_t st, const MsmPlan& P, const uint32_t* slice_W, const uint32_t* slice_T,
                           uint32_t* win, const int* flags, const uint8_t* rbad, int want_compress, uint8_t* out,
                           uint8_t* hout);
void launch_combine_records(hipStream_t st, uint32_t g, const uint8_t* recs, uint32_t stride, uint8_t* out);
void launch_combine(hipStream_t st, uint32_t g, const uint8_t* partials, int bad, int want_compress,
                    uint8_t* out);
// 256-byte result block src -> dst (dst may be a peer device's memory)
void launch_copy_block(hipStream_t st, const uint8_t* src, uint8_t* dst);
// g shard result blocks (256 bytes each, device) -> verdict block (as launch_combine)
void launch_combine_blocks(hipStream_t st, uint32_t g, const uint8_t* blocks, int want_compress, uint8_t* out);
size_t msm_entry_capacity(const MsmPlan& P, size_t short_terms, size_t full_terms);
// edc_single.hip
void launch_init_btable(hipStream_t st, uint32_t* btab);
void launch_verify_single(hipStream_t st, uint32_t n, const uint8_t* vk, const uint8_t* sig,
                          const uint32_t* k, const uint32_t* btab, uint32_t* vtab, uint8_t* verdict,
                          const KeyCacheView& kc, const uint32_t* bcomb);
// latency form for short item lists (one quad of lanes per item)
void launch_verify_quad(hipStream_t st, uint32_t n, const uint8_t* vk, const uint8_t* sig, const uint32_t* k,
                        const uint32_t* btab, uint8_t* verdict, const KeyCacheView& kc, const uint32_t* bcomb);
// key cache (edc_single.hip): decode m registered keys -> ext + ok, comb tables of m points
void launch_kc_decode(hipStream_t st, uint32_t m, const uint32_t* keys, uint32_t* ext, uint8_t* ok);
void launch_kc_basepoint(hipStream_t st, uint32_t* ext);
void launch_kc_comb(hipStream_t st, uint32_t m, const uint32_t* ext, uint32_t* comb);
// VerificationKey::try_from for n encodings: code[i] = 0 (Ok) or 2 (MalformedPublicKey)
void launch_vk_validate(hipStream_t st, uint32_t n, const uint8_t* enc, uint8_t* code);
size_t verify_single_scratch_words(size_t n);
void launch_sign(hipStream_t st, uint32_t n, const uint8_t* seeds, const uint32_t* seed_index,
                 const uint8_t* msg, const uint64_t* off, const uint32_t* btab, uint8_t* vk_out,
                 uint8_t* sig_out);
void launch_decode(hipStream_t st, uint32_t n, const uint8_t* enc, uint8_t* xy, uint8_t* ok);
void launch_chacha_fill(hipStream_t st, const uint32_t key[8], uint64_t blk0, uint64_t nblocks,
                        uint32_t* out);
}  // namespace edc
