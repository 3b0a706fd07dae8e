// C ABI (include/edc.h): context, workspace and the orchestration of the batch pipeline.
// Every entry point cites the reference API it replaces in include/edc.h.
#include <stdlib.h>
#include <string.h>
#include <string>
#include <random>
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>
#include <hip/hip_ext.h>
#include "edc.h"
#include "edc_common.h"
#include "edc_launch.h"

using namespace edc;

namespace {

// phases in enqueue order (each bracketed by HIP events on the slot stream)
enum Phase { PH_KEYS, PH_CHALLENGE, PH_COEF, PH_MSM_BIN, PH_DECOMP, PH_MSM_BUCKET, PH_MSM_TAIL, PH_N };
const char* kPhaseNames[PH_N] = {"keys_group", "challenge_sha512", "coef_chacha_scalar", "msm_bin",
                                 "decompress_R", "msm_bucket", "msm_window_final"};

template <typename T>
hipError_t dalloc(T** p, size_t count) {
  *p = nullptr;
  if (count == 0) count = 1;
  return hipMalloc((void**)p, count * sizeof(T));
}

#ifndef EDC_SLOTS
#define EDC_SLOTS 16
#endif
constexpr int kSlots = EDC_SLOTS;  // batches that can be in flight per context
// Timing probes only (make variant VFLAGS=-DEDC_PROBE_SKIP=<mask>, tools/phase_cost.sh): after a
// slot's first batch, skip a phase's launches (its outputs stay from that batch, which the bench
// repeats), to measure what the phase costs inside the pipeline: 2 SHA-512, 4 coefficients,
// 8 binning, 16 decompression, 32 accumulation, 64 bin reduction, 128 window combine + Horner,
// 256 bucket sort. The product build has mask 0.
#ifndef EDC_PROBE_SKIP
#define EDC_PROBE_SKIP 0
#endif
#define EDC_RUN(bit) ((EDC_PROBE_SKIP & (bit)) == 0 || s.probe_runs == 0)
#ifndef EDC_DUAL_STREAM
#define EDC_DUAL_STREAM 2   // slot 0 (synchronous calls) decodes on a second stream; see init_slot
#endif
#ifndef EDC_QUAD_VERIFY_MAX
#define EDC_QUAD_VERIFY_MAX (1u << 14)   // one lane per item beats a quad from ~32k items (r04ad)
#endif
constexpr size_t kQuadVerifyMax = EDC_QUAD_VERIFY_MAX;   // per-item lists up to this size use the quad kernel
constexpr uint32_t kMultiMax = 16;            // batches per edc_batch_submit_multi_device launch
constexpr uint32_t kMultiKeys = 4096;         // distinct keys with per-(batch, key) sums; more -> per signature

}  // namespace

// One in-flight batch: its own HIP stream and every per-batch device buffer.
struct Slot {
  hipStream_t st = nullptr;
  size_t cap_n = 0, cap_T = 0;
  uint32_t *k = nullptr, *key_slot = nullptr, *key_index = nullptr, *key_rep = nullptr;
  // the batch's challenges: k (computed by k_challenge) or a prehashed caller's device array
  const uint32_t* kin = nullptr;
  uint32_t *table = nullptr, *slot_key = nullptr;
  uint32_t *pts = nullptr, *scal = nullptr;
  unsigned long long *key_acc = nullptr, *u_acc = nullptr;
  uint32_t* coef_part = nullptr;     // k_coef's per-workgroup key slots (merged by k_coef_merge)
  uint8_t *itembad = nullptr, *keybad = nullptr;   // per-item / per-key failure bits (fallback)
  // MSM workspace, grown on demand to the plan's bins / entries
  uint32_t cap_bins = 0, cap_ranges = 0;
  size_t cap_entries = 0;
  uint32_t *counts = nullptr, *offsets = nullptr, *cursor = nullptr;
  uint2* entries = nullptr;
  uint32_t* sorted = nullptr;   // entries' point indices sorted by bucket within each bin
  uint32_t *slice_W = nullptr, *slice_T = nullptr, *win = nullptr;
  uint32_t* buckets = nullptr;  // bins x 256 bucket sums (extended)
  uint32_t* heads = nullptr;    // bins x 256 head partials of the segmented accumulation
  uint32_t* bucket_end = nullptr;   // bins x 256 bucket end positions of the sorted entries
  int* flags = nullptr;
  uint8_t* d_out = nullptr;     // 256-byte result block (kMultiMax of them for a multi-batch launch)
  uint8_t* h_out = nullptr;     // pinned mirror
  uint32_t* h_acc = nullptr;    // pinned: the last bin's offset and count (timed batches' entry count)
  // several batches in one launch (edc_batch_submit_multi_device): per-(batch, key) sums, listed
  // key / B terms, per-batch bad flags; nmulti = batches of the pending launch (0: one batch)
  unsigned long long* mb_acc = nullptr;
  uint32_t *mb_xpt = nullptr, *mb_xrg = nullptr, *mb_xscal = nullptr;
  uint8_t* mb_bad = nullptr;
  size_t mb_cap_acc = 0, mb_cap_terms = 0;
  uint32_t nmulti = 0;
  uint32_t acc_nbin = 0;        // bins of the last enqueued single-batch MSM (timing report)
  // union-first multi launch (edc_set_multi_union): the launch ran as ONE batch over all nb * n_per
  // items; its arguments are kept (device inputs are borrowed until the wait) to rerun it batch by
  // batch when that union fails
  bool mu_union = false;
  size_t mu_nper = 0;
  const uint8_t *mu_vk = nullptr, *mu_sig = nullptr, *mu_msg = nullptr;
  const uint64_t* mu_off = nullptr;
  const uint32_t* mu_k = nullptr;
  uint8_t mu_seed[32] = {};
  uint64_t mu_zbase = 0;
  int mu_compress = 0;
  hipEvent_t ev[PH_N + 1] = {};
  hipEvent_t ev_acc[2] = {};    // timed batches: around k_msm_accum_dma (edc_last_msm_accum)
  // EDC_DUAL_STREAM builds: the decode runs on a second stream beside SHA-512 / coefficients /
  // binning (joined before the accumulation)
  hipStream_t st2 = nullptr;
  hipEvent_t ev_keys = nullptr, ev_dec = nullptr;
  // host-buffer submissions (edc_batch_submit): this slot's own device copy of the inputs
  uint8_t *in_vk = nullptr, *in_sig = nullptr, *in_msg = nullptr;
  uint64_t* in_off = nullptr;
  uint32_t* in_idx = nullptr;         // key indices (edc_batch_submit_indexed)
  size_t in_cap_n = 0, in_cap_msg = 0;
  std::vector<uint64_t> in_rebased;   // offsets rebased to 0 (host side, alive until the slot is reused)
  bool pending = false;         // submitted, not yet waited
  bool timed = false;
  bool per_sig = false;         // this batch skipped key grouping (adaptive grouping)
  uint32_t n_batch = 0;
  int64_t ticket = -1;
  uint32_t probe_runs = 0;      // batches enqueued (EDC_PROBE_SKIP timing builds only)
  uint64_t t_submit_us = 0;     // host time of the submission (EDC_BATCH_STAMPS builds only)
};

struct edc_ctx {
  int device = 0;
  std::string err;
  uint32_t* btab = nullptr;     // [1..8]B, affine Niels
  Slot slot[kSlots];
  // staging for the host-pointer entry points (used on slot 0's stream)
  size_t cap_n = 0, cap_msg = 0, cap_aux = 0;
  uint8_t *vk = nullptr, *sig = nullptr, *msg = nullptr, *zexp = nullptr;
  uint64_t* off = nullptr;
  uint32_t* kbuf = nullptr;
  uint8_t* verdicts = nullptr;
  uint32_t* vtab = nullptr;     // per-item multiples tables of the per-signature kernel
  uint8_t* aux = nullptr;       // decode xy / sign outputs / partials
  // shard-partial combination on its own stream, so it never waits behind in-flight batches
  Slot comb;
  uint8_t* comb_in = nullptr;   // g x 128-byte partial records
  size_t comb_cap = 0;
  bool timing = false;
  float last_ms[PH_N] = {};
  float last_acc_ms = 0.f;      // k_msm_accum_dma of the last timed batch
  uint32_t last_acc_entries = 0;
  int nlast = 0;
  int64_t next_ticket = 0;
  int nslots = kSlots;          // in-flight slots the submissions rotate over (edc_set_slots)
  // adaptive key grouping (edc_set_key_grouping): mode 0 = auto, 1 = always group, 2 = never
  int key_grouping = 0;
  bool have_key_ratio = false;  // a grouped batch has completed on this context
  double last_key_ratio = 0.0;  // distinct keys / signatures of the last grouped batch
  int ungrouped_run = 0;        // consecutive ungrouped batches since the last grouped one
  int win_bits = 0;             // MSM window width override (edc_set_msm_shape), 0 = by batch size
  uint32_t bin_entries = 0;     // target entries per MSM bin (edc_set_msm_bin_entries), 0 = by batch size
  uint32_t msm_parts = 0;       // MSM parts override (edc_set_msm_shape), 0 = by batch size
  uint64_t secret = 0;          // key-grouping hash secret (OS randomness, per context)
  uint64_t nbatches = 0;
  // grouped fallback (range MSM) staging, slot 0 only
  size_t fb_cap_terms = 0, fb_cap_ranges = 0;
  uint32_t *fb_xpt = nullptr, *fb_xrg = nullptr, *fb_xscal = nullptr;
  uint8_t* fb_rv = nullptr;      // per-range verdict | pre-bad flag
  uint32_t* fb_idx = nullptr;    // items verified one by one
  size_t fb_cap_idx = 0;
  uint8_t* fb_g = nullptr;       // their gathered vk | sig | k (fb_cap_g items each)
  size_t fb_cap_g = 0;
  uint32_t fb_ranges = 128;     // target range count of the grouped fallback (sweep: profiles/r04/r04ad_fb_sweep.log)
  int fb_bits = 9;              // its window width
  // persistent validator-key cache (keycache.h), replaced by each edc_keycache_load, grown by
  // edc_keycache_add (device arrays hold kc_cap keys; the host keeps the key words and ok bytes
  // to rebuild the hash table and answer duplicates)
  uint32_t *kc_table = nullptr, *kc_keys = nullptr, *kc_comb = nullptr;
  uint8_t* kc_ok = nullptr;
  uint32_t* bcomb = nullptr;    // comb table of B, built with the first cache
  uint32_t kc_m = 0, kc_tmask = 0, kc_cap = 0;
  uint32_t kc_s0 = 0, kc_s1 = 0;        // table hash key, from `secret`
  std::vector<uint32_t> kc_words;       // kc_m x 8 raw key words
  std::vector<uint8_t> kc_okh;          // kc_m decode flags
  uint32_t* kc_reg = nullptr;   // registered position -> cache index (edc_batch_submit_indexed)
  uint32_t kc_reg_m = 0;
  // split coefficients (edc_common.h) while the key cache covers the batches' keys:
  // key_split 0 = auto, 1 = never; last_uncached = keys the last batch did not find in the cache
  int key_split = 0;
  uint32_t last_uncached = 0;
  int multi_union = 1;                  // edc_set_multi_union
  uint64_t mu_hits = 0, mu_reruns = 0;  // union-first launches that passed / were rerun per batch
  // chunked synchronous host-buffer calls (run_host_chunked): a copy stream and one event per
  // chunk (+ the keys / offsets piece), created on first use
  hipStream_t hcs = nullptr, hcs2 = nullptr;
  hipEvent_t hev[9] = {}, hev2[9] = {};   // piece 0 + signature chunks / k or message chunks
  hipStream_t st() const { return slot[0].st; }
  KeyCacheView kc() const {
    if (!kc_m) return KeyCacheView{nullptr, nullptr, nullptr, nullptr, 0, 0, nullptr, 0, 0};
    return KeyCacheView{kc_table, kc_keys, kc_ok, kc_comb, kc_tmask, kc_m, bcomb, kc_s0, kc_s1};
  }
};

// A failed HIP call also leaves the thread's last-error state set; it is cleared here, so that a
// later hipGetLastError() after a kernel launch reports only that launch.
#define CK(expr)                                                        \
  do {                                                                  \
    hipError_t e_ = (expr);                                             \
    if (e_ != hipSuccess) {                                             \
      (void)hipGetLastError();                                          \
      ctx->err = std::string(#expr) + ": " + hipGetErrorString(e_);     \
      return EDC_ERR_HIP;                                               \
    }                                                                   \
  } while (0)

static void free_msm_buffers(Slot& s) {
  void* ptrs[] = {s.counts, s.offsets, s.cursor, s.slice_W, s.slice_T, s.win, s.buckets, s.heads, s.entries, s.sorted,
                  s.bucket_end};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  s.counts = s.offsets = s.cursor = s.slice_W = s.slice_T = s.win = s.buckets = s.heads = s.sorted = nullptr;
  s.bucket_end = nullptr;
  s.entries = nullptr;
  s.cap_bins = s.cap_ranges = 0;
  s.cap_entries = 0;
}

static void free_slot_buffers(Slot& s) {
  void* ptrs[] = {s.k, s.key_slot, s.key_index, s.key_rep, s.table, s.slot_key, s.pts, s.scal, s.key_acc,
                  s.u_acc, s.itembad, s.keybad, s.coef_part};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  s.k = s.key_slot = s.key_index = s.key_rep = s.table = s.slot_key = s.pts = s.scal = nullptr;
  s.key_acc = s.u_acc = nullptr;
  s.coef_part = nullptr;
  s.itembad = s.keybad = nullptr;
  free_msm_buffers(s);
  s.cap_n = s.cap_T = 0;
}

static size_t next_pow2(size_t x) {
  size_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

// Every in-flight slot needs its own hardware queue: kernels of streams that share a queue run
// in order, so one batch's latency-bound tail would stall the bulk kernels of another. Streams
// created with an (all-CU) mask get a dedicated queue instead of one of the runtime's shared pool
// (GPU_MAX_HW_QUEUES, 4 by default, one of which the process's default stream already holds).
static hipError_t create_slot_stream(int device, hipStream_t* st) {
  int cus = 0;
  hipError_t e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
  if (e != hipSuccess || cus <= 0) return hipStreamCreateWithFlags(st, hipStreamNonBlocking);
  std::vector<uint32_t> mask((cus + 31) / 32, 0xFFFFFFFFu);
  if (cus % 32) mask.back() = (1u << (cus % 32)) - 1u;
  return hipExtStreamCreateWithCUMask(st, (uint32_t)mask.size(), mask.data());
}

static int init_slot(edc_ctx* ctx, Slot& s) {
  if (s.st) return 0;
  CK(create_slot_stream(ctx->device, &s.st));
  CK(dalloc(&s.flags, FLAG_ALLOC));
  CK(dalloc(&s.d_out, 256 * kMultiMax));
  CK(hipHostMalloc((void**)&s.h_out, 256 * kMultiMax));
  CK(hipHostMalloc((void**)&s.h_acc, 2 * sizeof(uint32_t)));
  for (int p = 0; p <= PH_N; ++p) CK(hipEventCreate(&s.ev[p]));
  for (int p = 0; p < 2; ++p) CK(hipEventCreate(&s.ev_acc[p]));
#if EDC_DUAL_STREAM
  // 1: every slot; 2: slot 0 only (the synchronous calls' slot), so the pipelined slots keep one
  // hardware queue each (past ~16 user queues per GPU the scheduler time-slices them).
  // EDC_SINGLE_STREAM=1 in the environment (measurement only: kernel traces of one batch at a time
  // that must not overlap the decode with SHA-512) keeps every slot on one stream.
  static const bool single_stream = getenv("EDC_SINGLE_STREAM") && getenv("EDC_SINGLE_STREAM")[0] == '1';
  if (!single_stream && (EDC_DUAL_STREAM == 1 || &s == &ctx->slot[0])) {
    CK(create_slot_stream(ctx->device, &s.st2));
    CK(hipEventCreateWithFlags(&s.ev_keys, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&s.ev_dec, hipEventDisableTiming));
  }
#endif
  return 0;
}

static int ensure_slot(edc_ctx* ctx, Slot& s, size_t n) {
  int rc = init_slot(ctx, s);
  if (rc) return rc;
  if (n <= s.cap_n && s.pts) return 0;
  CK(hipStreamSynchronize(s.st));
  free_slot_buffers(s);
  const size_t cap = n < 1024 ? 1024 : n + n / 8;
  const size_t T = next_pow2(2 * cap);
  CK(dalloc(&s.k, cap * 8));
  CK(dalloc(&s.key_slot, cap));
  CK(dalloc(&s.key_index, cap));
  CK(dalloc(&s.key_rep, cap));
  CK(dalloc(&s.table, T));
  CK(dalloc(&s.slot_key, T));
  // >= msm_num_points_split(n, m) for any m <= n (split coefficients add m + 1 points)
  CK(dalloc(&s.pts, (3 + 3 * cap) * NIELS_WORDS));
  CK(dalloc(&s.scal, (3 + 3 * cap) * 8));
  CK(dalloc(&s.key_acc, cap * KEY_ACC_LIMBS));
  CK(dalloc(&s.u_acc, (cap / COEF_CHUNK + 2) * KEY_ACC_LIMBS));   // one sum per fallback range
  CK(dalloc(&s.coef_part, coef_part_words(cap)));
  CK(dalloc(&s.itembad, 2 * cap));   // [0, cap): s bits (k_coef), [cap, 2 cap): R bits (k_decompress)
  CK(dalloc(&s.keybad, cap));
  launch_init_basepoint(s.st, s.pts);
  CK(hipGetLastError());
  s.cap_n = cap;
  s.cap_T = T;
  return 0;
}

// MSM workspace for plan P with up to `entries` digits (grow-only; the slot is idle when called)
static int ensure_msm(edc_ctx* ctx, Slot& s, const MsmPlan& P, size_t entries) {
  const uint32_t nbin = P.nbin();
  if (nbin > MSM_MAX_BINS || P.nwin > MSM_MAX_WIN) { ctx->err = "MSM plan too large"; return EDC_ERR_ARG; }
  if (nbin > s.cap_bins || P.nranges > s.cap_ranges) {
    CK(hipStreamSynchronize(s.st));
    for (void* p : {(void*)s.counts, (void*)s.offsets, (void*)s.cursor, (void*)s.slice_W, (void*)s.slice_T,
                    (void*)s.win, (void*)s.buckets, (void*)s.heads, (void*)s.bucket_end})
      if (p) (void)hipFree(p);
    const uint32_t nb = nbin > s.cap_bins ? nbin : s.cap_bins;
    const uint32_t nr = P.nranges > s.cap_ranges ? P.nranges : (s.cap_ranges ? s.cap_ranges : 1);
    s.counts = s.offsets = s.cursor = s.slice_W = s.slice_T = s.win = s.buckets = s.heads = nullptr;
    s.bucket_end = nullptr;
    s.cap_bins = s.cap_ranges = 0;
    CK(dalloc(&s.counts, nb));
    CK(dalloc(&s.offsets, nb));
    CK(dalloc(&s.cursor, nb));
    CK(dalloc(&s.slice_W, (size_t)nb * EXT_WORDS));
    CK(dalloc(&s.slice_T, (size_t)nb * EXT_WORDS));
    CK(dalloc(&s.win, (size_t)nr * MSM_MAX_WIN * EXT_WORDS));
    CK(dalloc(&s.buckets, msm_bucket_words(nb)));
    CK(dalloc(&s.heads, msm_bucket_words(nb)));
    CK(dalloc(&s.bucket_end, (size_t)nb * NSLICE));
    s.cap_bins = nb;
    s.cap_ranges = nr;
  }
  if (entries > s.cap_entries) {
    CK(hipStreamSynchronize(s.st));
    if (s.entries) (void)hipFree(s.entries);
    if (s.sorted) (void)hipFree(s.sorted);
    s.entries = nullptr;
    s.sorted = nullptr;
    s.cap_entries = 0;
    const size_t cap = entries + entries / 8 + 1024;
    CK(dalloc(&s.entries, cap));
    // + 256 per possible bin: each bin's lane-major region is padded to whole rounds (k_msm_sort)
    CK(dalloc(&s.sorted, cap + 256 * (size_t)MSM_MAX_BINS));
    s.cap_entries = cap;
  }
  return 0;
}

// ---- MSM plans ----
// Window width by batch size: wide windows amortize the 2 x buckets reduction work over many
// points; narrow ones keep enough digits per bucket for small batches. Below 2^13 signatures the
// windows are at most 9 bits (256 signed buckets, 8-bit unsigned top windows), i.e. one slice
// each, so no window-combine pass runs before the Horner pass (~90 us of latency per call).
static int auto_window_bits(size_t n) {
  if (n >= (1u << 19)) return 16;
  if (n >= (1u << 17)) return 15;   // 9 z windows; 14 bits 2 % and 16 bits 15 % slower at 2^17 (r06w)
  if (n >= (1u << 15)) return 13;
  if (n >= (1u << 13)) return 12;
  return 9;
}

// Windows of at most c bits over the 128 bits of a z (short scalars: windows 0..ws-1), then
// windows of at most hi bits over bits 128..252 of the full-width coefficients (< l < 2^253). The
// top window of each kind is unsigned (nothing sits above it, so no carry out): its digit reaches
// 2^bits, hence 2^bits buckets instead of 2^(bits-1). Widths are balanced: a window with only a
// few live bits would send every term's digit to a handful of buckets of one bin, i.e. one
// workgroup. Every slice starts as one bin (nsub = 1; batch_plan may split them).
static void plan_layout(MsmPlan& P) {
  uint32_t bin = 0;
  for (uint32_t w = 0; w < P.nwin; ++w) {
    P.bin0[w] = (uint16_t)bin;
    bin += (uint32_t)P.nslice[w] * P.nsub[w];
  }
  P.bins_per_range = bin;
}

static MsmPlan make_plan(int c, int hi, uint32_t nranges, bool hi_windows = true) {
  MsmPlan P{};
  uint32_t w = 0, off = 0;
  auto add = [&](uint32_t bits, uint32_t buckets) {
    P.off[w] = (uint16_t)off;
    P.bits[w] = (uint8_t)bits;
    P.nslice[w] = (uint16_t)((buckets + NSLICE - 1) / NSLICE);
    P.nsub[w] = 1;
    off += bits;
    ++w;
  };
  const uint32_t ws = (128 + c - 1) / c;
  for (uint32_t i = 0; i < ws; ++i) {
    const uint32_t bits = 128 / ws + (i < 128 % ws ? 1 : 0);
    add(bits, i + 1 == ws ? (1u << bits) : (1u << (bits - 1)));
  }
  P.nwin_short = ws;
  const uint32_t wh = hi_windows ? (125 + hi - 1) / hi : 0;
  for (uint32_t i = 0; i < wh; ++i) {
    const uint32_t bits = 125 / wh + (i < 125 % wh ? 1 : 0);
    add(bits, i + 1 == wh ? (1u << bits) : (1u << (bits - 1)));
  }
  P.nwin = w;
  P.nranges = nranges;
  plan_layout(P);
  return P;
}

static uint32_t floor_pow2(double x) {
  uint32_t p = 1;
  while (p * 2.0 <= x && p < 64) p *= 2;
  return p;
}

// Batch plan: few distinct keys (consensus votes; known from the previous grouped batch on this
// context) put the 253-bit B / key coefficients' high bits in 8-bit windows with ~m entries each
// (one bin per window instead of 128 nearly empty ones); otherwise every window has c bits.
// Small batches split the slices of their densest windows into sub-bins (terms interleaved by
// index, summed per slice by k_msm_window) so that every bin holds about the same number of
// entries and ~1-2k workgroups accumulate. edc_set_msm_shape's parts instead split the whole batch.
// Any plan is an exact MSM: the hint and the split only affect speed.
static MsmPlan batch_plan(const edc_ctx* ctx, size_t n, bool per_sig, bool split = false) {
  const int c = ctx->win_bits ? ctx->win_bits : auto_window_bits(n);
  const bool few = !per_sig && ctx->have_key_ratio && ctx->last_key_ratio * 16.0 <= 1.0 && n >= 4096;
  MsmPlan P = make_plan(c, few ? 8 : c, 1, !split);
  if (ctx->msm_parts) {
    uint32_t parts = ctx->msm_parts;
    while (parts > 1 && P.bins_per_range * parts > MSM_MAX_BINS) parts /= 2;
    P.nranges = parts;
    P.sum_ranges = parts > 1;
    return P;
  }
  // expected entries per slice of each window: short terms (the z_i) use the short windows, full
  // terms (B and the keys: m estimated from the last grouped batch, n per signature) all windows.
  // Only the lower half of two windows' slices is live: in the top short window the full terms'
  // digits are signed, and in the top full window bit 252 is set only by coefficients in
  // [2^252, l), a 2^-125 fraction.
  const double ns = (double)n;
  const double nf = 1.0 + (per_sig ? ns : (ctx->have_key_ratio ? ctx->last_key_ratio * ns : ns));
  double dens[MSM_MAX_WIN], total = 0;
  for (uint32_t w = 0; w < P.nwin; ++w) {
    const double sl = P.nslice[w], half = sl > 1 ? sl / 2 : 1;
    if (split) dens[w] = (ns + 2 * nf) / sl;      // every term short, top windows unsigned
    else if (w + 1 < P.nwin_short) dens[w] = (ns + nf) / sl;
    else if (w + 1 == P.nwin_short) dens[w] = ns / sl + nf / half;
    else if (w + 1 < P.nwin) dens[w] = nf / sl;
    else dens[w] = nf / half;
    total += split ? ns + 2 * nf : (w < P.nwin_short ? ns + nf : nf);
  }
  double target = ctx->bin_entries ? (double)ctx->bin_entries : (total / 1024.0 > 4096.0 ? total / 1024.0 : 4096.0);
  for (;;) {
    for (uint32_t w = 0; w < P.nwin; ++w) P.nsub[w] = (uint8_t)floor_pow2(dens[w] / target);
    plan_layout(P);
    if (P.bins_per_range <= MSM_MAX_BINS) break;
    target *= 2;
  }
  return P;
}

static MsmTerms batch_terms(const MsmPlan& P, const Slot& s, uint32_t n, bool split) {
  return MsmTerms{n, 0, 0, 0, P.sum_ranges ? P.nranges : 1u, s.scal, nullptr, nullptr, nullptr, split ? 1u : 0u};
}

// Split coefficients need [2^128]A of every key of the batch; the cache holds it for registered
// keys. They are planned while the previous batch found all its keys in the cache (a key missing
// from it still verifies exactly: k_decompress doubles it 128 times, and the next batches go back
// to the wide-coefficient plan until a batch finds every key again).
static bool choose_split(const edc_ctx* ctx) {
  return ctx->kc_m && ctx->bcomb && ctx->key_split == 0 && ctx->last_uncached == 0;
}

// host-staging buffers (inputs of the host-pointer entry points, per-item outputs)
static int ensure_n(edc_ctx* ctx, size_t n) {
  if (n <= ctx->cap_n && ctx->vk) return 0;
  CK(hipStreamSynchronize(ctx->st()));
  void* ptrs[] = {ctx->vk, ctx->sig, ctx->zexp, ctx->off, ctx->kbuf, ctx->verdicts, ctx->vtab};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  const size_t cap = n < 1024 ? 1024 : n + n / 8;
  CK(dalloc(&ctx->vtab, verify_single_scratch_words(cap)));
  CK(dalloc(&ctx->vk, cap * 32));
  CK(dalloc(&ctx->sig, cap * 64));
  CK(dalloc(&ctx->zexp, cap * 16));
  CK(dalloc(&ctx->off, cap + 1));
  CK(dalloc(&ctx->kbuf, cap * 8));
  CK(dalloc(&ctx->verdicts, cap));
  ctx->cap_n = cap;
  return 0;
}

static int ensure_msg(edc_ctx* ctx, size_t bytes) {
  if (bytes <= ctx->cap_msg && ctx->msg) return 0;
  CK(hipStreamSynchronize(ctx->st()));
  if (ctx->msg) (void)hipFree(ctx->msg);
  size_t cap = bytes < 4096 ? 4096 : bytes + bytes / 8;
  CK(dalloc(&ctx->msg, cap));
  ctx->cap_msg = cap;
  return 0;
}

static int ensure_aux(edc_ctx* ctx, size_t bytes) {
  if (bytes <= ctx->cap_aux && ctx->aux) return 0;
  CK(hipStreamSynchronize(ctx->st()));
  if (ctx->aux) (void)hipFree(ctx->aux);
  size_t cap = bytes < 4096 ? 4096 : bytes + bytes / 8;
  CK(dalloc(&ctx->aux, cap));
  ctx->cap_aux = cap;
  return 0;
}

static void seed_words(const uint8_t* seed, uint32_t w[8]) {
  for (int j = 0; j < 8; ++j)
    w[j] = seed ? ((uint32_t)seed[4 * j] | ((uint32_t)seed[4 * j + 1] << 8) | ((uint32_t)seed[4 * j + 2] << 16) |
                   ((uint32_t)seed[4 * j + 3] << 24))
                : 0u;
}

// Stage the message arena + offsets (0-based) into the context's device buffers (slot 0 stream).
static int upload_msgs(edc_ctx* ctx, size_t n, const uint8_t* msg, const uint64_t* msg_off) {
  if (n && !msg_off) { ctx->err = "null msg_off"; return EDC_ERR_ARG; }
  int rc = init_slot(ctx, ctx->slot[0]);
  if (rc) return rc;
  rc = ensure_n(ctx, n);
  if (rc) return rc;
  const size_t mbytes = n ? (size_t)(msg_off[n] - msg_off[0]) : 0;
  if (mbytes && !msg) { ctx->err = "null msg"; return EDC_ERR_ARG; }
  rc = ensure_msg(ctx, mbytes);
  if (rc) return rc;
  if (!n) return 0;
  hipStream_t st = ctx->st();
  if (mbytes) CK(hipMemcpyAsync(ctx->msg, msg + msg_off[0], mbytes, hipMemcpyHostToDevice, st));
  if (msg_off[0] == 0) {
    CK(hipMemcpyAsync(ctx->off, msg_off, (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, st));
  } else {
    std::vector<uint64_t> o(n + 1);
    for (size_t i = 0; i <= n; ++i) o[i] = msg_off[i] - msg_off[0];
    CK(hipMemcpyAsync(ctx->off, o.data(), (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    CK(hipStreamSynchronize(st));
  }
  return 0;
}

// Stage the host inputs (keys, signatures, messages) into the context's device buffers.
static int upload(edc_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg,
                  const uint64_t* msg_off) {
  if (n && (!vk || !sig)) { ctx->err = "null input"; return EDC_ERR_ARG; }
  int rc = upload_msgs(ctx, n, msg, msg_off);
  if (rc || !n) return rc;
  CK(hipMemcpyAsync(ctx->vk, vk, n * 32, hipMemcpyHostToDevice, ctx->st()));
  CK(hipMemcpyAsync(ctx->sig, sig, n * 64, hipMemcpyHostToDevice, ctx->st()));
  return 0;
}

// Stage host inputs into slot s's own device buffers on the slot's stream (edc_batch_submit), so
// the copy of one batch overlaps the kernels of the batches already in flight on other slots.
static int ensure_slot_inputs(edc_ctx* ctx, Slot& s, size_t n, size_t mbytes) {
  int rc = init_slot(ctx, s);
  if (rc) return rc;
  if (n > s.in_cap_n || !s.in_vk) {
    CK(hipStreamSynchronize(s.st));
    void* in[] = {s.in_vk, s.in_sig, s.in_off, s.in_idx};
    for (void* p : in)
      if (p) (void)hipFree(p);
    s.in_vk = s.in_sig = nullptr;
    s.in_off = nullptr;
    s.in_idx = nullptr;
    s.in_cap_n = 0;
    const size_t cap = n < 1024 ? 1024 : n + n / 8;
    CK(dalloc(&s.in_vk, cap * 32));
    CK(dalloc(&s.in_sig, cap * 64));
    CK(dalloc(&s.in_off, cap + 1));
    CK(dalloc(&s.in_idx, cap));
    s.in_cap_n = cap;
  }
  if (mbytes > s.in_cap_msg || !s.in_msg) {
    CK(hipStreamSynchronize(s.st));
    if (s.in_msg) (void)hipFree(s.in_msg);
    s.in_msg = nullptr;
    s.in_cap_msg = 0;
    const size_t cap = mbytes < 4096 ? 4096 : mbytes + mbytes / 8;
    CK(dalloc(&s.in_msg, cap));
    s.in_cap_msg = cap;
  }
  return 0;
}

static int upload_slot(edc_ctx* ctx, Slot& s, size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg,
                       const uint64_t* msg_off, const uint32_t* key_idx = nullptr) {
  if (n && ((!vk && !key_idx) || !sig || !msg_off)) { ctx->err = "null input"; return EDC_ERR_ARG; }
  const size_t mbytes = n ? (size_t)(msg_off[n] - msg_off[0]) : 0;
  if (mbytes && !msg) { ctx->err = "null msg"; return EDC_ERR_ARG; }
  int rc = ensure_slot_inputs(ctx, s, n, mbytes);
  if (rc) return rc;
  if (!n) return 0;
  hipStream_t st = s.st;
  const uint64_t* off = msg_off;
  if (msg_off[0] != 0) {
    s.in_rebased.resize(n + 1);
    for (size_t i = 0; i <= n; ++i) s.in_rebased[i] = msg_off[i] - msg_off[0];
    off = s.in_rebased.data();
  }
  CK(hipMemcpyAsync(s.in_off, off, (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, st));
  if (mbytes) CK(hipMemcpyAsync(s.in_msg, msg + msg_off[0], mbytes, hipMemcpyHostToDevice, st));
  if (key_idx) {                     // 4 bytes per item over PCIe instead of 32
    CK(hipMemcpyAsync(s.in_idx, key_idx, n * sizeof(uint32_t), hipMemcpyHostToDevice, st));
    launch_expand_keys(st, (uint32_t)n, s.in_idx, ctx->kc_reg, ctx->kc_keys, s.in_vk);
    CK(hipGetLastError());
  } else {
    CK(hipMemcpyAsync(s.in_vk, vk, n * 32, hipMemcpyHostToDevice, st));
  }
  CK(hipMemcpyAsync(s.in_sig, sig, n * 64, hipMemcpyHostToDevice, st));
  return 0;
}

// Prehashed host submissions (reference Item = {vk_bytes, sig, k}, src/batch.rs:76-80): keys and
// signatures into the slot's input buffers, the 32-byte challenges straight into the slot's k
// array (128 B per item over PCIe, no message bytes).
static int upload_slot_prehashed(edc_ctx* ctx, Slot& s, size_t n, const uint8_t* vk, const uint8_t* sig,
                                 const uint8_t* k, const uint32_t* key_idx = nullptr) {
  if (n && ((!vk && !key_idx) || !sig || !k)) { ctx->err = "null input"; return EDC_ERR_ARG; }
  int rc = ensure_slot_inputs(ctx, s, n, 0);
  if (rc) return rc;
  rc = ensure_slot(ctx, s, n);
  if (rc || !n) return rc;
  if (key_idx) {                     // 4 bytes per item over PCIe instead of 32: 100 B per item
    CK(hipMemcpyAsync(s.in_idx, key_idx, n * sizeof(uint32_t), hipMemcpyHostToDevice, s.st));
    launch_expand_keys(s.st, (uint32_t)n, s.in_idx, ctx->kc_reg, ctx->kc_keys, s.in_vk);
    CK(hipGetLastError());
  } else {
    CK(hipMemcpyAsync(s.in_vk, vk, n * 32, hipMemcpyHostToDevice, s.st));
  }
  CK(hipMemcpyAsync(s.in_sig, sig, n * 64, hipMemcpyHostToDevice, s.st));
  CK(hipMemcpyAsync(s.k, k, n * 32, hipMemcpyHostToDevice, s.st));
  return 0;
}

// caller-supplied device k arrays are read with 16-byte loads
static bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

static uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// Key grouping (the reference's HashMap<VerificationKeyBytes, _>, src/batch.rs:114-137) only
// saves work when keys repeat. When the last grouped batch had almost only distinct keys, the
// key terms stay per signature (A_i with coefficient z_i k_i): the same group element, so the
// same verdict and [8]check, without the hash table and the per-key atomics. Auto mode groups
// every 8th batch anyway, to notice when keys start repeating.
static bool choose_per_sig(const edc_ctx* ctx, size_t n) {
  return ctx->key_grouping == 2 || (ctx->key_grouping == 0 && n >= 4096 && ctx->have_key_ratio &&
                                    ctx->last_key_ratio > 0.5 && ctx->ungrouped_run < 7);
}

// Key lanes of a batch's decode launch. The distinct-key count m is only known on the device, so
// every possible key (m <= n) used to get a lane: at 2^20 votes from 150 validators, 2^20 lanes
// (16,384 waves) that exit at once. Grouped batches now get twice the previous grouped batch's key
// count (at least 4,096 lanes); a batch with more keys loops over them (k_decompress), so the
// hint only affects speed. One key term per signature: m = n exactly.
static uint32_t key_lanes(const edc_ctx* ctx, size_t n, bool per_sig) {
  if (per_sig || !ctx->have_key_ratio) return (uint32_t)n;
  const double m2 = 2.0 * ctx->last_key_ratio * (double)n;
  const size_t lanes = m2 < 4096.0 ? 4096 : (size_t)m2 + 64;
  return (uint32_t)(lanes < n ? lanes : n);
}

// Enqueue the per-signature prefix of the pipeline on slot s: key grouping, SHA-512 challenges,
// z and coefficients, ZIP215 decode of R_i and the keys. No host synchronization. With d_k (the
// prehashed entries: the caller's queue-time k, src/batch.rs:76-94) SHA-512 is skipped and the
// messages are not read (d_msg / d_off may be null).
static int enqueue_prefix(edc_ctx* ctx, Slot& s, size_t n, const uint8_t* d_vk, const uint8_t* d_sig,
                          const uint8_t* d_msg, const uint64_t* d_off, const uint8_t* z_seed, uint64_t z_base,
                          const uint8_t* d_z, bool with_bin, const MsmPlan* P, bool force_per_sig = false,
                          bool split = false, const uint32_t* d_k = nullptr) {
  if (n >= (1ull << 28)) { ctx->err = "batch too large for one call (max 2^28 items)"; return EDC_ERR_ARG; }
  if (n && (!aligned16(d_vk) || !aligned16(d_sig) || (d_z && !aligned16(d_z)) || (d_k && !aligned16(d_k)))) {
    ctx->err = "device vk / sig / z / k arrays must be 16-byte aligned";
    return EDC_ERR_ARG;
  }
  int rc = ensure_slot(ctx, s, n);
  if (rc) return rc;
  s.kin = d_k ? d_k : s.k;
  s.nmulti = 0;
  const uint32_t N = (uint32_t)n;
  const uint32_t T = (uint32_t)next_pow2(2 * (n < 128 ? 128 : n));
  if (T > s.cap_T) { ctx->err = "hash table capacity"; return EDC_ERR_ARG; }
  uint32_t seed[8];
  seed_words(z_seed, seed);
  hipStream_t st = s.st;
  s.timed = ctx->timing;
  auto mark = [&](int ph) {
    if (s.timed) (void)hipEventRecord(s.ev[ph], st);
  };
  const bool per_sig = force_per_sig || choose_per_sig(ctx, n);
  s.per_sig = per_sig;
  s.n_batch = N;
  mark(PH_KEYS);
  launch_init_batch(st, s.flags, per_sig ? (int)N : -1, s.u_acc, s.d_out, per_sig ? nullptr : s.table, per_sig ? 0u : T,
                    with_bin && EDC_RUN(8) ? s.counts : nullptr, with_bin && EDC_RUN(8) ? P->nbin() : 0u);
  if (!per_sig) {
    const uint64_t h = splitmix64(ctx->secret ^ splitmix64(ctx->nbatches++));
    const uint32_t salt[2] = {(uint32_t)h, (uint32_t)(h >> 32)};
    launch_keys(st, N, d_vk, s.table, T - 1, salt, ctx->key_grouping == 3, s.slot_key, s.key_slot, s.key_rep,
                s.key_index, s.key_acc, s.flags);
  }
  // dual-stream builds (untimed batches): the decode only needs the key grouping, so it runs on
  // the slot's second stream beside SHA-512 / coefficients / binning; its per-item R bits go to
  // their own array (itembad + cap_n), so no byte is written by both streams.
  // Contract while st2 runs (between ev_keys and the wait on ev_dec below): k_decompress reads
  // d_sig, d_vk, key_rep, flags[FLAG_NKEYS / FLAG_OVF] and the key cache, and writes pts,
  // itembad + cap_n, keybad and flags[FLAG_BAD / FLAG_UNCACHED] (atomics). The kernels enqueued on
  // st in between (coefficients, binning, bucket sort) must not read pts / keybad / itembad + cap_n,
  // write key_rep or FLAG_NKEYS / FLAG_OVF, or plain-store into flags; anything that does must
  // come after the ev_dec wait. tests/test_gpu_prehashed.py compares slot 0 (dual stream) with a
  // pipelined slot (one stream) on batches that fail in the decode and in the s check.
  // The decode is released after SHA-512, not right after the key grouping: both are VALU-bound,
  // and a decode launched first fills the GPU and starves SHA-512 (measured: the challenge took
  // ~1.0 ms beside the decode instead of 0.22 ms alone), so the light coefficient / binning /
  // sort chain queued behind SHA-512 ran after the decode instead of beside it.
  const bool dual = EDC_DUAL_STREAM && s.st2 && !s.timed;
  mark(PH_CHALLENGE);
  if (!d_k && EDC_RUN(2)) launch_challenge(st, N, d_vk, d_sig, d_msg, d_off, s.k);
  if (dual) {
    CK(hipEventRecord(s.ev_keys, st));
    CK(hipStreamWaitEvent(s.st2, s.ev_keys, 0));
    if (EDC_RUN(16))
      launch_decompress(s.st2, N, d_sig, d_vk, s.key_rep, per_sig, s.pts, s.itembad + s.cap_n, s.keybad, s.flags,
                        ctx->kc(), split, key_lanes(ctx, n, per_sig));
    CK(hipEventRecord(s.ev_dec, s.st2));
  }
  mark(PH_COEF);
  if (EDC_RUN(4)) launch_coef(st, N, d_sig, s.kin, d_z, seed, z_base, s.key_index, s.scal, s.key_acc, s.u_acc, s.itembad, s.flags,
              per_sig, s.coef_part, split);
  mark(PH_MSM_BIN);
  if (with_bin && EDC_RUN(8))
    launch_msm_bin(st, *P, batch_terms(*P, s, N, split), split ? 2 + 3 * N : 1 + 2 * N, s.counts, s.offsets, s.cursor,
                   s.entries, s.flags, true);
  // the per-bin bucket sort needs only the binning: before the decode join, so on the dual-stream
  // slot it runs beside the decode instead of after it
  if (with_bin && EDC_RUN(256))
    launch_msm_sort(st, *P, s.counts, s.offsets, s.entries, s.sorted, s.bucket_end, s.buckets);
  // the points are decoded last, right before the accumulation gathers them, so the freshly
  // written point table (134 MB at 2^20) is still in the Infinity Cache for the random row gathers
  mark(PH_DECOMP);
  if (dual) CK(hipStreamWaitEvent(st, s.ev_dec, 0));
  else if (EDC_RUN(16))
    launch_decompress(st, N, d_sig, d_vk, s.key_rep, per_sig, s.pts, s.itembad + s.cap_n, s.keybad, s.flags, ctx->kc(),
                      split, key_lanes(ctx, n, per_sig));
  CK(hipGetLastError());
  return 0;
}

// Enqueue the whole batch pipeline on slot s (device-resident inputs); no host synchronization.
static int enqueue_batch(edc_ctx* ctx, Slot& s, size_t n, const uint8_t* d_vk, const uint8_t* d_sig,
                         const uint8_t* d_msg, const uint64_t* d_off, const uint8_t* z_seed, uint64_t z_base,
                         const uint8_t* d_z, int want_compress, const uint32_t* d_k = nullptr,
                         bool latency = false) {
  if (n >= (1ull << 28)) { ctx->err = "batch too large for one call (max 2^28 items)"; return EDC_ERR_ARG; }
  int rc = ensure_slot(ctx, s, n);
  if (rc) return rc;
  const bool per_sig = choose_per_sig(ctx, n), split = choose_split(ctx);
  const MsmPlan P = batch_plan(ctx, n, per_sig, split);
  rc = ensure_msm(ctx, s, P, split ? msm_entry_capacity(P, 2 + 3 * n, 0) : msm_entry_capacity(P, n, n + 1));
  if (rc) return rc;
  rc = enqueue_prefix(ctx, s, n, d_vk, d_sig, d_msg, d_off, z_seed, z_base, d_z, true, &P, per_sig, split, d_k);
  if (rc) return rc;
  hipStream_t st = s.st;
  if (s.timed) (void)hipEventRecord(s.ev[PH_MSM_BUCKET], st);
  launch_msm_bucket(st, P, s.counts, s.offsets, s.entries, s.sorted, s.bucket_end, s.pts, s.buckets, s.heads, s.slice_W,
                    s.slice_T, s.probe_runs ? EDC_PROBE_SKIP : 0, s.timed ? s.ev_acc[0] : nullptr,
                    s.timed ? s.ev_acc[1] : nullptr, latency, s.flags);
  s.acc_nbin = P.nbin();
  if (s.timed) (void)hipEventRecord(s.ev[PH_MSM_TAIL], st);
  // the final kernel stores the result block to d_out and straight into the pinned h_out
  if (EDC_RUN(128)) launch_msm_tail(st, P, s.slice_W, s.slice_T, s.win, s.flags, want_compress, s.d_out, s.h_out);
  if (s.timed) {
    (void)hipEventRecord(s.ev[PH_N], st);
    // the accumulation's entry count (the last bin's offset + count), read at the wait without
    // another sync; queued after the last phase event so that no phase time includes the copies
    if (s.acc_nbin) {
      CK(hipMemcpyAsync(s.h_acc, s.offsets + s.acc_nbin - 1, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
      CK(hipMemcpyAsync(s.h_acc + 1, s.counts + s.acc_nbin - 1, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    }
  }
  CK(hipGetLastError());
  s.pending = true;
  s.probe_runs++;
  return 0;
}

// ---- several batches in one launch sequence (edc_batch_submit_multi_device) ----
// nb consecutive batches of n_per items each (a node verifying several blocks at once, or one
// GPU's shards of consecutive blocks): every per-item kernel runs once over all nb * n_per items,
// so small batches fill the GPU like one large batch, and the MSM is range-tagged (one range per
// batch, the plan of an n_per batch in each) with one Horner, verdict, check8 and partial per
// range. Batch b's z are drawn at z_base + b n_per + i: its results equal a separate
// edc_batch_verify_device / edc_batch_partial_device of batch b at that z_base. The grouped
// fallback's range machinery (k_coef range mode, listed key / B terms) with the key count left
// on the device: per-(batch, key) sums sit at b * kstride + key and the term layout is resolved
// from the key grouping by the binning kernels (MsmTerms::dyn).
static int multi_args(edc_ctx* ctx, uint32_t nb, size_t n_per, const uint8_t* d_vk, const uint8_t* d_sig,
                      const uint8_t* d_msg, const uint64_t* d_off, const uint32_t* d_k) {
  if (nb < 1 || nb > kMultiMax || n_per == 0 || n_per % COEF_CHUNK) {
    ctx->err = "multi-batch: 1..16 batches of a multiple of 2048 items each";
    return EDC_ERR_ARG;
  }
  if ((size_t)nb * n_per >= (1ull << 28)) { ctx->err = "batch too large for one call (max 2^28 items)"; return EDC_ERR_ARG; }
  if (!aligned16(d_vk) || !aligned16(d_sig) || (d_k && !aligned16(d_k))) {
    ctx->err = "device vk / sig / k arrays must be 16-byte aligned";
    return EDC_ERR_ARG;
  }
  if (!d_k && (!d_msg || !d_off)) { ctx->err = "null msg"; return EDC_ERR_ARG; }
  return 0;
}

static int enqueue_multi(edc_ctx* ctx, Slot& s, uint32_t nb, size_t n_per, const uint8_t* d_vk, const uint8_t* d_sig,
                         const uint8_t* d_msg, const uint64_t* d_off, const uint32_t* d_k, const uint8_t* z_seed,
                         uint64_t z_base, int want_compress) {
  int rc = multi_args(ctx, nb, n_per, d_vk, d_sig, d_msg, d_off, d_k);
  if (rc) return rc;
  const size_t N = (size_t)nb * n_per;
  rc = ensure_slot(ctx, s, N);
  if (rc) return rc;
  const bool per_sig = choose_per_sig(ctx, N);
  const uint32_t kstride = (uint32_t)(N < kMultiKeys ? N : kMultiKeys);
  MsmPlan P = batch_plan(ctx, n_per, per_sig, false);
  P.nranges = nb;
  P.sum_ranges = 0;
  if (P.bins_per_range * nb > MSM_MAX_BINS) {       // drop the sub-bins of the per-batch plan
    for (uint32_t w = 0; w < P.nwin; ++w) P.nsub[w] = 1;
    plan_layout(P);
  }
  if (P.bins_per_range * nb > MSM_MAX_BINS) { ctx->err = "multi-batch: too many batches for the MSM plan"; return EDC_ERR_ARG; }
  const size_t nx_max = (size_t)nb * kstride + nb;
  const size_t full_max = (N > (size_t)nb * kstride ? N : (size_t)nb * kstride) + nb;
  rc = ensure_msm(ctx, s, P, msm_entry_capacity(P, N, full_max));
  if (rc) return rc;
  if ((size_t)nb * kstride * KEY_ACC_LIMBS > s.mb_cap_acc || nx_max > s.mb_cap_terms || !s.mb_bad) {
    CK(hipStreamSynchronize(s.st));
    void* mb[] = {s.mb_acc, s.mb_xpt, s.mb_xrg, s.mb_xscal, s.mb_bad};
    for (void* p : mb)
      if (p) (void)hipFree(p);
    s.mb_acc = nullptr;
    s.mb_xpt = s.mb_xrg = s.mb_xscal = nullptr;
    s.mb_bad = nullptr;
    s.mb_cap_acc = s.mb_cap_terms = 0;
    const size_t acc = (size_t)kMultiMax * kMultiKeys * KEY_ACC_LIMBS, terms = (size_t)kMultiMax * kMultiKeys + kMultiMax;
    CK(dalloc(&s.mb_acc, acc));
    CK(dalloc(&s.mb_xpt, terms));
    CK(dalloc(&s.mb_xrg, terms));
    CK(dalloc(&s.mb_xscal, terms * 8));
    CK(dalloc(&s.mb_bad, kMultiMax));
    s.mb_cap_acc = acc;
    s.mb_cap_terms = terms;
  }
  const uint32_t n = (uint32_t)N;
  const uint32_t T = (uint32_t)next_pow2(2 * (N < 128 ? 128 : N));
  if (T > s.cap_T) { ctx->err = "hash table capacity"; return EDC_ERR_ARG; }
  uint32_t seed[8];
  seed_words(z_seed, seed);
  hipStream_t st = s.st;
  s.timed = false;
  s.kin = d_k ? d_k : s.k;
  s.per_sig = per_sig;
  s.n_batch = n;
  s.nmulti = nb;
  launch_init_batch(st, s.flags, per_sig ? (int)n : -1, s.u_acc, s.d_out, per_sig ? nullptr : s.table, per_sig ? 0u : T,
                    s.counts, P.nbin());
  if (!per_sig) {
    const uint64_t h = splitmix64(ctx->secret ^ splitmix64(ctx->nbatches++));
    const uint32_t salt[2] = {(uint32_t)h, (uint32_t)(h >> 32)};
    launch_keys(st, n, d_vk, s.table, T - 1, salt, ctx->key_grouping == 3, s.slot_key, s.key_slot, s.key_rep,
                s.key_index, s.key_acc, s.flags, kstride);
  }
  const bool dual = EDC_DUAL_STREAM && s.st2;       // same contract (and order) as enqueue_prefix
  if (!d_k) launch_challenge(st, n, d_vk, d_sig, d_msg, d_off, s.k);
  if (dual) {
    CK(hipEventRecord(s.ev_keys, st));
    CK(hipStreamWaitEvent(s.st2, s.ev_keys, 0));
    launch_decompress(s.st2, n, d_sig, d_vk, s.key_rep, per_sig, s.pts, s.itembad + s.cap_n, s.keybad, s.flags, ctx->kc(),
                      false, key_lanes(ctx, N, per_sig));
    CK(hipEventRecord(s.ev_dec, s.st2));
  }
  launch_multi_coef(st, n, nb, kstride, per_sig, d_sig, s.kin, seed, z_base, s.key_index, s.scal, s.mb_acc, s.u_acc,
                    s.itembad, s.flags, s.mb_xpt, s.mb_xrg, s.mb_xscal);
  const MsmTerms terms{n, (uint32_t)n_per, 0u, nb, 1u, s.scal, s.mb_xpt, s.mb_xrg, s.mb_xscal, 0u, per_sig ? 3u : 1u};
  launch_msm_bin(st, P, terms, (uint32_t)(N + full_max), s.counts, s.offsets, s.cursor, s.entries, s.flags, true);
  launch_msm_sort(st, P, s.counts, s.offsets, s.entries, s.sorted, s.bucket_end, s.buckets);
  if (dual) CK(hipStreamWaitEvent(st, s.ev_dec, 0));
  else
    launch_decompress(st, n, d_sig, d_vk, s.key_rep, per_sig, s.pts, s.itembad + s.cap_n, s.keybad, s.flags, ctx->kc(),
                      false, key_lanes(ctx, N, per_sig));
  CK(hipMemsetAsync(s.mb_bad, 0, nb, st));
  launch_range_prebad(st, n, (uint32_t)n_per, s.itembad, s.itembad + s.cap_n, s.keybad, s.key_index, per_sig, s.mb_bad,
                      s.flags);
  launch_msm_bucket(st, P, s.counts, s.offsets, s.entries, s.sorted, s.bucket_end, s.pts, s.buckets, s.heads, s.slice_W,
                    s.slice_T);
  launch_msm_multi_tail(st, P, s.slice_W, s.slice_T, s.win, s.flags, s.mb_bad, want_compress, s.d_out, s.h_out);
  CK(hipGetLastError());
  s.pending = true;
  return 0;
}

// Wait for a multi-batch slot: per batch verdict (EDC_OK / EDC_INVALID_SIGNATURE), optional
// check8 (nb x 32), partial (nb x 128) and bad flag; returns EDC_INVALID_SIGNATURE if any failed.
static int finish_multi(edc_ctx* ctx, Slot& s, size_t nb, int* verdicts, uint8_t* check8, uint8_t* partials, int* bad) {
  if (!s.pending || !s.nmulti) { ctx->err = "no multi-batch pending in this slot"; return EDC_ERR_ARG; }
  if (nb != s.nmulti) { ctx->err = "multi-batch count differs from the submission"; return EDC_ERR_ARG; }
  if (s.mu_union) {
    // The launch ran as one batch over all nb * n_per items (z at the same global indices). Its
    // equation is the sum of the nb batches' equations, so when it holds every batch holds (with
    // the probability batch verification itself gives: src/batch.rs:149-217) and each batch's
    // [8]*check is the identity. Otherwise, or when the caller wants the per-batch partials, the
    // launch is rerun range by range on the same slot (the inputs are still borrowed).
    s.mu_union = false;
    CK(hipStreamSynchronize(s.st));
    const int* u = reinterpret_cast<const int*>(s.h_out);
    if (u[45]) {
      s.pending = false;
      s.nmulti = 0;
      ctx->err = "prehashed k is not a canonical scalar (must be < l, as Scalar::from_hash returns)";
      return EDC_ERR_ARG;
    }
    if (!u[0] && !u[1] && !partials) {
      s.pending = false;
      s.nmulti = 0;
      if (s.per_sig) {
        ctx->ungrouped_run++;
      } else {
        ctx->ungrouped_run = 0;
        ctx->have_key_ratio = true;
        ctx->last_key_ratio = (double)u[2] / (double)s.n_batch;
      }
      if (ctx->kc_m) ctx->last_uncached = (uint32_t)u[44];
      ctx->mu_hits++;
      for (size_t g = 0; g < nb; ++g) {
        if (verdicts) verdicts[g] = EDC_OK;
        if (bad) bad[g] = 0;
        if (check8) {
          memset(check8 + 32 * g, 0, 32);
          check8[32 * g] = 1;                         // compressed identity
        }
      }
      return EDC_OK;
    }
    ctx->mu_reruns++;
    s.pending = false;
    s.nmulti = 0;
    int rc = enqueue_multi(ctx, s, (uint32_t)nb, s.mu_nper, s.mu_vk, s.mu_sig, s.mu_msg, s.mu_off, s.mu_k, s.mu_seed,
                           s.mu_zbase, s.mu_compress || check8 != nullptr);
    if (rc) return rc;
  }
  s.pending = false;
  s.nmulti = 0;
  CK(hipStreamSynchronize(s.st));
  const int* h0 = reinterpret_cast<const int*>(s.h_out);
  if (h0[45]) {
    ctx->err = "prehashed k is not a canonical scalar (must be < l, as Scalar::from_hash returns)";
    return EDC_ERR_ARG;
  }
  if (s.per_sig) {
    ctx->ungrouped_run++;
  } else {
    ctx->ungrouped_run = 0;
    ctx->have_key_ratio = true;
    ctx->last_key_ratio = (double)h0[2] / (double)s.n_batch;
  }
  if (ctx->kc_m) ctx->last_uncached = (uint32_t)h0[44];
  int any = 0;
  for (size_t g = 0; g < nb; ++g) {
    const uint8_t* b = s.h_out + 256 * g;
    const int v = reinterpret_cast<const int*>(b)[0], bd = reinterpret_cast<const int*>(b)[1];
    any |= v;
    if (verdicts) verdicts[g] = v ? EDC_INVALID_SIGNATURE : EDC_OK;
    if (bad) bad[g] = bd;
    if (check8) {
      if (bd) memset(check8 + 32 * g, 0, 32);
      else memcpy(check8 + 32 * g, b + 16, 32);
    }
    if (partials) memcpy(partials + 128 * g, b + 48, 128);
  }
  return any ? EDC_INVALID_SIGNATURE : EDC_OK;
}

#ifdef EDC_BATCH_STAMPS
// diagnostic build: one record per waited batch (ticket, n, host submit / wait-return time in us,
// the device phase stamps of edc_common.h BST_*), read and cleared by edc_debug_batch_stamps
static std::vector<uint32_t> g_bstamps;
static std::mutex g_bstamps_mu;    // contexts on several threads share the log
static uint64_t host_us() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}
extern "C" int edc_debug_batch_stamps(uint32_t* out, size_t cap_words) {
  std::lock_guard<std::mutex> g(g_bstamps_mu);
  const size_t n = std::min(cap_words, g_bstamps.size());
  if (out) memcpy(out, g_bstamps.data(), n * sizeof(uint32_t));
  g_bstamps.clear();
  return (int)(n / (4 + BST_N));
}
#endif

// Wait for slot s and harvest its result block (verdict, bad flag, check8, partial).
static int finish_batch(edc_ctx* ctx, Slot& s, uint8_t check8[32], uint8_t partial[128], int* bad_out) {
  if (!s.pending) { ctx->err = "no batch pending in this slot"; return EDC_ERR_ARG; }
  if (s.nmulti) { ctx->err = "multi-batch ticket: wait with edc_batch_wait_multi"; return EDC_ERR_ARG; }
  s.pending = false;
  CK(hipStreamSynchronize(s.st));
  if (s.timed) {
    for (int p = 0; p < PH_N; ++p) CK(hipEventElapsedTime(&ctx->last_ms[p], s.ev[p], s.ev[p + 1]));
    ctx->nlast = PH_N;
    CK(hipEventElapsedTime(&ctx->last_acc_ms, s.ev_acc[0], s.ev_acc[1]));
    // digit entries the accumulation added: the last bin's end (queued on s.st at the enqueue)
    ctx->last_acc_entries = s.acc_nbin ? s.h_acc[0] + s.h_acc[1] : 0;
  }
  const int verdict = reinterpret_cast<int*>(s.h_out)[0];
  const int bad = reinterpret_cast<int*>(s.h_out)[1];
#ifdef EDC_BATCH_STAMPS
  if (&s != &ctx->comb) {
    std::lock_guard<std::mutex> g(g_bstamps_mu);
    g_bstamps.push_back((uint32_t)s.ticket);
    g_bstamps.push_back(s.n_batch);
    g_bstamps.push_back((uint32_t)s.t_submit_us);
    g_bstamps.push_back((uint32_t)host_us());
    for (int k = 0; k < BST_N; ++k) g_bstamps.push_back(reinterpret_cast<uint32_t*>(s.h_out)[48 + k]);
  }
#endif
  if (&s != &ctx->comb && s.n_batch) {
    if (s.per_sig) {
      ctx->ungrouped_run++;
    } else {
      ctx->ungrouped_run = 0;
      ctx->have_key_ratio = true;
      ctx->last_key_ratio = (double)reinterpret_cast<int*>(s.h_out)[2] / (double)s.n_batch;
    }
    if (ctx->kc_m) ctx->last_uncached = (uint32_t)reinterpret_cast<int*>(s.h_out)[44];
  }
  if (&s != &ctx->comb && reinterpret_cast<int*>(s.h_out)[45]) {
    ctx->err = "prehashed k is not a canonical scalar (must be < l, as Scalar::from_hash returns)";
    return EDC_ERR_ARG;
  }
  if (check8) {
    if (bad) memset(check8, 0, 32);
    else memcpy(check8, s.h_out + 16, 32);
  }
  if (partial) memcpy(partial, s.h_out + 48, 128);
  if (bad_out) *bad_out = bad;
  return verdict ? EDC_INVALID_SIGNATURE : EDC_OK;
}

// Synchronous batch on slot 0.
static int run_batch_sync(edc_ctx* ctx, size_t n, const uint8_t* d_vk, const uint8_t* d_sig, const uint8_t* d_msg,
                          const uint64_t* d_off, const uint8_t* z_seed, uint64_t z_base, const uint8_t* d_z,
                          uint8_t check8[32], uint8_t partial[128], int* bad, const uint32_t* d_k = nullptr) {
  Slot& s = ctx->slot[0];
  if (s.pending) { ctx->err = "slot 0 busy: wait for submitted batches first"; return EDC_ERR_ARG; }
  // a synchronous call is one batch on an otherwise idle GPU: latency-shaped kernels (see
  // launch_msm_bucket); pipelined submissions keep the work-minimal ones
  int rc = enqueue_batch(ctx, s, n, d_vk, d_sig, d_msg, d_off, z_seed, z_base, d_z, check8 != nullptr, d_k, true);
  if (rc) return rc;
  return finish_batch(ctx, s, check8, partial, bad);
}

// ---- synchronous host-buffer calls, copy overlapped with compute ----
// A host-buffer call (the Rust shim's Verifier::verify, src/batch.rs:149) used to copy every input
// over PCIe and only then start the pipeline: at 2^20 prehashed items 134 MB (~2.5 ms at ~53 GB/s)
// + ~1.6 ms of compute. Here the inputs travel in pieces on a copy stream and each piece's work
// starts as it lands: the keys (and message offsets / caller z) first, so the key grouping and the
// keys' decode run under the signature copy; then the signatures (+ k or the message bytes) in
// chunks, each followed by its R decode (second stream) and its SHA-512 + coefficient pass (slot
// stream). A copy from pageable memory returns only when it has landed, so the calling thread
// issues nothing but copies and events, back to back, while a launcher thread enqueues each
// piece's kernels behind its event. The last chunk is small, so that little remains after the
// last byte: its decode and coefficients, the per-key merge, binning, sort and the MSM. Same
// kernels, same per-item / per-key arithmetic and the same integer sums (order-independent), so
// verdict and [8]*check are bit-identical to the one-piece path (tests/test_gpu_hostchunk.py).
constexpr size_t kHostChunkMin = 1u << 16;   // smaller calls copy in one piece (latency-bound anyway)
constexpr int kHostChunks = 8;               // chunks of signatures (ctx->hev: one event each + piece 0)

static bool host_chunked_ok(const edc_ctx* ctx, size_t n) {
  static const bool off = getenv("EDC_HOST_CHUNKS") && getenv("EDC_HOST_CHUNKS")[0] == '0';   // A/B measurement
  return !off && n >= kHostChunkMin && n < (1ull << 28) && !ctx->timing && ctx->slot[0].st2;
}

// chunk boundaries: kHostChunks - 1 equal chunks, then a last one of ~n/32; every boundary but n
// is a multiple of COEF_CHUNK (k_coef's workgroups start on one)
static std::vector<size_t> host_chunks(size_t n) {
  const size_t last = ((n + 31) / 32 + COEF_CHUNK - 1) / COEF_CHUNK * COEF_CHUNK;
  const size_t body = n > last ? (n - last) / COEF_CHUNK * COEF_CHUNK : 0;
  // body chunks of ~2^18 items: every pageable copy costs ~20-25 us of host time before the next
  // can start (r06c/r06d traces), and a 2^18 decode still ends under the next chunk's copy
  static const int env_chunks = getenv("EDC_HOST_BODY_CHUNKS") ? atoi(getenv("EDC_HOST_BODY_CHUNKS")) : 0;
  size_t k = env_chunks > 0 ? (size_t)env_chunks : (body + (1u << 17)) >> 18;
  if (k < 1) k = 1;
  if (k > kHostChunks - 1) k = kHostChunks - 1;
  const size_t c = ((body + k - 1) / k + COEF_CHUNK - 1) / COEF_CHUNK * COEF_CHUNK;
  std::vector<size_t> b{0};
  while (b.back() < body && c) b.push_back(b.back() + c < body ? b.back() + c : body);
  if (b.back() < n) b.push_back(n);
  return b;
}

// pieces landed so far (the copying thread counts up, the launcher thread waits)
struct HostGate {
  std::mutex m;
  std::condition_variable cv;
  int landed = 0;
  bool abort = false;
  void post(int k) {
    { std::lock_guard<std::mutex> g(m); landed = k; }
    cv.notify_all();
  }
  void stop() {
    { std::lock_guard<std::mutex> g(m); abort = true; }
    cv.notify_all();
  }
  bool wait(int k) {            // false: the copying thread gave up
    std::unique_lock<std::mutex> g(m);
    cv.wait(g, [&] { return landed >= k || abort; });
    return landed >= k;
  }
};

// Enqueue the whole chunked batch on slot 0 (inputs in host memory; k: prehashed challenges or
// null for the message path; z: caller-drawn z or null for the seed). The host buffers and
// `rebased` are read by the copies until the slot's wait.
static int enqueue_host_chunked(edc_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg,
                                const uint64_t* msg_off, const uint8_t* k, const uint8_t* z, const uint8_t* z_seed,
                                int want_compress, std::vector<uint64_t>& rebased) {
  Slot& s = ctx->slot[0];
  const size_t mbytes = k ? 0 : (size_t)(msg_off[n] - msg_off[0]);
  int rc = ensure_n(ctx, n);
  if (!rc) rc = ensure_slot(ctx, s, n);
  if (!rc && !k) rc = ensure_msg(ctx, mbytes);
  if (rc) return rc;
  if (!ctx->hcs) {
    CK(hipStreamCreateWithFlags(&ctx->hcs, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&ctx->hcs2, hipStreamNonBlocking));
    for (hipEvent_t& e : ctx->hev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (hipEvent_t& e : ctx->hev2) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  const bool per_sig = choose_per_sig(ctx, n), split = choose_split(ctx);
  const MsmPlan P = batch_plan(ctx, n, per_sig, split);
  rc = ensure_msm(ctx, s, P, split ? msm_entry_capacity(P, 2 + 3 * n, 0) : msm_entry_capacity(P, n, n + 1));
  if (rc) return rc;
  const uint32_t N = (uint32_t)n;
  const uint32_t T = (uint32_t)next_pow2(2 * (n < 128 ? 128 : n));
  if (T > s.cap_T) { ctx->err = "hash table capacity"; return EDC_ERR_ARG; }
  uint32_t seed[8];
  seed_words(z_seed, seed);
  hipStream_t st = s.st, st2 = s.st2, cs = ctx->hcs;
  s.kin = s.k;
  s.nmulti = 0;
  s.timed = false;
  s.per_sig = per_sig;
  s.n_batch = N;
  const std::vector<size_t> cb = host_chunks(n);
  const int nchunks = (int)cb.size() - 1;
  if (!k && msg_off[0] != 0) {
    rebased.resize(n + 1);
    for (size_t i = 0; i <= n; ++i) rebased[i] = msg_off[i] - msg_off[0];
  }
  const uint64_t salt64 = per_sig ? 0 : splitmix64(ctx->secret ^ splitmix64(ctx->nbatches++));
  const KeyCacheView kc = ctx->kc();

  // the launcher thread: every kernel, each piece's behind that piece's events. Two copying
  // threads: this one (keys / offsets / z, then the signature chunks) and a second one (the k or
  // message chunks) on its own stream, so that one thread's per-copy host work (~20-25 us per
  // pageable copy before its transfer starts) runs while the other's transfer is on the bus
  static const bool one_copier = getenv("EDC_HOST_COPY_THREADS") && getenv("EDC_HOST_COPY_THREADS")[0] == '1';
  HostGate gate, gate2;
  std::string lerr;
  int lrc = 0;
  std::thread launcher([&] {
    auto fail = [&](const char* what, hipError_t e) {
      (void)hipGetLastError();
      lerr = std::string(what) + ": " + hipGetErrorString(e);
      lrc = EDC_ERR_HIP;
    };
#define LK(expr)                                   \
  do {                                             \
    hipError_t e_ = (expr);                        \
    if (e_ != hipSuccess) return fail(#expr, e_);  \
  } while (0)
    LK(hipSetDevice(ctx->device));
    launch_init_batch(st, s.flags, per_sig ? (int)N : -1, s.u_acc, s.d_out, per_sig ? nullptr : s.table,
                      per_sig ? 0u : T, s.counts, P.nbin());
    if (!gate.wait(1)) return;
    LK(hipStreamWaitEvent(st, ctx->hev[0], 0));
    if (!per_sig) {
      const uint32_t salt[2] = {(uint32_t)salt64, (uint32_t)(salt64 >> 32)};
      launch_keys(st, N, ctx->vk, s.table, T - 1, salt, ctx->key_grouping == 3, s.slot_key, s.key_slot, s.key_rep,
                  s.key_index, s.key_acc, s.flags);
    }
    LK(hipEventRecord(s.ev_keys, st));
    LK(hipStreamWaitEvent(st2, s.ev_keys, 0));
    launch_decompress_range(st2, N, 0, 0, key_lanes(ctx, n, per_sig), ctx->sig, ctx->vk, s.key_rep, per_sig, s.pts,
                            s.itembad + s.cap_n, s.keybad, s.flags, kc, split);
    for (int c = 0; c < nchunks; ++c) {
      const size_t c0 = cb[c], cnt = cb[c + 1] - cb[c];
      if (!gate.wait(c + 2)) return;
      hipEvent_t ev = ctx->hev[c + 1];
      LK(hipStreamWaitEvent(st2, ev, 0));
      launch_decompress_range(st2, N, (uint32_t)c0, (uint32_t)cnt, 0, ctx->sig, ctx->vk, s.key_rep, per_sig, s.pts,
                              s.itembad + s.cap_n, s.keybad, s.flags, kc, split);
      LK(hipStreamWaitEvent(st, ev, 0));
      if (!one_copier) {
        if (!gate2.wait(c + 1)) return;
        LK(hipStreamWaitEvent(st, ctx->hev2[c], 0));
      }
      if (!k)
        launch_challenge(st, (uint32_t)cnt, ctx->vk + c0 * 32, ctx->sig + c0 * 64, ctx->msg, ctx->off + c0,
                         s.k + c0 * 8);
      launch_coef_range(st, N, (uint32_t)c0, (uint32_t)cnt, ctx->sig, s.k, z ? ctx->zexp : nullptr, seed, 0,
                        s.key_index, s.scal, s.key_acc, s.u_acc, s.itembad, s.flags, per_sig, s.coef_part, split);
    }
    LK(hipEventRecord(s.ev_dec, st2));
    launch_coef_finish(st, N, s.key_acc, s.u_acc, s.scal, s.flags, per_sig, s.coef_part, split);
    launch_msm_bin(st, P, batch_terms(P, s, N, split), split ? 2 + 3 * N : 1 + 2 * N, s.counts, s.offsets, s.cursor,
                   s.entries, s.flags, true);
    launch_msm_sort(st, P, s.counts, s.offsets, s.entries, s.sorted, s.bucket_end, s.buckets);
    LK(hipStreamWaitEvent(st, s.ev_dec, 0));
    launch_msm_bucket(st, P, s.counts, s.offsets, s.entries, s.sorted, s.bucket_end, s.pts, s.buckets, s.heads,
                      s.slice_W, s.slice_T, 0, nullptr, nullptr, true);
    launch_msm_tail(st, P, s.slice_W, s.slice_T, s.win, s.flags, want_compress, s.d_out, s.h_out);
    LK(hipGetLastError());
#undef LK
  });

  // the k / message chunks (second copying thread, or this one after each signature chunk)
  auto copy_second = [&](int c, hipStream_t str, hipEvent_t ev, std::string& err) -> int {
    const size_t c0 = cb[c], cnt = cb[c + 1] - cb[c];
    hipError_t e = hipSuccess;
    if (k) {
      e = hipMemcpyAsync(s.k + c0 * 8, k + c0 * 32, cnt * 32, hipMemcpyHostToDevice, str);
    } else {
      const size_t b0 = (size_t)(msg_off[c0] - msg_off[0]), b1 = (size_t)(msg_off[c0 + cnt] - msg_off[0]);
      if (b1 > b0) e = hipMemcpyAsync(ctx->msg + b0, msg + msg_off[c0], b1 - b0, hipMemcpyHostToDevice, str);
    }
    if (e == hipSuccess && ev) e = hipEventRecord(ev, str);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      err = std::string("host chunk copy: ") + hipGetErrorString(e);
      return EDC_ERR_HIP;
    }
    return 0;
  };
  std::string err2;
  int rc2 = 0;
  std::thread copier2;
  if (!one_copier)
    copier2 = std::thread([&] {
      if (hipSetDevice(ctx->device) != hipSuccess) { rc2 = EDC_ERR_HIP; gate2.stop(); return; }
      for (int c = 0; c < nchunks; ++c) {
        if ((rc2 = copy_second(c, ctx->hcs2, ctx->hev2[c], err2))) { gate2.stop(); return; }
        gate2.post(c + 1);
      }
    });
  // this thread: the copies, back to back, one event per piece
  auto copies = [&]() -> int {
    CK(hipMemcpyAsync(ctx->vk, vk, n * 32, hipMemcpyHostToDevice, cs));
    if (!k)
      CK(hipMemcpyAsync(ctx->off, rebased.empty() ? msg_off : rebased.data(), (n + 1) * sizeof(uint64_t),
                        hipMemcpyHostToDevice, cs));
    if (z) CK(hipMemcpyAsync(ctx->zexp, z, n * 16, hipMemcpyHostToDevice, cs));
    CK(hipEventRecord(ctx->hev[0], cs));
    gate.post(1);
    for (int c = 0; c < nchunks; ++c) {
      const size_t c0 = cb[c], cnt = cb[c + 1] - cb[c];
      CK(hipMemcpyAsync(ctx->sig + c0 * 64, sig + c0 * 64, cnt * 64, hipMemcpyHostToDevice, cs));
      if (one_copier) {
        std::string e1;
        if (int r = copy_second(c, cs, nullptr, e1)) { ctx->err = e1; return r; }
      }
      CK(hipEventRecord(ctx->hev[c + 1], cs));
      gate.post(c + 2);
    }
    return 0;
  };
  rc = copies();
  if (rc) { gate.stop(); gate2.stop(); }
  if (copier2.joinable()) copier2.join();
  if (rc2) gate.stop();
  launcher.join();
  if (rc) return rc;
  if (rc2) { ctx->err = err2; return rc2; }
  if (lrc) { ctx->err = lerr; return lrc; }
  s.acc_nbin = P.nbin();
  s.pending = true;
  return 0;
}

// One synchronous batch from host buffers, chunked when it pays (see above), else staged in one
// piece and run by run_batch_sync.
static int run_host_sync(edc_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg,
                         const uint64_t* msg_off, const uint8_t* k, const uint8_t* z, const uint8_t* z_seed,
                         uint8_t check8[32]) {
  Slot& s = ctx->slot[0];
  if (s.pending) { ctx->err = "slot 0 busy: wait for submitted batches first"; return EDC_ERR_ARG; }
  if (n && (!vk || !sig || (k ? false : !msg_off))) { ctx->err = "null input"; return EDC_ERR_ARG; }
  if (n && !k && msg_off[n] > msg_off[0] && !msg) { ctx->err = "null msg"; return EDC_ERR_ARG; }
  if (!host_chunked_ok(ctx, n)) {
    int rc = init_slot(ctx, s);
    if (rc) return rc;
    if (k) {
      if ((rc = ensure_n(ctx, n)) || (rc = ensure_slot(ctx, s, n))) return rc;
      if (n) {
        CK(hipMemcpyAsync(ctx->vk, vk, n * 32, hipMemcpyHostToDevice, ctx->st()));
        CK(hipMemcpyAsync(ctx->sig, sig, n * 64, hipMemcpyHostToDevice, ctx->st()));
        CK(hipMemcpyAsync(s.k, k, n * 32, hipMemcpyHostToDevice, ctx->st()));
      }
    } else if ((rc = upload(ctx, n, vk, sig, msg, msg_off))) {
      return rc;
    }
    if (z && n) CK(hipMemcpyAsync(ctx->zexp, z, n * 16, hipMemcpyHostToDevice, ctx->st()));
    return run_batch_sync(ctx, n, ctx->vk, ctx->sig, k ? nullptr : ctx->msg, k ? nullptr : ctx->off,
                          z ? nullptr : z_seed, 0, z ? ctx->zexp : nullptr, check8, nullptr, nullptr, k ? s.k : nullptr);
  }
  std::vector<uint64_t> rebased;
  const int rc = enqueue_host_chunked(ctx, n, vk, sig, msg, msg_off, k, z, z_seed, check8 != nullptr, rebased);
  if (rc) {     // nothing may still read the staging buffers or the caller's memory
    (void)hipStreamSynchronize(ctx->hcs);
    (void)hipStreamSynchronize(ctx->hcs2);
    (void)hipStreamSynchronize(s.st2);
    (void)hipStreamSynchronize(s.st);
    s.pending = false;
    return rc;
  }
  return finish_batch(ctx, s, check8, nullptr, nullptr);
}

extern "C" {

int edc_device_count(void) {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) return EDC_ERR_HIP;
  return c;
}

edc_ctx* edc_create(int device) {
  edc_ctx* ctx = new edc_ctx();
  ctx->device = device;
  {
    std::random_device rd;   // OS randomness: the key-grouping hash secret of this context
    ctx->secret = ((uint64_t)rd() << 32) ^ (uint64_t)rd();
    const uint64_t ks = splitmix64(ctx->secret ^ 0x6B657963616368ull);   // key-cache table hash key
    ctx->kc_s0 = (uint32_t)ks;
    ctx->kc_s1 = (uint32_t)(ks >> 32);
  }
  (void)hipGetLastError();   // launch checks below must not see an earlier, unrelated failure
  bool ok = hipSetDevice(device) == hipSuccess && msm_init_device() == hipSuccess && init_slot(ctx, ctx->slot[0]) == 0 &&
            dalloc(&ctx->btab, BTAB_TOTAL * NIELS_WORDS) == hipSuccess;
  if (ok) {
    launch_init_btable(ctx->st(), ctx->btab);
    ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(ctx->st()) == hipSuccess;
  }
  if (!ok) {
    (void)hipGetLastError();
    edc_destroy(ctx);
    (void)hipGetLastError();
    return nullptr;
  }
  return ctx;
}

static void free_keycache(edc_ctx* ctx) {
  void* ptrs[] = {ctx->kc_table, ctx->kc_keys, ctx->kc_comb, ctx->kc_ok, ctx->kc_reg};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  ctx->kc_table = ctx->kc_keys = ctx->kc_comb = ctx->kc_reg = nullptr;
  ctx->kc_reg_m = 0;
  ctx->kc_ok = nullptr;
  ctx->kc_m = ctx->kc_tmask = ctx->kc_cap = 0;
  ctx->kc_words.clear();
  ctx->kc_okh.clear();
}

static int sync_all(edc_ctx* ctx) {
  for (Slot& s : ctx->slot)
    if (s.st) CK(hipStreamSynchronize(s.st));
  return 0;
}

void edc_destroy(edc_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  (void)sync_all(ctx);
  free_keycache(ctx);
  if (ctx->bcomb) (void)hipFree(ctx->bcomb);
  for (Slot& s : ctx->slot) {
    if (s.st) (void)hipStreamSynchronize(s.st);
    free_slot_buffers(s);
    {
      void* in[] = {s.in_vk, s.in_sig, s.in_msg, s.in_off, s.in_idx};
      for (void* p : in)
        if (p) (void)hipFree(p);
    }
    {
      void* mb[] = {s.mb_acc, s.mb_xpt, s.mb_xrg, s.mb_xscal, s.mb_bad};
      for (void* p : mb)
        if (p) (void)hipFree(p);
    }
    if (s.flags) (void)hipFree(s.flags);
    if (s.d_out) (void)hipFree(s.d_out);
    if (s.h_out) (void)hipHostFree(s.h_out);
    if (s.h_acc) (void)hipHostFree(s.h_acc);
    for (int p = 0; p <= PH_N; ++p)
      if (s.ev[p]) (void)hipEventDestroy(s.ev[p]);
    for (hipEvent_t e : s.ev_acc)
      if (e) (void)hipEventDestroy(e);
    if (s.st) (void)hipStreamDestroy(s.st);
    if (s.st2) (void)hipStreamDestroy(s.st2);
    if (s.ev_keys) (void)hipEventDestroy(s.ev_keys);
    if (s.ev_dec) (void)hipEventDestroy(s.ev_dec);
  }
  {
    Slot& s = ctx->comb;
    if (s.st) (void)hipStreamSynchronize(s.st);
    if (s.flags) (void)hipFree(s.flags);
    if (s.d_out) (void)hipFree(s.d_out);
    if (s.h_out) (void)hipHostFree(s.h_out);
    if (s.h_acc) (void)hipHostFree(s.h_acc);
    for (int p = 0; p <= PH_N; ++p)
      if (s.ev[p]) (void)hipEventDestroy(s.ev[p]);
    for (hipEvent_t e : s.ev_acc)
      if (e) (void)hipEventDestroy(e);
    if (s.st) (void)hipStreamDestroy(s.st);
  }
  if (ctx->hcs) (void)hipStreamSynchronize(ctx->hcs);
  if (ctx->hcs2) (void)hipStreamSynchronize(ctx->hcs2);
  for (hipEvent_t e : ctx->hev)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : ctx->hev2)
    if (e) (void)hipEventDestroy(e);
  if (ctx->hcs) (void)hipStreamDestroy(ctx->hcs);
  if (ctx->hcs2) (void)hipStreamDestroy(ctx->hcs2);
  void* ptrs[] = {ctx->vk, ctx->sig, ctx->msg, ctx->zexp, ctx->off, ctx->kbuf, ctx->verdicts, ctx->vtab, ctx->aux,
                  ctx->btab, ctx->comb_in, ctx->fb_xpt, ctx->fb_xrg, ctx->fb_xscal, ctx->fb_rv, ctx->fb_idx,
                  ctx->fb_g};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  delete ctx;
}

const char* edc_last_error(const edc_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int edc_batch_verify(edc_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg,
                     const uint64_t* msg_off, const uint8_t z_seed[32], uint8_t check8[32]) {
  if (!ctx || !z_seed) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  return run_host_sync(ctx, n, vk, sig, msg, msg_off, nullptr, nullptr, z_seed, check8);
}

int edc_batch_verify_z(edc_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg,
                       const uint64_t* msg_off, const uint8_t* z, uint8_t check8[32]) {
  if (!ctx || (n && !z)) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  return run_host_sync(ctx, n, vk, sig, msg, msg_off, nullptr, n ? z : nullptr, nullptr, check8);
}

int edc_batch_verify_device(edc_ctx* ctx, size_t n, const uint8_t* d_vk, const uint8_t* d_sig,
                            const uint8_t* d_msg, const uint64_t* d_msg_off, const uint8_t z_seed[32],
                            uint64_t z_base, const uint8_t* d_z, uint8_t check8[32]) {
  if (!ctx || (!z_seed && !d_z)) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  return run_batch_sync(ctx, n, d_vk, d_sig, d_msg, d_msg_off, z_seed, z_base, d_z, check8, nullptr, nullptr);
}

int64_t edc_batch_submit_device(edc_ctx* ctx, size_t n, const uint8_t* d_vk, const uint8_t* d_sig,
                                const uint8_t* d_msg, const uint64_t* d_msg_off, const uint8_t z_seed[32],
                                uint64_t z_base, const uint8_t* d_z, int want_check8) {
  if (!ctx || (!z_seed && !d_z)) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  const int64_t ticket = ctx->next_ticket;
  Slot& s = ctx->slot[ticket % ctx->nslots];
  if (s.pending) { ctx->err = "all slots in flight: wait for the oldest ticket first"; return EDC_ERR_ARG; }
#ifdef EDC_BATCH_STAMPS
  s.t_submit_us = host_us();
#endif
  int rc = enqueue_batch(ctx, s, n, d_vk, d_sig, d_msg, d_msg_off, z_seed, z_base, d_z, want_check8 != 0);
  if (rc) return rc;
  s.ticket = ticket;
  ctx->next_ticket++;
  return ticket;
}

int64_t edc_batch_submit(edc_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg,
                         const uint64_t* msg_off, const uint8_t z_seed[32], uint64_t z_base, int want_check8) {
  if (!ctx || !z_seed) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  const int64_t ticket = ctx->next_ticket;
  Slot& s = ctx->slot[ticket % ctx->nslots];
  if (s.pending) { ctx->err = "all slots in flight: wait for the oldest ticket first"; return EDC_ERR_ARG; }
  int rc = upload_slot(ctx, s, n, vk, sig, msg, msg_off);
  if (rc) return rc;
  rc = enqueue_batch(ctx, s, n, s.in_vk, s.in_sig, s.in_msg, s.in_off, z_seed, z_base, nullptr, want_check8 != 0);
  if (rc) return rc;
  s.ticket = ticket;
  ctx->next_ticket++;
  return ticket;
}

int64_t edc_batch_submit_indexed(edc_ctx* ctx, size_t n, const uint32_t* key_idx, const uint8_t* sig,
                                 const uint8_t* msg, const uint64_t* msg_off, const uint8_t z_seed[32],
                                 uint64_t z_base, int want_check8) {
  if (!ctx || !z_seed || (n && !key_idx)) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  uint32_t mx = 0;
  for (size_t i = 0; i < n; ++i) mx = key_idx[i] > mx ? key_idx[i] : mx;
  if (n && mx >= ctx->kc_reg_m) { ctx->err = "key index outside the registered key list"; return EDC_ERR_ARG; }
  const int64_t ticket = ctx->next_ticket;
  Slot& s = ctx->slot[ticket % ctx->nslots];
  if (s.pending) { ctx->err = "all slots in flight: wait for the oldest ticket first"; return EDC_ERR_ARG; }
  int rc = upload_slot(ctx, s, n, nullptr, sig, msg, msg_off, key_idx);
  if (rc) return rc;
  rc = enqueue_batch(ctx, s, n, s.in_vk, s.in_sig, s.in_msg, s.in_off, z_seed, z_base, nullptr, want_check8 != 0);
  if (rc) return rc;
  s.ticket = ticket;
  ctx->next_ticket++;
  return ticket;
}

int edc_batch_wait(edc_ctx* ctx, int64_t ticket, uint8_t check8[32], uint8_t partial[128], int* bad) {
  if (!ctx || ticket < 0) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  Slot& s = ctx->slot[ticket % ctx->nslots];
  if (!s.pending || s.ticket != ticket) { ctx->err = "unknown or already-waited ticket"; return EDC_ERR_ARG; }
  return finish_batch(ctx, s, check8, partial, bad);
}

int64_t edc_batch_submit_multi_device(edc_ctx* ctx, size_t nb, size_t n_per, const uint8_t* d_vk, const uint8_t* d_sig,
                                      const uint8_t* d_msg, const uint64_t* d_msg_off, const uint8_t* d_k,
                                      const uint8_t z_seed[32], uint64_t z_base, int want_check8) {
  if (!ctx || !z_seed) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  const int64_t ticket = ctx->next_ticket;
  Slot& s = ctx->slot[ticket % ctx->nslots];
  if (s.pending) { ctx->err = "all slots in flight: wait for the oldest ticket first"; return EDC_ERR_ARG; }
  const uint32_t nbv = (uint32_t)(nb <= kMultiMax ? nb : 0);
  const uint32_t* dk = reinterpret_cast<const uint32_t*>(d_k);
  int rc;
  if (ctx->multi_union) {        // one batch over all items first (finish_multi)
    rc = multi_args(ctx, nbv, n_per, d_vk, d_sig, d_msg, d_msg_off, dk);
    if (!rc) rc = enqueue_batch(ctx, s, (size_t)nbv * n_per, d_vk, d_sig, d_msg, d_msg_off, z_seed, z_base, nullptr, 0, dk);
    if (rc) return rc;
    s.nmulti = nbv;
    s.mu_union = true;
    s.mu_nper = n_per;
    s.mu_vk = d_vk;
    s.mu_sig = d_sig;
    s.mu_msg = d_msg;
    s.mu_off = d_msg_off;
    s.mu_k = dk;
    memcpy(s.mu_seed, z_seed, 32);
    s.mu_zbase = z_base;
    s.mu_compress = want_check8 != 0;
  } else {
    rc = enqueue_multi(ctx, s, nbv, n_per, d_vk, d_sig, d_msg, d_msg_off, dk, z_seed, z_base, want_check8 != 0);
    if (rc) return rc;
    s.mu_union = false;
  }
  s.ticket = ticket;
  ctx->next_ticket++;
  return ticket;
}

int edc_batch_wait_multi(edc_ctx* ctx, int64_t ticket, size_t nb, int* verdicts, uint8_t* check8, uint8_t* partials,
                         int* bad) {
  if (!ctx || ticket < 0) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  Slot& s = ctx->slot[ticket % ctx->nslots];
  if (!s.pending || s.ticket != ticket) { ctx->err = "unknown or already-waited ticket"; return EDC_ERR_ARG; }
  return finish_multi(ctx, s, nb, verdicts, check8, partials, bad);
}

int edc_set_multi_union(edc_ctx* ctx, int on) {
  if (!ctx) return EDC_ERR_ARG;
  ctx->multi_union = on ? 1 : 0;
  return 0;
}

int edc_multi_union_stats(const edc_ctx* ctx, uint64_t* passed, uint64_t* rerun) {
  if (!ctx) return EDC_ERR_ARG;
  if (passed) *passed = ctx->mu_hits;
  if (rerun) *rerun = ctx->mu_reruns;
  return 0;
}

int edc_batch_partial_device(edc_ctx* ctx, size_t n, const uint8_t* d_vk, const uint8_t* d_sig,
                             const uint8_t* d_msg, const uint64_t* d_msg_off, const uint8_t z_seed[32],
                             uint64_t z_base, const uint8_t* d_z, uint8_t partial[128], int* bad) {
  if (!ctx || !partial || (!z_seed && !d_z)) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  int rc = run_batch_sync(ctx, n, d_vk, d_sig, d_msg, d_msg_off, z_seed, z_base, d_z, nullptr, partial, bad);
  return rc < 0 ? rc : 0;
}

// sum of g canonical partial points on the combine stream -> verdict of [8]*sum == 0 (with the
// bad flag), optional compressed check8 and canonical sum
static int combine_points(edc_ctx* ctx, size_t g, const uint8_t* partials, int bad, uint8_t check8[32],
                          uint8_t sum[128]) {
  Slot& s = ctx->comb;
  int rc = init_slot(ctx, s);
  if (rc) return rc;
  if (g * 128 > ctx->comb_cap) {
    if (ctx->comb_in) (void)hipFree(ctx->comb_in);
    ctx->comb_cap = 0;
    CK(dalloc(&ctx->comb_in, g * 128 + 1024));
    ctx->comb_cap = g * 128 + 1024;
  }
  if (g) CK(hipMemcpyAsync(ctx->comb_in, partials, g * 128, hipMemcpyHostToDevice, s.st));
  CK(hipMemsetAsync(s.d_out, 0, 256, s.st));
  launch_combine(s.st, (uint32_t)g, ctx->comb_in, bad ? 1 : 0, check8 != nullptr, s.d_out);
  CK(hipGetLastError());
  CK(hipMemcpyAsync(s.h_out, s.d_out, 256, hipMemcpyDeviceToHost, s.st));
  s.pending = true;
  s.timed = false;
  return finish_batch(ctx, s, check8, sum, nullptr);
}

int edc_combine_partials(edc_ctx* ctx, size_t g, const uint8_t* partials, int bad_any, uint8_t check8[32]) {
  if (!ctx || (g && !partials)) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  return combine_points(ctx, g, partials, bad_any, check8, nullptr);
}

int edc_debug_sc_reduce_wide(edc_ctx* ctx, size_t n, const uint8_t* d_in, uint8_t* d_out) {
  if (!ctx || (n && (!d_in || !d_out)) || n > (1u << 24)) return EDC_ERR_ARG;
  if (n && (!aligned16(d_in) || !aligned16(d_out))) {
    ctx->err = "device buffers must be 16-byte aligned";
    return EDC_ERR_ARG;
  }
  CK(hipSetDevice(ctx->device));
  Slot& s = ctx->slot[0];
  launch_sc_reduce_wide(s.st, (uint32_t)n, reinterpret_cast<const uint32_t*>(d_in), reinterpret_cast<uint32_t*>(d_out));
  CK(hipGetLastError());
  CK(hipStreamSynchronize(s.st));
  return 0;
}

int edc_combine_records_device(edc_ctx* ctx, void* stream, size_t g, const uint8_t* d_records, size_t stride,
                               uint8_t* d_out) {
  if (!ctx || !d_out || (g && !d_records) || stride < 129 || g > 4096) return EDC_ERR_ARG;
  if (!aligned16(d_out)) { ctx->err = "d_out must be 16-byte aligned"; return EDC_ERR_ARG; }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (st) {     // the caller's stream must belong to the context's GPU
    int sdev = -1;
    CK(hipStreamGetDevice(st, &sdev));
    if (sdev != ctx->device) { ctx->err = "stream is not on the context's device"; return EDC_ERR_ARG; }
  }
  // the launch needs the context's device current; the caller's current device is restored
  int prev = -1;
  CK(hipGetDevice(&prev));
  CK(hipSetDevice(ctx->device));
  launch_combine_records(st, (uint32_t)g, d_records, (uint32_t)stride, d_out);
  const hipError_t e = hipGetLastError();
  (void)hipSetDevice(prev);
  CK(e);
  return 0;
}

int edc_challenge(edc_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg,
                  const uint64_t* msg_off, uint8_t* k_out) {
  if (!ctx || (n && !k_out)) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  int rc = upload(ctx, n, vk, sig, msg, msg_off);
  if (rc) return rc;
  if (!n) return 0;
  launch_challenge(ctx->st(), (uint32_t)n, ctx->vk, ctx->sig, ctx->msg, ctx->off, ctx->kbuf);
  CK(hipGetLastError());
  CK(hipMemcpyAsync(k_out, ctx->kbuf, n * 32, hipMemcpyDeviceToHost, ctx->st()));
  CK(hipStreamSynchronize(ctx->st()));
  return 0;
}

int edc_verify_prehashed_each(edc_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* k,
                              uint8_t* verdicts) {
  if (!ctx || (n && (!vk || !sig || !k || !verdicts))) return EDC_ERR_ARG;
  for (size_t i = 0; i < n; ++i) {        // Scalar::from_hash never yields k >= l (batch paths: FLAG_KARG)
    uint32_t w[8];
    memcpy(w, k + 32 * i, 32);
    if (!sc_is_canonical(w)) { ctx->err = "prehashed k is not a canonical scalar"; return EDC_ERR_ARG; }
  }
  CK(hipSetDevice(ctx->device));
  int rc = ensure_n(ctx, n);
  if (rc) return rc;
  if (!n) return 0;
  hipStream_t st = ctx->st();
  CK(hipMemcpyAsync(ctx->vk, vk, n * 32, hipMemcpyHostToDevice, st));
  CK(hipMemcpyAsync(ctx->sig, sig, n * 64, hipMemcpyHostToDevice, st));
  CK(hipMemcpyAsync(ctx->kbuf, k, n * 32, hipMemcpyHostToDevice, st));
  launch_verify_single(st, (uint32_t)n, ctx->vk, ctx->sig, ctx->kbuf, ctx->btab, ctx->vtab, ctx->verdicts,
                       ctx->kc(), ctx->bcomb);
  CK(hipGetLastError());
  CK(hipMemcpyAsync(verdicts, ctx->verdicts, n, hipMemcpyDeviceToHost, st));
  CK(hipStreamSynchronize(st));
  return 0;
}

int edc_verify_each(edc_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg,
                    const uint64_t* msg_off, uint8_t* verdicts) {
  if (!ctx || (n && !verdicts)) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  int rc = upload(ctx, n, vk, sig, msg, msg_off);
  if (rc) return rc;
  if (!n) return 0;
  hipStream_t st = ctx->st();
  launch_challenge(st, (uint32_t)n, ctx->vk, ctx->sig, ctx->msg, ctx->off, ctx->kbuf);
  launch_verify_single(st, (uint32_t)n, ctx->vk, ctx->sig, ctx->kbuf, ctx->btab, ctx->vtab, ctx->verdicts,
                       ctx->kc(), ctx->bcomb);
  CK(hipGetLastError());
  CK(hipMemcpyAsync(verdicts, ctx->verdicts, n, hipMemcpyDeviceToHost, st));
  CK(hipStreamSynchronize(st));
  return 0;
}

int edc_verify_each_device(edc_ctx* ctx, size_t n, const uint8_t* d_vk, const uint8_t* d_sig, const uint8_t* d_msg,
                           const uint64_t* d_msg_off, uint8_t* d_verdicts) {
  if (!ctx || (n && (!d_vk || !d_sig || !d_msg_off || !d_verdicts))) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  int rc = ensure_n(ctx, n);
  if (rc) return rc;
  if (!n) return 0;
  hipStream_t st = ctx->st();
  launch_challenge(st, (uint32_t)n, d_vk, d_sig, d_msg, d_msg_off, ctx->kbuf);
  launch_verify_single(st, (uint32_t)n, d_vk, d_sig, ctx->kbuf, ctx->btab, ctx->vtab, d_verdicts,
                       ctx->kc(), ctx->bcomb);
  CK(hipGetLastError());
  CK(hipStreamSynchronize(st));
  return 0;
}

// ---- grouped fallback: one MSM pass over ~128 contiguous ranges (edc_set_fallback_shape) ----
static int ensure_fb(edc_ctx* ctx, size_t terms, size_t ranges) {
  if (terms > ctx->fb_cap_terms || !ctx->fb_xpt) {
    CK(hipStreamSynchronize(ctx->st()));
    for (void* p : {(void*)ctx->fb_xpt, (void*)ctx->fb_xrg, (void*)ctx->fb_xscal})
      if (p) (void)hipFree(p);
    ctx->fb_xpt = ctx->fb_xrg = ctx->fb_xscal = nullptr;
    ctx->fb_cap_terms = 0;
    const size_t cap = terms + terms / 8 + 64;
    CK(dalloc(&ctx->fb_xpt, cap));
    CK(dalloc(&ctx->fb_xrg, cap));
    CK(dalloc(&ctx->fb_xscal, cap * 8));
    ctx->fb_cap_terms = cap;
  }
  if (ranges > ctx->fb_cap_ranges || !ctx->fb_rv) {
    CK(hipStreamSynchronize(ctx->st()));
    if (ctx->fb_rv) (void)hipFree(ctx->fb_rv);
    ctx->fb_rv = nullptr;
    CK(dalloc(&ctx->fb_rv, 2 * ranges + 64));
    ctx->fb_cap_ranges = ranges;
  }
  return 0;
}

// Item::verify_single (src/batch.rs:104-107) for the listed items, with the batch's queue-time k
// (slot s): gathered into the staging buffers, one per-item launch, codes scattered into verdicts.
static int verify_listed(edc_ctx* ctx, Slot& s, const std::vector<uint32_t>& idx, const uint8_t* d_vk,
                         const uint8_t* d_sig, uint8_t* verdicts, int* invalid) {
  const size_t c = idx.size();
  if (!c) return 0;
  int rc = ensure_n(ctx, c);
  if (rc) return rc;
  if (c > ctx->fb_cap_idx || !ctx->fb_idx) {
    if (ctx->fb_idx) (void)hipFree(ctx->fb_idx);
    ctx->fb_idx = nullptr;
    CK(dalloc(&ctx->fb_idx, c + c / 8 + 64));
    ctx->fb_cap_idx = c + c / 8 + 64;
  }
  // gathered copies in their own buffer: the inputs may BE the context's staging buffers (host
  // entry points), and an in-place gather would race (item idx[j] > j is read while slot idx[j]
  // is written by another lane)
  if (c > ctx->fb_cap_g || !ctx->fb_g) {
    if (ctx->fb_g) (void)hipFree(ctx->fb_g);
    ctx->fb_g = nullptr;
    ctx->fb_cap_g = 0;
    CK(dalloc(&ctx->fb_g, (c + c / 8 + 64) * 128));
    ctx->fb_cap_g = c + c / 8 + 64;
  }
  uint8_t* g_vk = ctx->fb_g;
  uint8_t* g_sig = g_vk + ctx->fb_cap_g * 32;
  uint32_t* g_k = reinterpret_cast<uint32_t*>(g_sig + ctx->fb_cap_g * 64);
  hipStream_t st = s.st;
  CK(hipMemcpyAsync(ctx->fb_idx, idx.data(), c * sizeof(uint32_t), hipMemcpyHostToDevice, st));
  launch_gather_items(st, (uint32_t)c, ctx->fb_idx, d_vk, d_sig, s.kin, g_vk, g_sig, g_k);
  if (c <= kQuadVerifyMax)   // latency-bound: one quad of lanes per item
    launch_verify_quad(st, (uint32_t)c, g_vk, g_sig, g_k, ctx->btab, ctx->verdicts, ctx->kc(), ctx->bcomb);
  else
    launch_verify_single(st, (uint32_t)c, g_vk, g_sig, g_k, ctx->btab, ctx->vtab, ctx->verdicts, ctx->kc(),
                         ctx->bcomb);
  CK(hipGetLastError());
  std::vector<uint8_t> v(c);
  CK(hipMemcpyAsync(v.data(), ctx->verdicts, c, hipMemcpyDeviceToHost, st));
  CK(hipStreamSynchronize(st));
  for (size_t j = 0; j < c; ++j) {
    verdicts[idx[j]] = v[j];
    *invalid += v[j] != 0;
  }
  return 0;
}

// After a failed batch on slot s (its k, decoded points, key grouping and per-item failure bits
// still in place): the batch equation restricted to ~fb_ranges (default 32) contiguous ranges in
// ONE MSM pass (range-tagged bins, fb_bits = 9-bit windows by default), [8]P_g == 0 per range; ranges whose check fails or that
// hold an item with an undecodable R / key or a non-canonical s are verified item by item.
// Items of passing ranges are valid (ZIP215: batch == single, with a fresh secret z: see
// include/edc.h). verdicts (host, n bytes) receive Item::verify_single's code for every item.
static int fallback_ranges(edc_ctx* ctx, Slot& s, size_t n, const uint8_t* d_vk, const uint8_t* d_sig,
                           const uint8_t* d_msg, const uint64_t* d_off, const uint8_t* z_seed, uint64_t z_base,
                           bool per_sig, uint32_t m, uint8_t* verdicts) {
  memset(verdicts, 0, n);
  if (!n) return 0;
  // ~FB_RANGES ranges: each range-window bin then holds enough digits to amortize its fixed
  // 256-bucket reduction, and a failing range costs no more than a small one in the per-item pass
  // (that pass is latency-bound: one lane per item)
  // the range count is capped so that the range-tagged plan fits MSM_MAX_BINS (G * bins per range)
  const uint32_t bpr = make_plan(ctx->fb_bits, ctx->fb_bits, 1).bins_per_range;
  const uint32_t gmax = MSM_MAX_BINS / bpr;
  const uint32_t granges = ctx->fb_ranges < gmax ? ctx->fb_ranges : gmax;
  const size_t target = (n + granges - 1) / granges;
  const size_t rsize = (target + COEF_CHUNK - 1) / COEF_CHUNK * COEF_CHUNK;
  const uint32_t G = (uint32_t)((n + rsize - 1) / rsize);
  if (!per_sig && (size_t)G * m > s.cap_n) {
    // too many distinct keys for per-(range, key) sums: redo the prefix with one key term per
    // signature (the same group element)
    // (s.kin already holds this batch's k: computed by the first prefix or the caller's)
    int rc = enqueue_prefix(ctx, s, n, d_vk, d_sig, d_msg, d_off, z_seed, z_base, nullptr, false, nullptr, true, false,
                            s.kin);
    if (rc) return rc;
    CK(hipStreamSynchronize(s.st));
    per_sig = true;
  }
  const MsmPlan P = make_plan(ctx->fb_bits, ctx->fb_bits, G);
  const uint32_t mm = per_sig ? 0u : m;
  const size_t nx = (size_t)G * (mm + 1);
  const uint32_t npoint = (uint32_t)(per_sig ? 2 * n : n);
  int rc = ensure_msm(ctx, s, P, msm_entry_capacity(P, n, (per_sig ? n : 0) + nx));
  if (rc) return rc;
  rc = ensure_fb(ctx, nx, G);
  if (rc) return rc;
  uint32_t seed[8];
  seed_words(z_seed, seed);
  hipStream_t st = s.st;
  launch_range_coef(st, (uint32_t)n, (uint32_t)rsize, G, m, per_sig, d_sig, s.kin, nullptr, seed, z_base, s.key_index,
                    s.scal, s.key_acc, s.u_acc, s.flags, ctx->fb_xpt, ctx->fb_xrg, ctx->fb_xscal);
  const MsmTerms terms{(uint32_t)n, (uint32_t)rsize, npoint, (uint32_t)nx, 1, s.scal, ctx->fb_xpt, ctx->fb_xrg,
                       ctx->fb_xscal};
  launch_msm_bin(st, P, terms, npoint + (uint32_t)nx, s.counts, s.offsets, s.cursor, s.entries, s.flags);
  launch_msm_sort(st, P, s.counts, s.offsets, s.entries, s.sorted, s.bucket_end, s.buckets);
  launch_msm_bucket(st, P, s.counts, s.offsets, s.entries, s.sorted, s.bucket_end, s.pts, s.buckets, s.heads, s.slice_W,
                    s.slice_T);
  launch_msm_range_tail(st, P, s.slice_W, s.slice_T, s.win, ctx->fb_rv);
  CK(hipMemsetAsync(ctx->fb_rv + G, 0, G, st));
  launch_range_prebad(st, (uint32_t)n, (uint32_t)rsize, s.itembad, s.itembad + s.cap_n, s.keybad, s.key_index, per_sig,
                      ctx->fb_rv + G);
  CK(hipGetLastError());
  std::vector<uint8_t> rv(2 * (size_t)G);
  CK(hipMemcpyAsync(rv.data(), ctx->fb_rv, 2 * (size_t)G, hipMemcpyDeviceToHost, st));
  CK(hipStreamSynchronize(st));
  std::vector<uint32_t> idx;
  for (uint32_t g = 0; g < G; ++g)
    if (rv[g] || rv[G + g])
      for (size_t i = (size_t)g * rsize; i < n && i < (size_t)(g + 1) * rsize; ++i) idx.push_back((uint32_t)i);
  int invalid = 0;
  rc = verify_listed(ctx, s, idx, d_vk, d_sig, verdicts, &invalid);
  if (rc) return rc;
  return invalid;
}

// grouping state of the batch last enqueued on slot s (after it completed)
static int slot_grouping(edc_ctx* ctx, Slot& s, bool* per_sig, uint32_t* m) {
  int f[FLAG_COUNT];
  CK(hipMemcpy(f, s.flags, sizeof(f), hipMemcpyDeviceToHost));
  *per_sig = s.per_sig || f[FLAG_OVF] != 0;
  *m = (uint32_t)f[FLAG_NKEYS];
  return 0;
}

int edc_find_invalid_device(edc_ctx* ctx, size_t n, const uint8_t* d_vk, const uint8_t* d_sig,
                            const uint8_t* d_msg, const uint64_t* d_msg_off, const uint8_t z_seed[32],
                            size_t leaf, uint8_t* verdicts) {
  (void)leaf;
  if (!ctx || !z_seed || (n && (!d_vk || !d_sig || !d_msg_off || !verdicts))) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  Slot& s = ctx->slot[0];
  if (s.pending) { ctx->err = "slot 0 busy: wait for submitted batches first"; return EDC_ERR_ARG; }
  if (!n) return 0;
  int rc = enqueue_prefix(ctx, s, n, d_vk, d_sig, d_msg, d_msg_off, z_seed, 0, nullptr, false, nullptr);
  if (rc) return rc;
  CK(hipStreamSynchronize(s.st));
  bool per_sig;
  uint32_t m;
  rc = slot_grouping(ctx, s, &per_sig, &m);
  if (rc) return rc;
  return fallback_ranges(ctx, s, n, d_vk, d_sig, d_msg, d_msg_off, z_seed, 0, per_sig, m, verdicts);
}

}  // extern "C"

// batch on slot 0, then (on failure) the grouped fallback reusing its state; d_k: prehashed k
static int batch_with_fallback(edc_ctx* ctx, size_t n, const uint8_t* d_vk, const uint8_t* d_sig, const uint8_t* d_msg,
                               const uint64_t* d_msg_off, const uint32_t* d_k, const uint8_t* z_seed,
                               uint8_t* verdicts, int* n_invalid, uint8_t check8[32]) {
  if (n_invalid) *n_invalid = 0;
  int rc = run_batch_sync(ctx, n, d_vk, d_sig, d_msg, d_msg_off, z_seed, 0, nullptr, check8, nullptr, nullptr, d_k);
  if (rc <= 0) {
    if (rc == 0 && n) memset(verdicts, 0, n);
    return rc;
  }
  Slot& s = ctx->slot[0];
  bool per_sig;
  uint32_t m;
  int r2 = slot_grouping(ctx, s, &per_sig, &m);
  if (r2) return r2;
  r2 = fallback_ranges(ctx, s, n, d_vk, d_sig, d_msg, d_msg_off, z_seed, 0, per_sig, m, verdicts);
  if (r2 < 0) return r2;
  if (n_invalid) *n_invalid = r2;
  return EDC_INVALID_SIGNATURE;
}

extern "C" {

int edc_batch_verify_fallback_device(edc_ctx* ctx, size_t n, const uint8_t* d_vk, const uint8_t* d_sig,
                                     const uint8_t* d_msg, const uint64_t* d_msg_off, const uint8_t z_seed[32],
                                     uint8_t* verdicts, int* n_invalid, uint8_t check8[32]) {
  if (!ctx || !z_seed || (n && (!d_vk || !d_sig || !d_msg_off || !verdicts))) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  return batch_with_fallback(ctx, n, d_vk, d_sig, d_msg, d_msg_off, nullptr, z_seed, verdicts, n_invalid, check8);
}

// ---- prehashed items: the reference's batch::Item {vk_bytes, sig, k} (src/batch.rs:76-94) ----
int edc_batch_verify_prehashed(edc_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* k,
                               const uint8_t z_seed[32], const uint8_t* z, uint8_t check8[32]) {
  if (!ctx || (!z_seed && !z) || (n && (!vk || !sig || !k || (!z_seed && !z)))) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  if (!n) {     // empty batch: Ok through the one-piece path (no input is read)
    static const uint8_t none[1] = {0};
    return run_host_sync(ctx, 0, none, none, nullptr, nullptr, none, nullptr, z ? nullptr : z_seed, check8);
  }
  return run_host_sync(ctx, n, vk, sig, nullptr, nullptr, k, z, z_seed, check8);
}

int edc_batch_verify_prehashed_device(edc_ctx* ctx, size_t n, const uint8_t* d_vk, const uint8_t* d_sig,
                                      const uint8_t* d_k, const uint8_t z_seed[32], uint64_t z_base,
                                      const uint8_t* d_z, uint8_t check8[32]) {
  if (!ctx || (!z_seed && !d_z) || (n && (!d_vk || !d_sig || !d_k))) return EDC_ERR_ARG;
  if (!aligned16(d_k) || (d_z && !aligned16(d_z))) { ctx->err = "d_k / d_z must be 16-byte aligned"; return EDC_ERR_ARG; }
  CK(hipSetDevice(ctx->device));
  return run_batch_sync(ctx, n, d_vk, d_sig, nullptr, nullptr, z_seed, z_base, d_z, check8, nullptr, nullptr,
                        reinterpret_cast<const uint32_t*>(d_k));
}

int64_t edc_batch_submit_prehashed_indexed(edc_ctx* ctx, size_t n, const uint32_t* key_idx, const uint8_t* sig,
                                           const uint8_t* k, const uint8_t z_seed[32], uint64_t z_base,
                                           int want_check8) {
  if (!ctx || !z_seed || (n && !key_idx)) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  uint32_t mx = 0;
  for (size_t i = 0; i < n; ++i) mx = key_idx[i] > mx ? key_idx[i] : mx;
  if (n && mx >= ctx->kc_reg_m) { ctx->err = "key index outside the registered key list"; return EDC_ERR_ARG; }
  const int64_t ticket = ctx->next_ticket;
  Slot& s = ctx->slot[ticket % ctx->nslots];
  if (s.pending) { ctx->err = "all slots in flight: wait for the oldest ticket first"; return EDC_ERR_ARG; }
  int rc = upload_slot_prehashed(ctx, s, n, nullptr, sig, k, key_idx);
  if (rc) return rc;
  rc = enqueue_batch(ctx, s, n, s.in_vk, s.in_sig, nullptr, nullptr, z_seed, z_base, nullptr, want_check8 != 0, s.k);
  if (rc) return rc;
  s.ticket = ticket;
  ctx->next_ticket++;
  return ticket;
}

int64_t edc_batch_submit_prehashed(edc_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* k,
                                   const uint8_t z_seed[32], uint64_t z_base, int want_check8) {
  if (!ctx || !z_seed) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  const int64_t ticket = ctx->next_ticket;
  Slot& s = ctx->slot[ticket % ctx->nslots];
  if (s.pending) { ctx->err = "all slots in flight: wait for the oldest ticket first"; return EDC_ERR_ARG; }
  int rc = upload_slot_prehashed(ctx, s, n, vk, sig, k);
  if (rc) return rc;
  rc = enqueue_batch(ctx, s, n, s.in_vk, s.in_sig, nullptr, nullptr, z_seed, z_base, nullptr, want_check8 != 0, s.k);
  if (rc) return rc;
  s.ticket = ticket;
  ctx->next_ticket++;
  return ticket;
}

int64_t edc_batch_submit_prehashed_device(edc_ctx* ctx, size_t n, const uint8_t* d_vk, const uint8_t* d_sig,
                                          const uint8_t* d_k, const uint8_t z_seed[32], uint64_t z_base,
                                          const uint8_t* d_z, int want_check8) {
  if (!ctx || (!z_seed && !d_z) || (n && (!d_vk || !d_sig || !d_k))) return EDC_ERR_ARG;
  if (!aligned16(d_k) || (d_z && !aligned16(d_z))) { ctx->err = "d_k / d_z must be 16-byte aligned"; return EDC_ERR_ARG; }
  CK(hipSetDevice(ctx->device));
  const int64_t ticket = ctx->next_ticket;
  Slot& s = ctx->slot[ticket % ctx->nslots];
  if (s.pending) { ctx->err = "all slots in flight: wait for the oldest ticket first"; return EDC_ERR_ARG; }
  int rc = enqueue_batch(ctx, s, n, d_vk, d_sig, nullptr, nullptr, z_seed, z_base, d_z, want_check8 != 0,
                         reinterpret_cast<const uint32_t*>(d_k));
  if (rc) return rc;
  s.ticket = ticket;
  ctx->next_ticket++;
  return ticket;
}

int edc_batch_verify_prehashed_fallback(edc_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig,
                                        const uint8_t* k, const uint8_t z_seed[32], uint8_t* verdicts,
                                        int* n_invalid, uint8_t check8[32]) {
  if (!ctx || !z_seed || (n && (!vk || !sig || !k || !verdicts))) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  Slot& s = ctx->slot[0];
  if (s.pending) { ctx->err = "slot 0 busy: wait for submitted batches first"; return EDC_ERR_ARG; }
  int rc = ensure_n(ctx, n);
  if (rc) return rc;
  rc = ensure_slot(ctx, s, n);
  if (rc) return rc;
  if (n) {
    CK(hipMemcpyAsync(ctx->vk, vk, n * 32, hipMemcpyHostToDevice, ctx->st()));
    CK(hipMemcpyAsync(ctx->sig, sig, n * 64, hipMemcpyHostToDevice, ctx->st()));
    CK(hipMemcpyAsync(s.k, k, n * 32, hipMemcpyHostToDevice, ctx->st()));
  }
  return batch_with_fallback(ctx, n, ctx->vk, ctx->sig, nullptr, nullptr, s.k, z_seed, verdicts, n_invalid, check8);
}

int edc_batch_verify_prehashed_fallback_device(edc_ctx* ctx, size_t n, const uint8_t* d_vk, const uint8_t* d_sig,
                                               const uint8_t* d_k, const uint8_t z_seed[32], uint8_t* verdicts,
                                               int* n_invalid, uint8_t check8[32]) {
  if (!ctx || !z_seed || (n && (!d_vk || !d_sig || !d_k || !verdicts))) return EDC_ERR_ARG;
  if (!aligned16(d_k)) { ctx->err = "d_k must be 16-byte aligned"; return EDC_ERR_ARG; }
  CK(hipSetDevice(ctx->device));
  return batch_with_fallback(ctx, n, d_vk, d_sig, nullptr, nullptr, reinterpret_cast<const uint32_t*>(d_k), z_seed,
                             verdicts, n_invalid, check8);
}

int edc_decompress(edc_ctx* ctx, size_t n, const uint8_t* enc, uint8_t* xy, uint8_t* ok) {
  if (!ctx || (n && (!enc || !xy || !ok))) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  int rc = ensure_n(ctx, n);
  if (rc) return rc;
  rc = ensure_aux(ctx, n * 64);
  if (rc) return rc;
  if (!n) return 0;
  hipStream_t st = ctx->st();
  CK(hipMemcpyAsync(ctx->vk, enc, n * 32, hipMemcpyHostToDevice, st));
  launch_decode(st, (uint32_t)n, ctx->vk, ctx->aux, ctx->verdicts);
  CK(hipGetLastError());
  CK(hipMemcpyAsync(xy, ctx->aux, n * 64, hipMemcpyDeviceToHost, st));
  CK(hipMemcpyAsync(ok, ctx->verdicts, n, hipMemcpyDeviceToHost, st));
  CK(hipStreamSynchronize(st));
  return 0;
}

int edc_vk_validate(edc_ctx* ctx, size_t n, const uint8_t* vk, uint8_t* codes) {
  if (!ctx || (n && (!vk || !codes))) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  int rc = ensure_n(ctx, n);
  if (rc) return rc;
  if (!n) return 0;
  hipStream_t st = ctx->st();
  CK(hipMemcpyAsync(ctx->vk, vk, n * 32, hipMemcpyHostToDevice, st));
  launch_vk_validate(st, (uint32_t)n, ctx->vk, ctx->verdicts);
  CK(hipGetLastError());
  CK(hipMemcpyAsync(codes, ctx->verdicts, n, hipMemcpyDeviceToHost, st));
  CK(hipStreamSynchronize(st));
  return 0;
}

int edc_keycache_clear(edc_ctx* ctx) {
  if (!ctx) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  for (Slot& s : ctx->slot)
    if (s.pending) { ctx->err = "key cache change with a batch in flight"; return EDC_ERR_ARG; }
  int rc = sync_all(ctx);
  if (rc) return rc;
  free_keycache(ctx);
  return 0;
}

size_t edc_keycache_size(const edc_ctx* ctx) { return ctx ? ctx->kc_m : 0; }

// Appends the distinct new keys `neww` (un x 8 words) to the cache: grows the device arrays
// (capacity doubling; the cached keys keep their indices), decodes the new keys and builds their
// comb tables, builds B's comb table with the first key, and rebuilds the hash table over all
// keys. No batch may be in flight (callers check).
static int kc_append(edc_ctx* ctx, const std::vector<uint32_t>& neww) {
  const uint32_t u0 = ctx->kc_m, un = (uint32_t)(neww.size() / 8), u = u0 + un;
  if (!un) return 0;
  hipStream_t st = ctx->st();
  const size_t comb_words = (size_t)COMB_ENTRIES * NIELS_WORDS;
  if (u > ctx->kc_cap) {
    uint32_t cap = ctx->kc_cap ? 2 * ctx->kc_cap : 16;
    while (cap < u) cap *= 2;
    if (cap > KC_MAX_KEYS) cap = KC_MAX_KEYS;
    uint32_t *keys = nullptr, *comb = nullptr;
    uint8_t* okd = nullptr;
    if (dalloc(&keys, (size_t)cap * 8) != hipSuccess || dalloc(&okd, cap) != hipSuccess ||
        dalloc(&comb, (size_t)cap * comb_words) != hipSuccess) {
      (void)hipGetLastError();
      if (keys) (void)hipFree(keys);
      if (okd) (void)hipFree(okd);
      if (comb) (void)hipFree(comb);
      ctx->err = "key cache: out of device memory";
      return EDC_ERR_NOMEM;
    }
    if (u0) {
      CK(hipMemcpyAsync(keys, ctx->kc_keys, (size_t)u0 * 8 * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
      CK(hipMemcpyAsync(okd, ctx->kc_ok, u0, hipMemcpyDeviceToDevice, st));
      CK(hipMemcpyAsync(comb, ctx->kc_comb, (size_t)u0 * comb_words * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
      CK(hipStreamSynchronize(st));
    }
    if (ctx->kc_keys) (void)hipFree(ctx->kc_keys);
    if (ctx->kc_ok) (void)hipFree(ctx->kc_ok);
    if (ctx->kc_comb) (void)hipFree(ctx->kc_comb);
    ctx->kc_keys = keys;
    ctx->kc_ok = okd;
    ctx->kc_comb = comb;
    ctx->kc_cap = cap;
  }
  std::vector<uint32_t> all(ctx->kc_words);   // committed to the context only on success
  all.insert(all.end(), neww.begin(), neww.end());
  const uint32_t T = (uint32_t)next_pow2(2 * (size_t)(u < 8 ? 8 : u));
  std::vector<uint32_t> table(T, KC_EMPTY);
  for (uint32_t c = 0; c < u; ++c) {
    uint32_t h = kc_hash(&all[8 * c], ctx->kc_s0, ctx->kc_s1) & (T - 1);
    while (table[h] != KC_EMPTY) h = (h + 1) & (T - 1);
    table[h] = c;
  }
  // new table and scratch first: a failed allocation leaves the previous cache fully usable
  uint32_t *ntable = nullptr, *ext = nullptr;
  const bool new_table = T - 1 != ctx->kc_tmask || !ctx->kc_table;
  if ((new_table && dalloc(&ntable, T) != hipSuccess) || dalloc(&ext, (size_t)(un + 1) * EXT_WORDS) != hipSuccess) {
    (void)hipGetLastError();
    if (ntable) (void)hipFree(ntable);
    ctx->err = "key cache: out of device memory";
    return EDC_ERR_NOMEM;
  }
  if (new_table) {
    CK(hipStreamSynchronize(st));
    if (ctx->kc_table) (void)hipFree(ctx->kc_table);
    ctx->kc_table = ntable;
  }
  CK(hipMemcpyAsync(ctx->kc_table, table.data(), T * sizeof(uint32_t), hipMemcpyHostToDevice, st));
  CK(hipMemcpyAsync(ctx->kc_keys + (size_t)u0 * 8, neww.data(), neww.size() * sizeof(uint32_t),
                    hipMemcpyHostToDevice, st));
  launch_kc_decode(st, un, ctx->kc_keys + (size_t)u0 * 8, ext, ctx->kc_ok + u0);
  launch_kc_comb(st, un, ext, ctx->kc_comb + (size_t)u0 * comb_words);
  if (!ctx->bcomb) {
    CK(dalloc(&ctx->bcomb, comb_words));
    uint32_t* bext = ext + (size_t)un * EXT_WORDS;
    launch_kc_basepoint(st, bext);
    launch_kc_comb(st, 1, bext, ctx->bcomb);
  }
  CK(hipGetLastError());
  std::vector<uint8_t> okn(un);
  CK(hipMemcpyAsync(okn.data(), ctx->kc_ok + u0, un, hipMemcpyDeviceToHost, st));
  CK(hipStreamSynchronize(st));
  (void)hipFree(ext);
  ctx->kc_words.swap(all);
  ctx->kc_okh.insert(ctx->kc_okh.end(), okn.begin(), okn.end());
  ctx->kc_m = u;
  ctx->kc_tmask = T - 1;
  ctx->last_uncached = 0;                    // try split coefficients with the new key set
  return 0;
}

// distinct keys of vk (m x 32 bytes) not yet cached, in first-occurrence order; of[i] = the
// cache index key i will have
// (limit: the most keys the cache may then hold; edc_keycache_add checks it after dropping the
// keys that do not decode instead)
static int kc_collect(edc_ctx* ctx, size_t m, const uint8_t* vk, std::vector<uint32_t>& of,
                      std::vector<uint32_t>& neww, size_t limit = KC_MAX_KEYS) {
  std::unordered_map<std::string, uint32_t> idx;
  for (uint32_t c = 0; c < ctx->kc_m; ++c)
    idx.emplace(std::string(reinterpret_cast<const char*>(&ctx->kc_words[8 * c]), 32), c);
  of.resize(m);
  for (size_t i = 0; i < m; ++i) {
    auto it = idx.emplace(std::string(reinterpret_cast<const char*>(vk + 32 * i), 32), (uint32_t)idx.size());
    of[i] = it.first->second;
    if (it.second) {
      if (idx.size() > limit) { ctx->err = "key cache holds at most 65536 keys"; return EDC_ERR_ARG; }
      uint32_t w[8];
      memcpy(w, vk + 32 * i, 32);
      neww.insert(neww.end(), w, w + 8);
    }
  }
  return 0;
}

int64_t edc_keycache_load(edc_ctx* ctx, size_t m, const uint8_t* vk, uint8_t* ok) {
  if (!ctx || (m && !vk)) return EDC_ERR_ARG;
  int rc = edc_keycache_clear(ctx);
  if (rc) return rc;
  if (!m) return 0;
  // distinct keys in first-occurrence order (the cache is keyed on raw bytes, like the batch's
  // HashMap<VerificationKeyBytes, _>, src/batch.rs:114)
  std::vector<uint32_t> of, words;
  if ((rc = kc_collect(ctx, m, vk, of, words))) return rc;
  if ((rc = kc_append(ctx, words))) return rc;
  CK(dalloc(&ctx->kc_reg, m));
  CK(hipMemcpy(ctx->kc_reg, of.data(), m * sizeof(uint32_t), hipMemcpyHostToDevice));
  ctx->kc_reg_m = (uint32_t)m;
  if (ok)
    for (size_t i = 0; i < m; ++i) ok[i] = ctx->kc_okh[of[i]];
  return ctx->kc_m;
}

int64_t edc_keycache_add(edc_ctx* ctx, size_t m, const uint8_t* vk, uint8_t* ok) {
  if (!ctx || (m && !vk)) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  for (Slot& s : ctx->slot)
    if (s.pending) { ctx->err = "key cache change with a batch in flight"; return EDC_ERR_ARG; }
  int rc = sync_all(ctx);
  if (rc) return rc;
  std::vector<uint32_t> of, words;
  if ((rc = kc_collect(ctx, m, vk, of, words, SIZE_MAX))) return rc;
  // keys that fail to decode (VerificationKey::try_from's MalformedPublicKey) are not added: the
  // entry is meant for keys parsed from untrusted input, and a malformed one must not pin 64 KB of
  // comb table. of[] is remapped to the kept keys; a dropped key reports ok = 0.
  const uint32_t u0 = ctx->kc_m, un = (uint32_t)(words.size() / 8);
  std::vector<uint8_t> code(un, 0);
  if (un) {
    hipStream_t st = ctx->st();
    uint8_t *denc = nullptr, *dcode = nullptr;
    if (dalloc(&denc, (size_t)un * 32) != hipSuccess || dalloc(&dcode, un) != hipSuccess) {
      (void)hipGetLastError();
      if (denc) (void)hipFree(denc);
      ctx->err = "key cache: out of device memory";
      return EDC_ERR_NOMEM;
    }
    CK(hipMemcpyAsync(denc, words.data(), (size_t)un * 32, hipMemcpyHostToDevice, st));
    launch_vk_validate(st, un, denc, dcode);
    CK(hipGetLastError());
    CK(hipMemcpyAsync(code.data(), dcode, un, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    (void)hipFree(denc);
    (void)hipFree(dcode);
  }
  std::vector<uint32_t> keep, remap(un, UINT32_MAX);
  for (uint32_t j = 0; j < un; ++j)
    if (code[j] == EDC_OK) {
      remap[j] = u0 + (uint32_t)(keep.size() / 8);
      keep.insert(keep.end(), &words[8 * j], &words[8 * j] + 8);
    }
  if (u0 + keep.size() / 8 > KC_MAX_KEYS) { ctx->err = "key cache holds at most 65536 keys"; return EDC_ERR_ARG; }
  if ((rc = kc_append(ctx, keep))) return rc;
  if (ok)
    for (size_t i = 0; i < m; ++i) {
      const uint32_t c = of[i] < u0 ? of[i] : remap[of[i] - u0];
      ok[i] = c == UINT32_MAX ? 0 : ctx->kc_okh[c];
    }
  return ctx->kc_m;
}

int edc_sign_device(edc_ctx* ctx, size_t n, const uint8_t* d_seeds, const uint32_t* d_seed_index,
                    const uint8_t* d_msg, const uint64_t* d_msg_off, uint8_t* d_vk_out, uint8_t* d_sig_out) {
  if (!ctx) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  launch_sign(ctx->st(), (uint32_t)n, d_seeds, d_seed_index, d_msg, d_msg_off, ctx->btab, d_vk_out, d_sig_out);
  CK(hipGetLastError());
  CK(hipStreamSynchronize(ctx->st()));
  return 0;
}

int edc_sign(edc_ctx* ctx, size_t n, const uint8_t* seeds, size_t nseeds, const uint32_t* seed_index,
             const uint8_t* msg, const uint64_t* msg_off, uint8_t* vk_out, uint8_t* sig_out) {
  if (!ctx || (n && (!seeds || !vk_out || !sig_out || !msg_off))) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  if (seed_index) {
    for (size_t i = 0; i < n; ++i)
      if (seed_index[i] >= nseeds) { ctx->err = "seed_index out of range"; return EDC_ERR_ARG; }
  } else if (nseeds < n) {
    ctx->err = "need one seed per item when seed_index is NULL";
    return EDC_ERR_ARG;
  }
  int rc = upload_msgs(ctx, n, msg, msg_off);
  if (rc) return rc;
  if (!n) return 0;
  // aux: seeds (nseeds*32) | seed_index (n*4) | vk_out (n*32) | sig_out (n*64)
  const size_t sb = nseeds * 32, ib = seed_index ? n * 4 : 0;
  const size_t sb16 = (sb + 15) & ~(size_t)15, ib16 = (ib + 15) & ~(size_t)15;
  rc = ensure_aux(ctx, sb16 + ib16 + n * 96 + 64);
  if (rc) return rc;
  hipStream_t st = ctx->st();
  uint8_t* d_seeds = ctx->aux;
  uint32_t* d_idx = seed_index ? reinterpret_cast<uint32_t*>(ctx->aux + sb16) : nullptr;
  uint8_t* d_vk = ctx->aux + sb16 + ib16;
  uint8_t* d_sig = d_vk + n * 32;
  CK(hipMemcpyAsync(d_seeds, seeds, sb, hipMemcpyHostToDevice, st));
  if (d_idx) CK(hipMemcpyAsync(d_idx, seed_index, ib, hipMemcpyHostToDevice, st));
  launch_sign(st, (uint32_t)n, d_seeds, d_idx, ctx->msg, ctx->off, ctx->btab, d_vk, d_sig);
  CK(hipGetLastError());
  CK(hipMemcpyAsync(vk_out, d_vk, n * 32, hipMemcpyDeviceToHost, st));
  CK(hipMemcpyAsync(sig_out, d_sig, n * 64, hipMemcpyDeviceToHost, st));
  CK(hipStreamSynchronize(st));
  return 0;
}

int edc_chacha_fill_device(edc_ctx* ctx, const uint8_t key[32], uint64_t blk0, uint64_t nblocks, uint8_t* d_out) {
  if (!ctx || !key || (nblocks && !d_out)) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  uint32_t k[8];
  seed_words(key, k);
  launch_chacha_fill(ctx->st(), k, blk0, nblocks, reinterpret_cast<uint32_t*>(d_out));
  CK(hipGetLastError());
  CK(hipStreamSynchronize(ctx->st()));
  return 0;
}

int edc_set_slots(edc_ctx* ctx, int k) {
  if (!ctx || k < 1 || k > kSlots) return EDC_ERR_ARG;
  for (Slot& s : ctx->slot)
    if (s.pending) { ctx->err = "slot count change with a batch in flight"; return EDC_ERR_ARG; }
  ctx->nslots = k;
  ctx->next_ticket = 0;
  return 0;
}

int edc_set_key_grouping(edc_ctx* ctx, int mode) {
  if (!ctx || mode < 0 || mode > 3) return EDC_ERR_ARG;
  ctx->key_grouping = mode;
  ctx->ungrouped_run = 0;
  return 0;
}

int edc_set_key_split(edc_ctx* ctx, int mode) {
  if (!ctx || mode < 0 || mode > 1) return EDC_ERR_ARG;
  ctx->key_split = mode;
  return 0;
}

int edc_set_fallback_shape(edc_ctx* ctx, int ranges, int bits) {
  if (!ctx || ranges < 1 || ranges > 1024 || bits < 8 || bits > 13) return EDC_ERR_ARG;
  ctx->fb_ranges = (uint32_t)ranges;
  ctx->fb_bits = bits;
  return 0;
}

int edc_set_msm_shape(edc_ctx* ctx, int bits, int parts) {
  if (!ctx || bits < 0 || (bits && (bits < 8 || bits > 16)) || parts < 0 || parts > 64) return EDC_ERR_ARG;
  ctx->win_bits = bits;
  ctx->msm_parts = (uint32_t)parts;
  return 0;
}

int edc_set_msm_bin_entries(edc_ctx* ctx, int entries) {
  if (!ctx || entries < 0 || (entries && entries < 256)) return EDC_ERR_ARG;
  ctx->bin_entries = (uint32_t)entries;
  return 0;
}

int edc_reserve(edc_ctx* ctx, size_t n) {
  if (!ctx) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  const int c = ctx->win_bits ? ctx->win_bits : auto_window_bits(n);
  MsmPlan dense = make_plan(c, c, 1), few = make_plan(c, 8, 1);
  dense.nranges = few.nranges = MSM_MAX_BINS / (dense.bins_per_range > few.bins_per_range ? dense.bins_per_range
                                                                                          : few.bins_per_range);
  if (dense.nranges > 16) dense.nranges = few.nranges = 16;
  const MsmPlan splitp = make_plan(c, c, 1, false);
  size_t e1 = msm_entry_capacity(dense, n, n + 1), e2 = msm_entry_capacity(few, n, n + 1);
  const size_t e3 = msm_entry_capacity(splitp, 2 + 3 * n, 0);   // split coefficients (key cache)
  if (e3 > e1) e1 = e3;
  for (int i = 0; i < ctx->nslots; ++i) {
    Slot& s = ctx->slot[i];
    if (s.pending) { ctx->err = "reserve with a batch in flight"; return EDC_ERR_ARG; }
    int rc = ensure_slot(ctx, s, n);
    if (rc) return rc;
    rc = ensure_msm(ctx, s, dense.nbin() >= few.nbin() ? dense : few, e1 > e2 ? e1 : e2);
    if (rc) return rc;
  }
  return 0;
}

void edc_set_timing(edc_ctx* ctx, int enable) {
  if (ctx) ctx->timing = enable != 0;
}

int edc_last_timings(const edc_ctx* ctx, float* ms, int cap) {
  if (!ctx || !ms) return 0;
  int c = ctx->nlast < cap ? ctx->nlast : cap;
  for (int i = 0; i < c; ++i) ms[i] = ctx->last_ms[i];
  return c;
}

const char* edc_timing_name(int i) { return (i >= 0 && i < PH_N) ? kPhaseNames[i] : ""; }

int edc_last_msm_accum(const edc_ctx* ctx, float* ms, uint64_t* entries) {
  if (!ctx || !ctx->nlast) return EDC_ERR_ARG;
  if (ms) *ms = ctx->last_acc_ms;
  if (entries) *entries = ctx->last_acc_entries;
  return 0;
}

int edc_synchronize(edc_ctx* ctx) {
  if (!ctx) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  for (Slot& s : ctx->slot)
    if (s.st) CK(hipStreamSynchronize(s.st));
  return 0;
}

}  // extern "C"

// ---------------------------------------------------------------- several GPUs, one process
// A consensus node calls Verifier::verify once per block (src/batch.rs:149-217). edc_multi
// splits that one batch over the contexts of several devices: contiguous shards, shard g's z
// drawn at its global queue indices (z_base = shard start), so every shard evaluates its part of
// the same batch equation; each device reduces its shard to one partial point (128 bytes), the
// partials are gathered through the host (they already come back with each shard's verdict) and
// summed on the first device, then x8 and the identity test. One host thread per device drives
// its shard; the same device may appear several times (several contexts on one GPU).
// One in-flight multi-device batch (edc_multi_submit): every shard's 256-byte result block reaches
// `blocks` on the first device, whose combine stream waits for every shard's event and sums the
// partial points there (k_combine_blocks). The host only enqueues, and waits once per batch. How a
// block travels depends on the pair (edc_multi.route, fixed at edc_create_multi):
//  - ROUTE_LOCAL: the shard runs on the first device itself (listed twice): a one-wave kernel on
//    the shard's stream copies it;
//  - ROUTE_PEER: peer access from the shard's device to the first device was enabled: the same
//    kernel stores it over xGMI;
//  - ROUTE_STAGED: no peer access (or forced by edc_multi_debug_force_staged): the shard's final
//    kernel already wrote the block to its slot's pinned host mirror; the combine stream waits for
//    the shard's event and copies that mirror to `blocks` itself. No kernel ever stores to another
//    device's memory without peer access enabled.
struct MultiSlot {
  bool pending = false;
  int64_t ticket = -1;
  bool want = false;
  std::vector<int64_t> shard;        // shard tickets, one per context
  std::vector<hipEvent_t> copied;    // recorded on each shard's slot stream after its block copy
  hipEvent_t done = nullptr;         // first device, after the combine
  uint8_t* blocks = nullptr;         // first device: ndev x 256 bytes
  uint8_t* d_out = nullptr;          // first device: 256-byte verdict block
  uint8_t* h_out = nullptr;          // pinned mirror
};

enum { ROUTE_LOCAL = 0, ROUTE_PEER = 1, ROUTE_STAGED = 2 };

struct edc_multi {
  std::vector<edc_ctx*> ctx;
  std::vector<int> route;            // per shard: ROUTE_LOCAL / ROUTE_PEER / ROUTE_STAGED
  std::vector<int> route_auto;       // as found by edc_create_multi (edc_multi_debug_force_staged(0) restores it)
  std::string err;
  MultiSlot ms[kSlots];
  int ring = kSlots;                 // multi-batches in flight = the smallest shard context's slot count
  int64_t next_ticket = 0;
  hipStream_t comb = nullptr;        // first device: every batch's combine, in submission order
};

struct Shard {
  size_t lo = 0, hi = 0;
  int rc = 0, bad = 0;
  uint8_t partial[128] = {};
};

static void shard_bounds(size_t n, size_t g, std::vector<Shard>& sh) {
  sh.assign(g, Shard());
  for (size_t i = 0; i < g; ++i) {
    sh[i].lo = n * i / g;
    sh[i].hi = n * (i + 1) / g;
  }
}

template <typename F>
static void on_each_device(edc_multi* M, std::vector<Shard>& sh, F&& f) {
  std::vector<std::thread> th;
  for (size_t g = 1; g < sh.size(); ++g) th.emplace_back([&, g] { sh[g].rc = f(M->ctx[g], sh[g]); });
  sh[0].rc = f(M->ctx[0], sh[0]);
  for (auto& t : th) t.join();
}

// shard's part of the batch on its device: staged from the host, then the whole pipeline on
// slot 0 (so that a fallback can reuse its k, points and grouping), partial point + bad flag
static int shard_partial(edc_ctx* c, Shard& s, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg,
                         const uint64_t* msg_off, const uint8_t* z_seed) {
  if (hipSetDevice(c->device) != hipSuccess) return EDC_ERR_HIP;
  const size_t m = s.hi - s.lo;
  int rc = upload(c, m, vk + 32 * s.lo, sig + 64 * s.lo, msg, msg_off + s.lo);
  if (rc) return rc;
  rc = run_batch_sync(c, m, c->vk, c->sig, c->msg, c->off, z_seed, s.lo, nullptr, nullptr, s.partial, &s.bad);
  return rc < 0 ? rc : 0;
}

static int multi_batch(edc_multi* M, size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg,
                       const uint64_t* msg_off, const uint8_t* z_seed, uint8_t check8[32], std::vector<Shard>& sh) {
  shard_bounds(n, M->ctx.size(), sh);
  on_each_device(M, sh, [&](edc_ctx* c, Shard& s) { return shard_partial(c, s, vk, sig, msg, msg_off, z_seed); });
  std::vector<uint8_t> parts(128 * sh.size());
  int bad = 0;
  for (size_t g = 0; g < sh.size(); ++g) {
    if (sh[g].rc < 0) {
      M->err = std::string("device ") + std::to_string(M->ctx[g]->device) + ": " + M->ctx[g]->err;
      return sh[g].rc;
    }
    memcpy(&parts[128 * g], sh[g].partial, 128);
    bad |= sh[g].bad;
  }
  edc_ctx* c0 = M->ctx[0];
  if (hipSetDevice(c0->device) != hipSuccess) return EDC_ERR_HIP;
  const int rc = combine_points(c0, sh.size(), parts.data(), bad, check8, nullptr);
  if (rc < 0) M->err = c0->err;
  return rc;
}

#define MCK(expr)                                                       \
  do {                                                                  \
    hipError_t e_ = (expr);                                             \
    if (e_ != hipSuccess) {                                             \
      (void)hipGetLastError();                                          \
      M->err = std::string(#expr) + ": " + hipGetErrorString(e_);       \
      return EDC_ERR_HIP;                                               \
    }                                                                   \
  } while (0)

static int multi_slot_init(edc_multi* M, MultiSlot& ms) {
  for (edc_ctx* c : M->ctx)
    if (c->nslots < M->ring) {   // edc_set_slots on a shard context after edc_create_multi
      M->err = "a shard context has fewer in-flight slots than the multi-device ring";
      return EDC_ERR_ARG;
    }
  if (ms.done) return 0;
  const size_t g = M->ctx.size();
  MCK(hipSetDevice(M->ctx[0]->device));
  // the combines are tiny and in order: one ordinary stream for all of them (the shard contexts'
  // slot streams already hold a hardware queue each)
  if (!M->comb) MCK(hipStreamCreateWithFlags(&M->comb, hipStreamNonBlocking));
  MCK(hipEventCreateWithFlags(&ms.done, hipEventDisableTiming));
  MCK(hipMalloc((void**)&ms.blocks, 256 * g));
  MCK(hipMalloc((void**)&ms.d_out, 256));
  MCK(hipHostMalloc((void**)&ms.h_out, 256));
  ms.copied.assign(g, nullptr);
  for (size_t i = 0; i < g; ++i) {
    MCK(hipSetDevice(M->ctx[i]->device));
    MCK(hipEventCreateWithFlags(&ms.copied[i], hipEventDisableTiming));
  }
  return 0;
}

static void multi_slot_free(edc_multi* M, MultiSlot& ms) {
  if (!ms.done) return;
  (void)hipSetDevice(M->ctx[0]->device);
  (void)hipEventSynchronize(ms.done);
  for (hipEvent_t e : ms.copied)
    if (e) (void)hipEventDestroy(e);
  if (ms.done) (void)hipEventDestroy(ms.done);
  if (ms.blocks) (void)hipFree(ms.blocks);
  if (ms.d_out) (void)hipFree(ms.d_out);
  if (ms.h_out) (void)hipHostFree(ms.h_out);
  ms = MultiSlot();
}

// After shard g's batch was enqueued on its context (ticket t): copy its result block to the first
// device behind the batch, on the shard's slot stream, and let the combine stream wait for it.
static int multi_link_shard(edc_multi* M, MultiSlot& ms, size_t g, int64_t t) {
  edc_ctx* c = M->ctx[g];
  Slot& s = c->slot[t % c->nslots];
  if (!s.pending || s.ticket != t || !s.d_out) { M->err = "shard ticket has no pending slot"; return EDC_ERR_ARG; }
  MCK(hipSetDevice(c->device));
  const int route = M->route[g];
  if (route != ROUTE_STAGED) {
    launch_copy_block(s.st, s.d_out, ms.blocks + 256 * g);   // hipMemcpyPeerAsync blocks the host here
    MCK(hipGetLastError());
  }
  MCK(hipEventRecord(ms.copied[g], s.st));
  MCK(hipSetDevice(M->ctx[0]->device));
  MCK(hipStreamWaitEvent(M->comb, ms.copied[g], 0));
  // staged: the shard's final kernel stored its block to the slot's pinned host mirror (the slot is
  // not reused before edc_multi_wait has synchronized this combine)
  if (route == ROUTE_STAGED) MCK(hipMemcpyAsync(ms.blocks + 256 * g, s.h_out, 256, hipMemcpyHostToDevice, M->comb));
  return 0;
}

// enqueue the combine of every shard's block on the first device; the batch is then in flight
static int multi_finish_submit(edc_multi* M, MultiSlot& ms, int64_t ticket, int want_check8) {
  MCK(hipSetDevice(M->ctx[0]->device));
  launch_combine_blocks(M->comb, (uint32_t)M->ctx.size(), ms.blocks, want_check8 != 0, ms.d_out);
  MCK(hipGetLastError());
  MCK(hipMemcpyAsync(ms.h_out, ms.d_out, 256, hipMemcpyDeviceToHost, M->comb));
  MCK(hipEventRecord(ms.done, M->comb));
  ms.pending = true;
  ms.ticket = ticket;
  ms.want = want_check8 != 0;
  M->next_ticket++;
  return ticket >= 0 ? 0 : EDC_ERR_ARG;
}

// shard g's submission failed after earlier shards were enqueued: drain those so that their
// contexts' tickets stay consistent, and report the failure
static int multi_abort(edc_multi* M, MultiSlot& ms, size_t failed, bool link_failed, int rc) {
  const std::string why = link_failed ? M->err : std::string(edc_last_error(M->ctx[failed]));
  for (size_t g = 0; g < ms.shard.size(); ++g)
    if (ms.shard[g] >= 0) (void)edc_batch_wait(M->ctx[g], ms.shard[g], nullptr, nullptr, nullptr);
  M->err = std::string("device ") + std::to_string(M->ctx[failed]->device) + ": " + why;
  return rc < 0 ? rc : EDC_ERR_ARG;
}

extern "C" {

edc_multi* edc_create_multi(const int* devices, int ndev) {
  if (!devices || ndev < 1 || ndev > 64) return nullptr;
  edc_multi* M = new edc_multi();
  for (int i = 0; i < ndev; ++i) {
    edc_ctx* c = edc_create(devices[i]);
    if (!c) {
      edc_destroy_multi(M);
      return nullptr;
    }
    M->ctx.push_back(c);
  }
  // contexts sharing one GPU split its kSlots (16) in-flight slots (one hardware queue each), so
  // that a rehearsal with a device listed several times does not oversubscribe the queue scheduler;
  // the multi-batch ring is the smallest share, so a multi submission never finds a shard's slot busy
  M->ring = kSlots;
  for (int i = 0; i < ndev; ++i) {
    int same = 0;
    for (int j = 0; j < ndev; ++j) same += devices[j] == devices[i];
    M->ctx[i]->nslots = kSlots / same > 0 ? kSlots / same : 1;
    if (M->ctx[i]->nslots < M->ring) M->ring = M->ctx[i]->nslots;
  }
  // how each shard's result block reaches the first device (edc_multi_submit): a peer store over
  // xGMI only where peer access from the shard's device to the first device is actually enabled;
  // any other outcome of the enable than success / already-enabled is an error
  M->route.assign(ndev, ROUTE_LOCAL);
  for (int i = 1; i < ndev; ++i) {
    if (devices[i] == devices[0]) continue;
    int can = 0;
    if (hipDeviceCanAccessPeer(&can, devices[i], devices[0]) != hipSuccess || !can) {
      (void)hipGetLastError();
      M->route[i] = ROUTE_STAGED;
      continue;
    }
    const hipError_t e = hipSetDevice(devices[i]) == hipSuccess ? hipDeviceEnablePeerAccess(devices[0], 0)
                                                                 : hipErrorInvalidDevice;
    (void)hipGetLastError();
    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
      edc_destroy_multi(M);
      return nullptr;
    }
    M->route[i] = ROUTE_PEER;
  }
  M->route_auto = M->route;
  return M;
}

int edc_multi_debug_force_staged(edc_multi* M, int on) {
  if (!M) return EDC_ERR_ARG;
  for (const MultiSlot& ms : M->ms)
    if (ms.pending) { M->err = "route change with a batch in flight"; return EDC_ERR_ARG; }
  for (size_t i = 0; i < M->ctx.size(); ++i) M->route[i] = on ? (int)ROUTE_STAGED : M->route_auto[i];
  return 0;
}

int edc_multi_route(const edc_multi* M, int i) {
  return (M && i >= 0 && i < (int)M->route.size()) ? M->route[i] : EDC_ERR_ARG;
}

void edc_destroy_multi(edc_multi* M) {
  if (!M) return;
  for (MultiSlot& ms : M->ms) multi_slot_free(M, ms);
  if (M->comb) {
    (void)hipSetDevice(M->ctx[0]->device);
    (void)hipStreamDestroy(M->comb);
  }
  for (edc_ctx* c : M->ctx) edc_destroy(c);
  delete M;
}

int64_t edc_multi_submit(edc_multi* M, size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg,
                         const uint64_t* msg_off, const uint8_t z_seed[32], int want_check8) {
  if (!M || !z_seed || (n && (!vk || !sig || !msg_off))) return EDC_ERR_ARG;
  const int64_t ticket = M->next_ticket;
  MultiSlot& ms = M->ms[ticket % M->ring];
  if (ms.pending) { M->err = "all slots in flight: wait for the oldest ticket first"; return EDC_ERR_ARG; }
  int rc = multi_slot_init(M, ms);
  if (rc) return rc;
  std::vector<Shard> sh;
  shard_bounds(n, M->ctx.size(), sh);
  ms.shard.assign(sh.size(), -1);
  for (size_t g = 0; g < sh.size(); ++g) {
    const size_t lo = sh[g].lo, m = sh[g].hi - lo;
    const int64_t t = edc_batch_submit(M->ctx[g], m, vk + 32 * lo, sig + 64 * lo, msg, msg_off + lo, z_seed, lo, 0);
    if (t < 0) return multi_abort(M, ms, g, false, (int)t);
    ms.shard[g] = t;
    rc = multi_link_shard(M, ms, g, t);
    if (rc) return multi_abort(M, ms, g, true, rc);
  }
  rc = multi_finish_submit(M, ms, ticket, want_check8);
  return rc ? rc : ticket;
}

int64_t edc_multi_submit_device(edc_multi* M, const size_t* n, const uint8_t* const* d_vk, const uint8_t* const* d_sig,
                                const uint8_t* const* d_msg, const uint64_t* const* d_msg_off,
                                const uint8_t z_seed[32], int want_check8) {
  if (!M || !z_seed || !n || !d_vk || !d_sig || !d_msg || !d_msg_off) return EDC_ERR_ARG;
  const int64_t ticket = M->next_ticket;
  MultiSlot& ms = M->ms[ticket % M->ring];
  if (ms.pending) { M->err = "all slots in flight: wait for the oldest ticket first"; return EDC_ERR_ARG; }
  int rc = multi_slot_init(M, ms);
  if (rc) return rc;
  const size_t G = M->ctx.size();
  ms.shard.assign(G, -1);
  uint64_t base = 0;
  for (size_t g = 0; g < G; ++g) {
    const int64_t t = edc_batch_submit_device(M->ctx[g], n[g], d_vk[g], d_sig[g], d_msg[g], d_msg_off[g], z_seed,
                                              base, nullptr, 0);
    if (t < 0) return multi_abort(M, ms, g, false, (int)t);
    ms.shard[g] = t;
    rc = multi_link_shard(M, ms, g, t);
    if (rc) return multi_abort(M, ms, g, true, rc);
    base += n[g];
  }
  rc = multi_finish_submit(M, ms, ticket, want_check8);
  return rc ? rc : ticket;
}

int edc_multi_wait(edc_multi* M, int64_t ticket, uint8_t check8[32]) {
  if (!M || ticket < 0) return EDC_ERR_ARG;
  MultiSlot& ms = M->ms[ticket % M->ring];
  if (!ms.pending || ms.ticket != ticket) { M->err = "unknown or already-waited ticket"; return EDC_ERR_ARG; }
  ms.pending = false;
  int err = 0;
  for (size_t g = 0; g < ms.shard.size(); ++g) {   // retire the shard tickets (grouping statistics)
    const int r = edc_batch_wait(M->ctx[g], ms.shard[g], nullptr, nullptr, nullptr);
    if (r < 0 && !err) {
      err = r;
      M->err = std::string("device ") + std::to_string(M->ctx[g]->device) + ": " + edc_last_error(M->ctx[g]);
    }
  }
  MCK(hipSetDevice(M->ctx[0]->device));
  if (err) {   // the combine may still be running on M->comb: drain it before the slot can be reused
    (void)hipEventSynchronize(ms.done);
    (void)hipGetLastError();
    return err;
  }
  MCK(hipEventSynchronize(ms.done));
  const int verdict = reinterpret_cast<int*>(ms.h_out)[0];
  const int bad = reinterpret_cast<int*>(ms.h_out)[1];
  if (check8) {
    if (bad || !ms.want) memset(check8, 0, 32);
    else memcpy(check8, ms.h_out + 16, 32);
  }
  return verdict ? EDC_INVALID_SIGNATURE : EDC_OK;
}

int edc_multi_size(const edc_multi* M) { return M ? (int)M->ctx.size() : 0; }

edc_ctx* edc_multi_context(edc_multi* M, int i) {
  return (M && i >= 0 && i < (int)M->ctx.size()) ? M->ctx[i] : nullptr;
}

const char* edc_multi_last_error(const edc_multi* M) { return M ? M->err.c_str() : "null context"; }

int edc_multi_batch_verify(edc_multi* M, size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg,
                           const uint64_t* msg_off, const uint8_t z_seed[32], uint8_t check8[32]) {
  if (!M || !z_seed || (n && (!vk || !sig || !msg_off))) return EDC_ERR_ARG;
  std::vector<Shard> sh;
  return multi_batch(M, n, vk, sig, msg, msg_off, z_seed, check8, sh);
}

int edc_multi_batch_verify_fallback(edc_multi* M, size_t n, const uint8_t* vk, const uint8_t* sig,
                                    const uint8_t* msg, const uint64_t* msg_off, const uint8_t z_seed[32],
                                    uint8_t* verdicts, int* n_invalid, uint8_t check8[32]) {
  if (!M || !z_seed || (n && (!vk || !sig || !msg_off || !verdicts))) return EDC_ERR_ARG;
  if (n_invalid) *n_invalid = 0;
  std::vector<Shard> sh;
  const int rc = multi_batch(M, n, vk, sig, msg, msg_off, z_seed, check8, sh);
  if (rc <= 0) {
    if (rc == 0 && n) memset(verdicts, 0, n);
    return rc;
  }
  // every shard whose own partial fails (or that saw a decode / canonicity failure) localizes its
  // invalid items with the grouped fallback, reusing its batch state; the others are all valid
  on_each_device(M, sh, [&](edc_ctx* c, Shard& s) -> int {
    const size_t m = s.hi - s.lo;
    memset(verdicts + s.lo, 0, m);
    if (hipSetDevice(c->device) != hipSuccess) return EDC_ERR_HIP;
    const int ok = combine_points(c, 1, s.partial, s.bad, nullptr, nullptr);
    if (ok <= 0) return ok;
    Slot& sl = c->slot[0];
    bool per_sig;
    uint32_t keys;
    int r = slot_grouping(c, sl, &per_sig, &keys);
    if (r) return r;
    return fallback_ranges(c, sl, m, c->vk, c->sig, c->msg, c->off, z_seed, s.lo, per_sig, keys, verdicts + s.lo);
  });
  int total = 0;
  for (size_t g = 0; g < sh.size(); ++g) {
    if (sh[g].rc < 0) {
      M->err = std::string("device ") + std::to_string(M->ctx[g]->device) + ": " + M->ctx[g]->err;
      return sh[g].rc;
    }
    total += sh[g].rc;
  }
  if (n_invalid) *n_invalid = total;
  return EDC_INVALID_SIGNATURE;
}

}  // extern "C"
