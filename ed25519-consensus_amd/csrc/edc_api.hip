// C ABI (include/edc.h): context, workspace and the orchestration of the batch pipeline.
// Every entry point cites the reference API it replaces in include/edc.h.
#include <string.h>
#include <string>
#include <vector>
#include "edc.h"
#include "edc_common.h"
#include "edc_launch.h"

using namespace edc;

namespace {

enum Phase { PH_CHALLENGE, PH_DECOMP_R, PH_KEYS, PH_COEF, PH_MSM_BIN, PH_MSM_BUCKET, PH_MSM_TAIL, PH_N };
const char* kPhaseNames[PH_N] = {"challenge_sha512", "decompress_R", "keys_group_decompress_A",
                                 "coef_chacha_scalar", "msm_bin", "msm_bucket", "msm_window_final"};

template <typename T>
hipError_t dalloc(T** p, size_t count) {
  *p = nullptr;
  if (count == 0) count = 1;
  return hipMalloc((void**)p, count * sizeof(T));
}

}  // namespace

struct edc_ctx {
  int device = 0;
  hipStream_t st = nullptr;
  std::string err;
  uint32_t* btab = nullptr;   // [1..8]B affine Niels
  // grow-only workspace
  size_t cap_n = 0, cap_msg = 0, cap_T = 0;
  uint8_t *vk = nullptr, *sig = nullptr, *msg = nullptr, *zexp = nullptr;
  uint64_t* off = nullptr;
  uint32_t *k = nullptr, *key_slot = nullptr, *key_index = nullptr, *key_rep = nullptr;
  uint32_t *table = nullptr, *slot_key = nullptr;
  uint32_t *pts = nullptr, *scal = nullptr;
  unsigned long long *key_acc = nullptr, *u_acc = nullptr;
  uint32_t *counts = nullptr, *offsets = nullptr, *cursor = nullptr;
  uint2* entries = nullptr;
  uint32_t *slice_W = nullptr, *slice_T = nullptr, *win = nullptr;
  uint32_t* buckets = nullptr;  // NBIN x 256 bucket sums (extended), fixed size
  uint8_t* verdicts = nullptr;
  uint8_t* aux = nullptr;       // decode xy / sign outputs
  size_t cap_aux = 0;
  int* flags = nullptr;
  uint8_t* d_out = nullptr;     // 256-byte result block
  uint8_t* h_out = nullptr;     // pinned mirror
  bool timing = false;
  hipEvent_t ev[PH_N + 1] = {};
  float last_ms[PH_N] = {};
  int nlast = 0;
};

#define CK(expr)                                                        \
  do {                                                                  \
    hipError_t e_ = (expr);                                             \
    if (e_ != hipSuccess) {                                             \
      ctx->err = std::string(#expr) + ": " + hipGetErrorString(e_);     \
      return EDC_ERR_HIP;                                               \
    }                                                                   \
  } while (0)

static void free_workspace(edc_ctx* ctx) {
  void* ptrs[] = {ctx->vk, ctx->sig, ctx->msg, ctx->zexp, ctx->off, ctx->k, ctx->key_slot, ctx->key_index,
                  ctx->key_rep, ctx->table, ctx->slot_key, ctx->pts, ctx->scal, ctx->key_acc, ctx->u_acc,
                  ctx->counts, ctx->offsets, ctx->cursor, ctx->entries, ctx->slice_W, ctx->slice_T,
                  ctx->win, ctx->verdicts, ctx->buckets};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  ctx->vk = ctx->sig = ctx->msg = ctx->zexp = nullptr;
  ctx->off = nullptr;
  ctx->k = ctx->key_slot = ctx->key_index = ctx->key_rep = ctx->table = ctx->slot_key = nullptr;
  ctx->pts = ctx->scal = nullptr;
  ctx->key_acc = ctx->u_acc = nullptr;
  ctx->counts = ctx->offsets = ctx->cursor = nullptr;
  ctx->entries = nullptr;
  ctx->slice_W = ctx->slice_T = ctx->win = nullptr;
  ctx->buckets = nullptr;
  ctx->verdicts = nullptr;
  ctx->cap_n = ctx->cap_T = 0;
}

static size_t next_pow2(size_t x) {
  size_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

static int ensure_n(edc_ctx* ctx, size_t n) {
  if (n <= ctx->cap_n && ctx->pts) return 0;
  CK(hipStreamSynchronize(ctx->st));
  free_workspace(ctx);
  size_t cap = n < 1024 ? 1024 : n + n / 8;
  size_t T = next_pow2(2 * cap);
  CK(dalloc(&ctx->vk, cap * 32));
  CK(dalloc(&ctx->sig, cap * 64));
  CK(dalloc(&ctx->zexp, cap * 16));
  CK(dalloc(&ctx->off, cap + 1));
  CK(dalloc(&ctx->k, cap * 8));
  CK(dalloc(&ctx->key_slot, cap));
  CK(dalloc(&ctx->key_index, cap));
  CK(dalloc(&ctx->key_rep, cap));
  CK(dalloc(&ctx->table, T));
  CK(dalloc(&ctx->slot_key, T));
  CK(dalloc(&ctx->pts, (1 + 2 * cap) * NIELS_WORDS));
  CK(dalloc(&ctx->scal, (1 + 2 * cap) * 8));
  CK(dalloc(&ctx->key_acc, cap * KEY_ACC_LIMBS));
  CK(dalloc(&ctx->u_acc, KEY_ACC_LIMBS));
  CK(dalloc(&ctx->counts, NBIN));
  CK(dalloc(&ctx->offsets, NBIN));
  CK(dalloc(&ctx->cursor, NBIN));
  CK(dalloc(&ctx->entries, msm_entry_capacity((uint32_t)cap)));
  CK(dalloc(&ctx->slice_W, (size_t)NBIN * EXT_WORDS));
  CK(dalloc(&ctx->slice_T, (size_t)NBIN * EXT_WORDS));
  CK(dalloc(&ctx->win, (size_t)NWIN_FULL * EXT_WORDS));
  CK(dalloc(&ctx->buckets, msm_bucket_words()));
  CK(dalloc(&ctx->verdicts, cap));
  launch_init_basepoint(ctx->st, ctx->pts);
  CK(hipGetLastError());
  ctx->cap_n = cap;
  ctx->cap_T = T;
  return 0;
}

static int ensure_msg(edc_ctx* ctx, size_t bytes) {
  if (bytes <= ctx->cap_msg && ctx->msg) return 0;
  CK(hipStreamSynchronize(ctx->st));
  if (ctx->msg) (void)hipFree(ctx->msg);
  size_t cap = bytes < 4096 ? 4096 : bytes + bytes / 8;
  CK(dalloc(&ctx->msg, cap));
  ctx->cap_msg = cap;
  return 0;
}

static int ensure_aux(edc_ctx* ctx, size_t bytes) {
  if (bytes <= ctx->cap_aux && ctx->aux) return 0;
  CK(hipStreamSynchronize(ctx->st));
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

static inline void mark(edc_ctx* ctx, int ph) {
  if (ctx->timing) (void)hipEventRecord(ctx->ev[ph], ctx->st);
}

// Stage the message arena + offsets (0-based) into the context's device buffers.
static int upload_msgs(edc_ctx* ctx, size_t n, const uint8_t* msg, const uint64_t* msg_off) {
  if (n && !msg_off) { ctx->err = "null msg_off"; return EDC_ERR_ARG; }
  int rc = ensure_n(ctx, n);
  if (rc) return rc;
  const size_t mbytes = n ? (size_t)(msg_off[n] - msg_off[0]) : 0;
  if (mbytes && !msg) { ctx->err = "null msg"; return EDC_ERR_ARG; }
  rc = ensure_msg(ctx, mbytes);
  if (rc) return rc;
  if (!n) return 0;
  if (mbytes) CK(hipMemcpyAsync(ctx->msg, msg + msg_off[0], mbytes, hipMemcpyHostToDevice, ctx->st));
  if (msg_off[0] == 0) {
    CK(hipMemcpyAsync(ctx->off, msg_off, (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, ctx->st));
  } else {
    std::vector<uint64_t> o(n + 1);
    for (size_t i = 0; i <= n; ++i) o[i] = msg_off[i] - msg_off[0];
    CK(hipMemcpyAsync(ctx->off, o.data(), (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, ctx->st));
    CK(hipStreamSynchronize(ctx->st));
  }
  return 0;
}

// Stage the host inputs (keys, signatures, messages) into the context's device buffers.
static int upload(edc_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg,
                  const uint64_t* msg_off) {
  if (n && (!vk || !sig)) { ctx->err = "null input"; return EDC_ERR_ARG; }
  int rc = upload_msgs(ctx, n, msg, msg_off);
  if (rc || !n) return rc;
  CK(hipMemcpyAsync(ctx->vk, vk, n * 32, hipMemcpyHostToDevice, ctx->st));
  CK(hipMemcpyAsync(ctx->sig, sig, n * 64, hipMemcpyHostToDevice, ctx->st));
  return 0;
}

// The batch pipeline on device-resident inputs. Leaves the 256-byte result block in h_out.
static int run_batch(edc_ctx* ctx, size_t n, const uint8_t* d_vk, const uint8_t* d_sig, const uint8_t* d_msg,
                     const uint64_t* d_off, const uint8_t* z_seed, uint64_t z_base, const uint8_t* d_z,
                     int want_compress) {
  if (n >= (1ull << 28)) { ctx->err = "batch too large for one call (max 2^28 items)"; return EDC_ERR_ARG; }
  int rc = ensure_n(ctx, n);
  if (rc) return rc;
  const uint32_t N = (uint32_t)n;
  const uint32_t T = (uint32_t)next_pow2(2 * (n < 128 ? 128 : n));
  if (T > ctx->cap_T) { ctx->err = "hash table capacity"; return EDC_ERR_ARG; }
  uint32_t seed[8];
  seed_words(z_seed, seed);
  hipStream_t st = ctx->st;
  CK(hipMemsetAsync(ctx->flags, 0, FLAG_COUNT * sizeof(int), st));
  CK(hipMemsetAsync(ctx->table, 0xFF, (size_t)T * sizeof(uint32_t), st));
  CK(hipMemsetAsync(ctx->u_acc, 0, KEY_ACC_LIMBS * sizeof(unsigned long long), st));
  CK(hipMemsetAsync(ctx->d_out, 0, 256, st));
  mark(ctx, PH_CHALLENGE);
  launch_challenge(st, N, d_vk, d_sig, d_msg, d_off, ctx->k);
  mark(ctx, PH_DECOMP_R);
  launch_decompress_R(st, N, d_sig, ctx->pts, ctx->flags);
  mark(ctx, PH_KEYS);
  launch_keys(st, N, d_vk, ctx->table, T - 1, seed[0] ^ 0x5bd1e995u, ctx->slot_key, ctx->key_slot,
              ctx->key_rep, ctx->key_index, ctx->pts, ctx->key_acc, ctx->flags);
  mark(ctx, PH_COEF);
  launch_coef(st, N, d_sig, ctx->k, d_z, seed, z_base, ctx->key_index, ctx->scal, ctx->key_acc, ctx->u_acc,
              ctx->flags);
  mark(ctx, PH_MSM_BIN);
  launch_msm_bin(st, N, ctx->scal, ctx->counts, ctx->offsets, ctx->cursor, ctx->entries, ctx->flags);
  mark(ctx, PH_MSM_BUCKET);
  launch_msm_bucket(st, ctx->counts, ctx->offsets, ctx->entries, ctx->pts, ctx->buckets, ctx->slice_W,
                    ctx->slice_T);
  mark(ctx, PH_MSM_TAIL);
  launch_msm_tail(st, ctx->slice_W, ctx->slice_T, ctx->win, ctx->flags, want_compress, ctx->d_out);
  mark(ctx, PH_N);
  CK(hipGetLastError());
  CK(hipMemcpyAsync(ctx->h_out, ctx->d_out, 256, hipMemcpyDeviceToHost, st));
  CK(hipStreamSynchronize(st));
  if (ctx->timing) {
    for (int p = 0; p < PH_N; ++p) CK(hipEventElapsedTime(&ctx->last_ms[p], ctx->ev[p], ctx->ev[p + 1]));
    ctx->nlast = PH_N;
  }
  return 0;
}

static int verdict_from_out(edc_ctx* ctx, uint8_t check8[32]) {
  int verdict = reinterpret_cast<int*>(ctx->h_out)[0];
  int bad = reinterpret_cast<int*>(ctx->h_out)[1];
  if (check8) {
    if (bad) memset(check8, 0, 32);
    else memcpy(check8, ctx->h_out + 16, 32);
  }
  return verdict ? EDC_INVALID_SIGNATURE : EDC_OK;
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
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->st, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    return nullptr;
  }
  bool ok = dalloc(&ctx->btab, 8 * NIELS_WORDS) == hipSuccess && dalloc(&ctx->flags, FLAG_COUNT) == hipSuccess &&
            dalloc(&ctx->d_out, 256) == hipSuccess && hipHostMalloc((void**)&ctx->h_out, 256) == hipSuccess;
  for (int p = 0; ok && p <= PH_N; ++p) ok = hipEventCreate(&ctx->ev[p]) == hipSuccess;
  if (ok) {
    launch_init_btable(ctx->st, ctx->btab);
    ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(ctx->st) == hipSuccess;
  }
  if (!ok) {
    edc_destroy(ctx);
    return nullptr;
  }
  return ctx;
}

void edc_destroy(edc_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->st) (void)hipStreamSynchronize(ctx->st);
  free_workspace(ctx);
  if (ctx->msg) (void)hipFree(ctx->msg);
  if (ctx->aux) (void)hipFree(ctx->aux);
  if (ctx->btab) (void)hipFree(ctx->btab);
  if (ctx->flags) (void)hipFree(ctx->flags);
  if (ctx->d_out) (void)hipFree(ctx->d_out);
  if (ctx->h_out) (void)hipHostFree(ctx->h_out);
  for (int p = 0; p <= PH_N; ++p)
    if (ctx->ev[p]) (void)hipEventDestroy(ctx->ev[p]);
  if (ctx->st) (void)hipStreamDestroy(ctx->st);
  delete ctx;
}

const char* edc_last_error(const edc_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int edc_batch_verify(edc_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg,
                     const uint64_t* msg_off, const uint8_t z_seed[32], uint8_t check8[32]) {
  if (!ctx || !z_seed) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  int rc = upload(ctx, n, vk, sig, msg, msg_off);
  if (rc) return rc;
  rc = run_batch(ctx, n, ctx->vk, ctx->sig, ctx->msg, ctx->off, z_seed, 0, nullptr, check8 != nullptr);
  if (rc) return rc;
  return verdict_from_out(ctx, check8);
}

int edc_batch_verify_z(edc_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg,
                       const uint64_t* msg_off, const uint8_t* z, uint8_t check8[32]) {
  if (!ctx || (n && !z)) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  int rc = upload(ctx, n, vk, sig, msg, msg_off);
  if (rc) return rc;
  if (n) CK(hipMemcpyAsync(ctx->zexp, z, n * 16, hipMemcpyHostToDevice, ctx->st));
  rc = run_batch(ctx, n, ctx->vk, ctx->sig, ctx->msg, ctx->off, nullptr, 0, ctx->zexp, check8 != nullptr);
  if (rc) return rc;
  return verdict_from_out(ctx, check8);
}

int edc_batch_verify_device(edc_ctx* ctx, size_t n, const uint8_t* d_vk, const uint8_t* d_sig,
                            const uint8_t* d_msg, const uint64_t* d_msg_off, const uint8_t z_seed[32],
                            uint64_t z_base, const uint8_t* d_z, uint8_t check8[32]) {
  if (!ctx || (!z_seed && !d_z)) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  int rc = run_batch(ctx, n, d_vk, d_sig, d_msg, d_msg_off, z_seed, z_base, d_z, check8 != nullptr);
  if (rc) return rc;
  return verdict_from_out(ctx, check8);
}

int edc_batch_partial_device(edc_ctx* ctx, size_t n, const uint8_t* d_vk, const uint8_t* d_sig,
                             const uint8_t* d_msg, const uint64_t* d_msg_off, const uint8_t z_seed[32],
                             uint64_t z_base, const uint8_t* d_z, uint8_t partial[128], int* bad) {
  if (!ctx || !partial || (!z_seed && !d_z)) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  int rc = run_batch(ctx, n, d_vk, d_sig, d_msg, d_msg_off, z_seed, z_base, d_z, 0);
  if (rc) return rc;
  memcpy(partial, ctx->h_out + 48, 128);
  if (bad) *bad = reinterpret_cast<int*>(ctx->h_out)[1];
  return 0;
}

int edc_combine_partials(edc_ctx* ctx, size_t g, const uint8_t* partials, int bad_any, uint8_t check8[32]) {
  if (!ctx || (g && !partials)) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  int rc = ensure_aux(ctx, g * 128 + 1);
  if (rc) return rc;
  if (g) CK(hipMemcpyAsync(ctx->aux, partials, g * 128, hipMemcpyHostToDevice, ctx->st));
  CK(hipMemsetAsync(ctx->d_out, 0, 256, ctx->st));
  launch_combine(ctx->st, (uint32_t)g, ctx->aux, bad_any ? 1 : 0, check8 != nullptr, ctx->d_out);
  CK(hipGetLastError());
  CK(hipMemcpyAsync(ctx->h_out, ctx->d_out, 256, hipMemcpyDeviceToHost, ctx->st));
  CK(hipStreamSynchronize(ctx->st));
  return verdict_from_out(ctx, check8);
}

int edc_challenge(edc_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg,
                  const uint64_t* msg_off, uint8_t* k_out) {
  if (!ctx || (n && !k_out)) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  int rc = upload(ctx, n, vk, sig, msg, msg_off);
  if (rc) return rc;
  if (!n) return 0;
  launch_challenge(ctx->st, (uint32_t)n, ctx->vk, ctx->sig, ctx->msg, ctx->off, ctx->k);
  CK(hipGetLastError());
  CK(hipMemcpyAsync(k_out, ctx->k, n * 32, hipMemcpyDeviceToHost, ctx->st));
  CK(hipStreamSynchronize(ctx->st));
  return 0;
}

int edc_verify_prehashed_each(edc_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* k,
                              uint8_t* verdicts) {
  if (!ctx || (n && (!vk || !sig || !k || !verdicts))) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  int rc = ensure_n(ctx, n);
  if (rc) return rc;
  if (!n) return 0;
  CK(hipMemcpyAsync(ctx->vk, vk, n * 32, hipMemcpyHostToDevice, ctx->st));
  CK(hipMemcpyAsync(ctx->sig, sig, n * 64, hipMemcpyHostToDevice, ctx->st));
  CK(hipMemcpyAsync(ctx->k, k, n * 32, hipMemcpyHostToDevice, ctx->st));
  launch_verify_single(ctx->st, (uint32_t)n, ctx->vk, ctx->sig, ctx->k, ctx->btab, ctx->verdicts);
  CK(hipGetLastError());
  CK(hipMemcpyAsync(verdicts, ctx->verdicts, n, hipMemcpyDeviceToHost, ctx->st));
  CK(hipStreamSynchronize(ctx->st));
  return 0;
}

int edc_verify_each(edc_ctx* ctx, size_t n, const uint8_t* vk, const uint8_t* sig, const uint8_t* msg,
                    const uint64_t* msg_off, uint8_t* verdicts) {
  if (!ctx || (n && !verdicts)) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  int rc = upload(ctx, n, vk, sig, msg, msg_off);
  if (rc) return rc;
  if (!n) return 0;
  launch_challenge(ctx->st, (uint32_t)n, ctx->vk, ctx->sig, ctx->msg, ctx->off, ctx->k);
  launch_verify_single(ctx->st, (uint32_t)n, ctx->vk, ctx->sig, ctx->k, ctx->btab, ctx->verdicts);
  CK(hipGetLastError());
  CK(hipMemcpyAsync(verdicts, ctx->verdicts, n, hipMemcpyDeviceToHost, ctx->st));
  CK(hipStreamSynchronize(ctx->st));
  return 0;
}

int edc_decompress(edc_ctx* ctx, size_t n, const uint8_t* enc, uint8_t* xy, uint8_t* ok) {
  if (!ctx || (n && (!enc || !xy || !ok))) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  int rc = ensure_n(ctx, n);
  if (rc) return rc;
  rc = ensure_aux(ctx, n * 64);
  if (rc) return rc;
  if (!n) return 0;
  CK(hipMemcpyAsync(ctx->vk, enc, n * 32, hipMemcpyHostToDevice, ctx->st));
  launch_decode(ctx->st, (uint32_t)n, ctx->vk, ctx->aux, ctx->verdicts);
  CK(hipGetLastError());
  CK(hipMemcpyAsync(xy, ctx->aux, n * 64, hipMemcpyDeviceToHost, ctx->st));
  CK(hipMemcpyAsync(ok, ctx->verdicts, n, hipMemcpyDeviceToHost, ctx->st));
  CK(hipStreamSynchronize(ctx->st));
  return 0;
}

int edc_sign_device(edc_ctx* ctx, size_t n, const uint8_t* d_seeds, const uint32_t* d_seed_index,
                    const uint8_t* d_msg, const uint64_t* d_msg_off, uint8_t* d_vk_out, uint8_t* d_sig_out) {
  if (!ctx) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  launch_sign(ctx->st, (uint32_t)n, d_seeds, d_seed_index, d_msg, d_msg_off, ctx->btab, d_vk_out, d_sig_out);
  CK(hipGetLastError());
  CK(hipStreamSynchronize(ctx->st));
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
  size_t sb = nseeds * 32, ib = seed_index ? n * 4 : 0;
  rc = ensure_aux(ctx, sb + ib + n * 96 + 64);
  if (rc) return rc;
  uint8_t* d_seeds = ctx->aux;
  uint32_t* d_idx = seed_index ? reinterpret_cast<uint32_t*>(ctx->aux + ((sb + 15) & ~(size_t)15)) : nullptr;
  uint8_t* d_vk = ctx->aux + ((sb + 15) & ~(size_t)15) + ((ib + 15) & ~(size_t)15);
  uint8_t* d_sig = d_vk + n * 32;
  CK(hipMemcpyAsync(d_seeds, seeds, sb, hipMemcpyHostToDevice, ctx->st));
  if (d_idx) CK(hipMemcpyAsync(d_idx, seed_index, ib, hipMemcpyHostToDevice, ctx->st));
  launch_sign(ctx->st, (uint32_t)n, d_seeds, d_idx, ctx->msg, ctx->off, ctx->btab, d_vk, d_sig);
  CK(hipGetLastError());
  CK(hipMemcpyAsync(vk_out, d_vk, n * 32, hipMemcpyDeviceToHost, ctx->st));
  CK(hipMemcpyAsync(sig_out, d_sig, n * 64, hipMemcpyDeviceToHost, ctx->st));
  CK(hipStreamSynchronize(ctx->st));
  return 0;
}

int edc_chacha_fill_device(edc_ctx* ctx, const uint8_t key[32], uint64_t blk0, uint64_t nblocks, uint8_t* d_out) {
  if (!ctx || !key || (nblocks && !d_out)) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  uint32_t k[8];
  seed_words(key, k);
  launch_chacha_fill(ctx->st, k, blk0, nblocks, reinterpret_cast<uint32_t*>(d_out));
  CK(hipGetLastError());
  CK(hipStreamSynchronize(ctx->st));
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

int edc_synchronize(edc_ctx* ctx) {
  if (!ctx) return EDC_ERR_ARG;
  CK(hipSetDevice(ctx->device));
  CK(hipStreamSynchronize(ctx->st));
  return 0;
}

}  // extern "C"
