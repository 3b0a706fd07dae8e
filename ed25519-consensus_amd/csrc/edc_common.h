// Shared device-side storage helpers and the workspace layout used by every kernel.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "fe25519.h"
#include "ge25519.h"
#include "sc25519.h"
#include "sha512.h"
#include "chacha20.h"
#include "keycache.h"

namespace edc {

// ---- HBM record layouts ----
// affine Niels point: ypx | ymx | xy2d as 9 radix-2^29 limbs each (27 words), padded to 32 words
// so that every record is exactly one 128-byte cache line: the MSM gathers points in random
// order, and a 112-byte record straddled two lines most of the time.
constexpr int NIELS_WORDS = 32;
// extended point: X | Y | Z | T, 36 words (144 B)
constexpr int EXT_WORDS = 36;

__device__ __forceinline__ fe ld_fe(const uint32_t* p) {
  fe r;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = p[i];
  return r;
}
__device__ __forceinline__ void st_fe(uint32_t* p, const fe& a) {
#pragma unroll
  for (int i = 0; i < 9; ++i) p[i] = a.v[i];
}

__device__ __forceinline__ ge_niels ld_niels(const uint32_t* base, uint32_t idx) {
  const uint4* q = reinterpret_cast<const uint4*>(base + (size_t)idx * NIELS_WORDS);
  uint32_t w[28];
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    uint4 t = q[i];
    w[4 * i] = t.x; w[4 * i + 1] = t.y; w[4 * i + 2] = t.z; w[4 * i + 3] = t.w;
  }
  ge_niels n;
#pragma unroll
  for (int i = 0; i < 9; ++i) { n.ypx.v[i] = w[i]; n.ymx.v[i] = w[9 + i]; n.xy2d.v[i] = w[18 + i]; }
  return n;
}
__device__ __forceinline__ void st_niels(uint32_t* base, uint32_t idx, const ge_niels& n) {
  uint32_t w[28];
#pragma unroll
  for (int i = 0; i < 9; ++i) { w[i] = n.ypx.v[i]; w[9 + i] = n.ymx.v[i]; w[18 + i] = n.xy2d.v[i]; }
  w[27] = 0;
  uint4* q = reinterpret_cast<uint4*>(base + (size_t)idx * NIELS_WORDS);
#pragma unroll
  for (int i = 0; i < 7; ++i) q[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
}

__device__ __forceinline__ ge_p3 ld_ext(const uint32_t* p) {
  ge_p3 r;
  r.X = ld_fe(p); r.Y = ld_fe(p + 9); r.Z = ld_fe(p + 18); r.T = ld_fe(p + 27);
  return r;
}
__device__ __forceinline__ void st_ext(uint32_t* p, const ge_p3& a) {
  st_fe(p, a.X); st_fe(p + 9, a.Y); st_fe(p + 18, a.Z); st_fe(p + 27, a.T);
}

__device__ __forceinline__ void ld_words8(const uint8_t* p, uint32_t w[8]) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  uint4 a = q[0], b = q[1];
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}

// ---- Pippenger plan: windows of the scalar bits, buckets, bins ----
// An MSM term is (point, scalar, range). Terms with a "short" scalar (the 128-bit z_i of R_i) use
// windows [0, nwin_short) only; full-width scalars (253-bit coefficients of B and the keys) use
// every window. Window w covers scalar bits [off[w], off[w] + bits[w]) as a signed digit
// (carry into the next window); the top short window is unsigned for short scalars (they have no
// window above it), so its digit can reach 2^bits when bits divides 128. Digit magnitude m >= 1
// goes to bucket m - 1; a bin is one slice of 256 consecutive buckets of one window of one range
// and is reduced by one workgroup. Ranges (>1 only in the grouped fallback) are independent MSMs
// over contiguous slices of the signatures.
constexpr int MSM_MAX_WIN = 32;
constexpr int SLICE_BITS = 8;      // 256 buckets per slice (one workgroup)
constexpr int NSLICE = 1 << SLICE_BITS;
constexpr uint32_t MSM_MAX_BINS = 8192;

struct MsmPlan {
  uint32_t nwin, nwin_short;
  uint32_t nranges;               // ranges (grouped fallback) or parts of one batch (sum_ranges)
  uint32_t sum_ranges;            // 1: the ranges are parts of ONE MSM, summed per window
  uint32_t bins_per_range;        // sum of nslice * nsub over the windows
  uint16_t off[MSM_MAX_WIN];      // first scalar bit of window w
  uint8_t bits[MSM_MAX_WIN];      // width of window w (<= 16)
  uint8_t nsub[MSM_MAX_WIN];      // sub-bins per slice of window w (power of 2; term t -> t mod nsub)
  uint16_t bin0[MSM_MAX_WIN];     // first bin of window w inside a range
  uint16_t nslice[MSM_MAX_WIN];   // slices of window w
  __host__ __device__ uint32_t nbin() const { return nranges * bins_per_range; }
};

// The terms of one MSM. Batch (rsize = 0): point terms t = 0..n+m (B, R_i, keys), in part
// t mod nparts (parts only spread a small batch over more workgroups; their sums are added per
// window; interleaved, so that each part holds the same mix of short z_i and full-width terms).
// Ranges (grouped fallback, rsize > 0): point terms t < npoint are R_i (t < n, point 1+t, range
// t / rsize) and, for one key term per signature, A_i (point 1+t, range (t-n) / rsize); then nx
// listed terms (point xpt, range xrg, scalar xscal): the per-(range, key) and per-range B terms.
struct MsmTerms {
  uint32_t n, rsize, npoint, nx;
  uint32_t nparts;                // batch split into nparts interleaved parts (nparts <= 1: one part)
  const uint32_t* scal;
  const uint32_t* xpt;
  const uint32_t* xrg;
  const uint32_t* xscal;
  uint32_t split;                 // batch with split coefficients (msm_num_points_split): all terms short
  // several batches in one launch (edc_batch_submit_multi_device): bit 0 set = the layout is
  // resolved on the device from the key grouping (flags): npoint = n (or 2n with one key term per
  // signature: bit 1 = per signature by the host's choice, or FLAG_OVF), nx = nranges * m + nranges
  // listed terms, where the host passes nranges in nx
  uint32_t dyn;
};

// signed digit of window w (bits <= 16) with carry in/out; top_unsigned keeps the raw value
__device__ __forceinline__ int plan_digit(const uint32_t s[8], uint32_t off, uint32_t bits, int& carry,
                                          bool top_unsigned) {
  const uint32_t k = off >> 5, sh = off & 31;
  const uint64_t two = (uint64_t)s[k] | ((uint64_t)(k < 7 ? s[k + 1] : 0u) << 32);
  const uint32_t raw = ((uint32_t)(two >> sh) & ((1u << bits) - 1u)) + (uint32_t)carry;
  if (top_unsigned) { carry = 0; return (int)raw; }
  if (raw >= (1u << (bits - 1))) { carry = 1; return (int)raw - (int)(1u << bits); }
  carry = 0;
  return (int)raw;
}

// 64-bit limb-sum accumulators per distinct key (12 limbs of a 128 x 256-bit product)
constexpr int KEY_ACC_LIMBS = 12;

// flags slot indices. FLAG_OVF: key grouping gave up (probe limit, section "Key grouping" of
// DESIGN.md): the batch continues with one key term per signature, which is the same group element.
// FLAG_UNCACHED: keys of the batch not found in the context's key cache (reported to the host,
// which only plans split coefficients while the previous batch had none).
// FLAG_KARG: a caller-supplied challenge k (prehashed entries) was not a canonical scalar (>= l):
// a broken caller contract, reported as EDC_ERR_ARG, never as a verdict.
enum { FLAG_BAD = 0, FLAG_NKEYS = 1, FLAG_VERDICT = 2, FLAG_OVF = 3, FLAG_UNCACHED = 4, FLAG_KARG = 5, FLAG_COUNT = 8 };
// A slot's flags array holds FLAG_ALLOC words: [0, FLAG_COUNT) the per-batch flags above (reset by
// k_init_batch), [FLAG_STAMP0, FLAG_STAMP0 + BST_N) the phase stamps of the EDC_BATCH_STAMPS
// diagnostic build (make variant VARIANT=bstamps VFLAGS=-DEDC_BATCH_STAMPS, tools/batch_timeline.py):
// workgroup 0 of each stamped kernel stores the 100 MHz realtime counter as it starts, k_msm_final
// copies them (and its own end) into words 48.. of the result block. Results are unchanged.
constexpr int FLAG_ALLOC = 32, FLAG_STAMP0 = 16;
enum { BST_INIT, BST_COEF, BST_COUNT, BST_DECODE, BST_ACCUM, BST_REDUCE, BST_FINAL, BST_END, BST_N };
#ifdef EDC_BATCH_STAMPS
#define BATCH_STAMP(fl, k)                                                                          \
  do {                                                                                              \
    if (blockIdx.x == 0 && threadIdx.x == 0 && (fl))                                                \
      const_cast<int*>(fl)[FLAG_STAMP0 + (k)] = (int)__builtin_amdgcn_s_memrealtime();              \
  } while (0)
#else
#define BATCH_STAMP(fl, k) do { } while (0)
#endif

// Points of a batch MSM: 0 = B, 1..n = R_i, n+1..n+m = the distinct keys (grouped) or each
// signature's own key (m = n, one key term per signature).
__host__ __device__ __forceinline__ uint32_t msm_num_points(uint32_t n, uint32_t m) { return 1 + n + m; }

// Split coefficients (a batch whose keys are all in the context's key cache): every 253-bit
// coefficient c of B and of the keys is written c = lo + 2^128 hi, lo on the point itself and hi on
// its [2^128] multiple, which the cache holds (comb[32][0] = [16^32]A). Every term is then at most
// 128 bits, the plan has no windows above bit 128 and the Horner chain is ~128 doublings instead of
// ~250. Points: 0 = B, 1..n = R_i, 1+n..n+m = A_j, 1+n+m = [2^128]B, 2+n+m+j = [2^128]A_j.
__host__ __device__ __forceinline__ uint32_t msm_num_points_split(uint32_t n, uint32_t m) { return 2 + n + 2 * m; }
__host__ __device__ __forceinline__ uint32_t split_hi_point(uint32_t n, uint32_t m, uint32_t j) { return 2 + n + m + j; }
__host__ __device__ __forceinline__ uint32_t split_b_hi_point(uint32_t n, uint32_t m) { return 1 + n + m; }

constexpr int BTAB_ENTRIES = 8;
// radix-256 comb of B behind the 8 multiples in the same table: entry 8 + 128 j + d - 1 =
// [d 256^j]B (j = 0..31, d = 1..128), affine Niels; the per-item kernels take [s]B from it with 32
// additions and no doublings (instead of 64 additions inside the doubling loop)
constexpr int B256_POS = 32, B256_MULT = 128, B256_ENTRIES = B256_POS * B256_MULT;
constexpr int BTAB_TOTAL = BTAB_ENTRIES + B256_ENTRIES;
constexpr uint32_t COEF_CHUNK = 2048;   // signatures per k_coef workgroup (range sizes are multiples)   // context table [1..8]B (per-item fallback, signer)

// Per-item failure bits written by the prefix kernels (the grouped fallback reads them).
enum { ITEM_BAD_S = 1, ITEM_BAD_R = 2 };

}  // namespace edc
