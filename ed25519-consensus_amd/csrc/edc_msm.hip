// Pippenger multi-scalar multiplication for the batch equation (K4)
//   check = [B_coeff]B + sum_keys [A_coeff]A + sum_i [z_i]R_i
// (reference src/batch.rs:205-210, EdwardsPoint::vartime_multiscalar_mul; any exact algorithm
// yields the same group element).
//
// The windows, buckets and bins follow an MsmPlan (edc_common.h) chosen per batch on the host:
// 128-bit z_i use the low windows only, full-width coefficients (B, keys) every window. Digits
// are binned by (range, window, slice of 256 buckets) by a count / scan / scatter pass
// (LDS-aggregated histograms, no global sort); each bin's workgroup counting-sorts its entries,
// accumulates its buckets with 7M mixed additions (segmented lanes, LDS-DMA row gathers); a
// lane-parallel pass reduces each bin to (sum_t (t+1) S_t, sum_t S_t). Windows with several slices combine them; a
// Horner pass per range joins the windows, multiplies by the cofactor and tests the identity
// (src/batch.rs:212-216). Ranges > 1 only in the grouped fallback: independent MSMs over
// contiguous slices of the signatures, one verdict each.
#include "edc_common.h"
#include "edc_launch.h"
#include "ge_quad.h"
#include "ge_row.h"

namespace edc {


// the multi-batch layout (MsmTerms::dyn) from the batch's key grouping
__device__ __forceinline__ MsmTerms resolve_terms(MsmTerms T, const int* flags) {
  if (T.dyn & 1u) {
    const bool per_sig = (T.dyn & 2u) || flags[FLAG_OVF];
    const uint32_t nr = T.nx, m = per_sig ? 0u : (uint32_t)flags[FLAG_NKEYS];
    T.npoint = per_sig ? 2 * T.n : T.n;
    T.nx = nr * m + nr;
  }
  return T;
}

__device__ __forceinline__ uint32_t terms_count(const MsmTerms& T, const int* flags) {
  if (T.rsize) return T.npoint + T.nx;
  const uint32_t m = (uint32_t)flags[FLAG_NKEYS];
  return T.split ? msm_num_points_split(T.n, m) : msm_num_points(T.n, m);
}

// term t -> point index, range, short scalar?, scalar words
__device__ __forceinline__ void term_get(const MsmTerms& T, uint32_t t, uint32_t& pt, uint32_t& rg, bool& shrt,
                                         uint32_t s[8]) {
  const uint32_t* src;
  if (!T.rsize) {
    pt = t;
    rg = T.nparts > 1 ? t % T.nparts : 0;   // interleaved: every part gets its share of R, keys and B
    shrt = T.split || (t >= 1 && t <= T.n);
    src = T.scal + (size_t)t * 8;
  } else if (t < T.npoint) {       // R_i (t < n), then one key term per signature
    pt = 1 + t;
    rg = (t < T.n ? t : t - T.n) / T.rsize;
    shrt = t < T.n;
    src = T.scal + (size_t)pt * 8;
  } else {                          // listed (range, key) and per-range B terms
    const uint32_t q = t - T.npoint;
    pt = T.xpt[q];
    rg = T.xrg[q];
    shrt = false;
    src = T.xscal + (size_t)q * 8;
  }
  const uint4* q4 = reinterpret_cast<const uint4*>(src);
  const uint4 a = q4[0], b = shrt ? make_uint4(0u, 0u, 0u, 0u) : q4[1];   // a z_i is 128 bits
  s[0] = a.x; s[1] = a.y; s[2] = a.z; s[3] = a.w; s[4] = b.x; s[5] = b.y; s[6] = b.z; s[7] = b.w;
}

// digits of term t: calls f(bin, local bucket, negative) for every non-zero digit. A term's top
// window is unsigned (nothing sits above it: bit 128 for a z_i, bit 253 for a coefficient < l);
// slice s of window w is split into nsub[w] sub-bins by term index.
template <typename F>
__device__ __forceinline__ void term_digits(const MsmPlan& P, uint32_t t, bool shrt, uint32_t rg, const uint32_t s[8],
                                            F&& f) {
  const uint32_t nw = shrt ? P.nwin_short : P.nwin;
  const uint32_t rbase = rg * P.bins_per_range;
  int carry = 0;
  for (uint32_t w = 0; w < nw; ++w) {
    const int d = plan_digit(s, P.off[w], P.bits[w], carry, w + 1 == nw);
    if (d) {
      const uint32_t b = (uint32_t)(d < 0 ? -d : d) - 1;
      const uint32_t ns = P.nsub[w];
      f(rbase + P.bin0[w] + (b >> SLICE_BITS) * ns + (t & (ns - 1)), b & (NSLICE - 1), d < 0);
    }
  }
}

__global__ void __launch_bounds__(256) k_msm_count(MsmPlan P, MsmTerms T, uint32_t per_block,
                                                   uint32_t* __restrict__ counts, const int* __restrict__ flags) {
  extern __shared__ uint32_t hist[];
  BATCH_STAMP(flags, BST_COUNT);
  const uint32_t nbin = P.nbin();
  for (uint32_t b = threadIdx.x; b < nbin; b += blockDim.x) hist[b] = 0;
  __syncthreads();
  T = resolve_terms(T, flags);
  const uint32_t cnt = terms_count(T, flags);
  const uint32_t t0 = blockIdx.x * per_block;
  for (uint32_t u = threadIdx.x; u < per_block; u += blockDim.x) {
    const uint32_t t = t0 + u;
    if (t >= cnt) break;
    uint32_t pt, rg, s[8];
    bool shrt;
    term_get(T, t, pt, rg, shrt, s);
    term_digits(P, t, shrt, rg, s, [&](uint32_t bin, uint32_t, bool) { atomicAdd(&hist[bin], 1u); });
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nbin; b += blockDim.x)
    if (hist[b]) atomicAdd(&counts[b], hist[b]);
}

// exclusive scan of nbin counts (one workgroup of 1024 lanes, consecutive bins per lane)
__global__ void __launch_bounds__(1024) k_msm_scan(uint32_t nbin, const uint32_t* __restrict__ counts,
                                                   uint32_t* __restrict__ offsets,
                                                   uint32_t* __restrict__ cursor) {
  __shared__ uint32_t part[1024];
  const uint32_t t = threadIdx.x;
  const uint32_t per = (nbin + 1023) / 1024;
  const uint32_t b0 = t * per, b1 = min(nbin, b0 + per);
  uint32_t s = 0;
  for (uint32_t b = b0; b < b1; ++b) s += counts[b];
  part[t] = s;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    uint32_t v = t >= (uint32_t)d ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - s;
  for (uint32_t b = b0; b < b1; ++b) {
    offsets[b] = run;
    cursor[b] = run;
    run += counts[b];
  }
}

// Scatter of every digit into its bin's run of `entries`. Pass 1 counts the workgroup's digits per
// bin; each bin's run is reserved with one global atomic. Staged path (the workgroup's entries fit
// its LDS stage, `stage_cap` > 0): pass 2 counting-sorts the entries by bin into the LDS stage
// (bin kept in .y's upper bits), then the workgroup writes the stage out in order, so consecutive
// lanes store consecutive entries of one run and every run leaves in whole-run wave stores
// instead of one 8-byte store per digit spread over pass 2 (the scattered stores re-opened
// partially written lines in L2: ~2.9x the entry bytes reached HBM). Direct path otherwise.
// Workgroup -> terms of the scatter. Batches with full-width terms use two regions, so that every
// workgroup's entries fit the LDS stage: region A holds the short terms 1..n (R_i, nwin_short
// digits each) at per_a terms per workgroup; region B the full-width terms (B, then the keys:
// term 0 and terms n+1.., all windows) at per_b = per_a * nwin_short / nwin. One region
// (grid_a = grid, a0 = 0) otherwise. Term t of a workgroup is its u-th: region A t = a0 + base + u
// (t < a_end); region B v = base + u, t = v ? b_base + v : 0.
struct ScatterBlocks {
  uint32_t grid_a, per_a, a0, a_end, per_b, b_base;
};
template <typename F>
__device__ __forceinline__ void scatter_terms(const ScatterBlocks& S, uint32_t cnt, F&& f) {
  if (blockIdx.x < S.grid_a) {
    const uint32_t t0 = S.a0 + blockIdx.x * S.per_a, lim = min(cnt, S.a_end);
    for (uint32_t u = threadIdx.x; u < S.per_a; u += blockDim.x) {
      if (t0 + u >= lim) break;
      f(t0 + u);
    }
  } else {
    const uint32_t v0 = (blockIdx.x - S.grid_a) * S.per_b;
    for (uint32_t u = threadIdx.x; u < S.per_b; u += blockDim.x) {
      const uint32_t v = v0 + u, t = v ? S.b_base + v : 0u;
      if (t >= cnt) break;
      f(t);
    }
  }
}

#ifndef EDC_SCATTER_THREADS
#define EDC_SCATTER_THREADS 1024
#endif
constexpr int SCATTER_THREADS = EDC_SCATTER_THREADS;
__global__ void __launch_bounds__(SCATTER_THREADS) k_msm_scatter(MsmPlan P, MsmTerms T, ScatterBlocks SB,
                                                     uint32_t* __restrict__ cursor, uint2* __restrict__ entries,
                                                     const int* __restrict__ flags, uint32_t stage_cap) {
  extern __shared__ uint32_t smem_hist[];
  __shared__ uint32_t wsum[SCATTER_THREADS / 64];
  const uint32_t nbin = P.nbin();
  uint32_t* hist = smem_hist;
  uint32_t* gbase = smem_hist + nbin;
  uint32_t* lbase = smem_hist + 2 * nbin;                                   // staged path only
  uint2* stage = reinterpret_cast<uint2*>(smem_hist + 3 * nbin + (nbin & 1));  // 8-byte aligned
  for (uint32_t b = threadIdx.x; b < nbin; b += blockDim.x) hist[b] = 0;
  __syncthreads();
  T = resolve_terms(T, flags);
  const uint32_t cnt = terms_count(T, flags);
  // pass 1: local counts (recomputed in pass 2 from the same digits)
  scatter_terms(SB, cnt, [&](uint32_t t) {
    uint32_t pt, rg, s[8];
    bool shrt;
    term_get(T, t, pt, rg, shrt, s);
    term_digits(P, t, shrt, rg, s, [&](uint32_t bin, uint32_t, bool) { atomicAdd(&hist[bin], 1u); });
  });
  __syncthreads();
  // reserve each bin's run; staged path: exclusive scan of the counts over the bins (each lane
  // takes a block of consecutive bins) into lbase, and the counters restart at lbase
  const uint32_t per_lane = (nbin + blockDim.x - 1) / blockDim.x;
  const uint32_t b0 = min(nbin, threadIdx.x * per_lane), b1 = min(nbin, b0 + per_lane);
  uint32_t mine = 0;
  for (uint32_t b = b0; b < b1; ++b) {
    const uint32_t c = hist[b];
    gbase[b] = c ? atomicAdd(&cursor[b], c) : 0u;
    mine += c;
  }
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t incl = mine;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t v = __shfl_up(incl, d, 64);
    if (lane >= (uint32_t)d) incl += v;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  uint32_t before = 0, total = 0;
  for (uint32_t k = 0; k < blockDim.x / 64; ++k) {
    if (k < wave) before += wsum[k];
    total += wsum[k];
  }
  const bool staged = total <= stage_cap;       // uniform over the workgroup
  uint32_t run = before + incl - mine;
  for (uint32_t b = b0; b < b1; ++b) {
    const uint32_t c = hist[b];
    if (staged) { lbase[b] = run; hist[b] = run; } else { hist[b] = 0; }
    run += c;
  }
  __syncthreads();
  scatter_terms(SB, cnt, [&](uint32_t t) {
    uint32_t pt, rg, s[8];
    bool shrt;
    term_get(T, t, pt, rg, shrt, s);
    term_digits(P, t, shrt, rg, s, [&](uint32_t bin, uint32_t local, bool neg) {
      const uint32_t r = atomicAdd(&hist[bin], 1u);
      if (staged) stage[r] = make_uint2(pt | (neg ? 0x80000000u : 0u), local | (bin << SLICE_BITS));
      else entries[gbase[bin] + r] = make_uint2(pt | (neg ? 0x80000000u : 0u), local);
    });
  });
  if (!staged) return;
  __syncthreads();
  for (uint32_t e = threadIdx.x; e < total; e += blockDim.x) {
    const uint2 v = stage[e];
    const uint32_t bin = v.y >> SLICE_BITS;
    entries[gbase[bin] + (e - lbase[bin])] = make_uint2(v.x, v.y & (NSLICE - 1));
  }
}

// ---- workgroup point reductions through LDS (quad-cooperative point arithmetic) ----
// weighted_sum_256: 256 extended points lds_pts[0..255], 256 lanes = 64 quads.
//   returns (sum_t t * P_t, sum_t P_t), valid in quad 0 (threads 0..3).
// Quad g folds points 4g..4g+3 (res_g = P1 + 2P2 + 3P3, run_g = sum), then a Hillis-Steele
// suffix scan of run over the 64 quads gives sum_g 4g run_g = 4 sum_{g>=1} Suf_g; two trees
// finish (R on quads 0-31, S on quads 32-63). Serial depth: 5 + 6 + 6 + 3 quad point ops. R and S are 64-point LDS scratch; they
// may alias lds_pts (every point is read before the first scratch write).
__device__ __forceinline__ void weighted_sum_256(const uint32_t* lds_pts, uint32_t* R, uint32_t* S, ge_p3& wsum, ge_p3& tot) {
  const int g = threadIdx.x >> 2;
  const bool leader = (threadIdx.x & 3) == 0;
  {
    ge_p3 run = quad_add(ld_ext(lds_pts + (4 * g + 3) * EXT_WORDS), ld_ext(lds_pts + (4 * g + 2) * EXT_WORDS));
    ge_p3 res = quad_add(run, ld_ext(lds_pts + (4 * g + 3) * EXT_WORDS));
    run = quad_add(run, ld_ext(lds_pts + (4 * g + 1) * EXT_WORDS));
    res = quad_add(res, run);
    run = quad_add(run, ld_ext(lds_pts + (4 * g + 0) * EXT_WORDS));
    __syncthreads();
    if (leader) { st_ext(R + g * EXT_WORDS, res); st_ext(S + g * EXT_WORDS, run); }
  }
  __syncthreads();
  // inclusive suffix scan of run over the 64 quads: S[g] = Suf_g
  for (int d = 1; d < 64; d <<= 1) {
    const bool has = g + d < 64;
    ge_p3 mine, other;
    if (has) { mine = ld_ext(S + g * EXT_WORDS); other = ld_ext(S + (g + d) * EXT_WORDS); }
    __syncthreads();
    if (has) {
      mine = quad_add(mine, other);
      if (leader) st_ext(S + g * EXT_WORDS, mine);
    }
    __syncthreads();
  }
  if (g == 0) tot = ld_ext(S);
  __syncthreads();
  if (g == 0 && leader) st_ext(S, ge_identity());   // sum_{g>=1} Suf_g
  // two trees at once: R (sum of res_g) on quads 0..31, S (sum of suffixes) on quads 32..63, so
  // each level is one quad addition deep (waves 0-1 take R, waves 2-3 take S: no divergence)
  const bool on_s = g >= 32;
  const int h = on_s ? g - 32 : g;
  uint32_t* const tree = on_s ? S : R;
  for (int d = 32; d >= 1; d >>= 1) {
    __syncthreads();
    ge_p3 x;
    if (h < d) x = quad_add(ld_ext(tree + h * EXT_WORDS), ld_ext(tree + (h + d) * EXT_WORDS));
    __syncthreads();   // every lane reaches both barriers: none sits in a divergent branch
    if (h < d && leader) st_ext(tree + h * EXT_WORDS, x);
  }
  __syncthreads();
  if (g == 0) wsum = quad_add(ld_ext(R), quad_dbl(quad_dbl(ld_ext(S))));
}

// plain sum of 256 extended points held one per lane (lane t has P_t); valid in quad 0.
__device__ __forceinline__ ge_p3 sum_256(const ge_p3& mine, uint32_t* scratch) {
  // stage, then quad g folds 4 points, then a 64-quad tree
  st_ext(scratch + threadIdx.x * EXT_WORDS, mine);
  __syncthreads();
  const int g = threadIdx.x >> 2;
  const bool leader = (threadIdx.x & 3) == 0;
  ge_p3 a = quad_add(quad_add(ld_ext(scratch + (4 * g) * EXT_WORDS), ld_ext(scratch + (4 * g + 1) * EXT_WORDS)),
                     quad_add(ld_ext(scratch + (4 * g + 2) * EXT_WORDS), ld_ext(scratch + (4 * g + 3) * EXT_WORDS)));
  for (int d = 32; d >= 1; d >>= 1) {
    __syncthreads();
    if (leader && g >= d && g < 2 * d) st_ext(scratch + (g - d) * EXT_WORDS, a);
    __syncthreads();
    if (g < d) a = quad_add(a, ld_ext(scratch + g * EXT_WORDS));
  }
  return a;
}

// ---- bucket accumulation with coalesced row gathers ----
// One workgroup per bin, one lane per bucket (buckets handed to lanes by decreasing entry count,
// so the lanes of a wave run about the same number of rounds). The bin's entries are counting-
// sorted by bucket through LDS counters into `sorted` (global, so a bin of any size is sorted in
// one pass and LDS stays free for the row buffers). Each round, every wave gathers the next Niels
// record of each of its 64 lanes with 7 LDS-DMA wave-instructions (global_load_lds_dwordx4):
// instruction k moves pieces 64k..64k+63 of the wave's 64 x 7 sixteen-byte pieces, i.e. whole
// 112-byte rows, 9-10 rows per instruction, instead of 64 scattered 16-byte pieces per load
// instruction as a row-per-lane register gather issues. Rows land row-major (112-byte stride:
// 28 words, odd multiple of 4 banks, so the row reads are conflict-free) and each lane reads its
// own row back.
constexpr int ROW_PIECES = 7;                        // 16-byte pieces of a record carrying data
constexpr int ROW_WORDS = ROW_PIECES * 4;            // 28
constexpr int WAVE_ROWS_WORDS = 64 * ROW_WORDS;      // 7 KB of LDS per wave

__device__ __forceinline__ void dma_piece(const uint32_t* gsrc, uint32_t* lds_wave_dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gsrc,
                                   (__attribute__((address_space(3))) void*)lds_wave_dst, 16, 0, 0);
}

__device__ __forceinline__ ge_niels ld_row_lds(const uint32_t* p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
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

// Lane balance (segmented accumulation): lane t takes the sorted positions [E t/256, E (t+1)/256)
// of its bin, so every lane runs the same number of rounds whatever the Poisson spread of the
// bucket sizes (one bucket per lane ran each workgroup as long as its largest bucket). A lane
// flushes its running sum whenever its positions cross a bucket end: a bucket that starts and
// ends inside the lane's range is stored whole; the partial of a bucket that began before the
// range ("head") goes to the lane's scratch slot; the lane holding a bucket's first entry adds the
// heads of the following lanes the bucket covers after a barrier and stores the bucket.
// Diagnostic build only (make variant VARIANT=stamps VFLAGS=-DEDC_STAMPS, tools/accum_stamps.py):
// per-workgroup shader-clock stamps of the accumulation's phases; results are unchanged.
#ifdef EDC_STAMPS
__device__ unsigned long long g_acc_stamps[MSM_MAX_BINS * 8];
#define ACC_STAMP(k, v) do { if (threadIdx.x == 0) g_acc_stamps[(size_t)blockIdx.x * 8 + (k)] = (v); } while (0)
#else
#define ACC_STAMP(k, v) do { } while (0)
#endif

__device__ __forceinline__ uint32_t* bucket_slot(uint32_t* buckets, uint32_t bin, uint32_t b) {
  return buckets + ((size_t)bin * NSLICE + b) * EXT_WORDS;
}

// Counting sort of each bin's entries by bucket (one workgroup per bin): the point indices (sign in
// bit 31) go out bucket by bucket, bucket_end[] gets the exclusive end position of every bucket,
// and empty buckets get the identity. The accumulation's lane t walks the sorted positions
// [lo_t, hi_t) = [E t / 256, E (t+1) / 256) one per round, so position q is stored LANE-MAJOR at
// sorted_slot(bin, q) = offsets[bin] + 256 bin + 256 j + t (t its lane, j = q - lo_t its round): a
// round's 64 lanes then read one contiguous 256-byte run of `sorted` instead of 64 words on 64
// lines (each lane re-reading its own line every round, which the row gathers evicted from L2
// in between). Each bin's region is padded to 256 x rounds slots: 256 more per bin in total. A kernel of its own, so the memory-bound sort of one
// batch overlaps the VALU-bound accumulation of another instead of idling the accumulation's CUs
// (every workgroup of a launch sorts at the same time).
// lane of the accumulation that owns sorted position q of a bin of E entries (lo_t <= q < hi_t
// with lo_t = (E t) >> 8): the largest t with lo_t <= q, which is floor((256 q + 255) / E) -- with
// E < 256 several lanes share one lo and only the last of them owns it. A float estimate of that
// quotient is within one of it; one exact step fixes it.
__device__ __forceinline__ uint32_t acc_lane_of(uint32_t q, uint32_t E, float invE) {
  uint32_t t = (uint32_t)(((float)q * 256.0f + 255.0f) * invE);
  t = t > 255u ? 255u : t;
  if ((uint32_t)(((uint64_t)E * t) >> 8) > q) --t;
  else if (t < 255u && (uint32_t)(((uint64_t)E * (t + 1)) >> 8) <= q) ++t;
  return t;
}
#ifndef EDC_SORT_LANE_MAJOR
#define EDC_SORT_LANE_MAJOR 1   // measurement knob: 0 = the round-5 position-major layout (A/B builds)
#endif
__device__ __forceinline__ uint32_t sorted_slot(uint32_t base, uint32_t q, uint32_t E, float invE) {
#if EDC_SORT_LANE_MAJOR
  const uint32_t t = acc_lane_of(q, E, invE);
  return base + 256u * (q - (uint32_t)(((uint64_t)E * t) >> 8)) + t;
#else
  return base + q;
#endif
}

#ifndef EDC_SORT_REG
#define EDC_SORT_REG 40
#endif
constexpr int SORT_REG = EDC_SORT_REG;               // entries per lane held in registers (0: two reads)
__global__ void __launch_bounds__(256) k_msm_sort(const uint32_t* __restrict__ counts,
                                                  const uint32_t* __restrict__ offsets,
                                                  const uint2* __restrict__ entries, uint32_t* __restrict__ sorted,
                                                  uint32_t* __restrict__ bucket_end, uint32_t* __restrict__ buckets) {
  __shared__ uint32_t lcnt[NSLICE];
  __shared__ uint32_t lcur[NSLICE];
  const int t = threadIdx.x;
  const uint32_t bin = blockIdx.x;
  const uint32_t E = counts[bin];
  if (E == 0) return;
  const uint32_t off = offsets[bin];
  const uint32_t tbase = off + 256u * bin;            // the bin's lane-major region
  const float invE = 1.0f / (float)E;
  lcnt[t] = 0;
  __syncthreads();
  // the first SORT_REG * 256 entries are read once and kept in registers for the second pass
  // (a 2^20 batch's bins hold ~8k entries); any beyond are read twice, in batches of 8
  uint2 reg[SORT_REG];
#pragma unroll
  for (int u = 0; u < SORT_REG; ++u)
    reg[u] = t + 256u * u < E ? entries[off + t + 256u * u] : make_uint2(0u, 0xFFFFFFFFu);
#pragma unroll
  for (int u = 0; u < SORT_REG; ++u)
    if (reg[u].y != 0xFFFFFFFFu) atomicAdd(&lcnt[reg[u].y], 1u);
  constexpr int SB = 8;
  for (uint32_t e0 = t + 256u * SORT_REG; e0 < E; e0 += 256 * SB) {
    uint32_t y[SB];
#pragma unroll
    for (int u = 0; u < SB; ++u) y[u] = e0 + 256u * u < E ? entries[off + e0 + 256u * u].y : 0xFFFFFFFFu;
#pragma unroll
    for (int u = 0; u < SB; ++u)
      if (y[u] != 0xFFFFFFFFu) atomicAdd(&lcnt[y[u]], 1u);
  }
  __syncthreads();
  if (t < 64) {
    uint32_t c[4], sum = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) { c[q] = lcnt[4 * t + q]; sum += c[q]; }
    uint32_t incl = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      uint32_t v = __shfl_up(incl, d, 64);
      if (t >= d) incl += v;
    }
    uint32_t run = incl - sum;
    uint32_t* be = bucket_end + (size_t)bin * NSLICE + 4 * t;
#pragma unroll
    for (int q = 0; q < 4; ++q) { lcur[4 * t + q] = run; run += c[q]; be[q] = run; }
  }
  __syncthreads();
  if (lcnt[t] == 0) st_ext(bucket_slot(buckets, bin, t), ge_identity());
#pragma unroll
  for (int u = 0; u < SORT_REG; ++u)
    if (reg[u].y != 0xFFFFFFFFu) sorted[sorted_slot(tbase, atomicAdd(&lcur[reg[u].y], 1u), E, invE)] = reg[u].x;
  for (uint32_t e0 = t + 256u * SORT_REG; e0 < E; e0 += 256 * SB) {
    uint2 en[SB];
#pragma unroll
    for (int u = 0; u < SB; ++u) en[u] = e0 + 256u * u < E ? entries[off + e0 + 256u * u] : make_uint2(0u, 0xFFFFFFFFu);
#pragma unroll
    for (int u = 0; u < SB; ++u)
      if (en[u].y != 0xFFFFFFFFu) sorted[sorted_slot(tbase, atomicAdd(&lcur[en[u].y], 1u), E, invE)] = en[u].x;
  }
}

#ifndef EDC_ACC_OCC
#define EDC_ACC_OCC 4
#endif
#ifndef EDC_ACC_HOIST
#define EDC_ACC_HOIST 0   // measurement knob: let the compiler hoist the DMA piece map (needs VGPRs)
#endif
#ifndef EDC_ACC_PROBE
#define EDC_ACC_PROBE 0   // measurement knob: 1 = no row gathers after the first round, 2 = no LDS row reads either
#endif
__global__ void __launch_bounds__(256, EDC_ACC_OCC) k_msm_accum_dma(const uint32_t* __restrict__ counts,
                                                                   const uint32_t* __restrict__ offsets,
                                                                   const uint32_t* __restrict__ sorted,
                                                                   const uint32_t* __restrict__ bucket_end,
                                                                   const uint32_t* __restrict__ pts,
                                                                   uint32_t* __restrict__ buckets,
                                                                   uint32_t* __restrict__ heads,
                                                                   uint32_t* __restrict__ slice_W,
                                                                   uint32_t* __restrict__ slice_T,
                                                                   int* __restrict__ stampf) {
  __shared__ uint32_t lend[NSLICE];                 // exclusive end position of each bucket
  BATCH_STAMP(stampf, BST_ACCUM);
#ifndef EDC_ACC_LDS_PAD
#define EDC_ACC_LDS_PAD 0   // measurement knob: extra LDS words per workgroup (caps workgroups per CU)
#endif
  __shared__ __attribute__((aligned(16))) uint32_t lbuf[4 * WAVE_ROWS_WORDS + EDC_ACC_LDS_PAD];   // row buffers of the 4 waves
  const int t = threadIdx.x;
  const int lane = t & 63, wv = t >> 6;
  const uint32_t bin = blockIdx.x;
  const uint32_t E = counts[bin];
  ACC_STAMP(0, __builtin_amdgcn_s_memtime());
  ACC_STAMP(5, __builtin_amdgcn_s_memrealtime());
  ACC_STAMP(7, E);
  if (E == 0) {
    if (t == 0) {
      st_ext(slice_W + (size_t)bin * EXT_WORDS, ge_identity());
      st_ext(slice_T + (size_t)bin * EXT_WORDS, ge_identity());
    }
    return;
  }
  const uint32_t off = offsets[bin];
  lend[t] = bucket_end[(size_t)bin * NSLICE + t];
  __syncthreads();
  ACC_STAMP(1, __builtin_amdgcn_s_memtime());
  const uint32_t lo = (uint32_t)(((uint64_t)E * t) >> 8), hi = (uint32_t)(((uint64_t)E * (t + 1)) >> 8);
  // bucket holding position lo: the first b with lend[b] > lo
  uint32_t cb = 0;
#pragma unroll
  for (int step = 128; step >= 1; step >>= 1)
    if (lend[cb + step - 1] <= lo) cb += step;
  cb = min(cb, (uint32_t)NSLICE - 1);              // lanes with an empty range (E < 256)
  const bool head0 = lo < hi && (cb ? lend[cb - 1] : 0u) < lo;   // first bucket began in an earlier lane
  bool in_head = head0;
  uint32_t cend = lend[cb];
  const uint32_t rounds = __builtin_amdgcn_readfirstlane(((uint64_t)E + 255) >> 8);
  uint32_t* wrows = lbuf + wv * WAVE_ROWS_WORDS;
  uint32_t* my_head = heads + ((size_t)bin * NSLICE + t) * EXT_WORDS;
  ge_p3 acc = ge_identity();
  // DMA piece map of this lane: instruction k moves piece g - 7 src of the wave's row
  // src = g / 7, g = 64 k + lane; the seven 6-bit src fields are packed in two registers
  uint32_t pmap0 = 0, pmap1 = 0;
#pragma unroll
  for (int k = 0; k < ROW_PIECES; ++k) {
    const uint32_t src = (64u * k + lane) / 7u;
    if (k < 5) pmap0 |= src << (6 * k); else pmap1 |= src << (6 * (k - 5));
  }
  // one round of row gathers: the wave's 64 rows (one per lane, `row`) -> wrows, row-major
  auto gather_rows = [&](uint32_t row) {
#if !EDC_ACC_HOIST
    asm volatile("" : "+v"(pmap0), "+v"(pmap1));   // unpacked each round, never hoisted (VGPRs)
#endif
#pragma unroll
    for (int k = 0; k < ROW_PIECES; ++k) {
      const uint32_t src = k < 5 ? (pmap0 >> (6 * k)) & 63u : (pmap1 >> (6 * (k - 5))) & 63u;
      const uint32_t piece = 64u * k + lane - 7u * src;
      const uint32_t r = (uint32_t)__shfl((int)row, (int)src, 64);
      dma_piece(pts + (size_t)r * NIELS_WORDS + piece * 4, wrows + k * 256);
    }
  };
  // software pipeline: the rows of round j + 1 are in flight while round j's addition runs
  // this lane's positions, lane-major (k_msm_sort): round j's index at srow[256 j]
#if EDC_SORT_LANE_MAJOR
  const uint32_t* srow = sorted + off + 256u * bin + t;
  constexpr uint32_t SSTEP = 256;
#else
  const uint32_t* srow = sorted + off + 256u * bin + lo;
  constexpr uint32_t SSTEP = 1;
#endif
  uint32_t e = lo < hi ? srow[0] : 0u;
  uint32_t e_next = lo + 1 < hi ? srow[SSTEP] : e;
  gather_rows(e & 0x7FFFFFFFu);
#if EDC_ACC_PROBE >= 2
  __builtin_amdgcn_s_waitcnt(0x0F70);
  const ge_niels q0 = ld_row_lds(wrows + lane * ROW_WORDS);
#endif
  for (uint32_t j = 0; j < rounds; ++j) {
    const uint32_t pos = lo + j;
    if (pos < hi && pos == cend) {                 // the running bucket ended: flush it
      st_ext(in_head ? my_head : bucket_slot(buckets, bin, cb), acc);
      acc = ge_identity();
      in_head = false;
      do { ++cb; } while (lend[cb] <= pos);        // skip empty buckets
      cend = lend[cb];
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);            // vmcnt(0): round j's rows are in LDS
#if EDC_ACC_PROBE >= 2                             // measurement builds only (wrong results)
    ge_niels q = q0;
#else
    ge_niels q = ld_row_lds(wrows + lane * ROW_WORDS);
#endif
    __builtin_amdgcn_s_waitcnt(0xC07F);            // lgkmcnt(0): row in VGPRs before the refill
#if EDC_ACC_PROBE == 0
    if (j + 1 < rounds) gather_rows(e_next & 0x7FFFFFFFu);   // lanes past their range re-read a row
#endif
    const uint32_t e_cur = e;
    e = e_next;
    if (pos + 2 < hi) e_next = srow[SSTEP * (j + 2)];
    if (pos < hi) {
      acc = ge_madd_sgn(acc, q, (e_cur >> 31) != 0);
    }
  }
  ACC_STAMP(2, __builtin_amdgcn_s_memtime());
  // the open segment: a head partial, a whole bucket ending at hi, or the first part of a bucket
  // that continues into the next lanes
  const bool owns_open = lo < hi && !in_head;
  const bool continues = owns_open && cend > hi;
  if (lo < hi && in_head) st_ext(my_head, acc);
  if (owns_open && !continues) st_ext(bucket_slot(buckets, bin, cb), acc);
  __syncthreads();   // heads visible to the owners
  if (continues) {
    for (uint32_t u = t + 1; u < NSLICE; ++u) {
      const uint32_t lo_u = (uint32_t)(((uint64_t)E * u) >> 8), hi_u = (uint32_t)(((uint64_t)E * (u + 1)) >> 8);
      if (lo_u < hi_u) acc = ge_add(acc, ld_ext(heads + ((size_t)bin * NSLICE + u) * EXT_WORDS));  // lanes
      if (cend <= hi_u) break;                     // with an empty range (E < 256) hold no head
    }
    st_ext(bucket_slot(buckets, bin, cb), acc);
  }
  ACC_STAMP(3, __builtin_amdgcn_s_memtime());
  ACC_STAMP(6, __builtin_amdgcn_s_memrealtime());
}

// ---- bin reduction: W = sum_t (t+1) S_t and T = sum_t S_t over a bin's 256 bucket sums ----
// Lane-parallel (every lane adds its own points; quad-cooperative arithmetic would spend a whole
// wave-instruction on 16 additions instead of 64): L lanes per bin, 256 / L consecutive buckets
// per lane, 64 / L bins per wave. Lane j runs the chunk's running sums from the top bucket down
// (s_j = sum_i B_i, r_j = sum_i (i+1) B_i), then the lanes of a bin combine through shuffles:
// sum_t (t+1) B_t = sum_j r_j + (256 / L) * sum_{j>=1} Suf_j with Suf_j = sum_{k>=j} s_k (a suffix
// scan), and T = Suf_0. L = 32 for large batches (least work: 1-2 workgroups per CU anyway);
// L = 64 when there are few bins and the serial depth (2 * 256 / L + 2 log2 L + log2(256 / L)
// additions) is the latency of the whole pass.
template <int L>
__device__ __forceinline__ fe shfl_down_fe(const fe& a, int d) {
  fe r;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = (uint32_t)__shfl_down((int)a.v[i], d, L);
  return r;
}
template <int L>
__device__ __forceinline__ ge_p3 shfl_down_pt(const ge_p3& P, int d) {
  return ge_p3{shfl_down_fe<L>(P.X, d), shfl_down_fe<L>(P.Y, d), shfl_down_fe<L>(P.Z, d), shfl_down_fe<L>(P.T, d)};
}

template <int L>
__global__ void __launch_bounds__(256) k_msm_reduce(uint32_t nbin, const uint32_t* __restrict__ counts,
                                                    const uint32_t* __restrict__ buckets,
                                                    uint32_t* __restrict__ slice_W, uint32_t* __restrict__ slice_T,
                                                    int* __restrict__ stampf) {
  BATCH_STAMP(stampf, BST_REDUCE);
  constexpr int CHUNK = NSLICE / L;
  const uint32_t bin = blockIdx.x * (256 / L) + threadIdx.x / L;
  const int j = (int)(threadIdx.x % L);
  const bool live = bin < nbin && counts[bin] != 0;     // empty bins: the accumulation wrote W = T = 0
  ge_p3 run = ge_identity(), acc = ge_identity();
  if (live) {
    const uint32_t* base = buckets + ((size_t)bin * NSLICE + (size_t)j * CHUNK) * EXT_WORDS;
    ge_p3 nxt = ld_ext(base + (CHUNK - 1) * EXT_WORDS);
    run = nxt;
    acc = nxt;
    for (int i = CHUNK - 2; i >= 0; --i) {
      const ge_p3 cur = ld_ext(base + i * EXT_WORDS);
      run = ge_add(run, cur);
      acc = ge_add(acc, run);
    }
  }
  // suffix scan of s_j = run over the bin's lanes (all lanes of a wave take part in the shuffles)
  ge_p3 suf = run;
  for (int d = 1; d < L; d <<= 1) {
    const ge_p3 o = shfl_down_pt<L>(suf, d);
    if (j + d < L) suf = ge_add(suf, o);
  }
  // x_j = r_j + CHUNK * Suf_j (j >= 1), x_0 = r_0; then the sum over the bin's lanes
  ge_p3 x = acc;
  if (j >= 1) {
    ge_p3 y = suf;
    for (int k = 1; k < CHUNK; k <<= 1) y = ge_dbl(y);
    x = ge_add(x, y);
  }
  for (int d = L / 2; d >= 1; d >>= 1) {
    const ge_p3 o = shfl_down_pt<L>(x, d);
    if (j < d) x = ge_add(x, o);
  }
  if (live && j == 0) {
    st_ext(slice_W + (size_t)bin * EXT_WORDS, x);
    st_ext(slice_T + (size_t)bin * EXT_WORDS, suf);
  }
}

// Bin reduction for few bins (small batches, where it is latency): one workgroup per bin, its 64
// quads run the cooperative weighted sum over the bin's 256 bucket sums (serial depth 26 quad
// additions of 2 multiplication rounds each, instead of ~20 one-lane additions of 9 rounds).
// About 4x the instructions of k_msm_reduce, so large batches keep the lane-parallel form.
constexpr uint32_t REDUCE_QUAD_MAX_BINS = 128;
// synchronous calls: up to what one round of k_msm_reduce_quad workgroups holds (143 VGPRs: 3
// per CU, 768 on 256 CUs); past it a second round costs more than the lane-parallel form (measured:
// configs[2]'s 1,040 bins 1.83 vs 1.79 ms per call, 2^17's 592 bins 0.54 vs 0.56 ms, profiles/r05)
#ifndef EDC_REDUCE_QUAD_LATENCY_MAX_BINS
#define EDC_REDUCE_QUAD_LATENCY_MAX_BINS 768u
#endif
constexpr uint32_t REDUCE_QUAD_LATENCY_MAX_BINS = EDC_REDUCE_QUAD_LATENCY_MAX_BINS;
#ifndef EDC_REDUCE64_MAX_BINS
#define EDC_REDUCE64_MAX_BINS 256
#endif
constexpr uint32_t REDUCE64_MAX_BINS = EDC_REDUCE64_MAX_BINS;   // 64 lanes per bin below this many bins
// lanes per bin from that many bins up. 16 lanes do the least VALU work (672 point additions per
// bin against 864 with 32) but double the serial depth: one configs[2] batch's reduction 102 ->
// 139 us (rocprof, one batch at a time) for a pipelined rate within noise (+0.3 %,
// profiles/r05/r05y_reduce16_vs_32_ab.log), so 32
#ifndef EDC_REDUCE_WIDE_LANES
#define EDC_REDUCE_WIDE_LANES 32
#endif
constexpr int REDUCE_WIDE_LANES = EDC_REDUCE_WIDE_LANES;
__global__ void __launch_bounds__(256) k_msm_reduce_quad(const uint32_t* __restrict__ counts,
                                                         const uint32_t* __restrict__ buckets,
                                                         uint32_t* __restrict__ slice_W, uint32_t* __restrict__ slice_T,
                                                         int* __restrict__ stampf) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  BATCH_STAMP(stampf, BST_REDUCE);
  const uint32_t bin = blockIdx.x;
  if (counts[bin] == 0) return;                     // the accumulation wrote W = T = 0
  const int t = threadIdx.x;
  st_ext(smem + t * EXT_WORDS, ld_ext(buckets + ((size_t)bin * NSLICE + t) * EXT_WORDS));
  __syncthreads();
  __builtin_amdgcn_s_setprio(3);
  ge_p3 ws, tot;
  weighted_sum_256(smem, smem, smem + 64 * EXT_WORDS, ws, tot);   // (sum_t t B_t, sum_t B_t)
  if (t < 4) {
    const ge_p3 W = quad_add(ws, tot);              // sum_t (t + 1) B_t
    if (t == 0) {
      st_ext(slice_W + (size_t)bin * EXT_WORDS, W);
      st_ext(slice_T + (size_t)bin * EXT_WORDS, tot);
    }
  }
}

// Win(range g, window w) = sum_s W_s + 256 * sum_s s T_s over the window's slices, for windows
// with more than one slice (single-slice windows are read straight from their bin): one
// 256-lane workgroup, `smem` = kReduceLds bytes of LDS.
__device__ __forceinline__ bool window_needs_combine(const MsmPlan& P, uint32_t w) {
  return P.nslice[w] * P.nsub[w] > 1 || P.sum_ranges;
}
__device__ __forceinline__ void window_combine(const MsmPlan& P, uint32_t g, uint32_t w, const uint32_t* __restrict__ slice_W,
                                               const uint32_t* __restrict__ slice_T, uint32_t* __restrict__ win,
                                               uint32_t* smem) {
  const uint32_t ns = P.nslice[w], nsub = P.nsub[w];
  const int t = threadIdx.x;
  const uint32_t b0 = g * P.bins_per_range + P.bin0[w];
  // slice t's sums: its sub-bins, and the parts of one batch (sum_ranges), are added first
  ge_p3 sT = ge_identity(), sW = ge_identity();
  if ((uint32_t)t < ns) {
    const uint32_t np = P.sum_ranges ? P.nranges : 1u;
    for (uint32_t p = 0; p < np; ++p)
      for (uint32_t u = 0; u < nsub; ++u) {
        const size_t b = (P.sum_ranges ? (size_t)p * P.bins_per_range + P.bin0[w] : b0) + (size_t)t * nsub + u;
        const ge_p3 T = ld_ext(slice_T + b * EXT_WORDS), W = ld_ext(slice_W + b * EXT_WORDS);
        if (p == 0 && u == 0) { sT = T; sW = W; } else { sT = ge_add(sT, T); sW = ge_add(sW, W); }
      }
  }
  uint32_t* lpts = smem;
  st_ext(lpts + t * EXT_WORDS, sT);
  __syncthreads();
  ge_p3 ws, tot;
  weighted_sum_256(lpts, lpts, lpts + 64 * EXT_WORDS, ws, tot);  // R/S scratch aliases the consumed points
  __syncthreads();
  ge_p3 a = sum_256(sW, lpts);
  __syncthreads();   // sum_256's last reads of lpts are done
  if (t == 0) { st_ext(lpts, ws); st_ext(lpts + EXT_WORDS, a); }
  __syncthreads();
  if (t < 64) {      // 2^8 ws + a on wave 0's limb-sliced point (ge_row.h)
    const RowCtx c = row_ctx();
    const uint32_t bq = row_cached(c, lpts + EXT_WORDS, row_d2(c));
    uint32_t x = row_ld_ext(c, lpts);
    for (int k = 0; k < SLICE_BITS; ++k) x = row_dbl(c, x);
    row_st_ext(c, win + ((size_t)g * MSM_MAX_WIN + w) * EXT_WORDS, row_add(c, x, bq));
  }
}

// One workgroup per (range, window) (grouped fallback ranges).
__global__ void __launch_bounds__(256) k_msm_window(MsmPlan P, const uint32_t* __restrict__ slice_W,
                                                    const uint32_t* __restrict__ slice_T, uint32_t* __restrict__ win) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t g = blockIdx.x / P.nwin, w = blockIdx.x % P.nwin;
  if (!window_needs_combine(P, w)) return;
  __builtin_amdgcn_s_setprio(3);   // latency-bound tail: issue ahead of co-resident bulk waves
  window_combine(P, g, w, slice_W, slice_T, win, smem);
}

__device__ __forceinline__ void fe_to_bytes32(const fe& a, uint8_t* out) {
  uint32_t w[8];
  fe_to_words(a, w);
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int b = 0; b < 4; ++b) out[4 * j + b] = (uint8_t)(w[j] >> (8 * b));
}

__device__ __forceinline__ void ext_to_canonical_bytes(const ge_p3& P, uint8_t* out) {
  fe_to_bytes32(P.X, out);
  fe_to_bytes32(P.Y, out + 32);
  fe_to_bytes32(P.Z, out + 64);
  fe_to_bytes32(P.T, out + 96);
}

__device__ __forceinline__ fe fe_from_bytes32(const uint8_t* in) {
  uint32_t w[8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
    w[j] = (uint32_t)in[4 * j] | ((uint32_t)in[4 * j + 1] << 8) | ((uint32_t)in[4 * j + 2] << 16) |
           ((uint32_t)in[4 * j + 3] << 24);
  return fe_from_words(w);
}

__device__ __forceinline__ ge_p3 ext_from_canonical_bytes(const uint8_t* in) {
  ge_p3 P;
  P.X = fe_from_bytes32(in);
  P.Y = fe_from_bytes32(in + 32);
  P.Z = fe_from_bytes32(in + 64);
  P.T = fe_from_bytes32(in + 96);
  return P;
}

// result block (device): [0] verdict, [1] bad flag, [2..] pad; bytes 16..48 check8, 48..176 partial
__device__ void finish_point(const ge_p3& check, int bad, int want_compress, uint8_t* out) {
  ext_to_canonical_bytes(check, out + 48);
  ge_p3 c8 = ge_mul_by_cofactor(check);
  bool ident = ge_is_identity(c8);
  reinterpret_cast<int*>(out)[0] = (!bad && ident) ? 0 : 1;
  reinterpret_cast<int*>(out)[1] = bad;
  if (want_compress) {
    uint32_t w[8];
    ge_compress(c8, w);
    for (int j = 0; j < 8; ++j)
      for (int b = 0; b < 4; ++b) out[16 + 4 * j + b] = (uint8_t)(w[j] >> (8 * b));
  }
}

// window sum of (range g, window w): combined by k_msm_window, or the single bin's W
__device__ __forceinline__ const uint32_t* window_ptr(const MsmPlan& P, uint32_t g, uint32_t w, const uint32_t* slice_W,
                                                      const uint32_t* win) {
  if (P.nslice[w] * P.nsub[w] > 1 || P.sum_ranges) return win + ((size_t)g * MSM_MAX_WIN + w) * EXT_WORDS;
  return slice_W + (size_t)(g * P.bins_per_range + P.bin0[w]) * EXT_WORDS;
}

// Horner over the windows of range g, sum_w 2^off[w] Win_w, on the wave's limb-sliced point
// (ge_row.h: ~890 cycles per doubling against ~1980 on a quad). `cached` holds the second-operand
// form of every window but the top one (row_cached, one word per lane, 64 words per window);
// returns Win and [8]Win in `res` (two extended points, X | Y | Z | T).
__device__ __forceinline__ void horner_row(const RowCtx& c, const MsmPlan& P, uint32_t g, const uint32_t* slice_W,
                                           const uint32_t* win, const uint32_t* cached, uint32_t* res,
                                           const uint32_t* from = nullptr, uint32_t from_w = 0) {
  // from: the Horner value after windows from_w..nwin-1 (k_msm_window2), else start at the top
  const uint32_t lane = threadIdx.x & 63;
  uint32_t acc = row_ld_ext(c, from ? from : window_ptr(P, g, P.nwin - 1, slice_W, win));
  for (int w = (from ? (int)from_w : (int)P.nwin - 1) - 1; w >= 0; --w) {
    const uint32_t bq = cached[w * 64 + lane];
    for (uint32_t k = 0; k < P.bits[w]; ++k) acc = row_dbl(c, acc);
    acc = row_add(c, acc, bq);
  }
  row_st_ext(c, res, acc);
  acc = row_dbl(c, row_dbl(c, row_dbl(c, acc)));
  row_st_ext(c, res + EXT_WORDS, acc);
}

// second-operand forms of range g's windows 0..nwin-2 into cached[] by the workgroup's `nwave` waves
__device__ __forceinline__ void cache_windows(const RowCtx& c, const MsmPlan& P, uint32_t g, const uint32_t* slice_W,
                                              const uint32_t* win, uint32_t* cached, uint32_t wave, uint32_t nwave,
                                              uint32_t upto = MSM_MAX_WIN) {
  const uint32_t d2 = row_d2(c), lane = threadIdx.x & 63;
  for (uint32_t w = wave; w + 1 < P.nwin && w < upto; w += nwave)
    cached[w * 64 + lane] = row_cached(c, window_ptr(P, g, w, slice_W, win), d2);
}

// batch: Horner, x8, identity (requires Z != 0), optional compression, partial point. Four waves
// form the windows' addition operands, then wave 0 runs the serial chain. The 256-byte result
// block is assembled in LDS and stored whole to `out` (device) and, when given, to `hout` (the
// slot's pinned host mirror, written through the device mapping: no copy packet per batch).
__global__ void __launch_bounds__(256) k_msm_final(MsmPlan P, const uint32_t* __restrict__ slice_W,
                                                   const uint32_t* __restrict__ win, const int* __restrict__ flags,
                                                   int want_compress, uint8_t* __restrict__ out,
                                                   uint8_t* __restrict__ hout, const uint32_t* __restrict__ from,
                                                   uint32_t from_w) {
  __shared__ uint32_t cached[MSM_MAX_WIN * 64];
  __shared__ uint32_t res[2 * EXT_WORDS];
  __shared__ uint32_t blk[64];
  if (blockIdx.x != 0) return;
  __builtin_amdgcn_s_setprio(3);   // a serial chain: issue ahead of co-resident bulk waves
  BATCH_STAMP(flags, BST_FINAL);
  const RowCtx c = row_ctx();
  const uint32_t wave = threadIdx.x >> 6;
  if (threadIdx.x < 64) blk[threadIdx.x] = 0;
  cache_windows(c, P, 0, slice_W, win, cached, wave, 4, from ? from_w : MSM_MAX_WIN);
  __syncthreads();
  if (wave == 0) horner_row(c, P, 0, slice_W, win, cached, res, from, from_w);
  __syncthreads();
  if (threadIdx.x == 0) {
    // a batch rejected by its bad flag (undecodable R / key, s >= l) reports the identity as its
    // partial and check point: the MSM sum then holds an off-curve point, whose value depends on
    // the order the additions ran in, and a public output must be the same on every run
    const int bad = flags[FLAG_BAD];
    const ge_p3 acc = bad ? ge_identity() : ld_ext(res), c8 = bad ? ge_identity() : ld_ext(res + EXT_WORDS);
    uint8_t* b = reinterpret_cast<uint8_t*>(blk);
    ext_to_canonical_bytes(acc, b + 48);
    blk[0] = (!bad && ge_is_identity(c8)) ? 0u : 1u;
    blk[1] = (uint32_t)bad;
    blk[2] = (uint32_t)flags[FLAG_NKEYS];   // distinct keys seen (adaptive grouping)
    blk[3] = (uint32_t)flags[FLAG_OVF];
    blk[44] = (uint32_t)flags[FLAG_UNCACHED];   // byte 176, after the partial point
    blk[45] = (uint32_t)flags[FLAG_KARG];       // byte 180: a caller's k was not canonical
    if (want_compress) ge_compress(c8, blk + 4);   // bytes 16..48 (little-endian words)
#ifdef EDC_BATCH_STAMPS
    for (int k = 0; k < BST_END; ++k) blk[48 + k] = (uint32_t)flags[FLAG_STAMP0 + k];
    blk[48 + BST_END] = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    reinterpret_cast<uint32_t*>(out)[threadIdx.x] = blk[threadIdx.x];
    if (hout) {
      reinterpret_cast<uint32_t*>(hout)[threadIdx.x] = blk[threadIdx.x];
      __threadfence_system();   // visible to the host once the stream's completion is observed
    }
  }
}

// Batch tail with the top-run Horner overlapped (plans whose top windows need no combine: for
// vote batches the 16 single-bin 8-bit windows of bits 128..252, ~125 doublings). k_msm_window2
// runs nwin + 1 workgroups: 0..nwin-1 combine the windows that have several slices, the extra one
// runs the Horner over windows r..nwin-1 into `hbuf` at the same time; k_msm_final then continues
// the Horner from hbuf over windows r-1..0. Serial depth: max(window combine, top-run Horner) +
// the rest of the Horner, instead of their sum. (A single launch with an arrival counter needs an
// L2 writeback per workgroup for the hand-off and measured slower.)
__host__ __device__ __forceinline__ uint32_t top_run_start(const MsmPlan& P) {
  uint32_t r = P.nwin;
  while (r > 0 && !(P.nslice[r - 1] * P.nsub[r - 1] > 1 || P.sum_ranges)) --r;
  return r;
}
__global__ void __launch_bounds__(256) k_msm_window2(MsmPlan P, const uint32_t* __restrict__ slice_W,
                                                     const uint32_t* __restrict__ slice_T, uint32_t* __restrict__ win,
                                                     uint32_t* __restrict__ hbuf) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  __builtin_amdgcn_s_setprio(3);
  if (blockIdx.x < P.nwin) {
    if (window_needs_combine(P, blockIdx.x)) window_combine(P, 0, blockIdx.x, slice_W, slice_T, win, smem);
    return;
  }
  const uint32_t r = top_run_start(P);
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t* cached = smem;                              // windows r..nwin-2, 64 words each
  const RowCtx c = row_ctx();
  const uint32_t d2 = row_d2(c);
  for (uint32_t w = r + wave; w + 1 < P.nwin; w += 4) cached[w * 64 + lane] = row_cached(c, window_ptr(P, 0, w, slice_W, win), d2);
  __syncthreads();
  if (wave != 0) return;
  uint32_t acc = row_ld_ext(c, window_ptr(P, 0, P.nwin - 1, slice_W, win));
  for (int w = (int)P.nwin - 2; w >= (int)r; --w) {
    const uint32_t bq = cached[w * 64 + lane];
    for (uint32_t k = 0; k < P.bits[w]; ++k) acc = row_dbl(c, acc);
    acc = row_add(c, acc, bq);
  }
  row_st_ext(c, hbuf, acc);
}

// ranges: rverdict[g] = 0 iff [8] * (range g's check point) is the identity; one wave per range
__global__ void __launch_bounds__(64) k_msm_range_final(MsmPlan P, const uint32_t* __restrict__ slice_W,
                                                        const uint32_t* __restrict__ win,
                                                        uint8_t* __restrict__ rverdict) {
  __shared__ uint32_t cached[MSM_MAX_WIN * 64];
  __shared__ uint32_t res[2 * EXT_WORDS];
  const uint32_t g = blockIdx.x;
  if (g >= P.nranges) return;
  __builtin_amdgcn_s_setprio(3);
  const RowCtx c = row_ctx();
  cache_windows(c, P, g, slice_W, win, cached, 0, 1);
  horner_row(c, P, g, slice_W, win, cached, res);
  __syncthreads();
  if (threadIdx.x == 0) rverdict[g] = ge_is_identity(ld_ext(res + EXT_WORDS)) ? 0 : 1;
}

// Several batches in one launch: range g's Horner, x8, identity -> result block g (the layout of
// k_msm_final's, at out + 256 g and, when given, hout + 256 g): verdict, bad flag (its range's
// failed decodes / s checks, rbad[g]), check8, partial point. One workgroup per range.
__global__ void __launch_bounds__(64) k_msm_multi_final(MsmPlan P, const uint32_t* __restrict__ slice_W,
                                                        const uint32_t* __restrict__ win, const int* __restrict__ flags,
                                                        const uint8_t* __restrict__ rbad, int want_compress,
                                                        uint8_t* __restrict__ out, uint8_t* __restrict__ hout) {
  __shared__ uint32_t cached[MSM_MAX_WIN * 64];
  __shared__ uint32_t res[2 * EXT_WORDS];
  __shared__ uint32_t blk[64];
  const uint32_t g = blockIdx.x;
  if (g >= P.nranges) return;
  __builtin_amdgcn_s_setprio(3);
  const RowCtx c = row_ctx();
  blk[threadIdx.x] = 0;
  cache_windows(c, P, g, slice_W, win, cached, 0, 1);
  horner_row(c, P, g, slice_W, win, cached, res);
  __syncthreads();
  if (threadIdx.x == 0) {
    const int bad = rbad[g] ? 1 : 0;     // rejected by its bad flag: identity (see k_msm_final)
    const ge_p3 acc = bad ? ge_identity() : ld_ext(res), c8 = bad ? ge_identity() : ld_ext(res + EXT_WORDS);
    ext_to_canonical_bytes(acc, reinterpret_cast<uint8_t*>(blk) + 48);
    blk[0] = (!bad && ge_is_identity(c8)) ? 0u : 1u;
    blk[1] = (uint32_t)bad;
    blk[2] = (uint32_t)flags[FLAG_NKEYS];
    blk[3] = (uint32_t)flags[FLAG_OVF];
    blk[44] = (uint32_t)flags[FLAG_UNCACHED];
    blk[45] = (uint32_t)flags[FLAG_KARG];
    if (want_compress) ge_compress(c8, blk + 4);
  }
  __syncthreads();
  reinterpret_cast<uint32_t*>(out + 256 * (size_t)g)[threadIdx.x] = blk[threadIdx.x];
  if (hout) {
    reinterpret_cast<uint32_t*>(hout + 256 * (size_t)g)[threadIdx.x] = blk[threadIdx.x];
    __threadfence_system();
  }
}

// combine G partial check points (canonical 128-byte records) from G shards
__global__ void k_combine(uint32_t g, const uint8_t* __restrict__ partials, int bad,
                          int want_compress, uint8_t* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  ge_p3 acc = ge_identity();
  for (uint32_t i = 0; i < g; ++i) acc = ge_add(acc, ext_from_canonical_bytes(partials + 128 * (size_t)i));
  finish_point(acc, bad, want_compress, out);
}

// combine the result blocks of g shards (256-byte blocks: int[1] bad flag, bytes 48..176 the
// canonical partial point), as the pipelined multi-device path gathers them device to device
__global__ void k_combine_blocks(uint32_t g, const uint8_t* __restrict__ blocks, int want_compress,
                                 uint8_t* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  ge_p3 acc = ge_identity();
  int bad = 0;
  for (uint32_t i = 0; i < g; ++i) {
    acc = ge_add(acc, ext_from_canonical_bytes(blocks + 256 * (size_t)i + 48));
    bad |= reinterpret_cast<const int*>(blocks + 256 * (size_t)i)[1];
  }
  for (int j = 0; j < 64; ++j) reinterpret_cast<int*>(out)[j] = 0;
  finish_point(acc, bad, want_compress, out);
}

// combine g exchange records (stride bytes apart: canonical 128-byte partial, then the bad byte),
// as the multi-rank all-gather leaves them in device memory
__global__ void k_combine_records(uint32_t g, const uint8_t* __restrict__ recs, uint32_t stride,
                                  uint8_t* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  ge_p3 acc = ge_identity();
  int bad = 0;
  for (uint32_t i = 0; i < g; ++i) {
    acc = ge_add(acc, ext_from_canonical_bytes(recs + (size_t)stride * i));
    bad |= recs[(size_t)stride * i + 128] ? 1 : 0;
  }
  for (int j = 0; j < 64; ++j) reinterpret_cast<int*>(out)[j] = 0;
  finish_point(acc, bad, 0, out);
}

// one shard's 256-byte result block to the first device's gather buffer (a peer store over xGMI
// when the devices differ): a kernel on the shard's stream, so the copy stays asynchronous
__global__ void k_copy_block(const uint4* __restrict__ src, uint4* __restrict__ dst) {
  if (threadIdx.x < 16) dst[threadIdx.x] = src[threadIdx.x];
}

// ---------------------------------------------------------------- launchers
static inline uint32_t cdiv(uint64_t a, uint32_t b) { return (uint32_t)((a + b - 1) / b); }
static constexpr size_t kScatterLdsMax = 160 * 1024 - 256;   // k_msm_scatter's dynamic LDS ceiling
// entries of the scatter's LDS stage (process-wide; edc_debug_set_scatter_stage lowers it so that
// tests can drive the direct-store path, which the default stage covers only at large bin counts)
#ifndef EDC_SCATTER_STAGE
#define EDC_SCATTER_STAGE 16384   // measurement knob (A/B builds); the debug entry lowers it at run time
#endif
static uint32_t g_scatter_stage_max = EDC_SCATTER_STAGE;
extern "C" int edc_debug_set_scatter_stage(uint32_t max_entries) {
  g_scatter_stage_max = max_entries > 16384 ? 16384u : max_entries;
  return 0;
}

void launch_msm_bin(hipStream_t st, const MsmPlan& P, const MsmTerms& T, uint32_t max_terms, uint32_t* counts,
                    uint32_t* offsets, uint32_t* cursor, uint2* entries, const int* flags, bool counts_zeroed) {
  const uint32_t nbin = P.nbin();
  if (!counts_zeroed) (void)hipMemsetAsync(counts, 0, nbin * sizeof(uint32_t), st);
  // terms per workgroup: up to 4096 (long runs of entries per bin for the scatter's writes), but
  // at least ~256 workgroups so small batches still fill the GPU
  uint32_t per = max_terms / 256;
  per = per < 256 ? 256 : (per > 4096 ? 4096 : (per + 255) / 256 * 256);
  // the scatter's LDS stage: what is left of 160 KB after three per-bin arrays, at most 16k
  // entries; terms per workgroup then sized so that every workgroup's digits fit it (ScatterBlocks)
  const size_t lds_max = kScatterLdsMax, bins_bytes = (3 * (size_t)nbin + 1) * sizeof(uint32_t);
  uint32_t stage_cap = bins_bytes + 2048 * sizeof(uint2) <= lds_max
                           ? (uint32_t)std::min<size_t>(g_scatter_stage_max, (lds_max - bins_bytes) / sizeof(uint2) / 256 * 256)
                           : 0u;
  const uint32_t grid = cdiv(max_terms ? max_terms : 1, per);
  ScatterBlocks SB{grid, per, 0u, 0xFFFFFFFFu, per, 0u};
  uint32_t sgrid = grid;
  if (stage_cap) {
    const auto fit = [&](uint32_t digits) { return stage_cap / std::max(1u, digits) / 256 * 256; };
    const uint32_t fa = fit(P.nwin_short), fb = fit(P.nwin);
    if (!T.rsize && !T.split && P.nwin > P.nwin_short && fa >= 256 && fb >= 256) {   // batch: short region, then full-width
      SB.per_a = std::min(per, fa);
      SB.per_b = std::min(per, fb);
      SB.a0 = 1;
      SB.a_end = 1 + T.n;
      SB.b_base = T.n;
      SB.grid_a = cdiv(T.n ? T.n : 1, SB.per_a);
      sgrid = SB.grid_a + cdiv(max_terms > T.n ? max_terms - T.n : 1, SB.per_b);
    } else if (fa >= 256 && per > fa) {
      SB.per_a = SB.per_b = fa;
      SB.grid_a = sgrid = cdiv(max_terms ? max_terms : 1, fa);
    }
  }
#ifndef EDC_COUNT_SPLIT
#define EDC_COUNT_SPLIT 4
#endif
  // the count pass needs no long runs: EDC_COUNT_SPLIT times the scatter's workgroups (at 2^20, 257
  // workgroups of 4096 terms leave one workgroup per CU, latency-bound: 49.5 us; 1,025 of 1024
  // terms 34.0 us; past ~2,000 the per-workgroup flush of the bin counts to global atomics costs
  // more, 84 us at 4,097; profiles/r05/r05ar, r05as)
  const uint32_t cper = std::max(256u, per / EDC_COUNT_SPLIT);
  hipLaunchKernelGGL(k_msm_count, dim3(cdiv(max_terms ? max_terms : 1, cper)), dim3(256), nbin * sizeof(uint32_t), st, P, T,
                     cper, counts, flags);
  hipLaunchKernelGGL(k_msm_scan, dim3(1), dim3(1024), 0, st, nbin, counts, offsets, cursor);
#ifdef EDC_PROBE_EXTRA_SCANS   // measurement only: N more (idempotent) dependent launches per batch
  for (int r = 0; r < EDC_PROBE_EXTRA_SCANS; ++r)
    hipLaunchKernelGGL(k_msm_scan, dim3(1), dim3(1024), 0, st, nbin, counts, offsets, cursor);
#endif
  hipLaunchKernelGGL(k_msm_scatter, dim3(sgrid), dim3(SCATTER_THREADS), bins_bytes + (size_t)stage_cap * sizeof(uint2), st, P, T,
                     SB, cursor, entries, flags, stage_cap);
}

hipError_t msm_init_device() {
  return hipFuncSetAttribute(reinterpret_cast<const void*>(&k_msm_scatter), hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)kScatterLdsMax);
}

static const size_t kReduceLds = (size_t)NSLICE * EXT_WORDS * sizeof(uint32_t);  // 256 points; scans reuse them

void launch_msm_sort(hipStream_t st, const MsmPlan& P, const uint32_t* counts, const uint32_t* offsets,
                     const uint2* entries, uint32_t* sorted, uint32_t* bucket_end, uint32_t* buckets) {
  hipLaunchKernelGGL(k_msm_sort, dim3(P.nbin()), dim3(256), 0, st, counts, offsets, entries, sorted, bucket_end, buckets);
}

void launch_msm_bucket(hipStream_t st, const MsmPlan& P, const uint32_t* counts, const uint32_t* offsets,
                       const uint2* entries, uint32_t* sorted, uint32_t* bucket_end, const uint32_t* pts,
                       uint32_t* buckets, uint32_t* heads, uint32_t* slice_W, uint32_t* slice_T, int probe_skip,
                       hipEvent_t acc_begin, hipEvent_t acc_end, bool latency, int* stamp_flags) {
  // one workgroup per bin (accumulation of the entries k_msm_sort ordered), then the bin
  // reductions (probe_skip: timing-probe builds only, edc_api.hip EDC_PROBE_SKIP; 0 in the product)
  if (acc_begin) (void)hipEventRecord(acc_begin, st);      // timed batches: the accumulation alone
  if (!(probe_skip & 32))
    hipLaunchKernelGGL(k_msm_accum_dma, dim3(P.nbin()), dim3(256), 0, st, counts, offsets, sorted, bucket_end, pts,
                       buckets, heads, slice_W, slice_T, stamp_flags);
  if (acc_end) (void)hipEventRecord(acc_end, st);
  if (probe_skip & 64) return;
  // latency: one synchronous batch on an idle GPU (edc_batch_verify*): the quad-cooperative weighted
  // sum (one workgroup per bin) has ~1/3 of the lane-parallel form's serial instruction count per
  // wave -- a lone wave issues one VALU instruction per ~5.5 cycles whatever its dependencies --
  // at ~2x its VALU work, which only the pipelined submissions (other batches to overlap) mind
  if (P.nbin() <= REDUCE_QUAD_MAX_BINS || (latency && P.nbin() <= REDUCE_QUAD_LATENCY_MAX_BINS))
    hipLaunchKernelGGL(k_msm_reduce_quad, dim3(P.nbin()), dim3(256), kReduceLds, st, counts, buckets, slice_W, slice_T,
                       stamp_flags);
  else if (P.nbin() < REDUCE64_MAX_BINS)
    hipLaunchKernelGGL(k_msm_reduce<64>, dim3(cdiv(P.nbin(), 4)), dim3(256), 0, st, P.nbin(), counts, buckets, slice_W,
                       slice_T, stamp_flags);
  else
    hipLaunchKernelGGL(k_msm_reduce<REDUCE_WIDE_LANES>, dim3(cdiv(P.nbin(), 256 / REDUCE_WIDE_LANES)), dim3(256), 0, st,
                       P.nbin(), counts, buckets, slice_W, slice_T, stamp_flags);
}

#ifdef EDC_STAMPS
extern "C" int edc_debug_acc_stamps(void* out, size_t bytes) {
  if (bytes > sizeof(g_acc_stamps)) bytes = sizeof(g_acc_stamps);
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_acc_stamps), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

size_t msm_bucket_words(uint32_t nbin) { return (size_t)nbin * NSLICE * EXT_WORDS; }

static bool plan_multi(const MsmPlan& P) {
  for (uint32_t w = 0; w < P.nwin; ++w)
    if (P.nslice[w] * P.nsub[w] > 1) return true;
  return false;
}

void launch_msm_tail(hipStream_t st, const MsmPlan& P, const uint32_t* slice_W, const uint32_t* slice_T,
                     uint32_t* win, int* flags, int want_compress, uint8_t* out, uint8_t* hout) {
  const uint32_t r = top_run_start(P);
  if (plan_multi(P) && r < P.nwin && r > 0 && P.nwin < MSM_MAX_WIN) {
    // window combines beside the top-run Horner; hbuf = the unused last window record of range 0
    uint32_t* hbuf = win + (size_t)(MSM_MAX_WIN - 1) * EXT_WORDS;
    hipLaunchKernelGGL(k_msm_window2, dim3(P.nwin + 1), dim3(256), kReduceLds, st, P, slice_W, slice_T, win, hbuf);
    hipLaunchKernelGGL(k_msm_final, dim3(1), dim3(256), 0, st, P, slice_W, win, flags, want_compress, out, hout,
                       (const uint32_t*)hbuf, r);
    return;
  }
  if (plan_multi(P) || P.sum_ranges)
    hipLaunchKernelGGL(k_msm_window, dim3(P.nwin), dim3(256), kReduceLds, st, P, slice_W, slice_T, win);
  hipLaunchKernelGGL(k_msm_final, dim3(1), dim3(256), 0, st, P, slice_W, win, flags, want_compress, out, hout,
                     (const uint32_t*)nullptr, 0u);
}

void launch_msm_range_tail(hipStream_t st, const MsmPlan& P, const uint32_t* slice_W, const uint32_t* slice_T,
                           uint32_t* win, uint8_t* rverdict) {
  if (plan_multi(P))
    hipLaunchKernelGGL(k_msm_window, dim3(P.nwin * P.nranges), dim3(256), kReduceLds, st, P, slice_W, slice_T, win);
  hipLaunchKernelGGL(k_msm_range_final, dim3(P.nranges), dim3(64), 0, st, P, slice_W, win, rverdict);
}

void launch_msm_multi_tail(hipStream_t st, const MsmPlan& P, const uint32_t* slice_W, const uint32_t* slice_T,
                           uint32_t* win, const int* flags, const uint8_t* rbad, int want_compress, uint8_t* out,
                           uint8_t* hout) {
  if (plan_multi(P))
    hipLaunchKernelGGL(k_msm_window, dim3(P.nwin * P.nranges), dim3(256), kReduceLds, st, P, slice_W, slice_T, win);
  hipLaunchKernelGGL(k_msm_multi_final, dim3(P.nranges), dim3(64), 0, st, P, slice_W, win, flags, rbad, want_compress,
                     out, hout);
}

void launch_copy_block(hipStream_t st, const uint8_t* src, uint8_t* dst) {
  hipLaunchKernelGGL(k_copy_block, dim3(1), dim3(64), 0, st, reinterpret_cast<const uint4*>(src),
                     reinterpret_cast<uint4*>(dst));
}

void launch_combine_blocks(hipStream_t st, uint32_t g, const uint8_t* blocks, int want_compress, uint8_t* out) {
  hipLaunchKernelGGL(k_combine_blocks, dim3(1), dim3(64), 0, st, g, blocks, want_compress, out);
}

void launch_combine_records(hipStream_t st, uint32_t g, const uint8_t* recs, uint32_t stride, uint8_t* out) {
  hipLaunchKernelGGL(k_combine_records, dim3(1), dim3(64), 0, st, g, recs, stride, out);
}

void launch_combine(hipStream_t st, uint32_t g, const uint8_t* partials, int bad, int want_compress,
                    uint8_t* out) {
  hipLaunchKernelGGL(k_combine, dim3(1), dim3(64), 0, st, g, partials, bad, want_compress, out);
}

// entries of a plan: every term can put one digit in each of its windows
size_t msm_entry_capacity(const MsmPlan& P, size_t short_terms, size_t full_terms) {
  return (size_t)P.nwin_short * short_terms + (size_t)P.nwin * full_terms;
}

}  // namespace edc
