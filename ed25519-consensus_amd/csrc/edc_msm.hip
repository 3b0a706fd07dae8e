// Pippenger multi-scalar multiplication for the batch equation (K4)
//   check = [B_coeff]B + sum_keys [A_coeff]A + sum_i [z_i]R_i
// (reference src/batch.rs:205-210, EdwardsPoint::vartime_multiscalar_mul; any exact algorithm
// yields the same group element).
//
// Points p: 0 = B, 1..n = R_i (128-bit z, 8 windows, top digit unsigned up to 2^16),
//           n+1..n+m = distinct keys (253-bit, 16 signed windows); in few-key mode
//           (edc_common.h) B and the keys carry 128-bit halves and their [2^128] twins follow,
//           so every point has 8 windows.
// Buckets: signed radix-2^16 digits d, bucket |d| in window w. A bin = (window, slice of 256
// consecutive buckets) = one workgroup. Entries are binned by a count / scan / scatter pass
// (LDS-aggregated histograms, no global sort), then each bin's workgroup counting-sorts its
// entries in LDS, accumulates one bucket per lane with 7M mixed additions, and reduces its 256
// buckets to (sum_t (t+1) S_t, sum_t S_t). Windows combine slices; a final Horner pass joins
// windows, multiplies by the cofactor and tests the identity (src/batch.rs:212-216).
#include "edc_common.h"
#include "edc_launch.h"
#include "ge_quad.h"

namespace edc {

constexpr int CNT_PTS_PER_BLOCK = 4096;   // points per count/scatter workgroup

__device__ __forceinline__ void load_scalar(const uint32_t* scal, uint32_t p, uint32_t s[8]) {
  const uint4* q = reinterpret_cast<const uint4*>(scal + (size_t)p * 8);
  uint4 a = q[0], b = q[1];
  s[0] = a.x; s[1] = a.y; s[2] = a.z; s[3] = a.w; s[4] = b.x; s[5] = b.y; s[6] = b.z; s[7] = b.w;
}

__global__ void __launch_bounds__(256) k_msm_count(uint32_t n, const uint32_t* __restrict__ scal,
                                                   uint32_t* __restrict__ counts,
                                                   const int* __restrict__ flags) {
  __shared__ uint32_t hist[NBIN];
  for (int b = threadIdx.x; b < NBIN; b += blockDim.x) hist[b] = 0;
  __syncthreads();
  const uint32_t m = (uint32_t)flags[FLAG_NKEYS];
  const bool few = few_key_mode(n, m);
  const uint32_t npts = msm_num_points(n, m);
  const uint32_t p0 = blockIdx.x * CNT_PTS_PER_BLOCK;
  for (uint32_t t = threadIdx.x; t < CNT_PTS_PER_BLOCK; t += blockDim.x) {
    uint32_t p = p0 + t;
    if (p >= npts) break;
    uint32_t s[8];
    load_scalar(scal, p, s);
    const bool isR = msm_short_scalar(p, n, few);
    const int nwin = isR ? NWIN_Z : NWIN_FULL;
    int carry = 0;
    for (int w = 0; w < nwin; ++w) {
      int d = scalar_digit(s, w, carry, isR && w == NWIN_Z - 1);
      if (d) {
        uint32_t b = (uint32_t)(d < 0 ? -d : d) - 1;
        atomicAdd(&hist[w * NSLICE + (b >> SLICE_BITS)], 1u);
      }
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < NBIN; b += blockDim.x)
    if (hist[b]) atomicAdd(&counts[b], hist[b]);
}

// exclusive scan of NBIN counts (one workgroup of 1024 lanes, 4 bins per lane)
__global__ void __launch_bounds__(1024) k_msm_scan(const uint32_t* __restrict__ counts,
                                                   uint32_t* __restrict__ offsets,
                                                   uint32_t* __restrict__ cursor) {
  __shared__ uint32_t part[1024];
  const int t = threadIdx.x;
  uint32_t c[4], s = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) { c[j] = counts[4 * t + j]; s += c[j]; }
  part[t] = s;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    uint32_t v = t >= d ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - s;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    offsets[4 * t + j] = run;
    cursor[4 * t + j] = run;
    run += c[j];
  }
}

__global__ void __launch_bounds__(256) k_msm_scatter(uint32_t n, const uint32_t* __restrict__ scal,
                                                     uint32_t* __restrict__ cursor,
                                                     uint2* __restrict__ entries,
                                                     const int* __restrict__ flags) {
  __shared__ uint32_t hist[NBIN];
  __shared__ uint32_t gbase[NBIN];
  for (int b = threadIdx.x; b < NBIN; b += blockDim.x) hist[b] = 0;
  __syncthreads();
  const uint32_t m = (uint32_t)flags[FLAG_NKEYS];
  const bool few = few_key_mode(n, m);
  const uint32_t npts = msm_num_points(n, m);
  const uint32_t p0 = blockIdx.x * CNT_PTS_PER_BLOCK;
  // pass 1: local ranks (recomputed in pass 2 from the same digits)
  for (uint32_t t = threadIdx.x; t < CNT_PTS_PER_BLOCK; t += blockDim.x) {
    uint32_t p = p0 + t;
    if (p >= npts) break;
    uint32_t s[8];
    load_scalar(scal, p, s);
    const bool isR = msm_short_scalar(p, n, few);
    const int nwin = isR ? NWIN_Z : NWIN_FULL;
    int carry = 0;
    for (int w = 0; w < nwin; ++w) {
      int d = scalar_digit(s, w, carry, isR && w == NWIN_Z - 1);
      if (d) {
        uint32_t b = (uint32_t)(d < 0 ? -d : d) - 1;
        atomicAdd(&hist[w * NSLICE + (b >> SLICE_BITS)], 1u);
      }
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < NBIN; b += blockDim.x) {
    uint32_t c = hist[b];
    gbase[b] = c ? atomicAdd(&cursor[b], c) : 0u;
    hist[b] = 0;
  }
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < CNT_PTS_PER_BLOCK; t += blockDim.x) {
    uint32_t p = p0 + t;
    if (p >= npts) break;
    uint32_t s[8];
    load_scalar(scal, p, s);
    const bool isR = msm_short_scalar(p, n, few);
    const int nwin = isR ? NWIN_Z : NWIN_FULL;
    int carry = 0;
    for (int w = 0; w < nwin; ++w) {
      int d = scalar_digit(s, w, carry, isR && w == NWIN_Z - 1);
      if (d) {
        uint32_t b = (uint32_t)(d < 0 ? -d : d) - 1;
        uint32_t bin = w * NSLICE + (b >> SLICE_BITS);
        uint32_t r = atomicAdd(&hist[bin], 1u);
        entries[gbase[bin] + r] = make_uint2(p | (d < 0 ? 0x80000000u : 0u), b & (NSLICE - 1));
      }
    }
  }
}

// ---- workgroup point reductions through LDS (quad-cooperative point arithmetic) ----
// weighted_sum_256: 256 extended points lds_pts[0..255], 256 lanes = 64 quads.
//   returns (sum_t t * P_t, sum_t P_t), valid in quad 0 (threads 0..3).
// Quad g folds points 4g..4g+3 (res_g = P1 + 2P2 + 3P3, run_g = sum), then a Hillis-Steele
// suffix scan of run over the 64 quads gives sum_g 4g run_g = 4 sum_{g>=1} Suf_g; two trees
// finish. Serial depth: 5 + 6 + 2*6 + 3 quad point ops. R and S are 64-point LDS scratch; they
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
  // two trees: R (sum of res_g) and S (sum of suffixes), interleaved per step
  for (int d = 32; d >= 1; d >>= 1) {
    __syncthreads();
    ge_p3 x, y;
    if (g < d) {
      x = quad_add(ld_ext(R + g * EXT_WORDS), ld_ext(R + (g + d) * EXT_WORDS));
      y = quad_add(ld_ext(S + g * EXT_WORDS), ld_ext(S + (g + d) * EXT_WORDS));
    }
    __syncthreads();   // every lane reaches both barriers: none sits in a divergent branch
    if (g < d && leader) { st_ext(R + g * EXT_WORDS, x); st_ext(S + g * EXT_WORDS, y); }
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

constexpr int BKT_CHUNK = 4096;

// one workgroup per bin (window w, slice s) of 256 buckets: S_b for b = 256 s + t + 1.
// Entries are counting-sorted by local bucket in LDS (chunks of BKT_CHUNK). ACC_LANES lanes share
// a bucket (lane group (t, t + 256, ...) walks entries j = half, half + ACC_LANES, ...; the group
// is summed at the end), which shortens the serial chains of the dense bins. Bucket sizes are
// Poisson-distributed and a wave runs as long as its fullest lane, so buckets are handed to lanes
// in order of decreasing entry count. With ACC_PREFETCH the next Niels point is loaded under the
// current 7M mixed addition.
#ifndef EDC_ACC_LANES
#define EDC_ACC_LANES 1
#endif
#ifndef EDC_ACC_PREFETCH
#define EDC_ACC_PREFETCH 0
#endif
#ifndef EDC_ACC_WAVES
#define EDC_ACC_WAVES 4
#endif
constexpr int ACC_LANES = EDC_ACC_LANES;
constexpr int ACC_THREADS = ACC_LANES * NSLICE;

__global__ void __launch_bounds__(ACC_THREADS, EDC_ACC_WAVES) k_msm_accum(const uint32_t* __restrict__ counts,
                                                              const uint32_t* __restrict__ offsets,
                                                              const uint2* __restrict__ entries,
                                                              const uint32_t* __restrict__ pts,
                                                              uint32_t* __restrict__ buckets) {
  __shared__ uint32_t lidx[BKT_CHUNK];
  __shared__ uint32_t lcnt[NSLICE];
  __shared__ uint32_t lstart[NSLICE];
  __shared__ uint32_t lcur[NSLICE];
  __shared__ uint32_t lorder[NSLICE];   // bucket handled by lane group t (by decreasing count)
#if EDC_ACC_LANES > 1
  __shared__ __attribute__((aligned(16))) uint32_t lpart[NSLICE * EXT_WORDS];
#endif
  const int t = threadIdx.x;
  const int lane_b = t & (NSLICE - 1);  // bucket slot of this lane group
  const uint32_t half = (uint32_t)t >> 8;
  const uint32_t bin = blockIdx.x;
  const uint32_t E = counts[bin];
  if (E == 0) return;
  const uint32_t off = offsets[bin];
  ge_p3 acc = ge_identity();
  uint32_t my_bucket = lane_b;
  for (uint32_t c0 = 0; c0 < E; c0 += BKT_CHUNK) {
    const uint32_t ch = min((uint32_t)BKT_CHUNK, E - c0);
    if (t < NSLICE) lcnt[t] = 0;
    __syncthreads();
    for (uint32_t e = t; e < ch; e += ACC_THREADS) atomicAdd(&lcnt[entries[off + c0 + e].y], 1u);
    __syncthreads();
    if (t < 64) {
      uint32_t c[4], s = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) { c[j] = lcnt[4 * t + j]; s += c[j]; }
      uint32_t incl = s;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        uint32_t v = __shfl_up(incl, d, 64);
        if (t >= d) incl += v;
      }
      uint32_t run = incl - s;
#pragma unroll
      for (int j = 0; j < 4; ++j) { lstart[4 * t + j] = run; lcur[4 * t + j] = run; run += c[j]; }
    }
    if (c0 == 0 && t >= ACC_THREADS - NSLICE) {
      // rank bucket b by (count desc, index)
      const int b = t - (ACC_THREADS - NSLICE);
      const uint32_t mine = lcnt[b];
      uint32_t rank = 0;
      for (int u = 0; u < NSLICE; ++u) {
        const uint32_t o = lcnt[u];
        rank += (o > mine) || (o == mine && u < b);
      }
      lorder[rank] = b;
    }
    __syncthreads();
    if (c0 == 0) my_bucket = lorder[lane_b];
    for (uint32_t e = t; e < ch; e += ACC_THREADS) {
      uint2 en = entries[off + c0 + e];
      uint32_t pos = atomicAdd(&lcur[en.y], 1u);
      lidx[pos] = en.x;
    }
    __syncthreads();
    const uint32_t beg = lstart[my_bucket], cnt = lcnt[my_bucket];
#if EDC_ACC_PREFETCH
    if (half < cnt) {
      uint32_t e = lidx[beg + half];
      ge_niels q = ld_niels(pts, e & 0x7FFFFFFFu);
      for (uint32_t j = half; j < cnt; j += ACC_LANES) {
        const uint32_t e_next = (j + ACC_LANES < cnt) ? lidx[beg + j + ACC_LANES] : e;
        ge_niels q_next = ld_niels(pts, e_next & 0x7FFFFFFFu);
        if (e >> 31) q = ge_niels_neg(q);
        acc = ge_madd(acc, q);
        e = e_next;
        q = q_next;
      }
    }
#else
#if EDC_ACC_PROBE == 3      // measurement probe: LDS sort only, no accumulation (result wrong)
    if (cnt > 100000) acc.X.v[0] = lidx[beg];
#elif EDC_ACC_PROBE == 4    // measurement probe: accumulate unsorted entries straight from HBM
    for (uint32_t j = t; j < ch; j += ACC_THREADS) {
      const uint32_t e = entries[off + c0 + j].x;
      ge_niels q = ld_niels(pts, e & 0x7FFFFFFFu);
      if (e >> 31) q = ge_niels_neg(q);
      acc = ge_madd(acc, q);
    }
#else
    for (uint32_t j = half; j < cnt; j += ACC_LANES) {
      const uint32_t e = lidx[beg + j];
#endif
#if EDC_ACC_PROBE == 3 || EDC_ACC_PROBE == 4
    for (uint32_t j = 0; j < 0; ++j) {
      const uint32_t e = 0;
#endif
#if EDC_ACC_PROBE == 1      // measurement probe: gathers + sort only (result wrong)
      ge_niels q = ld_niels(pts, e & 0x7FFFFFFFu);
#pragma unroll
      for (int k = 0; k < 9; ++k) acc.X.v[k] ^= q.ypx.v[k] ^ q.ymx.v[k] ^ q.xy2d.v[k];
#elif EDC_ACC_PROBE == 2    // measurement probe: arithmetic only, no gather (result wrong)
      ge_niels q = ld_niels(pts, 1 + (e & 1));
      if (e >> 31) q = ge_niels_neg(q);
      acc = ge_madd(acc, q);
#else
      ge_niels q = ld_niels(pts, e & 0x7FFFFFFFu);
      if (e >> 31) q = ge_niels_neg(q);
      acc = ge_madd(acc, q);
#endif
    }
#endif
    __syncthreads();
  }
#if EDC_ACC_LANES > 1
  if (half) st_ext(lpart + lane_b * EXT_WORDS, acc);
  __syncthreads();
  if (half) return;
  acc = ge_add(acc, ld_ext(lpart + lane_b * EXT_WORDS));
#endif
  st_ext(buckets + ((size_t)bin * NSLICE + my_bucket) * EXT_WORDS, acc);
}

#ifndef EDC_ACC_DMA
#define EDC_ACC_DMA 1
#endif

// ---- bucket accumulation with coalesced row gathers (EDC_ACC_DMA) ----
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
__device__ __forceinline__ uint32_t* bucket_slot(uint32_t* buckets, uint32_t bin, uint32_t b) {
  return buckets + ((size_t)bin * NSLICE + b) * EXT_WORDS;
}

__global__ void __launch_bounds__(256, EDC_ACC_WAVES) k_msm_accum_dma(const uint32_t* __restrict__ counts,
                                                                   const uint32_t* __restrict__ offsets,
                                                                   const uint2* __restrict__ entries,
                                                                   uint32_t* __restrict__ sorted,
                                                                   const uint32_t* __restrict__ pts,
                                                                   uint32_t* __restrict__ buckets,
                                                                   uint32_t* __restrict__ heads,
                                                                   uint32_t* __restrict__ slice_W,
                                                                   uint32_t* __restrict__ slice_T) {
  __shared__ uint32_t lcnt[NSLICE];
  __shared__ uint32_t lend[NSLICE];                 // exclusive end position of each bucket
  __shared__ uint32_t lcur[NSLICE];
  // row buffers of the 4 waves during accumulation, then the 256 bucket sums for the reduction
  __shared__ __attribute__((aligned(16))) uint32_t lbuf[NSLICE * EXT_WORDS];
  static_assert(4 * WAVE_ROWS_WORDS <= NSLICE * EXT_WORDS, "row buffers fit the bucket image");
  const int t = threadIdx.x;
  const int lane = t & 63, wv = t >> 6;
  const uint32_t bin = blockIdx.x;
  const uint32_t E = counts[bin];
  if (E == 0) {
    if (t == 0) {
      st_ext(slice_W + (size_t)bin * EXT_WORDS, ge_identity());
      st_ext(slice_T + (size_t)bin * EXT_WORDS, ge_identity());
    }
    return;
  }
  const uint32_t off = offsets[bin];
  lcnt[t] = 0;
  __syncthreads();
  // counting sort by bucket; loads are batched 8 deep so the passes are not latency-bound
  constexpr int SB = 8;
  for (uint32_t e0 = t; e0 < E; e0 += 256 * SB) {
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
#pragma unroll
    for (int q = 0; q < 4; ++q) { lcur[4 * t + q] = run; run += c[q]; lend[4 * t + q] = run; }
  }
  __syncthreads();
  if (lcnt[t] == 0) st_ext(bucket_slot(buckets, bin, t), ge_identity());
  for (uint32_t e0 = t; e0 < E; e0 += 256 * SB) {
    uint2 en[SB];
#pragma unroll
    for (int u = 0; u < SB; ++u) en[u] = e0 + 256u * u < E ? entries[off + e0 + 256u * u] : make_uint2(0u, 0xFFFFFFFFu);
#pragma unroll
    for (int u = 0; u < SB; ++u)
      if (en[u].y != 0xFFFFFFFFu) sorted[off + atomicAdd(&lcur[en[u].y], 1u)] = en[u].x;
  }
  __syncthreads();   // workgroup-scope release/acquire: the sorted lists are read back below
  const uint32_t lo = (uint32_t)(((uint64_t)E * t) >> 8), hi = (uint32_t)(((uint64_t)E * (t + 1)) >> 8);
  // bucket holding position lo: the first b with lend[b] > lo
  uint32_t cb = 0;
#pragma unroll
  for (int step = 128; step >= 1; step >>= 1)
    if (lend[cb + step - 1] <= lo) cb += step;
  cb = min(cb, (uint32_t)NSLICE - 1);              // lanes with an empty range (E < 256)
  const bool head0 = lo < hi && lend[cb] - lcnt[cb] < lo;   // first bucket began in an earlier lane
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
#if EDC_ACC_PROBE == 5      // measurement probe: 64-byte rows (4 pieces, 4 DMA instructions)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t g = 64u * k + lane;
      const uint32_t r = (uint32_t)__shfl((int)row, (int)(g >> 2), 64);
      dma_piece(pts + (size_t)r * NIELS_WORDS + (g & 3) * 4, wrows + k * 256);
    }
    return;
#endif
    asm volatile("" : "+v"(pmap0), "+v"(pmap1));   // unpacked each round, never hoisted (VGPRs)
#pragma unroll
    for (int k = 0; k < ROW_PIECES; ++k) {
      const uint32_t src = k < 5 ? (pmap0 >> (6 * k)) & 63u : (pmap1 >> (6 * (k - 5))) & 63u;
      const uint32_t piece = 64u * k + lane - 7u * src;
      const uint32_t r = (uint32_t)__shfl((int)row, (int)src, 64);
      dma_piece(pts + (size_t)r * NIELS_WORDS + piece * 4, wrows + k * 256);
    }
  };
  // software pipeline: the rows of round j + 1 are in flight while round j's addition runs
  uint32_t e = lo < hi ? sorted[off + lo] : 0u;
  uint32_t e_next = lo + 1 < hi ? sorted[off + lo + 1] : e;
#if EDC_ACC_PROBE != 2 && EDC_ACC_PROBE != 6
  gather_rows(e & 0x7FFFFFFFu);
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
#if EDC_ACC_PROBE == 2 || EDC_ACC_PROBE == 6   // measurement probes: no gather (result wrong)
    ge_niels q = ld_niels(pts, 1 + (e & 1));
#else
    __builtin_amdgcn_s_waitcnt(0x0F70);            // vmcnt(0): round j's rows are in LDS
    ge_niels q = ld_row_lds(wrows + lane * ROW_WORDS);
    __builtin_amdgcn_s_waitcnt(0xC07F);            // lgkmcnt(0): row in VGPRs before the refill
    if (j + 1 < rounds) gather_rows(e_next & 0x7FFFFFFFu);   // lanes past their range re-read a row
#endif
    const uint32_t e_cur = e;
    e = e_next;
    if (pos + 2 < hi) e_next = sorted[off + pos + 2];
    if (pos < hi) {
#if EDC_ACC_PROBE == 1 || EDC_ACC_PROBE == 5 || EDC_ACC_PROBE == 6   // probes: no addition (result wrong)
#pragma unroll
      for (int k = 0; k < 9; ++k) acc.X.v[k] ^= q.ypx.v[k] ^ q.ymx.v[k] ^ q.xy2d.v[k];
#else
      if (e_cur >> 31) q = ge_niels_neg(q);
      acc = ge_madd(acc, q);
#endif
    }
  }
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
  // the bin's reduction (fused: its latency-bound steps overlap the other workgroups of the CU)
  // W = sum_t (t+1) S_t and T = sum_t S_t over the 256 bucket sums (quad-cooperative)
  __syncthreads();   // every bucket of the bin is stored
  st_ext(lbuf + t * EXT_WORDS, ld_ext(bucket_slot(buckets, bin, t)));
  __syncthreads();
  ge_p3 ws, tot;
  weighted_sum_256(lbuf, lbuf, lbuf + 64 * EXT_WORDS, ws, tot);  // R/S scratch aliases the consumed points
  if (t < 4) {
    ge_p3 W = quad_add(ws, tot);       // sum_t (t+1) S_t = sum_t t S_t + sum_t S_t
    if (t == 0) {
      st_ext(slice_W + (size_t)bin * EXT_WORDS, W);
      st_ext(slice_T + (size_t)bin * EXT_WORDS, tot);
    }
  }
}

// one workgroup per bin: W_s = sum_t (t+1) S_t and T_s = sum_t S_t (quad-cooperative)
__global__ void __launch_bounds__(256) k_msm_reduce(const uint32_t* __restrict__ counts,
                                                    const uint32_t* __restrict__ buckets,
                                                    uint32_t* __restrict__ slice_W,
                                                    uint32_t* __restrict__ slice_T) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int t = threadIdx.x;
  const uint32_t bin = blockIdx.x;
  if (counts[bin] == 0) {
    if (t == 0) {
      st_ext(slice_W + (size_t)bin * EXT_WORDS, ge_identity());
      st_ext(slice_T + (size_t)bin * EXT_WORDS, ge_identity());
    }
    return;
  }
  uint32_t* lpts = smem;
  st_ext(lpts + t * EXT_WORDS, ld_ext(buckets + ((size_t)bin * NSLICE + t) * EXT_WORDS));
  __syncthreads();
  ge_p3 ws, tot;
  weighted_sum_256(lpts, lpts, lpts + 64 * EXT_WORDS, ws, tot);  // R/S scratch aliases the consumed points
  if (t < 4) {
    ge_p3 W = quad_add(ws, tot);       // sum_t (t+1) S_t = sum_t t S_t + sum_t S_t
    if (t == 0) {
      st_ext(slice_W + (size_t)bin * EXT_WORDS, W);
      st_ext(slice_T + (size_t)bin * EXT_WORDS, tot);
    }
  }
}

// one workgroup per window: Win_w = sum_s W_s + 256 * sum_s s T_s
// (a window without entries -- windows 8..15 in few-key mode -- is skipped; FLAG_WINMASK records
// the non-empty ones for the Horner pass)
__global__ void __launch_bounds__(256) k_msm_window(const uint32_t* __restrict__ counts,
                                                    const uint32_t* __restrict__ slice_W,
                                                    const uint32_t* __restrict__ slice_T,
                                                    uint32_t* __restrict__ win, int* __restrict__ flags) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int t = threadIdx.x;
  const uint32_t w = blockIdx.x;
  if (!__syncthreads_or(counts[w * NSLICE + t] != 0)) return;
  if (t == 0) atomicOr(&flags[FLAG_WINMASK], 1 << w);
  uint32_t* lpts = smem;
  st_ext(lpts + t * EXT_WORDS, ld_ext(slice_T + (size_t)(w * NSLICE + t) * EXT_WORDS));
  __syncthreads();
  ge_p3 ws, tot;
  weighted_sum_256(lpts, lpts, lpts + 64 * EXT_WORDS, ws, tot);  // R/S scratch aliases the consumed points
  __syncthreads();
  ge_p3 a = sum_256(ld_ext(slice_W + (size_t)(w * NSLICE + t) * EXT_WORDS), lpts);
  if (t < 4) {
    ge_p3 x = ws;
    for (int k = 0; k < 8; ++k) x = quad_dbl(x);
    ge_p3 r = quad_add(a, x);
    if (t == 0) st_ext(win + (size_t)w * EXT_WORDS, r);
  }
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

// Horner over windows on one quad (4 cooperating lanes), then x8 / identity / optional
// compression (single lane; only when the caller asked for check8).
__global__ void k_msm_final(const uint32_t* __restrict__ win, const int* __restrict__ flags,
                            int want_compress, uint8_t* __restrict__ out) {
  if (threadIdx.x >= 4 || blockIdx.x != 0) return;
  // Horner from the highest non-empty window (windows without entries were never written)
  const uint32_t mask = (uint32_t)flags[FLAG_WINMASK];
  const int top = mask ? 31 - __builtin_clz(mask) : -1;
  ge_p3 acc = ge_identity();
  for (int w = top; w >= 0; --w) {
    if (w != top)
      for (int k = 0; k < WIN_BITS; ++k) acc = quad_dbl(acc);
    if (mask & (1u << w)) acc = quad_add(acc, ld_ext(win + (size_t)w * EXT_WORDS));
  }
  ge_p3 c8 = quad_dbl(quad_dbl(quad_dbl(acc)));
  if (threadIdx.x != 0) return;
  ext_to_canonical_bytes(acc, out + 48);
  const int bad = flags[FLAG_BAD];
  reinterpret_cast<int*>(out)[0] = (!bad && ge_is_identity(c8)) ? 0 : 1;
  reinterpret_cast<int*>(out)[1] = bad;
  reinterpret_cast<int*>(out)[2] = flags[FLAG_NKEYS];   // distinct keys seen (adaptive grouping)
  if (want_compress) {
    uint32_t w8[8];
    ge_compress(c8, w8);
    for (int j = 0; j < 8; ++j)
      for (int b = 0; b < 4; ++b) out[16 + 4 * j + b] = (uint8_t)(w8[j] >> (8 * b));
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

// ---------------------------------------------------------------- launchers
static inline uint32_t cdiv(uint64_t a, uint32_t b) { return (uint32_t)((a + b - 1) / b); }

void launch_msm_bin(hipStream_t st, uint32_t n, const uint32_t* scal, uint32_t* counts,
                    uint32_t* offsets, uint32_t* cursor, uint2* entries, const int* flags) {
  const uint32_t maxpts = 1 + 2 * n;
  (void)hipMemsetAsync(counts, 0, NBIN * sizeof(uint32_t), st);
  hipLaunchKernelGGL(k_msm_count, dim3(cdiv(maxpts, CNT_PTS_PER_BLOCK)), dim3(256), 0, st, n, scal, counts,
                     flags);
  hipLaunchKernelGGL(k_msm_scan, dim3(1), dim3(1024), 0, st, counts, offsets, cursor);
  hipLaunchKernelGGL(k_msm_scatter, dim3(cdiv(maxpts, CNT_PTS_PER_BLOCK)), dim3(256), 0, st, n, scal,
                     cursor, entries, flags);
}

static const size_t kReduceLds = (size_t)NSLICE * EXT_WORDS * sizeof(uint32_t);  // 256 points; scans reuse them

void launch_msm_bucket(hipStream_t st, const uint32_t* counts, const uint32_t* offsets,
                       const uint2* entries, uint32_t* sorted, const uint32_t* pts, uint32_t* buckets,
                       uint32_t* heads, uint32_t* slice_W, uint32_t* slice_T) {
#if EDC_ACC_DMA
  hipLaunchKernelGGL(k_msm_accum_dma, dim3(NBIN), dim3(256), 0, st, counts, offsets, entries, sorted, pts, buckets,
                     heads, slice_W, slice_T);
  return;                              // the reduction is fused into the accumulation
#else
  (void)sorted;
  (void)heads;
  hipLaunchKernelGGL(k_msm_accum, dim3(NBIN), dim3(ACC_THREADS), 0, st, counts, offsets, entries, pts, buckets);
#endif
  hipLaunchKernelGGL(k_msm_reduce, dim3(NBIN), dim3(256), kReduceLds, st, counts, buckets, slice_W, slice_T);
}

size_t msm_bucket_words() { return (size_t)NBIN * NSLICE * EXT_WORDS; }

void launch_msm_tail(hipStream_t st, const uint32_t* counts, const uint32_t* slice_W, const uint32_t* slice_T,
                     uint32_t* win, int* flags, int want_compress, uint8_t* out) {
  hipLaunchKernelGGL(k_msm_window, dim3(NWIN_FULL), dim3(256), kReduceLds, st, counts, slice_W, slice_T, win, flags);
  hipLaunchKernelGGL(k_msm_final, dim3(1), dim3(64), 0, st, win, flags, want_compress, out);
}

void launch_combine(hipStream_t st, uint32_t g, const uint8_t* partials, int bad, int want_compress,
                    uint8_t* out) {
  hipLaunchKernelGGL(k_combine, dim3(1), dim3(64), 0, st, g, partials, bad, want_compress, out);
}

size_t msm_entry_capacity(uint32_t n) { return (size_t)NWIN_Z * n + (size_t)NWIN_FULL * (n + 1); }

}  // namespace edc
