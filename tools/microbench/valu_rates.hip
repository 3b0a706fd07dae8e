// Phase-0 microbenchmark: sustained issue rate of the integer VALU instructions the
// GF(2^255-19) arithmetic can be built from, on gfx950 (wave64, all CUs busy).
// Each lane runs 8 independent chains of one instruction inside an unrolled loop; the
// printed figure is lane-ops per second over the whole chip.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 2048;

__global__ void k_mad_u64_u32(uint64_t* out, uint32_t a, uint32_t b) {
  uint64_t c[8];
  uint32_t x = a + threadIdx.x, y = b ^ blockIdx.x;
#pragma unroll
  for (int i = 0; i < 8; ++i) c[i] = (uint64_t)(x + i) << 7;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      { uint64_t cc; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(c[i]), "=&s"(cc) : "v"(x), "v"(y)); }
  }
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s ^= c[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mad_u64_u32_carry(uint64_t* out, uint32_t a, uint32_t b) {
  // mad with carry-out to SGPR pair + addc consuming it (the column-sum idiom)
  uint64_t c[4]; uint32_t h[4];
  uint32_t x = a + threadIdx.x, y = b ^ blockIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) { c[i] = (uint64_t)(x + i) << 7; h[i] = i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint64_t cc;
      asm volatile("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32 %2, vcc, %2, 0, %1"
                   : "+v"(c[i]), "=&s"(cc), "+v"(h[i]) : "v"(x), "v"(y) : "vcc");
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) s ^= c[i] + h[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mul_lo_u32(uint64_t* out, uint32_t a, uint32_t b) {
  uint32_t c[8];
  uint32_t y = b ^ blockIdx.x;
#pragma unroll
  for (int i = 0; i < 8; ++i) c[i] = a + threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(c[i]) : "v"(y));
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s ^= c[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mul_hi_u32(uint64_t* out, uint32_t a, uint32_t b) {
  uint32_t c[8];
  uint32_t y = b ^ blockIdx.x;
#pragma unroll
  for (int i = 0; i < 8; ++i) c[i] = a + threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(c[i]) : "v"(y));
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s ^= c[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mad_u32_u24(uint64_t* out, uint32_t a, uint32_t b) {
  uint32_t c[8];
  uint32_t x = (a + threadIdx.x) & 0xffffff, y = (b ^ blockIdx.x) & 0xffffff;
#pragma unroll
  for (int i = 0; i < 8; ++i) c[i] = a + threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(c[i]) : "v"(x), "v"(y));
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s ^= c[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_add_co(uint64_t* out, uint32_t a, uint32_t b) {
  uint32_t c[8];
  uint32_t y = b ^ blockIdx.x;
#pragma unroll
  for (int i = 0; i < 8; ++i) c[i] = a + threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(c[i]) : "v"(y) : "vcc");
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s ^= c[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_add_u32(uint64_t* out, uint32_t a, uint32_t b) {
  uint32_t c[8];
  uint32_t y = b ^ blockIdx.x;
#pragma unroll
  for (int i = 0; i < 8; ++i) c[i] = a + threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(c[i]) : "v"(y));
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s ^= c[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_fma_f64(uint64_t* out, uint32_t a, uint32_t b) {
  double c[8];
  double x = 1.0 + 1e-9 * threadIdx.x, y = 0.999999 + 1e-12 * b;
#pragma unroll
  for (int i = 0; i < 8; ++i) c[i] = (double)(a + i);
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(c[i]) : "v"(x), "v"(y));
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += c[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}

__global__ void k_fma_f32(uint64_t* out, uint32_t a, uint32_t b) {
  float c[8];
  float x = 1.0f + 1e-6f * threadIdx.x, y = 0.5f;
#pragma unroll
  for (int i = 0; i < 8; ++i) c[i] = (float)(a + i);
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(c[i]) : "v"(x), "v"(y));
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += c[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}


// 32-bit two-operand ops (c = op(c, y)) and 64-bit ops used by the carry chains / SHA-512
#define K32(NAME, ASM)                                                                 \
  __global__ void NAME(uint64_t* out, uint32_t a, uint32_t b) {                        \
    uint32_t c[8];                                                                     \
    uint32_t y = b ^ blockIdx.x;                                                       \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) c[i] = a + threadIdx.x + i;          \
    for (int it = 0; it < ITERS; ++it) {                                               \
      _Pragma("unroll") for (int i = 0; i < 8; ++i) asm volatile(ASM : "+v"(c[i]) : "v"(y)); \
    }                                                                                  \
    uint32_t s = 0;                                                                    \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) s ^= c[i];                           \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                    \
  }
K32(k_alignbit, "v_alignbit_b32 %0, %0, %1, 29")
K32(k_and_b32, "v_and_b32 %0, %0, %1")
K32(k_bitop3, "v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96")
#define K64(NAME, ASM)                                                                 \
  __global__ void NAME(uint64_t* out, uint32_t a, uint32_t b) {                        \
    uint64_t c[8];                                                                     \
    uint64_t y = ((uint64_t)b << 32) ^ blockIdx.x;                                     \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) c[i] = (uint64_t)(a + threadIdx.x + i) << 20; \
    for (int it = 0; it < ITERS; ++it) {                                               \
      _Pragma("unroll") for (int i = 0; i < 8; ++i) asm volatile(ASM : "+v"(c[i]) : "v"(y)); \
    }                                                                                  \
    uint64_t s = 0;                                                                    \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) s ^= c[i];                           \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                    \
  }
K64(k_lshrrev_b64, "v_lshrrev_b64 %0, 29, %0")
K64(k_lshl_add_u64, "v_lshl_add_u64 %0, %0, 0, %1")

typedef void (*kfn)(uint64_t*, uint32_t, uint32_t);

int run(const char* name, kfn f, int ops_per_iter, uint64_t* d, int blocks, int threads) {
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, d, 3u, 5u);
  CHK(hipDeviceSynchronize());
  const int reps = 5;
  CHK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, d, 3u + r, 5u);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
  double lane_ops = (double)blocks * threads * ITERS * ops_per_iter * reps;
  double rate = lane_ops / (ms * 1e-3);
  // cycles per wave-instruction per SIMD at 2.4 GHz: 1024 SIMDs
  double wave_instr_per_s = rate / 64.0;
  double cyc = 1024.0 * 2.4e9 / wave_instr_per_s;
  printf("%-22s %8.3f ms  %10.3f T lane-ops/s  ~%5.2f cyc/wave-instr/SIMD @2.4GHz\n", name, ms / reps, rate / 1e12, cyc);
  return 0;
}

int main() {
  int blocks = 256 * 8 * 4, threads = 256;
  uint64_t* d;
  CHK(hipMalloc(&d, (size_t)blocks * threads * 8));
  hipDeviceProp_t p; CHK(hipGetDeviceProperties(&p, 0));
  printf("device %s CUs %d clock %d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  run("v_fma_f32", k_fma_f32, 8, d, blocks, threads);
  run("v_add_u32", k_add_u32, 8, d, blocks, threads);
  run("v_add_co_u32", k_add_co, 8, d, blocks, threads);
  run("v_mad_u32_u24", k_mad_u32_u24, 8, d, blocks, threads);
  run("v_mul_lo_u32", k_mul_lo_u32, 8, d, blocks, threads);
  run("v_mul_hi_u32", k_mul_hi_u32, 8, d, blocks, threads);
  run("v_mad_u64_u32", k_mad_u64_u32, 8, d, blocks, threads);
  run("mad_u64_u32+addc(pair)", k_mad_u64_u32_carry, 4, d, blocks, threads);
  run("v_fma_f64", k_fma_f64, 8, d, blocks, threads);
  run("v_alignbit_b32", k_alignbit, 8, d, blocks, threads);
  run("v_and_b32", k_and_b32, 8, d, blocks, threads);
  run("v_bitop3_b32", k_bitop3, 8, d, blocks, threads);
  run("v_lshrrev_b64", k_lshrrev_b64, 8, d, blocks, threads);
  run("v_lshl_add_u64", k_lshl_add_u64, 8, d, blocks, threads);
  CHK(hipFree(d));
  return 0;
}
