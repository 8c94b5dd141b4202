// Microbenchmark: per-instruction VALU throughput on gfx950 for the candidate
// arithmetic of the exact negacyclic product (f64 FMA vs 32/64-bit integer multiply).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 4096
#define CH 8

template <int OP>
__global__ void __launch_bounds__(256) kern(uint64_t* out, uint64_t seed) {
  uint64_t t = threadIdx.x + blockIdx.x * 256ull + seed;
  if constexpr (OP == 0) {  // f64 fma
    double a[CH]; double b = 1.0000001, c = 1e-9;
    for (int i = 0; i < CH; i++) a[i] = (double)(t + i);
    for (int it = 0; it < ITERS; it++)
#pragma unroll
      for (int i = 0; i < CH; i++) a[i] = __builtin_fma(a[i], b, c);
    double s = 0; for (int i = 0; i < CH; i++) s += a[i];
    out[t & 1023] = __double_as_longlong(s);
  } else if constexpr (OP == 1) {  // f32 fma
    float a[CH]; float b = 1.0000001f, c = 1e-9f;
    for (int i = 0; i < CH; i++) a[i] = (float)(t + i);
    for (int it = 0; it < ITERS; it++)
#pragma unroll
      for (int i = 0; i < CH; i++) a[i] = __builtin_fmaf(a[i], b, c);
    float s = 0; for (int i = 0; i < CH; i++) s += a[i];
    out[t & 1023] = __float_as_uint(s);
  } else if constexpr (OP == 2) {  // u32 mul lo
    uint32_t a[CH]; uint32_t b = (uint32_t)seed | 1;
    for (int i = 0; i < CH; i++) a[i] = (uint32_t)(t + i);
    for (int it = 0; it < ITERS; it++)
#pragma unroll
      for (int i = 0; i < CH; i++) a[i] = a[i] * b;
    uint32_t s = 0; for (int i = 0; i < CH; i++) s ^= a[i];
    out[t & 1023] = s;
  } else if constexpr (OP == 3) {  // u32 mul hi
    uint32_t a[CH]; uint32_t b = (uint32_t)seed | 0x80000001u;
    for (int i = 0; i < CH; i++) a[i] = (uint32_t)(t + i) | 0x80000000u;
    for (int it = 0; it < ITERS; it++)
#pragma unroll
      for (int i = 0; i < CH; i++) a[i] = __umulhi(a[i], b) | 0x80000000u;
    uint32_t s = 0; for (int i = 0; i < CH; i++) s ^= a[i];
    out[t & 1023] = s;
  } else if constexpr (OP == 4) {  // u64 mul lo (64x64)
    uint64_t a[CH]; uint64_t b = seed | 1;
    for (int i = 0; i < CH; i++) a[i] = t + i;
    for (int it = 0; it < ITERS; it++)
#pragma unroll
      for (int i = 0; i < CH; i++) a[i] = a[i] * b;
    uint64_t s = 0; for (int i = 0; i < CH; i++) s ^= a[i];
    out[t & 1023] = s;
  } else if constexpr (OP == 5) {  // u32 add (baseline int)
    uint32_t a[CH]; uint32_t b = (uint32_t)seed | 1;
    for (int i = 0; i < CH; i++) a[i] = (uint32_t)(t + i);
    for (int it = 0; it < ITERS; it++)
#pragma unroll
      for (int i = 0; i < CH; i++) a[i] = (a[i] ^ b) + 0x9e37;
    uint32_t s = 0; for (int i = 0; i < CH; i++) s ^= a[i];
    out[t & 1023] = s;
  } else if constexpr (OP == 6) {  // f64 add
    double a[CH]; double b = 1e-9;
    for (int i = 0; i < CH; i++) a[i] = (double)(t + i);
    for (int it = 0; it < ITERS; it++)
#pragma unroll
      for (int i = 0; i < CH; i++) a[i] = a[i] + b;
    double s = 0; for (int i = 0; i < CH; i++) s += a[i];
    out[t & 1023] = __double_as_longlong(s);
  } else if constexpr (OP == 7) {  // u24 mul
    uint32_t a[CH]; uint32_t b = ((uint32_t)seed | 1) & 0xffffff;
    for (int i = 0; i < CH; i++) a[i] = (uint32_t)(t + i);
    for (int it = 0; it < ITERS; it++)
#pragma unroll
      for (int i = 0; i < CH; i++) a[i] = __umul24(a[i], b) ^ 0x5;  // clamps to 24 bits in hw
    uint32_t s = 0; for (int i = 0; i < CH; i++) s ^= a[i];
    out[t & 1023] = s;
  } else if constexpr (OP == 8) {  // f64 mul
    double a[CH]; double b = 1.0000001;
    for (int i = 0; i < CH; i++) a[i] = (double)(t + i);
    for (int it = 0; it < ITERS; it++)
#pragma unroll
      for (int i = 0; i < CH; i++) a[i] = a[i] * b;
    double s = 0; for (int i = 0; i < CH; i++) s += a[i];
    out[t & 1023] = __double_as_longlong(s);
  }
}

template <int OP>
void run(const char* name, uint64_t* d, int ops_per_iter) {
  int blocks = 256 * 16;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  kern<OP><<<blocks, 256>>>(d, 1);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; r++) kern<OP><<<blocks, 256>>>(d, 12345 + r);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double lane_ops = 5.0 * blocks * 256.0 * ITERS * CH * ops_per_iter;
  double per_cu_clk = lane_ops / (ms * 1e-3) / 256.0 / 2.4e9;
  printf("%-12s %8.3f ms  %8.2f T lane-op/s  %7.1f lane-ops/clk/CU (at 2.4GHz)\n", name, ms, lane_ops / (ms * 1e-3) / 1e12, per_cu_clk);
}

int main() {
  uint64_t* d; hipMalloc(&d, 1024 * 8);
  run<1>("f32_fma", d, 1);
  run<0>("f64_fma", d, 1);
  run<6>("f64_add", d, 1);
  run<8>("f64_mul", d, 1);
  run<5>("u32_xor_add", d, 2);
  run<2>("u32_mul_lo", d, 1);
  run<3>("u32_mul_hi", d, 2);
  run<7>("u24_mul", d, 2);
  run<4>("u64_mul", d, 1);
  return 0;
}
