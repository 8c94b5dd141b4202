// Microbenchmark: cost of the one-wave 512-point transform (fft512.hpp) on gfx950.
// Each wave runs R forward+inverse round trips on its own data; one workgroup per CU.
// MODE 0: full transforms; 1: butterflies/twiddles only (transposes skipped, values wrong);
// 2: transposes only.  Reports cycles per transform per wave and per SIMD.
// Build: hipcc -O3 --offload-arch=gfx950 -I../../concrete_amd/csrc fft_bench.cpp -o fft_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "fft512.hpp"

using namespace chip;

constexpr int R = 200;

template <int MODE>
__device__ __forceinline__ void fwd(cplx (&v)[8], cplx* xch, const Fft512Tables& T, int lane) {
  const int hi = lane >> 3, lo = lane & 7;
  if constexpr (MODE != 2) fwd_p1(v, T, lane);
  if constexpr (MODE == 4) {
    xpose_hi(v);
  } else if constexpr (MODE != 1) {
    fwd_w1(v, xch, hi, lo);
    wave_lds_fence();
    fwd_r1(v, xch, hi, lo);
    wave_lds_fence();
  }
  if constexpr (MODE != 2) fwd_p2(v, T, lo);
  if constexpr (MODE != 1) {
    fwd_w2(v, xch, hi, lo);
    wave_lds_fence();
    fwd_r2(v, xch, hi, lo);
    wave_lds_fence();
  }
  if constexpr (MODE != 2) dft8<false>(v);
}
template <int MODE>
__device__ __forceinline__ void inv(cplx (&v)[8], cplx* xch, const Fft512Tables& T, int lane) {
  const int hi = lane >> 3, lo = lane & 7;
  if constexpr (MODE != 2) inv_p1(v, T, lo);
  if constexpr (MODE != 1) {
    inv_w1(v, xch, hi, lo);
    wave_lds_fence();
    inv_r1(v, xch, hi, lo);
    wave_lds_fence();
  }
  if constexpr (MODE != 2) inv_p2(v, T, hi, lo);
  if constexpr (MODE == 4) {
    xpose_hi(v);
  } else if constexpr (MODE != 1) {
    inv_w2(v, xch, hi, lo);
    wave_lds_fence();
    inv_r2(v, xch, hi, lo);
    wave_lds_fence();
  }
  if constexpr (MODE != 2) inv_p3(v);
}

// two transforms per wave, software-pipelined through one scratch
__device__ __forceinline__ void inv2(cplx (&a)[8], cplx (&b)[8], cplx* xch, const Fft512Tables& T, int lane) {
  const int hi = lane >> 3, lo = lane & 7;
  inv_p1(a, T, lo);
  inv_w1(a, xch, hi, lo);
  wave_lds_fence();
  inv_r1(a, xch, hi, lo);
  wave_lds_fence();
  inv_p1(b, T, lo);
  wave_lds_fence();
  inv_w1(b, xch, hi, lo);
  wave_lds_fence();
  inv_r1(b, xch, hi, lo);
  wave_lds_fence();
  inv_p2(a, T, hi, lo);
  wave_lds_fence();
  inv_w2(a, xch, hi, lo);
  wave_lds_fence();
  inv_r2(a, xch, hi, lo);
  wave_lds_fence();
  inv_p2(b, T, hi, lo);
  wave_lds_fence();
  inv_w2(b, xch, hi, lo);
  wave_lds_fence();
  inv_r2(b, xch, hi, lo);
  wave_lds_fence();
  inv_p3(a);
  inv_p3(b);
}

template <int NWAVES>
__global__ void __launch_bounds__(NWAVES * 64) kern2(double* out, unsigned long long* cyc) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  cplx* T1 = reinterpret_cast<cplx*>(smem);
  cplx* T2 = T1 + 8 * T1_STRIDE;
  cplx* xall = T2 + 64;
  build_fft512_tables(T1, T2, threadIdx.x, NWAVES * 64);
  __syncthreads();
  const Fft512Tables T{T1, T2};
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  cplx* xch = xall + w * 576;
  cplx a[8], b[8];
  for (int m = 0; m < 8; ++m) {
    a[m] = {(double)((lane * 7 + m * 3) % 17 - 8), (double)((lane + m) % 5 - 2)};
    b[m] = {(double)((lane * 5 + m * 3) % 13 - 6), (double)((lane + 2 * m) % 7 - 3)};
  }
  long long c0 = clock64();
  for (int r = 0; r < R / 2; ++r) {
    fft512_fwd2(a, b, xch, T, lane);
    inv2(a, b, xch, T, lane);
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      a[m] = {a[m].re * (1.0 / 512), a[m].im * (1.0 / 512)};
      b[m] = {b[m].re * (1.0 / 512), b[m].im * (1.0 / 512)};
    }
  }
  long long c1 = clock64();
  double s = 0;
  for (int m = 0; m < 8; ++m) s += a[m].re + a[m].im + b[m].re + b[m].im;
  out[blockIdx.x * NWAVES * 64 + threadIdx.x] = s;
  if (lane == 0) cyc[blockIdx.x * NWAVES + w] = (unsigned long long)(c1 - c0);
}

template <int MODE, int NWAVES>
__global__ void __launch_bounds__(NWAVES * 64) kern(double* out, unsigned long long* cyc) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  cplx* T1 = reinterpret_cast<cplx*>(smem);
  cplx* T2 = T1 + 8 * T1_STRIDE;
  cplx* xall = T2 + 64;
  build_fft512_tables(T1, T2, threadIdx.x, NWAVES * 64);
  __syncthreads();
  const Fft512Tables T{T1, T2};
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  cplx* xch = xall + w * 576;
  cplx v[8];
  for (int m = 0; m < 8; ++m) v[m] = {(double)((lane * 7 + m * 3) % 17 - 8), (double)((lane + m) % 5 - 2)};
  unsigned long long t0 = wall_clock64();
  long long c0 = clock64();
  for (int r = 0; r < R; ++r) {
    fwd<MODE>(v, xch, T, lane);
    inv<MODE>(v, xch, T, lane);
#pragma unroll
    for (int m = 0; m < 8; ++m) v[m] = {v[m].re * (1.0 / 512), v[m].im * (1.0 / 512)};
  }
  long long c1 = clock64();
  (void)t0;
  double s = 0;
  for (int m = 0; m < 8; ++m) s += v[m].re + v[m].im;
  out[blockIdx.x * NWAVES * 64 + threadIdx.x] = s;
  if (lane == 0) cyc[blockIdx.x * NWAVES + w] = (unsigned long long)(c1 - c0);
}

static double* ref_out = nullptr;  // outputs of the last MODE 0 run

template <int MODE, int NWAVES>
void run(const char* name) {
  auto K = MODE == 3 ? kern2<NWAVES> : kern<MODE == 3 ? 0 : MODE, NWAVES>;
  int ncu = 256;
  size_t lds = FFT512_TABLE_ENTRIES * 16 + NWAVES * 576 * 16;
  // pad LDS so that exactly one workgroup fits per CU
  size_t lds_req = lds < 90 * 1024 ? 90 * 1024 : lds;
  double* out;
  unsigned long long* cyc;
  hipMalloc(&out, ncu * NWAVES * 64 * sizeof(double));
  hipMalloc(&cyc, ncu * NWAVES * sizeof(unsigned long long));
  (void)hipFuncSetAttribute((const void*)K, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_req);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  K<<<ncu, NWAVES * 64, lds_req>>>(out, cyc);
  (void)hipEventRecord(e0);
  K<<<ncu, NWAVES * 64, lds_req>>>(out, cyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  // correctness: modes 0 and 4 compute the same transforms (bit-identical outputs)
  if (MODE == 0 || MODE == 4) {
    size_t cnt = (size_t)ncu * NWAVES * 64;
    double* hv = (double*)malloc(cnt * sizeof(double));
    hipMemcpy(hv, out, cnt * sizeof(double), hipMemcpyDeviceToHost);
    if (MODE == 0) {
      free(ref_out);
      ref_out = hv;
    } else {
      size_t bad = 0;
      for (size_t i = 0; i < cnt; ++i) bad += hv[i] != ref_out[i];
      printf("  register-transpose results identical to LDS transposes: %s (%zu mismatches)\n", bad ? "NO" : "yes", bad);
      free(hv);
    }
  }
  unsigned long long* h = (unsigned long long*)malloc(ncu * NWAVES * sizeof(unsigned long long));
  hipMemcpy(h, cyc, ncu * NWAVES * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < ncu * NWAVES; ++i) avg += (double)h[i];
  avg /= ncu * NWAVES;
  const double per_fft = avg / (2.0 * R);
  printf("%-28s waves/CU %d  %.3f ms  %.0f clk per transform per wave  (%.0f per transform per SIMD)\n", name,
         NWAVES, ms, per_fft, per_fft / (NWAVES / 4.0));
  free(h);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  run<0, 4>("full");
  run<4, 4>("full, hi transposes in regs");
  run<0, 8>("full");
  run<4, 8>("full, hi transposes in regs");
  run<1, 4>("butterflies only");
  run<1, 8>("butterflies only");
  run<2, 4>("transposes only");
  run<2, 8>("transposes only");
  run<3, 4>("two interleaved per wave");
  run<3, 8>("two interleaved per wave");
  return 0;
}
