// Microbenchmark: cost of the one-wave 512-point transform (fft512.hpp) on gfx950.
// Each wave runs R forward+inverse round trips on its own data; one workgroup per CU.
// MODE 0: full transforms (fft512_fwd / fft512_inv); 1: butterflies and twiddles only (the LDS
// transposes skipped, values wrong); 2: transposes only (LDS and register transposes, no
// butterflies).  Reports cycles per transform per wave and per SIMD.
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
  if constexpr (MODE == 0) {
    fft512_fwd(v, xch, T, lane);
    return;
  }
  if constexpr (MODE == 1) fwd_p1(v);
  xpose_hi(v);
  cplx tw3[4];
  fwd_p3_tw(tw3, T, lane);
  if constexpr (MODE == 1) fwd_p2(v, T, hi);
  if constexpr (MODE == 2) {
    fwd_w2(v, xch, hi, lo);
    wave_lds_fence();
    fwd_r2(v, xch, hi, lo);
    wave_lds_fence();
  }
  if constexpr (MODE == 1) geo8<false>(v, tw3, 0);
}

template <int MODE>
__device__ __forceinline__ void inv(cplx (&v)[8], cplx* xch, const Fft512Tables& T, int lane) {
  const int hi = lane >> 3, lo = lane & 7;
  if constexpr (MODE == 0) {
    fft512_inv(v, xch, T, lane);
    return;
  }
  if constexpr (MODE == 1) inv_p1(v);
  if constexpr (MODE == 2) {
    inv_w1(v, xch, hi, lo);
    wave_lds_fence();
    inv_r1(v, xch, hi, lo);
    wave_lds_fence();
  }
  if constexpr (MODE == 1) inv_p2(v, T, hi, lo);
  xpose_hi(v);
  if constexpr (MODE == 1) inv_p3(v);
}

template <int MODE, int NWAVES>
__global__ void __launch_bounds__(NWAVES * 64) kern(double* out, unsigned long long* cyc) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  cplx* tbl = reinterpret_cast<cplx*>(smem);
  cplx* xall = tbl + FFT512_TABLE_ENTRIES;
  build_fft512_tables(tbl, threadIdx.x, NWAVES * 64);
  __syncthreads();
  const Fft512Tables T = fft512_tables_at(tbl);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  cplx* xch = xall + w * XCH_SLOTS;
  cplx v[8];
  for (int m = 0; m < 8; ++m) v[m] = {(double)((lane * 7 + m * 3) % 17 - 8), (double)((lane + m) % 5 - 2)};
  long long c0 = clock64();
  for (int r = 0; r < R; ++r) {
    fwd<MODE>(v, xch, T, lane);
    inv<MODE>(v, xch, T, lane);
#pragma unroll
    for (int m = 0; m < 8; ++m) v[m] = {v[m].re * (1.0 / 512), v[m].im * (1.0 / 512)};
  }
  long long c1 = clock64();
  double s = 0;
  for (int m = 0; m < 8; ++m) s += v[m].re + v[m].im;
  out[blockIdx.x * NWAVES * 64 + threadIdx.x] = s;
  if (lane == 0) cyc[blockIdx.x * NWAVES + w] = (unsigned long long)(c1 - c0);
}

template <int MODE, int NWAVES>
void run(const char* name) {
  auto K = kern<MODE, NWAVES>;
  int ncu = 256;
  size_t lds = (FFT512_TABLE_ENTRIES + NWAVES * XCH_SLOTS) * 16;
  // pad LDS so that exactly one workgroup fits per CU
  size_t lds_req = lds < 90 * 1024 ? 90 * 1024 : lds;
  double* out;
  unsigned long long* cyc;
  (void)hipMalloc(&out, ncu * NWAVES * 64 * sizeof(double));
  (void)hipMalloc(&cyc, ncu * NWAVES * sizeof(unsigned long long));
  (void)hipFuncSetAttribute((const void*)K, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_req);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  K<<<ncu, NWAVES * 64, lds_req>>>(out, cyc);
  (void)hipEventRecord(e0);
  K<<<ncu, NWAVES * 64, lds_req>>>(out, cyc);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  unsigned long long* h = (unsigned long long*)malloc(ncu * NWAVES * sizeof(unsigned long long));
  (void)hipMemcpy(h, cyc, ncu * NWAVES * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < ncu * NWAVES; ++i) avg += (double)h[i];
  avg /= ncu * NWAVES;
  const double per_fft = avg / (2.0 * R);
  printf("%-28s waves/CU %d  %.3f ms  %.0f clk per transform per wave  (%.0f per transform per SIMD)\n", name,
         NWAVES, ms, per_fft, per_fft / (NWAVES / 4.0));
  free(h);
  (void)hipFree(out);
  (void)hipFree(cyc);
}

int main() {
  run<0, 4>("full");
  run<0, 8>("full");
  run<1, 4>("butterflies only");
  run<1, 8>("butterflies only");
  run<2, 4>("transposes only");
  run<2, 8>("transposes only");
  return 0;
}
