// Device check of fft512.hpp: one wave runs fft512_fwd / fft512_inv on random data; the host
// compares against a long-double DFT (forward: Z_f = sum_j x_j zeta^j w512^{jf}).
// Build: hipcc -O3 --offload-arch=gfx950 -I concrete_amd/csrc tools/microbench/fft_check.hip -o /tmp/fft_check
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "fft512.hpp"
using namespace chip;

__global__ void __launch_bounds__(64) fft_kernel(cplx* data, uint64_t sign) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  cplx* tbl = reinterpret_cast<cplx*>(smem);
  build_fft512_tables(tbl, threadIdx.x, 64);
  __syncthreads();
  const Fft512Tables T = fft512_tables_at(tbl);
  cplx* xch = tbl + FFT512_TABLE_ENTRIES;
  const int lane = threadIdx.x;
  cplx v[8];
  for (int m = 0; m < 8; ++m) v[m] = data[lane + 64 * m];
  fft512_fwd(v, xch, T, lane, sign);
  for (int m = 0; m < 8; ++m) data[512 + lane * 8 + m] = v[m];
  wave_lds_fence();
  fft512_inv(v, xch, T, lane, sign);
  for (int m = 0; m < 8; ++m) data[1024 + lane + 64 * m] = v[m];
}

int main() {
  typedef std::complex<long double> C;
  int bad = 0;
  for (int sg = 0; sg < 2; ++sg) {
    std::vector<cplx> h(1536);
    for (int j = 0; j < 512; ++j) h[j] = {rand() / (double)RAND_MAX - 0.5, rand() / (double)RAND_MAX - 0.5};
    cplx* d;
    hipMalloc(&d, h.size() * sizeof(cplx));
    hipMemcpy(d, h.data(), h.size() * sizeof(cplx), hipMemcpyHostToDevice);
    const size_t lds = FFT512_TABLE_ENTRIES * sizeof(cplx) + 576 * sizeof(cplx);
    hipLaunchKernelGGL(fft_kernel, dim3(1), dim3(64), lds, 0, d, sg ? (1ull << 63) : 0ull);
    hipMemcpy(h.data(), d, h.size() * sizeof(cplx), hipMemcpyDeviceToHost);
    hipFree(d);
    double ef = 0, ei = 0;
    for (int lane = 0; lane < 64; ++lane)
      for (int k2 = 0; k2 < 8; ++k2) {
        const int f = fft512_freq(lane, sg ? (k2 ^ 4) : k2);
        C acc = 0;
        for (int j = 0; j < 512; ++j) {
          const long double a = M_PIl * ((long double)j / 1024 - 2.0L * j * f / 512);
          acc += C(h[j].re, h[j].im) * C(cosl(a), sinl(a));
        }
        const cplx g = h[512 + lane * 8 + k2];
        { const double e = (double)std::abs(acc - C(g.re, g.im)); if (!(e <= ef)) ef = e; }  // NaN-propagating
      }
    for (int j = 0; j < 512; ++j)
      { const double e = fabs(h[1024 + j].re / 512 - h[j].re) + fabs(h[1024 + j].im / 512 - h[j].im); if (!(e <= ei)) ei = e; }
    printf("relabel %d: forward max err %.3g, inverse(forward)/512 max err %.3g\n", sg, ef, ei);
    bad |= !(ef < 1e-13 && ei < 1e-14);
  }
  printf(bad ? "FFT CHECK FAILED\n" : "FFT CHECK OK\n");
  return bad;
}
