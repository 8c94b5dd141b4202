// Microbenchmark: does a residue-number-system (RNS / NTT) product beat
// the f64 limb-FFT on gfx950?  The survey's §7.2 candidates replace the 512-point complex FFT of an
// N = 1024 negacyclic polynomial (fft512.hpp) by an N-point negacyclic NTT over Z_p per residue.
// This measures one wave's N = 1024 negacyclic NTT over a 30-bit prime (Harvey's lazy butterflies,
// Shoup multiplication: 3 32-bit multiplies per butterfly, values in [0, 4p)), forward + inverse, in
// registers with two LDS transposes per direction — the same shape as fft512 (16 values per lane) —
// and, in the same binary, the fft512 round trip, both at 2 and 3 waves per SIMD.  The round trip is
// checked (inverse(forward(x)) = N x mod p, and fft512's = 512 x to 1e-9) before timing.
//
// Cost model the numbers feed: an exact product needs residues whose product P
// exceeds twice the largest convolution coefficient; with the u64 key that is 3 primes of 30 bits at
// cfg2 (2 * 6 * 1024 * 2^6 * 2^63 ~ 2^83.6) and 4 at cfg4 (2 * 2 * 2048 * 2^22 * 2^63 ~ 2^98), so a
// CMUX step takes (k+1) l P forward and (k+1) P inverse NTTs plus a CRT per coefficient, against the
// f64 path's 12 (cfg2) and 24 (cfg4) 512-point transforms.
//
// Build: hipcc -O3 --offload-arch=gfx950 -I../../concrete_amd/csrc ntt_bench.hip -o ntt_bench
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "fft512.hpp"

using namespace chip;

constexpr uint32_t P = 1073479681u;  // 2^30 - 2^18 + 1: prime, P = 1 mod 2048
constexpr int NN = 1024, LOGN = 10;
constexpr int R = 200;  // round trips per wave

// ---- host modular arithmetic -----------------------------------------------------------------
static uint64_t mulm(uint64_t a, uint64_t b) { return (a * b) % P; }
static uint64_t powm(uint64_t a, uint64_t e) {
  uint64_t r = 1;
  while (e) {
    if (e & 1) r = mulm(r, a);
    a = mulm(a, a);
    e >>= 1;
  }
  return r;
}
static uint32_t bitrev(uint32_t x, int bits) { return __builtin_bitreverse32(x) >> (32 - bits); }

// ---- device: Harvey butterflies ----------------------------------------------------------------
struct Tw {
  uint32_t w, ws;  // w and floor(w 2^32 / P)
};
// t = w y mod P in [0, 2P) (Shoup): q = mulhi(ws, y), t = w y - q P (mod 2^32)
__device__ __forceinline__ uint32_t shoup(uint32_t y, Tw t) {
  const uint32_t q = __umulhi(t.ws, y);
  return t.w * y - q * P;
}
// forward (Cooley-Tukey, lazy): x, y in [0, 4P) -> x + wy, x - wy + 2P in [0, 4P)
__device__ __forceinline__ void ct_bf(uint32_t& x, uint32_t& y, Tw t) {
  uint32_t a = x - 2 * P;
  a = a < x ? a : x;  // x mod 2P (x < 4P)
  const uint32_t v = shoup(y, t);
  x = a + v;
  y = a - v + 2 * P;
}
// inverse (Gentleman-Sande, lazy): x, y in [0, 2P) -> x + y mod 2P, (x - y + 2P) w mod [0, 2P)
__device__ __forceinline__ void gs_bf(uint32_t& x, uint32_t& y, Tw t) {
  uint32_t s = x + y;
  const uint32_t s2 = s - 2 * P;
  s = s2 < s ? s2 : s;
  const uint32_t d = x - y + 2 * P;
  x = s;
  y = shoup(d, t);
}
__device__ __forceinline__ uint32_t red2(uint32_t x) {  // [0, 4P) -> [0, P)
  uint32_t a = x - 2 * P;
  a = a < x ? a : x;
  const uint32_t b = a - P;
  return b < a ? b : a;
}

// Index bits of the coefficient j (10 bits) across (lane, register) in the three layouts:
//   A: register m = bits 9..6, lane = bits 5..0                       (stages on bits 9..6)
//   B: register m = bits 5..2, lane = (bits 9..6) << 2 | bits 1..0     (stages on bits 5..2)
//   C: register m = bits 1..0 | (bits 9..8) << 2, lane = bits 7..2     (stages on bits 1..0)
// Twiddle of the CT stage on bit b for coefficient j: psi_rev[2^(9-b) + (j >> (b + 1))].
__device__ __forceinline__ int jA(int lane, int m) { return (m << 6) | lane; }
__device__ __forceinline__ int jB(int lane, int m) { return ((lane >> 2) << 6) | (m << 2) | (lane & 3); }
__device__ __forceinline__ int jC(int lane, int m) { return ((m >> 2) << 8) | (lane << 2) | (m & 3); }

template <class JF>
__device__ __forceinline__ void store16(const uint32_t (&v)[16], uint32_t* s, int lane, JF jf) {
#pragma unroll
  for (int m = 0; m < 16; ++m) s[jf(lane, m) + (jf(lane, m) >> 5)] = v[m];  // +1 pad per 32
}
template <class JF>
__device__ __forceinline__ void load16(uint32_t (&v)[16], const uint32_t* s, int lane, JF jf) {
#pragma unroll
  for (int m = 0; m < 16; ++m) v[m] = s[jf(lane, m) + (jf(lane, m) >> 5)];
}

// stages of one layout: register pairs (m, m ^ (1 << rb)) for register bit rb = the coefficient bit b
template <bool INV, class JF>
__device__ __forceinline__ void stage(uint32_t (&v)[16], const Tw* tw, int lane, int b, int rb, JF jf) {
  const int base = 1 << (9 - b);
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    if (m & (1 << rb)) continue;
    const int j = jf(lane, m);
    const Tw t = tw[base + (j >> (b + 1))];
    if (INV) gs_bf(v[m], v[m | (1 << rb)], t);
    else ct_bf(v[m], v[m | (1 << rb)], t);
  }
}

__device__ __forceinline__ void ntt_fwd(uint32_t (&v)[16], const Tw* tw, uint32_t* s, int lane) {
  stage<false>(v, tw, lane, 9, 3, jA);
  stage<false>(v, tw, lane, 8, 2, jA);
  stage<false>(v, tw, lane, 7, 1, jA);
  stage<false>(v, tw, lane, 6, 0, jA);
  store16(v, s, lane, jA);
  wave_lds_fence();
  load16(v, s, lane, jB);
  wave_lds_fence();
  stage<false>(v, tw, lane, 5, 3, jB);
  stage<false>(v, tw, lane, 4, 2, jB);
  stage<false>(v, tw, lane, 3, 1, jB);
  stage<false>(v, tw, lane, 2, 0, jB);
  store16(v, s, lane, jB);
  wave_lds_fence();
  load16(v, s, lane, jC);
  wave_lds_fence();
  stage<false>(v, tw, lane, 1, 1, jC);
  stage<false>(v, tw, lane, 0, 0, jC);
}
// inverse: the same stages backwards with the inverse twiddles (GS), output in layout A
__device__ __forceinline__ void ntt_inv(uint32_t (&v)[16], const Tw* itw, uint32_t* s, int lane) {
#pragma unroll
  for (int m = 0; m < 16; ++m) v[m] = red2(v[m]) ;  // [0, 4P) -> [0, P) before the GS stages
  stage<true>(v, itw, lane, 0, 0, jC);
  stage<true>(v, itw, lane, 1, 1, jC);
  store16(v, s, lane, jC);
  wave_lds_fence();
  load16(v, s, lane, jB);
  wave_lds_fence();
  stage<true>(v, itw, lane, 2, 0, jB);
  stage<true>(v, itw, lane, 3, 1, jB);
  stage<true>(v, itw, lane, 4, 2, jB);
  stage<true>(v, itw, lane, 5, 3, jB);
  store16(v, s, lane, jB);
  wave_lds_fence();
  load16(v, s, lane, jA);
  wave_lds_fence();
  stage<true>(v, itw, lane, 6, 0, jA);
  stage<true>(v, itw, lane, 7, 1, jA);
  stage<true>(v, itw, lane, 8, 2, jA);
  stage<true>(v, itw, lane, 9, 3, jA);
}

constexpr int SCR = NN + NN / 32;  // u32 per wave scratch (padded)

template <int NWAVES, bool CHECK>
__global__ void __launch_bounds__(NWAVES * 64) ntt_kern(const Tw* __restrict__ gtw, const Tw* __restrict__ gitw,
                                                        uint32_t* out, unsigned long long* cyc) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  Tw* tw = reinterpret_cast<Tw*>(smem);
  Tw* itw = tw + NN;
  uint32_t* scr = reinterpret_cast<uint32_t*>(itw + NN);
  for (int e = threadIdx.x; e < NN; e += NWAVES * 64) tw[e] = gtw[e], itw[e] = gitw[e];
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t* s = scr + w * SCR;
  uint32_t v[16];
  for (int m = 0; m < 16; ++m) v[m] = (uint32_t)(((uint64_t)jA(lane, m) * 2654435761ull) % P);
  const long long c0 = clock64();
  for (int r = 0; r < (CHECK ? 1 : R); ++r) {
    ntt_fwd(v, tw, s, lane);
    ntt_inv(v, itw, s, lane);
  }
  const long long c1 = clock64();
  for (int m = 0; m < 16; ++m) out[(blockIdx.x * NWAVES + w) * NN + jA(lane, m)] = v[m];
  if (lane == 0) cyc[blockIdx.x * NWAVES + w] = (unsigned long long)(c1 - c0);
}

template <int NWAVES, bool CHECK>
__global__ void __launch_bounds__(NWAVES * 64) fft_kern(double* out, unsigned long long* cyc) {
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
  const long long c0 = clock64();
  for (int r = 0; r < (CHECK ? 1 : R); ++r) {
    fft512_fwd(v, xch, T, lane);
    fft512_inv(v, xch, T, lane);
#pragma unroll
    for (int m = 0; m < 8; ++m) v[m] = {v[m].re * (1.0 / 512), v[m].im * (1.0 / 512)};
  }
  const long long c1 = clock64();
  for (int m = 0; m < 8; ++m) {
    out[((blockIdx.x * NWAVES + w) * 64 + lane) * 16 + 2 * m] = v[m].re;
    out[((blockIdx.x * NWAVES + w) * 64 + lane) * 16 + 2 * m + 1] = v[m].im;
  }
  if (lane == 0) cyc[blockIdx.x * NWAVES + w] = (unsigned long long)(c1 - c0);
}

static double avg_cycles(unsigned long long* d, int n) {
  std::vector<unsigned long long> h(n);
  (void)hipMemcpy(h.data(), d, n * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  double a = 0;
  for (auto x : h) a += (double)x;
  return a / n;
}

int main() {
  // twiddles: psi a primitive 2N-th root of unity; CT forward uses psi_rev[k] = psi^bitrev(k),
  // GS inverse psi^-bitrev(k); the inverse leaves N x (no N^-1 scaling)
  uint64_t g = 3, psi = 0;
  for (; g < P; ++g) {
    const uint64_t c = powm(g, (P - 1) / (2 * NN));
    if (powm(c, NN) == P - 1) {
      psi = c;
      break;
    }
  }
  const uint64_t ipsi = powm(psi, P - 2);
  std::vector<Tw> tw(NN), itw(NN);
  for (int k = 0; k < NN; ++k) {
    const uint64_t a = powm(psi, bitrev(k, LOGN)), b = powm(ipsi, bitrev(k, LOGN));
    tw[k] = {(uint32_t)a, (uint32_t)((a << 32) / P)};
    itw[k] = {(uint32_t)b, (uint32_t)((b << 32) / P)};
  }
  const int ncu = 256;
  Tw *dtw, *ditw;
  uint32_t* dout;
  double* dfo;
  unsigned long long* dcyc;
  (void)hipMalloc(&dtw, NN * sizeof(Tw));
  (void)hipMalloc(&ditw, NN * sizeof(Tw));
  (void)hipMalloc(&dout, (size_t)ncu * 12 * NN * 4);
  (void)hipMalloc(&dfo, (size_t)ncu * 12 * 64 * 16 * 8);
  (void)hipMalloc(&dcyc, ncu * 12 * 8);
  (void)hipMemcpy(dtw, tw.data(), NN * sizeof(Tw), hipMemcpyHostToDevice);
  (void)hipMemcpy(ditw, itw.data(), NN * sizeof(Tw), hipMemcpyHostToDevice);
  // ---- correctness: one round trip = N x mod P
  {
    const size_t lds = 2 * NN * sizeof(Tw) + 8 * SCR * 4;
    (void)hipFuncSetAttribute((const void*)ntt_kern<8, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    ntt_kern<8, true><<<1, 512, lds>>>(dtw, ditw, dout, dcyc);
    std::vector<uint32_t> h(8 * NN);
    (void)hipMemcpy(h.data(), dout, h.size() * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int j = 0; j < NN; ++j) {
      const uint64_t x = ((uint64_t)j * 2654435761u) % P;
      if ((h[j] % P) != mulm(x, NN)) ++bad;
    }
    // forward alone vs the negacyclic definition: NTT(x)[k] = sum_j x_j psi^((2 bitrev(k) + 1) j)
    printf("ntt round trip: %s (%d of %d wrong)\n", bad ? "WRONG" : "ok", bad, NN);
    if (bad) return 1;
  }
  {
    const size_t lds = (FFT512_TABLE_ENTRIES + 8 * XCH_SLOTS) * 16;
    (void)hipFuncSetAttribute((const void*)fft_kern<8, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    fft_kern<8, true><<<1, 512, lds>>>(dfo, dcyc);
    std::vector<double> h(64 * 16);
    (void)hipMemcpy(h.data(), dfo, h.size() * 8, hipMemcpyDeviceToHost);
    double err = 0;
    for (int lane = 0; lane < 64; ++lane)
      for (int m = 0; m < 8; ++m) {
        const double re = (double)((lane * 7 + m * 3) % 17 - 8), im = (double)((lane + m) % 5 - 2);
        err = fmax(err, fabs(h[lane * 16 + 2 * m] - re) + fabs(h[lane * 16 + 2 * m + 1] - im));
      }
    printf("fft512 round trip: max error %.3g (%s)\n", err, err < 1e-9 ? "ok" : "WRONG");
  }
  // ---- timing: 2 and 3 waves per SIMD (8 / 12 waves per CU, one workgroup per CU)
  auto time_ntt = [&](auto kern, int nw) {
    const size_t lds = 2 * NN * sizeof(Tw) + nw * SCR * 4;
    const size_t req = lds < 90 * 1024 ? 90 * 1024 : lds;
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)req);
    kern<<<ncu, nw * 64, req>>>(dtw, ditw, dout, dcyc);
    kern<<<ncu, nw * 64, req>>>(dtw, ditw, dout, dcyc);
    (void)hipDeviceSynchronize();
    const double c = avg_cycles(dcyc, ncu * nw) / (2.0 * R);
    printf("ntt1024 (30-bit Shoup, lazy)  waves/CU %2d: %6.0f clk per transform per wave, %6.0f per SIMD\n", nw, c,
           c / (nw / 4.0));
    return c / (nw / 4.0);
  };
  auto time_fft = [&](auto kern, int nw) {
    const size_t lds = (FFT512_TABLE_ENTRIES + nw * XCH_SLOTS) * 16;
    const size_t req = lds < 90 * 1024 ? 90 * 1024 : lds;
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)req);
    kern<<<ncu, nw * 64, req>>>(dfo, dcyc);
    kern<<<ncu, nw * 64, req>>>(dfo, dcyc);
    (void)hipDeviceSynchronize();
    const double c = avg_cycles(dcyc, ncu * nw) / (2.0 * R);
    printf("fft512 (f64, this backend)    waves/CU %2d: %6.0f clk per transform per wave, %6.0f per SIMD\n", nw, c,
           c / (nw / 4.0));
    return c / (nw / 4.0);
  };
  const double n8 = time_ntt(ntt_kern<8, false>, 8), n12 = time_ntt(ntt_kern<12, false>, 12);
  const double f8 = time_fft(fft_kern<8, false>, 8), f12 = time_fft(fft_kern<12, false>, 12);
  printf("ratio ntt1024 / fft512 per SIMD: %.2f (2 waves/SIMD), %.2f (3 waves/SIMD)\n", n8 / f8, n12 / f12);
  // transforms per ciphertext and CMUX step (header): cfg2 f64 12 vs RNS (3 primes) 6*3 + 2*3 = 24;
  // cfg4 f64 24 (512-point) vs RNS (4 primes, N = 2048 ~ 2 x N = 1024 + a stage) 2*4*2 + 2*4*2 = 32
  printf("cfg2 transform cost per step, RNS / f64: %.2f  (24 ntt1024 vs 12 fft512)\n", 24 * n12 / (12 * f12));
  printf("cfg4 transform cost per step, RNS / f64: %.2f  (32 ntt1024-equivalents vs 24 fft512)\n",
         32 * n8 / (24 * f8));
  return 0;
}
