// pbs.hip — batched classic programmable bootstrap for CDNA4 (gfx950).
//
// Reference semantics: concrete-cpu c_api/bootstrap.rs:347-414 -> tfhe 0.10
// programmable_bootstrap_lwe_ciphertext_mem_optimized (blind_rotate_assign + sample extract),
// restated in oracle/tfhe_oracle.c:ora_pbs.  Batched call shape: tfhe-cuda-backend
// cuda_programmable_bootstrap_lwe_ciphertext_vector_64 as invoked by the runtime
// (compiler lib/Runtime/wrappers.cpp:237-240, lib/Runtime/GPUDFG.cpp:1214-1218).
//
// Exact arithmetic: the product digit-poly x key-poly over Z_{2^64}[X]/(X^N+1) is computed
// as LIMBS exact integer negacyclic convolutions d * g_j (g = sum_j 2^{s_j} g_j, g_j balanced
// limbs of 22/21/21 bits) evaluated with an f64 negacyclic FFT whose worst-case rounding
// error is certified < 1/2, so rounding recovers the exact integers; the
// limbs are recombined modulo 2^64.  Results are bit-identical to the schoolbook definition.
//
// Mapping (N = 1024): one wave64 per ciphertext, the whole 630-step CMUX loop inside one
// launch.  Lane t owns coefficients t + 64 m of every polynomial.  The GLWE accumulator
// (16 KB) lives in the wave's LDS slice; the six digit spectra live in VGPRs; the Fourier
// key slice of step i is streamed from L2/HBM with 1 KB coalesced loads.
#include "common.hpp"
#include "fft512.hpp"
#include "pbs.hpp"

namespace chip {

// ------------------------------------------------------------------------------------
// In-kernel twiddle tables (computed once per workgroup with sincospi; <= 1 ulp class error)
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void build_tables_1024(cplx* tw1, cplx* tw2, cplx* zeta) {
  for (int e = threadIdx.x; e < 512; e += blockDim.x) {
    const int k0 = e >> 6, t = e & 63;
    double s, c;
    // w512^{t k0} = exp(-2 pi i t k0 / 512)
    sincospi(-2.0 * (double)((t * k0) & 511) / 512.0, &s, &c);
    tw1[e] = {c, s};
    // zeta^{t + 64 m} = exp(i pi (t + 64 m) / 1024), e = m * 64 + t
    sincospi((double)e / 1024.0, &s, &c);
    zeta[e] = {c, s};
  }
  for (int e = threadIdx.x; e < 64; e += blockDim.x) {
    const int k1 = e >> 3, t0 = e & 7;
    double s, c;
    sincospi(-2.0 * (double)((t0 * k1) & 63) / 64.0, &s, &c);
    tw2[e] = {c, s};
  }
}

__device__ __forceinline__ int64_t round_to_i64(double v) {
  // v + 1.5*2^52 rounds v to the nearest integer (|v| < 2^51); the mantissa carries it.
  const double magic = 6755399441055744.0;
  double t = v + magic;
  return (int64_t)(__double_as_longlong(t) - __double_as_longlong(magic));
}

template <int K, int L, int LIMBS, bool RESID>
__global__ void __launch_bounds__(PBS1024_WAVES * 64, 1)
pbs1024_kernel(uint64_t* __restrict__ out, const uint64_t* __restrict__ out_idx,
               const uint64_t* __restrict__ luts, const uint64_t* __restrict__ lut_idx,
               const uint64_t* __restrict__ in, const uint64_t* __restrict__ in_idx,
               const cplx* __restrict__ fbsk, uint32_t n, uint32_t base_log, uint32_t num_samples,
               unsigned long long* __restrict__ resid_out) {
  constexpr int N = 1024, LOG2_2N = 11, K1 = K + 1, RQ = K1 * L;
  constexpr int PER_I = K1 * LIMBS * RQ * 8 * 64;  // complex values of one Fourier GGSW
  extern __shared__ __attribute__((aligned(16))) char smem[];
  cplx* tw1 = reinterpret_cast<cplx*>(smem);
  cplx* tw2 = tw1 + 512;
  cplx* zeta = tw2 + 64;
  char* wave_base = smem + PBS1024_TABLE_BYTES;

  build_tables_1024(tw1, tw2, zeta);
  __syncthreads();

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t s = blockIdx.x * PBS1024_WAVES + wave;
  if (s >= num_samples) return;

  uint64_t* acc = reinterpret_cast<uint64_t*>(wave_base + wave * pbs1024_wave_bytes(K));
  cplx* xch = reinterpret_cast<cplx*>(acc + K1 * N);
  const Fft512Tables T{tw1, tw2};

  const uint64_t* lwe = in + (in_idx ? in_idx[s] : s) * (uint64_t)(n + 1);
  const uint64_t* lut = luts + (lut_idx ? lut_idx[s] : 0ull) * (uint64_t)(K1 * N);

  // acc <- LUT * X^{-ms(b)}   (blind_rotate_assign: polynomial_wrapping_monic_monomial_div)
  {
    const uint32_t bt = modswitch(lwe[n], LOG2_2N);
#pragma unroll
    for (int r = 0; r < K1; ++r)
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const int j = lane + 64 * m;
        const uint32_t src = (j + bt) & (2 * N - 1);
        const uint64_t v = lut[r * N + (src & (N - 1))];
        acc[r * N + j] = src < N ? v : 0ull - v;
      }
  }
  wave_lds_fence();

  const int nrep = 64 - L * (int)base_log;
  const int logB = (int)base_log;
  double max_resid = 0.0;

  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t ai = lwe[i];
    if (ai == 0ull) continue;  // tfhe: a zero mask element skips the CMUX
    const uint32_t at = modswitch(ai, LOG2_2N);
    if (at == 0u) continue;    // X^0 acc - acc = 0: the external product of 0 is exactly 0

    // ---- ct1 = acc * X^{at} - acc, decomposition, forward transforms -------------------
    cplx X[RQ][8];
#pragma unroll
    for (int r = 0; r < K1; ++r) {
      int32_t dig[L][16];
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const int j = lane + 64 * m;
        const uint32_t src = (uint32_t)(j - (int)at) & (2 * N - 1);
        const uint64_t rv = acc[r * N + (src & (N - 1))];
        const uint64_t c1 = (src < N ? rv : 0ull - rv) - acc[r * N + j];
        uint64_t st = decomp_init(c1, nrep);
#pragma unroll
        for (int q = 0; q < L; ++q) dig[q][m] = decomp_next(st, logB);
      }
#pragma unroll
      for (int q = 0; q < L; ++q) {
        cplx v[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) {
          const cplx z = zeta[m * 64 + lane];
          const double a = (double)dig[q][m], b = (double)dig[q][m + 8];
          v[m] = {a * z.re - b * z.im, a * z.im + b * z.re};
        }
        fft512_fwd(v, xch, T, lane);
#pragma unroll
        for (int e = 0; e < 8; ++e) X[r * L + q][e] = v[e];
      }
    }

    // ---- multiply-accumulate with the Fourier GGSW, inverse transforms, exact recombination
    const cplx* Gi = fbsk + (uint64_t)i * PER_I;
#pragma unroll 1
    for (int c = 0; c < K1; ++c) {
      uint64_t R[16];
#pragma unroll
      for (int m = 0; m < 16; ++m) R[m] = 0ull;
      int shift = 0;
#pragma unroll
      for (int li = 0; li < LIMBS; ++li) {
        const cplx* G = Gi + (c * LIMBS + li) * (RQ * 512);
        cplx Y[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) Y[e] = {0.0, 0.0};
#pragma unroll
        for (int rq = 0; rq < RQ; ++rq) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const cplx g = G[rq * 512 + e * 64 + lane];
            const cplx x = X[rq][e];
            Y[e].re = __builtin_fma(x.re, g.re, __builtin_fma(-x.im, g.im, Y[e].re));
            Y[e].im = __builtin_fma(x.re, g.im, __builtin_fma(x.im, g.re, Y[e].im));
          }
        }
        fft512_inv(Y, xch, T, lane);
#pragma unroll
        for (int m = 0; m < 8; ++m) {
          const cplx z = zeta[m * 64 + lane];
          const double cr = __builtin_fma(Y[m].re, z.re, Y[m].im * z.im);
          const double ci = __builtin_fma(Y[m].im, z.re, -Y[m].re * z.im);
          const int64_t rr = round_to_i64(cr), ri = round_to_i64(ci);
          if constexpr (RESID) {
            max_resid = fmax(max_resid, fabs(cr - (double)rr));
            max_resid = fmax(max_resid, fabs(ci - (double)ri));
          }
          R[m] += (uint64_t)rr << shift;
          R[m + 8] += (uint64_t)ri << shift;
        }
        shift += (64 / LIMBS) + (li < (64 % LIMBS) ? 1 : 0);
      }
#pragma unroll
      for (int m = 0; m < 16; ++m) acc[c * N + lane + 64 * m] += R[m];
    }
    wave_lds_fence();
  }

  // ---- sample extract (nth = 0) -------------------------------------------------------
  uint64_t* o = out + (out_idx ? out_idx[s] : s) * (uint64_t)(K * N + 1);
  for (int e = lane; e < K * N; e += 64) {
    const int r = e / N, j = e % N;
    const uint64_t v = acc[r * N + ((N - j) & (N - 1))];
    o[e] = j == 0 ? v : 0ull - v;
  }
  if (lane == 0) o[K * N] = acc[K * N];

  if constexpr (RESID) {
    // wave max then one atomic (non-negative doubles order like their bit patterns)
    for (int off = 32; off > 0; off >>= 1) max_resid = fmax(max_resid, __shfl_xor(max_resid, off));
    if (lane == 0) atomicMax(resid_out, (unsigned long long)__double_as_longlong(max_resid));
  }
}

// ------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------
template <int K, int L, int LIMBS>
static int launch_1024(const PbsArgs& a) {
  const size_t lds = pbs1024_lds_bytes(K);
  const uint32_t blocks = (a.num_samples + PBS1024_WAVES - 1) / PBS1024_WAVES;
  if (blocks == 0) return 0;
  if (a.resid) {
    auto kern = pbs1024_kernel<K, L, LIMBS, true>;
    CHIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(PBS1024_WAVES * 64), lds, a.stream, a.out, a.out_idx, a.luts,
                       a.lut_idx, a.in, a.in_idx, reinterpret_cast<const cplx*>(a.fbsk), a.n, a.base_log,
                       a.num_samples, a.resid);
  } else {
    auto kern = pbs1024_kernel<K, L, LIMBS, false>;
    CHIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(PBS1024_WAVES * 64), lds, a.stream, a.out, a.out_idx, a.luts,
                       a.lut_idx, a.in, a.in_idx, reinterpret_cast<const cplx*>(a.fbsk), a.n, a.base_log,
                       a.num_samples, a.resid);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("pbs launch failed: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

int pbs_launch(const PbsArgs& a) {
  if (a.N == 1024 && a.k == 1 && a.limbs == 3) {
    switch (a.level) {
      case 1: return launch_1024<1, 1, 3>(a);
      case 2: return launch_1024<1, 2, 3>(a);
      case 3: return launch_1024<1, 3, 3>(a);
      case 4: return launch_1024<1, 4, 3>(a);
      default: break;
    }
  }
  set_error("unsupported PBS parameters: N=%u k=%u level=%u limbs=%u", a.N, a.k, a.level, a.limbs);
  return -2;
}

}  // namespace chip
