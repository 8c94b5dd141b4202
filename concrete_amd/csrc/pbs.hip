// pbs.hip — batched classic programmable bootstrap for CDNA4 (gfx950).
//
// Reference semantics: concrete-cpu c_api/bootstrap.rs:347-414 -> tfhe 0.10
// programmable_bootstrap_lwe_ciphertext_mem_optimized (blind_rotate_assign + sample extract),
// restated in oracle/tfhe_oracle.c:ora_pbs.  Batched call shape: tfhe-cuda-backend
// cuda_programmable_bootstrap_lwe_ciphertext_vector_64 as invoked by the runtime
// (compiler lib/Runtime/wrappers.cpp:237-240, lib/Runtime/GPUDFG.cpp:1214-1218).
//
// Exact arithmetic: the product digit-poly x key-poly over Z_{2^64}[X]/(X^N+1) is computed
// as LIMBS exact integer negacyclic convolutions d * g_j (g = sum_j 2^{s_j} g_j, balanced
// limbs of 22/21/21 bits) evaluated with an f64 negacyclic FFT whose worst-case rounding
// error is certified < 1/2, so rounding recovers the exact integers; the
// limbs are recombined modulo 2^64.  Results are bit-identical to the schoolbook definition.
//
// Mapping (N = 1024): one wave64 per ciphertext, 4 ciphertexts per workgroup, the whole
// n-step CMUX loop inside one launch.  Lane t owns coefficients t + 64 m of every polynomial.
//   VGPRs: GLWE accumulator (2 x 16 u64 per lane) and the six digit spectra (6 x 8 complex).
//   LDS  : twiddle tables, one 8 KB transpose scratch per wave, and a 2-slot ring of Fourier
//          key slices (one slice = the 48 KB a (column, limb) output needs from GGSW_i)
//          filled by LDS-DMA (global_load_lds_dwordx4) and shared by the 4 waves, so the
//          key is read from L2 once per 4 ciphertexts.  The waves run the CMUX loop in
//          lockstep (two raw s_barriers per slice); the DMA for slice g+2 is in flight while
//          slice g+1 is consumed.
#include <type_traits>

#include "common.hpp"
#include "fft512.hpp"
#include "pbs.hpp"

namespace chip {

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E)
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

__device__ __forceinline__ void build_tables_1024(cplx* tw1, cplx* tw2, cplx* zeta) {
  for (int e = threadIdx.x; e < 512; e += blockDim.x) {
    const int k0 = e >> 6, t = e & 63;
    double s, c;
    sincospi(-2.0 * (double)((t * k0) & 511) / 512.0, &s, &c);  // w512^{t k0}
    tw1[e] = {c, s};
    sincospi((double)e / 1024.0, &s, &c);  // zeta^{t + 64 m}, e = 64 m + t
    zeta[e] = {c, s};
  }
  for (int e = threadIdx.x; e < 64; e += blockDim.x) {
    const int k1 = e >> 3, t0 = e & 7;
    double s, c;
    sincospi(-2.0 * (double)((t0 * k1) & 63) / 64.0, &s, &c);  // w64^{t0 k1}
    tw2[e] = {c, s};
  }
}

// bits(v + 1.5 * 2^52) = bits(1.5 * 2^52) + round(v) for |v| < 2^51
constexpr double RND_MAGIC = 6755399441055744.0;
constexpr uint64_t RND_MAGIC_BITS = 0x4338000000000000ull;
// sum over limbs of RND_MAGIC_BITS << shift(limb), for LIMBS = 3 (shifts 0, 22, 43)
constexpr uint64_t MAGIC_ALL = RND_MAGIC_BITS + (RND_MAGIC_BITS << 22) + (RND_MAGIC_BITS << 43);

template <int N_WAIT>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N_WAIT >= 0 && N_WAIT < 64, "vmcnt range");
  // gfx9 encoding: vmcnt[3:0] | expcnt[6:4]=7 | lgkmcnt[11:8]=15 | vmcnt_hi[15:14]
  __builtin_amdgcn_s_waitcnt((N_WAIT & 15) | (7 << 4) | (15 << 8) | ((N_WAIT >> 4) << 14));
}

template <int K, int L, int LIMBS, bool RESID, bool DIRECT_G>
__global__ void __launch_bounds__(PBS1024_WAVES * 64, 1)
pbs1024_kernel(uint64_t* __restrict__ out, const uint64_t* __restrict__ out_idx,
               const uint64_t* __restrict__ luts, const uint64_t* __restrict__ lut_idx,
               const uint64_t* __restrict__ in, const uint64_t* __restrict__ in_idx,
               const cplx* __restrict__ fbsk, uint32_t n, uint32_t base_log, uint32_t num_samples,
               unsigned long long* __restrict__ resid_out) {
  static_assert(LIMBS == 3, "MAGIC_ALL assumes limb shifts 0, 22, 43");
  constexpr int N = 1024, LOG2_2N = 11, K1 = K + 1, RQ = K1 * L;
  constexpr int NSL = K1 * LIMBS;                    // key slices per CMUX step
  constexpr int SLICE = RQ * 512;                    // complex values per slice
  constexpr int PER_I = NSL * SLICE;                 // complex values per Fourier GGSW
  constexpr int GLDS = SLICE / 64 / PBS1024_WAVES;   // 1 KB LDS-DMA pieces per wave per slice
  static_assert(SLICE % (64 * PBS1024_WAVES) == 0, "slice split");
  static_assert(GLDS < 32, "vmcnt range");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  cplx* tw1 = reinterpret_cast<cplx*>(smem);
  cplx* tw2 = tw1 + 512;
  cplx* zeta = tw2 + 64;
  cplx* xch_all = zeta + 512;
  cplx* ring = xch_all + PBS1024_WAVES * 512;  // 2 slots of SLICE

  // wave index made wave-uniform (SGPR) so per-ciphertext addresses and a_i use scalar loads
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t s = blockIdx.x * PBS1024_WAVES + wave;
  const bool active = s < num_samples;
  cplx* xch = xch_all + wave * 512;
  uint64_t* xch64 = reinterpret_cast<uint64_t*>(xch);
  const Fft512Tables T{tw1, tw2};

  // ---- LDS-DMA of key slice g (step g / NSL, slice g % NSL) into ring slot g & 1 -------
  const uint64_t total_slices = (uint64_t)n * NSL;
  auto issue_slice = [&](uint64_t g) {
    const cplx* src = fbsk + (g / NSL) * (uint64_t)PER_I + (g % NSL) * (uint64_t)SLICE;
    cplx* dst = ring + (g & 1) * SLICE;
#pragma unroll
    for (int j = 0; j < GLDS; ++j) {
      const int piece = wave * GLDS + j;
      __builtin_amdgcn_global_load_lds(src + piece * 64 + lane, (lds_ptr_t)(dst + piece * 64), 16, 0, 0);
    }
  };
  issue_slice(0);
  if (total_slices > 1) issue_slice(1);

  build_tables_1024(tw1, tw2, zeta);
  __syncthreads();

  const uint64_t* lwe = in + (active ? (in_idx ? in_idx[s] : s) : 0) * (uint64_t)(n + 1);
  const uint64_t* lut = luts + (active && lut_idx ? lut_idx[s] : 0ull) * (uint64_t)(K1 * N);

  // ---- accumulator: acc = LUT * X^{-ms(b)} (polynomial_wrapping_monic_monomial_div) ----
  uint64_t A[K1][16];
  {
    const uint32_t bt = active ? modswitch(lwe[n], LOG2_2N) : 0u;
#pragma unroll
    for (int r = 0; r < K1; ++r)
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const uint32_t src = (uint32_t)(lane + 64 * m + bt) & (2 * N - 1);
        const uint64_t v = active ? lut[r * N + (src & (N - 1))] : 0ull;
        A[r][m] = src < N ? v : 0ull - v;
      }
  }

  const int nrep = 64 - L * (int)base_log;
  const int logB = (int)base_log;
  double max_resid = 0.0;

  uint64_t a_next = active ? lwe[0] : 0ull;
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t ai = a_next;
    if (i + 1 < n) a_next = active ? lwe[i + 1] : 0ull;
    const uint32_t at = modswitch(ai, LOG2_2N);
    // tfhe skips a zero mask element; at == 0 gives X^0 acc - acc = 0, whose product is 0
    const bool work = ai != 0ull && at != 0u;

    // ---- ct1 = acc * X^{at} - acc, decomposition, forward transforms (per wave) -------
    cplx X[RQ][8];
    if (work) {
#pragma unroll
      for (int r = 0; r < K1; ++r) {
#pragma unroll
        for (int m = 0; m < 16; ++m) xch64[lane + 64 * m] = A[r][m];
        wave_lds_fence();
        int32_t dig[L][16];
#pragma unroll
        for (int m = 0; m < 16; ++m) {
          const uint32_t src = (uint32_t)(lane + 64 * m - (int)at) & (2 * N - 1);
          const uint64_t rv = xch64[src & (N - 1)];
          const uint64_t c1 = (src < N ? rv : 0ull - rv) - A[r][m];
          uint64_t st = decomp_init(c1, nrep);
#pragma unroll
          for (int q = 0; q < L; ++q) dig[q][m] = decomp_next(st, logB);
        }
        wave_lds_fence();
#pragma unroll
        for (int q = 0; q < L; ++q) {
          cplx v[8];
#pragma unroll
          for (int m = 0; m < 8; ++m) {
            const cplx z = zeta[m * 64 + lane];
            const double a = (double)dig[q][m], b = (double)dig[q][m + 8];
            v[m] = {__builtin_fma(a, z.re, -b * z.im), __builtin_fma(a, z.im, b * z.re)};
          }
          fft512_fwd(v, xch, T, lane);
#pragma unroll
          for (int e = 0; e < 8; ++e) X[r * L + q][e] = v[e];
        }
      }
    }

    // ---- per key slice: MAC from the LDS ring, inverse transform, exact recombination --
    static_for<0, NSL>([&](auto SL) {
      constexpr int sl = decltype(SL)::value;
      const uint64_t g = (uint64_t)i * NSL + sl;
      // slice g landed for this wave's pieces (slice g+1's pieces may stay in flight) ...
      if (g + 1 < total_slices) wait_vmcnt<GLDS>();
      else wait_vmcnt<0>();
      // ... and for every wave's pieces
      __builtin_amdgcn_s_barrier();
      const cplx* G = DIRECT_G ? fbsk + (g / NSL) * (uint64_t)PER_I + (g % NSL) * (uint64_t)SLICE
                               : ring + (g & 1) * SLICE;
      cplx Y[8];
      if (work) {
#pragma unroll
        for (int e = 0; e < 8; ++e) Y[e] = {0.0, 0.0};
#pragma unroll
        for (int rq = 0; rq < RQ; ++rq) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const cplx gv = G[rq * 512 + e * 64 + lane];
            const cplx x = X[rq][e];
            Y[e].re = __builtin_fma(x.re, gv.re, __builtin_fma(-x.im, gv.im, Y[e].re));
            Y[e].im = __builtin_fma(x.re, gv.im, __builtin_fma(x.im, gv.re, Y[e].im));
          }
        }
      }
      // every wave has read slot g & 1: refill it with slice g + 2
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (g + 2 < total_slices) issue_slice(g + 2);
      if (work) {
        constexpr int c = sl / LIMBS, li = sl % LIMBS;
        constexpr int shift = li * (64 / LIMBS) + (li < (64 % LIMBS) ? li : (64 % LIMBS));
        fft512_inv(Y, xch, T, lane);
#pragma unroll
        for (int m = 0; m < 8; ++m) {
          const cplx z = zeta[m * 64 + lane];
          const double cr = __builtin_fma(Y[m].re, z.re, Y[m].im * z.im);
          const double ci = __builtin_fma(Y[m].im, z.re, -Y[m].re * z.im);
          const double tr = cr + RND_MAGIC, ti = ci + RND_MAGIC;
          if constexpr (RESID) {
            max_resid = fmax(max_resid, fabs(cr - (tr - RND_MAGIC)));
            max_resid = fmax(max_resid, fabs(ci - (ti - RND_MAGIC)));
          }
          // bits(t) = MAGIC_BITS + round(v): the constant of all limbs is removed with limb 0
          // (it must not survive into the next step's rotation: X^a * const != const)
          if constexpr (li == 0) {
            A[c][m] += (uint64_t)__double_as_longlong(tr) - MAGIC_ALL;
            A[c][m + 8] += (uint64_t)__double_as_longlong(ti) - MAGIC_ALL;
          } else {
            A[c][m] += (uint64_t)__double_as_longlong(tr) << shift;
            A[c][m + 8] += (uint64_t)__double_as_longlong(ti) << shift;
          }
        }
      }
    });
  }

  if (active) {
    // ---- sample extract (nth = 0): out[rN + j] = -A_r[N - j] (j > 0), A_r[0]; body B[0] --
    uint64_t* o = out + (out_idx ? out_idx[s] : s) * (uint64_t)(K * N + 1);
#pragma unroll
    for (int r = 0; r < K; ++r) {
#pragma unroll
      for (int m = 0; m < 16; ++m) xch64[lane + 64 * m] = A[r][m];
      wave_lds_fence();
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const int j = lane + 64 * m;
        const uint64_t v = xch64[(N - j) & (N - 1)];
        o[r * N + j] = j == 0 ? v : 0ull - v;
      }
      wave_lds_fence();
    }
    if (lane == 0) o[K * N] = A[K][0];
  }

  if constexpr (RESID) {
    for (int off = 32; off > 0; off >>= 1) max_resid = fmax(max_resid, __shfl_xor(max_resid, off));
    if (lane == 0 && active && resid_out) atomicMax(resid_out, (unsigned long long)__double_as_longlong(max_resid));
  }
}

// ------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------
template <int K, int L, int LIMBS, bool RESID, bool DIRECT_G = false>
static int launch_1024_t(const PbsArgs& a) {
  const size_t lds = pbs1024_lds_bytes(K, L);
  const uint32_t blocks = (a.num_samples + PBS1024_WAVES - 1) / PBS1024_WAVES;
  auto kern = pbs1024_kernel<K, L, LIMBS, RESID, DIRECT_G>;
  CHIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(PBS1024_WAVES * 64), lds, a.stream, a.out, a.out_idx, a.luts, a.lut_idx,
                     a.in, a.in_idx, reinterpret_cast<const cplx*>(a.fbsk), a.n, a.base_log, a.num_samples, a.resid);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("pbs launch failed: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

template <int K, int L, int LIMBS>
static int launch_1024(const PbsArgs& a) {
  if (a.num_samples == 0 || a.n == 0) return a.n == 0 ? -3 : 0;
  // diagnostic: CONCRETE_HIP_PBS_DIRECT_KEY=1 reads the key from global memory instead of the LDS ring
  static const bool direct = getenv("CONCRETE_HIP_PBS_DIRECT_KEY") && atoi(getenv("CONCRETE_HIP_PBS_DIRECT_KEY"));
  if (direct) return launch_1024_t<K, L, LIMBS, true, true>(a);
  return a.resid ? launch_1024_t<K, L, LIMBS, true>(a) : launch_1024_t<K, L, LIMBS, false>(a);
}

int pbs_launch(const PbsArgs& a) {
  if (a.N == 1024 && a.k == 1 && a.limbs == 3) {
    switch (a.level) {
      case 1: return launch_1024<1, 1, 3>(a);
      case 2: return launch_1024<1, 2, 3>(a);
      case 3: return launch_1024<1, 3, 3>(a);
      default: break;
    }
  }
  set_error("unsupported PBS parameters: N=%u k=%u level=%u limbs=%u", a.N, a.k, a.level, a.limbs);
  return -2;
}

}  // namespace chip
