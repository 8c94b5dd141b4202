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
// Mapping (N = 1024, k = 1): a workgroup of two waves bootstraps one ciphertext.  Wave h
//   * owns GLWE polynomial h of the accumulator (16 u64 per lane: lane t holds t + 64 m),
//   * computes the l forward transforms of its own polynomial's digits,
//   * keeps frequency slots k2 in [4h, 4h + 4) of all (k+1) l digit spectra (the other half
//     goes to its partner through LDS),
//   * runs the multiply-accumulate with the Fourier key on its half of the frequencies for
//     both output polynomials, trades the partner's half, and runs the l inverse transforms
//     of its own output polynomial.
// So each wave needs < 256 VGPRs (two waves per SIMD) and the 630-step CMUX loop stays in one
// launch; the two waves meet at 2l + 2 workgroup barriers per step.
#include <type_traits>

#include "common.hpp"
#include "fft512.hpp"
#include "pbs.hpp"

namespace chip {

// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E)
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// bits(v + 1.5 * 2^52) = bits(1.5 * 2^52) + round(v) for |v| < 2^51
constexpr double RND_MAGIC = 6755399441055744.0;
constexpr uint64_t RND_MAGIC_BITS = 0x4338000000000000ull;
// sum over limbs of RND_MAGIC_BITS << shift(limb), LIMBS = 3 (shifts 0, 22, 43)
constexpr uint64_t MAGIC_ALL = RND_MAGIC_BITS + (RND_MAGIC_BITS << 22) + (RND_MAGIC_BITS << 43);
constexpr int limb_shift(int li) { return li * 21 + (li > 0 ? 1 : 0); }

// Workgroup barrier for the two waves of a ciphertext: LDS writes drained, compiler fence,
// no vmcnt drain (key loads may stay in flight).
__device__ __forceinline__ void pair_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Diagnostic cycle stamps (STAMPS builds only; never in the product kernel).
__device__ __forceinline__ uint64_t stamp() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
constexpr int NSTAMP = 8;  // rot+decomp, fwd+xchg, mac, y-xchg, inv+recomb, -, total, steps

template <int L, bool RESID, bool STAMPS>
__global__ void __launch_bounds__(128, 2)
pbs1024_pair_kernel(uint64_t* __restrict__ out, const uint64_t* __restrict__ out_idx,
                    const uint64_t* __restrict__ luts, const uint64_t* __restrict__ lut_idx,
                    const uint64_t* __restrict__ in, const uint64_t* __restrict__ in_idx,
                    const cplx* __restrict__ fbsk, uint32_t n, uint32_t base_log,
                    unsigned long long* __restrict__ resid_out) {
  constexpr int K = 1, K1 = 2, N = 1024, LOG2_2N = 11, LIMBS = 3, RQ = K1 * L;
  constexpr int SLICE = RQ * 512;            // complex values per (column, limb) key slice
  constexpr int PER_I = K1 * LIMBS * SLICE;  // complex values per Fourier GGSW
  static_assert(XCH_SLOTS <= (int)PBS1024_XCH_SLOTS, "transpose scratch");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  cplx* T1 = reinterpret_cast<cplx*>(smem);
  cplx* T2 = T1 + 512;
  cplx* xch_all = T2 + 64;  // 2 x PBS1024_XCH_SLOTS: per-wave transpose scratch, also the mailbox

  const int h = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave = polynomial = half
  const int lane = threadIdx.x & 63;
  const uint32_t s = blockIdx.x;
  cplx* xch = xch_all + h * PBS1024_XCH_SLOTS;
  uint64_t* xch64 = reinterpret_cast<uint64_t*>(xch);
  cplx* mybox = xch;                                  // the half-spectrum mailbox is the
  const cplx* partnerbox = xch_all + (1 - h) * PBS1024_XCH_SLOTS;   // transpose scratch, between transforms

  build_fft512_tables(T1, T2, threadIdx.x, 128);
  __syncthreads();
  const Fft512Tables T{T1, T2};

  const uint64_t* lwe = in + (in_idx ? in_idx[s] : s) * (uint64_t)(n + 1);
  const uint64_t* lut = luts + (lut_idx ? lut_idx[s] : 0ull) * (uint64_t)(K1 * N);

  // acc_h = LUT_h * X^{-ms(b)}  (blind_rotate_assign: polynomial_wrapping_monic_monomial_div)
  uint64_t A[16];
  {
    const uint32_t bt = modswitch(lwe[n], LOG2_2N);
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const uint32_t src = (uint32_t)(lane + 64 * m + bt) & (2 * N - 1);
      const uint64_t v = lut[h * N + (src & (N - 1))];
      A[m] = src < N ? v : 0ull - v;
    }
  }

  const int nrep = 64 - L * (int)base_log;
  const int logB = (int)base_log;
  double max_resid = 0.0;
  uint64_t acc_t[NSTAMP] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t t_begin = 0, tp = 0;
  if constexpr (STAMPS) t_begin = stamp();

  uint64_t a_next = lwe[0];
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t ai = a_next;
    if (i + 1 < n) a_next = lwe[i + 1];
    const uint32_t at = modswitch(ai, LOG2_2N);
    // tfhe skips a zero mask element; at == 0 gives X^0 acc - acc = 0 whose product is 0.
    // The condition depends only on the ciphertext: uniform across the pair.
    if (ai == 0ull || at == 0u) continue;
    if constexpr (STAMPS) {
      tp = stamp();
      acc_t[7] += 1;
    }

    // ---- own polynomial: ct1 = acc * X^{at} - acc, decomposer state per coefficient ------
    uint64_t st[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) xch64[lane + 64 * m] = A[m];
    wave_lds_fence();
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const uint32_t src = (uint32_t)(lane + 64 * m - (int)at) & (2 * N - 1);
      const uint64_t rv = xch64[src & (N - 1)];
      st[m] = decomp_init((src < N ? rv : 0ull - rv) - A[m], nrep);
    }
    wave_lds_fence();
    if constexpr (STAMPS) {
      uint64_t t = stamp();
      acc_t[0] += t - tp;
      tp = t;
    }

    // ---- forward transforms; keep my half of the slots, mail the other half -------------
    // X[row][q][j]: digit spectrum (row, level q) at slot k2 = 4h + j
    cplx X[K1][L][4];
#pragma unroll
    for (int q = 0; q < L; ++q) {
      cplx v[8];
      // digits of level l - q (the decomposition iterator yields the least significant first)
      int32_t d[16];
#pragma unroll
      for (int m = 0; m < 16; ++m) d[m] = decomp_next(st[m], logB);
#pragma unroll
      for (int m = 0; m < 8; ++m) v[m] = {(double)d[m], (double)d[m + 8]};
      fft512_fwd(v, xch, T, lane);
      if (h == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          X[0][q][j] = v[j];
          mybox[j * 64 + lane] = v[4 + j];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          X[1][q][j] = v[4 + j];
          mybox[j * 64 + lane] = v[j];
        }
      }
      pair_barrier();
      if (h == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) X[1][q][j] = partnerbox[j * 64 + lane];
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) X[0][q][j] = partnerbox[j * 64 + lane];
      }
      pair_barrier();  // partner has read my mailbox: my scratch is free again
    }
    if constexpr (STAMPS) {
      uint64_t t = stamp();
      acc_t[1] += t - tp;
      tp = t;
    }

    // ---- per limb: MAC for both output polynomials on my half, trade halves, inverse ----
    const cplx* Gi = fbsk + (uint64_t)i * PER_I + (4 * h) * 64 + lane;
    static_for<0, LIMBS>([&](auto LI) {
      constexpr int li = decltype(LI)::value;
      cplx Ymine[4];
#pragma unroll
      for (int cc = 0; cc < K1; ++cc) {
        // the partner's polynomial first (its half goes to the mailbox), then mine
        const int c = cc == 0 ? 1 - h : h;
        const cplx* G = Gi + (c * LIMBS + li) * SLICE;
        cplx Y[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) Y[j] = {0.0, 0.0};
        // rolling prefetch: key slots of spectrum rq + PF are in flight while rq is consumed
        constexpr int PF = 2;
        cplx gq[PF + 1][4];
#pragma unroll
        for (int p = 0; p < PF; ++p)
#pragma unroll
          for (int j = 0; j < 4; ++j) gq[p][j] = G[(p * 8 + j) * 64];
        static_for<0, RQ>([&](auto RQI) {
          constexpr int rq = decltype(RQI)::value;
          if constexpr (rq + PF < RQ) {
            // an opaque copy of the pointer pins these loads here (no hoisting of the whole slice)
            const cplx* Gl = G;
            asm volatile("" : "+v"(Gl));
#pragma unroll
            for (int j = 0; j < 4; ++j) gq[(rq + PF) % (PF + 1)][j] = Gl[((rq + PF) * 8 + j) * 64];
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const cplx gv = gq[rq % (PF + 1)][j];
            const cplx x = X[rq / L][rq % L][j];
            Y[j].re = __builtin_fma(x.re, gv.re, __builtin_fma(-x.im, gv.im, Y[j].re));
            Y[j].im = __builtin_fma(x.re, gv.im, __builtin_fma(x.im, gv.re, Y[j].im));
          }
          __builtin_amdgcn_sched_barrier(0);
        });
        if (cc == 0) {
#pragma unroll
          for (int j = 0; j < 4; ++j) mybox[j * 64 + lane] = Y[j];
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) Ymine[j] = Y[j];
        }
      }
      if constexpr (STAMPS) {
        uint64_t t = stamp();
        acc_t[2] += t - tp;
        tp = t;
      }
      pair_barrier();
      cplx v[8];
      if (h == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] = Ymine[j];
          v[4 + j] = partnerbox[j * 64 + lane];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] = partnerbox[j * 64 + lane];
          v[4 + j] = Ymine[j];
        }
      }
      pair_barrier();
      if constexpr (STAMPS) {
        uint64_t t = stamp();
        acc_t[3] += t - tp;
        tp = t;
      }
      fft512_inv(v, xch, T, lane);
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const double tr = v[m].re + RND_MAGIC, ti = v[m].im + RND_MAGIC;
        if constexpr (RESID) {
          max_resid = fmax(max_resid, fabs(v[m].re - (tr - RND_MAGIC)));
          max_resid = fmax(max_resid, fabs(v[m].im - (ti - RND_MAGIC)));
        }
        // bits(t) = MAGIC_BITS + round(v): the constant of all limbs is removed with limb 0
        // (it must not survive into the next step's rotation: X^a * const != const)
        if constexpr (li == 0) {
          A[m] += (uint64_t)__double_as_longlong(tr) - MAGIC_ALL;
          A[m + 8] += (uint64_t)__double_as_longlong(ti) - MAGIC_ALL;
        } else {
          A[m] += (uint64_t)__double_as_longlong(tr) << limb_shift(li);
          A[m + 8] += (uint64_t)__double_as_longlong(ti) << limb_shift(li);
        }
      }
      if constexpr (STAMPS) {
        uint64_t t = stamp();
        acc_t[4] += t - tp;
        tp = t;
      }
    });
  }

  if constexpr (STAMPS) {
    acc_t[6] = stamp() - t_begin;
    if (lane == 0 && resid_out) {
      unsigned long long* dst = resid_out + ((uint64_t)blockIdx.x * 2 + h) * NSTAMP;
      for (int q = 0; q < NSTAMP; ++q) dst[q] = acc_t[q];
    }
  }

  // ---- sample extract (nth = 0): out[j] = -A_0[N - j] (j > 0), A_0[0]; body B[0] -------
  uint64_t* o = out + (out_idx ? out_idx[s] : s) * (uint64_t)(K * N + 1);
  if (h == 0) {
#pragma unroll
    for (int m = 0; m < 16; ++m) xch64[lane + 64 * m] = A[m];
    wave_lds_fence();
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int j = lane + 64 * m;
      const uint64_t v = xch64[(N - j) & (N - 1)];
      o[j] = j == 0 ? v : 0ull - v;
    }
  } else if (lane == 0) {
    o[K * N] = A[0];
  }

  if constexpr (RESID && !STAMPS) {
    for (int off = 32; off > 0; off >>= 1) max_resid = fmax(max_resid, __shfl_xor(max_resid, off));
    if (lane == 0 && resid_out) atomicMax(resid_out, (unsigned long long)__double_as_longlong(max_resid));
  }
}

// ------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------
template <int L, bool RESID, bool STAMPS>
static int launch_pair_t(const PbsArgs& a) {
  const size_t lds = pbs1024_pair_lds_bytes(L);
  auto kern = pbs1024_pair_kernel<L, RESID, STAMPS>;
  CHIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(kern, dim3(a.num_samples), dim3(128), lds, a.stream, a.out, a.out_idx, a.luts, a.lut_idx, a.in,
                     a.in_idx, reinterpret_cast<const cplx*>(a.fbsk), a.n, a.base_log, a.resid);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("pbs launch failed: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

template <int L>
static int launch_pair(const PbsArgs& a) {
  if (a.num_samples == 0) return 0;
  // diagnostic: CONCRETE_HIP_PBS_STAMPS=1 runs the s_memtime-instrumented build; `resid` must then
  // point at 2 * num_samples * 8 u64 (per-wave cycle sums per phase)
  static const bool stamps = getenv("CONCRETE_HIP_PBS_STAMPS") && atoi(getenv("CONCRETE_HIP_PBS_STAMPS"));
  if (stamps) return launch_pair_t<L, true, true>(a);
  return a.resid ? launch_pair_t<L, true, false>(a) : launch_pair_t<L, false, false>(a);
}

int pbs_launch(const PbsArgs& a) {
  if (a.N == 1024 && a.k == 1 && a.limbs == 3) {
    switch (a.level) {
      case 1: return launch_pair<1>(a);
      case 2: return launch_pair<2>(a);
      case 3: return launch_pair<3>(a);
      default: break;
    }
  }
  set_error("unsupported PBS parameters: N=%u k=%u level=%u limbs=%u", a.N, a.k, a.level, a.limbs);
  return -2;
}

}  // namespace chip
