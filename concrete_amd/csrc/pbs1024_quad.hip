// pbs1024_quad.hip — the N = 1024, k = 1 PBS (cfg2) for small batches: four waves per ciphertext.
//
// Same semantics, key, key layout, ring and exact arithmetic as pbs1024_pair_kernel (pbs.hip).
// Why: at <= 2 ciphertexts per CU (the metric's whole-node batch of 4096 on 8 GPUs is 512 per GPU)
// the pair kernel has one wave per SIMD, and a wave alone on a SIMD issues its transforms and key
// products no faster than when it shares the SIMD with a second wave (stamps, DESIGN.md §4.1:
// 9.0k vs 9.5k cycles per step for the forward phase): the step is bound by one wave's issue
// and latency, not by the SIMD.  Interleaving two transforms in one wave did not change that
// (+2 %).  Here each ciphertext gets four waves, so two share every SIMD:
//
//   wave role v = 2c + h (c = GLWE polynomial, h = half).  Both waves of polynomial c hold its
//   (negated) accumulator and run the rotation and decomposition.
//   forward: h = 0 transforms levels 0 and 1, h = 1 level 2 (rounds F1 = {0, 2}, F2 = {1})
//   key products: frequency slots {2v, 2v + 1} of all six digit spectra, for both outputs
//   inverse: limb 0 by h = 0 and limb 1 by h = 1 (round IA), limb 2 by h = 1 (round IB)
//   each wave's rounded limb contributions reach its sibling through LDS once per step.
//
// The two ciphertexts of a workgroup are laid out so that every SIMD holds one h = 0 and one
// h = 1 wave (ciphertext 1's roles are those of ciphertext 0 with h flipped): in the rounds only
// one half works in (F2, IB), every SIMD still has one busy wave.
#include "common.hpp"
#include "fft512.hpp"
#include "kernel_util.hpp"
#include "pbs.hpp"

namespace chip {

namespace {

constexpr uint64_t Q_MAGIC_ALL = RND_MAGIC_BITS + (RND_MAGIC_BITS << 22) + (RND_MAGIC_BITS << 43);
constexpr int q_limb_shift(int li) { return li * 21 + (li > 0 ? 1 : 0); }

// Synchronisation of the four waves of one ciphertext (counters qf[ct * 4 + role]).
__device__ __forceinline__ void q_sync(uint32_t* qf, int ct, int v, uint32_t& cnt, const SyncGuard& guard) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  ++cnt;
  __hip_atomic_store(&qf[ct * 4 + v], cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
  for (int o = 1; o < 4; ++o) spin_until_ge(&qf[ct * 4 + ((v + o) & 3)], cnt, guard);
}
__device__ __forceinline__ void q_signal(uint32_t* qf, int ct, int v, uint32_t& cnt) {
  asm volatile("" ::: "memory");
  ++cnt;
  __hip_atomic_store(&qf[ct * 4 + v], cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void q_wait(uint32_t* qf, int ct, int v, uint32_t cnt, const SyncGuard& guard) {
#pragma unroll
  for (int o = 1; o < 4; ++o) spin_until_ge(&qf[ct * 4 + ((v + o) & 3)], cnt, guard);
  asm volatile("" ::: "memory");
}
// the two waves of one polynomial (separate counters pf[ct * 4 + role])
__device__ __forceinline__ void q_pair_sync(uint32_t* pf, int ct, int v, uint32_t& cnt, const SyncGuard& guard) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  ++cnt;
  __hip_atomic_store(&pf[ct * 4 + v], cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  spin_until_ge(&pf[ct * 4 + (v ^ 1)], cnt, guard);
}

}  // namespace

template <int CTS, bool RESID>
__global__ void __launch_bounds__(CTS * 256, 1)
pbs1024_quad_kernel(uint64_t* __restrict__ out, const uint64_t* __restrict__ out_idx,
                    const uint64_t* __restrict__ luts, const uint64_t* __restrict__ lut_idx,
                    const uint64_t* __restrict__ in, const uint64_t* __restrict__ in_idx,
                    const cplx* __restrict__ fbsk, uint32_t n, uint32_t base_log, uint32_t num_samples,
                    unsigned long long* __restrict__ resid_out, SyncGuard guard) {
  constexpr int K = 1, K1 = 2, N = 1024, LOG2_2N = 11, LIMBS = 3, L = 3, RQ = K1 * L;
  constexpr int PER_I = K1 * LIMBS * RQ * 512;  // complex values per Fourier GGSW
  constexpr int XS = (int)PBS1024_XCH_SLOTS;
  constexpr int NW = 4 * CTS;
  constexpr int GROUP = L * 512;           // one (limb, column, row) slice: the L level spectra
  constexpr int NGRP = K1 * K1 * LIMBS;
  constexpr int GLDS = GROUP / 64 / NW;    // 1 KB LDS-DMA pieces per wave per group
  static_assert(GROUP % (64 * NW) == 0 && NGRP % 3 == 0, "ring geometry");
  static_assert(XCH_SLOTS <= XS, "transpose scratch");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  cplx* tbl = reinterpret_cast<cplx*>(smem);
  cplx* xch_all = tbl + FFT512_TABLE_ENTRIES;  // NW scratches (transposes, spectra, mailboxes, deltas)
  cplx* ring = xch_all + NW * XS;              // 3 x GROUP key ring
  uint32_t* qf = reinterpret_cast<uint32_t*>(ring + 3 * GROUP);  // NW quad-sync counters
  uint32_t* pf = qf + NW;                                         // NW pair-sync counters

  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int ctl = w >> 2;
  const int v = (w & 3) ^ (ctl & 1);  // role (ciphertext 1: h flipped, see the header)
  const int c = v >> 1, h = v & 1;
  const uint32_t s = blockIdx.x * CTS + ctl;
  const bool active = s < num_samples;
  auto scr = [&](int role) __attribute__((always_inline)) {
    return xch_all + (ctl * 4 + (role ^ (ctl & 1))) * XS;
  };
  cplx* xch = xch_all + w * XS;
  uint64_t* xch64 = reinterpret_cast<uint64_t*>(xch);

  // ---- key ring (pbs1024_pair_kernel): group r = (li, co, ro) of the step -> slot r % 3
  const cplx* key_w = fbsk + (uint64_t)w * GLDS * 64;
  cplx* ring_w = ring + w * GLDS * 64;
  const uint32_t lane_b = (uint32_t)lane * (uint32_t)sizeof(cplx);
  auto issue_group = [&](const cplx* key_step, int r) __attribute__((always_inline)) {
    const char* src = reinterpret_cast<const char*>(key_step + r * GROUP);
    cplx* dst = ring_w + (r % 3) * GROUP;
#pragma unroll
    for (int j = 0; j < GLDS; ++j) {
      const cplx* gp = reinterpret_cast<const cplx*>(src + j * 1024 + lane_b);
      const uint32_t m0 = (uint32_t)(uintptr_t)(lds_ptr_t)(dst + j * 64);
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
      asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" : : "v"(gp), "s"(m0) : "m0", "memory");
#pragma clang diagnostic pop
    }
  };
  if (n > 0) {
    issue_group(key_w, 0);
    issue_group(key_w, 1);
  }

  build_fft512_tables(tbl, threadIdx.x, NW * 64);
  if (lane == 0) qf[w] = 0u, pf[w] = 0u;
  uint32_t qcnt = 0, pcnt = 0;
  __syncthreads();
  const Fft512Tables T = fft512_tables_at(tbl);

  const uint64_t* lwe = in + (active ? (in_idx ? in_idx[s] : s) : 0) * (uint64_t)(n + 1);
  const uint64_t* lut = luts + (active && lut_idx ? lut_idx[s] : 0ull) * (uint64_t)(K1 * N);

  // the negated accumulator B = -acc_c (pbs1024_pair_kernel), held by both waves of polynomial c
  uint64_t B[16];
  {
    const uint32_t bt = active ? modswitch(lwe[n], LOG2_2N) : 0u;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const uint32_t src = (uint32_t)(lane + 64 * m + bt) & (2 * N - 1);
      const uint64_t val = active ? lut[c * N + (src & (N - 1))] : 0ull;
      B[m] = src < N ? 0ull - val : val;
    }
  }

  const int nrep = 64 - L * (int)base_log;
  const int logB = (int)base_log;
  const int32_t neg_base = -(1 << logB);
  const uint32_t half_m1 = (1u << (logB - 1)) - 1u;
  double max_resid = 0.0;

  // my rounded limb contributions of the step (bits(MAGIC - v): negated, as B)
  uint64_t D[16];
  auto recombine = [&](const cplx (&vv)[8], auto LIc) __attribute__((always_inline)) {
    constexpr int lr = decltype(LIc)::value;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const double tr = RND_MAGIC - vv[m].re, ti = RND_MAGIC - vv[m].im;
      if constexpr (RESID) {
        max_resid = fmax(max_resid, fabs(vv[m].re - (RND_MAGIC - tr)));
        max_resid = fmax(max_resid, fabs(vv[m].im - (RND_MAGIC - ti)));
      }
      if constexpr (lr == 0) {
        D[m] += (uint64_t)__double_as_longlong(tr) - Q_MAGIC_ALL;
        D[m + 8] += (uint64_t)__double_as_longlong(ti) - Q_MAGIC_ALL;
      } else {
        D[m] += (uint64_t)__double_as_longlong(tr) << q_limb_shift(lr);
        D[m + 8] += (uint64_t)__double_as_longlong(ti) << q_limb_shift(lr);
      }
    }
  };
  auto inverse = [&](cplx (&vv)[8]) __attribute__((always_inline)) {
    cplx gi2[4];
    inv_p2_stage_tw(gi2, T, lane & 7);
    fft512_inv_tw(vv, xch, T, lane, gi2, 0);
  };

  uint64_t a_next = active ? lwe[0] : 0ull;
  for (uint32_t i = 0; i < n; ++i) {
    const cplx* key_step = key_w + (uint64_t)i * PER_I;
    const bool last_step = i + 1 >= n;
    const uint64_t ai = a_next;
    if (i + 1 < n) a_next = active ? lwe[i + 1] : 0ull;
    const uint32_t at = modswitch(ai, LOG2_2N);

    // ---- rotation and decomposer state in my own scratch (pbs1024_pair_kernel) ---------
    uint32_t st[16];
    {
#pragma unroll
      for (int m = 0; m < 16; ++m) xch64[lane + 64 * m] = B[m];
      wave_lds_fence();
      const uint32_t o0 = ((uint32_t)(lane - (int)at) << 3) + 8u * N;
      const uint32_t khi = 1u << (nrep - 33);
      uint64_t rv[16];
#pragma unroll
      for (int m = 0; m < 16; ++m)
        rv[m] = *reinterpret_cast<const uint64_t*>(reinterpret_cast<const char*>(xch64) + ((o0 + 512u * m) & 8191u));
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const uint32_t o = o0 + 512u * m;
        const uint32_t s32 = (uint32_t)((int32_t)(o << 18) >> 31);
        const uint64_t rvs = rv[m] ^ (((uint64_t)s32 << 32) | s32);
        const uint64_t x = B[m] + rvs + (uint64_t)(s32 & 1u);
        st[m] = ((uint32_t)(x >> 32) + khi) >> (nrep - 32);
      }
      wave_lds_fence();
    }

    // ---- digits: h = 0 keeps levels 0 and 1, h = 1 level 2 --------------------------------
    int32_t dA[16], dB[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int32_t d0 = decomp_level32(st[m], 0u, logB, half_m1, neg_base, true);
      const int32_t d1 = decomp_level32(st[m], (uint32_t)logB, logB, half_m1, neg_base, true);
      const int32_t d2 = decomp_level32(st[m], (uint32_t)(2 * logB), logB, half_m1, neg_base, false);
      dA[m] = h ? d2 : d0;
      dB[m] = d1;
    }

    // X[r][q][jj]: spectrum of digit polynomial (input row r ^ c, level q) at slot 2v + jj —
    // rows relative to my polynomial, as the key layout stores them (bsk.hip: slots 0..3 hold
    // column co / row ro of group (li, co, ro), slots 4..7 column 1 - co / row 1 - ro)
    cplx X[K1][L][2];
    cplx tw2[4], tw3[4];
    fwd_p2_tw(tw2, T, lane >> 3);
    fwd_p3_tw(tw3, T, lane);
    {  // F1: level 0 (h = 0) / level 2 (h = 1)
      cplx vv[8];
#pragma unroll
      for (int m = 0; m < 8; ++m) vv[m] = {(double)dA[m], (double)dA[m + 8]};
      fft512_fwd_tw(vv, xch, lane, tw2, tw3, 0, []() {});
#pragma unroll
      for (int k2 = 0; k2 < 8; ++k2) xch[k2 * 64 + lane] = vv[k2];
    }
    q_sync(qf, ctl, v, qcnt, guard);
#pragma unroll
    for (int r = 0; r < K1; ++r) {
      const int p = r ^ c;
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        X[r][0][jj] = scr(2 * p)[(2 * v + jj) * 64 + lane];
        X[r][2][jj] = scr(2 * p + 1)[(2 * v + jj) * 64 + lane];
      }
    }
#pragma unroll
    for (int r = 0; r < K1; ++r)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) pin(X[r][0][jj]), pin(X[r][2][jj]);
    q_signal(qf, ctl, v, qcnt);
    if (h == 0) {  // F2: level 1, published by the first key window's barrier
      cplx vv[8];
#pragma unroll
      for (int m = 0; m < 8; ++m) vv[m] = {(double)dB[m], (double)dB[m + 8]};
      fft512_fwd_tw(vv, xch, lane, tw2, tw3, 0, [&]() __attribute__((always_inline)) {
        q_wait(qf, ctl, v, qcnt, guard);  // my F1 spectrum has been read
      });
#pragma unroll
      for (int k2 = 0; k2 < 8; ++k2) xch[k2 * 64 + lane] = vv[k2];
    }

    // ---- key windows: both outputs, all three limbs, my two slots ------------------------
    // Y[li][co][jj]: output column co ^ c, slot 2v + jj
    cplx Y[LIMBS][K1][2];
    static_for<0, LIMBS>([&](auto LI) __attribute__((always_inline)) {
      constexpr int li = decltype(LI)::value;
#pragma unroll
      for (int co = 0; co < K1; ++co) {
#pragma unroll
        for (int ro = 0; ro < K1; ++ro) {
          const int r = (li * K1 + co) * K1 + ro;
          if (r + 1 < NGRP || !last_step) wait_vmcnt<GLDS>();
          else wait_vmcnt<0>();
          pair_barrier();
          if (r + 2 < NGRP) issue_group(key_step, r + 2);
          else if (!last_step) issue_group(key_step + PER_I, r + 2 - NGRP);
          if constexpr (li == 0) {
            if (co == 0 && ro == 0) {
#pragma unroll
              for (int rr = 0; rr < K1; ++rr)
#pragma unroll
                for (int jj = 0; jj < 2; ++jj) X[rr][1][jj] = scr(2 * (rr ^ c))[(2 * v + jj) * 64 + lane];
            }
          }
          const cplx* G = ring + (r % 3) * GROUP + (2 * v) * 64 + lane;
          cplx gv[L][2];
#pragma unroll
          for (int q = 0; q < L; ++q)
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) gv[q][jj] = G[q * 512 + jj * 64];
#pragma unroll
          for (int q = 0; q < L; ++q) {
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) {
              const cplx x = X[ro][q][jj];
              cplx& y = Y[li][co][jj];
              if (ro == 0 && q == 0) {
                y.re = __builtin_fma(x.re, gv[q][jj].re, -x.im * gv[q][jj].im);
                y.im = __builtin_fma(x.re, gv[q][jj].im, x.im * gv[q][jj].re);
              } else {
                y.re = __builtin_fma(x.re, gv[q][jj].re, __builtin_fma(-x.im, gv[q][jj].im, y.re));
                y.im = __builtin_fma(x.re, gv[q][jj].im, __builtin_fma(x.im, gv[q][jj].re, y.im));
              }
            }
          }
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) pin(Y[li][co][jj]);
        }
      }
    });

    // ---- inverse rounds ---------------------------------------------------------------
    // mailbox of (polynomial C, limb 0) = scratch of role 2C, (C, 1) and (C, 2) = role 2C + 1.
    // Every scratch is free: the last spectra were read right after the first window's barrier.
#pragma unroll
    for (int co = 0; co < K1; ++co) {
      const int C = co ^ c;
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        scr(2 * C)[(2 * v + jj) * 64 + lane] = Y[0][co][jj];
        scr(2 * C + 1)[(2 * v + jj) * 64 + lane] = Y[1][co][jj];
      }
    }
#pragma unroll
    for (int m = 0; m < 16; ++m) D[m] = 0ull;
    q_sync(qf, ctl, v, qcnt, guard);  // S1: mailboxes of limbs 0 and 1 complete
    {  // IA: limb h of my polynomial
      cplx vv[8];
#pragma unroll
      for (int k2 = 0; k2 < 8; ++k2) vv[k2] = xch[k2 * 64 + lane];
      inverse(vv);
      if (h == 0) recombine(vv, std::integral_constant<int, 0>{});
      else recombine(vv, std::integral_constant<int, 1>{});
    }
    if (h == 0) {  // my delta (limb 0) for my sibling, in my scratch
#pragma unroll
      for (int m = 0; m < 16; ++m) xch64[lane + 64 * m] = D[m];
    }
    q_sync(qf, ctl, v, qcnt, guard);  // S2: IA done everywhere; h = 0 deltas written
    uint64_t Dsib[16];
    if (h == 1) {
      const uint64_t* sib = reinterpret_cast<const uint64_t*>(scr(2 * c));
#pragma unroll
      for (int m = 0; m < 16; ++m) Dsib[m] = sib[lane + 64 * m];
    }
#pragma unroll
    for (int co = 0; co < K1; ++co) {
      const int C = co ^ c;
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) scr(2 * C + 1)[(2 * v + jj) * 64 + lane] = Y[2][co][jj];
    }
    q_sync(qf, ctl, v, qcnt, guard);  // S3: mailboxes of limb 2 complete (h = 1 scratches)
    if (h == 1) {  // IB: limb 2; then my delta (limbs 1 + 2) into my sibling's scratch
      cplx vv[8];
#pragma unroll
      for (int k2 = 0; k2 < 8; ++k2) vv[k2] = xch[k2 * 64 + lane];
      inverse(vv);
      recombine(vv, std::integral_constant<int, 2>{});
      uint64_t* sib = reinterpret_cast<uint64_t*>(scr(2 * c));
#pragma unroll
      for (int m = 0; m < 16; ++m) sib[lane + 64 * m] = D[m];
    }
    q_pair_sync(pf, ctl, v, pcnt, guard);  // P1: the h = 1 delta is in the h = 0 scratch
    if (h == 0) {
#pragma unroll
      for (int m = 0; m < 16; ++m) Dsib[m] = xch64[lane + 64 * m];
    }
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      B[m] += D[m] + Dsib[m];
      pin(B[m]);
    }
    if constexpr (RESID) pin(max_resid);
  }

  // ---- sample extract of acc = -B (pbs1024_pair_kernel), by the h = 0 waves -------------
  uint64_t* o = out + (active ? (out_idx ? out_idx[s] : s) : 0) * (uint64_t)(K * N + 1);
  if (!active || h != 0) {
  } else if (c == 0) {
#pragma unroll
    for (int m = 0; m < 16; ++m) xch64[lane + 64 * m] = B[m];
    wave_lds_fence();
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int j = lane + 64 * m;
      const uint64_t val = xch64[(N - j) & (N - 1)];
      o[j] = j == 0 ? 0ull - val : val;
    }
  } else if (lane == 0) {
    o[K * N] = 0ull - B[0];
  }

  if constexpr (RESID) {
    for (int off = 32; off > 0; off >>= 1) max_resid = fmax(max_resid, __shfl_xor(max_resid, off));
    if (lane == 0 && active && resid_out) atomicMax(resid_out, (unsigned long long)__double_as_longlong(max_resid));
  }
}

template <int CTS, bool RESID>
static int launch_quad_t(const PbsArgs& a) {
  const size_t lds = pbs1024_quad_lds_bytes(CTS);
  auto kern = pbs1024_quad_kernel<CTS, RESID>;
  CHIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const uint32_t blocks = (a.num_samples + CTS - 1) / CTS;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(CTS * 256), lds, a.stream, a.out, a.out_idx, a.luts, a.lut_idx, a.in,
                     a.in_idx, reinterpret_cast<const cplx*>(a.fbsk), a.n, a.base_log, a.num_samples, a.resid,
                     a.guard);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("pbs launch failed: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

int pbs1024_quad_launch(const PbsArgs& a, int cts) {
  if (!(a.N == 1024 && a.k == 1 && a.level == 3 && a.limbs == 3 && pbs1024_exact(1, 3, a.base_log))) {
    set_error("unsupported PBS parameters for the four-wave kernel: N=%u k=%u level=%u base_log=%u", a.N, a.k,
              a.level, a.base_log);
    return -2;
  }
  if (a.num_samples == 0) return 0;
  if (cts == 1) return a.resid ? launch_quad_t<1, true>(a) : launch_quad_t<1, false>(a);
  return a.resid ? launch_quad_t<2, true>(a) : launch_quad_t<2, false>(a);
}

}  // namespace chip
