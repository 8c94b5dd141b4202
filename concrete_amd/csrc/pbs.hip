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
// Mapping (N = 1024, k = 1): two waves per ciphertext, P ciphertexts per workgroup (P = 4; 2 or 1
// for batches too small to give every CU a workgroup of 4: launch_pair).
// Wave h of a pair
//   * owns GLWE polynomial h of the accumulator (16 u64 per lane: lane t holds t + 64 m),
//   * computes the l forward transforms of its own polynomial's digits,
//   * keeps frequency slots k2 in [4h, 4h + 4) of all (k+1) l digit spectra (the other half
//     goes to its partner through LDS),
//   * runs the multiply-accumulate with the Fourier key on its half of the frequencies for
//     both output polynomials, trades the partner's half, and runs the l inverse transforms
//     of its own output polynomial.
// Each wave stays < 256 VGPRs (two waves per SIMD).  The Fourier key is streamed through a
// 3-group LDS ring (24 KB groups = three spectra of one (column, limb) slice) filled by
// LDS-DMA (global_load_lds_dwordx4) and read by all P pairs, so it crosses the L2->CU
// port once per workgroup instead of once per ciphertext.  The whole CMUX loop runs in one
// launch with the workgroup in lockstep (one raw s_barrier per key group and per half-spectrum
// exchange).
#include <type_traits>

#include "common.hpp"
#include "fft512.hpp"
#include "kernel_util.hpp"
#include "pbs.hpp"
#include "pbs1024_plan.hpp"
#include "pbs_hex.hpp"

namespace chip {

// sum over limbs of RND_MAGIC_BITS << shift(limb), LIMBS = 3 (shifts 0, 22, 43)
constexpr uint64_t MAGIC_ALL = RND_MAGIC_BITS + (RND_MAGIC_BITS << 22) + (RND_MAGIC_BITS << 43);
constexpr int limb_shift(int li) { return li * 21 + (li > 0 ? 1 : 0); }

#ifndef FWD_LAST_VIA_WINDOW
#define FWD_LAST_VIA_WINDOW 1  // last forward exchange published by the first key window's barrier
#endif
#ifndef FWD_TW2_EARLY
#define FWD_TW2_EARLY 1  // forward pass-2 twiddles issued ahead of pass 1 (+0.4 %)
#endif
#ifndef DIAG_NOMAC
#define DIAG_NOMAC 0  // diagnostic builds only: skip the key MAC (wrong results)
#endif

#ifndef FWD_XBATCH
#define FWD_XBATCH 2  // forward levels traded per exchange (mailbox: 4 KB per level, <= 2)
#endif
#ifndef PAIR_FLAGS
#define PAIR_FLAGS 1  // half-spectrum exchanges synchronise the two waves of a pair only
#endif

// Synchronisation point of the half-spectrum exchanges.  PAIR_FLAGS: a pair-local barrier on
// LDS counters — each wave publishes how many sync points it has passed and waits for its
// partner to reach the same count — so the other pairs of the workgroup are not held up.
// Only LDS traffic is drained (lgkmcnt), never the key DMA (no release fence: that would add
// vmcnt(0)).  LDS operations are coherent across the waves of a CU.
// (DIAG_NOXBAR: timing-only builds without any exchange synchronisation.)
// Split form: pair_signal publishes that this wave has issued its reads of the partner's
// scratch (LDS operations of a wave execute in issue order, so the count is seen only after
// them); pair_wait, before this wave next overwrites its own scratch, waits for the partner's.
__device__ __forceinline__ void pair_signal(uint32_t* flags, int w, uint32_t& cnt) {
  asm volatile("" ::: "memory");
  ++cnt;
#if !defined(DIAG_NOXBAR)
  __hip_atomic_store(&flags[w], cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#endif
}
__device__ __forceinline__ void pair_wait(uint32_t* flags, int w, uint32_t cnt, const SyncGuard& guard) {
#if defined(DIAG_NOXBAR)
  (void)flags, (void)w, (void)cnt, (void)guard;
#else
  spin_until_ge(&flags[w ^ 1], cnt, guard);
#endif
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void xchg_barrier(uint32_t* flags, int w, uint32_t& cnt, const SyncGuard& guard) {
#if defined(DIAG_NOXBAR)
  (void)flags, (void)w, (void)cnt, (void)guard;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#elif PAIR_FLAGS
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  ++cnt;
  __hip_atomic_store(&flags[w], cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  spin_until_ge(&flags[w ^ 1], cnt, guard);
#else
  (void)flags, (void)w, (void)cnt, (void)guard;
  pair_barrier();
#endif
}

template <int P, int L, bool RESID, bool STAMPS>
__global__ void __launch_bounds__(P * 128, 2)
pbs1024_pair_kernel(uint64_t* __restrict__ out, const uint64_t* __restrict__ out_idx,
                    const uint64_t* __restrict__ luts, const uint64_t* __restrict__ lut_idx,
                    const uint64_t* __restrict__ in, const uint64_t* __restrict__ in_idx,
                    const cplx* __restrict__ fbsk, uint32_t n, uint32_t base_log, uint32_t num_samples,
                    unsigned long long* __restrict__ resid_out, SyncGuard guard) {
  constexpr int K = 1, K1 = 2, N = 1024, LOG2_2N = 11, LIMBS = 3, RQ = K1 * L;
  constexpr int PER_I = K1 * LIMBS * RQ * 512;  // complex values per Fourier GGSW
  static_assert(XCH_SLOTS <= (int)PBS1024_XCH_SLOTS, "transpose scratch");
  static_assert(FFT512_TABLE_ENTRIES * sizeof(cplx) == PBS1024_TABLE_BYTES, "table bytes");
  constexpr int NW = 2 * P;                   // waves per workgroup
  constexpr int GROUP = L * 512;              // complex values per ring group (one row of a slice)
  constexpr int NGRP = K1 * K1 * LIMBS;       // ring groups per CMUX step
  constexpr int GLDS = GROUP / 64 / NW;       // 1 KB LDS-DMA pieces per wave per group
  static_assert(GROUP % (64 * NW) == 0, "group split");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  cplx* tbl = reinterpret_cast<cplx*>(smem);      // FFT tables (fft512.hpp)
  cplx* xch_all = tbl + FFT512_TABLE_ENTRIES;     // NW x PBS1024_XCH_SLOTS: transpose scratch,
  cplx* ring = xch_all + NW * PBS1024_XCH_SLOTS;  // also the mailbox; 3 x GROUP key ring
  uint32_t* pflags = reinterpret_cast<uint32_t*>(ring + 3 * GROUP);  // NW pair-sync counters

  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = w & 1;  // polynomial = frequency half
  const uint64_t hsign = (uint64_t)h << 63;  // sign mask of the k2 ^ 4 relabeling (h = 1)
  const int lane = threadIdx.x & 63;
  const uint32_t s = blockIdx.x * P + (w >> 1);
  const bool active = s < num_samples;
  cplx* xch = xch_all + w * PBS1024_XCH_SLOTS;
  uint64_t* xch64 = reinterpret_cast<uint64_t*>(xch);
  cplx* mybox = xch;                                  // the half-spectrum mailbox is the
  const cplx* partnerbox = xch_all + (w ^ 1) * PBS1024_XCH_SLOTS;   // transpose scratch, between transforms
  cplx* partnermail = xch_all + (w ^ 1) * PBS1024_XCH_SLOTS;

  // ---- key ring: group g = (step g / NGRP, limb, co, ro) -> slot g % 3 ---------------------
  // Both waves of a pair read the same group at the same time, each its own half of the slots:
  // group (li, co, ro) holds, for slots 0..3, column co / row ro and, for slots 4..7, column
  // 1 - co / row 1 - ro, i.e. "own"/"other" relative to the reading wave (bsk.hip).
  // Within a step every group index r = (li K1 + co) K1 + ro is a compile-time constant and
  // NGRP is a multiple of 3, so a group's slot (r % 3) and its offset from the step's key base
  // are constants too: the refill is one wave-uniform base plus immediates, no division.
  static_assert(NGRP % 3 == 0, "ring slot of a group must not depend on the step");
  const cplx* key_w = fbsk + (uint64_t)w * GLDS * 64;  // this wave's pieces of every group
  cplx* ring_w = ring + w * GLDS * 64;
  const uint32_t lane_b = (uint32_t)lane * (uint32_t)sizeof(cplx);  // zero-extended lane offset
  auto issue_group = [&](const cplx* key_step, int r) __attribute__((always_inline)) {
    const char* src = reinterpret_cast<const char*>(key_step + r * GROUP);
    cplx* dst = ring_w + (r % 3) * GROUP;
#pragma unroll
    for (int j = 0; j < GLDS; ++j)
    {
      // Issued from inline assembly so that the compiler does not see an LDS write: with the
      // builtin it treats every window's key reads as possibly aliasing the DMA and waits for
      // all twelve (lgkmcnt(0)) before the first FMA; here it counts them (lgkmcnt(4) ...):
      // +1.1 % PBS/s.  The ring is ordered by the explicit vmcnt waits and workgroup barriers
      // alone.  M0 (the LDS base of the piece) is set inside the statement; nothing else in the
      // kernel uses M0.
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

  build_fft512_tables(tbl, threadIdx.x, P * 128);
  if (lane == 0) pflags[w] = 0u;
  uint32_t pcnt = 0;
  __syncthreads();
  const Fft512Tables T = fft512_tables_at(tbl);

  const uint64_t* lwe = in + (active ? (in_idx ? in_idx[s] : s) : 0) * (uint64_t)(n + 1);
  const uint64_t* lut = luts + (active && lut_idx ? lut_idx[s] : 0ull) * (uint64_t)(K1 * N);

  // acc_h = LUT_h * X^{-ms(b)}  (blind_rotate_assign: polynomial_wrapping_monic_monomial_div).
  // The wave keeps the NEGATED accumulator B = -acc_h (16 u64 per lane): the step's
  // X^a acc - acc = B - X^a B then needs no 64-bit negation, and the recombination adds the
  // rounded negated products, which the f64 rounding gives for free (MAGIC - v).
  uint64_t B[16];
  {
    const uint32_t bt = active ? modswitch(lwe[n], LOG2_2N) : 0u;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const uint32_t src = (uint32_t)(lane + 64 * m + bt) & (2 * N - 1);
      const uint64_t v = active ? lut[h * N + (src & (N - 1))] : 0ull;
      B[m] = src < N ? 0ull - v : v;
    }
  }

  const int nrep = 64 - L * (int)base_log;
  const int logB = (int)base_log;
  const int32_t neg_base = -(1 << logB);
  const uint32_t half_m1 = (1u << (logB - 1)) - 1u;
  double max_resid = 0.0;
  uint64_t acc_t[NSTAMP] = {};
  uint64_t t_begin = 0, tp = 0;
  if constexpr (STAMPS) t_begin = stamp();

  // forward pass-3 twiddles of my lane: constant for the whole kernel, kept in registers
  cplx tw3[4];
  fwd_p3_tw(tw3, T, lane);

  uint64_t a_next = active ? lwe[0] : 0ull;
  for (uint32_t i = 0; i < n; ++i) {
    const cplx* key_step = key_w + (uint64_t)i * PER_I;
    const uint64_t ai = a_next;
    if (i + 1 < n) a_next = active ? lwe[i + 1] : 0ull;

    const uint32_t at = modswitch(ai, LOG2_2N);
    // tfhe skips a zero mask element (and at == 0 changes nothing): the step still runs, on
    // ct1 = X^0 acc - acc = 0, whose digits, spectra and products are exact zeros, so the
    // recombination adds exactly 0 (the limb constants cancel).  Running every step keeps the
    // compiler from hoisting undefined values of skipped-step arrays out of the loop, where
    // they pinned ~110 VGPRs.
    if constexpr (STAMPS) {
      tp = stamp();
      acc_t[7] += ai != 0ull && at != 0u;
    }

    // ---- own polynomial: ct1 = acc * X^{at} - acc = B - X^{at} B, decomposer state per
    //      coefficient.  Coefficient j = lane + 64 m reads B[src & (N-1)], src = j - at mod 2N,
    //      negated when src >= N; o = 8 src + 8N (mod 2^32) carries the byte offset in bits 0..12
    //      and "src < N" in bit 13, so ct1 = B + (rv ^ s) - s with s = -(bit 13 of o).
    //      decomp_init(x) = (x >> nrep) + bit(nrep - 1) = (x + 2^(nrep-1)) >> nrep (a wrap of
    //      x + 2^(nrep-1) past 2^64 gives state 0 instead of 2^(l logB), both decomposing to zero
    //      digits); nrep >= 37 under the exactness gate, so only the high word is shifted.
    uint32_t st[16];
    {
#pragma unroll
      for (int m = 0; m < 16; ++m) xch64[lane + 64 * m] = B[m];
      wave_lds_fence();
      const uint32_t o0 = ((uint32_t)(lane - (int)at) << 3) + 8u * N;
      const uint32_t khi = 1u << (nrep - 33);  // 2^(nrep-1) in the high word
      // all 16 reads in flight at once (left to itself the scheduler issues them four at a time,
      // one LDS round trip each)
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
    if constexpr (STAMPS) {
      uint64_t t = stamp();
      acc_t[0] += t - tp;
      tp = t;
    }

    // ---- forward transforms; keep my half of the slots, mail the other half -------------
    // Xo[q][j] / Xp[q][j]: spectrum of my own / my partner's digit polynomial (level q) at
    // frequency slot 4h + j.  The wave owning the upper half (h = 1) emits its spectrum in slot
    // order k2 ^ 4, so every wave keeps v[0..3] and mails v[4..7]: no h-dependent registers.
    cplx Xo[L][4], Xp[L][4];
    // levels are traded in batches of up to FWD_XBATCH (one mailbox of 4 KB per level): the
    // mailed halves of a batch wait in registers until its last transform is done
    constexpr int XB = FWD_XBATCH;
#pragma unroll
    for (int q0 = 0; q0 < L; q0 += XB) {
      const int nq = (q0 + XB <= L) ? XB : L - q0;
      cplx out[XB][4];
      {
#pragma unroll
        for (int t = 0; t < XB; ++t) {
          if (t < nq) {
            // digits of level l - q (the decomposition iterator yields the least significant first)
            cplx v[8];
            int32_t d[16];
#pragma unroll
            for (int m = 0; m < 16; ++m)
              d[m] = decomp_level32(st[m], (uint32_t)((q0 + t) * logB), logB, half_m1, neg_base, q0 + t + 1 < L);
#pragma unroll
            for (int m = 0; m < 8; ++m) v[m] = {(double)d[m], (double)d[m + 8]};
            // the first transform after a mailbox exchange overwrites my scratch: my partner
            // must have read the mailbox (it signals right after its reads)
            cplx tw2[4];
            fwd_p2_tw(tw2, T, lane >> 3);
            // issued here, ahead of pass 1 and the register transpose that hide their latency
            // (left alone the scheduler sinks each read to its butterfly stage, one exposed LDS
            // round trip per stage)
            if (FWD_TW2_EARLY) __builtin_amdgcn_sched_barrier(0);
            fft512_fwd_tw(v, xch, lane, tw2, tw3, hsign, [&]() __attribute__((always_inline)) {
              if (q0 > 0 && t == 0) pair_wait(pflags, w, pcnt, guard);
            });
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              Xo[q0 + t][j] = v[j];
              out[t][j] = v[4 + j];
            }
          }
        }
#pragma unroll
        for (int t = 0; t < XB; ++t)
          if (t < nq)
#pragma unroll
            for (int j = 0; j < 4; ++j) mybox[(t * 4 + j) * 64 + lane] = out[t][j];
      }
      // The last batch's halves need no pair sync: the first key window's workgroup barrier
      // (which drains every wave's LDS writes) publishes them, and they are first used in the
      // second window (row 1); they are read right after that barrier.
      const bool last_batch = q0 + XB >= L;
      if (!last_batch || !FWD_LAST_VIA_WINDOW) {
        xchg_barrier(pflags, w, pcnt, guard);
#pragma unroll
        for (int t = 0; t < XB; ++t)
          if (t < nq)
#pragma unroll
            for (int j = 0; j < 4; ++j) Xp[q0 + t][j] = partnerbox[(t * 4 + j) * 64 + lane];
      }
      // materialise this batch's spectra here (else its transforms sink into the key windows)
#pragma unroll
      for (int t = 0; t < XB; ++t)
        if (t < nq)
#pragma unroll
          for (int j = 0; j < 4; ++j) pin(Xo[q0 + t][j]);
      // my partner's mailbox has been read: signal it (it waits before its next transform writes
      // its scratch).  After the last batch the scratch is next written behind the key windows'
      // workgroup barriers.
      if (q0 + XB < L) pair_signal(pflags, w, pcnt);
    }
    if constexpr (STAMPS) {
      uint64_t t = stamp();
      acc_t[1] += t - tp;
      tp = t;
    }

    // ---- per limb: MAC for both output polynomials on my half (key from the LDS ring),
    //      trade halves through the mailbox, inverse transform of my polynomial. ------------
    // bits(MAGIC - v) = MAGIC_BITS - round(v): limb li's exact integers, negated (B = -acc),
    // shifted into B.  The constant of all limbs is removed with limb 0 (it must not survive into
    // the next step's rotation: X^a * const != const).
    auto recombine = [&](const cplx (&v)[8], auto LIc) __attribute__((always_inline)) {
      constexpr int lr = decltype(LIc)::value;
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const double tr = RND_MAGIC - v[m].re, ti = RND_MAGIC - v[m].im;
        if constexpr (RESID) {
          max_resid = fmax(max_resid, fabs(v[m].re - (RND_MAGIC - tr)));
          max_resid = fmax(max_resid, fabs(v[m].im - (RND_MAGIC - ti)));
        }
        if constexpr (lr == 0) {
          B[m] += (uint64_t)__double_as_longlong(tr) - MAGIC_ALL;
          B[m + 8] += (uint64_t)__double_as_longlong(ti) - MAGIC_ALL;
        } else {
          B[m] += (uint64_t)__double_as_longlong(tr) << limb_shift(lr);
          B[m + 8] += (uint64_t)__double_as_longlong(ti) << limb_shift(lr);
        }
      }
    };
    static_for<0, LIMBS>([&](auto LI) __attribute__((always_inline)) {
      constexpr int li = decltype(LI)::value;
      cplx Ymine[4];
      // co / ro: my own (0) or my partner's (1) output polynomial / input row; group
      // (li, co, ro) holds exactly those spectra for both halves (layout: bsk.hip)
#pragma unroll
      for (int co = 0; co < K1; ++co) {
        cplx Y[4];  // set by the first product of window ro = 0 (no zeroing)
        if constexpr (DIAG_NOMAC) {
#pragma unroll
          for (int j = 0; j < 4; ++j) Y[j] = {0.0, 0.0};
        }
#pragma unroll
        for (int ro = 0; ro < K1; ++ro) {
          const int r = (li * K1 + co) * K1 + ro;  // group within the step (constant)
          const bool last_step = i + 1 >= n;
          if constexpr (STAMPS) {
            uint64_t t = stamp();
            acc_t[2] += t - tp;
            tp = t;
          }
          // group g landed for this wave's pieces (group g + 1 may stay in flight) ...
          if (r + 1 < NGRP || !last_step) wait_vmcnt<GLDS>();
          else wait_vmcnt<0>();
          if constexpr (STAMPS) {
            uint64_t t = stamp();
            acc_t[8] += t - tp;
            tp = t;
          }
          // ... and for every wave's pieces; everyone is also done with group g - 1
#ifndef DIAG_NOBAR
          pair_barrier();
#endif
          if constexpr (STAMPS) {
            uint64_t t = stamp();
            acc_t[5] += t - tp;
            tp = t;
          }
          // refill the slot of group g - 1 with group g + 2, right after the barrier (the DMA
          // needs the lead time: issued after the window's reads or FMAs it measured slower)
#ifndef DIAG_NODMA
          if (r + 2 < NGRP) issue_group(key_step, r + 2);
          else if (!last_step) issue_group(key_step + PER_I, r + 2 - NGRP);
#endif
          if constexpr (FWD_LAST_VIA_WINDOW && li == 0) {
            if (co == 0 && ro == 0) {
              constexpr int QL = (L - 1) / FWD_XBATCH * FWD_XBATCH;  // first level of the last batch
#pragma unroll
              for (int q = QL; q < L; ++q)
#pragma unroll
                for (int j = 0; j < 4; ++j) Xp[q][j] = partnerbox[((q - QL) * 4 + j) * 64 + lane];
            }
          }
          const cplx* G = ring + (r % 3) * GROUP + (4 * h) * 64 + lane;
          // all key values of the window first, then the FMAs
          cplx gv[L][4];
#pragma unroll
          for (int q = 0; q < L; ++q)
#pragma unroll
            for (int j = 0; j < 4; ++j) gv[q][j] = G[(q * 8 + j) * 64];
#pragma unroll
          for (int q = 0; q < (DIAG_NOMAC ? 0 : L); ++q) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const cplx x = ro == 0 ? Xo[q][j] : Xp[q][j];
              if (ro == 0 && q == 0) {  // fma(a, b, 0) == a * b: same bits as accumulating from 0
                Y[j].re = __builtin_fma(x.re, gv[q][j].re, -x.im * gv[q][j].im);
                Y[j].im = __builtin_fma(x.re, gv[q][j].im, x.im * gv[q][j].re);
              } else {
                Y[j].re = __builtin_fma(x.re, gv[q][j].re, __builtin_fma(-x.im, gv[q][j].im, Y[j].re));
                Y[j].im = __builtin_fma(x.re, gv[q][j].im, __builtin_fma(x.im, gv[q][j].re, Y[j].im));
              }
            }
          }
          // this window's products are done here, not sunk past the next window's barrier
#pragma unroll
          for (int j = 0; j < 4; ++j) pin(Y[j]);
        }
        if (co == 0) {
#pragma unroll
          for (int j = 0; j < 4; ++j) Ymine[j] = Y[j];
        } else {
          // straight into my partner's mailbox (its scratch has been idle since the key
          // windows' workgroup barriers), so no "partner has read" sync is needed afterwards
#pragma unroll
          for (int j = 0; j < 4; ++j) partnermail[j * 64 + lane] = Y[j];
        }
      }
      if constexpr (STAMPS) {
        uint64_t t = stamp();
        acc_t[2] += t - tp;
        tp = t;
      }
      xchg_barrier(pflags, w, pcnt, guard);
      // my output polynomial's spectrum, slots in order k2 ^ 4h (undone by the inverse pass 1)
      cplx vp[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        vp[j] = Ymine[j];
        vp[4 + j] = mybox[j * 64 + lane];
      }
      // no second sync: the only writes into my scratch by my partner are these Y mailboxes,
      // one per limb, always behind key-window workgroup barriers (the forward exchange only
      // reads the partner's scratch, under its own two syncs)
      if constexpr (STAMPS) {
        uint64_t t = stamp();
        acc_t[3] += t - tp;
        tp = t;
      }
      cplx gi2[4];  // inverse pass-2 stage twiddles, read ahead of the transpose
      inv_p2_stage_tw(gi2, T, lane & 7);
      fft512_inv_tw(vp, xch, T, lane, gi2, hsign);
      recombine(vp, LI);
      // materialise B here (else the inverse tail sinks into the next limb's key windows)
#pragma unroll
      for (int m = 0; m < 16; ++m) pin(B[m]);
      if constexpr (RESID) pin(max_resid);
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
      unsigned long long* dst = resid_out + ((uint64_t)blockIdx.x * NW + w) * NSTAMP;
      for (int q = 0; q < NSTAMP; ++q) dst[q] = acc_t[q];
    }
  }

  // ---- sample extract (nth = 0) of acc = -B: out[j] = -acc_0[N - j] (j > 0), acc_0[0]; body acc_1[0]
  uint64_t* o = out + (active ? (out_idx ? out_idx[s] : s) : 0) * (uint64_t)(K * N + 1);
  if (!active) {
  } else if (h == 0) {
    // acc = -B
#pragma unroll
    for (int m = 0; m < 16; ++m) xch64[lane + 64 * m] = B[m];
    wave_lds_fence();
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int j = lane + 64 * m;
      const uint64_t v = xch64[(N - j) & (N - 1)];
      o[j] = j == 0 ? 0ull - v : v;
    }
  } else if (lane == 0) {
    o[K * N] = 0ull - B[0];
  }

  if constexpr (RESID && !STAMPS) {
    for (int off = 32; off > 0; off >>= 1) max_resid = fmax(max_resid, __shfl_xor(max_resid, off));
    if (lane == 0 && active && resid_out) atomicMax(resid_out, (unsigned long long)__double_as_longlong(max_resid));
  }
}

// ------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------
template <int P, int L, bool RESID, bool STAMPS>
static int launch_pair_t(const PbsArgs& a) {
  const size_t lds = pbs1024_pair_lds_bytes(L, P);
  // the exactness gate (pbs1024_exact) keeps l * logB <= 27: the decomposer state fits 32 bits
  if (!pbs1024_exact(1, L, a.base_log)) {
    set_error("pbs: N=1024 l=%d logB=%u is outside the exact range", L, a.base_log);
    return -2;
  }
  auto kern = pbs1024_pair_kernel<P, L, RESID, STAMPS>;
  CHIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const uint32_t blocks = (a.num_samples + P - 1) / P;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(P * 128), lds, a.stream, a.out, a.out_idx, a.luts, a.lut_idx,
                     a.in, a.in_idx, reinterpret_cast<const cplx*>(a.fbsk), a.n, a.base_log, a.num_samples, a.resid,
                     a.guard);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("pbs launch failed: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

// compute units of the current device (cached per device)
static uint32_t device_cus() {
  static uint32_t cus[64] = {};
  int dev = 0;
  CHIP_CHECK(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) return 256;
  if (!cus[dev]) {
    int n = 0;
    CHIP_CHECK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
    cus[dev] = n > 0 ? (uint32_t)n : 256u;
  }
  return cus[dev];
}

template <int P, int L>
static int launch_pair_p(const PbsArgs& a) {
  // diagnostic: CONCRETE_HIP_PBS_STAMPS=1 runs the s_memtime-instrumented build; `resid` must then
  // point at 2 * P * ceil(num_samples / P) * NSTAMP u64 (per-wave cycle sums)
  static const bool stamps = getenv("CONCRETE_HIP_PBS_STAMPS") && atoi(getenv("CONCRETE_HIP_PBS_STAMPS"));
  if (stamps) return launch_pair_t<P, L, true, true>(a);
  return a.resid ? launch_pair_t<P, L, true, false>(a) : launch_pair_t<P, L, false, false>(a);
}

// the contiguous part [start, start + count) of a batched call: the index arrays (the runtime's u64
// in / out / LUT indexes, wrappers.cpp:215-232) advance with it, or without them the LWE rows do
static PbsArgs pbs_args_range(const PbsArgs& a, uint32_t start, uint32_t count) {
  PbsArgs r = a;
  r.num_samples = count;
  if (a.in_idx) r.in_idx = a.in_idx + start;
  else r.in = a.in + (uint64_t)start * (a.n + 1);
  if (a.out_idx) r.out_idx = a.out_idx + start;
  else r.out = a.out + (uint64_t)start * (a.k * a.N + 1);
  if (a.lut_idx) r.lut_idx = a.lut_idx + start;
  return r;
}

template <int L>
static int launch_pair(const PbsArgs& a) {
  if (a.num_samples == 0) return 0;
  // Ciphertexts per workgroup: a workgroup runs alone on its CU (LDS), so 4 per workgroup leaves
  // CUs idle below 4 x CUs ciphertexts.  The round time of a workgroup falls with fewer waves per
  // SIMD, but not in proportion: 2 per workgroup pays off while their workgroups fit one round
  // (<= 2 x CUs ciphertexts), 1 per workgroup at <= CUs.  CONCRETE_HIP_PBS_PAIRS=1/2/4 forces it.
  const char* fe = getenv("CONCRETE_HIP_PBS_PAIRS");  // read per call (tests switch it)
  const int forced = fe ? atoi(fe) : 0;
  const uint32_t cus = device_cus();
  const int P = forced == 1 || forced == 2 || forced == 4 ? forced
                : a.num_samples <= cus ? 1 : a.num_samples <= 2 * cus ? 2 : 4;
  // <= 1 ciphertext per CU at l = 3: four waves per ciphertext (pbs1024_quad.hip), +7 % at B = 256
  // (at 2 per CU, B = 512, it measured 0.9x the pair kernel: DESIGN.md §4.1).  CONCRETE_HIP_PBS_QUAD=0
  // keeps the pair kernel, =1 / =2 forces it with that many ciphertexts per workgroup (read per
  // call: tests, A/B).
  // Six waves per ciphertext (pbs1024_hex.hip, round 5), two ciphertexts per CU: a round of 2 x CUs
  // ciphertexts takes ~5.41 ms against ~10.2 ms for the pair kernel's round of 4 x CUs (cfg2, one
  // MI355X, profiles/r05/ab5_sweep.json), so it wins whenever it needs fewer than 1.886x the pair
  // kernel's rounds — every batch of <= 2 x CUs (the metric's 512 per GPU on 8 GPUs: 92k vs 70k
  // PBS/s), 1536, 2560 ... — and one ciphertext per workgroup at <= CUs (52.5k vs 40.6k at 256).
  // CONCRETE_HIP_PBS_HEX=1 / =2 forces it with that many ciphertexts per workgroup, =0 keeps it off;
  // a forced CONCRETE_HIP_PBS_PAIRS / _QUAD selects those kernels (read per call: tests, A/B).
  // Round 6: the call is split over the kernels by pbs1024_plan.hpp (whole pair rounds, six-wave
  // rounds, at most one round of one ciphertext per workgroup), each part a contiguous range of the
  // batch launched on the caller's stream.
  if (L == 3) {
    const char* he = getenv("CONCRETE_HIP_PBS_HEX");
    const int hx = he ? atoi(he) : -1;
    if (hx == 1 || hx == 2) return pbs1024_hex_launch(a, hx);
    if (hx != 0 && !fe && !getenv("CONCRETE_HIP_PBS_QUAD") && !getenv("CONCRETE_HIP_PBS_STAMPS")) {
      const Pbs1024Plan plan = plan_pbs1024(a.num_samples, cus);
      uint32_t start = 0;
      int rc = 0;
      if (plan.pair) {
        rc = launch_pair_p<4, L>(pbs_args_range(a, start, plan.pair));
        start += plan.pair;
      }
      if (rc == 0 && plan.hex2) {
        rc = pbs1024_hex_launch(pbs_args_range(a, start, plan.hex2), 2);
        start += plan.hex2;
      }
      if (rc == 0 && plan.hex1) rc = pbs1024_hex_launch(pbs_args_range(a, start, plan.hex1), 1);
      return rc;
    }
  }
  if (L == 3 && P <= 2 && !getenv("CONCRETE_HIP_PBS_STAMPS")) {
    const char* qe = getenv("CONCRETE_HIP_PBS_QUAD");
    const int q = qe ? atoi(qe) : -1;
    if (q == 1 || q == 2) return pbs1024_quad_launch(a, q);
    if (q != 0 && P == 1) return pbs1024_quad_launch(a, 1);
  }
  if (P == 1) return launch_pair_p<1, L>(a);
  if (P == 2) return launch_pair_p<2, L>(a);
  return launch_pair_p<4, L>(a);
}

int pbs_launch(const PbsArgs& a) {
  const KeyKind kind = key_format(a.k, a.N, a.level).kind;
  if (kind == KeyKind::GENERIC) return pbs_generic_launch(a);
  if (kind == KeyKind::N2048) return pbs2048_launch(a);
  if (kind == KeyKind::K2N1024) return pbs1024k2_launch(a);
  if (kind == KeyKind::SMALL) return pbs_small_launch(a);
  if (kind == KeyKind::N1024 && a.limbs == 3) {
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
