// pbs2048.hip — batched classic PBS for N = 2048, k = 1, l = 1 (BASELINE.json configs[3],
// "cfg4": n = 742, logB = 23) on CDNA4 (gfx950).
//
// Same semantics as pbs.hip (concrete-cpu c_api/bootstrap.rs:347-414 -> tfhe 0.10
// blind_rotate_assign + sample extract; restated in oracle/tfhe_oracle.c:ora_pbs), same exact
// arithmetic, re-planned for the larger ring:
//
// * Even/odd split.  With Z = X^2, a(X) = a_e(Z) + X a_o(Z) and
//       a * b mod (X^2048 + 1) = (a_e b_e + Z a_o b_o) + X (a_e b_o + a_o b_e),
//   where every product is negacyclic in Z modulo Z^1024 + 1: the N = 1024 product of pbs.hip
//   (512-point folded, twisted transform, fft512.hpp).  Multiplying by Z is pointwise
//   multiplication by the evaluation point alpha_k = exp(i pi (1 - 4k) / 1024) of frequency k.
// * Sub-digits on the limb grid.  The key polynomial g is split into 4 balanced 16-bit limbs,
//   g = sum_j 2^{16 j} g_j, and a 23-bit digit d exactly into d = d_lo + 2^16 d_hi with d_lo
//   balanced 16-bit (|d_lo| <= 2^15) and |d_hi| <= 2^(logB-17) + 1.  Then
//       d g = sum_m 2^{16 m} (d_lo g_m + d_hi g_{m-1})   (mod 2^64, slots m = 0..3)
//   so every slot is one exact integer convolution sum (certified error < 1/2,
//   oracle/pyoracle.py:gpu2048_error_bound) and each key limb serves two slots: limb j's key
//   window adds d_lo g_j to slot j and d_hi g_j to slot j + 1 (carried into the next limb).
//
// Mapping: four waves per ciphertext; wave v = 2c + p owns the parity-p half of GLWE polynomial c
// (16 u64 per lane, lane t holds coefficient 2(t + 64m) + p), runs the forward transforms of its
// own sub-digit polynomials, keeps frequency slots k2 in {2v, 2v + 1} of all of them (the rest
// goes to its three partners through LDS), does the key MAC for all four outputs on its quarter
// of the frequencies, trades quarters back and runs the inverse transforms of its own output.
// PBS2_CTS ciphertexts per workgroup share a ring of 16 KB key groups filled by LDS-DMA.
//
// Products at the square roots (P2_PM, pbs.hpp).  With s_k^2 = alpha_k, the N = 2048 polynomial
// evaluated at +-s_k is A+-_k = A_e(alpha_k) +- s_k A_o(alpha_k) (its 1024-point negacyclic
// spectrum: the even/odd 512-point transforms plus one radix-2 stage), so
//     C+- = A+- B+-,   C_e = (C+ + C-) / 2,   C_o = (C+ - C-) / (2 s_k)
// — two complex multiplies per frequency and key value instead of the four of the even/odd form.
// The key holds K+- = B+- / 2 (bsk.hip); each wave forms A+- of its frequency quarter after the
// spectrum exchange, accumulates U+- = sum A+- K+- in the key windows, and a completed slot is
// unfolded to C_e = U+ + U-, C_o = (U+ - U-) conj(s_k) before it is mailed to its owners.
#include "common.hpp"
#include "fft512.hpp"
#include "kernel_util.hpp"
#include "pbs.hpp"

#include <type_traits>

namespace chip {

constexpr uint64_t P2_MAGIC_ALL =
    RND_MAGIC_BITS + (RND_MAGIC_BITS << 16) + (RND_MAGIC_BITS << 32) + (RND_MAGIC_BITS << 48);

// Synchronisation of the four waves of one ciphertext (the exchanges never involve the other
// ciphertext of the workgroup): each wave publishes how many sync points it has passed and
// waits until its three partners have reached the same count.  LDS traffic is drained, the
// key DMA is not.
__device__ __forceinline__ void quad_sync(uint32_t* flags, int ctl, int v, uint32_t& cnt, const SyncGuard& guard) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#if defined(D4_NOQS) && D4_NOQS
  return;
#endif
  ++cnt;
  __hip_atomic_store(&flags[ctl * 4 + v], cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
  for (int o = 1; o < 4; ++o) spin_until_ge(&flags[ctl * 4 + ((v + o) & 3)], cnt, guard);
}

// Diagnostic builds only (timing, wrong results): D4_NOBAR (no key-window barriers), D4_NOMAC
// (no key MAC FMAs), D4_NOINV (no inverse transforms), D4_NOFWD (no forward transforms),
// D4_NOQS (no quad syncs).
#ifndef D4_NOBAR
#define D4_NOBAR 0
#endif
#ifndef D4_NOMAC
#define D4_NOMAC 0
#endif
#ifndef D4_NOINV
#define D4_NOINV 0
#endif
#ifndef D4_NOFWD
#define D4_NOFWD 0
#endif
#ifndef D4_NOQS
#define D4_NOQS 0
#endif

#ifndef P2_DEFER_INV
#define P2_DEFER_INV 1  // limb li's inverse after limb li + 1's first key-window barrier, no quad sync (+1.0 %)
#endif
#ifndef P2_SPLIT_XSYNC
#define P2_SPLIT_XSYNC 1  // split second sync of the sub-0 exchange (+1.1 %)
#endif
// Split form of quad_sync: quad_signal publishes that this wave's reads of the partners'
// scratches have been issued (LDS operations of a wave execute in order, so the count is seen
// after them); quad_wait, before this wave next overwrites its scratch, waits for the partners.
__device__ __forceinline__ void quad_signal(uint32_t* flags, int ctl, int v, uint32_t& cnt) {
  asm volatile("" ::: "memory");
  ++cnt;
  __hip_atomic_store(&flags[ctl * 4 + v], cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void quad_wait(uint32_t* flags, int ctl, int v, uint32_t cnt, const SyncGuard& guard) {
#pragma unroll
  for (int o = 1; o < 4; ++o) spin_until_ge(&flags[ctl * 4 + ((v + o) & 3)], cnt, guard);
  asm volatile("" ::: "memory");
}

// The same counters for the two parity waves of one polynomial (v, v ^ 1) only.
__device__ __forceinline__ void pair_sync2048(uint32_t* flags, int ctl, int v, uint32_t& cnt, const SyncGuard& guard) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  ++cnt;
  __hip_atomic_store(&flags[ctl * 4 + v], cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  spin_until_ge(&flags[ctl * 4 + (v ^ 1)], cnt, guard);
}

// NQ = 1: one digit split into d_lo + 2^16 d_hi (logB <= 24); NQ = l = 2 .. 4: whole digits
// (l 2^(logB-1) <= 2^15), each level's products landing in the same slot (the key holds the levels,
// [n][limb][col][q][row][+-][512], one ring group per (column, level, row)).
template <bool RESID, int NQ>
__global__ void __launch_bounds__(PBS2_CTS * 256, 2)
pbs2048_quad_kernel(uint64_t* __restrict__ out, const uint64_t* __restrict__ out_idx,
                    const uint64_t* __restrict__ luts, const uint64_t* __restrict__ lut_idx,
                    const uint64_t* __restrict__ in, const uint64_t* __restrict__ in_idx,
                    const cplx* __restrict__ fbsk, uint32_t n, uint32_t base_log, uint32_t num_samples,
                    unsigned long long* __restrict__ resid_out, SyncGuard guard) {
  constexpr int N = 2048, LOG2_2N = 12, K1 = 2;
  constexpr int NW = 4 * PBS2_CTS;                          // waves per workgroup
  constexpr int GROUP = 2 * 512;                            // (limb, col, row): parity e and o spectra
  constexpr int NGRP = PBS2_LIMBS * K1 * K1 * NQ;           // ring groups per CMUX step
  constexpr int NF = NQ == 1 ? PBS2_SUBS : NQ;              // forward transforms per step
  using StT = std::conditional_t<(NQ > 1), uint64_t, uint32_t>;  // decomposition state (l logB bits)
  constexpr int PER_I = NGRP * GROUP;                       // complex values per Fourier GGSW
  constexpr int RS = PBS2_RING_SLOTS, DIST = PBS2_RING_DIST;
  constexpr int GLDS = GROUP / 64 / NW;                     // 1 KB LDS-DMA pieces per wave per group
  constexpr int XS = (int)PBS1024_XCH_SLOTS;
  static_assert(GROUP % (64 * NW) == 0 && DIST < RS, "ring geometry");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  cplx* tbl = reinterpret_cast<cplx*>(smem);  // FFT tables (fft512.hpp)
  cplx* xch_all = tbl + FFT512_TABLE_ENTRIES;  // NW x XS: transpose scratch and mailboxes
  cplx* ring = xch_all + NW * XS;         // RS x GROUP key ring
  uint32_t* qflags = reinterpret_cast<uint32_t*>(ring + RS * GROUP);  // NW sync counters

  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int ctl = w >> 2;            // ciphertext within the workgroup
  const int v = w & 3;               // virtual polynomial = frequency quarter
  const int c = v >> 1, par = v & 1;
  const uint32_t s = blockIdx.x * PBS2_CTS + ctl;
  const bool active = s < num_samples;
  cplx* xch = xch_all + w * XS;
  uint64_t* xch64 = reinterpret_cast<uint64_t*>(xch);
  const cplx* ctx = xch_all + ctl * 4 * XS;  // the four scratches of this ciphertext
  cplx* ctxw = xch_all + ctl * 4 * XS;

  // ---- key ring: group g = (step g / NGRP, r = g % NGRP) -> slot g % RS.  NGRP is a multiple
  // of RS, so within a step a group's slot (r % RS) and its offset from the step's key base are
  // compile-time constants: the refill is one wave-uniform base plus immediates.
  static_assert(NGRP % RS == 0, "ring slot of a group must not depend on the step");
  const cplx* key_w = fbsk + (uint64_t)w * GLDS * 64;  // this wave's pieces of every group
  cplx* ring_w = ring + w * GLDS * 64;
  const uint32_t lane_b = (uint32_t)lane * (uint32_t)sizeof(cplx);  // zero-extended lane offset
  auto issue_group = [&](const cplx* key_step, int r) __attribute__((always_inline)) {
    const char* src = reinterpret_cast<const char*>(key_step + r * GROUP);
    cplx* dst = ring_w + (r % RS) * GROUP;
#pragma unroll
    for (int j = 0; j < GLDS; ++j)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const cplx*>(src + j * 1024 + lane_b),
                                       (lds_ptr_t)(dst + j * 64), 16, 0, 0);
  };
  if (n > 0) {
#pragma unroll
    for (int g = 0; g < DIST; ++g) issue_group(key_w, g);
  }

  build_fft512_tables(tbl, threadIdx.x, NW * 64);
  if (lane == 0) qflags[w] = 0u;
  uint32_t qcnt = 0;
  __syncthreads();
  const Fft512Tables T = fft512_tables_at(tbl);

  const uint64_t* lwe = in + (active ? (in_idx ? in_idx[s] : s) : 0) * (uint64_t)(n + 1);
  const uint64_t* lut = luts + (active && lut_idx ? lut_idx[s] : 0ull) * (uint64_t)(K1 * N);

  // acc_c = LUT_c * X^{-ms(b)}; this wave holds coefficients 2(lane + 64 m) + par of polynomial c
  uint64_t A[16];
  {
    const uint32_t bt = active ? modswitch(lwe[n], LOG2_2N) : 0u;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const uint32_t src = (uint32_t)(2 * (lane + 64 * m) + par + bt) & (2 * N - 1);
      const uint64_t val = active ? lut[c * N + (src & (N - 1))] : 0ull;
      A[m] = src < N ? val : 0ull - val;
    }
  }

#if P2_PM
  // square roots s_k = exp(i pi (1 - 4k) / 2048) of the evaluation points of my two frequency slots
  cplx sroot[2];
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const int k = fft512_freq(lane, 2 * v + jj);
    const int num = (1 - 4 * k) & 4095;  // in units of pi / 2048
    double sn, cs;
    sincospi((double)num / 2048.0, &sn, &cs);
    sroot[jj] = {cs, sn};
  }
  // X[2 row][sub] / X[2 row + 1][sub] (parity e / o spectra of one row) -> A+ / A- in place
  auto to_pm = [&](cplx (&X)[4][NF][2], int sub) __attribute__((always_inline)) {
#pragma unroll
    for (int row = 0; row < 2; ++row)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const cplx so = cmul(X[2 * row + 1][sub][jj], sroot[jj]);
        const cplx xe = X[2 * row][sub][jj];
        X[2 * row][sub][jj] = cadd(xe, so);
        X[2 * row + 1][sub][jj] = csub(xe, so);
      }
  };
#else
  // evaluation points of my two frequency slots (multiplication by Z = X^2)
  cplx alpha[2];
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const int k = fft512_freq(lane, 2 * v + jj);
    const int num = (1 - 4 * k) & 2047;  // in units of pi / 1024
    double sn, cs;
    sincospi((double)num / 1024.0, &sn, &cs);
    alpha[jj] = {cs, sn};
  }
#endif

  const int nrep = 64 - NQ * (int)base_log;
  const int logB = (int)base_log;
  double max_resid = 0.0;

  uint64_t a_next = active ? lwe[0] : 0ull;
  for (uint32_t i = 0; i < n; ++i) {
    const cplx* key_step = key_w + (uint64_t)i * PER_I;
    const bool last_step = i + 1 >= n;
    const uint64_t ai = a_next;
    if (i + 1 < n) a_next = active ? lwe[i + 1] : 0ull;
    const uint32_t at = modswitch(ai, LOG2_2N);
    // tfhe skips a zero mask element (and at == 0 changes nothing): the step still runs, on
    // ct1 = X^0 acc - acc = 0, whose digits, spectra and products are exact zeros, so the
    // recombination adds exactly 0 (the limb constants cancel).  Running every step keeps the
    // compiler from hoisting undefined values of skipped-step arrays out of the loop.

    // ---- ct1 = X^{at} acc - acc: the source coefficient may sit in the other parity's wave --
    StT st[16];
    {
#pragma unroll
      for (int m = 0; m < 16; ++m) xch64[lane + 64 * m] = A[m];
    }
    // An even shift keeps every coefficient in its parity class: the sources are my own
    // scratch, no other wave is involved.  An odd one swaps the classes: the sources are my
    // parity partner's (v ^ 1) scratch — a pair sync before the reads and one after (before my
    // next transform overwrites my scratch, which my partner reads).  `at` is the same for all
    // four waves, so the four sync counters stay equal.
    const bool odd = (at & 1u) != 0u;
    if (odd) pair_sync2048(qflags, ctl, v, qcnt, guard);
    else wave_lds_fence();
    {
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const uint32_t sp = (uint32_t)(2 * (lane + 64 * m) + par - (int)at) & (2 * N - 1);
        const uint32_t sj = sp & (N - 1);
        const uint64_t* box = reinterpret_cast<const uint64_t*>(ctx + (c * 2 + (int)(sj & 1)) * XS);
        const uint64_t rv = box[sj >> 1];
        st[m] = (StT)decomp_init((sp < N ? rv : 0ull - rv) - A[m], nrep);
      }
    }
    if (odd) pair_sync2048(qflags, ctl, v, qcnt, guard);  // my partner has read my scratch

    // ---- digit polynomials (two sub-digits of one level, or NQ levels), forward transforms --
    // X[vv][f][jj]: spectrum of digit polynomial f (virtual poly vv = 2 row + parity) at
    // frequency slot 2v + jj
    cplx X[4][NF][2];
    int32_t dlo[16], dhi[16];
    if constexpr (NQ == 1) {
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const int32_t d = decomp_next_t(st[m], logB);
        const int32_t lo = ((d + (1 << (PBS2_SUB_BITS - 1))) & ((1 << PBS2_SUB_BITS) - 1)) - (1 << (PBS2_SUB_BITS - 1));
        dlo[m] = lo;
        dhi[m] = (d - lo) >> PBS2_SUB_BITS;  // exact: d - lo is a multiple of 2^16
      }
    }
#pragma unroll
    for (int sub = 0; sub < NF; ++sub) {
      {
        if constexpr (NQ > 1) {
#pragma unroll
          for (int m = 0; m < 16; ++m) dlo[m] = decomp_next_t(st[m], logB);  // level q = sub
        }
        cplx vv8[8];
#pragma unroll
        for (int m = 0; m < 8; ++m)
          vv8[m] = sub == 0 || NQ > 1 ? cplx{(double)dlo[m], (double)dlo[m + 8]} : cplx{(double)dhi[m], (double)dhi[m + 8]};
#if P2_SPLIT_XSYNC
        if (!D4_NOFWD) {
          cplx tw2[4], tw3[4];
          fwd_p2_tw(tw2, T, lane >> 3);
          fwd_p3_tw(tw3, T, lane);
          // the sub-0 exchange's "everyone has read my spectrum" wait, right before this
          // transform's first LDS write (the partners signalled right after their reads)
          fft512_fwd_tw(vv8, xch, lane, tw2, tw3, 0, [&]() __attribute__((always_inline)) {
            if (sub > 0) quad_wait(qflags, ctl, v, qcnt, guard);
          });
        }
#else
        if (!D4_NOFWD) fft512_fwd(vv8, xch, T, lane);
#endif
#pragma unroll
        for (int k2 = 0; k2 < 8; ++k2) xch[k2 * 64 + lane] = vv8[k2];
      }
      // The last sub-digit's spectra need no quad sync: the first key window's workgroup barrier
      // (which drains every wave's LDS writes) publishes them, and they are first used in the
      // second window (sub 1); they are read right after that barrier.
      if (sub + 1 < NF) {
        quad_sync(qflags, ctl, v, qcnt, guard);
#pragma unroll
        for (int vv = 0; vv < 4; ++vv)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) X[vv][sub][jj] = ctx[vv * XS + (2 * v + jj) * 64 + lane];
#if P2_PM
        to_pm(X, sub);
#endif
#pragma unroll
        for (int vv = 0; vv < 4; ++vv)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) pin(X[vv][sub][jj]);
      }
      // everyone has read my spectrum before my next transform writes the scratch; after the
      // last sub-digit the scratches are next written behind the key windows' barriers
#if P2_SPLIT_XSYNC
      if (sub + 1 < NF) quad_signal(qflags, ctl, v, qcnt);
#else
      if (sub + 1 < NF) quad_sync(qflags, ctl, v, qcnt, guard);
#endif
    }

    // ---- per limb: MAC for the four outputs on my quarter, trade quarters, inverse ---------
    // Slot li = sum over rows of d_lo * g_li + d_hi * g_{li-1}: Ya/Pa hold slot li (its d_hi part
    // from the previous limb's windows), Yb/Pb start slot li + 1 with d_hi * g_li.  Y[cc][par][jj]:
    // output (column cc, parity par) at my frequency slot 2v + jj; P: the odd x odd products, times
    // alpha when the slot is folded (after its windows: once for the d_hi part, once for d_lo).
    cplx Ya[2][2][2], Pa[2][2];
#pragma unroll
    for (int cc = 0; cc < 2; ++cc)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) Ya[cc][0][jj] = Ya[cc][1][jj] = Pa[cc][jj] = {0.0, 0.0};
    // inverse transform of output (c, par) for limb LJ from my mailbox, exact rounding into A
    auto inverse_limb = [&](auto LJc) __attribute__((always_inline)) {
      constexpr int lj = decltype(LJc)::value;
      cplx V[8];
#pragma unroll
      for (int vv = 0; vv < 4; ++vv)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) V[2 * vv + jj] = xch[(vv * 2 + jj) * 64 + lane];
      if (!D4_NOINV) {
        // stage twiddles ahead of the transpose, output twiddles after it (as pbs.hip): +0.8 %
        cplx gi2[4];
        inv_p2_stage_tw(gi2, T, lane & 7);
        fft512_inv_tw(V, xch, T, lane, gi2, 0);
      }
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const double tr = V[m].re + RND_MAGIC, ti = V[m].im + RND_MAGIC;
        if constexpr (RESID) {
          max_resid = fmax(max_resid, fabs(V[m].re - (tr - RND_MAGIC)));
          max_resid = fmax(max_resid, fabs(V[m].im - (ti - RND_MAGIC)));
        }
        if constexpr (lj == 0) {
          A[m] += (uint64_t)__double_as_longlong(tr) - P2_MAGIC_ALL;
          A[m + 8] += (uint64_t)__double_as_longlong(ti) - P2_MAGIC_ALL;
        } else {
          A[m] += (uint64_t)__double_as_longlong(tr) << (16 * lj);
          A[m + 8] += (uint64_t)__double_as_longlong(ti) << (16 * lj);
        }
      }
      // materialise A here (else the inverse tail sinks into the next limb's key windows)
#pragma unroll
      for (int m = 0; m < 16; ++m) pin(A[m]);
      if constexpr (RESID) pin(max_resid);
    };
    static_for<0, PBS2_LIMBS>([&](auto LI) __attribute__((always_inline)) {
      constexpr int li = decltype(LI)::value;
      constexpr bool HI = NQ == 1 && li + 1 < PBS2_LIMBS;  // d_hi * g_3 lands at 2^64: vanishes
      if constexpr (NQ > 1 && li > 0) {  // levels: no carry, every slot starts from zero
#pragma unroll
        for (int cc = 0; cc < 2; ++cc)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) Ya[cc][0][jj] = Ya[cc][1][jj] = Pa[cc][jj] = {0.0, 0.0};
      }
      cplx Yb[2][2][2], Pb[2][2];
#pragma unroll
      for (int cc = 0; cc < 2; ++cc)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) Yb[cc][0][jj] = Yb[cc][1][jj] = Pb[cc][jj] = {0.0, 0.0};
#if P2_PM
      // U+ += A+ K+, U- += A- K- of one row (Y[0] / Y[1] hold U+ / U-; P unused)
      auto mac = [&](cplx (&Y)[2][2], cplx (&P)[2], const cplx& xp, const cplx& xm, const cplx& kp, const cplx& km,
                     int jj) __attribute__((always_inline)) {
        (void)P;
        Y[0][jj].re = __builtin_fma(xp.re, kp.re, __builtin_fma(-xp.im, kp.im, Y[0][jj].re));
        Y[0][jj].im = __builtin_fma(xp.re, kp.im, __builtin_fma(xp.im, kp.re, Y[0][jj].im));
        Y[1][jj].re = __builtin_fma(xm.re, km.re, __builtin_fma(-xm.im, km.im, Y[1][jj].re));
        Y[1][jj].im = __builtin_fma(xm.re, km.im, __builtin_fma(xm.im, km.re, Y[1][jj].im));
      };
#else
      // (a_e b_e + Z a_o b_o) and (a_e b_o + a_o b_e) of one row into (Y, P)
      auto mac = [&](cplx (&Y)[2][2], cplx (&P)[2], const cplx& xe, const cplx& xo, const cplx& ge, const cplx& go,
                     int jj) __attribute__((always_inline)) {
        Y[0][jj].re = __builtin_fma(xe.re, ge.re, __builtin_fma(-xe.im, ge.im, Y[0][jj].re));
        Y[0][jj].im = __builtin_fma(xe.re, ge.im, __builtin_fma(xe.im, ge.re, Y[0][jj].im));
        P[jj].re = __builtin_fma(xo.re, go.re, __builtin_fma(-xo.im, go.im, P[jj].re));
        P[jj].im = __builtin_fma(xo.re, go.im, __builtin_fma(xo.im, go.re, P[jj].im));
        Y[1][jj].re = __builtin_fma(xe.re, go.re, __builtin_fma(-xe.im, go.im, Y[1][jj].re));
        Y[1][jj].im = __builtin_fma(xe.re, go.im, __builtin_fma(xe.im, go.re, Y[1][jj].im));
        Y[1][jj].re = __builtin_fma(xo.re, ge.re, __builtin_fma(-xo.im, ge.im, Y[1][jj].re));
        Y[1][jj].im = __builtin_fma(xo.re, ge.im, __builtin_fma(xo.im, ge.re, Y[1][jj].im));
      };
#endif
#pragma unroll
      for (int cc = 0; cc < K1; ++cc) {
#pragma unroll
        for (int rq = 0; rq < K1 * NQ; ++rq) {
          const int q = rq / K1, row = rq % K1;  // level (NQ > 1), row
          const int r = (li * K1 + cc) * K1 * NQ + rq;  // group within the step
          // group r landed for this wave's pieces (the next DIST - 1 may stay in flight) ...
          if (r + DIST - 1 < NGRP || !last_step) wait_vmcnt<GLDS * (DIST - 1)>();
          else if (r + 1 == NGRP) wait_vmcnt<0>();
          else if (r + 2 == NGRP) wait_vmcnt<GLDS>();
          else wait_vmcnt<GLDS * 2>();
          if (!D4_NOBAR) pair_barrier();  // ... for every wave; everyone is done with group r - 1
          // refill the slot of group r - 1 with group r + DIST (RS = DIST + 1)
          if (r + DIST < NGRP) issue_group(key_step, r + DIST);
          else if (!last_step) issue_group(key_step + PER_I, r + DIST - NGRP);
          if constexpr (P2_DEFER_INV && li > 0) {
            if (cc == 0 && rq == 0) inverse_limb(std::integral_constant<int, li - 1>{});
          }
          if constexpr (li == 0) {
            if (cc == 0 && rq == 0) {  // the last digit polynomial's spectra (see above)
#pragma unroll
              for (int vv = 0; vv < 4; ++vv)
#pragma unroll
                for (int jj = 0; jj < 2; ++jj)
                  X[vv][NF - 1][jj] = ctx[vv * XS + (2 * v + jj) * 64 + lane];
#if P2_PM
              to_pm(X, NF - 1);
#endif
            }
          }
          {
            const cplx* G = ring + (r % RS) * GROUP + (2 * v) * 64 + lane;
            cplx ge[2], go[2];
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) ge[jj] = G[jj * 64], go[jj] = G[512 + jj * 64];
            // all four reads in flight before the first FMA (left to itself the scheduler issues
            // them one at a time, each behind its own LDS round trip): +1.1 %, 255 VGPRs
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int jj = 0; jj < (D4_NOMAC ? 0 : 2); ++jj) mac(Ya[cc], Pa[cc], X[2 * row][q][jj], X[2 * row + 1][q][jj], ge[jj], go[jj], jj);
            if constexpr (HI) {
#pragma unroll
              for (int jj = 0; jj < (D4_NOMAC ? 0 : 2); ++jj)
                mac(Yb[cc], Pb[cc], X[2 * row][1][jj], X[2 * row + 1][1][jj], ge[jj], go[jj], jj);
            }
            // this window's products are done here, not sunk past the next window's barrier
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) {
              pin(Ya[cc][0][jj]), pin(Ya[cc][1][jj]), pin(Pa[cc][jj]);
              if constexpr (HI) pin(Yb[cc][0][jj]), pin(Yb[cc][1][jj]), pin(Pb[cc][jj]);
            }
          }
        }
        // column cc of slot li is complete: fold Z a_o b_o in and send my quarter of outputs
        // vo = 2 cc + par straight into wave vo's mailbox, slot pair (v, jj).  Every scratch has been
        // idle since this limb's first key-window barrier (the last sub-digit's spectra were read
        // before the second), and nobody writes it again before the next limb's windows.
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
#if P2_PM
          // C_e = U+ + U-, C_o = (U+ - U-) conj(s)
          const cplx ce = cadd(Ya[cc][0][jj], Ya[cc][1][jj]);
          const cplx co = cmulc(csub(Ya[cc][0][jj], Ya[cc][1][jj]), sroot[jj]);
          ctxw[(2 * cc) * XS + (v * 2 + jj) * 64 + lane] = ce;
          ctxw[(2 * cc + 1) * XS + (v * 2 + jj) * 64 + lane] = co;
#else
          Ya[cc][0][jj] = cadd(Ya[cc][0][jj], cmul(Pa[cc][jj], alpha[jj]));
          ctxw[(2 * cc) * XS + (v * 2 + jj) * 64 + lane] = Ya[cc][0][jj];
          ctxw[(2 * cc + 1) * XS + (v * 2 + jj) * 64 + lane] = Ya[cc][1][jj];
#endif
        }
      }
      // slot li + 1 so far (d_hi * g_li): fold its odd products now, so that only the Y values are
      // carried across the inverse; the next limb's d_lo products restart P from zero
      if constexpr (HI) {
#pragma unroll
        for (int cc = 0; cc < 2; ++cc)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
#if P2_PM
            Ya[cc][0][jj] = Yb[cc][0][jj];
#else
            Ya[cc][0][jj] = cadd(Yb[cc][0][jj], cmul(Pb[cc][jj], alpha[jj]));
#endif
            Ya[cc][1][jj] = Yb[cc][1][jj];
            Pa[cc][jj] = {0.0, 0.0};
            pin(Ya[cc][0][jj]), pin(Ya[cc][1][jj]);
          }
      }
      // limb li's outputs are in the mailboxes: its inverse runs here for the last limb, and for the
      // others after the next limb's first key-window barrier (P2_DEFER_INV), which publishes the
      // mailboxes as this quad sync does
      if constexpr (!P2_DEFER_INV || li + 1 == PBS2_LIMBS) {
        quad_sync(qflags, ctl, v, qcnt, guard);
        inverse_limb(LI);
      }
    });
  }

  // ---- sample extract (nth = 0): out[j] = -A_0[N - j] (j > 0), A_0[0]; body B[0] ---------
  uint64_t* o = out + (active ? (out_idx ? out_idx[s] : s) : 0) * (uint64_t)(N + 1);
  if (!active) {
  } else if (c == 0) {
    // N - j has the parity of j: each half reverses its own coefficients
#pragma unroll
    for (int m = 0; m < 16; ++m) xch64[lane + 64 * m] = A[m];
    wave_lds_fence();
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int uj = lane + 64 * m;
      const int j = 2 * uj + par;
      const int u = par == 0 ? ((1024 - uj) & 1023) : 1023 - uj;
      const uint64_t val = xch64[u];
      o[j] = j == 0 ? val : 0ull - val;
    }
  } else if (par == 0 && lane == 0) {
    o[N] = A[0];
  }

  if constexpr (RESID) {
    for (int off = 32; off > 0; off >>= 1) max_resid = fmax(max_resid, __shfl_xor(max_resid, off));
    if (lane == 0 && active && resid_out) atomicMax(resid_out, (unsigned long long)__double_as_longlong(max_resid));
  }
}

template <bool RESID, int NQ>
static int launch2048_t(const PbsArgs& a) {
  const size_t lds = pbs2048_lds_bytes();
  auto kern = pbs2048_quad_kernel<RESID, NQ>;
  CHIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const uint32_t blocks = (a.num_samples + PBS2_CTS - 1) / PBS2_CTS;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(PBS2_CTS * 256), lds, a.stream, a.out, a.out_idx, a.luts, a.lut_idx,
                     a.in, a.in_idx, reinterpret_cast<const cplx*>(a.fbsk), a.n, a.base_log, a.num_samples, a.resid,
                     a.guard);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("pbs launch failed: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

int pbs2048_launch(const PbsArgs& a) {
  if (!(a.N == 2048 && a.k == 1 && a.limbs == (uint32_t)PBS2_LIMBS && pbs2048_ok(a.level, a.base_log))) {
    set_error("unsupported PBS parameters: N=%u k=%u level=%u base_log=%u limbs=%u", a.N, a.k, a.level, a.base_log,
              a.limbs);
    return -2;
  }
  if (a.num_samples == 0) return 0;
  switch (a.level) {
    case 1: return a.resid ? launch2048_t<true, 1>(a) : launch2048_t<false, 1>(a);
    case 2: return a.resid ? launch2048_t<true, 2>(a) : launch2048_t<false, 2>(a);
    case 3: return a.resid ? launch2048_t<true, 3>(a) : launch2048_t<false, 3>(a);
    default: return a.resid ? launch2048_t<true, 4>(a) : launch2048_t<false, 4>(a);
  }
}

}  // namespace chip
