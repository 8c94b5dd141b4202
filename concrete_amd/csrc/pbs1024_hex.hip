// pbs1024_hex.hip — the N = 1024, k = 1, l = 3 PBS (cfg2) with six waves per ciphertext.
//
// Same semantics, Fourier key, key layout and exact arithmetic as pbs1024_pair_kernel (pbs.hip;
// reference call site: tfhe-cuda-backend cuda_programmable_bootstrap_lwe_ciphertext_vector_64 as
// invoked by compiler lib/Runtime/wrappers.cpp:237-240 and lib/Runtime/GPUDFG.cpp:1214-1218,
// semantics concrete-cpu c_api/bootstrap.rs:347-414, restated in oracle/tfhe_oracle.c:ora_pbs).
//
// Why: at <= 2 ciphertexts per CU (the metric's whole-node batch of 4096 is 512 per GPU on 8 GPUs)
// the pair kernel runs one wave per SIMD, and a lone wave is latency-bound.  A
// ciphertext's CMUX step holds 6 forward transforms (2 polynomials x 3 levels) and 6 inverse
// transforms (2 output polynomials x 3 key limbs), so six waves take one of each — a balanced split
// with the register fft512 unchanged — and two ciphertexts per workgroup put three waves on every
// SIMD.  Wave u = 3 c + j of a ciphertext, per CMUX step:
//   * produce (two ciphertexts per workgroup): rotation X^a B - B of polynomial c and its balanced
//     decomposition at every level for the coefficient pairs (m, m + 8), m in the wave's third of
//     the register slots; level q's digits (packed int16 pairs) go to the scratch of wave (c, q).
//     The negated accumulators B_c live in LDS, shared by the three waves of c.  [barrier D]
//   * forward transform of the level-j digit polynomial, spectrum published in the wave's scratch
//     (all 8 frequency slots, fft512's natural order).  [barrier A]
//   * key products of output c, limb j: the two waves of role u (one per ciphertext) split the
//     slots — wave h computes [4h, 4h + 4) for BOTH ciphertexts over their six spectra (LDS) — so
//     each key value is read once per CU, straight from L2 into registers, six batches of four
//     16-byte values per step, the next step's first three issued in the inverse phase.  [barrier B]
//   * the other ciphertext's half mailed into its wave's scratch (pair counter), inverse transform
//     with the k2 ^ 4 relabeling for h = 1, exact rounding, and the limb's contribution added into
//     B_c with 64-bit LDS atomics (integer adds mod 2^64: exact in any order).  [barrier C]
// The key layout is the pair kernel's (bsk.hip: group (limb, co, ro) holds column co / row ro in
// slots 0..3 and column 1 - co / row 1 - ro in slots 4..7, so wave (c, j) reads slots 0..3 of groups
// (j, c, r) and slots 4..7 of groups (j, 1 - c, 1 - r)).  One ciphertext per workgroup (batches of
// <= CUs): every wave rotates and decomposes its own digits and computes all eight slots of its own
// ciphertext's product; the syncs are per-ciphertext LDS counters.
#include <type_traits>

#include "common.hpp"
#include "fft512.hpp"
#include "kernel_util.hpp"
#include "pbs.hpp"
#include "pbs_hex.hpp"

#ifndef HX_SHARED_DIGITS
#define HX_SHARED_DIGITS 1  // rotation + decomposition shared by the three waves of a polynomial (XM)
#endif
#ifndef HX_DIAG_NOKEY
#define HX_DIAG_NOKEY 0  // timing-only builds: no key loads (the key values are the spectra's)
#endif
#ifndef HX_DIAG_NOATOMIC
#define HX_DIAG_NOATOMIC 0
#endif

namespace chip {

namespace {

constexpr uint64_t HX_MAGIC_ALL = RND_MAGIC_BITS + (RND_MAGIC_BITS << 22) + (RND_MAGIC_BITS << 43);
constexpr int hx_limb_shift(int li) { return li * 21 + (li > 0 ? 1 : 0); }

__device__ __forceinline__ void hx_signal(uint32_t* ctr, uint32_t& cnt) {
  asm volatile("" ::: "memory");
  ++cnt;
  __hip_atomic_store(ctr, cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// wait until counters ctr[0 .. NC) all reach target: the NC reads are issued together per poll
template <int NC>
__device__ __forceinline__ void hx_wait(const uint32_t* ctr, uint32_t target, const SyncGuard& guard) {
  for (uint32_t it = 0;; ++it) {
    uint32_t lo = 0xffffffffu;
#pragma unroll
    for (int o = 0; o < NC; ++o) {
      const uint32_t x = __hip_atomic_load(ctr + o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      lo = x < lo ? x : lo;
    }
    if (lo >= target) break;
    if (it >= guard.spin_limit) {
      __hip_atomic_fetch_or(guard.status, DEV_STATUS_SYNC_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    __builtin_amdgcn_s_sleep(0);
  }
  asm volatile("" ::: "memory");
}

}  // namespace

template <int CTS, bool RESID, bool STAMPS = false>
__global__ void __launch_bounds__(CTS * 384, 1)
pbs1024_hex_kernel(uint64_t* __restrict__ out, const uint64_t* __restrict__ out_idx,
                   const uint64_t* __restrict__ luts, const uint64_t* __restrict__ lut_idx,
                   const uint64_t* __restrict__ in, const uint64_t* __restrict__ in_idx,
                   const cplx* __restrict__ fbsk, uint32_t n, uint32_t base_log, uint32_t num_samples,
                   unsigned long long* __restrict__ resid_out, SyncGuard guard) {
  constexpr int K = 1, K1 = 2, N = 1024, LOG2_2N = 11, LIMBS = 3, L = 3;
  constexpr int GROUP = L * 512;                      // one (limb, co, ro) group: the L level spectra
  constexpr int PER_I = K1 * K1 * LIMBS * GROUP;      // complex values per Fourier GGSW
  constexpr int XS = (int)PBS1024_XCH_SLOTS;
  constexpr int NW = 6 * CTS;
  static_assert(XCH_SLOTS <= XS, "transpose scratch");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  cplx* tbl = reinterpret_cast<cplx*>(smem);
  cplx* xch_all = tbl + FFT512_TABLE_ENTRIES;                               // NW scratches
  uint64_t* acc_all = reinterpret_cast<uint64_t*>(xch_all + NW * XS);       // CTS x 2 x N: B_c
  uint32_t* hf = reinterpret_cast<uint32_t*>(acc_all + CTS * K1 * N);       // 8 counters per ciphertext

  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int ctl = w / 6, u = w - 6 * ctl;
  const int c = u >= 3 ? 1 : 0, j = u - 3 * c;
  const uint32_t s = blockIdx.x * CTS + ctl;
  const bool active = s < num_samples;
  cplx* xch = xch_all + w * XS;
  uint64_t* accc = acc_all + (ctl * K1 + c) * N;
  uint32_t* myctr = hf + ctl * 8 + u;
  const uint32_t* ctctr = hf + ctl * 8;         // the ciphertext's six counters
  const uint32_t* polyctr = hf + ctl * 8 + 3 * c;

  const uint64_t* lwe = in + (active ? (in_idx ? in_idx[s] : s) : 0) * (uint64_t)(n + 1);
  const uint64_t* lut = luts + (active && lut_idx ? lut_idx[s] : 0ull) * (uint64_t)(K1 * N);

  build_fft512_tables(tbl, threadIdx.x, NW * 64);
  if (lane == 0) *myctr = 0u;
  // acc_c = LUT_c * X^{-ms(b)} (blind_rotate_assign: polynomial_wrapping_monic_monomial_div), stored
  // negated (pbs1024_pair_kernel): written by wave j = 0 of each polynomial
  if (j == 0) {
    const uint32_t bt = active ? modswitch(lwe[n], LOG2_2N) : 0u;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const uint32_t src = (uint32_t)(lane + 64 * m + bt) & (2 * N - 1);
      const uint64_t v = active ? lut[c * N + (src & (N - 1))] : 0ull;
      accc[lane + 64 * m] = src < N ? 0ull - v : v;
    }
  }
  uint32_t cnt = 0;
  __syncthreads();
  const Fft512Tables T = fft512_tables_at(tbl);

  const int nrep = 64 - L * (int)base_log;
  const int logB = (int)base_log;
  const int32_t neg_base = -(1 << logB);
  const uint32_t half_m1 = (1u << (logB - 1)) - 1u;
  const uint32_t khi = 1u << (nrep - 33);  // 2^(nrep-1) in the high word (nrep >= 37 under the gate)
  double max_resid = 0.0;
  // diagnostic stamps (STAMPS builds only): cycles per phase, summed over the steps
  uint64_t acc_t[NSTAMP] = {};
  uint64_t t_begin = 0, tp = 0;
  auto lap = [&](int k) __attribute__((always_inline)) {
    if constexpr (STAMPS) {
      const uint64_t t = stamp();
      acc_t[k] += t - tp;
      tp = t;
    }
  };
  if constexpr (STAMPS) t_begin = tp = stamp();

  // ---- this wave's key slice: output column c, limb j.  Slots 0..3 of row r: group (j, c, r);
  //      slots 4..7 of row r: group (j, 1 - c, 1 - r) (the pair layout's own/other halves).
  // (wave-uniform bases: the loads take the scalar-base + 32-bit lane-offset form)
  const cplx* key_lo = fbsk + (uint64_t)(((j * K1 + c) * K1) * GROUP);            // + r GROUP
  const cplx* key_hi = fbsk + (uint64_t)(((j * K1 + (1 - c)) * K1 + 1) * GROUP);  // - r GROUP
  // Two ciphertexts per workgroup (XM): the key products of output (c, j) are split by frequency
  // half between the two waves of role u — wave h = ctl computes slots [4h, 4h + 4) for BOTH
  // ciphertexts — so each key value crosses L2 -> CU once per workgroup; the halves of the other
  // ciphertext's product are then mailed to its wave (the pair kernel's k2 ^ 4 relabeling lets the
  // h = 1 wave keep its own half in v[0..3]).  One ciphertext: all eight slots in the wave.
  constexpr bool XM = CTS == 2;
  constexpr int KS = XM ? 4 : 8;       // key slots per batch
  constexpr int PF = XM ? 3 : 2;       // batches in flight
  constexpr int NB = K1 * L;           // batches (r, q) per step
  const int h = XM ? ctl : 0;
  const uint64_t hsign = (uint64_t)h << 63;
  // batch b = (r, q) = (b / L, b % L): key slots [4h, 4h + KS) of that row and level.  XM: one
  // wave-uniform base per row (no per-load select): h = 0 reads slots 0..3 of (j, c, r), h = 1 slots
  // 4..7 of (j, 1 - c, 1 - r)
  const cplx* krow0 = XM && h ? key_hi + 4 * 64 : key_lo;
  const cplx* krow1 = XM && h ? key_hi + 4 * 64 - GROUP : key_lo + GROUP;
  auto load_batch = [&](cplx (&g)[KS], uint64_t step_off, int b) __attribute__((always_inline)) {
    const int r = b / L, q = b % L;
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const cplx* kb;
      if (XM) kb = (r ? krow1 : krow0) + (step_off + q * 512 + k * 64);
      else kb = k < 4 ? key_lo + (step_off + r * GROUP + q * 512 + k * 64)
                      : key_hi + (step_off - r * GROUP + q * 512 + k * 64);
#if HX_DIAG_NOKEY
      g[k] = {(double)(k + 1), (double)(size_t)kb};
#else
      g[k] = kb[lane];
#endif
    }
  };
  cplx gb[PF][KS];
  if (n > 0) {
#pragma unroll
    for (int b = 0; b < PF; ++b) load_batch(gb[b], 0, b);
  }

  uint64_t a_next = active && n > 0 ? lwe[0] : 0ull;
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t step_off = (uint64_t)i * PER_I;
    const uint64_t next_off = i + 1 < n ? step_off + PER_I : step_off;  // past the last step: re-read (unused)
    const uint64_t ai = a_next;
    if (i + 1 < n) a_next = active ? lwe[i + 1] : 0ull;
    const uint32_t at = modswitch(ai, LOG2_2N);

    // ---- ct1 = acc X^at - acc = B - X^at B of polynomial c (pbs1024_pair_kernel's offsets: bit 13
    //      of o says "src < N", i.e. no wrap, where the rotated term is subtracted), decomposer state
    const uint32_t o0 = ((uint32_t)(lane - (int)at) << 3) + 8u * N;
    const char* accb = reinterpret_cast<const char*>(accc);
    auto state_of = [&](uint64_t rv, uint64_t bv, int m) __attribute__((always_inline)) {
      const uint32_t o = o0 + 512u * m;
      const uint32_t s32 = (uint32_t)((int32_t)(o << 18) >> 31);
      const uint64_t rvs = rv ^ (((uint64_t)s32 << 32) | s32);
      const uint64_t x = bv + rvs + (uint64_t)(s32 & 1u);
      return ((uint32_t)(x >> 32) + khi) >> (nrep - 32);
    };
    auto rot_read = [&](int m) __attribute__((always_inline)) {
      return *reinterpret_cast<const uint64_t*>(accb + ((o0 + 512u * m) & 8191u));
    };
    int32_t d[16];
    if constexpr (XM && HX_SHARED_DIGITS) {
      // Shared: wave (c, j) rotates and decomposes (every level) only the coefficient pairs
      // (m, m + 8) with m in [MB, ME) of its role — 3 / 3 / 2 of the 8 — and stores level q's digits
      // (two int16 per u32) in the scratch of wave (c, q); after barrier D each wave reads its level's
      // 16 digits from its own scratch.  (Every scratch is idle between the C and D barriers.)
      auto produce = [&](auto JC) __attribute__((always_inline)) {
        constexpr int JJ = decltype(JC)::value;
        constexpr int MB = JJ == 0 ? 0 : JJ == 1 ? 3 : 6, ME = JJ == 0 ? 3 : JJ == 1 ? 6 : 8, NM = ME - MB;
        uint64_t rv[2][NM], bv[2][NM];
#pragma unroll
        for (int t = 0; t < NM; ++t)
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            const int m = MB + t + 8 * hh;
            rv[hh][t] = rot_read(m);
            bv[hh][t] = accc[lane + 64 * m];
          }
        __builtin_amdgcn_sched_barrier(0);
        uint32_t* dst = reinterpret_cast<uint32_t*>(xch_all + (ctl * 6 + 3 * c) * XS) + lane;
#pragma unroll
        for (int t = 0; t < NM; ++t) {
          const int m = MB + t;
          uint32_t s0 = state_of(rv[0][t], bv[0][t], m), s1 = state_of(rv[1][t], bv[1][t], m + 8);
#pragma unroll
          for (int q = 0; q < L; ++q) {
            const int32_t d0 = decomp_level32(s0, (uint32_t)(q * logB), logB, half_m1, neg_base, q + 1 < L);
            const int32_t d1 = decomp_level32(s1, (uint32_t)(q * logB), logB, half_m1, neg_base, q + 1 < L);
            dst[q * XS * 4 + m * 64] = ((uint32_t)d0 & 0xffffu) | ((uint32_t)d1 << 16);
          }
        }
      };
      if (j == 0) produce(std::integral_constant<int, 0>{});
      else if (j == 1) produce(std::integral_constant<int, 1>{});
      else produce(std::integral_constant<int, 2>{});
      lap(0);  // rotation + shared digits
      pair_barrier();  // D
      const uint32_t* mine = reinterpret_cast<const uint32_t*>(xch) + lane;
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const uint32_t pk = mine[m * 64];
        d[m] = (int32_t)__builtin_amdgcn_sbfe(pk, 0u, 16u);
        d[m + 8] = (int32_t)pk >> 16;
      }
    } else {
      uint32_t st[16];
      {
        uint64_t rv[16], bv[16];
#pragma unroll
        for (int m = 0; m < 16; ++m) {
          rv[m] = rot_read(m);
          bv[m] = accc[lane + 64 * m];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < 16; ++m) st[m] = state_of(rv[m], bv[m], m);
      }
      lap(0);  // rotation + state
      // the levels up to mine (the lower ones only carry into it): one uniform branch around whole
      // loops (a branch per coefficient and level, or every level for every role, cost more)
      auto digits = [&](auto JC) __attribute__((always_inline)) {
        constexpr int JJ = decltype(JC)::value;
#pragma unroll
        for (int m = 0; m < 16; ++m) {
          int32_t dig = 0;
#pragma unroll
          for (int q = 0; q <= JJ; ++q)
            dig = decomp_level32(st[m], (uint32_t)(q * logB), logB, half_m1, neg_base, q < JJ);
          d[m] = dig;
        }
      };
      if (j == 0) digits(std::integral_constant<int, 0>{});
      else if (j == 1) digits(std::integral_constant<int, 1>{});
      else digits(std::integral_constant<int, 2>{});
    }
    // ---- forward transform of my level's digit polynomial, spectrum published in my scratch
    {
      cplx v[8];
#pragma unroll
      for (int m = 0; m < 8; ++m) v[m] = {(double)d[m], (double)d[m + 8]};
      fft512_fwd(v, xch, T, lane, 0ull);
      // my scratch was last read by my own transpose (wave order); B of the previous step released it
#pragma unroll
      for (int k2 = 0; k2 < 8; ++k2) xch[k2 * 64 + lane] = v[k2];
    }
    lap(1);  // digits + forward + publish
    // A: the spectra of the workgroup are published (XM reads both ciphertexts': a workgroup barrier)
    if constexpr (XM) {
      pair_barrier();
    } else {
      hx_signal(myctr, cnt);
      hx_wait<6>(ctctr, cnt, guard);
    }
    lap(2);  // wait A

    // ---- key product of output c, limb j: XM both ciphertexts at slots [4h, 4h + 4), else mine at
    //      all eight; the key PF batches ahead
    constexpr int NT = XM ? 2 : 1;
    cplx Y[NT][KS];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int r = b / L, q = b % L;
      cplx x[NT][KS];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        // t = 0: my ciphertext, t = 1 (XM): the other one
        const cplx* X = xch_all + ((t == 0 ? ctl : 1 - ctl) * 6 + r * L + q) * XS + (4 * h) * 64 + lane;
#pragma unroll
        for (int k = 0; k < KS; ++k) x[t][k] = X[k * 64];
      }
      cplx (&g)[KS] = gb[b % PF];
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int k = 0; k < KS; ++k) {
          const cplx xv = x[t][k], gv = g[k];
          if (b == 0) {  // fma(a, b, 0) == a * b: the same bits as accumulating from zero
            Y[t][k].re = __builtin_fma(xv.re, gv.re, -xv.im * gv.im);
            Y[t][k].im = __builtin_fma(xv.re, gv.im, xv.im * gv.re);
          } else {
            Y[t][k].re = __builtin_fma(xv.re, gv.re, __builtin_fma(-xv.im, gv.im, Y[t][k].re));
            Y[t][k].im = __builtin_fma(xv.re, gv.im, __builtin_fma(xv.im, gv.re, Y[t][k].im));
          }
        }
      if (!XM && b == NB - 1) hx_signal(myctr, cnt);  // B: every spectrum read of this wave is issued
      // refill: batch b + PF of this step (the next step's first PF batches are issued in the
      // inverse phase: issued here, all of a step's key loads crowded into this phase, where the
      // CU's vector-memory path — 288 KB per step — bounded it: +5.8 % without key loads, diagnostic)
      if (b + PF < NB) load_batch(g, step_off, b + PF);
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int k = 0; k < KS; ++k) pin(Y[t][k]);
    lap(3);  // key products

    // ---- inverse transform of (c, j): my scratch is rewritten only after every reader of the
    //      spectra is done (B)
    cplx v[8];
    if constexpr (XM) {
      pair_barrier();  // B
      // the other ciphertext's half straight into its wave's scratch, then signal it
      // (Y[0] is my ciphertext's, Y[1] the other's: compile-time indexes, registers only)
      cplx* partner = xch_all + ((1 - ctl) * 6 + u) * XS + lane;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        partner[k * 64] = Y[1][k];
        v[k] = Y[0][k];  // my half: natural slots 4h + k (k2 ^ 4 order for h = 1)
      }
      hx_signal(myctr, cnt);  // M
      hx_wait<1>(hf + (1 - ctl) * 8 + u, cnt, guard);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[4 + k] = xch[k * 64 + lane];  // the partner's: slots 4 (1 - h) + k
    } else {
      hx_wait<6>(ctctr, cnt, guard);  // B
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = Y[0][k];
    }
    lap(4);  // wait B (+ mailbox)
    // the next step's first key batches, in flight during the inverse and the next rotation and
    // forward transform
#pragma unroll
    for (int b = 0; b < PF; ++b) load_batch(gb[b], next_off, b);
    fft512_inv(v, xch, T, lane, hsign);
    {
      const int lsh = j == 0 ? 0 : j == 1 ? hx_limb_shift(1) : hx_limb_shift(2);
      const uint64_t lsub = j == 0 ? HX_MAGIC_ALL : 0ull;
      // limb j's exact integers, negated (B = -acc), shifted; limb 0 removes the constant of all limbs
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const double tr = RND_MAGIC - v[m].re, ti = RND_MAGIC - v[m].im;
        if constexpr (RESID) {
          max_resid = fmax(max_resid, fabs(v[m].re - (RND_MAGIC - tr)));
          max_resid = fmax(max_resid, fabs(v[m].im - (RND_MAGIC - ti)));
        }
        // (branch-free: wave-uniform shift and constant)
        const uint64_t cre = ((uint64_t)__double_as_longlong(tr) << lsh) - lsub;
        const uint64_t cim = ((uint64_t)__double_as_longlong(ti) << lsh) - lsub;
#if HX_DIAG_NOATOMIC  // timing-only builds: plain stores (wrong results)
        if (j == 0) accc[lane + 64 * m] = cre, accc[lane + 64 * (m + 8)] = cim;
#else
        __hip_atomic_fetch_add(&accc[lane + 64 * m], cre, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add(&accc[lane + 64 * (m + 8)], cim, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#endif
      }
    }
    lap(5);  // inverse + rounding + atomic adds
    // C: the limbs of polynomial c are in.  XM: a workgroup barrier (every wave runs the same phases
    // between the A and B barriers anyway; spinning waves would take VALU issue slots)
    if constexpr (XM) {
      pair_barrier();
    } else {
      hx_signal(myctr, cnt);
      hx_wait<3>(polyctr, cnt, guard);
    }
    lap(7);  // wait C
  }
  if constexpr (STAMPS) {
    acc_t[6] = stamp() - t_begin;
    if (lane == 0 && resid_out) {
      unsigned long long* dst = resid_out + ((uint64_t)blockIdx.x * NW + w) * NSTAMP;
      for (int q = 0; q < NSTAMP; ++q) dst[q] = acc_t[q];
    }
  }

  // ---- sample extract (nth = 0) of acc = -B: out[j'] = -acc_0[N - j'] (j' > 0), acc_0[0]; body acc_1[0].
  //      The three waves of polynomial 0 split the mask words (m = j mod 3); wave (1, 0) the body.
  //      (B_1 is final once polynomial 1's last C sync has passed: the waves of polynomial 1 only.)
  uint64_t* o = out + (active ? (out_idx ? out_idx[s] : s) : 0) * (uint64_t)(K * N + 1);
  if (active) {
    if (c == 0) {
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        if (m % 3 != j) continue;
        const int jj = lane + 64 * m;
        const uint64_t val = accc[(N - jj) & (N - 1)];
        o[jj] = jj == 0 ? 0ull - val : val;
      }
    } else if (j == 0 && lane == 0) {
      o[K * N] = 0ull - accc[0];
    }
  }

  if constexpr (RESID && !STAMPS) {
    for (int off = 32; off > 0; off >>= 1) max_resid = fmax(max_resid, __shfl_xor(max_resid, off));
    if (lane == 0 && active && resid_out) atomicMax(resid_out, (unsigned long long)__double_as_longlong(max_resid));
  }
}

template <int CTS, bool RESID, bool STAMPS = false>
static int launch_hex_t(const PbsArgs& a) {
  const size_t lds = pbs1024_hex_lds_bytes(CTS);
  auto kern = pbs1024_hex_kernel<CTS, RESID, STAMPS>;
  CHIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const uint32_t blocks = (a.num_samples + CTS - 1) / CTS;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(CTS * 384), lds, a.stream, a.out, a.out_idx, a.luts, a.lut_idx, a.in,
                     a.in_idx, reinterpret_cast<const cplx*>(a.fbsk), a.n, a.base_log, a.num_samples, a.resid,
                     a.guard);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("pbs launch failed: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

int pbs1024_hex_launch(const PbsArgs& a, int cts) {
  if (!(a.N == 1024 && a.k == 1 && a.level == 3 && a.limbs == 3 && pbs1024_exact(1, 3, a.base_log))) {
    set_error("unsupported PBS parameters for the six-wave kernel: N=%u k=%u level=%u base_log=%u", a.N, a.k,
              a.level, a.base_log);
    return -2;
  }
  if (a.num_samples == 0) return 0;
  // diagnostic: CONCRETE_HIP_PBS_STAMPS=1 runs the s_memtime-instrumented build (2 ciphertexts per
  // workgroup); `resid` must then hold 6 * 2 * ceil(num_samples / 2) * NSTAMP u64
  static const bool stamps = getenv("CONCRETE_HIP_PBS_STAMPS") && atoi(getenv("CONCRETE_HIP_PBS_STAMPS"));
  if (stamps) return launch_hex_t<2, true, true>(a);
  if (cts == 1) return a.resid ? launch_hex_t<1, true>(a) : launch_hex_t<1, false>(a);
  return a.resid ? launch_hex_t<2, true>(a) : launch_hex_t<2, false>(a);
}

}  // namespace chip
