// pbs_small.hip — batched classic PBS for the optimizer's small rings: N = 512, k = 3 and
// N = 256, k = 5 / 6, l = 1 (v0_last_128's 1- to 3-bit rows: opt3 n = 722 logB = 18, opt1 n = 592
// logB = 15, the k = 6 rows at log norm2 1-4 with logB = 18) on CDNA4 (gfx950).
//
// Same semantics as pbs.hip (concrete-cpu c_api/bootstrap.rs:347-414 -> tfhe 0.10
// blind_rotate_assign + sample extract; oracle/tfhe_oracle.c:ora_pbs) and the exact arithmetic of
// pbs1024k2.hip: 4 balanced 16-bit key limbs, digits split on the limb grid (d = d_lo + 2^16 d_hi;
// logB <= 15 needs no split), slot m = sum over rows of d_lo g_m + d_hi g_{m-1}, certified error
// < 1/2 (oracle/pyoracle.py:gpu_small_error_bound; logB <= 24).
//
// P = 1024 / N polynomials share one register fft512 (fft512.hpp).  With z_{P j + p} = a_p[j] (the
// folded N-point polynomial p), the transform's built-in twist zeta_1024^{P j + p} is the N-ring
// twist zeta_2N^j times the constant zeta_1024^p, and
//     Z[k + q M] = sum_p w_P^{p q} tz_p(k) E_p[k],   tz_p(k) = zeta_1024^p w_512^{p k},  M = N / 2,
// where E_p is the M-point negacyclic spectrum of polynomial p: a P-point DFT over the slots
// k2, k2 + 8/P, ... of one lane separates them (unzip), and the inverse runs the same steps
// backwards (zip, one inverse fft512 for P output polynomials).  Unnormalised unzip and zip scale the
// products by P^2 M: the key is stored scaled by 1 / (512 P).
//
// Mapping: two waves per ciphertext, wave v owning polynomials [vP, vP + P) (N = 256: the second
// wave's last two (k = 5) or one (k = 6) are empty) — 16 u64 per lane, lane t holding coefficients
// t / P + (64 / P) m and that + N / 2 of its polynomial t mod P.  Each wave transforms its own
// polynomials' sub-digits, keeps half of the spectrum slots of every row, runs the key products
// for all outputs on them, mails the outputs to their owners and runs the inverse of its own.
// Four ciphertexts per workgroup (8 waves, 2 per SIMD) share a ring of key groups (one limb and
// one output column: the K1 row spectra) filled by LDS-DMA.
#include "common.hpp"
#include "fft512.hpp"
#include "kernel_util.hpp"
#include "pbs.hpp"

#include <type_traits>

// Diagnostic builds only (timing; wrong results): SMD_NOMAC / SMD_NOINV / SMD_NOFWD drop the key
// products / inverse transforms / forward transforms, SMD_NOZIP the unzip and zip.
#ifndef SMD_NOMAC
#define SMD_NOMAC 0
#endif
#ifndef SMD_NOINV
#define SMD_NOINV 0
#endif
#ifndef SMD_NOFWD
#define SMD_NOFWD 0
#endif
#ifndef SMD_NOZIP
#define SMD_NOZIP 0
#endif

namespace chip {

namespace {

constexpr uint64_t SM_MAGIC_ALL =
    RND_MAGIC_BITS + (RND_MAGIC_BITS << 16) + (RND_MAGIC_BITS << 32) + (RND_MAGIC_BITS << 48);

// the two waves of one ciphertext (counters f[ct * 2 + v])
__device__ __forceinline__ void sm_sync(uint32_t* f, int ct, int v, uint32_t& cnt, const SyncGuard& guard) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  ++cnt;
  __hip_atomic_store(&f[ct * 2 + v], cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  spin_until_ge(&f[ct * 2 + (v ^ 1)], cnt, guard);
}
__device__ __forceinline__ void sm_signal(uint32_t* f, int ct, int v, uint32_t& cnt) {
  asm volatile("" ::: "memory");
  ++cnt;
  __hip_atomic_store(&f[ct * 2 + v], cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void sm_wait(uint32_t* f, int ct, int v, uint32_t cnt, const SyncGuard& guard) {
  spin_until_ge(&f[ct * 2 + (v ^ 1)], cnt, guard);
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ cplx mul_i(cplx a) { return {-a.im, a.re}; }
__device__ __forceinline__ cplx mul_mi(cplx a) { return {a.im, -a.re}; }

// P-point DFTs over the slots of one lane: unzip F_p = sum_q w_P^{-pq} Y_q, zip Y_q = sum_p w_P^{pq} F_p
// (w_P = exp(-2 pi i / P), unnormalised)
template <int P>
__device__ __forceinline__ void dftp(cplx (&x)[P], bool inverse) {
  if constexpr (P == 2) {
    const cplx a = x[0], b = x[1];
    x[0] = cadd(a, b);
    x[1] = csub(a, b);
  } else {
    static_assert(P == 4, "P = 2 or 4");
    const cplx s02 = cadd(x[0], x[2]), d02 = csub(x[0], x[2]);
    const cplx s13 = cadd(x[1], x[3]), d13 = csub(x[1], x[3]);
    const cplx r = inverse ? mul_i(d13) : mul_mi(d13);  // i^{pq} (unzip) or (-i)^{pq} (zip) at p q = 1
    x[0] = cadd(s02, s13);
    x[2] = csub(s02, s13);
    x[1] = cadd(d02, r);
    x[3] = csub(d02, r);
  }
}

}  // namespace

// SUBS = 2, NQ = 1: one digit split into d_lo + 2^16 d_hi (16 < logB <= 24); SUBS = 1: NQ = l whole
// digits (l = 2, 3 with l 2^(logB-1) <= 2^15), each level's products landing in the same slot (the
// key holds the levels, [n][limb][cg][q][c2][row][M], one ring group per level).
template <int N, int K1, int SUBS, int NQ, bool RESID>
__global__ void __launch_bounds__(SM_CTS * 128, 1)
pbs_small_kernel(uint64_t* __restrict__ out, const uint64_t* __restrict__ out_idx,
                 const uint64_t* __restrict__ luts, const uint64_t* __restrict__ lut_idx,
                 const uint64_t* __restrict__ in, const uint64_t* __restrict__ in_idx,
                 const cplx* __restrict__ fbsk, uint32_t n, uint32_t base_log, uint32_t num_samples,
                 unsigned long long* __restrict__ resid_out, SyncGuard guard) {
  constexpr int P = 1024 / N;               // polynomials per wave
  constexpr int M = N / 2;                  // spectrum points per polynomial
  constexpr int SL = 8 / P;                 // spectrum slots per polynomial
  constexpr int W = 2;                      // waves per ciphertext
  static_assert((K1 + P - 1) / P == W, "two waves per ciphertext");
  constexpr int MS = SL / W;                // key-product slots per wave
  constexpr int NW = W * SM_CTS;
  constexpr int LOG2_2N = N == 512 ? 10 : 9;
  constexpr int GC = sm_gc(N, K1);          // output columns per key group
  constexpr int GROUP = GC * K1 * M;        // (limb, GC columns): their K1 row spectra each
  constexpr int NCG = K1 / GC;              // column groups per limb
  static_assert(K1 % GC == 0, "column groups");
  constexpr int NGRP = SM_LIMBS * NCG * NQ;
  constexpr int NF = SUBS * NQ;             // forward transforms per step (sub-digits or levels)
  static_assert(SUBS == 1 || NQ == 1, "sub-digits or levels");
  using StT = std::conditional_t<(NQ > 1), uint64_t, uint32_t>;  // decomposition state (l logB bits)
  constexpr int PER_I = NGRP * GROUP;
  constexpr int RS = sm_rs(N, K1), DIST = RS - 1;
  constexpr int PB = (GROUP * 16) % (NW * 1024) == 0 ? 16 : 4;  // LDS-DMA bytes per lane
  constexpr int GLDS = GROUP * 16 / (64 * PB) / NW;              // DMA instructions per wave per group
  constexpr int XS = (int)PBS1024_XCH_SLOTS;
  static_assert(GROUP * 16 % (64 * PB * NW) == 0 && NGRP % RS == 0, "ring geometry");
  static_assert(XCH_SLOTS <= XS && P * N * 8 <= XS * 16, "scratch");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  cplx* tbl = reinterpret_cast<cplx*>(smem);
  cplx* xch_all = tbl + FFT512_TABLE_ENTRIES;
  cplx* ring = xch_all + NW * XS;
  uint32_t* sflags = reinterpret_cast<uint32_t*>(ring + RS * GROUP);

  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int ctl = w >> 1, v = w & 1;
  const int pl = lane & (P - 1);            // my lane's polynomial (local)
  const int pa = v * P + pl;                // ... absolute (>= K1: an empty slot of the last wave)
  const int jb = lane / P;                  // coefficient index base: j(m) = jb + (64 / P) m
  const int sv = v * MS;                    // my first key-product slot
  const uint32_t s = blockIdx.x * SM_CTS + ctl;
  const bool active = s < num_samples;
  cplx* xch = xch_all + w * XS;
  uint64_t* xch64 = reinterpret_cast<uint64_t*>(xch);
  cplx* ctx = xch_all + ctl * W * XS;       // the two scratches of this ciphertext

  const cplx* key_w = fbsk + (uint64_t)w * GLDS * (64 * PB / 16);
  cplx* ring_w = ring + w * GLDS * (64 * PB / 16);
  const uint32_t lane_b = (uint32_t)lane * (uint32_t)PB;
  auto issue_group = [&](const cplx* key_step, int r) __attribute__((always_inline)) {
    const char* src = reinterpret_cast<const char*>(key_step + r * GROUP);
    cplx* dst = ring_w + (r % RS) * GROUP;
#pragma unroll
    for (int j = 0; j < GLDS; ++j) {
      const void* gp = src + j * 64 * PB + lane_b;
      lds_ptr_t lp = (lds_ptr_t)(reinterpret_cast<char*>(dst) + j * 64 * PB);
      if constexpr (PB == 16) __builtin_amdgcn_global_load_lds(gp, lp, 16, 0, 0);
      else __builtin_amdgcn_global_load_lds(gp, lp, 4, 0, 0);
    }
  };
  if (n > 0) {
#pragma unroll
    for (int g = 0; g < DIST; ++g) issue_group(key_w, g);
  }

  build_fft512_tables(tbl, threadIdx.x, NW * 64);
  if (lane == 0) sflags[w] = 0u;
  uint32_t scnt = 0;
  __syncthreads();
  const Fft512Tables T = fft512_tables_at(tbl);

  // tz[p][sl] = zeta_1024^p w_512^{p k}, k = fft512_freq(lane, sl) (p >= 1)
  cplx tz[P][SL];
#pragma unroll
  for (int p = 1; p < P; ++p)
#pragma unroll
    for (int sl = 0; sl < SL; ++sl) {
      const int k = fft512_freq(lane, sl);
      const int num = (p * (1 - 4 * k)) & 2047;  // units of pi / 1024
      double sn, cs;
      sincospi((double)num / 1024.0, &sn, &cs);
      tz[p][sl] = {cs, sn};
    }

  const uint64_t* lwe = in + (active ? (in_idx ? in_idx[s] : s) : 0) * (uint64_t)(n + 1);
  const uint64_t* lut = luts + (active && lut_idx ? lut_idx[s] : 0ull) * (uint64_t)(K1 * N);
  const bool real = pa < K1;

  // acc_pa = LUT_pa * X^{-ms(b)}: A[m] coefficient j(m), A[m + 8] coefficient j(m) + N / 2
  uint64_t A[16];
  {
    const uint32_t bt = active ? modswitch(lwe[n], LOG2_2N) : 0u;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int c = jb + (64 / P) * (m & 7) + (m >= 8 ? M : 0);
      const uint32_t src = (uint32_t)(c + bt) & (2 * N - 1);
      const uint64_t val = active && real ? lut[pa * N + (src & (N - 1))] : 0ull;
      A[m] = src < N ? val : 0ull - val;
    }
  }

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

    // ---- ct1 = X^{at} acc - acc in my own scratch (P polynomials of N u64) ---------------
    StT st[16];
    {
#pragma unroll
      for (int m = 0; m < 16; ++m) xch64[pl * N + jb + (64 / P) * (m & 7) + (m >= 8 ? M : 0)] = A[m];
      wave_lds_fence();
      uint64_t rv[16];
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const int c = jb + (64 / P) * (m & 7) + (m >= 8 ? M : 0);
        rv[m] = xch64[pl * N + ((uint32_t)(c - (int)at) & (N - 1))];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const int c = jb + (64 / P) * (m & 7) + (m >= 8 ? M : 0);
        const uint32_t sp = (uint32_t)(c - (int)at) & (2 * N - 1);
        st[m] = (StT)decomp_init((sp < N ? rv[m] : 0ull - rv[m]) - A[m], nrep);
      }
      wave_lds_fence();
    }

    // ---- digits and forward transforms; X[row][f][js]: row's spectrum of digit polynomial f
    //      (sub-digit or level) at slot sv + js
    cplx X[K1][NF][MS];
    int32_t dd[SUBS][16];  // SUBS = 2: both sub-digits; else the current level's digits
    if constexpr (SUBS == 2) {
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const int32_t d = decomp_next_t(st[m], logB);
        const int32_t lo = ((d + (1 << (SM_SUB_BITS - 1))) & ((1 << SM_SUB_BITS) - 1)) - (1 << (SM_SUB_BITS - 1));
        dd[0][m] = lo;
        dd[1][m] = (d - lo) >> SM_SUB_BITS;
      }
    }
#pragma unroll
    for (int sub = 0; sub < NF; ++sub) {
      {
        if constexpr (SUBS == 1) {
#pragma unroll
          for (int m = 0; m < 16; ++m) dd[0][m] = decomp_next_t(st[m], logB);  // level q = sub
        }
        cplx vv[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) vv[m] = {(double)dd[SUBS == 2 ? sub : 0][m], (double)dd[SUBS == 2 ? sub : 0][m + 8]};
        cplx tw2[4], tw3[4];
        fwd_p2_tw(tw2, T, lane >> 3);
        fwd_p3_tw(tw3, T, lane);
        if (!SMD_NOFWD)
          fft512_fwd_tw(vv, xch, lane, tw2, tw3, 0, [&]() __attribute__((always_inline)) {
            if (sub > 0) sm_wait(sflags, ctl, v, scnt, guard);
          });
        // unzip: E_p = conj(tz_p) sum_q w_P^{-pq} Z[slot sl + q SL]
#pragma unroll
        for (int sl = 0; sl < SL; ++sl) {
          cplx y[P];
#pragma unroll
          for (int q = 0; q < P; ++q) y[q] = vv[sl + q * SL];
          if (!SMD_NOZIP) dftp<P>(y, true);
#pragma unroll
          for (int p = 0; p < P; ++p)
            xch[(p * SL + sl) * 64 + lane] = p == 0 || SMD_NOZIP ? y[p] : cmulc(y[p], tz[p][sl]);
        }
      }
      // the last digit polynomial's spectra are published by the first key window's barrier
      if (sub + 1 < NF) {
        sm_sync(sflags, ctl, v, scnt, guard);
#pragma unroll
        for (int row = 0; row < K1; ++row)
#pragma unroll
          for (int js = 0; js < MS; ++js)
            X[row][sub][js] = ctx[(row / P) * XS + ((row % P) * SL + sv + js) * 64 + lane];
#pragma unroll
        for (int row = 0; row < K1; ++row)
#pragma unroll
          for (int js = 0; js < MS; ++js) pin(X[row][sub][js]);
        sm_signal(sflags, ctl, v, scnt);
      }
    }

    // ---- per limb: key products for all outputs on my slots, mail, zip + inverse ---------
    cplx Yc[K1][MS];
#pragma unroll
    for (int cc = 0; cc < K1; ++cc)
#pragma unroll
      for (int js = 0; js < MS; ++js) Yc[cc][js] = {0.0, 0.0};
    static_for<0, SM_LIMBS>([&](auto LI) __attribute__((always_inline)) {
      constexpr int li = decltype(LI)::value;
      if constexpr (NQ == 1) {
        constexpr bool HI = SUBS == 2 && li + 1 < SM_LIMBS;
        cplx Yn[K1][MS];
#pragma unroll
        for (int cc = 0; cc < K1; ++cc)
#pragma unroll
          for (int js = 0; js < MS; ++js) Yn[cc][js] = {0.0, 0.0};
#pragma unroll
        for (int cg = 0; cg < NCG; ++cg) {
          const int r = li * NCG + cg;
          static_assert(DIST <= 3, "vmcnt tail cases");
          if (r + DIST - 1 < NGRP || !last_step) wait_vmcnt<GLDS * (DIST - 1)>();
          else if (r + 1 == NGRP) wait_vmcnt<0>();
          else if (r + 2 == NGRP) wait_vmcnt<GLDS>();
          else wait_vmcnt<GLDS * 2>();
          pair_barrier();
          if (r + DIST < NGRP) issue_group(key_step, r + DIST);
          else if (!last_step) issue_group(key_step + PER_I, r + DIST - NGRP);
          if constexpr (li == 0) {
            if (cg == 0) {
#pragma unroll
              for (int row = 0; row < K1; ++row)
#pragma unroll
                for (int js = 0; js < MS; ++js)
                  X[row][SUBS - 1][js] = ctx[(row / P) * XS + ((row % P) * SL + sv + js) * 64 + lane];
            }
          }
#pragma unroll
        for (int c2 = 0; c2 < GC; ++c2) {
          const int cc = cg * GC + c2;
          cplx Ya[MS];
#pragma unroll
          for (int js = 0; js < MS; ++js) Ya[js] = Yc[cc][js];
          const cplx* G = ring + (r % RS) * GROUP + c2 * K1 * M + sv * 64 + lane;
#pragma unroll
          for (int row = 0; row < K1; ++row) {
            cplx g[MS];
#pragma unroll
            for (int js = 0; js < MS; ++js) g[js] = G[row * M + js * 64];
#pragma unroll
            for (int js = 0; js < (SMD_NOMAC ? 0 : MS); ++js) {
              const cplx x0 = X[row][0][js];
              Ya[js].re = __builtin_fma(x0.re, g[js].re, __builtin_fma(-x0.im, g[js].im, Ya[js].re));
              Ya[js].im = __builtin_fma(x0.re, g[js].im, __builtin_fma(x0.im, g[js].re, Ya[js].im));
              if constexpr (HI) {
                const cplx x1 = X[row][SUBS - 1][js];
                Yn[cc][js].re = __builtin_fma(x1.re, g[js].re, __builtin_fma(-x1.im, g[js].im, Yn[cc][js].re));
                Yn[cc][js].im = __builtin_fma(x1.re, g[js].im, __builtin_fma(x1.im, g[js].re, Yn[cc][js].im));
              }
            }
          }
          // column cc of slot li: my slots into its owner's mailbox (each wave only ever touches its
          // own slots of a partner's scratch; the owner reads it behind the limb's pair sync)
#pragma unroll
          for (int js = 0; js < MS; ++js) ctx[(cc / P) * XS + ((cc % P) * SL + sv + js) * 64 + lane] = Ya[js];
#pragma unroll
          for (int js = 0; js < MS; ++js) {
            pin(Ya[js]);
            if constexpr (HI) pin(Yn[cc][js]);
          }
        }
        }
        if constexpr (HI) {
#pragma unroll
          for (int cc = 0; cc < K1; ++cc)
#pragma unroll
            for (int js = 0; js < MS; ++js) Yc[cc][js] = Yn[cc][js];
        }
      } else {
        // levels: each column group's windows sum the NQ levels' groups, then mail
#pragma unroll
        for (int cg = 0; cg < NCG; ++cg) {
          cplx Ya[GC][MS];
#pragma unroll
          for (int c2 = 0; c2 < GC; ++c2)
#pragma unroll
            for (int js = 0; js < MS; ++js) Ya[c2][js] = {0.0, 0.0};
#pragma unroll
          for (int q = 0; q < NQ; ++q) {
            const int r = (li * NCG + cg) * NQ + q;
            if (r + DIST - 1 < NGRP || !last_step) wait_vmcnt<GLDS * (DIST - 1)>();
            else if (r + 1 == NGRP) wait_vmcnt<0>();
            else if (r + 2 == NGRP) wait_vmcnt<GLDS>();
            else wait_vmcnt<GLDS * 2>();
            pair_barrier();
            if (r + DIST < NGRP) issue_group(key_step, r + DIST);
            else if (!last_step) issue_group(key_step + PER_I, r + DIST - NGRP);
            if constexpr (li == 0) {
              if (cg == 0 && q == 0) {  // the last level's spectra (published by this barrier)
#pragma unroll
                for (int row = 0; row < K1; ++row)
#pragma unroll
                  for (int js = 0; js < MS; ++js)
                    X[row][NF - 1][js] = ctx[(row / P) * XS + ((row % P) * SL + sv + js) * 64 + lane];
              }
            }
#pragma unroll
            for (int c2 = 0; c2 < GC; ++c2) {
              const cplx* G = ring + (r % RS) * GROUP + c2 * K1 * M + sv * 64 + lane;
#pragma unroll
              for (int row = 0; row < K1; ++row) {
#pragma unroll
                for (int js = 0; js < MS; ++js) {
                  const cplx g = G[row * M + js * 64];
                  const cplx x = X[row][q][js];
                  Ya[c2][js].re = __builtin_fma(x.re, g.re, __builtin_fma(-x.im, g.im, Ya[c2][js].re));
                  Ya[c2][js].im = __builtin_fma(x.re, g.im, __builtin_fma(x.im, g.re, Ya[c2][js].im));
                }
              }
            }
#pragma unroll
            for (int c2 = 0; c2 < GC; ++c2)
#pragma unroll
              for (int js = 0; js < MS; ++js) pin(Ya[c2][js]);
          }
#pragma unroll
          for (int c2 = 0; c2 < GC; ++c2) {
            const int cc = cg * GC + c2;
#pragma unroll
            for (int js = 0; js < MS; ++js)
              ctx[(cc / P) * XS + ((cc % P) * SL + sv + js) * 64 + lane] = Ya[c2][js];
          }
        }
      }
      sm_sync(sflags, ctl, v, scnt, guard);
      cplx V[8];
#pragma unroll
      for (int sl = 0; sl < SL; ++sl) {
        cplx y[P];
#pragma unroll
        for (int p = 0; p < P; ++p) {
          // an empty polynomial slot of the last wave has no mailbox writer: zero
          const cplx e = v * P + p < K1 ? xch[(p * SL + sl) * 64 + lane] : cplx{0.0, 0.0};
          y[p] = p == 0 || SMD_NOZIP ? e : cmul(e, tz[p][sl]);
        }
        if (!SMD_NOZIP) dftp<P>(y, false);
#pragma unroll
        for (int q = 0; q < P; ++q) V[sl + q * SL] = y[q];
      }
      {
        cplx gi2[4];
        inv_p2_stage_tw(gi2, T, lane & 7);
        if (!SMD_NOINV) fft512_inv_tw(V, xch, T, lane, gi2, 0);
      }
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const double tr = V[m].re + RND_MAGIC, ti = V[m].im + RND_MAGIC;
        if constexpr (RESID) {
          max_resid = fmax(max_resid, fabs(V[m].re - (tr - RND_MAGIC)));
          max_resid = fmax(max_resid, fabs(V[m].im - (ti - RND_MAGIC)));
        }
        if constexpr (li == 0) {
          A[m] += (uint64_t)__double_as_longlong(tr) - SM_MAGIC_ALL;
          A[m + 8] += (uint64_t)__double_as_longlong(ti) - SM_MAGIC_ALL;
        } else {
          A[m] += (uint64_t)__double_as_longlong(tr) << (16 * li);
          A[m + 8] += (uint64_t)__double_as_longlong(ti) << (16 * li);
        }
      }
#pragma unroll
      for (int m = 0; m < 16; ++m) pin(A[m]);
      if constexpr (RESID) pin(max_resid);
    });
  }

  // ---- sample extract (nth = 0): mask segment c: out[c N + j] = -A_c[N - j] (j > 0), A_c[0];
  //      body out[k N] = A_k[0]
  uint64_t* o = out + (active ? (out_idx ? out_idx[s] : s) : 0) * (uint64_t)((K1 - 1) * N + 1);
  if (active) {
#pragma unroll
    for (int m = 0; m < 16; ++m) xch64[pl * N + jb + (64 / P) * (m & 7) + (m >= 8 ? M : 0)] = A[m];
    wave_lds_fence();
    if (pa < K1 - 1) {
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const int j = jb + (64 / P) * (m & 7) + (m >= 8 ? M : 0);
        const uint64_t val = xch64[pl * N + ((N - j) & (N - 1))];
        o[pa * N + j] = j == 0 ? val : 0ull - val;
      }
    } else if (pa == K1 - 1 && jb == 0) {
      o[(K1 - 1) * N] = A[0];
    }
  }

  if constexpr (RESID) {
    for (int off = 32; off > 0; off >>= 1) max_resid = fmax(max_resid, __shfl_xor(max_resid, off));
    if (lane == 0 && active && resid_out) atomicMax(resid_out, (unsigned long long)__double_as_longlong(max_resid));
  }
}

template <int N, int K1, int SUBS, int NQ, bool RESID>
static int launch_small_t(const PbsArgs& a) {
  const size_t lds = pbs_small_lds_bytes(N, K1);
  auto kern = pbs_small_kernel<N, K1, SUBS, NQ, RESID>;
  CHIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const uint32_t blocks = (a.num_samples + SM_CTS - 1) / SM_CTS;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(SM_CTS * 128), lds, a.stream, a.out, a.out_idx, a.luts, a.lut_idx, a.in,
                     a.in_idx, reinterpret_cast<const cplx*>(a.fbsk), a.n, a.base_log, a.num_samples, a.resid,
                     a.guard);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("pbs launch failed: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

template <int N, int K1, int SUBS, int NQ>
static int launch_small_r(const PbsArgs& a) {
  return a.resid ? launch_small_t<N, K1, SUBS, NQ, true>(a) : launch_small_t<N, K1, SUBS, NQ, false>(a);
}

template <int N, int K1>
static int launch_small_n(const PbsArgs& a) {
  if (a.level == 2) return launch_small_r<N, K1, 1, 2>(a);
  if (a.level == 3) return launch_small_r<N, K1, 1, 3>(a);
  // logB <= 15: |digit| <= 2^14 fits the 16-bit grid whole (one sub-digit)
  return a.base_log <= 15 ? launch_small_r<N, K1, 1, 1>(a) : launch_small_r<N, K1, 2, 1>(a);
}

int pbs_small_launch(const PbsArgs& a) {
  if (a.N == 512 && a.k == 4) return pbs512k4_launch(a);  // five polynomials: four waves (pbs512k4.hip)
  if (!(a.limbs == (uint32_t)SM_LIMBS && pbs_small_ok(a.k, a.N, a.level, a.base_log))) {
    set_error("unsupported PBS parameters: N=%u k=%u level=%u base_log=%u limbs=%u", a.N, a.k, a.level, a.base_log,
              a.limbs);
    return -2;
  }
  if (a.num_samples == 0) return 0;
  if (a.N == 512) return launch_small_n<512, 4>(a);
  return a.k == 5 ? launch_small_n<256, 6>(a) : launch_small_n<256, 7>(a);
}

}  // namespace chip
