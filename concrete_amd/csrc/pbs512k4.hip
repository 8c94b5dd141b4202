// pbs512k4.hip — batched classic PBS for N = 512, k = 4, l = 1 (v0_last_128's 1- to 3-bit rows at
// log norm2 3-9: br 1/23, n = 605-745, thirteen rows) on CDNA4 (gfx950).
//
// Same semantics as pbs.hip (concrete-cpu c_api/bootstrap.rs:347-414 -> tfhe 0.10
// blind_rotate_assign + sample extract; oracle/tfhe_oracle.c:ora_pbs) and pbs_small.hip's exact
// arithmetic and packing: 4 balanced 16-bit key limbs, the digit split on the limb grid
// (d = d_lo + 2^16 d_hi; logB <= 15 needs no split), two N = 512 polynomials in one register fft512
// (z_{2j + p} = a_p[j]; unzip / zip = a 2-point DFT per slot pair and one twiddle), key scaled 1/1024;
// certified error < 1/2 (oracle/pyoracle.py:gpu_small_error_bound with k = 4).
//
// Mapping: five polynomials make three packed transforms, so four waves per ciphertext: the
// owners (roles 0-2) hold polynomials 2v, 2v + 1 (role 2: polynomial 4 and an empty half), rotate
// them in their own scratch, transform their sub-digits and run the inverse of their pair; role 3
// holds no accumulator.  Each role keeps one of the four spectrum slots of every row and runs the key
// products for all five outputs on it, mailing each output column to its owner.  A workgroup of two
// ciphertexts is eight waves, two per SIMD (w % 4); the second ciphertext's roles are rotated by one
// so that the two transform-free waves land on different SIMDs (2 and 3).  (Three waves per
// ciphertext with a 2 / 1 / 1 slot split held twice the spectra and carries in the two-slot wave:
// 44-54 spilled VGPRs.)  The two ciphertexts share a ring of 20 KB key groups (one limb and one output
// column: five row spectra) filled by LDS-DMA.
#include "common.hpp"
#include "fft512.hpp"
#include "kernel_util.hpp"
#include "pbs.hpp"

#include <type_traits>

namespace chip {

namespace {

// sum over the key limbs of the rounding constant at each limb's shift (LB bits per limb)
constexpr uint64_t k4_magic_all(int limbs, int lb) {
  uint64_t m = 0;
  for (int li = 0; li < limbs; ++li) m += RND_MAGIC_BITS << (lb * li);
  return m;
}

// the four waves of one ciphertext (counters f[ct * 4 + role]): publish how many sync points this
// wave has passed; wait until the other three have reached a count.  LDS traffic is drained, the key
// DMA is not.
__device__ __forceinline__ void k4_signal(uint32_t* f, int ctl, int role, uint32_t& cnt) {
  asm volatile("" ::: "memory");
  ++cnt;
  __hip_atomic_store(&f[ctl * 4 + role], cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void k4_wait(uint32_t* f, int ctl, int role, uint32_t cnt, const SyncGuard& guard) {
#pragma unroll
  for (int o = 1; o < 4; ++o) spin_until_ge(&f[ctl * 4 + ((role + o) & 3)], cnt, guard);
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void k4_sync(uint32_t* f, int ctl, int role, uint32_t& cnt, const SyncGuard& guard) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  k4_signal(f, ctl, role, cnt);
  k4_wait(f, ctl, role, cnt, guard);
}

}  // namespace

// SUBS = 2, NQ = 1: one digit split into d_lo + 2^16 d_hi (16 < logB <= 24); SUBS = 1: NQ = l whole
// digits, each level's products landing in the same slot (the key holds the levels,
// [n][limb][col][q][row][M], one ring group per level): l = 1 at logB <= 15 and l = 2 on 13-bit limbs;
// from l = 3 pbs512k4_many_kernel runs one level at a time.
// LIMBS = 4 balanced 16-bit key limbs, or 5 of 13 bits (l = 2 at logB = 16: two whole 16-bit digits
// against 16-bit limbs would put the certified bound at 0.69; 13-bit limbs cut the key spectra 8x).
template <int SUBS, int NQ, int LIMBS, bool RESID>
__global__ void __launch_bounds__(K4_CTS * 256, 1)
pbs512k4_kernel(uint64_t* __restrict__ out, const uint64_t* __restrict__ out_idx,
                const uint64_t* __restrict__ luts, const uint64_t* __restrict__ lut_idx,
                const uint64_t* __restrict__ in, const uint64_t* __restrict__ in_idx,
                const cplx* __restrict__ fbsk, uint32_t n, uint32_t base_log, uint32_t num_samples,
                unsigned long long* __restrict__ resid_out, SyncGuard guard) {
  constexpr int N = 512, LOG2_2N = 10, K1 = 5;
  constexpr int M = N / 2;                  // spectrum points per polynomial
  constexpr int SL = 4;                     // spectrum slots per polynomial (two per transform)
  constexpr int NW = 4 * K4_CTS;            // waves per workgroup
  constexpr int GROUP = K1 * M;             // (limb, column): the five row spectra
  constexpr int LB = LIMBS == 4 ? 16 : 13;  // limb grid: limb li at 2^{LB li} (the last of 5: 12 bits)
  static_assert(LIMBS == 4 || (LIMBS == 5 && SUBS == 1), "sub-digits need the 16-bit grid");
  constexpr uint64_t MAGIC_ALL = k4_magic_all(LIMBS, LB);
  constexpr int NGRP = LIMBS * K1 * NQ;     // ring groups per CMUX step
  constexpr int NF = SUBS * NQ;             // forward transforms per step (sub-digits or levels)
  static_assert(SUBS == 1 || NQ == 1, "sub-digits or levels");
  using StT = std::conditional_t<(NQ > 1), uint64_t, uint32_t>;  // decomposition state (l logB bits)
  constexpr int PER_I = NGRP * GROUP;
  constexpr int RS = K4_RING_SLOTS, DIST = RS - 1;
  constexpr int GLDS = 4;                   // 1 KB LDS-DMA pieces per issuing wave per group
  constexpr int NISS = GROUP / 64 / GLDS;   // waves 0 .. NISS - 1 issue a group's pieces
  static_assert(GROUP / 64 == GLDS * NISS && NISS <= NW, "ring geometry");
  static_assert(NGRP % 2 == 0 && RS == 4 && DIST <= 3, "ring geometry");
  constexpr int XS = (int)PBS1024_XCH_SLOTS;
  static_assert(XCH_SLOTS <= XS && 2 * N * 8 <= XS * 16, "scratch");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  cplx* tbl = reinterpret_cast<cplx*>(smem);
  cplx* xch_all = tbl + FFT512_TABLE_ENTRIES;
  cplx* ring = xch_all + 3 * K4_CTS * XS;   // (role 3 has no scratch)
  uint32_t* tflags = reinterpret_cast<uint32_t*>(ring + RS * GROUP);  // NW sync counters

  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int ctl = w >> 2;
  const int role = ctl == 0 ? (w & 3) : ((w + 1) & 3);  // = my key-product slot
  const bool owner = role < 3;
  const int v = owner ? role : 0;           // owned pair (role 3: none)
  const int pl = lane & 1;                  // my lane's polynomial within the pair
  const int pa = 2 * v + pl;                // ... absolute (5: the empty half of role 2)
  const int jb = lane >> 1;                 // coefficient j(m) = jb + 32 m (+ M for m >= 8)
  const uint32_t s = blockIdx.x * K4_CTS + ctl;
  const bool active = s < num_samples;
  cplx* ctx = xch_all + ctl * 3 * XS;       // the three owners' scratches of this ciphertext
  cplx* xch = ctx + v * XS;
  uint64_t* xch64 = reinterpret_cast<uint64_t*>(xch);
  cplx* myslot = ctx + role * 64 + lane;    // + poly-slot region * 64 + scratch * XS

  const bool issuer = w < NISS;
  const cplx* key_w = fbsk + (uint64_t)(issuer ? w : 0) * GLDS * 64;
  cplx* ring_w = ring + (issuer ? w : 0) * GLDS * 64;
  const uint32_t lane_b = (uint32_t)lane * (uint32_t)sizeof(cplx);
  // group r of step i (r may run past NGRP into step i + 1) sits in ring slot (i NGRP + r) % RS:
  // with NGRP % RS == 0 a compile-time constant, else (NGRP even, RS = 4) the step's parity adds 2
  auto slot_of = [&](uint32_t i, int r) __attribute__((always_inline)) {
    return NGRP % RS == 0 ? r % RS : (int)((i * (uint32_t)NGRP + (uint32_t)r) & (RS - 1));
  };
  auto issue_group = [&](const cplx* key_step, uint32_t i, int r) __attribute__((always_inline)) {
    if (!issuer) return;
    const char* src = reinterpret_cast<const char*>(key_step + r * GROUP);
    cplx* dst = ring_w + slot_of(i, r) * GROUP;
#pragma unroll
    for (int j = 0; j < GLDS; ++j)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const cplx*>(src + j * 1024 + lane_b),
                                       (lds_ptr_t)(dst + j * 64), 16, 0, 0);
  };
  if (n > 0) {
#pragma unroll
    for (int g = 0; g < DIST; ++g) issue_group(key_w, 0u, g);
  }

  build_fft512_tables(tbl, threadIdx.x, NW * 64);
  if (lane == 0) tflags[w] = 0u;
  uint32_t tcnt = 0;
  __syncthreads();
  const Fft512Tables T = fft512_tables_at(tbl);

  // tz[sl] = zeta_1024 w_512^k, k = fft512_freq(lane, sl): the odd polynomial's unzip twiddle
  cplx tz[SL];
#pragma unroll
  for (int sl = 0; sl < SL; ++sl) {
    const int k = fft512_freq(lane, sl);
    double sn, cs;
    sincospi((double)((1 - 4 * k) & 2047) / 1024.0, &sn, &cs);
    tz[sl] = {cs, sn};
  }

  const uint64_t* lwe = in + (active ? (in_idx ? in_idx[s] : s) : 0) * (uint64_t)(n + 1);
  const uint64_t* lut = luts + (active && lut_idx ? lut_idx[s] : 0ull) * (uint64_t)(K1 * N);
  const bool real = owner && pa < K1;

  // acc_pa = LUT_pa * X^{-ms(b)}: A[m] coefficient j(m), A[m + 8] coefficient j(m) + M
  uint64_t A[16];
  {
    const uint32_t bt = active ? modswitch(lwe[n], LOG2_2N) : 0u;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int c = jb + 32 * (m & 7) + (m >= 8 ? M : 0);
      const uint32_t src = (uint32_t)(c + bt) & (2 * N - 1);
      const uint64_t val = active && real ? lut[pa * N + (src & (N - 1))] : 0ull;
      A[m] = src < N ? val : 0ull - val;
    }
  }

  const int nrep = 64 - NQ * (int)base_log;
  const int logB = (int)base_log;
  double max_resid = 0.0;

  uint64_t a_next = active && owner ? lwe[0] : 0ull;
  for (uint32_t i = 0; i < n; ++i) {
    const cplx* key_step = key_w + (uint64_t)i * PER_I;
    const bool last_step = i + 1 >= n;
    const uint64_t ai = a_next;
    if (i + 1 < n) a_next = active && owner ? lwe[i + 1] : 0ull;
    const uint32_t at = modswitch(ai, LOG2_2N);

    // X[row][f]: row's spectrum of digit polynomial f (sub-digit or level) at my slot
    cplx X[K1][NF];
    if (owner) {
      // ---- ct1 = X^{at} acc - acc in my own scratch (two polynomials of N u64) -------------
      StT st[16];
      {
#pragma unroll
        for (int m = 0; m < 16; ++m) xch64[pl * N + jb + 32 * (m & 7) + (m >= 8 ? M : 0)] = A[m];
        wave_lds_fence();
        uint64_t rv[16];
#pragma unroll
        for (int m = 0; m < 16; ++m) {
          const int c = jb + 32 * (m & 7) + (m >= 8 ? M : 0);
          rv[m] = xch64[pl * N + ((uint32_t)(c - (int)at) & (N - 1))];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < 16; ++m) {
          const int c = jb + 32 * (m & 7) + (m >= 8 ? M : 0);
          const uint32_t sp = (uint32_t)(c - (int)at) & (2 * N - 1);
          st[m] = (StT)decomp_init((sp < N ? rv[m] : 0ull - rv[m]) - A[m], nrep);
        }
        wave_lds_fence();
      }
      // ---- digit polynomials and forward transforms ------------------------------------------
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
          // sub > 0: everyone has read my previous spectra before this transform's first LDS write
          fft512_fwd_tw(vv, xch, lane, tw2, tw3, 0, [&]() __attribute__((always_inline)) {
            if (sub > 0) k4_wait(tflags, ctl, role, tcnt, guard);
          });
          // unzip: E_0 = Z[sl] + Z[sl + 4], E_1 = conj(tz) (Z[sl] - Z[sl + 4])
#pragma unroll
          for (int sl = 0; sl < SL; ++sl) {
            const cplx a = vv[sl], b = vv[sl + SL];
            xch[sl * 64 + lane] = cadd(a, b);
            xch[(SL + sl) * 64 + lane] = cmulc(csub(a, b), tz[sl]);
          }
        }
        // the last digit polynomial's spectra are published by the first key window's barrier
        if (sub + 1 < NF) {
          k4_sync(tflags, ctl, role, tcnt, guard);
#pragma unroll
          for (int row = 0; row < K1; ++row) X[row][sub] = myslot[(row >> 1) * XS + (row & 1) * SL * 64];
#pragma unroll
          for (int row = 0; row < K1; ++row) pin(X[row][sub]);
          k4_signal(tflags, ctl, role, tcnt);
        }
      }
    } else {
      // role 3: the owners' spectra of all but the last digit polynomial
#pragma unroll
      for (int f = 0; f + 1 < NF; ++f) {
        k4_sync(tflags, ctl, role, tcnt, guard);
#pragma unroll
        for (int row = 0; row < K1; ++row) X[row][f] = myslot[(row >> 1) * XS + (row & 1) * SL * 64];
#pragma unroll
        for (int row = 0; row < K1; ++row) pin(X[row][f]);
        k4_signal(tflags, ctl, role, tcnt);
      }
    }

    // ---- per limb: key products for all outputs on my slot, mail, zip + inverse --------------
    // Slot li of output cc = sum over rows of d_lo g_li + d_hi g_{li-1}: Yc[cc] carries the d_hi
    // part into limb li's column-cc window, Yn[cc] starts slot li + 1 with d_hi g_li.
    cplx Yc[K1];
#pragma unroll
    for (int cc = 0; cc < K1; ++cc) Yc[cc] = {0.0, 0.0};
    static_for<0, LIMBS>([&](auto LI) __attribute__((always_inline)) {
      constexpr int li = decltype(LI)::value;
      if constexpr (NQ == 1) {
        constexpr bool HI = SUBS == 2 && li + 1 < LIMBS;  // d_hi g_3 lands at 2^64: vanishes
        cplx Yn[K1];
#pragma unroll
        for (int cc = 0; cc < K1; ++cc) Yn[cc] = {0.0, 0.0};
#pragma unroll
        for (int cc = 0; cc < K1; ++cc) {
          const int r = li * K1 + cc;  // group within the step
          // group r landed for this wave's pieces (the next DIST - 1 may stay in flight) ...
          if (issuer) {
            if (r + DIST - 1 < NGRP || !last_step) wait_vmcnt<GLDS * (DIST - 1)>();
            else if (r + 1 == NGRP) wait_vmcnt<0>();
            else if (r + 2 == NGRP) wait_vmcnt<GLDS>();
            else wait_vmcnt<GLDS * 2>();
          }
          pair_barrier();  // ... for every wave; everyone is done with group r - 1
          if (r + DIST < NGRP || !last_step) issue_group(key_step, i, r + DIST);
          if constexpr (li == 0) {
            if (cc == 0) {
#pragma unroll
              for (int row = 0; row < K1; ++row) X[row][SUBS - 1] = myslot[(row >> 1) * XS + (row & 1) * SL * 64];
            }
          }
          cplx Ya = Yc[cc];
          const cplx* G = ring + slot_of(i, r) * GROUP + role * 64 + lane;
#pragma unroll
          for (int row = 0; row < K1; ++row) {
            const cplx g = G[row * M];
            const cplx x0 = X[row][0];
            Ya.re = __builtin_fma(x0.re, g.re, __builtin_fma(-x0.im, g.im, Ya.re));
            Ya.im = __builtin_fma(x0.re, g.im, __builtin_fma(x0.im, g.re, Ya.im));
            if constexpr (HI) {
              const cplx x1 = X[row][SUBS - 1];
              Yn[cc].re = __builtin_fma(x1.re, g.re, __builtin_fma(-x1.im, g.im, Yn[cc].re));
              Yn[cc].im = __builtin_fma(x1.re, g.im, __builtin_fma(x1.im, g.re, Yn[cc].im));
            }
          }
          // column cc of slot li: my slot into its owner's mailbox (each wave only ever touches its
          // own slot of an owner's scratch; the owner reads it behind the limb's sync)
          myslot[(cc >> 1) * XS + (cc & 1) * SL * 64] = Ya;
          pin(Ya);
          if constexpr (HI) pin(Yn[cc]);
        }
        if constexpr (HI) {
#pragma unroll
          for (int cc = 0; cc < K1; ++cc) Yc[cc] = Yn[cc];
        }
      } else {
        // levels: each output window sums the NQ levels' groups, then mails
#pragma unroll
        for (int cc = 0; cc < K1; ++cc) {
          cplx Ya = {0.0, 0.0};
#pragma unroll
          for (int q = 0; q < NQ; ++q) {
            const int r = (li * K1 + cc) * NQ + q;  // group within the step
            if (issuer) {
              if (r + DIST - 1 < NGRP || !last_step) wait_vmcnt<GLDS * (DIST - 1)>();
              else if (r + 1 == NGRP) wait_vmcnt<0>();
              else if (r + 2 == NGRP) wait_vmcnt<GLDS>();
              else wait_vmcnt<GLDS * 2>();
            }
            pair_barrier();
            if (r + DIST < NGRP || !last_step) issue_group(key_step, i, r + DIST);
            if constexpr (li == 0) {
              if (cc == 0 && q == 0) {  // the last level's spectra (published by this barrier)
#pragma unroll
                for (int row = 0; row < K1; ++row) X[row][NF - 1] = myslot[(row >> 1) * XS + (row & 1) * SL * 64];
              }
            }
            const cplx* G = ring + slot_of(i, r) * GROUP + role * 64 + lane;
#pragma unroll
            for (int row = 0; row < K1; ++row) {
              const cplx g = G[row * M];
              const cplx x = X[row][q];
              Ya.re = __builtin_fma(x.re, g.re, __builtin_fma(-x.im, g.im, Ya.re));
              Ya.im = __builtin_fma(x.re, g.im, __builtin_fma(x.im, g.re, Ya.im));
            }
            pin(Ya);
          }
          myslot[(cc >> 1) * XS + (cc & 1) * SL * 64] = Ya;
        }
      }
      if (!owner) {
        // role 3 only mails: it publishes, and the next window's barrier keeps it from mailing
        // into a scratch its owner still transforms in
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        k4_signal(tflags, ctl, role, tcnt);
        return;
      }
      k4_sync(tflags, ctl, role, tcnt, guard);
      // zip: Z[sl] = E_0 + tz E_1, Z[sl + 4] = E_0 - tz E_1 (role 2's second half has no mail: 0)
      cplx V[8];
#pragma unroll
      for (int sl = 0; sl < SL; ++sl) {
        const cplx e0 = xch[sl * 64 + lane];
        const cplx e1 = v < 2 ? cmul(xch[(SL + sl) * 64 + lane], tz[sl]) : cplx{0.0, 0.0};
        V[sl] = cadd(e0, e1);
        V[sl + SL] = csub(e0, e1);
      }
      {
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
        if constexpr (li == 0) {
          A[m] += (uint64_t)__double_as_longlong(tr) - MAGIC_ALL;
          A[m + 8] += (uint64_t)__double_as_longlong(ti) - MAGIC_ALL;
        } else {
          A[m] += (uint64_t)__double_as_longlong(tr) << (LB * li);
          A[m + 8] += (uint64_t)__double_as_longlong(ti) << (LB * li);
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
  if (active && owner) {
#pragma unroll
    for (int m = 0; m < 16; ++m) xch64[pl * N + jb + 32 * (m & 7) + (m >= 8 ? M : 0)] = A[m];
    wave_lds_fence();
    if (pa < K1 - 1) {
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const int j = jb + 32 * (m & 7) + (m >= 8 ? M : 0);
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

// Many levels (l = K4_MANY_MIN .. 64, runtime), whole digits: one level at a time.  Per level the
// owners transform its digit polynomials, and every role runs the 20 key windows of that level
// (limb, column) into Y[limb][column] at its slot; the key is level-major, [n][q][limb][col][row][M],
// so the ring's group sequence stays contiguous.  After the last level, per limb: mail, sync, zip +
// inverse, a workgroup barrier before the next limb's mail.  Registers: one level's spectra and the
// 20 accumulators, whatever l is.
template <bool RESID>
__global__ void __launch_bounds__(K4_CTS * 256, 1)
pbs512k4_many_kernel(uint64_t* __restrict__ out, const uint64_t* __restrict__ out_idx,
                     const uint64_t* __restrict__ luts, const uint64_t* __restrict__ lut_idx,
                     const uint64_t* __restrict__ in, const uint64_t* __restrict__ in_idx,
                     const cplx* __restrict__ fbsk, uint32_t n, uint32_t level, uint32_t base_log,
                     uint32_t num_samples, unsigned long long* __restrict__ resid_out, SyncGuard guard) {
  constexpr int N = 512, LOG2_2N = 10, K1 = 5, LIMBS = 4, LB = 16;
  constexpr int M = N / 2, SL = 4;
  constexpr int NW = 4 * K4_CTS;
  constexpr int GROUP = K1 * M;             // (level, limb, column): the five row spectra
  constexpr int WPL = LIMBS * K1;           // key windows per level
  constexpr uint64_t MAGIC_ALL = k4_magic_all(LIMBS, LB);
  constexpr int RS = K4_RING_SLOTS, DIST = RS - 1;
  constexpr int GLDS = 4;
  constexpr int NISS = GROUP / 64 / GLDS;
  static_assert(GROUP / 64 == GLDS * NISS && NISS <= NW && WPL % RS == 0 && DIST <= 3, "ring geometry");
  constexpr int XS = (int)PBS1024_XCH_SLOTS;
  const uint32_t NGRP = (uint32_t)WPL * level;  // ring groups per CMUX step
  const uint64_t PER_I = (uint64_t)NGRP * GROUP;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  cplx* tbl = reinterpret_cast<cplx*>(smem);
  cplx* xch_all = tbl + FFT512_TABLE_ENTRIES;
  cplx* ring = xch_all + 3 * K4_CTS * XS;
  uint32_t* tflags = reinterpret_cast<uint32_t*>(ring + RS * GROUP);
  cplx* tzt = reinterpret_cast<cplx*>(tflags + 4 * K4_CTS * 2);  // [slot][lane] unzip twiddles (16-B aligned)

  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int ctl = w >> 2;
  const int role = ctl == 0 ? (w & 3) : ((w + 1) & 3);
  const bool owner = role < 3;
  const int v = owner ? role : 0;
  const int pl = lane & 1, pa = 2 * v + pl, jb = lane >> 1;
  const uint32_t s = blockIdx.x * K4_CTS + ctl;
  const bool active = s < num_samples;
  cplx* ctx = xch_all + ctl * 3 * XS;
  cplx* xch = ctx + v * XS;
  uint64_t* xch64 = reinterpret_cast<uint64_t*>(xch);
  cplx* myslot = ctx + role * 64 + lane;

  const bool issuer = w < NISS;
  const cplx* key_w = fbsk + (uint64_t)(issuer ? w : 0) * GLDS * 64;
  cplx* ring_w = ring + (issuer ? w : 0) * GLDS * 64;
  const uint32_t lane_b = (uint32_t)lane * (uint32_t)sizeof(cplx);
  // group g of the step (g may run past NGRP into the next step, whose key follows contiguously);
  // NGRP is a multiple of RS, so the ring slot is g % RS
  auto issue_group = [&](const cplx* key_step, uint32_t g) __attribute__((always_inline)) {
    if (!issuer) return;
    const char* src = reinterpret_cast<const char*>(key_step + (uint64_t)g * GROUP);
    cplx* dst = ring_w + (g % RS) * GROUP;
#pragma unroll
    for (int j = 0; j < GLDS; ++j)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const cplx*>(src + j * 1024 + lane_b),
                                       (lds_ptr_t)(dst + j * 64), 16, 0, 0);
  };
  if (n > 0) {
#pragma unroll
    for (int g = 0; g < DIST; ++g) issue_group(key_w, (uint32_t)g);
  }

  build_fft512_tables(tbl, threadIdx.x, NW * 64);
  if (lane == 0) tflags[w] = 0u;
  if (threadIdx.x < SL * 64) {  // tz[sl] = zeta_1024 w_512^k, k = fft512_freq(lane, sl), in LDS
    const int k = fft512_freq((int)threadIdx.x & 63, (int)threadIdx.x >> 6);
    double sn, cs;
    sincospi((double)((1 - 4 * k) & 2047) / 1024.0, &sn, &cs);
    tzt[threadIdx.x] = {cs, sn};
  }
  uint32_t tcnt = 0;
  __syncthreads();
  const Fft512Tables T = fft512_tables_at(tbl);

  const uint64_t* lwe = in + (active ? (in_idx ? in_idx[s] : s) : 0) * (uint64_t)(n + 1);
  const uint64_t* lut = luts + (active && lut_idx ? lut_idx[s] : 0ull) * (uint64_t)(K1 * N);
  const bool real = owner && pa < K1;

  uint64_t A[16];
  {
    const uint32_t bt = active ? modswitch(lwe[n], LOG2_2N) : 0u;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int c = jb + 32 * (m & 7) + (m >= 8 ? M : 0);
      const uint32_t src = (uint32_t)(c + bt) & (2 * N - 1);
      const uint64_t val = active && real ? lut[pa * N + (src & (N - 1))] : 0ull;
      A[m] = src < N ? val : 0ull - val;
    }
  }

  const int nrep = 64 - (int)level * (int)base_log;
  const int logB = (int)base_log;
  double max_resid = 0.0;

  uint64_t a_next = active && owner ? lwe[0] : 0ull;
  for (uint32_t i = 0; i < n; ++i) {
    const cplx* key_step = key_w + (uint64_t)i * PER_I;
    const bool last_step = i + 1 >= n;
    const uint64_t ai = a_next;
    if (i + 1 < n) a_next = active && owner ? lwe[i + 1] : 0ull;
    const uint32_t at = modswitch(ai, LOG2_2N);

    uint64_t st[16];
    if (owner) {
#pragma unroll
      for (int m = 0; m < 16; ++m) xch64[pl * N + jb + 32 * (m & 7) + (m >= 8 ? M : 0)] = A[m];
      wave_lds_fence();
      uint64_t rv[16];
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const int c = jb + 32 * (m & 7) + (m >= 8 ? M : 0);
        rv[m] = xch64[pl * N + ((uint32_t)(c - (int)at) & (N - 1))];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const int c = jb + 32 * (m & 7) + (m >= 8 ? M : 0);
        const uint32_t sp = (uint32_t)(c - (int)at) & (2 * N - 1);
        st[m] = decomp_init((sp < N ? rv[m] : 0ull - rv[m]) - A[m], nrep);
      }
      wave_lds_fence();
    }

    cplx Y[LIMBS][K1];
#pragma unroll
    for (int li = 0; li < LIMBS; ++li)
#pragma unroll
      for (int cc = 0; cc < K1; ++cc) Y[li][cc] = {0.0, 0.0};
#pragma unroll 1
    for (uint32_t q = 0; q < level; ++q) {
      // ---- level q: the owners' digit polynomials and forward transforms (published by the
      //      level's first key window barrier; every wave read the previous level's spectra
      //      right after that level's first barrier, 19 windows ago)
      if (owner) {
        cplx vv[8];
        {
          int32_t d[16];
#pragma unroll
          for (int m = 0; m < 16; ++m) d[m] = decomp_next_t(st[m], logB);
#pragma unroll
          for (int m = 0; m < 8; ++m) vv[m] = {(double)d[m], (double)d[m + 8]};
        }
        cplx tw2[4], tw3[4];
        fwd_p2_tw(tw2, T, lane >> 3);
        fwd_p3_tw(tw3, T, lane);
        fft512_fwd_tw(vv, xch, lane, tw2, tw3, 0, []() __attribute__((always_inline)) {});
#pragma unroll
        for (int sl = 0; sl < SL; ++sl) {
          const cplx a = vv[sl], b = vv[sl + SL];
          xch[sl * 64 + lane] = cadd(a, b);
          xch[(SL + sl) * 64 + lane] = cmulc(csub(a, b), tzt[sl * 64 + lane]);
        }
      }
      cplx X[K1];
#pragma unroll
      for (int wi = 0; wi < WPL; ++wi) {
        const int li = wi / K1, cc = wi % K1;
        const uint32_t r = q * (uint32_t)WPL + (uint32_t)wi;  // group within the step
        if (issuer) {
          if (r + DIST - 1 < NGRP || !last_step) wait_vmcnt<GLDS * (DIST - 1)>();
          else if (r + 1 == NGRP) wait_vmcnt<0>();
          else if (r + 2 == NGRP) wait_vmcnt<GLDS>();
          else wait_vmcnt<GLDS * 2>();
        }
        pair_barrier();
        if (r + DIST < NGRP || !last_step) issue_group(key_step, r + DIST);
        if (wi == 0) {
#pragma unroll
          for (int row = 0; row < K1; ++row) X[row] = myslot[(row >> 1) * XS + (row & 1) * SL * 64];
        }
        const cplx* G = ring + (wi % RS) * GROUP + role * 64 + lane;
#pragma unroll
        for (int row = 0; row < K1; ++row) {
          const cplx g = G[row * M];
          Y[li][cc].re = __builtin_fma(X[row].re, g.re, __builtin_fma(-X[row].im, g.im, Y[li][cc].re));
          Y[li][cc].im = __builtin_fma(X[row].re, g.im, __builtin_fma(X[row].im, g.re, Y[li][cc].im));
        }
        pin(Y[li][cc]);
      }
    }

    // ---- per limb: mail my slot of the five outputs, sync, zip + inverse, barrier -------------
#pragma unroll
    for (int li = 0; li < LIMBS; ++li) {
#pragma unroll
      for (int cc = 0; cc < K1; ++cc) myslot[(cc >> 1) * XS + (cc & 1) * SL * 64] = Y[li][cc];
      if (owner) {
        k4_sync(tflags, ctl, role, tcnt, guard);
        cplx V[8];
#pragma unroll
        for (int sl = 0; sl < SL; ++sl) {
          const cplx e0 = xch[sl * 64 + lane];
          const cplx e1 = v < 2 ? cmul(xch[(SL + sl) * 64 + lane], tzt[sl * 64 + lane]) : cplx{0.0, 0.0};
          V[sl] = cadd(e0, e1);
          V[sl + SL] = csub(e0, e1);
        }
        {
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
          if (li == 0) {
            A[m] += (uint64_t)__double_as_longlong(tr) - MAGIC_ALL;
            A[m + 8] += (uint64_t)__double_as_longlong(ti) - MAGIC_ALL;
          } else {
            A[m] += (uint64_t)__double_as_longlong(tr) << (LB * li);
            A[m + 8] += (uint64_t)__double_as_longlong(ti) << (LB * li);
          }
        }
#pragma unroll
        for (int m = 0; m < 16; ++m) pin(A[m]);
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        k4_signal(tflags, ctl, role, tcnt);
      }
      // every owner is done with its scratch (the next limb's mail, the next step's rotation)
      pair_barrier();
    }
  }

  uint64_t* o = out + (active ? (out_idx ? out_idx[s] : s) : 0) * (uint64_t)((K1 - 1) * N + 1);
  if (active && owner) {
#pragma unroll
    for (int m = 0; m < 16; ++m) xch64[pl * N + jb + 32 * (m & 7) + (m >= 8 ? M : 0)] = A[m];
    wave_lds_fence();
    if (pa < K1 - 1) {
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const int j = jb + 32 * (m & 7) + (m >= 8 ? M : 0);
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

template <int SUBS, int NQ, int LIMBS, bool RESID>
static int launch_k4_t(const PbsArgs& a) {
  const size_t lds = pbs512k4_lds_bytes();
  auto kern = pbs512k4_kernel<SUBS, NQ, LIMBS, RESID>;
  CHIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const uint32_t blocks = (a.num_samples + K4_CTS - 1) / K4_CTS;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(K4_CTS * 256), lds, a.stream, a.out, a.out_idx, a.luts, a.lut_idx,
                     a.in, a.in_idx, reinterpret_cast<const cplx*>(a.fbsk), a.n, a.base_log, a.num_samples, a.resid,
                     a.guard);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("pbs launch failed: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

template <int SUBS, int NQ, int LIMBS = 4>
static int launch_k4_r(const PbsArgs& a) {
  return a.resid ? launch_k4_t<SUBS, NQ, LIMBS, true>(a) : launch_k4_t<SUBS, NQ, LIMBS, false>(a);
}

template <bool RESID>
static int launch_k4_many_t(const PbsArgs& a) {
  const size_t lds = pbs512k4_lds_bytes();
  auto kern = pbs512k4_many_kernel<RESID>;
  CHIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const uint32_t blocks = (a.num_samples + K4_CTS - 1) / K4_CTS;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(K4_CTS * 256), lds, a.stream, a.out, a.out_idx, a.luts, a.lut_idx,
                     a.in, a.in_idx, reinterpret_cast<const cplx*>(a.fbsk), a.n, a.level, a.base_log,
                     a.num_samples, a.resid, a.guard);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("pbs launch failed: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

int pbs512k4_launch(const PbsArgs& a) {
  if (!(a.N == 512 && a.k == 4 && a.limbs == small_limbs(a.k, a.N, a.level) &&
        pbs_small_ok(a.k, a.N, a.level, a.base_log))) {
    set_error("unsupported PBS parameters: N=%u k=%u level=%u base_log=%u limbs=%u", a.N, a.k, a.level, a.base_log,
              a.limbs);
    return -2;
  }
  if (a.num_samples == 0) return 0;
  if (a.level >= K4_MANY_MIN) return a.resid ? launch_k4_many_t<true>(a) : launch_k4_many_t<false>(a);
  switch (a.level) {
    // logB <= 15: |digit| <= 2^14 fits the 16-bit grid whole (one sub-digit)
    case 1: return a.base_log <= 15 ? launch_k4_r<1, 1>(a) : launch_k4_r<2, 1>(a);
    default: return launch_k4_r<1, 2, 5>(a);  // l = 2: 13-bit key limbs
  }
}

}  // namespace chip
