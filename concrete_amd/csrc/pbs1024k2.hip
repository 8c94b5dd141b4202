// pbs1024k2.hip — batched classic PBS for N = 1024, k = 2, l = 1 (the optimizer's 4-bit rows,
// v0-parameters: n = 801, logB = 23; bench.py --config opt4) and l = 2 at logB <= 15 (its rows at
// log norm2 >= 1: br 2/15) on CDNA4 (gfx950).
//
// Same semantics as pbs.hip (concrete-cpu c_api/bootstrap.rs:347-414 -> tfhe 0.10
// blind_rotate_assign + sample extract; restated in oracle/tfhe_oracle.c:ora_pbs) and the same
// exact arithmetic as pbs2048.hip:
//
// * Sub-digits on the limb grid.  The key polynomial g is split into 4 balanced 16-bit limbs,
//   g = sum_j 2^{16 j} g_j, and a digit d (logB <= 24) exactly into d = d_lo + 2^16 d_hi with d_lo
//   balanced 16-bit and |d_hi| <= 2^(logB-17) + 1, so
//       d g = sum_m 2^{16 m} (d_lo g_m + d_hi g_{m-1})   (mod 2^64, slots m = 0..3)
//   and each slot is one exact integer convolution sum over the three rows (certified error
//   < 1/2, oracle/pyoracle.py:gpu1024k2_error_bound).  Limb j's key serves slot j (d_lo) and slot
//   j + 1 (d_hi, carried into the next limb's windows).
// * The N = 1024 negacyclic products are pbs.hip's: one-wave 512-point folded, twisted
//   transforms in registers (fft512.hpp), key spectra in the same (lane, slot) order, scaled 1/512.
//
// Mapping: three waves per ciphertext; wave v owns GLWE polynomial v of the accumulator (16 u64
// per lane, lane t holds coefficient t + 64 m), runs the forward transforms of its own two
// sub-digit polynomials, keeps frequency slots [SB(v), SB(v+1)) of all three rows' spectra (the
// rest is read by its partners from its scratch), runs the key MAC for all three outputs on its
// slots, mails each output's slots to the owning wave and runs the four inverse transforms of its
// own output.  The slot shares are 3 / 2 / 3: a workgroup of two ciphertexts is six waves, which
// land on the four SIMDs as {0, 4}, {1, 5}, {2}, {3}, so the two SIMDs holding two waves each carry
// one 3-slot and one 2-slot wave (ciphertext 0's waves 0, 1 and ciphertext 1's waves 1, 2).
// The two ciphertexts of a workgroup share a ring of 24 KB key groups (one limb and one output
// column: three row spectra) filled by LDS-DMA, so the key crosses the L2->CU port once per
// workgroup.
#include "common.hpp"
#include "fft512.hpp"
#include "kernel_util.hpp"
#include "pbs.hpp"

#include <type_traits>

namespace chip {

namespace {

constexpr uint64_t K2_MAGIC_ALL =
    RND_MAGIC_BITS + (RND_MAGIC_BITS << 16) + (RND_MAGIC_BITS << 32) + (RND_MAGIC_BITS << 48);

// first frequency slot of wave v's share (v = 0, 1, 2; SB(3) = 8)
#ifndef K2_SB1
#define K2_SB1 3
#endif
#ifndef K2_SB2
#define K2_SB2 5
#endif
#ifndef K2_ASM_DMA
#define K2_ASM_DMA 0
#endif
// Diagnostic builds only (timing; wrong results): K2D_NOBAR (no key-window barriers), K2D_NOMAC
// (no key MAC FMAs), K2D_NOINV / K2D_NOFWD (no inverse / forward transforms), K2D_NOTRI (no
// three-wave syncs).
#ifndef K2D_NOBAR
#define K2D_NOBAR 0
#endif
#ifndef K2D_NOMAC
#define K2D_NOMAC 0
#endif
#ifndef K2D_NOINV
#define K2D_NOINV 0
#endif
#ifndef K2D_NOFWD
#define K2D_NOFWD 0
#endif
#ifndef K2D_NOTRI
#define K2D_NOTRI 0
#endif
#ifndef K2D_NOROT
#define K2D_NOROT 0
#endif
#ifndef K2D_NOXRD
#define K2D_NOXRD 0
#endif
__device__ __forceinline__ int k2_slot_base(int v) { return v == 0 ? 0 : (v == 1 ? K2_SB1 : K2_SB2); }

// Synchronisation of the three waves of one ciphertext (never the other ciphertext of the
// workgroup): each wave publishes how many sync points it has passed and waits until its two
// partners have reached the same count.  LDS traffic is drained, the key DMA is not.
__device__ __forceinline__ void tri_sync(uint32_t* flags, int ctl, int v, uint32_t& cnt, const SyncGuard& guard) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (K2D_NOTRI) return;
  ++cnt;
  __hip_atomic_store(&flags[ctl * 3 + v], cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  spin_until_ge(&flags[ctl * 3 + (v == 2 ? 0 : v + 1)], cnt, guard);
  spin_until_ge(&flags[ctl * 3 + (v == 0 ? 2 : v - 1)], cnt, guard);
}
// Split form: tri_signal publishes that this wave's reads of its partners' scratches have been
// issued (LDS operations of a wave execute in order); tri_wait, before this wave next overwrites
// its own scratch, waits for its partners' signals.
__device__ __forceinline__ void tri_signal(uint32_t* flags, int ctl, int v, uint32_t& cnt) {
  asm volatile("" ::: "memory");
  ++cnt;
  __hip_atomic_store(&flags[ctl * 3 + v], cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void tri_wait(uint32_t* flags, int ctl, int v, uint32_t cnt, const SyncGuard& guard) {
  if (K2D_NOTRI) return;
  spin_until_ge(&flags[ctl * 3 + (v == 2 ? 0 : v + 1)], cnt, guard);
  spin_until_ge(&flags[ctl * 3 + (v == 0 ? 2 : v - 1)], cnt, guard);
  asm volatile("" ::: "memory");
}

// the four waves of one ciphertext in the many-level kernel (counters f[ct * 4 + role])
__device__ __forceinline__ void k2q_signal(uint32_t* f, int ctl, int role, uint32_t& cnt) {
  asm volatile("" ::: "memory");
  ++cnt;
  __hip_atomic_store(&f[ctl * 4 + role], cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void k2q_sync(uint32_t* f, int ctl, int role, uint32_t& cnt, const SyncGuard& guard) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  k2q_signal(f, ctl, role, cnt);
#pragma unroll
  for (int o = 1; o < 4; ++o) spin_until_ge(&f[ctl * 4 + ((role + o) & 3)], cnt, guard);
  asm volatile("" ::: "memory");
}

}  // namespace

// NQ = 1: l = 1, the two sub-digits of one digit (d_hi carried into the next slot); NQ = l = 2 (from
// l = 3 pbs1024k2_many_kernel runs one level at a time):
// whole digits (l 2^(logB-1) <= 2^15), the levels' products in the same slot (the key
// holds both levels, [n][limb][col][q][row][512], one ring group per level).
template <bool RESID, int NQ>
__global__ void __launch_bounds__(K2_CTS * 192, 1)
pbs1024k2_kernel(uint64_t* __restrict__ out, const uint64_t* __restrict__ out_idx,
                 const uint64_t* __restrict__ luts, const uint64_t* __restrict__ lut_idx,
                 const uint64_t* __restrict__ in, const uint64_t* __restrict__ in_idx,
                 const cplx* __restrict__ fbsk, uint32_t n, uint32_t base_log, uint32_t num_samples,
                 unsigned long long* __restrict__ resid_out, SyncGuard guard) {
  constexpr int N = 1024, LOG2_2N = 11, K1 = 3;
  constexpr int NW = 3 * K2_CTS;              // waves per workgroup
  constexpr bool LEVELS = NQ > 1;             // key levels per (limb, column): NQ
  constexpr int NF = LEVELS ? NQ : K2_SUBS;   // digit polynomials (sub-digits or levels) per step
  using StT = std::conditional_t<(NQ > 2), uint64_t, uint32_t>;  // decomposition state (l logB bits)
  constexpr int GROUP = K1 * 512;             // (limb, column[, level]): the three row spectra
  constexpr int NGRP = K2_LIMBS * K1 * NQ;    // ring groups per CMUX step
  constexpr int PER_I = NGRP * GROUP;         // complex values per Fourier GGSW
  constexpr int RS = K2_RING_SLOTS, DIST = K2_RING_SLOTS - 1;
  constexpr int GLDS = GROUP / 64 / NW;       // 1 KB LDS-DMA pieces per wave per group
  constexpr int XS = (int)PBS1024_XCH_SLOTS;
  constexpr int MS = 3;                       // largest slot share
  static_assert(GROUP % (64 * NW) == 0 && NGRP % RS == 0, "ring geometry");
  static_assert(XCH_SLOTS <= XS, "transpose scratch");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  cplx* tbl = reinterpret_cast<cplx*>(smem);   // FFT tables (fft512.hpp)
  cplx* xch_all = tbl + FFT512_TABLE_ENTRIES;  // NW x XS: transpose scratch and mailboxes
  cplx* ring = xch_all + NW * XS;              // RS x GROUP key ring
  uint32_t* tflags = reinterpret_cast<uint32_t*>(ring + RS * GROUP);  // NW sync counters

  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int ctl = w / 3;  // ciphertext within the workgroup
  const int v = w - 3 * ctl;  // own polynomial
  const int sb = k2_slot_base(v);
  // slots of my share; every share has at least 2 (K2_SB1, K2_SB2), so only slot 2 is conditional
  const int ns = (v == 2 ? 8 : k2_slot_base(v + 1)) - sb;
  static_assert(K2_SB1 >= 2 && K2_SB2 - K2_SB1 >= 2 && 8 - K2_SB2 >= 2 && K2_SB1 <= 3 && K2_SB2 - K2_SB1 <= 3 &&
                    8 - K2_SB2 <= 3,
                "slot shares of 2 or 3");
  auto has = [&](int jj) __attribute__((always_inline)) { return jj < 2 || ns > 2; };
  const uint32_t s = blockIdx.x * K2_CTS + ctl;
  const bool active = s < num_samples;
  cplx* xch = xch_all + w * XS;
  uint64_t* xch64 = reinterpret_cast<uint64_t*>(xch);
  cplx* ctx = xch_all + ctl * 3 * XS;  // the three scratches of this ciphertext

  // ---- key ring: group g = (step g / NGRP, r = g % NGRP) -> slot g % RS (a constant within a
  // step: NGRP is a multiple of RS), so the refill is one wave-uniform base plus immediates.
  const cplx* key_w = fbsk + (uint64_t)w * GLDS * 64;  // this wave's pieces of every group
  cplx* ring_w = ring + w * GLDS * 64;
  const uint32_t lane_b = (uint32_t)lane * (uint32_t)sizeof(cplx);
  auto issue_group = [&](const cplx* key_step, int r) __attribute__((always_inline)) {
    const char* src = reinterpret_cast<const char*>(key_step + r * GROUP);
    cplx* dst = ring_w + (r % RS) * GROUP;
#pragma unroll
    for (int j = 0; j < GLDS; ++j) {
#if K2_ASM_DMA
      const cplx* gp = reinterpret_cast<const cplx*>(src + j * 1024 + lane_b);
      const uint32_t m0 = (uint32_t)(uintptr_t)(lds_ptr_t)(dst + j * 64);
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
      asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" : : "v"(gp), "s"(m0) : "m0", "memory");
#pragma clang diagnostic pop
#else
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const cplx*>(src + j * 1024 + lane_b),
                                       (lds_ptr_t)(dst + j * 64), 16, 0, 0);
#endif
    }
  };
  if (n > 0) {
#pragma unroll
    for (int g = 0; g < DIST; ++g) issue_group(key_w, g);
  }

  build_fft512_tables(tbl, threadIdx.x, NW * 64);
  if (lane == 0) tflags[w] = 0u;
  uint32_t tcnt = 0;
  __syncthreads();
  const Fft512Tables T = fft512_tables_at(tbl);

  const uint64_t* lwe = in + (active ? (in_idx ? in_idx[s] : s) : 0) * (uint64_t)(n + 1);
  const uint64_t* lut = luts + (active && lut_idx ? lut_idx[s] : 0ull) * (uint64_t)(K1 * N);

  // acc_v = LUT_v * X^{-ms(b)}: lane t holds coefficients t + 64 m
  uint64_t A[16];
  {
    const uint32_t bt = active ? modswitch(lwe[n], LOG2_2N) : 0u;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const uint32_t src = (uint32_t)(lane + 64 * m + bt) & (2 * N - 1);
      const uint64_t val = active ? lut[v * N + (src & (N - 1))] : 0ull;
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
    // a zero mask element (tfhe skips it) runs on ct1 = 0: exact zeros throughout (pbs.hip)

    // ---- ct1 = X^{at} acc - acc within my own scratch (nobody else reads or writes it between
    //      the last limb's mailbox read and this step's first spectrum exchange)
    StT st[16];
    {
#pragma unroll
      for (int m = 0; m < 16; ++m) xch64[lane + 64 * m] = A[m];
      wave_lds_fence();
      uint64_t rv[16];
#pragma unroll
      for (int m = 0; m < 16; ++m) rv[m] = K2D_NOROT ? A[m] ^ at : xch64[(uint32_t)(lane + 64 * m - (int)at) & (N - 1)];
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const uint32_t sp = (uint32_t)(lane + 64 * m - (int)at) & (2 * N - 1);
        st[m] = (StT)decomp_init((sp < N ? rv[m] : 0ull - rv[m]) - A[m], nrep);
      }
      wave_lds_fence();
    }

    // ---- one level, two sub-digit polynomials, forward transforms ------------------------
    // X[row][sub][jj]: spectrum of row `row`'s sub-digit polynomial at my slot sb + jj
    cplx X[K1][NF][MS];
    int32_t dlo[16], dhi[16];
#pragma unroll
    for (int m = 0; m < (NQ <= 2 ? 16 : 0); ++m) {  // NQ > 2: each level's digits before its transform
      const int32_t d = decomp_next_t(st[m], logB);
      if constexpr (LEVELS) {
        dlo[m] = d;                           // level q = 0 (least significant first)
        dhi[m] = decomp_next_t(st[m], logB);  // level q = 1
      } else {
        const int32_t lo = ((d + (1 << (K2_SUB_BITS - 1))) & ((1 << K2_SUB_BITS) - 1)) - (1 << (K2_SUB_BITS - 1));
        dlo[m] = lo;
        dhi[m] = (d - lo) >> K2_SUB_BITS;  // exact: d - lo is a multiple of 2^16
      }
    }
#pragma unroll
    for (int sub = 0; sub < NF; ++sub) {
      {
        if constexpr (NQ > 2) {
#pragma unroll
          for (int m = 0; m < 16; ++m) dlo[m] = decomp_next_t(st[m], logB);  // level q = sub
        }
        cplx vv8[8];
#pragma unroll
        for (int m = 0; m < 8; ++m)
          vv8[m] = sub == 0 || NQ > 2 ? cplx{(double)dlo[m], (double)dlo[m + 8]} : cplx{(double)dhi[m], (double)dhi[m + 8]};
        cplx tw2[4], tw3[4];
        fwd_p2_tw(tw2, T, lane >> 3);
        fwd_p3_tw(tw3, T, lane);
        // the sub-0 exchange's "everyone has read my spectrum" wait, right before this
        // transform's first LDS write (the partners signalled right after their reads)
        if (!K2D_NOFWD)
          fft512_fwd_tw(vv8, xch, lane, tw2, tw3, 0, [&]() __attribute__((always_inline)) {
            if (sub > 0) tri_wait(tflags, ctl, v, tcnt, guard);
          });
#pragma unroll
        for (int k2 = 0; k2 < 8; ++k2) xch[k2 * 64 + lane] = vv8[k2];
      }
      // The last sub-digit's spectra need no sync: the first key window's workgroup barrier
      // (which drains every wave's LDS writes) publishes them; they are read right after it.
      if (sub + 1 < NF) {
        tri_sync(tflags, ctl, v, tcnt, guard);
#pragma unroll
        for (int row = 0; row < K1; ++row)
#pragma unroll
          for (int jj = 0; jj < MS; ++jj)
            if (has(jj)) X[row][sub][jj] = ctx[(K2D_NOXRD ? v : row) * XS + (sb + jj) * 64 + lane];
#pragma unroll
        for (int row = 0; row < K1; ++row)
#pragma unroll
          for (int jj = 0; jj < MS; ++jj) pin(X[row][sub][jj]);
        tri_signal(tflags, ctl, v, tcnt);
      }
    }

    // ---- per limb: MAC for the three outputs on my slots, mail them, inverse of my own -----
    // Slot li of output cc = sum over rows of d_lo g_li + d_hi g_{li-1}: Yc[cc] carries the d_hi
    // part (from the previous limb's windows) into limb li's column-cc window, Yn[cc] starts
    // slot li + 1 with d_hi g_li.
    cplx Yc[K1][MS];
#pragma unroll
    for (int cc = 0; cc < K1; ++cc)
#pragma unroll
      for (int jj = 0; jj < MS; ++jj) Yc[cc][jj] = {0.0, 0.0};
    static_for<0, K2_LIMBS>([&](auto LI) __attribute__((always_inline)) {
      constexpr int li = decltype(LI)::value;
      if constexpr (!LEVELS) {
        constexpr bool HI = li + 1 < K2_LIMBS;  // d_hi g_3 lands at 2^64: vanishes
        cplx Yn[K1][MS];
#pragma unroll
        for (int cc = 0; cc < K1; ++cc)
#pragma unroll
          for (int jj = 0; jj < MS; ++jj) Yn[cc][jj] = {0.0, 0.0};
#pragma unroll
        for (int cc = 0; cc < K1; ++cc) {
          const int r = li * K1 + cc;  // group within the step
          // group r landed for this wave's pieces (the next DIST - 1 may stay in flight) ...
          if (r + DIST - 1 < NGRP || !last_step) wait_vmcnt<GLDS * (DIST - 1)>();
          else wait_vmcnt<0>();
          if (!K2D_NOBAR) pair_barrier();  // ... for every wave; everyone is done with group r - 1
          // refill the slot of group r - 1 with group r + DIST (RS = DIST + 1)
          if (r + DIST < NGRP) issue_group(key_step, r + DIST);
          else if (!last_step) issue_group(key_step + PER_I, r + DIST - NGRP);
          if constexpr (li == 0) {
            if (cc == 0) {  // the last sub-digit's spectra (see above)
#pragma unroll
              for (int row = 0; row < K1; ++row)
#pragma unroll
                for (int jj = 0; jj < MS; ++jj)
                  if (has(jj)) X[row][NF - 1][jj] = ctx[(K2D_NOXRD ? v : row) * XS + (sb + jj) * 64 + lane];
            }
          }
          cplx Ya[MS];
#pragma unroll
          for (int jj = 0; jj < MS; ++jj) Ya[jj] = Yc[cc][jj];
          const cplx* G = ring + (r % RS) * GROUP + sb * 64 + lane;
#pragma unroll
          for (int row = 0; row < K1; ++row) {
            cplx g[MS];
#pragma unroll
            for (int jj = 0; jj < MS; ++jj)
              if (has(jj)) g[jj] = G[row * 512 + jj * 64];
#pragma unroll
            for (int jj = 0; jj < (K2D_NOMAC ? 0 : MS); ++jj) {
              if (has(jj)) {
                const cplx x0 = X[row][0][jj];
                Ya[jj].re = __builtin_fma(x0.re, g[jj].re, __builtin_fma(-x0.im, g[jj].im, Ya[jj].re));
                Ya[jj].im = __builtin_fma(x0.re, g[jj].im, __builtin_fma(x0.im, g[jj].re, Ya[jj].im));
                if constexpr (HI) {
                  const cplx x1 = X[row][1][jj];
                  Yn[cc][jj].re = __builtin_fma(x1.re, g[jj].re, __builtin_fma(-x1.im, g[jj].im, Yn[cc][jj].re));
                  Yn[cc][jj].im = __builtin_fma(x1.re, g[jj].im, __builtin_fma(x1.im, g[jj].re, Yn[cc][jj].im));
                }
              }
            }
          }
          // column cc of slot li is complete: my slots straight into wave cc's mailbox.  Every
          // scratch has been idle (for writes of its owner) since this limb's first barrier, and
          // each wave only ever touches its own slots of a partner's scratch.
#pragma unroll
          for (int jj = 0; jj < MS; ++jj)
            if (has(jj)) ctx[cc * XS + (sb + jj) * 64 + lane] = Ya[jj];
#pragma unroll
          for (int jj = 0; jj < MS; ++jj) {
            pin(Ya[jj]);
            if constexpr (HI) pin(Yn[cc][jj]);
          }
        }
        if constexpr (HI) {
#pragma unroll
          for (int cc = 0; cc < K1; ++cc)
#pragma unroll
            for (int jj = 0; jj < MS; ++jj) Yc[cc][jj] = Yn[cc][jj];
        }
      } else {
        // l = 2: both levels' products land in slot li, one key window per (column, level)
#pragma unroll
        for (int cc = 0; cc < K1; ++cc) {
          cplx Ya[MS];
#pragma unroll
          for (int jj = 0; jj < MS; ++jj) Ya[jj] = {0.0, 0.0};
#pragma unroll
          for (int q = 0; q < NQ; ++q) {
            const int r = (li * K1 + cc) * NQ + q;  // group within the step
            if (r + DIST - 1 < NGRP || !last_step) wait_vmcnt<GLDS * (DIST - 1)>();
            else wait_vmcnt<0>();
            if (!K2D_NOBAR) pair_barrier();
            if (r + DIST < NGRP) issue_group(key_step, r + DIST);
            else if (!last_step) issue_group(key_step + PER_I, r + DIST - NGRP);
            if constexpr (li == 0) {
              if (cc == 0 && q == 0) {  // the second level's spectra (published by this barrier)
#pragma unroll
                for (int row = 0; row < K1; ++row)
#pragma unroll
                  for (int jj = 0; jj < MS; ++jj)
                    if (has(jj)) X[row][NF - 1][jj] = ctx[row * XS + (sb + jj) * 64 + lane];
              }
            }
            const cplx* G = ring + (r % RS) * GROUP + sb * 64 + lane;
#pragma unroll
            for (int row = 0; row < K1; ++row) {
              cplx g[MS];
#pragma unroll
              for (int jj = 0; jj < MS; ++jj)
                if (has(jj)) g[jj] = G[row * 512 + jj * 64];
#pragma unroll
              for (int jj = 0; jj < MS; ++jj) {
                if (has(jj)) {
                  const cplx x = X[row][q][jj];
                  Ya[jj].re = __builtin_fma(x.re, g[jj].re, __builtin_fma(-x.im, g[jj].im, Ya[jj].re));
                  Ya[jj].im = __builtin_fma(x.re, g[jj].im, __builtin_fma(x.im, g[jj].re, Ya[jj].im));
                }
              }
            }
#pragma unroll
            for (int jj = 0; jj < MS; ++jj) pin(Ya[jj]);
          }
#pragma unroll
          for (int jj = 0; jj < MS; ++jj)
            if (has(jj)) ctx[cc * XS + (sb + jj) * 64 + lane] = Ya[jj];
        }
      }
      cplx V[8];
      tri_sync(tflags, ctl, v, tcnt, guard);
#pragma unroll
      for (int k2 = 0; k2 < 8; ++k2) V[k2] = xch[k2 * 64 + lane];
      {
        cplx gi2[4];
        inv_p2_stage_tw(gi2, T, lane & 7);
        if (!K2D_NOINV) fft512_inv_tw(V, xch, T, lane, gi2, 0);
      }
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const double tr = V[m].re + RND_MAGIC, ti = V[m].im + RND_MAGIC;
        if constexpr (RESID) {
          max_resid = fmax(max_resid, fabs(V[m].re - (tr - RND_MAGIC)));
          max_resid = fmax(max_resid, fabs(V[m].im - (ti - RND_MAGIC)));
        }
        if constexpr (li == 0) {
          A[m] += (uint64_t)__double_as_longlong(tr) - K2_MAGIC_ALL;
          A[m + 8] += (uint64_t)__double_as_longlong(ti) - K2_MAGIC_ALL;
        } else {
          A[m] += (uint64_t)__double_as_longlong(tr) << (16 * li);
          A[m + 8] += (uint64_t)__double_as_longlong(ti) << (16 * li);
        }
      }
      // materialise A here (else the inverse tail sinks into the next limb's key windows)
#pragma unroll
      for (int m = 0; m < 16; ++m) pin(A[m]);
      if constexpr (RESID) pin(max_resid);
    });
  }

  // ---- sample extract (nth = 0): mask segment c: out[c N + j] = -A_c[N - j] (j > 0), A_c[0];
  //      body out[k N] = A_k[0]
  uint64_t* o = out + (active ? (out_idx ? out_idx[s] : s) : 0) * (uint64_t)(2 * N + 1);
  if (!active) {
  } else if (v < 2) {
#pragma unroll
    for (int m = 0; m < 16; ++m) xch64[lane + 64 * m] = A[m];
    wave_lds_fence();
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int j = lane + 64 * m;
      const uint64_t val = xch64[(N - j) & (N - 1)];
      o[v * N + j] = j == 0 ? val : 0ull - val;
    }
  } else if (lane == 0) {
    o[2 * N] = A[0];
  }

  if constexpr (RESID) {
    for (int off = 32; off > 0; off >>= 1) max_resid = fmax(max_resid, __shfl_xor(max_resid, off));
    if (lane == 0 && active && resid_out) atomicMax(resid_out, (unsigned long long)__double_as_longlong(max_resid));
  }
}

template <bool RESID, int NQ>
static int launch_k2_t(const PbsArgs& a) {
  const size_t lds = pbs1024k2_lds_bytes();
  auto kern = pbs1024k2_kernel<RESID, NQ>;
  CHIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const uint32_t blocks = (a.num_samples + K2_CTS - 1) / K2_CTS;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(K2_CTS * 192), lds, a.stream, a.out, a.out_idx, a.luts, a.lut_idx,
                     a.in, a.in_idx, reinterpret_cast<const cplx*>(a.fbsk), a.n, a.base_log, a.num_samples, a.resid,
                     a.guard);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("pbs launch failed: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

// Many levels (l >= K2_MANY_MIN, runtime), whole digits, one level at a time (as
// pbs512k4_many_kernel): four waves per ciphertext — the three polynomial owners and a fourth with
// no accumulator — each keeping two of the eight spectrum slots and Y[limb][column][slot] for them
// (24 accumulators, whatever l is); the key level-major, [n][q][limb][col][row][512].
template <bool RESID>
__global__ void __launch_bounds__(K2_CTS * 256, 1)
pbs1024k2_many_kernel(uint64_t* __restrict__ out, const uint64_t* __restrict__ out_idx,
                      const uint64_t* __restrict__ luts, const uint64_t* __restrict__ lut_idx,
                      const uint64_t* __restrict__ in, const uint64_t* __restrict__ in_idx,
                      const cplx* __restrict__ fbsk, uint32_t n, uint32_t level, uint32_t base_log,
                      uint32_t num_samples, unsigned long long* __restrict__ resid_out, SyncGuard guard) {
  constexpr int N = 1024, LOG2_2N = 11, K1 = 3, LIMBS = K2_LIMBS, MS = 2;
  constexpr int NW = 4 * K2_CTS;
  constexpr int GROUP = K1 * 512;           // (level, limb, column): the three row spectra
  constexpr int WPL = LIMBS * K1;           // key windows per level
  constexpr int RS = K2_RING_SLOTS, DIST = RS - 1;
  constexpr int GLDS = 4;
  constexpr int NISS = GROUP / 64 / GLDS;   // waves 0 .. NISS - 1 issue a group's pieces
  static_assert(GROUP / 64 == GLDS * NISS && NISS <= NW && WPL % RS == 0 && DIST <= 3, "ring geometry");
  constexpr int XS = (int)PBS1024_XCH_SLOTS;
  const uint32_t NGRP = (uint32_t)WPL * level;
  const uint64_t PER_I = (uint64_t)NGRP * GROUP;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  cplx* tbl = reinterpret_cast<cplx*>(smem);
  cplx* xch_all = tbl + FFT512_TABLE_ENTRIES;
  cplx* ring = xch_all + 3 * K2_CTS * XS;   // (the fourth wave has no scratch)
  uint32_t* tflags = reinterpret_cast<uint32_t*>(ring + RS * GROUP);

  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int ctl = w >> 2;
  const int role = ctl == 0 ? (w & 3) : ((w + 1) & 3);  // slots 2 role, 2 role + 1
  const bool owner = role < 3;
  const int v = owner ? role : 0;           // owned polynomial
  const uint32_t s = blockIdx.x * K2_CTS + ctl;
  const bool active = s < num_samples;
  cplx* ctx = xch_all + ctl * 3 * XS;
  cplx* xch = ctx + v * XS;
  uint64_t* xch64 = reinterpret_cast<uint64_t*>(xch);
  cplx* myslot = ctx + 2 * role * 64 + lane;  // + jj * 64 + scratch * XS

  const bool issuer = w < NISS;
  const cplx* key_w = fbsk + (uint64_t)(issuer ? w : 0) * GLDS * 64;
  cplx* ring_w = ring + (issuer ? w : 0) * GLDS * 64;
  const uint32_t lane_b = (uint32_t)lane * (uint32_t)sizeof(cplx);
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
  uint32_t tcnt = 0;
  __syncthreads();
  const Fft512Tables T = fft512_tables_at(tbl);

  const uint64_t* lwe = in + (active ? (in_idx ? in_idx[s] : s) : 0) * (uint64_t)(n + 1);
  const uint64_t* lut = luts + (active && lut_idx ? lut_idx[s] : 0ull) * (uint64_t)(K1 * N);

  // acc_v = LUT_v * X^{-ms(b)}: lane t holds coefficients t + 64 m
  uint64_t A[16];
  {
    const uint32_t bt = active ? modswitch(lwe[n], LOG2_2N) : 0u;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const uint32_t src = (uint32_t)(lane + 64 * m + bt) & (2 * N - 1);
      const uint64_t val = active && owner ? lut[v * N + (src & (N - 1))] : 0ull;
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
      for (int m = 0; m < 16; ++m) xch64[lane + 64 * m] = A[m];
      wave_lds_fence();
      uint64_t rv[16];
#pragma unroll
      for (int m = 0; m < 16; ++m) rv[m] = xch64[(uint32_t)(lane + 64 * m - (int)at) & (N - 1)];
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const uint32_t sp = (uint32_t)(lane + 64 * m - (int)at) & (2 * N - 1);
        st[m] = decomp_init((sp < N ? rv[m] : 0ull - rv[m]) - A[m], nrep);
      }
      wave_lds_fence();
    }

    cplx Y[LIMBS][K1][MS];
#pragma unroll
    for (int li = 0; li < LIMBS; ++li)
#pragma unroll
      for (int cc = 0; cc < K1; ++cc)
#pragma unroll
        for (int jj = 0; jj < MS; ++jj) Y[li][cc][jj] = {0.0, 0.0};
#pragma unroll 1
    for (uint32_t q = 0; q < level; ++q) {
      // ---- level q: the owners' digit polynomials and forward transforms, published by the
      //      level's first key-window barrier (every wave read the previous level's spectra right
      //      after that level's first barrier, 11 windows ago)
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
        for (int k2 = 0; k2 < 8; ++k2) xch[k2 * 64 + lane] = vv[k2];
      }
      cplx X[K1][MS];
#pragma unroll
      for (int wi = 0; wi < WPL; ++wi) {
        const int li = wi / K1, cc = wi % K1;
        const uint32_t r = q * (uint32_t)WPL + (uint32_t)wi;
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
          for (int row = 0; row < K1; ++row)
#pragma unroll
            for (int jj = 0; jj < MS; ++jj) X[row][jj] = myslot[row * XS + jj * 64];
        }
        const cplx* G = ring + (wi % RS) * GROUP + 2 * role * 64 + lane;
#pragma unroll
        for (int row = 0; row < K1; ++row) {
#pragma unroll
          for (int jj = 0; jj < MS; ++jj) {
            const cplx g = G[row * 512 + jj * 64];
            cplx& y = Y[li][cc][jj];
            y.re = __builtin_fma(X[row][jj].re, g.re, __builtin_fma(-X[row][jj].im, g.im, y.re));
            y.im = __builtin_fma(X[row][jj].re, g.im, __builtin_fma(X[row][jj].im, g.re, y.im));
          }
        }
#pragma unroll
        for (int jj = 0; jj < MS; ++jj) pin(Y[li][cc][jj]);
      }
    }

    // ---- per limb: mail my slots of the three outputs, sync, inverse, barrier ---------------
#pragma unroll
    for (int li = 0; li < LIMBS; ++li) {
#pragma unroll
      for (int cc = 0; cc < K1; ++cc)
#pragma unroll
        for (int jj = 0; jj < MS; ++jj) myslot[cc * XS + jj * 64] = Y[li][cc][jj];
      if (owner) {
        k2q_sync(tflags, ctl, role, tcnt, guard);
        cplx V[8];
#pragma unroll
        for (int k2 = 0; k2 < 8; ++k2) V[k2] = xch[k2 * 64 + lane];
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
            A[m] += (uint64_t)__double_as_longlong(tr) - K2_MAGIC_ALL;
            A[m + 8] += (uint64_t)__double_as_longlong(ti) - K2_MAGIC_ALL;
          } else {
            A[m] += (uint64_t)__double_as_longlong(tr) << (16 * li);
            A[m + 8] += (uint64_t)__double_as_longlong(ti) << (16 * li);
          }
        }
#pragma unroll
        for (int m = 0; m < 16; ++m) pin(A[m]);
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        k2q_signal(tflags, ctl, role, tcnt);
      }
      pair_barrier();  // every owner is done with its scratch
    }
  }

  uint64_t* o = out + (active ? (out_idx ? out_idx[s] : s) : 0) * (uint64_t)(2 * N + 1);
  if (!active || !owner) {
  } else if (v < 2) {
#pragma unroll
    for (int m = 0; m < 16; ++m) xch64[lane + 64 * m] = A[m];
    wave_lds_fence();
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int j = lane + 64 * m;
      const uint64_t val = xch64[(N - j) & (N - 1)];
      o[v * N + j] = j == 0 ? val : 0ull - val;
    }
  } else if (lane == 0) {
    o[2 * N] = A[0];
  }

  if constexpr (RESID) {
    for (int off = 32; off > 0; off >>= 1) max_resid = fmax(max_resid, __shfl_xor(max_resid, off));
    if (lane == 0 && active && resid_out) atomicMax(resid_out, (unsigned long long)__double_as_longlong(max_resid));
  }
}

template <bool RESID>
static int launch_k2_many_t(const PbsArgs& a) {
  const size_t lds = pbs1024k2_many_lds_bytes();
  auto kern = pbs1024k2_many_kernel<RESID>;
  CHIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const uint32_t blocks = (a.num_samples + K2_CTS - 1) / K2_CTS;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(K2_CTS * 256), lds, a.stream, a.out, a.out_idx, a.luts, a.lut_idx,
                     a.in, a.in_idx, reinterpret_cast<const cplx*>(a.fbsk), a.n, a.level, a.base_log,
                     a.num_samples, a.resid, a.guard);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("pbs launch failed: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

int pbs1024k2_launch(const PbsArgs& a) {
  if (!(a.N == 1024 && a.k == 2 && a.limbs == (uint32_t)K2_LIMBS && k2_ok(a.level, a.base_log))) {
    set_error("unsupported PBS parameters: N=%u k=%u level=%u base_log=%u limbs=%u", a.N, a.k, a.level, a.base_log,
              a.limbs);
    return -2;
  }
  if (a.num_samples == 0) return 0;
  if (a.level >= K2_MANY_MIN) return a.resid ? launch_k2_many_t<true>(a) : launch_k2_many_t<false>(a);
  switch (a.level) {
    case 1: return a.resid ? launch_k2_t<true, 1>(a) : launch_k2_t<false, 1>(a);
    default: return a.resid ? launch_k2_t<true, 2>(a) : launch_k2_t<false, 2>(a);
  }
}

}  // namespace chip
