// pbs_generic.hip — batched PBS for the general parameter sets of the concrete optimizer
// (SURVEY.md §8f item 4): GLWE dimension k >= 1 and polynomial sizes N = 256 .. 16384, e.g.
// the v0_last_128 table's 1-2 bit sets (k = 4..6, N = 256), 3 bits (k = 3, N = 512), 4 bits
// (k = 2, N = 1024), 6-8 bits (k = 1, N = 4096 .. 16384; 8 bits: n = 1006, l = 2, logB = 15).
//
// Same semantics as pbs.hip / pbs2048.hip (concrete-cpu c_api/bootstrap.rs:347-414 -> tfhe 0.10
// blind_rotate_assign + sample extract; oracle/tfhe_oracle.c:ora_pbs) and the same exactness
// recipe: every digit x key product over Z_{2^64}[X]/(X^N+1) is evaluated as
// exact integer convolutions with an f64 negacyclic FFT (M = N/2 complex points, folded
// x_j + i x_{j+M}, twisted by zeta^j), whose certified rounding error stays below 1/2:
//   * the key polynomial g is split into L balanced limbs of b bits, g = sum_j 2^{jb} g_j;
//   * a decomposition digit wider than b bits is split into T balanced b-bit sub-digits,
//     d = sum_t 2^{tb} s_t, so the product s_t * g_j lands on "slot" m = j + t: the slot sums
//     Y_m = sum_t S_t * G_{m-t} are inverse-transformed once per slot (L per output
//     polynomial; slots >= L vanish mod 2^64) and recombined as sum_m 2^{mb} round(y_m).
//   b depends on (k, N, l) only, so the key format is fixed at conversion time (the runtime's
//   conversion call carries no base_log); the PBS gate checks the bound for the actual logB.
//
// A GLWE accumulator at these sizes (up to 256 KB) does not fit a CU's LDS next to its
// transforms, so the blind rotation runs as two batched launches per CMUX step:
//   gen_mac_kernel   Y[ct][c][m] = sum_{r,q,t} X[ct][r][q][t] * G_i[c][m-t][r][q]   (each key
//                    value read once per 16-ciphertext tile: HBM-bound on the X/Y spectra)
//   gen_step_kernel  per (ciphertext, polynomial): inverse transforms of the L slots, exact
//                    recombination into the accumulator, then the next step's rotation
//                    X^{a_{i+1}} acc - acc, decomposition and forward transforms -> X.
// Transforms are radix-8 Stockham FFTs in LDS (one polynomial per wave group of a workgroup).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <map>
#include <mutex>
#include <vector>

#include "common.hpp"
#include "fft512.hpp"
#include "kernel_util.hpp"
#include "keycheck.hpp"
#include "pbs.hpp"
#include "companion.hpp"

// Streaming (non-temporal) accesses of the per-call spectra and accumulators, which cross HBM once
// per CMUX step and are not re-read from L2 (round 6, A/B in DESIGN.md §4.5): GEN_NT_STORES 2 = every
// X / Y / H / accumulator store of the two-launch and split paths (1: X and Y of the two-launch path
// only); GEN_NT_LOADS 1 = the two-launch path's X and Y loads (the split path's measured slower)
#ifndef GEN_NT_STORES
#define GEN_NT_STORES 2
#endif
#ifndef GEN_NT_LOADS
#define GEN_NT_LOADS 1
#endif
#ifndef MAC_CTS
#define MAC_CTS 16  // ciphertexts per block (key values loaded once per tile)
#endif

namespace chip {

// abi.hip: raise the device's default memory-pool release threshold once, so stream-ordered
// scratch freed by one call stays pooled for the next (each keyswitch call at cfg2 otherwise paid
// ~0.1 ms of allocation).
void keep_pool_memory();

// ------------------------------------------------------------------------------------------
// key format and exactness gate (host)
// ------------------------------------------------------------------------------------------

// Rounding bound of one slot of the product (oracle ora_fft_error_bound): R
// products of a digit polynomial (||d||_2 <= sqrt(N) 2^(dbits-1)) with a key limb spectrum
// (|G| <= maxG) through a forward transform, the pointwise product and an inverse transform
// (Higham, Accuracy and Stability, Thm 24.2, twiddle error mu = 5u for the two-level twiddle
// tables; gamma doubled for the radix-8/4 schedule), plus the
// f64 key transform (||dG||_2 <= gamma ||g||_2, ||g||_2 <= sqrt(N) 2^(b-1)) and the final
// rounding of the largest output.  maxG <= 0 selects the random-key estimate
// 8 sqrt(M) 2^(b-1) sqrt(2) used by the gate; tests certify each key with its measured maxG
// (oracle/pyoracle.py:generic_error_bound).
double generic_error_bound(uint32_t k, uint32_t N, uint32_t level, uint32_t base_log, uint32_t bits,
                           double maxG) {
  const double u = std::ldexp(1.0, -53);
  const double M = N / 2.0;
  const double logM = std::log2(M);
  // twiddles are products of two correctly rounded table entries: |error| <= mu = 5u
  const double mu = 5.0 * u;
  const double eta = mu + 4.0 * u / (1.0 - 4.0 * u) * (std::sqrt(2.0) + mu);
  const double gamma = 2.0 * logM * eta / (1.0 - 2.0 * logM * eta);
  const uint32_t T = (base_log + bits - 1) / bits;
  const uint32_t dbits = base_log < bits ? base_log : bits;
  const double R = (double)(k + 1) * level * T;
  const double dnorm = std::sqrt((double)N) * std::ldexp(1.0, (int)dbits - 1);
  const double gnorm = std::sqrt((double)N) * std::ldexp(1.0, (int)bits - 1);
  if (maxG <= 0.0) maxG = 8.0 * std::sqrt(M) * std::ldexp(1.0, (int)bits - 1) * std::sqrt(2.0);
  const double max_out = R * (double)N * std::ldexp(1.0, (int)dbits - 1) * std::ldexp(1.0, (int)bits - 1);
  return R * dnorm * (maxG * (4.0 * gamma + 3.0 * u) + gamma * gnorm) * 1.0001 + 4.0 * u * max_out;
}

// Levels up to 64 (l logB <= 64: the optimizer's rows reach l = 44 at logB = 1, v0_last_128).
static bool generic_shape_ok(uint32_t k, uint32_t N, uint32_t level) {
  if (k < 1 || k > (uint32_t)GEN_MAX_K || level < 1 || level > 64) return false;
  return N >= 256 && N <= 65536 && (N & (N - 1)) == 0;
}

// Limb width b for (k, N, l): the widest b whose bound holds for digits of up to 2b bits
// (T <= 2 sub-digits), which covers every logB the optimizer pairs with these sizes; a digit is
// never wider than 64 / l bits (l logB <= 64), so many-level keys get wider limbs.
uint32_t generic_limb_bits(uint32_t k, uint32_t N, uint32_t level) {
  for (uint32_t b = 24; b >= 8; --b)
    if (generic_error_bound(k, N, level, std::min<uint32_t>(2 * b, 64 / level), b, 0.0) < 0.25) return b;
  return 0;
}

KeyFormat generic_key_format(uint32_t k, uint32_t N, uint32_t level) {
  if (generic_shape_ok(k, N, level)) {
    const uint32_t b = generic_limb_bits(k, N, level);
    const uint32_t L = b ? (64 + b - 1) / b : 0;
    if (b && L <= (uint32_t)GEN_MAX_LIMBS) return {KeyKind::GENERIC, L, b};
  }
  return {KeyKind::NONE, 0, 0};
}

KeyFormat key_format(uint32_t k, uint32_t N, uint32_t level) {
  if (k == 1 && N == 1024 && level >= 1 && level <= 3) return {KeyKind::N1024, 3, 22};
  if (k == 1 && N == 2048 && level >= 1 && level <= PBS2_MAX_LEVEL) return {KeyKind::N2048, (uint32_t)PBS2_LIMBS, 16};
  if (k == 2 && N == 1024 && level >= 1 && level <= 64) return {KeyKind::K2N1024, (uint32_t)K2_LIMBS, 16};
  if (pbs_small_shape(k, N, level))
    return {KeyKind::SMALL, small_limbs(k, N, level), small_limbs(k, N, level) == K4_L2_LIMBS ? 13u : 16u};
  return generic_key_format(k, N, level);
}

// The general path's own gate, for its key format (also for the shapes whose primary key is a
// hand-tuned kernel's: their wide-digit PBS runs here on a companion key, pbs_needs_generic_key).
bool generic_pbs_ok(uint32_t k, uint32_t N, uint32_t level, uint32_t base_log) {
  const KeyFormat f = generic_key_format(k, N, level);
  if (f.kind != KeyKind::GENERIC || base_log < 1 || (uint64_t)level * base_log > 64) return false;
  // any number of product terms (k + 1) l T: the register-tiled products cover the optimizer's
  // log-norm2-0 shapes, gen_mac_kernel the rest in chunks of GEN_MAX_TERMS
  return generic_error_bound(k, N, level, base_log, f.bits, 0.0) < 0.25;
}

static hipStream_t side_stream(int idx);  // a library stream per device (defined below)

namespace gen {

// a spectrum value read once (the previous launch's X / Y): streaming load under GEN_NT_LOADS
__device__ __forceinline__ cplx ld_once(const cplx* p) {
#if GEN_NT_LOADS
  return {__builtin_nontemporal_load(&p->re), __builtin_nontemporal_load(&p->im)};
#else
  return *p;
#endif
}


// ------------------------------------------------------------------------------------------
// block FFT (LDS, in place, radix-8 Stockham passes after one radix-2/4 pass; radix-4 for M <= 256)
// ------------------------------------------------------------------------------------------
template <int M>
struct Geo {
  static constexpr int THREADS = M >= 512 ? M / 8 : (M >= 256 ? 64 : M / 4);  // per polynomial
  static constexpr int VPT = M / THREADS;                  // complex values per thread
  static constexpr int PPB = THREADS >= 256 ? 1 : 256 / THREADS;  // polynomials per workgroup
  static constexpr int BLOCK = THREADS * PPB;
  static constexpr int LOG = M == 128 ? 7 : M == 256 ? 8 : M == 512 ? 9 : M == 1024 ? 10 : M == 2048 ? 11
                           : M == 4096 ? 12 : 13;
  static_assert((1 << LOG) == M, "M");
  static_assert(VPT % 4 == 0, "values per thread");
};

// Synchronisation of one polynomial's threads around its LDS passes: a polynomial of up to 64
// threads lives in one wave, whose LDS operations execute in issue order, so only the compiler
// has to be fenced; larger polynomials span waves and take a workgroup barrier.
template <int M>
__device__ __forceinline__ void poly_sync() {
  if constexpr (Geo<M>::THREADS <= 64) wave_lds_fence();
  else __syncthreads();
}

// Twiddle e^{-+2 pi i idx/M} from LDS: the full correctly rounded table for M <= FULL_TW_MAX,
// else two tables, W[j] = Wlo[j mod TW_LO] * Whi[j / TW_LO] (error <= 5u: the bound's mu).
constexpr int TW_LO = 128;
constexpr int FULL_TW_MAX = 2048;
template <int M>
constexpr int tw_entries() {
  return M <= FULL_TW_MAX ? M : TW_LO + (M / TW_LO > 1 ? M / TW_LO : 1);
}
template <int M, bool INV>
__device__ __forceinline__ cplx twiddle(const cplx* W, int idx) {
  cplx w;
  if constexpr (M <= FULL_TW_MAX) w = W[idx];
  else w = cmul(W[idx & (TW_LO - 1)], W[TW_LO + (idx >> 7)]);
  return INV ? cplx{w.re, -w.im} : w;
}
static_assert(TW_LO == 128, "twiddle split");

// stage the twiddle table(s) of size M into LDS (tw_entries<M>() entries)
template <int M>
__device__ __forceinline__ void load_twiddles(cplx* tw, const cplx* Wfull, const cplx* Wlo, const cplx* Whi, int t,
                                              int nt) {
  if constexpr (M <= FULL_TW_MAX) {
    for (int e = t; e < M; e += nt) tw[e] = Wfull[e];
  } else {
    constexpr int NHI = M / TW_LO > 1 ? M / TW_LO : 1;
    for (int e = t; e < TW_LO + NHI; e += nt) tw[e] = e < TW_LO ? Wlo[e] : Whi[e - TW_LO];
  }
}

// LDS slot of complex element i: bits 1-3 XOR bits 4-6, so the strided writes of the first
// Stockham passes (stride 8, 16, 32 elements) and the contiguous reads hit 8 distinct 16-byte
// bank groups per 8-lane group (gfx950 ds_write_b128/ds_read_b128 lane groups).
__device__ __forceinline__ int sw(int i) { return i ^ (((i >> 4) & 7) << 1); }

// One Stockham pass of radix R at stride Ns (natural order in, natural order out).  Every
// thread reads all its inputs before the barrier and writes after it, so the pass is in place.
template <int M, int R, bool INV>
__device__ __forceinline__ void stockham_pass(cplx* buf, const cplx* W, int tid, int Ns) {
  constexpr int TH = Geo<M>::THREADS;
  constexpr int NB = M / R / TH;  // butterflies per thread
  static_assert(NB >= 1 && (M / R) % TH == 0, "pass split");
  cplx v[NB][R];
#pragma unroll
  for (int s = 0; s < NB; ++s) {
    const int j = tid + s * TH;
#pragma unroll
    for (int r = 0; r < R; ++r) v[s][r] = buf[sw(j + r * (M / R))];
  }
  poly_sync<M>();
#pragma unroll
  for (int s = 0; s < NB; ++s) {
    const int j = tid + s * TH;
    const int kk = j & (Ns - 1);
    const int step = M / (Ns * R);
#pragma unroll
    for (int r = 1; r < R; ++r) v[s][r] = cmul(v[s][r], twiddle<M, INV>(W, kk * r * step));
    if constexpr (R == 2) {
      const cplx x0 = v[s][0], x1 = v[s][1];
      v[s][0] = cadd(x0, x1);
      v[s][1] = csub(x0, x1);
    } else if constexpr (R == 4) {
      const cplx t0 = cadd(v[s][0], v[s][2]), t1 = csub(v[s][0], v[s][2]);
      const cplx t2 = cadd(v[s][1], v[s][3]), t3 = mul_mi<INV>(csub(v[s][1], v[s][3]));
      v[s][0] = cadd(t0, t2);
      v[s][2] = csub(t0, t2);
      v[s][1] = cadd(t1, t3);
      v[s][3] = csub(t1, t3);
    } else {
      dft8<INV>(v[s]);
    }
    const int d = (j - kk) * R + kk;
#pragma unroll
    for (int r = 0; r < R; ++r) buf[sw(d + r * Ns)] = v[s][r];
  }
  poly_sync<M>();
}

// Unnormalised DFT of buf (M complex, natural order) in place: forward e^{-2 pi i jk/M},
// inverse e^{+2 pi i jk/M}; W[j] = e^{-2 pi i j/M}.  Callers synchronise before the call.
template <int M, bool INV>
__device__ __forceinline__ void fft_block(cplx* buf, const cplx* W, int tid) {
  constexpr int LOG = Geo<M>::LOG;
  if constexpr (Geo<M>::VPT >= 8) {
    // radix-8 passes (three 8-point stages in registers per LDS round trip), the leftover
    // factor 2 or 4 first (its stride-1 pass needs no twiddles)
    int Ns = 1;
    if constexpr (LOG % 3 == 1) {
      stockham_pass<M, 2, INV>(buf, W, tid, Ns);
      Ns = 2;
    } else if constexpr (LOG % 3 == 2) {
      stockham_pass<M, 4, INV>(buf, W, tid, Ns);
      Ns = 4;
    }
#pragma unroll 1
    for (; Ns < M; Ns *= 8) stockham_pass<M, 8, INV>(buf, W, tid, Ns);
  } else {
    int Ns = 1;
    if constexpr (LOG & 1) {
      stockham_pass<M, 2, INV>(buf, W, tid, Ns);
      Ns = 2;
    }
#pragma unroll 1
    for (; Ns < M; Ns *= 4) stockham_pass<M, 4, INV>(buf, W, tid, Ns);
  }
}

// Tile transforms (M <= 256, radix-4 Stockham as fft_block) with each pass's twiddles laid out
// per pass, TWP[off(Ns) + kk (R-1) + r - 1] = W[kk r M / (Ns R)] (copies of the correctly rounded
// table, so the bound is unchanged): the lanes of a ds_read_b128 group read consecutive kk at a
// 48-byte stride instead of the full table's 2-8-way conflicted strides, and the first pass
// (all twiddles 1) multiplies by nothing.
// threads per polynomial in the tile kernels: the step kernel's for M <= 256, 128 (two waves,
// four values each) at M = 512
#ifndef TILE128_CP
#define TILE128_CP 2
#endif
#ifndef TILE_GROUPS
#define TILE_GROUPS 1
#endif
#ifndef TILE512_TH
#define TILE512_TH 128
#endif
template <int M>
constexpr int tile_threads() { return M == 512 ? TILE512_TH : Geo<M>::THREADS; }
template <int TH>
__device__ __forceinline__ void tile_sync() {
  if constexpr (TH <= 64) wave_lds_fence();
  else __syncthreads();  // every polynomial of the tile transforms in lockstep
}

// radix of the tile transforms' passes (values per thread) and of the first pass (the leftover
// factor, or a full pass: its twiddles are all 1)
template <int M, int TH>
constexpr int tile_radix() { return M / TH; }
template <int M, int TH>
constexpr int tile_first_radix() {
  constexpr int LR = tile_radix<M, TH>() == 8 ? 3 : 2, REM = Geo<M>::LOG % LR;
  return REM ? (1 << REM) : tile_radix<M, TH>();
}
template <int M, int TH>
constexpr int tile_tw_entries() {
  int n = 0;
  for (int Ns = tile_first_radix<M, TH>(); Ns < M; Ns *= tile_radix<M, TH>()) n += (tile_radix<M, TH>() - 1) * Ns;
  return n;
}

template <int M, int TH>
__device__ __forceinline__ void build_tile_tw(cplx* TWP, const cplx* W, int t, int nt) {
  constexpr int R = tile_radix<M, TH>();
  int off = 0;
  for (int Ns = tile_first_radix<M, TH>(); Ns < M; Ns *= R) {
    const int step = M / (Ns * R);
    for (int e = t; e < (R - 1) * Ns; e += nt) TWP[off + e] = W[(e / (R - 1)) * (e % (R - 1) + 1) * step];
    off += (R - 1) * Ns;
  }
}

template <int M, int TH, int R, bool INV, bool FIRST>
__device__ __forceinline__ void tile_pass(cplx* buf, const cplx* TW, int tid, int Ns) {
  constexpr int NB = M / R / TH;
  static_assert(NB >= 1 && (M / R) % TH == 0, "pass split");
  cplx v[NB][R];
#pragma unroll
  for (int s = 0; s < NB; ++s) {
    const int j = tid + s * TH;
#pragma unroll
    for (int r = 0; r < R; ++r) v[s][r] = buf[sw(j + r * (M / R))];
  }
  tile_sync<TH>();
#pragma unroll
  for (int s = 0; s < NB; ++s) {
    const int j = tid + s * TH;
    const int kk = FIRST ? 0 : (j & (Ns - 1));
    if constexpr (!FIRST) {
#pragma unroll
      for (int r = 1; r < R; ++r) {
        const cplx w = TW[kk * (R - 1) + r - 1];
        v[s][r] = INV ? cmulc(v[s][r], w) : cmul(v[s][r], w);
      }
    }
    if constexpr (R == 2) {
      const cplx x0 = v[s][0], x1 = v[s][1];
      v[s][0] = cadd(x0, x1);
      v[s][1] = csub(x0, x1);
    } else if constexpr (R == 4) {
      const cplx t0 = cadd(v[s][0], v[s][2]), t1 = csub(v[s][0], v[s][2]);
      const cplx t2 = cadd(v[s][1], v[s][3]), t3 = mul_mi<INV>(csub(v[s][1], v[s][3]));
      v[s][0] = cadd(t0, t2);
      v[s][2] = csub(t0, t2);
      v[s][1] = cadd(t1, t3);
      v[s][3] = csub(t1, t3);
    } else {
      dft8<INV>(v[s]);
    }
    const int d = (j - kk) * R + kk;
#pragma unroll
    for (int r = 0; r < R; ++r) buf[sw(d + r * Ns)] = v[s][r];
  }
  tile_sync<TH>();
}

template <int M, int TH, bool INV>
__device__ __forceinline__ void tile_fft(cplx* buf, const cplx* TWP, int tid) {
  constexpr int R = tile_radix<M, TH>(), R0 = tile_first_radix<M, TH>();
  static_assert(R == 4 || R == 8, "tile radix");
  tile_pass<M, TH, R0, INV, true>(buf, nullptr, tid, 1);
  int off = 0;
#pragma unroll 1
  for (int Ns = R0; Ns < M; Ns *= R) {
    tile_pass<M, TH, R, INV, false>(buf, TWP + off, tid, Ns);
    off += (R - 1) * Ns;
  }
}

// tfhe SignedDecomposer::decompose_one_level on a 64-bit state (digits up to 64 bits)
__device__ __forceinline__ int64_t decomp_next64(uint64_t& state, int logB) {
  const uint64_t mask = logB >= 64 ? ~0ull : (1ull << logB) - 1ull;
  const uint64_t res = state & mask;
  state = logB >= 64 ? 0ull : state >> logB;
  const uint64_t carry = (((res - 1ull) | state) & res) >> (logB - 1);
  state += carry;
  return (int64_t)(res - (logB >= 64 ? 0ull : carry << logB));
}

// ------------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------------
struct StepArgs {
  uint64_t* acc;       // [chunk][K1][N] accumulators
  cplx* X;             // [chunk][K1 r][l q][T t][M] digit spectra
  const cplx* Y;       // [chunk][K1 c][L m][M] slot spectra
  const cplx* Wfull;   // e^{-2 pi i j/M}, j < M
  const cplx* Wlo;     // e^{-2 pi i j/M}, j < TW_LO
  const cplx* Whi;     // e^{-2 pi i j TW_LO/M}
  const cplx* Z;       // zeta^j = e^{i pi j/N}
  const uint64_t* in;  // LWE inputs (rows of n+1)
  const uint64_t* in_idx;
  const uint64_t* luts;
  const uint64_t* lut_idx;
  unsigned long long* resid;
  uint32_t base;   // first sample of the chunk
  uint32_t count;  // samples in the chunk
  uint32_t n, k, level, base_log, bits, limbs, subs;
  uint32_t step;     // FRONT: the mask position whose rotation is prepared
  const cplx* Tau;   // four-step column twiddles [R][512] + row/slot factors [R][8] (gen_big_step_kernel)
};

enum { MODE_INIT = 1, MODE_BACK = 2, MODE_FRONT = 4 };

template <int M, int MODE>
__global__ void __launch_bounds__(Geo<M>::BLOCK) gen_step_kernel(StepArgs a) {
  constexpr int N = 2 * M, TH = Geo<M>::THREADS, VPT = Geo<M>::VPT, LOG2_2N = Geo<M>::LOG + 2;
  constexpr int PPB = Geo<M>::PPB;
  // ZLDS: the twist table in LDS next to the twiddles; YDMA: the slot spectra of the inverse
  // transforms double-buffered by LDS-DMA (slot m + 1 lands while slot m is transformed)
  constexpr bool ZLDS = M <= 1024;
  constexpr bool YDMA = TH >= 64 && M <= 512;
  constexpr int NBUF = YDMA ? 2 : 1;
  // PP: per-pass twiddle tables (tile_fft; they do not fit next to an M = 8192 polynomial,
  // which keeps the two-level table of fft_block)
  constexpr bool PP = M <= 4096;
  constexpr int TWN = PP ? tile_tw_entries<M, TH>() : tw_entries<M>();
  __shared__ cplx lds[NBUF * PPB * M + TWN + (ZLDS ? M : 0)];
  cplx* W = lds + NBUF * PPB * M;
  if constexpr (PP)
    build_tile_tw<M, TH>(W, a.Wfull, threadIdx.x, Geo<M>::BLOCK);
  else
    load_twiddles<M>(W, a.Wfull, a.Wlo, a.Whi, threadIdx.x, Geo<M>::BLOCK);
  cplx* Zl = W + TWN;
  if constexpr (ZLDS)
    for (int e = threadIdx.x; e < M; e += Geo<M>::BLOCK) Zl[e] = a.Z[e];
  auto zeta = [&](int j) { return ZLDS ? Zl[j] : a.Z[j]; };
  __syncthreads();
  // polynomial group g of this workgroup: (ciphertext, GLWE polynomial) = divmod(poly, k + 1).
  // Groups past the batch keep taking part in the workgroup barriers of the transforms.
  const int g = threadIdx.x / TH, tid = threadIdx.x % TH;
  auto fwd = [&](cplx* b) {
    if constexpr (PP) tile_fft<M, TH, false>(b, W, tid);
    else fft_block<M, false>(b, W, tid);
  };
  cplx* buf = lds + g * NBUF * M;
  const uint32_t K1 = a.k + 1;
  const uint64_t poly = (uint64_t)blockIdx.x * PPB + g;
  const bool live = poly < (uint64_t)a.count * K1;
  const uint32_t ct = live ? (uint32_t)(poly / K1) : 0u, c = (uint32_t)(poly % K1);
  const uint32_t s = a.base + ct;
  const uint64_t row = live ? (a.in_idx ? a.in_idx[s] : s) : 0ull;
  const uint64_t* lwe = a.in + row * (uint64_t)(a.n + 1);
  uint64_t* acc = a.acc + ((uint64_t)ct * K1 + c) * N;
  // this thread's coefficients: j = tid + e TH (e < VPT) and j + M (element e + VPT)
  auto coef = [&](int e) { return (uint32_t)(tid + (e % VPT) * TH + (e / VPT) * M); };
  uint64_t A[2 * VPT];
  double max_resid = 0.0;

  if constexpr ((MODE & MODE_INIT) != 0) {
    // acc_c = LUT_c * X^{-ms(b)} (blind_rotate_assign: polynomial_wrapping_monic_monomial_div)
    const uint64_t* lut =
        a.luts + (live && a.lut_idx ? a.lut_idx[s] : 0ull) * (uint64_t)(K1 * N) + (uint64_t)c * N;
    const uint32_t bt = live ? modswitch(lwe[a.n], LOG2_2N) : 0u;
#pragma unroll
    for (int e = 0; e < 2 * VPT; ++e) {
      const uint32_t src = (coef(e) + bt) & (2 * N - 1);
      const uint64_t v = live ? lut[src & (N - 1)] : 0ull;
      A[e] = src < (uint32_t)N ? v : 0ull - v;
    }
  } else {
#pragma unroll
    for (int e = 0; e < 2 * VPT; ++e) A[e] = live ? acc[coef(e)] : 0ull;
  }

  if constexpr ((MODE & MODE_BACK) != 0) {
    // acc_c += sum_m 2^{m b} round(iFFT(Y_m) conj(zeta^j)); the key spectra carry the 1/M.
    // bits(v + MAGIC) - MAGIC_BITS = round(v) mod 2^64 for |v| < 2^51 (either sign).
    const cplx* Yc = a.Y + ((uint64_t)ct * K1 + c) * a.limbs * (uint64_t)M;
    // YDMA: wave-linear LDS destination, swizzle applied on the source side (slot p holds
    // element sw(p)); a group past the batch loads ciphertext 0's rows (in bounds, unused)
    auto issue_y = [&](uint32_t m, cplx* dst) {
      const cplx* Ym = Yc + (uint64_t)m * M;
      const int w0 = tid & ~63, ln = tid & 63;
#pragma unroll
      for (int e = 0; e < VPT; ++e) {
        const int L0 = w0 + e * TH;
        __builtin_amdgcn_global_load_lds(Ym + sw(L0 + ln), (lds_ptr_t)(dst + L0), 16, 0, 0);
      }
    };
    // PREF (up to M = 4096; M = 8192 has no registers to spare): slot m + 1 is loaded into
    // registers while slot m is transformed
    constexpr bool PREF = !YDMA && M <= 4096;
    cplx nx[PREF ? VPT : 1];
    if constexpr (YDMA) {
      issue_y(0, buf);
    } else if constexpr (PREF) {
#pragma unroll
      for (int e = 0; e < VPT; ++e) nx[e] = live ? Yc[tid + e * TH] : cplx{0.0, 0.0};
    }
#pragma unroll 1
    for (uint32_t m = 0; m < a.limbs; ++m) {
      cplx* cur = buf;
      if constexpr (YDMA) {
        cur = buf + (m & 1) * M;
        wait_vmcnt<0>();
        poly_sync<M>();
        if (m + 1 < a.limbs) issue_y(m + 1, buf + ((m + 1) & 1) * M);
      } else if constexpr (PREF) {
#pragma unroll
        for (int e = 0; e < VPT; ++e) cur[sw(tid + e * TH)] = nx[e];
        if (m + 1 < a.limbs) {
          const cplx* Yn = Yc + (uint64_t)(m + 1) * M;
#pragma unroll
          for (int e = 0; e < VPT; ++e) nx[e] = live ? Yn[tid + e * TH] : cplx{0.0, 0.0};
        }
        poly_sync<M>();
      } else {
        const cplx* Ym = Yc + (uint64_t)m * M;
#pragma unroll
        for (int e = 0; e < VPT; ++e) cur[sw(tid + e * TH)] = live ? Ym[tid + e * TH] : cplx{0.0, 0.0};
        poly_sync<M>();
      }
      if constexpr (PP)
        tile_fft<M, TH, true>(cur, W, tid);
      else
        fft_block<M, true>(cur, W, tid);
      const uint32_t sh = m * a.bits;
#pragma unroll
      for (int e = 0; e < VPT; ++e) {
        const int j = tid + e * TH;
        const cplx z = cmulc(cur[sw(j)], zeta(j));
        const double tr = z.re + RND_MAGIC, ti = z.im + RND_MAGIC;
        max_resid = fmax(max_resid, fmax(fabs(z.re - (tr - RND_MAGIC)), fabs(z.im - (ti - RND_MAGIC))));
        if (sh < 64) {
          A[e] += ((uint64_t)__double_as_longlong(tr) - RND_MAGIC_BITS) << sh;
          A[e + VPT] += ((uint64_t)__double_as_longlong(ti) - RND_MAGIC_BITS) << sh;
        }
      }
      poly_sync<M>();
    }
  }

  if constexpr ((MODE & (MODE_BACK | MODE_INIT)) != 0) {
    if (live)
#pragma unroll
      for (int e = 0; e < 2 * VPT; ++e) acc[coef(e)] = A[e];
  }

  if constexpr ((MODE & MODE_FRONT) != 0) {
    // ct1 = X^{ms(a_i)} acc - acc; balanced decomposition; b-bit sub-digits; forward transforms
    const uint32_t at = live ? modswitch(lwe[a.step], LOG2_2N) : 0u;
    uint64_t* accl = reinterpret_cast<uint64_t*>(buf);
#pragma unroll
    for (int e = 0; e < 2 * VPT; ++e) accl[coef(e)] = A[e];
    poly_sync<M>();
    const int nrep = 64 - (int)(a.level * a.base_log);
#pragma unroll
    for (int e = 0; e < 2 * VPT; ++e) {
      const uint32_t src = (coef(e) - at) & (2 * N - 1);
      const uint64_t rv = accl[src & (N - 1)];
      const uint64_t x = (src < (uint32_t)N ? rv : 0ull - rv) - A[e];
      A[e] = nrep > 0 ? decomp_init(x, nrep) : x;  // decomposer state (reuses A)
    }
    poly_sync<M>();
    cplx* Xc = a.X + ((uint64_t)ct * K1 + c) * a.level * a.subs * (uint64_t)M;
    const int logB = (int)a.base_log;
    const int sb = (int)a.bits;
    const uint64_t half = 1ull << (sb - 1);
    const uint64_t bmask = (1ull << sb) - 1ull;
    // STAGE (large M): the twisted sub-digit inputs of all l T transforms go to their X slots
    // first, so no decomposition state is live across the transforms (no register spills at
    // 1024 threads); each slot is then transformed in place through LDS.
    constexpr bool STAGE = M >= 8192;
#pragma unroll 1
    for (uint32_t q = 0; q < a.level; ++q) {
      int64_t D[2 * VPT];
#pragma unroll
      for (int e = 0; e < 2 * VPT; ++e) D[e] = decomp_next64(A[e], logB);
#pragma unroll 1
      for (uint32_t t = 0; t < a.subs; ++t) {
        cplx* dst = Xc + ((uint64_t)q * a.subs + t) * M;
#pragma unroll
        for (int e = 0; e < VPT; ++e) {
          int64_t s0 = D[e], s1 = D[e + VPT];
          if (a.subs > 1) {  // balanced b-bit sub-digit, exact: D - s is a multiple of 2^b
            s0 = (int64_t)(((uint64_t)D[e] + half) & bmask) - (int64_t)half;
            s1 = (int64_t)(((uint64_t)D[e + VPT] + half) & bmask) - (int64_t)half;
            D[e] = (D[e] - s0) >> sb;
            D[e + VPT] = (D[e + VPT] - s1) >> sb;
          }
          const int j = tid + e * TH;
          const cplx z = cmul(cplx{(double)s0, (double)s1}, zeta(j));
          if constexpr (STAGE) {
            if (live) dst[j] = z;
          } else {
            buf[sw(j)] = z;
          }
        }
        if constexpr (!STAGE) {
          poly_sync<M>();
          fwd(buf);
          if (live)
#pragma unroll
            for (int e = 0; e < VPT; ++e) dst[tid + e * TH] = buf[sw(tid + e * TH)];
          poly_sync<M>();
        }
      }
    }
    if constexpr (STAGE) {
#pragma unroll 1
      for (uint32_t x = 0; x < a.level * a.subs; ++x) {
        cplx* dst = Xc + (uint64_t)x * M;
#pragma unroll
        for (int e = 0; e < VPT; ++e) buf[sw(tid + e * TH)] = live ? dst[tid + e * TH] : cplx{0.0, 0.0};
        poly_sync<M>();
        fwd(buf);
        if (live)
#pragma unroll
          for (int e = 0; e < VPT; ++e) dst[tid + e * TH] = buf[sw(tid + e * TH)];
        poly_sync<M>();
      }
    }
  }

  if constexpr ((MODE & MODE_BACK) != 0) {
    if (a.resid) {
      for (int off = 32; off > 0; off >>= 1) max_resid = fmax(max_resid, __shfl_xor(max_resid, off));
      if ((threadIdx.x & 63) == 0) atomicMax(a.resid, (unsigned long long)__double_as_longlong(max_resid));
    }
  }
}

// ------------------------------------------------------------------------------------------
// N >= 2048: four-step step kernel.  The M-point transform (M = R x 512) splits into R rows of
// 512 points (row j1 = the coefficients n = j1 + R J, J < 1024, folded as J and J + 512) done by
// the one-wave fft512 transforms (fft512.hpp) in registers, and 512 R-point column DFTs across
// the rows, one LDS exchange apart: with j = j1 + R j2 and f = k2 + 512 k1,
//   Z_f = sum_j1 w_R^{j1 k1} tau(j1, k2) FFT512_j1[k2],  tau(j1, k2) = zeta_N^{j1} w_M^{j1 k2},
// where FFT512_j1 is the row's 512-point transform with its own twist zeta_N^R = exp(i pi / 1024)
// (exactly the twist fft512 folds into its first pass), and the inverse runs the same steps
// backwards with conjugate twiddles.  Each path through the transform still takes log2 M
// butterfly stages and at most log2 M inexact twiddle products (fft512's stages, tau, and at
// most two inexact constants inside an R-point DFT of log2 R stages), each within the mu = 5u of
// the certified bound (tau: one correctly rounded table entry), so generic_error_bound holds
// unchanged; the tests check the measured residual against it.
// Against gen_step_kernel<M> (one polynomial per workgroup through log M / 3 radix-8 LDS passes
// of the whole polynomial, ~10 barriers per transform, digit spectra staged through HBM at
// M = 8192): one LDS round trip of the polynomial and two barriers per transform.
// Data layout: spectra in the order f' = k1 512 + pos (pos = slot 64 + lane of fft512's
// output, frequency k2 = fft512_freq(lane, slot)); the Fourier key is stored in the same order
// (gen_convert_kernel, perm), the product kernels are elementwise and unchanged.  Accumulators
// in row order, acc[j1 1024 + J] (gen_extract_kernel, rlog).
// LDS: R rows of 576 complex (512 + the pad that makes room for a wave's transpose scratch in
// its own first row), the fft512 tables, at R = 16 the column-twiddle slot factors beta: 160 KB
// at M = 8192, one workgroup of 8 waves per CU.
// ------------------------------------------------------------------------------------------
template <int M>
struct Big {
  static constexpr int R = M / 512;
  static constexpr int LOGR = R == 2 ? 1 : R == 4 ? 2 : R == 8 ? 3 : 4;
  static constexpr int NW = R < 8 ? R : 8;  // waves
  static constexpr int SPW = R / NW;        // rows per wave
  static constexpr int NT = 64 * NW;
  static constexpr int CPT = 512 / NT;      // column positions per thread
  static constexpr int RS = 576;            // row stride (complex)
  static constexpr int BIG = R * RS;
  static constexpr int BETA = SPW == 1 ? 0 : R * 8;  // tau slot factors in LDS (rows per wave > 1)
  static constexpr int LDS = (BIG + FFT512_TABLE_ENTRIES + BETA) * 16;
  static_assert((1 << LOGR) == R && R <= 16 && RS >= XCH_SLOTS, "rows");
  static_assert(BIG >= M && LDS <= 160 * 1024, "LDS");
};
constexpr int ROWLEN = 1024;  // coefficients per row (N / R)

// frequency held at spectrum position p of the four-step order
__host__ __device__ constexpr uint32_t big_freq(uint32_t p) {
  return (uint32_t)fft512_freq((int)(p & 63), (int)((p >> 6) & 7)) + 512u * (p >> 9);
}

// R-point DFT across the rows, natural order in and out (forward exp(-2 pi i jk/R), inverse +)
constexpr double C16_1 = 0.92387953251128675613, S16_1 = 0.38268343236508977173;  // cos, sin pi/8
constexpr double R2H = 0.70710678118654752440;
template <int R, bool INV>
__device__ __forceinline__ void dft_col(cplx (&u)[R]) {
  if constexpr (R == 2) {
    const cplx x0 = u[0], x1 = u[1];
    u[0] = cadd(x0, x1);
    u[1] = csub(x0, x1);
  } else if constexpr (R == 4) {
    const cplx t0 = cadd(u[0], u[2]), t1 = csub(u[0], u[2]);
    const cplx t2 = cadd(u[1], u[3]), t3 = mul_mi<INV>(csub(u[1], u[3]));
    u[0] = cadd(t0, t2);
    u[2] = csub(t0, t2);
    u[1] = cadd(t1, t3);
    u[3] = csub(t1, t3);
  } else if constexpr (R == 8) {
    dft8<INV>(u);
  } else {
    static_assert(R == 16, "column radix");
    // even / odd halves, then X[k] = E[k] + w16^k O[k], X[k + 8] = E[k] - w16^k O[k]
    cplx e[8], o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) e[i] = u[2 * i], o[i] = u[2 * i + 1];
    dft8<INV>(e);
    dft8<INV>(o);
    const cplx w16[8] = {{1.0, 0.0},     {C16_1, -S16_1}, {R2H, -R2H},     {S16_1, -C16_1},
                         {0.0, -1.0},    {-S16_1, -C16_1}, {-R2H, -R2H},   {-C16_1, -S16_1}};
#pragma unroll
    for (int k = 1; k < 8; ++k) o[k] = k == 4 ? mul_mi<INV>(o[4]) : INV ? cmulc(o[k], w16[k]) : cmul(o[k], w16[k]);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      u[k] = cadd(e[k], o[k]);
      u[k + 8] = csub(e[k], o[k]);
    }
  }
}

// W32: decomposition state and digits in 32 bits (level * base_log <= 31), else 64
template <int M, int MODE, bool W32>
__global__ void __launch_bounds__(Big<M>::NT) gen_big_step_kernel(StepArgs a) {
  using G = Big<M>;
  constexpr int N = 2 * M, R = G::R, LOGR = G::LOGR, SPW = G::SPW, NT = G::NT, CPT = G::CPT, RS = G::RS;
  constexpr int LOG2_2N = Geo<M>::LOG + 2;
  using St = typename std::conditional<W32, uint32_t, uint64_t>::type;
  using Dg = typename std::conditional<W32, int32_t, int64_t>::type;
  __shared__ cplx lds[G::BIG + FFT512_TABLE_ENTRIES + G::BETA];
  cplx* E = lds;  // rows j1 at E + j1 RS
  build_fft512_tables(lds + G::BIG, threadIdx.x, NT);
  cplx* beta = lds + G::BIG + FFT512_TABLE_ENTRIES;
  for (int x = threadIdx.x; x < G::BETA; x += NT) beta[x] = a.Tau[R * 512 + x];
  const Fft512Tables T = fft512_tables_at(lds + G::BIG);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  cplx* xch = E + w * SPW * RS;  // transpose scratch: the wave's first row and its pad
  const uint32_t K1 = a.k + 1, poly = blockIdx.x, ct = poly / K1, c = poly % K1;
  const uint32_t s = a.base + ct;
  const uint64_t row = a.in_idx ? a.in_idx[s] : s;
  const uint64_t* lwe = a.in + row * (uint64_t)(a.n + 1);
  uint64_t* acc = a.acc + (uint64_t)poly * N;
  // this thread's column positions and rows / coefficients: row jrow(sr), J = jcol(e) (e < 8:
  // the real parts J = lane + 64 e, e >= 8: the imaginary parts J + 512)
  auto pos_of = [&](int p) { return (int)threadIdx.x + p * NT; };
  auto jrow = [&](int sr) { return w * SPW + sr; };
  auto jcol = [&](int e) { return lane + 64 * (e & 7) + 512 * (e >> 3); };
  // column twiddles tau(j1, pos), applied by the row waves (row j1 = jrow(sr), positions
  // e 64 + lane): in registers for SPW = 1.  At R = 16 (16 per thread would not fit next to the
  // accumulator's 32 words) tau(j1, e 64 + lane) = alpha(j1, lane) beta(j1, e), the lane factor
  // alpha = tau(j1, lane) in registers and the slot factor beta(j1, e) = exp(-256 i pi j1 e / N)
  // from LDS (a broadcast read): no global load inside the row phases, whose vmcnt(0) waits would
  // also drain the next slot's prefetched columns.  Both factors are correctly rounded, so the
  // computed twiddle is within 3u of tau (0.5u + 0.5u + 2u for the FMA complex product), inside
  // the mu = 5u the certified bound allows each twiddle.
  constexpr bool TAUREG = SPW == 1;
  cplx tau_r[TAUREG ? 8 : SPW];
  if constexpr (TAUREG) {
#pragma unroll
    for (int e = 0; e < 8; ++e) tau_r[e] = a.Tau[jrow(0) * 512 + e * 64 + lane];
  } else {
#pragma unroll
    for (int sr = 0; sr < SPW; ++sr) tau_r[sr] = a.Tau[jrow(sr) * 512 + lane];
  }
  auto tau = [&](int sr, int e) -> cplx {
    if constexpr (TAUREG) {
      return tau_r[e];
    } else {
#ifdef DG_NOTAU  // timing diagnostic only (wrong results)
      return cplx{1.0, 0.0};
#endif
      return e == 0 ? tau_r[sr] : cmul(tau_r[sr], beta[jrow(sr) * 8 + e]);
    }
  };
  uint64_t A[SPW][16];
  double max_resid = 0.0;
  // BACK: slot m + 1's columns are loaded while slot m's columns and rows are transformed, the
  // first slot's ahead of the accumulator: every HBM read of Y overlaps work
  const cplx* Yc = a.Y + (uint64_t)poly * a.limbs * M;
  cplx pf[CPT][R];
  auto load_cols = [&](uint32_t m) {
    const cplx* Ym = Yc + (uint64_t)m * M;
#pragma unroll
    for (int p = 0; p < CPT; ++p)
#pragma unroll
      for (int k1 = 0; k1 < R; ++k1) {
#ifdef DG_NOY  // timing diagnostic only (wrong results)
        pf[p][k1] = cplx{(double)(k1 + m), (double)pos_of(p)};
#else
        pf[p][k1] = ld_once(&Ym[k1 * 512 + pos_of(p)]);
#endif
      }
    __builtin_amdgcn_sched_barrier(0);  // issued here, not sunk to their first use
  };
  if constexpr ((MODE & MODE_BACK) != 0) load_cols(0);

  if constexpr ((MODE & MODE_INIT) != 0) {
    // acc_c = LUT_c * X^{-ms(b)} (blind_rotate_assign: polynomial_wrapping_monic_monomial_div)
    const uint64_t* lut = a.luts + (a.lut_idx ? a.lut_idx[s] : 0ull) * (uint64_t)(K1 * N) + (uint64_t)c * N;
    const uint32_t bt = modswitch(lwe[a.n], LOG2_2N);
#pragma unroll
    for (int sr = 0; sr < SPW; ++sr)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const uint32_t src = ((uint32_t)(jrow(sr) + R * jcol(e)) + bt) & (2 * N - 1);
        const uint64_t v = lut[src & (N - 1)];
        A[sr][e] = src < (uint32_t)N ? v : 0ull - v;
      }
  } else {
#pragma unroll
    for (int sr = 0; sr < SPW; ++sr)
#pragma unroll
      for (int e = 0; e < 16; ++e) A[sr][e] = acc[jrow(sr) * ROWLEN + jcol(e)];
  }
  pair_barrier();  // fft512 tables

  if constexpr ((MODE & MODE_BACK) != 0) {
    // acc += sum_m 2^{m b} round(iFFT(Y_m) conj(zeta^j)); the key spectra carry the 1/M
#pragma unroll 1
    for (uint32_t m = 0; m < a.limbs; ++m) {
      cplx u[CPT][R];
#pragma unroll
      for (int p = 0; p < CPT; ++p)
#pragma unroll
        for (int k1 = 0; k1 < R; ++k1) u[p][k1] = pf[p][k1];
      if (m + 1 < a.limbs) load_cols(m + 1);
#pragma unroll
      for (int p = 0; p < CPT; ++p) {
#ifndef DG_NOCOL
        dft_col<R, true>(u[p]);
#endif
#pragma unroll
        for (int j1 = 0; j1 < R; ++j1) E[j1 * RS + pos_of(p)] = u[p][j1];
      }
      pair_barrier();
      // slot shifts stay below 64: the top limb is 64 - (L - 1) b bits wide (key_format), so no
      // guard (a per-element `sh < 64` test had become one branch per coefficient, with the
      // accumulator spilled around each)
      const uint32_t sh = (m * a.bits) & 63u;
#pragma unroll
      for (int sr = 0; sr < SPW; ++sr) {
        // row 0 of the wave is read whole before its transform writes the scratch over it
        cplx v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = E[jrow(sr) * RS + e * 64 + lane];
        wave_lds_fence();
        if (jrow(sr) != 0)  // tau(0, .) = 1
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = cmulc(v[e], tau(sr, e));
        // output twiddles read after the transpose (fft512_inv_tw): 32 fewer VGPRs live across
        // it, which the next slot's prefetched columns need
        cplx gi2[4];
        inv_p2_stage_tw(gi2, T, lane & 7);
#ifndef DG_NOROW
        fft512_inv_tw(v, xch, T, lane, gi2, 0);
#endif
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const double tr = v[e].re + RND_MAGIC, ti = v[e].im + RND_MAGIC;
          max_resid = fmax(max_resid, fmax(fabs(v[e].re - (tr - RND_MAGIC)), fabs(v[e].im - (ti - RND_MAGIC))));
          A[sr][e] += ((uint64_t)__double_as_longlong(tr) - RND_MAGIC_BITS) << sh;
          A[sr][e + 8] += ((uint64_t)__double_as_longlong(ti) - RND_MAGIC_BITS) << sh;
        }
      }
      pair_barrier();
    }
  }

  if constexpr ((MODE & (MODE_BACK | MODE_INIT)) != 0) {
#pragma unroll
    for (int sr = 0; sr < SPW; ++sr)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
#if GEN_NT_STORES >= 2
        __builtin_nontemporal_store(A[sr][e], &acc[jrow(sr) * ROWLEN + jcol(e)]);
#else
        acc[jrow(sr) * ROWLEN + jcol(e)] = A[sr][e];
#endif
      }
  }

  if constexpr ((MODE & MODE_FRONT) != 0) {
    // ct1 = X^{ms(a_i)} acc - acc through the LDS copy of the accumulator (row order)
    const uint32_t at = modswitch(lwe[a.step], LOG2_2N);
    uint64_t* accl = reinterpret_cast<uint64_t*>(E);
#pragma unroll
    for (int sr = 0; sr < SPW; ++sr)
#pragma unroll
      for (int e = 0; e < 16; ++e) accl[jrow(sr) * ROWLEN + jcol(e)] = A[sr][e];
    pair_barrier();
    const int nrep = 64 - (int)(a.level * a.base_log);
    St S[SPW][16];
#pragma unroll
    for (int sr = 0; sr < SPW; ++sr)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const uint32_t src = ((uint32_t)(jrow(sr) + R * jcol(e)) - at) & (2 * N - 1);
        const uint32_t idx = src & (N - 1);
        const uint64_t rv = accl[(idx & (R - 1)) * ROWLEN + (idx >> LOGR)];
        const uint64_t x = (src < (uint32_t)N ? rv : 0ull - rv) - A[sr][e];
        S[sr][e] = (St)(nrep > 0 ? decomp_init(x, nrep) : x);
      }
    pair_barrier();
    cplx* Xc = a.X + (uint64_t)poly * a.level * a.subs * M;
    const int logB = (int)a.base_log, sb = (int)a.bits;
    // one sub-digit: half = 0 and an all-ones mask make s = D and leave D = 0 (no per-element branch)
    const bool split = a.subs > 1;
    const St half = split ? (St)1 << (sb - 1) : (St)0, bmask = split ? ((St)1 << sb) - (St)1 : ~(St)0;
#ifdef DG_NOFRONT  // timing diagnostic only (wrong results): no forward transforms / X stores
    if (S[0][0] != (St)0x12345) return;
#endif
#pragma unroll 1
    for (uint32_t q = 0; q < a.level; ++q) {
      Dg D[SPW][16];
#pragma unroll
      for (int sr = 0; sr < SPW; ++sr)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          if constexpr (W32) D[sr][e] = decomp_next_t<uint32_t>(S[sr][e], logB);
          else D[sr][e] = decomp_next64(S[sr][e], logB);
        }
#pragma unroll 1
      for (uint32_t t = 0; t < a.subs; ++t) {
        cplx hold[8];  // SPW = 2: the first row's spectrum, until the second row's transform is done
#pragma unroll
        for (int sr = 0; sr < SPW; ++sr) {
          cplx v[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            // balanced b-bit sub-digit, exact: D - s is a multiple of 2^b
            const Dg s0 = (Dg)(((St)D[sr][e] + half) & bmask) - (Dg)half;
            const Dg s1 = (Dg)(((St)D[sr][e + 8] + half) & bmask) - (Dg)half;
            D[sr][e] = (D[sr][e] - s0) >> sb;
            D[sr][e + 8] = (D[sr][e + 8] - s1) >> sb;
            v[e] = {(double)s0, (double)s1};
          }
#ifndef DG_NOROW
          fft512_fwd(v, xch, T, lane);
#endif
          if (jrow(sr) != 0)
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = cmul(v[e], tau(sr, e));
          if (SPW == 2 && sr == 0) {
#pragma unroll
            for (int e = 0; e < 8; ++e) hold[e] = v[e];
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) E[jrow(sr) * RS + e * 64 + lane] = v[e];
          }
        }
        if constexpr (SPW == 2) {
          wave_lds_fence();
#pragma unroll
          for (int e = 0; e < 8; ++e) E[jrow(0) * RS + e * 64 + lane] = hold[e];
        }
        pair_barrier();
        cplx* dst = Xc + ((uint64_t)q * a.subs + t) * M;
#pragma unroll
        for (int p = 0; p < CPT; ++p) {
          cplx u[R];
#pragma unroll
          for (int j1 = 0; j1 < R; ++j1) u[j1] = E[j1 * RS + pos_of(p)];
#ifndef DG_NOCOL
          dft_col<R, false>(u);
#endif
#pragma unroll
          for (int k1 = 0; k1 < R; ++k1) {
#if GEN_NT_STORES  // variant: streaming (non-temporal) stores of the spectra the next launch reads
            __builtin_nontemporal_store(u[k1].re, &dst[k1 * 512 + pos_of(p)].re);
            __builtin_nontemporal_store(u[k1].im, &dst[k1 * 512 + pos_of(p)].im);
#else
            dst[k1 * 512 + pos_of(p)] = u[k1];
#endif
          }
        }
        pair_barrier();
      }
    }
  }

  if constexpr ((MODE & MODE_BACK) != 0) {
    if (a.resid) {
      for (int off = 32; off > 0; off >>= 1) max_resid = fmax(max_resid, __shfl_xor(max_resid, off));
      if (lane == 0) atomicMax(a.resid, (unsigned long long)__double_as_longlong(max_resid));
    }
  }
}

// ------------------------------------------------------------------------------------------
// N = 32768 / 65536 (the optimizer's 9- and 10-bit rows, v0_last_128): a polynomial spread over
// S = N / 16384 workgroups (round 4).  The M-point spectrum (M = R x 512, R = 32 / 64 rows of the
// four-step order) no longer fits one CU's LDS, so the R-point column DFT splits by row class:
// with j1 = S a + h (h < S, a < 16) and f = k2 + 512 k1,
//   Z_f = sum_h w_R^{h k1} G_h[k1 mod 16](k2),  G_h = DFT16_a( tau(S a + h, k2) FFT512_{S a + h}[k2] )
// i.e. workgroup h of a polynomial runs the 16 rows of its class exactly as gen_big_step_kernel
// runs an M' = 8192 polynomial (fft512 rows in registers, tau, one LDS exchange, DFT16 columns) and
// writes G_h; the product kernel combines the S classes when it loads X (gen_mac_split_kernel), and
// the inverse splits Y back the same way, H_h[k1'] = sum_u conj(w_R^{h (k1' + 16 u)}) Y[k1' + 16 u],
// before workgroup h's inverse DFT16 and row transforms.  Every path through the transform still
// has log2 M butterfly stages with at most log2 M inexact twiddle products, each a correctly rounded
// table entry (tau, w_R) or fft512 / DFT16 constant, so generic_error_bound holds unchanged.  The
// front half (rotation, decomposition, forward transforms) reads the rotated accumulator rows of
// the other classes from HBM, so the back half and the front half are separate launches.
// ------------------------------------------------------------------------------------------
constexpr int SPLIT_ROWS = 16;  // rows per workgroup (the M' = 8192 four-step shape)

struct SplitArgs {
  uint64_t* acc;        // [chunk][K1][N] in the four-step row order (n at (n mod R) ROWLEN + n / R)
  cplx* X;              // [chunk][K1 r][l q][T t][S h][16][512]: the column-class transforms G_h
  const cplx* Y;        // [chunk][K1 c][L m][M], position p = k1 512 + pos (k1 < R)
  const cplx* Tau;      // tau(j1, pos) [R][512], then the slot factors [R][8]
  const cplx* WR;       // w_R^x = exp(-2 pi i x / R), x < R
  const uint64_t* in;   // LWE inputs (rows of n + 1)
  const uint64_t* in_idx;
  const uint64_t* luts;
  const uint64_t* lut_idx;
  unsigned long long* resid;
  uint32_t base, count, n, k, level, base_log, bits, limbs, subs;
  uint32_t step;  // front: the mask position whose rotation is prepared
  uint32_t xcd = 1;  // the S class workgroups of a polynomial on one XCD (split_block)
};

// workgroup -> (polynomial, class h).  Each class workgroup reads its polynomial's whole slot
// spectra (back) and rotated accumulator (front), so with xcd the S classes of a polynomial are
// placed on one XCD — workgroups b and b + 8 share one under the round-robin dispatch — and the
// second to S-th reads can hit that XCD's L2; the last partial group of fewer than 8 polynomials
// keeps the plain order
template <int S>
__device__ __forceinline__ void split_block(uint32_t b, uint32_t polys, bool xcd, uint32_t& poly, uint32_t& h) {
  const uint32_t g = b / (8 * S), r = b % (8 * S);
  if (xcd && (g + 1) * 8 <= polys) {
    poly = g * 8 + (r & 7);
    h = r >> 3;
  } else {
    poly = b / S;
    h = b % S;
  }
}

template <int S>
struct Split {
  static constexpr int R = SPLIT_ROWS * S, M = R * 512, N = 2 * M;
  static constexpr int LOGR = S == 2 ? 5 : 6;
  static constexpr int NT = 512, SPW = 2, RS = 576;  // 8 waves, two rows each
  static constexpr int LDS_CPLX = SPLIT_ROWS * RS + FFT512_TABLE_ENTRIES + SPLIT_ROWS * 8;
  static_assert(S == 2 || S == 4, "split");
  static_assert(LDS_CPLX * 16 <= 160 * 1024, "LDS");
};

// acc = LUT * X^{-ms(b)}, row order (blind_rotate_assign: polynomial_wrapping_monic_monomial_div)
template <int S>
__global__ void __launch_bounds__(256) gen_split_init_kernel(SplitArgs a) {
  using G = Split<S>;
  constexpr int N = G::N, LOG2_2N = G::LOGR + 9 + 2;
  const uint32_t K1 = a.k + 1;
  const uint64_t total = (uint64_t)a.count * K1 * N;
  for (uint64_t g = blockIdx.x * 256ull + threadIdx.x; g < total; g += (uint64_t)gridDim.x * 256) {
    const uint32_t nn = (uint32_t)(g % N);
    const uint64_t poly = g / N;
    const uint32_t ct = (uint32_t)(poly / K1), c = (uint32_t)(poly % K1), s = a.base + ct;
    const uint64_t row = a.in_idx ? a.in_idx[s] : s;
    const uint32_t bt = modswitch(a.in[row * (uint64_t)(a.n + 1) + a.n], LOG2_2N);
    const uint64_t* lut = a.luts + (a.lut_idx ? a.lut_idx[s] : 0ull) * (uint64_t)(K1 * N) + (uint64_t)c * N;
    const uint32_t src = (nn + bt) & (2 * N - 1);
    const uint64_t v = lut[src & (N - 1)];
    a.acc[poly * N + (uint64_t)(nn & (G::R - 1)) * (N / G::R) + (nn >> G::LOGR)] = src < (uint32_t)N ? v : 0ull - v;
  }
}

// The rows of class h of one polynomial: tables, tau factors (lane factor in registers, slot factor
// in LDS, as gen_big_step_kernel at R = 16) and the global row of local row jl.
template <int S>
struct SplitRows {
  cplx* E;
  cplx* beta;
  Fft512Tables T;
  cplx tau_r[2];
  int w, lane, h;
  __device__ int jg(int sr) const { return S * (w * 2 + sr) + h; }
  __device__ cplx tau(int sr, int e) const { return e == 0 ? tau_r[sr] : cmul(tau_r[sr], beta[(w * 2 + sr) * 8 + e]); }
};

template <int S>
__device__ __forceinline__ SplitRows<S> split_rows_setup(cplx* lds, const SplitArgs& a, int h) {
  using G = Split<S>;
  SplitRows<S> q;
  q.E = lds;
  build_fft512_tables(lds + SPLIT_ROWS * G::RS, threadIdx.x, G::NT);
  q.beta = lds + SPLIT_ROWS * G::RS + FFT512_TABLE_ENTRIES;
  q.w = threadIdx.x >> 6, q.lane = threadIdx.x & 63, q.h = h;
  for (int x = threadIdx.x; x < SPLIT_ROWS * 8; x += G::NT)
    q.beta[x] = a.Tau[G::R * 512 + (S * (x >> 3) + h) * 8 + (x & 7)];
  q.T = fft512_tables_at(lds + SPLIT_ROWS * G::RS);
#pragma unroll
  for (int sr = 0; sr < 2; ++sr) q.tau_r[sr] = a.Tau[q.jg(sr) * 512 + q.lane];
  return q;
}

// front: X^{a_i} acc - acc from the accumulator in HBM, decomposition, sub-digits, the class-h
// transforms of every digit polynomial -> X (G_h)
template <int S, bool W32>
__global__ void __launch_bounds__(512) gen_split_front_kernel(SplitArgs a) {
  using G = Split<S>;
  constexpr int N = G::N, R = G::R, RS = G::RS, LOG2_2N = G::LOGR + 9 + 2, ROWLEN = N / R;
  using St = typename std::conditional<W32, uint32_t, uint64_t>::type;
  using Dg = typename std::conditional<W32, int32_t, int64_t>::type;
  __shared__ cplx lds[G::LDS_CPLX];
  const uint32_t K1 = a.k + 1;
  uint32_t poly, h;
  split_block<S>(blockIdx.x, a.count * K1, a.xcd != 0, poly, h);
  const uint32_t ct = poly / K1;
  const SplitRows<S> q = split_rows_setup<S>(lds, a, (int)h);
  const int lane = q.lane;
  cplx* xch = q.E + q.w * 2 * RS;  // the wave's first row and its pad
  const uint32_t s = a.base + ct;
  const uint64_t row = a.in_idx ? a.in_idx[s] : s;
  const uint32_t at = modswitch(a.in[row * (uint64_t)(a.n + 1) + a.step], LOG2_2N);
  const uint64_t* acc = a.acc + (uint64_t)poly * N;
  auto jcol = [&](int e) { return lane + 64 * (e & 7) + 512 * (e >> 3); };
  const int nrep = 64 - (int)(a.level * a.base_log);
  St Sx[2][16];
#pragma unroll
  for (int sr = 0; sr < 2; ++sr)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const uint32_t nn = (uint32_t)(q.jg(sr) + R * jcol(e));
      const uint32_t src = (nn - at) & (2 * N - 1), idx = src & (N - 1);
      const uint64_t rv = acc[(uint64_t)(idx & (R - 1)) * ROWLEN + (idx >> G::LOGR)];
      const uint64_t x = (src < (uint32_t)N ? rv : 0ull - rv) - acc[(uint64_t)q.jg(sr) * ROWLEN + jcol(e)];
      Sx[sr][e] = (St)(nrep > 0 ? decomp_init(x, nrep) : x);
    }
  pair_barrier();  // fft512 tables, beta
  cplx* Xc = a.X + (uint64_t)poly * a.level * a.subs * S * (SPLIT_ROWS * 512) + (uint64_t)h * SPLIT_ROWS * 512;
  const int logB = (int)a.base_log, sb = (int)a.bits;
  const bool split = a.subs > 1;
  const St half = split ? (St)1 << (sb - 1) : (St)0, bmask = split ? ((St)1 << sb) - (St)1 : ~(St)0;
#pragma unroll 1
  for (uint32_t qq = 0; qq < a.level; ++qq) {
    Dg D[2][16];
#pragma unroll
    for (int sr = 0; sr < 2; ++sr)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        if constexpr (W32) D[sr][e] = decomp_next_t<uint32_t>(Sx[sr][e], logB);
        else D[sr][e] = decomp_next64(Sx[sr][e], logB);
      }
#pragma unroll 1
    for (uint32_t t = 0; t < a.subs; ++t) {
      cplx hold[8];  // the first row's spectrum, until the second row's transform is done
#pragma unroll
      for (int sr = 0; sr < 2; ++sr) {
        cplx v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const Dg s0 = (Dg)(((St)D[sr][e] + half) & bmask) - (Dg)half;
          const Dg s1 = (Dg)(((St)D[sr][e + 8] + half) & bmask) - (Dg)half;
          D[sr][e] = (D[sr][e] - s0) >> sb;
          D[sr][e + 8] = (D[sr][e + 8] - s1) >> sb;
          v[e] = {(double)s0, (double)s1};
        }
        fft512_fwd(v, xch, q.T, lane);
        if (q.jg(sr) != 0)
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = cmul(v[e], q.tau(sr, e));
        if (sr == 0) {
#pragma unroll
          for (int e = 0; e < 8; ++e) hold[e] = v[e];
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) q.E[(q.w * 2 + 1) * RS + e * 64 + lane] = v[e];
        }
      }
      wave_lds_fence();
#pragma unroll
      for (int e = 0; e < 8; ++e) q.E[(q.w * 2) * RS + e * 64 + lane] = hold[e];
      pair_barrier();
      cplx* dst = Xc + ((uint64_t)qq * a.subs + t) * S * (SPLIT_ROWS * 512);
      const int pos = threadIdx.x;
      cplx u[SPLIT_ROWS];
#pragma unroll
      for (int jl = 0; jl < SPLIT_ROWS; ++jl) u[jl] = q.E[jl * RS + pos];
      dft_col<SPLIT_ROWS, false>(u);
#pragma unroll
      for (int k1 = 0; k1 < SPLIT_ROWS; ++k1) {
#if GEN_NT_STORES >= 2
        __builtin_nontemporal_store(u[k1].re, &dst[k1 * 512 + pos].re);
        __builtin_nontemporal_store(u[k1].im, &dst[k1 * 512 + pos].im);
#else
        dst[k1 * 512 + pos] = u[k1];
#endif
      }
      pair_barrier();
    }
  }
}

// back: acc += sum_m 2^{m b} round(iFFT(Y_m) conj(zeta^j)) for the rows of class h
// HPRE: the product kernel has already split the slot spectra by class (gen_mac_split_kernel writes
// H_h[m][k1'][pos] in Y's place), so class h loads its 16 values per slot directly — a third of the
// loads at S = 2 with no combination — and the next slot's are loaded while this slot is transformed
template <int S, bool HPRE>
__global__ void __launch_bounds__(512) gen_split_back_kernel(SplitArgs a) {
  using G = Split<S>;
  constexpr int N = G::N, R = G::R, RS = G::RS, M = G::M, ROWLEN = N / R;
  __shared__ cplx lds[G::LDS_CPLX];
  uint32_t poly, h;
  split_block<S>(blockIdx.x, a.count * (a.k + 1), a.xcd != 0, poly, h);
  const SplitRows<S> q = split_rows_setup<S>(lds, a, (int)h);
  const int lane = q.lane, pos = threadIdx.x;
  cplx* xch = q.E + q.w * 2 * RS;
  uint64_t* acc = a.acc + (uint64_t)poly * N;
  auto jcol = [&](int e) { return lane + 64 * (e & 7) + 512 * (e >> 3); };
  uint64_t A[2][16];
#pragma unroll
  for (int sr = 0; sr < 2; ++sr)
#pragma unroll
    for (int e = 0; e < 16; ++e) A[sr][e] = acc[(uint64_t)q.jg(sr) * ROWLEN + jcol(e)];
  // conj(w_R^{h (k1' + 16 u)}) for this class, k1' < 16, u < S
  const cplx* Yc = a.Y + (uint64_t)poly * a.limbs * M + pos;
  double max_resid = 0.0;
#ifndef SPLIT_HPF
// HPRE: how the next slot's values are loaded ahead.  3 (kept): half of them, issued once this slot's
// columns are in LDS (254 VGPRs; +2 % against none at opt9 and opt10, profiles/r06/split_path);
// 1: all of them before this slot's transforms (spills 39 VGPRs, -1 %); 2: all of them after the
// columns (spills 29, -1 %); 0: none
#define SPLIT_HPF 3
#endif
  constexpr bool PF = HPRE && SPLIT_HPF == 1;
  constexpr bool LATE = HPRE && (SPLIT_HPF == 2 || SPLIT_HPF == 3);  // variant: issued after this slot's columns are in LDS
  constexpr int NPF = SPLIT_HPF == 3 ? SPLIT_ROWS / 2 : SPLIT_ROWS;  // values loaded ahead (3: half)
  cplx pf[HPRE ? SPLIT_ROWS : 1];
  auto load_h = [&](uint32_t m, int k0 = 0, int k9 = SPLIT_ROWS) {
    const cplx* Hm = Yc + (uint64_t)m * M + (uint64_t)h * SPLIT_ROWS * 512;
#pragma unroll
    for (int k1 = 0; k1 < SPLIT_ROWS; ++k1)
      if (k1 >= k0 && k1 < k9) pf[k1] = Hm[(uint64_t)k1 * 512];
    __builtin_amdgcn_sched_barrier(0);  // issued here, not sunk to their first use
  };
  if constexpr (PF || LATE) load_h(0, 0, NPF);
  pair_barrier();  // fft512 tables, beta
#pragma unroll 1
  for (uint32_t m = 0; m < a.limbs; ++m) {
    const cplx* Ym = Yc + (uint64_t)m * M;
    cplx u[SPLIT_ROWS];
    if constexpr (HPRE) {
      if constexpr (!PF && !LATE) load_h(m);
      if constexpr (LATE && NPF < SPLIT_ROWS) load_h(m, NPF, SPLIT_ROWS);
#pragma unroll
      for (int k1 = 0; k1 < SPLIT_ROWS; ++k1) u[k1] = pf[k1];
      if (PF && m + 1 < a.limbs) load_h(m + 1);
    } else {
#pragma unroll
      for (int k1 = 0; k1 < SPLIT_ROWS; ++k1) {
        cplx hsum = {0.0, 0.0};
#pragma unroll
        for (int uu = 0; uu < S; ++uu) {
          const int kk = k1 + SPLIT_ROWS * uu;
          const cplx y = Ym[(uint64_t)kk * 512];
          const cplx w = a.WR[(h * kk) & (R - 1)];
          hsum = cadd(hsum, cmulc(y, w));
        }
        u[k1] = hsum;
      }
    }
    dft_col<SPLIT_ROWS, true>(u);
#pragma unroll
    for (int jl = 0; jl < SPLIT_ROWS; ++jl) q.E[jl * RS + pos] = u[jl];
    if (LATE && m + 1 < a.limbs) load_h(m + 1, 0, NPF);
    pair_barrier();
    const uint32_t sh = (m * a.bits) & 63u;
#pragma unroll
    for (int sr = 0; sr < 2; ++sr) {
      // row 0 of the wave is read whole before its transform writes the scratch over it
      cplx v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = q.E[(q.w * 2 + sr) * RS + e * 64 + lane];
      wave_lds_fence();
      if (q.jg(sr) != 0)
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = cmulc(v[e], q.tau(sr, e));
      cplx gi2[4];
      inv_p2_stage_tw(gi2, q.T, lane & 7);
      fft512_inv_tw(v, xch, q.T, lane, gi2, 0);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const double tr = v[e].re + RND_MAGIC, ti = v[e].im + RND_MAGIC;
        max_resid = fmax(max_resid, fmax(fabs(v[e].re - (tr - RND_MAGIC)), fabs(v[e].im - (ti - RND_MAGIC))));
        A[sr][e] += ((uint64_t)__double_as_longlong(tr) - RND_MAGIC_BITS) << sh;
        A[sr][e + 8] += ((uint64_t)__double_as_longlong(ti) - RND_MAGIC_BITS) << sh;
      }
    }
    pair_barrier();
  }
#pragma unroll
  for (int sr = 0; sr < 2; ++sr)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
#if GEN_NT_STORES >= 2
      __builtin_nontemporal_store(A[sr][e], &acc[(uint64_t)q.jg(sr) * ROWLEN + jcol(e)]);
#else
      acc[(uint64_t)q.jg(sr) * ROWLEN + jcol(e)] = A[sr][e];
#endif
    }
  if (a.resid) {
    for (int off = 32; off > 0; off >>= 1) max_resid = fmax(max_resid, __shfl_xor(max_resid, off));
    if (lane == 0) atomicMax(a.resid, (unsigned long long)__double_as_longlong(max_resid));
  }
}

// Y[ct][c][m][p] = sum over (r, q, t) with 0 <= m - t < L of X_p[r][q][t] G_i[c][m-t][r][q][p], with
// X_p = sum_h w_R^{h k1} G_h[k1 mod 16][pos] combined on load (p = k1 512 + pos): one thread per
// (position, output polynomial), the key values of the thread in registers across the tile
struct MacSplitArgs {
  const cplx* X;
  cplx* Y;
  const cplx* G;  // Fourier key [n][K1 c][L lim][K1 l rq][M]
  const cplx* WR;
  uint32_t count, k, level, limbs, subs, M, R;
  uint32_t i;
};

// The slot spectra leave already split by class for gen_split_back_kernel<S, true>.  A wave covers
// 64 / S positions of one k1' < 16 at its S frequencies k1' + 16 u (lane = u 64 / S + position), so
// the S values of a position meet inside the wave: the digit spectra are combined from the S class
// transforms (each lane loads its own class's value, the others arrive by lane shuffles), and lane
// (u, position) writes class h = u's H_h[k1'] = sum_u' conj(w_R^{h (k1' + 16 u')}) Y[k1' + 16 u'] —
// the back kernel's former combination, same terms in the same order — at [ct][c][m][h][k1'][pos], in
// Y's place and size.  (Exchanging through LDS behind a workgroup barrier per ciphertext instead:
// 1018 vs 798 us per step at opt10.)
template <int KL, int L, int T, int S>
__global__ void __launch_bounds__(256) gen_mac_split_kernel(MacSplitArgs a) {
  constexpr int QW = 64 / S, PB = 256 / S;  // positions per wave / per block
  const uint32_t b = blockIdx.x, kl = b / (2 * S), lane = threadIdx.x & 63;
  const uint32_t u = lane / QW, pl = lane % QW;
  const uint32_t pos = (b % (2 * S)) * PB + (threadIdx.x >> 6) * QW + pl;
  const uint32_t k1 = kl + SPLIT_ROWS * u, p = k1 * 512 + pos;
  const uint32_t c = blockIdx.y, K1 = a.k + 1;
  const uint64_t M = a.M;
  cplx wr[S], wi[S];
#pragma unroll
  for (int hh = 0; hh < S; ++hh) {
    wr[hh] = a.WR[(hh * k1) & (a.R - 1)];
    wi[hh] = a.WR[(u * (kl + SPLIT_ROWS * hh)) & (a.R - 1)];
  }
  auto from = [&](cplx v, int hh) -> cplx {  // lane (hh, pl)'s value
    const int src = hh * QW + (int)pl;
    return {__shfl(v.re, src, 64), __shfl(v.im, src, 64)};
  };
  cplx kv[L][KL];
#pragma unroll
  for (int lim = 0; lim < L; ++lim)
#pragma unroll
    for (int rq = 0; rq < KL; ++rq) kv[lim][rq] = a.G[((((uint64_t)a.i * K1 + c) * L + lim) * KL + rq) * M + p];
  const uint32_t ct0 = blockIdx.z * MAC_CTS;
  for (uint32_t ct = ct0; ct < ct0 + MAC_CTS && ct < a.count; ++ct) {
    // my class's transform value at (k1', pos) of every digit polynomial
    const cplx* Xct = a.X + (uint64_t)ct * KL * T * M + (uint64_t)u * SPLIT_ROWS * 512 + (uint64_t)kl * 512 + pos;
    cplx xv[KL][T];
#pragma unroll
    for (int rq = 0; rq < KL; ++rq)
#pragma unroll
      for (int t = 0; t < T; ++t) xv[rq][t] = Xct[(uint64_t)(rq * T + t) * M];
#pragma unroll
    for (int rq = 0; rq < KL; ++rq)
#pragma unroll
      for (int t = 0; t < T; ++t) {
        const cplx g = xv[rq][t];
        cplx x = from(g, 0);  // class 0: w_R^0 = 1
#pragma unroll
        for (int hh = 1; hh < S; ++hh) {
          const cplx gh = from(g, hh), w = wr[hh];
          x.re = __builtin_fma(gh.re, w.re, __builtin_fma(-gh.im, w.im, x.re));
          x.im = __builtin_fma(gh.re, w.im, __builtin_fma(gh.im, w.re, x.im));
        }
        xv[rq][t] = x;
      }
    cplx* Hct = a.Y + ((uint64_t)ct * K1 + c) * L * M + (uint64_t)(u * SPLIT_ROWS + kl) * 512 + pos;
#pragma unroll
    for (int m = 0; m < L; ++m) {
      cplx y = {0.0, 0.0};
#pragma unroll
      for (int t = 0; t < T; ++t) {
        if (m - t < 0 || m - t >= L) continue;
#pragma unroll
        for (int rq = 0; rq < KL; ++rq) {
          const cplx xg = xv[rq][t], g = kv[m - t][rq];
          y.re = __builtin_fma(xg.re, g.re, __builtin_fma(-xg.im, g.im, y.re));
          y.im = __builtin_fma(xg.re, g.im, __builtin_fma(xg.im, g.re, y.im));
        }
      }
      cplx hsum = {0.0, 0.0};
#pragma unroll
      for (int uu = 0; uu < S; ++uu) hsum = cadd(hsum, cmulc(from(y, uu), wi[uu]));
#if GEN_NT_STORES >= 2
      __builtin_nontemporal_store(hsum.re, &Hct[(uint64_t)m * M].re);
      __builtin_nontemporal_store(hsum.im, &Hct[(uint64_t)m * M].im);
#else
      Hct[(uint64_t)m * M] = hsum;
#endif
    }
  }
}

// Any (k, l, T, L): one thread per (position, output polynomial, slot), the key values of
// GEN_MAX_TERMS terms at a time in registers (as gen_mac_kernel), X combined on load.
template <int S>
__global__ void __launch_bounds__(256) gen_mac_split_generic_kernel(MacSplitArgs a) {
  const uint32_t p = blockIdx.x * 256 + threadIdx.x;
  const uint32_t K1 = a.k + 1, L = a.limbs, T = a.subs;
  const uint32_t c = blockIdx.y / L, m = blockIdx.y % L;
  const uint32_t terms = K1 * a.level * T;
  const uint64_t M = a.M;
  if (p >= M) return;
  const uint32_t k1 = p >> 9, pos = p & 511, kl = k1 & (SPLIT_ROWS - 1);
  cplx wr[S];
#pragma unroll
  for (int h = 0; h < S; ++h) wr[h] = a.WR[(h * k1) & (a.R - 1)];
  const uint32_t ct0 = blockIdx.z * MAC_CTS;
#pragma unroll 1
  for (uint32_t x0 = 0; x0 < terms; x0 += GEN_MAX_TERMS) {
    cplx kv[GEN_MAX_TERMS];
#pragma unroll
    for (int x = 0; x < GEN_MAX_TERMS; ++x) {
      kv[x] = {0.0, 0.0};
      const uint32_t xx = x0 + x;
      if (xx < terms) {
        const uint32_t t = xx % T, rq = xx / T;  // xx = (r l + q) T + t
        if (m >= t && m - t < L) kv[x] = a.G[((((uint64_t)a.i * K1 + c) * L + (m - t)) * K1 * a.level + rq) * M + p];
      }
    }
    for (uint32_t ct = ct0; ct < ct0 + MAC_CTS && ct < a.count; ++ct) {
      const cplx* Xct = a.X + (uint64_t)ct * terms * M + (uint64_t)kl * 512 + pos;
      cplx* Yp = a.Y + (((uint64_t)ct * K1 + c) * L + m) * M + p;
      cplx y = x0 ? *Yp : cplx{0.0, 0.0};
#pragma unroll
      for (int x = 0; x < GEN_MAX_TERMS; ++x) {
        if (x0 + x < terms) {
          const cplx* g = Xct + (uint64_t)(x0 + x) * M;
          cplx xv = g[0];
#pragma unroll
          for (int h = 1; h < S; ++h) xv = cadd(xv, cmul(g[(uint64_t)h * SPLIT_ROWS * 512], wr[h]));
          y.re = __builtin_fma(xv.re, kv[x].re, __builtin_fma(-xv.im, kv[x].im, y.re));
          y.im = __builtin_fma(xv.re, kv[x].im, __builtin_fma(xv.im, kv[x].re, y.im));
        }
      }
      *Yp = y;
    }
  }
}

// Key conversion at N >= 32768: the class-h transforms of every limb of every standard polynomial
// (the front kernel's transform with the limb as input) into scratch, then the combine and 1/M.
struct SplitConvArgs {
  cplx* Gs;             // [poly in batch][limb][S h][16][512]
  const uint64_t* src;  // standard key, [i][v][r][c][N]
  const cplx* Tau;
  const cplx* WR;
  cplx* dest;           // Fourier key [i][c][lim][r][q][M]
  uint64_t poly0;       // first standard polynomial of this batch
  uint32_t polys, k, level, bits, limbs;
  unsigned long long* smax;  // keycheck.hpp sink (or nullptr)
};

template <int S>
__global__ void __launch_bounds__(512) gen_split_convert_kernel(SplitConvArgs a) {
  using G = Split<S>;
  constexpr int N = G::N, R = G::R, RS = G::RS;
  __shared__ cplx lds[G::LDS_CPLX];
  const uint32_t h = blockIdx.x % S, item = blockIdx.x / S;  // item = (poly in batch, limb)
  const uint32_t lim = item % a.limbs, pb = item / a.limbs;
  SplitArgs t{};
  t.Tau = a.Tau;
  const SplitRows<S> q = split_rows_setup<S>(lds, t, (int)h);
  const int lane = q.lane, pos = threadIdx.x;
  cplx* xch = q.E + q.w * 2 * RS;
  const uint64_t* g = a.src + (a.poly0 + pb) * (uint64_t)N;
  auto jcol = [&](int e) { return lane + 64 * (e & 7) + 512 * (e >> 3); };
  pair_barrier();  // fft512 tables, beta
  cplx hold[8];
#pragma unroll
  for (int sr = 0; sr < 2; ++sr) {
    cplx v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      // limb lim of the coefficient: balanced limbs as gen_convert_kernel (top limb in its own width)
      int64_t sv[2];
#pragma unroll
      for (int z = 0; z < 2; ++z) {
        uint64_t gv = g[(uint64_t)(q.jg(sr) + R * jcol(e + 8 * z))];
        int64_t s0 = 0;
        for (uint32_t j = 0; j <= lim; ++j) {
          const uint32_t w = j + 1 < a.limbs ? a.bits : 64 - (a.limbs - 1) * a.bits;
          const uint64_t half = 1ull << (w - 1), bmask = (1ull << w) - 1ull;
          s0 = (int64_t)((gv + half) & bmask) - (int64_t)half;
          gv = (gv - (uint64_t)s0) >> a.bits;
        }
        sv[z] = s0;
      }
      v[e] = {(double)sv[0], (double)sv[1]};
    }
    fft512_fwd(v, xch, q.T, lane);
    if (q.jg(sr) != 0)
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = cmul(v[e], q.tau(sr, e));
    if (sr == 0) {
#pragma unroll
      for (int e = 0; e < 8; ++e) hold[e] = v[e];
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) q.E[(q.w * 2 + 1) * RS + e * 64 + lane] = v[e];
    }
  }
  wave_lds_fence();
#pragma unroll
  for (int e = 0; e < 8; ++e) q.E[(q.w * 2) * RS + e * 64 + lane] = hold[e];
  pair_barrier();
  cplx u[SPLIT_ROWS];
#pragma unroll
  for (int jl = 0; jl < SPLIT_ROWS; ++jl) u[jl] = q.E[jl * RS + pos];
  dft_col<SPLIT_ROWS, false>(u);
  cplx* dst = a.Gs + ((uint64_t)item * S + h) * SPLIT_ROWS * 512;
#pragma unroll
  for (int k1 = 0; k1 < SPLIT_ROWS; ++k1) dst[k1 * 512 + pos] = u[k1];
}

template <int S>
__global__ void __launch_bounds__(256) gen_split_combine_kernel(SplitConvArgs a) {
  using G = Split<S>;
  constexpr int M = G::M, R = G::R;
  const uint64_t total = (uint64_t)a.polys * a.limbs * M;
  const uint32_t K1 = a.k + 1;
  const double scale = 1.0 / (double)M;
  double m2 = 0.0;  // max |G|^2 of the stored values (keycheck.hpp)
  for (uint64_t gi = blockIdx.x * 256ull + threadIdx.x; gi < total; gi += (uint64_t)gridDim.x * 256) {
    const uint32_t p = (uint32_t)(gi % M);
    const uint64_t item = gi / M;
    const uint32_t lim = (uint32_t)(item % a.limbs);
    const uint64_t pb = item / a.limbs;
    const uint32_t k1 = p >> 9, pos = p & 511, kl = k1 & (SPLIT_ROWS - 1);
    const cplx* gs = a.Gs + (item * S) * SPLIT_ROWS * 512 + (uint64_t)kl * 512 + pos;
    cplx x = gs[0];
#pragma unroll
    for (int h = 1; h < S; ++h) x = cadd(x, cmul(gs[(uint64_t)h * SPLIT_ROWS * 512], a.WR[(h * k1) & (R - 1)]));
    // standard polynomial index -> Fourier key slot (gen_convert_kernel)
    uint64_t sp = a.poly0 + pb;
    const uint32_t c = (uint32_t)(sp % K1);
    sp /= K1;
    const uint32_t r = (uint32_t)(sp % K1);
    sp /= K1;
    const uint32_t v = (uint32_t)(sp % a.level);
    const uint64_t i = sp / a.level;
    const uint32_t qq = a.level - 1 - v;
    a.dest[((((i * K1 + c) * a.limbs + lim) * K1 + r) * a.level + qq) * (uint64_t)M + p] = {x.re * scale, x.im * scale};
    m2 = fmax(m2, spec_mag2(x.re * scale, x.im * scale));
  }
  spec_max_commit(a.smax, m2);
}

// ------------------------------------------------------------------------------------------
// N = 4096, k = 1: the whole blind rotation of a ciphertext in ONE workgroup and one launch, the
// digit and slot spectra on chip (round 4).  The two-launch path above moves ~0.57 MB of X / Y
// spectra and accumulator per ciphertext and CMUX step through HBM at N = 4096 (8x the
// algorithmic bytes, profiles/r04_opt6_pmc.json); here only the key is streamed (from L2: every
// CU walks the same GGSW at about the same time) and the LWE rows are read and written once.
//
// Mapping: 8 waves; wave w owns row j1 = w mod R of GLWE polynomial c = w / R of the accumulator
// in registers (the four-step row order of gen_big_step_kernel: coefficient n = j1 + R J, lane
// holds J = lane + 64 e and J + 512, 16 u64).  Per CMUX step:
//   forward  the rotated difference X^{a} acc - acc through an LDS copy of both polynomials,
//            decomposition, sub-digits; per (q, t) every wave transforms its row (fft512_fwd,
//            column twiddle tau), one barrier, then thread p runs the R-point column DFT of
//            position p for both polynomials: X[(r q) T + t][k1] = frequency k1 512 + p stays in
//            the thread's registers (2 l T R complex);
//   product  slot m of output polynomial c at the thread's R frequencies, Y = sum_{r,q,t} X G,
//            key values read straight from L2 (coalesced: position p is the fastest index of the
//            key, gen_convert_kernel perm);
//   inverse  the R-point inverse column DFT in registers into the rows of E, one barrier, every
//            wave the inverse row transform of its row, exact rounding and the 2^{m b} shift-add
//            into its accumulator row.
// The arithmetic is gen_big_step_kernel's (same transforms, twiddles, key and rounding), so the
// certified bound and generic_pbs_ok hold unchanged; the tests compare bit for bit with the
// oracle.  LDS: 2R rows of 576 complex (each wave's row doubles as its transpose scratch), the
// fft512 tables and tau: 118 KB, one workgroup per CU.
// ------------------------------------------------------------------------------------------
struct FusedArgs {
  uint64_t* out;
  const uint64_t* out_idx;
  const uint64_t* in;
  const uint64_t* in_idx;
  const uint64_t* luts;
  const uint64_t* lut_idx;
  const cplx* G;    // Fourier key [n][c][lim][r][q][M], four-step frequency order
  const cplx* Tau;  // column twiddles [R][512]
  unsigned long long* resid;
  uint32_t count, n, base_log, bits;
};

template <int R, int LV, int T, int L>
struct Fused {
  static constexpr int M = R * 512, N = 2 * M;
  static constexpr int NW = 2 * R, NT = 64 * NW;  // one wave per accumulator row
  static constexpr int RS = 576;                  // row stride (complex): 512 + transpose pad
  static constexpr int NX = 2 * LV * T;           // digit spectra per ciphertext and step
  static constexpr int LDS_CPLX = NW * RS + FFT512_TABLE_ENTRIES + R * 512;
  static_assert(NT == 512, "one column position per thread");
  static_assert(LDS_CPLX * 16 <= 160 * 1024, "LDS");
  static_assert(NW * RS * 16 >= 2 * N * 8, "the accumulator copy fits the rows");
};

#ifndef FUSED_PF
#define FUSED_PF 1
#endif
template <int R, int LV, int T, int L, bool W32>
__global__ void __launch_bounds__(512) gen_fused_kernel(FusedArgs a) {
  using F = Fused<R, LV, T, L>;
  constexpr int M = F::M, N = F::N, RS = F::RS, NX = F::NX;
  constexpr int LOGR = R == 2 ? 1 : R == 4 ? 2 : 3, LOG2_2N = Geo<M>::LOG + 2;
  using St = typename std::conditional<W32, uint32_t, uint64_t>::type;
  using Dg = typename std::conditional<W32, int32_t, int64_t>::type;
  __shared__ cplx lds[F::LDS_CPLX];
  cplx* E = lds;
  cplx* tab = lds + F::NW * RS;
  cplx* tau = tab + FFT512_TABLE_ENTRIES;
  build_fft512_tables(tab, threadIdx.x, F::NT);
  for (int x = threadIdx.x; x < R * 512; x += F::NT) tau[x] = a.Tau[x];
  const Fft512Tables TB = fft512_tables_at(tab);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c = w / R, j1 = w % R;
  const int pos = threadIdx.x;  // column position of this thread
  cplx* row = E + w * RS;       // the wave's row (and transpose scratch)
  const uint32_t ct = blockIdx.x;
  const uint64_t in_row = a.in_idx ? a.in_idx[ct] : ct;
  const uint64_t* lwe = a.in + in_row * (uint64_t)(a.n + 1);
  auto jcol = [&](int e) { return lane + 64 * (e & 7) + 512 * (e >> 3); };
  uint64_t A[16];
  {
    // acc_c = LUT_c * X^{-ms(b)} (blind_rotate_assign: polynomial_wrapping_monic_monomial_div)
    const uint64_t* lut = a.luts + (a.lut_idx ? a.lut_idx[ct] : 0ull) * (uint64_t)(2 * N) + (uint64_t)c * N;
    const uint32_t bt = modswitch(lwe[a.n], LOG2_2N);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const uint32_t src = ((uint32_t)(j1 + R * jcol(e)) + bt) & (2 * N - 1);
      const uint64_t v = lut[src & (N - 1)];
      A[e] = src < (uint32_t)N ? v : 0ull - v;
    }
  }
  const int logB = (int)a.base_log, sb = (int)a.bits;
  const int nrep = 64 - LV * logB;
  const bool split = T > 1;
  const St half = split ? (St)1 << (sb - 1) : (St)0, bmask = split ? ((St)1 << sb) - (St)1 : ~(St)0;
  double max_resid = 0.0;
  pair_barrier();  // tables, tau

#pragma unroll 1
  for (uint32_t i = 0; i < a.n; ++i) {
    // ---- forward: X^{a_i} acc - acc through the LDS copy of both polynomials (row order)
    const uint32_t at = modswitch(lwe[i], LOG2_2N);
    uint64_t* accl = reinterpret_cast<uint64_t*>(E);
#pragma unroll
    for (int e = 0; e < 16; ++e) accl[c * N + j1 * (N / R) + jcol(e)] = A[e];
    pair_barrier();
    St S[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const uint32_t src = ((uint32_t)(j1 + R * jcol(e)) - at) & (2 * N - 1);
      const uint32_t idx = src & (N - 1);
      const uint64_t rv = accl[c * N + (idx & (R - 1)) * (N / R) + (idx >> LOGR)];
      const uint64_t x = (src < (uint32_t)N ? rv : 0ull - rv) - A[e];
      S[e] = (St)(nrep > 0 ? decomp_init(x, nrep) : x);
    }
    pair_barrier();  // the rows are free again
    cplx X[NX][R];
#pragma unroll
    for (int q = 0; q < LV; ++q) {
      Dg D[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        if constexpr (W32) D[e] = decomp_next_t<uint32_t>(S[e], logB);
        else D[e] = decomp_next64(S[e], logB);
      }
#pragma unroll
      for (int t = 0; t < T; ++t) {
        cplx v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          // balanced b-bit sub-digit, exact: D - s is a multiple of 2^b
          const Dg s0 = (Dg)(((St)D[e] + half) & bmask) - (Dg)half;
          const Dg s1 = (Dg)(((St)D[e + 8] + half) & bmask) - (Dg)half;
          D[e] = (D[e] - s0) >> sb;
          D[e + 8] = (D[e + 8] - s1) >> sb;
          v[e] = {(double)s0, (double)s1};
        }
        fft512_fwd(v, row, TB, lane);
        if (j1 != 0)
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = cmul(v[e], tau[j1 * 512 + e * 64 + lane]);
#pragma unroll
        for (int e = 0; e < 8; ++e) row[e * 64 + lane] = v[e];
        pair_barrier();
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          cplx u[R];
#pragma unroll
          for (int jj = 0; jj < R; ++jj) u[jj] = E[(r * R + jj) * RS + pos];
          dft_col<R, false>(u);
#pragma unroll
          for (int k1 = 0; k1 < R; ++k1) X[(r * LV + q) * T + t][k1] = u[k1];
        }
        pair_barrier();
      }
    }

    // ---- products and inverse transforms, slot by slot
    const cplx* Gi = a.G + (uint64_t)i * (2 * L * 2 * LV) * M + pos;
    // FUSED_PF: the first output polynomial's t = 0 key values of slot m + 1 (lim = m + 1, q = 0)
    // are loaded while slot m's inverse transforms run, so their L2 latency hides behind them
    cplx kp[FUSED_PF ? 2 : 1][R];
    auto load_kp = [&](int lim) {
      if constexpr (FUSED_PF) {
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
          for (int k1 = 0; k1 < R; ++k1) kp[r][k1] = Gi[(uint64_t)((lim * 2 + r) * LV) * M + k1 * 512];
        __builtin_amdgcn_sched_barrier(0);  // issued here, not sunk to their use
      }
    };
    load_kp(0);
#pragma unroll 1
    for (int m = 0; m < L; ++m) {
#pragma unroll
      for (int cc = 0; cc < 2; ++cc) {
        cplx y[R];
#pragma unroll
        for (int k1 = 0; k1 < R; ++k1) y[k1] = {0.0, 0.0};
#pragma unroll
        for (int t = 0; t < T; ++t) {
          const int lim = m - t;
          if (lim < 0) continue;  // lim < L always (m < L)
#pragma unroll
          for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int q = 0; q < LV; ++q) {
              const cplx* g = Gi + (uint64_t)(((cc * L + lim) * 2 + r) * LV + q) * M;
              const bool pre = FUSED_PF && cc == 0 && t == 0 && q == 0;
#pragma unroll
              for (int k1 = 0; k1 < R; ++k1) {
                const cplx gv = pre ? kp[FUSED_PF ? r : 0][k1] : g[k1 * 512], xv = X[(r * LV + q) * T + t][k1];
                y[k1].re = __builtin_fma(xv.re, gv.re, __builtin_fma(-xv.im, gv.im, y[k1].re));
                y[k1].im = __builtin_fma(xv.re, gv.im, __builtin_fma(xv.im, gv.re, y[k1].im));
              }
            }
        }
        dft_col<R, true>(y);
#pragma unroll
        for (int jj = 0; jj < R; ++jj) E[(cc * R + jj) * RS + pos] = y[jj];
      }
      if (m + 1 < L) load_kp(m + 1);
      pair_barrier();
      cplx v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = row[e * 64 + lane];
      wave_lds_fence();  // the row is read whole before the transform writes its scratch over it
      if (j1 != 0)
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = cmulc(v[e], tau[j1 * 512 + e * 64 + lane]);
      cplx gi2[4];
      inv_p2_stage_tw(gi2, TB, lane & 7);
      fft512_inv_tw(v, row, TB, lane, gi2, 0);
      // slot shifts stay below 64: the top limb is 64 - (L - 1) b bits wide (key_format)
      const uint32_t sh = ((uint32_t)m * a.bits) & 63u;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const double tr = v[e].re + RND_MAGIC, ti = v[e].im + RND_MAGIC;
        max_resid = fmax(max_resid, fmax(fabs(v[e].re - (tr - RND_MAGIC)), fabs(v[e].im - (ti - RND_MAGIC))));
        A[e] += ((uint64_t)__double_as_longlong(tr) - RND_MAGIC_BITS) << sh;
        A[e + 8] += ((uint64_t)__double_as_longlong(ti) - RND_MAGIC_BITS) << sh;
      }
      pair_barrier();  // the rows are written by the next slot's column DFTs
    }
  }

  // sample extract (nth = 0): out[j] = -A_0[N - j] (j > 0), out[0] = A_0[0], out[N] = A_1[0]
  const uint64_t orow = a.out_idx ? a.out_idx[ct] : ct;
  uint64_t* o = a.out + orow * (uint64_t)(N + 1);
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const uint32_t j = (uint32_t)(j1 + R * jcol(e));
    if (c == 0)
      o[(N - j) & (N - 1)] = j == 0 ? A[e] : 0ull - A[e];
    else if (j == 0)
      o[N] = A[e];
  }
  if (a.resid) {
    for (int off = 32; off > 0; off >>= 1) max_resid = fmax(max_resid, __shfl_xor(max_resid, off));
    if (lane == 0) atomicMax(a.resid, (unsigned long long)__double_as_longlong(max_resid));
  }
}


// ------------------------------------------------------------------------------------------
// gen_coop_kernel: k = 1, N = 8192 (M = 4096, R = 8 rows) with one ciphertext on TWO workgroups
// (round 5; the optimizer's 7-bit rows, v0_last_128:194).  gen_fused_kernel's one-CU form does
// not fit at N = 8192 (both polynomials' rows, X and the accumulator exceed one CU), and the
// two-launch path moves X, Y and the accumulator through HBM every step (9x the algorithmic bytes).
// Here workgroup c of a pair owns GLWE polynomial c: its accumulator (in registers, rows as in
// gen_fused_kernel), the rotation, decomposition and forward transforms of its digits, and the
// inverse transforms of output c.  Per CMUX step the two workgroups exchange, through L2/MALL:
//   X  each keeps the column DFT outputs k1 in [4c, 4c + 4) of its digit spectra and hands the
//      other half to its partner, so each holds BOTH polynomials' spectra at its four k1;
//   Y  per slot m, the products of both outputs at its k1 (key values straight from L2), the
//      other output's half handed over, its own output's eight k1 then go through the inverse
//      column DFT and the row transforms.
// Hand-offs: MI355X_MICROARCH.md / cdna_hip_programming.md §6 Guideline 16, R1: 16-B payload
// stores with sc1 (write-through), every storing wave drained (vmcnt(0)), a workgroup barrier,
// one lane's agent-scope flag store; the consumer's wave 0 polls the flag (relaxed, agent), a
// barrier, then every payload load a 16-B buffer load with sc1.  Events are counted per call
// (flags zeroed by the launcher), placement-independent.  Pairs form by ticket (the order in which
// workgroups start): a workgroup that waits has a running or next-to-start partner, so the launch
// cannot deadlock while two CUs are free for it; every wait is bounded (guard.spin_limit polls,
// then DEV_STATUS_SYNC_TIMEOUT).
// Why no agent-scope release / acquire fences: the LLVM gfx950 model's release
// (buffer_wbl2 sc1, a write-back of the XCD's whole L2, ~1.7-6.5 us) and acquire (buffer_inv sc1,
// ~1.7 us) would cost more than a hand-off's payload at seven hand-offs per CMUX step.  The hand-off
// instead takes the form MI355X_MICROARCH.md §"Workgroup dispatch, XCD placement & inter-workgroup
// visibility" lists as valid without them (its "Valid forms" table, first row, and the Consumer
// bullet's conditions 1-4): EVERY payload byte is stored sc1 (write-through past the producer's L2,
// so the partner's XCD, wherever it is, reads it from memory) and loaded by a buffer sc1 load to
// registers (L1-bypassing; no stale line of this CU's L1 can be hit); every storing wave drains its
// stores (vmcnt(0)) before the workgroup barrier that precedes the one-lane flag store (sc1: an
// agent-scope relaxed store); the consumer's polling wave sees the flag with an sc1 load, the other
// waves load only after the barrier that wave joins; hipMalloc'd buffers, one workgroup per CU.  It
// is the measured form, not an architectural guarantee; the tests compare every hand-off's result
// bit for bit (test_generic_coop_kernel*, the N = 8192 rows in full).
// Arithmetic: gen_fused_kernel's / gen_big_step_kernel's (same transforms, tau, key, rounding), so
// the certified bound (generic_pbs_ok) holds unchanged; the tests compare bit for bit.
// ------------------------------------------------------------------------------------------
struct CoopArgs {
  uint64_t* out;
  const uint64_t* out_idx;
  const uint64_t* in;
  const uint64_t* in_idx;
  const uint64_t* luts;
  const uint64_t* lut_idx;
  const cplx* G;    // Fourier key [n][c][lim][r][q][M], four-step frequency order
  const cplx* Tau;  // column twiddles [R][512]
  unsigned long long* resid;
  cplx* xb;         // X halves [pair][sender][l T][4][512]
  cplx* yb;         // Y halves [pair][sender][2 (slot parity)][4][512]
  uint32_t* flags;  // [pair][sender] published events, then the ticket counter
  uint32_t* status;
  uint32_t spin_limit, base, count, n, base_log, bits, xb_bytes, yb_bytes;
};
constexpr int COOP_R = 8;
// timing-only builds (wrong results): COOP_DIAG_NOSYNC (no hand-off waits or flags),
// COOP_DIAG_NOKEY (no key loads)
#ifndef COOP_DIAG_NOSYNC
#define COOP_DIAG_NOSYNC 0
#endif
#ifndef COOP_DIAG_NOKEY
#define COOP_DIAG_NOKEY 0
#endif
#ifndef COOP_LIMB
#define COOP_LIMB 1  // limb-major products: each key value read once per step (2.53k vs 2.30k PBS/s)
#endif

using v4u = __attribute__((ext_vector_type(4))) unsigned int;
__device__ __forceinline__ v4u cplx_bits(cplx v) {
  const uint64_t r = (uint64_t)__double_as_longlong(v.re), i = (uint64_t)__double_as_longlong(v.im);
  v4u o;
  o.x = (uint32_t)r, o.y = (uint32_t)(r >> 32), o.z = (uint32_t)i, o.w = (uint32_t)(i >> 32);
  return o;
}
__device__ __forceinline__ cplx bits_cplx(v4u o) {
  return {__longlong_as_double((long long)(((uint64_t)o.y << 32) | o.x)),
          __longlong_as_double((long long)(((uint64_t)o.w << 32) | o.z))};
}

template <int LV, int T, int L, bool W32>
__global__ void __launch_bounds__(512) gen_coop_kernel(CoopArgs a) {
  constexpr int R = COOP_R, M = R * 512, N = 2 * M, RS = 576, LOGR = 3, LOG2_2N = Geo<M>::LOG + 2;
  constexpr int NXH = LV * T;  // digit spectra of one polynomial per step
  constexpr uint32_t SC1 = 16;  // cache-policy aux bit: sc1 (write-through stores, L1-bypassing loads)
  using St = typename std::conditional<W32, uint32_t, uint64_t>::type;
  using Dg = typename std::conditional<W32, int32_t, int64_t>::type;
  __shared__ cplx lds[R * RS + FFT512_TABLE_ENTRIES + R * 512];
  __shared__ uint32_t sh_ticket;
  cplx* E = lds;
  cplx* tab = lds + R * RS;
  cplx* tau = tab + FFT512_TABLE_ENTRIES;
  build_fft512_tables(tab, threadIdx.x, 512);
  for (int x = threadIdx.x; x < R * 512; x += 512) tau[x] = a.Tau[x];
  if (threadIdx.x == 0)
    sh_ticket = __hip_atomic_fetch_add(a.flags + 2 * a.count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const Fft512Tables TB = fft512_tables_at(tab);
  const uint32_t tk = __builtin_amdgcn_readfirstlane(sh_ticket);
  const uint32_t p = tk >> 1;
  const int c = (int)(tk & 1u);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int j1 = w, pos = threadIdx.x;
  cplx* row = E + w * RS;
  const uint64_t ct = a.base + p;
  const uint64_t in_row = a.in_idx ? a.in_idx[ct] : ct;
  const uint64_t* lwe = a.in + in_row * (uint64_t)(a.n + 1);
  auto jcol = [&](int e) { return lane + 64 * (e & 7) + 512 * (e >> 3); };
  uint64_t A[16];
  {
    const uint64_t* lut = a.luts + (a.lut_idx ? a.lut_idx[ct] : 0ull) * (uint64_t)(2 * N) + (uint64_t)c * N;
    const uint32_t bt = modswitch(lwe[a.n], LOG2_2N);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const uint32_t src = ((uint32_t)(j1 + R * jcol(e)) + bt) & (2 * N - 1);
      const uint64_t v = lut[src & (N - 1)];
      A[e] = src < (uint32_t)N ? v : 0ull - v;
    }
  }
  const int logB = (int)a.base_log, sb = (int)a.bits;
  const int nrep = 64 - LV * logB;
  const bool split = T > 1;
  const St half = split ? (St)1 << (sb - 1) : (St)0, bmask = split ? ((St)1 << sb) - (St)1 : ~(St)0;
  double max_resid = 0.0;

  // ---- hand-off endpoints (byte offsets: per-lane voffset of the sc1 buffer accesses)
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(a.xb, 0, (int)a.xb_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(a.yb, 0, (int)a.yb_bytes, 0x00020000);
  const uint32_t x_out = (p * 2 + c) * (uint32_t)(NXH * 4 * 512 * 16) + pos * 16;
  const uint32_t x_in = (p * 2 + (1 - c)) * (uint32_t)(NXH * 4 * 512 * 16) + pos * 16;
  const uint32_t y_out = (p * 2 + c) * (uint32_t)(2 * 4 * 512 * 16) + pos * 16;
  const uint32_t y_in = (p * 2 + (1 - c)) * (uint32_t)(2 * 4 * 512 * 16) + pos * 16;
  uint32_t* myflag = a.flags + 2 * p + c;
  const uint32_t* pflag = a.flags + 2 * p + (1 - c);
  auto publish = [&](uint32_t ev) __attribute__((always_inline)) {
    if (COOP_DIAG_NOSYNC) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(myflag, ev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  auto consume = [&](uint32_t ev) __attribute__((always_inline)) {
    if (COOP_DIAG_NOSYNC) return;
    if (w == 0) {
      for (uint32_t it = 0;; ++it) {
        if (__hip_atomic_load(pflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= ev) break;
        if (it >= a.spin_limit) {
          if (lane == 0) __hip_atomic_fetch_or(a.status, DEV_STATUS_SYNC_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // payload loads stay below the poll
  };
  pair_barrier();  // tables, tau

#pragma unroll 1
  for (uint32_t i = 0; i < a.n; ++i) {
    const uint32_t ev0 = i * (uint32_t)(L + 1);
    // ---- forward: X^{a_i} acc - acc through the LDS copy of polynomial c (row order)
    const uint32_t at = modswitch(lwe[i], LOG2_2N);
    uint64_t* accl = reinterpret_cast<uint64_t*>(E);
#pragma unroll
    for (int e = 0; e < 16; ++e) accl[j1 * (N / R) + jcol(e)] = A[e];
    pair_barrier();
    St S[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const uint32_t src = ((uint32_t)(j1 + R * jcol(e)) - at) & (2 * N - 1);
      const uint32_t idx = src & (N - 1);
      const uint64_t rv = accl[(idx & (R - 1)) * (N / R) + (idx >> LOGR)];
      const uint64_t x = (src < (uint32_t)N ? rv : 0ull - rv) - A[e];
      S[e] = (St)(nrep > 0 ? decomp_init(x, nrep) : x);
    }
    pair_barrier();  // the rows are free again
    // X[r][s][kh]: r = 0 my polynomial, r = 1 the partner's; s = q T + t; frequencies (4 c + kh) 512 + pos
    cplx X[2][NXH][4];
#pragma unroll
    for (int q = 0; q < LV; ++q) {
      Dg D[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        if constexpr (W32) D[e] = decomp_next_t<uint32_t>(S[e], logB);
        else D[e] = decomp_next64(S[e], logB);
      }
#pragma unroll
      for (int t = 0; t < T; ++t) {
        cplx v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const Dg s0 = (Dg)(((St)D[e] + half) & bmask) - (Dg)half;
          const Dg s1 = (Dg)(((St)D[e + 8] + half) & bmask) - (Dg)half;
          D[e] = (D[e] - s0) >> sb;
          D[e + 8] = (D[e + 8] - s1) >> sb;
          v[e] = {(double)s0, (double)s1};
        }
        fft512_fwd(v, row, TB, lane);
        if (j1 != 0)
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = cmul(v[e], tau[j1 * 512 + e * 64 + lane]);
#pragma unroll
        for (int e = 0; e < 8; ++e) row[e * 64 + lane] = v[e];
        pair_barrier();
        cplx u[R];
#pragma unroll
        for (int jj = 0; jj < R; ++jj) u[jj] = E[jj * RS + pos];
        dft_col<R, false>(u);
        const int s = q * T + t;
        // (uniform branches: a select on c would become an indexed, scratch-backed array)
        auto keep_send = [&](auto CC) __attribute__((always_inline)) {
          constexpr int C0 = decltype(CC)::value;
#pragma unroll
          for (int kh = 0; kh < 4; ++kh) {
            X[0][s][kh] = u[4 * C0 + kh];
            __builtin_amdgcn_raw_buffer_store_b128(cplx_bits(u[4 * (1 - C0) + kh]), xr,
                                                   x_out + (uint32_t)((s * 4 + kh) * 512 * 16), 0, SC1);
          }
        };
        if (c) keep_send(std::integral_constant<int, 1>{});
        else keep_send(std::integral_constant<int, 0>{});
        pair_barrier();
      }
    }
    publish(ev0 + 1);
    consume(ev0 + 1);
#pragma unroll
    for (int s = 0; s < NXH; ++s)
#pragma unroll
      for (int kh = 0; kh < 4; ++kh)
        X[1][s][kh] = bits_cplx(__builtin_amdgcn_raw_buffer_load_b128(xr, x_in + (uint32_t)((s * 4 + kh) * 512 * 16), 0, SC1));

    // ---- products and inverse transforms, slot by slot (the key values straight from L2; loading
    //      the next slot's ahead, across the hand-off and inverse, spills at two waves per SIMD and
    //      measured slower: 1.94k vs 2.27k PBS/s, profiles/r05/coop_ab.json)
    const cplx* Gi = a.G + (uint64_t)i * (2 * L * 2 * LV) * M + (uint64_t)(4 * c * 512) + pos;
    cplx Yn[2][4];  // COOP_LIMB: slot m's t = 1 terms (limb m - 1), carried from the previous slot
#pragma unroll 1
    for (int m = 0; m < L; ++m) {
      cplx y[2][4];
#pragma unroll
      for (int cc = 0; cc < 2; ++cc)
#pragma unroll
        for (int kh = 0; kh < 4; ++kh) y[cc][kh] = COOP_LIMB && T == 2 && m > 0 ? Yn[cc][kh] : cplx{0.0, 0.0};
      if constexpr (COOP_LIMB && T == 2) {
        // limb m's key values once: its t = 0 terms into slot m, its t = 1 terms into slot m + 1
        // (half the key bytes of the slot-major form); one output's values in flight at a time.
        // (The last limb's t = 1 terms land in slot L, zero mod 2^64; skipping them in a second
        // copy of the loop spilled 13 VGPRs.)
#pragma unroll
        for (int cc = 0; cc < 2; ++cc) {
#pragma unroll
          for (int kh = 0; kh < 4; ++kh) Yn[cc][kh] = {0.0, 0.0};
#pragma unroll
          for (int r = 0; r < 2; ++r) {
            const int rr = r == 0 ? c : 1 - c;
#pragma unroll
            for (int q = 0; q < LV; ++q) {
              const cplx* g = Gi + (uint64_t)(((cc * L + m) * 2 + rr) * LV + q) * M;
#pragma unroll
              for (int kh = 0; kh < 4; ++kh) {
                const cplx x0 = X[r][q * T][kh], x1 = X[r][q * T + 1][kh];
                const cplx gv = COOP_DIAG_NOKEY ? cplx{x0.im, (double)m} : g[kh * 512];
                y[cc][kh].re = __builtin_fma(x0.re, gv.re, __builtin_fma(-x0.im, gv.im, y[cc][kh].re));
                y[cc][kh].im = __builtin_fma(x0.re, gv.im, __builtin_fma(x0.im, gv.re, y[cc][kh].im));
                Yn[cc][kh].re = __builtin_fma(x1.re, gv.re, __builtin_fma(-x1.im, gv.im, Yn[cc][kh].re));
                Yn[cc][kh].im = __builtin_fma(x1.re, gv.im, __builtin_fma(x1.im, gv.re, Yn[cc][kh].im));
              }
            }
          }
          // one output's key values in flight at a time (without this barrier: 2.34k vs 2.51k)
          __builtin_amdgcn_sched_barrier(0);
        }
      }
#pragma unroll
      for (int t = 0; t < (COOP_LIMB && T == 2 ? 0 : T); ++t) {
        const int lim = m - t;
        if (lim < 0) continue;
#pragma unroll
        for (int cc = 0; cc < 2; ++cc)
#pragma unroll
          for (int r = 0; r < 2; ++r) {
            const int rr = r == 0 ? c : 1 - c;  // the key row of X[r]
#pragma unroll
            for (int q = 0; q < LV; ++q) {
              const cplx* g = Gi + (uint64_t)(((cc * L + lim) * 2 + rr) * LV + q) * M;
#pragma unroll
              for (int kh = 0; kh < 4; ++kh) {
                const cplx xv = X[r][q * T + t][kh];
                const cplx gv = COOP_DIAG_NOKEY ? cplx{xv.im, (double)lim} : g[kh * 512];
                y[cc][kh].re = __builtin_fma(xv.re, gv.re, __builtin_fma(-xv.im, gv.im, y[cc][kh].re));
                y[cc][kh].im = __builtin_fma(xv.re, gv.im, __builtin_fma(xv.im, gv.re, y[cc][kh].im));
              }
            }
          }
      }
      // the partner's output at my k1 to the partner; its half of mine back
      const uint32_t par = (uint32_t)(m & 1) * (4 * 512 * 16);
      auto send = [&](auto CC) __attribute__((always_inline)) {
        constexpr int C0 = decltype(CC)::value;
#pragma unroll
        for (int kh = 0; kh < 4; ++kh)
          __builtin_amdgcn_raw_buffer_store_b128(cplx_bits(y[1 - C0][kh]), yr, y_out + par + (uint32_t)(kh * 512 * 16),
                                                 0, SC1);
      };
      if (c) send(std::integral_constant<int, 1>{});
      else send(std::integral_constant<int, 0>{});
      publish(ev0 + 2 + (uint32_t)m);
      consume(ev0 + 2 + (uint32_t)m);
      cplx u[R];
      auto gather = [&](auto CC) __attribute__((always_inline)) {
        constexpr int C0 = decltype(CC)::value;
#pragma unroll
        for (int kh = 0; kh < 4; ++kh) {
          u[4 * C0 + kh] = y[C0][kh];
          u[4 * (1 - C0) + kh] =
              bits_cplx(__builtin_amdgcn_raw_buffer_load_b128(yr, y_in + par + (uint32_t)(kh * 512 * 16), 0, SC1));
        }
      };
      if (c) gather(std::integral_constant<int, 1>{});
      else gather(std::integral_constant<int, 0>{});
      dft_col<R, true>(u);
#pragma unroll
      for (int jj = 0; jj < R; ++jj) E[jj * RS + pos] = u[jj];
      pair_barrier();
      cplx v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = row[e * 64 + lane];
      wave_lds_fence();  // the row is read whole before the transform writes its scratch over it
      if (j1 != 0)
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = cmulc(v[e], tau[j1 * 512 + e * 64 + lane]);
      cplx gi2[4];
      inv_p2_stage_tw(gi2, TB, lane & 7);
      fft512_inv_tw(v, row, TB, lane, gi2, 0);
      const uint32_t sh = ((uint32_t)m * a.bits) & 63u;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const double tr = v[e].re + RND_MAGIC, ti = v[e].im + RND_MAGIC;
        max_resid = fmax(max_resid, fmax(fabs(v[e].re - (tr - RND_MAGIC)), fabs(v[e].im - (ti - RND_MAGIC))));
        A[e] += ((uint64_t)__double_as_longlong(tr) - RND_MAGIC_BITS) << sh;
        A[e + 8] += ((uint64_t)__double_as_longlong(ti) - RND_MAGIC_BITS) << sh;
      }
      pair_barrier();  // the rows are written by the next slot's column DFTs
    }
  }

  // sample extract (nth = 0): out[j] = -A_0[N - j] (j > 0), out[0] = A_0[0], out[N] = A_1[0]
  const uint64_t orow = a.out_idx ? a.out_idx[ct] : ct;
  uint64_t* o = a.out + orow * (uint64_t)(N + 1);
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const uint32_t j = (uint32_t)(j1 + R * jcol(e));
    if (c == 0)
      o[(N - j) & (N - 1)] = j == 0 ? A[e] : 0ull - A[e];
    else if (j == 0)
      o[N] = A[e];
  }
  if (a.resid) {
    for (int off = 32; off > 0; off >>= 1) max_resid = fmax(max_resid, __shfl_xor(max_resid, off));
    if (lane == 0) atomicMax(a.resid, (unsigned long long)__double_as_longlong(max_resid));
  }
}

// Y[ct][c][m][f] = sum over (r, q, t) with 0 <= m - t < L of X[ct][r][q][t][f] * G_i[c][m-t][r][q][f]
struct MacArgs {
  const cplx* X;
  cplx* Y;
  const cplx* G;  // Fourier key [n][K1 c][L lim][K1 r][l q][M]
  uint32_t count, k, level, limbs, subs, M;
  uint32_t i;  // GGSW index (LWE mask position)
};

// Any number of terms: the key values of GEN_MAX_TERMS terms at a time in registers, the slot
// sum carried through Y between the chunks (each thread re-reads only what it wrote).
__global__ void __launch_bounds__(256) gen_mac_kernel(MacArgs a) {
  const uint32_t f = blockIdx.x * 256 + threadIdx.x;
  const uint32_t K1 = a.k + 1, L = a.limbs, T = a.subs;
  const uint32_t c = blockIdx.y / L, m = blockIdx.y % L;
  const uint32_t terms = K1 * a.level * T;
  const uint64_t M = a.M;
  if (f >= M) return;
  const uint32_t ct0 = blockIdx.z * MAC_CTS;
#pragma unroll 1
  for (uint32_t x0 = 0; x0 < terms; x0 += GEN_MAX_TERMS) {
    cplx kv[GEN_MAX_TERMS];
#pragma unroll
    for (int x = 0; x < GEN_MAX_TERMS; ++x) {
      kv[x] = {0.0, 0.0};
      const uint32_t xx = x0 + x;
      if (xx < terms) {
        const uint32_t t = xx % T, rq = xx / T;  // xx = (r l + q) T + t
        if (m >= t && m - t < L) kv[x] = a.G[((((uint64_t)a.i * K1 + c) * L + (m - t)) * K1 * a.level + rq) * M + f];
      }
    }
    for (uint32_t ct = ct0; ct < ct0 + MAC_CTS && ct < a.count; ++ct) {
      const cplx* Xct = a.X + (uint64_t)ct * terms * M + f;
      cplx* Yp = a.Y + (((uint64_t)ct * K1 + c) * L + m) * M + f;
      cplx y = x0 ? *Yp : cplx{0.0, 0.0};
#pragma unroll
      for (int x = 0; x < GEN_MAX_TERMS; ++x) {
        if (x0 + x < terms) {
          const cplx xv = Xct[(uint64_t)(x0 + x) * M];
          y.re = __builtin_fma(xv.re, kv[x].re, __builtin_fma(-xv.im, kv[x].im, y.re));
          y.im = __builtin_fma(xv.re, kv[x].im, __builtin_fma(xv.im, kv[x].re, y.im));
        }
      }
      *Yp = y;
    }
  }
}

// Same product, one thread per (frequency, output polynomial c) computing all L slots: each X
// value is read once per output polynomial instead of once per (polynomial, slot), and the
// key values of the thread (L x K1 l) stay in registers across the ciphertext tile.
template <int KL, int L, int T>
__global__ void __launch_bounds__(256) gen_mac2_kernel(MacArgs a) {
  const uint32_t f = blockIdx.x * 256 + threadIdx.x;
  const uint32_t c = blockIdx.y, K1 = a.k + 1;
  const uint64_t M = a.M;
  if (f >= M) return;
  cplx kv[L][KL];
#pragma unroll
  for (int lim = 0; lim < L; ++lim)
#pragma unroll
    for (int rq = 0; rq < KL; ++rq) kv[lim][rq] = a.G[((((uint64_t)a.i * K1 + c) * L + lim) * KL + rq) * M + f];
  const uint32_t ct0 = blockIdx.z * MAC_CTS;
  for (uint32_t ct = ct0; ct < ct0 + MAC_CTS && ct < a.count; ++ct) {
    const cplx* Xct = a.X + (uint64_t)ct * KL * T * M + f;
    cplx xv[KL][T];
#pragma unroll
    for (int rq = 0; rq < KL; ++rq)
#pragma unroll
      for (int t = 0; t < T; ++t) xv[rq][t] = Xct[(uint64_t)(rq * T + t) * M];
    cplx* Yct = a.Y + ((uint64_t)ct * K1 + c) * L * M + f;
#pragma unroll
    for (int m = 0; m < L; ++m) {
      cplx y = {0.0, 0.0};
#pragma unroll
      for (int t = 0; t < T; ++t) {
        if (m - t < 0 || m - t >= L) continue;
#pragma unroll
        for (int rq = 0; rq < KL; ++rq) {
          const cplx xg = xv[rq][t], g = kv[m - t][rq];
          y.re = __builtin_fma(xg.re, g.re, __builtin_fma(-xg.im, g.im, y.re));
          y.im = __builtin_fma(xg.re, g.im, __builtin_fma(xg.im, g.re, y.im));
        }
      }
      Yct[(uint64_t)m * M] = y;
    }
  }
}

// k = 1 (two output polynomials): one thread per frequency computing both outputs, so each
// digit spectrum value is read once per tile instead of once per output polynomial (the
// product is HBM-bound on the X/Y spectra at N >= 2048).  (Tried: the next ciphertext's spectra
// double-buffered by LDS-DMA, twice the loads in flight per wave: opt8 823.0 vs 822.7 PBS/s.)
template <int KL, int L, int T>
__global__ void __launch_bounds__(256) gen_mac2k1_kernel(MacArgs a) {
  const uint32_t f = blockIdx.x * 256 + threadIdx.x;
  const uint64_t M = a.M;
  if (f >= M) return;
  cplx kv[2][L][KL];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int lim = 0; lim < L; ++lim)
#pragma unroll
      for (int rq = 0; rq < KL; ++rq)
        kv[c][lim][rq] = a.G[((((uint64_t)a.i * 2 + c) * L + lim) * KL + rq) * M + f];
  const uint32_t ct0 = blockIdx.z * MAC_CTS;
  for (uint32_t ct = ct0; ct < ct0 + MAC_CTS && ct < a.count; ++ct) {
    const cplx* Xct = a.X + (uint64_t)ct * KL * T * M + f;
    cplx xv[KL][T];
#pragma unroll
    for (int rq = 0; rq < KL; ++rq)
#pragma unroll
      for (int t = 0; t < T; ++t) xv[rq][t] = ld_once(&Xct[(uint64_t)(rq * T + t) * M]);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      cplx* Yct = a.Y + ((uint64_t)ct * 2 + c) * L * M + f;
#pragma unroll
      for (int m = 0; m < L; ++m) {
        cplx y = {0.0, 0.0};
#pragma unroll
        for (int t = 0; t < T; ++t) {
          if (m - t < 0 || m - t >= L) continue;
#pragma unroll
          for (int rq = 0; rq < KL; ++rq) {
            const cplx xg = xv[rq][t], g = kv[c][m - t][rq];
            y.re = __builtin_fma(xg.re, g.re, __builtin_fma(-xg.im, g.im, y.re));
            y.im = __builtin_fma(xg.re, g.im, __builtin_fma(xg.im, g.re, y.im));
          }
        }
        #if GEN_NT_STORES
        __builtin_nontemporal_store(y.re, &Yct[(uint64_t)m * M].re);
        __builtin_nontemporal_store(y.im, &Yct[(uint64_t)m * M].im);
#else
        Yct[(uint64_t)m * M] = y;
#endif
      }
    }
  }
}

// launch the register-tiled product for (K1 l, L, T) when instantiated, else the generic one
static bool launch_mac2(const MacArgs& m, uint32_t cnt, hipStream_t st) {
  const uint32_t KL = (m.k + 1) * m.level;
  if (m.k == 1 && m.M >= 1024) {
    const dim3 g1((m.M + 255) / 256, 1, (cnt + MAC_CTS - 1) / MAC_CTS);
#define GEN_MAC2K1(KLv, Lv, Tv)                                                              \
    if (KL == KLv && m.limbs == Lv && m.subs == Tv) {                                        \
      hipLaunchKernelGGL((gen_mac2k1_kernel<KLv, Lv, Tv>), g1, dim3(256), 0, st, m);         \
      return true;                                                                           \
    }
    GEN_MAC2K1(2, 5, 2) GEN_MAC2K1(2, 6, 2) GEN_MAC2K1(4, 6, 2) GEN_MAC2K1(4, 5, 2) GEN_MAC2K1(4, 5, 1)
    GEN_MAC2K1(4, 6, 1)
#undef GEN_MAC2K1
  }
  const dim3 grid((m.M + 255) / 256, m.k + 1, (cnt + MAC_CTS - 1) / MAC_CTS);
#define GEN_MAC2(KLv, Lv, Tv)                                                               \
  if (KL == KLv && m.limbs == Lv && m.subs == Tv) {                                           \
    hipLaunchKernelGGL((gen_mac2_kernel<KLv, Lv, Tv>), grid, dim3(256), 0, st, m);            \
    return true;                                                                              \
  }
#define GEN_MAC2_L(KLv, Tv) GEN_MAC2(KLv, 4, Tv) GEN_MAC2(KLv, 5, Tv) GEN_MAC2(KLv, 6, Tv)
  GEN_MAC2_L(2, 1) GEN_MAC2_L(2, 2) GEN_MAC2_L(3, 1) GEN_MAC2_L(3, 2) GEN_MAC2_L(4, 1) GEN_MAC2_L(4, 2)
  GEN_MAC2_L(5, 1) GEN_MAC2_L(5, 2) GEN_MAC2_L(6, 1) GEN_MAC2_L(6, 2)
  GEN_MAC2(7, 4, 1) GEN_MAC2(7, 5, 1) GEN_MAC2(7, 4, 2) GEN_MAC2(7, 5, 2)
  GEN_MAC2(8, 4, 1) GEN_MAC2(8, 4, 2)
#undef GEN_MAC2_L
#undef GEN_MAC2
  return false;
}

// ------------------------------------------------------------------------------------------
// N <= 512: the whole bootstrap of a tile of C ciphertexts in one workgroup (one launch per
// call).  The accumulator lives in the registers of the polynomial's thread group, the digit
// spectra and one slot spectrum per polynomial in LDS; the key is the only data streamed per
// CMUX step, each key value loaded once per tile and used for its C ciphertexts.  No spectra
// go through HBM (the two-launch path moves ~170 KB of X/Y spectra per ciphertext and step).
// ------------------------------------------------------------------------------------------
struct TileArgs {
  uint64_t* out;
  const uint64_t* out_idx;
  const uint64_t* in;
  const uint64_t* in_idx;
  const uint64_t* luts;
  const uint64_t* lut_idx;
  const cplx* G;  // Fourier key [n][K1 c][L lim][K1 l rq][M]
  const cplx* Wfull;
  const cplx* Z;
  unsigned long long* resid;
  uint32_t count, n, base_log, bits;
};

template <int M, int K1, int KL, int T, int L, int C>
struct TileGeo {
  static constexpr int TH = tile_threads<M>();  // threads per polynomial
  static constexpr int NT = C * K1 * TH;      // threads per workgroup
  static constexpr int BASE = ((C * KL * T + C * K1) * M + tile_tw_entries<M, TH>()) * 16;
  static constexpr bool ZLDS = BASE + M * 16 <= 160 * 1024;  // twist table in LDS when it fits
  static constexpr int LDS = BASE + (ZLDS ? M * 16 : 0);
  static_assert(M <= 512 && NT <= 1024 && LDS <= 160 * 1024, "tile shape");
};

template <int M, int K1, int KL, int T, int L, int C>
__global__ void __launch_bounds__((TileGeo<M, K1, KL, T, L, C>::NT)) gen_tile_kernel(TileArgs a) {
  using TG = TileGeo<M, K1, KL, T, L, C>;
  constexpr int N = 2 * M, TH = TG::TH, VPT = M / TH, NT = TG::NT, LOG2_2N = Geo<M>::LOG + 2;
  constexpr int LV = KL / K1;                           // decomposition levels
  constexpr int ITEMS = K1 * M, IPT = (ITEMS + NT - 1) / NT;  // product items (c, f) per thread
  extern __shared__ __attribute__((aligned(16))) char smem[];
  cplx* Xs = reinterpret_cast<cplx*>(smem);  // [C][KL rq][T t][M] digit spectra (slots sw(f))
  cplx* Ys = Xs + C * KL * T * M;            // [C][K1 c][M] slot spectra / rotation scratch
  cplx* W = Ys + C * K1 * M;  // per-pass twiddles (tile_fft)
  cplx* Zl = W + tile_tw_entries<M, TH>();
  build_tile_tw<M, TH>(W, a.Wfull, threadIdx.x, NT);
  if constexpr (TG::ZLDS)
    for (int e = threadIdx.x; e < M; e += NT) Zl[e] = a.Z[e];
  auto zeta = [&](int j) { return TG::ZLDS ? Zl[j] : a.Z[j]; };
  const int g = threadIdx.x / TH, tid = threadIdx.x % TH;
  const int lct = g / K1, c = g % K1;  // this group's polynomial: (ciphertext of the tile, c)
  const uint32_t ct = blockIdx.x * C + lct;
  const bool live = ct < a.count;  // groups past the batch run on row 0 and write nothing
  const uint64_t row = live ? (a.in_idx ? a.in_idx[ct] : ct) : 0ull;
  const uint64_t* lwe = a.in + row * (uint64_t)(a.n + 1);
  cplx* ybuf = Ys + g * M;
  auto coef = [&](int e) { return (uint32_t)(tid + (e % VPT) * TH + (e / VPT) * M); };
  uint64_t A[2 * VPT];
  double max_resid = 0.0;
  {
    const uint64_t* lut =
        a.luts + (live && a.lut_idx ? a.lut_idx[ct] : 0ull) * (uint64_t)(K1 * N) + (uint64_t)c * N;
    const uint32_t bt = live ? modswitch(lwe[a.n], LOG2_2N) : 0u;
#pragma unroll
    for (int e = 0; e < 2 * VPT; ++e) {
      const uint32_t src = (coef(e) + bt) & (2 * N - 1);
      const uint64_t v = live ? lut[src & (N - 1)] : 0ull;
      A[e] = src < (uint32_t)N ? v : 0ull - v;
    }
  }
  __syncthreads();
  const int logB = (int)a.base_log, sb = (int)a.bits;
  const int nrep = 64 - LV * logB;
  const uint64_t half = 1ull << (sb - 1), bmask = (1ull << sb) - 1ull;
  // key values of product item (c, f) = (it / M, it % M), it = threadIdx.x + s NT, for slot m
  // Output-group items (PAIR): an item = (frequency, CP output polynomials, C / LCS ciphertexts
  // of the tile), so each digit-spectrum value read from LDS serves CP outputs (the product
  // phase is LDS-bound): N = 256: CP = 2, LCS = 2 (55.4k -> 61.3k PBS/s at opt1); N = 1024:
  // CP = 3, LCS = 1 with the key prefetch (512 items, a third of the threads idle in the
  // product).  N = 512 keeps per-(output, frequency) items with shared-frequency reads: CP = 4
  // measured 34.1k (33.5k with prefetch) vs 35.9k.  N = 256 with CP = 3 (512 items): 55.4k.
  constexpr int CP = !TILE_GROUPS ? 0 : (M == 128 && K1 == 6 && C == 4) ? TILE128_CP : (M == 512 && K1 == 3 && C == 2) ? 3 : 0;
#ifndef TILE_GPF
#define TILE_GPF 1  // re-measured round 2: 18.8k with (10 VGPRs spilled) vs 18.3k without
#endif
  constexpr bool GPF = TILE_GPF && M == 512 && CP == 3;  // N = 1024: next-limb key values prefetched (18.5k -> 18.8k)
  constexpr int LCS = M == 128 ? 2 : 1;
  constexpr bool PAIR = CP > 0;
  constexpr int NGRP = PAIR ? K1 / CP : 1, LPG = PAIR ? C / LCS : 1, GITEMS = NGRP * M * LCS;
  static_assert(!PAIR || (K1 % CP == 0 && C % LCS == 0 && GITEMS <= NT), "output groups");
  cplx gn[IPT][KL];
  auto load_key = [&](uint32_t step, int m) {
#pragma unroll
    for (int s = 0; s < IPT; ++s) {
      const int it = threadIdx.x + s * NT;
      if (ITEMS % NT == 0 || it < ITEMS) {
        const cplx* Gp = a.G + (((uint64_t)step * K1 + it / M) * L + m) * (uint64_t)(KL * M) + it % M;
#pragma unroll
        for (int rq = 0; rq < KL; ++rq) gn[s][rq] = Gp[rq * M];
      }
    }
  };
  if (!PAIR && a.n > 0) load_key(0, 0);
  cplx gp2[GPF ? CP : 1][KL];  // GPF: the group's key values of the next limb
  if constexpr (GPF) {
    const int f = threadIdx.x % M, cg = (threadIdx.x / M) % NGRP;
    if (a.n > 0 && (GITEMS == NT || (int)threadIdx.x < GITEMS))
#pragma unroll
      for (int p = 0; p < CP; ++p)
#pragma unroll
        for (int rq = 0; rq < KL; ++rq) gp2[p][rq] = a.G[((uint64_t)(cg * CP + p) * L * KL + rq) * M + f];
  }
#pragma unroll 1
  for (uint32_t i = 0; i < a.n; ++i) {
    // ct1 = X^{ms(a_i)} acc - acc (rotation through this group's slot buffer), decomposition,
    // b-bit sub-digits, forward transforms into the tile's digit spectra
    const uint32_t at = live ? modswitch(lwe[i], LOG2_2N) : 0u;
    uint64_t* rot = reinterpret_cast<uint64_t*>(ybuf);
#pragma unroll
    for (int e = 0; e < 2 * VPT; ++e) rot[coef(e)] = A[e];
    tile_sync<TH>();
    uint64_t S[2 * VPT];
#pragma unroll
    for (int e = 0; e < 2 * VPT; ++e) {
      const uint32_t src = (coef(e) - at) & (2 * N - 1);
      const uint64_t rv = rot[src & (N - 1)];
      const uint64_t x = (src < (uint32_t)N ? rv : 0ull - rv) - A[e];
      S[e] = nrep > 0 ? decomp_init(x, nrep) : x;
    }
#pragma unroll 1
    for (int q = 0; q < LV; ++q) {
      int64_t D[2 * VPT];
#pragma unroll
      for (int e = 0; e < 2 * VPT; ++e) D[e] = decomp_next64(S[e], logB);
#pragma unroll
      for (int t = 0; t < T; ++t) {
        cplx* xs = Xs + ((lct * KL + c * LV + q) * T + t) * M;
#pragma unroll
        for (int e = 0; e < VPT; ++e) {
          int64_t s0 = D[e], s1 = D[e + VPT];
          if constexpr (T > 1) {
            s0 = (int64_t)(((uint64_t)D[e] + half) & bmask) - (int64_t)half;
            s1 = (int64_t)(((uint64_t)D[e + VPT] + half) & bmask) - (int64_t)half;
            D[e] = (D[e] - s0) >> sb;
            D[e + VPT] = (D[e + VPT] - s1) >> sb;
          }
          const int j = tid + e * TH;
          xs[sw(j)] = cmul(cplx{(double)s0, (double)s1}, zeta(j));
        }
        tile_sync<TH>();
        tile_fft<M, TH, false>(xs, W, tid);
      }
    }
    __syncthreads();
    // slots m = 0 .. L-1: Y_m = sum_rq X[rq][0] G[m][rq] + X[rq][1] G[m-1][rq]; inverse; acc += 2^{mb} round
    // limb j's key values serve slot j (sub-digit 0) and slot j + 1 (sub-digit 1); the
    // sub-digit-1 partial of slot j + 1 waits in registers (same thread, same item)
    cplx carry[IPT][C];
    cplx carry2[PAIR ? CP : 1][LPG];
#pragma unroll 1
    for (int m = 0; m < L; ++m) {
      // this limb's key values were loaded one limb ahead; issue the next limb's now
      cplx gk[IPT][KL];
      if constexpr (!PAIR) {
#pragma unroll
        for (int s = 0; s < IPT; ++s)
#pragma unroll
          for (int rq = 0; rq < KL; ++rq) gk[s][rq] = gn[s][rq];
        if (m + 1 < L)
          load_key(i, m + 1);
        else if (i + 1 < a.n)
          load_key(i + 1, 0);
      }
      if constexpr (PAIR) {
        const int it = threadIdx.x;
        if (GITEMS == NT || it < GITEMS) {
          const int f = it % M, r1 = it / M, cg = r1 % NGRP, lg = r1 / NGRP;
          const int sf = sw(f);
          // key values loaded at the start of the limb: a prefetch (24 more VGPRs at N = 256)
          // spills at 768 threads and measured slower (55.2k vs 61.3k PBS/s at opt1)
          cplx g2[CP][KL];
          if constexpr (GPF) {
#pragma unroll
            for (int p = 0; p < CP; ++p)
#pragma unroll
              for (int rq = 0; rq < KL; ++rq) g2[p][rq] = gp2[p][rq];
            const uint32_t ni = m + 1 < L ? i : i + 1;
            const int nm = m + 1 < L ? m + 1 : 0;
            if (ni < a.n) {
#pragma unroll
              for (int p = 0; p < CP; ++p) {
                const cplx* Gp = a.G + (((uint64_t)ni * K1 + cg * CP + p) * L + nm) * (uint64_t)(KL * M) + f;
#pragma unroll
                for (int rq = 0; rq < KL; ++rq) gp2[p][rq] = Gp[rq * M];
              }
            }
          } else {
#pragma unroll
            for (int p = 0; p < CP; ++p) {
              const cplx* Gp = a.G + (((uint64_t)i * K1 + cg * CP + p) * L + m) * (uint64_t)(KL * M) + f;
#pragma unroll
              for (int rq = 0; rq < KL; ++rq) g2[p][rq] = Gp[rq * M];
            }
          }
#pragma unroll
          for (int lcl = 0; lcl < LPG; ++lcl) {
            const int lc = lg * LPG + lcl;
            // sub-digit 0 (completes slot m), then sub-digit 1 (starts slot m + 1): one
            // spectrum row in registers at a time
            cplx y[CP];
#pragma unroll
            for (int p = 0; p < CP; ++p) y[p] = (T > 1 && m > 0) ? carry2[p][lcl] : cplx{0.0, 0.0};
#pragma unroll
            for (int rq = 0; rq < KL; ++rq) {
              const cplx xv = Xs[((lc * KL + rq) * T) * M + sf];
#pragma unroll
              for (int p = 0; p < CP; ++p) {
                const cplx gv = g2[p][rq];
                y[p].re = __builtin_fma(xv.re, gv.re, __builtin_fma(-xv.im, gv.im, y[p].re));
                y[p].im = __builtin_fma(xv.re, gv.im, __builtin_fma(xv.im, gv.re, y[p].im));
              }
            }
#pragma unroll
            for (int p = 0; p < CP; ++p) Ys[(lc * K1 + cg * CP + p) * M + sf] = y[p];
            if constexpr (T > 1) {
              cplx z[CP];
#pragma unroll
              for (int p = 0; p < CP; ++p) z[p] = {0.0, 0.0};
#pragma unroll
              for (int rq = 0; rq < KL; ++rq) {
                const cplx xv = Xs[((lc * KL + rq) * T + 1) * M + sf];
#pragma unroll
                for (int p = 0; p < CP; ++p) {
                  const cplx gv = g2[p][rq];
                  z[p].re = __builtin_fma(xv.re, gv.re, __builtin_fma(-xv.im, gv.im, z[p].re));
                  z[p].im = __builtin_fma(xv.re, gv.im, __builtin_fma(xv.im, gv.re, z[p].im));
                }
              }
#pragma unroll
              for (int p = 0; p < CP; ++p) carry2[p][lcl] = z[p];
            }
          }
        }
      } else if constexpr (NT % M == 0 && IPT > 1) {
        // a thread's items share one frequency (it % M = threadIdx.x % M): each digit spectrum
        // value is read from LDS once per limb for all its output polynomials
        const int sf = sw(threadIdx.x % M);
#pragma unroll
        for (int lc = 0; lc < C; ++lc) {
          cplx x0[KL], x1[KL];
#pragma unroll
          for (int rq = 0; rq < KL; ++rq) {
            x0[rq] = Xs[((lc * KL + rq) * T) * M + sf];
            if constexpr (T > 1) x1[rq] = Xs[((lc * KL + rq) * T + 1) * M + sf];
          }
#pragma unroll
          for (int s = 0; s < IPT; ++s) {
            const int cc = (threadIdx.x + s * NT) / M;
            cplx y = (T > 1 && m > 0) ? carry[s][lc] : cplx{0.0, 0.0};
#pragma unroll
            for (int rq = 0; rq < KL; ++rq) {
              const cplx xv = x0[rq], gv = gk[s][rq];
              y.re = __builtin_fma(xv.re, gv.re, __builtin_fma(-xv.im, gv.im, y.re));
              y.im = __builtin_fma(xv.re, gv.im, __builtin_fma(xv.im, gv.re, y.im));
            }
            Ys[(lc * K1 + cc) * M + sf] = y;
            if constexpr (T > 1) {
              cplx z = {0.0, 0.0};
#pragma unroll
              for (int rq = 0; rq < KL; ++rq) {
                const cplx xv = x1[rq], gv = gk[s][rq];
                z.re = __builtin_fma(xv.re, gv.re, __builtin_fma(-xv.im, gv.im, z.re));
                z.im = __builtin_fma(xv.re, gv.im, __builtin_fma(xv.im, gv.re, z.im));
              }
              carry[s][lc] = z;
            }
          }
        }
      } else {
#pragma unroll
      for (int s = 0; s < IPT; ++s) {
        const int it = threadIdx.x + s * NT;
        if (ITEMS % NT == 0 || it < ITEMS) {
          const int cc = it / M, f = it % M;
          const int sf = sw(f);
#pragma unroll
          for (int lc = 0; lc < C; ++lc) {
            cplx y = (T > 1 && m > 0) ? carry[s][lc] : cplx{0.0, 0.0};
#pragma unroll
            for (int rq = 0; rq < KL; ++rq) {
              const cplx xv = Xs[((lc * KL + rq) * T) * M + sf], gv = gk[s][rq];
              y.re = __builtin_fma(xv.re, gv.re, __builtin_fma(-xv.im, gv.im, y.re));
              y.im = __builtin_fma(xv.re, gv.im, __builtin_fma(xv.im, gv.re, y.im));
            }
            Ys[(lc * K1 + cc) * M + sf] = y;
            if constexpr (T > 1) {
              cplx z = {0.0, 0.0};
#pragma unroll
              for (int rq = 0; rq < KL; ++rq) {
                const cplx xv = Xs[((lc * KL + rq) * T + 1) * M + sf], gv = gk[s][rq];
                z.re = __builtin_fma(xv.re, gv.re, __builtin_fma(-xv.im, gv.im, z.re));
                z.im = __builtin_fma(xv.re, gv.im, __builtin_fma(xv.im, gv.re, z.im));
              }
              carry[s][lc] = z;
            }
          }
        }
      }
      }
      __syncthreads();
      tile_fft<M, TH, true>(ybuf, W, tid);
      const uint32_t sh = m * a.bits;
#pragma unroll
      for (int e = 0; e < VPT; ++e) {
        const int j = tid + e * TH;
        const cplx z = cmulc(ybuf[sw(j)], zeta(j));
        const double tr = z.re + RND_MAGIC, ti = z.im + RND_MAGIC;
        max_resid = fmax(max_resid, fmax(fabs(z.re - (tr - RND_MAGIC)), fabs(z.im - (ti - RND_MAGIC))));
        if (sh < 64) {
          A[e] += ((uint64_t)__double_as_longlong(tr) - RND_MAGIC_BITS) << sh;
          A[e + VPT] += ((uint64_t)__double_as_longlong(ti) - RND_MAGIC_BITS) << sh;
        }
      }
      __syncthreads();
    }
  }
  // sample extract (nth = 0): out[r N + 0] = A_r[0], out[r N + j] = -A_r[N - j], out[k N] = B[0]
  if (live) {
    const uint64_t orow = a.out_idx ? a.out_idx[ct] : ct;
    uint64_t* o = a.out + orow * ((uint64_t)(K1 - 1) * N + 1);
#pragma unroll
    for (int e = 0; e < 2 * VPT; ++e) {
      const uint32_t j = coef(e);
      if (c < K1 - 1)
        o[(uint64_t)c * N + ((N - j) & (N - 1))] = j == 0 ? A[e] : 0ull - A[e];
      else if (j == 0)
        o[(uint64_t)(K1 - 1) * N] = A[e];
    }
  }
  if (a.resid) {
    for (int off = 32; off > 0; off >>= 1) max_resid = fmax(max_resid, __shfl_xor(max_resid, off));
    if ((threadIdx.x & 63) == 0) atomicMax(a.resid, (unsigned long long)__double_as_longlong(max_resid));
  }
}

// sample extract (nth = 0): out[r N + 0] = A_r[0], out[r N + j] = -A_r[N - j], out[k N] = B[0].
// rlog > 0: accumulators in the four-step row order (coefficient n at (n mod R) N/R + n / R).
__global__ void gen_extract_kernel(uint64_t* out, const uint64_t* out_idx, const uint64_t* acc, uint32_t base,
                                   uint32_t count, uint32_t k, uint32_t N, uint32_t rlog) {
  const uint64_t width = (uint64_t)k * N + 1;
  const uint64_t total = width * count;
  const uint32_t rmask = (1u << rlog) - 1u, rowlen = N >> rlog;
  auto at = [&](uint32_t j) { return (j & rmask) * rowlen + (j >> rlog); };
  for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < total; g += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t ct = (uint32_t)(g / width), e = (uint32_t)(g % width);
    const uint32_t s = base + ct;
    const uint64_t orow = out_idx ? out_idx[s] : s;
    const uint64_t* A = acc + (uint64_t)ct * (k + 1) * N;
    uint64_t v;
    if (e == k * N) {
      v = A[(uint64_t)k * N];  // coefficient 0 sits at 0 in either order
    } else {
      const uint32_t r = e / N, j = e % N;
      const uint64_t x = A[(uint64_t)r * N + at((N - j) & (N - 1))];
      v = j == 0 ? x : 0ull - x;
    }
    out[orow * width + e] = v;
  }
}

// Fourier key: G[i][c][lim][r][q][f] = FFT(twist(limb_lim(std[i][l-1-q][r][c])))[f] / M, frequencies
// in natural order, or (perm) in the four-step order of gen_big_step_kernel: position p holds
// frequency big_freq(p)
template <int M>
__global__ void __launch_bounds__(Geo<M>::THREADS) gen_convert_kernel(cplx* G, const uint64_t* src, const cplx* Wfull,
                                                                        const cplx* Wlo,
                                                                        const cplx* Whi, const cplx* Z, uint32_t k,
                                                                        uint32_t level, uint32_t bits, uint32_t limbs,
                                                                        uint32_t perm, unsigned long long* smax) {
  constexpr int N = 2 * M, TH = Geo<M>::THREADS, VPT = Geo<M>::VPT;
  constexpr bool PP = M <= 4096;  // as gen_step_kernel
  __shared__ cplx buf[M + (PP ? tile_tw_entries<M, TH>() : tw_entries<M>())];
  cplx* W = buf + M;
  if constexpr (PP)
    build_tile_tw<M, TH>(W, Wfull, threadIdx.x, TH);
  else
    load_twiddles<M>(W, Wfull, Wlo, Whi, threadIdx.x, TH);
  __syncthreads();
  const int tid = threadIdx.x;
  const uint32_t K1 = k + 1;
  // block = one standard polynomial [i][v][row r][col c] (concrete-cpu bootstrap.rs:417-429)
  uint64_t p = blockIdx.x;
  const uint32_t c = p % K1;
  p /= K1;
  const uint32_t r = p % K1;
  p /= K1;
  const uint32_t v = p % level;
  const uint64_t i = p / level;
  const uint32_t q = level - 1 - v;
  const uint64_t* g = src + (uint64_t)blockIdx.x * N;
  uint64_t gv[2 * VPT];
#pragma unroll
  for (int e = 0; e < 2 * VPT; ++e) gv[e] = g[tid + (e % VPT) * TH + (e / VPT) * M];
  const double scale = 1.0 / (double)M;
  double m2 = 0.0;  // max |G|^2 of the stored values (keycheck.hpp)
#pragma unroll 1
  for (uint32_t lim = 0; lim < limbs; ++lim) {
    // balanced limbs: g = sum_j 2^{jb} g_j mod 2^64, |g_j| <= 2^(b-1); the top limb only matters
    // mod 2^(64 - (L-1) b), so it is balanced in that width (no DC offset in its spectrum)
    const uint32_t w = lim + 1 < limbs ? bits : 64 - (limbs - 1) * bits;
    const uint64_t half = 1ull << (w - 1);
    const uint64_t bmask = (1ull << w) - 1ull;
#pragma unroll
    for (int e = 0; e < VPT; ++e) {
      const int64_t s0 = (int64_t)((gv[e] + half) & bmask) - (int64_t)half;
      const int64_t s1 = (int64_t)((gv[e + VPT] + half) & bmask) - (int64_t)half;
      gv[e] = (gv[e] - (uint64_t)s0) >> bits;
      gv[e + VPT] = (gv[e + VPT] - (uint64_t)s1) >> bits;
      const int j = tid + e * TH;
      buf[sw(j)] = cmul(cplx{(double)s0, (double)s1}, Z[j]);
    }
    __syncthreads();
    if constexpr (PP)
      tile_fft<M, TH, false>(buf, W, tid);
    else
      fft_block<M, false>(buf, W, tid);
    cplx* dst = G + ((((i * K1 + c) * limbs + lim) * K1 + r) * level + q) * (uint64_t)M;
#pragma unroll
    for (int e = 0; e < VPT; ++e) {
      const uint32_t p = tid + e * TH;
      const cplx x = buf[sw(perm ? (int)big_freq(p) : (int)p)];
      dst[p] = {x.re * scale, x.im * scale};
      m2 = fmax(m2, spec_mag2(x.re * scale, x.im * scale));
    }
    __syncthreads();
  }
  spec_max_commit(smax, m2);
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
struct Tables {
  cplx* Wfull = nullptr;  // e^{-2 pi i j/M}, j < M
  cplx* Wlo = nullptr;  // e^{-2 pi i j/M}, j < TW_LO
  cplx* Whi = nullptr;  // e^{-2 pi i j TW_LO/M}, j < max(1, M/TW_LO)
  cplx* Z = nullptr;    // zeta^j, j < M
  cplx* Tau = nullptr;  // four-step column twiddles tau(j1, k2(pos)) [R][512] (M >= 1024)
  cplx* WR = nullptr;   // w_R^x = exp(-2 pi i x / R), x < R (N >= 32768: the column-class combine)
};

// Whether N runs on the four-step step kernel (and its keys are converted to the four-step
// frequency order).  CONCRETE_HIP_GEN_FOURSTEP=0 selects gen_step_kernel for A/B runs; the choice
// is made once per process, so conversion and PBS always agree.
static bool four_step(uint32_t N) {
  static const bool on = !getenv("CONCRETE_HIP_GEN_FOURSTEP") || atoi(getenv("CONCRETE_HIP_GEN_FOURSTEP")) != 0;
  return on && N >= 2048 && N <= 16384;
}

// Twiddle and twist tables for polynomial size N on the current device, built once in long
// double (correctly rounded to f64) and kept for the life of the process.
static Tables tables_for(uint32_t N) {
  static std::mutex mu;
  static std::map<std::pair<int, uint32_t>, Tables> cache;
  int dev = 0;
  CHIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find({dev, N});
  if (it != cache.end()) return it->second;
  const uint32_t M = N / 2, NHI = M / TW_LO > 1 ? M / TW_LO : 1;
  const long double PI = 3.14159265358979323846264338327950288L;
  auto ex = [&](long double ang) { return cplx{(double)cosl(ang), (double)sinl(ang)}; };
  std::vector<cplx> full(M), lo(TW_LO), hi(NHI), z(M);
  for (uint32_t j = 0; j < M; ++j) full[j] = ex(-2.0L * PI * (long double)j / (long double)M);
  for (uint32_t j = 0; j < (uint32_t)TW_LO; ++j) lo[j] = ex(-2.0L * PI * (long double)j / (long double)M);
  for (uint32_t j = 0; j < NHI; ++j) hi[j] = ex(-2.0L * PI * (long double)(j * TW_LO) / (long double)M);
  for (uint32_t j = 0; j < M; ++j) z[j] = ex(PI * (long double)j / (long double)N);
  Tables t;
  CHIP_CHECK(hipMalloc((void**)&t.Wfull, M * sizeof(cplx)));
  CHIP_CHECK(hipMemcpy(t.Wfull, full.data(), M * sizeof(cplx), hipMemcpyHostToDevice));
  CHIP_CHECK(hipMalloc((void**)&t.Wlo, TW_LO * sizeof(cplx)));
  CHIP_CHECK(hipMalloc((void**)&t.Whi, NHI * sizeof(cplx)));
  CHIP_CHECK(hipMalloc((void**)&t.Z, M * sizeof(cplx)));
  CHIP_CHECK(hipMemcpy(t.Wlo, lo.data(), TW_LO * sizeof(cplx), hipMemcpyHostToDevice));
  CHIP_CHECK(hipMemcpy(t.Whi, hi.data(), NHI * sizeof(cplx), hipMemcpyHostToDevice));
  CHIP_CHECK(hipMemcpy(t.Z, z.data(), M * sizeof(cplx), hipMemcpyHostToDevice));
  if (M >= 1024) {
    // tau(j1, k2) = zeta^{j1} w_M^{j1 k2} = exp(i pi j1 (1 - 4 k2) / N), correctly rounded
    const uint32_t R = M / 512;
    std::vector<cplx> tau((size_t)R * 512);
    for (uint32_t j1 = 0; j1 < R; ++j1)
      for (uint32_t p = 0; p < 512; ++p) {
        const int64_t e = ((int64_t)j1 * (1 - 4 * (int64_t)big_freq(p))) % (2 * (int64_t)N);
        tau[(size_t)j1 * 512 + p] = ex(PI * (long double)(e < 0 ? e + 2 * (int64_t)N : e) / (long double)N);
      }
    // slot factors beta(j1, e) = exp(-256 i pi j1 e / N) = tau(j1, e 64 + lane) / tau(j1, lane)
    for (uint32_t j1 = 0; j1 < R; ++j1)
      for (uint32_t e = 0; e < 8; ++e) {
        const int64_t x = (-(int64_t)256 * j1 * e) % (2 * (int64_t)N);
        tau.push_back(ex(PI * (long double)(x < 0 ? x + 2 * (int64_t)N : x) / (long double)N));
      }
    CHIP_CHECK(hipMalloc((void**)&t.Tau, tau.size() * sizeof(cplx)));
    CHIP_CHECK(hipMemcpy(t.Tau, tau.data(), tau.size() * sizeof(cplx), hipMemcpyHostToDevice));
    std::vector<cplx> wr(R);
    for (uint32_t x = 0; x < R; ++x) wr[x] = ex(-2.0L * PI * (long double)x / (long double)R);
    CHIP_CHECK(hipMalloc((void**)&t.WR, R * sizeof(cplx)));
    CHIP_CHECK(hipMemcpy(t.WR, wr.data(), R * sizeof(cplx), hipMemcpyHostToDevice));
  }
  cache[{dev, N}] = t;
  return t;
}

template <int M, int MODE>
static void launch_step(const StepArgs& s, uint32_t K1, hipStream_t st) {
  const uint64_t polys = (uint64_t)s.count * K1;
  const uint32_t blocks = (uint32_t)((polys + Geo<M>::PPB - 1) / Geo<M>::PPB);
  hipLaunchKernelGGL((gen_step_kernel<M, MODE>), dim3(blocks), dim3(Geo<M>::BLOCK), 0, st, s);
}

template <int M, int MODE>
static void launch_big_step(const StepArgs& s, uint32_t K1, hipStream_t st) {
  const uint32_t blocks = s.count * K1;  // one workgroup per polynomial
  if (s.level * s.base_log <= 31)
    hipLaunchKernelGGL((gen_big_step_kernel<M, MODE, true>), dim3(blocks), dim3(Big<M>::NT), 0, st, s);
  else
    hipLaunchKernelGGL((gen_big_step_kernel<M, MODE, false>), dim3(blocks), dim3(Big<M>::NT), 0, st, s);
}

template <int MODE>
static int step_dispatch(uint32_t N, const StepArgs& s, uint32_t K1, hipStream_t st) {
  if (four_step(N)) {
    switch (N) {
      case 2048: launch_big_step<1024, MODE>(s, K1, st); return 0;
      case 4096: launch_big_step<2048, MODE>(s, K1, st); return 0;
      case 8192: launch_big_step<4096, MODE>(s, K1, st); return 0;
      case 16384: launch_big_step<8192, MODE>(s, K1, st); return 0;
      default: return -2;
    }
  }
  switch (N) {
    case 256: launch_step<128, MODE>(s, K1, st); break;
    case 512: launch_step<256, MODE>(s, K1, st); break;
    case 1024: launch_step<512, MODE>(s, K1, st); break;
    case 2048: launch_step<1024, MODE>(s, K1, st); break;
    case 4096: launch_step<2048, MODE>(s, K1, st); break;
    case 8192: launch_step<4096, MODE>(s, K1, st); break;
    case 16384: launch_step<8192, MODE>(s, K1, st); break;
    default: return -2;
  }
  return 0;
}

// one-launch tile path for the instantiated shapes
template <int M, int K1, int KL, int T, int L, int C>
static void launch_tile(const TileArgs& t, hipStream_t st) {
  using TG = TileGeo<M, K1, KL, T, L, C>;
  auto kern = gen_tile_kernel<M, K1, KL, T, L, C>;
  CHIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, TG::LDS));
  hipLaunchKernelGGL(kern, dim3((t.count + C - 1) / C), dim3(TG::NT), TG::LDS, st, t);
}

// Tile sizes (ciphertexts per workgroup) measured on MI355X: N = 256, k = 5: C = 4 (55.4k PBS/s;
// C = 2: 44.3k); N = 512, k = 3: C = 2 (35.7k; C = 1: 22.3k at 269 VGPRs); N = 1024, k = 2:
// C = 2 (18.5k; C = 1: 12.1k).  CONCRETE_HIP_TILE_C selects the alternative for A/B runs.
// false: no tile instance for this shape (two-launch path).
static bool tile_dispatch(uint32_t N, uint32_t K1, uint32_t KL, uint32_t T, uint32_t L, const TileArgs& t,
                          hipStream_t st) {
  static const int tile_c = getenv("CONCRETE_HIP_TILE_C") ? atoi(getenv("CONCRETE_HIP_TILE_C")) : 0;
  if (N == 256 && K1 == 6 && KL == 6 && T == 2 && L == 5) {
    if (tile_c == 2) launch_tile<128, 6, 6, 2, 5, 2>(t, st);
    else launch_tile<128, 6, 6, 2, 5, 4>(t, st);
    return true;
  }
  if (N == 512 && K1 == 4 && KL == 4 && T == 2 && L == 5) {
    if (tile_c == 1) launch_tile<256, 4, 4, 2, 5, 1>(t, st);
    else launch_tile<256, 4, 4, 2, 5, 2>(t, st);
    return true;
  }
  if (N == 1024 && K1 == 3 && KL == 3 && T == 2 && L == 5) {
    if (tile_c == 1) launch_tile<512, 3, 3, 2, 5, 1>(t, st);
    else launch_tile<512, 3, 3, 2, 5, 2>(t, st);
    return true;
  }
  return false;
}

// k = 1, N = 4096 with an instance for (l, T, L): the one-launch gen_fused_kernel.  false: no instance
// (or CONCRETE_HIP_GEN_FUSED=0, A/B runs): the two-launch path runs.
static bool fused_dispatch(const FusedArgs& f, uint32_t k, uint32_t N, uint32_t level, uint32_t T, uint32_t L,
                           hipStream_t st) {
  const char* fe = getenv("CONCRETE_HIP_GEN_FUSED");  // read per call (tests cover both paths)
  if ((fe && atoi(fe) == 0) || k != 1 || !four_step(N)) return false;
  const bool w32 = (uint64_t)level * f.base_log <= 31;
  if (N != 4096) return false;
#define GEN_FUSED(LVv, Tv, Lv)                                                                               \
  if (level == LVv && T == Tv && L == Lv) {                                                                  \
    if (w32)                                                                                                 \
      hipLaunchKernelGGL((gen_fused_kernel<4, LVv, Tv, Lv, true>), dim3(f.count), dim3(512), 0, st, f);     \
    else                                                                                                     \
      hipLaunchKernelGGL((gen_fused_kernel<4, LVv, Tv, Lv, false>), dim3(f.count), dim3(512), 0, st, f);    \
    return true;                                                                                             \
  }
  GEN_FUSED(1, 2, 5)
#undef GEN_FUSED
  return false;
}

// k = 1, N = 8192 with an instance for (l, T, L): gen_coop_kernel, one ciphertext on two workgroups.
// false: no instance (or CONCRETE_HIP_GEN_COOP=0, A/B runs and tests): the two-launch path runs.
// Hand-off scratch per ciphertext: X halves 2 x l T x 32 KB, Y halves 2 x 2 x 32 KB; the flags are
// zeroed before every chunk (events are counted from 1 within a launch).
static bool coop_dispatch(const PbsArgs& a, const Tables& tb, uint32_t T, uint32_t L, uint32_t b, int* rc) {
  const char* ce = getenv("CONCRETE_HIP_GEN_COOP");  // read per call (tests cover both paths)
  if ((ce && atoi(ce) == 0) || a.k != 1 || a.N != 8192 || !four_step(a.N)) return false;
  const bool w32 = (uint64_t)a.level * a.base_log <= 31;
  void (*kern)(CoopArgs) = nullptr;
#define GEN_COOP(LVv, Tv, Lv)                                                                    \
  if (a.level == LVv && T == Tv && L == Lv) kern = w32 ? gen_coop_kernel<LVv, Tv, Lv, true> : gen_coop_kernel<LVv, Tv, Lv, false>;
  GEN_COOP(1, 2, 6)
#undef GEN_COOP
  if (!kern) return false;
  const uint64_t xb_ct = 2ull * a.level * T * 4 * 512 * sizeof(cplx), yb_ct = 2ull * 2 * 4 * 512 * sizeof(cplx);
  const char* ke = getenv("CONCRETE_HIP_GEN_CHUNK");
  // (<= 8192 ciphertexts per launch: the kernel's hand-off buffer descriptors count bytes in 31 bits)
  const uint32_t chunk = (uint32_t)std::min<uint64_t>(
      a.num_samples, std::min<uint64_t>(ke && atoi(ke) > 0 ? (uint64_t)atoi(ke) : 4096, 8192));
  const uint64_t flag_bytes = ((2ull * chunk + 1) * 4 + 15) / 16 * 16;
  char* scratch = nullptr;
  keep_pool_memory();
  CHIP_CHECK(hipMallocAsync((void**)&scratch, flag_bytes + (xb_ct + yb_ct) * chunk, a.stream));
  uint32_t* flags = reinterpret_cast<uint32_t*>(scratch);
  cplx* xb = reinterpret_cast<cplx*>(scratch + flag_bytes);
  cplx* yb = reinterpret_cast<cplx*>(scratch + flag_bytes + xb_ct * chunk);
  *rc = 0;
  for (uint32_t base = 0; base < a.num_samples; base += chunk) {
    const uint32_t cnt = std::min(chunk, a.num_samples - base);
    CHIP_CHECK(hipMemsetAsync(flags, 0, flag_bytes, a.stream));
    const CoopArgs ca{a.out, a.out_idx, a.in, a.in_idx, a.luts, a.lut_idx, reinterpret_cast<const cplx*>(a.fbsk),
                      tb.Tau, a.resid, xb, yb, flags, a.guard.status, a.guard.spin_limit, base, cnt, a.n, a.base_log,
                      b, (uint32_t)(xb_ct * cnt), (uint32_t)(yb_ct * cnt)};
    hipLaunchKernelGGL(kern, dim3(2 * cnt), dim3(512), 0, a.stream, ca);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      set_error("generic pbs (coop) launch failed: %s", hipGetErrorString(e));
      *rc = -1;
      break;
    }
  }
  CHIP_CHECK(hipFreeAsync(scratch, a.stream));
  return true;
}

// N >= 32768: the split path (S = N / 16384 workgroups per polynomial), one stream, chunks of
// <= 2 GB of scratch run one after another: init, then per CMUX step the product, the back half
// and the next step's front half.
// true: the register-tiled product ran, which leaves the slot spectra split by class (HPRE)
template <int S>
static bool launch_split_mac(const MacSplitArgs& m, uint32_t KL, uint32_t cnt, hipStream_t st) {
  const dim3 g1((m.M + 255) / 256, m.k + 1, (cnt + MAC_CTS - 1) / MAC_CTS);
  if (KL == 4 && m.limbs == 7 && m.subs == 2) {
    hipLaunchKernelGGL((gen_mac_split_kernel<4, 7, 2, S>), g1, dim3(256), 0, st, m);
    return true;
  }
  const dim3 g2((m.M + 255) / 256, (m.k + 1) * m.limbs, (cnt + MAC_CTS - 1) / MAC_CTS);
  hipLaunchKernelGGL((gen_mac_split_generic_kernel<S>), g2, dim3(256), 0, st, m);
  return false;
}

template <int S>
static void launch_split_front(const SplitArgs& s, uint32_t K1, hipStream_t st) {
  const dim3 grid(s.count * K1 * S);
  if ((uint64_t)s.level * s.base_log <= 31)
    hipLaunchKernelGGL((gen_split_front_kernel<S, true>), grid, dim3(512), 0, st, s);
  else
    hipLaunchKernelGGL((gen_split_front_kernel<S, false>), grid, dim3(512), 0, st, s);
}

// Chunks run in groups of NS on NS streams (the caller's and library streams, as the two-launch
// path), their launches interleaved, so one chunk's product kernel (HBM streaming) runs beside
// another's back / front kernels (one LDS-filling workgroup per CU).  CONCRETE_HIP_GEN_STREAMS=n
// (1..4, default 2) sets NS.
template <int S>
static int pbs_split_launch(const PbsArgs& a, const KeyFormat& fmt, const Tables& tb, uint32_t T) {
  using G = Split<S>;
  const uint32_t K1 = a.k + 1, M = G::M, L = fmt.limbs;
  const uint64_t per_ct = generic_scratch_bytes_per_sample(a.k, a.N, a.level, a.base_log);
  const char* be = getenv("CONCRETE_HIP_GEN_BUDGET_MB");
  const uint64_t budget = be && atoi(be) > 0 ? (uint64_t)atoi(be) << 20 : 2ull << 30;
  const char* ce = getenv("CONCRETE_HIP_GEN_CHUNK");
  const uint64_t cap = ce && atoi(ce) > 0 ? (uint64_t)atoi(ce) : 65536;
  const uint32_t chunk_max = (uint32_t)std::min<uint64_t>(std::min<uint64_t>(a.num_samples, cap),
                                                          std::max<uint64_t>(1, budget / per_ct));
  uint32_t nchunks = (a.num_samples + chunk_max - 1) / chunk_max;
  constexpr int MAX_NS = 4;
  const char* se = getenv("CONCRETE_HIP_GEN_STREAMS");
  const int want = se && atoi(se) >= 1 ? std::min(atoi(se), MAX_NS) : 2;
  const int NS = (int)std::min<uint32_t>((uint32_t)want, nchunks);
  nchunks = (nchunks + NS - 1) / NS * NS;  // balanced groups of NS chunks
  const uint32_t chunk = (a.num_samples + nchunks - 1) / nchunks;
  hipStream_t st[MAX_NS];
  for (int q = 0; q < MAX_NS; ++q) st[q] = q == 0 || q >= NS ? a.stream : side_stream(q);
  void* scratch = nullptr;
  keep_pool_memory();
  CHIP_CHECK(hipMallocAsync(&scratch, per_ct * chunk * NS, a.stream));
  hipEvent_t ev_in = nullptr;
  if (NS > 1) {  // the library streams start after the caller's prior work and the allocation
    CHIP_CHECK(hipEventCreateWithFlags(&ev_in, hipEventDisableTiming));
    CHIP_CHECK(hipEventRecord(ev_in, a.stream));
    for (int q = 1; q < NS; ++q) CHIP_CHECK(hipStreamWaitEvent(st[q], ev_in, 0));
  }
  const char* xe = getenv("CONCRETE_HIP_SPLIT_XCD");  // 0: plain workgroup order (A/B)
  const bool xcd = !(xe && atoi(xe) == 0);
  struct Lane {
    SplitArgs s;
    MacSplitArgs m;
    uint32_t cnt;
  };
  int rc = 0;
  for (uint32_t base0 = 0; base0 < a.num_samples && rc == 0; base0 += NS * chunk) {
    Lane ln[MAX_NS];
    int nl = 0;
    for (int q = 0; q < NS; ++q) {
      const uint32_t base = base0 + q * chunk;
      if (base >= a.num_samples) break;
      const uint32_t cnt = std::min(chunk, a.num_samples - base);
      cplx* X = reinterpret_cast<cplx*>(static_cast<char*>(scratch) + (uint64_t)q * per_ct * chunk);
      cplx* Y = X + (uint64_t)chunk * K1 * a.level * T * M;
      uint64_t* acc = reinterpret_cast<uint64_t*>(Y + (uint64_t)chunk * K1 * L * M);
      ln[q].s = SplitArgs{acc, X, Y, tb.Tau, tb.WR, a.in, a.in_idx, a.luts, a.lut_idx, a.resid,
                          base, cnt, a.n, a.k, a.level, a.base_log, fmt.bits, L, T, 0};
      ln[q].s.xcd = xcd ? 1u : 0u;
      ln[q].m = MacSplitArgs{X, Y, reinterpret_cast<const cplx*>(a.fbsk), tb.WR, cnt, a.k, a.level, L, T, M, G::R, 0};
      ln[q].cnt = cnt;
      ++nl;
    }
    for (int q = 0; q < nl; ++q) {
      const uint64_t elems = (uint64_t)ln[q].cnt * K1 * a.N;
      hipLaunchKernelGGL((gen_split_init_kernel<S>), dim3((uint32_t)std::min<uint64_t>((elems + 255) / 256, 65535)),
                         dim3(256), 0, st[q], ln[q].s);
      launch_split_front<S>(ln[q].s, K1, st[q]);
    }
    for (uint32_t i = 0; i < a.n; ++i) {
      for (int q = 0; q < nl; ++q) {
        Lane& l = ln[q];
        l.m.i = i;
        if (launch_split_mac<S>(l.m, K1 * a.level, l.cnt, st[q]))
          hipLaunchKernelGGL((gen_split_back_kernel<S, true>), dim3(l.cnt * K1 * S), dim3(512), 0, st[q], l.s);
        else
          hipLaunchKernelGGL((gen_split_back_kernel<S, false>), dim3(l.cnt * K1 * S), dim3(512), 0, st[q], l.s);
        if (i + 1 < a.n) {
          l.s.step = i + 1;
          launch_split_front<S>(l.s, K1, st[q]);
        }
      }
    }
    for (int q = 0; q < nl; ++q) {
      const uint64_t total = ((uint64_t)a.k * a.N + 1) * ln[q].cnt;
      const uint32_t eb = (uint32_t)std::min<uint64_t>((total + 255) / 256, 65535);
      hipLaunchKernelGGL(gen_extract_kernel, dim3(eb), dim3(256), 0, st[q], a.out, a.out_idx, ln[q].s.acc,
                         ln[q].s.base, ln[q].cnt, a.k, a.N, (uint32_t)G::LOGR);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      set_error("generic pbs (split) launch failed: %s", hipGetErrorString(e));
      rc = -1;
    }
  }
  if (NS > 1) {  // the caller's stream resumes after the library streams' chunks
    for (int q = 1; q < NS; ++q) {
      hipEvent_t ev = nullptr;
      CHIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      CHIP_CHECK(hipEventRecord(ev, st[q]));
      CHIP_CHECK(hipStreamWaitEvent(a.stream, ev, 0));
      CHIP_CHECK(hipEventDestroy(ev));
    }
    CHIP_CHECK(hipEventDestroy(ev_in));
  }
  CHIP_CHECK(hipFreeAsync(scratch, a.stream));
  return rc;
}

template <int S>
static int convert_split_launch(const ConvertArgs& a, const KeyFormat& fmt, const Tables& tb) {
  using G = Split<S>;
  const uint64_t polys = (uint64_t)a.n * a.level * (a.k + 1) * (a.k + 1);
  const uint64_t per_poly = (uint64_t)fmt.limbs * G::M * sizeof(cplx);
  const uint32_t batch = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(polys, (1ull << 30) / per_poly));
  void* scratch = nullptr;
  keep_pool_memory();
  CHIP_CHECK(hipMallocAsync(&scratch, per_poly * batch, a.stream));
  for (uint64_t p0 = 0; p0 < polys; p0 += batch) {
    const uint32_t nb = (uint32_t)std::min<uint64_t>(batch, polys - p0);
    SplitConvArgs c{reinterpret_cast<cplx*>(scratch), a.src_dev, tb.Tau, tb.WR, reinterpret_cast<cplx*>(a.dest), p0,
                    nb, a.k, a.level, fmt.bits, fmt.limbs, a.smax};
    hipLaunchKernelGGL((gen_split_convert_kernel<S>), dim3(nb * fmt.limbs * S), dim3(512), 0, a.stream, c);
    const uint64_t total = (uint64_t)nb * fmt.limbs * G::M;
    hipLaunchKernelGGL((gen_split_combine_kernel<S>), dim3((uint32_t)std::min<uint64_t>((total + 255) / 256, 65535)),
                       dim3(256), 0, a.stream, c);
  }
  CHIP_CHECK(hipFreeAsync(scratch, a.stream));
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("generic convert (split) launch failed: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

}  // namespace gen

uint64_t generic_scratch_bytes_per_sample(uint32_t k, uint32_t N, uint32_t level, uint32_t base_log) {
  const KeyFormat f = generic_key_format(k, N, level);
  if (f.kind != KeyKind::GENERIC) return 0;
  const uint64_t K1 = k + 1, M = N / 2, T = (base_log + f.bits - 1) / f.bits;
  return K1 * level * T * M * 16 + K1 * f.limbs * M * 16 + K1 * N * 8;
}

// A second stream per device for the two-launch and split paths' chunk groups (created once, never
// destroyed: it lives as long as the process, like the device tables).
static hipStream_t side_stream(int idx) {
  static std::mutex mu;
  static std::map<std::pair<int, int>, hipStream_t> streams;
  int dev = 0;
  CHIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> g(mu);
  auto it = streams.find({dev, idx});
  if (it != streams.end()) return it->second;
  hipStream_t s = nullptr;
  CHIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  streams[{dev, idx}] = s;
  return s;
}

int pbs_generic_launch(const PbsArgs& a) {
  using namespace gen;
  if (a.num_samples == 0) return 0;
  if (!generic_pbs_ok(a.k, a.N, a.level, a.base_log)) {
    set_error("pbs: k=%u N=%u level=%u base_log=%u outside the generic path's exact range", a.k, a.N, a.level,
              a.base_log);
    return -2;
  }
  const KeyFormat fmt = generic_key_format(a.k, a.N, a.level);
  const uint32_t K1 = a.k + 1, M = a.N / 2, L = fmt.limbs, b = fmt.bits;
  const uint32_t T = (a.base_log + b - 1) / b;
  const Tables tb = tables_for(a.N);
  if (a.N == 32768) return pbs_split_launch<2>(a, fmt, tb, T);
  {
    int rc = 0;
    if (coop_dispatch(a, tb, T, L, b, &rc)) return rc;
  }
  if (a.N == 65536) return pbs_split_launch<4>(a, fmt, tb, T);
  {
    const FusedArgs f{a.out, a.out_idx, a.in, a.in_idx, a.luts, a.lut_idx, reinterpret_cast<const cplx*>(a.fbsk),
                      tb.Tau, a.resid, a.num_samples, a.n, a.base_log, b};
    if (fused_dispatch(f, a.k, a.N, a.level, T, L, a.stream)) {
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) {
        set_error("generic pbs (fused) launch failed: %s", hipGetErrorString(e));
        return -1;
      }
      return 0;
    }
  }
  {
    const TileArgs t{a.out,   a.out_idx, a.in,    a.in_idx, a.luts,         a.lut_idx, reinterpret_cast<const cplx*>(a.fbsk),
                     tb.Wfull, tb.Z,     a.resid, a.num_samples, a.n, a.base_log, b};
    if (tile_dispatch(a.N, K1, K1 * a.level, T, L, t, a.stream)) {
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) {
        set_error("generic pbs (tile) launch failed: %s", hipGetErrorString(e));
        return -1;
      }
      return 0;
    }
  }
  // Two-launch path: chunks of <= 2 GB of X / Y / accumulator scratch.  With two or more chunks,
  // groups of NS chunks run on NS streams (the caller's and library streams of the device), their
  // launches interleaved: the step kernel (one LDS-filling workgroup per CU, its HBM traffic in
  // phase-locked bursts) and the product kernel (HBM streaming) of different chunks then share
  // the chip instead of alternating on it.  CONCRETE_HIP_GEN_STREAMS=n (1..4, default 2) sets NS.
  const uint64_t per_ct = generic_scratch_bytes_per_sample(a.k, a.N, a.level, a.base_log);
  const char* be = getenv("CONCRETE_HIP_GEN_BUDGET_MB");  // scratch per chunk (A/B runs)
  const uint64_t budget = be && atoi(be) > 0 ? (uint64_t)atoi(be) << 20 : 2ull << 30;
  // CONCRETE_HIP_GEN_CHUNK caps the ciphertexts per chunk (tests: several chunks at small batches);
  // both knobs are read per call
  const char* ce = getenv("CONCRETE_HIP_GEN_CHUNK");
  const uint64_t cap = ce && atoi(ce) > 0 ? (uint64_t)atoi(ce) : 65536;
  const uint32_t chunk_max = (uint32_t)std::min<uint64_t>(std::min<uint64_t>(a.num_samples, cap),
                                                          std::max<uint64_t>(1, budget / per_ct));
  uint32_t nchunks = (a.num_samples + chunk_max - 1) / chunk_max;
  constexpr int MAX_NS = 4;
  const char* se = getenv("CONCRETE_HIP_GEN_STREAMS");
  const int want = se && atoi(se) >= 1 ? std::min(atoi(se), MAX_NS) : 2;
  const int NS = (int)std::min<uint32_t>((uint32_t)want, nchunks);
  nchunks = (nchunks + NS - 1) / NS * NS;  // balanced groups of NS chunks
  const uint32_t chunk = (a.num_samples + nchunks - 1) / nchunks;
  hipStream_t st[MAX_NS];
  for (int q = 0; q < MAX_NS; ++q) st[q] = q == 0 || q >= NS ? a.stream : side_stream(q);
  hipEvent_t ev_in = nullptr, ev_out[MAX_NS] = {};
  void* scratch = nullptr;
  keep_pool_memory();
  CHIP_CHECK(hipMallocAsync(&scratch, per_ct * chunk * NS, a.stream));
  if (NS > 1) {  // the library streams start after the caller's prior work and the allocation
    CHIP_CHECK(hipEventCreateWithFlags(&ev_in, hipEventDisableTiming));
    CHIP_CHECK(hipEventRecord(ev_in, a.stream));
    for (int q = 1; q < NS; ++q) CHIP_CHECK(hipStreamWaitEvent(st[q], ev_in, 0));
  }
  struct Lane {
    StepArgs s;
    MacArgs m;
    uint64_t* acc;
    uint32_t cnt;
  };
  int rc = 0;
  for (uint32_t base0 = 0; base0 < a.num_samples && rc == 0; base0 += NS * chunk) {
    Lane ln[MAX_NS];
    int nl = 0;
    for (int q = 0; q < NS; ++q) {
      const uint32_t base = base0 + q * chunk;
      if (base >= a.num_samples) break;
      const uint32_t cnt = std::min(chunk, a.num_samples - base);
      cplx* X = reinterpret_cast<cplx*>(static_cast<char*>(scratch) + (uint64_t)q * per_ct * chunk);
      cplx* Y = X + (uint64_t)chunk * K1 * a.level * T * M;
      uint64_t* acc = reinterpret_cast<uint64_t*>(Y + (uint64_t)chunk * K1 * L * M);
      ln[q].s = StepArgs{acc,     X,    Y,   tb.Wfull, tb.Wlo,  tb.Whi,     tb.Z, a.in, a.in_idx, a.luts, a.lut_idx,
                         a.resid, base, cnt, a.n,      a.k,     a.level,    a.base_log, b, L,      T,      0, tb.Tau};
      ln[q].m = MacArgs{X, Y, reinterpret_cast<const cplx*>(a.fbsk), cnt, a.k, a.level, L, T, M, 0};
      ln[q].acc = acc;
      ln[q].cnt = cnt;
      ++nl;
    }
    for (int q = 0; q < nl && rc == 0; ++q) rc = step_dispatch<MODE_INIT | MODE_FRONT>(a.N, ln[q].s, K1, st[q]);
    for (uint32_t i = 0; i < a.n && rc == 0; ++i) {
      for (int q = 0; q < nl && rc == 0; ++q) {
        Lane& l = ln[q];
        l.m.i = i;
        if (!launch_mac2(l.m, l.cnt, st[q])) {
          const dim3 mg((M + 255) / 256, K1 * L, (l.cnt + MAC_CTS - 1) / MAC_CTS);
          hipLaunchKernelGGL(gen_mac_kernel, mg, dim3(256), 0, st[q], l.m);
        }
        l.s.step = i + 1;
        rc = i + 1 < a.n ? step_dispatch<MODE_BACK | MODE_FRONT>(a.N, l.s, K1, st[q])
                         : step_dispatch<MODE_BACK>(a.N, l.s, K1, st[q]);
      }
    }
    for (int q = 0; q < nl && rc == 0; ++q) {
      const uint64_t total = ((uint64_t)a.k * a.N + 1) * ln[q].cnt;
      const uint32_t eb = (uint32_t)std::min<uint64_t>((total + 255) / 256, 65535);
      const uint32_t rlog = four_step(a.N) ? (uint32_t)__builtin_ctz(M / 512) : 0u;
      hipLaunchKernelGGL(gen_extract_kernel, dim3(eb), dim3(256), 0, st[q], a.out, a.out_idx, ln[q].acc, ln[q].s.base,
                         ln[q].cnt, a.k, a.N, rlog);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      set_error("generic pbs launch failed: %s", hipGetErrorString(e));
      rc = -1;
    }
  }
  if (NS > 1) {  // the caller's stream resumes after the library streams' chunks
    for (int q = 1; q < NS; ++q) {
      CHIP_CHECK(hipEventCreateWithFlags(&ev_out[q], hipEventDisableTiming));
      CHIP_CHECK(hipEventRecord(ev_out[q], st[q]));
      CHIP_CHECK(hipStreamWaitEvent(a.stream, ev_out[q], 0));
      CHIP_CHECK(hipEventDestroy(ev_out[q]));
    }
    CHIP_CHECK(hipEventDestroy(ev_in));
  }
  CHIP_CHECK(hipFreeAsync(scratch, a.stream));
  return rc;
}

int convert_bsk_generic_launch(const ConvertArgs& a) {
  using namespace gen;
  const KeyFormat fmt = generic_key_format(a.k, a.N, a.level);
  if (fmt.kind != KeyKind::GENERIC) {
    set_error("generic BSK conversion: unsupported k=%u N=%u level=%u", a.k, a.N, a.level);
    return -2;
  }
  const Tables tb = tables_for(a.N);
  const uint64_t blocks = (uint64_t)a.n * a.level * (a.k + 1) * (a.k + 1);
  if (blocks == 0) return 0;
  if (a.N == 32768) return convert_split_launch<2>(a, fmt, tb);
  if (a.N == 65536) return convert_split_launch<4>(a, fmt, tb);
  cplx* G = reinterpret_cast<cplx*>(a.dest);
#define GEN_CONV(MM)                                                                                        \
  hipLaunchKernelGGL(gen_convert_kernel<MM>, dim3((uint32_t)blocks), dim3(Geo<MM>::THREADS), 0, a.stream, G, \
                     a.src_dev, tb.Wfull, tb.Wlo, tb.Whi, tb.Z, a.k, a.level, fmt.bits, fmt.limbs,        \
                     four_step(a.N) ? 1u : 0u, a.smax)
  switch (a.N) {
    case 256: GEN_CONV(128); break;
    case 512: GEN_CONV(256); break;
    case 1024: GEN_CONV(512); break;
    case 2048: GEN_CONV(1024); break;
    case 4096: GEN_CONV(2048); break;
    case 8192: GEN_CONV(4096); break;
    case 16384: GEN_CONV(8192); break;
    default: set_error("generic BSK conversion: N=%u", a.N); return -2;
  }
#undef GEN_CONV
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("generic convert launch failed: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

}  // namespace chip
