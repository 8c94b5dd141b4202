// pbs.hpp — host-side descriptors for the PBS and BSK-conversion kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace chip {

// N = 1024 kernel geometry: a workgroup of two waves per ciphertext (one GLWE polynomial and
// one half of the frequency slots per wave).  LDS: the two pass-1/pass-2 twiddle tables and one
// 9.2 KB transpose scratch per wave (which doubles as the half-spectrum mailbox).
constexpr size_t PBS1024_TABLE_BYTES = (8 * 72 + 4 * (8 + 64 + 8)) * 16;  // FFT512_TABLE_ENTRIES (fft512.hpp)
// Ciphertexts (wave pairs) per workgroup: PBS_PAIRS = 4 (8 waves, 2 per SIMD, one workgroup per CU
// by LDS) for batches that fill the chip; 2 or 1 for batches of <= 2 or <= 1 ciphertexts per CU, where
// 4 per workgroup would leave CUs idle (pbs.hip launch_pair: strong scaling, 512 per GPU on 8 GPUs).
constexpr int PBS_PAIRS = 4;
constexpr size_t PBS1024_XCH_SLOTS = 576;  // >= XCH_SLOTS (fft512.hpp), 16-B slots per wave
constexpr size_t pbs1024_pair_lds_bytes(int level, int pairs = PBS_PAIRS) {
  return PBS1024_TABLE_BYTES + 2 * (size_t)pairs * PBS1024_XCH_SLOTS * 16 + 3 * (size_t)level * 512 * 16 +
         2 * (size_t)pairs * 4;  // + pair-sync counters
}

// Small batches at l = 3 (pbs1024_quad.hip): four waves per ciphertext, CTS = 1 or 2 ciphertexts per
// workgroup; the pair kernel's ring and tables, one transpose scratch per wave, two counter sets.
constexpr size_t pbs1024_quad_lds_bytes(int cts) {
  return PBS1024_TABLE_BYTES + 4 * (size_t)cts * PBS1024_XCH_SLOTS * 16 + 3 * 3 * 512 * 16 + 2 * 4 * (size_t)cts * 4;
}

// N = 2048 kernel geometry (pbs2048.hip): four waves per ciphertext (one per even/odd half of
// each GLWE polynomial), PBS2_CTS ciphertexts per workgroup, a ring of 16 KB key groups.
constexpr int PBS2_CTS = 2;
constexpr int PBS2_RING_SLOTS = 4;
constexpr int PBS2_RING_DIST = 3;
constexpr int PBS2_LIMBS = 4;     // 16-bit key limbs
constexpr int PBS2_SUBS = 2;      // sub-digits per decomposition digit: balanced 16-bit d_lo, d_hi
constexpr int PBS2_SUB_BITS = 16; // on the key-limb grid (pbs2048.hip)
constexpr int PBS2_MAX_LOGB = 24; // |d_hi| <= 2^(logB-17) + 1 keeps the certified bound < 1/2
// l = 2 .. PBS2_MAX_LEVEL: whole digits with l 2^(logB-1) <= 2^15 (the l = 1 digit's magnitude), the
// levels' products summed into the same slot (the optimizer's 5-bit rows at br 2/15, 3/11, 4/9)
constexpr uint32_t PBS2_MAX_LEVEL = 4;
inline bool pbs2048_ok(uint32_t level, uint32_t base_log) {
  if (level == 1) return base_log >= 1 && base_log <= (uint32_t)PBS2_MAX_LOGB;
  return level >= 2 && level <= PBS2_MAX_LEVEL && base_log >= 1 && base_log <= 15 &&
         ((uint64_t)level << (base_log - 1)) <= (1ull << 15);
}
// P2_PM = 1: the key holds the spectra at the two square roots +-s_k of each evaluation point
// alpha_k, K+- = (G_e +- s G_o) / 2 (the N = 2048 polynomial evaluated at +-s_k, i.e. its
// 1024-point negacyclic spectrum), so a product costs 2 complex multiplies per frequency instead
// of the 4 of the even/odd form (a_e b_e + Z a_o b_o, a_e b_o + a_o b_e); 0: the even/odd key
// (pbs2048.hip, bsk.hip; A/B builds only, the key format follows it).
#ifndef P2_PM
#define P2_PM 1
#endif
constexpr size_t pbs2048_lds_bytes() {
  return PBS1024_TABLE_BYTES + 4 * PBS2_CTS * PBS1024_XCH_SLOTS * 16 + (size_t)PBS2_RING_SLOTS * 1024 * 16 +
         4 * PBS2_CTS * 4;  // + per-wave sync counters
}

// N = 1024, k = 2, l = 1 kernel geometry (pbs1024k2.hip): three waves per ciphertext (one per GLWE
// polynomial), K2_CTS ciphertexts per workgroup, a ring of 24 KB key groups (one limb and one output
// column: the three row spectra).  Key: 4 balanced 16-bit limbs, digits split as in pbs2048.hip.
constexpr int K2_CTS = 2;
constexpr int K2_RING_SLOTS = 3;
constexpr int K2_LIMBS = 4;
constexpr int K2_SUBS = 2;
constexpr int K2_SUB_BITS = 16;
constexpr int K2_MAX_LOGB = 24;  // certified bound < 1/2 (oracle/pyoracle.py:gpu1024k2_error_bound)
// l = 1: one digit split into two sub-digits (logB <= 24); l = 2: two whole digits with
// l 2^(logB-1) <= 2^15 (the l = 1 digit's magnitude; the optimizer's br 2/15 rows), both levels'
// spectra held in registers (pbs1024k2_kernel)
constexpr uint32_t K2_MAX_LEVEL = 2;  // pbs1024k2_kernel's levels
// l >= K2_MANY_MIN: one level at a time (pbs1024k2_many_kernel), the key level-major
// ([n][q][limb][col][row][512]); whole digits with l 2^(logB-1) <= 2^15 and l logB < 64.  From l = 3
// it is faster than holding every level's spectra (3.6 % at l = 3, profiles/r04manyab_rows.log).
#ifndef K2_MANY_MIN_LEVEL
#define K2_MANY_MIN_LEVEL 3
#endif
constexpr uint32_t K2_MANY_MIN = K2_MANY_MIN_LEVEL;
inline bool k2_ok(uint32_t level, uint32_t base_log) {
  if (level == 1) return base_log >= 1 && base_log <= (uint32_t)K2_MAX_LOGB;
  if (level >= K2_MANY_MIN && (uint64_t)level * base_log >= 64) return false;
  return level >= 2 && level <= 64 && base_log >= 1 && base_log <= 15 &&
         ((uint64_t)level << (base_log - 1)) <= (1ull << 15);
}
constexpr size_t pbs1024k2_many_lds_bytes() {  // four waves per ciphertext, three scratches
  return PBS1024_TABLE_BYTES + 3 * K2_CTS * PBS1024_XCH_SLOTS * 16 + (size_t)K2_RING_SLOTS * 3 * 512 * 16 +
         4 * K2_CTS * 4;
}
constexpr size_t pbs1024k2_lds_bytes() {
  return PBS1024_TABLE_BYTES + 3 * K2_CTS * PBS1024_XCH_SLOTS * 16 + (size_t)K2_RING_SLOTS * 3 * 512 * 16 +
         3 * K2_CTS * 4;  // + per-wave sync counters
}

// N = 512, k = 3 and N = 256, k = 5 / 6, l <= 3 (pbs_small.hip): P = 1024 / N polynomials per register
// fft512, two waves per ciphertext, SM_CTS ciphertexts per workgroup, a ring of key groups (one limb
// and one output column: the k + 1 row spectra).  Key: 4 balanced 16-bit limbs, scaled 1 / (512 P).
constexpr int SM_CTS = 4;
constexpr int SM_LIMBS = 4;
constexpr int SM_SUB_BITS = 16;
// l = 2, 3: whole digits (l 2^(logB-1) <= 2^15, the l = 1, logB = 16 magnitude), the levels' products
// summed into the same slot (the optimizer's rows at br 2/10, 2/12, 3/9)
constexpr uint32_t SM_MAX_LEVEL = 3;
// largest digit: the certified bound (oracle/pyoracle.py:gpu_small_error_bound) on random keys of
// the table rows' size is 0.28 at N = 512, k = 3 and 0.34 / 0.39 at N = 256, k = 5 / 6 for any
// logB <= 24 (0.17 / 0.19 with one sub-digit, logB <= 15); wider digits run on the general path
inline uint32_t pbs_small_max_logb(uint32_t N) { return N == 512 || N == 256 ? 24u : 0u; }
// key group = one limb and SM_GC(N) output columns (K1 row spectra each); SM_RS(N) ring slots
// (two columns at N = 256 when k + 1 is even: half the key windows, 3 x 24 KB slots)
#ifndef SM_GC256
#define SM_GC256 2
#endif
constexpr int sm_gc(int N, int K1) { return N == 256 && K1 % SM_GC256 == 0 ? SM_GC256 : 1; }
constexpr int sm_rs(int N, int K1) { return sm_gc(N, K1) == 2 ? 3 : 4; }
constexpr size_t pbs_small_lds_bytes(int N, int K1) {
  return PBS1024_TABLE_BYTES + 2 * SM_CTS * PBS1024_XCH_SLOTS * 16 +
         (size_t)sm_rs(N, K1) * sm_gc(N, K1) * K1 * (N / 2) * 16 + 2 * SM_CTS * 4;
}
// N = 512, k = 4 (pbs512k4.hip): the same key format and packing; five polynomials make three packed
// transforms: four waves per ciphertext (three transform owners, one slot each), K4_CTS ciphertexts per
// workgroup and a ring of K4_RING_SLOTS 20 KB key groups.  l = 1 (logB <= 24), and whole digits with
// l 2^(logB-1) <= 2^15 (the l = 1, logB = 16 magnitude: certified bound 0.35) one level at a time from
// l = 3.  l = 2: the optimizer's rows have logB = 16, where two whole digits against 16-bit limbs would put the
// bound at 0.69, so that shape's key has five 13-bit limbs (bound 0.09; the format depends on (k, N, l)
// only, so the whole shape takes it).
constexpr int K4_CTS = 2;
constexpr int K4_RING_SLOTS = 4;
constexpr uint32_t K4_MAX_LEVEL = 2;  // pbs512k4_kernel's levels (l = 2: 13-bit limbs)
// l >= K4_MANY_MIN: one level at a time (pbs512k4_many_kernel), the key level-major
// ([n][q][limb][col][row][M]); whole digits with l 2^(logB-1) <= 2^15 and l logB < 64.  From l = 3
// it is faster than holding every level's spectra (3-7 % at l = 3 .. 5, profiles/r04manyab_rows.log).
#ifndef K4_MANY_MIN_LEVEL
#define K4_MANY_MIN_LEVEL 3
#endif
constexpr uint32_t K4_MANY_MIN = K4_MANY_MIN_LEVEL;
constexpr size_t pbs512k4_lds_bytes() {
  return PBS1024_TABLE_BYTES + 3 * K4_CTS * PBS1024_XCH_SLOTS * 16 + (size_t)K4_RING_SLOTS * 5 * 256 * 16 +
         4 * K4_CTS * 4 * 2 + 4 * 64 * 16;  // + sync counters (padded to 16 B) + the many-level kernel's tz
}
inline bool pbs_small_shape(uint32_t k, uint32_t N, uint32_t level) {
  if (N == 512 && k == 4) return level >= 1 && level <= 64;
  return level >= 1 && level <= SM_MAX_LEVEL && ((N == 512 && k == 3) || (N == 256 && (k == 5 || k == 6)));
}
// key limbs of a small-ring key: 4 of 16 bits, 5 of 13 bits at k = 4, N = 512, l = 2 (K4_L2_LIMBS)
constexpr uint32_t K4_L2_LIMBS = 5;
inline uint32_t small_limbs(uint32_t k, uint32_t N, uint32_t level) {
  return N == 512 && k == 4 && level == 2 ? K4_L2_LIMBS : (uint32_t)SM_LIMBS;
}
inline bool pbs_small_ok(uint32_t k, uint32_t N, uint32_t level, uint32_t base_log) {
  if (!pbs_small_shape(k, N, level) || base_log < 1) return false;
  if (level == 1) return base_log <= pbs_small_max_logb(N);
  // 13-bit limbs: two whole digits up to 16 bits (certified bound 0.09 on the table rows' keys)
  if (small_limbs(k, N, level) == K4_L2_LIMBS) return base_log <= 16;
  if ((uint64_t)level * base_log >= 64) return false;
  return base_log <= 15 && ((uint64_t)level << (base_log - 1)) <= (1ull << 15);
}

// Device key formats.  N1024 / N2048: the hand-tuned kernels' layouts (pbs.hip, pbs2048.hip);
// GENERIC: pbs_generic.hip, L balanced limbs of `bits` bits for any k <= GEN_MAX_K and
// N = 256 .. 16384.  The format depends on (k, N, l) only: the runtime's key conversion call
// carries no base_log (context.h:106-109).
// K2N1024: pbs1024k2.hip (k = 2, N = 1024, any l); SMALL: pbs_small.hip (N = 512, k = 3 and
// N = 256, k = 5 / 6, l <= 3) and pbs512k4.hip (N = 512, k = 4, l = 1 .. 64: l >= K4_MANY_MIN one
// level at a time).  The values are the ABI's format codes
// (concrete_hip_bsk_format).
enum class KeyKind { NONE, N1024, N2048, GENERIC, K2N1024, SMALL };
struct KeyFormat {
  KeyKind kind;
  uint32_t limbs, bits;
};
constexpr int GEN_MAX_K = 8;       // GLWE dimension
constexpr int GEN_MAX_LIMBS = 8;   // key limbs
constexpr int GEN_MAX_TERMS = 24; // key values per register chunk of the generic product (gen_mac_kernel)
KeyFormat key_format(uint32_t k, uint32_t N, uint32_t level);                              // pbs_generic.hip
bool generic_pbs_ok(uint32_t k, uint32_t N, uint32_t level, uint32_t base_log);            // pbs_generic.hip
uint32_t generic_limb_bits(uint32_t k, uint32_t N, uint32_t level);                        // pbs_generic.hip
double generic_error_bound(uint32_t k, uint32_t N, uint32_t level, uint32_t base_log, uint32_t bits,
                           double maxG);                                                   // pbs_generic.hip
uint64_t generic_scratch_bytes_per_sample(uint32_t k, uint32_t N, uint32_t level, uint32_t base_log);

// Number of exact limbs of the key polynomial for a parameter set.
inline uint32_t default_limbs(uint32_t k, uint32_t N, uint32_t level) { return key_format(k, N, level).limbs; }

// N = 1024 exactness gate.  The 3-limb product's certified rounding bound grows with the number
// of digit rows (k+1)l and the digit magnitude 2^(logB-1): measured on random keys it is
// 0.044 at l=3/logB=7 (cfg2) and ~0.22-0.24 at (k+1) l 2^logB = 4096 (oracle fft_error_bound;
// DESIGN.md §3).  Sets beyond that could round a coefficient the wrong way, so they are refused.
inline bool pbs1024_exact(uint32_t k, uint32_t level, uint32_t base_log) {
  return level >= 1 && level <= 3 && base_log >= 1 && base_log <= 11 &&
         ((uint64_t)(k + 1) * level << base_log) <= 4096ull;
}

// Whether a (k, N, l, logB) PBS runs, exactly, on one of the kernels.
inline bool pbs_params_ok(uint32_t k, uint32_t N, uint32_t level, uint32_t base_log) {
  const KeyFormat f = key_format(k, N, level);
  switch (f.kind) {
    case KeyKind::N1024: return pbs1024_exact(k, level, base_log);
    // one level whose digit splits into d_lo + 2^16 d_hi (pbs2048.hip)
    case KeyKind::N2048: return pbs2048_ok(level, base_log);
    case KeyKind::GENERIC: return generic_pbs_ok(k, N, level, base_log);
    case KeyKind::K2N1024: return k2_ok(level, base_log);
    case KeyKind::SMALL: return pbs_small_ok(k, N, level, base_log);
    default: return false;
  }
}

// Size in bytes of the device Fourier bootstrapping key.
//   N1024:   [n][limb][co][ro][q][512] complex f64; slots 0..3 of group (limb, co, ro) hold column co /
//            row ro, slots 4..7 column 1 - co / row 1 - ro (bsk.hip: each wave of a pair reads its
//            "own" and "other" spectra at fixed positions)
//   N2048:   [n][limb][col][q][row][+-][512] complex f64 (pbs2048.hip; l <= 4)
//   GENERIC: [n][col][limb][row][q][N/2] complex f64 (pbs_generic.hip)
//   K2N1024: [n][limb][col][q][row][512] complex f64 (pbs1024k2.hip; l < K2_MANY_MIN;
//            l >= K2_MANY_MIN: [n][q][limb][col][row][512])
//   SMALL:   [n][limb][cg][q][c2][row][N/2] complex f64, col = cg GC + c2 (pbs_small.hip, pbs512k4.hip;
//            GC = sm_gc(N, k + 1)); k = 4, N = 512, l >= K4_MANY_MIN: [n][q][limb][col][row][N/2]
inline uint64_t fourier_bsk_bytes(uint32_t n, uint32_t k, uint32_t level, uint32_t N) {
  const KeyFormat f = key_format(k, N, level);
  switch (f.kind) {
    case KeyKind::N2048: return (uint64_t)n * f.limbs * (k + 1) * (k + 1) * 2 * 512 * 16ull * level;
    case KeyKind::N1024:
    case KeyKind::K2N1024:
    case KeyKind::SMALL:
    case KeyKind::GENERIC: return (uint64_t)n * level * (k + 1) * (k + 1) * f.limbs * (N / 2) * 16ull;
    default: return 0;
  }
}

struct PbsArgs {
  hipStream_t stream;
  uint64_t* out;
  const uint64_t* out_idx;
  const uint64_t* luts;
  const uint64_t* lut_idx;
  const uint64_t* in;
  const uint64_t* in_idx;
  const void* fbsk;
  uint32_t n, k, N, base_log, level, limbs, num_samples;
  unsigned long long* resid;  // optional: max |x - round(x)| over all outputs (f64 bits)
  SyncGuard guard;            // device status word + spin bound of the wave-pair/quad syncs
};

int pbs_launch(const PbsArgs& a);
int pbs2048_launch(const PbsArgs& a);         // pbs2048.hip
int pbs1024_quad_launch(const PbsArgs& a, int cts);  // pbs1024_quad.hip (cts = 1 or 2)
int pbs_generic_launch(const PbsArgs& a);     // pbs_generic.hip
int pbs1024k2_launch(const PbsArgs& a);       // pbs1024k2.hip
int pbs_small_launch(const PbsArgs& a);       // pbs_small.hip
int pbs512k4_launch(const PbsArgs& a);        // pbs512k4.hip

struct ConvertArgs {
  hipStream_t stream;
  void* dest;               // Fourier key, fourier_bsk_bytes()
  const uint64_t* src_dev;  // standard-domain key on the device [n][l][k+1][k+1][N]
  uint32_t n, k, level, N, limbs;
  unsigned long long* smax = nullptr;  // keycheck.hpp sink: max |G|^2 of the stored key (or none)
};
int convert_bsk_launch(const ConvertArgs& a);
int convert_bsk_generic_launch(const ConvertArgs& a);  // pbs_generic.hip

struct KsArgs {
  hipStream_t stream;
  uint64_t* out;
  const uint64_t* out_idx;
  const uint64_t* in;
  const uint64_t* in_idx;
  const uint64_t* ksk;
  uint32_t n_in, n_out, base_log, level, num_samples;
};
int keyswitch_launch(const KsArgs& a);
bool keyswitch_params_ok(uint32_t level, uint32_t base_log, uint32_t n_in, uint32_t n_out);  // keyswitch.hip
// keyswitch.hip: drop the int8 key bytes cached for the KSK at device pointer p (freed on stream s,
// or synchronously when s is null; untrack when p itself is being freed); returns the number of
// entries released.  track_device_buffer: p's lifetime is visible to the backend (cuda_malloc_async,
// keyset keys), so key bytes derived from it may be cached.
int release_key_bytes(const void* p, hipStream_t s, bool untrack);
void track_device_buffer(const void* p);

}  // namespace chip
