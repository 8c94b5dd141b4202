// keyswitch.hip — batched LWE keyswitch (exact u64 torus arithmetic).
//
// Reference semantics: concrete-cpu c_api/keyswitch.rs:185-223 -> tfhe 0.10
// keyswitch_lwe_ciphertext (restated in oracle/tfhe_oracle.c:ora_keyswitch):
//   out = (0, ..., 0, b) - sum_i sum_t d_{i,t} * KSK[i][t],  digits yielded level l first,
// KSK layout [n_in][l][n_out+1] u64 exactly as the runtime uploads it (context.h:117-145).
// Batched call shape: cuda_keyswitch_lwe_ciphertext_vector_64 (GPUDFG.cpp:1098-1101).
//
// Mapping: a workgroup owns KS_TILE samples; each KSK row (one (i, t) pair, n_out+1 words)
// is read once per tile with 2 KB coalesced loads and applied to all KS_TILE samples, so
// the 20.7 MB (cfg2) key is streamed B / KS_TILE times instead of B times.
#include <algorithm>
#include <mutex>
#include <type_traits>
#include <unordered_set>
#include <vector>

#include "common.hpp"
#include "kernel_util.hpp"
#include "pbs.hpp"

namespace chip {

// abi.hip: raise the device's default memory-pool release threshold once (released and re-reserved
// pool memory reads stale data on this stack; pooled scratch also saves ~0.1 ms per call at cfg2).
void keep_pool_memory();

constexpr int KS_TILE = 8;
constexpr int KS_THREADS = 256;
constexpr int KS_ICHUNK = 32;
constexpr int KS_MAX_U = 4;                       // output words per thread per sample
constexpr int KS_MAX_OUT = KS_MAX_U * KS_THREADS;  // output words per block (wider rows: windows in blockIdx.z)
constexpr uint32_t KS_MAX_ROW = 1u << 16;           // n_out + 1 accepted (LWE dimensions are far below)
// Levels: any l with l * logB < 64 (the optimizer's keyswitches reach l = 23 at logB = 1,
// v0_last_128 9-bit log-norm2 16).  The VALU kernel stages the digits of KS_DIG_ROWS (position,
// level) pairs per chunk in LDS: KS_ICHUNK positions up to KS_ICHUNK_L levels, fewer positions
// per chunk above that.
constexpr int KS_ICHUNK_L = 8;
constexpr int KS_DIG_ROWS = KS_ICHUNK * KS_ICHUNK_L;
__host__ __device__ constexpr uint32_t ks_ichunk(uint32_t level) {
  return level <= (uint32_t)KS_ICHUNK_L ? (uint32_t)KS_ICHUNK : (uint32_t)KS_DIG_ROWS / level;
}
// batches from this size take the MFMA path when it is exact (CONCRETE_HIP_KS_PATH: 0 = never,
// 1 = always when exact; A/B and test switch)
constexpr uint32_t KS_MFMA_MIN_BATCH = 64;

// Split-K (SPLIT): blockIdx.y takes mask positions [i_begin, i_end) and adds its partial sums
// into pre-zeroed outputs with 64-bit atomics (wrapping addition is exact and order-free, so
// the result is bit-identical); split 0 adds the body.  Used when the batch alone gives too
// few workgroups for the chip (large n_in, small batches).
__global__ void keyswitch_zero_kernel(uint64_t* out, const uint64_t* out_idx, uint32_t W, uint32_t num_samples) {
  const uint64_t total = (uint64_t)W * num_samples;
  for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < total; g += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t smp = (uint32_t)(g / W), j = (uint32_t)(g % W);
    out[(out_idx ? out_idx[smp] : smp) * (uint64_t)W + j] = 0ull;
  }
}

// NCH > 0: the 64-bit products d * k split into NCH key chunks (3: 22/21/21 bits, 4: 16 bits
// each), d * k_c summed in int32 with full-rate 24-bit multiply-adds (|d| <= 2^(logB-1), so a
// block of FP positions x level rows stays below 2^31 — the host picks NCH by that bound, see
// keyswitch_launch) and folded into the u64 accumulators once per block: exact, and it
// replaces the quarter-rate 32-bit multiplies.  NCH = 0: the 64-bit products.
template <int U, bool SPLIT, int NCH>
__global__ void __launch_bounds__(KS_THREADS)
keyswitch_kernel(uint64_t* __restrict__ out, const uint64_t* __restrict__ out_idx, const uint64_t* __restrict__ in,
                 const uint64_t* __restrict__ in_idx, const uint64_t* __restrict__ ksk, uint32_t n_in,
                 uint32_t n_out, uint32_t base_log, uint32_t level, uint32_t num_samples, uint32_t i_per_split) {
  // digits sample-minor: the KS_TILE digits of one (position, level) are two 16-byte reads.
  // The chunked paths need |d| <= 2^(logB-1) small anyway (int32); the 64-bit path keeps int64
  // digits, so any base_log with level * base_log < 64 is exact (a balanced digit can be +2^31).
  using dig_t = typename std::conditional<NCH == 0, int64_t, int32_t>::type;
  __shared__ __attribute__((aligned(16))) dig_t dig[KS_DIG_ROWS][KS_TILE];  // [position in chunk][level]
  const uint32_t ich = ks_ichunk(level);
  const uint32_t s0 = blockIdx.x * KS_TILE;
  const int tid = threadIdx.x;
  const uint32_t W = n_out + 1;
  const uint32_t jz = blockIdx.z * (uint32_t)KS_MAX_OUT;  // this block's window of output words
  uint64_t acc[KS_TILE][U];
#pragma unroll
  for (int s = 0; s < KS_TILE; ++s)
#pragma unroll
    for (int u = 0; u < U; ++u) acc[s][u] = 0ull;
  const int nrep = 64 - (int)(level * base_log);

  const uint32_t i_begin = SPLIT ? blockIdx.y * i_per_split : 0u;
  const uint32_t i_end = SPLIT ? min(n_in, i_begin + i_per_split) : n_in;
  for (uint32_t i0 = i_begin; i0 < i_end; i0 += ich) {
    __syncthreads();
    for (uint32_t e = tid; e < KS_TILE * ich; e += KS_THREADS) {
      const uint32_t s = e / ich, ii = e % ich;
      const uint32_t smp = s0 + s, i = i0 + ii;
      uint64_t a = 0ull;
      if (smp < num_samples && i < i_end) a = in[(in_idx ? in_idx[smp] : smp) * (uint64_t)(n_in + 1) + i];
      uint64_t st = decomp_init(a, nrep);
      for (uint32_t t = 0; t < level; ++t) dig[ii * level + t][s] = (dig_t)decomp_next64(st, (int)base_log);
    }
    __syncthreads();
    const uint32_t iend = min(ich, i_end - i0);
    if constexpr (NCH > 0) {
      constexpr int FP = NCH == 3 ? 16 : KS_ICHUNK;  // positions per int32 block
      for (uint32_t b0 = 0; b0 < iend; b0 += FP) {
        int32_t ca[KS_TILE][U][NCH];
#pragma unroll
        for (int s = 0; s < KS_TILE; ++s)
#pragma unroll
          for (int u = 0; u < U; ++u)
#pragma unroll
            for (int c = 0; c < NCH; ++c) ca[s][u][c] = 0;
        const uint32_t b1 = min(b0 + FP, iend);
        for (uint32_t ii = b0; ii < b1; ++ii) {
          for (uint32_t t = 0; t < level; ++t) {
            const uint64_t* row = ksk + ((uint64_t)(i0 + ii) * level + t) * W;
#pragma unroll
            for (int u = 0; u < U; ++u) {
              const uint32_t j = jz + tid + u * KS_THREADS;
              const uint64_t kv = j < W ? row[j] : 0ull;
              int32_t kc[NCH];
              if constexpr (NCH == 3) {
                kc[0] = (int32_t)(kv & 0x3fffffu);
                kc[1] = (int32_t)((kv >> 22) & 0x1fffffu);
                kc[2] = (int32_t)(kv >> 43);
              } else {
#pragma unroll
                for (int c = 0; c < NCH; ++c) kc[c] = (int32_t)((kv >> (16 * c)) & 0xffffu);
              }
#pragma unroll
              for (int s = 0; s < KS_TILE; ++s) {
                const int32_t d = dig[ii * level + t][s];
#pragma unroll
                for (int c = 0; c < NCH; ++c) ca[s][u][c] += __mul24(d, kc[c]);
              }
            }
          }
        }
#pragma unroll
        for (int s = 0; s < KS_TILE; ++s)
#pragma unroll
          for (int u = 0; u < U; ++u) {
            uint64_t sum = 0ull;
#pragma unroll
            for (int c = 0; c < NCH; ++c)
              sum += (uint64_t)(int64_t)ca[s][u][c] << (NCH == 3 ? (c == 0 ? 0 : c == 1 ? 22 : 43) : 16 * c);
            acc[s][u] -= sum;
          }
      }
    } else {
      for (uint32_t ii = 0; ii < iend; ++ii) {
        for (uint32_t t = 0; t < level; ++t) {
          const uint64_t* row = ksk + ((uint64_t)(i0 + ii) * level + t) * W;
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const uint32_t j = jz + tid + u * KS_THREADS;
            const uint64_t kv = j < W ? row[j] : 0ull;
#pragma unroll
            for (int s = 0; s < KS_TILE; ++s) acc[s][u] -= (uint64_t)dig[ii * level + t][s] * kv;
          }
        }
      }
    }
  }
#pragma unroll
  for (int s = 0; s < KS_TILE; ++s) {
    const uint32_t smp = s0 + s;
    if (smp >= num_samples) break;
    const uint64_t* ci = in + (in_idx ? in_idx[smp] : smp) * (uint64_t)(n_in + 1);
    uint64_t* co = out + (out_idx ? out_idx[smp] : smp) * (uint64_t)W;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t j = jz + tid + u * KS_THREADS;
      if (j >= W) continue;
      const uint64_t v = acc[s][u] + (j == n_out && (!SPLIT || blockIdx.y == 0) ? ci[n_in] : 0ull);
      if constexpr (SPLIT) atomicAdd((unsigned long long*)&co[j], (unsigned long long)v);
      else co[j] = v;
    }
  }
}

// ------------------------------------------------------------------------------------------
// MFMA path (base_log <= 7): the digit x key-word products as exact int8 matrix products.
// Every KSK word k is split into 8 balanced signed bytes, k = sum_c 2^{8c} k_c (mod 2^64),
// k_c in [-128, 127]; every digit fits int8 (|d| <= 2^(logB-1) <= 64).  With A[b][r] the digit
// of KSK row r = i l + t of sample b and B_c[r][j] = k_c of KSK[r][j], the int32 products
//     S_c = A B_c   (|S_c| <= K 2^(logB-1) 128 < 2^31, checked by the host)
// are exact on the i8 matrix cores (v_mfma_i32_32x32x32_i8), and
//     out[b][j] = (j == n_out ? b_in : 0) - sum_c 2^{8c} S_c[b][j]   (mod 2^64)
// is the keyswitch bit for bit.  Operands are K-contiguous rows (digits [Bp][Ks], key chunks
// [8][NP][Ks], zero padded; a launch sums k < Kp <= Ks); A and B fragments use the same lane/element -> k map, so the
// products sum over exactly the k of each step whatever order the hardware gives them.
// ------------------------------------------------------------------------------------------
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
constexpr int KSM_ROWS = 128;  // rows (samples) per 4-wave workgroup
constexpr int KSM_COLS = 64;   // columns (output words) per 4-wave workgroup
constexpr int KSM_KB = 64;     // K per register block (Kp is padded to a multiple of it)

__global__ void __launch_bounds__(256) ks_digits_i8_kernel(int8_t* __restrict__ A, const uint64_t* __restrict__ in,
                                                         const uint64_t* __restrict__ in_idx, uint32_t n_in,
                                                         uint32_t level, uint32_t base_log, uint32_t num_samples,
                                                         uint32_t Ks, uint32_t ipr) {
  // thread = (sample row b, mask position i); rows past the batch and positions past n_in: zeros
  const uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint32_t b = (uint32_t)(g / ipr), i = (uint32_t)(g % ipr);
  const int nrep = 64 - (int)(level * base_log);
  uint64_t a = 0ull;
  if (b < num_samples && i < n_in) a = in[(in_idx ? in_idx[b] : b) * (uint64_t)(n_in + 1) + i];
  uint64_t st = decomp_init(a, nrep);
  int8_t* row = A + (uint64_t)b * Ks;
  for (uint32_t t = 0; t < level; ++t) {
    const int8_t d = (int8_t)decomp_next64(st, (int)base_log);
    const uint32_t k = i * level + t;
    if (k < Ks) row[k] = d;
  }
}

// thread = (output word j, 16 consecutive KSK rows): 16 coalesced u64 reads (lanes along j),
// then one 16-byte store per chunk c into B_c[j][k0 .. k0 + 15]
__global__ void __launch_bounds__(256) ks_chunks_i8_kernel(int8_t* __restrict__ Bt, const uint64_t* __restrict__ ksk,
                                                         uint32_t K, uint32_t W, uint32_t NP, uint32_t Ks) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t k0 = blockIdx.y * 16;
  if (j >= NP) return;
  uint32_t w[8][4] = {};
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const uint32_t k = k0 + e;
    uint64_t v = (j < W && k < K) ? ksk[(uint64_t)k * W + j] : 0ull;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int32_t kc = (int32_t)(int8_t)(uint8_t)(v & 0xffull);  // balanced byte
      v = (v - (uint64_t)(int64_t)kc) >> 8;
      w[c][e >> 2] |= ((uint32_t)(uint8_t)kc) << (8 * (e & 3));
    }
  }
#pragma unroll
  for (int c = 0; c < 8; ++c)
    *reinterpret_cast<uint4*>(Bt + ((uint64_t)c * NP + j) * Ks + k0) = make_uint4(w[c][0], w[c][1], w[c][2], w[c][3]);
}

// one wave = 64 samples (two 32-row tiles) x 32 output words, all 8 chunks: 16 int32
// accumulator tiles (256 AGPRs), so each key-chunk fragment it loads serves two MFMAs; 4 waves
// per workgroup cover 128 x 64.  K in register blocks of KSM_KB = 64: lane half h reads the 32
// contiguous bytes [32 h, 32 h + 32) of the block for its row / column and feeds bytes
// 16 s .. 16 s + 15 to step s (any k order is exact as long as A and B use the same one); the
// next block's 20 fragments are loaded while the current block's 32 MFMAs run.
__global__ void __launch_bounds__(256) ks_mfma_kernel(uint64_t* __restrict__ out, const uint64_t* __restrict__ out_idx,
                                                    const uint64_t* __restrict__ in, const uint64_t* __restrict__ in_idx,
                                                    const int8_t* __restrict__ A, const int8_t* __restrict__ Bt,
                                                    uint32_t n_in, uint32_t n_out, uint32_t num_samples, uint32_t NP,
                                                    uint32_t Kp, uint32_t Ks, uint32_t k_per_split) {
  constexpr int RT = 2, SPB = KSM_KB / 32;  // row tiles per wave, MFMA k-steps per block
  // split-K (gridDim.z > 1): this workgroup sums k in [k_begin, k_end) and adds its partial
  // result into pre-zeroed outputs with 64-bit atomics (wrapping addition: exact, order-free);
  // split 0 adds the body
  const uint32_t k_begin = blockIdx.z * k_per_split, k_end = min(Kp, k_begin + k_per_split);
  const bool split = gridDim.z > 1;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t row0 = blockIdx.y * KSM_ROWS + 64 * (w >> 1), col0 = blockIdx.x * KSM_COLS + 32 * (w & 1);
  const int8_t* ap = A + (uint64_t)(row0 + (lane & 31)) * Ks + (KSM_KB / 2) * (lane >> 5);
  const int8_t* bp = Bt + (uint64_t)(col0 + (lane & 31)) * Ks + (KSM_KB / 2) * (lane >> 5);
  const uint64_t cstride = (uint64_t)NP * Ks, rstride = 32ull * Ks;
  v16i acc[RT][8];
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][c][r] = 0;
  v4i av[RT][SPB], bv[8][SPB];
  auto load_block = [&](uint32_t k0, v4i (&a4)[RT][SPB], v4i (&b4)[8][SPB]) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
      for (int s4 = 0; s4 < SPB; ++s4) a4[t][s4] = *reinterpret_cast<const v4i*>(ap + t * rstride + k0 + 16 * s4);
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
      for (int s4 = 0; s4 < SPB; ++s4) b4[c][s4] = *reinterpret_cast<const v4i*>(bp + c * cstride + k0 + 16 * s4);
  };
  load_block(k_begin, av, bv);
  for (uint32_t k0 = k_begin; k0 < k_end; k0 += KSM_KB) {
    v4i an[RT][SPB], bn[8][SPB];
    const uint32_t kn = k0 + KSM_KB < k_end ? k0 + KSM_KB : k0;  // last block: a harmless reload
    load_block(kn, an, bn);
    __builtin_amdgcn_sched_barrier(0);  // all next-block loads issued before this block's MFMAs
#pragma unroll
    for (int s4 = 0; s4 < SPB; ++s4)
#pragma unroll
      for (int c = 0; c < 8; ++c)
#pragma unroll
        for (int t = 0; t < RT; ++t)
          acc[t][c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(av[t][s4], bv[c][s4], acc[t][c], 0, 0, 0);
#pragma unroll
    for (int s4 = 0; s4 < SPB; ++s4) {
#pragma unroll
      for (int t = 0; t < RT; ++t) av[t][s4] = an[t][s4];
#pragma unroll
      for (int c = 0; c < 8; ++c) bv[c][s4] = bn[c][s4];
    }
  }
  // C/D map (gfx950, dtype-independent): col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
  const uint32_t W = n_out + 1;
  const uint32_t j = col0 + (lane & 31);
  if (j >= W) return;
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const uint32_t b = row0 + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (b >= num_samples) continue;
      uint64_t sum = 0ull;
#pragma unroll
      for (int c = 0; c < 8; ++c) sum += (uint64_t)(int64_t)acc[t][c][r] << (8 * c);
      uint64_t v = 0ull - sum;
      if (j == n_out && blockIdx.z == 0) v += in[(in_idx ? in_idx[b] : b) * (uint64_t)(n_in + 1) + n_in];
      uint64_t* o = out + (out_idx ? out_idx[b] : b) * (uint64_t)W + j;
      if (split) atomicAdd((unsigned long long*)o, (unsigned long long)v);
      else *o = v;
    }
}

// LDS-staged form (KS_LDS): 8 waves share a 128-sample x 64-word tile; each 64-k block of the
// tile's operands (digits 8 KB + key bytes 32 KB) is brought into an LDS ring of 3 stages by
// LDS-DMA (2 stages in flight), so every operand byte crosses L2 -> CU once per workgroup instead
// of once per wave.  LDS layout of a stage: A[kc][row] and B[c][kc][col], 16-byte cells, kc =
// 16-byte k chunk: each DMA piece (64 lanes x 16 B) is one (kc, 64 rows / cols) run, and a
// fragment read (lanes along rows / columns) is conflict-free.
#ifndef KS_LDS
#define KS_LDS 1
#endif
constexpr int KSL_ROWS = 128, KSL_COLS = 64, KSL_KB = 64, KSL_RS = 3;
constexpr int KSL_A_CELLS = (KSL_KB / 16) * KSL_ROWS;                 // 512 cells = 8 KB
constexpr int KSL_STAGE_CELLS = KSL_A_CELLS + 8 * (KSL_KB / 16) * KSL_COLS;  // + 2048 cells = 32 KB
constexpr int KSL_PIECES = KSL_STAGE_CELLS / 64;                      // 40 DMA pieces per stage
constexpr int KSL_PPW = KSL_PIECES / 8;                               // 5 per wave
constexpr size_t KSL_LDS = (size_t)KSL_RS * KSL_STAGE_CELLS * 16;     // 120 KB

__global__ void __launch_bounds__(512) ks_mfma_lds_kernel(uint64_t* __restrict__ out, const uint64_t* __restrict__ out_idx,
                                                        const uint64_t* __restrict__ in,
                                                        const uint64_t* __restrict__ in_idx, const int8_t* __restrict__ A,
                                                        const int8_t* __restrict__ Bt, uint32_t n_in, uint32_t n_out,
                                                        uint32_t num_samples, uint32_t NP, uint32_t Kp,
                                                        uint32_t Ks, uint32_t k_per_split) {
  extern __shared__ __attribute__((aligned(16))) v4i lds[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int rt = w & 3, ct = w >> 2;
  const uint32_t row_base = blockIdx.y * KSL_ROWS, col_base = blockIdx.x * KSL_COLS;
  const uint32_t k_begin = blockIdx.z * k_per_split, k_end = min(Kp, k_begin + k_per_split);
  const uint32_t nst = (k_end - k_begin) / KSL_KB;
  const bool split = gridDim.z > 1;
  const uint64_t cstride = (uint64_t)NP * Ks;
  // this wave's DMA pieces of a stage: global source of its lane and LDS cell offset of the piece
  const int8_t* src[KSL_PPW];
  int dst[KSL_PPW];
#pragma unroll
  for (int q = 0; q < KSL_PPW; ++q) {
    const int p = w * KSL_PPW + q;
    if (p < 8) {  // A: kc = p >> 1, rows 64 (p & 1) .. + 63
      const int kc = p >> 1, rh = p & 1;
      src[q] = A + (uint64_t)(row_base + 64 * rh + lane) * Ks + 16 * kc;
      dst[q] = kc * KSL_ROWS + 64 * rh;
    } else {  // B: c, kc
      const int pb = p - 8, c = pb >> 2, kc = pb & 3;
      src[q] = Bt + c * cstride + (uint64_t)(col_base + lane) * Ks + 16 * kc;
      dst[q] = KSL_A_CELLS + (c * 4 + kc) * KSL_COLS;
    }
  }
  auto issue = [&](uint32_t t) __attribute__((always_inline)) {
    const uint32_t kb = k_begin + t * KSL_KB;
    v4i* stage = lds + (t % KSL_RS) * KSL_STAGE_CELLS;
#pragma unroll
    for (int q = 0; q < KSL_PPW; ++q)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src[q] + kb), (lds_ptr_t)(stage + dst[q]), 16, 0, 0);
  };
  v16i acc[8];
#pragma unroll
  for (int c = 0; c < 8; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[c][r] = 0;
  if (nst > 0) issue(0);
  if (nst > 1) issue(1);
  const int r32 = lane & 31, h = lane >> 5;
  for (uint32_t t = 0; t < nst; ++t) {
    // stage t landed for this wave (stage t + 1 may stay in flight) ...
    if (t + 1 < nst) wait_vmcnt<KSL_PPW>();
    else wait_vmcnt<0>();
    pair_barrier();  // ... and for every wave; everyone is done with stage t - 1
    if (t + 2 < nst) issue(t + 2);  // into the slot of stage t - 1
    const v4i* stage = lds + (t % KSL_RS) * KSL_STAGE_CELLS;
#pragma unroll
    for (int s4 = 0; s4 < KSL_KB / 32; ++s4) {
      const int kc = 2 * s4 + h;
      const v4i av = stage[kc * KSL_ROWS + 32 * rt + r32];
      v4i bv[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) bv[c] = stage[KSL_A_CELLS + (c * 4 + kc) * KSL_COLS + 32 * ct + r32];
#pragma unroll
      for (int c = 0; c < 8; ++c) acc[c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv[c], acc[c], 0, 0, 0);
    }
  }
  const uint32_t W = n_out + 1;
  const uint32_t j = col_base + 32 * ct + r32;
  if (j >= W) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const uint32_t b = row_base + 32 * rt + (r & 3) + 8 * (r >> 2) + 4 * h;
    if (b >= num_samples) continue;
    uint64_t sum = 0ull;
#pragma unroll
    for (int c = 0; c < 8; ++c) sum += (uint64_t)(int64_t)acc[c][r] << (8 * c);
    uint64_t v = 0ull - sum;
    if (j == n_out && blockIdx.z == 0) v += in[(in_idx ? in_idx[b] : b) * (uint64_t)(n_in + 1) + n_in];
    uint64_t* o = out + (out_idx ? out_idx[b] : b) * (uint64_t)W + j;
    if (split) atomicAdd((unsigned long long*)o, (unsigned long long)v);
    else *o = v;
  }
}

// Four-wave form of the LDS-staged kernel (same stages, same operand layout): each wave covers 64
// samples (two 32-row tiles) x 32 words, so every key-chunk fragment it reads from LDS serves two
// MFMAs (16 per 32-k step from 10 fragment reads, against 8 from 9 in the eight-wave form): LDS
// reads per MFMA fall from 1.125 to 0.625 fragments, for one wave per SIMD whose 256 accumulator
// registers (AGPRs) leave room for the next step's fragments (read ahead of the MFMAs).
constexpr int KSL4_PPW = KSL_PIECES / 4;  // 10 DMA pieces per wave per stage
__global__ void __launch_bounds__(256) ks_mfma_lds4_kernel(uint64_t* __restrict__ out, const uint64_t* __restrict__ out_idx,
                                                         const uint64_t* __restrict__ in,
                                                         const uint64_t* __restrict__ in_idx, const int8_t* __restrict__ A,
                                                         const int8_t* __restrict__ Bt, uint32_t n_in, uint32_t n_out,
                                                         uint32_t num_samples, uint32_t NP, uint32_t Kp,
                                                         uint32_t Ks, uint32_t k_per_split) {
  extern __shared__ __attribute__((aligned(16))) v4i lds[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int rh = w >> 1, ch = w & 1;  // rows 64 rh .. + 63 (two 32-row tiles), words 32 ch .. + 31
  const uint32_t row_base = blockIdx.y * KSL_ROWS, col_base = blockIdx.x * KSL_COLS;
  const uint32_t k_begin = blockIdx.z * k_per_split, k_end = min(Kp, k_begin + k_per_split);
  const uint32_t nst = (k_end - k_begin) / KSL_KB;
  const bool split = gridDim.z > 1;
  const uint64_t cstride = (uint64_t)NP * Ks;
  const int8_t* src[KSL4_PPW];
  int dst[KSL4_PPW];
#pragma unroll
  for (int q = 0; q < KSL4_PPW; ++q) {
    const int p = w * KSL4_PPW + q;
    if (p < 8) {  // A: kc = p >> 1, rows 64 (p & 1) .. + 63
      const int kc = p >> 1, r2 = p & 1;
      src[q] = A + (uint64_t)(row_base + 64 * r2 + lane) * Ks + 16 * kc;
      dst[q] = kc * KSL_ROWS + 64 * r2;
    } else {  // B: c, kc
      const int pb = p - 8, c = pb >> 2, kc = pb & 3;
      src[q] = Bt + c * cstride + (uint64_t)(col_base + lane) * Ks + 16 * kc;
      dst[q] = KSL_A_CELLS + (c * 4 + kc) * KSL_COLS;
    }
  }
  auto issue = [&](uint32_t t) __attribute__((always_inline)) {
    const uint32_t kb = k_begin + t * KSL_KB;
    v4i* stage = lds + (t % KSL_RS) * KSL_STAGE_CELLS;
#pragma unroll
    for (int q = 0; q < KSL4_PPW; ++q)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src[q] + kb), (lds_ptr_t)(stage + dst[q]), 16, 0, 0);
  };
  v16i acc[2][8];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][c][r] = 0;
  if (nst > 0) issue(0);
  if (nst > 1) issue(1);
  const int r32 = lane & 31, h = lane >> 5;
  for (uint32_t t = 0; t < nst; ++t) {
    if (t + 1 < nst) wait_vmcnt<KSL4_PPW>();
    else wait_vmcnt<0>();
    pair_barrier();
    if (t + 2 < nst) issue(t + 2);
    const v4i* stage = lds + (t % KSL_RS) * KSL_STAGE_CELLS;
    v4i av[2][2], bv[2][8];
#pragma unroll
    for (int s4 = 0; s4 < KSL_KB / 32; ++s4) {
      const int kc = 2 * s4 + h;
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) av[s4][rt] = stage[kc * KSL_ROWS + 64 * rh + 32 * rt + r32];
#pragma unroll
      for (int c = 0; c < 8; ++c) bv[s4][c] = stage[KSL_A_CELLS + (c * 4 + kc) * KSL_COLS + 32 * ch + r32];
    }
#pragma unroll
    for (int s4 = 0; s4 < KSL_KB / 32; ++s4)
#pragma unroll
      for (int c = 0; c < 8; ++c)
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
          acc[rt][c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(av[s4][rt], bv[s4][c], acc[rt][c], 0, 0, 0);
  }
  const uint32_t W = n_out + 1;
  const uint32_t j = col_base + 32 * ch + r32;
  if (j >= W) return;
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const uint32_t b = row_base + 64 * rh + 32 * rt + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (b >= num_samples) continue;
      uint64_t sum = 0ull;
#pragma unroll
      for (int c = 0; c < 8; ++c) sum += (uint64_t)(int64_t)acc[rt][c][r] << (8 * c);
      uint64_t v = 0ull - sum;
      if (j == n_out && blockIdx.z == 0) v += in[(in_idx ? in_idx[b] : b) * (uint64_t)(n_in + 1) + n_in];
      uint64_t* o = out + (out_idx ? out_idx[b] : b) * (uint64_t)W + j;
      if (split) atomicAdd((unsigned long long*)o, (unsigned long long)v);
      else *o = v;
    }
}

// Whether the MFMA path is exact for these parameters (int8 digits, int32 sums): a sum has K =
// n_in l products of |d| <= 2^(logB-1) and |k_c| <= 128 (the zero padding adds nothing).
static bool ks_mfma_ok(const KsArgs& a) {
  if (a.base_log > 7) return false;
  const uint64_t K = (uint64_t)a.n_in * a.level;
  return K * (1ull << (a.base_log - 1)) * 128ull <= 0x7fffffffull;
}

// Key bytes B_c of a KSK, [8][NP][Ks] int8 (zero padded in j and k), built from the caller's u64 key.
// Cached per (key pointer, device, shape) so that the runtime's repeated keyswitches with one key
// (context.h:117-145 uploads it once) split it once — but only for buffers whose lifetime the
// backend sees: allocated by cuda_malloc_async (how the runtime allocates its KSK, context.h:134)
// or by the keyset (runtime.hip).  cuda_drop / cuda_drop_async / a cuda_memcpy_async_to_gpu onto the
// buffer release the entry (concrete_hip_release_device_buffer).  Any other pointer (e.g. memory of
// a caching allocator, which hands the same address to the next tensor) gets fresh key bytes on
// every call.  CONCRETE_HIP_KS_KEY_CACHE=0 disables the cache.
struct KeyBytes {
  const uint64_t* ksk;
  int dev;
  uint32_t K, W, NP, Ks;
  int8_t* bt;
  hipEvent_t built;  // other streams wait on the build
};
static std::mutex g_kb_mu;
static std::vector<KeyBytes> g_kb;
static std::unordered_set<const void*> g_tracked;  // buffers whose release the backend sees

void track_device_buffer(const void* p) {
  std::lock_guard<std::mutex> g(g_kb_mu);
  g_tracked.insert(p);
}

static bool key_cache_on() {
  static const bool on = !getenv("CONCRETE_HIP_KS_KEY_CACHE") || atoi(getenv("CONCRETE_HIP_KS_KEY_CACHE")) != 0;
  return on;
}

// nullptr when the device memory could not be allocated (the caller falls back to the VALU kernel)
static int8_t* key_bytes(const KsArgs& a, uint32_t K, uint32_t W, uint32_t NP, uint32_t Ks, bool& owned) {
  int dev = 0;
  CHIP_CHECK(hipGetDevice(&dev));
  keep_pool_memory();
  bool cache = key_cache_on();
  if (cache) {
    std::lock_guard<std::mutex> g(g_kb_mu);
    cache = g_tracked.count(a.ksk) > 0;
  }
  std::unique_lock<std::mutex> lk(g_kb_mu, std::defer_lock);
  if (cache) {
    lk.lock();
    for (const KeyBytes& e : g_kb)
      if (e.ksk == a.ksk && e.dev == dev && e.K == K && e.W == W && e.NP == NP && e.Ks == Ks) {
        CHIP_CHECK(hipStreamWaitEvent(a.stream, e.built, 0));
        owned = false;
        return e.bt;
      }
  }
  int8_t* bt = nullptr;
  const size_t bytes = (size_t)8 * NP * Ks;
  if ((cache ? hipMalloc((void**)&bt, bytes) : hipMallocAsync((void**)&bt, bytes, a.stream)) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  hipLaunchKernelGGL(ks_chunks_i8_kernel, dim3((NP + 255) / 256, Ks / 16), dim3(256), 0, a.stream, bt, a.ksk, K, W,
                     NP, Ks);
  owned = !cache;
  if (cache) {
    KeyBytes e{a.ksk, dev, K, W, NP, Ks, bt, nullptr};
    CHIP_CHECK(hipEventCreateWithFlags(&e.built, hipEventDisableTiming));
    CHIP_CHECK(hipEventRecord(e.built, a.stream));
    g_kb.push_back(e);
  }
  return bt;
}

// drop the cached key bytes derived from device buffer `p` (any device); returns how many.
// untrack: p is being freed (its address may come back for other data)
int release_key_bytes(const void* p, hipStream_t s, bool untrack) {
  std::vector<KeyBytes> gone;
  {
    std::lock_guard<std::mutex> g(g_kb_mu);
    if (untrack) g_tracked.erase(p);
    for (auto it = g_kb.begin(); it != g_kb.end();)
      if ((const void*)it->ksk == p) {
        gone.push_back(*it);
        it = g_kb.erase(it);
      } else {
        ++it;
      }
  }
  int prev = 0;
  if (!gone.empty()) CHIP_CHECK(hipGetDevice(&prev));
  for (KeyBytes& e : gone) {
    CHIP_CHECK(hipSetDevice(e.dev));
    if (s) CHIP_CHECK(hipFreeAsync(e.bt, s));
    else CHIP_CHECK(hipFree(e.bt));
    CHIP_CHECK(hipEventDestroy(e.built));
  }
  if (!gone.empty()) CHIP_CHECK(hipSetDevice(prev));
  return (int)gone.size();
}

static int keyswitch_mfma_launch(const KsArgs& a) {
  const uint32_t W = a.n_out + 1, NP = (W + KSM_COLS - 1) / KSM_COLS * KSM_COLS;
  const uint32_t K = a.n_in * a.level, kb = (K + KSM_KB - 1) / KSM_KB;
  // samples per pass: the int8 digit matrix of a pass stays <= 1 GiB (8-bit rows: K = 81,920);
  // rows are Ks = (kb + 7) KSM_KB bytes apart (below)
  const uint64_t kmax = (uint64_t)(kb + 7) * KSM_KB;
  // (CONCRETE_HIP_KS_CHUNK: a smaller pass size, read per call — the multi-pass test uses it)
  const char* cap_env = getenv("CONCRETE_HIP_KS_CHUNK");
  const uint64_t cap = cap_env && atoll(cap_env) > 0 ? (uint64_t)atoll(cap_env) : (1ull << 30) / kmax;
  const uint32_t chunk = (uint32_t)std::max<uint64_t>(
      KSM_ROWS, std::min<uint64_t>((uint64_t)(a.num_samples + KSM_ROWS - 1) / KSM_ROWS * KSM_ROWS,
                                   cap / KSM_ROWS * KSM_ROWS));
  // split K over s workgroups so that the rounds of the chip (one workgroup per CU: 512 registers
  // x 4 waves, or 120 KB of LDS) come out even: time ~ ceil(wgs s / 256) / s, smallest s on ties
  // (cfg2 batch 4096: 320 workgroups -> s = 4, 5 full rounds)
  const uint32_t wgs = (NP / KSM_COLS) * (chunk / KSM_ROWS);
  uint32_t splits = 1;
  {
    double best = 1e30;
    for (uint32_t sp = 1; sp <= std::min<uint32_t>(8, std::max<uint32_t>(1, kb / 2)); ++sp) {
      const double t = (double)((wgs * sp + 255) / 256) / sp;
      if (t < best - 1e-9) best = t, splits = sp;
    }
  }
  const uint32_t k_per_split = (kb + splits - 1) / splits * KSM_KB;
  splits = (kb * KSM_KB + k_per_split - 1) / k_per_split;
  const uint32_t Kp = splits * k_per_split;  // zero padded: whole blocks in every split
  // operand row stride: covers the padding of any split count (<= 8), so one key-byte layout
  // serves every batch size
  const uint32_t Ks = (kb + 7) * KSM_KB;
  static_assert(KSL_ROWS == KSM_ROWS && KSL_COLS == KSM_COLS && KSL_KB == KSM_KB, "one padding for both kernels");
  // CONCRETE_HIP_KS_WAVES=4: the four-wave LDS kernel (A/B), read per call
  const char* kw = getenv("CONCRETE_HIP_KS_WAVES");
  const bool four = KS_LDS && kw && atoi(kw) == 4;
  if (KS_LDS) CHIP_CHECK(hipFuncSetAttribute(four ? (const void*)ks_mfma_lds4_kernel : (const void*)ks_mfma_lds_kernel,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)KSL_LDS));
  keep_pool_memory();
  // test hook: refuse operand scratch above this many bytes (the VALU fallback then runs)
  if (const char* lim = getenv("CONCRETE_HIP_KS_SCRATCH_LIMIT"))
    if ((uint64_t)chunk * Ks + 8ull * NP * Ks > strtoull(lim, nullptr, 10)) return -5;
  bool bt_owned = false;
  int8_t* Bt = key_bytes(a, K, W, NP, Ks, bt_owned);
  int8_t* A = nullptr;
  if (!Bt || hipMallocAsync((void**)&A, (size_t)chunk * Ks, a.stream) != hipSuccess) {
    // not enough device memory for the matrix-core operands: the scratch-free VALU kernel
    (void)hipGetLastError();
    if (Bt && bt_owned) CHIP_CHECK(hipFreeAsync(Bt, a.stream));
    return -5;
  }
  const uint32_t ipr = (Ks + a.level - 1) / a.level;  // positions per digit row (covers the padding)
  for (uint32_t s0 = 0; s0 < a.num_samples; s0 += chunk) {
    const uint32_t cn = std::min(chunk, a.num_samples - s0);
    const uint32_t Bp = (cn + KSM_ROWS - 1) / KSM_ROWS * KSM_ROWS;
    // this pass's rows: shift the index arrays when given, else the row pointers
    const uint64_t* in_idx = a.in_idx ? a.in_idx + s0 : nullptr;
    const uint64_t* out_idx = a.out_idx ? a.out_idx + s0 : nullptr;
    const uint64_t* in = a.in_idx ? a.in : a.in + (uint64_t)s0 * (a.n_in + 1);
    uint64_t* out = a.out_idx ? a.out : a.out + (uint64_t)s0 * W;
    const uint64_t nd = (uint64_t)Bp * ipr;
    hipLaunchKernelGGL(ks_digits_i8_kernel, dim3((uint32_t)((nd + 255) / 256)), dim3(256), 0, a.stream, A, in, in_idx,
                       a.n_in, a.level, a.base_log, cn, Ks, ipr);
    if (splits > 1) {
      const uint64_t total = (uint64_t)W * cn;
      hipLaunchKernelGGL(keyswitch_zero_kernel, dim3((uint32_t)std::min<uint64_t>((total + 255) / 256, 4096)),
                         dim3(256), 0, a.stream, out, out_idx, W, cn);
    }
    if (four)
      hipLaunchKernelGGL(ks_mfma_lds4_kernel, dim3(NP / KSL_COLS, Bp / KSL_ROWS, splits), dim3(256), KSL_LDS, a.stream,
                         out, out_idx, in, in_idx, A, Bt, a.n_in, a.n_out, cn, NP, Kp, Ks, k_per_split);
    else if (KS_LDS)
      hipLaunchKernelGGL(ks_mfma_lds_kernel, dim3(NP / KSL_COLS, Bp / KSL_ROWS, splits), dim3(512), KSL_LDS, a.stream,
                         out, out_idx, in, in_idx, A, Bt, a.n_in, a.n_out, cn, NP, Kp, Ks, k_per_split);
    else
      hipLaunchKernelGGL(ks_mfma_kernel, dim3(NP / KSM_COLS, Bp / KSM_ROWS, splits), dim3(256), 0, a.stream, out,
                         out_idx, in, in_idx, A, Bt, a.n_in, a.n_out, cn, NP, Kp, Ks, k_per_split);
  }
  hipError_t e = hipGetLastError();
  CHIP_CHECK(hipFreeAsync(A, a.stream));
  if (bt_owned) CHIP_CHECK(hipFreeAsync(Bt, a.stream));
  if (e != hipSuccess) {
    set_error("keyswitch launch failed: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

// parameters the keyswitch kernels accept (64-bit arithmetic: the arguments may come from an
// imported key message, keyio.cpp)
bool keyswitch_params_ok(uint32_t level, uint32_t base_log, uint32_t n_in, uint32_t n_out) {
  return level >= 1 && base_log >= 1 && (uint64_t)level * base_log < 64 && n_in >= 1 &&
         (uint64_t)n_out + 1 <= KS_MAX_ROW;
}

int keyswitch_launch(const KsArgs& a) {
  if (!keyswitch_params_ok(a.level, a.base_log, a.n_in, a.n_out)) {
    set_error("unsupported keyswitch parameters: n_out=%u level=%u base_log=%u", a.n_out, a.level, a.base_log);
    return -2;
  }
  const uint32_t blocks = (a.num_samples + KS_TILE - 1) / KS_TILE;
  if (blocks == 0) return 0;
  static const int ks_path = getenv("CONCRETE_HIP_KS_PATH") ? atoi(getenv("CONCRETE_HIP_KS_PATH")) : -1;
  if (ks_path != 0 && ks_mfma_ok(a) && (ks_path == 1 || a.num_samples >= KS_MFMA_MIN_BATCH)) {
    const int rc = keyswitch_mfma_launch(a);
    if (rc != -5) return rc;  // -5: operand memory unavailable, run the VALU kernel below
  }
  // output words in windows of KS_MAX_OUT (blockIdx.z): U words per thread in each
  const uint32_t zw = (a.n_out + 1 + KS_MAX_OUT - 1) / KS_MAX_OUT;
  const uint32_t U = (std::min<uint32_t>(a.n_out + 1, KS_MAX_OUT) + KS_THREADS - 1) / KS_THREADS;
  // enough workgroups for 256 CUs: split the mask positions when the batch alone is short
  uint32_t splits = 1;
  if (blocks < 512) splits = std::min<uint32_t>((512 + blocks - 1) / blocks, std::max<uint32_t>(1, a.n_in / 128));
  const uint32_t per = ((a.n_in + splits - 1) / splits + KS_ICHUNK - 1) / KS_ICHUNK * KS_ICHUNK;
  splits = (a.n_in + per - 1) / per;
  if (splits > 1) {
    const uint64_t total = (uint64_t)(a.n_out + 1) * a.num_samples;
    hipLaunchKernelGGL(keyswitch_zero_kernel, dim3((uint32_t)std::min<uint64_t>((total + 255) / 256, 4096)), dim3(256),
                       0, a.stream, a.out, a.out_idx, a.n_out + 1, a.num_samples);
  }
  // int32 chunk sums of one block: FP * dmax * (max chunk) <= 2^31 - 1 with dmax = l 2^(logB-1)
  // (the largest digit row sum): 3 chunks (<= 22 bits, FP = 16) when dmax <= 32, 4 chunks
  // (16 bits, FP = 32) when dmax <= 1024, else the 64-bit products.  Compared by division so
  // nothing overflows for any accepted base_log.
  const uint64_t dmax = a.base_log - 1 >= 40 ? ~0ull : (1ull << (a.base_log - 1)) * a.level;
  const int nch = dmax <= 0x7fffffffull / (16ull * ((1ull << 22) - 1)) ? 3
                  : dmax <= 0x7fffffffull / ((uint64_t)KS_ICHUNK * 65535ull) ? 4 : 0;
#define KS_LAUNCH2(UU, CH)                                                                                         \
  if (splits > 1)                                                                                                  \
    hipLaunchKernelGGL((keyswitch_kernel<UU, true, CH>), dim3(blocks, splits, zw), dim3(KS_THREADS), 0, a.stream,     \
                       a.out, a.out_idx, a.in, a.in_idx, a.ksk, a.n_in, a.n_out, a.base_log, a.level,              \
                       a.num_samples, per);                                                                        \
  else                                                                                                             \
    hipLaunchKernelGGL((keyswitch_kernel<UU, false, CH>), dim3(blocks, 1, zw), dim3(KS_THREADS), 0, a.stream, a.out,     \
                       a.out_idx, a.in, a.in_idx, a.ksk, a.n_in, a.n_out, a.base_log, a.level, a.num_samples, per)
#define KS_LAUNCH(UU)          \
  if (nch == 3) {              \
    KS_LAUNCH2(UU, 3);         \
  } else if (nch == 4) {       \
    KS_LAUNCH2(UU, 4);         \
  } else {                     \
    KS_LAUNCH2(UU, 0);         \
  }
  switch (U) {
    case 1: KS_LAUNCH(1); break;
    case 2: KS_LAUNCH(2); break;
    case 3: KS_LAUNCH(3); break;
    default: KS_LAUNCH(4); break;
  }
#undef KS_LAUNCH
#undef KS_LAUNCH2
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("keyswitch launch failed: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

}  // namespace chip
