// common.hpp — shared host/device helpers for libconcrete_hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

namespace chip {

// Reference behaviour for the cuda_* ABI: void returns, failures abort the process
// (concrete-cpu c_api.rs:22-36 `nounwind`; tfhe-cuda-backend check_cuda_error).
#define CHIP_CHECK(expr)                                                                      \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    if (_e != hipSuccess) ::chip::hip_fatal(#expr, __FILE__, __LINE__, _e);                   \
  } while (0)

// abi.hip: prints the failed call, the HIP error, what hipGetDeviceCount reports now and the
// device-visibility environment (the round-3 abort left no such record), flushes, aborts
[[noreturn]] void hip_fatal(const char* expr, const char* file, int line, hipError_t e);
// the same state report without aborting (rt_die)
void report_hip_state(FILE* f);

// Error state for the concrete_hip_* extension entry points (which return status codes).
void set_error(const char* fmt, ...);
const char* last_error();

// Sticky per-device status word written by the PBS kernels, read back at synchronisation points
// (cuda_synchronize_device, concrete_hip_device_status, the runtime's batch completion).
constexpr uint32_t DEV_STATUS_SYNC_TIMEOUT = 1u;  // a wave-pair/quad sync spin hit its bound
constexpr uint32_t DEFAULT_SPIN_LIMIT = 1u << 22;  // LDS-counter polls (s_sleep 0 each, >= ~30 ms) before giving up
struct SyncGuard {
  uint32_t* status;     // device word, OR-ed with DEV_STATUS_* bits
  uint32_t spin_limit;  // polls before a sync spin gives up and flags DEV_STATUS_SYNC_TIMEOUT
};
SyncGuard sync_guard(int gpu, hipStream_t s);  // abi.hip: the word of (gpu, stream), lazily allocated
int take_device_status(int gpu);     // abi.hip: synchronises the device, returns and clears every word

// Torus helpers -------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint32_t modswitch(uint64_t x, int log2_2n) {
  // pbs_modulus_switch (tfhe 0.10) == simulation.cpp:64-75: round(x * 2N / 2^64) mod 2N
  return (uint32_t)((x + (1ull << (63 - log2_2n))) >> (64 - log2_2n));
}

// Balanced signed decomposition (tfhe 0.10 SignedDecomposer::init_decomposer_state +
// decompose_one_level; restated in oracle/tfhe_oracle.c:ora_decomp_*).
__device__ __forceinline__ uint64_t decomp_init(uint64_t x, int nrep) {
  return (x >> nrep) + ((x >> (nrep - 1)) & 1ull);
}
__device__ __forceinline__ int32_t decomp_next(uint64_t& state, int logB) {
  const uint64_t mask = (1ull << logB) - 1ull;
  uint64_t res = state & mask;
  state >>= logB;
  uint64_t carry = (((res - 1ull) | state) & res) >> (logB - 1);
  state += carry;
  return (int32_t)(int64_t)(res - (carry << logB));
}

// full-width digit (any base_log < 64; a balanced digit may be +2^(logB-1), so int32 is not enough
// past logB = 31)
__device__ __forceinline__ int64_t decomp_next64(uint64_t& state, int logB) {
  const uint64_t mask = (1ull << logB) - 1ull;
  uint64_t res = state & mask;
  state >>= logB;
  uint64_t carry = (((res - 1ull) | state) & res) >> (logB - 1);
  state += carry;
  return (int64_t)(res - (carry << logB));
}

// 32-bit state, digit as res + carry * (-2^logB) (one 24-bit multiply-add instead of a shift and
// a subtraction); valid when level * base_log <= 31
__device__ __forceinline__ int32_t decomp_next32(uint32_t& state, int logB, int32_t neg_base) {
  const uint32_t mask = (1u << logB) - 1u;
  const uint32_t res = state & mask;
  state >>= logB;
  const uint32_t carry = (((res - 1u) | state) & res) >> (logB - 1);
  state += carry;
  return __mul24((int)carry, neg_base) + (int32_t)res;  // v_mad_i32_i24
}

// The same recurrence on an UNSHIFTED 32-bit state S: level q's raw digit is bits
// [q logB, (q+1) logB) of S, the tie bit is bit (q+2) logB - 1 (the next level's top bit), and
// the carry is added back at bit (q+1) logB.  ((res - 1) | next) & res has bit logB-1 set exactly
// when res + next_top > B/2, i.e. carry = (res + next_top + B/2 - 1) >> logB.  Five or six
// operations per digit instead of seven; valid when level * base_log <= 31.
__device__ __forceinline__ int32_t decomp_level32(uint32_t& S, uint32_t off, int logB, uint32_t half_m1,
                                                  int32_t neg_base, bool update) {
  const uint32_t res = __builtin_amdgcn_ubfe(S, off, (uint32_t)logB);
  // bit (q+2) logB - 1; past bit 31 it is zero (S < 2^(level logB + 1) <= 2^28), as is bit 31
  const uint32_t tb = off + 2u * (uint32_t)logB - 1u;
  const uint32_t top = __builtin_amdgcn_ubfe(S, tb < 31u ? tb : 31u, 1u);
  const uint32_t carry = (res + top + half_m1) >> logB;
  if (update) S += carry << (off + (uint32_t)logB);
  return __mul24((int)carry, neg_base) + (int32_t)res;  // v_mad_i32_i24
}

// same recurrence on a 32-bit state (valid when level * base_log <= 31)
template <class U>
__device__ __forceinline__ int32_t decomp_next_t(U& state, int logB) {
  const U mask = ((U)1 << logB) - (U)1;
  U res = state & mask;
  state >>= logB;
  U carry = (((res - (U)1) | state) & res) >> (logB - 1);
  state += carry;
  return (int32_t)res - (int32_t)(carry << logB);
}

}  // namespace chip
