// kernel_util.hpp — device helpers shared by the PBS kernels (pbs.hip, pbs2048.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "common.hpp"

namespace chip {

// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E)
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// bits(v + 1.5 * 2^52) = bits(1.5 * 2^52) + round(v) for |v| < 2^51
constexpr double RND_MAGIC = 6755399441055744.0;
constexpr uint64_t RND_MAGIC_BITS = 0x4338000000000000ull;

// Workgroup barrier for the two waves of a ciphertext: LDS writes drained, compiler fence,
// no vmcnt drain (key loads may stay in flight).
__device__ __forceinline__ void pair_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Bounded spin on an LDS counter: returns once *ctr >= target.  A wave that polls more than
// guard.spin_limit times (default 2^22 polls, far beyond any legitimate wait) stops waiting so a
// synchronisation bug cannot hang the GPU, and flags DEV_STATUS_SYNC_TIMEOUT in the device status
// word (a vector atomic): the results of that launch are then wrong, and the host reports it at
// the next synchronisation point (cuda_synchronize_device aborts, concrete_hip_device_status
// returns an error).
__device__ __forceinline__ void spin_until_ge(const uint32_t* ctr, uint32_t target, const SyncGuard& guard) {
  for (uint32_t it = 0;; ++it) {
    if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) break;
    if (it >= guard.spin_limit) {
      __hip_atomic_fetch_or(guard.status, DEV_STATUS_SYNC_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    __builtin_amdgcn_s_sleep(0);  // shortest back-off (s_sleep 1 measured -0.3 %, none -1.8 %)
  }
  asm volatile("" ::: "memory");
}

// Diagnostic cycle stamps (STAMPS builds only; never in the product kernel).
__device__ __forceinline__ uint64_t stamp() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
constexpr int NSTAMP = 10;  // rot+decomp, fwd+xchg, mac, y-xchg, inv+recomb, ring barrier, total, steps, vmcnt, -

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// Optimisation barrier on a register value: the value is computed here and not later (the
// compiler otherwise sinks pure arithmetic past LDS barriers into later phases, where its
// operands stay live and push the kernel past 256 VGPRs).  No instruction is emitted.
__device__ __forceinline__ void pin(uint64_t& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void pin(double& x) { asm volatile("" : "+v"(x)); }

template <int N_WAIT>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N_WAIT >= 0 && N_WAIT < 64, "vmcnt range");
  // gfx9 encoding: vmcnt[3:0] | expcnt[6:4]=7 | lgkmcnt[11:8]=15 | vmcnt_hi[15:14]
  __builtin_amdgcn_s_waitcnt((N_WAIT & 15) | (7 << 4) | (15 << 8) | ((N_WAIT >> 4) << 14));
}

}  // namespace chip
