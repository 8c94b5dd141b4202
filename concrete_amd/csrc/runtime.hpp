// runtime.hpp — host-side internals shared by the circuit-facing runtime glue (runtime.hip) and
// the SDFG stream emulator (sdfg.hip): the keyset (the RuntimeContext key caches of compiler
// include/concretelang/Runtime/context.h:86-145), its device-resident keys, and the device
// helpers both routes launch (lut.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>
#include <vector>

#include "../../include/concrete_hip.h"

namespace chip {

constexpr int RT_MAX_DEV = 16;

[[noreturn]] void rt_die(const char* fmt, ...);
#define RT_ASSERT(cond)                                          \
  do {                                                           \
    if (!(cond)) ::chip::rt_die("assertion failed: %s", #cond);  \
  } while (0)

struct BskEntry {
  std::vector<uint64_t> host;
  uint32_t n = 0, k = 0, level = 0, base_log = 0, N = 0;
  void* dev[RT_MAX_DEV] = {};
  std::mutex m;
};
struct KskEntry {
  std::vector<uint64_t> host;
  uint32_t level = 0, base_log = 0, n_in = 0, n_out = 0;
  void* dev[RT_MAX_DEV] = {};
  std::mutex m;
};

// Per-slice resources of the memref route, reused across calls (grow-only device buffers, one
// non-blocking stream, timing events).  Slot r serves slice r of a call.
struct SliceSlot {
  uint32_t gpu = 0;
  hipStream_t s = nullptr;
  void* buf[4] = {};      // in, out, luts (+ accumulators), lut indexes
  uint64_t cap[4] = {};   // bytes
  hipEvent_t ev[5] = {};  // start, after H2D, after kernel, after D2H; ev[4] unused
  std::vector<void*> retired;  // outgrown buffers, freed once every slice thread has joined
};

}  // namespace chip

struct concrete_hip_keyset {
  std::mutex m;
  std::vector<chip::BskEntry*> bsk;  // indexed by bsk_index
  std::vector<chip::KskEntry*> ksk;
  std::vector<uint32_t> devices{0};
  // one memref call at a time uses the slots (a circuit's calls are sequential per context)
  std::mutex call_m;
  std::vector<chip::SliceSlot> slots;
  bool timing = false;
  std::vector<double> timeline;  // 6 per slice of the last call (concrete_hip_keyset_timeline)
};

namespace chip {

// device Fourier key of bsk_index on `gpu`, converted (or peer-copied) on first use
void* keyset_bsk_on(concrete_hip_keyset* ks, uint32_t idx, uint32_t gpu, hipStream_t s);
// device copy of the standard KSK on `gpu`, uploaded on first use
void* keyset_ksk_on(concrete_hip_keyset* ks, uint32_t idx, uint32_t gpu, hipStream_t s);
BskEntry* keyset_bsk_entry(concrete_hip_keyset* ks, uint32_t idx);
KskEntry* keyset_ksk_entry(concrete_hip_keyset* ks, uint32_t idx);
// keyset bound to a runtime context pointer (concrete_hip_context_bind / resolver); aborts if none
concrete_hip_keyset* keyset_of_context(const void* ctx);

// lut.hip: accumulators = trivial GLWEs (k zero masks, body = LUT row) built on the device from
// num_luts LUT rows of N words (compiler lib/Runtime/wrappers.cpp:199-209, GPUDFG.cpp:1122-1136)
void launch_trivial_glwe(hipStream_t s, uint64_t* acc, const uint64_t* luts, uint64_t num_luts, uint32_t k,
                         uint32_t N);
// lut.hip: idx[i] = i for i < count
void launch_iota(hipStream_t s, uint64_t* idx, uint64_t count);
// linear.hip: the four linear ops with a per-sample (b_stride 1) or broadcast (b_stride 0) operand
void launch_linear_op(hipStream_t s, int op, uint64_t* out, const uint64_t* a, const uint64_t* b,
                      uint64_t b_stride, uint32_t lwe_dimension, uint64_t num_samples);
enum { LINOP_ADD = 0, LINOP_ADD_PT = 1, LINOP_MUL_CT = 2, LINOP_NEG = 3 };

}  // namespace chip
