// runtime.hpp — host-side internals shared by the circuit-facing runtime glue (runtime.hip) and
// the SDFG stream emulator (sdfg.hip): the keyset (the RuntimeContext key caches of compiler
// include/concretelang/Runtime/context.h:86-145), its device-resident keys, and the device
// helpers both routes launch (lut.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <thread>
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

// Host memory the devices copy from and to: grow-only page-locked memory (hipHostMalloc), so H2D /
// D2H copies are DMA at link speed and asynchronous (pageable copies are staged by the runtime in
// small blocking pieces: the stream emulator's KS -> PBS route at cfg2 spent ~25 of its 66 ms per
// 4096 samples in them); pageable fallback when pinning fails.  Contents are not zeroed on growth.
// Used for the stream emulator's stream buffers (sdfg.hip) and the memref route's staging
// (runtime.hip).
class HostBuf {
 public:
  HostBuf() = default;
  HostBuf(const HostBuf&) = delete;
  HostBuf& operator=(const HostBuf&) = delete;
  HostBuf(HostBuf&& o) noexcept : p_(o.p_), n_(o.n_), cap_(o.cap_), pinned_(o.pinned_) { o.p_ = nullptr, o.n_ = o.cap_ = 0; }
  HostBuf& operator=(HostBuf&& o) noexcept {
    if (this != &o) {
      release();
      p_ = o.p_, n_ = o.n_, cap_ = o.cap_, pinned_ = o.pinned_;
      o.p_ = nullptr, o.n_ = o.cap_ = 0;
    }
    return *this;
  }
  ~HostBuf() { release(); }
  uint64_t* data() { return p_; }
  const uint64_t* data() const { return p_; }
  uint64_t size() const { return n_; }
  bool pinned() const { return pinned_; }
  uint64_t& operator[](uint64_t i) { return p_[i]; }
  const uint64_t* begin() const { return p_; }
  const uint64_t* end() const { return p_ + n_; }
  void resize(uint64_t n) {
    if (n > cap_) {
      uint64_t* q = nullptr;
      bool pinned = hipHostMalloc((void**)&q, std::max<uint64_t>(n, 1) * 8, hipHostMallocDefault) == hipSuccess;
      if (!pinned) {
        (void)hipGetLastError();
        q = (uint64_t*)malloc(std::max<uint64_t>(n, 1) * 8);
        if (!q) rt_die("host buffer: out of host memory (%llu words)", (unsigned long long)n);
      }
      if (n_) memcpy(q, p_, n_ * 8);
      release();
      p_ = q, cap_ = n, pinned_ = pinned;
    }
    n_ = n;
  }

 private:
  void release() {
    if (!p_) return;
    if (pinned_) (void)hipHostFree(p_);
    else free(p_);
    p_ = nullptr, cap_ = 0;
  }
  uint64_t* p_ = nullptr;
  uint64_t n_ = 0, cap_ = 0;
  bool pinned_ = false;
};

// Host <-> device copy of a HostBuf range: asynchronous DMA when page-locked; the blocking form
// for the pageable fallback (the staged tail of an asynchronous pageable D2H was seen to land after
// hipStreamSynchronize had returned).
inline hipError_t copy_h2d(void* dev, const HostBuf& h, const uint64_t* src, uint64_t bytes, hipStream_t s) {
  return h.pinned() ? hipMemcpyAsync(dev, src, bytes, hipMemcpyHostToDevice, s)
                    : hipMemcpyWithStream(dev, src, bytes, hipMemcpyHostToDevice, s);
}
inline hipError_t copy_d2h(uint64_t* dst, const HostBuf& h, const void* dev, uint64_t bytes, hipStream_t s) {
  return h.pinned() ? hipMemcpyAsync(dst, dev, bytes, hipMemcpyDeviceToHost, s)
                    : hipMemcpyWithStream(dst, dev, bytes, hipMemcpyDeviceToHost, s);
}

// Row-wise copy between host memrefs and stream buffers, split over a few threads for large
// batches (a single core moves ~10 GB/s: 3-4 ms per 4096 x 1025 words).
inline void copy_rows(uint64_t* dst, uint64_t dst_stride, const uint64_t* src, uint64_t src_stride, uint64_t rows,
               uint64_t cols) {
  auto part = [&](uint64_t r0, uint64_t r1) {
    if (dst_stride == cols && src_stride == cols) {
      memcpy(dst + r0 * cols, src + r0 * cols, (r1 - r0) * cols * 8);
      return;
    }
    for (uint64_t r = r0; r < r1; ++r) memcpy(dst + r * dst_stride, src + r * src_stride, cols * 8);
  };
  const uint64_t bytes = rows * cols * 8;
  const uint64_t nt = std::min<uint64_t>(std::min<uint64_t>(8, rows), bytes >> 22);  // >= 4 MB per thread
  if (nt <= 1) {
    part(0, rows);
    return;
  }
  std::vector<std::thread> th;
  for (uint64_t t = 0; t < nt; ++t) th.emplace_back(part, rows * t / nt, rows * (t + 1) / nt);
  for (auto& x : th) x.join();
}

// Per-slice resources of the memref route, reused across calls (grow-only device buffers, one
// non-blocking stream, timing events).  Slot r serves slice r of a call.
struct SliceSlot {
  uint32_t gpu = 0;
  hipStream_t s = nullptr;
  void* buf[4] = {};      // in, out, luts (+ accumulators), lut indexes
  uint64_t cap[4] = {};   // bytes
  hipEvent_t ev[4] = {};  // start, after H2D, after kernel, after D2H
  std::vector<void*> retired;  // outgrown buffers, freed once every slice thread has joined
  HostBuf stage_in, stage_out, stage_lut;  // page-locked staging of the caller's (pageable) memrefs
  uint32_t* status_h = nullptr;  // page-locked landing word of the stream-ordered status read
  bool timing = false;           // this call records its events (captured once at the call's start)
};

// The slots of one call.  A keyset keeps a pool of them: concurrent calls on one keyset (several
// RuntimeContexts sharing it) each take their own set, so they overlap instead of
// queueing behind one lock (round 4; the reference runs one scheduler thread per device,
// GPUDFG.cpp:852-895).
struct SlotSet {
  std::vector<SliceSlot> slots;
};

// Device status of the work issued so far on stream s (abi.hip): the status word is read on s itself
// into h (page-locked) and s is synchronised — no device-wide synchronisation, so other streams'
// calls keep running.  Returns 0, or -4 with the message set when a PBS wave synchronisation gave up.
int take_stream_status(int gpu, hipStream_t s, uint32_t* h);
// abi.hip: a stream about to be destroyed (its work synchronised): clear its word, free its slot
void release_stream_status(int gpu, hipStream_t s);

}  // namespace chip

struct concrete_hip_keyset {
  std::mutex m;
  std::vector<chip::BskEntry*> bsk;  // indexed by bsk_index
  std::vector<chip::KskEntry*> ksk;
  std::vector<uint32_t> devices{0};
  // call_m guards the pool and the timing state; it is held only to take or return a slot set
  std::mutex call_m;
  std::vector<chip::SlotSet*> idle_sets, all_sets;
  bool timing = false;
  uint64_t timing_epoch = 0;  // bumped by every set_timing: a call's events are read back only in its epoch
  hipEvent_t timing_base[chip::RT_MAX_DEV] = {};  // recorded when timing was enabled, per device
  std::vector<double> timeline;  // 6 per slice of every call since timing was enabled
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
