// runtime.hip — circuit-facing runtime glue (SURVEY.md §8b layer B2, direct GPU route), host code.
//
// Mirrors the memref wrappers a compiled circuit calls on the direct GPU route
// (compiler include/concretelang/Runtime/wrappers.h:240-300; lib/Runtime/wrappers.cpp:70-363)
// with the same memref-descriptor arguments and shape assertions, over a keyset that plays the
// part of RuntimeContext's key caches (include/concretelang/Runtime/context.h:86-145):
//   * keys are registered once in standard form (host copies);
//   * per device, the Fourier key is produced on first use under double-checked locking
//     (context.h:90-115) — converted on the first device that needs it and peer-copied to the
//     others — and stays resident for every later call;
//   * a batched call is split into contiguous slices over the keyset's device list and every
//     slice runs on its own host thread (as the reference's per-device scheduler threads,
//     GPUDFG.cpp:852-895), on a stream and device buffers cached per slice slot across calls:
//     slice r + 1's copies and kernel are issued while slice r's are in flight;
//   * accumulators are built on the device from the LUT rows (lut.hip), so only N words per LUT
//     cross PCIe instead of the (k+1)N-word trivial GLWE (wrappers.cpp:199-209).
// The caller's (pageable) ciphertext and LUT rows go through page-locked staging per slice slot
// (host copies on a few threads, then asynchronous DMA; runtime.hpp HostBuf), so issuing a slice
// never blocks on a copy.  Each slice's thread waits on its own stream only.
// Two name sets: memref_*_hip_u64 take the keyset handle itself; memref_*_cuda_u64 carry the
// reference names and take the caller's runtime context pointer, resolved to a keyset through
// concrete_hip_context_bind / concrete_hip_set_context_resolver.
#include <stdarg.h>

#include <algorithm>
#include <chrono>
#include <thread>
#include <unordered_map>
#include <unordered_set>

#include "common.hpp"
#include "pbs.hpp"
#include "companion.hpp"
#include "runtime.hpp"

namespace chip {

void rt_die(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  fprintf(stderr, "concrete-hip runtime: ");
  vfprintf(stderr, fmt, ap);
  fprintf(stderr, "\n");
  va_end(ap);
  report_hip_state(stderr);
  abort();
}

namespace {

// CONCRETE_HIP_ROUTE_TRACE=1: host-side phase times of every memref-route PBS slice on stderr
// (diagnostic; the device side is the keyset timeline)
bool route_trace() {
  static const bool on = getenv("CONCRETE_HIP_ROUTE_TRACE") != nullptr;
  return on;
}
double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

template <class E>
E* entry(std::vector<E*>& v, uint32_t idx, std::mutex& m, bool create) {
  std::lock_guard<std::mutex> g(m);
  if (idx >= v.size()) {
    if (!create) return nullptr;
    v.resize(idx + 1, nullptr);
  }
  if (!v[idx] && create) v[idx] = new E();
  return v[idx];
}

// live keysets (a context pointer that is itself a keyset resolves to it) and bound contexts
std::mutex g_ctx_mu;
std::unordered_set<const concrete_hip_keyset*> g_live;
std::unordered_map<const void*, concrete_hip_keyset*> g_bound;
concrete_hip_context_resolver g_resolver = nullptr;
void* g_resolver_user = nullptr;

}  // namespace

BskEntry* keyset_bsk_entry(concrete_hip_keyset* ks, uint32_t idx) { return entry(ks->bsk, idx, ks->m, false); }
KskEntry* keyset_ksk_entry(concrete_hip_keyset* ks, uint32_t idx) { return entry(ks->ksk, idx, ks->m, false); }

void* keyset_bsk_on(concrete_hip_keyset* ks, uint32_t idx, uint32_t gpu, hipStream_t s) {
  BskEntry* e = keyset_bsk_entry(ks, idx);
  if (!e) rt_die("bootstrap key index %u not registered", idx);
  RT_ASSERT(gpu < RT_MAX_DEV);
  if (e->dev[gpu]) return e->dev[gpu];
  std::lock_guard<std::mutex> g(e->m);
  if (e->dev[gpu]) return e->dev[gpu];
  const uint64_t bytes = concrete_hip_fourier_bsk_size_bytes(e->n, e->k, e->level, e->N);
  CHIP_CHECK(hipSetDevice((int)gpu));
  void* d = nullptr;
  CHIP_CHECK(hipMalloc(&d, bytes));
  int src = -1;
  for (int o = 0; o < RT_MAX_DEV; ++o)
    if (e->dev[o]) src = o;
  if (src >= 0) {
    // one conversion per keyset; the other devices get the converted bytes (xGMI peer copy)
    CHIP_CHECK(hipMemcpyPeerAsync(d, (int)gpu, e->dev[src], src, bytes, s));
    key_spectrum_copy(d, e->dev[src]);  // the copy carries the source's measured spectrum (keycheck.hip)
  } else if (concrete_hip_convert_bsk(s, gpu, d, e->host.data(), 0, e->n, e->k, e->level, e->N) != 0) {
    rt_die("%s", concrete_hip_last_error());
  }
  // publication only after the key is complete (context.h:110-113)
  CHIP_CHECK(hipStreamSynchronize(s));
  // the host copy is the source of a general-format companion for wide-digit calls
  if (key_format(e->k, e->N, e->level).kind != KeyKind::GENERIC)
    register_std_source(d, e->host.data(), false, gpu, e->n, e->k, e->level, e->N);
  e->dev[gpu] = d;
  return d;
}

void* keyset_ksk_on(concrete_hip_keyset* ks, uint32_t idx, uint32_t gpu, hipStream_t s) {
  KskEntry* e = keyset_ksk_entry(ks, idx);
  if (!e) rt_die("keyswitch key index %u not registered", idx);
  RT_ASSERT(gpu < RT_MAX_DEV);
  if (e->dev[gpu]) return e->dev[gpu];
  std::lock_guard<std::mutex> g(e->m);
  if (e->dev[gpu]) return e->dev[gpu];
  CHIP_CHECK(hipSetDevice((int)gpu));
  void* d = nullptr;
  const uint64_t bytes = e->host.size() * 8ull;
  CHIP_CHECK(hipMalloc(&d, bytes));
  CHIP_CHECK(hipMemcpyAsync(d, e->host.data(), bytes, hipMemcpyHostToDevice, s));
  CHIP_CHECK(hipStreamSynchronize(s));
  track_device_buffer(d);  // resident for the keyset's lifetime: its int8 key bytes may be cached
  e->dev[gpu] = d;
  return d;
}

concrete_hip_keyset* keyset_of_context(const void* ctx) {
  if (!ctx) rt_die("null runtime context");
  concrete_hip_context_resolver fn;
  void* user;
  {
    std::lock_guard<std::mutex> g(g_ctx_mu);
    auto it = g_bound.find(ctx);
    if (it != g_bound.end()) return it->second;
    if (g_live.count((const concrete_hip_keyset*)ctx)) return (concrete_hip_keyset*)ctx;
    fn = g_resolver, user = g_resolver_user;
  }
  concrete_hip_keyset* ks = fn ? fn(ctx, user) : nullptr;
  if (!ks) rt_die("no keyset bound to runtime context %p (concrete_hip_context_bind)", ctx);
  std::lock_guard<std::mutex> g(g_ctx_mu);
  g_bound[ctx] = ks;  // a context's keys do not change during its lifetime (context.h:42-57)
  return ks;
}

namespace {

// contiguous slice of `total` for part r of `parts` (the first total % parts get one more)
void slice_of(uint64_t total, uint64_t parts, uint64_t r, uint64_t& start, uint64_t& count) {
  const uint64_t base = total / parts, extra = total % parts;
  count = base + (r < extra ? 1 : 0);
  start = r * base + (r < extra ? r : extra);
}

void slot_release(SliceSlot& sl) {
  if (!sl.s) return;
  CHIP_CHECK(hipSetDevice((int)sl.gpu));
  CHIP_CHECK(hipStreamSynchronize(sl.s));
  for (int i = 0; i < 4; ++i)
    if (sl.buf[i]) CHIP_CHECK(hipFree(sl.buf[i]));
  for (void* p : sl.retired) CHIP_CHECK(hipFree(p));
  for (int i = 0; i < 4; ++i)
    if (sl.ev[i]) CHIP_CHECK(hipEventDestroy(sl.ev[i]));
  if (sl.status_h) CHIP_CHECK(hipHostFree(sl.status_h));
  release_stream_status((int)sl.gpu, sl.s);
  CHIP_CHECK(hipStreamDestroy(sl.s));
  sl = SliceSlot{};
}

void slot_init(SliceSlot& sl, uint32_t gpu) {
  if (sl.s && sl.gpu == gpu) return;
  slot_release(sl);
  sl.gpu = gpu;
  CHIP_CHECK(hipSetDevice((int)gpu));
  CHIP_CHECK(hipStreamCreateWithFlags(&sl.s, hipStreamNonBlocking));
  for (int i = 0; i < 4; ++i) CHIP_CHECK(hipEventCreate(&sl.ev[i]));
  CHIP_CHECK(hipHostMalloc((void**)&sl.status_h, sizeof(uint32_t), hipHostMallocDefault));
}

SlotSet* take_set(concrete_hip_keyset* ks) {
  std::lock_guard<std::mutex> g(ks->call_m);
  if (!ks->idle_sets.empty()) {
    SlotSet* s = ks->idle_sets.back();
    ks->idle_sets.pop_back();
    return s;
  }
  ks->all_sets.push_back(new SlotSet());
  return ks->all_sets.back();
}

void return_set(concrete_hip_keyset* ks, SlotSet* s) {
  std::lock_guard<std::mutex> g(ks->call_m);
  ks->idle_sets.push_back(s);
}

// grow-only device buffer i of the slot (the slot's stream is idle between calls).  hipFree
// synchronises the whole device, so an outgrown buffer is retired and freed after the slice
// threads join: freeing it here stalled this slice until the other slices' kernels on the same
// device had finished (seen in tests/test_gpu_runtime.py::test_slices_overlap_and_bit_exact).
uint64_t* slot_buf(SliceSlot& sl, int i, uint64_t bytes) {
  bytes = std::max<uint64_t>(bytes, 8);
  if (sl.cap[i] < bytes) {
    if (sl.buf[i]) sl.retired.push_back(sl.buf[i]);
    sl.buf[i] = nullptr;
    CHIP_CHECK(hipMalloc(&sl.buf[i], bytes));
    sl.cap[i] = bytes;
  }
  return (uint64_t*)sl.buf[i];
}

void mark(concrete_hip_keyset*, SliceSlot& sl, int i) {
  // sl.timing is the keyset's flag captured when the call started (re-reading it here
  // raced with set_timing, leaving some events unrecorded before their readback)
  if (sl.timing) CHIP_CHECK(hipEventRecord(sl.ev[i], sl.s));
}

// Run body(slot, start, count) for every contiguous slice of the batch, one host thread per slice
// when there are several, on a slot set of this call's own (concurrent calls on one keyset overlap),
// then read every slice stream's status word on that stream (a PBS whose wave synchronisation gave
// up produced wrong outputs: abort, as the reference's wrappers do).
template <class F>
void run_sliced(concrete_hip_keyset* ks, uint64_t num_samples, F&& body) {
  std::vector<uint32_t> devs;
  {
    std::lock_guard<std::mutex> g(ks->m);
    devs = ks->devices;
  }
  const uint64_t parts = std::max<uint64_t>(1, std::min<uint64_t>(devs.size(), num_samples));
  SlotSet* set = take_set(ks);
  std::vector<SliceSlot>& slots = set->slots;
  if (slots.size() < parts) slots.resize(parts);
  std::vector<uint64_t> start(parts), count(parts);
  for (uint64_t r = 0; r < parts; ++r) {
    slot_init(slots[r], devs[r]);
    slice_of(num_samples, parts, r, start[r], count[r]);
  }
  bool timing;
  uint64_t epoch;
  {
    std::lock_guard<std::mutex> g(ks->call_m);
    timing = ks->timing;
    epoch = ks->timing_epoch;
  }
  for (uint64_t r = 0; r < parts; ++r) slots[r].timing = timing;
  auto slice = [&](uint64_t r) {
    SliceSlot& sl = slots[r];
    body(sl, start[r], count[r]);
    if (take_stream_status((int)sl.gpu, sl.s, sl.status_h) != 0) rt_die("%s", concrete_hip_last_error());
  };
  if (parts == 1) {
    slice(0);
  } else {
    std::vector<std::thread> th;
    th.reserve(parts);
    for (uint64_t r = 0; r < parts; ++r) th.emplace_back(slice, r);
    for (auto& t : th) t.join();
  }
  for (uint64_t r = 0; r < parts; ++r) {
    SliceSlot& sl = slots[r];
    if (sl.retired.empty()) continue;
    CHIP_CHECK(hipSetDevice((int)sl.gpu));
    for (void* p : sl.retired) CHIP_CHECK(hipFree(p));
    sl.retired.clear();
  }
  if (timing) {
    std::vector<double> tl(parts * 6, 0.0);
    std::lock_guard<std::mutex> g(ks->call_m);
    // every event of this call was recorded (sl.timing); timing switched off or re-based since the
    // call started: its events are not on the current time axis, so they are dropped
    const bool same_epoch = ks->timing && ks->timing_epoch == epoch;
    for (uint64_t r = 0; r < parts && same_epoch; ++r) {
      SliceSlot& sl = slots[r];
      if (!ks->timing_base[sl.gpu]) continue;  // a device added after timing was enabled
      CHIP_CHECK(hipSetDevice((int)sl.gpu));
      double* t = &tl[r * 6];
      t[0] = sl.gpu;
      for (int i = 0; i < 4; ++i) {
        float ms = 0.f;
        CHIP_CHECK(hipEventElapsedTime(&ms, ks->timing_base[sl.gpu], sl.ev[i]));
        t[1 + i] = ms;
      }
      t[5] = (double)count[r];
    }
    if (same_epoch) ks->timeline.insert(ks->timeline.end(), tl.begin(), tl.end());
  }
  return_set(ks, set);
}

struct PbsCall {
  const uint64_t* ct0;
  uint64_t* out;
  const uint64_t* tlu;  // num_luts rows of N words, row stride tlu_stride0
  uint64_t num_luts, tlu_stride0;
  uint32_t n, N, level, base_log, k, bsk_index;
};

void run_batched_pbs(concrete_hip_keyset* ks, uint64_t num_samples, const PbsCall& c) {
  if (num_samples == 0) return;
  {
    // the registered key must have the call's parameters: its device format (and size) follows
    // them, so a mismatch would read past the key or reinterpret its layout
    BskEntry* e = keyset_bsk_entry(ks, c.bsk_index);
    if (!e) rt_die("bootstrap key index %u not registered", c.bsk_index);
    RT_ASSERT(e->n == c.n && e->k == c.k && e->N == c.N && e->level == c.level && e->base_log == c.base_log);
  }
  const uint64_t in_w = c.n + 1, out_w = (uint64_t)c.k * c.N + 1, glwe = (uint64_t)(c.k + 1) * c.N;
  run_sliced(ks, num_samples, [&](SliceSlot& sl, uint64_t start, uint64_t count) {
    CHIP_CHECK(hipSetDevice((int)sl.gpu));
    void* fbsk = keyset_bsk_on(ks, c.bsk_index, sl.gpu, sl.s);
    const bool mapped = c.num_luts > 1;
    const uint64_t rows = mapped ? count : 1;
    uint64_t* d_in = slot_buf(sl, 0, count * in_w * 8);
    uint64_t* d_out = slot_buf(sl, 1, count * out_w * 8);
    uint64_t* d_lut = slot_buf(sl, 2, rows * (c.N + glwe) * 8);  // LUT rows, then their accumulators
    uint64_t* d_acc = d_lut + rows * c.N;
    uint64_t* d_lidx = mapped ? slot_buf(sl, 3, count * 8) : nullptr;
    mark(ks, sl, 0);
    const auto t0 = std::chrono::steady_clock::now();
    // the caller's memref is pageable: its rows go through the slot's page-locked staging, whose
    // copy to the device is asynchronous DMA
    sl.stage_in.resize(count * in_w);
    copy_rows(sl.stage_in.data(), in_w, c.ct0 + start * in_w, in_w, count, in_w);
    const double t_in = ms_since(t0);
    CHIP_CHECK(copy_h2d(d_in, sl.stage_in, sl.stage_in.data(), count * in_w * 8, sl.s));
    const double t_h2d = ms_since(t0);
    // one LUT per sample: this slice's rows, indexed 0..count-1 (wrappers.cpp:317-325)
    // (packed into page-locked staging too: a blocking pageable copy here was seen to stall the
    // issue of the call for tens of ms on some boxes)
    const uint64_t* src = c.tlu + (mapped ? start * c.tlu_stride0 : 0);
    sl.stage_lut.resize(rows * c.N);
    copy_rows(sl.stage_lut.data(), c.N, src, c.tlu_stride0, rows, c.N);
    CHIP_CHECK(copy_h2d(d_lut, sl.stage_lut, sl.stage_lut.data(), rows * c.N * 8, sl.s));
    const double t_lut = ms_since(t0);
    launch_trivial_glwe(sl.s, d_acc, d_lut, rows, c.k, c.N);
    if (mapped) launch_iota(sl.s, d_lidx, count);
    mark(ks, sl, 1);
    const double t_acc = ms_since(t0);
    if (concrete_hip_pbs(sl.s, sl.gpu, d_out, nullptr, d_acc, d_lidx, d_in, nullptr, fbsk, c.n, c.k, c.N, c.base_log,
                         c.level, (uint32_t)count, nullptr) != 0)
      rt_die("%s", concrete_hip_last_error());
    mark(ks, sl, 2);
    const double t_pbs = ms_since(t0);
    sl.stage_out.resize(count * out_w);
    CHIP_CHECK(copy_d2h(sl.stage_out.data(), sl.stage_out, d_out, count * out_w * 8, sl.s));
    mark(ks, sl, 3);
    const double t_issue = ms_since(t0);
    CHIP_CHECK(hipStreamSynchronize(sl.s));
    const double t_wait = ms_since(t0);
    copy_rows(c.out + start * out_w, out_w, sl.stage_out.data(), out_w, count, out_w);
    if (route_trace())
      fprintf(stderr, "route trace: slice %llu (%llu rows): stage-in %.2f, h2d %.2f, lut %.2f, acc %.2f, pbs %.2f, "
              "issued %.2f, synced %.2f, copied out %.2f ms\n",
              (unsigned long long)start, (unsigned long long)count, t_in, t_h2d, t_lut, t_acc, t_pbs, t_issue, t_wait,
              ms_since(t0));
  });
}

void run_batched_ks(concrete_hip_keyset* ks, uint64_t num_samples, const uint64_t* ct0, uint64_t* out, uint32_t level,
                    uint32_t base_log, uint32_t n_in, uint32_t n_out, uint32_t ksk_index) {
  if (num_samples == 0) return;
  KskEntry* e = keyset_ksk_entry(ks, ksk_index);
  if (!e) rt_die("keyswitch key index %u not registered", ksk_index);
  RT_ASSERT(e->level == level && e->base_log == base_log && e->n_in == n_in && e->n_out == n_out);
  const uint64_t in_w = n_in + 1, out_w = n_out + 1;
  run_sliced(ks, num_samples, [&](SliceSlot& sl, uint64_t start, uint64_t count) {
    CHIP_CHECK(hipSetDevice((int)sl.gpu));
    void* dk = keyset_ksk_on(ks, ksk_index, sl.gpu, sl.s);
    uint64_t* d_in = slot_buf(sl, 0, count * in_w * 8);
    uint64_t* d_out = slot_buf(sl, 1, count * out_w * 8);
    mark(ks, sl, 0);
    sl.stage_in.resize(count * in_w);
    copy_rows(sl.stage_in.data(), in_w, ct0 + start * in_w, in_w, count, in_w);
    CHIP_CHECK(copy_h2d(d_in, sl.stage_in, sl.stage_in.data(), count * in_w * 8, sl.s));
    mark(ks, sl, 1);
    if (concrete_hip_keyswitch(sl.s, sl.gpu, d_out, nullptr, d_in, nullptr, (const uint64_t*)dk, n_in, n_out, base_log,
                               level, (uint32_t)count) != 0)
      rt_die("%s", concrete_hip_last_error());
    mark(ks, sl, 2);
    sl.stage_out.resize(count * out_w);
    CHIP_CHECK(copy_d2h(sl.stage_out.data(), sl.stage_out, d_out, count * out_w * 8, sl.s));
    mark(ks, sl, 3);
    CHIP_CHECK(hipStreamSynchronize(sl.s));
    copy_rows(out + start * out_w, out_w, sl.stage_out.data(), out_w, count, out_w);
  });
}

void free_keys(concrete_hip_keyset* ks) {
  for (BskEntry* e : ks->bsk) {
    if (!e) continue;
    for (int d = 0; d < RT_MAX_DEV; ++d)
      if (e->dev[d]) {
        CHIP_CHECK(hipSetDevice(d));
        release_std_source(e->dev[d]);  // and its general-format companion, if one was built
        CHIP_CHECK(hipFree(e->dev[d]));
      }
    delete e;
  }
  for (KskEntry* e : ks->ksk) {
    if (!e) continue;
    for (int d = 0; d < RT_MAX_DEV; ++d)
      if (e->dev[d]) {
        CHIP_CHECK(hipSetDevice(d));
        release_key_bytes(e->dev[d], nullptr, true);  // int8 key bytes cached for this KSK
        CHIP_CHECK(hipFree(e->dev[d]));
      }
    delete e;
  }
}

}  // namespace
}  // namespace chip

using namespace chip;

extern "C" {

concrete_hip_keyset* concrete_hip_keyset_create(void) {
  concrete_hip_keyset* ks = new concrete_hip_keyset();
  std::lock_guard<std::mutex> g(g_ctx_mu);
  g_live.insert(ks);
  return ks;
}

void concrete_hip_keyset_destroy(concrete_hip_keyset* ks) {
  if (!ks) return;
  {
    std::lock_guard<std::mutex> g(g_ctx_mu);
    g_live.erase(ks);
    for (auto it = g_bound.begin(); it != g_bound.end();)
      it = it->second == ks ? g_bound.erase(it) : std::next(it);
  }
  for (SlotSet* set : ks->all_sets) {
    for (auto& sl : set->slots) slot_release(sl);
    delete set;
  }
  for (int d = 0; d < RT_MAX_DEV; ++d)
    if (ks->timing_base[d]) {
      CHIP_CHECK(hipSetDevice(d));
      CHIP_CHECK(hipEventDestroy(ks->timing_base[d]));
    }
  free_keys(ks);
  delete ks;
}

int concrete_hip_keyset_add_bsk(concrete_hip_keyset* ks, uint32_t bsk_index, const uint64_t* bsk,
                                uint32_t input_lwe_dim, uint32_t glwe_dim, uint32_t level, uint32_t base_log,
                                uint32_t poly_size) {
  if (!ks || !bsk || input_lwe_dim == 0) {
    set_error("keyset_add_bsk: bad argument");
    return -3;
  }
  if (!concrete_hip_pbs_supported(glwe_dim, poly_size, level, base_log)) {
    set_error("keyset_add_bsk: unsupported parameters k=%u N=%u level=%u base_log=%u", glwe_dim, poly_size, level,
              base_log);
    return -2;
  }
  BskEntry* e = entry(ks->bsk, bsk_index, ks->m, true);
  std::lock_guard<std::mutex> g(e->m);
  for (int d = 0; d < RT_MAX_DEV; ++d)
    if (e->dev[d]) {
      set_error("keyset_add_bsk: index %u already resident", bsk_index);
      return -3;
    }
  const uint64_t len = (uint64_t)input_lwe_dim * level * ((uint64_t)glwe_dim + 1) * ((uint64_t)glwe_dim + 1) * poly_size;
  e->host.assign(bsk, bsk + len);
  e->n = input_lwe_dim, e->k = glwe_dim, e->level = level, e->base_log = base_log, e->N = poly_size;
  return 0;
}

int concrete_hip_keyset_add_ksk(concrete_hip_keyset* ks, uint32_t ksk_index, const uint64_t* ksk, uint32_t level,
                                uint32_t base_log, uint32_t input_lwe_dim, uint32_t output_lwe_dim) {
  if (!ks || !ksk) {
    set_error("keyset_add_ksk: bad argument");
    return -3;
  }
  // 64-bit checks: the parameters may come from an imported key message (keyio.cpp)
  if (!keyswitch_params_ok(level, base_log, input_lwe_dim, output_lwe_dim)) {
    set_error("keyset_add_ksk: unsupported parameters level=%u base_log=%u n_in=%u n_out=%u", level, base_log,
              input_lwe_dim, output_lwe_dim);
    return -2;
  }
  KskEntry* e = entry(ks->ksk, ksk_index, ks->m, true);
  std::lock_guard<std::mutex> g(e->m);
  for (int d = 0; d < RT_MAX_DEV; ++d)
    if (e->dev[d]) {
      set_error("keyset_add_ksk: index %u already resident", ksk_index);
      return -3;
    }
  const uint64_t len = (uint64_t)input_lwe_dim * level * ((uint64_t)output_lwe_dim + 1);
  e->host.assign(ksk, ksk + len);
  e->level = level, e->base_log = base_log, e->n_in = input_lwe_dim, e->n_out = output_lwe_dim;
  return 0;
}

int concrete_hip_keyset_set_devices(concrete_hip_keyset* ks, const uint32_t* devices, uint32_t count) {
  if (!ks || !devices || count == 0) {
    set_error("keyset_set_devices: bad argument");
    return -3;
  }
  const int nd = concrete_hip_device_count();
  for (uint32_t i = 0; i < count; ++i)
    if ((int)devices[i] >= nd || devices[i] >= RT_MAX_DEV) {
      set_error("keyset_set_devices: device %u not visible", devices[i]);
      return -3;
    }
  // calls in flight keep the devices they started with (run_sliced copies the list)
  std::lock_guard<std::mutex> g(ks->m);
  ks->devices.assign(devices, devices + count);
  return 0;
}

void concrete_hip_keyset_set_timing(concrete_hip_keyset* ks, int enable) {
  if (!ks) return;
  std::vector<uint32_t> devs;
  {
    std::lock_guard<std::mutex> g(ks->m);
    devs = ks->devices;
  }
  std::lock_guard<std::mutex> call(ks->call_m);
  ks->timeline.clear();
  ks->timing = false;
  ++ks->timing_epoch;
  if (!enable) return;
  // one base event per device, in the past of every later call: slices of different calls (and
  // streams) share the time axis
  int prev = 0;
  CHIP_CHECK(hipGetDevice(&prev));
  for (uint32_t d : devs) {
    CHIP_CHECK(hipSetDevice((int)d));
    if (!ks->timing_base[d]) CHIP_CHECK(hipEventCreate(&ks->timing_base[d]));
    CHIP_CHECK(hipEventRecord(ks->timing_base[d], nullptr));
    CHIP_CHECK(hipEventSynchronize(ks->timing_base[d]));
  }
  CHIP_CHECK(hipSetDevice(prev));
  ks->timing = true;
}

uint32_t concrete_hip_keyset_timeline(concrete_hip_keyset* ks, double* out, uint32_t max_slices) {
  if (!ks) return 0;
  std::lock_guard<std::mutex> call(ks->call_m);
  const uint32_t n = (uint32_t)(ks->timeline.size() / 6);
  if (out) std::copy(ks->timeline.begin(), ks->timeline.begin() + 6 * std::min(n, max_slices), out);
  return n;
}

int concrete_hip_context_bind(const void* runtime_context, concrete_hip_keyset* ks) {
  if (!runtime_context) {
    set_error("context_bind: null context");
    return -3;
  }
  std::lock_guard<std::mutex> g(g_ctx_mu);
  if (ks) {
    if (!g_live.count(ks)) {
      set_error("context_bind: %p is not a live keyset", (void*)ks);
      return -3;
    }
    g_bound[runtime_context] = ks;
  } else {
    g_bound.erase(runtime_context);
  }
  return 0;
}

void concrete_hip_set_context_resolver(concrete_hip_context_resolver fn, void* user) {
  std::lock_guard<std::mutex> g(g_ctx_mu);
  g_resolver = fn, g_resolver_user = user;
}

// ------------------------------------------------------------------------------------------
// memref_*_hip_u64: the keyset handle is the context
// ------------------------------------------------------------------------------------------
void memref_batched_bootstrap_lwe_hip_u64(uint64_t* out_allocated, uint64_t* out_aligned, uint64_t out_offset,
                                          uint64_t out_size0, uint64_t out_size1, uint64_t out_stride0,
                                          uint64_t out_stride1, uint64_t* ct0_allocated, uint64_t* ct0_aligned,
                                          uint64_t ct0_offset, uint64_t ct0_size0, uint64_t ct0_size1,
                                          uint64_t ct0_stride0, uint64_t ct0_stride1, uint64_t* tlu_allocated,
                                          uint64_t* tlu_aligned, uint64_t tlu_offset, uint64_t tlu_size,
                                          uint64_t tlu_stride, uint32_t input_lwe_dim, uint32_t poly_size,
                                          uint32_t level, uint32_t base_log, uint32_t glwe_dim, uint32_t bsk_index,
                                          concrete_hip_keyset* context) {
  (void)out_allocated, (void)ct0_allocated, (void)tlu_allocated;
  // wrappers.cpp:174-175
  RT_ASSERT(out_size0 == ct0_size0);
  RT_ASSERT(out_size1 == (uint64_t)glwe_dim * poly_size + 1);
  RT_ASSERT(ct0_size1 == (uint64_t)input_lwe_dim + 1);
  RT_ASSERT(tlu_size == poly_size && tlu_stride == 1);
  RT_ASSERT(out_stride1 == 1 && out_stride0 == out_size1 && ct0_stride1 == 1 && ct0_stride0 == ct0_size1);
  RT_ASSERT(context);
  run_batched_pbs(context, out_size0,
                  PbsCall{ct0_aligned + ct0_offset, out_aligned + out_offset, tlu_aligned + tlu_offset, 1, poly_size,
                          input_lwe_dim, poly_size, level, base_log, glwe_dim, bsk_index});
}

void memref_batched_mapped_bootstrap_lwe_hip_u64(
    uint64_t* out_allocated, uint64_t* out_aligned, uint64_t out_offset, uint64_t out_size0, uint64_t out_size1,
    uint64_t out_stride0, uint64_t out_stride1, uint64_t* ct0_allocated, uint64_t* ct0_aligned, uint64_t ct0_offset,
    uint64_t ct0_size0, uint64_t ct0_size1, uint64_t ct0_stride0, uint64_t ct0_stride1, uint64_t* tlu_allocated,
    uint64_t* tlu_aligned, uint64_t tlu_offset, uint64_t tlu_size0, uint64_t tlu_size1, uint64_t tlu_stride0,
    uint64_t tlu_stride1, uint32_t input_lwe_dim, uint32_t poly_size, uint32_t level, uint32_t base_log,
    uint32_t glwe_dim, uint32_t bsk_index, concrete_hip_keyset* context) {
  (void)out_allocated, (void)ct0_allocated, (void)tlu_allocated;
  // wrappers.cpp:269-272, 308-312
  RT_ASSERT(out_size0 == ct0_size0);
  RT_ASSERT(out_size1 == (uint64_t)glwe_dim * poly_size + 1);
  RT_ASSERT(ct0_size1 == (uint64_t)input_lwe_dim + 1);
  RT_ASSERT((out_size0 == tlu_size0 || tlu_size0 == 1) && "Number of LUTs does not match batch size");
  RT_ASSERT(tlu_size1 == poly_size && tlu_stride1 == 1 && tlu_stride0 >= poly_size);
  RT_ASSERT(out_stride1 == 1 && out_stride0 == out_size1 && ct0_stride1 == 1 && ct0_stride0 == ct0_size1);
  RT_ASSERT(context);
  run_batched_pbs(context, out_size0,
                  PbsCall{ct0_aligned + ct0_offset, out_aligned + out_offset, tlu_aligned + tlu_offset, tlu_size0,
                          tlu_stride0, input_lwe_dim, poly_size, level, base_log, glwe_dim, bsk_index});
}

void memref_bootstrap_lwe_hip_u64(uint64_t* out_allocated, uint64_t* out_aligned, uint64_t out_offset,
                                  uint64_t out_size, uint64_t out_stride, uint64_t* ct0_allocated,
                                  uint64_t* ct0_aligned, uint64_t ct0_offset, uint64_t ct0_size, uint64_t ct0_stride,
                                  uint64_t* tlu_allocated, uint64_t* tlu_aligned, uint64_t tlu_offset,
                                  uint64_t tlu_size, uint64_t tlu_stride, uint32_t input_lwe_dim, uint32_t poly_size,
                                  uint32_t level, uint32_t base_log, uint32_t glwe_dim, uint32_t bsk_index,
                                  concrete_hip_keyset* context) {
  // a single ciphertext is a batch of one (wrappers.cpp:88-106)
  RT_ASSERT(out_stride == 1 && ct0_stride == 1);
  memref_batched_bootstrap_lwe_hip_u64(out_allocated, out_aligned, out_offset, 1, out_size, out_size, 1,
                                       ct0_allocated, ct0_aligned, ct0_offset, 1, ct0_size, ct0_size, 1,
                                       tlu_allocated, tlu_aligned, tlu_offset, tlu_size, tlu_stride, input_lwe_dim,
                                       poly_size, level, base_log, glwe_dim, bsk_index, context);
}

void memref_batched_keyswitch_lwe_hip_u64(uint64_t* out_allocated, uint64_t* out_aligned, uint64_t out_offset,
                                          uint64_t out_size0, uint64_t out_size1, uint64_t out_stride0,
                                          uint64_t out_stride1, uint64_t* ct0_allocated, uint64_t* ct0_aligned,
                                          uint64_t ct0_offset, uint64_t ct0_size0, uint64_t ct0_size1,
                                          uint64_t ct0_stride0, uint64_t ct0_stride1, uint32_t level,
                                          uint32_t base_log, uint32_t input_lwe_dim, uint32_t output_lwe_dim,
                                          uint32_t ksk_index, concrete_hip_keyset* context) {
  (void)out_allocated, (void)ct0_allocated;
  // wrappers.cpp:118-120
  RT_ASSERT(out_size0 == ct0_size0);
  RT_ASSERT(out_size1 == (uint64_t)output_lwe_dim + 1 && ct0_size1 == (uint64_t)input_lwe_dim + 1);
  RT_ASSERT(out_stride1 == 1 && out_stride0 == out_size1 && ct0_stride1 == 1 && ct0_stride0 == ct0_size1);
  RT_ASSERT(context);
  run_batched_ks(context, out_size0, ct0_aligned + ct0_offset, out_aligned + out_offset, level, base_log,
                 input_lwe_dim, output_lwe_dim, ksk_index);
}

void memref_keyswitch_lwe_hip_u64(uint64_t* out_allocated, uint64_t* out_aligned, uint64_t out_offset,
                                  uint64_t out_size, uint64_t out_stride, uint64_t* ct0_allocated,
                                  uint64_t* ct0_aligned, uint64_t ct0_offset, uint64_t ct0_size, uint64_t ct0_stride,
                                  uint32_t level, uint32_t base_log, uint32_t input_lwe_dim,
                                  uint32_t output_lwe_dim, uint32_t ksk_index, concrete_hip_keyset* context) {
  // wrappers.cpp:70-86
  RT_ASSERT(out_stride == 1 && ct0_stride == 1);
  memref_batched_keyswitch_lwe_hip_u64(out_allocated, out_aligned, out_offset, 1, out_size, out_size, 1,
                                       ct0_allocated, ct0_aligned, ct0_offset, 1, ct0_size, ct0_size, 1, level,
                                       base_log, input_lwe_dim, output_lwe_dim, ksk_index, context);
}

// ------------------------------------------------------------------------------------------
// memref_*_cuda_u64: the reference's names (wrappers.h:246-300); the last argument is the
// caller's runtime context, resolved to its keyset
// ------------------------------------------------------------------------------------------
void memref_keyswitch_lwe_cuda_u64(uint64_t* out_allocated, uint64_t* out_aligned, uint64_t out_offset,
                                   uint64_t out_size, uint64_t out_stride, uint64_t* ct0_allocated,
                                   uint64_t* ct0_aligned, uint64_t ct0_offset, uint64_t ct0_size,
                                   uint64_t ct0_stride, uint32_t level, uint32_t base_log, uint32_t input_lwe_dim,
                                   uint32_t output_lwe_dim, uint32_t ksk_index, void* context) {
  memref_keyswitch_lwe_hip_u64(out_allocated, out_aligned, out_offset, out_size, out_stride, ct0_allocated,
                               ct0_aligned, ct0_offset, ct0_size, ct0_stride, level, base_log, input_lwe_dim,
                               output_lwe_dim, ksk_index, keyset_of_context(context));
}

void memref_bootstrap_lwe_cuda_u64(uint64_t* out_allocated, uint64_t* out_aligned, uint64_t out_offset,
                                   uint64_t out_size, uint64_t out_stride, uint64_t* ct0_allocated,
                                   uint64_t* ct0_aligned, uint64_t ct0_offset, uint64_t ct0_size,
                                   uint64_t ct0_stride, uint64_t* tlu_allocated, uint64_t* tlu_aligned,
                                   uint64_t tlu_offset, uint64_t tlu_size, uint64_t tlu_stride,
                                   uint32_t input_lwe_dim, uint32_t poly_size, uint32_t level, uint32_t base_log,
                                   uint32_t glwe_dim, uint32_t bsk_index, void* context) {
  memref_bootstrap_lwe_hip_u64(out_allocated, out_aligned, out_offset, out_size, out_stride, ct0_allocated,
                               ct0_aligned, ct0_offset, ct0_size, ct0_stride, tlu_allocated, tlu_aligned, tlu_offset,
                               tlu_size, tlu_stride, input_lwe_dim, poly_size, level, base_log, glwe_dim, bsk_index,
                               keyset_of_context(context));
}

void memref_batched_keyswitch_lwe_cuda_u64(uint64_t* out_allocated, uint64_t* out_aligned, uint64_t out_offset,
                                           uint64_t out_size0, uint64_t out_size1, uint64_t out_stride0,
                                           uint64_t out_stride1, uint64_t* ct0_allocated, uint64_t* ct0_aligned,
                                           uint64_t ct0_offset, uint64_t ct0_size0, uint64_t ct0_size1,
                                           uint64_t ct0_stride0, uint64_t ct0_stride1, uint32_t level,
                                           uint32_t base_log, uint32_t input_lwe_dim, uint32_t output_lwe_dim,
                                           uint32_t ksk_index, void* context) {
  memref_batched_keyswitch_lwe_hip_u64(out_allocated, out_aligned, out_offset, out_size0, out_size1, out_stride0,
                                       out_stride1, ct0_allocated, ct0_aligned, ct0_offset, ct0_size0, ct0_size1,
                                       ct0_stride0, ct0_stride1, level, base_log, input_lwe_dim, output_lwe_dim,
                                       ksk_index, keyset_of_context(context));
}

void memref_batched_bootstrap_lwe_cuda_u64(uint64_t* out_allocated, uint64_t* out_aligned, uint64_t out_offset,
                                           uint64_t out_size0, uint64_t out_size1, uint64_t out_stride0,
                                           uint64_t out_stride1, uint64_t* ct0_allocated, uint64_t* ct0_aligned,
                                           uint64_t ct0_offset, uint64_t ct0_size0, uint64_t ct0_size1,
                                           uint64_t ct0_stride0, uint64_t ct0_stride1, uint64_t* tlu_allocated,
                                           uint64_t* tlu_aligned, uint64_t tlu_offset, uint64_t tlu_size,
                                           uint64_t tlu_stride, uint32_t input_lwe_dim, uint32_t poly_size,
                                           uint32_t level, uint32_t base_log, uint32_t glwe_dim, uint32_t bsk_index,
                                           void* context) {
  memref_batched_bootstrap_lwe_hip_u64(out_allocated, out_aligned, out_offset, out_size0, out_size1, out_stride0,
                                       out_stride1, ct0_allocated, ct0_aligned, ct0_offset, ct0_size0, ct0_size1,
                                       ct0_stride0, ct0_stride1, tlu_allocated, tlu_aligned, tlu_offset, tlu_size,
                                       tlu_stride, input_lwe_dim, poly_size, level, base_log, glwe_dim, bsk_index,
                                       keyset_of_context(context));
}

void memref_batched_mapped_bootstrap_lwe_cuda_u64(
    uint64_t* out_allocated, uint64_t* out_aligned, uint64_t out_offset, uint64_t out_size0, uint64_t out_size1,
    uint64_t out_stride0, uint64_t out_stride1, uint64_t* ct0_allocated, uint64_t* ct0_aligned, uint64_t ct0_offset,
    uint64_t ct0_size0, uint64_t ct0_size1, uint64_t ct0_stride0, uint64_t ct0_stride1, uint64_t* tlu_allocated,
    uint64_t* tlu_aligned, uint64_t tlu_offset, uint64_t tlu_size0, uint64_t tlu_size1, uint64_t tlu_stride0,
    uint64_t tlu_stride1, uint32_t input_lwe_dim, uint32_t poly_size, uint32_t level, uint32_t base_log,
    uint32_t glwe_dim, uint32_t bsk_index, void* context) {
  memref_batched_mapped_bootstrap_lwe_hip_u64(
      out_allocated, out_aligned, out_offset, out_size0, out_size1, out_stride0, out_stride1, ct0_allocated,
      ct0_aligned, ct0_offset, ct0_size0, ct0_size1, ct0_stride0, ct0_stride1, tlu_allocated, tlu_aligned, tlu_offset,
      tlu_size0, tlu_size1, tlu_stride0, tlu_stride1, input_lwe_dim, poly_size, level, base_log, glwe_dim, bsk_index,
      keyset_of_context(context));
}

}  // extern "C"
