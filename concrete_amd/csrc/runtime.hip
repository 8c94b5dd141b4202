// runtime.hip — circuit-facing runtime glue (SURVEY.md §8b layer B2), host code.
//
// Mirrors the memref wrappers the compiled circuit calls on the direct GPU route
// (compiler include/concretelang/Runtime/wrappers.h:240-300; lib/Runtime/wrappers.cpp:88-363)
// with the same memref-descriptor arguments and shape assertions, over an opaque keyset that
// plays the part of RuntimeContext's key caches (include/concretelang/Runtime/context.h:86-145):
//   * keys are registered once in standard form (host copies);
//   * per device, the Fourier key is produced on first use under double-checked locking
//     (context.h:90-115) — converted on the first device that needs it and peer-copied to the
//     others — and stays resident for every later call;
//   * a batched call is split into contiguous slices over the keyset's device list, one stream
//     per slice, all slices in flight before the single synchronisation.
#include <algorithm>
#include <mutex>
#include <vector>

#include "../../include/concrete_hip.h"
#include "common.hpp"
#include "pbs.hpp"

using namespace chip;

namespace {

constexpr int MAX_DEV = 16;

[[noreturn]] void die(const char* what) {
  fprintf(stderr, "concrete-hip runtime: %s\n", what);
  abort();
}
#define RT_ASSERT(cond)                                     \
  do {                                                      \
    if (!(cond)) die("assertion failed: " #cond);           \
  } while (0)

struct BskEntry {
  std::vector<uint64_t> host;
  uint32_t n = 0, k = 0, level = 0, base_log = 0, N = 0;
  void* dev[MAX_DEV] = {};
  std::mutex m;
};
struct KskEntry {
  std::vector<uint64_t> host;
  uint32_t level = 0, base_log = 0, n_in = 0, n_out = 0;
  void* dev[MAX_DEV] = {};
  std::mutex m;
};

}  // namespace

struct concrete_hip_keyset {
  std::mutex m;
  std::vector<BskEntry*> bsk;  // indexed by bsk_index
  std::vector<KskEntry*> ksk;
  std::vector<uint32_t> devices{0};
};

namespace {

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

// device Fourier key of bsk_index on `gpu` (context.h:86-115 double-checked locking)
void* bsk_on(concrete_hip_keyset* ks, uint32_t idx, uint32_t gpu, hipStream_t s) {
  BskEntry* e = entry(ks->bsk, idx, ks->m, false);
  if (!e) die("bootstrap key index not registered");
  RT_ASSERT(gpu < MAX_DEV);
  if (e->dev[gpu]) return e->dev[gpu];
  std::lock_guard<std::mutex> g(e->m);
  if (e->dev[gpu]) return e->dev[gpu];
  const uint64_t bytes = concrete_hip_fourier_bsk_size_bytes(e->n, e->k, e->level, e->N);
  CHIP_CHECK(hipSetDevice((int)gpu));
  void* d = nullptr;
  CHIP_CHECK(hipMalloc(&d, bytes));
  int src = -1;
  for (int o = 0; o < MAX_DEV; ++o)
    if (e->dev[o]) src = o;
  if (src >= 0) {
    // one conversion per keyset; the other devices get the converted bytes (xGMI peer copy)
    CHIP_CHECK(hipMemcpyPeerAsync(d, (int)gpu, e->dev[src], src, bytes, s));
  } else if (concrete_hip_convert_bsk(s, gpu, d, e->host.data(), 0, e->n, e->k, e->level, e->N) != 0) {
    die(concrete_hip_last_error());
  }
  // publication only after the key is complete (context.h:110-113)
  CHIP_CHECK(hipStreamSynchronize(s));
  e->dev[gpu] = d;
  return d;
}

void* ksk_on(concrete_hip_keyset* ks, uint32_t idx, uint32_t gpu, hipStream_t s) {
  KskEntry* e = entry(ks->ksk, idx, ks->m, false);
  if (!e) die("keyswitch key index not registered");
  RT_ASSERT(gpu < MAX_DEV);
  if (e->dev[gpu]) return e->dev[gpu];
  std::lock_guard<std::mutex> g(e->m);
  if (e->dev[gpu]) return e->dev[gpu];
  CHIP_CHECK(hipSetDevice((int)gpu));
  void* d = nullptr;
  const uint64_t bytes = e->host.size() * 8ull;
  CHIP_CHECK(hipMalloc(&d, bytes));
  CHIP_CHECK(hipMemcpyAsync(d, e->host.data(), bytes, hipMemcpyHostToDevice, s));
  CHIP_CHECK(hipStreamSynchronize(s));
  e->dev[gpu] = d;
  return d;
}

// contiguous slice of `total` for part r of `parts` (the first total % parts get one more)
void slice(uint64_t total, uint64_t parts, uint64_t r, uint64_t& start, uint64_t& count) {
  const uint64_t base = total / parts, extra = total % parts;
  count = base + (r < extra ? 1 : 0);
  start = r * base + (r < extra ? r : extra);
}

struct Slice {
  uint32_t gpu;
  hipStream_t s;
  uint64_t start, count;
  std::vector<void*> bufs;
};

void* dmalloc(Slice& sl, uint64_t bytes) {
  void* p = nullptr;
  CHIP_CHECK(hipMallocAsync(&p, bytes ? bytes : 8, sl.s));
  sl.bufs.push_back(p);
  return p;
}

void finish(std::vector<Slice>& slices) {
  for (auto& sl : slices) {
    CHIP_CHECK(hipSetDevice((int)sl.gpu));
    for (void* p : sl.bufs) CHIP_CHECK(hipFreeAsync(p, sl.s));
  }
  for (auto& sl : slices) {
    CHIP_CHECK(hipSetDevice((int)sl.gpu));
    CHIP_CHECK(hipStreamSynchronize(sl.s));
    CHIP_CHECK(hipStreamDestroy(sl.s));
  }
  // a PBS whose wave synchronisation gave up produced wrong outputs: abort, as the reference's
  // wrappers do on any backend failure
  for (auto& sl : slices)
    if (take_device_status((int)sl.gpu) != 0) die(concrete_hip_last_error());
}

std::vector<Slice> make_slices(concrete_hip_keyset* ks, uint64_t num_samples) {
  std::vector<uint32_t> devs;
  {
    std::lock_guard<std::mutex> g(ks->m);
    devs = ks->devices;
  }
  const uint64_t parts = std::max<uint64_t>(1, std::min<uint64_t>(devs.size(), num_samples));
  std::vector<Slice> out(parts);
  for (uint64_t r = 0; r < parts; ++r) {
    out[r].gpu = devs[r];
    CHIP_CHECK(hipSetDevice((int)devs[r]));
    CHIP_CHECK(hipStreamCreateWithFlags(&out[r].s, hipStreamNonBlocking));
    slice(num_samples, parts, r, out[r].start, out[r].count);
  }
  return out;
}

// batched PBS shared by the plain and mapped wrappers: luts = num_luts trivial GLWEs on host
void run_batched_pbs(uint64_t* out, const uint64_t* ct0, uint64_t num_samples, const std::vector<uint64_t>& acc,
                     uint64_t num_luts, uint32_t n, uint32_t N, uint32_t level, uint32_t base_log, uint32_t k,
                     uint32_t bsk_index, concrete_hip_keyset* ks) {
  if (num_samples == 0) return;
  {
    // the registered key must have the call's parameters: its device format (and size) follows
    // them, so a mismatch would read past the key or reinterpret its layout
    BskEntry* e = entry(ks->bsk, bsk_index, ks->m, false);
    if (!e) die("bootstrap key index not registered");
    RT_ASSERT(e->n == n && e->k == k && e->N == N && e->level == level && e->base_log == base_log);
  }
  const uint64_t in_w = n + 1, out_w = (uint64_t)k * N + 1, glwe = (uint64_t)(k + 1) * N;
  auto slices = make_slices(ks, num_samples);
  for (auto& sl : slices) {
    CHIP_CHECK(hipSetDevice((int)sl.gpu));
    void* fbsk = bsk_on(ks, bsk_index, sl.gpu, sl.s);
    uint64_t* d_in = (uint64_t*)dmalloc(sl, sl.count * in_w * 8);
    uint64_t* d_out = (uint64_t*)dmalloc(sl, sl.count * out_w * 8);
    CHIP_CHECK(hipMemcpyAsync(d_in, ct0 + sl.start * in_w, sl.count * in_w * 8, hipMemcpyHostToDevice, sl.s));
    uint64_t* d_acc;
    uint64_t* d_lidx = nullptr;
    if (num_luts == 1) {
      d_acc = (uint64_t*)dmalloc(sl, glwe * 8);
      CHIP_CHECK(hipMemcpyAsync(d_acc, acc.data(), glwe * 8, hipMemcpyHostToDevice, sl.s));
    } else {
      // one LUT per sample: this slice's LUTs, indexed 0..count-1 (wrappers.cpp:317-325)
      d_acc = (uint64_t*)dmalloc(sl, sl.count * glwe * 8);
      CHIP_CHECK(hipMemcpyAsync(d_acc, acc.data() + sl.start * glwe, sl.count * glwe * 8, hipMemcpyHostToDevice,
                                sl.s));
      std::vector<uint64_t> idx(sl.count);
      for (uint64_t i = 0; i < sl.count; ++i) idx[i] = i;
      d_lidx = (uint64_t*)dmalloc(sl, sl.count * 8);
      CHIP_CHECK(hipMemcpyAsync(d_lidx, idx.data(), sl.count * 8, hipMemcpyHostToDevice, sl.s));
      CHIP_CHECK(hipStreamSynchronize(sl.s));  // idx is a host temporary
    }
    if (concrete_hip_pbs(sl.s, sl.gpu, d_out, nullptr, d_acc, d_lidx, d_in, nullptr, fbsk, n, k, N, base_log, level,
                         (uint32_t)sl.count, nullptr) != 0)
      die(concrete_hip_last_error());
    CHIP_CHECK(hipMemcpyAsync(out + sl.start * out_w, d_out, sl.count * out_w * 8, hipMemcpyDeviceToHost, sl.s));
  }
  finish(slices);
}

std::vector<uint64_t> trivial_glwes(const uint64_t* tlu, uint64_t num_luts, uint64_t tlu_stride0, uint32_t N,
                                    uint32_t k) {
  // (wrappers.cpp:199-209, 296-305): k zero masks, body = LUT
  const uint64_t glwe = (uint64_t)(k + 1) * N;
  std::vector<uint64_t> acc(num_luts * glwe, 0);
  for (uint64_t l = 0; l < num_luts; ++l)
    for (uint32_t i = 0; i < N; ++i) acc[l * glwe + (uint64_t)k * N + i] = tlu[l * tlu_stride0 + i];
  return acc;
}

}  // namespace

extern "C" {

concrete_hip_keyset* concrete_hip_keyset_create(void) { return new concrete_hip_keyset(); }

void concrete_hip_keyset_destroy(concrete_hip_keyset* ks) {
  if (!ks) return;
  for (BskEntry* e : ks->bsk) {
    if (!e) continue;
    for (int d = 0; d < MAX_DEV; ++d)
      if (e->dev[d]) {
        CHIP_CHECK(hipSetDevice(d));
        CHIP_CHECK(hipFree(e->dev[d]));
      }
    delete e;
  }
  for (KskEntry* e : ks->ksk) {
    if (!e) continue;
    for (int d = 0; d < MAX_DEV; ++d)
      if (e->dev[d]) {
        CHIP_CHECK(hipSetDevice(d));
        CHIP_CHECK(hipFree(e->dev[d]));
      }
    delete e;
  }
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
  for (int d = 0; d < MAX_DEV; ++d)
    if (e->dev[d]) {
      set_error("keyset_add_bsk: index %u already resident", bsk_index);
      return -3;
    }
  const uint64_t len = (uint64_t)input_lwe_dim * level * (glwe_dim + 1) * (glwe_dim + 1) * poly_size;
  e->host.assign(bsk, bsk + len);
  e->n = input_lwe_dim, e->k = glwe_dim, e->level = level, e->base_log = base_log, e->N = poly_size;
  return 0;
}

int concrete_hip_keyset_add_ksk(concrete_hip_keyset* ks, uint32_t ksk_index, const uint64_t* ksk, uint32_t level,
                                uint32_t base_log, uint32_t input_lwe_dim, uint32_t output_lwe_dim) {
  if (!ks || !ksk || level == 0 || base_log == 0 || level * base_log >= 64 || output_lwe_dim + 1 > 1024) {
    set_error("keyset_add_ksk: bad argument");
    return -3;
  }
  KskEntry* e = entry(ks->ksk, ksk_index, ks->m, true);
  std::lock_guard<std::mutex> g(e->m);
  const uint64_t len = (uint64_t)input_lwe_dim * level * (output_lwe_dim + 1);
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
    if ((int)devices[i] >= nd || devices[i] >= MAX_DEV) {
      set_error("keyset_set_devices: device %u not visible", devices[i]);
      return -3;
    }
  std::lock_guard<std::mutex> g(ks->m);
  ks->devices.assign(devices, devices + count);
  return 0;
}

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
  auto acc = trivial_glwes(tlu_aligned + tlu_offset, 1, poly_size, poly_size, glwe_dim);
  run_batched_pbs(out_aligned + out_offset, ct0_aligned + ct0_offset, out_size0, acc, 1, input_lwe_dim, poly_size,
                  level, base_log, glwe_dim, bsk_index, context);
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
  RT_ASSERT(tlu_size1 == poly_size && tlu_stride1 == 1);
  RT_ASSERT(out_stride1 == 1 && out_stride0 == out_size1 && ct0_stride1 == 1 && ct0_stride0 == ct0_size1);
  RT_ASSERT(context);
  auto acc = trivial_glwes(tlu_aligned + tlu_offset, tlu_size0, tlu_stride0, poly_size, glwe_dim);
  run_batched_pbs(out_aligned + out_offset, ct0_aligned + ct0_offset, out_size0, acc, tlu_size0, input_lwe_dim,
                  poly_size, level, base_log, glwe_dim, bsk_index, context);
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
  RT_ASSERT(out_size0 == ct0_size0);
  RT_ASSERT(out_size1 == (uint64_t)output_lwe_dim + 1 && ct0_size1 == (uint64_t)input_lwe_dim + 1);
  RT_ASSERT(out_stride1 == 1 && out_stride0 == out_size1 && ct0_stride1 == 1 && ct0_stride0 == ct0_size1);
  RT_ASSERT(context);
  const uint64_t num_samples = out_size0;
  if (num_samples == 0) return;
  KskEntry* e = entry(context->ksk, ksk_index, context->m, false);
  if (!e) die("keyswitch key index not registered");
  RT_ASSERT(e->level == level && e->base_log == base_log && e->n_in == input_lwe_dim && e->n_out == output_lwe_dim);
  const uint64_t in_w = input_lwe_dim + 1, out_w = output_lwe_dim + 1;
  const uint64_t* ct0 = ct0_aligned + ct0_offset;
  uint64_t* out = out_aligned + out_offset;
  auto slices = make_slices(context, num_samples);
  for (auto& sl : slices) {
    CHIP_CHECK(hipSetDevice((int)sl.gpu));
    void* dk = ksk_on(context, ksk_index, sl.gpu, sl.s);
    uint64_t* d_in = (uint64_t*)dmalloc(sl, sl.count * in_w * 8);
    uint64_t* d_out = (uint64_t*)dmalloc(sl, sl.count * out_w * 8);
    CHIP_CHECK(hipMemcpyAsync(d_in, ct0 + sl.start * in_w, sl.count * in_w * 8, hipMemcpyHostToDevice, sl.s));
    if (concrete_hip_keyswitch(sl.s, sl.gpu, d_out, nullptr, d_in, nullptr, (const uint64_t*)dk, input_lwe_dim,
                               output_lwe_dim, base_log, level, (uint32_t)sl.count) != 0)
      die(concrete_hip_last_error());
    CHIP_CHECK(hipMemcpyAsync(out + sl.start * out_w, d_out, sl.count * out_w * 8, hipMemcpyDeviceToHost, sl.s));
  }
  finish(slices);
}

void memref_keyswitch_lwe_hip_u64(uint64_t* out_allocated, uint64_t* out_aligned, uint64_t out_offset,
                                  uint64_t out_size, uint64_t out_stride, uint64_t* ct0_allocated,
                                  uint64_t* ct0_aligned, uint64_t ct0_offset, uint64_t ct0_size, uint64_t ct0_stride,
                                  uint32_t level, uint32_t base_log, uint32_t input_lwe_dim,
                                  uint32_t output_lwe_dim, uint32_t ksk_index, concrete_hip_keyset* context) {
  RT_ASSERT(out_stride == 1 && ct0_stride == 1);
  memref_batched_keyswitch_lwe_hip_u64(out_allocated, out_aligned, out_offset, 1, out_size, out_size, 1,
                                       ct0_allocated, ct0_aligned, ct0_offset, 1, ct0_size, ct0_size, 1, level,
                                       base_log, input_lwe_dim, output_lwe_dim, ksk_index, context);
}

}  // extern "C"
