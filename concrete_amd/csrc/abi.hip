// abi.hip — extern "C" entry points of libconcrete_hip.so (declared in include/concrete_hip.h).
//
// The cuda_* names are the backend ABI the Concrete runtime links; they
// keep the reference conventions: void return, abort on failure, stream-ordered work.
// The concrete_hip_* extensions return status codes for testability.
#include <stdarg.h>
#include <unistd.h>

#include <atomic>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "../../include/concrete_hip.h"
#include "common.hpp"
#include "pbs.hpp"
#include "companion.hpp"
#include "pbs1024_plan.hpp"

namespace chip {

// Every stream-ordered allocation of the library (cuda_malloc_async, key-conversion and keyswitch
// scratch, the general PBS path's spectra) comes from the device's default pool, whose release
// threshold is raised to "never" before the first one: freed blocks stay mapped and are reused.
// Measured on gfx950 / ROCm 7.2 (tools/microbench/pool_copy.hip): with the default threshold (0) the
// pool hands memory back to the driver at each synchronisation, and a later allocation of >= ~20 MB
// on the same stream then reads / writes stale pages — 19 of 20 rounds of "allocate, H2D copy,
// kernel, D2H, free, sync" returned wrong data, pinned or pageable, async or blocking copies; with
// the threshold raised, 0 of 20.  The cost: the pool keeps the library's peak stream-ordered usage
// (e.g. <= 1 GiB of keyswitch digits per pass, <= 2 GB of general-path spectra) reserved for the
// process; trimming it (hipMemPoolTrimTo) would bring the failure back, so it is not offered.
void keep_pool_memory() {
  static std::atomic<uint64_t> done{0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return;
  const uint64_t bit = 1ull << dev;
  if (done.load(std::memory_order_acquire) & bit) return;
  hipMemPool_t pool;
  if (hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess) {
    uint64_t thr = ~0ull;
    (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
  }
  done.fetch_or(bit, std::memory_order_acq_rel);
}

static thread_local char g_err[512] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
}
const char* last_error() { return g_err; }

static void die(const char* what) {
  fprintf(stderr, "concrete-hip: %s: %s\n", what, g_err);
  abort();
}

// Registry of device Fourier keys created through the legacy convert entry point, keyed by
// the caller's `dest` allocation (see concrete_hip.h, cuda_convert_lwe_programmable_bootstrap_key_64).
struct KeyEntry {
  void* fourier;
  uint32_t gpu, n, k, level, N;
};
static std::mutex g_keys_mu;
static std::unordered_map<const void*, KeyEntry> g_keys;

static void set_device(uint32_t gpu) { CHIP_CHECK(hipSetDevice((int)gpu)); }

// Status words (common.hpp SyncGuard), one per (device, stream): a launch flags the word of the stream
// it runs on, so a call reading its own stream's word is told about its own launches only (round 5;
// the round-4 word was per device, and a spin-bound failure in one call's kernel aborted whichever
// concurrent call read the word first).  Per device a slab of STATUS_SLOTS words (+ one reduction
// word) is allocated on first use, zeroed, never freed; slot 0 serves the null stream and every
// stream that arrives while all other slots are taken (shared, mapped explicitly so that reads find
// the word launches write).  A stream's slot returns to the device's free list when the stream is
// destroyed (release_stream_status: cuda_destroy_stream, the runtime's and the SDFG's slot release),
// so a server that creates and destroys a stream per call (wrappers.cpp:129/160, 185/255, 283/362)
// never runs out (round 6).
constexpr int STATUS_MAX_DEV = 64;
constexpr uint32_t STATUS_SLOTS = 4096;
struct DevStatus {
  uint32_t* slab = nullptr;  // STATUS_SLOTS words + the take_device_status reduction word
  uint32_t used = 0;         // high-water mark of handed-out slots (slot 0 included)
  uint32_t live = 0;         // slots other than 0 held by live streams
  std::vector<uint32_t> free_slots;
  std::unordered_map<hipStream_t, uint32_t> slot;
};
static std::mutex g_status_mu;
static DevStatus g_status[STATUS_MAX_DEV];
static std::mutex g_take_mu[STATUS_MAX_DEV];  // one take_device_status per device at a time (reduction word)
static uint32_t g_status_cap = STATUS_SLOTS;  // test hook (concrete_hip_set_status_slot_cap), g_status_mu
static std::atomic<uint32_t> g_spin_limit{DEFAULT_SPIN_LIMIT};
static thread_local uint32_t t_spin_limit = 0;  // per-thread override (test hook), 0 = the global bound

static void check_gpu_index(int gpu) {
  if (gpu < 0 || gpu >= STATUS_MAX_DEV) {
    fprintf(stderr, "concrete-hip: device index %d out of range\n", gpu);
    abort();
  }
}

// the status word of (gpu, s), allocating the device's slab on first use (g_status_mu held);
// nullptr when !create and s has no word yet (no PBS kernel has run on it)
static uint32_t* status_word_locked(int gpu, hipStream_t s, bool create) {
  DevStatus& d = g_status[gpu];
  if (!d.slab) {
    if (!create) return nullptr;
    int prev = 0;
    CHIP_CHECK(hipGetDevice(&prev));
    CHIP_CHECK(hipSetDevice(gpu));
    void* p = nullptr;
    CHIP_CHECK(hipMalloc(&p, (STATUS_SLOTS + 1) * sizeof(uint32_t)));
    CHIP_CHECK(hipMemset(p, 0, (STATUS_SLOTS + 1) * sizeof(uint32_t)));
    CHIP_CHECK(hipSetDevice(prev));
    d.slab = (uint32_t*)p;
    d.used = 1;  // slot 0: null stream / overflow
  }
  if (!s) return d.slab;
  auto it = d.slot.find(s);
  if (it != d.slot.end()) return d.slab + it->second;
  if (!create) return nullptr;
  uint32_t k = 0;  // overflow: the shared word, recorded so that the stream's reads find it
  if (d.live + 1 < g_status_cap) {
    if (!d.free_slots.empty()) {
      k = d.free_slots.back();
      d.free_slots.pop_back();
    } else {
      k = d.used++;  // used = live + 1 + free slots <= cap <= STATUS_SLOTS
    }
    ++d.live;
  }
  d.slot.emplace(s, k);
  return d.slab + k;
}

SyncGuard sync_guard(int gpu, hipStream_t s) {
  check_gpu_index(gpu);
  uint32_t* w;
  {
    std::lock_guard<std::mutex> g(g_status_mu);
    w = status_word_locked(gpu, s, true);
  }
  const uint32_t lim = t_spin_limit ? t_spin_limit : g_spin_limit.load(std::memory_order_relaxed);
  return SyncGuard{w, lim};
}

void report_hip_state(FILE* f) {
  int n = -1;
  const hipError_t e = hipGetDeviceCount(&n);
  int dev = -1;
  (void)hipGetDevice(&dev);
  fprintf(f, "concrete-hip: process %d: hipGetDeviceCount -> %s, %d device(s); current device %d", (int)getpid(),
          hipGetErrorString(e), n, dev);
  for (const char* v : {"HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "GPU_DEVICE_ORDINAL"})
    if (const char* x = getenv(v)) fprintf(f, "; %s=%s", v, x);
  fprintf(f, "\n");
  fflush(f);
}

[[noreturn]] void hip_fatal(const char* expr, const char* file, int line, hipError_t e) {
  fprintf(stderr, "concrete-hip: %s failed at %s:%d: %s\n", expr, file, line, hipGetErrorString(e));
  report_hip_state(stderr);
  abort();
}

static int status_error(int gpu, uint32_t v, const char* scope) {
  if (v & DEV_STATUS_SYNC_TIMEOUT) {
    set_error("device %d: a PBS wave synchronisation exceeded its spin bound on %s; that launch's outputs are wrong",
              gpu, scope);
    return -4;
  }
  set_error("device %d: status word 0x%x on %s", gpu, v, scope);
  return -4;
}

// Every word is taken with an atomic exchange and OR-ed into the reduction word (slab[STATUS_SLOTS]):
// a flag that a kernel still running on another stream sets while the slab is being read is either
// taken here or left for its own stream's read, never wiped unseen (the round-5 form copied
// the slab and then zeroed all of it).
__global__ void status_take_kernel(uint32_t* slab, uint32_t used) {
  uint32_t acc = 0;
  for (uint32_t i = threadIdx.x; i < used; i += blockDim.x) acc |= atomicExch(slab + i, 0u);
  if (acc) atomicOr(slab + STATUS_SLOTS, acc);
}

// Device-wide form: synchronises the device and takes (reads and clears) the words of every stream.
int take_device_status(int gpu) {
  if (gpu < 0 || gpu >= STATUS_MAX_DEV) return 0;
  std::lock_guard<std::mutex> tg(g_take_mu[gpu]);
  uint32_t* slab = nullptr;
  uint32_t used = 0;
  {
    std::lock_guard<std::mutex> g(g_status_mu);
    slab = g_status[gpu].slab, used = g_status[gpu].used;
  }
  if (!slab) return 0;  // no PBS kernel has run on this device
  int prev = 0;
  CHIP_CHECK(hipGetDevice(&prev));  // the caller's current device is restored (torch shares it)
  CHIP_CHECK(hipSetDevice(gpu));
  CHIP_CHECK(hipDeviceSynchronize());
  status_take_kernel<<<1, 256, 0, nullptr>>>(slab, used);
  CHIP_CHECK(hipGetLastError());
  uint32_t any = 0;
  CHIP_CHECK(hipMemcpy(&any, slab + STATUS_SLOTS, sizeof(uint32_t), hipMemcpyDeviceToHost));
  if (any) CHIP_CHECK(hipMemset(slab + STATUS_SLOTS, 0, sizeof(uint32_t)));
  CHIP_CHECK(hipSetDevice(prev));
  return any ? status_error(gpu, any, "some stream") : 0;
}

// Stream-ordered form: the word of stream s is read on s after the work issued there (the runtime's
// slice and shard streams), so concurrent calls on other streams are neither waited for nor blamed.
// (An overflowed stream shares slot 0 and may be told of another overflowed stream's failure.)
int take_stream_status(int gpu, hipStream_t s, uint32_t* h) {
  uint32_t* w;
  {
    std::lock_guard<std::mutex> g(g_status_mu);
    w = (gpu >= 0 && gpu < STATUS_MAX_DEV) ? status_word_locked(gpu, s, false) : nullptr;
  }
  if (!w) {  // no PBS kernel has run on this stream: only the stream's own work to wait for
    CHIP_CHECK(hipStreamSynchronize(s));
    return 0;
  }
  CHIP_CHECK(hipMemcpyAsync(h, w, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  CHIP_CHECK(hipStreamSynchronize(s));
  const uint32_t v = *h;
  if (v == 0) return 0;
  CHIP_CHECK(hipMemsetAsync(w, 0, sizeof(uint32_t), s));
  CHIP_CHECK(hipStreamSynchronize(s));
  return status_error(gpu, v, "this call's stream");
}

// A stream about to be destroyed (its work synchronised by the caller): its word is cleared and its
// slot goes back to the device's free list.  Slot 0 (shared) is never cleared here.
void release_stream_status(int gpu, hipStream_t s) {
  if (gpu < 0 || gpu >= STATUS_MAX_DEV || !s) return;
  uint32_t* w = nullptr;
  {
    std::lock_guard<std::mutex> g(g_status_mu);
    DevStatus& d = g_status[gpu];
    auto it = d.slot.find(s);
    if (it == d.slot.end()) return;
    const uint32_t k = it->second;
    d.slot.erase(it);
    if (k == 0) return;
    --d.live;
    w = d.slab + k;
    // cleared before the slot can be handed out again (the lock is held across the clear)
    int prev = 0;
    CHIP_CHECK(hipGetDevice(&prev));
    CHIP_CHECK(hipSetDevice(gpu));
    CHIP_CHECK(hipMemset(w, 0, sizeof(uint32_t)));
    CHIP_CHECK(hipSetDevice(prev));
    d.free_slots.push_back(k);
  }
}

uint32_t status_slots_in_use(int gpu) {
  if (gpu < 0 || gpu >= STATUS_MAX_DEV) return 0;
  std::lock_guard<std::mutex> g(g_status_mu);
  return g_status[gpu].live;
}

// ---- general-format companion keys (pbs_needs_generic_key) ------------------------------
// A primary device key in a hand-tuned kernel's format (N = 1024 / 2048) whose standard-domain
// source the backend can reach — the keyset's host copy, or the `dest` buffer of
// cuda_convert_lwe_programmable_bootstrap_key_64, which holds the standard key on the device — is
// registered with that source; the first PBS with digits wider than the hand-tuned kernel accepts
// converts it once into the general path's format (its companion), kept until the primary goes.
struct StdSource {
  const uint64_t* src;
  bool on_device;
  uint32_t gpu, n, k, level, N;
  void* companion;  // general-format key, built on first use
};
static std::mutex g_src_mu;
static std::unordered_map<const void*, StdSource> g_src;

void register_std_source(const void* primary, const uint64_t* src, bool on_device, uint32_t gpu, uint32_t n,
                         uint32_t k, uint32_t level, uint32_t N) {
  void* old = nullptr;
  {
    std::lock_guard<std::mutex> g(g_src_mu);
    auto it = g_src.find(primary);
    if (it != g_src.end()) old = it->second.companion;
    g_src[primary] = StdSource{src, on_device, gpu, n, k, level, N, nullptr};
  }
  if (old) CHIP_CHECK(hipFree(old));
}

void release_std_source(const void* primary) {
  void* c = nullptr;
  int gpu = 0;
  {
    std::lock_guard<std::mutex> g(g_src_mu);
    auto it = g_src.find(primary);
    if (it == g_src.end()) return;
    c = it->second.companion;
    gpu = (int)it->second.gpu;
    g_src.erase(it);
  }
  if (c) {
    key_spectrum_forget(c);
    int prev = 0;
    CHIP_CHECK(hipGetDevice(&prev));
    CHIP_CHECK(hipSetDevice(gpu));
    CHIP_CHECK(hipFree(c));
    CHIP_CHECK(hipSetDevice(prev));
  }
}

// The companion of `primary` for (n, k, l, N), converted on `s` (and synchronised: published
// complete, context.h:110-113) on first use; nullptr when the primary has no registered source or
// other parameters.
const void* generic_companion_key(const void* primary, uint32_t n, uint32_t k, uint32_t level, uint32_t N,
                                  hipStream_t s) {
  std::lock_guard<std::mutex> g(g_src_mu);  // held across the one-time conversion
  auto it = g_src.find(primary);
  if (it == g_src.end()) return nullptr;
  StdSource& e = it->second;
  if (e.n != n || e.k != k || e.level != level || e.N != N) return nullptr;
  if (e.companion) return e.companion;
  const uint64_t bytes = generic_fourier_bsk_bytes(n, k, level, N);
  if (!bytes) return nullptr;
  void* d = nullptr;
  CHIP_CHECK(hipMalloc(&d, bytes));
  const uint64_t std_bytes = (uint64_t)n * level * (k + 1) * (k + 1) * N * 8ull;
  const uint64_t* src_dev = e.src;
  void* tmp = nullptr;
  if (!e.on_device) {
    CHIP_CHECK(hipMalloc(&tmp, std_bytes));
    CHIP_CHECK(hipMemcpyAsync(tmp, e.src, std_bytes, hipMemcpyHostToDevice, s));
    src_dev = (const uint64_t*)tmp;
  }
  ConvertArgs a{s, d, src_dev, n, k, level, N, generic_key_format(k, N, level).limbs, key_spectrum_sink(s)};
  int rc = convert_bsk_generic_launch(a);
  const int rs = key_spectrum_record(s, rc == 0 ? d : nullptr, generic_key_format(k, N, level), n, k, N, level, a.smax);
  if (rc == 0) rc = rs;
  CHIP_CHECK(hipStreamSynchronize(s));
  if (tmp) CHIP_CHECK(hipFree(tmp));
  if (rc != 0) {
    key_spectrum_forget(d);
    CHIP_CHECK(hipFree(d));
    return nullptr;
  }
  e.companion = d;
  return d;
}

}  // namespace chip

using namespace chip;

extern "C" {

// ----------------------------------------------------------------------------------------
// device / stream / memory management
// ----------------------------------------------------------------------------------------
void* cuda_create_stream(uint32_t gpu_index) {
  set_device(gpu_index);
  hipStream_t s;
  CHIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  return (void*)s;
}

void cuda_destroy_stream(void* stream, uint32_t gpu_index) {
  set_device(gpu_index);
  CHIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
  release_stream_status((int)gpu_index, (hipStream_t)stream);
  CHIP_CHECK(hipStreamDestroy((hipStream_t)stream));
}

void* cuda_malloc_async(uint64_t size, void* stream, uint32_t gpu_index) {
  set_device(gpu_index);
  void* p = nullptr;
  if (size == 0) return nullptr;
  keep_pool_memory();
  CHIP_CHECK(hipMallocAsync(&p, size, (hipStream_t)stream));
  track_device_buffer(p);
  return p;
}

void cuda_memcpy_async_to_gpu(void* dest, void* src, uint64_t size, void* stream, uint32_t gpu_index) {
  if (size == 0) return;
  set_device(gpu_index);
  release_key_bytes(dest, nullptr, false);  // new contents: derived key bytes are stale
  CHIP_CHECK(hipMemcpyAsync(dest, src, size, hipMemcpyHostToDevice, (hipStream_t)stream));
}

void cuda_memcpy_async_to_cpu(void* dest, const void* src, uint64_t size, void* stream, uint32_t gpu_index) {
  if (size == 0) return;
  set_device(gpu_index);
  CHIP_CHECK(hipMemcpyAsync(dest, src, size, hipMemcpyDeviceToHost, (hipStream_t)stream));
}

static void release_registered(void* ptr) {
  void* f = nullptr;
  {
    std::lock_guard<std::mutex> g(g_keys_mu);
    auto it = g_keys.find(ptr);
    if (it != g_keys.end()) {
      f = it->second.fourier;
      g_keys.erase(it);
    }
  }
  if (f) {
    release_std_source(f);
    key_spectrum_forget(f);
    CHIP_CHECK(hipFree(f));
  }
}

void cuda_drop(void* ptr, uint32_t gpu_index) {
  if (!ptr) return;
  set_device(gpu_index);
  release_registered(ptr);
  release_key_bytes(ptr, nullptr, true);
  key_spectrum_forget(ptr);
  CHIP_CHECK(hipFree(ptr));
}

void cuda_drop_async(void* ptr, void* stream, uint32_t gpu_index) {
  if (!ptr) return;
  set_device(gpu_index);
  release_registered(ptr);
  release_key_bytes(ptr, (hipStream_t)stream, true);
  key_spectrum_forget(ptr);
  CHIP_CHECK(hipFreeAsync(ptr, (hipStream_t)stream));
}

int concrete_hip_release_device_buffer(const void* ptr) {
  if (!ptr) return 0;
  release_registered((void*)ptr);
  key_spectrum_forget(ptr);
  return release_key_bytes(ptr, nullptr, false);
}

void cuda_synchronize_device(uint32_t gpu_index) {
  set_device(gpu_index);
  CHIP_CHECK(hipDeviceSynchronize());
  // the PBS kernels report synchronisation failures through the device status word: abort here,
  // the reference's failure behaviour for the cuda_* entry points
  if (take_device_status((int)gpu_index) != 0) die("cuda_synchronize_device");
}

// ----------------------------------------------------------------------------------------
// extensions
// ----------------------------------------------------------------------------------------
uint32_t concrete_hip_abi_version(void) { return 5u; }
const char* concrete_hip_last_error(void) { return last_error(); }
int concrete_hip_device_status(uint32_t gpu_index) { return take_device_status((int)gpu_index); }
int concrete_hip_stream_status(void* stream, uint32_t gpu_index) {
  if (gpu_index >= (uint32_t)STATUS_MAX_DEV) {
    set_error("stream_status: device index %u out of range", gpu_index);
    return -3;
  }
  set_device(gpu_index);
  static thread_local uint32_t* landing = nullptr;  // page-locked landing word of this thread
  if (!landing) CHIP_CHECK(hipHostMalloc((void**)&landing, sizeof(uint32_t), hipHostMallocDefault));
  return take_stream_status((int)gpu_index, (hipStream_t)stream, landing);
}
void concrete_hip_set_thread_spin_limit(uint32_t polls) { t_spin_limit = polls; }

uint64_t concrete_hip_pbs1024_plan(uint64_t num_samples, uint32_t cus, uint32_t* parts) {
  const Pbs1024Plan p = plan_pbs1024(num_samples, cus);
  if (parts) parts[0] = p.pair, parts[1] = p.hex2, parts[2] = p.hex1;
  return p.cost;
}

uint32_t concrete_hip_status_slots_in_use(uint32_t gpu_index) { return status_slots_in_use((int)gpu_index); }

void concrete_hip_set_status_slot_cap(uint32_t slots) {
  std::lock_guard<std::mutex> g(g_status_mu);
  g_status_cap = (slots == 0 || slots > STATUS_SLOTS) ? STATUS_SLOTS : slots;
}

void concrete_hip_set_spin_limit(uint32_t polls) {
  g_spin_limit.store(polls ? polls : DEFAULT_SPIN_LIMIT, std::memory_order_relaxed);
}

int concrete_hip_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int concrete_hip_pbs_supported(uint32_t glwe_dim, uint32_t polynomial_size, uint32_t level_count,
                               uint32_t base_log) {
  return pbs_params_ok(glwe_dim, polynomial_size, level_count, base_log) ||
                 pbs_needs_generic_key(glwe_dim, polynomial_size, level_count, base_log)
             ? 1
             : 0;
}

int concrete_hip_keyswitch_supported(uint32_t level_count, uint32_t base_log, uint32_t input_lwe_dim,
                                     uint32_t output_lwe_dim) {
  return keyswitch_params_ok(level_count, base_log, input_lwe_dim, output_lwe_dim) ? 1 : 0;
}

uint32_t concrete_hip_bsk_limbs(uint32_t polynomial_size, uint32_t level_count, uint32_t base_log) {
  (void)base_log;
  return default_limbs(1, polynomial_size, level_count);
}

int concrete_hip_bsk_format(uint32_t glwe_dim, uint32_t polynomial_size, uint32_t level_count, uint32_t* limbs,
                            uint32_t* limb_bits) {
  const KeyFormat f = key_format(glwe_dim, polynomial_size, level_count);
  if (limbs) *limbs = f.limbs;
  if (limb_bits) *limb_bits = f.bits;
  return (int)f.kind;
}

double concrete_hip_generic_error_bound(uint32_t glwe_dim, uint32_t polynomial_size, uint32_t level_count,
                                        uint32_t base_log, double max_key_spectrum) {
  const KeyFormat f = key_format(glwe_dim, polynomial_size, level_count);
  if (f.kind != KeyKind::GENERIC) return -1.0;
  return generic_error_bound(glwe_dim, polynomial_size, level_count, base_log, f.bits, max_key_spectrum);
}

uint64_t concrete_hip_fourier_bsk_size_bytes(uint32_t input_lwe_dim, uint32_t glwe_dim, uint32_t level_count,
                                             uint32_t polynomial_size) {
  return fourier_bsk_bytes(input_lwe_dim, glwe_dim, level_count, polynomial_size);
}

int concrete_hip_convert_bsk(void* stream, uint32_t gpu_index, void* dest_fourier, const void* src,
                             int src_is_device, uint32_t input_lwe_dim, uint32_t glwe_dim, uint32_t level_count,
                             uint32_t polynomial_size) {
  if (!dest_fourier || !src) {
    set_error("convert_bsk: null pointer");
    return -1;
  }
  if (key_format(glwe_dim, polynomial_size, level_count).kind == KeyKind::NONE) {
    set_error("convert_bsk: unsupported parameters k=%u N=%u level=%u", glwe_dim, polynomial_size, level_count);
    return -2;
  }
  set_device(gpu_index);
  hipStream_t s = (hipStream_t)stream;
  const uint64_t std_bytes =
      (uint64_t)input_lwe_dim * level_count * (glwe_dim + 1) * (glwe_dim + 1) * polynomial_size * 8ull;
  const uint64_t* src_dev = (const uint64_t*)src;
  void* tmp = nullptr;
  keep_pool_memory();
  if (!src_is_device) {
    CHIP_CHECK(hipMallocAsync(&tmp, std_bytes, s));
    CHIP_CHECK(hipMemcpyAsync(tmp, src, std_bytes, hipMemcpyHostToDevice, s));
    src_dev = (const uint64_t*)tmp;
  }
  ConvertArgs a{s, dest_fourier, src_dev, input_lwe_dim, glwe_dim, level_count, polynomial_size,
                default_limbs(glwe_dim, polynomial_size, level_count), key_spectrum_sink(s)};
  int rc = convert_bsk_launch(a);
  // the key's measured spectrum against the certified bound (keycheck.hip; synchronises s, as the
  // reference does after its conversion, context.h:110-113)
  const int rs = key_spectrum_record(s, rc == 0 ? dest_fourier : nullptr,
                                     key_format(glwe_dim, polynomial_size, level_count), input_lwe_dim, glwe_dim,
                                     polynomial_size, level_count, a.smax);
  if (rc == 0) rc = rs;
  else key_spectrum_forget(dest_fourier);
  if (tmp) CHIP_CHECK(hipFreeAsync(tmp, s));
  return rc;
}

int concrete_hip_pbs(void* stream, uint32_t gpu_index, uint64_t* lwe_array_out, const uint64_t* lwe_output_indexes,
                     const uint64_t* lut_vector, const uint64_t* lut_vector_indexes, const uint64_t* lwe_array_in,
                     const uint64_t* lwe_input_indexes, const void* fourier_bsk, uint32_t lwe_dimension,
                     uint32_t glwe_dimension, uint32_t polynomial_size, uint32_t base_log, uint32_t level_count,
                     uint32_t num_samples, uint64_t* resid_bits) {
  if (num_samples == 0) return 0;
  if (!lwe_array_out || !lut_vector || !lwe_array_in || !fourier_bsk) {
    set_error("pbs: null pointer");
    return -1;
  }
  if (lwe_dimension == 0) {
    set_error("pbs: lwe_dimension must be > 0");
    return -3;
  }
  bool generic = !pbs_params_ok(glwe_dimension, polynomial_size, level_count, base_log);
  if (generic && !pbs_needs_generic_key(glwe_dimension, polynomial_size, level_count, base_log)) {
    set_error("pbs: unsupported parameters k=%u N=%u level=%u base_log=%u", glwe_dimension, polynomial_size,
              level_count, base_log);
    return -2;
  }
  set_device(gpu_index);
  const void* key = fourier_bsk;
  uint32_t limbs = default_limbs(glwe_dimension, polynomial_size, level_count);
  const KeyKind kind = key_format(glwe_dimension, polynomial_size, level_count).kind;
  if (!generic && key_bound_check(fourier_bsk, kind, glwe_dimension, polynomial_size, level_count, base_log) != 0) {
    // this key's spectrum is too large for the hand-tuned kernel at this base_log: the general path's
    // narrower limbs may still be exact (its companion's own bound is checked below)
    if (kind == KeyKind::GENERIC ||
        !generic_pbs_ok(glwe_dimension, polynomial_size, level_count, base_log) ||
        !generic_companion_key(fourier_bsk, lwe_dimension, glwe_dimension, level_count, polynomial_size,
                               (hipStream_t)stream))
      return -2;  // message set by key_bound_check
    generic = true;
  }
  if (generic) {
    // digits wider than the hand-tuned kernel takes: the general path, on this key's companion
    key = generic_companion_key(fourier_bsk, lwe_dimension, glwe_dimension, level_count, polynomial_size,
                                (hipStream_t)stream);
    if (!key) {
      set_error("pbs: k=%u N=%u level=%u base_log=%u runs on the general path, whose key format this key is not "
                "in and cannot be derived from (convert it through a keyset or "
                "cuda_convert_lwe_programmable_bootstrap_key_64, or use concrete_hip_convert_bsk_generic + "
                "concrete_hip_pbs_generic)",
                glwe_dimension, polynomial_size, level_count, base_log);
      return -2;
    }
    limbs = generic_key_format(glwe_dimension, polynomial_size, level_count).limbs;
    if (key_bound_check(key, KeyKind::GENERIC, glwe_dimension, polynomial_size, level_count, base_log) != 0)
      return -2;
  }
  PbsArgs a{(hipStream_t)stream,
            lwe_array_out,
            lwe_output_indexes,
            lut_vector,
            lut_vector_indexes,
            lwe_array_in,
            lwe_input_indexes,
            key,
            lwe_dimension,
            glwe_dimension,
            polynomial_size,
            base_log,
            level_count,
            limbs,
            num_samples,
            (unsigned long long*)resid_bits,
            sync_guard((int)gpu_index, (hipStream_t)stream)};
  return generic ? pbs_generic_launch(a) : pbs_launch(a);
}

uint64_t concrete_hip_generic_bsk_size_bytes(uint32_t input_lwe_dim, uint32_t glwe_dim, uint32_t level_count,
                                             uint32_t polynomial_size) {
  return generic_fourier_bsk_bytes(input_lwe_dim, glwe_dim, level_count, polynomial_size);
}

int concrete_hip_convert_bsk_generic(void* stream, uint32_t gpu_index, void* dest, const void* src, int src_is_device,
                                     uint32_t input_lwe_dim, uint32_t glwe_dim, uint32_t level_count,
                                     uint32_t polynomial_size) {
  if (!dest || !src) {
    set_error("convert_bsk_generic: null pointer");
    return -1;
  }
  const KeyFormat f = generic_key_format(glwe_dim, polynomial_size, level_count);
  if (f.kind != KeyKind::GENERIC) {
    set_error("convert_bsk_generic: k=%u N=%u level=%u is not on the general path", glwe_dim, polynomial_size,
              level_count);
    return -2;
  }
  set_device(gpu_index);
  hipStream_t s = (hipStream_t)stream;
  const uint64_t std_bytes =
      (uint64_t)input_lwe_dim * level_count * (glwe_dim + 1) * (glwe_dim + 1) * polynomial_size * 8ull;
  const uint64_t* src_dev = (const uint64_t*)src;
  void* tmp = nullptr;
  keep_pool_memory();
  if (!src_is_device) {
    CHIP_CHECK(hipMallocAsync(&tmp, std_bytes, s));
    CHIP_CHECK(hipMemcpyAsync(tmp, src, std_bytes, hipMemcpyHostToDevice, s));
    src_dev = (const uint64_t*)tmp;
  }
  ConvertArgs a{s, dest, src_dev, input_lwe_dim, glwe_dim, level_count, polynomial_size, f.limbs,
                key_spectrum_sink(s)};
  int rc = convert_bsk_generic_launch(a);
  const int rs = key_spectrum_record(s, rc == 0 ? dest : nullptr, f, input_lwe_dim, glwe_dim, polynomial_size,
                                     level_count, a.smax);
  if (rc == 0) rc = rs;
  else key_spectrum_forget(dest);
  if (tmp) CHIP_CHECK(hipFreeAsync(tmp, s));
  return rc;
}

int concrete_hip_pbs_generic(void* stream, uint32_t gpu_index, uint64_t* lwe_array_out,
                             const uint64_t* lwe_output_indexes, const uint64_t* lut_vector,
                             const uint64_t* lut_vector_indexes, const uint64_t* lwe_array_in,
                             const uint64_t* lwe_input_indexes, const void* generic_bsk, uint32_t lwe_dimension,
                             uint32_t glwe_dimension, uint32_t polynomial_size, uint32_t base_log,
                             uint32_t level_count, uint32_t num_samples, uint64_t* resid_bits) {
  if (num_samples == 0) return 0;
  if (!lwe_array_out || !lut_vector || !lwe_array_in || !generic_bsk || lwe_dimension == 0) {
    set_error("pbs_generic: null pointer or zero dimension");
    return -1;
  }
  if (!generic_pbs_ok(glwe_dimension, polynomial_size, level_count, base_log)) {
    set_error("pbs_generic: k=%u N=%u level=%u base_log=%u outside the general path's exact range", glwe_dimension,
              polynomial_size, level_count, base_log);
    return -2;
  }
  if (key_bound_check(generic_bsk, KeyKind::GENERIC, glwe_dimension, polynomial_size, level_count, base_log) != 0)
    return -2;
  set_device(gpu_index);
  PbsArgs a{(hipStream_t)stream, lwe_array_out, lwe_output_indexes, lut_vector, lut_vector_indexes, lwe_array_in,
            lwe_input_indexes, generic_bsk, lwe_dimension, glwe_dimension, polynomial_size, base_log, level_count,
            generic_key_format(glwe_dimension, polynomial_size, level_count).limbs, num_samples,
            (unsigned long long*)resid_bits, sync_guard((int)gpu_index, (hipStream_t)stream)};
  return pbs_generic_launch(a);
}

int concrete_hip_keyswitch(void* stream, uint32_t gpu_index, uint64_t* lwe_array_out,
                           const uint64_t* lwe_output_indexes, const uint64_t* lwe_array_in,
                           const uint64_t* lwe_input_indexes, const uint64_t* ksk, uint32_t lwe_dimension_in,
                           uint32_t lwe_dimension_out, uint32_t base_log, uint32_t level_count,
                           uint32_t num_samples) {
  if (num_samples == 0) return 0;
  if (!lwe_array_out || !lwe_array_in || !ksk) {
    set_error("keyswitch: null pointer");
    return -1;
  }
  set_device(gpu_index);
  KsArgs a{(hipStream_t)stream, lwe_array_out, lwe_output_indexes, lwe_array_in, lwe_input_indexes, ksk,
           lwe_dimension_in,    lwe_dimension_out, base_log,       level_count,  num_samples};
  return keyswitch_launch(a);
}

const void* concrete_hip_lookup_bsk(const void* bootstrapping_key) {
  std::lock_guard<std::mutex> g(g_keys_mu);
  auto it = g_keys.find(bootstrapping_key);
  return it == g_keys.end() ? nullptr : it->second.fourier;
}

// ----------------------------------------------------------------------------------------
// runtime-facing PBS / KS entry points
// ----------------------------------------------------------------------------------------
void cuda_convert_lwe_programmable_bootstrap_key_64(void* stream, uint32_t gpu_index, void* dest, void* src,
                                                    uint32_t input_lwe_dim, uint32_t glwe_dim,
                                                    uint32_t level_count, uint32_t polynomial_size) {
  set_device(gpu_index);
  const uint64_t bytes = concrete_hip_fourier_bsk_size_bytes(input_lwe_dim, glwe_dim, level_count, polynomial_size);
  void* f = nullptr;
  CHIP_CHECK(hipMalloc(&f, bytes));
  // dest (caller-sized at n*l*(k+1)^2*N*8 bytes) receives the standard key verbatim and is the
  // conversion source; the Fourier form (larger: exact limbs) lives in the registry.
  const uint64_t std_bytes =
      (uint64_t)input_lwe_dim * level_count * (glwe_dim + 1) * (glwe_dim + 1) * polynomial_size * 8ull;
  CHIP_CHECK(hipMemcpyAsync(dest, src, std_bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
  if (concrete_hip_convert_bsk(stream, gpu_index, f, dest, 1, input_lwe_dim, glwe_dim, level_count,
                               polynomial_size) != 0)
    die("cuda_convert_lwe_programmable_bootstrap_key_64");
  void* old = nullptr;
  {
    std::lock_guard<std::mutex> g(g_keys_mu);
    auto it = g_keys.find(dest);
    if (it != g_keys.end()) old = it->second.fourier;
    g_keys[dest] = KeyEntry{f, gpu_index, input_lwe_dim, glwe_dim, level_count, polynomial_size};
  }
  if (old) {
    CHIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
    release_std_source(old);
    CHIP_CHECK(hipFree(old));
  }
  // dest keeps the standard key: the source of a general-format companion for wide-digit calls
  if (key_format(glwe_dim, polynomial_size, level_count).kind != KeyKind::GENERIC)
    register_std_source(f, (const uint64_t*)dest, true, gpu_index, input_lwe_dim, glwe_dim, level_count,
                        polynomial_size);
}

void scratch_cuda_programmable_bootstrap_64(void* stream, uint32_t gpu_index, int8_t** pbs_buffer,
                                            uint32_t glwe_dimension, uint32_t polynomial_size,
                                            uint32_t level_count, uint32_t input_lwe_ciphertext_count,
                                            bool allocate_gpu_memory) {
  (void)input_lwe_ciphertext_count;
  if (key_format(glwe_dimension, polynomial_size, level_count).kind == KeyKind::NONE) {
    set_error("scratch: unsupported parameters k=%u N=%u level=%u", glwe_dimension, polynomial_size, level_count);
    die("scratch_cuda_programmable_bootstrap_64");
  }
  // The kernel keeps all per-ciphertext state in LDS/VGPRs: the buffer is a 256-byte token
  // (diagnostics word at offset 0) so that the caller's ownership protocol is unchanged.
  if (!allocate_gpu_memory) {
    *pbs_buffer = nullptr;
    return;
  }
  set_device(gpu_index);
  keep_pool_memory();
  void* p = nullptr;
  CHIP_CHECK(hipMallocAsync(&p, 256, (hipStream_t)stream));
  CHIP_CHECK(hipMemsetAsync(p, 0, 256, (hipStream_t)stream));
  *pbs_buffer = (int8_t*)p;
}

void cleanup_cuda_programmable_bootstrap(void* stream, uint32_t gpu_index, int8_t** pbs_buffer) {
  if (!pbs_buffer || !*pbs_buffer) return;
  set_device(gpu_index);
  CHIP_CHECK(hipFreeAsync(*pbs_buffer, (hipStream_t)stream));
  *pbs_buffer = nullptr;
}

void cuda_programmable_bootstrap_lwe_ciphertext_vector_64(
    void* stream, uint32_t gpu_index, void* lwe_array_out, void* lwe_output_indexes, void* lut_vector,
    void* lut_vector_indexes, void* lwe_array_in, void* lwe_input_indexes, void* bootstrapping_key,
    int8_t* pbs_buffer, uint32_t lwe_dimension, uint32_t glwe_dimension, uint32_t polynomial_size,
    uint32_t base_log, uint32_t level_count, uint32_t num_samples, uint32_t num_many_lut, uint32_t lut_stride) {
  (void)pbs_buffer;
  if (num_many_lut != 1 || lut_stride != 1) {
    set_error("num_many_lut=%u lut_stride=%u (only 1, 1 is used by the runtime)", num_many_lut, lut_stride);
    die("cuda_programmable_bootstrap_lwe_ciphertext_vector_64");
  }
  KeyEntry e{};
  {
    std::lock_guard<std::mutex> g(g_keys_mu);
    auto it = g_keys.find(bootstrapping_key);
    if (it != g_keys.end()) e = it->second;
  }
  if (!e.fourier) {
    set_error("bootstrapping key %p was not converted by cuda_convert_lwe_programmable_bootstrap_key_64",
              bootstrapping_key);
    die("cuda_programmable_bootstrap_lwe_ciphertext_vector_64");
  }
  // the device format follows the conversion's (n, k, l, N): a call with other parameters would
  // read past the key or reinterpret its layout
  if (e.n != lwe_dimension || e.k != glwe_dimension || e.level != level_count || e.N != polynomial_size ||
      e.gpu != gpu_index) {
    set_error("bootstrapping key converted for n=%u k=%u level=%u N=%u on gpu %u, called with n=%u k=%u level=%u "
              "N=%u on gpu %u",
              e.n, e.k, e.level, e.N, e.gpu, lwe_dimension, glwe_dimension, level_count, polynomial_size, gpu_index);
    die("cuda_programmable_bootstrap_lwe_ciphertext_vector_64");
  }
  const void* f = e.fourier;
  if (concrete_hip_pbs(stream, gpu_index, (uint64_t*)lwe_array_out, (const uint64_t*)lwe_output_indexes,
                       (const uint64_t*)lut_vector, (const uint64_t*)lut_vector_indexes,
                       (const uint64_t*)lwe_array_in, (const uint64_t*)lwe_input_indexes, f, lwe_dimension,
                       glwe_dimension, polynomial_size, base_log, level_count, num_samples, nullptr) != 0)
    die("cuda_programmable_bootstrap_lwe_ciphertext_vector_64");
}

void cuda_keyswitch_lwe_ciphertext_vector_64(void* stream, uint32_t gpu_index, void* lwe_array_out,
                                             void* lwe_output_indexes, void* lwe_array_in,
                                             void* lwe_input_indexes, void* ksk, uint32_t lwe_dimension_in,
                                             uint32_t lwe_dimension_out, uint32_t base_log,
                                             uint32_t level_count, uint32_t num_samples) {
  if (concrete_hip_keyswitch(stream, gpu_index, (uint64_t*)lwe_array_out, (const uint64_t*)lwe_output_indexes,
                             (const uint64_t*)lwe_array_in, (const uint64_t*)lwe_input_indexes,
                             (const uint64_t*)ksk, lwe_dimension_in, lwe_dimension_out, base_log, level_count,
                             num_samples) != 0)
    die("cuda_keyswitch_lwe_ciphertext_vector_64");
}

}  // extern "C"
