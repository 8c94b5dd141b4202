// sdfg.hip — the SDFG stream emulator (SURVEY.md §8b layer B2, the default GPU route), host code.
//
// A circuit compiled with the GPU backend and SDFG extraction does not call the memref wrappers: it
// builds a dataflow graph at run time through the stream_emulator_* C API
// (compiler include/concretelang/Runtime/stream_emulator_api.h:30-106, emitted by
// lib/Conversion/SDFGToStreamEmulator/SDFGToStreamEmulator.cpp:25-73) — streams, processes
// (keyswitch, bootstrap, mapped bootstrap, the four linear operations), puts of the inputs — and
// then gets an output, which evaluates the subgraph producing it.  The reference's implementation
// is lib/Runtime/GPUDFG.cpp:1467-1799 (semantics kept: stream kinds, put copies the data,
// generations so only stale processes rerun, output sizes of KS/PBS, constant / per-sample LUT
// and plaintext operands, SDFG_NUM_GPUS).
//
// Redesigned for the MI355X node rather than translated:
//   * the whole subgraph runs on the device: inputs cross PCIe once, intermediates (the
//     keyswitch output feeding the bootstrap, linear-op results) stay in HBM, accumulators are
//     built on the device from the LUT rows (lut.hip), and only outputs that somebody reads are
//     copied back.  The reference moves chunks host<->device around every process and builds the
//     accumulators on the host per chunk (GPUDFG.cpp:451-479, 1122-1136);
//   * the batch is cut into one contiguous shard per device entry, each run by its own host thread
//     on a stream cached in the graph (the reference's per-device scheduler threads,
//     GPUDFG.cpp:852-895, without its CPU-worker split: this backend is GPU-only), and a shard is
//     chunked only when the device's free memory asks for it (GPUDFG.cpp:696-731);
//   * keys come from the keyset bound to the process's context pointer (runtime.hip), resident on
//     every device after first use.
// Device list: CONCRETE_HIP_SDFG_DEVICES="0,0,1" (entries may repeat), else SDFG_NUM_GPUS (first
// N visible devices, capped at the visible count as GPUDFG.cpp:1745-1758), else every device.
#include <stdarg.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>

#include "common.hpp"
#include "pbs.hpp"
#include "runtime.hpp"

namespace chip {
namespace sdfg {

enum StreamKind { SK_U64, SK_MEMREF, SK_BATCH };
enum ProcKind { P_ADD, P_ADD_PT, P_MUL_CT, P_NEG, P_KS, P_PBS };

struct Dfg;
struct Proc;

struct Stream {
  std::string name;
  int stype = 0;
  StreamKind kind = SK_MEMREF;
  HostBuf host;                // rows x cols, row-major, valid when host_ok
  uint64_t rows = 0, cols = 0;
  bool host_ok = false;
  uint64_t version = 0;        // put streams: clock value of the last put
  bool computed = false;       // produced streams: host or device result exists for computed_eff
  uint64_t computed_eff = 0;
  Proc* producer = nullptr;
  std::vector<Proc*> consumers;
  Dfg* dfg = nullptr;
};

struct Proc {
  ProcKind kind;
  Stream* in[2] = {nullptr, nullptr};
  Stream* out = nullptr;
  uint32_t level = 0, base_log = 0, n_in = 0, n_out = 0, poly = 0, glwe = 0, output_size = 0, key_index = 0;
  void* ctx = nullptr;
};

// one shard's device context: a stream and grow-only device buffers reused by every chunk and get
// (buffer i = the i-th allocation of run_chunk; hipMalloc'd: pageable copies into memory that the
// stream-ordered pool had freed and handed out again were seen to read stale data)
struct Slot {
  uint32_t gpu = 0;
  hipStream_t s = nullptr;
  std::vector<void*> buf;
  std::vector<uint64_t> cap;
  std::vector<void*> retired;  // outgrown buffers, freed once every shard thread has joined
  uint32_t* status_h = nullptr;  // page-locked landing word of the stream-ordered status read
};

// hipFree synchronises the whole device, so a buffer outgrown while other shards' kernels run on
// the same device is retired and freed after the threads join
void slot_free_retired(Slot& sl) {
  if (sl.retired.empty()) return;
  CHIP_CHECK(hipSetDevice((int)sl.gpu));
  for (void* p : sl.retired) CHIP_CHECK(hipFree(p));
  sl.retired.clear();
}

void slot_free(Slot& sl) {
  if (!sl.s) return;
  CHIP_CHECK(hipSetDevice((int)sl.gpu));
  CHIP_CHECK(hipStreamSynchronize(sl.s));
  for (void* p : sl.buf)
    if (p) CHIP_CHECK(hipFree(p));
  for (void* p : sl.retired) CHIP_CHECK(hipFree(p));
  if (sl.status_h) CHIP_CHECK(hipHostFree(sl.status_h));
  release_stream_status((int)sl.gpu, sl.s);
  CHIP_CHECK(hipStreamDestroy(sl.s));
  sl = Slot{};
}

struct Dfg {
  std::mutex m;
  std::vector<Proc*> procs;
  std::unordered_set<Stream*> streams;
  std::vector<uint32_t> devices;
  std::vector<Slot> slots;
};

std::atomic<uint64_t> g_clock{0};

std::vector<uint32_t> default_devices() {
  const int visible = concrete_hip_device_count();
  if (visible <= 0) rt_die("stream_emulator_init: no GPUs available on system (device count %d)", visible);
  std::vector<uint32_t> d;
  if (const char* e = getenv("CONCRETE_HIP_SDFG_DEVICES")) {
    for (const char* p = e; *p;) {
      char* end = nullptr;
      const unsigned long v = strtoul(p, &end, 10);
      if (end == p) break;
      if ((int)v >= visible || v >= (unsigned long)RT_MAX_DEV) rt_die("CONCRETE_HIP_SDFG_DEVICES: device %lu not visible", v);
      d.push_back((uint32_t)v);
      p = *end ? end + 1 : end;
    }
    if (!d.empty()) return d;
  }
  size_t n = (size_t)std::min(visible, RT_MAX_DEV);
  if (const char* e = getenv("SDFG_NUM_GPUS")) {
    size_t req = strtoul(e, nullptr, 10);
    if (req == 0) {
      fprintf(stderr, "WARNING: no GPUs requested (%zu available) - continuing with one device.\n", n);
      req = 1;
    }
    if (req > n)
      fprintf(stderr, "WARNING: requested more GPUs (%zu) than available (%zu) - continuing with available devices.\n",
              req, n);
    else
      n = req;
  }
  for (size_t i = 0; i < n; ++i) d.push_back((uint32_t)i);
  return d;
}

void attach(Dfg* g, Proc* p) {
  for (Stream* s : p->in)
    if (s) {
      s->consumers.push_back(p);
      s->dfg = g;
      g->streams.insert(s);
    }
  p->out->producer = p;
  p->out->dfg = g;
  g->streams.insert(p->out);
  g->procs.push_back(p);
}

Proc* make(void* dfg, ProcKind k, void* sin1, void* sin2, void* sout) {
  if (!dfg || !sin1 || !sout) rt_die("stream_emulator: null graph or stream");
  Proc* p = new Proc();
  p->kind = k;
  p->in[0] = (Stream*)sin1;
  p->in[1] = (Stream*)sin2;
  p->out = (Stream*)sout;
  attach((Dfg*)dfg, p);
  return p;
}

// ---- scheduling ------------------------------------------------------------------------------

// newest put reaching s (memoised per get).  A produced stream counts its own puts too: a value
// put on an intermediate stream makes every consumer computed before it stale.
uint64_t eff(Stream* s, std::unordered_map<Stream*, uint64_t>& memo) {
  if (!s->producer) return s->version;
  auto it = memo.find(s);
  if (it != memo.end()) return it->second;
  uint64_t v = s->version;
  for (Stream* i : s->producer->in)
    if (i) v = std::max(v, eff(i, memo));
  memo[s] = v;
  return v;
}

// processes to run (post-order) so that s is available: a produced stream is recomputed when an
// input changed since it was computed (the reference's generations, GPUDFG.cpp:580-599) or when its
// value only ever lived on the device
void need(Stream* s, std::vector<Proc*>& q, std::unordered_set<Proc*>& queued,
          std::unordered_map<Stream*, uint64_t>& memo) {
  if (!s->producer) {
    if (!s->host_ok) rt_die("stream_emulator: no data was put on stream %s", s->name.c_str());
    return;
  }
  if (queued.count(s->producer)) return;
  const bool fresh = s->computed && s->computed_eff == eff(s, memo);
  if (fresh && s->host_ok) return;
  for (Stream* i : s->producer->in)
    if (i) need(i, q, queued, memo);
  queued.insert(s->producer);
  q.push_back(s->producer);
}

uint64_t out_width(const Proc* p, const std::unordered_map<Stream*, uint64_t>& width) {
  switch (p->kind) {
    case P_KS: return p->output_size ? p->output_size : p->n_out + 1;
    case P_PBS: return p->output_size;
    default: return width.at(p->in[0]);
  }
}

// role of a subgraph input for sharding: ciphertext rows, LUT rows, or per-sample scalars
enum Role { R_CT, R_LUT, R_SCALAR };

struct Input {
  Stream* s;
  Role role;
  bool broadcast;   // one LUT / one scalar for every sample
  uint64_t width;   // words per sample (ciphertext, LUT row) or 1 (scalar)
};

struct Plan {
  std::vector<Proc*> q;
  std::vector<Input> inputs;
  std::vector<Stream*> produced;            // outputs of q, in order
  std::unordered_set<Stream*> download;     // produced streams copied back to the host
  std::unordered_map<Stream*, uint64_t> width;
  uint64_t batch = 0;
};

Role role_of(const Stream* s, const Plan& P) {
  for (const Proc* p : P.q) {
    if (p->in[0] == s) return R_CT;
    if (p->in[1] == s) {
      if (p->kind == P_ADD) return R_CT;
      if (p->kind == P_PBS) return R_LUT;
      return R_SCALAR;
    }
  }
  return R_CT;
}

Plan plan_for(Stream* target) {
  Plan P;
  std::unordered_set<Proc*> queued;
  std::unordered_map<Stream*, uint64_t> memo;
  need(target, P.q, queued, memo);
  std::unordered_set<Stream*> produced;
  for (Proc* p : P.q) produced.insert(p->out);
  std::unordered_set<Stream*> seen;
  for (Proc* p : P.q)
    for (Stream* s : p->in)
      if (s && !produced.count(s) && seen.insert(s).second) P.inputs.push_back(Input{s, role_of(s, P), false, 0});
  // the batch: rows of the ciphertext inputs (GPUDFG.cpp:673-681)
  for (auto& in : P.inputs)
    if (in.role == R_CT) P.batch = std::max(P.batch, in.s->rows);
  if (P.batch == 0) P.batch = 1;
  for (auto& in : P.inputs) {
    const uint64_t elems = in.s->rows * in.s->cols;
    if (in.role == R_CT) {
      if (in.s->rows != P.batch) rt_die("stream %s: %llu ciphertexts, the batch has %llu", in.s->name.c_str(),
                                        (unsigned long long)in.s->rows, (unsigned long long)P.batch);
      in.width = in.s->cols;
    } else if (in.role == R_LUT) {
      // one LUT for all, or one per sample (the mapped bootstrap, GPUDFG.cpp:1234-1243)
      in.broadcast = in.s->rows == 1;
      if (!in.broadcast && in.s->rows != P.batch) rt_die("stream %s: number of LUTs does not match batch size", in.s->name.c_str());
      in.width = in.s->cols;
    } else {
      // a constant (GPUDFG.cpp:1321, 1379) or one value per sample
      in.broadcast = elems == 1;
      if (!in.broadcast && elems != P.batch) rt_die("stream %s: %llu values for a batch of %llu", in.s->name.c_str(),
                                                    (unsigned long long)elems, (unsigned long long)P.batch);
      in.width = 1;
    }
    P.width[in.s] = in.width;
  }
  for (Proc* p : P.q) {
    P.width[p->out] = out_width(p, P.width);
    P.produced.push_back(p->out);
    // read back: the requested stream, streams the host reads (device_to_host / device_to_both,
    // SDFGToStreamEmulator.cpp:334-343) and streams a process outside this subgraph consumes
    bool outside = p->out == target || p->out->stype == CONCRETE_HIP_TS_STREAM_TYPE_TOPO_TO_X86_LSAP ||
                   p->out->stype == CONCRETE_HIP_TS_STREAM_TYPE_TOPO_TO_BOTH;
    for (Proc* c : p->out->consumers)
      if (!queued.count(c)) outside = true;
    if (outside) P.download.insert(p->out);
  }
  return P;
}

// The registered key of a KS / PBS process must have the process's parameters (as the memref
// route asserts, runtime.hip run_batched_pbs / run_batched_ks): the device key's layout and size
// follow them, so a mismatch would read past the key or reinterpret it.
void check_proc(const Proc* p, const Plan& P) {
  const uint64_t w0 = P.width.at(p->in[0]);
  switch (p->kind) {
    case P_KS: {
      RT_ASSERT(w0 == (uint64_t)p->n_in + 1);
      RT_ASSERT(P.width.at(p->out) == (uint64_t)p->n_out + 1);
      KskEntry* e = keyset_ksk_entry(keyset_of_context(p->ctx), p->key_index);
      if (!e) rt_die("stream_emulator: keyswitch key index %u not registered", p->key_index);
      if (e->level != p->level || e->base_log != p->base_log || e->n_in != p->n_in || e->n_out != p->n_out)
        rt_die("stream_emulator: keyswitch key %u is (l=%u, logB=%u, %u -> %u), the process asks (l=%u, logB=%u, "
               "%u -> %u)", p->key_index, e->level, e->base_log, e->n_in, e->n_out, p->level, p->base_log, p->n_in,
               p->n_out);
      break;
    }
    case P_PBS: {
      // GPUDFG.cpp:1116
      RT_ASSERT(p->output_size == p->glwe * p->poly + 1);
      RT_ASSERT(w0 == (uint64_t)p->n_in + 1);
      RT_ASSERT(P.width.at(p->in[1]) == p->poly);
      BskEntry* e = keyset_bsk_entry(keyset_of_context(p->ctx), p->key_index);
      if (!e) rt_die("stream_emulator: bootstrap key index %u not registered", p->key_index);
      if (e->n != p->n_in || e->k != p->glwe || e->N != p->poly || e->level != p->level || e->base_log != p->base_log)
        rt_die("stream_emulator: bootstrap key %u is (n=%u, k=%u, N=%u, l=%u, logB=%u), the process asks (n=%u, k=%u, "
               "N=%u, l=%u, logB=%u)", p->key_index, e->n, e->k, e->N, e->level, e->base_log, p->n_in, p->glwe,
               p->poly, p->level, p->base_log);
      break;
    }
    case P_ADD:
      RT_ASSERT(P.width.at(p->in[1]) == w0);
      break;
    default:
      break;
  }
}

struct Shard {
  uint64_t start, count;
};

// bytes of device memory one sample of the subgraph needs (inputs, every produced stream, the
// mapped accumulators and indexes); the per-sample spectra of the general PBS path are inside
// concrete_hip_pbs's own (pooled) allocation
uint64_t bytes_per_sample(const Plan& P) {
  uint64_t b = 0;
  for (const auto& in : P.inputs)
    if (!in.broadcast) b += in.width * 8;
  for (Stream* s : P.produced) b += P.width.at(s) * 8;
  for (const Proc* p : P.q)
    if (p->kind == P_PBS) b += ((uint64_t)(p->glwe + 1) * p->poly + 1) * 8;
  return std::max<uint64_t>(b, 8);
}

bool trace_on() {
  static const bool on = getenv("CONCRETE_HIP_SDFG_TRACE") && atoi(getenv("CONCRETE_HIP_SDFG_TRACE")) != 0;
  return on;
}

void run_chunk(const Plan& P, Slot& sl, uint64_t start, uint64_t cnt) {
  hipStream_t s = sl.s;
  std::unordered_map<Stream*, uint64_t*> dev;
  size_t nbuf = 0;
  auto alloc = [&](uint64_t bytes) {  // the slot's nbuf-th buffer, grown to `bytes` (stream idle here)
    bytes = std::max<uint64_t>(bytes, 8);
    if (nbuf == sl.buf.size()) sl.buf.push_back(nullptr), sl.cap.push_back(0);
    if (sl.cap[nbuf] < bytes) {
      if (sl.buf[nbuf]) sl.retired.push_back(sl.buf[nbuf]);
      sl.buf[nbuf] = nullptr;
      CHIP_CHECK(hipMalloc(&sl.buf[nbuf], bytes));
      sl.cap[nbuf] = bytes;
    }
    return (uint64_t*)sl.buf[nbuf++];
  };
  // inputs: this chunk's rows (or the whole broadcast operand)
  for (const auto& in : P.inputs) {
    const uint64_t rows = in.broadcast ? 1 : cnt;
    uint64_t* d = alloc(rows * in.width * 8);
    const uint64_t* src = in.s->host.data() + (in.broadcast ? 0 : start * in.width);
    CHIP_CHECK(copy_h2d(d, in.s->host, src, rows * in.width * 8, s));
    dev[in.s] = d;
  }
  auto is_broadcast = [&](Stream* x) {
    for (const auto& in : P.inputs)
      if (in.s == x) return in.broadcast;
    return false;
  };
  for (Proc* p : P.q) {
    const uint64_t w = P.width.at(p->out);
    uint64_t* o = alloc(cnt * w * 8);
    dev[p->out] = o;
    const uint64_t* a = dev.at(p->in[0]);
    switch (p->kind) {
      case P_KS: {
        concrete_hip_keyset* ks = keyset_of_context(p->ctx);
        const void* dk = keyset_ksk_on(ks, p->key_index, sl.gpu, s);
        if (concrete_hip_keyswitch(s, sl.gpu, o, nullptr, a, nullptr, (const uint64_t*)dk, p->n_in, p->n_out,
                                   p->base_log, p->level, (uint32_t)cnt) != 0)
          rt_die("%s", concrete_hip_last_error());
        break;
      }
      case P_PBS: {
        concrete_hip_keyset* ks = keyset_of_context(p->ctx);
        const void* fbsk = keyset_bsk_on(ks, p->key_index, sl.gpu, s);
        const bool mapped = !is_broadcast(p->in[1]);
        const uint64_t rows = mapped ? cnt : 1, glwe = (uint64_t)(p->glwe + 1) * p->poly;
        uint64_t* acc = alloc(rows * glwe * 8);
        launch_trivial_glwe(s, acc, dev.at(p->in[1]), rows, p->glwe, p->poly);
        uint64_t* lidx = nullptr;
        if (mapped) {
          lidx = alloc(cnt * 8);
          launch_iota(s, lidx, cnt);
        }
        if (concrete_hip_pbs(s, sl.gpu, o, nullptr, acc, lidx, a, nullptr, fbsk, p->n_in, p->glwe, p->poly,
                             p->base_log, p->level, (uint32_t)cnt, nullptr) != 0)
          rt_die("%s", concrete_hip_last_error());
        break;
      }
      case P_ADD:
        launch_linear_op(s, LINOP_ADD, o, a, dev.at(p->in[1]), 1, (uint32_t)(w - 1), cnt);
        break;
      case P_ADD_PT:
        launch_linear_op(s, LINOP_ADD_PT, o, a, dev.at(p->in[1]), is_broadcast(p->in[1]) ? 0 : 1, (uint32_t)(w - 1),
                         cnt);
        break;
      case P_MUL_CT:
        launch_linear_op(s, LINOP_MUL_CT, o, a, dev.at(p->in[1]), is_broadcast(p->in[1]) ? 0 : 1, (uint32_t)(w - 1),
                         cnt);
        break;
      case P_NEG:
        launch_linear_op(s, LINOP_NEG, o, a, nullptr, 0, (uint32_t)(w - 1), cnt);
        break;
    }
  }
  // copies to and from the streams' page-locked host buffers are stream-ordered DMA; the stream is
  // idle when the chunk returns
  for (Stream* x : P.produced)
    if (P.download.count(x)) {
      const uint64_t w = P.width.at(x);
      CHIP_CHECK(copy_d2h(x->host.data() + start * w, x->host, dev.at(x), cnt * w * 8, s));
    }
  CHIP_CHECK(hipStreamSynchronize(s));
  if (trace_on()) {
    for (const auto& in : P.inputs) {
      uint64_t h = 0;
      for (uint64_t v : in.s->host) h = h * 31 + v;
      fprintf(stderr, "[sdfg]   input %s %llux%llu hash %llx\n", in.s->name.c_str(), (unsigned long long)in.s->rows,
              (unsigned long long)in.s->cols, (unsigned long long)h);
    }
    for (Stream* x : P.produced)
      if (P.download.count(x)) {
        uint64_t h = 0;
        for (uint64_t v : x->host) h ^= v;
        fprintf(stderr, "[sdfg]   output %s hash %llx\n", x->name.c_str(), (unsigned long long)h);
      }
  }
}

void execute(Dfg* g, Stream* target) {
  Plan P = plan_for(target);
  if (trace_on()) {
    fprintf(stderr, "[sdfg] get %s: %zu processes, batch %llu, %zu devices:", target->name.c_str(), P.q.size(),
            (unsigned long long)P.batch, g->devices.size());
    for (Proc* p : P.q) fprintf(stderr, " %d->%s%s", (int)p->kind, p->out->name.c_str(), P.download.count(p->out) ? "(D2H)" : "");
    fprintf(stderr, "\n");
  }
  if (P.q.empty()) return;
  for (Proc* p : P.q) check_proc(p, P);
  // host space of the results read back (threads fill disjoint row ranges)
  for (Stream* x : P.produced)
    if (P.download.count(x)) {
      x->rows = P.batch, x->cols = P.width.at(x);
      x->host.resize(x->rows * x->cols);  // every row is written by its shard's D2H
    }
  const uint64_t parts = std::max<uint64_t>(1, std::min<uint64_t>(g->devices.size(), P.batch));
  if (g->slots.size() < parts) g->slots.resize(parts);
  std::vector<Shard> shard(parts);
  for (uint64_t r = 0; r < parts; ++r) {
    Slot& sl = g->slots[r];
    if (!sl.s || sl.gpu != g->devices[r]) {
      slot_free(sl);
      sl.gpu = g->devices[r];
      CHIP_CHECK(hipSetDevice((int)sl.gpu));
      CHIP_CHECK(hipStreamCreateWithFlags(&sl.s, hipStreamNonBlocking));
      CHIP_CHECK(hipHostMalloc((void**)&sl.status_h, sizeof(uint32_t), hipHostMallocDefault));
    }
    const uint64_t base = P.batch / parts, extra = P.batch % parts;
    shard[r].count = base + (r < extra ? 1 : 0);
    shard[r].start = r * base + std::min<uint64_t>(r, extra);
  }
  const uint64_t per_sample = bytes_per_sample(P);
  auto work = [&](uint64_t r) {
    Slot& sl = g->slots[r];
    CHIP_CHECK(hipSetDevice((int)sl.gpu));
    size_t free_b = 0, total_b = 0;
    CHIP_CHECK(hipMemGetInfo(&free_b, &total_b));
    // half of the free memory for this shard's chunks (several shards may share the device)
    const uint64_t chunk = std::max<uint64_t>(1, (uint64_t)(free_b / 2 / parts) / per_sample);
    for (uint64_t s0 = 0; s0 < shard[r].count; s0 += chunk)
      run_chunk(P, sl, shard[r].start + s0, std::min(chunk, shard[r].count - s0));
    // the shard stream's own status read (no device-wide synchronisation)
    if (take_stream_status((int)sl.gpu, sl.s, sl.status_h) != 0) rt_die("%s", concrete_hip_last_error());
  };
  if (parts == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (uint64_t r = 0; r < parts; ++r) th.emplace_back(work, r);
    for (auto& t : th) t.join();
  }
  for (uint64_t r = 0; r < parts; ++r) slot_free_retired(g->slots[r]);
  std::unordered_map<Stream*, uint64_t> memo;
  for (Stream* x : P.produced) {
    x->computed = true;
    x->computed_eff = eff(x, memo);
    x->host_ok = P.download.count(x) > 0;
  }
}

void get_host(Stream* s) {
  if (!s) rt_die("stream_emulator: null stream");
  if (s->producer) {
    Dfg* g = s->dfg;
    std::lock_guard<std::mutex> lk(g->m);
    execute(g, s);
  } else if (!s->host_ok) {
    rt_die("stream_emulator: no data on stream %s", s->name.c_str());
  }
}

void put(Stream* s, const uint64_t* data, uint64_t rows, uint64_t cols, uint64_t stride0) {
  if (!s) rt_die("stream_emulator: null stream");
  s->rows = rows, s->cols = cols;
  s->host.resize(rows * cols);
  copy_rows(s->host.data(), cols, data, stride0, rows, cols);
  s->host_ok = true;
  s->version = ++g_clock;
  if (s->producer) {  // a value put on a produced stream stands until its inputs change
    std::unordered_map<Stream*, uint64_t> memo;
    s->computed = true;
    s->computed_eff = eff(s, memo);
  }
}

void copy_out(Stream* s, uint64_t* out, uint64_t rows, uint64_t cols, uint64_t stride0) {
  if (s->rows * s->cols != rows * cols || (rows > 1 && s->cols != cols))
    rt_die("stream_emulator: stream %s holds %llux%llu words, the output memref is %llux%llu", s->name.c_str(),
           (unsigned long long)s->rows, (unsigned long long)s->cols, (unsigned long long)rows,
           (unsigned long long)cols);
  copy_rows(out, stride0, s->host.data(), cols, rows, cols);
  if (trace_on()) {
    uint64_t h = 0;
    for (uint64_t v : s->host) h ^= v;
    fprintf(stderr, "[sdfg] copy_out %s %llux%llu xor %llx first %llx out %p\n", s->name.c_str(),
            (unsigned long long)rows, (unsigned long long)cols, (unsigned long long)h,
            (unsigned long long)s->host[0], (void*)out);
  }
}

Stream* new_stream(const char* name, int stype, StreamKind kind) {
  static std::atomic<uint64_t> id{0};
  Stream* s = new Stream();
  s->name = name ? name : "stream" + std::to_string(id++);
  s->stype = stype;
  s->kind = kind;
  return s;
}

}  // namespace sdfg
}  // namespace chip

using namespace chip;
using namespace chip::sdfg;

extern "C" {

void* stream_emulator_init(void) {
  Dfg* g = new Dfg();
  g->devices = default_devices();
  return g;
}

void stream_emulator_run(void* dfg) { (void)dfg; }  // the graph runs at the first get (GPUDFG.cpp:1795-1798)

void stream_emulator_delete(void* dfg) {
  Dfg* g = (Dfg*)dfg;
  if (!g) return;
  for (Slot& sl : g->slots) slot_free(sl);
  for (Proc* p : g->procs) delete p;
  for (Stream* s : g->streams) delete s;
  delete g;
}

// ---- processes (GPUDFG.cpp:1467-1648) --------------------------------------------------------
void stream_emulator_make_memref_add_lwe_ciphertexts_u64_process(void* dfg, void* sin1, void* sin2, void* sout) {
  make(dfg, P_ADD, sin1, sin2, sout);
}
void stream_emulator_make_memref_add_plaintext_lwe_ciphertext_u64_process(void* dfg, void* sin1, void* sin2,
                                                                          void* sout) {
  make(dfg, P_ADD_PT, sin1, sin2, sout);
}
void stream_emulator_make_memref_mul_cleartext_lwe_ciphertext_u64_process(void* dfg, void* sin1, void* sin2,
                                                                          void* sout) {
  make(dfg, P_MUL_CT, sin1, sin2, sout);
}
void stream_emulator_make_memref_negate_lwe_ciphertext_u64_process(void* dfg, void* sin1, void* sout) {
  make(dfg, P_NEG, sin1, nullptr, sout);
}
void stream_emulator_make_memref_keyswitch_lwe_u64_process(void* dfg, void* sin1, void* sout, uint32_t level,
                                                           uint32_t base_log, uint32_t input_lwe_dim,
                                                           uint32_t output_lwe_dim, uint32_t output_size,
                                                           uint32_t ksk_index, void* context) {
  Proc* p = make(dfg, P_KS, sin1, nullptr, sout);
  p->level = level, p->base_log = base_log, p->n_in = input_lwe_dim, p->n_out = output_lwe_dim;
  p->output_size = output_size, p->key_index = ksk_index, p->ctx = context;
}
void stream_emulator_make_memref_bootstrap_lwe_u64_process(void* dfg, void* sin1, void* sin2, void* sout,
                                                           uint32_t input_lwe_dim, uint32_t poly_size,
                                                           uint32_t level, uint32_t base_log, uint32_t glwe_dim,
                                                           uint32_t output_size, uint32_t bsk_index, void* context) {
  Proc* p = make(dfg, P_PBS, sin1, sin2, sout);
  p->n_in = input_lwe_dim, p->poly = poly_size, p->level = level, p->base_log = base_log, p->glwe = glwe_dim;
  p->output_size = output_size, p->key_index = bsk_index, p->ctx = context;
}
// the batched forms only mark stream kinds in the reference; execution is the same here
void stream_emulator_make_memref_batched_add_lwe_ciphertexts_u64_process(void* dfg, void* sin1, void* sin2,
                                                                         void* sout) {
  make(dfg, P_ADD, sin1, sin2, sout);
}
void stream_emulator_make_memref_batched_add_plaintext_lwe_ciphertext_u64_process(void* dfg, void* sin1, void* sin2,
                                                                                  void* sout) {
  make(dfg, P_ADD_PT, sin1, sin2, sout);
}
void stream_emulator_make_memref_batched_add_plaintext_cst_lwe_ciphertext_u64_process(void* dfg, void* sin1,
                                                                                      void* sin2, void* sout) {
  make(dfg, P_ADD_PT, sin1, sin2, sout);
}
void stream_emulator_make_memref_batched_mul_cleartext_lwe_ciphertext_u64_process(void* dfg, void* sin1, void* sin2,
                                                                                  void* sout) {
  make(dfg, P_MUL_CT, sin1, sin2, sout);
}
void stream_emulator_make_memref_batched_mul_cleartext_cst_lwe_ciphertext_u64_process(void* dfg, void* sin1,
                                                                                      void* sin2, void* sout) {
  make(dfg, P_MUL_CT, sin1, sin2, sout);
}
void stream_emulator_make_memref_batched_negate_lwe_ciphertext_u64_process(void* dfg, void* sin1, void* sout) {
  make(dfg, P_NEG, sin1, nullptr, sout);
}
void stream_emulator_make_memref_batched_keyswitch_lwe_u64_process(void* dfg, void* sin1, void* sout, uint32_t level,
                                                                   uint32_t base_log, uint32_t input_lwe_dim,
                                                                   uint32_t output_lwe_dim, uint32_t output_size,
                                                                   uint32_t ksk_index, void* context) {
  stream_emulator_make_memref_keyswitch_lwe_u64_process(dfg, sin1, sout, level, base_log, input_lwe_dim,
                                                        output_lwe_dim, output_size, ksk_index, context);
}
void stream_emulator_make_memref_batched_bootstrap_lwe_u64_process(void* dfg, void* sin1, void* sin2, void* sout,
                                                                   uint32_t input_lwe_dim, uint32_t poly_size,
                                                                   uint32_t level, uint32_t base_log,
                                                                   uint32_t glwe_dim, uint32_t output_size,
                                                                   uint32_t bsk_index, void* context) {
  stream_emulator_make_memref_bootstrap_lwe_u64_process(dfg, sin1, sin2, sout, input_lwe_dim, poly_size, level,
                                                        base_log, glwe_dim, output_size, bsk_index, context);
}
void stream_emulator_make_memref_batched_mapped_bootstrap_lwe_u64_process(void* dfg, void* sin1, void* sin2,
                                                                          void* sout, uint32_t input_lwe_dim,
                                                                          uint32_t poly_size, uint32_t level,
                                                                          uint32_t base_log, uint32_t glwe_dim,
                                                                          uint32_t output_size, uint32_t bsk_index,
                                                                          void* context) {
  stream_emulator_make_memref_bootstrap_lwe_u64_process(dfg, sin1, sin2, sout, input_lwe_dim, poly_size, level,
                                                        base_log, glwe_dim, output_size, bsk_index, context);
}

// ---- streams (GPUDFG.cpp:1650-1736) ------------------------------------------------------------
void* stream_emulator_make_uint64_stream(const char* name, int stype) { return new_stream(name, stype, SK_U64); }
void stream_emulator_put_uint64(void* stream, uint64_t e) { put((Stream*)stream, &e, 1, 1, 1); }
uint64_t stream_emulator_get_uint64(void* stream) {
  Stream* s = (Stream*)stream;
  get_host(s);
  if (s->rows * s->cols != 1) rt_die("stream_emulator_get_uint64: stream %s is not a scalar", s->name.c_str());
  return s->host[0];
}

void* stream_emulator_make_memref_stream(const char* name, int stype) { return new_stream(name, stype, SK_MEMREF); }
void stream_emulator_put_memref(void* stream, uint64_t* allocated, uint64_t* aligned, uint64_t offset, uint64_t size,
                                uint64_t stride, uint64_t data_ownership) {
  if (stride != 1) rt_die("stream_emulator_put_memref: strided memrefs not supported");
  put((Stream*)stream, aligned + offset, 1, size, size);
  if (data_ownership) free(allocated);  // the data was copied; ownership ends here
}
void stream_emulator_get_memref(void* stream, uint64_t* out_allocated, uint64_t* out_aligned, uint64_t out_offset,
                                uint64_t out_size, uint64_t out_stride) {
  (void)out_allocated;
  if (out_stride != 1) rt_die("stream_emulator_get_memref: strided memrefs not supported");
  Stream* s = (Stream*)stream;
  get_host(s);
  copy_out(s, out_aligned + out_offset, 1, out_size, out_size);
}

void* stream_emulator_make_memref_batch_stream(const char* name, int stype) {
  return new_stream(name, stype, SK_BATCH);
}
void stream_emulator_put_memref_batch(void* stream, uint64_t* allocated, uint64_t* aligned, uint64_t offset,
                                      uint64_t size0, uint64_t size1, uint64_t stride0, uint64_t stride1,
                                      uint64_t data_ownership) {
  if (stride1 != 1) rt_die("stream_emulator_put_memref_batch: strided memrefs not supported");
  put((Stream*)stream, aligned + offset, size0, size1, stride0);
  if (data_ownership) free(allocated);
}
void stream_emulator_get_memref_batch(void* stream, uint64_t* out_allocated, uint64_t* out_aligned,
                                      uint64_t out_offset, uint64_t out_size0, uint64_t out_size1,
                                      uint64_t out_stride0, uint64_t out_stride1) {
  (void)out_allocated;
  if (out_stride1 != 1) rt_die("stream_emulator_get_memref_batch: strided memrefs not supported");
  Stream* s = (Stream*)stream;
  get_host(s);
  copy_out(s, out_aligned + out_offset, out_size0, out_size1, out_stride0);
}

}  // extern "C"
