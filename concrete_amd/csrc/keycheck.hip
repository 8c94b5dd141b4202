// keycheck.hip — the exactness gate checked against the key actually converted (round 6).
//
// Every kernel computes the exact negacyclic product with f64 transforms and rounds each output to
// the nearest integer; that is exact while the certified rounding bound stays below
// 1/2.  The bound grows with the largest magnitude max|G| of the key's limb spectra.  The static
// gates (pbs.hpp: pbs1024_exact, pbs2048_ok, k2_ok, pbs_small_ok, generic_pbs_ok) were set with
// max|G| of random-looking keys; an imported key whose spectra are larger (a crafted or degenerate
// key: constant-coefficient rows reach 8x the random-key value at N = 1024) would round some
// coefficient the wrong way without any error.  So every conversion (concrete_hip_convert_bsk, the
// general-format conversions and companions) has its conversion kernels reduce max|G| over the
// values they store (keycheck.hpp: free beside the transforms, no extra pass over the key) and
// records it with the key's device address.  Each PBS call then evaluates the certified bound of its kernel for its actual
// base_log with that max|G| and refuses (-2) when it reaches 1/2 (concrete_hip_pbs: a hand-tuned
// kernel's key that fails first tries the general path's companion, whose narrower limbs give a
// smaller bound).  A key the backend did not convert (copied in by the caller) has no record and
// keeps the static gate.  The reference requires a converted key to be complete and correct before
// it is published (compiler include/concretelang/Runtime/context.h:104-112); the bound functions
// restate oracle/pyoracle.py (gpu2048_error_bound, gpu1024k2_error_bound, gpu_small_error_bound,
// generic_error_bound) and oracle/tfhe_oracle.c:ora_fft_error_bound, which the GPU tests already check
// every kernel's measured residual against.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <unordered_map>

#include "common.hpp"
#include "companion.hpp"
#include "keycheck.hpp"
#include "pbs.hpp"

namespace chip {

void keep_pool_memory();  // abi.hip

// scale of the stored spectra (the kernels' inverse normalisation folded into the key)
static double stored_scale(const KeyFormat& f, uint32_t N) {
  switch (f.kind) {
    case KeyKind::N1024: return 512.0;
    case KeyKind::N2048: return 1024.0;  // K+- = G(+-s) / 1024 (pbs2048.hip, bsk.hip)
    case KeyKind::K2N1024: return 512.0;
    case KeyKind::SMALL: return 512.0 * (1024.0 / N);  // 1 / (512 P), P = 1024 / N
    case KeyKind::GENERIC: return N / 2.0;
    default: return 0.0;
  }
}

namespace {
struct SpecRec {
  double maxG;  // unscaled max |G| over every limb spectrum of the key
  KeyKind kind;
  uint32_t k, N, level, bits;
};
std::mutex g_spec_mu;
std::unordered_map<const void*, SpecRec> g_spec;

double higham_gamma(double logM, double mu) {
  const double u = std::ldexp(1.0, -53);
  const double eta = mu + 4.0 * u / (1.0 - 4.0 * u) * (std::sqrt(2.0) + mu);
  return logM * eta / (1.0 - logM * eta);
}
}  // namespace

// Certified rounding bound of the kernel that runs (kind, k, N, l, logB) on a key with max|G| = maxG.
double certified_bound(KeyKind kind, uint32_t k, uint32_t N, uint32_t level, uint32_t logB, uint32_t bits,
                       double maxG) {
  const double u = std::ldexp(1.0, -53);
  switch (kind) {
    case KeyKind::N1024: {  // tfhe_oracle.c:ora_fft_error_bound (3 limbs of 22/21/21 bits)
      const double gamma = higham_gamma(9.0, u);
      const double rows = (double)(k + 1) * level;
      const double dnorm = std::sqrt((double)N) * std::ldexp(1.0, (int)logB - 1);
      const double max_out = rows * N * std::ldexp(1.0, (int)logB - 1) * std::ldexp(1.0, 22 - 1);
      return rows * dnorm * maxG * (4.0 * gamma + 3.0 * u) * 1.0001 + 4.0 * u * max_out;
    }
    case KeyKind::N2048: {  // pyoracle.py:gpu2048_error_bound
      const double gamma = higham_gamma(10.0, 2.0 * u);
      const double dsum = level > 1 ? 2.0 * level * std::ldexp(1.0, (int)logB - 1)
                                    : 2.0 * (std::ldexp(1.0, 15) + std::ldexp(1.0, logB > 17 ? (int)logB - 17 : 0) + 1.0);
      const double main = std::sqrt(2048.0) * dsum * maxG * (4.0 * gamma + 5.0 * u) * 1.0001;
      return main + 4.0 * u * (2048.0 * dsum * std::ldexp(1.0, 15));
    }
    case KeyKind::K2N1024: {  // pyoracle.py:gpu1024k2_error_bound
      const double gamma = higham_gamma(9.0, u);
      const double dsum = level == 1 ? 3.0 * (std::ldexp(1.0, 15) + std::ldexp(1.0, logB > 17 ? (int)logB - 17 : 0) + 1.0)
                                     : 3.0 * level * std::ldexp(1.0, (int)logB - 1);
      const double main = std::sqrt(1024.0) * dsum * maxG * (4.0 * gamma + 5.0 * u) * 1.0001;
      return main + 4.0 * u * (1024.0 * dsum * std::ldexp(1.0, 15));
    }
    case KeyKind::SMALL: {  // pyoracle.py:gpu_small_error_bound
      const double P = 1024.0 / N;
      const double gamma = higham_gamma(9.0 + std::log2(P) + 1.0, 2.0 * u);
      const double dmax = (logB <= 15 || level > 1)
                              ? std::ldexp(1.0, (int)logB - 1) * level
                              : std::ldexp(1.0, 15) + std::ldexp(1.0, logB > 17 ? (int)logB - 17 : 0) + 1.0;
      const double dsum = (k + 1) * dmax;
      const double main = std::sqrt(1024.0) * dsum * maxG * (4.0 * gamma + 5.0 * u) * 1.0001;
      return main + 4.0 * u * (N * dsum * std::ldexp(1.0, 15));
    }
    case KeyKind::GENERIC: return generic_error_bound(k, N, level, logB, bits, maxG);
    default: return INFINITY;
  }
}

// A zeroed sink for the conversion kernels' max |G|^2 (keycheck.hpp), stream-ordered.
unsigned long long* key_spectrum_sink(hipStream_t s) {
  unsigned long long* d = nullptr;
  keep_pool_memory();
  CHIP_CHECK(hipMallocAsync((void**)&d, SPEC_SINK_WORDS * sizeof(unsigned long long), s));
  CHIP_CHECK(hipMemsetAsync(d, 0, SPEC_SINK_WORDS * sizeof(unsigned long long), s));
  return d;
}

// The key just converted on s into `dest` (format f of (k, N, l)) left max |G|^2 in `sink` (the
// conversion kernels reduce it as they store the key: no pass of its own): wait for it, record
// max |G|, free the sink, and refuse (-2) a key that no base_log could use exactly.
int key_spectrum_record(hipStream_t s, const void* dest, const KeyFormat& f, uint32_t n, uint32_t k, uint32_t N,
                        uint32_t level, unsigned long long* sink) {
  (void)n;
  if (!sink) return 0;
  static thread_local unsigned long long* landing = nullptr;  // page-locked words of this thread
  if (!landing)
    CHIP_CHECK(hipHostMalloc((void**)&landing, SPEC_SINK_WORDS * sizeof(unsigned long long), hipHostMallocDefault));
  CHIP_CHECK(hipMemcpyAsync(landing, sink, SPEC_SINK_WORDS * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
  CHIP_CHECK(hipFreeAsync(sink, s));
  CHIP_CHECK(hipStreamSynchronize(s));
  double m2 = 0.0;
  for (int w = 0; w < SPEC_SINK_WORDS; ++w) {
    double x;
    const unsigned long long bits = landing[w];
    memcpy(&x, &bits, sizeof x);
    m2 = std::max(m2, x);
  }
  // |z|^2 by one FMA and a product is within 2u of the exact square (a relative 1u on |z|); the
  // margin keeps the recorded value an upper bound of the stored key's largest magnitude
  const double maxG = std::sqrt(m2) * stored_scale(f, N) * (1.0 + std::ldexp(1.0, -48));
  if (!dest) return 0;
  {
    std::lock_guard<std::mutex> g(g_spec_mu);
    g_spec[dest] = SpecRec{maxG, f.kind, k, N, level, f.bits};
  }
  if (!(certified_bound(f.kind, k, N, level, 1, f.bits, maxG) < 0.5)) {
    set_error("convert: the converted key's largest limb spectrum |G| = %.4g puts the certified rounding bound at "
              "or above 1/2 for every base_log (k=%u N=%u level=%u): no exact product is possible with this key",
              maxG, k, N, level);
    return -2;
  }
  return 0;
}

void key_spectrum_copy(const void* dest, const void* src) {
  std::lock_guard<std::mutex> g(g_spec_mu);
  auto it = g_spec.find(src);
  if (it == g_spec.end())
    g_spec.erase(dest);
  else
    g_spec[dest] = it->second;
}

void key_spectrum_forget(const void* key) {
  std::lock_guard<std::mutex> g(g_spec_mu);
  g_spec.erase(key);
}

// max|G| recorded for `key` converted in format `kind` for (k, N, l); -1 when none
double key_spectrum_max(const void* key, KeyKind kind, uint32_t k, uint32_t N, uint32_t level, uint32_t* bits) {
  std::lock_guard<std::mutex> g(g_spec_mu);
  auto it = g_spec.find(key);
  if (it == g_spec.end()) return -1.0;
  const SpecRec& r = it->second;
  if ((kind != KeyKind::NONE && r.kind != kind) || r.k != k || r.N != N || r.level != level) return -1.0;
  if (bits) *bits = r.bits;
  return r.maxG;
}

// 0 when the PBS on `key` is certified exact at logB (or the key has no record: the static gate
// holds), -2 with the message set when its measured spectrum puts the bound at or above 1/2.
int key_bound_check(const void* key, KeyKind kind, uint32_t k, uint32_t N, uint32_t level, uint32_t logB) {
  uint32_t bits = 0;
  const double maxG = key_spectrum_max(key, kind, k, N, level, &bits);
  if (maxG < 0.0) return 0;
  const double b = certified_bound(kind, k, N, level, logB, bits, maxG);
  if (b < 0.5) return 0;
  set_error("pbs: this key's largest limb spectrum |G| = %.4g puts the certified rounding bound at %.3f >= 1/2 for "
            "k=%u N=%u level=%u base_log=%u: the product would not be exact (a key with random-looking spectra "
            "stays below it; see DESIGN.md §3)",
            maxG, b, k, N, level, logB);
  return -2;
}

}  // namespace chip

using namespace chip;

extern "C" {

double concrete_hip_key_spectrum_max(const void* fourier_key) {
  std::lock_guard<std::mutex> g(g_spec_mu);
  auto it = g_spec.find(fourier_key);
  return it == g_spec.end() ? -1.0 : it->second.maxG;
}

double concrete_hip_key_error_bound(const void* fourier_key, uint32_t base_log) {
  SpecRec r;
  {
    std::lock_guard<std::mutex> g(g_spec_mu);
    auto it = g_spec.find(fourier_key);
    if (it == g_spec.end()) return -1.0;
    r = it->second;
  }
  return certified_bound(r.kind, r.k, r.N, r.level, base_log, r.bits, r.maxG);
}

}  // extern "C"
