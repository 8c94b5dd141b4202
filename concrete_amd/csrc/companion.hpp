// companion.hpp — general-format companion keys (host side of libconcrete_hip).
//
// A PBS whose digits are wider than the hand-tuned kernel of its (k, N, l) accepts (N = 1024: the
// gate (k+1) l 2^logB <= 4096, pbs.hpp pbs1024_exact; N = 2048: logB <= 24) but which the general
// path (pbs_generic.hip) runs exactly runs there, on a companion key in the general format built
// from the standard key (abi.hip generic_companion_key; concrete_hip_pbs_generic for caller-held
// keys).  Kept apart from pbs.hpp, whose contents are the kernels' geometry.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pbs.hpp"

namespace chip {

KeyFormat generic_key_format(uint32_t k, uint32_t N, uint32_t level);  // pbs_generic.hip: any shape it runs

inline bool pbs_needs_generic_key(uint32_t k, uint32_t N, uint32_t level, uint32_t base_log) {
  const KeyFormat f = key_format(k, N, level);
  if (f.kind == KeyKind::N1024 && !pbs1024_exact(k, level, base_log)) return generic_pbs_ok(k, N, level, base_log);
  if (f.kind == KeyKind::N2048 && !pbs2048_ok(level, base_log))
    return generic_pbs_ok(k, N, level, base_log);
  if (f.kind == KeyKind::K2N1024 && !k2_ok(level, base_log))
    return generic_pbs_ok(k, N, level, base_log);
  if (f.kind == KeyKind::SMALL && !pbs_small_ok(k, N, level, base_log))
    return generic_pbs_ok(k, N, level, base_log);
  return false;
}

// Size in bytes of a general-format key ([n][col][limb][row][q][N/2] complex f64).
inline uint64_t generic_fourier_bsk_bytes(uint32_t n, uint32_t k, uint32_t level, uint32_t N) {
  const KeyFormat f = generic_key_format(k, N, level);
  return f.kind == KeyKind::GENERIC ? (uint64_t)n * level * (k + 1) * (k + 1) * f.limbs * (N / 2) * 16ull : 0;
}

// abi.hip: companions of hand-tuned-format keys.  `src` is the standard key (host or device
// memory) and must outlive the registration.
void register_std_source(const void* primary, const uint64_t* src, bool on_device, uint32_t gpu, uint32_t n,
                         uint32_t k, uint32_t level, uint32_t N);
void release_std_source(const void* primary);
const void* generic_companion_key(const void* primary, uint32_t n, uint32_t k, uint32_t level, uint32_t N,
                                  hipStream_t s);

// keycheck.hip: the exactness gate against the converted key's measured spectrum (round 6).
// key_spectrum_record reads the max|G| the conversion kernels left in the sink (synchronises s),
// records it for `dest`, and returns -2 when no base_log could use the key exactly; key_bound_check returns -2
// (message set) when the PBS on `key` at logB would not be certified exact (0 without a record).
unsigned long long* key_spectrum_sink(hipStream_t s);  // zeroed sink for ConvertArgs::smax
int key_spectrum_record(hipStream_t s, const void* dest, const KeyFormat& f, uint32_t n, uint32_t k, uint32_t N,
                        uint32_t level, unsigned long long* sink);
int key_bound_check(const void* key, KeyKind kind, uint32_t k, uint32_t N, uint32_t level, uint32_t logB);
void key_spectrum_copy(const void* dest, const void* src);
void key_spectrum_forget(const void* key);

}  // namespace chip
