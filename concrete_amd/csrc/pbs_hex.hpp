// pbs_hex.hpp — host-side geometry of the six-wave N = 1024 kernel (pbs1024_hex.hip).
#pragma once
#include <stddef.h>

#include "pbs.hpp"

namespace chip {

// Six waves per ciphertext (one forward and one inverse transform each), CTS = 1 or 2 ciphertexts per
// workgroup (2: three waves per SIMD).  LDS: the fft512 tables, one transpose scratch per wave (which
// also publishes the wave's digit spectrum), the two negated accumulators per ciphertext, and eight
// sync counters per ciphertext.  No key ring: each wave reads its key slice from L2 into registers.
constexpr size_t pbs1024_hex_lds_bytes(int cts) {
  return PBS1024_TABLE_BYTES + 6 * (size_t)cts * PBS1024_XCH_SLOTS * 16 + (size_t)cts * 2 * 1024 * 8 +
         8 * (size_t)cts * 4;
}
int pbs1024_hex_launch(const PbsArgs& a, int cts);

}  // namespace chip
