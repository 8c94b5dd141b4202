// keycheck.hpp — the converted key's largest limb-spectrum magnitude, reduced inside the key
// conversion kernels (bsk.hip, pbs_generic.hip) as they store each value (round 6; keycheck.hip
// says what the value is for).  Each wave reduces max |z|^2 over the values its lanes stored and one
// lane folds it into one of SPEC_SINK_WORDS sharded words (the f64 bit pattern of a non-negative
// double orders as an unsigned integer, so atomicMax on the bits is a max on the values); the host
// takes the max of the words.  Sharding by block keeps the per-word contention of a 10^4-block
// conversion low.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace chip {

constexpr int SPEC_SINK_WORDS = 256;

// |z|^2 of a stored spectrum value
__device__ __forceinline__ double spec_mag2(double re, double im) { return __builtin_fma(re, re, im * im); }

// wave-reduce m2 (max |z|^2 of this lane's stored values) and fold it into the sink (nullptr: off)
__device__ __forceinline__ void spec_max_commit(unsigned long long* sink, double m2) {
  if (!sink) return;
  for (int o = 32; o >= 1; o >>= 1) m2 = fmax(m2, __shfl_xor(m2, o, 64));
  if ((threadIdx.x & 63) == 0 && m2 > 0.0)
    atomicMax(sink + (blockIdx.x & (SPEC_SINK_WORDS - 1)), (unsigned long long)__double_as_longlong(m2));
}

}  // namespace chip
