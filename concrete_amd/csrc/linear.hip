// linear.hip — the four LWE linear-operation vectors of the runtime's GPU dataflow route
// (compiler lib/Runtime/GPUDFG.cpp:1286-1289, 1344-1346, 1402-1404, 1445-1446), which keep
// whole SDFG subgraphs on the device between bootstraps.  Exact wrapping u64 arithmetic on
// batch-major (num_samples, lwe_dimension + 1) ciphertext arrays, the semantics of the CPU
// route (memref_batched_{add,add_plaintext,mul_cleartext,negate}_lwe_ciphertext_u64):
//   add:       out = a + b                       (every word)
//   plaintext: out = a, out.body += p[sample]    (last word of each ciphertext)
//   cleartext: out = a * c[sample]               (every word)
//   negate:    out = -a                          (every word)
// HBM-bound streams: one thread per 2 words (16-B accesses), grid-stride.
#include "../../include/concrete_hip.h"
#include <algorithm>

#include "common.hpp"
#include "runtime.hpp"

namespace chip {

enum LinOp { LIN_ADD = 0, LIN_ADD_PT = 1, LIN_MUL_CT = 2, LIN_NEG = 3 };

template <int OP>
__global__ void __launch_bounds__(256) linear_kernel(uint64_t* __restrict__ out, const uint64_t* __restrict__ a,
                                                     const uint64_t* __restrict__ b, uint64_t width,
                                                     uint64_t total, uint64_t b_stride) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * 2;
  for (uint64_t e = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 2; e < total; e += stride) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const uint64_t idx = e + u;
      if (idx >= total) break;
      const uint64_t x = a[idx];
      uint64_t y;
      if constexpr (OP == LIN_ADD) y = x + b[idx];
      else if constexpr (OP == LIN_ADD_PT) y = (idx % width == width - 1) ? x + b[idx / width * b_stride] : x;
      else if constexpr (OP == LIN_MUL_CT) y = x * b[idx / width * b_stride];
      else y = 0ull - x;
      out[idx] = y;
    }
  }
}

template <int OP>
static void launch_linear_on(hipStream_t stream, uint64_t* out, const uint64_t* a, const uint64_t* b,
                             uint64_t b_stride, uint32_t lwe_dimension, uint64_t num_samples) {
  const uint64_t width = (uint64_t)lwe_dimension + 1, total = width * num_samples;
  if (total == 0) return;
  const uint64_t threads = (total + 1) / 2;
  const uint32_t blocks = (uint32_t)std::min<uint64_t>((threads + 255) / 256, 256ull * 64);
  hipLaunchKernelGGL((linear_kernel<OP>), dim3(blocks), dim3(256), 0, stream, out, a, b, width, total, b_stride);
  CHIP_CHECK(hipGetLastError());
}

template <int OP>
static void launch_linear(void* stream, uint32_t gpu, void* out, const void* a, const void* b, uint32_t lwe_dimension,
                          uint32_t num_samples) {
  CHIP_CHECK(hipSetDevice((int)gpu));
  launch_linear_on<OP>((hipStream_t)stream, (uint64_t*)out, (const uint64_t*)a, (const uint64_t*)b, 1, lwe_dimension,
                       num_samples);
}

// the SDFG route's form (sdfg.hip): the current device, a per-sample (b_stride 1) or broadcast
// (b_stride 0) plaintext / cleartext operand (the *_cst processes, GPUDFG.cpp:1321-1328, 1379-1386)
void launch_linear_op(hipStream_t s, int op, uint64_t* out, const uint64_t* a, const uint64_t* b, uint64_t b_stride,
                      uint32_t lwe_dimension, uint64_t num_samples) {
  switch (op) {
    case LINOP_ADD: launch_linear_on<LIN_ADD>(s, out, a, b, 1, lwe_dimension, num_samples); break;
    case LINOP_ADD_PT: launch_linear_on<LIN_ADD_PT>(s, out, a, b, b_stride, lwe_dimension, num_samples); break;
    case LINOP_MUL_CT: launch_linear_on<LIN_MUL_CT>(s, out, a, b, b_stride, lwe_dimension, num_samples); break;
    default: launch_linear_on<LIN_NEG>(s, out, a, b, 1, lwe_dimension, num_samples); break;
  }
}

}  // namespace chip

using namespace chip;

extern "C" {

void cuda_add_lwe_ciphertext_vector_64(void* stream, uint32_t gpu_index, void* lwe_array_out,
                                       const void* lwe_array_in_1, const void* lwe_array_in_2,
                                       uint32_t input_lwe_dimension, uint32_t input_lwe_ciphertext_count) {
  launch_linear<LIN_ADD>(stream, gpu_index, lwe_array_out, lwe_array_in_1, lwe_array_in_2, input_lwe_dimension,
                         input_lwe_ciphertext_count);
}

void cuda_add_lwe_ciphertext_vector_plaintext_vector_64(void* stream, uint32_t gpu_index, void* lwe_array_out,
                                                        const void* lwe_array_in, const void* plaintext_array_in,
                                                        uint32_t input_lwe_dimension,
                                                        uint32_t input_lwe_ciphertext_count) {
  launch_linear<LIN_ADD_PT>(stream, gpu_index, lwe_array_out, lwe_array_in, plaintext_array_in, input_lwe_dimension,
                            input_lwe_ciphertext_count);
}

void cuda_mult_lwe_ciphertext_vector_cleartext_vector_64(void* stream, uint32_t gpu_index, void* lwe_array_out,
                                                         const void* lwe_array_in, const void* cleartext_array_in,
                                                         uint32_t input_lwe_dimension,
                                                         uint32_t input_lwe_ciphertext_count) {
  launch_linear<LIN_MUL_CT>(stream, gpu_index, lwe_array_out, lwe_array_in, cleartext_array_in, input_lwe_dimension,
                            input_lwe_ciphertext_count);
}

void cuda_negate_lwe_ciphertext_vector_64(void* stream, uint32_t gpu_index, void* lwe_array_out,
                                          const void* lwe_array_in, uint32_t input_lwe_dimension,
                                          uint32_t input_lwe_ciphertext_count) {
  launch_linear<LIN_NEG>(stream, gpu_index, lwe_array_out, lwe_array_in, nullptr, input_lwe_dimension,
                         input_lwe_ciphertext_count);
}

}  // extern "C"
