// lut.hip — LUT encoding and accumulator construction on the device, so that a
// dataflow subgraph (encode -> KS -> PBS -> linear ops) stays resident between its processes.
//
//   encode/expand: compiler lib/Runtime/wrappers.cpp:388-450 (memref_encode_expand_lut_for_bootstrap)
//     out[o] = enc(in[map(t)]), t = (o + mega/2) / mega, mega = out_size / in_size, with the first
//     entry's half-box at both ends (negated at the top, t == in_size) and map the half rotation of
//     signed LUTs; enc(v) = v << (64 - out_bits - 1).  Host twin: keygen.cpp concrete_hip_encode_expand_lut.
//   accumulators: the trivial GLWE of a LUT row, k zero mask polynomials then the row as body
//     (wrappers.cpp:199-209, 296-310; GPUDFG.cpp:1122-1136 builds it on the host per chunk).
// Both are HBM-bound streams of 8-byte words (one thread per output word, coalesced).
#include <algorithm>

#include "../../include/concrete_hip.h"
#include "common.hpp"
#include "runtime.hpp"

namespace chip {

__global__ void __launch_bounds__(256) encode_expand_lut_kernel(uint64_t* __restrict__ out, uint64_t out_size,
                                                                const uint64_t* __restrict__ in, uint64_t in_size,
                                                                uint32_t sh, int is_signed, uint64_t total) {
  const uint64_t mega = out_size / in_size, half = in_size / 2;
  for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total; g += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t row = g / out_size, o = g - row * out_size;
    const uint64_t t = (o + mega / 2) / mega;  // in [0, in_size]
    const uint64_t li = t == in_size ? 0 : t;
    const uint64_t src = is_signed ? (li < half ? li + half : li - half) : li;
    const uint64_t v = in[row * in_size + src] << sh;
    out[g] = t == in_size ? 0ull - v : v;
  }
}

__global__ void __launch_bounds__(256) trivial_glwe_kernel(uint64_t* __restrict__ acc, const uint64_t* __restrict__ luts,
                                                           uint64_t glwe, uint64_t body, uint32_t N, uint64_t total) {
  for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total; g += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t l = g / glwe, c = g - l * glwe;
    acc[g] = c < body ? 0ull : luts[l * N + (c - body)];
  }
}

__global__ void __launch_bounds__(256) iota_kernel(uint64_t* __restrict__ idx, uint64_t count) {
  for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < count; g += (uint64_t)gridDim.x * blockDim.x)
    idx[g] = g;
}

static uint32_t grid_for(uint64_t total) { return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((total + 255) / 256, 8192)); }

void launch_trivial_glwe(hipStream_t s, uint64_t* acc, const uint64_t* luts, uint64_t num_luts, uint32_t k, uint32_t N) {
  const uint64_t glwe = (uint64_t)(k + 1) * N, total = glwe * num_luts;
  if (total == 0) return;
  hipLaunchKernelGGL(trivial_glwe_kernel, dim3(grid_for(total)), dim3(256), 0, s, acc, luts, glwe, (uint64_t)k * N, N,
                     total);
  CHIP_CHECK(hipGetLastError());
}

void launch_iota(hipStream_t s, uint64_t* idx, uint64_t count) {
  if (count == 0) return;
  hipLaunchKernelGGL(iota_kernel, dim3(grid_for(count)), dim3(256), 0, s, idx, count);
  CHIP_CHECK(hipGetLastError());
}

}  // namespace chip

using namespace chip;

extern "C" {

int concrete_hip_encode_expand_lut_device(void* stream, uint32_t gpu_index, uint64_t* out, uint64_t out_size,
                                          const uint64_t* in, uint64_t in_size, uint64_t num_luts,
                                          uint32_t out_message_bits, int is_signed) {
  if (num_luts == 0) return 0;
  if (!out || !in) {
    set_error("encode_expand_lut_device: null pointer");
    return -1;
  }
  // wrappers.cpp:402-404: power-of-two sizes, an even mega-case
  if (in_size == 0 || out_size % in_size != 0 || (out_size / in_size) % 2 != 0 || out_message_bits >= 63) {
    set_error("encode_expand_lut_device: out_size %llu is not an even multiple of in_size %llu (or out bits %u)",
              (unsigned long long)out_size, (unsigned long long)in_size, out_message_bits);
    return -3;
  }
  CHIP_CHECK(hipSetDevice((int)gpu_index));
  const uint64_t total = out_size * num_luts;
  hipLaunchKernelGGL(encode_expand_lut_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, out, out_size,
                     in, in_size, 64u - out_message_bits - 1u, is_signed, total);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("encode_expand_lut_device: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

int concrete_hip_build_accumulators(void* stream, uint32_t gpu_index, uint64_t* acc, const uint64_t* luts,
                                    uint64_t num_luts, uint32_t glwe_dim, uint32_t polynomial_size) {
  if (num_luts == 0) return 0;
  if (!acc || !luts) {
    set_error("build_accumulators: null pointer");
    return -1;
  }
  CHIP_CHECK(hipSetDevice((int)gpu_index));
  launch_trivial_glwe((hipStream_t)stream, acc, luts, num_luts, glwe_dim, polynomial_size);
  return 0;
}

}  // extern "C"
