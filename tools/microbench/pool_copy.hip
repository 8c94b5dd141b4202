// pool_copy.hip — does a host->device copy into stream-ordered pool memory that was freed and
// handed out again land where the next kernel reads it?  (sdfg.hip saw stale rows.)
// Build: hipcc --offload-arch=gfx950 -O2 pool_copy.hip -o pool_copy ; run: ./pool_copy
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      printf("%s failed: %s\n", #x, hipGetErrorString(e));                  \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

__global__ void copy_k(uint64_t* o, const uint64_t* a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) o[i] = a[i];
}

// mode bits: 1 = pinned host buffers, 2 = blocking copies (hipMemcpyWithStream), 4 = keep pool (threshold max)
static int run(int mode, size_t n, int rounds) {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  {
    hipMemPool_t pool;
    CK(hipDeviceGetDefaultMemPool(&pool, 0));
    uint64_t thr = (mode & 4) ? ~0ull : 0ull;
    CK(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr));
  }
  uint64_t *h_in, *h_out;
  std::vector<uint64_t> v_in(n), v_out(n);
  if (mode & 1) {
    CK(hipHostMalloc((void**)&h_in, n * 8));
    CK(hipHostMalloc((void**)&h_out, n * 8));
  } else {
    h_in = v_in.data(), h_out = v_out.data();
  }
  int bad = 0;
  for (int r = 0; r < rounds; ++r) {
    for (size_t i = 0; i < n; ++i) h_in[i] = (uint64_t)r * 0x9e3779b97f4a7c15ull + i;
    uint64_t *a, *b;
    CK(hipMallocAsync((void**)&a, n * 8, s));
    CK(hipMallocAsync((void**)&b, n * 8, s));
    if (mode & 2) CK(hipMemcpyWithStream(a, h_in, n * 8, hipMemcpyHostToDevice, s));
    else CK(hipMemcpyAsync(a, h_in, n * 8, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(copy_k, dim3(256), dim3(256), 0, s, b, a, n);
    memset(h_out, 0, n * 8);
    if (mode & 2) CK(hipMemcpyWithStream(h_out, b, n * 8, hipMemcpyDeviceToHost, s));
    else CK(hipMemcpyAsync(h_out, b, n * 8, hipMemcpyDeviceToHost, s));
    CK(hipFreeAsync(a, s));
    CK(hipFreeAsync(b, s));
    CK(hipStreamSynchronize(s));
    size_t wrong = 0;
    for (size_t i = 0; i < n; ++i) wrong += h_out[i] != h_in[i];
    if (wrong) ++bad;
    if (wrong && bad <= 3) printf("  mode %d round %d: %zu of %zu words wrong\n", mode, r, wrong, n);
  }
  if (mode & 1) {
    CK(hipHostFree(h_in));
    CK(hipHostFree(h_out));
  }
  CK(hipStreamDestroy(s));
  return bad;
}

int main() {
  const size_t sizes[] = {10 * 1025, 4096 * 631, 1 << 22};
  for (size_t n : sizes)
    for (int mode = 0; mode < 8; ++mode) {
      const int bad = run(mode, n, 20);
      printf("n=%zu mode=%d (pinned=%d blocking=%d keep_pool=%d): %d of 20 rounds wrong\n", n, mode, mode & 1,
             (mode >> 1) & 1, (mode >> 2) & 1, bad);
    }
  return 0;
}
