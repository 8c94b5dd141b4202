/* A plain C client of libconcrete_hip.so: what a C host (or a cgo / JNI / N-API shim) binding
 * include/concrete_hip.h sees.  Device-free calls only (queries and argument validation), so
 * it runs on a CPU-only machine; tests/test_c_abi.py compiles it with gcc -std=c99 and runs it. */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "concrete_hip.h"

#define CHECK(cond)                                            \
  do {                                                         \
    if (!(cond)) {                                             \
      fprintf(stderr, "FAILED line %d: %s\n", __LINE__, #cond); \
      return 1;                                                \
    }                                                          \
  } while (0)

int main(void) {
  CHECK(concrete_hip_abi_version() == 5);
  /* cfg2 and cfg4 (BASELINE.json) are supported, N = 2^17 is not (up to 2^16 since round 4) */
  CHECK(concrete_hip_pbs_supported(1, 1024, 3, 7) == 1);
  CHECK(concrete_hip_pbs_supported(1, 2048, 1, 23) == 1);
  CHECK(concrete_hip_pbs_supported(1, 131072, 1, 7) == 0);
  uint32_t limbs = 0, bits = 0;
  CHECK(concrete_hip_bsk_format(1, 1024, 3, &limbs, &bits) == 1 && limbs == 3);
  /* n (k+1)^2 l x 3 limbs x N/2 complex f64 */
  CHECK(concrete_hip_fourier_bsk_size_bytes(630, 1, 3, 1024) == 630ull * 4 * 3 * 3 * 512 * 16);
  /* null buffers are refused (-1); unsupported parameters are refused before any device call
   * (-2, with a message): the dummy host pointers below are never dereferenced */
  static uint64_t dummy[4];
  CHECK(concrete_hip_pbs(NULL, 0, NULL, NULL, NULL, NULL, NULL, NULL, NULL, 630, 1, 1024, 7, 3, 4, NULL) == -1);
  CHECK(concrete_hip_pbs(NULL, 0, dummy, NULL, dummy, NULL, dummy, NULL, dummy, 630, 1, 131072, 7, 3, 4, NULL) == -2);
  CHECK(strstr(concrete_hip_last_error(), "unsupported") != NULL);
  /* an empty batch is a no-op */
  CHECK(concrete_hip_pbs(NULL, 0, NULL, NULL, NULL, NULL, NULL, NULL, NULL, 630, 1, 1024, 7, 3, 0, NULL) == 0);
  printf("abi_client ok\n");
  return 0;
}
