/* keyio_client.c — loads a serialized server keyset through include/concrete_hip.h Part 6 from
 * plain C99 (the surface a cgo / JNI / N-API binding uses) and prints what it read, one line per
 * key: kind index id level base_log glwe_dim poly_size n_in n_out compression key_words checksum.
 * Usage: keyio_client FILE   (exit 0, or 1 with the library's error message) */
#include <stdio.h>
#include <stdlib.h>

#include "concrete_hip.h"

static uint64_t checksum(const uint64_t *w, uint64_t n) {
  uint64_t h = 1469598103934665603ull;
  for (uint64_t i = 0; i < n; ++i) h = (h ^ w[i]) * 1099511628211ull;
  return h;
}

static int dump(const concrete_hip_server_keyset *sk, int bsk, uint32_t i) {
  concrete_hip_key_info k;
  if ((bsk ? concrete_hip_server_keyset_bsk_info(sk, i, &k) : concrete_hip_server_keyset_ksk_info(sk, i, &k)) != 0)
    return 1;
  uint64_t *buf = malloc(k.key_words * sizeof(uint64_t) + 8);
  if (!buf) return 1;
  int rc = bsk ? concrete_hip_server_keyset_read_bsk(sk, i, buf, k.key_words)
               : concrete_hip_server_keyset_read_ksk(sk, i, buf, k.key_words);
  if (rc == 0)
    printf("%s %u %u %u %u %u %u %u %u %u %llu %llu\n", bsk ? "bsk" : "ksk", i, k.id, k.level_count, k.base_log,
           k.glwe_dim, k.poly_size, k.input_lwe_dim, k.output_lwe_dim, k.compression,
           (unsigned long long)k.key_words, (unsigned long long)checksum(buf, k.key_words));
  free(buf);
  return rc != 0;
}

int main(int argc, char **argv) {
  if (argc != 2) return 2;
  concrete_hip_server_keyset *sk = NULL;
  if (concrete_hip_server_keyset_load_file(argv[1], CONCRETE_HIP_ROOT_SERVER_KEYSET, &sk) != 0) {
    fprintf(stderr, "%s\n", concrete_hip_last_error());
    return 1;
  }
  int bad = 0;
  for (uint32_t i = 0; i < concrete_hip_server_keyset_bsk_count(sk); ++i) bad |= dump(sk, 1, i);
  for (uint32_t i = 0; i < concrete_hip_server_keyset_ksk_count(sk); ++i) bad |= dump(sk, 0, i);
  if (bad) fprintf(stderr, "%s\n", concrete_hip_last_error());
  concrete_hip_server_keyset_destroy(sk);
  return bad;
}
