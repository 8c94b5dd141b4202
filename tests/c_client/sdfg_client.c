/* A compiled circuit's view of the SDFG route, replayed in C: the call sequence
 * SDFGToStreamEmulator.cpp:25-73 lowers a table lookup to (stream_emulator_init, make streams,
 * make processes, run, put inputs, get outputs, delete), for the KS -> PBS atomic pattern of
 * FHEToTFHEScalar.cpp:373-437, against libconcrete_hip.so.  The keys come from the keyset API and
 * are bound to an opaque "runtime context" pointer, as a RuntimeContext would be.
 *
 * Usage: sdfg_client IN OUT.  IN (u64 words): n k N l logB ks_l ks_logB B, the BSK
 * [n][l][k+1][k+1][N], the KSK [kN][ks_l][n+1], the B input ciphertexts (B x (kN+1), big key),
 * the plaintext p, B per-sample LUT rows (B x N; row 0 is also the single LUT).  OUT: four B x
 * (kN+1) results, then the fifth:
 *   graph 1:  r1 = PBS_lut0(KS(x + p)),  r2 = -r1          (r1 TOPO_TO_BOTH, r2 TOPO_TO_X86)
 *             r3 = r1 after a new put of x with its rows reversed (the subgraph reruns: r3 = r1 reversed)
 *   graph 2:  r4 = mapped PBS_{lut_i}(KS(x_i))
 *   graph 3:  r5 = PBS_lut0(KS(x)) for ciphertext 0 alone (rank-1 memref streams, scalar processes)
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "concrete_hip.h"

static uint64_t *read_all(const char *path, size_t *words) {
  FILE *f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  long sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  uint64_t *buf = (uint64_t *)malloc((size_t)sz);
  if (fread(buf, 1, (size_t)sz, f) != (size_t)sz) {
    fclose(f);
    return NULL;
  }
  fclose(f);
  *words = (size_t)sz / 8;
  return buf;
}

int main(int argc, char **argv) {
  if (argc != 3) return 2;
  size_t words = 0;
  uint64_t *in = read_all(argv[1], &words);
  if (!in || words < 8) return 3;
  const uint64_t n = in[0], k = in[1], N = in[2], l = in[3], logB = in[4], ks_l = in[5], ks_logB = in[6], B = in[7];
  const uint64_t big = k * N, bsk_len = n * l * (k + 1) * (k + 1) * N, ksk_len = big * ks_l * (n + 1);
  const uint64_t *bsk = in + 8, *ksk = bsk + bsk_len, *cts = ksk + ksk_len;
  const uint64_t p = cts[B * (big + 1)];
  const uint64_t *luts = cts + B * (big + 1) + 1;
  if (words != 8 + bsk_len + ksk_len + B * (big + 1) + 1 + B * N) return 4;

  concrete_hip_keyset *ks = concrete_hip_keyset_create();
  if (concrete_hip_keyset_add_bsk(ks, 0, bsk, (uint32_t)n, (uint32_t)k, (uint32_t)l, (uint32_t)logB, (uint32_t)N) ||
      concrete_hip_keyset_add_ksk(ks, 0, ksk, (uint32_t)ks_l, (uint32_t)ks_logB, (uint32_t)big, (uint32_t)n)) {
    fprintf(stderr, "keyset: %s\n", concrete_hip_last_error());
    return 5;
  }
  static int runtime_context; /* stands for the circuit's RuntimeContext* */
  void *ctx = &runtime_context;
  if (concrete_hip_context_bind(ctx, ks)) return 6;

  const uint64_t W = big + 1;
  uint64_t *out = (uint64_t *)calloc(5 * B * W, 8);
  uint64_t *x2 = (uint64_t *)malloc(B * W * 8);

  /* ---- graph 1: x + p -> KS -> PBS -> r1, r2 = -r1 ---- */
  void *dfg = stream_emulator_init();
  void *s_x = stream_emulator_make_memref_batch_stream("x", CONCRETE_HIP_TS_STREAM_TYPE_X86_TO_TOPO_LSAP);
  void *s_p = stream_emulator_make_uint64_stream("p", CONCRETE_HIP_TS_STREAM_TYPE_X86_TO_TOPO_LSAP);
  void *s_xp = stream_emulator_make_memref_batch_stream("x+p", CONCRETE_HIP_TS_STREAM_TYPE_TOPO_TO_TOPO_LSAP);
  void *s_small = stream_emulator_make_memref_batch_stream("ks", CONCRETE_HIP_TS_STREAM_TYPE_TOPO_TO_TOPO_LSAP);
  void *s_lut = stream_emulator_make_memref_stream("lut", CONCRETE_HIP_TS_STREAM_TYPE_X86_TO_TOPO_LSAP);
  void *s_r1 = stream_emulator_make_memref_batch_stream("r1", CONCRETE_HIP_TS_STREAM_TYPE_TOPO_TO_BOTH);
  void *s_r2 = stream_emulator_make_memref_batch_stream("r2", CONCRETE_HIP_TS_STREAM_TYPE_TOPO_TO_X86_LSAP);
  stream_emulator_make_memref_batched_add_plaintext_cst_lwe_ciphertext_u64_process(dfg, s_x, s_p, s_xp);
  stream_emulator_make_memref_batched_keyswitch_lwe_u64_process(dfg, s_xp, s_small, (uint32_t)ks_l, (uint32_t)ks_logB,
                                                                (uint32_t)big, (uint32_t)n, (uint32_t)(n + 1), 0, ctx);
  stream_emulator_make_memref_batched_bootstrap_lwe_u64_process(dfg, s_small, s_lut, s_r1, (uint32_t)n, (uint32_t)N,
                                                                (uint32_t)l, (uint32_t)logB, (uint32_t)k,
                                                                (uint32_t)W, 0, ctx);
  stream_emulator_make_memref_batched_negate_lwe_ciphertext_u64_process(dfg, s_r1, s_r2);
  stream_emulator_run(dfg);
  stream_emulator_put_memref_batch(s_x, (uint64_t *)cts, (uint64_t *)cts, 0, B, W, W, 1, 0);
  stream_emulator_put_uint64(s_p, p);
  stream_emulator_put_memref(s_lut, (uint64_t *)luts, (uint64_t *)luts, 0, N, 1, 0);
  stream_emulator_get_memref_batch(s_r2, out + B * W, out + B * W, 0, B, W, W, 1);
  stream_emulator_get_memref_batch(s_r1, out, out, 0, B, W, W, 1); /* kept on the host: no rerun */
  /* a new put on x (its rows reversed): the generations make the subgraph rerun */
  for (uint64_t b = 0; b < B; ++b) memcpy(x2 + b * W, cts + (B - 1 - b) * W, W * 8);
  stream_emulator_put_memref_batch(s_x, x2, x2, 0, B, W, W, 1, 0);
  stream_emulator_get_memref_batch(s_r1, out + 2 * B * W, out + 2 * B * W, 0, B, W, W, 1);
  stream_emulator_delete(dfg);

  /* ---- graph 2: mapped bootstrap, one LUT row per sample ---- */
  dfg = stream_emulator_init();
  s_x = stream_emulator_make_memref_batch_stream("x", CONCRETE_HIP_TS_STREAM_TYPE_X86_TO_TOPO_LSAP);
  s_small = stream_emulator_make_memref_batch_stream("ks", CONCRETE_HIP_TS_STREAM_TYPE_TOPO_TO_TOPO_LSAP);
  void *s_luts = stream_emulator_make_memref_batch_stream("luts", CONCRETE_HIP_TS_STREAM_TYPE_X86_TO_TOPO_LSAP);
  void *s_r4 = stream_emulator_make_memref_batch_stream("r4", CONCRETE_HIP_TS_STREAM_TYPE_TOPO_TO_X86_LSAP);
  stream_emulator_make_memref_batched_keyswitch_lwe_u64_process(dfg, s_x, s_small, (uint32_t)ks_l, (uint32_t)ks_logB,
                                                                (uint32_t)big, (uint32_t)n, (uint32_t)(n + 1), 0, ctx);
  stream_emulator_make_memref_batched_mapped_bootstrap_lwe_u64_process(dfg, s_small, s_luts, s_r4, (uint32_t)n,
                                                                       (uint32_t)N, (uint32_t)l, (uint32_t)logB,
                                                                       (uint32_t)k, (uint32_t)W, 0, ctx);
  stream_emulator_run(dfg);
  stream_emulator_put_memref_batch(s_x, (uint64_t *)cts, (uint64_t *)cts, 0, B, W, W, 1, 0);
  stream_emulator_put_memref_batch(s_luts, (uint64_t *)luts, (uint64_t *)luts, 0, B, N, N, 1, 0);
  stream_emulator_get_memref_batch(s_r4, out + 3 * B * W, out + 3 * B * W, 0, B, W, W, 1);
  stream_emulator_delete(dfg);

  /* ---- graph 3: one ciphertext, scalar processes on rank-1 memref streams ---- */
  dfg = stream_emulator_init();
  void *s_c = stream_emulator_make_memref_stream("c", CONCRETE_HIP_TS_STREAM_TYPE_X86_TO_TOPO_LSAP);
  void *s_cs = stream_emulator_make_memref_stream("cs", CONCRETE_HIP_TS_STREAM_TYPE_TOPO_TO_TOPO_LSAP);
  void *s_l1 = stream_emulator_make_memref_stream("lut", CONCRETE_HIP_TS_STREAM_TYPE_X86_TO_TOPO_LSAP);
  void *s_r5 = stream_emulator_make_memref_stream("r5", CONCRETE_HIP_TS_STREAM_TYPE_TOPO_TO_X86_LSAP);
  stream_emulator_make_memref_keyswitch_lwe_u64_process(dfg, s_c, s_cs, (uint32_t)ks_l, (uint32_t)ks_logB,
                                                        (uint32_t)big, (uint32_t)n, (uint32_t)(n + 1), 0, ctx);
  stream_emulator_make_memref_bootstrap_lwe_u64_process(dfg, s_cs, s_l1, s_r5, (uint32_t)n, (uint32_t)N, (uint32_t)l,
                                                        (uint32_t)logB, (uint32_t)k, (uint32_t)W, 0, ctx);
  stream_emulator_run(dfg);
  stream_emulator_put_memref(s_c, (uint64_t *)cts, (uint64_t *)cts, 0, W, 1, 0);
  stream_emulator_put_memref(s_l1, (uint64_t *)luts, (uint64_t *)luts, 0, N, 1, 0);
  stream_emulator_get_memref(s_r5, out + 4 * B * W, out + 4 * B * W, 0, W, 1);
  stream_emulator_delete(dfg);

  concrete_hip_context_bind(ctx, NULL);
  concrete_hip_keyset_destroy(ks);
  FILE *f = fopen(argv[2], "wb");
  if (!f) return 7;
  /* r5 is one row: write B rows for a uniform file (rows 1.. of r5 stay zero) */
  fwrite(out, 8, 5 * B * W, f);
  fclose(f);
  free(out);
  free(x2);
  free(in);
  printf("sdfg_client ok\n");
  return 0;
}
