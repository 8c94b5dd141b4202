/*
 * tfhe_oracle.h — CPU restatement of the concrete-cpu / tfhe 0.10 semantics of the
 * batched programmable-bootstrap (PBS) path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the HIP backend
 * (libconcrete_hip.so).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it; the product path never calls it.
 *
 * Provenance (the reference's arithmetic lives in the un-vendored crate tfhe 0.10.0,
 * backends/concrete-cpu/implementation/Cargo.lock:867-870; its published algorithms are
 * restated here, anchored on the reference call sites):
 *   - LWE/GLWE/GGSW/BSK/KSK layouts ........ concrete-cpu c_api/bootstrap.rs:417-444,
 *                                             keyswitch.rs:226-236, secret_key.rs:343-357
 *   - PBS entry ............................. concrete-cpu c_api/bootstrap.rs:347-414
 *   - keyswitch entry ....................... concrete-cpu c_api/keyswitch.rs:185-223
 *   - trivial-GLWE accumulator from a LUT ... compiler lib/Runtime/wrappers.cpp:773-783
 *   - LUT expansion ......................... compiler lib/Runtime/wrappers.cpp:388-450
 *   - modulus switch (plaintext semantics) .. compiler lib/Runtime/simulation.cpp:64-84
 *   - native encode/decode .................. compiler lib/Common/Transformers.cpp:364-427
 *   - noise std from the 128-bit curve ...... compiler lib/Common/Security.cpp:16-27,
 *                                             tools/parameter-curves/.../curves.gen.h:2
 *
 * Parity contract: ciphertext bits of the reference's fft64 PBS are
 * approximate (f64 FFT); this oracle computes the EXACT product over Z_{2^64}[X]/(X^N+1).
 * Two independent exact paths are provided: a schoolbook definition and a Karatsuba
 * ring product (both pure integer arithmetic), plus a fast limb-split f64 FFT path whose
 * rounding is certified exact and is itself checked against the
 * integer paths in tests/test_oracle.py.
 */
#ifndef TFHE_ORACLE_H
#define TFHE_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- deterministic PRNG (NOT the tfhe CSPRNG; synthetic inputs only) ---- */
typedef struct ora_rng { uint64_t s[4]; int has_spare; double spare; } ora_rng;
void ora_rng_seed(ora_rng *r, uint64_t seed);
uint64_t ora_rng_u64(ora_rng *r);
double ora_rng_gauss(ora_rng *r);
/* round(N(0, std_torus) * 2^64) wrapped to u64 */
uint64_t ora_gauss_torus(ora_rng *r, double std_torus);

/* 128-bit security curve: log2(std) = max(slope*size + bias, 2 - 64); Security.cpp:16-27 */
double ora_secure_log2_std(uint64_t glwe_dim, uint64_t poly_size);

/* ---------------- sizes (concrete-cpu c_api) ---------------- */
size_t ora_lwe_size(size_t lwe_dim);                                    /* n+1 */
size_t ora_glwe_size(size_t k, size_t N);                               /* (k+1)N */
size_t ora_ggsw_size(size_t k, size_t N, size_t l);                     /* l(k+1)^2 N */
size_t ora_bsk_size(size_t n, size_t k, size_t N, size_t l);            /* n l (k+1)^2 N */
size_t ora_ksk_size(size_t n_in, size_t n_out, size_t l);               /* n_in l (n_out+1) */

/* ---------------- keys / encryption ---------------- */
void ora_binary_key(uint64_t *sk, size_t len, ora_rng *r);
void ora_lwe_encrypt(const uint64_t *sk, uint64_t *ct, uint64_t pt, size_t n, double std_torus, ora_rng *r);
uint64_t ora_lwe_decrypt(const uint64_t *sk, const uint64_t *ct, size_t n);
/* body already holds the message polynomial; mask sampled, body += <mask,S> + e */
void ora_glwe_encrypt_assign(const uint64_t *glwe_sk, uint64_t *ct, size_t k, size_t N, double std_torus, ora_rng *r);
void ora_glwe_decrypt(const uint64_t *glwe_sk, const uint64_t *ct, uint64_t *out, size_t k, size_t N);
void ora_ggsw_encrypt(const uint64_t *glwe_sk, uint64_t *ggsw, uint64_t cleartext, size_t k, size_t N,
                      size_t l, size_t logB, double std_torus, ora_rng *r);
void ora_bsk_generate(uint64_t *bsk, const uint64_t *lwe_sk, const uint64_t *glwe_sk, size_t n, size_t k,
                      size_t N, size_t l, size_t logB, double std_torus, uint64_t seed);
void ora_ksk_generate(uint64_t *ksk, const uint64_t *sk_in, const uint64_t *sk_out, size_t n_in,
                      size_t n_out, size_t l, size_t logB, double std_torus, uint64_t seed);

/* ---------------- primitives ---------------- */
uint64_t ora_decomp_init_state(uint64_t x, size_t l, size_t logB);
/* one level of the balanced signed decomposition; returns the digit as wrapping u64 */
uint64_t ora_decomp_one_level(uint64_t *state, size_t logB);
/* digits[q] for q = 0..l-1, q = 0 is level l (least significant), as the tfhe iterator yields */
void ora_decompose(uint64_t x, size_t l, size_t logB, int64_t *digits);
size_t ora_modswitch(uint64_t x, size_t N); /* round(x * 2N / 2^64) mod 2N */
void ora_monomial_mul(uint64_t *out, const uint64_t *in, size_t d, size_t N); /* out = in * X^d */
void ora_monomial_div(uint64_t *out, const uint64_t *in, size_t d, size_t N); /* out = in * X^-d */
/* out += d * g mod (X^N + 1) over Z_{2^64}; d small signed */
void ora_polymul_acc_schoolbook(uint64_t *out, const int64_t *d, const uint64_t *g, size_t N);
void ora_polymul_acc_karatsuba(uint64_t *out, const int64_t *d, const uint64_t *g, size_t N);
void ora_sample_extract(uint64_t *lwe_out, const uint64_t *glwe, size_t k, size_t N);

/* ---------------- Fourier limb key (CPU side, oracle-private layout) ---------------- */
/* limb split of a u64 into L balanced signed limbs; returns limb bit widths via widths[] */
void ora_limb_widths(size_t L, int *widths);
void ora_limb_split(uint64_t g, size_t L, int64_t *limbs);
size_t ora_fourier_bsk_len(size_t n, size_t k, size_t N, size_t l, size_t L); /* in doubles */
void ora_bsk_to_fourier(double *fbsk, const uint64_t *bsk, size_t n, size_t k, size_t N, size_t l, size_t L);
/* certified bound on max |rounding error| of the limb FFT product for this key */
double ora_fft_error_bound(const double *fbsk, size_t n, size_t k, size_t N, size_t l, size_t logB, size_t L);

/* ---------------- PBS / KS ---------------- */
/* ORA_MODE_FFT64: the limb-FFT path with ONE 64-bit key limb (fbsk from limbs = 1), i.e. the
 * arithmetic of concrete-cpu's fft64 (tfhe 0.10: u64 -> i64 -> f64 key spectrum, f64 products,
 * rounding mod 2^64): NOT exact (the low output bits carry FFT noise, which decryption absorbs);
 * bench.py times it as the closer-to-reference CPU baseline, never as a parity check. */
enum { ORA_MODE_SCHOOLBOOK = 0, ORA_MODE_KARATSUBA = 1, ORA_MODE_FFT = 2, ORA_MODE_FFT64 = 3 };
/* acc (k+1)N in/out: acc += ExtProd(GGSW_i, ct1) */
void ora_external_product_acc(uint64_t *acc, const uint64_t *ggsw_std, const double *ggsw_fourier,
                              const uint64_t *ct1, size_t k, size_t N, size_t l, size_t logB, size_t L,
                              int mode, double *max_resid);
void ora_blind_rotate(uint64_t *acc, const uint64_t *lwe_in, const uint64_t *bsk_std, const double *fbsk,
                      size_t n, size_t k, size_t N, size_t l, size_t logB, size_t L, int mode, double *max_resid);
void ora_pbs(uint64_t *lwe_out, const uint64_t *lwe_in, const uint64_t *accumulator, const uint64_t *bsk_std,
             const double *fbsk, size_t n, size_t k, size_t N, size_t l, size_t logB, size_t L, int mode,
             double *max_resid);
/* batched PBS with the runtime's index arrays (GPUDFG.cpp:1149-1205 semantics), OpenMP over samples */
void ora_pbs_batch(uint64_t *out, const uint64_t *out_idx, const uint64_t *luts, const uint64_t *lut_idx,
                   const uint64_t *in, const uint64_t *in_idx, const uint64_t *bsk_std, const double *fbsk,
                   size_t n, size_t k, size_t N, size_t l, size_t logB, size_t L, size_t num_samples, int mode,
                   int nthreads, double *max_resid);
void ora_keyswitch(uint64_t *out, const uint64_t *in, const uint64_t *ksk, size_t l, size_t logB, size_t n_in,
                   size_t n_out);
void ora_keyswitch_batch(uint64_t *out, const uint64_t *out_idx, const uint64_t *in, const uint64_t *in_idx,
                         const uint64_t *ksk, size_t l, size_t logB, size_t n_in, size_t n_out,
                         size_t num_samples, int nthreads);

/* ---------------- encoding (compiler runtime) ---------------- */
uint64_t ora_encode_native(uint64_t m, uint32_t width);                 /* Transformers.cpp:364-382 */
uint64_t ora_decode_native(uint64_t x, uint32_t width, int is_signed);  /* Transformers.cpp:384-427 */
void ora_encode_expand_lut(uint64_t *out, size_t out_size, const uint64_t *in, size_t in_size,
                           uint32_t out_message_bits, int is_signed);   /* wrappers.cpp:388-450 */
void ora_trivial_glwe_from_lut(uint64_t *glwe, const uint64_t *lut, size_t k, size_t N); /* wrappers.cpp:773-783 */

#ifdef __cplusplus
}
#endif
#endif
