/*
 * concrete_hip.h — C ABI of libconcrete_hip.so, the MI355X-native (gfx950) backend for the
 * batched programmable-bootstrap path of the Concrete compiler runtime.
 *
 * Part 1 (cuda_* / scratch_* / cleanup_* names) is exactly the set of backend entry points
 * libConcretelangRuntime calls when built with CONCRETELANG_CUDA_SUPPORT; the names are kept
 * because the runtime's compiled call sites use them.  Each declaration cites the reference
 * call site it replaces (paths relative to /root/reference/compilers/concrete-compiler/compiler).
 * Conventions: void returns, failures abort (reference `nounwind`,
 * backends/concrete-cpu/implementation/src/c_api.rs:22-36); everything is stream-ordered;
 * the caller synchronises.  `stream` is a hipStream_t created by cuda_create_stream.
 *
 * Part 2 (concrete_hip_*) are extensions: a size query for the device key format (fixes the
 * runtime's `len * sizeof(double)` allocation hazard, include/concretelang/Runtime/context.h:101-105),
 * status-returning variants, and the direct (no key registry) PBS used by the multi-GPU glue.
 */
#ifndef CONCRETE_HIP_H
#define CONCRETE_HIP_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------------------------
 * Part 1: runtime-facing ABI (tfhe-cuda-backend names)
 * ------------------------------------------------------------------------------------------ */

/* lib/Runtime/wrappers.cpp:129,185,283; lib/Runtime/GPUDFG.cpp:191 */
void *cuda_create_stream(uint32_t gpu_index);
/* lib/Runtime/wrappers.cpp:160,255,362; lib/Runtime/GPUDFG.cpp:168 */
void cuda_destroy_stream(void *stream, uint32_t gpu_index);
/* lib/Runtime/wrappers.cpp:50,146,194; include/concretelang/Runtime/context.h:103-104 */
void *cuda_malloc_async(uint64_t size, void *stream, uint32_t gpu_index);
/* lib/Runtime/wrappers.cpp:51,222; lib/Runtime/GPUDFG.cpp:475,1194; context.h:137-139 */
void cuda_memcpy_async_to_gpu(void *dest, void *src, uint64_t size, void *stream, uint32_t gpu_index);
/* lib/Runtime/wrappers.cpp:59; lib/Runtime/GPUDFG.cpp:407,463,1034 */
void cuda_memcpy_async_to_cpu(void *dest, const void *src, uint64_t size, void *stream, uint32_t gpu_index);
/* lib/Runtime/wrappers.cpp:65,157-159; include/concretelang/Runtime/context.h:47-55 */
void cuda_drop(void *ptr, uint32_t gpu_index);
/* lib/Runtime/wrappers.cpp:246-250; lib/Runtime/GPUDFG.cpp:392,422,432,1102 */
void cuda_drop_async(void *ptr, void *stream, uint32_t gpu_index);
/* lib/Runtime/wrappers.cpp:155 */
void cuda_synchronize_device(uint32_t gpu_index);

/* include/concretelang/Runtime/context.h:104-109: H2D + conversion of the standard u64 BSK
 * (host pointer `src`, layout [n][l][k+1][k+1][N], concrete-cpu bootstrap.rs:417-429) into the
 * device key format.  `dest` is the caller's allocation of n*l*(k+1)^2*N*8 bytes; the device
 * format is larger (exact limbs), so the backend keeps it in a registry keyed by `dest` and
 * releases it when cuda_drop(dest) is called.  The key is usable once the stream is synced. */
void cuda_convert_lwe_programmable_bootstrap_key_64(void *stream, uint32_t gpu_index, void *dest, void *src,
                                                    uint32_t input_lwe_dim, uint32_t glwe_dim,
                                                    uint32_t level_count, uint32_t polynomial_size);

/* lib/Runtime/wrappers.cpp:234,341; lib/Runtime/GPUDFG.cpp:126 */
void scratch_cuda_programmable_bootstrap_64(void *stream, uint32_t gpu_index, int8_t **pbs_buffer,
                                            uint32_t glwe_dimension, uint32_t polynomial_size,
                                            uint32_t level_count, uint32_t input_lwe_ciphertext_count,
                                            bool allocate_gpu_memory);
/* lib/Runtime/wrappers.cpp:241,348; lib/Runtime/GPUDFG.cpp:131 */
void cleanup_cuda_programmable_bootstrap(void *stream, uint32_t gpu_index, int8_t **pbs_buffer);

/* lib/Runtime/wrappers.cpp:237-240,344-347; lib/Runtime/GPUDFG.cpp:1214-1218: batched classic PBS.
 *   out[out_idx[s]] (kN+1 u64) = PBS(in[in_idx[s]] (n+1 u64), lut_vector[lut_idx[s]] ((k+1)N u64))
 * bootstrapping_key is the `dest` of cuda_convert_lwe_programmable_bootstrap_key_64.
 * The last two arguments are passed as (1, 1) by every reference call site (one LUT per
 * sample, stride 1); other values abort. */
void cuda_programmable_bootstrap_lwe_ciphertext_vector_64(
    void *stream, uint32_t gpu_index, void *lwe_array_out, void *lwe_output_indexes, void *lut_vector,
    void *lut_vector_indexes, void *lwe_array_in, void *lwe_input_indexes, void *bootstrapping_key,
    int8_t *pbs_buffer, uint32_t lwe_dimension, uint32_t glwe_dimension, uint32_t polynomial_size,
    uint32_t base_log, uint32_t level_count, uint32_t num_samples, uint32_t num_many_lut, uint32_t lut_stride);

/* lib/Runtime/wrappers.cpp:149-151, GPUDFG.cpp:1098-1101: batched LWE keyswitch; ksk is the
 * standard u64 key [n_in][l][n_out+1] copied verbatim to the device (context.h:117-145).
 * Exact u64 result.  For base_log <= 7 and >= 64 samples it runs on the int8 matrix cores
 * (key words split into bytes, exact int32 sums) with stream-ordered scratch: the key bytes
 * (8 (n_out+1) n_in l B) and the batch's int8 digits (<= 1 GiB per pass). */
void cuda_keyswitch_lwe_ciphertext_vector_64(void *stream, uint32_t gpu_index, void *lwe_array_out,
                                             void *lwe_output_indexes, void *lwe_array_in,
                                             void *lwe_input_indexes, void *ksk, uint32_t lwe_dimension_in,
                                             uint32_t lwe_dimension_out, uint32_t base_log,
                                             uint32_t level_count, uint32_t num_samples);

/* The four linear-operation vectors of the dataflow route (GPUDFG.cpp:1286-1289, 1344-1346,
 * 1402-1404, 1445-1446): batch-major (count, lwe_dimension + 1) u64 ciphertexts, wrapping.
 * plaintext/cleartext arrays hold one u64 per ciphertext. */
void cuda_add_lwe_ciphertext_vector_64(void *stream, uint32_t gpu_index, void *lwe_array_out,
                                       const void *lwe_array_in_1, const void *lwe_array_in_2,
                                       uint32_t input_lwe_dimension, uint32_t input_lwe_ciphertext_count);
void cuda_add_lwe_ciphertext_vector_plaintext_vector_64(void *stream, uint32_t gpu_index, void *lwe_array_out,
                                                        const void *lwe_array_in, const void *plaintext_array_in,
                                                        uint32_t input_lwe_dimension,
                                                        uint32_t input_lwe_ciphertext_count);
void cuda_mult_lwe_ciphertext_vector_cleartext_vector_64(void *stream, uint32_t gpu_index, void *lwe_array_out,
                                                         const void *lwe_array_in, const void *cleartext_array_in,
                                                         uint32_t input_lwe_dimension,
                                                         uint32_t input_lwe_ciphertext_count);
void cuda_negate_lwe_ciphertext_vector_64(void *stream, uint32_t gpu_index, void *lwe_array_out,
                                          const void *lwe_array_in, uint32_t input_lwe_dimension,
                                          uint32_t input_lwe_ciphertext_count);

/* ------------------------------------------------------------------------------------------
 * Part 2: extensions (return 0 on success, < 0 on error; message via concrete_hip_last_error)
 * ------------------------------------------------------------------------------------------ */

/* ABI version of this header (2: round 3 — context-resolved memref_*_cuda_u64, stream emulator;
 * 3: round 4 — keyswitch support query, key level-order check against client keys;
 * 4: round 5 — status words per (device, stream): concrete_hip_stream_status,
 *    concrete_hip_set_thread_spin_limit;
 * 5: round 6 — status slots recycled on stream destroy (concrete_hip_status_slots_in_use,
 *    concrete_hip_set_status_slot_cap), converted keys checked against the certified bound
 *    (concrete_hip_key_spectrum_max)). */
uint32_t concrete_hip_abi_version(void);
/* thread-local message of the last failed concrete_hip_* call */
const char *concrete_hip_last_error(void);
/* 1 if (k, N, level, base_log) has a compiled PBS kernel (wide digits: the general path), else 0 */
int concrete_hip_pbs_supported(uint32_t glwe_dim, uint32_t polynomial_size, uint32_t level_count,
                               uint32_t base_log);
/* 1 if the batched keyswitch runs (level, base_log, n_in -> n_out): level * base_log < 64,
 * n_out + 1 <= 65536; else 0 (round 4) */
int concrete_hip_keyswitch_supported(uint32_t level_count, uint32_t base_log, uint32_t input_lwe_dim,
                                     uint32_t output_lwe_dim);
/* DEPRECATED (kept for ABI version 2 callers): number of exact key limbs of the device format for
 * k = 1 only (it takes no glwe_dim; the k-dependent formats of round 4 differ, e.g. 5 limbs at
 * k = 4, N = 512, l = 2).  Use concrete_hip_bsk_format, which takes k. */
uint32_t concrete_hip_bsk_limbs(uint32_t polynomial_size, uint32_t level_count, uint32_t base_log);
/* device key format of (k, N, l): 0 unsupported, 1 / 2 the N = 1024 / 2048 (k = 1) kernels' layouts,
 * 3 the general path (pbs_generic.hip), 4 the k = 2, N = 1024 kernels' layout (pbs1024k2.hip,
 * round 4), 5 the small-ring kernels' (N = 512, k = 3 / N = 256, k = 5, 6, l <= 3: pbs_small.hip; N = 512,
 * k = 4, any l: pbs512k4.hip; round 4); code 2 covers N = 2048, l <= 4; *limbs
 * balanced key limbs of *limb_bits bits each */
int concrete_hip_bsk_format(uint32_t glwe_dim, uint32_t polynomial_size, uint32_t level_count, uint32_t *limbs,
                            uint32_t *limb_bits);
/* rounding-error bound of the general path's exact product for a key whose largest
 * limb-spectrum magnitude is max_key_spectrum (<= 0: the random-key estimate the gate uses);
 * -1 when (k, N, l) is not on the general path */
double concrete_hip_generic_error_bound(uint32_t glwe_dim, uint32_t polynomial_size, uint32_t level_count,
                                        uint32_t base_log, double max_key_spectrum);
/* The exactness gate against the converted key (round 6).  Every conversion (concrete_hip_convert_bsk,
 * concrete_hip_convert_bsk_generic, cuda_convert_lwe_programmable_bootstrap_key_64, keyset keys and
 * general-format companions) reduces the largest limb-spectrum magnitude max|G| of the key it wrote,
 * records it with the key's device address, and returns -2 when no base_log could use the key exactly;
 * it synchronises its stream (the reference does too, context.h:110-113).  A PBS on a recorded key
 * evaluates its kernel's certified rounding bound with that max|G| at its base_log and
 * returns -2 when the bound reaches 1/2 (a hand-tuned kernel's key first falls back to the general
 * path's companion when the backend holds its standard key and the companion's bound holds).
 * concrete_hip_key_spectrum_max: the recorded max|G| of a converted key, -1 when none;
 * concrete_hip_key_error_bound: the certified bound of a PBS on that key at base_log, -1 when none. */
double concrete_hip_key_spectrum_max(const void *fourier_key);
double concrete_hip_key_error_bound(const void *fourier_key, uint32_t base_log);
/* bytes of the device (Fourier, exact-limb) bootstrapping key */
uint64_t concrete_hip_fourier_bsk_size_bytes(uint32_t input_lwe_dim, uint32_t glwe_dim, uint32_t level_count,
                                             uint32_t polynomial_size);
/* convert a standard u64 BSK (host pointer if src_is_device == 0, else device pointer) into a
 * caller-owned device buffer of concrete_hip_fourier_bsk_size_bytes() bytes */
int concrete_hip_convert_bsk(void *stream, uint32_t gpu_index, void *dest_fourier, const void *src,
                             int src_is_device, uint32_t input_lwe_dim, uint32_t glwe_dim, uint32_t level_count,
                             uint32_t polynomial_size);
/* Wide digits.  A (k, N, l) with a hand-tuned kernel (concrete_hip_bsk_format code 1, 2, 4 or 5)
 * accepts only digits that kernel keeps exact (k = 1, N = 1024: (k+1) l 2^logB <= 4096; l = 1 on the
 * 16-bit-limb kernels: logB <= 24; whole-digit levels: l 2^(logB-1) <= 2^15, or logB <= 16 on the
 * 13-bit-limb key of k = 4, N = 512, l = 2); wider ones run on the general path (pbs_generic.hip),
 * which needs the key in its own format.  Keys converted
 * through a keyset or cuda_convert_lwe_programmable_bootstrap_key_64 get that companion built from
 * their standard key on first use (concrete_hip_pbs, the memref / stream-emulator routes); a
 * caller holding its own key converts it with these two and calls concrete_hip_pbs_generic. */
uint64_t concrete_hip_generic_bsk_size_bytes(uint32_t input_lwe_dim, uint32_t glwe_dim, uint32_t level_count,
                                             uint32_t polynomial_size);
int concrete_hip_convert_bsk_generic(void *stream, uint32_t gpu_index, void *dest, const void *src,
                                     int src_is_device, uint32_t input_lwe_dim, uint32_t glwe_dim,
                                     uint32_t level_count, uint32_t polynomial_size);
int concrete_hip_pbs_generic(void *stream, uint32_t gpu_index, uint64_t *lwe_array_out,
                             const uint64_t *lwe_output_indexes, const uint64_t *lut_vector,
                             const uint64_t *lut_vector_indexes, const uint64_t *lwe_array_in,
                             const uint64_t *lwe_input_indexes, const void *generic_bsk, uint32_t lwe_dimension,
                             uint32_t glwe_dimension, uint32_t polynomial_size, uint32_t base_log,
                             uint32_t level_count, uint32_t num_samples, uint64_t *resid_bits);
/* batched PBS on a caller-owned Fourier key (no registry lookup); index arrays may be NULL
 * (identity for in/out, LUT 0 for lut).  resid_bits: optional device u64 receiving the f64
 * bits of max |x - round(x)| seen in the exact recombination (diagnostics; slower kernel). */
int concrete_hip_pbs(void *stream, uint32_t gpu_index, uint64_t *lwe_array_out, const uint64_t *lwe_output_indexes,
                     const uint64_t *lut_vector, const uint64_t *lut_vector_indexes, const uint64_t *lwe_array_in,
                     const uint64_t *lwe_input_indexes, const void *fourier_bsk, uint32_t lwe_dimension,
                     uint32_t glwe_dimension, uint32_t polynomial_size, uint32_t base_log, uint32_t level_count,
                     uint32_t num_samples, uint64_t *resid_bits);
/* batched keyswitch, status-returning variant */
int concrete_hip_keyswitch(void *stream, uint32_t gpu_index, uint64_t *lwe_array_out,
                           const uint64_t *lwe_output_indexes, const uint64_t *lwe_array_in,
                           const uint64_t *lwe_input_indexes, const uint64_t *ksk, uint32_t lwe_dimension_in,
                           uint32_t lwe_dimension_out, uint32_t base_log, uint32_t level_count,
                           uint32_t num_samples);
/* Fourier key registered for a `dest` of cuda_convert_lwe_programmable_bootstrap_key_64, or NULL */
const void *concrete_hip_lookup_bsk(const void *bootstrapping_key);
/* Release what the backend derived from device buffer `ptr` (a registered Fourier key whose `dest`
 * is ptr, the int8 key bytes the matrix-core keyswitch cached for a KSK at ptr — cached only for
 * buffers from cuda_malloc_async or a keyset) without freeing ptr itself; cuda_drop /
 * cuda_drop_async do this for every pointer, and cuda_memcpy_async_to_gpu for its destination.
 * Returns the number of cached key-byte entries released. */
int concrete_hip_release_device_buffer(const void *ptr);
/* LUT encoding on the device (compiler lib/Runtime/wrappers.cpp:388-450,
 * memref_encode_expand_lut_for_bootstrap, for num_luts rows at once): out is num_luts x out_size,
 * in is num_luts x in_size, device pointers; stream-ordered. */
int concrete_hip_encode_expand_lut_device(void *stream, uint32_t gpu_index, uint64_t *out, uint64_t out_size,
                                          const uint64_t *in, uint64_t in_size, uint64_t num_luts,
                                          uint32_t out_message_bits, int is_signed);
/* Trivial-GLWE accumulators on the device (wrappers.cpp:199-209): acc is num_luts x (k+1)N, row l =
 * k zero polynomials then LUT row l of luts (num_luts x N); device pointers; stream-ordered. */
int concrete_hip_build_accumulators(void *stream, uint32_t gpu_index, uint64_t *acc, const uint64_t *luts,
                                    uint64_t num_luts, uint32_t glwe_dim, uint32_t polynomial_size);
/* number of visible devices */
int concrete_hip_device_count(void);
/* Synchronise the device and return (and clear) the sticky status of every stream on it: 0 ok, -4
 * when a PBS kernel's wave synchronisation gave up after its spin bound since the last check (that
 * launch's outputs are wrong).  cuda_synchronize_device performs the same check and aborts. */
int concrete_hip_device_status(uint32_t gpu_index);
/* Stream-ordered status of one stream (round 5): waits for the work issued on `stream` (nothing
 * else), then returns (and clears) the status of the PBS launches made on that stream since its last
 * check: 0 ok, -4 when one of them gave up a wave synchronisation (its outputs are wrong).  Status
 * words are per (device, stream), so concurrent calls on other streams are never blamed. */
int concrete_hip_stream_status(void *stream, uint32_t gpu_index);
/* Spin bound (LDS-counter polls) of the PBS kernels' wave synchronisation for later launches;
 * 0 restores the default (2^22).  Test hook: a tiny bound forces the timeout path. */
void concrete_hip_set_spin_limit(uint32_t polls);
/* The same bound for launches issued by the calling host thread only (0: the process-wide bound).
 * Test hook: forces the timeout path on one of several concurrent calls. */
void concrete_hip_set_thread_spin_limit(uint32_t polls);
/* How a cfg2-shaped call (k = 1, N = 1024, l = 3) of num_samples ciphertexts is split on a device of
 * `cus` compute units (round 6): parts[0..2] = ciphertexts run on the pair kernel (4 per CU), the
 * six-wave kernel at 2 per CU and at 1 per CU, in that launch order; returns the estimated time in
 * 1/100 ms per round at n = 630 (concrete_amd/csrc/pbs1024_plan.hpp). */
uint64_t concrete_hip_pbs1024_plan(uint64_t num_samples, uint32_t cus, uint32_t *parts);
/* Status slots held by live streams of the device (round 6): a stream gets a slot on its first PBS
 * launch and returns it when it is destroyed (cuda_destroy_stream, the runtime's own streams), so a
 * caller that creates and destroys a stream per call (wrappers.cpp:129/160) never exhausts them. */
uint32_t concrete_hip_status_slots_in_use(uint32_t gpu_index);
/* Test hook: at most `slots` status slots per device (0 restores 4096); a stream arriving while all
 * are taken shares slot 0, whose reads still report that stream's launches. */
void concrete_hip_set_status_slot_cap(uint32_t slots);

/* ------------------------------------------------------------------------------------------
 * Part 3: client-side helpers (host code; synthetic workloads and LUT encoding).
 * INSECURE — FOR TESTS AND BENCHMARKS ONLY: keys, masks and noise come from xoshiro256** seeded
 * with the caller's 64-bit seed (Box-Muller Gaussians), not from a CSPRNG; reusing a seed reuses
 * the encryption masks.  Real key material comes from the reference's client (concrete-csprng).
 * Mirrors the
 * concrete-cpu client ABI (backends/concrete-cpu/implementation/include/concrete-cpu.h:
 * concrete_cpu_init_secret_key_u64, concrete_cpu_encrypt_lwe_ciphertext_u64,
 * concrete_cpu_init_lwe_bootstrap_key_u64, concrete_cpu_init_lwe_keyswitch_key_u64) and the
 * runtime's LUT expansion (compiler lib/Runtime/wrappers.cpp:388-450).  Deterministic per seed.
 * ------------------------------------------------------------------------------------------ */
double concrete_hip_secure_log2_std(uint64_t glwe_dim, uint64_t poly_size);
void concrete_hip_keygen_binary(uint64_t *sk, uint64_t len, uint64_t seed);
void concrete_hip_lwe_encrypt_batch(const uint64_t *sk, uint64_t *out, const uint64_t *plaintexts, uint64_t count,
                                    uint64_t n, double std_torus, uint64_t seed);
uint64_t concrete_hip_lwe_decrypt(const uint64_t *sk, const uint64_t *ct, uint64_t n);
void concrete_hip_bsk_generate(uint64_t *bsk, const uint64_t *lwe_sk, const uint64_t *glwe_sk, uint64_t n,
                               uint64_t k, uint64_t N, uint64_t l, uint64_t logB, double std_torus, uint64_t seed);
void concrete_hip_ksk_generate(uint64_t *ksk, const uint64_t *sk_in, const uint64_t *sk_out, uint64_t n_in,
                               uint64_t n_out, uint64_t l, uint64_t logB, double std_torus, uint64_t seed);
void concrete_hip_encode_expand_lut(uint64_t *out, uint64_t out_size, const uint64_t *in, uint64_t in_size,
                                    uint32_t out_message_bits, int is_signed);

/* ------------------------------------------------------------------------------------------
 * Part 4: circuit-facing runtime glue (SURVEY.md §8b layer B2).  Mirrors of the runtime's
 * memref wrappers (compiler include/concretelang/Runtime/wrappers.h:240-300, implementation
 * lib/Runtime/wrappers.cpp:88-363) over an opaque keyset handle instead of the C++
 * RuntimeContext (include/concretelang/Runtime/context.h:42-145): MLIR memref descriptors
 * expanded as (allocated, aligned, offset, sizes..., strides...), host memory in and out, the
 * same shape assertions (violations abort), trivial GLWE accumulators built from the LUT
 * (wrappers.cpp:199-209), one LUT per sample for the mapped form (wrappers.cpp:317-325).
 * Differences by design: device keys are converted once per keyset and device and reused
 * across calls (the reference re-converts per RuntimeContext, ServerLib.cpp:579); a keyset may
 * list several devices, across which every batched call is sharded in contiguous slices
 * (the reference's direct route is "TODO: Multi GPU", wrappers.cpp:176-177), the converted key
 * reaching the other devices by peer copy.
 * ------------------------------------------------------------------------------------------ */
typedef struct concrete_hip_keyset concrete_hip_keyset;
concrete_hip_keyset *concrete_hip_keyset_create(void);
void concrete_hip_keyset_destroy(concrete_hip_keyset *ks);
/* standard-domain keys (host buffers, copied): BSK [n][l][k+1][k+1][N], KSK [n_in][l][n_out+1] */
int concrete_hip_keyset_add_bsk(concrete_hip_keyset *ks, uint32_t bsk_index, const uint64_t *bsk, uint32_t input_lwe_dim,
                                uint32_t glwe_dim, uint32_t level, uint32_t base_log, uint32_t poly_size);
int concrete_hip_keyset_add_ksk(concrete_hip_keyset *ks, uint32_t ksk_index, const uint64_t *ksk, uint32_t level,
                                uint32_t base_log, uint32_t input_lwe_dim, uint32_t output_lwe_dim);
/* devices the batched calls shard across (default: device 0); entries may repeat.  Every slice of
 * a call runs on its own host thread, stream and cached device buffers. */
int concrete_hip_keyset_set_devices(concrete_hip_keyset *ks, const uint32_t *devices, uint32_t count);
/* Diagnostics: record HIP events around every slice of the following calls ... */
void concrete_hip_keyset_set_timing(concrete_hip_keyset *ks, int enable);
/* ... and read them for every call since timing was enabled, in completion order: 6 doubles per
 * slice (device, then ms since timing was enabled on that device: slice start, inputs copied
 * (kernel issue), kernel done, outputs copied, then the slice's sample count); returns the number
 * of slices (copies at most max_slices).  Concurrent calls on one keyset run on slot sets of their
 * own, so their slices share this time axis (round 4). */
uint32_t concrete_hip_keyset_timeline(concrete_hip_keyset *ks, double *out, uint32_t max_slices);

/* The runtime's context pointer (mlir::concretelang::RuntimeContext *, context.h:42-154) is what
 * the circuit passes to memref_*_cuda_u64 and to the stream emulator's KS / PBS processes.  The
 * backend resolves it to a keyset: a pointer bound with concrete_hip_context_bind (NULL keyset
 * unbinds), else the resolver's answer (cached per context), else the pointer itself when it is a
 * live keyset handle.  An unresolvable context aborts (reference failure behaviour). */
int concrete_hip_context_bind(const void *runtime_context, concrete_hip_keyset *ks);
typedef concrete_hip_keyset *(*concrete_hip_context_resolver)(const void *runtime_context, void *user);
void concrete_hip_set_context_resolver(concrete_hip_context_resolver fn, void *user);

void memref_keyswitch_lwe_hip_u64(uint64_t *out_allocated, uint64_t *out_aligned, uint64_t out_offset,
                                  uint64_t out_size, uint64_t out_stride, uint64_t *ct0_allocated,
                                  uint64_t *ct0_aligned, uint64_t ct0_offset, uint64_t ct0_size, uint64_t ct0_stride,
                                  uint32_t level, uint32_t base_log, uint32_t input_lwe_dim,
                                  uint32_t output_lwe_dim, uint32_t ksk_index, concrete_hip_keyset *context);
void memref_bootstrap_lwe_hip_u64(uint64_t *out_allocated, uint64_t *out_aligned, uint64_t out_offset,
                                  uint64_t out_size, uint64_t out_stride, uint64_t *ct0_allocated,
                                  uint64_t *ct0_aligned, uint64_t ct0_offset, uint64_t ct0_size, uint64_t ct0_stride,
                                  uint64_t *tlu_allocated, uint64_t *tlu_aligned, uint64_t tlu_offset,
                                  uint64_t tlu_size, uint64_t tlu_stride, uint32_t input_lwe_dim, uint32_t poly_size,
                                  uint32_t level, uint32_t base_log, uint32_t glwe_dim, uint32_t bsk_index,
                                  concrete_hip_keyset *context);
void memref_batched_keyswitch_lwe_hip_u64(uint64_t *out_allocated, uint64_t *out_aligned, uint64_t out_offset,
                                          uint64_t out_size0, uint64_t out_size1, uint64_t out_stride0,
                                          uint64_t out_stride1, uint64_t *ct0_allocated, uint64_t *ct0_aligned,
                                          uint64_t ct0_offset, uint64_t ct0_size0, uint64_t ct0_size1,
                                          uint64_t ct0_stride0, uint64_t ct0_stride1, uint32_t level,
                                          uint32_t base_log, uint32_t input_lwe_dim, uint32_t output_lwe_dim,
                                          uint32_t ksk_index, concrete_hip_keyset *context);
void memref_batched_bootstrap_lwe_hip_u64(uint64_t *out_allocated, uint64_t *out_aligned, uint64_t out_offset,
                                          uint64_t out_size0, uint64_t out_size1, uint64_t out_stride0,
                                          uint64_t out_stride1, uint64_t *ct0_allocated, uint64_t *ct0_aligned,
                                          uint64_t ct0_offset, uint64_t ct0_size0, uint64_t ct0_size1,
                                          uint64_t ct0_stride0, uint64_t ct0_stride1, uint64_t *tlu_allocated,
                                          uint64_t *tlu_aligned, uint64_t tlu_offset, uint64_t tlu_size,
                                          uint64_t tlu_stride, uint32_t input_lwe_dim, uint32_t poly_size,
                                          uint32_t level, uint32_t base_log, uint32_t glwe_dim, uint32_t bsk_index,
                                          concrete_hip_keyset *context);
void memref_batched_mapped_bootstrap_lwe_hip_u64(
    uint64_t *out_allocated, uint64_t *out_aligned, uint64_t out_offset, uint64_t out_size0, uint64_t out_size1,
    uint64_t out_stride0, uint64_t out_stride1, uint64_t *ct0_allocated, uint64_t *ct0_aligned, uint64_t ct0_offset,
    uint64_t ct0_size0, uint64_t ct0_size1, uint64_t ct0_stride0, uint64_t ct0_stride1, uint64_t *tlu_allocated,
    uint64_t *tlu_aligned, uint64_t tlu_offset, uint64_t tlu_size0, uint64_t tlu_size1, uint64_t tlu_stride0,
    uint64_t tlu_stride1, uint32_t input_lwe_dim, uint32_t poly_size, uint32_t level, uint32_t base_log,
    uint32_t glwe_dim, uint32_t bsk_index, concrete_hip_keyset *context);

/* The direct GPU route under the reference's own names and argument lists
 * (compiler include/concretelang/Runtime/wrappers.h:246-300, lib/Runtime/wrappers.cpp:70-363):
 * `context` is the caller's runtime context, resolved as described above.  Same semantics as the
 * memref_*_hip_u64 forms (every batched call sharded over the keyset's devices). */
void memref_keyswitch_lwe_cuda_u64(uint64_t *out_allocated, uint64_t *out_aligned, uint64_t out_offset,
                                   uint64_t out_size, uint64_t out_stride, uint64_t *ct0_allocated,
                                   uint64_t *ct0_aligned, uint64_t ct0_offset, uint64_t ct0_size,
                                   uint64_t ct0_stride, uint32_t level, uint32_t base_log, uint32_t input_lwe_dim,
                                   uint32_t output_lwe_dim, uint32_t ksk_index, void *context);
void memref_bootstrap_lwe_cuda_u64(uint64_t *out_allocated, uint64_t *out_aligned, uint64_t out_offset,
                                   uint64_t out_size, uint64_t out_stride, uint64_t *ct0_allocated,
                                   uint64_t *ct0_aligned, uint64_t ct0_offset, uint64_t ct0_size,
                                   uint64_t ct0_stride, uint64_t *tlu_allocated, uint64_t *tlu_aligned,
                                   uint64_t tlu_offset, uint64_t tlu_size, uint64_t tlu_stride,
                                   uint32_t input_lwe_dim, uint32_t poly_size, uint32_t level, uint32_t base_log,
                                   uint32_t glwe_dim, uint32_t bsk_index, void *context);
void memref_batched_keyswitch_lwe_cuda_u64(uint64_t *out_allocated, uint64_t *out_aligned, uint64_t out_offset,
                                           uint64_t out_size0, uint64_t out_size1, uint64_t out_stride0,
                                           uint64_t out_stride1, uint64_t *ct0_allocated, uint64_t *ct0_aligned,
                                           uint64_t ct0_offset, uint64_t ct0_size0, uint64_t ct0_size1,
                                           uint64_t ct0_stride0, uint64_t ct0_stride1, uint32_t level,
                                           uint32_t base_log, uint32_t input_lwe_dim, uint32_t output_lwe_dim,
                                           uint32_t ksk_index, void *context);
void memref_batched_bootstrap_lwe_cuda_u64(uint64_t *out_allocated, uint64_t *out_aligned, uint64_t out_offset,
                                           uint64_t out_size0, uint64_t out_size1, uint64_t out_stride0,
                                           uint64_t out_stride1, uint64_t *ct0_allocated, uint64_t *ct0_aligned,
                                           uint64_t ct0_offset, uint64_t ct0_size0, uint64_t ct0_size1,
                                           uint64_t ct0_stride0, uint64_t ct0_stride1, uint64_t *tlu_allocated,
                                           uint64_t *tlu_aligned, uint64_t tlu_offset, uint64_t tlu_size,
                                           uint64_t tlu_stride, uint32_t input_lwe_dim, uint32_t poly_size,
                                           uint32_t level, uint32_t base_log, uint32_t glwe_dim, uint32_t bsk_index,
                                           void *context);
void memref_batched_mapped_bootstrap_lwe_cuda_u64(
    uint64_t *out_allocated, uint64_t *out_aligned, uint64_t out_offset, uint64_t out_size0, uint64_t out_size1,
    uint64_t out_stride0, uint64_t out_stride1, uint64_t *ct0_allocated, uint64_t *ct0_aligned, uint64_t ct0_offset,
    uint64_t ct0_size0, uint64_t ct0_size1, uint64_t ct0_stride0, uint64_t ct0_stride1, uint64_t *tlu_allocated,
    uint64_t *tlu_aligned, uint64_t tlu_offset, uint64_t tlu_size0, uint64_t tlu_size1, uint64_t tlu_stride0,
    uint64_t tlu_stride1, uint32_t input_lwe_dim, uint32_t poly_size, uint32_t level, uint32_t base_log,
    uint32_t glwe_dim, uint32_t bsk_index, void *context);

/* ------------------------------------------------------------------------------------------
 * Part 5: the SDFG stream emulator — the default GPU route of a circuit compiled with SDFG
 * extraction (compiler include/concretelang/Runtime/stream_emulator_api.h:30-106; reference
 * implementation lib/Runtime/GPUDFG.cpp:1467-1799; call sequence emitted by
 * lib/Conversion/SDFGToStreamEmulator/SDFGToStreamEmulator.cpp:25-73: init, make streams, make
 * processes, run, put inputs, get outputs, delete).  Same names and argument lists; `stype` is the
 * reference's `stream_type` enum (passed as int; values below).  A get evaluates the processes its
 * stream depends on whose inputs changed since their last evaluation, the whole subgraph resident
 * on the devices (sdfg.hip).  Devices: CONCRETE_HIP_SDFG_DEVICES ("0,0,1", repeats allowed), else
 * SDFG_NUM_GPUS, else all visible devices.  `context` of KS / PBS processes: as in Part 4.
 * ------------------------------------------------------------------------------------------ */
enum {
  CONCRETE_HIP_TS_STREAM_TYPE_X86_TO_TOPO_LSAP = 0,
  CONCRETE_HIP_TS_STREAM_TYPE_TOPO_TO_TOPO_LSAP = 1,
  CONCRETE_HIP_TS_STREAM_TYPE_TOPO_TO_X86_LSAP = 2,
  CONCRETE_HIP_TS_STREAM_TYPE_TOPO_TO_BOTH = 3,
  CONCRETE_HIP_TS_STREAM_TYPE_X86_TO_X86_LSAP = 4
};
void *stream_emulator_init(void);
void stream_emulator_run(void *dfg);
void stream_emulator_delete(void *dfg);
void stream_emulator_make_memref_add_lwe_ciphertexts_u64_process(void *dfg, void *sin1, void *sin2, void *sout);
void stream_emulator_make_memref_add_plaintext_lwe_ciphertext_u64_process(void *dfg, void *sin1, void *sin2,
                                                                          void *sout);
void stream_emulator_make_memref_mul_cleartext_lwe_ciphertext_u64_process(void *dfg, void *sin1, void *sin2,
                                                                          void *sout);
void stream_emulator_make_memref_negate_lwe_ciphertext_u64_process(void *dfg, void *sin1, void *sout);
void stream_emulator_make_memref_keyswitch_lwe_u64_process(void *dfg, void *sin1, void *sout, uint32_t level,
                                                           uint32_t base_log, uint32_t input_lwe_dim,
                                                           uint32_t output_lwe_dim, uint32_t output_size,
                                                           uint32_t ksk_index, void *context);
void stream_emulator_make_memref_bootstrap_lwe_u64_process(void *dfg, void *sin1, void *sin2, void *sout,
                                                           uint32_t input_lwe_dim, uint32_t poly_size,
                                                           uint32_t level, uint32_t base_log, uint32_t glwe_dim,
                                                           uint32_t output_size, uint32_t bsk_index, void *context);
void stream_emulator_make_memref_batched_add_lwe_ciphertexts_u64_process(void *dfg, void *sin1, void *sin2,
                                                                         void *sout);
void stream_emulator_make_memref_batched_add_plaintext_lwe_ciphertext_u64_process(void *dfg, void *sin1, void *sin2,
                                                                                  void *sout);
void stream_emulator_make_memref_batched_add_plaintext_cst_lwe_ciphertext_u64_process(void *dfg, void *sin1,
                                                                                      void *sin2, void *sout);
void stream_emulator_make_memref_batched_mul_cleartext_lwe_ciphertext_u64_process(void *dfg, void *sin1, void *sin2,
                                                                                  void *sout);
void stream_emulator_make_memref_batched_mul_cleartext_cst_lwe_ciphertext_u64_process(void *dfg, void *sin1,
                                                                                      void *sin2, void *sout);
void stream_emulator_make_memref_batched_negate_lwe_ciphertext_u64_process(void *dfg, void *sin1, void *sout);
void stream_emulator_make_memref_batched_keyswitch_lwe_u64_process(void *dfg, void *sin1, void *sout, uint32_t level,
                                                                   uint32_t base_log, uint32_t input_lwe_dim,
                                                                   uint32_t output_lwe_dim, uint32_t output_size,
                                                                   uint32_t ksk_index, void *context);
void stream_emulator_make_memref_batched_bootstrap_lwe_u64_process(void *dfg, void *sin1, void *sin2, void *sout,
                                                                   uint32_t input_lwe_dim, uint32_t poly_size,
                                                                   uint32_t level, uint32_t base_log,
                                                                   uint32_t glwe_dim, uint32_t output_size,
                                                                   uint32_t bsk_index, void *context);
void stream_emulator_make_memref_batched_mapped_bootstrap_lwe_u64_process(void *dfg, void *sin1, void *sin2,
                                                                          void *sout, uint32_t input_lwe_dim,
                                                                          uint32_t poly_size, uint32_t level,
                                                                          uint32_t base_log, uint32_t glwe_dim,
                                                                          uint32_t output_size, uint32_t bsk_index,
                                                                          void *context);
void *stream_emulator_make_uint64_stream(const char *name, int stype);
void stream_emulator_put_uint64(void *stream, uint64_t e);
uint64_t stream_emulator_get_uint64(void *stream);
void *stream_emulator_make_memref_stream(const char *name, int stype);
void stream_emulator_put_memref(void *stream, uint64_t *allocated, uint64_t *aligned, uint64_t offset, uint64_t size,
                                uint64_t stride, uint64_t data_ownership);
void stream_emulator_get_memref(void *stream, uint64_t *out_allocated, uint64_t *out_aligned, uint64_t out_offset,
                                uint64_t out_size, uint64_t out_stride);
void *stream_emulator_make_memref_batch_stream(const char *name, int stype);
void stream_emulator_put_memref_batch(void *stream, uint64_t *allocated, uint64_t *aligned, uint64_t offset,
                                      uint64_t size0, uint64_t size1, uint64_t stride0, uint64_t stride1,
                                      uint64_t data_ownership);
void stream_emulator_get_memref_batch(void *stream, uint64_t *out_allocated, uint64_t *out_aligned,
                                      uint64_t out_offset, uint64_t out_size0, uint64_t out_size1,
                                      uint64_t out_stride0, uint64_t out_stride1);

/* ------------------------------------------------------------------------------------------
 * Part 6: key wire-format import (concrete_amd/csrc/keyio.cpp).
 * Reads the evaluation keys of a serialized concrete keyset — the Cap'n Proto messages
 * `ServerKeyset.serialize()` / `Keyset.serialize()` write (capnp::writeMessage, unpacked framing,
 * include/concretelang/Common/Protocol.h:158-175; schema tools/concrete-protocol/src/
 * concrete-protocol.capnp:149-297) — and registers them in a runtime keyset under the indexes the
 * runtime context uses (list position, lib/Runtime/context.cpp:36-94), replacing the reference's
 * ServerKeyset::fromProto + LweBootstrapKey/LweKeyswitchKey::fromProto (lib/Common/Keys.cpp:142-163,
 * 262-283).  Payloads: List(Data) blobs concatenated (Protocol.h:349-372).  Seeded keys
 * (Compression::SEED, Keys.cpp:193-218) are expanded by concrete-cpu's own decompressors, which the
 * caller installs (the runtime already links concrete-cpu); without them a seeded key is refused.
 * Only 64-bit keys over the native modulus are accepted (the PBS / KS kernels' torus).
 * Returns 0, or < 0 with concrete_hip_last_error() set (malformed message, size mismatch, ...).
 * ------------------------------------------------------------------------------------------ */
typedef struct concrete_hip_server_keyset concrete_hip_server_keyset;
enum {
  CONCRETE_HIP_ROOT_SERVER_KEYSET = 0,    /* ServerKeyset (ServerKeyset.serialize()) */
  CONCRETE_HIP_ROOT_KEYSET = 1,           /* Keyset: its `server` part (Keyset.serialize()) */
  CONCRETE_HIP_ROOT_LWE_BOOTSTRAP_KEY = 2, /* one LweBootstrapKey */
  CONCRETE_HIP_ROOT_LWE_KEYSWITCH_KEY = 3  /* one LweKeyswitchKey */
};
typedef struct concrete_hip_key_info {
  uint32_t id, input_id, output_id;          /* LweBootstrapKeyInfo / LweKeyswitchKeyInfo */
  uint32_t level_count, base_log;
  uint32_t glwe_dim, poly_size;              /* bootstrap keys only */
  uint32_t input_lwe_dim, output_lwe_dim;    /* bootstrap keys: output = glwe_dim * poly_size */
  uint32_t integer_precision;
  uint32_t key_type;                         /* KeyType: 0 binary, 1 ternary */
  uint32_t compression;                      /* Compression: 0 none, 1 seed, 2 paillier */
  uint32_t modulus_kind, modulus_value;      /* Modulus union: 0 native, 1 power of two, 2 integer */
  double variance;
  uint64_t payload_words;                    /* u64 words on the wire */
  uint64_t key_words;                        /* u64 words of the standard-domain key */
} concrete_hip_key_info;
int concrete_hip_server_keyset_deserialize(const void *bytes, uint64_t size, uint32_t root,
                                           concrete_hip_server_keyset **out);
int concrete_hip_server_keyset_load_file(const char *path, uint32_t root, concrete_hip_server_keyset **out);
void concrete_hip_server_keyset_destroy(concrete_hip_server_keyset *sk);
uint32_t concrete_hip_server_keyset_bsk_count(const concrete_hip_server_keyset *sk);
uint32_t concrete_hip_server_keyset_ksk_count(const concrete_hip_server_keyset *sk);
int concrete_hip_server_keyset_bsk_info(const concrete_hip_server_keyset *sk, uint32_t index,
                                        concrete_hip_key_info *out);
int concrete_hip_server_keyset_ksk_info(const concrete_hip_server_keyset *sk, uint32_t index,
                                        concrete_hip_key_info *out);
/* the standard-domain key (BSK [n][l][k+1][k+1][N], KSK [n_in][l][n_out+1]); dst holds >= key_words */
/* Level order of evaluation key `index` (is_bsk: bootstrap, else keyswitch), found when it was last
 * read (read_bsk / read_ksk / keyset_add_server_keyset) against the client secret keys a Keyset
 * message carries: one GGSW / keyswitch row per level is decrypted.  A key stored in the reversed
 * level order is re-ordered on read; one that decrypts in neither order is refused (round 4). */
enum {
  CONCRETE_HIP_LEVEL_ORDER_UNCHECKED = 0,   /* no client keys (ServerKeyset), one level, or not read yet */
  CONCRETE_HIP_LEVEL_ORDER_AS_EXPECTED = 1, /* the order the standard layouts assume */
  CONCRETE_HIP_LEVEL_ORDER_REVERSED = 2     /* stored reversed: re-ordered on read */
};
int concrete_hip_server_keyset_level_order(const concrete_hip_server_keyset *sk, int is_bsk, uint32_t index);
/* client secret keys read from a Keyset message (0 for the other roots) */
uint32_t concrete_hip_server_keyset_secret_count(const concrete_hip_server_keyset *sk);
int concrete_hip_server_keyset_read_bsk(const concrete_hip_server_keyset *sk, uint32_t index, uint64_t *dst,
                                        uint64_t dst_words);
int concrete_hip_server_keyset_read_ksk(const concrete_hip_server_keyset *sk, uint32_t index, uint64_t *dst,
                                        uint64_t dst_words);
/* every bootstrap key i -> bsk_index i, every keyswitch key i -> ksk_index i */
int concrete_hip_keyset_add_server_keyset(concrete_hip_keyset *ks, const concrete_hip_server_keyset *sk);
/* Same layout and calling convention as concrete-cpu's Uint128 and its decompressors
 * (backends/concrete-cpu/implementation/include/concrete-cpu.h:49-51,185-207), so
 * concrete_cpu_decompress_seeded_lwe_{bootstrap,keyswitch}_key_u64 install directly.  The last
 * argument is concrete-cpu's Parallelism (1 = Rayon, what Keys.cpp:209-211 passes). */
typedef struct concrete_hip_uint128 {
  uint8_t little_endian_bytes[16];
} concrete_hip_uint128;
typedef void (*concrete_hip_bsk_decompressor)(uint64_t *lwe_bsk, const uint64_t *seeded_lwe_bsk,
                                              size_t input_lwe_dimension, size_t output_polynomial_size,
                                              size_t output_glwe_dimension, size_t decomposition_level_count,
                                              size_t decomposition_base_log, concrete_hip_uint128 compression_seed,
                                              uint32_t parallelism);
typedef void (*concrete_hip_ksk_decompressor)(uint64_t *lwe_ksk, const uint64_t *seeded_lwe_ksk,
                                              size_t input_lwe_dimension, size_t output_lwe_dimension,
                                              size_t decomposition_level_count, size_t decomposition_base_log,
                                              concrete_hip_uint128 compression_seed, uint32_t parallelism);
void concrete_hip_set_seeded_key_decompressors(concrete_hip_bsk_decompressor bsk, concrete_hip_ksk_decompressor ksk);

#ifdef __cplusplus
}
#endif
#endif /* CONCRETE_HIP_H */
