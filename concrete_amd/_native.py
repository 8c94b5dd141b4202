"""ctypes binding of libconcrete_hip.so (the C ABI declared in include/concrete_hip.h).

The shared library is built in-tree (``make -C concrete_amd/csrc``); there is no fallback:
if it is missing or fails to load, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
# CONCRETE_HIP_LIB: alternative build of the same ABI (kernel experiments, tools/variant.sh)
LIB_PATH = os.environ.get("CONCRETE_HIP_LIB") or os.path.join(_HERE, "libconcrete_hip.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "concrete_hip.h")

u32, u64, i32, vp, dbl = C.c_uint32, C.c_uint64, C.c_int, C.c_void_p, C.c_double
u64p = C.POINTER(C.c_uint64)

# name -> (restype, argtypes)
SIGNATURES = {
    "cuda_create_stream": (vp, [u32]),
    "cuda_destroy_stream": (None, [vp, u32]),
    "cuda_malloc_async": (vp, [u64, vp, u32]),
    "cuda_memcpy_async_to_gpu": (None, [vp, vp, u64, vp, u32]),
    "cuda_memcpy_async_to_cpu": (None, [vp, vp, u64, vp, u32]),
    "cuda_drop": (None, [vp, u32]),
    "cuda_drop_async": (None, [vp, vp, u32]),
    "cuda_synchronize_device": (None, [u32]),
    "cuda_convert_lwe_programmable_bootstrap_key_64": (None, [vp, u32, vp, vp, u32, u32, u32, u32]),
    "scratch_cuda_programmable_bootstrap_64": (None, [vp, u32, C.POINTER(vp), u32, u32, u32, u32, C.c_bool]),
    "cleanup_cuda_programmable_bootstrap": (None, [vp, u32, C.POINTER(vp)]),
    "cuda_programmable_bootstrap_lwe_ciphertext_vector_64": (
        None, [vp, u32, vp, vp, vp, vp, vp, vp, vp, vp, u32, u32, u32, u32, u32, u32, u32, u32]),
    "cuda_keyswitch_lwe_ciphertext_vector_64": (None, [vp, u32, vp, vp, vp, vp, vp, u32, u32, u32, u32, u32]),
    "cuda_add_lwe_ciphertext_vector_64": (None, [vp, u32, vp, vp, vp, u32, u32]),
    "cuda_add_lwe_ciphertext_vector_plaintext_vector_64": (None, [vp, u32, vp, vp, vp, u32, u32]),
    "cuda_mult_lwe_ciphertext_vector_cleartext_vector_64": (None, [vp, u32, vp, vp, vp, u32, u32]),
    "cuda_negate_lwe_ciphertext_vector_64": (None, [vp, u32, vp, vp, u32, u32]),
    "concrete_hip_abi_version": (u32, []),
    "concrete_hip_last_error": (C.c_char_p, []),
    "concrete_hip_pbs_supported": (i32, [u32, u32, u32, u32]),
    "concrete_hip_keyswitch_supported": (i32, [u32, u32, u32, u32]),
    "concrete_hip_server_keyset_level_order": (i32, [vp, i32, u32]),
    "concrete_hip_server_keyset_secret_count": (u32, [vp]),
    "concrete_hip_bsk_limbs": (u32, [u32, u32, u32]),
    "concrete_hip_bsk_format": (C.c_int, [u32, u32, u32, C.POINTER(u32), C.POINTER(u32)]),
    "concrete_hip_generic_error_bound": (C.c_double, [u32, u32, u32, u32, C.c_double]),
    "concrete_hip_fourier_bsk_size_bytes": (u64, [u32, u32, u32, u32]),
    "concrete_hip_convert_bsk": (i32, [vp, u32, vp, vp, i32, u32, u32, u32, u32]),
    "concrete_hip_pbs": (i32, [vp, u32, vp, vp, vp, vp, vp, vp, vp, u32, u32, u32, u32, u32, u32, vp]),
    "concrete_hip_keyswitch": (i32, [vp, u32, vp, vp, vp, vp, vp, u32, u32, u32, u32, u32]),
    "concrete_hip_lookup_bsk": (vp, [vp]),
    "concrete_hip_generic_bsk_size_bytes": (u64, [u32, u32, u32, u32]),
    "concrete_hip_convert_bsk_generic": (i32, [vp, u32, vp, vp, i32, u32, u32, u32, u32]),
    "concrete_hip_pbs_generic": (i32, [vp, u32, vp, vp, vp, vp, vp, vp, vp, u32, u32, u32, u32, u32, u32, vp]),
    "concrete_hip_device_count": (i32, []),
    "concrete_hip_device_status": (i32, [u32]),
    "concrete_hip_set_spin_limit": (None, [u32]),
    "concrete_hip_stream_status": (i32, [vp, u32]),
    "concrete_hip_set_thread_spin_limit": (None, [u32]),
    "concrete_hip_status_slots_in_use": (u32, [u32]),
    "concrete_hip_set_status_slot_cap": (None, [u32]),
    "concrete_hip_key_spectrum_max": (C.c_double, [vp]),
    "concrete_hip_pbs1024_plan": (u64, [u64, u32, C.POINTER(u32)]),
    "concrete_hip_key_error_bound": (C.c_double, [vp, u32]),
    "concrete_hip_secure_log2_std": (dbl, [u64, u64]),
    "concrete_hip_keygen_binary": (None, [vp, u64, u64]),
    "concrete_hip_lwe_encrypt_batch": (None, [vp, vp, vp, u64, u64, dbl, u64]),
    "concrete_hip_lwe_decrypt": (u64, [vp, vp, u64]),
    "concrete_hip_bsk_generate": (None, [vp, vp, vp, u64, u64, u64, u64, u64, dbl, u64]),
    "concrete_hip_ksk_generate": (None, [vp, vp, vp, u64, u64, u64, u64, dbl, u64]),
    "concrete_hip_encode_expand_lut": (None, [vp, u64, vp, u64, u32, i32]),
    # Part 4: runtime glue (memref descriptors expanded: allocated, aligned, offset, sizes, strides)
    "concrete_hip_keyset_create": (vp, []),
    "concrete_hip_keyset_destroy": (None, [vp]),
    "concrete_hip_keyset_add_bsk": (i32, [vp, u32, vp, u32, u32, u32, u32, u32]),
    "concrete_hip_keyset_add_ksk": (i32, [vp, u32, vp, u32, u32, u32, u32]),
    "concrete_hip_keyset_set_devices": (i32, [vp, vp, u32]),
    "memref_keyswitch_lwe_hip_u64": (None, [vp, vp, u64, u64, u64, vp, vp, u64, u64, u64, u32, u32, u32, u32, u32, vp]),
    "memref_bootstrap_lwe_hip_u64": (None, [vp, vp, u64, u64, u64, vp, vp, u64, u64, u64, vp, vp, u64, u64, u64,
                                            u32, u32, u32, u32, u32, u32, vp]),
    "memref_batched_keyswitch_lwe_hip_u64": (None, [vp, vp, u64, u64, u64, u64, u64, vp, vp, u64, u64, u64, u64, u64,
                                                    u32, u32, u32, u32, u32, vp]),
    "memref_batched_bootstrap_lwe_hip_u64": (None, [vp, vp, u64, u64, u64, u64, u64, vp, vp, u64, u64, u64, u64, u64,
                                                    vp, vp, u64, u64, u64, u32, u32, u32, u32, u32, u32, vp]),
    "memref_batched_mapped_bootstrap_lwe_hip_u64": (None, [vp, vp, u64, u64, u64, u64, u64, vp, vp, u64, u64, u64, u64,
                                                           u64, vp, vp, u64, u64, u64, u64, u64, u32, u32, u32, u32,
                                                           u32, u32, vp]),
    "concrete_hip_keyset_set_timing": (None, [vp, i32]),
    "concrete_hip_keyset_timeline": (u32, [vp, vp, u32]),
    "concrete_hip_context_bind": (i32, [vp, vp]),
    "concrete_hip_set_context_resolver": (None, [vp, vp]),
    "concrete_hip_release_device_buffer": (i32, [vp]),
    "concrete_hip_encode_expand_lut_device": (i32, [vp, u32, vp, u64, vp, u64, u64, u32, i32]),
    "concrete_hip_build_accumulators": (i32, [vp, u32, vp, vp, u64, u32, u32]),
    # the reference's names, context pointer last (wrappers.h:246-300)
    "memref_keyswitch_lwe_cuda_u64": (None, [vp, vp, u64, u64, u64, vp, vp, u64, u64, u64, u32, u32, u32, u32, u32, vp]),
    "memref_bootstrap_lwe_cuda_u64": (None, [vp, vp, u64, u64, u64, vp, vp, u64, u64, u64, vp, vp, u64, u64, u64,
                                             u32, u32, u32, u32, u32, u32, vp]),
    "memref_batched_keyswitch_lwe_cuda_u64": (None, [vp, vp, u64, u64, u64, u64, u64, vp, vp, u64, u64, u64, u64, u64,
                                                     u32, u32, u32, u32, u32, vp]),
    "memref_batched_bootstrap_lwe_cuda_u64": (None, [vp, vp, u64, u64, u64, u64, u64, vp, vp, u64, u64, u64, u64, u64,
                                                     vp, vp, u64, u64, u64, u32, u32, u32, u32, u32, u32, vp]),
    "memref_batched_mapped_bootstrap_lwe_cuda_u64": (None, [vp, vp, u64, u64, u64, u64, u64, vp, vp, u64, u64, u64,
                                                            u64, u64, vp, vp, u64, u64, u64, u64, u64, u32, u32, u32,
                                                            u32, u32, u32, vp]),
    # Part 5: stream emulator (stream_emulator_api.h:30-106)
    "stream_emulator_init": (vp, []),
    "stream_emulator_run": (None, [vp]),
    "stream_emulator_delete": (None, [vp]),
    "stream_emulator_make_memref_add_lwe_ciphertexts_u64_process": (None, [vp, vp, vp, vp]),
    "stream_emulator_make_memref_add_plaintext_lwe_ciphertext_u64_process": (None, [vp, vp, vp, vp]),
    "stream_emulator_make_memref_mul_cleartext_lwe_ciphertext_u64_process": (None, [vp, vp, vp, vp]),
    "stream_emulator_make_memref_negate_lwe_ciphertext_u64_process": (None, [vp, vp, vp]),
    "stream_emulator_make_memref_keyswitch_lwe_u64_process": (None, [vp, vp, vp, u32, u32, u32, u32, u32, u32, vp]),
    "stream_emulator_make_memref_bootstrap_lwe_u64_process": (None, [vp, vp, vp, vp, u32, u32, u32, u32, u32, u32, u32,
                                                                     vp]),
    "stream_emulator_make_memref_batched_add_lwe_ciphertexts_u64_process": (None, [vp, vp, vp, vp]),
    "stream_emulator_make_memref_batched_add_plaintext_lwe_ciphertext_u64_process": (None, [vp, vp, vp, vp]),
    "stream_emulator_make_memref_batched_add_plaintext_cst_lwe_ciphertext_u64_process": (None, [vp, vp, vp, vp]),
    "stream_emulator_make_memref_batched_mul_cleartext_lwe_ciphertext_u64_process": (None, [vp, vp, vp, vp]),
    "stream_emulator_make_memref_batched_mul_cleartext_cst_lwe_ciphertext_u64_process": (None, [vp, vp, vp, vp]),
    "stream_emulator_make_memref_batched_negate_lwe_ciphertext_u64_process": (None, [vp, vp, vp]),
    "stream_emulator_make_memref_batched_keyswitch_lwe_u64_process": (None, [vp, vp, vp, u32, u32, u32, u32, u32, u32,
                                                                             vp]),
    "stream_emulator_make_memref_batched_bootstrap_lwe_u64_process": (None, [vp, vp, vp, vp, u32, u32, u32, u32, u32,
                                                                             u32, u32, vp]),
    "stream_emulator_make_memref_batched_mapped_bootstrap_lwe_u64_process": (None, [vp, vp, vp, vp, u32, u32, u32, u32,
                                                                                    u32, u32, u32, vp]),
    "stream_emulator_make_uint64_stream": (vp, [C.c_char_p, i32]),
    "stream_emulator_put_uint64": (None, [vp, u64]),
    "stream_emulator_get_uint64": (u64, [vp]),
    "stream_emulator_make_memref_stream": (vp, [C.c_char_p, i32]),
    "stream_emulator_put_memref": (None, [vp, vp, vp, u64, u64, u64, u64]),
    "stream_emulator_get_memref": (None, [vp, vp, vp, u64, u64, u64]),
    "stream_emulator_make_memref_batch_stream": (vp, [C.c_char_p, i32]),
    "stream_emulator_put_memref_batch": (None, [vp, vp, vp, u64, u64, u64, u64, u64, u64]),
    "stream_emulator_get_memref_batch": (None, [vp, vp, vp, u64, u64, u64, u64, u64]),
    # Part 6: key wire-format import (concrete-protocol.capnp)
    "concrete_hip_server_keyset_deserialize": (i32, [vp, u64, u32, C.POINTER(vp)]),
    "concrete_hip_server_keyset_load_file": (i32, [C.c_char_p, u32, C.POINTER(vp)]),
    "concrete_hip_server_keyset_destroy": (None, [vp]),
    "concrete_hip_server_keyset_bsk_count": (u32, [vp]),
    "concrete_hip_server_keyset_ksk_count": (u32, [vp]),
    "concrete_hip_server_keyset_bsk_info": (i32, [vp, u32, vp]),
    "concrete_hip_server_keyset_ksk_info": (i32, [vp, u32, vp]),
    "concrete_hip_server_keyset_read_bsk": (i32, [vp, u32, vp, u64]),
    "concrete_hip_server_keyset_read_ksk": (i32, [vp, u32, vp, u64]),
    "concrete_hip_keyset_add_server_keyset": (i32, [vp, vp]),
    "concrete_hip_set_seeded_key_decompressors": (None, [vp, vp]),
}

_lib = None


class NativeMissing(RuntimeError):
    pass


def lib():
    """Load libconcrete_hip.so (raises NativeMissing if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeMissing(f"{LIB_PATH} not built: run `make -C concrete_amd/csrc` "
                                "(or __graft_entry__.build()); there is no CPU fallback")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def declared_symbols():
    """Function names declared in include/concrete_hip.h."""
    txt = open(HEADER_PATH).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    # a name followed by "(" that does not open a function-pointer declarator "(*"
    return sorted(set(re.findall(r"\b([a-z_][a-z0-9_]*)\s*\((?!\s*\*)", txt)) - {"defined"})


def check(rc, what):
    if rc != 0:
        msg = lib().concrete_hip_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed ({rc}): {msg}")
