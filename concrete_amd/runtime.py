"""ctypes front of the native runtime glue (concrete_amd/csrc/runtime.hip, include/concrete_hip.h
Part 4): what a compiled circuit's memref calls look like, driven from numpy arrays.

Each wrapper passes an MLIR memref descriptor expanded as (allocated, aligned, offset, sizes...,
strides...) exactly as the compiled circuit does (compiler include/concretelang/Runtime/
wrappers.h:240-300).  All memory is host memory; the native code moves it to the devices.
"""
from __future__ import annotations

import numpy as np

from . import _native


def _desc(a: np.ndarray):
    assert a.dtype == np.uint64 and a.flags.c_contiguous
    p = a.ctypes.data
    if a.ndim == 1:
        return [p, p, 0, a.shape[0], 1]
    return [p, p, 0, a.shape[0], a.shape[1], a.shape[1], 1]


class Keyset:
    """Opaque native keyset: standard-domain keys registered once, device keys resident."""

    def __init__(self, devices=None):
        self.lib = _native.lib()
        self.h = self.lib.concrete_hip_keyset_create()
        if devices is not None:
            arr = np.asarray(devices, dtype=np.uint32)
            _native.check(self.lib.concrete_hip_keyset_set_devices(self.h, arr.ctypes.data, len(arr)),
                          "keyset_set_devices")

    def add_bsk(self, index, bsk, p):
        bsk = np.ascontiguousarray(bsk, dtype=np.uint64)
        _native.check(self.lib.concrete_hip_keyset_add_bsk(self.h, index, bsk.ctypes.data, p.n, p.k, p.level,
                                                           p.base_log, p.N), "keyset_add_bsk")

    def add_ksk(self, index, ksk, p):
        ksk = np.ascontiguousarray(ksk, dtype=np.uint64)
        _native.check(self.lib.concrete_hip_keyset_add_ksk(self.h, index, ksk.ctypes.data, p.ks_level,
                                                           p.ks_base_log, p.big_n, p.n), "keyset_add_ksk")

    def close(self):
        if self.h:
            self.lib.concrete_hip_keyset_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


def batched_bootstrap(ks: Keyset, p, cts: np.ndarray, tlu: np.ndarray, bsk_index=0) -> np.ndarray:
    """memref_batched_bootstrap_lwe_hip_u64: (B, n+1) ciphertexts, one N-entry LUT -> (B, kN+1)."""
    cts = np.ascontiguousarray(cts, dtype=np.uint64)
    tlu = np.ascontiguousarray(tlu, dtype=np.uint64)
    out = np.zeros((cts.shape[0], p.k * p.N + 1), dtype=np.uint64)
    ks.lib.memref_batched_bootstrap_lwe_hip_u64(*_desc(out), *_desc(cts), *_desc(tlu), p.n, p.N, p.level,
                                                p.base_log, p.k, bsk_index, ks.h)
    return out


def batched_mapped_bootstrap(ks: Keyset, p, cts: np.ndarray, tlus: np.ndarray, bsk_index=0) -> np.ndarray:
    """memref_batched_mapped_bootstrap_lwe_hip_u64: one LUT row per sample (or a single row)."""
    cts = np.ascontiguousarray(cts, dtype=np.uint64)
    tlus = np.ascontiguousarray(np.atleast_2d(tlus), dtype=np.uint64)
    out = np.zeros((cts.shape[0], p.k * p.N + 1), dtype=np.uint64)
    ks.lib.memref_batched_mapped_bootstrap_lwe_hip_u64(*_desc(out), *_desc(cts), *_desc(tlus), p.n, p.N, p.level,
                                                       p.base_log, p.k, bsk_index, ks.h)
    return out


def bootstrap(ks: Keyset, p, ct: np.ndarray, tlu: np.ndarray, bsk_index=0) -> np.ndarray:
    """memref_bootstrap_lwe_hip_u64: one ciphertext."""
    ct = np.ascontiguousarray(ct, dtype=np.uint64)
    tlu = np.ascontiguousarray(tlu, dtype=np.uint64)
    out = np.zeros(p.k * p.N + 1, dtype=np.uint64)
    ks.lib.memref_bootstrap_lwe_hip_u64(*_desc(out), *_desc(ct), *_desc(tlu), p.n, p.N, p.level, p.base_log, p.k,
                                        bsk_index, ks.h)
    return out


def batched_keyswitch(ks: Keyset, p, cts: np.ndarray, ksk_index=0) -> np.ndarray:
    """memref_batched_keyswitch_lwe_hip_u64: (B, kN+1) -> (B, n+1)."""
    cts = np.ascontiguousarray(cts, dtype=np.uint64)
    out = np.zeros((cts.shape[0], p.n + 1), dtype=np.uint64)
    ks.lib.memref_batched_keyswitch_lwe_hip_u64(*_desc(out), *_desc(cts), p.ks_level, p.ks_base_log, p.big_n, p.n,
                                                ksk_index, ks.h)
    return out


def keyswitch(ks: Keyset, p, ct: np.ndarray, ksk_index=0) -> np.ndarray:
    """memref_keyswitch_lwe_hip_u64: one ciphertext."""
    ct = np.ascontiguousarray(ct, dtype=np.uint64)
    out = np.zeros(p.n + 1, dtype=np.uint64)
    ks.lib.memref_keyswitch_lwe_hip_u64(*_desc(out), *_desc(ct), p.ks_level, p.ks_base_log, p.big_n, p.n, ksk_index,
                                        ks.h)
    return out
