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

    def set_timing(self, on=True):
        """Record HIP events around every slice of the following calls (concrete_hip_keyset_set_timing)."""
        self.lib.concrete_hip_keyset_set_timing(self.h, int(on))

    def timeline(self) -> np.ndarray:
        """Per slice of the last call: (device, start, inputs copied, kernel done, outputs copied, count),
        times in ms since the call's start on that device."""
        n = self.lib.concrete_hip_keyset_timeline(self.h, None, 0)
        buf = np.zeros((max(n, 1), 6), dtype=np.float64)
        self.lib.concrete_hip_keyset_timeline(self.h, buf.ctypes.data, n)
        return buf[:n]

    def bind(self, context_ptr: int):
        """Bind a runtime-context pointer to this keyset (concrete_hip_context_bind)."""
        _native.check(self.lib.concrete_hip_context_bind(context_ptr, self.h), "context_bind")

    def close(self):
        if self.h:
            self.lib.concrete_hip_keyset_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


def batched_bootstrap(ks: Keyset, p, cts: np.ndarray, tlu: np.ndarray, bsk_index=0, out=None) -> np.ndarray:
    """memref_batched_bootstrap_lwe_hip_u64: (B, n+1) ciphertexts, one N-entry LUT -> (B, kN+1)
    (into `out` when given: a C-contiguous uint64 array of that shape)."""
    cts = np.ascontiguousarray(cts, dtype=np.uint64)
    tlu = np.ascontiguousarray(tlu, dtype=np.uint64)
    shape = (cts.shape[0], p.k * p.N + 1)
    if out is None:
        out = np.zeros(shape, dtype=np.uint64)
    elif out.shape != shape or out.dtype != np.uint64 or not out.flags.c_contiguous:
        raise ValueError(f"out must be a C-contiguous uint64 array of shape {shape}")
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


# ------------------------------------------------------------------------------------------
# the reference's names (memref_*_cuda_u64, wrappers.h:246-300): the last argument is the caller's
# runtime-context pointer, resolved to a keyset by the backend
# ------------------------------------------------------------------------------------------
def batched_bootstrap_cuda(context: int, p, cts: np.ndarray, tlu: np.ndarray, bsk_index=0) -> np.ndarray:
    L = _native.lib()
    cts = np.ascontiguousarray(cts, dtype=np.uint64)
    tlu = np.ascontiguousarray(tlu, dtype=np.uint64)
    out = np.zeros((cts.shape[0], p.k * p.N + 1), dtype=np.uint64)
    L.memref_batched_bootstrap_lwe_cuda_u64(*_desc(out), *_desc(cts), *_desc(tlu), p.n, p.N, p.level, p.base_log,
                                            p.k, bsk_index, context)
    return out


def batched_mapped_bootstrap_cuda(context: int, p, cts: np.ndarray, tlus: np.ndarray, bsk_index=0) -> np.ndarray:
    L = _native.lib()
    cts = np.ascontiguousarray(cts, dtype=np.uint64)
    tlus = np.ascontiguousarray(np.atleast_2d(tlus), dtype=np.uint64)
    out = np.zeros((cts.shape[0], p.k * p.N + 1), dtype=np.uint64)
    L.memref_batched_mapped_bootstrap_lwe_cuda_u64(*_desc(out), *_desc(cts), *_desc(tlus), p.n, p.N, p.level,
                                                   p.base_log, p.k, bsk_index, context)
    return out


def bootstrap_cuda(context: int, p, ct: np.ndarray, tlu: np.ndarray, bsk_index=0) -> np.ndarray:
    L = _native.lib()
    ct = np.ascontiguousarray(ct, dtype=np.uint64)
    tlu = np.ascontiguousarray(tlu, dtype=np.uint64)
    out = np.zeros(p.k * p.N + 1, dtype=np.uint64)
    L.memref_bootstrap_lwe_cuda_u64(*_desc(out), *_desc(ct), *_desc(tlu), p.n, p.N, p.level, p.base_log, p.k,
                                    bsk_index, context)
    return out


def batched_keyswitch_cuda(context: int, p, cts: np.ndarray, ksk_index=0) -> np.ndarray:
    L = _native.lib()
    cts = np.ascontiguousarray(cts, dtype=np.uint64)
    out = np.zeros((cts.shape[0], p.n + 1), dtype=np.uint64)
    L.memref_batched_keyswitch_lwe_cuda_u64(*_desc(out), *_desc(cts), p.ks_level, p.ks_base_log, p.big_n, p.n,
                                            ksk_index, context)
    return out


def keyswitch_cuda(context: int, p, ct: np.ndarray, ksk_index=0) -> np.ndarray:
    L = _native.lib()
    ct = np.ascontiguousarray(ct, dtype=np.uint64)
    out = np.zeros(p.n + 1, dtype=np.uint64)
    L.memref_keyswitch_lwe_cuda_u64(*_desc(out), *_desc(ct), p.ks_level, p.ks_base_log, p.big_n, p.n, ksk_index,
                                    context)
    return out


# ------------------------------------------------------------------------------------------
# the SDFG stream emulator (include/concrete_hip.h Part 5), driven from Python
# ------------------------------------------------------------------------------------------
TS_X86_TO_TOPO, TS_TOPO_TO_TOPO, TS_TOPO_TO_X86, TS_TOPO_TO_BOTH, TS_X86_TO_X86 = range(5)


class Dfg:
    """One stream-emulator graph (stream_emulator_init ... stream_emulator_delete)."""

    def __init__(self):
        self.lib = _native.lib()
        self.h = self.lib.stream_emulator_init()

    def batch_stream(self, name, stype=TS_TOPO_TO_TOPO):
        return self.lib.stream_emulator_make_memref_batch_stream(name.encode(), stype)

    def memref_stream(self, name, stype=TS_TOPO_TO_TOPO):
        return self.lib.stream_emulator_make_memref_stream(name.encode(), stype)

    def uint64_stream(self, name, stype=TS_X86_TO_TOPO):
        return self.lib.stream_emulator_make_uint64_stream(name.encode(), stype)

    def put_batch(self, s, a: np.ndarray):
        a = np.ascontiguousarray(a, dtype=np.uint64)
        self.lib.stream_emulator_put_memref_batch(s, a.ctypes.data, a.ctypes.data, 0, a.shape[0], a.shape[1],
                                                  a.shape[1], 1, 0)

    def put_memref(self, s, a: np.ndarray):
        a = np.ascontiguousarray(a, dtype=np.uint64)
        self.lib.stream_emulator_put_memref(s, a.ctypes.data, a.ctypes.data, 0, a.shape[0], 1, 0)

    def put_uint64(self, s, v: int):
        self.lib.stream_emulator_put_uint64(s, int(v))

    def get_batch(self, s, rows, cols, out=None) -> np.ndarray:
        """The stream's (rows, cols) batch, into `out` when given (C-contiguous uint64 of that shape)."""
        if out is None:
            out = np.zeros((rows, cols), dtype=np.uint64)
        elif out.shape != (rows, cols) or out.dtype != np.uint64 or not out.flags.c_contiguous:
            raise ValueError(f"out must be a C-contiguous uint64 array of shape {(rows, cols)}")
        self.lib.stream_emulator_get_memref_batch(s, out.ctypes.data, out.ctypes.data, 0, rows, cols, cols, 1)
        return out

    def get_memref(self, s, size) -> np.ndarray:
        out = np.zeros(size, dtype=np.uint64)
        self.lib.stream_emulator_get_memref(s, out.ctypes.data, out.ctypes.data, 0, size, 1)
        return out

    def keyswitch(self, sin, sout, p, context, ksk_index=0, batched=True):
        f = (self.lib.stream_emulator_make_memref_batched_keyswitch_lwe_u64_process if batched
             else self.lib.stream_emulator_make_memref_keyswitch_lwe_u64_process)
        f(self.h, sin, sout, p.ks_level, p.ks_base_log, p.big_n, p.n, p.n + 1, ksk_index, context)

    def bootstrap(self, sin, slut, sout, p, context, bsk_index=0, mapped=False, batched=True):
        f = (self.lib.stream_emulator_make_memref_batched_mapped_bootstrap_lwe_u64_process if mapped else
             self.lib.stream_emulator_make_memref_batched_bootstrap_lwe_u64_process if batched else
             self.lib.stream_emulator_make_memref_bootstrap_lwe_u64_process)
        f(self.h, sin, slut, sout, p.n, p.N, p.level, p.base_log, p.k, p.k * p.N + 1, bsk_index, context)

    def linear(self, op, sin1, sin2, sout):
        """op: add, add_pt, add_pt_cst, mul, mul_cst, neg (the batched processes)."""
        L = self.lib
        f = {"add": L.stream_emulator_make_memref_batched_add_lwe_ciphertexts_u64_process,
             "add_pt": L.stream_emulator_make_memref_batched_add_plaintext_lwe_ciphertext_u64_process,
             "add_pt_cst": L.stream_emulator_make_memref_batched_add_plaintext_cst_lwe_ciphertext_u64_process,
             "mul": L.stream_emulator_make_memref_batched_mul_cleartext_lwe_ciphertext_u64_process,
             "mul_cst": L.stream_emulator_make_memref_batched_mul_cleartext_cst_lwe_ciphertext_u64_process}
        if op == "neg":
            L.stream_emulator_make_memref_batched_negate_lwe_ciphertext_u64_process(self.h, sin1, sout)
        else:
            f[op](self.h, sin1, sin2, sout)

    def run(self):
        self.lib.stream_emulator_run(self.h)

    def close(self):
        if self.h:
            self.lib.stream_emulator_delete(self.h)
            self.h = None

    def __del__(self):
        self.close()
