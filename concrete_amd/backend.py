"""Host-side mirror of the runtime's use of the backend ABI (Python plumbing for tests/bench).

The reference runtime drives the backend from C++ (compiler lib/Runtime/wrappers.cpp:164-363,
GPUDFG.cpp:1114-1250, context.h:86-145).  This module replays that call sequence over the C
ABI with device memory owned by PyTorch (plumbing only: every computation is a HIP kernel of
libconcrete_hip.so).  Names follow the reference domain: LWE/GLWE ciphertexts, bootstrapping
key (BSK), keyswitching key (KSK), lookup tables (LUT).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _native

vp = C.c_void_p


@dataclass(frozen=True)
class PbsParams:
    """n = LWE dimension of the PBS input, k = GLWE dimension, N = polynomial size,
    level/base_log = PBS decomposition, ks_level/ks_base_log = KS decomposition."""
    n: int
    k: int
    N: int
    level: int
    base_log: int
    ks_level: int = 4
    ks_base_log: int = 3

    @property
    def big_n(self) -> int:
        return self.k * self.N

    @property
    def lwe_in_size(self) -> int:
        return self.n + 1

    @property
    def lwe_out_size(self) -> int:
        return self.k * self.N + 1

    @property
    def glwe_size(self) -> int:
        return (self.k + 1) * self.N

    @property
    def bsk_len(self) -> int:  # u64 words, concrete-cpu bootstrap.rs:417-429
        return self.n * self.level * (self.k + 1) ** 2 * self.N

    @property
    def ksk_len(self) -> int:  # u64 words, concrete-cpu keyswitch.rs:226-236
        return self.big_n * self.ks_level * (self.n + 1)

    def bsk_bytes_per_pbs(self) -> int:
        """Algorithmic HBM bytes of one PBS: BSK + LWE in + LWE out."""
        return 8 * (self.bsk_len + self.lwe_in_size + self.lwe_out_size)


# BASELINE.json configs[1]/[2] (cfg2) and configs[3] (cfg4)
CFG2 = PbsParams(n=630, k=1, N=1024, level=3, base_log=7, ks_level=4, ks_base_log=3)
CFG4 = PbsParams(n=742, k=1, N=2048, level=1, base_log=23, ks_level=5, ks_base_log=3)

# The concrete optimizer's 128-bit parameter rows at log norm2 = 0 (compilers/concrete-optimizer/
# v0-parameters/ref/v0_last_128: k, log2 N, n, br_l, br_b, ks_l, ks_b), keyed by message bits.
# All but 5 bits run on the general path (pbs_generic.hip).
OPTIMIZER_SETS = {
    1: PbsParams(n=592, k=5, N=256, level=1, base_log=15, ks_level=3, ks_base_log=3),
    2: PbsParams(n=700, k=5, N=256, level=1, base_log=15, ks_level=3, ks_base_log=4),
    3: PbsParams(n=722, k=3, N=512, level=1, base_log=18, ks_level=3, ks_base_log=4),
    4: PbsParams(n=801, k=2, N=1024, level=1, base_log=23, ks_level=3, ks_base_log=4),
    5: PbsParams(n=783, k=1, N=2048, level=1, base_log=23, ks_level=5, ks_base_log=3),
    6: PbsParams(n=880, k=1, N=4096, level=1, base_log=22, ks_level=4, ks_base_log=4),
    7: PbsParams(n=915, k=1, N=8192, level=1, base_log=22, ks_level=6, ks_base_log=3),
    8: PbsParams(n=1006, k=1, N=16384, level=2, base_log=15, ks_level=5, ks_base_log=4),
    9: PbsParams(n=1039, k=1, N=32768, level=2, base_log=15, ks_level=7, ks_base_log=3),
    10: PbsParams(n=1136, k=1, N=65536, level=2, base_log=14, ks_level=6, ks_base_log=4),
}


def _ptr(a) -> int:
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return a.data_ptr()  # torch tensor


# ---------------------------------------------------------------------------------------
# client-side generation (product keygen; deterministic per seed)
# ---------------------------------------------------------------------------------------
def secure_std(glwe_dim: int, poly_size: int) -> float:
    return 2.0 ** _native.lib().concrete_hip_secure_log2_std(glwe_dim, poly_size)


def binary_key(length: int, seed: int) -> np.ndarray:
    sk = np.zeros(length, dtype=np.uint64)
    _native.lib().concrete_hip_keygen_binary(_ptr(sk), length, seed)
    return sk


def lwe_encrypt(sk: np.ndarray, plaintexts, n: int, std: float, seed: int) -> np.ndarray:
    pts = np.ascontiguousarray(plaintexts, dtype=np.uint64)
    out = np.zeros((len(pts), n + 1), dtype=np.uint64)
    _native.lib().concrete_hip_lwe_encrypt_batch(_ptr(sk), _ptr(out), _ptr(pts), len(pts), n, std, seed)
    return out


def lwe_decrypt(sk: np.ndarray, cts: np.ndarray, n: int) -> np.ndarray:
    L = _native.lib()
    cts = np.ascontiguousarray(cts, dtype=np.uint64)
    return np.array([L.concrete_hip_lwe_decrypt(_ptr(sk), cts[i].ctypes.data, n) for i in range(cts.shape[0])],
                    dtype=np.uint64)


def bsk_generate(p: PbsParams, lwe_sk, glwe_sk, seed: int, std: float | None = None) -> np.ndarray:
    bsk = np.zeros(p.bsk_len, dtype=np.uint64)
    _native.lib().concrete_hip_bsk_generate(_ptr(bsk), _ptr(lwe_sk), _ptr(glwe_sk), p.n, p.k, p.N, p.level,
                                           p.base_log, secure_std(p.k, p.N) if std is None else std, seed)
    return bsk


def ksk_generate(p: PbsParams, sk_in, sk_out, seed: int, std: float | None = None) -> np.ndarray:
    ksk = np.zeros(p.ksk_len, dtype=np.uint64)
    _native.lib().concrete_hip_ksk_generate(_ptr(ksk), _ptr(sk_in), _ptr(sk_out), p.big_n, p.n, p.ks_level,
                                           p.ks_base_log, secure_std(1, p.n) if std is None else std, seed)
    return ksk


def encode(m, width: int):
    """Native integer encoding, compiler lib/Common/Transformers.cpp:364-382."""
    return np.uint64((int(m) << (64 - (width + 1))) & 0xFFFFFFFFFFFFFFFF)


def decode(x, width: int, signed: bool = False) -> int:
    """Native decoding, compiler lib/Common/Transformers.cpp:384-427 (signed: sign-extended)."""
    x = int(x)
    out = x >> (64 - width - 2)
    carry = out % 2
    out = ((out >> 1) + carry) % (1 << (width + 1))
    if signed and out >= (1 << (width - 1)):
        # Transformers.cpp:414-419: output |= UINT64_MAX << precision, read as int64
        out = (out & ((1 << width) - 1)) - (1 << width)
    return out


def expand_lut(table, N: int, out_bits: int, signed: bool = False) -> np.ndarray:
    tab = np.ascontiguousarray(table, dtype=np.uint64)
    out = np.zeros(N, dtype=np.uint64)
    _native.lib().concrete_hip_encode_expand_lut(_ptr(out), N, _ptr(tab), len(tab), out_bits, int(signed))
    return out


def trivial_glwe(p: PbsParams, lut_poly: np.ndarray) -> np.ndarray:
    """Trivial GLWE accumulator [0 .. 0 | LUT] (compiler lib/Runtime/wrappers.cpp:199-209)."""
    g = np.zeros(p.glwe_size, dtype=np.uint64)
    g[p.k * p.N:] = lut_poly
    return g


# ---------------------------------------------------------------------------------------
# device side (torch owns memory; kernels run on torch's current stream of that device)
# ---------------------------------------------------------------------------------------
def _torch():
    import torch
    return torch


def to_device(a: np.ndarray, device):
    torch = _torch()
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(device)


def to_host(t) -> np.ndarray:
    return t.cpu().numpy().view(np.uint64)


def _stream(device) -> int:
    torch = _torch()
    return torch.cuda.current_stream(device).cuda_stream


def _gpu_index(device) -> int:
    torch = _torch()
    return torch.device(device).index or 0


class RuntimeBuffer:
    """A device buffer allocated and filled the way the reference runtime does it
    (cuda_malloc_async + cuda_memcpy_async_to_gpu, include/concretelang/Runtime/context.h:134-139),
    released by cuda_drop: the backend sees its lifetime, so derived data (the matrix-core
    keyswitch's key bytes) may be cached for it.  Has data_ptr() like a torch tensor."""

    def __init__(self, host: np.ndarray, gpu: int = 0):
        L = _native.lib()
        host = np.ascontiguousarray(host)
        self.gpu = gpu
        self.stream = L.cuda_create_stream(gpu)
        self.nbytes = host.nbytes
        self.ptr = L.cuda_malloc_async(self.nbytes, self.stream, gpu)
        self.write(host)

    def write(self, host: np.ndarray):
        L = _native.lib()
        host = np.ascontiguousarray(host)
        assert host.nbytes == self.nbytes
        L.cuda_memcpy_async_to_gpu(self.ptr, host.ctypes.data, self.nbytes, self.stream, self.gpu)
        L.cuda_synchronize_device(self.gpu)

    def data_ptr(self) -> int:
        return self.ptr

    def free(self):
        if self.ptr:
            L = _native.lib()
            L.cuda_drop(self.ptr, self.gpu)
            L.cuda_destroy_stream(self.stream, self.gpu)
            self.ptr = None


def pbs_supported(p: PbsParams) -> bool:
    """Whether the kernels take this parameter set (and compute it exactly: pbs.hpp)."""
    return bool(_native.lib().concrete_hip_pbs_supported(p.k, p.N, p.level, p.base_log))


def bsk_format(p: PbsParams) -> tuple[int, int, int]:
    """Device key format of (k, N, l): (kind, limbs, limb bits); kind 1 / 2 = the N = 1024 /
    2048 kernels' layouts, 3 = the general path (pbs_generic.hip), 0 = unsupported."""
    limbs, bits = C.c_uint32(0), C.c_uint32(0)
    kind = _native.lib().concrete_hip_bsk_format(p.k, p.N, p.level, C.byref(limbs), C.byref(bits))
    return int(kind), int(limbs.value), int(bits.value)


def fourier_bsk_bytes(p: PbsParams) -> int:
    return int(_native.lib().concrete_hip_fourier_bsk_size_bytes(p.n, p.k, p.level, p.N))


def convert_bsk(p: PbsParams, bsk, device="cuda:0", out=None):
    """Standard u64 BSK (numpy host array or torch device tensor) -> device Fourier key."""
    torch = _torch()
    nbytes = fourier_bsk_bytes(p)
    if out is None:
        out = torch.empty(nbytes // 8, dtype=torch.int64, device=device)
    src_is_dev = not isinstance(bsk, np.ndarray)
    src = bsk if src_is_dev else np.ascontiguousarray(bsk, dtype=np.uint64)
    _native.check(_native.lib().concrete_hip_convert_bsk(_stream(device), _gpu_index(device), _ptr(out), _ptr(src),
                                                          int(src_is_dev), p.n, p.k, p.level, p.N),
                  "concrete_hip_convert_bsk")
    return out


def pbs(p: PbsParams, fbsk, lwe_in, luts, lut_idx=None, in_idx=None, out_idx=None, out=None,
        num_samples=None, resid=None):
    """Batched PBS on device tensors: lwe_in (B, n+1), luts (L, (k+1)N) -> out (B, kN+1)."""
    torch = _torch()
    device = lwe_in.device
    B = lwe_in.shape[0] if num_samples is None else num_samples
    if out is None:
        out = torch.empty((B, p.lwe_out_size), dtype=torch.int64, device=device)
    _native.check(_native.lib().concrete_hip_pbs(
        _stream(device), _gpu_index(device), _ptr(out), _ptr(out_idx), _ptr(luts), _ptr(lut_idx), _ptr(lwe_in),
        _ptr(in_idx), _ptr(fbsk), p.n, p.k, p.N, p.base_log, p.level, B, _ptr(resid)), "concrete_hip_pbs")
    return out


def device_status(device="cuda:0") -> int:
    """Synchronise the device and return (and clear) its sticky status: 0, or -4 when a PBS
    kernel's wave synchronisation gave up since the last check (concrete_hip_device_status)."""
    return int(_native.lib().concrete_hip_device_status(_gpu_index(device)))


def stream_status(device="cuda:0", stream=None) -> int:
    """Wait for the work issued on `stream` (default: torch's current stream of `device`) and return
    (and clear) the status of the PBS launches made on it: 0, or -4 when one gave up a wave
    synchronisation (concrete_hip_stream_status; status words are per stream)."""
    s = _stream(device) if stream is None else stream.cuda_stream
    return int(_native.lib().concrete_hip_stream_status(s, _gpu_index(device)))


def set_spin_limit(polls: int) -> None:
    """Spin bound of the PBS kernels' wave synchronisation (0 = default); a test hook."""
    _native.lib().concrete_hip_set_spin_limit(int(polls))


def set_thread_spin_limit(polls: int) -> None:
    """The same bound for launches issued by the calling thread only (0 = the process bound)."""
    _native.lib().concrete_hip_set_thread_spin_limit(int(polls))


def keyswitch(p: PbsParams, ksk_dev, lwe_in, out=None, in_idx=None, out_idx=None, num_samples=None):
    """Batched LWE keyswitch kN -> n on device tensors."""
    torch = _torch()
    device = lwe_in.device
    B = lwe_in.shape[0] if num_samples is None else num_samples
    if out is None:
        out = torch.empty((B, p.n + 1), dtype=torch.int64, device=device)
    _native.check(_native.lib().concrete_hip_keyswitch(
        _stream(device), _gpu_index(device), _ptr(out), _ptr(out_idx), _ptr(lwe_in), _ptr(in_idx), _ptr(ksk_dev),
        p.big_n, p.n, p.ks_base_log, p.ks_level, B), "concrete_hip_keyswitch")
    return out
