"""ctypes bindings for the CPU restatement (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product path (concrete_amd/).  See tfhe_oracle.h for the
reference file:line each routine restates.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

u64p = C.POINTER(C.c_uint64)
i64p = C.POINTER(C.c_int64)
f64p = C.POINTER(C.c_double)
sz = C.c_size_t

MODE_SCHOOLBOOK, MODE_KARATSUBA, MODE_FFT, MODE_FFT64 = 0, 1, 2, 3  # FFT64: approximate (tfhe_oracle.h)


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        L.ora_secure_log2_std.restype = C.c_double
        L.ora_secure_log2_std.argtypes = [C.c_uint64, C.c_uint64]
        L.ora_lwe_decrypt.restype = C.c_uint64
        L.ora_modswitch.restype = sz
        L.ora_modswitch.argtypes = [C.c_uint64, sz]
        L.ora_decomp_init_state.restype = C.c_uint64
        L.ora_decomp_init_state.argtypes = [C.c_uint64, sz, sz]
        L.ora_fourier_bsk_len.restype = sz
        L.ora_fourier_bsk_len.argtypes = [sz] * 5
        L.ora_fft_error_bound.restype = C.c_double
        L.ora_fft_error_bound.argtypes = [f64p, sz, sz, sz, sz, sz, sz]
        L.ora_encode_native.restype = C.c_uint64
        L.ora_encode_native.argtypes = [C.c_uint64, C.c_uint32]
        L.ora_decode_native.restype = C.c_uint64
        L.ora_decode_native.argtypes = [C.c_uint64, C.c_uint32, C.c_int]
        L.ora_bsk_generate.argtypes = [u64p, u64p, u64p, sz, sz, sz, sz, sz, C.c_double, C.c_uint64]
        L.ora_ksk_generate.argtypes = [u64p, u64p, u64p, sz, sz, sz, sz, C.c_double, C.c_uint64]
        L.ora_bsk_to_fourier.argtypes = [f64p, u64p, sz, sz, sz, sz, sz]
        L.ora_pbs_batch.argtypes = [u64p, u64p, u64p, u64p, u64p, u64p, u64p, f64p,
                                    sz, sz, sz, sz, sz, sz, sz, C.c_int, C.c_int, f64p]
        L.ora_keyswitch_batch.argtypes = [u64p, u64p, u64p, u64p, u64p, sz, sz, sz, sz, sz, C.c_int]
        L.ora_polymul_acc_schoolbook.argtypes = [u64p, i64p, u64p, sz]
        L.ora_polymul_acc_karatsuba.argtypes = [u64p, i64p, u64p, sz]
        L.ora_decompose.argtypes = [C.c_uint64, sz, sz, i64p]
        L.ora_limb_split.argtypes = [C.c_uint64, sz, i64p]
        L.ora_monomial_mul.argtypes = [u64p, u64p, sz, sz]
        L.ora_monomial_div.argtypes = [u64p, u64p, sz, sz]
        L.ora_sample_extract.argtypes = [u64p, u64p, sz, sz]
        L.ora_encode_expand_lut.argtypes = [u64p, sz, u64p, sz, C.c_uint32, C.c_int]
        L.ora_external_product_acc.argtypes = [u64p, u64p, f64p, u64p, sz, sz, sz, sz, sz, C.c_int, f64p]
        _lib = L
    return _lib


def P(a, t=u64p):
    return a.ctypes.data_as(t) if a is not None else None


@dataclass(frozen=True)
class Params:
    """PBS/KS parameter set (names follow the reference: n = LWE dim after KS, k = GLWE dim,
    N = polynomial size, l/logB = PBS decomposition, ks_l/ks_logB = KS decomposition)."""
    n: int
    k: int
    N: int
    l: int
    logB: int
    ks_l: int = 4
    ks_logB: int = 3
    limbs: int = 3

    @property
    def big_n(self):  # LWE dimension of the PBS output / KS input
        return self.k * self.N


# BASELINE.json configs[1] (cfg2) and configs[3] (cfg4); KS params from SURVEY.md §8.
CFG2 = Params(n=630, k=1, N=1024, l=3, logB=7, ks_l=4, ks_logB=3, limbs=3)
CFG4 = Params(n=742, k=1, N=2048, l=1, logB=23, ks_l=5, ks_logB=3, limbs=8)  # 8 limbs: certified bound 0.16
SMALL = Params(n=16, k=1, N=256, l=3, logB=7, ks_l=4, ks_logB=3, limbs=3)


def limbs_for(N: int) -> int:
    """Key limbs the oracle's certified FFT path needs (fft_error_bound < 1/2): 3 at N = 1024
    (l = 3, logB = 7), 8 at N = 2048 (l = 1, logB = 23)."""
    return 3 if N <= 1024 else 8


def gpu2048_error_bound(fbsk_gpu: np.ndarray, logB: int = 23, level: int = 1) -> float:
    """Certified bound on |x - round(x)| for the GPU's N = 2048 scheme (concrete_amd/csrc/
    pbs2048.hip).  The products are taken at the square roots +-s_k of the
    N = 1024 evaluation points (P2_PM): each digit polynomial's 1024-point negacyclic spectrum is
    its two parity halves' 512-point transforms plus one radix-2 stage with twiddle s_k, and the
    output is unfolded by the inverse stage (C_e = U+ + U-, C_o = (U+ - U-) conj s_k) before the
    512-point inverse transforms: Higham's bound for a 1024-point transform (log M = 10) with
    twiddle error mu = 2u (s_k from sincospi, <= 1 ulp per component; the tables are correctly
    rounded).  The digit split on the 16-bit key-limb grid, d = d_lo + 2^16 d_hi (|d_lo| <= 2^15,
    |d_hi| <= 2^(logB-17) + 1), makes output slot m the sum of d_lo g_m + d_hi g_{m-1} over both
    rows: 4 full N = 2048 products.  level > 1 (logB <= 15): the l levels' whole digits sum into the
    same slot, dsum = 2 l 2^(logB-1).  fbsk_gpu: the device key (f64 view; K+- = G(+-s) / 1024)."""
    u = 2.0 ** -53
    logM = 10.0
    mu = 2.0 * u
    eta = mu + 4.0 * u / (1.0 - 4.0 * u) * (np.sqrt(2.0) + mu)
    gamma = logM * eta / (1.0 - logM * eta)
    f = np.asarray(fbsk_gpu, dtype=np.float64).reshape(-1, 2)
    maxG = float(np.max(np.hypot(f[:, 0], f[:, 1]))) * 1024.0
    if level > 1:
        dsum = 2.0 * level * 2.0 ** (logB - 1)  # whole digits of every level, both rows
    else:
        dlo = 2.0 ** 15
        dhi = 2.0 ** max(logB - 17, 0) + 1.0
        dsum = 2.0 * (dlo + dhi)                # sum over the 4 products of max |digit|
    # forward transform, key rounding, pointwise product and inverse of each product, plus the
    # accumulation and unfold additions: (4 gamma + 5 u), as for the N = 1024 products
    main = np.sqrt(2048.0) * dsum * maxG * (4.0 * gamma + 5.0 * u) * 1.0001
    max_out = 2048.0 * dsum * 2.0 ** 15
    return float(main + 4.0 * u * max_out)


def gpu1024k2_error_bound(fbsk_gpu: np.ndarray, logB: int = 23, level: int = 1) -> float:
    """Certified bound on |x - round(x)| for the GPU's k = 2, N = 1024, l = 1 scheme
    (concrete_amd/csrc/pbs1024k2.hip): the N = 1024 products of pbs.hip
    (512-point folded, twisted transforms, log M = 9, correctly rounded tables: mu = u) on the
    digit split of pbs2048.hip, d = d_lo + 2^16 d_hi (|d_lo| <= 2^15, |d_hi| <= 2^(logB-17) + 1)
    against 16-bit key limbs: output slot m is the sum of d_lo g_m + d_hi g_{m-1} over the three
    rows, 6 N = 1024 products.  fbsk_gpu: the device key (f64 view; spectra scaled by 1/512)."""
    u = 2.0 ** -53
    logM = 9.0
    mu = u
    eta = mu + 4.0 * u / (1.0 - 4.0 * u) * (np.sqrt(2.0) + mu)
    gamma = logM * eta / (1.0 - logM * eta)
    f = np.asarray(fbsk_gpu, dtype=np.float64).reshape(-1, 2)
    maxG = float(np.max(np.hypot(f[:, 0], f[:, 1]))) * 512.0
    if level == 1:
        dlo = 2.0 ** 15
        dhi = 2.0 ** max(logB - 17, 0) + 1.0
        dsum = 3.0 * (dlo + dhi)                # sum over the 6 products of max |digit|
    else:                                       # l = 2, logB <= 15: two whole digits per row
        dsum = 3.0 * level * 2.0 ** (logB - 1)
    # forward transform, key rounding, pointwise product and inverse of each product, plus the
    # accumulation additions: (4 gamma + 5 u), as for the N = 2048 products
    main = np.sqrt(1024.0) * dsum * maxG * (4.0 * gamma + 5.0 * u) * 1.0001
    max_out = 1024.0 * dsum * 2.0 ** 15
    return float(main + 4.0 * u * max_out)


def gpu_small_error_bound(fbsk_gpu: np.ndarray, N: int, k: int, logB: int, level: int = 1) -> float:
    """Certified bound on |x - round(x)| for the GPU's small-ring scheme (concrete_amd/csrc/
    pbs_small.hip, DESIGN.md §4.9: N = 512, k = 3 / N = 256, k = 5, l = 1).  P = 1024 / N
    polynomials share one 512-point transform: their M-point spectra come out of the fft512 through a
    P-point DFT and one twiddle product (sincospi, mu = 2u), i.e. a transform of 9 + log2 P + 1
    stages, and its error is relative to the norm of all P polynomials together: the 2-norm factor
    is sqrt(P N) = 32 instead of sqrt(N).  Digits on the 16-bit limb grid as in pbs1024k2.hip
    (logB <= 15: one sub-digit, |d| <= 2^(logB-1)); level > 1 (pbs512k4.hip, logB <= 15): the l
    levels' whole digits sum into the same slot, dsum = (k + 1) l 2^(logB-1) (k = 4, l = 2: 13-bit key
    limbs, which the measured key spectrum carries).  fbsk_gpu: the device key (f64 view; spectra
    scaled by 1 / (512 P))."""
    u = 2.0 ** -53
    P = 1024 // N
    logM = 9.0 + np.log2(P) + 1.0
    mu = 2.0 * u
    eta = mu + 4.0 * u / (1.0 - 4.0 * u) * (np.sqrt(2.0) + mu)
    gamma = logM * eta / (1.0 - logM * eta)
    f = np.asarray(fbsk_gpu, dtype=np.float64).reshape(-1, 2)
    maxG = float(np.max(np.hypot(f[:, 0], f[:, 1]))) * 512.0 * P
    if logB <= 15 or level > 1:  # whole digits (level > 1: pbs512k4.hip's l = 2 reaches logB 16)
        dmax = 2.0 ** (logB - 1) * level
    else:
        dmax = 2.0 ** 15 + 2.0 ** max(logB - 17, 0) + 1.0
    dsum = (k + 1) * dmax
    main = np.sqrt(1024.0) * dsum * maxG * (4.0 * gamma + 5.0 * u) * 1.0001
    max_out = N * dsum * 2.0 ** 15
    return float(main + 4.0 * u * max_out)


def generic_error_bound(k: int, N: int, l: int, logB: int, bits: int, fbsk_gpu=None) -> float:
    """Certified bound on |x - round(x)| for the GPU's general path (concrete_amd/csrc/
    pbs_generic.hip:generic_error_bound): R = (k+1) l T products per slot of a
    digit (or b-bit sub-digit) polynomial with a b-bit key-limb spectrum through radix-4
    forward/inverse transforms (gamma doubled), plus the f64 key transform and the final
    rounding.  fbsk_gpu: the device key (f64 view, spectra scaled by 1/M) -> measured max|G|;
    None -> the random-key estimate the kernel's gate uses."""
    u = 2.0 ** -53
    M = N / 2.0
    logM = np.log2(M)
    mu = 5.0 * u  # two-level twiddle tables: products of two correctly rounded entries
    eta = mu + 4.0 * u / (1.0 - 4.0 * u) * (np.sqrt(2.0) + mu)
    gamma = 2.0 * logM * eta / (1.0 - 2.0 * logM * eta)
    T = -(-logB // bits)
    dbits = min(logB, bits)
    R = (k + 1) * l * T
    dnorm = np.sqrt(N) * 2.0 ** (dbits - 1)
    gnorm = np.sqrt(N) * 2.0 ** (bits - 1)
    if fbsk_gpu is None:
        maxG = 8.0 * np.sqrt(M) * 2.0 ** (bits - 1) * np.sqrt(2.0)
    else:
        f = np.asarray(fbsk_gpu, dtype=np.float64).reshape(-1, 2)
        maxG = float(np.max(np.hypot(f[:, 0], f[:, 1]))) * M
    max_out = R * N * 2.0 ** (dbits - 1) * 2.0 ** (bits - 1)
    return float(R * dnorm * (maxG * (4.0 * gamma + 3.0 * u) + gamma * gnorm) * 1.0001 + 4.0 * u * max_out)


def bsk_std_torus(p: Params) -> float:
    return 2.0 ** lib().ora_secure_log2_std(p.k, p.N)


def lwe_std_torus(p: Params) -> float:
    return 2.0 ** lib().ora_secure_log2_std(1, p.n)


def keygen_bsk(p: Params, lwe_sk, glwe_sk, seed: int, std=None):
    L = lib()
    bsk = np.zeros(p.n * p.l * (p.k + 1) ** 2 * p.N, dtype=np.uint64)
    L.ora_bsk_generate(P(bsk), P(lwe_sk), P(glwe_sk), p.n, p.k, p.N, p.l, p.logB,
                       bsk_std_torus(p) if std is None else std, seed)
    return bsk


def keygen_ksk(p: Params, sk_in, sk_out, seed: int, std=None):
    L = lib()
    ksk = np.zeros(p.big_n * p.ks_l * (p.n + 1), dtype=np.uint64)
    L.ora_ksk_generate(P(ksk), P(sk_in), P(sk_out), p.big_n, p.n, p.ks_l, p.ks_logB,
                       lwe_std_torus(p) if std is None else std, seed)
    return ksk


def bsk_to_fourier(p: Params, bsk):
    L = lib()
    f = np.zeros(L.ora_fourier_bsk_len(p.n, p.k, p.N, p.l, p.limbs), dtype=np.float64)
    L.ora_bsk_to_fourier(P(f, f64p), P(bsk), p.n, p.k, p.N, p.l, p.limbs)
    return f


def fft_error_bound(p: Params, fbsk) -> float:
    return lib().ora_fft_error_bound(P(fbsk, f64p), p.n, p.k, p.N, p.l, p.logB, p.limbs)


def pbs_batch(p: Params, lwe_in, luts, bsk=None, fbsk=None, lut_idx=None, mode=MODE_FFT,
              nthreads=0, in_idx=None, out_idx=None):
    """Batched PBS with the runtime's index-array semantics (GPUDFG.cpp:1149-1205).
    lwe_in: (B, n+1) u64; luts: (num_luts, (k+1)N) u64 trivial GLWE accumulators."""
    L = lib()
    lwe_in = np.ascontiguousarray(lwe_in, dtype=np.uint64)
    luts = np.ascontiguousarray(luts, dtype=np.uint64)
    B = lwe_in.shape[0] if in_idx is None else len(in_idx)
    out_rows = B if out_idx is None else int(np.max(out_idx)) + 1
    out = np.zeros((out_rows, p.big_n + 1), dtype=np.uint64)
    resid = C.c_double(0.0)
    li = None if lut_idx is None else np.ascontiguousarray(lut_idx, dtype=np.uint64)
    ii = None if in_idx is None else np.ascontiguousarray(in_idx, dtype=np.uint64)
    oi = None if out_idx is None else np.ascontiguousarray(out_idx, dtype=np.uint64)
    L.ora_pbs_batch(P(out), P(oi), P(luts), P(li), P(lwe_in), P(ii), P(bsk), P(fbsk, f64p),
                    p.n, p.k, p.N, p.l, p.logB, p.limbs, B, mode, nthreads, C.byref(resid))
    return out, resid.value


def keyswitch_batch(p: Params, lwe_in, ksk, nthreads=0):
    L = lib()
    lwe_in = np.ascontiguousarray(lwe_in, dtype=np.uint64)
    B = lwe_in.shape[0]
    out = np.zeros((B, p.n + 1), dtype=np.uint64)
    L.ora_keyswitch_batch(P(out), None, P(lwe_in), None, P(ksk), p.ks_l, p.ks_logB, p.big_n, p.n, B, nthreads)
    return out


def encode(m, width):
    return np.uint64(lib().ora_encode_native(int(m), width))


def decode(x, width, signed=False):
    return int(lib().ora_decode_native(int(x), width, int(signed)))


def expand_lut(table, N, out_bits, signed=False):
    L = lib()
    tab = np.ascontiguousarray(table, dtype=np.uint64)
    out = np.zeros(N, dtype=np.uint64)
    L.ora_encode_expand_lut(P(out), N, P(tab), len(tab), out_bits, int(signed))
    return out


def trivial_glwe(p: Params, lut_poly):
    g = np.zeros((p.k + 1) * p.N, dtype=np.uint64)
    g[p.k * p.N:] = lut_poly
    return g


class Rng:
    """numpy-side wrapper around the C xoshiro256** stream (so Python and C agree)."""

    def __init__(self, seed):
        self._r = (C.c_uint64 * 6)()
        lib().ora_rng_seed(C.byref(self._r), C.c_uint64(seed))
        lib().ora_rng_u64.restype = C.c_uint64

    def u64(self):
        return lib().ora_rng_u64(C.byref(self._r))


def binary_key(length, seed):
    sk = np.zeros(length, dtype=np.uint64)
    r = (C.c_uint64 * 6)()
    lib().ora_rng_seed(C.byref(r), C.c_uint64(seed))
    lib().ora_binary_key(P(sk), C.c_size_t(length), C.byref(r))
    return sk


def lwe_encrypt_batch(sk, msgs_encoded, n, std, seed):
    L = lib()
    B = len(msgs_encoded)
    out = np.zeros((B, n + 1), dtype=np.uint64)
    r = (C.c_uint64 * 6)()
    L.ora_rng_seed(C.byref(r), C.c_uint64(seed))
    L.ora_lwe_encrypt.argtypes = [u64p, u64p, C.c_uint64, sz, C.c_double, C.c_void_p]
    for i in range(B):
        row = out[i]
        L.ora_lwe_encrypt(P(sk), row.ctypes.data_as(u64p), C.c_uint64(int(msgs_encoded[i])), n, std, C.byref(r))
    return out


def lwe_decrypt_batch(sk, cts, n):
    L = lib()
    L.ora_lwe_decrypt.argtypes = [u64p, u64p, sz]
    return np.array([L.ora_lwe_decrypt(P(sk), cts[i].ctypes.data_as(u64p), n) for i in range(cts.shape[0])],
                    dtype=np.uint64)
