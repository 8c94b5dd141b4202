"""Restatement of the reference noise model for the PBS path (TEST INFRASTRUCTURE ONLY).

Follows backends/concrete-cpu/noise-model/src/gaussian_noise/noise/external_product_glwe.rs:4-89,
blind_rotate.rs:8-28, conversion.rs, and tools/parameter-curves/concrete-security-curves-rust
src/gaussian/security.rs:29-45 + security_weights.rs:9-23 (128-bit weights from curves_gen.rs).
Pinned by the reference's own golden unit tests (blind_rotate.rs:38-109) in tests/test_oracle.py.
"""
from __future__ import annotations

import math

FFT_SCALING_WEIGHT = -2.577_224_94  # external_product_glwe.rs:71
WEIGHTS = {128: (-0.025696778711484593, 2.675931372549016, 450),
           132: (-0.024891456582633045, 2.65734593837534, 450)}


def secure_log2_std(lwe_dimension: int, log_q: float, security: int = 128) -> float:
    slope, bias, min_dim = WEIGHTS[security]
    eps = 2.0 - log_q
    if min_dim <= lwe_dimension:
        return max(slope * lwe_dimension + bias, eps)
    return log_q


def minimal_variance_glwe(glwe_dim: int, poly_size: int, log_q: int, security: int = 128) -> float:
    return 2.0 ** (2.0 * secure_log2_std(glwe_dim * poly_size, float(log_q), security))


def modular_variance_to_variance(mv: float, log_q: int) -> float:
    return mv / 2.0 ** (2 * log_q)


def variance_to_modular_variance(v: float, log_q: int) -> float:
    return v * 2.0 ** (2 * log_q)


def theoretical_variance_external_product_glwe(k, N, log2_base, level, log_q, variance_ggsw):
    var_key_bin = modular_variance_to_variance(1.0 / 4.0, log_q)
    sq_exp_key_bin = modular_variance_to_variance((1.0 / 2.0) ** 2, log_q)
    b = 2.0 ** log2_base
    b2l = 2.0 ** (log2_base * 2 * level)
    q2 = 2.0 ** (2 * log_q)
    res_1 = level * (k + 1.0) * N * (b * b + 2.0) / 12.0 * variance_ggsw
    res_2 = ((q2 - b2l) / (24.0 * b2l) * (modular_variance_to_variance(1.0, log_q)
                                          + k * N * (var_key_bin + sq_exp_key_bin))
             + k * N / 8.0 * var_key_bin
             + 1.0 / 16.0 * (1.0 - k * N) ** 2 * sq_exp_key_bin)
    return res_1 + res_2


def fft_noise_variance_external_product_glwe(k, N, log2_base, level, log_q, fft_precision):
    b = 2.0 ** log2_base
    lost_bits = log_q - fft_precision
    scale_margin = 2.0 ** (2 * lost_bits)
    res = 2.0 ** FFT_SCALING_WEIGHT * scale_margin * level * b * b * N ** 2 * (k + 1.0)
    return modular_variance_to_variance(res, log_q)


def variance_blind_rotate(n, k, N, log2_base, level, log_q, fft_precision, variance_bsk, exact=False):
    """n * variance_cmux; exact=True drops the FFT term (this backend's arithmetic is exact)."""
    v = theoretical_variance_external_product_glwe(k, N, log2_base, level, log_q, variance_bsk)
    if not exact:
        v += fft_noise_variance_external_product_glwe(k, N, log2_base, level, log_q, fft_precision)
    return n * v
