"""GPU tests of the four LWE linear-operation vectors (concrete_amd/csrc/linear.hip;
compiler lib/Runtime/GPUDFG.cpp:1286-1446): exact wrapping u64 results vs numpy, and the
homomorphic meaning checked by decryption."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    from concrete_amd import _native
    from concrete_amd import backend as B
    return torch, _native.lib(), B


def _run(env, fn, *arrays, n, count, extra_in=None):
    torch, L, B = env
    dev = "cuda:0"
    ins = [B.to_device(a, dev) for a in arrays]
    out = torch.zeros((count, n + 1), dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    getattr(L, fn)(s, 0, out.data_ptr(), *[t.data_ptr() for t in ins], n, count)
    torch.cuda.synchronize()
    return B.to_host(out)


@pytest.mark.parametrize("n,count", [(630, 1), (630, 37), (2048, 300), (1, 5)])
def test_linear_ops_exact(env, n, count):
    rng = np.random.default_rng(n + count)
    a = rng.integers(0, 2 ** 64, size=(count, n + 1), dtype=np.uint64)
    b = rng.integers(0, 2 ** 64, size=(count, n + 1), dtype=np.uint64)
    p = rng.integers(0, 2 ** 64, size=count, dtype=np.uint64)
    c = rng.integers(0, 2 ** 64, size=count, dtype=np.uint64)
    with np.errstate(over="ignore"):
        assert np.array_equal(_run(env, "cuda_add_lwe_ciphertext_vector_64", a, b, n=n, count=count), a + b)
        ref = a.copy()
        ref[:, n] += p
        assert np.array_equal(_run(env, "cuda_add_lwe_ciphertext_vector_plaintext_vector_64", a, p, n=n, count=count), ref)
        assert np.array_equal(_run(env, "cuda_mult_lwe_ciphertext_vector_cleartext_vector_64", a, c, n=n, count=count),
                              a * c[:, None])
        assert np.array_equal(_run(env, "cuda_negate_lwe_ciphertext_vector_64", a, n=n, count=count),
                              (np.uint64(0) - a))


def test_linear_ops_decrypt(env):
    """Enc(m1) + Enc(m2), Enc(m) + encode(p), Enc(m) * c, -Enc(m) decrypt to the cleartext results."""
    torch, L, B = env
    n, width = 630, 4
    sk = B.binary_key(n, 5)
    m1 = np.array([1, 2, 3, 4, 5, 6])
    m2 = np.array([2, 2, 7, 0, 1, 3])
    ct1 = B.lwe_encrypt(sk, [B.encode(m, width) for m in m1], n, 2.0 ** -30, 11)
    ct2 = B.lwe_encrypt(sk, [B.encode(m, width) for m in m2], n, 2.0 ** -30, 12)
    dec = lambda cts: [B.decode(d, width) for d in B.lwe_decrypt(sk, cts, n)]
    k = len(m1)
    assert dec(_run(env, "cuda_add_lwe_ciphertext_vector_64", ct1, ct2, n=n, count=k)) == list((m1 + m2) % 16)
    pts = np.array([B.encode(int(x), width) for x in m2], dtype=np.uint64)
    assert dec(_run(env, "cuda_add_lwe_ciphertext_vector_plaintext_vector_64", ct1, pts, n=n, count=k)) == \
        list((m1 + m2) % 16)
    cl = np.array([1, 2, 3, 1, 2, 2], dtype=np.uint64)
    assert dec(_run(env, "cuda_mult_lwe_ciphertext_vector_cleartext_vector_64", ct1, cl, n=n, count=k)) == \
        list((m1 * cl.astype(np.int64)) % 16)
    # the encoding keeps a padding bit: -m decodes modulo 2^(width + 1)
    assert dec(_run(env, "cuda_negate_lwe_ciphertext_vector_64", ct1, n=n, count=k)) == list((-m1) % 32)
