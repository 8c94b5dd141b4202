"""BASELINE configs[0] (the README's add(x, y)) and the reference's other leveled single-op cases,
encrypted and run through the four cuda_*_lwe_ciphertext_vector_64 entry points on the GPU
(linear.hip; GPUDFG.cpp:1286-1447), decrypting to the reference's expected outputs
(tests/golden/reference_leveled_fixtures.json, lowering in tests/leveled_cases.py).  Precisions
up to 55 bits: a 4096-word LWE key at the 128-bit curve's noise floor (2^-62)."""
import numpy as np
import pytest

import leveled_cases as LC

pytestmark = pytest.mark.gpu

N_LWE = 4096
MASK = (1 << 64) - 1


def test_reference_leveled_cases_through_linear_ops():
    import torch
    assert torch.cuda.is_available()
    from concrete_amd import _native
    from concrete_amd import backend as B
    L = _native.lib()
    dev = "cuda:0"
    s = torch.cuda.current_stream().cuda_stream
    sk = B.binary_key(N_LWE, 909)
    std = B.secure_std(1, N_LWE)
    cases = LC.load()
    got, want = [], []
    for ci, c in enumerate(cases):
        p = c["precision"]
        encs, _ = LC.operands(c)
        cts = B.lwe_encrypt(sk, [B.encode(m, p) for m in encs], N_LWE, std, 10_000 + ci)
        regs = [B.to_device(cts[i:i + 1], dev) for i in range(len(encs))]
        for st in LC.program(c):
            out = torch.empty((1, N_LWE + 1), dtype=torch.int64, device=dev)
            if st[0] == "add":
                L.cuda_add_lwe_ciphertext_vector_64(s, 0, out.data_ptr(), regs[st[1]].data_ptr(),
                                                    regs[st[2]].data_ptr(), N_LWE, 1)
            elif st[0] == "add_pt":
                pt = B.to_device(np.array([int(B.encode(st[2] % (1 << (p + 1)), p))], dtype=np.uint64), dev)
                L.cuda_add_lwe_ciphertext_vector_plaintext_vector_64(s, 0, out.data_ptr(), regs[st[1]].data_ptr(),
                                                                     pt.data_ptr(), N_LWE, 1)
            elif st[0] == "mul":
                cl = B.to_device(np.array([st[2] & MASK], dtype=np.uint64), dev)
                L.cuda_mult_lwe_ciphertext_vector_cleartext_vector_64(s, 0, out.data_ptr(), regs[st[1]].data_ptr(),
                                                                      cl.data_ptr(), N_LWE, 1)
            else:
                L.cuda_negate_lwe_ciphertext_vector_64(s, 0, out.data_ptr(), regs[st[1]].data_ptr(), N_LWE, 1)
            regs.append(out)
        torch.cuda.synchronize()
        res = B.to_host(regs[-1])
        got.append(B.decode(B.lwe_decrypt(sk, res, N_LWE)[0], p))
        want.append(c["expected"])
    bad = [(c["description"], g, w) for c, g, w in zip(cases, got, want) if g != w]
    assert not bad, bad[:10]
