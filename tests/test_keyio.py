"""Key wire-format import (include/concrete_hip.h Part 6, concrete_amd/csrc/keyio.cpp): CPU tests.

Parity unpinned: the reference holds no serialized keyset (no capnp library or fixture in the
image), so these tests pin the reader against (a) capnp's struct-layout rule recomputed here from
the schema's field lists (concrete-protocol.capnp:149-207), (b) round trips through the writer in
concrete_amd/keys.py in every pointer form capnp produces (near, single far, double far; one or
many segments and blobs), (c) refusal of malformed or unsupported messages, and (d) the seeded-key
hand-off to an installed concrete-cpu-signature decompressor.
"""
import ctypes as C
import struct

import numpy as np
import pytest

from concrete_amd import _native
from concrete_amd import keys as K


# ---- (a) capnp layout rule ------------------------------------------------------------------
def _capnp_layout(fields):
    """Byte offsets of data fields under capnp's allocation rule (fields in ordinal order, each in
    the first free hole of its size, splitting larger holes, else a new word).  fields: list of
    (name, bits) in ordinal order, bits = 0 for pointer fields.  Returns ({name: byte offset},
    data words)."""
    holes = {}  # lg size -> offset in units of that size
    words = 0
    out = {}

    def try_alloc(lg):
        if lg >= 6:
            return None
        if holes.get(lg):
            v = holes.pop(lg)
            return v
        nxt = try_alloc(lg + 1)
        if nxt is None:
            return None
        holes[lg] = nxt * 2 + 1
        return nxt * 2

    for name, bits in fields:
        if bits == 0:
            continue
        lg = {8: 3, 16: 4, 32: 5, 64: 6}[bits]
        off = try_alloc(lg)
        if off is None:
            off = words << (6 - lg)
            words += 1
            # the rest of the new word becomes holes of sizes lg .. 32 bits
            o, s = off + 1, lg
            while s < 6:
                holes[s] = o
                s += 1
                o = (o + 1) // 2
        out[name] = off * bits // 8
    return out, words


def test_schema_offsets_follow_capnp_layout():
    info, w = _capnp_layout([("id", 32), ("input_id", 32), ("output_id", 32), ("params", 0), ("compression", 16)])
    assert info == K.INFO_OFF and w == K.INFO_WORDS
    bsk, w = _capnp_layout([("level_count", 32), ("base_log", 32), ("glwe_dim", 32), ("poly_size", 32),
                            ("variance", 64), ("integer_precision", 32), ("modulus", 0), ("key_type", 16),
                            ("input_lwe_dim", 32)])
    assert bsk == K.BSK_PARAMS_OFF and w == K.BSK_PARAMS_WORDS
    ksk, w = _capnp_layout([("level_count", 32), ("base_log", 32), ("variance", 64), ("integer_precision", 32),
                            ("modulus", 0), ("key_type", 16), ("input_lwe_dim", 32), ("output_lwe_dim", 32)])
    assert ksk == K.KSK_PARAMS_OFF and w == K.KSK_PARAMS_WORDS


# ---- (b) round trips ------------------------------------------------------------------------
class _P:  # a small backend.PbsParams-like parameter set
    n, k, N, level, base_log, ks_level, ks_base_log = 5, 1, 16, 2, 7, 3, 4
    big_n = 16


def _keys(rng, n_bsk=2, n_ksk=1):
    bsks, ksks = [], []
    for i in range(n_bsk):
        info = K.bsk_info(_P, id=i, input_id=2 * i, output_id=2 * i + 1, variance=2.0 ** -60 * (i + 1))
        bsks.append((info, rng.integers(0, 2 ** 64, size=info.bsk_words(), dtype=np.uint64)))
    for i in range(n_ksk):
        info = K.ksk_info(_P, id=10 + i, input_id=1, output_id=0, variance=2.0 ** -30, key_type=0)
        ksks.append((info, rng.integers(0, 2 ** 64, size=info.ksk_words(), dtype=np.uint64)))
    return bsks, ksks


def _check(sk, bsks, ksks):
    assert len(sk.bootstrap_keys) == len(bsks) and len(sk.keyswitch_keys) == len(ksks)
    for i, (info, payload) in enumerate(bsks):
        got = sk.bootstrap_keys[i]
        for f in ("id", "input_id", "output_id", "level_count", "base_log", "glwe_dim", "poly_size",
                  "input_lwe_dim", "integer_precision", "key_type", "compression", "variance"):
            assert getattr(got, f) == getattr(info, f), f
        assert got.output_lwe_dim == info.glwe_dim * info.poly_size
        assert got.payload_words == payload.size == got.key_words
        assert np.array_equal(sk.bsk(i), payload)
    for i, (info, payload) in enumerate(ksks):
        got = sk.keyswitch_keys[i]
        for f in ("id", "input_id", "output_id", "level_count", "base_log", "input_lwe_dim", "output_lwe_dim",
                  "integer_precision", "variance"):
            assert getattr(got, f) == getattr(info, f), f
        assert np.array_equal(sk.ksk(i), payload)


@pytest.mark.parametrize("layout", ["flat", "single_far", "double_far", "mixed"])
@pytest.mark.parametrize("blob_words", [K.BLOB_WORDS, 7])
def test_server_keyset_round_trip(layout, blob_words):
    rng = np.random.default_rng(1)
    bsks, ksks = _keys(rng)
    data = K.serialize_server_keyset(bsks, ksks, layout=layout, blob_words=blob_words)
    nseg = struct.unpack_from("<I", data)[0] + 1
    assert (nseg == 1) == (layout == "flat")
    _check(K.ServerKeyset.deserialize(data), bsks, ksks)


def test_keyset_and_single_key_roots(tmp_path):
    rng = np.random.default_rng(2)
    bsks, ksks = _keys(rng, 1, 2)
    _check(K.ServerKeyset.deserialize(K.serialize_server_keyset(bsks, ksks, root="keyset", layout="mixed"),
                                      root="keyset"), bsks, ksks)
    one = K.serialize_server_keyset(bsks, root="bootstrap_key", layout="single_far")
    _check(K.ServerKeyset.deserialize(one, root="bootstrap_key"), bsks, [])
    one = K.serialize_server_keyset(ksks=ksks[1:], root="keyswitch_key")
    _check(K.ServerKeyset.deserialize(one, root="keyswitch_key"), [], ksks[1:])
    path = tmp_path / "server.keys"
    path.write_bytes(K.serialize_server_keyset(bsks, ksks, layout="double_far"))
    _check(K.ServerKeyset.load(path), bsks, ksks)
    empty = K.ServerKeyset.deserialize(K.serialize_server_keyset())
    assert empty.bootstrap_keys == [] and empty.keyswitch_keys == []


def test_unaligned_input_is_copied():
    rng = np.random.default_rng(3)
    bsks, ksks = _keys(rng, 1, 1)
    data = K.serialize_server_keyset(bsks, ksks)
    buf = np.zeros(len(data) + 8, dtype=np.uint8)
    raw = buf[1:1 + len(data)]
    raw[:] = np.frombuffer(data, dtype=np.uint8)
    lib = _native.lib()
    h = C.c_void_p()
    _native.check(lib.concrete_hip_server_keyset_deserialize(raw.ctypes.data, len(data), 0, C.byref(h)), "deser")
    sk = K.ServerKeyset(h.value)
    _check(sk, bsks, ksks)


# ---- (c) refusals -----------------------------------------------------------------------------
def _deser_rc(data: bytes, root=0):
    lib = _native.lib()
    h = C.c_void_p()
    buf = np.frombuffer(data, dtype=np.uint8).copy() if data else np.zeros(8, np.uint8)
    rc = lib.concrete_hip_server_keyset_deserialize(buf.ctypes.data, len(data), root, C.byref(h))
    if rc == 0:
        lib.concrete_hip_server_keyset_destroy(h.value)
    return rc


def test_malformed_messages_are_refused():
    rng = np.random.default_rng(4)
    bsks, ksks = _keys(rng, 1, 1)
    good = K.serialize_server_keyset(bsks, ksks, layout="mixed")
    assert _deser_rc(good) == 0
    assert _deser_rc(b"") < 0
    assert _deser_rc(good[:-8]) < 0  # last segment truncated
    assert _deser_rc(good[:-3]) < 0  # not whole words
    assert _deser_rc(struct.pack("<II", 10000, 1) + b"\0" * 8) < 0  # absurd segment count
    # root pointer aimed past the segment
    bad = bytearray(good)
    nseg = struct.unpack_from("<I", bad)[0] + 1
    hdr = ((4 * (1 + nseg) + 7) // 8) * 8
    struct.pack_into("<Q", bad, hdr, (0x1000 << 2) | (3 << 48))
    assert _deser_rc(bytes(bad)) < 0
    # a far pointer into a segment that does not exist
    struct.pack_into("<Q", bad, hdr, 2 | (0 << 3) | (77 << 32))
    assert _deser_rc(bytes(bad)) < 0
    # a capability pointer as root
    struct.pack_into("<Q", bad, hdr, 3)
    assert _deser_rc(bytes(bad)) < 0
    assert _deser_rc(good, root=9) < 0


def test_unsupported_and_mismatched_keys_are_refused():
    rng = np.random.default_rng(5)
    (info, payload), = _keys(rng, 1, 0)[0]
    short = K.serialize_server_keyset([(info, payload[:-1])])
    sk = K.ServerKeyset.deserialize(short)  # parses: sizes are checked when the key is read
    with pytest.raises(RuntimeError, match="payload has"):
        sk.bsk(0)
    info32 = K.KeyInfo(**{**info.__dict__, "integer_precision": 32})
    sk = K.ServerKeyset.deserialize(K.serialize_server_keyset([(info32, payload)]))
    with pytest.raises(RuntimeError, match="64-bit"):
        sk.bsk(0)
    pow2 = K.KeyInfo(**{**info.__dict__, "modulus_kind": 1, "modulus_value": 62})
    sk = K.ServerKeyset.deserialize(K.serialize_server_keyset([(pow2, payload)]))
    assert sk.bootstrap_keys[0].modulus_kind == 1 and sk.bootstrap_keys[0].modulus_value == 62
    with pytest.raises(RuntimeError, match="native modulus"):
        sk.bsk(0)


# ---- (d) seeded keys --------------------------------------------------------------------------
class _U128(C.Structure):
    _fields_ = [("little_endian_bytes", C.c_uint8 * 16)]


_BSK_DEC = C.CFUNCTYPE(None, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_size_t, C.c_size_t, C.c_size_t,
                       C.c_size_t, C.c_size_t, _U128, C.c_uint32)
_KSK_DEC = C.CFUNCTYPE(None, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_size_t, C.c_size_t, C.c_size_t,
                       C.c_size_t, _U128, C.c_uint32)


def test_seeded_keys_use_the_installed_decompressors():
    lib = _native.lib()
    calls = []

    def fake_mask(seed_bytes, i):  # stand-in for concrete-csprng's mask stream (test only)
        return (int.from_bytes(seed_bytes, "little") * 0x9E3779B97F4A7C15 + i) % 2 ** 64

    @_BSK_DEC
    def bsk_dec(out, seeded, n, N, k, l, logB, seed, par):
        sb = bytes(seed.little_endian_bytes)
        calls.append(("bsk", n, N, k, l, logB, sb, par))
        # standard layout [n][l][k+1 rows][k+1 polys][N]: masks from the "stream", bodies copied
        body = 0
        for row in range(n * l * (k + 1)):
            for poly in range(k + 1):
                for c in range(N):
                    dst = (row * (k + 1) + poly) * N + c
                    if poly == k:
                        out[dst] = seeded[body]
                        body += 1
                    else:
                        out[dst] = fake_mask(sb, dst)

    @_KSK_DEC
    def ksk_dec(out, seeded, n_in, n_out, l, logB, seed, par):
        sb = bytes(seed.little_endian_bytes)
        calls.append(("ksk", n_in, n_out, l, logB, sb, par))
        for row in range(n_in * l):
            for c in range(n_out):
                out[row * (n_out + 1) + c] = fake_mask(sb, row * (n_out + 1) + c)
            out[row * (n_out + 1) + n_out] = seeded[row]

    rng = np.random.default_rng(6)
    bi = K.bsk_info(_P, compression=1)
    ki = K.ksk_info(_P, compression=1)
    seed = [0x0706050403020100, 0x0F0E0D0C0B0A0908]  # writeSeed: byte b at word b // 8, bits 8 (b % 8)
    b_bodies = rng.integers(0, 2 ** 64, size=_P.n * _P.level * (_P.k + 1) * _P.N, dtype=np.uint64)
    k_bodies = rng.integers(0, 2 ** 64, size=_P.big_n * _P.ks_level, dtype=np.uint64)
    data = K.serialize_server_keyset([(bi, np.concatenate([np.array(seed, np.uint64), b_bodies]))],
                                     [(ki, np.concatenate([np.array(seed, np.uint64), k_bodies]))])
    sk = K.ServerKeyset.deserialize(data)
    assert sk.bootstrap_keys[0].compression == 1
    assert sk.bootstrap_keys[0].payload_words == 2 + b_bodies.size
    assert sk.bootstrap_keys[0].key_words == bi.bsk_words()
    lib.concrete_hip_set_seeded_key_decompressors(None, None)
    with pytest.raises(RuntimeError, match="seeded"):
        sk.bsk(0)
    lib.concrete_hip_set_seeded_key_decompressors(C.cast(bsk_dec, C.c_void_p), C.cast(ksk_dec, C.c_void_p))
    try:
        b = sk.bsk(0).reshape(_P.n * _P.level * (_P.k + 1), _P.k + 1, _P.N)
        kk = sk.ksk(0).reshape(_P.big_n * _P.ks_level, _P.n + 1)
    finally:
        lib.concrete_hip_set_seeded_key_decompressors(None, None)
    sb = bytes(range(16))
    assert calls[0] == ("bsk", _P.n, _P.N, _P.k, _P.level, _P.base_log, sb, 1)
    assert calls[1] == ("ksk", _P.big_n, _P.n, _P.ks_level, _P.ks_base_log, sb, 1)
    assert np.array_equal(b[:, _P.k, :].ravel(), b_bodies)
    assert int(b[0, 0, 3]) == fake_mask(sb, 3)
    assert np.array_equal(kk[:, _P.n], k_bodies)
    # a seeded payload of the wrong size is refused before the decompressor runs
    bad = K.serialize_server_keyset([(bi, np.concatenate([np.array(seed, np.uint64), b_bodies[:-1]]))])
    with pytest.raises(RuntimeError, match="seeded payload"):
        K.ServerKeyset.deserialize(bad).bsk(0)


# ---- (e) the C boundary ------------------------------------------------------------------------
def _fnv(words: np.ndarray) -> int:
    h = 1469598103934665603
    for w in words.tolist():
        h = ((h ^ w) * 1099511628211) % 2 ** 64
    return h


def test_c_client_reads_the_same_keys(tmp_path):
    """tests/c_client/keyio_client.c (C99) loads the file and reports every key's info and a
    checksum of its words: the C struct layout and the ctypes one agree."""
    import os
    import shutil
    import subprocess
    if shutil.which("gcc") is None:
        pytest.skip("gcc not installed")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    libdir = os.path.join(root, "concrete_amd")
    exe = tmp_path / "keyio_client"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(root, "include"),
                    os.path.join(root, "tests", "c_client", "keyio_client.c"), "-L", libdir, "-lconcrete_hip",
                    f"-Wl,-rpath,{libdir}", "-o", str(exe)], check=True)
    rng = np.random.default_rng(7)
    bsks, ksks = _keys(rng, 2, 2)
    path = tmp_path / "server.keys"
    path.write_bytes(K.serialize_server_keyset(bsks, ksks, layout="mixed", blob_words=9))
    out = subprocess.run([str(exe), str(path)], check=True, capture_output=True, text=True, timeout=60).stdout
    want = []
    for kind, keys in (("bsk", bsks), ("ksk", ksks)):
        for i, (info, payload) in enumerate(keys):
            n_out = info.glwe_dim * info.poly_size if kind == "bsk" else info.output_lwe_dim
            want.append(f"{kind} {i} {info.id} {info.level_count} {info.base_log} {info.glwe_dim} {info.poly_size} "
                        f"{info.input_lwe_dim} {n_out} {info.compression} {payload.size} {_fnv(payload)}")
    assert out.split("\n")[:-1] == want
    bad = tmp_path / "bad.keys"
    bad.write_bytes(path.read_bytes()[:-8])
    r = subprocess.run([str(exe), str(bad)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "segment" in r.stderr


def test_aliased_blobs_cannot_amplify_the_payload():
    """A crafted List(Data) whose many pointers all name one blob would make a naive reader
    allocate (pointers x blob) bytes; the reader caps a payload at the message's own size."""
    m = K._Message("flat")
    key = m.new_struct(0, 2)
    m.set_root(key)
    info = K.bsk_info(_P)
    inf = m.new_struct(K.INFO_WORDS, 1)
    par = m.new_struct(K.BSK_PARAMS_WORDS, 1)
    for name, off in K.BSK_PARAMS_OFF.items():
        fmt = "d" if name == "variance" else ("H" if name == "key_type" else "I")
        m.set_data(par, off, fmt, getattr(info, name))
    m.set_struct_ptr(inf, 0, par)
    m.set_struct_ptr(key, 0, inf)
    pl = m.new_struct(0, 1)
    n_ptr = 4096
    plist = m.new_ptr_list(n_ptr)
    blob = m.new_data(b"\x01" * 4096)
    for b in range(n_ptr):
        m.set_list_elem_ptr(plist, b, blob)  # every element points at the same 4 KB
    m.set_list_ptr(pl, 0, plist)
    m.set_struct_ptr(key, 1, pl)
    data = m.to_bytes()
    assert len(data) < 64 * 1024  # 16 MB of payload if the aliases were followed
    assert _deser_rc(data, root=2) < 0
    assert "aliased" in _native.lib().concrete_hip_last_error().decode()


def test_many_keys_sharing_one_payload_are_refused():
    """the aliasing cap was per key, so a composite list of K keys naming one payload
    could allocate ~K x message bytes; the budget is now one per parse."""
    m = K._Message("flat")
    srv = m.new_struct(0, 3)
    m.set_root(srv)
    n_keys = 64
    lst, elems = m.new_struct_list(n_keys, 0, 2)
    m.set_list_ptr(srv, 0, lst)
    info = K.bsk_info(_P)
    inf = m.new_struct(K.INFO_WORDS, 1)
    par = m.new_struct(K.BSK_PARAMS_WORDS, 1)
    for name, off in K.BSK_PARAMS_OFF.items():
        fmt = "d" if name == "variance" else ("H" if name == "key_type" else "I")
        m.set_data(par, off, fmt, getattr(info, name))
    m.set_struct_ptr(inf, 0, par)
    pl = m.new_struct(0, 1)
    plist = m.new_ptr_list(1)
    m.set_list_elem_ptr(plist, 0, m.new_data(b"\x02" * 4096))
    m.set_list_ptr(pl, 0, plist)
    for el in elems:  # every key: the same info, the same 4 KB payload
        m.set_struct_ptr(el, 0, inf)
        m.set_struct_ptr(el, 1, pl)
    data = m.to_bytes()
    assert len(data) < 8 * 1024  # 256 KB of payload copies if every alias were followed
    assert _deser_rc(data) < 0
    assert "payloads total" in _native.lib().concrete_hip_last_error().decode()


@pytest.mark.parametrize("dims,msg", [
    # u32 products that wrapped to a tiny size before round 4
    ({"input_lwe_dim": 1 << 31, "level_count": 2, "base_log": 2, "glwe_dim": 1, "poly_size": 4}, "out of range"),
    ({"input_lwe_dim": 8, "level_count": 1 << 31, "base_log": 2, "glwe_dim": 1, "poly_size": 4}, "out of range"),
    ({"input_lwe_dim": 8, "level_count": 2, "base_log": 7, "glwe_dim": 1, "poly_size": 3}, "out of range"),
    # within every per-dimension bound, but the product exceeds the size bound
    ({"input_lwe_dim": 1 << 20, "level_count": 16, "base_log": 4, "glwe_dim": 64, "poly_size": 1 << 17}, "overflows"),
])
def test_key_dimensions_are_bounded_before_anything_is_sized(dims, msg):
    """A seeded key whose dimensions make its size wrap would have passed the 2-word payload check
    and let the decompressor write the real size through a short buffer: the dimensions are now
    bounded and the sizes computed with overflow checks when the message is parsed."""
    info = K.KeyInfo(**{**K.bsk_info(_P, compression=1).__dict__, **dims})
    data = K.serialize_server_keyset([(info, np.array([1, 2], np.uint64))])
    assert _deser_rc(data) < 0
    assert msg in _native.lib().concrete_hip_last_error().decode()


def test_keyswitch_support_is_checked_before_expansion():
    """keyset_add_server_keyset checks every key's parameters against the kernels before any key is
    expanded (a decompressor never runs for a key the keyset would refuse)."""
    lib = _native.lib()
    assert lib.concrete_hip_keyswitch_supported(_P.ks_level, _P.ks_base_log, _P.big_n, _P.n) == 1
    assert lib.concrete_hip_keyswitch_supported(23, 1, 16384, 1006) == 1  # v0_last_128 9-bit log-norm2 16
    assert lib.concrete_hip_keyswitch_supported(16, 4, 1024, 600) == 0   # 64 bits of digits
    assert lib.concrete_hip_keyswitch_supported(2, 4, 1024, 65535) == 1
    assert lib.concrete_hip_keyswitch_supported(2, 4, 1024, 65536) == 0
    assert lib.concrete_hip_keyswitch_supported(2, 4, 1024, 0xFFFFFFFF) == 0  # n_out + 1 wraps in u32


# ---- (f) level orders, checked against the client secret keys of a Keyset message ---------------
def _reverse_levels(key: np.ndarray, n: int, l: int) -> np.ndarray:
    return key.reshape(n, l, -1)[:, ::-1, :].copy().ravel()


def test_level_order_checked_against_client_keys():
    """the GGSW level order (level 1 first, keygen.cpp) and the keyswitch key's
    reversed levels are restated, not pinned.  A Keyset message carries the client secret keys, so
    on read one row per level is decrypted: a key in the expected order passes, a level-reversed key
    is detected and re-ordered, one that decrypts in neither order is refused, and a ServerKeyset
    (no secret keys) stays unchecked."""
    from dataclasses import dataclass

    from concrete_amd import backend as B

    @dataclass
    class P:
        n: int = 12
        k: int = 2
        N: int = 64
        level: int = 3
        base_log: int = 7
        ks_level: int = 4
        ks_base_log: int = 5

        @property
        def big_n(self):
            return self.k * self.N

        bsk_len = property(lambda s: s.n * s.level * (s.k + 1) ** 2 * s.N)
        ksk_len = property(lambda s: s.big_n * s.ks_level * (s.n + 1))

    p = P()
    lwe_sk = B.binary_key(p.n, 31)
    glwe_sk = B.binary_key(p.big_n, 32)
    assert lwe_sk.any() and glwe_sk.any()
    bsk = B.bsk_generate(p, lwe_sk, glwe_sk, 33, std=2.0 ** -45)
    ksk = B.ksk_generate(p, glwe_sk, lwe_sk, 34, std=2.0 ** -45)
    var = (2.0 ** -45) ** 2  # every level's scale is far above this noise: all levels are compared
    bi = [K.bsk_info(p, id=i, input_id=0, output_id=1, variance=var) for i in range(3)]
    ki = [K.ksk_info(p, id=10 + i, input_id=1, output_id=0, variance=var) for i in range(3)]
    rng = np.random.default_rng(35)
    junk_b = rng.integers(0, 2 ** 64, size=bsk.size, dtype=np.uint64)
    junk_k = rng.integers(0, 2 ** 64, size=ksk.size, dtype=np.uint64)
    bsks = [(bi[0], bsk), (bi[1], _reverse_levels(bsk, p.n, p.level)), (bi[2], junk_b)]
    ksks = [(ki[0], ksk), (ki[1], _reverse_levels(ksk, p.big_n, p.ks_level)), (ki[2], junk_k)]
    data = K.serialize_server_keyset(bsks, ksks, root="keyset", layout="mixed", secrets=[(0, lwe_sk), (1, glwe_sk)])
    sk = K.ServerKeyset.deserialize(data, "keyset")
    assert sk.secret_count == 2
    assert sk.level_order("bsk", 0) == "unchecked"  # not read yet
    assert np.array_equal(sk.bsk(0), bsk) and sk.level_order("bsk", 0) == "as_expected"
    assert np.array_equal(sk.bsk(1), bsk) and sk.level_order("bsk", 1) == "reversed"
    assert np.array_equal(sk.ksk(0), ksk) and sk.level_order("ksk", 0) == "as_expected"
    assert np.array_equal(sk.ksk(1), ksk) and sk.level_order("ksk", 1) == "reversed"
    for kind in ("bsk", "ksk"):
        with pytest.raises(RuntimeError, match="in either level order"):
            getattr(sk, kind)(2)
    # the same keys in a ServerKeyset message: nothing to check against
    srv = K.ServerKeyset.deserialize(K.serialize_server_keyset(bsks[:2], ksks[:2]))
    assert srv.secret_count == 0
    assert np.array_equal(srv.bsk(1), bsks[1][1]) and srv.level_order("bsk", 1) == "unchecked"


@pytest.mark.parametrize("name,n,l,logb", [
    ("cfg4_ks", 742, 5, 3),    # BASELINE configs[3]'s keyswitch: deepest level at the noise floor
    ("opt7_ks", 915, 5, 3),    # v0_last_128 7-bit row's keyswitch
    ("v0_l23", 880, 23, 1),    # 23 levels of 1 bit: most levels below the noise
])
def test_level_order_at_secure_noise(name, n, l, logb):
    """keys generated at the secure noise (secure_std(1, n), the KSK's output
    dimension) put the deepest keyswitch levels at or below the noise floor.  The order is decided by
    the most significant level, deeper levels are compared only where their scale clears 64 sigma of
    the key's variance: such keys read back 'as_expected', and their level-reversed copies
    'reversed' (re-ordered), whatever the noise draws."""
    from dataclasses import dataclass

    from concrete_amd import backend as B

    @dataclass
    class P:
        n: int
        k: int
        N: int
        ks_level: int
        ks_base_log: int

        @property
        def big_n(self):
            return self.k * self.N

        ksk_len = property(lambda s: s.big_n * s.ks_level * (s.n + 1))

    # only the first 64 input positions carry key rows here (the check reads up to 16 positions
    # whose secret bit is 1); the rest of the key is irrelevant to the level order
    p = P(n=n, k=1, N=64, ks_level=l, ks_base_log=logb)
    std = B.secure_std(1, n)
    glwe_sk = B.binary_key(p.big_n, 41)
    lwe_sk = B.binary_key(n, 42)
    ksk = B.ksk_generate(p, glwe_sk, lwe_sk, 43, std=std)
    info = [K.KeyInfo(id=i, input_id=1, output_id=0, level_count=l, base_log=logb, input_lwe_dim=p.big_n,
                      output_lwe_dim=n, variance=std * std) for i in range(2)]
    rev = _reverse_levels(ksk, p.big_n, l)
    data = K.serialize_server_keyset([], [(info[0], ksk), (info[1], rev)], root="keyset", layout="mixed",
                                     secrets=[(0, lwe_sk), (1, glwe_sk)])
    sk = K.ServerKeyset.deserialize(data, "keyset")
    assert np.array_equal(sk.ksk(0), ksk) and sk.level_order("ksk", 0) == "as_expected"
    assert np.array_equal(sk.ksk(1), ksk) and sk.level_order("ksk", 1) == "reversed"
