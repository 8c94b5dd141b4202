"""Key wire format: concrete keysets as Cap'n Proto messages.

Reading is native (``concrete_amd/csrc/keyio.cpp``, include/concrete_hip.h Part 6): a server
keyset written by the reference's ``ServerKeyset.serialize()`` / ``Keyset.serialize()``
(capnp::writeMessage, compiler include/concretelang/Common/Protocol.h:158-175; schema
tools/concrete-protocol/src/concrete-protocol.capnp:149-297) loads into a runtime keyset under
the list positions the runtime context indexes keys by (lib/Runtime/context.cpp:36-94).

Writing (``serialize_server_keyset``) is the host-side mirror of ``ServerKeyset::toProto`` +
``vectorToProtoPayload`` (lib/Common/Keysets.cpp, Protocol.h:274-317): the payload is split into
``Data`` blobs of at most MAX_TEXT_SIZE bytes.  It can lay objects out in one segment or behind
single / double far pointers, the forms capnp's MallocMessageBuilder produces for large keys, so
the reader's handling of each is exercised (tests/test_keyio.py).

The field offsets (bytes in each struct's data section) follow capnp's layout rule for the
schema's ordinals; tests/test_keyio.py recomputes them with that rule.
"""
from __future__ import annotations

import ctypes as C
import struct
from dataclasses import dataclass, fields

import numpy as np

from . import _native

ROOTS = {"server": 0, "keyset": 1, "bootstrap_key": 2, "keyswitch_key": 3}
# capnp::MAX_TEXT_SIZE (2^29 - 2 bytes); vectorToProtoPayload stores this many u64 per blob
BLOB_WORDS = (2 ** 29 - 2) // 8

# data-section byte offsets (concrete-protocol.capnp; see keyio.cpp)
INFO_OFF = {"id": 0, "input_id": 4, "output_id": 8, "compression": 12}
BSK_PARAMS_OFF = {"level_count": 0, "base_log": 4, "glwe_dim": 8, "poly_size": 12, "variance": 16,
                  "integer_precision": 24, "key_type": 28, "input_lwe_dim": 32}
KSK_PARAMS_OFF = {"level_count": 0, "base_log": 4, "variance": 8, "integer_precision": 16, "key_type": 20,
                  "input_lwe_dim": 24, "output_lwe_dim": 28}
INFO_WORDS, BSK_PARAMS_WORDS, KSK_PARAMS_WORDS = 2, 5, 4
# LweSecretKeyInfo: id u32 @0 (1 data word, params pointer); LweSecretKeyParams: lweDimension u32 @0,
# integerPrecision u32 @4, keyType u16 @8 (2 data words)
SK_INFO_WORDS, SK_PARAMS_WORDS = 1, 2
SK_PARAMS_OFF = {"lwe_dimension": 0, "integer_precision": 4, "key_type": 8}
# concrete_hip_server_keyset_level_order
LEVEL_ORDER = {0: "unchecked", 1: "as_expected", 2: "reversed"}


class _CKeyInfo(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in ("id", "input_id", "output_id", "level_count", "base_log", "glwe_dim",
                                          "poly_size", "input_lwe_dim", "output_lwe_dim", "integer_precision",
                                          "key_type", "compression", "modulus_kind", "modulus_value")] + [
        ("variance", C.c_double), ("payload_words", C.c_uint64), ("key_words", C.c_uint64)]


@dataclass
class KeyInfo:
    """concrete_hip_key_info: LweBootstrapKeyInfo / LweKeyswitchKeyInfo and their params."""
    id: int = 0
    input_id: int = 0
    output_id: int = 0
    level_count: int = 0
    base_log: int = 0
    glwe_dim: int = 0
    poly_size: int = 0
    input_lwe_dim: int = 0
    output_lwe_dim: int = 0
    integer_precision: int = 64
    key_type: int = 0
    compression: int = 0
    modulus_kind: int = 0
    modulus_value: int = 0
    variance: float = 0.0
    payload_words: int = 0
    key_words: int = 0

    @classmethod
    def _from_c(cls, c: _CKeyInfo) -> "KeyInfo":
        return cls(**{f.name: getattr(c, f.name) for f in fields(cls)})

    def bsk_words(self) -> int:  # concrete_cpu_bootstrap_key_size_u64
        g = self.glwe_dim + 1
        return self.input_lwe_dim * self.level_count * g * g * self.poly_size

    def ksk_words(self) -> int:  # concrete_cpu_keyswitch_key_size_u64
        return self.input_lwe_dim * self.level_count * (self.output_lwe_dim + 1)


def bsk_info(p, **kw) -> KeyInfo:
    """KeyInfo of a bootstrap key for backend.PbsParams p."""
    return KeyInfo(level_count=p.level, base_log=p.base_log, glwe_dim=p.k, poly_size=p.N, input_lwe_dim=p.n,
                   output_lwe_dim=p.k * p.N, **kw)


def ksk_info(p, **kw) -> KeyInfo:
    """KeyInfo of the keyswitch key kN -> n for backend.PbsParams p."""
    return KeyInfo(level_count=p.ks_level, base_log=p.ks_base_log, input_lwe_dim=p.big_n, output_lwe_dim=p.n, **kw)


class ServerKeyset:
    """Evaluation keys read from their wire form (concrete_hip_server_keyset)."""

    def __init__(self, handle):
        self.lib = _native.lib()
        self.h = handle
        n_b = self.lib.concrete_hip_server_keyset_bsk_count(self.h)
        n_k = self.lib.concrete_hip_server_keyset_ksk_count(self.h)
        self.bootstrap_keys = [self._info(self.lib.concrete_hip_server_keyset_bsk_info, i) for i in range(n_b)]
        self.keyswitch_keys = [self._info(self.lib.concrete_hip_server_keyset_ksk_info, i) for i in range(n_k)]

    def _info(self, fn, i) -> KeyInfo:
        c = _CKeyInfo()
        _native.check(fn(self.h, i, C.byref(c)), "server_keyset_info")
        return KeyInfo._from_c(c)

    @classmethod
    def deserialize(cls, data: bytes, root: str = "server") -> "ServerKeyset":
        lib = _native.lib()
        h = C.c_void_p()
        buf = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(0, np.uint8)
        _native.check(lib.concrete_hip_server_keyset_deserialize(buf.ctypes.data if len(buf) else None, len(buf),
                                                                 ROOTS[root], C.byref(h)), "server_keyset_deserialize")
        return cls(h.value)

    @classmethod
    def load(cls, path: str, root: str = "server") -> "ServerKeyset":
        lib = _native.lib()
        h = C.c_void_p()
        _native.check(lib.concrete_hip_server_keyset_load_file(str(path).encode(), ROOTS[root], C.byref(h)),
                      "server_keyset_load_file")
        return cls(h.value)

    def bsk(self, i: int) -> np.ndarray:
        out = np.zeros(self.bootstrap_keys[i].key_words, dtype=np.uint64)
        _native.check(self.lib.concrete_hip_server_keyset_read_bsk(self.h, i, out.ctypes.data, out.size), "read_bsk")
        return out

    def ksk(self, i: int) -> np.ndarray:
        out = np.zeros(self.keyswitch_keys[i].key_words, dtype=np.uint64)
        _native.check(self.lib.concrete_hip_server_keyset_read_ksk(self.h, i, out.ctypes.data, out.size), "read_ksk")
        return out

    def level_order(self, kind: str, i: int) -> str:
        """Level order found when key i ("bsk" / "ksk") was last read, checked against the client
        secret keys of a Keyset message: "unchecked", "as_expected" or "reversed" (re-ordered)."""
        rc = self.lib.concrete_hip_server_keyset_level_order(self.h, int(kind == "bsk"), i)
        _native.check(rc if rc < 0 else 0, "server_keyset_level_order")
        return LEVEL_ORDER[rc]

    @property
    def secret_count(self) -> int:
        return self.lib.concrete_hip_server_keyset_secret_count(self.h)

    def add_to(self, keyset) -> None:
        """Register every key in a runtime.Keyset (bsk_index / ksk_index = list position)."""
        _native.check(self.lib.concrete_hip_keyset_add_server_keyset(keyset.h, self.h), "keyset_add_server_keyset")

    def close(self):
        if self.h:
            self.lib.concrete_hip_server_keyset_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


# ---------------------------------------------------------------------------------------------
# writer
# ---------------------------------------------------------------------------------------------
class _Message:
    """Minimal Cap'n Proto message builder (unpacked stream framing).

    layout: "flat" (one segment), "single_far" (every object after the root in its own segment
    behind a one-word landing pad), "double_far" (objects in their own segments, two-word landing
    pads in a separate segment), "mixed" (alternating single / double).
    """

    def __init__(self, layout: str = "flat"):
        assert layout in ("flat", "single_far", "double_far", "mixed")
        self.layout = layout
        self.segs: list[list[int]] = [[0]]  # segment 0 starts with the root pointer
        self.pad_seg = None
        self.n_obj = 0

    def _alloc(self, words: int):
        """(segment, first word, pad word or None) of a new object of `words` words."""
        self.n_obj += 1
        mode = self.layout
        if mode == "mixed":
            mode = "single_far" if self.n_obj % 2 else "double_far"
        if mode == "flat" or self.n_obj == 1:  # the root object stays next to the root pointer
            seg = self.segs[0]
            start = len(seg)
            seg.extend([0] * words)
            return 0, start, None
        if mode == "single_far":
            self.segs.append([0] * (1 + words))
            return len(self.segs) - 1, 1, 0
        self.segs.append([0] * words)
        return len(self.segs) - 1, 0, None

    def _pad_words(self):
        if self.pad_seg is None:
            self.segs.append([])
            self.pad_seg = len(self.segs) - 1
        return self.pad_seg

    def _point(self, src_seg: int, src_word: int, obj, tag: int):
        """Writes at (src_seg, src_word) a pointer to obj = (seg, start, pad) described by tag
        (a struct / list pointer word with a zero offset field)."""
        seg, start, pad = obj
        if seg == src_seg:
            off = start - (src_word + 1)
            self.segs[src_seg][src_word] = tag | ((off & 0x3FFFFFFF) << 2)
            return
        if pad is not None:  # single far: landing pad right before the object
            self.segs[seg][pad] = tag | (((start - (pad + 1)) & 0x3FFFFFFF) << 2)
            self.segs[src_seg][src_word] = 2 | (pad << 3) | (seg << 32)
            return
        ps = self._pad_words()
        at = len(self.segs[ps])
        self.segs[ps].extend([2 | (start << 3) | (seg << 32), tag])  # far to the content, then its tag
        self.segs[src_seg][src_word] = 2 | 4 | (at << 3) | (ps << 32)

    # objects -----------------------------------------------------------------------------------
    def new_struct(self, dw: int, pw: int):
        seg, start, pad = self._alloc(dw + pw)
        return {"obj": (seg, start, pad), "dw": dw, "pw": pw}

    def struct_tag(self, s) -> int:
        return (s["dw"] << 32) | (s["pw"] << 48)

    def set_root(self, s):
        self._point(0, 0, s["obj"], self.struct_tag(s))

    def set_data(self, s, byte_off: int, fmt: str, value):
        seg, start, _ = s["obj"]
        word = start + byte_off // 8
        raw = bytearray(struct.pack("<Q", self.segs[seg][word]))
        struct.pack_into("<" + fmt, raw, byte_off % 8, value)
        self.segs[seg][word] = struct.unpack("<Q", bytes(raw))[0]

    def set_struct_ptr(self, s, idx: int, child):
        seg, start, _ = s["obj"]
        self._point(seg, start + s["dw"] + idx, child["obj"], self.struct_tag(child))

    def new_struct_list(self, n: int, dw: int, pw: int):
        """Composite list of n structs; returns (list handle, element handles)."""
        words = n * (dw + pw)
        seg, start, pad = self._alloc(1 + words)
        self.segs[seg][start] = (n << 2) | (dw << 32) | (pw << 48)  # tag word
        elems = [{"obj": (seg, start + 1 + i * (dw + pw), None), "dw": dw, "pw": pw} for i in range(n)]
        return {"obj": (seg, start, pad), "tag": 1 | (7 << 32) | (words << 35)}, elems

    def new_ptr_list(self, n: int):
        seg, start, pad = self._alloc(n)
        return {"obj": (seg, start, pad), "tag": 1 | (6 << 32) | (n << 35), "n": n}

    def new_data(self, payload: bytes):
        words = (len(payload) + 7) // 8
        seg, start, pad = self._alloc(words)
        padded = payload + b"\0" * (words * 8 - len(payload))
        self.segs[seg][start:start + words] = list(np.frombuffer(padded, dtype="<u8").tolist())
        return {"obj": (seg, start, pad), "tag": 1 | (2 << 32) | (len(payload) << 35)}

    def set_list_ptr(self, s, idx: int, lst):
        seg, start, _ = s["obj"]
        self._point(seg, start + s["dw"] + idx, lst["obj"], lst["tag"])

    def set_list_elem_ptr(self, plist, i: int, lst):
        seg, start, _ = plist["obj"]
        self._point(seg, start + i, lst["obj"], lst["tag"])

    def to_bytes(self) -> bytes:
        n = len(self.segs)
        head = [n - 1] + [len(s) for s in self.segs]
        if len(head) % 2:
            head.append(0)
        out = struct.pack("<%dI" % len(head), *head)
        for s in self.segs:
            out += np.asarray(s, dtype=np.uint64).astype("<u8").tobytes()
        return out


def _write_key(m: _Message, key, info: KeyInfo, payload: np.ndarray, is_bsk: bool, blob_words: int):
    inf = m.new_struct(INFO_WORDS, 1)
    for name, off in INFO_OFF.items():
        m.set_data(inf, off, "H" if name == "compression" else "I", getattr(info, name))
    offs = BSK_PARAMS_OFF if is_bsk else KSK_PARAMS_OFF
    par = m.new_struct(BSK_PARAMS_WORDS if is_bsk else KSK_PARAMS_WORDS, 1)
    for name, off in offs.items():
        fmt = "d" if name == "variance" else ("H" if name == "key_type" else "I")
        m.set_data(par, off, fmt, getattr(info, name))
    mod = m.new_struct(1, 1)  # Modulus: discriminant @0, member pointer 0
    m.set_data(mod, 0, "H", info.modulus_kind)
    member = m.new_struct(1 if info.modulus_kind else 0, 0)
    if info.modulus_kind:
        m.set_data(member, 0, "I", info.modulus_value)
    m.set_struct_ptr(mod, 0, member)
    m.set_struct_ptr(par, 0, mod)
    m.set_struct_ptr(inf, 0, par)
    m.set_struct_ptr(key, 0, inf)
    pl = m.new_struct(0, 1)  # Payload
    words = np.ascontiguousarray(payload, dtype=np.uint64)
    nblobs = max(1, -(-words.size // blob_words)) if words.size else 0
    plist = m.new_ptr_list(nblobs)
    for b in range(nblobs):
        chunk = words[b * blob_words:(b + 1) * blob_words]
        m.set_list_elem_ptr(plist, b, m.new_data(chunk.astype("<u8").tobytes()))
    m.set_list_ptr(pl, 0, plist)
    m.set_struct_ptr(key, 1, pl)


def _write_secret(m: _Message, key, sk_id: int, words: np.ndarray, blob_words: int):
    inf = m.new_struct(SK_INFO_WORDS, 1)
    m.set_data(inf, 0, "I", sk_id)
    par = m.new_struct(SK_PARAMS_WORDS, 0)
    m.set_data(par, SK_PARAMS_OFF["lwe_dimension"], "I", int(words.size))
    m.set_data(par, SK_PARAMS_OFF["integer_precision"], "I", 64)
    m.set_data(par, SK_PARAMS_OFF["key_type"], "H", 0)
    m.set_struct_ptr(inf, 0, par)
    m.set_struct_ptr(key, 0, inf)
    pl = m.new_struct(0, 1)
    w = np.ascontiguousarray(words, dtype=np.uint64)
    nblobs = max(1, -(-w.size // blob_words))
    plist = m.new_ptr_list(nblobs)
    for b in range(nblobs):
        m.set_list_elem_ptr(plist, b, m.new_data(w[b * blob_words:(b + 1) * blob_words].astype("<u8").tobytes()))
    m.set_list_ptr(pl, 0, plist)
    m.set_struct_ptr(key, 1, pl)


def serialize_server_keyset(bsks=(), ksks=(), *, root: str = "server", layout: str = "flat",
                            blob_words: int = BLOB_WORDS, secrets=()) -> bytes:
    """Wire form of a server keyset: bsks / ksks are lists of (KeyInfo, u64 payload).
    root: "server" (ServerKeyset), "keyset" (Keyset with the server part, and the client part's
    LweSecretKeys when `secrets` lists (id, u64 words) pairs), or "bootstrap_key" /
    "keyswitch_key" (a single key message)."""
    m = _Message(layout)
    if root in ("bootstrap_key", "keyswitch_key"):
        is_bsk = root == "bootstrap_key"
        (info, payload), = bsks if is_bsk else ksks
        key = m.new_struct(0, 2)
        m.set_root(key)
        _write_key(m, key, info, payload, is_bsk, blob_words)
        return m.to_bytes()
    if root == "keyset":
        top = m.new_struct(0, 2)
        m.set_root(top)
        srv = m.new_struct(0, 3)
        m.set_struct_ptr(top, 0, srv)
        if secrets:
            client = m.new_struct(0, 1)
            m.set_struct_ptr(top, 1, client)
            lst, elems = m.new_struct_list(len(secrets), 0, 2)
            m.set_list_ptr(client, 0, lst)
            for el, (sk_id, words) in zip(elems, secrets):
                _write_secret(m, el, sk_id, np.asarray(words), blob_words)
    else:
        srv = m.new_struct(0, 3)
        m.set_root(srv)
    for idx, (keys, is_bsk) in enumerate(((bsks, True), (ksks, False))):
        if not keys:
            continue
        lst, elems = m.new_struct_list(len(keys), 0, 2)
        m.set_list_ptr(srv, idx, lst)
        for el, (info, payload) in zip(elems, keys):
            _write_key(m, el, info, payload, is_bsk, blob_words)
    return m.to_bytes()
