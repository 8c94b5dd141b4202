// keyio.cpp — key wire-format import (host code of libconcrete_hip).
//
// Reads the evaluation keys of a concrete keyset from its Cap'n Proto wire form, the messages
// the reference writes with capnp::writeMessage (compiler include/concretelang/Common/
// Protocol.h:158-175, unpacked stream framing) for the schema
// tools/concrete-protocol/src/concrete-protocol.capnp:149-297 (ServerKeyset, Keyset,
// LweBootstrapKey, LweKeyswitchKey and their Info / Params structs), and hands the standard-domain
// keys to a runtime keyset (runtime.hip) in the order the runtime context indexes them
// (context.cpp:36-94: position in the ServerKeyset's lists).
//
// No capnp library is in the image, so this is a self-contained reader of the published encoding:
//   * stream framing: u32 (segment count - 1), u32 size (words) per segment, padding to 8 bytes,
//     then the segments;
//   * pointers: struct (kind 0: signed 30-bit word offset, data / pointer section sizes), list
//     (kind 1: element size code, count; composite lists with a tag word), far (kind 2: landing
//     pad in another segment, single or double), null = 0; out-of-range fields read as defaults;
//   * field placement inside each struct follows capnp's layout rule (fields in ordinal order,
//     each in the first free aligned hole of the data section), computed by hand for the structs
//     read here (offsets below, one comment per struct).
// Payloads are `List(Data)` blobs concatenated in order (Protocol.h:349-372), little-endian u64.
// Seeded keys (Compression::SEED: 2 seed words + bodies, Keys.cpp:121-137,193-218) are expanded by
// the caller-installed concrete-cpu decompressors (concrete_cpu_decompress_seeded_lwe_*_u64, the
// functions Keys.cpp calls): their mask stream is concrete-csprng's, which is not restated here.
//
// Parity: unpinned — the reference holds no serialized keyset; tests/test_keyio.py round-trips the
// writer in concrete_amd/keys.py (single-segment, single-far and double-far layouts) and checks
// malformed messages are refused.  The restated level orders of the standard layouts are checked
// on read whenever the message carries the client secret keys (a Keyset): check_level_order.
#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <exception>
#include <initializer_list>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/concrete_hip.h"

namespace chip {
void set_error(const char* fmt, ...);
}
using chip::set_error;

struct concrete_hip_server_keyset {
  struct Key {
    concrete_hip_key_info info;
    std::vector<uint64_t> payload;  // concatenated blobs (u64 words)
    // level order found when the key was last expanded against the client secret keys
    // (CONCRETE_HIP_LEVEL_ORDER_*).  Expansion is a const read of the keyset that several threads may
    // run on one key at once: the field is atomic (every expansion of one key finds the same order).
    struct Order {
      std::atomic<int> v{0};
      Order() = default;
      Order(const Order& o) : v(o.v.load()) {}
      Order& operator=(const Order& o) {
        v.store(o.v.load());
        return *this;
      }
    };
    mutable Order level_order;
  };
  struct Secret {  // a client LweSecretKey (Keyset.client, concrete-protocol.capnp:139-145, 298-303)
    uint32_t id = 0;
    std::vector<uint64_t> words;  // lweDimension u64 words (binary keys: 0 / 1)
  };
  std::vector<Key> bsk, ksk;
  std::vector<Secret> secrets;
  const Secret* secret(uint32_t id, uint64_t dim) const {
    for (const auto& x : secrets)
      if (x.id == id && x.words.size() == dim) return &x;
    return nullptr;
  }
};

namespace {

constexpr uint64_t MAX_WORDS = 1ull << 37;  // 1 TiB: sanity bound on declared segment sizes

class Reader {
 public:
  // words: the message body (segments back to back), seg_start / seg_size in words
  Reader(const uint64_t* words, std::vector<uint64_t> start, std::vector<uint64_t> size)
      : w_(words), start_(std::move(start)), size_(std::move(size)) {}

  struct Struct {
    bool present = false;
    uint32_t seg = 0;
    uint64_t data = 0;  // word index within the segment
    uint32_t dw = 0, pw = 0;
  };
  struct List {
    bool present = false;
    uint32_t seg = 0;
    uint64_t start = 0;   // first element (word index; byte lists: word index of the first byte)
    uint32_t esize = 0;   // capnp element size code
    uint64_t count = 0;   // elements
    uint32_t dw = 0, pw = 0;  // composite element layout
  };

  bool ok() const { return err_.empty(); }
  uint64_t message_bytes() const {
    uint64_t w = 0;
    for (uint64_t x : size_) w += x;
    return w * 8;
  }
  const std::string& err() const { return err_; }
  // Payload bytes copied so far by the whole parse.  Blobs may alias (several pointers to one Data),
  // and a composite list may hold many keys: the sum over every key stays within the message's own
  // size, so a crafted message cannot make the reader allocate more than it was given (capnp's
  // per-message traversal limit plays this role).
  bool charge_payload(uint64_t bytes) {
    if (bytes > message_bytes() - copied_) return false;
    copied_ += bytes;
    return true;
  }

  uint64_t word(uint32_t seg, uint64_t i) const { return w_[start_[seg] + i]; }

  Struct root() {
    if (size_.empty() || size_[0] < 1) return fail_s("empty message");
    return read_struct_ptr(0, 0);
  }

  // --- fields ---------------------------------------------------------------------------------
  uint32_t u32(const Struct& s, uint32_t byte_off) const {
    if ((byte_off + 4) > s.dw * 8ull) return 0;  // beyond the data section: default
    uint64_t v = word(s.seg, s.data + byte_off / 8);
    return (uint32_t)(v >> (8 * (byte_off % 8)));
  }
  uint16_t u16(const Struct& s, uint32_t byte_off) const {
    if ((byte_off + 2) > s.dw * 8ull) return 0;
    uint64_t v = word(s.seg, s.data + byte_off / 8);
    return (uint16_t)(v >> (8 * (byte_off % 8)));
  }
  double f64(const Struct& s, uint32_t byte_off) const {
    if ((byte_off + 8) > s.dw * 8ull) return 0.0;
    uint64_t v = word(s.seg, s.data + byte_off / 8);
    double d;
    memcpy(&d, &v, 8);
    return d;
  }
  Struct ptr_struct(const Struct& s, uint32_t idx) {
    if (idx >= s.pw) return Struct{};
    return read_struct_ptr(s.seg, s.data + s.dw + idx);
  }
  List ptr_list(const Struct& s, uint32_t idx) {
    if (idx >= s.pw) return List{};
    return read_list_ptr(s.seg, s.data + s.dw + idx);
  }
  Struct list_struct(const List& l, uint64_t i) {
    Struct r;
    if (!l.present || i >= l.count) return r;
    if (l.esize != 7) {
      fail("list of structs expected (element size %u)", l.esize);
      return r;
    }
    r.present = true;
    r.seg = l.seg;
    r.data = l.start + i * (uint64_t)(l.dw + l.pw);
    r.dw = l.dw;
    r.pw = l.pw;
    return r;
  }
  List list_ptr_list(const List& l, uint64_t i) {  // element i of a List(Data) / List(List(..))
    if (!l.present || i >= l.count) return List{};
    if (l.esize != 6) {
      fail("list of pointers expected (element size %u)", l.esize);
      return List{};
    }
    return read_list_ptr(l.seg, l.start + i);
  }
  const uint8_t* bytes(const List& l) const {
    return reinterpret_cast<const uint8_t*>(w_ + start_[l.seg] + l.start);
  }

 private:
  uint64_t copied_ = 0;
  const uint64_t* w_;
  std::vector<uint64_t> start_, size_;
  std::string err_;

  void fail(const char* fmt, ...) __attribute__((format(printf, 2, 3))) {
    if (!err_.empty()) return;
    char b[256];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(b, sizeof b, fmt, ap);
    va_end(ap);
    err_ = b;
  }
  Struct fail_s(const char* m) {
    fail("%s", m);
    return Struct{};
  }

  static int64_t off30(uint64_t w) { return (int64_t)((int32_t)(uint32_t)w >> 2); }

  // Follows the pointer at (seg, at): the target's segment, first word and the tag describing it
  // (the pointer itself, or the landing pad's tag for far pointers).  false: null or malformed.
  bool deref(uint32_t seg, uint64_t at, uint32_t& tseg, uint64_t& tstart, uint64_t& tag) {
    if (at >= size_[seg]) {
      fail("pointer outside its segment");
      return false;
    }
    const uint64_t p = word(seg, at);
    if (p == 0) return false;
    const uint32_t kind = p & 3;
    if (kind == 3) {
      fail("capability pointer in a key message");
      return false;
    }
    if (kind != 2) {
      tseg = seg;
      tag = p;
      const int64_t t = (int64_t)at + 1 + off30(p);
      if (t < 0 || (uint64_t)t > size_[seg]) {
        fail("pointer target outside its segment");
        return false;
      }
      tstart = (uint64_t)t;
      return true;
    }
    const bool dbl = (p >> 2) & 1;
    const uint64_t pad = (p >> 3) & 0x1fffffffu;
    const uint32_t sid = (uint32_t)(p >> 32);
    if (sid >= size_.size() || pad + (dbl ? 2 : 1) > size_[sid]) {
      fail("far pointer outside the message");
      return false;
    }
    const uint64_t l0 = word(sid, pad);
    if (!dbl) {
      if ((l0 & 3) == 2 || (l0 & 3) == 3) {
        fail("far pointer landing pad is not a struct or list pointer");
        return false;
      }
      tseg = sid;
      tag = l0;
      const int64_t t = (int64_t)pad + 1 + off30(l0);
      if (t < 0 || (uint64_t)t > size_[sid]) {
        fail("landing pad target outside its segment");
        return false;
      }
      tstart = (uint64_t)t;
      return true;
    }
    // double far: pad[0] = single far pointer to the content's start, pad[1] = its tag
    if ((l0 & 7) != 2) {
      fail("double-far landing pad is not a single far pointer");
      return false;
    }
    const uint32_t cseg = (uint32_t)(l0 >> 32);
    const uint64_t cstart = (l0 >> 3) & 0x1fffffffu;
    if (cseg >= size_.size() || cstart > size_[cseg]) {
      fail("double-far content outside the message");
      return false;
    }
    tseg = cseg;
    tstart = cstart;
    tag = word(sid, pad + 1);
    return true;
  }

  Struct read_struct_ptr(uint32_t seg, uint64_t at) {
    Struct s;
    uint32_t tseg;
    uint64_t tstart, tag;
    if (!deref(seg, at, tseg, tstart, tag)) return s;
    if ((tag & 3) != 0) return fail_s("struct pointer expected");
    s.dw = (uint32_t)((tag >> 32) & 0xffff);
    s.pw = (uint32_t)(tag >> 48);
    if (tstart + s.dw + s.pw > size_[tseg]) return fail_s("struct outside its segment");
    s.present = true;
    s.seg = tseg;
    s.data = tstart;
    return s;
  }

  List read_list_ptr(uint32_t seg, uint64_t at) {
    List l;
    uint32_t tseg;
    uint64_t tstart, tag;
    if (!deref(seg, at, tseg, tstart, tag)) return l;
    if ((tag & 3) != 1) {
      fail("list pointer expected");
      return l;
    }
    l.esize = (uint32_t)((tag >> 32) & 7);
    const uint64_t n = tag >> 35;
    l.seg = tseg;
    if (l.esize == 7) {  // composite: n = words after the tag word
      if (tstart + 1 + n > size_[tseg]) {
        fail("composite list outside its segment");
        return l;
      }
      const uint64_t t = word(tseg, tstart);
      if ((t & 3) != 0) {
        fail("composite list tag is not a struct tag");
        return l;
      }
      l.count = (t >> 2) & 0x3fffffffu;
      l.dw = (uint32_t)((t >> 32) & 0xffff);
      l.pw = (uint32_t)(t >> 48);
      if (l.count * (uint64_t)(l.dw + l.pw) > n) {
        fail("composite list elements exceed its word count");
        return l;
      }
      l.start = tstart + 1;
    } else {
      static const uint32_t bits[7] = {0, 1, 8, 16, 32, 64, 64};
      const uint64_t words = (n * bits[l.esize] + 63) / 64;
      if (tstart + words > size_[tseg]) {
        fail("list outside its segment");
        return l;
      }
      l.count = n;
      l.start = tstart;
    }
    l.present = true;
    return l;
  }
};

// --- schema offsets (concrete-protocol.capnp; capnp layout rule, bytes in the data section) ------
// LweBootstrapKey / LweKeyswitchKey: data 0 words; ptr 0 info, ptr 1 payload.
// *KeyInfo: id u32 @0, inputId u32 @4, outputId u32 @8, compression u16 @12 (enum);
//           ptr 0 params.
// LweBootstrapKeyParams: levelCount @0, baseLog @4, glweDimension @8, polynomialSize @12,
//           variance f64 @16, integerPrecision @24, keyType u16 @28, inputLweDimension @32;
//           ptr 0 modulus.
// LweKeyswitchKeyParams: levelCount @0, baseLog @4, variance f64 @8, integerPrecision @16,
//           keyType u16 @20, inputLweDimension @24, outputLweDimension @28; ptr 0 modulus.
// Modulus: union discriminant u16 @0 (0 native, 1 powerOfTwo, 2 integer); ptr 0 the member,
//           PowerOfTwoModulus.power / IntegerModulus.modulus u32 @0.
// Payload: ptr 0 data (List(Data)).
// ServerKeyset: ptr 0 lweBootstrapKeys, ptr 1 lweKeyswitchKeys, ptr 2 packingKeyswitchKeys.
// Keyset: ptr 0 server, ptr 1 client.

bool read_modulus(Reader& r, const Reader::Struct& params, concrete_hip_key_info& k) {
  Reader::Struct m = r.ptr_struct(params, 0);
  k.modulus_kind = 0;
  k.modulus_value = 0;
  if (!m.present) return r.ok();  // default: native
  k.modulus_kind = r.u16(m, 0);
  if (k.modulus_kind == 1 || k.modulus_kind == 2) {
    Reader::Struct v = r.ptr_struct(m, 0);
    if (v.present) k.modulus_value = r.u32(v, 0);
  }
  return r.ok();
}

bool read_payload(Reader& r, const Reader::Struct& key, std::vector<uint64_t>& out, uint64_t& words) {
  Reader::Struct payload = r.ptr_struct(key, 1);
  out.clear();
  words = 0;
  if (!payload.present) return r.ok();
  Reader::List blobs = r.ptr_list(payload, 0);
  if (!blobs.present) return r.ok();
  if (blobs.esize != 6) {
    set_error("key payload: List(Data) expected");
    return false;
  }
  uint64_t total = 0;
  std::vector<Reader::List> parts(blobs.count);
  for (uint64_t i = 0; i < blobs.count; ++i) {
    parts[i] = r.list_ptr_list(blobs, i);
    if (!r.ok()) return false;
    if (parts[i].present && parts[i].esize != 2) {
      set_error("key payload: blob %llu is not Data", (unsigned long long)i);
      return false;
    }
    total += parts[i].present ? parts[i].count : 0;
    // blobs may alias (several pointers to one Data): cap the payload at the message's own size
    if (total > r.message_bytes()) {
      set_error("key payload: blobs total more bytes than the message holds (aliased blobs?)");
      return false;
    }
  }
  // ... and every key's payload together (many keys naming one payload)
  if (!r.charge_payload(total)) {
    set_error("key payload: the keys' payloads total more bytes than the message holds (aliased blobs?)");
    return false;
  }
  if (total % 8) {
    set_error("key payload: %llu bytes is not a whole number of u64 words", (unsigned long long)total);
    return false;
  }
  out.resize(total / 8);
  uint8_t* dst = reinterpret_cast<uint8_t*>(out.data());
  for (const auto& p : parts)
    if (p.present && p.count) {
      memcpy(dst, r.bytes(p), p.count);
      dst += p.count;
    }
  words = total / 8;
  return true;
}

// Key sizes from the message's dimensions.  Those are untrusted u32 fields: every product is
// checked (a wrapped size would let a seeded key's decompressor write the real size through a
// buffer sized by the wrapped one), and read_info bounds the dimensions first.
bool mul_words(std::initializer_list<uint64_t> f, uint64_t& out) {
  uint64_t p = 1;
  for (uint64_t x : f)
    if (__builtin_mul_overflow(p, x, &p)) return false;
  out = p;
  return p <= MAX_WORDS;
}
bool bsk_words(const concrete_hip_key_info& k, uint64_t& w) {  // concrete_cpu_bootstrap_key_size_u64
  const uint64_t g = (uint64_t)k.glwe_dim + 1;
  return mul_words({k.input_lwe_dim, k.level_count, g, g, k.poly_size}, w);
}
bool seeded_bsk_words(const concrete_hip_key_info& k, uint64_t& w) {  // 2 seed words + seeded GGSW bodies
  if (!mul_words({k.input_lwe_dim, k.level_count, (uint64_t)k.glwe_dim + 1, k.poly_size}, w)) return false;
  w += 2;
  return true;
}
bool ksk_words(const concrete_hip_key_info& k, uint64_t& w) {  // concrete_cpu_keyswitch_key_size_u64
  return mul_words({k.input_lwe_dim, k.level_count, (uint64_t)k.output_lwe_dim + 1}, w);
}
bool seeded_ksk_words(const concrete_hip_key_info& k, uint64_t& w) {
  if (!mul_words({k.input_lwe_dim, k.level_count}, w)) return false;
  w += 2;
  return true;
}

// Dimension bounds a key must meet before anything is sized from it: a decomposition of at most
// 64 bits, LWE dimensions up to 2^20, GLWE dimension up to 64 and a power-of-two polynomial of
// at most 2^17 coefficients (concrete's optimizer tables stay far inside these).
bool key_dims_ok(const concrete_hip_key_info& k, bool is_bsk) {
  if (k.level_count < 1 || k.base_log < 1 || (uint64_t)k.level_count * k.base_log > 64) return false;
  if (k.input_lwe_dim < 1 || k.input_lwe_dim > (1u << 20)) return false;
  if (is_bsk)
    return k.glwe_dim >= 1 && k.glwe_dim <= 64 && k.poly_size >= 2 && k.poly_size <= (1u << 17) &&
           (k.poly_size & (k.poly_size - 1)) == 0;
  return k.output_lwe_dim >= 1 && k.output_lwe_dim <= (1u << 20);
}

bool read_info(Reader& r, const Reader::Struct& key, bool is_bsk, concrete_hip_key_info& k) {
  memset(&k, 0, sizeof k);
  Reader::Struct info = r.ptr_struct(key, 0);
  if (!info.present) {
    set_error("key without info");
    return false;
  }
  k.id = r.u32(info, 0);
  k.input_id = r.u32(info, 4);
  k.output_id = r.u32(info, 8);
  k.compression = r.u16(info, 12);
  Reader::Struct p = r.ptr_struct(info, 0);
  if (!p.present) {
    set_error("key info without params");
    return false;
  }
  k.level_count = r.u32(p, 0);
  k.base_log = r.u32(p, 4);
  if (is_bsk) {
    k.glwe_dim = r.u32(p, 8);
    k.poly_size = r.u32(p, 12);
    k.variance = r.f64(p, 16);
    k.integer_precision = r.u32(p, 24);
    k.key_type = r.u16(p, 28);
    k.input_lwe_dim = r.u32(p, 32);
    k.output_lwe_dim = k.glwe_dim * k.poly_size;
  } else {
    k.variance = r.f64(p, 8);
    k.integer_precision = r.u32(p, 16);
    k.key_type = r.u16(p, 20);
    k.input_lwe_dim = r.u32(p, 24);
    k.output_lwe_dim = r.u32(p, 28);
  }
  if (!read_modulus(r, p, k)) return false;
  if (!key_dims_ok(k, is_bsk)) {
    set_error("%s %u: dimensions out of range (level %u, base_log %u, glwe %u, N %u, n_in %u, n_out %u)",
              is_bsk ? "bootstrap key" : "keyswitch key", k.id, k.level_count, k.base_log, k.glwe_dim, k.poly_size,
              k.input_lwe_dim, k.output_lwe_dim);
    return false;
  }
  // the standard-domain (decompressed) size
  if (!(is_bsk ? bsk_words(k, k.key_words) : ksk_words(k, k.key_words))) {
    set_error("%s %u: key size overflows", is_bsk ? "bootstrap key" : "keyswitch key", k.id);
    return false;
  }
  return r.ok();
}

bool read_keys(Reader& r, const Reader::List& list, bool is_bsk, std::vector<concrete_hip_server_keyset::Key>& out) {
  if (!list.present) return r.ok();
  for (uint64_t i = 0; i < list.count; ++i) {
    Reader::Struct key = r.list_struct(list, i);
    if (!r.ok()) return false;
    concrete_hip_server_keyset::Key k;
    if (!read_info(r, key, is_bsk, k.info)) return false;
    if (!read_payload(r, key, k.payload, k.info.payload_words)) return false;
    out.push_back(std::move(k));
  }
  return true;
}

// ClientKeyset.lweSecretKeys: LweSecretKey { info @0 (LweSecretKeyInfo: id u32 @0; ptr 0 params:
// LweSecretKeyParams lweDimension u32 @0, integerPrecision u32 @4, keyType u16 @8), payload @1 }
bool read_secrets(Reader& r, const Reader::List& list, std::vector<concrete_hip_server_keyset::Secret>& out) {
  if (!list.present) return r.ok();
  for (uint64_t i = 0; i < list.count; ++i) {
    Reader::Struct key = r.list_struct(list, i);
    if (!r.ok()) return false;
    Reader::Struct info = r.ptr_struct(key, 0);
    if (!info.present) continue;
    concrete_hip_server_keyset::Secret sec;
    sec.id = r.u32(info, 0);
    Reader::Struct par = r.ptr_struct(info, 0);
    const uint32_t dim = par.present ? r.u32(par, 0) : 0;
    const uint32_t prec = par.present ? r.u32(par, 4) : 0;
    uint64_t words = 0;
    if (!read_payload(r, key, sec.words, words)) return false;
    // only 64-bit secret keys of their declared dimension take part in the level-order check
    if (prec == 64 && dim > 0 && words == dim) out.push_back(std::move(sec));
  }
  return r.ok();
}

int parse_impl(const uint64_t* words, uint64_t n_words, uint32_t root, concrete_hip_server_keyset** out);

// no C++ exception crosses the C ABI: allocation failures (a 1 GB key on a short host) are errors
int parse(const uint64_t* words, uint64_t n_words, uint32_t root, concrete_hip_server_keyset** out) {
  try {
    return parse_impl(words, n_words, root, out);
  } catch (const std::exception& e) {
    set_error("deserialize: %s", e.what());
    return -3;
  }
}

int parse_impl(const uint64_t* words, uint64_t n_words, uint32_t root, concrete_hip_server_keyset** out) {
  if (n_words < 1) {
    set_error("deserialize: empty input");
    return -3;
  }
  const uint32_t* h = reinterpret_cast<const uint32_t*>(words);
  const uint64_t nseg = (uint64_t)h[0] + 1;
  const uint64_t header_words = (4 * (1 + nseg) + 7) / 8;
  if (nseg > 512 || header_words > n_words) {
    set_error("deserialize: bad segment table (%llu segments)", (unsigned long long)nseg);
    return -3;
  }
  std::vector<uint64_t> start(nseg), size(nseg);
  uint64_t at = header_words;
  for (uint64_t s = 0; s < nseg; ++s) {
    size[s] = h[1 + s];
    start[s] = at;
    at += size[s];
    if (size[s] > MAX_WORDS || at > n_words) {
      set_error("deserialize: segment %llu extends past the input (%llu of %llu words)", (unsigned long long)s,
                (unsigned long long)at, (unsigned long long)n_words);
      return -3;
    }
  }
  Reader r(words, start, size);
  Reader::Struct top = r.root();
  if (!r.ok() || !top.present) {
    set_error("deserialize: %s", r.ok() ? "null root" : r.err().c_str());
    return -3;
  }
  auto* ks = new concrete_hip_server_keyset();
  bool ok = true;
  switch (root) {
    case CONCRETE_HIP_ROOT_KEYSET: {
      // Keyset.client (secret keys: the level orders of the evaluation keys are checked against them)
      Reader::Struct client = r.ptr_struct(top, 1);
      if (client.present && !read_secrets(r, r.ptr_list(client, 0), ks->secrets)) {
        ok = false;
        break;
      }
      top = r.ptr_struct(top, 0);  // Keyset.server
      if (!top.present) break;
    }
      /* fallthrough */
    case CONCRETE_HIP_ROOT_SERVER_KEYSET:
      ok = read_keys(r, r.ptr_list(top, 0), true, ks->bsk) && read_keys(r, r.ptr_list(top, 1), false, ks->ksk);
      break;
    case CONCRETE_HIP_ROOT_LWE_BOOTSTRAP_KEY:
    case CONCRETE_HIP_ROOT_LWE_KEYSWITCH_KEY: {
      const bool is_bsk = root == CONCRETE_HIP_ROOT_LWE_BOOTSTRAP_KEY;
      concrete_hip_server_keyset::Key k;
      ok = read_info(r, top, is_bsk, k.info) && read_payload(r, top, k.payload, k.info.payload_words);
      if (ok) (is_bsk ? ks->bsk : ks->ksk).push_back(std::move(k));
      break;
    }
    default:
      set_error("deserialize: unknown root type %u", root);
      ok = false;
  }
  if (ok && !r.ok()) {
    set_error("deserialize: %s", r.err().c_str());
    ok = false;
  }
  if (!ok) {
    delete ks;
    return -3;
  }
  *out = ks;
  return 0;
}

// ---- level order of an evaluation key, checked against the client secret keys ---------------
// The standard layouts restate tfhe's storage orders (unpinned: no serialized keyset exists
// offline): GGSW level position v of a bootstrap key encrypts s_i 2^(64 - logB (v + 1)) (keygen.cpp,
// level 1 first); keyswitch row t of block i encrypts s_in[i] 2^(64 - logB (l - t)) (levels reversed,
// keyswitch.rs:185-223).  When the keyset carries the client keys, one row per level of the first
// mask position whose secret bit is 1 is decrypted: a key stored in the other order is re-ordered,
// one that decrypts to neither is refused (a silent wrong order would bootstrap to garbage).
// dist(a, b): |a - b| on the torus
inline uint64_t tdist(uint64_t a, uint64_t b) {
  const uint64_t d = a - b;
  return (int64_t)d < 0 ? 0 - d : d;
}
// Classify the per-level decryptions d[p][v] (p over checked mask positions) against the expected
// scales e[v] and their reversal.  The order is decided by the most significant level, whose scale
// sits far above any key's noise; a deeper level is compared too only when its scale / 4 is at
// least 64 sigma of the key's noise (sigma from the key's variance field; unknown: top level only).
// A keyswitch key at secure noise puts its deepest level at the noise floor by design (CFG4's
// n = 742, l = 5, logB = 3: sigma ~ 2^47.6 against scale / 4 = 2^47), so requiring every level to
// decrypt would refuse valid keys.  Junk passes one position's top-level check with
// probability ~2^-(logB + 1) per order; every checked position must agree.
int classify_levels(const std::vector<std::vector<uint64_t>>& d, const std::vector<uint64_t>& e, double sigma) {
  const size_t l = e.size();
  size_t vt = 0;
  for (size_t v = 1; v < l; ++v)
    if (e[v] > e[vt]) vt = v;
  const double floor = 256.0 * sigma;  // scale / 4 >= 64 sigma
  auto resolvable = [&](size_t v) { return v == vt || (sigma > 0.0 && (double)e[v] >= floor); };
  bool as_is = true, reversed = true;
  for (const auto& dp : d)
    for (size_t v = 0; v < l; ++v) {
      // stored position v holds expected scale e[v] (as is) or e[l - 1 - v] (reversed)
      if (resolvable(v) && !(tdist(dp[v], e[v]) < e[v] / 4)) as_is = false;
      const size_t r = l - 1 - v;
      if (resolvable(r) && !(tdist(dp[v], e[r]) < e[r] / 4)) reversed = false;
    }
  if (as_is && !reversed) return CONCRETE_HIP_LEVEL_ORDER_AS_EXPECTED;
  if (reversed && !as_is) return CONCRETE_HIP_LEVEL_ORDER_REVERSED;
  return -1;  // neither, or both (indistinguishable): refuse
}

// key: standard-domain words; returns CONCRETE_HIP_LEVEL_ORDER_* or -1 (refuse)
int check_level_order(const concrete_hip_server_keyset* ks, const concrete_hip_key_info& i, bool is_bsk,
                      uint64_t* key) {
  const uint32_t l = i.level_count, logB = i.base_log;
  if (!ks || l < 2) return CONCRETE_HIP_LEVEL_ORDER_UNCHECKED;  // one level: nothing to order
  const uint64_t n_out = is_bsk ? (uint64_t)i.glwe_dim * i.poly_size : i.output_lwe_dim;
  const auto* s_in = ks->secret(i.input_id, i.input_lwe_dim);
  const auto* s_out = ks->secret(i.output_id, n_out);
  if (!s_in || !s_out) return CONCRETE_HIP_LEVEL_ORDER_UNCHECKED;
  // up to 16 mask positions whose secret bit is 1 (each row decryption is one constant coefficient:
  // O(k N) or O(n_out) work)
  constexpr size_t MAX_POS = 16;
  std::vector<uint64_t> pos;
  for (uint64_t m = 0; m < i.input_lwe_dim && pos.size() < MAX_POS; ++m)
    if (s_in->words[m] == 1) pos.push_back(m);
  if (pos.empty()) return CONCRETE_HIP_LEVEL_ORDER_UNCHECKED;
  std::vector<std::vector<uint64_t>> d(pos.size(), std::vector<uint64_t>(l));
  std::vector<uint64_t> e(l);
  const uint64_t* so = s_out->words.data();
  for (size_t pi = 0; pi < pos.size(); ++pi) {
    if (is_bsk) {
      // [n][l][k+1 rows][k+1 polys][N]: row k of level v, constant coefficient of B - sum_r A_r S_r
      const uint64_t k = i.glwe_dim, N = i.poly_size, glwe = (k + 1) * N;
      for (uint32_t v = 0; v < l; ++v) {
        const uint64_t* ct = key + ((pos[pi] * l + v) * (k + 1) + k) * glwe;
        uint64_t acc = ct[k * N];
        for (uint64_t r = 0; r < k; ++r) {
          const uint64_t* a = ct + r * N;
          const uint64_t* sr = so + r * N;
          acc -= a[0] * sr[0];
          for (uint64_t j = 1; j < N; ++j) acc += a[j] * sr[N - j];  // negacyclic: X^N = -1
        }
        d[pi][v] = acc;
        e[v] = 1ull << (64 - logB * (v + 1));
      }
    } else {
      // [n_in][l][n_out + 1]: row t decrypts to s_in[pos] 2^(64 - logB (l - t))
      for (uint32_t t = 0; t < l; ++t) {
        const uint64_t* ct = key + (pos[pi] * l + t) * (n_out + 1);
        uint64_t acc = ct[n_out];
        for (uint64_t j = 0; j < n_out; ++j) acc -= ct[j] * so[j];
        d[pi][t] = acc;
        e[t] = 1ull << (64 - logB * (l - t));
      }
    }
  }
  // the key's noise: concrete-protocol's variance is on the unit torus
  const double sigma = (i.variance > 0.0 && i.variance < 1.0) ? sqrt(i.variance) * 18446744073709551616.0 : 0.0;
  const int c = classify_levels(d, e, sigma);
  if (c != CONCRETE_HIP_LEVEL_ORDER_REVERSED) return c;
  // re-order: reverse the level blocks of every mask position
  const uint64_t blk = is_bsk ? ((uint64_t)i.glwe_dim + 1) * ((uint64_t)i.glwe_dim + 1) * i.poly_size : n_out + 1;
  for (uint64_t m = 0; m < i.input_lwe_dim; ++m)
    for (uint32_t v = 0; v < l / 2; ++v)
      std::swap_ranges(key + (m * l + v) * blk, key + (m * l + v + 1) * blk, key + (m * l + (l - 1 - v)) * blk);
  return c;
}

std::mutex g_dec_mu;
concrete_hip_bsk_decompressor g_bsk_dec = nullptr;
concrete_hip_ksk_decompressor g_ksk_dec = nullptr;

int expand_raw(const concrete_hip_server_keyset::Key& k, bool is_bsk, uint64_t* dst, uint64_t dst_words);

// Checks a key's parameters and payload size, writes its standard-domain form to dst, and checks
// (and if needed fixes) its level order against the keyset's client secret keys.
int expand(const concrete_hip_server_keyset* ks, const concrete_hip_server_keyset::Key& k, bool is_bsk, uint64_t* dst,
           uint64_t dst_words) {
  const int rc = expand_raw(k, is_bsk, dst, dst_words);
  if (rc) return rc;
  const int order = check_level_order(ks, k.info, is_bsk, dst);
  if (order < 0) {
    set_error("%s %u: no GGSW / keyswitch row decrypts to its level under the keyset's client keys, in either "
              "level order", is_bsk ? "bootstrap key" : "keyswitch key", k.info.id);
    return -3;
  }
  k.level_order.v.store(order);
  return 0;
}

int expand_raw(const concrete_hip_server_keyset::Key& k, bool is_bsk, uint64_t* dst, uint64_t dst_words) {
  const concrete_hip_key_info& i = k.info;
  const char* what = is_bsk ? "bootstrap key" : "keyswitch key";
  if (i.integer_precision != 64 || i.modulus_kind != 0) {
    set_error("%s %u: only 64-bit keys over the native modulus are supported (precision %u, modulus kind %u)", what,
              i.id, i.integer_precision, i.modulus_kind);
    return -2;
  }
  if (dst_words < i.key_words) {
    set_error("%s %u: destination holds %llu words, the key needs %llu", what, i.id, (unsigned long long)dst_words,
              (unsigned long long)i.key_words);
    return -3;
  }
  if (i.compression == 0) {
    if (k.payload.size() != i.key_words) {
      set_error("%s %u: payload has %llu words, its parameters need %llu", what, i.id,
                (unsigned long long)k.payload.size(), (unsigned long long)i.key_words);
      return -3;
    }
    memcpy(dst, k.payload.data(), i.key_words * 8);
    return 0;
  }
  if (i.compression != 1) {
    set_error("%s %u: unsupported compression %u", what, i.id, i.compression);
    return -2;
  }
  uint64_t need = 0;
  if (!(is_bsk ? seeded_bsk_words(i, need) : seeded_ksk_words(i, need)) || k.payload.size() != need) {
    set_error("%s %u: seeded payload has %llu words, its parameters need %llu", what, i.id,
              (unsigned long long)k.payload.size(), (unsigned long long)need);
    return -3;
  }
  // Csprng.cpp:125-140 readSeed: word 0 = bytes 0-7, word 1 = bytes 8-15, little endian
  concrete_hip_uint128 seed;
  for (int b = 0; b < 16; ++b) seed.little_endian_bytes[b] = (uint8_t)(k.payload[b / 8] >> (8 * (b % 8)));
  concrete_hip_bsk_decompressor bf;
  concrete_hip_ksk_decompressor kf;
  {
    std::lock_guard<std::mutex> g(g_dec_mu);
    bf = g_bsk_dec;
    kf = g_ksk_dec;
  }
  if (is_bsk ? !bf : !kf) {
    set_error("%s %u is seeded: install concrete-cpu's decompressor with concrete_hip_set_seeded_key_decompressors",
              what, i.id);
    return -2;
  }
  if (is_bsk)
    bf(dst, k.payload.data() + 2, i.input_lwe_dim, i.poly_size, i.glwe_dim, i.level_count, i.base_log, seed, 1u);
  else
    kf(dst, k.payload.data() + 2, i.input_lwe_dim, i.output_lwe_dim, i.level_count, i.base_log, seed, 1u);
  return 0;
}

}  // namespace

static int add_server_keyset(concrete_hip_keyset* ks, const concrete_hip_server_keyset* sk) {
  // every key's parameters are checked against what the backend runs before any key is expanded
  // (a decompressor runs only on a key the keyset would accept)
  for (uint32_t i = 0; i < sk->bsk.size(); ++i) {
    const concrete_hip_key_info& k = sk->bsk[i].info;
    if (!concrete_hip_pbs_supported(k.glwe_dim, k.poly_size, k.level_count, k.base_log)) {
      set_error("keyset_add_server_keyset: bootstrap key %u: unsupported parameters k=%u N=%u level=%u base_log=%u",
                i, k.glwe_dim, k.poly_size, k.level_count, k.base_log);
      return -2;
    }
  }
  for (uint32_t i = 0; i < sk->ksk.size(); ++i) {
    const concrete_hip_key_info& k = sk->ksk[i].info;
    if (!concrete_hip_keyswitch_supported(k.level_count, k.base_log, k.input_lwe_dim, k.output_lwe_dim)) {
      set_error("keyset_add_server_keyset: keyswitch key %u: unsupported parameters level=%u base_log=%u n_out=%u", i,
                k.level_count, k.base_log, k.output_lwe_dim);
      return -2;
    }
  }
  std::vector<uint64_t> buf;
  for (uint32_t i = 0; i < sk->bsk.size(); ++i) {
    const concrete_hip_key_info& k = sk->bsk[i].info;
    buf.assign(k.key_words, 0);
    int rc = expand(sk, sk->bsk[i], true, buf.data(), buf.size());
    if (rc) return rc;
    rc = concrete_hip_keyset_add_bsk(ks, i, buf.data(), k.input_lwe_dim, k.glwe_dim, k.level_count, k.base_log,
                                     k.poly_size);
    if (rc) return rc;
  }
  for (uint32_t i = 0; i < sk->ksk.size(); ++i) {
    const concrete_hip_key_info& k = sk->ksk[i].info;
    buf.assign(k.key_words, 0);
    int rc = expand(sk, sk->ksk[i], false, buf.data(), buf.size());
    if (rc) return rc;
    rc = concrete_hip_keyset_add_ksk(ks, i, buf.data(), k.level_count, k.base_log, k.input_lwe_dim,
                                     k.output_lwe_dim);
    if (rc) return rc;
  }
  return 0;
}

extern "C" {

int concrete_hip_server_keyset_deserialize(const void* bytes, uint64_t size, uint32_t root,
                                           concrete_hip_server_keyset** out) {
  if (!out || (!bytes && size)) {
    set_error("server_keyset_deserialize: bad argument");
    return -3;
  }
  *out = nullptr;
  if (size % 8) {
    set_error("server_keyset_deserialize: %llu bytes is not a whole number of words", (unsigned long long)size);
    return -3;
  }
  if ((uintptr_t)bytes % 8 == 0) return parse((const uint64_t*)bytes, size / 8, root, out);
  try {
    std::vector<uint64_t> copy(size / 8);
    memcpy(copy.data(), bytes, size);
    return parse(copy.data(), copy.size(), root, out);
  } catch (const std::exception& e) {
    set_error("server_keyset_deserialize: %s", e.what());
    return -3;
  }
}

int concrete_hip_server_keyset_load_file(const char* path, uint32_t root, concrete_hip_server_keyset** out) {
  if (!path || !out) {
    set_error("server_keyset_load_file: bad argument");
    return -3;
  }
  *out = nullptr;
  FILE* f = fopen(path, "rb");
  if (!f) {
    set_error("server_keyset_load_file: cannot open %s", path);
    return -3;
  }
  std::vector<uint64_t> buf;
  uint64_t got = 0;
  try {
    if (fseek(f, 0, SEEK_END) == 0) {
      long len = ftell(f);
      if (len > 0 && len % 8 == 0 && fseek(f, 0, SEEK_SET) == 0) {
        buf.resize((uint64_t)len / 8);
        got = fread(buf.data(), 1, (size_t)len, f);
      }
    }
  } catch (const std::exception& e) {
    fclose(f);
    set_error("server_keyset_load_file: %s", e.what());
    return -3;
  }
  fclose(f);
  if (buf.empty() || got != buf.size() * 8) {
    set_error("server_keyset_load_file: %s is empty, unreadable or not a whole number of words", path);
    return -3;
  }
  return parse(buf.data(), buf.size(), root, out);
}

void concrete_hip_server_keyset_destroy(concrete_hip_server_keyset* sk) { delete sk; }

uint32_t concrete_hip_server_keyset_bsk_count(const concrete_hip_server_keyset* sk) {
  return sk ? (uint32_t)sk->bsk.size() : 0;
}
uint32_t concrete_hip_server_keyset_ksk_count(const concrete_hip_server_keyset* sk) {
  return sk ? (uint32_t)sk->ksk.size() : 0;
}

int concrete_hip_server_keyset_bsk_info(const concrete_hip_server_keyset* sk, uint32_t index,
                                        concrete_hip_key_info* out) {
  if (!sk || !out || index >= sk->bsk.size()) {
    set_error("server_keyset_bsk_info: bad argument or index %u", index);
    return -3;
  }
  *out = sk->bsk[index].info;
  return 0;
}

int concrete_hip_server_keyset_ksk_info(const concrete_hip_server_keyset* sk, uint32_t index,
                                        concrete_hip_key_info* out) {
  if (!sk || !out || index >= sk->ksk.size()) {
    set_error("server_keyset_ksk_info: bad argument or index %u", index);
    return -3;
  }
  *out = sk->ksk[index].info;
  return 0;
}

int concrete_hip_server_keyset_read_bsk(const concrete_hip_server_keyset* sk, uint32_t index, uint64_t* dst,
                                        uint64_t dst_words) {
  if (!sk || !dst || index >= sk->bsk.size()) {
    set_error("server_keyset_read_bsk: bad argument or index %u", index);
    return -3;
  }
  return expand(sk, sk->bsk[index], true, dst, dst_words);
}

int concrete_hip_server_keyset_read_ksk(const concrete_hip_server_keyset* sk, uint32_t index, uint64_t* dst,
                                        uint64_t dst_words) {
  if (!sk || !dst || index >= sk->ksk.size()) {
    set_error("server_keyset_read_ksk: bad argument or index %u", index);
    return -3;
  }
  return expand(sk, sk->ksk[index], false, dst, dst_words);
}

int concrete_hip_server_keyset_level_order(const concrete_hip_server_keyset* sk, int is_bsk, uint32_t index) {
  if (!sk || index >= (is_bsk ? sk->bsk.size() : sk->ksk.size())) {
    set_error("server_keyset_level_order: bad argument or index %u", index);
    return -3;
  }
  return (is_bsk ? sk->bsk[index] : sk->ksk[index]).level_order.v.load();
}

uint32_t concrete_hip_server_keyset_secret_count(const concrete_hip_server_keyset* sk) {
  return sk ? (uint32_t)sk->secrets.size() : 0;
}

void concrete_hip_set_seeded_key_decompressors(concrete_hip_bsk_decompressor bsk, concrete_hip_ksk_decompressor ksk) {
  std::lock_guard<std::mutex> g(g_dec_mu);
  g_bsk_dec = bsk;
  g_ksk_dec = ksk;
}

int concrete_hip_keyset_add_server_keyset(concrete_hip_keyset* ks, const concrete_hip_server_keyset* sk) {
  if (!ks || !sk) {
    set_error("keyset_add_server_keyset: bad argument");
    return -3;
  }
  try {
    return add_server_keyset(ks, sk);
  } catch (const std::exception& e) {
    set_error("keyset_add_server_keyset: %s", e.what());
    return -3;
  }
}

}  // extern "C"
