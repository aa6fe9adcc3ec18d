// am_txid.hip -- transaction-id identity at the boundary (host code).
//
// clocksi_materializer:is_op_in_snapshot/7 uses a TxId only for equality: an op whose
// #clocksi_payload.txid == the reading transaction's TxId is a candidate even when the base
// snapshot already covers it (src/clocksi_materializer.erl:232).  A TxId is
// #tx_id{local_start_time, server_pid} (include/antidote.hrl:192-195): it holds a pid, which
// the ORDERED term codec (am_codec.hip) cannot label, and a fresh TxId per transaction would
// make an ordered label space grow and re-spread without bound.  So TxIds get their own
// equality-only map: the external-term-format bytes of the term (enif_term_to_binary) are
// canonicalised -- every encoding of one term (ATOM_EXT / SMALL_ATOM_UTF8_EXT, PID_EXT /
// NEW_PID_EXT, REFERENCE_EXT / NEW_REFERENCE_EXT / NEWER_REFERENCE_EXT, the port forms,
// STRING_EXT / LIST_EXT, BIT_BINARY_EXT with 8 bits / BINARY_EXT, minimal integers) maps to one
// byte string -- and interned into a dense u64 id, never reordered or relabeled.  Two TxIds
// get the same id iff they are the same term (exact, no hashing).  Ids start at 1 and are
// never reused; am_txid_forget drops a finished transaction's entry (its ops keep the id, and
// no later read carries that TxId), and am_txid_expire drops the entries of ops the stable
// snapshot covers (below).  Floats compare by bits (a TxId holds none).  Maps and funs
// are AM_ERR_UNSUPPORTED.
#include <map>
#include <string>
#include <unordered_map>

#include "am_internal.h"

namespace {

struct Canon {
  const uint8_t *p, *e;
  std::string out;
  bool ok = true, unsupported = false;
  bool need(uint64_t n) {
    if ((uint64_t)(e - p) < n) ok = false;
    return ok;
  }
  uint32_t u8() { return need(1) ? *p++ : 0; }
  uint32_t u16() {
    if (!need(2)) return 0;
    const uint32_t v = (uint32_t)p[0] << 8 | p[1];
    p += 2;
    return v;
  }
  uint32_t u32() {
    if (!need(4)) return 0;
    const uint32_t v = (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
    p += 4;
    return v;
  }
  void put32(uint32_t v) {
    out.push_back((char)(v >> 24)), out.push_back((char)(v >> 16)), out.push_back((char)(v >> 8)), out.push_back((char)v);
  }
  void put_bytes(const uint8_t *b, uint64_t n) { out.append((const char *)b, n); }

  // an atom's text as UTF-8 (ATOM_EXT / SMALL_ATOM_EXT are Latin-1)
  bool atom_text(uint32_t tag, std::string &txt) {
    uint32_t n = 0;
    if (tag == 100 || tag == 118) n = u16();
    else n = u8();
    if (!need(n)) return false;
    if (tag == 100 || tag == 115) {
      for (uint32_t i = 0; i < n; ++i) {
        const uint8_t c = p[i];
        if (c < 0x80) {
          txt.push_back((char)c);
        } else {
          txt.push_back((char)(0xC0 | (c >> 6)));
          txt.push_back((char)(0x80 | (c & 0x3F)));
        }
      }
    } else {
      txt.assign((const char *)p, n);
    }
    p += n;
    return true;
  }
  void put_atom(const std::string &txt) {
    if (txt.size() < 256) {
      out.push_back((char)119);
      out.push_back((char)txt.size());
    } else {
      out.push_back((char)118);
      out.push_back((char)(txt.size() >> 8));
      out.push_back((char)txt.size());
    }
    out += txt;
  }
  // the node atom of a pid / port / reference
  bool node() {
    const uint32_t tag = u8();
    if (tag != 100 && tag != 115 && tag != 118 && tag != 119) return ok = false;
    std::string txt;
    if (!atom_text(tag, txt)) return false;
    put_atom(txt);
    return true;
  }
  // integer magnitude (little-endian digits) -> canonical SMALL_INTEGER / INTEGER / BIG
  void put_int(bool neg, const uint8_t *le, uint32_t n) {
    while (n && le[n - 1] == 0) --n;
    if (n == 0) neg = false;
    if (n <= 8) {
      uint64_t m = 0;
      for (uint32_t i = 0; i < n; ++i) m |= (uint64_t)le[i] << (8 * i);
      if (!neg && m < 256) {
        out.push_back((char)97);
        out.push_back((char)m);
        return;
      }
      if ((!neg && m <= 0x7FFFFFFFull) || (neg && m <= 0x80000000ull)) {
        out.push_back((char)98);
        put32(neg ? (uint32_t)(0u - (uint32_t)m) : (uint32_t)m);
        return;
      }
    }
    if (n < 256) {
      out.push_back((char)110);
      out.push_back((char)n);
    } else {
      out.push_back((char)111);
      put32(n);
    }
    out.push_back(neg ? 1 : 0);
    put_bytes(le, n);
  }
  bool term(int depth) {
    if (depth > 256) return ok = false;
    const uint32_t tag = u8();
    if (!ok) return false;
    switch (tag) {
      case 97: {  // SMALL_INTEGER_EXT
        const uint8_t v = (uint8_t)u8();
        put_int(false, &v, 1);
        return ok;
      }
      case 98: {  // INTEGER_EXT
        const int32_t v = (int32_t)u32();
        const uint32_t m = v < 0 ? 0u - (uint32_t)v : (uint32_t)v;
        const uint8_t le[4] = {(uint8_t)m, (uint8_t)(m >> 8), (uint8_t)(m >> 16), (uint8_t)(m >> 24)};
        put_int(v < 0, le, 4);
        return ok;
      }
      case 110: case 111: {  // SMALL_BIG_EXT / LARGE_BIG_EXT
        const uint32_t n = tag == 110 ? u8() : u32();
        const bool neg = u8() != 0;
        if (!need(n)) return false;
        const uint8_t *d = p;
        p += n;
        put_int(neg, d, n);
        return ok;
      }
      case 70: {  // NEW_FLOAT_EXT
        if (!need(8)) return false;
        out.push_back((char)70);
        put_bytes(p, 8);
        p += 8;
        return ok;
      }
      case 100: case 115: case 118: case 119: {  // atoms
        std::string txt;
        if (!atom_text(tag, txt)) return false;
        put_atom(txt);
        return ok;
      }
      case 104: case 105: {  // tuples
        const uint32_t n = tag == 104 ? u8() : u32();
        if (n < 256) {
          out.push_back((char)104);
          out.push_back((char)n);
        } else {
          out.push_back((char)105);
          put32(n);
        }
        for (uint32_t k = 0; k < n && ok; ++k) term(depth + 1);
        return ok;
      }
      case 106:  // NIL_EXT
        out.push_back((char)106);
        return ok;
      case 107: case 108: {  // STRING_EXT / LIST_EXT: canonical LIST_EXT, proper tails merged
        std::string items;
        uint32_t count = 0;
        uint32_t t = tag;
        std::string tail;
        for (;;) {
          if (t == 107) {
            const uint32_t n = u16();
            if (!need(n)) return false;
            for (uint32_t k = 0; k < n; ++k) {
              items.push_back((char)97);
              items.push_back((char)p[k]);
            }
            p += n;
            count += n;
            tail.assign(1, (char)106);
            break;
          }
          const uint32_t n = u32();
          std::string saved;
          saved.swap(out);
          for (uint32_t k = 0; k < n && ok; ++k) term(depth + 1);
          items += out;
          out.swap(saved);
          count += n;
          if (!ok) return false;
          const uint32_t nt = u8();
          if (nt == 106) {
            tail.assign(1, (char)106);
            break;
          }
          if (nt == 107 || nt == 108) {  // [a | "bc"] / [a | [b]] are the list [a, b, c]
            t = nt;
            continue;
          }
          --p;  // an improper tail: a term of its own
          std::string outer;
          outer.swap(out);
          term(depth + 1);
          tail.swap(out);
          out.swap(outer);
          if (!ok) return false;
          break;
        }
        if (count == 0) {
          out += tail;
          return ok;
        }
        out.push_back((char)108);
        put32(count);
        out += items;
        out += tail;
        return ok;
      }
      case 109: {  // BINARY_EXT
        const uint32_t n = u32();
        if (!need(n)) return false;
        out.push_back((char)109);
        put32(n);
        put_bytes(p, n);
        p += n;
        return ok;
      }
      case 77: {  // BIT_BINARY_EXT: whole bytes -> BINARY_EXT; unused trailing bits zeroed
        const uint32_t n = u32();
        const uint32_t bits = u8();
        if (!need(n) || bits < 1 || bits > 8 || n == 0) return ok = false;
        if (bits == 8) {
          out.push_back((char)109);
          put32(n);
          put_bytes(p, n);
        } else {
          out.push_back((char)77);
          put32(n);
          out.push_back((char)bits);
          put_bytes(p, n - 1);
          out.push_back((char)(p[n - 1] & (uint8_t)(0xFF << (8 - bits))));
        }
        p += n;
        return ok;
      }
      case 103: case 88: {  // PID_EXT / NEW_PID_EXT -> NEW_PID_EXT
        out.push_back((char)88);
        if (!node()) return false;
        const uint32_t id = u32(), serial = u32();
        const uint32_t creation = tag == 103 ? u8() : u32();
        put32(id), put32(serial), put32(creation);
        return ok;
      }
      case 102: case 89: case 120: {  // PORT_EXT / NEW_PORT_EXT / V4_PORT_EXT -> V4_PORT_EXT
        out.push_back((char)120);
        if (!node()) return false;
        uint64_t id = 0;
        if (tag == 120) {
          id = (uint64_t)u32() << 32;
          id |= u32();
        } else {
          id = u32();
        }
        const uint32_t creation = tag == 102 ? u8() : u32();
        put32((uint32_t)(id >> 32)), put32((uint32_t)id), put32(creation);
        return ok;
      }
      case 101: case 114: case 90: {  // REFERENCE_EXT / NEW_ / NEWER_REFERENCE_EXT -> NEWER_
        if (tag == 101) {
          out.push_back((char)90);
          out.push_back(0), out.push_back(1);
          if (!node()) return false;
          const uint32_t id = u32();
          const uint32_t creation = u8();
          put32(creation), put32(id);
          return ok;
        }
        const uint32_t len = u16();
        if (len > 5) return ok = false;
        out.push_back((char)90);
        out.push_back((char)(len >> 8)), out.push_back((char)len);
        if (!node()) return false;
        const uint32_t creation = tag == 114 ? u8() : u32();
        put32(creation);
        for (uint32_t k = 0; k < len && ok; ++k) put32(u32());
        return ok;
      }
      default:  // maps, funs, exports, compressed terms, FLOAT_EXT
        unsupported = true;
        ok = false;
        return false;
    }
  }
};

// the canonical byte string of an encoded term (AM_ERR_UNSUPPORTED / AM_ERR_INVALID)
int canonical(const uint8_t *b, uint64_t len, std::string &out) {
  if (!b || len < 2 || b[0] != 131) return AM_ERR_INVALID;
  Canon c{b + 1, b + len};
  c.term(0);
  if (!c.ok) return c.unsupported ? AM_ERR_UNSUPPORTED : AM_ERR_INVALID;  // else truncated / malformed
  if (c.p != c.e) return AM_ERR_INVALID;
  out.swap(c.out);
  return AM_OK;
}

}  // namespace

// An entry is HELD while a reader interned it (am_txid_intern, until am_txid_forget) and STAMPED
// with its ops' commit time {DcId, CT} when ops interned it (am_txid_intern_op).  A stamped entry
// that no reader holds is dropped by am_txid_expire once the stable snapshot covers its commit
// time: the transaction committed (its ops reach the ops cache at commit) and every partition has
// applied it, so no live reader carries that TxId -- ops replicated from other DCs, whose TxIds no
// local coordinator ever forgets, leave the map this way.  Ids are never reused, so an op whose
// entry was dropped can never equal a later reader's TxId.
struct am_txid_ent {
  uint64_t id = 0, ct = 0;
  uint32_t dc = 0;
  bool stamped = false, held = false;
};
struct am_txids {
  std::mutex mu;
  std::unordered_map<std::string, am_txid_ent> ids;
  std::map<uint32_t, std::multimap<uint64_t, std::string>> by_ct;  // stamped entries per DC (may hold stale keys)
  uint64_t next = 1;
};

extern "C" {

int am_txid_create(am_txids **out) {
  if (!out) return AM_ERR_INVALID;
  *out = new (std::nothrow) am_txids();
  return *out ? AM_OK : AM_ERR_NOMEM;
}

int am_txid_destroy(am_txids *t) {
  delete t;
  return AM_OK;
}

int am_txid_intern(am_txids *t, const uint8_t *term, uint64_t len, uint64_t *id) {
  if (!t || !id) return AM_ERR_INVALID;
  std::string k;
  const int rc = canonical(term, len, k);
  if (rc != AM_OK) {
    am_set_error("am_txid_intern: %s external term", rc == AM_ERR_UNSUPPORTED ? "unsupported" : "malformed");
    return rc;
  }
  std::lock_guard<std::mutex> g(t->mu);
  am_txid_ent &e = t->ids[k];
  if (!e.id) e.id = t->next++;
  e.held = true;
  *id = e.id;
  return AM_OK;
}

int am_txid_intern_op(am_txids *t, const uint8_t *term, uint64_t len, uint32_t dc, uint64_t ct, uint64_t *id) {
  if (!t || !id) return AM_ERR_INVALID;
  std::string k;
  const int rc = canonical(term, len, k);
  if (rc != AM_OK) {
    am_set_error("am_txid_intern_op: %s external term", rc == AM_ERR_UNSUPPORTED ? "unsupported" : "malformed");
    return rc;
  }
  std::lock_guard<std::mutex> g(t->mu);
  auto it = t->ids.find(k);
  if (it == t->ids.end()) it = t->ids.emplace(k, am_txid_ent{}).first;
  am_txid_ent &e = it->second;
  if (!e.id) e.id = t->next++;
  if (!e.stamped || e.dc != dc || e.ct < ct) {  // every op of a transaction carries one commit time
    e.stamped = true, e.dc = dc, e.ct = ct;
    t->by_ct[dc].emplace(ct, k);
  }
  *id = e.id;
  return AM_OK;
}

int am_txid_lookup(am_txids *t, const uint8_t *term, uint64_t len, uint64_t *id) {
  if (!t || !id) return AM_ERR_INVALID;
  std::string k;
  const int rc = canonical(term, len, k);
  if (rc != AM_OK) return rc;
  std::lock_guard<std::mutex> g(t->mu);
  auto it = t->ids.find(k);
  if (it == t->ids.end()) return AM_CODEC_ABSENT;
  *id = it->second.id;
  return AM_OK;
}

int am_txid_forget(am_txids *t, const uint8_t *term, uint64_t len) {
  if (!t) return AM_ERR_INVALID;
  std::string k;
  const int rc = canonical(term, len, k);
  if (rc != AM_OK) return rc;
  std::lock_guard<std::mutex> g(t->mu);
  return t->ids.erase(k) ? AM_OK : AM_CODEC_ABSENT;
}

int am_txid_expire(am_txids *t, uint32_t n_dc, const uint64_t *stable_vc, uint32_t stable_pres, uint64_t *dropped) {
  if (!t || (n_dc && !stable_vc) || n_dc > 32) return AM_ERR_INVALID;
  std::lock_guard<std::mutex> g(t->mu);
  uint64_t n = 0;
  for (auto &dm : t->by_ct) {
    const uint32_t dc = dm.first;
    if (dc >= n_dc || !((stable_pres >> dc) & 1u)) continue;  // a DC the stable snapshot lacks
    auto &idx = dm.second;
    const uint64_t s = stable_vc[dc];
    while (!idx.empty() && idx.begin()->first <= s) {
      auto ie = idx.begin();
      auto it = t->ids.find(ie->second);
      if (it != t->ids.end() && it->second.stamped && it->second.dc == dc && it->second.ct == ie->first) {
        if (it->second.held) it->second.stamped = false;  // a reader still holds it: forget drops it
        else t->ids.erase(it), ++n;
      }
      idx.erase(ie);
    }
  }
  if (dropped) *dropped = n;
  return AM_OK;
}

uint64_t am_txid_size(am_txids *t) {
  if (!t) return 0;
  std::lock_guard<std::mutex> g(t->mu);
  return t->ids.size();
}

int am_txid_canonical(const uint8_t *term, uint64_t len, uint8_t *buf, uint64_t cap, uint64_t *out_len) {
  if (!out_len) return AM_ERR_INVALID;
  std::string k;
  const int rc = canonical(term, len, k);
  if (rc != AM_OK) return rc;
  *out_len = (uint64_t)k.size() + 1;
  if (!buf || cap < *out_len) return AM_ERR_CAPACITY;
  buf[0] = 131;
  memcpy(buf + 1, k.data(), k.size());
  return AM_OK;
}

}  // extern "C"
