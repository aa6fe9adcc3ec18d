// am_codec.hip -- the term codec at the boundary: Erlang terms <-> the u64 words of the op
// log, the snapshot cache and the results.
//
// The device never does arithmetic on a CRDT value, element or token: it only compares them
// (equality: a remove kills the tokens it observed; order: the add-wins set is an orddict by
// element, the MV register an ordered list of {Value, Token}, the LWW register a max of
// {Timestamp, Value} -- antidote_crdt, used by clocksi_materializer:materialize_intern/11).
// So a partition interns every such term into a LABEL whose u64 order is Erlang term order
// (number < atom < ... < tuple < map < nil < list < bitstring): sorting labels on the device
// gives the reference's orddict order, and decoding the labels gives back the terms.
//
// Terms arrive in the external term format (enif_term_to_binary; the NIF of INTEGRATION.md)
// and are compared by a restatement of the runtime's term order over the parsed form:
// integers (small, 32-bit, big) and floats by value, atoms by text, tuples by arity then
// elements, lists element-wise (nil first, improper tails as terms), bitstrings bit-wise.
// Maps, pids, ports, references and funs are not CRDT payloads here: AM_ERR_UNSUPPORTED.
// Terms that compare equal (1 and 1.0) share a label, as orddict keys do.
//
// Labels lie in [1, 2^64 - 2] (0 and ~0 are the kernels' "none" sentinels).  A new term gets
// a label between its neighbours' (a fixed stride past the last one, the midpoint inside);
// when a gap is used up every label is re-spread evenly, ORDER PRESERVED.  The caller then
// takes the old -> new map (am_codec_take_relabel) and applies it to every device structure
// holding labels (am_store_relabel, am_snapcache_relabel, am_vnode_relabel) before it puts
// the labels of the relabelling call on the device; interning is refused until then.
#include <algorithm>
#include <cmath>
#include <memory>
#include <set>
#include <string>
#include <unordered_map>

#include "am_internal.h"

namespace {

// ---------------------------------------------------------------- parsed terms
enum Cls : uint8_t { C_NUM = 0, C_ATOM = 1, C_TUPLE = 6, C_NIL = 8, C_LIST = 9, C_BITS = 10 };

struct Node {
  Cls cls = C_NIL;
  bool is_float = false, neg = false;
  double f = 0;
  std::string mag;   // integers: big-endian magnitude without leading zeros
  std::string text;  // atom (UTF-8) / bitstring bytes
  uint8_t last_bits = 8;  // bitstring: bits used in the last byte
  std::vector<Node> kids;             // tuple elements / list elements
  std::unique_ptr<Node> tail;         // list: improper tail (null = [])
};

struct Parser {
  const uint8_t *p, *e;
  bool ok = true;
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
  std::string bytes(uint64_t n) {
    if (!need(n)) return std::string();
    std::string s((const char *)p, n);
    p += n;
    return s;
  }
  static std::string strip(std::string be) {
    size_t i = 0;
    while (i < be.size() && be[i] == 0) ++i;
    return be.substr(i);
  }
  void set_int(Node &n, bool neg, std::string be_mag) {
    n.cls = C_NUM;
    n.mag = strip(std::move(be_mag));
    n.neg = neg && !n.mag.empty();
  }
  static std::string latin1_to_utf8(const std::string &s) {
    std::string o;
    for (unsigned char ch : s) {
      if (ch < 0x80) o += (char)ch;
      else o += (char)(0xC0 | (ch >> 6)), o += (char)(0x80 | (ch & 0x3F));
    }
    return o;
  }
  int term(Node &n, int depth) {
    if (depth > 512) return AM_ERR_UNSUPPORTED;
    const uint32_t tag = u8();
    if (!ok) return AM_ERR_INVALID;
    switch (tag) {
      case 97: {  // SMALL_INTEGER_EXT
        const uint32_t v = u8();
        set_int(n, false, std::string(1, (char)v));
        break;
      }
      case 98: {  // INTEGER_EXT (signed 32)
        const int32_t v = (int32_t)u32();
        const uint32_t a = v < 0 ? (uint32_t)(-(int64_t)v) : (uint32_t)v;
        std::string be(4, 0);
        for (int i = 0; i < 4; ++i) be[i] = (char)(a >> (24 - 8 * i));
        set_int(n, v < 0, be);
        break;
      }
      case 110: case 111: {  // SMALL_BIG_EXT / LARGE_BIG_EXT: little-endian digits
        const uint32_t len = tag == 110 ? u8() : u32();
        const bool neg = u8() != 0;
        std::string le = bytes(len);
        std::reverse(le.begin(), le.end());
        set_int(n, neg, le);
        break;
      }
      case 70: {  // NEW_FLOAT_EXT
        uint64_t b = (uint64_t)u32() << 32;
        b |= u32();
        n.cls = C_NUM;
        n.is_float = true;
        memcpy(&n.f, &b, 8);
        if (!std::isfinite(n.f)) return AM_ERR_INVALID;
        break;
      }
      case 100: case 115: case 118: case 119: {  // ATOM_EXT, SMALL_ATOM_EXT, *_UTF8_EXT
        const uint32_t len = (tag == 100 || tag == 118) ? u16() : u8();
        n.cls = C_ATOM;
        n.text = bytes(len);
        if (tag == 100 || tag == 115) n.text = latin1_to_utf8(n.text);
        break;
      }
      case 104: case 105: {  // SMALL_TUPLE_EXT / LARGE_TUPLE_EXT
        const uint32_t ar = tag == 104 ? u8() : u32();
        if (!ok || ar > (uint64_t)(e - p)) return AM_ERR_INVALID;
        n.cls = C_TUPLE;
        n.kids.resize(ar);
        for (auto &k : n.kids)
          if (int rc = term(k, depth + 1)) return rc;
        break;
      }
      case 106:  // NIL_EXT
        n.cls = C_NIL;
        break;
      case 107: {  // STRING_EXT: a list of bytes
        const uint32_t len = u16();
        const std::string s = bytes(len);
        n.cls = len ? C_LIST : C_NIL;
        n.kids.resize(s.size());
        for (size_t i = 0; i < s.size(); ++i) set_int(n.kids[i], false, std::string(1, s[i]));
        break;
      }
      case 108: {  // LIST_EXT: len elements, then the tail
        const uint32_t len = u32();
        if (!ok || len > (uint64_t)(e - p)) return AM_ERR_INVALID;
        n.cls = C_LIST;
        n.kids.resize(len);
        for (auto &k : n.kids)
          if (int rc = term(k, depth + 1)) return rc;
        Node t;
        if (int rc = term(t, depth + 1)) return rc;
        if (t.cls == C_LIST) {  // a proper continuation: flatten
          for (auto &k : t.kids) n.kids.push_back(std::move(k));
          n.tail = std::move(t.tail);
        } else if (t.cls != C_NIL) {
          n.tail.reset(new Node(std::move(t)));
        }
        if (n.kids.empty() && !n.tail) n.cls = C_NIL;
        break;
      }
      case 109: {  // BINARY_EXT
        const uint32_t len = u32();
        n.cls = C_BITS;
        n.text = bytes(len);
        break;
      }
      case 77: {  // BIT_BINARY_EXT
        const uint32_t len = u32();
        const uint32_t bits = u8();
        n.cls = C_BITS;
        n.text = bytes(len);
        if (!ok || bits < 1 || bits > 8 || len == 0) return AM_ERR_INVALID;
        n.last_bits = (uint8_t)bits;
        n.text.back() = (char)((uint8_t)n.text.back() & (uint8_t)(0xFF << (8 - bits)));
        break;
      }
      default:
        return AM_ERR_UNSUPPORTED;  // maps, pids, ports, references, funs, compressed
    }
    return ok ? AM_OK : AM_ERR_INVALID;
  }
};

int parse_etf(const uint8_t *b, uint64_t len, Node &n) {
  if (!b || len < 2 || b[0] != 131) return AM_ERR_INVALID;
  Parser P{b + 1, b + len};
  int rc = P.term(n, 0);
  if (!rc && P.p != P.e) rc = AM_ERR_INVALID;  // trailing bytes
  return rc;
}

// ---------------------------------------------------------------- term order
int sgn(int x) { return (x > 0) - (x < 0); }

int cmp_mag(const std::string &a, const std::string &b) {
  if (a.size() != b.size()) return a.size() < b.size() ? -1 : 1;
  return sgn(memcmp(a.data(), b.data(), a.size()));
}

long double as_ld(const Node &n) {
  if (n.is_float) return n.f;
  long double v = 0;
  for (unsigned char ch : n.mag) v = v * 256 + ch;
  return n.neg ? -v : v;
}

int cmp_num(const Node &a, const Node &b) {
  if (!a.is_float && !b.is_float) {
    if (a.neg != b.neg) return a.neg ? -1 : 1;
    const int m = cmp_mag(a.mag, b.mag);
    return a.neg ? -m : m;
  }
  const long double x = as_ld(a), y = as_ld(b);
  return (x > y) - (x < y);
}

int cmp_bits(const Node &a, const Node &b) {
  const uint64_t la = a.text.empty() ? 0 : (a.text.size() - 1) * 8 + a.last_bits;
  const uint64_t lb = b.text.empty() ? 0 : (b.text.size() - 1) * 8 + b.last_bits;
  const uint64_t full = std::min(la, lb) / 8;
  if (int c = memcmp(a.text.data(), b.text.data(), full)) return sgn(c);
  for (uint64_t i = full * 8; i < std::min(la, lb); ++i) {
    const int x = ((uint8_t)a.text[i / 8] >> (7 - i % 8)) & 1, y = ((uint8_t)b.text[i / 8] >> (7 - i % 8)) & 1;
    if (x != y) return x < y ? -1 : 1;
  }
  return (la > lb) - (la < lb);
}

int cmp(const Node &a, const Node &b);

// a list from element i on: a cons cell while elements remain, then the tail term
int cmp_list(const Node &a, const Node &b) {
  static const Node nil;
  size_t i = 0;
  for (;; ++i) {
    const bool ca = i < a.kids.size(), cb = i < b.kids.size();
    if (ca && cb) {
      if (int c = cmp(a.kids[i], b.kids[i])) return c;
      continue;
    }
    const Node &ta = a.tail ? *a.tail : nil, &tb = b.tail ? *b.tail : nil;
    if (ca) return tb.cls < C_LIST ? 1 : -1;   // cons vs a non-list tail (tail classes are never C_LIST)
    if (cb) return ta.cls < C_LIST ? -1 : 1;
    return cmp(ta, tb);
  }
}

int cmp(const Node &a, const Node &b) {
  if (a.cls != b.cls) return a.cls < b.cls ? -1 : 1;
  switch (a.cls) {
    case C_NUM: return cmp_num(a, b);
    case C_ATOM: {
      const int c = memcmp(a.text.data(), b.text.data(), std::min(a.text.size(), b.text.size()));
      return c ? sgn(c) : (a.text.size() > b.text.size()) - (a.text.size() < b.text.size());
    }
    case C_TUPLE: {
      if (a.kids.size() != b.kids.size()) return a.kids.size() < b.kids.size() ? -1 : 1;
      for (size_t i = 0; i < a.kids.size(); ++i)
        if (int c = cmp(a.kids[i], b.kids[i])) return c;
      return 0;
    }
    case C_NIL: return 0;
    case C_LIST: return cmp_list(a, b);
    case C_BITS: return cmp_bits(a, b);
  }
  return 0;
}

// ---------------------------------------------------------------- the dictionary
struct Entry {
  std::string etf;
  Node node;
  uint64_t label = 0;
  uint64_t dev = 0;  // the label the caller's device state holds (differs after a relabel)
};
struct Less {
  bool operator()(const Entry *a, const Entry *b) const { return cmp(a->node, b->node) < 0; }
};

constexpr uint64_t LMIN = 1, LMAX = ~0ull - 1;  // usable labels [LMIN, LMAX]
constexpr uint64_t STRIDE = 1ull << 32;         // spacing of labels appended at either end

}  // namespace

struct am_codec {
  std::mutex mu;
  std::set<Entry *, Less> ord;
  std::unordered_map<std::string, Entry *> by_etf;
  std::unordered_map<uint64_t, Entry *> by_label;
  std::vector<std::unique_ptr<Entry>> all;
  bool pending = false;
  uint64_t relabels = 0;

  void respread() {
    const uint64_t n = ord.size();
    const uint64_t step = (LMAX - LMIN) / (n + 1);
    uint64_t i = 1;
    by_label.clear();
    for (Entry *e : ord) {
      e->label = LMIN + step * i++;
      by_label[e->label] = e;
    }
    pending = true;
    ++relabels;
  }
  // the label for a new entry at position `it` of ord (before insertion); false: no room
  bool place(std::set<Entry *, Less>::iterator it, uint64_t &out) {
    const bool first = it == ord.begin(), last = it == ord.end();
    const uint64_t lo = first ? LMIN - 1 : (*std::prev(it))->label;  // exclusive bounds
    const uint64_t hi = last ? LMAX + 1 : (*it)->label;
    if (hi - lo < 2) return false;
    if (last && !first && hi - lo > 2 * STRIDE) out = lo + STRIDE;
    else if (first && !last && hi - lo > 2 * STRIDE) out = hi - STRIDE;
    else out = lo + (hi - lo) / 2;
    return true;
  }
  int intern(const uint8_t *b, uint64_t len, Entry **out, std::vector<Entry *> &created) {
    std::string key((const char *)b, len);
    auto f = by_etf.find(key);
    if (f != by_etf.end()) {
      *out = f->second;
      return AM_OK;
    }
    std::unique_ptr<Entry> e(new Entry());
    if (int rc = parse_etf(b, len, e->node)) return rc;
    auto it = ord.lower_bound(e.get());
    if (it != ord.end() && cmp((*it)->node, e->node) == 0) {  // an equal term, other bytes
      by_etf[key] = *it;
      *out = *it;
      return AM_OK;
    }
    uint64_t lab = 0;
    if (!place(it, lab)) {
      respread();
      it = ord.lower_bound(e.get());
      if (!place(it, lab)) return AM_ERR_NOMEM;  // 2^64 - 2 terms
    }
    e->etf = std::move(key);
    e->label = e->dev = lab;
    Entry *p = e.get();
    ord.insert(it, p);
    by_etf[p->etf] = p;
    by_label[lab] = p;
    all.push_back(std::move(e));
    created.push_back(p);
    *out = p;
    return AM_OK;
  }
};

extern "C" {

int am_codec_create(am_codec **out) {
  if (!out) return AM_ERR_INVALID;
  *out = new am_codec();
  return AM_OK;
}

int am_codec_destroy(am_codec *c) {
  delete c;
  return AM_OK;
}

int am_codec_compare(const uint8_t *a, uint64_t la, const uint8_t *b, uint64_t lb, int *out) {
  if (!out) return AM_ERR_INVALID;
  Node x, y;
  if (int rc = parse_etf(a, la, x)) return rc;
  if (int rc = parse_etf(b, lb, y)) return rc;
  *out = cmp(x, y);
  return AM_OK;
}

int am_codec_intern(am_codec *c, uint64_t n, const uint8_t *const *terms, const uint64_t *lens, uint64_t *labels,
                    int *relabeled) {
  if (!c || (n && (!terms || !lens || !labels))) return AM_ERR_INVALID;
  std::lock_guard<std::mutex> g(c->mu);
  if (c->pending) {
    am_set_error("am_codec_intern: a relabel map is pending (am_codec_take_relabel first)");
    return AM_ERR_INVALID;
  }
  const uint64_t before = c->relabels;
  std::vector<Entry *> got(n, nullptr), created;
  int rc = AM_OK;
  uint64_t i = 0;
  for (; i < n && !rc; ++i) rc = c->intern(terms[i], lens[i], &got[i], created);
  // the terms this call created are not on the device yet: they hold the current labelling
  for (Entry *e : created) e->dev = e->label;
  for (uint64_t j = 0; j < n && got[j]; ++j) labels[j] = got[j]->label;
  const bool rl = c->relabels != before;
  if (rc) {
    am_set_error("am_codec_intern: term %llu: %s", (unsigned long long)(i - 1),
                 rc == AM_ERR_UNSUPPORTED ? "unsupported term (map, pid, port, reference, fun)" : "malformed term");
    if (relabeled) *relabeled = rl ? 1 : 0;  // a relabel still has to reach the device
    return rc;
  }
  if (relabeled) *relabeled = rl ? 1 : 0;
  return AM_OK;
}

int am_codec_lookup(am_codec *c, const uint8_t *term, uint64_t len, uint64_t *label) {
  if (!c || !term || !label) return AM_ERR_INVALID;
  std::lock_guard<std::mutex> g(c->mu);
  auto f = c->by_etf.find(std::string((const char *)term, len));
  if (f != c->by_etf.end()) {
    *label = f->second->label;
    return AM_OK;
  }
  Entry probe;
  if (int rc = parse_etf(term, len, probe.node)) return rc;
  auto it = c->ord.find(&probe);
  if (it == c->ord.end()) return AM_CODEC_ABSENT;
  *label = (*it)->label;
  return AM_OK;
}

int am_codec_term(am_codec *c, uint64_t label, uint8_t *buf, uint64_t cap, uint64_t *len) {
  if (!c || !len) return AM_ERR_INVALID;
  std::lock_guard<std::mutex> g(c->mu);
  auto f = c->by_label.find(label);
  if (f == c->by_label.end()) return AM_ERR_INVALID;
  const std::string &s = f->second->etf;
  *len = s.size();
  if (buf && cap >= s.size()) memcpy(buf, s.data(), s.size());
  return (buf && cap < s.size()) ? AM_ERR_CAPACITY : AM_OK;
}

uint64_t am_codec_size(am_codec *c) {
  if (!c) return 0;
  std::lock_guard<std::mutex> g(c->mu);
  return c->ord.size();
}

int am_codec_take_relabel(am_codec *c, uint64_t *old_labels, uint64_t *new_labels, uint64_t cap, uint64_t *n) {
  if (!c || !n) return AM_ERR_INVALID;
  std::lock_guard<std::mutex> g(c->mu);
  uint64_t m = 0;
  for (Entry *e : c->ord) m += e->dev != e->label;
  *n = m;
  if (!old_labels || !new_labels) return AM_OK;  // size query
  if (cap < m) return AM_ERR_CAPACITY;
  uint64_t i = 0;
  for (Entry *e : c->ord)  // term order == old-label order (relabelling preserves order)
    if (e->dev != e->label) {
      old_labels[i] = e->dev;
      new_labels[i] = e->label;
      e->dev = e->label;
      ++i;
    }
  c->pending = false;
  return AM_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- device relabelling
namespace {

__device__ __forceinline__ void relabel_word(uint64_t *w, const uint64_t *old, const uint64_t *nw, uint64_t n) {
  const uint64_t x = *w;
  if (x == 0 || x == ~0ull) return;  // the kernels' sentinels are never labels
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) / 2;
    if (old[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  if (lo < n && old[lo] == x) *w = nw[lo];
}

// one wave per key: the label words of its ops (by type) and of its token groups
__global__ void k_store_relabel(am_op_log L, uint64_t *p0, uint64_t *p1, uint64_t *vd, uint64_t *grp,
                                const uint64_t *old, const uint64_t *nw, uint64_t n) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / 64);
  for (uint64_t k = (uint64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64; k < L.n_keys; k += waves) {
    const uint32_t t = L.key_type[k];
    if (t != AM_LWW && t != AM_AWSET && t != AM_MVREG) continue;
    for (uint64_t p = L.key_off[k] + lane; p < am_kend(L, k); p += 64) {
      if (t == AM_LWW) {
        relabel_word(p1 + p, old, nw, n);  // {Ts, Value}: the value
        continue;
      }
      const uint64_t vo = L.var_off ? L.var_off[p] : 0, ve = L.var_off ? L.var_off[p + 1] : 0;
      if (t == AM_MVREG) {  // {Value, Token, Overridden}
        relabel_word(p0 + p, old, nw, n);
        relabel_word(p1 + p, old, nw, n);
        for (uint64_t q = vo; q < ve; ++q) relabel_word(vd + q, old, nw, n);
        continue;
      }
      for (uint64_t q = vo; q + 3 <= ve;) {  // [{Elem, AddTokens, RemoveTokens}]: [elem, na, nr, tok...]
        const uint64_t na = vd[q + 1], nr = vd[q + 2];
        if (na > ve - q || nr > ve - q || q + 3 + na + nr > ve) break;  // malformed: Type:update raises anyway
        relabel_word(vd + q, old, nw, n);
        for (uint64_t j = 0; j < na + nr; ++j) relabel_word(vd + q + 3 + j, old, nw, n);
        q += 3 + na + nr;
      }
    }
    if (grp && L.key_ngrp && L.rec_key_off && t != AM_LWW) {
      const uint32_t ng = am_ngrp_count(L.key_ngrp[k]);
      if (ng == 0) continue;
      const uint64_t r0 = L.rec_key_off[k];
      for (uint32_t j = lane; j < ng; j += 64) {
        relabel_word(grp + 2 * (r0 + j), old, nw, n);
        relabel_word(grp + 2 * (r0 + j) + 1, old, nw, n);
      }
      if (L.prec && L.rec_g && !am_ngrp_big(L.key_ngrp[k])) {  // the birth-ordered pairs of its births
        uint64_t *pr = const_cast<uint64_t *>(L.prec);
        for (uint64_t r = r0 + lane; r < am_rkend(L, k); r += 64) {
          const uint32_t x = L.rec_g[r];
          if (x == 0xFFFFFFFFu || (x & AM_REC_KILL)) continue;
          relabel_word(pr + 2 * r, old, nw, n);
          relabel_word(pr + 2 * r + 1, old, nw, n);
        }
      }
    }
  }
}

}  // namespace

// the old -> new map in device memory (caller frees with hipFree)
int am_relabel_upload(am_ctx *c, const uint64_t *old_labels, const uint64_t *new_labels, uint64_t n, uint64_t **d_old,
                      uint64_t **d_new) {
  for (uint64_t i = 1; i < n; ++i)
    if (old_labels[i - 1] >= old_labels[i]) {
      am_set_error("relabel: old labels must be strictly increasing (am_codec_take_relabel order)");
      return AM_ERR_INVALID;
    }
  *d_old = *d_new = nullptr;
  if (hipMalloc((void **)d_old, n * 8) != hipSuccess || hipMalloc((void **)d_new, n * 8) != hipSuccess) {
    if (*d_old) (void)hipFree(*d_old);
    *d_old = nullptr;
    am_set_error("relabel: out of device memory");
    return AM_ERR_NOMEM;
  }
  if (hipMemcpyAsync(*d_old, old_labels, n * 8, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
      hipMemcpyAsync(*d_new, new_labels, n * 8, hipMemcpyHostToDevice, c->stream) != hipSuccess) {
    (void)hipFree(*d_old);
    (void)hipFree(*d_new);
    am_set_error("relabel: upload failed");
    return AM_ERR_HIP;
  }
  return AM_OK;
}

extern "C" int am_store_relabel(am_ctx *c, am_store *st, const uint64_t *old_labels, const uint64_t *new_labels,
                                uint64_t n) {
  if (!c || !st || (n && (!old_labels || !new_labels))) return AM_ERR_INVALID;
  AM_LOCK(c);
  if (n == 0 || st->dev.n_keys == 0) return AM_OK;
  AM_HIP(hipSetDevice(c->device));
  uint64_t *d_old = nullptr, *d_new = nullptr;
  if (int rc = am_relabel_upload(c, old_labels, new_labels, n, &d_old, &d_new)) return rc;
  const am_op_log &L = st->dev;
  const uint64_t blocks = (L.n_keys + 3) / 4 < 65536 ? (L.n_keys + 3) / 4 : 65536;
  hipLaunchKernelGGL(k_store_relabel, dim3((unsigned)blocks), dim3(256), 0, c->stream, L, const_cast<uint64_t *>(L.p0),
                     const_cast<uint64_t *>(L.p1), const_cast<uint64_t *>(L.var_data), const_cast<uint64_t *>(L.grp),
                     d_old, d_new, n);
  const bool ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(c->stream) == hipSuccess;
  (void)hipFree(d_old);
  (void)hipFree(d_new);
  if (!ok) {
    am_set_error("am_store_relabel: kernel failed");
    return AM_ERR_HIP;
  }
  return AM_OK;
}
