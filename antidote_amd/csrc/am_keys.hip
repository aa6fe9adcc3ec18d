// am_keys.hip -- log_utilities:convert_key/1 + get_key_partition/1 (src/log_utilities.erl:
// 60-79, 100-118) for the keys the NIF hands over as bytes (host code):
//   binary key whose text is an integer  list_to_integer(binary_to_list(Key)): optional sign,
//                                        decimal digits, any length -> abs(...) rem N
//   any other binary key                 riak_core_util:chash_key({?BUCKET, Key}) =
//                                        SHA-1 of term_to_binary({<<"antidote">>, Key})
//   any other term (not an integer)      chash_key({?BUCKET, term_to_binary(Key)}): the caller
//                                        passes term_to_binary(Key) (enif_term_to_binary)
// then crypto:bytes_to_integer (big-endian) rem N; the partition is that index (Pos - 1 in
// get_primaries_preflist/1).  Integer keys: am_key_partition (am_runtime.hip).
#include <cstring>

#include "am_internal.h"

namespace {

struct Sha1 {
  uint32_t h[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
  uint8_t buf[64];
  uint64_t n = 0;  // bytes hashed
  static uint32_t rol(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }
  void block(const uint8_t *p) {
    uint32_t w[80];
    for (int i = 0; i < 16; ++i) w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
    for (int i = 16; i < 80; ++i) w[i] = rol(w[i - 3] ^ w[i - 8] ^ w[i - 14] ^ w[i - 16], 1);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
    for (int i = 0; i < 80; ++i) {
      uint32_t f, k;
      if (i < 20) f = (b & c) | (~b & d), k = 0x5A827999u;
      else if (i < 40) f = b ^ c ^ d, k = 0x6ED9EBA1u;
      else if (i < 60) f = (b & c) | (b & d) | (c & d), k = 0x8F1BBCDCu;
      else f = b ^ c ^ d, k = 0xCA62C1D6u;
      const uint32_t t = rol(a, 5) + f + e + k + w[i];
      e = d, d = c, c = rol(b, 30), b = a, a = t;
    }
    h[0] += a, h[1] += b, h[2] += c, h[3] += d, h[4] += e;
  }
  void update(const uint8_t *p, uint64_t len) {
    for (uint64_t i = 0; i < len; ++i) {
      buf[n % 64] = p[i];
      if (++n % 64 == 0) block(buf);
    }
  }
  void digest(uint8_t out[20]) {
    const uint64_t bits = n * 8;
    const uint8_t one = 0x80, zero = 0;
    update(&one, 1);
    while (n % 64 != 56) update(&zero, 1);
    uint8_t l[8];
    for (int i = 0; i < 8; ++i) l[i] = (uint8_t)(bits >> (56 - 8 * i));
    update(l, 8);
    for (int i = 0; i < 5; ++i)
      for (int j = 0; j < 4; ++j) out[4 * i + j] = (uint8_t)(h[i] >> (24 - 8 * j));
  }
};

// big-endian unsigned bytes rem m
uint32_t bytes_rem(const uint8_t *p, uint64_t len, uint32_t m) {
  uint64_t r = 0;
  for (uint64_t i = 0; i < len; ++i) r = ((r << 8) | p[i]) % m;
  return (uint32_t)r;
}

// list_to_integer/1 on the key's text: [+-]?[0-9]+ -> abs(value) rem m; false if not an integer
bool int_text_rem(const uint8_t *p, uint64_t len, uint32_t m, uint32_t *out) {
  uint64_t i = 0;
  if (len && (p[0] == '+' || p[0] == '-')) i = 1;
  if (i == len) return false;
  uint64_t r = 0;
  for (; i < len; ++i) {
    if (p[i] < '0' || p[i] > '9') return false;
    r = (r * 10 + (p[i] - '0')) % m;
  }
  *out = (uint32_t)r;
  return true;
}

}  // namespace

extern "C" {

int am_chash_key(const uint8_t *bytes, uint64_t len, uint8_t out[20]) {
  if ((!bytes && len) || !out) return AM_ERR_INVALID;
  // term_to_binary({<<"antidote">>, Bytes}): SMALL_TUPLE_EXT of two BINARY_EXT
  static const uint8_t head[] = {131, 104, 2, 109, 0, 0, 0, 8, 'a', 'n', 't', 'i', 'd', 'o', 't', 'e', 109};
  const uint8_t blen[4] = {(uint8_t)(len >> 24), (uint8_t)(len >> 16), (uint8_t)(len >> 8), (uint8_t)len};
  Sha1 s;
  s.update(head, sizeof(head));
  s.update(blen, 4);
  s.update(bytes, len);
  s.digest(out);
  return AM_OK;
}

uint32_t am_key_partition_bytes(const uint8_t *bytes, uint64_t len, int kind, uint32_t n_partitions) {
  if (n_partitions == 0 || (!bytes && len)) return 0;
  uint32_t r = 0;
  if (kind == AM_KEY_BINARY && int_text_rem(bytes, len, n_partitions, &r)) return r;
  uint8_t d[20];
  am_chash_key(bytes, len, d);
  return bytes_rem(d, 20, n_partitions);
}

}  // extern "C"
