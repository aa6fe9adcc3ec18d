// synth.h -- deterministic synthetic op logs (bench + parity), shared by the
// device generator kernel and the host regenerator (am_synth_host).
//
// Counter-based: every field of op i of key k is a pure function of
// (seed, k, i), so any key range can be regenerated on the host to check the
// device results against the oracle without copying the whole log back.
//
// Model (one timeline per key; D = n_dc):
//   g(i)          = BASE + i*STEP + jitter(k,i)       jitter < STEP, so g is strictly
//                                                     increasing in i (g(j<0) = BASE + j*STEP)
//   commit_dc(i)  = h(k,i,1) mod D
//   commit_time(i)= g(i)
//   snap_vc(i)[d] = g(i - lag_d), lag_d = 1 + h(k,i,2+d) mod max_lag   (causally earlier;
//                   snap_vc[commit_dc] < commit_time as ClockSI guarantees)
//   read clock(q) = BASE + floor(q * N) * STEP + d * STEP/2   per DC d
//   (esc_ppm > 0: a fraction of ops carry one remote DC's entry 2^33 us behind, am_syn_snap_e)
// Payloads:
//   PN   delta uniform in [-1000, 1000]
//   LWW  ts = BASE + perm_k(i) * STEP + jitter  (perm_k a bijection of [0, 2^ceil(log2 N)),
//        so timestamps are unique per key and not ordered like commits); value = h(k,i,20)
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define AM_HD __host__ __device__ __forceinline__
#else
#define AM_HD static inline
#endif

#define AM_SYN_BASE 1700000000000000ull
#define AM_SYN_STEP 1000ull

AM_HD uint64_t am_splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

AM_HD uint64_t am_syn_h(uint64_t seed, uint64_t key, uint64_t i, uint64_t stream) {
  return am_splitmix64(seed ^ am_splitmix64(key * 0xD1B54A32D192ED03ull ^
                                             (i * 0x8CB92BA72F3D8DD7ull + stream * 0x9E3779B97F4A7C15ull)));
}

AM_HD uint64_t am_syn_g(uint64_t seed, uint64_t key, int64_t i) {
  if (i < 0) return (uint64_t)((int64_t)AM_SYN_BASE + i * (int64_t)AM_SYN_STEP);
  return AM_SYN_BASE + (uint64_t)i * AM_SYN_STEP + am_syn_h(seed, key, (uint64_t)i, 0) % AM_SYN_STEP;
}

AM_HD uint32_t am_syn_dc(uint64_t seed, uint64_t key, uint64_t i, uint32_t n_dc) {
  return (uint32_t)(am_syn_h(seed, key, i, 1) % n_dc);
}

AM_HD uint64_t am_syn_snap(uint64_t seed, uint64_t key, uint64_t i, uint32_t d, uint32_t max_lag) {
  uint64_t lag = 1 + am_syn_h(seed, key, i, 2 + d) % (max_lag ? max_lag : 1);
  return am_syn_g(seed, key, (int64_t)i - (int64_t)lag);
}

// A lagging DC (the packed view's escape path): with probability esc_ppm / 10^6 an op's
// snapshot entry of one remote DC -- never its commit DC, whose entry the commit time replaces
// in the inclusion test -- lags by AM_SYN_ESC_LAG us (2.4 h), outside the 2^32-us window of the
// packed view around the key's time base.  snapshot_time is a full vectorclock
// (include/antidote.hrl:197-204); a partitioned DC's entry stays where the partition left it
// (src/inter_dc_dep_vnode.erl:206-232), so such entries are real, and the view escapes the op.
#define AM_SYN_ESC_LAG (1ull << 33)
AM_HD uint64_t am_syn_snap_e(uint64_t seed, uint64_t key, uint64_t i, uint32_t d, uint32_t max_lag, uint32_t n_dc,
                             uint32_t esc_ppm) {
  const uint64_t s = am_syn_snap(seed, key, i, d, max_lag);
  if (!esc_ppm || n_dc < 2 || am_syn_h(seed, key, i, 60) % 1000000u >= esc_ppm) return s;
  const uint32_t cdc = (uint32_t)(am_syn_h(seed, key, i, 1) % n_dc);  // am_syn_dc
  const uint32_t ed = (cdc + 1u + (uint32_t)(am_syn_h(seed, key, i, 61) % (n_dc - 1))) % n_dc;
  return d == ed ? s - AM_SYN_ESC_LAG : s;
}

AM_HD uint64_t am_syn_read_clock(uint64_t n_ops_per_key, double q, uint32_t d) {
  uint64_t pos = (uint64_t)(q * (double)n_ops_per_key);
  return AM_SYN_BASE + pos * AM_SYN_STEP + (uint64_t)d * (AM_SYN_STEP / 2);
}

AM_HD int64_t am_syn_pn_delta(uint64_t seed, uint64_t key, uint64_t i) {
  return (int64_t)(am_syn_h(seed, key, i, 10) % 2001) - 1000;
}

AM_HD uint64_t am_syn_lww_ts(uint64_t seed, uint64_t key, uint64_t i, uint32_t n) {
  uint32_t bits = 0;
  while ((1u << bits) < n) ++bits;
  uint64_t mask = bits >= 63 ? ~0ull : ((1ull << bits) - 1);
  uint64_t hk = am_syn_h(seed, key, 0, 21);
  uint64_t a = (hk | 1ull), b = hk >> 17;
  uint64_t perm = (i * a + b) & mask;
  return AM_SYN_BASE + perm * AM_SYN_STEP + am_syn_h(seed, key, i, 22) % AM_SYN_STEP;
}

AM_HD uint64_t am_syn_lww_val(uint64_t seed, uint64_t key, uint64_t i) {
  return am_syn_h(seed, key, i, 20);
}

// ---- mixed workloads: the key's CRDT type ----
//   C4 mixed (type 0): 40% PN, 20% LWW, 20% AW-set, 20% MV register
//   C5 (type 6):       50% MV register, 50% bounded counter
AM_HD uint32_t am_syn_key_type(uint64_t seed, uint64_t key, uint32_t type) {
  const uint64_t h = am_syn_h(seed, key, 0, 40) % 10;
  if (type == 0) return h < 4 ? 1u : h < 6 ? 2u : h < 8 ? 3u : 4u;
  if (type == 6) return h < 5 ? 4u : 5u;
  return type;
}

// ---- add-wins set: causal history, every op observes every earlier op ----
// Op i touches element elem(i) = (i*A + B) mod U (U a power of two, A odd: a
// bijection on each period of U ops, so the previous op on the same element is
// op i-U).  70% adds {e, [tok(i)], Observed}, 30% removes {e, [], Observed},
// where Observed = [tok(i-U)] if op i-U was an add (the element's only live token
// in a sequential history), else [].
AM_HD uint64_t am_syn_aw_elem(uint64_t seed, uint64_t key, uint64_t i, uint32_t U) {
  const uint64_t hk = am_syn_h(seed, key, 0, 41);
  return (i * (hk | 1ull) + (hk >> 20)) & (uint64_t)(U - 1);
}
AM_HD bool am_syn_aw_is_add(uint64_t seed, uint64_t key, uint64_t i) { return am_syn_h(seed, key, i, 42) % 10 < 7; }
AM_HD uint64_t am_syn_tok(uint64_t seed, uint64_t key, uint64_t i) { return am_syn_h(seed, key, i, 43); }
AM_HD uint32_t am_syn_aw_words(uint64_t seed, uint64_t key, uint64_t i, uint32_t U) {
  const bool rm = i >= U && am_syn_aw_is_add(seed, key, i - U);
  return 3u + (am_syn_aw_is_add(seed, key, i) ? 1u : 0u) + (rm ? 1u : 0u);
}

// ---- MV register: assign {val(i), tok(i), [tok(i-1)]} (sequential overrides) ----
AM_HD uint64_t am_syn_mv_val(uint64_t seed, uint64_t key, uint64_t i) { return am_syn_h(seed, key, i, 44) % 1000; }
AM_HD uint32_t am_syn_mv_words(uint64_t i) { return i >= 1 ? 1u : 0u; }

// ---- bounded counter: {{increment,V},Id} | {{decrement,V},Id} | {{transfer,V,To},From} ----
AM_HD uint32_t am_syn_bc_kind(uint64_t seed, uint64_t key, uint64_t i) { return (uint32_t)(am_syn_h(seed, key, i, 45) % 3); }
AM_HD uint32_t am_syn_bc_from(uint64_t seed, uint64_t key, uint64_t i, uint32_t D) {
  return (uint32_t)(am_syn_h(seed, key, i, 46) % D);
}
AM_HD uint32_t am_syn_bc_to(uint64_t seed, uint64_t key, uint64_t i, uint32_t D) {
  return (uint32_t)(am_syn_h(seed, key, i, 47) % D);
}
AM_HD uint64_t am_syn_bc_amount(uint64_t seed, uint64_t key, uint64_t i) { return 1 + am_syn_h(seed, key, i, 48) % 100; }
