// am_synth.hip -- on-device generation of the synthetic op logs (the C3-sized
// logs do not fit through the host), and the bit-identical host regenerator
// used by the parity tests.  Model: synth.h.  Log lengths are uniform or Zipf
// (computed on the host in double precision and shared by both paths, so the
// device and host logs agree to the bit).
#include <hipcub/hipcub.hpp>

#include <cmath>
#include <vector>

#include "am_internal.h"
#include "synth.h"

namespace {

struct SynOp {
  uint8_t meta;
  uint64_t ct;
  uint64_t p0, p1;
};

AM_HD uint32_t universe_of(const am_synth_params &p) { return p.universe ? p.universe : 64u; }

AM_HD void syn_op(const am_synth_params &p, uint64_t key, uint64_t i, uint32_t ktype, uint32_t n, SynOp &o) {
  const uint32_t dc = am_syn_dc(p.seed, key, i, p.n_dc);
  uint32_t kind = 0;
  o.ct = am_syn_g(p.seed, key, (int64_t)i);
  o.p0 = o.p1 = 0;
  if (ktype == AM_PN) {
    o.p0 = (uint64_t)am_syn_pn_delta(p.seed, key, i);
  } else if (ktype == AM_LWW) {
    o.p0 = am_syn_lww_ts(p.seed, key, i, n);
    o.p1 = am_syn_lww_val(p.seed, key, i);
  } else if (ktype == AM_MVREG) {
    o.p0 = am_syn_mv_val(p.seed, key, i);
    o.p1 = am_syn_tok(p.seed, key, i);
  } else if (ktype == AM_BCOUNTER) {
    kind = am_syn_bc_kind(p.seed, key, i);
    o.p0 = am_syn_bc_amount(p.seed, key, i);
    o.p1 = am_syn_bc_from(p.seed, key, i, p.n_dc) | ((uint64_t)am_syn_bc_to(p.seed, key, i, p.n_dc) << 8);
  }
  o.meta = (uint8_t)((dc & 31u) | (kind << 5));
}

AM_HD uint32_t var_words(const am_synth_params &p, uint64_t key, uint64_t i, uint32_t ktype) {
  if (ktype == AM_AWSET) return am_syn_aw_words(p.seed, key, i, universe_of(p));
  if (ktype == AM_MVREG) return am_syn_mv_words(i);
  return 0;
}

AM_HD void var_write(const am_synth_params &p, uint64_t key, uint64_t i, uint32_t ktype, uint64_t *dst) {
  if (ktype == AM_AWSET) {
    const uint32_t U = universe_of(p);
    const bool add = am_syn_aw_is_add(p.seed, key, i);
    const bool rm = i >= U && am_syn_aw_is_add(p.seed, key, i - U);
    dst[0] = am_syn_aw_elem(p.seed, key, i, U);
    dst[1] = add ? 1 : 0;
    dst[2] = rm ? 1 : 0;
    uint32_t w = 3;
    if (add) dst[w++] = am_syn_tok(p.seed, key, i);
    if (rm) dst[w++] = am_syn_tok(p.seed, key, i - U);
  } else if (ktype == AM_MVREG) {
    if (i >= 1) dst[0] = am_syn_tok(p.seed, key, i - 1);
  }
}

// Global key of local key k: contiguous from key_base, or the k-th key of the owned
// partitions (key mod 64 in part_mask), so a rank holds exactly the keys
// get_key_partition/1 sends to its partitions (src/log_utilities.erl:60-79).
AM_HD uint64_t global_key(const am_synth_params &p, uint64_t k) {
  if (!p.part_mask) return p.key_base + k;
  const uint32_t m = (uint32_t)__builtin_popcountll(p.part_mask);
  uint64_t r = k % m, bits = p.part_mask;
  for (; r; --r) bits &= bits - 1;  // drop the r lowest owned partitions
  const uint64_t base = ((uint64_t)p.key_base + 63) / 64 * 64;
  return base + (k / m) * 64 + (uint64_t)__builtin_ctzll(bits);
}

bool needs_var(const am_synth_params &p) { return p.type == 0 || p.type == AM_AWSET || p.type == AM_MVREG || p.type == AM_SYNTH_MV_BC; }
bool needs_p1(const am_synth_params &p) { return p.type != AM_PN; }

int check_params(const am_synth_params *p) {
  if (!p || p->n_dc == 0 || p->n_dc > AM_MAX_DC || p->n_keys == 0) {
    am_set_error("synth: bad params (n_dc 1..32, n_keys > 0)");
    return AM_ERR_INVALID;
  }
  if (p->zipf_milli == 0 && p->ops_per_key == 0) {
    am_set_error("synth: ops_per_key == 0 with uniform lengths");
    return AM_ERR_INVALID;
  }
  const uint32_t U = universe_of(*p);
  if (U & (U - 1)) {
    am_set_error("synth: universe must be a power of two");
    return AM_ERR_INVALID;
  }
  if (!(p->type <= AM_BCOUNTER || p->type == AM_SYNTH_MV_BC)) {
    am_set_error("synth: unknown type %u", p->type);
    return AM_ERR_INVALID;
  }
  if (p->esc_ppm > 1000000u) {
    am_set_error("synth: esc_ppm %u above 10^6", p->esc_ppm);
    return AM_ERR_INVALID;
  }
  return AM_OK;
}

// Log length of keys [k0, k0+nk): uniform, or Zipf(s) over the key index with
// n_k = min(cap, max(1, floor(Z (k+1)^-s))), Z = total_ops / H(n_keys, s).
void key_lengths(const am_synth_params &p, uint64_t k0, uint64_t nk, std::vector<uint32_t> &len) {
  len.resize(nk);
  if (p.zipf_milli == 0) {
    for (uint64_t k = 0; k < nk; ++k) len[k] = p.ops_per_key;
    return;
  }
  const double s = p.zipf_milli / 1000.0;
  double H = 0;
  for (uint64_t r = 1; r <= p.n_keys; ++r) H += std::pow((double)r, -s);
  const double Z = (double)p.total_ops / H;
  const uint32_t cap = p.hot_cap ? p.hot_cap : (1u << 20);
  for (uint64_t k = 0; k < nk; ++k) {
    double x = std::floor(Z * std::pow((double)(k0 + k + 1), -s));
    if (x < 1) x = 1;
    if (x > cap) x = cap;
    len[k] = (uint32_t)x;
  }
}

__global__ void k_gen_ops(am_synth_params p, const uint64_t *key_off, uint64_t stride, uint8_t *key_type,
                          uint8_t *meta, uint64_t *ct, uint64_t *snap, uint64_t *p0, uint64_t *p1, uint64_t *vlen) {
  for (uint64_t k = blockIdx.x; k < p.n_keys; k += gridDim.x) {
    const uint64_t key = global_key(p, k);
    const uint32_t kt = am_syn_key_type(p.seed, key, p.type);
    if (threadIdx.x == 0) key_type[k] = (uint8_t)kt;
    const uint64_t off = key_off[k], n = key_off[k + 1] - off;
    for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) {
      const uint64_t q = off + i;
      SynOp o;
      syn_op(p, key, i, kt, (uint32_t)n, o);
      meta[q] = o.meta;
      ct[q] = o.ct;
      p0[q] = o.p0;
      if (p1) p1[q] = o.p1;
      for (uint32_t d = 0; d < p.n_dc; ++d) snap[(uint64_t)d * stride + q] = am_syn_snap_e(p.seed, key, i, d, p.max_lag, p.n_dc, p.esc_ppm);
      if (vlen) vlen[q] = var_words(p, key, i, kt);
    }
  }
}

__global__ void k_gen_var(am_synth_params p, const uint64_t *key_off, const uint64_t *var_off, uint64_t *var_data) {
  for (uint64_t k = blockIdx.x; k < p.n_keys; k += gridDim.x) {
    const uint64_t key = global_key(p, k);
    const uint32_t kt = am_syn_key_type(p.seed, key, p.type);
    const uint64_t off = key_off[k], n = key_off[k + 1] - off;
    for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) var_write(p, key, i, kt, var_data + var_off[off + i]);
  }
}

}  // namespace

extern "C" {

int am_synth_store(am_ctx *c, const am_synth_params *p, am_store **out) {
  if (!c) return AM_ERR_INVALID;
  AM_LOCK(c);
  int rc = check_params(p);
  if (rc) return rc;
  if (!c || !out) return AM_ERR_INVALID;
  AM_HIP(hipSetDevice(c->device));
  std::vector<uint32_t> len;
  key_lengths(*p, 0, p->n_keys, len);
  std::vector<uint64_t> off(p->n_keys + 1, 0);
  for (uint64_t k = 0; k < p->n_keys; ++k) off[k + 1] = off[k] + len[k];
  const uint64_t n_ops = off[p->n_keys];
  const uint64_t na = am_round_up(n_ops, AM_OP_PAD) + AM_OP_PAD;
  am_store *st = new am_store();
  st->ctx = c;
  am_op_log &d = st->dev;
  d.n_dc = p->n_dc;
  d.n_keys = p->n_keys;
  d.n_ops = n_ops;
  d.snap_stride = na;
  auto alloc = [&](size_t bytes, void **o) -> int {
    void *q = nullptr;
    int r = am_dev_alloc(c, bytes, &q);
    if (r) return r;
    st->allocs.push_back(q);
    *o = q;
    return hipMemsetAsync(q, 0, bytes, c->stream) == hipSuccess ? AM_OK : AM_ERR_HIP;
  };
  void *key_off = nullptr, *key_type = nullptr, *meta = nullptr, *ct = nullptr, *snap = nullptr, *p0 = nullptr,
       *p1 = nullptr, *var_off = nullptr, *var_data = nullptr;
  if (!rc) rc = alloc((p->n_keys + 1) * 8, &key_off);
  if (!rc) rc = alloc(p->n_keys + 16, &key_type);
  if (!rc) rc = alloc(na, &meta);
  if (!rc) rc = alloc(na * 8, &ct);
  if (!rc) rc = alloc((size_t)p->n_dc * na * 8, &snap);
  if (!rc) rc = alloc(na * 8, &p0);
  if (!rc && needs_p1(*p)) rc = alloc(na * 8, &p1);
  if (!rc && needs_var(*p)) rc = alloc((n_ops + 1) * 8, &var_off);
  if (!rc) {
    hipError_t e = hipMemcpyAsync(key_off, off.data(), off.size() * 8, hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) rc = AM_ERR_HIP;
  }
  const unsigned grid = (unsigned)(p->n_keys < 65536 ? p->n_keys : 65536);
  if (!rc) {
    hipLaunchKernelGGL(k_gen_ops, dim3(grid), dim3(256), 0, c->stream, *p, (const uint64_t *)key_off, na,
                       (uint8_t *)key_type, (uint8_t *)meta, (uint64_t *)ct, (uint64_t *)snap, (uint64_t *)p0,
                       (uint64_t *)p1, (uint64_t *)var_off);
    if (hipGetLastError() != hipSuccess) rc = AM_ERR_HIP;
  }
  uint64_t n_var = 0;
  if (!rc && var_off) {
    // var_off := exclusive prefix sum of the per-op word counts (last slot = total)
    size_t tmp = 0;
    void *tbuf = nullptr;
    uint64_t *vo = (uint64_t *)var_off;
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, vo, vo, n_ops + 1, c->stream) != hipSuccess) rc = AM_ERR_HIP;
    if (!rc) rc = alloc(tmp + 16, &tbuf);
    if (!rc && hipcub::DeviceScan::ExclusiveSum(tbuf, tmp, vo, vo, n_ops + 1, c->stream) != hipSuccess) rc = AM_ERR_HIP;
    if (!rc && hipMemcpyAsync(&n_var, vo + n_ops, 8, hipMemcpyDeviceToHost, c->stream) != hipSuccess) rc = AM_ERR_HIP;
    if (!rc && hipStreamSynchronize(c->stream) != hipSuccess) rc = AM_ERR_HIP;
    if (!rc) rc = alloc((n_var + 4) * 8, &var_data);
    if (!rc) {
      hipLaunchKernelGGL(k_gen_var, dim3(grid), dim3(256), 0, c->stream, *p, (const uint64_t *)key_off,
                         (const uint64_t *)var_off, (uint64_t *)var_data);
      if (hipGetLastError() != hipSuccess) rc = AM_ERR_HIP;
    }
  }
  if (!rc && hipStreamSynchronize(c->stream) != hipSuccess) rc = AM_ERR_HIP;
  if (rc) {
    if (rc == AM_ERR_HIP) am_set_error("synth generation failed");
    am_store_destroy(st);
    return rc;
  }
  d.key_off = (const uint64_t *)key_off;
  d.key_type = (const uint8_t *)key_type;
  d.op_meta = (const uint8_t *)meta;
  d.commit_time = (const uint64_t *)ct;
  d.snap_vc = (const uint64_t *)snap;
  d.p0 = (const uint64_t *)p0;
  d.p1 = (const uint64_t *)p1;
  d.var_off = (const uint64_t *)var_off;
  d.var_data = (const uint64_t *)var_data;
  d.n_var = n_var;
  rc = am_store_pack(st);
  if (rc) {
    am_store_destroy(st);
    return rc;
  }
  *out = st;
  return AM_OK;
}

int am_synth_read_clock(const am_synth_params *p, double q, uint64_t *out_vc) {
  if (!p || !out_vc || p->n_dc == 0 || p->n_dc > AM_MAX_DC) return AM_ERR_INVALID;
  // Uniform logs: the q-quantile of every key's timeline.  Zipf: every key shares the
  // timeline g(i), so one snapshot position i* covers min(len_k, i*) ops of key k;
  // pick the smallest i* that covers a fraction q of all ops.
  if (!p->zipf_milli) {
    for (uint32_t d = 0; d < p->n_dc; ++d) out_vc[d] = am_syn_read_clock(p->ops_per_key, q, d);
    return AM_OK;
  }
  std::vector<uint32_t> len;
  key_lengths(*p, 0, p->n_keys, len);
  uint64_t total = 0, hi = 0;
  for (uint32_t l : len) {
    total += l;
    hi = l > hi ? l : hi;
  }
  const double target = q * (double)total;
  uint64_t lo = 0;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) / 2;
    uint64_t cov = 0;
    for (uint32_t l : len) cov += l < mid ? l : mid;
    if ((double)cov >= target) hi = mid;
    else lo = mid + 1;
  }
  for (uint32_t d = 0; d < p->n_dc; ++d) out_vc[d] = am_syn_read_clock(lo, 1.0, d);
  return AM_OK;
}

uint64_t am_synth_key(const am_synth_params *p, uint64_t k) { return p ? global_key(*p, k) : 0; }

int am_synth_host_sizes(const am_synth_params *p, uint64_t k0, uint64_t nk, uint64_t *n_ops, uint64_t *n_var) {
  int rc = check_params(p);
  if (rc) return rc;
  std::vector<uint32_t> len;
  key_lengths(*p, k0, nk, len);
  uint64_t no = 0, nv = 0;
  for (uint64_t k = 0; k < nk; ++k) {
    const uint64_t key = global_key(*p, k0 + k);
    const uint32_t kt = am_syn_key_type(p->seed, key, p->type);
    for (uint64_t i = 0; i < len[k]; ++i) nv += var_words(*p, key, i, kt);
    no += len[k];
  }
  if (n_ops) *n_ops = no;
  if (n_var) *n_var = nv;
  return AM_OK;
}

// Fills caller-provided host buffers (out->snap_stride describes snap_vc; var_off /
// var_data may be NULL when the workload has no variable payloads); key_off is
// relative to the regenerated range.
int am_synth_host(const am_synth_params *p, uint64_t k0, uint64_t nk, am_op_log *o) {
  int rc = check_params(p);
  if (rc) return rc;
  if (!o || !o->key_off || !o->key_type || !o->op_meta || !o->commit_time || !o->snap_vc || !o->p0) return AM_ERR_INVALID;
  std::vector<uint32_t> len;
  key_lengths(*p, k0, nk, len);
  uint64_t total = 0;
  for (uint64_t k = 0; k < nk; ++k) total += len[k];
  const uint64_t stride = o->snap_stride ? o->snap_stride : total;
  uint64_t *key_off = const_cast<uint64_t *>(o->key_off);
  uint8_t *key_type = const_cast<uint8_t *>(o->key_type);
  uint8_t *meta = const_cast<uint8_t *>(o->op_meta);
  uint64_t *ct = const_cast<uint64_t *>(o->commit_time);
  uint64_t *snap = const_cast<uint64_t *>(o->snap_vc);
  uint64_t *p0 = const_cast<uint64_t *>(o->p0);
  uint64_t *p1 = const_cast<uint64_t *>(o->p1);
  uint64_t *var_off = const_cast<uint64_t *>(o->var_off);
  uint64_t *var_data = const_cast<uint64_t *>(o->var_data);
  uint64_t q = 0, w = 0;
  key_off[0] = 0;
  for (uint64_t k = 0; k < nk; ++k) {
    const uint64_t key = global_key(*p, k0 + k);
    const uint32_t kt = am_syn_key_type(p->seed, key, p->type);
    key_type[k] = (uint8_t)kt;
    for (uint64_t i = 0; i < len[k]; ++i, ++q) {
      SynOp op;
      syn_op(*p, key, i, kt, len[k], op);
      meta[q] = op.meta;
      ct[q] = op.ct;
      p0[q] = op.p0;
      if (p1) p1[q] = op.p1;
      for (uint32_t d = 0; d < p->n_dc; ++d) snap[(uint64_t)d * stride + q] = am_syn_snap_e(p->seed, key, i, d, p->max_lag, p->n_dc, p->esc_ppm);
      if (var_off) {
        var_off[q] = w;
        if (var_data) var_write(*p, key, i, kt, var_data + w);
        w += var_words(*p, key, i, kt);
      }
    }
    key_off[k + 1] = q;
  }
  if (var_off) var_off[q] = w;
  return AM_OK;
}

}  // extern "C"
