// am_pack.hip -- the packed streaming view of a device op log (am_op_log.key_tbase, .pk_vc).
// The scan kernels are HBM-bound and their per-op work is the ClockSI inclusion test, a
// compare of the op's commit vector against the read clock per DC.  Entries of one key's ops
// lie within minutes of each other, so relative to a per-key time base they fit in u32: the
// test and the LastOpCt max run on 32-bit lanes and each op streams 4 B per DC.  Ops that do
// not fit (or carry AM_META_BAD) are flagged (pk_vc[0] = AM_PK_ESC) and read from the full
// columns, so results stay bit-exact.
//
// The token-group view (am_op_log.rec_* / grp_* / key_ngrp, include/antidote_mat.h)
// flattens the add-wins-set / MV-register effects of every op into u32 birth / kill records
// of per-key token groups, a key's records contiguous in op order, so the set kernels
// stream effects like any other column instead of chasing var_off -> var_data:
//   k_op_key_mark + inclusive max-scan   op -> key
//   k_rec_count + exclusive scan         per-op record counts -> record offsets (malformed
//                                        effects: AM_META_BAD in op_meta, escaped in pk_vc)
//   k_rec_key_off                        per-key record ranges
//   k_grp_build (am_group.hip)           per key: token groups in output order + u32 records
#include <hipcub/hipcub.hpp>

#include "am_block.h"
#include "am_packop.h"

using namespace amk;

namespace {

// one wave per key: the key's base from its first op, then its ops' entries
__global__ void k_pack(am_op_log L, uint64_t *tbase, uint32_t *pk_vc) {
  const uint64_t stride = L.snap_stride ? L.snap_stride : L.n_ops;
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / WAVE);
  for (uint64_t k = (uint64_t)blockIdx.x * (blockDim.x / WAVE) + threadIdx.x / WAVE; k < L.n_keys; k += waves) {
    const uint64_t o0 = L.key_off[k], o1 = L.key_off[k + 1];
    uint64_t base = 0;
    if (o1 > o0) {
      uint64_t s[AM_MAX_DC];
      for (uint32_t d = 0; d < L.n_dc; ++d) s[d] = L.snap_vc[(uint64_t)d * stride + o0];
      base = am_pk_base(L.commit_time[o0], s, L.n_dc, 0xFFFFFFFFu, AM_META_DC(L.op_meta[o0]));
    }
    if (lane == 0) tbase[k] = base;
    for (uint64_t p = o0 + lane; p < o1; p += WAVE)
      am_pk_write(pk_vc, stride, p, L.n_dc, base, L.commit_time[p], L.op_meta[p],
                  [&](uint32_t d) { return L.snap_vc[(uint64_t)d * stride + p]; });
  }
}

// op -> key: the first op of every non-empty key gets the key index; an inclusive
// max-scan spreads it over the key's ops
__global__ void k_op_key_mark(const uint64_t *key_off, uint64_t n_keys, uint32_t *okey) {
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n_keys; k += (uint64_t)gridDim.x * blockDim.x)
    if (key_off[k] < key_off[k + 1]) okey[key_off[k]] = (uint32_t)k;
}

struct CountSink {
  uint32_t n = 0;
  __device__ void births(uint64_t, const uint64_t *, uint32_t c, int32_t) { n += c; }
  __device__ void birth(uint64_t, uint64_t, int32_t) { n += 1; }
  __device__ void kills(const uint64_t *, uint32_t c, uint64_t, int32_t) { n += c; }
};
template <class Sink>
__device__ __forceinline__ bool op_effects(const am_op_log &L, uint64_t p, uint32_t type, uint32_t meta, Sink &sk) {
  if (type == AM_AWSET) return set_effects<AM_AWSET>(L, p, meta, 0, sk);
  return set_effects<AM_MVREG>(L, p, meta, 0, sk);
}

// records reserved per free op slot of a slack store (an AW add with one token and a remove,
// an MV assign overriding one token); a key whose appends need more is rebuilt
constexpr uint64_t REC_SLACK = 2;

__global__ void k_rec_count(am_op_log L, const uint32_t *okey, uint64_t *cnt, uint32_t *pk_vc, uint8_t *op_meta) {
  for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < L.n_ops; p += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t k = okey[p];
    const uint32_t type = L.key_type[k];
    const bool setk = type == AM_AWSET || type == AM_MVREG;
    if (L.key_end && p >= L.key_end[k]) {  // a free slot: room for its records, as many as the
      uint64_t per = REC_SLACK;            // key's ops average (records <= effect words + 1)
      const uint64_t o0 = L.key_off[k], e = L.key_end[k];
      if (setk && L.var_off) {
        const uint64_t w = e > o0 ? (L.var_off[e] - L.var_off[o0] + (e - o0) - 1) / (e - o0) + 1 : 0;
        per = w > per ? w : per;
      }
      // a key with no ops yet carries the placeholder type (PN): its first ops may be of a set
      // type, so its free slots keep set room too (no O(store) rebuild for a new set key)
      cnt[p] = (setk || e == o0) ? per : 0;
      continue;
    }
    const uint32_t meta = L.op_meta[p];
    // a hot MV key's chunked view starts with its chunk table (include/antidote_mat.h)
    uint64_t c = (p == L.key_off[k] && am_big_grp_key(L, k)) ? am_big_hdr(am_kend(L, k) - p) : 0;
    if (setk && !(meta & AM_META_BAD)) {
      CountSink cs;
      if (op_effects(L, p, type, meta, cs)) {
        c += cs.n;
      } else {  // Type:update/2 raises on this effect: flagged, escaped, no records
        if (pk_vc) pk_vc[p] = AM_PK_ESC;
        op_meta[p] = (uint8_t)(meta | AM_META_BAD);
      }
    }
    cnt[p] = c;
  }
}

// the group-mask view (include/antidote_mat.h gmask): a key with at most AM_GMASK_MAX_GRP
// groups gets its records folded per op -- births into bits 0-31, effective kills into 32-63
// (the builder already dropped the ineffective kills: those slots are 0xFFFFFFFF).  One thread
// per key walks its records (a key's records are few when it has so few groups); every other op
// keeps the zero of the memset.
__global__ void k_gmask(am_op_log L, uint64_t *gm) {
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < L.n_keys; k += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t G = L.key_ngrp[k];
    if (G == AM_NGRP_NONE || G > AM_GMASK_MAX_GRP) continue;
    const uint64_t off0 = L.key_off[k], r1 = am_rkend(L, k);
    for (uint64_t r = L.rec_key_off[k]; r < r1; ++r) {
      const uint32_t x = L.rec_g[r];
      if (x == 0xFFFFFFFFu) continue;
      gm[off0 + AM_REC_OP(x)] |= 1ull << (AM_REC_GRP(x) + ((x & AM_REC_KILL) ? 32u : 0u));
    }
  }
}

__global__ void k_rec_key_off(const uint64_t *key_off, const uint64_t *key_end, uint64_t n_keys, const uint64_t *off,
                              uint64_t *rko, uint64_t *rke) {
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k <= n_keys; k += (uint64_t)gridDim.x * blockDim.x) {
    rko[k] = off[key_off[k]];
    if (key_end && k < n_keys) rke[k] = off[key_end[k]];
  }
}

// the zone map (include/antidote_mat.h zone_vc): one wave per block of AM_ZONE_OPS op slots,
// the max of every op's commit vector X per DC (X[commit dc] = commit_time; a snapshot entry
// the op does not carry reads as 0, as in is_op_in_snapshot/7); with `exact_on`, row n_dc marks
// the exact blocks
__global__ void k_zone(am_op_log L, uint64_t *zone, uint64_t nz, int exact_on) {
  const uint64_t stride = L.snap_stride ? L.snap_stride : L.n_ops;
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / WAVE);
  for (uint64_t z = (uint64_t)blockIdx.x * (blockDim.x / WAVE) + threadIdx.x / WAVE; z < nz; z += waves) {
    uint64_t mx[AM_MAX_DC];
    for (uint32_t d = 0; d < L.n_dc; ++d) mx[d] = 0;
    for (uint64_t p = z * AM_ZONE_OPS + lane; p < (z + 1) * AM_ZONE_OPS && p < L.n_ops; p += WAVE) {
      const uint32_t dc = AM_META_DC(L.op_meta[p]);
      const uint32_t sp = L.snap_pres ? L.snap_pres[p] : 0xFFFFFFFFu;
      for (uint32_t d = 0; d < L.n_dc; ++d) {
        const uint64_t x = d == dc ? L.commit_time[p] : (((sp >> d) & 1u) ? L.snap_vc[(uint64_t)d * stride + p] : 0);
        mx[d] = x > mx[d] ? x : mx[d];
      }
    }
    for (uint32_t d = 0; d < L.n_dc; ++d) {
      const uint64_t m = wave_max_u64(mx[d]);
      if (lane == 0) zone[(uint64_t)d * nz + z] = m;
    }
    // exact: every slot a used op of the block's first key, in the packed view, valid
    const uint64_t z0 = z * AM_ZONE_OPS, z1 = z0 + AM_ZONE_OPS;
    bool exact = exact_on && z1 <= L.n_ops && L.pk_vc && L.key_tbase;
    if (exact) {
      uint64_t lo = 0, hi = L.n_keys;  // the key holding slot z0: last k with key_off[k] <= z0
      while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (L.key_off[mid] <= z0) lo = mid;
        else hi = mid;
      }
      exact = L.key_off[lo] <= z0 && z1 <= am_kend(L, lo);
    }
    for (uint64_t p = z0 + lane; exact && p < z1; p += WAVE)
      if (L.pk_vc[p] == AM_PK_ESC || (L.op_meta[p] & AM_META_BAD)) exact = false;
    exact = __ballot(!exact) == 0;
    if (lane == 0) zone[(uint64_t)L.n_dc * nz + z] = exact ? 1u : 0u;
  }
}

struct MaxOp {
  __device__ __forceinline__ uint32_t operator()(uint32_t a, uint32_t b) const { return a > b ? a : b; }
};

unsigned grid_of(uint64_t n) { return (unsigned)((n + 255) / 256 < 65536 ? (n + 255) / 256 : 65536); }

// builds the record view of a packed store (no-op for logs without set payloads)
// ---- escape rows (am_op_log.esc_rows): every escaped op's commit time, meta byte and
//      snapshot entries in one row of 2 + n_dc words, its index + 1 in the op's DC-1 packed
//      entry.  One wave per key, the key's escaped ops compacted by ballot, rows claimed with one
//      atomic per 64 ops; rows == null counts only ----
__global__ void k_esc_rows(am_op_log L, uint32_t *pk_vc, uint64_t *rows, unsigned long long *cnt, uint64_t cap) {
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / WAVE);
  const uint64_t stride = L.snap_stride ? L.snap_stride : L.n_ops;
  const uint32_t nd = L.n_dc, E = 2 + nd;
  for (uint64_t k = (uint64_t)blockIdx.x * (blockDim.x / WAVE) + threadIdx.x / WAVE; k < L.n_keys; k += waves) {
    const uint64_t o0 = L.key_off[k], o1 = am_kend(L, k);
    for (uint64_t b = o0; b < o1; b += WAVE) {
      const uint64_t p = b + lane;
      const bool e = p < o1 && pk_vc[p] == AM_PK_ESC;
      const uint64_t m = __ballot(e);
      if (!m) continue;
      uint64_t base = 0;
      if (lane == 0) base = atomicAdd(cnt, (unsigned long long)__popcll(m));
      base = shfl_u64(base, 0);
      if (!e || !rows) continue;
      const uint64_t row = base + (uint64_t)__popcll(m & ((1ull << lane) - 1ull));
      if (row >= cap) continue;
      uint64_t *w = rows + row * E;
      w[0] = L.commit_time[p];
      w[1] = L.op_meta[p];
      for (uint32_t d = 0; d < nd; ++d) w[2 + d] = L.snap_vc[(uint64_t)d * stride + p];
      pk_vc[stride + p] = (uint32_t)(row + 1);
    }
  }
}

int build_esc_rows(am_store *st) {
  am_ctx *c = st->ctx;
  am_op_log &d = st->dev;
  d.esc_rows = nullptr;
  if (!d.pk_vc || d.n_dc < 2 || !d.n_ops || !d.n_keys) return AM_OK;
  void *cnt = nullptr;
  if (int rc = am_ctx_scratch(c, AM_SCR_MISC, 256, &cnt)) return rc;
  const uint64_t blocks = (d.n_keys + 3) / 4 < 65536 ? (d.n_keys + 3) / 4 : 65536;
  AM_HIP(hipMemsetAsync(cnt, 0, 8, c->stream));
  hipLaunchKernelGGL(k_esc_rows, dim3((unsigned)blocks), dim3(256), 0, c->stream, d, const_cast<uint32_t *>(d.pk_vc),
                     (uint64_t *)nullptr, (unsigned long long *)cnt, (uint64_t)0);
  AM_HIP(hipGetLastError());
  uint64_t n_esc = 0;
  if (int rc = am_ctx_fetch(c, cnt, 1, &n_esc)) return rc;
  if (n_esc == 0) return AM_OK;
  void *rows = nullptr;
  if (int rc = am_dev_alloc(c, n_esc * (2 + d.n_dc) * 8, &rows)) return rc;
  st->allocs.push_back(rows);
  AM_HIP(hipMemsetAsync(cnt, 0, 8, c->stream));
  hipLaunchKernelGGL(k_esc_rows, dim3((unsigned)blocks), dim3(256), 0, c->stream, d, const_cast<uint32_t *>(d.pk_vc),
                     (uint64_t *)rows, (unsigned long long *)cnt, n_esc);
  AM_HIP(hipGetLastError());
  AM_HIP(hipStreamSynchronize(c->stream));
  d.esc_rows = (const uint64_t *)rows;
  return AM_OK;
}

// ---- the lag view (am_op_log.lag_ct / lag / key_lag) from the packed view: one wave per key.
//      Pass 1: key_lag[k][d] = min over the key's packed ops of (ct - X[d]) = entry(dc) - entry(d);
//      pass 2: each op's commit entry and lags, or AM_PK_ESC when a lag exceeds 16 bits ----
constexpr uint32_t LAG_MAX_DC = 16;
__global__ void k_lag(am_op_log L, uint32_t *lag_ct, uint16_t *lag, int32_t *key_lag) {
  const uint32_t lane = threadIdx.x & (WAVE - 1);
  const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / WAVE);
  const uint64_t stride = L.snap_stride ? L.snap_stride : L.n_ops;
  const uint32_t nd = L.n_dc;
  for (uint64_t k = (uint64_t)blockIdx.x * (blockDim.x / WAVE) + threadIdx.x / WAVE; k < L.n_keys; k += waves) {
    const uint64_t o0 = L.key_off[k], o1 = am_kend(L, k);
    int64_t lb[LAG_MAX_DC];
    bool fit = true;  // every lag base within int32
    for (uint32_t d = 0; d < nd; ++d) {
      uint64_t m = ~0ull;  // min of (ct - X[d]) + 2^32 (biased: the difference lies in (-2^32, 2^32))
      for (uint64_t p = o0 + lane; p < o1; p += WAVE) {
        if (L.pk_vc[p] == AM_PK_ESC) continue;
        const uint32_t c = L.pk_vc[(uint64_t)AM_META_DC(L.op_meta[p]) * stride + p];
        const uint64_t v = (uint64_t)c + (1ull << 32) - L.pk_vc[(uint64_t)d * stride + p];
        m = v < m ? v : m;
      }
      m = wave_min_u64(m);
      lb[d] = m == ~0ull ? 0 : (int64_t)m - (int64_t)(1ull << 32);
      fit &= lb[d] >= INT32_MIN && lb[d] <= INT32_MAX;
      if (lane == 0) key_lag[k * nd + d] = fit ? (int32_t)lb[d] : 0;
    }
    for (uint64_t p = o0 + lane; p < o1; p += WAVE) {
      bool ok = fit && L.pk_vc[p] != AM_PK_ESC;
      const uint32_t c = ok ? L.pk_vc[(uint64_t)AM_META_DC(L.op_meta[p]) * stride + p] : 0u;
      for (uint32_t d = 0; d < nd; ++d) {
        const int64_t l = ok ? (int64_t)c - (int64_t)L.pk_vc[(uint64_t)d * stride + p] - lb[d] : 0;
        ok = ok && l >= 0 && l <= 0xFFFF;
        lag[(uint64_t)d * stride + p] = (uint16_t)(ok ? l : 0);
      }
      lag_ct[p] = ok ? c : AM_PK_ESC;
    }
  }
}

int build_lag(am_store *st) {
  am_ctx *c = st->ctx;
  am_op_log &d = st->dev;
  d.lag_ct = nullptr, d.lag = nullptr, d.key_lag = nullptr;
  if (!d.pk_vc || d.n_dc > LAG_MAX_DC || !d.n_keys) return AM_OK;
  const uint64_t stride = d.snap_stride ? d.snap_stride : d.n_ops;
  void *ct = nullptr, *lg = nullptr, *kl = nullptr;
  if (int rc = am_dev_alloc(c, stride * 4 + 16, &ct)) return rc;
  st->allocs.push_back(ct);
  if (int rc = am_dev_alloc(c, (size_t)d.n_dc * stride * 2 + 16, &lg)) return rc;
  st->allocs.push_back(lg);
  if (int rc = am_dev_alloc(c, d.n_keys * d.n_dc * 4 + 16, &kl)) return rc;
  st->allocs.push_back(kl);
  // free slots (room for appends, padding) stay escaped: 0xFF bytes
  AM_HIP(hipMemsetAsync(ct, 0xFF, stride * 4 + 16, c->stream));
  AM_HIP(hipMemsetAsync(lg, 0, (size_t)d.n_dc * stride * 2 + 16, c->stream));
  const uint64_t blocks = (d.n_keys + 3) / 4 < 65536 ? (d.n_keys + 3) / 4 : 65536;
  hipLaunchKernelGGL(k_lag, dim3((unsigned)blocks), dim3(256), 0, c->stream, d, (uint32_t *)ct, (uint16_t *)lg,
                     (int32_t *)kl);
  AM_HIP(hipGetLastError());
  AM_HIP(hipStreamSynchronize(c->stream));
  d.lag_ct = (const uint32_t *)ct, d.lag = (const uint16_t *)lg, d.key_lag = (const int32_t *)kl;
  return AM_OK;
}

int build_records(am_store *st) {
  am_ctx *c = st->ctx;
  am_op_log &d = st->dev;
  if (!d.var_off || d.n_ops == 0 || d.n_ops > 0xFFFFFFFFull) return AM_OK;
  const uint64_t n = d.n_ops;
  uint32_t *okey = nullptr;
  uint64_t *cnt = nullptr;
  void *tmp = nullptr;
  size_t tmp_b = 0, t2 = 0;
  int rc = AM_OK;
  auto cleanup = [&]() {
    (void)hipStreamSynchronize(c->stream);
    am_dev_release(c, okey);  // temporaries from the context's caching allocator (stream-ordered reuse)
    am_dev_release(c, cnt);
    am_dev_release(c, tmp);
  };
  if (hipcub::DeviceScan::InclusiveScan(nullptr, tmp_b, okey, okey, MaxOp(), n, c->stream) != hipSuccess ||
      hipcub::DeviceScan::ExclusiveSum(nullptr, t2, cnt, cnt, n + 1, c->stream) != hipSuccess) {
    am_set_error("record view: scan sizing failed");
    return AM_ERR_HIP;
  }
  if (t2 > tmp_b) tmp_b = t2;
  if (am_dev_alloc(c, n * 4, (void **)&okey) || am_dev_alloc(c, (n + 1) * 8, (void **)&cnt) ||
      am_dev_alloc(c, tmp_b + 16, &tmp)) {
    cleanup();
    am_set_error("record view: out of device memory");
    return AM_ERR_NOMEM;
  }
  uint64_t n_rec = 0;
  do {
    if (hipMemsetAsync(okey, 0, n * 4, c->stream) != hipSuccess) break;
    if (hipMemsetAsync(cnt + n, 0, 8, c->stream) != hipSuccess) break;
    hipLaunchKernelGGL(k_op_key_mark, dim3(grid_of(d.n_keys)), dim3(256), 0, c->stream, d.key_off, d.n_keys, okey);
    if (hipcub::DeviceScan::InclusiveScan(tmp, tmp_b, okey, okey, MaxOp(), n, c->stream) != hipSuccess) break;
    hipLaunchKernelGGL(k_rec_count, dim3(grid_of(n)), dim3(256), 0, c->stream, d, okey, cnt,
                       const_cast<uint32_t *>(d.pk_vc), const_cast<uint8_t *>(d.op_meta));
    if (hipcub::DeviceScan::ExclusiveSum(tmp, tmp_b, cnt, cnt, n + 1, c->stream) != hipSuccess) break;
    if (hipMemcpyAsync(&n_rec, cnt + n, 8, hipMemcpyDeviceToHost, c->stream) != hipSuccess) break;
    if (hipStreamSynchronize(c->stream) != hipSuccess) break;
    rc = -1;
  } while (0);
  if (rc != -1) {
    cleanup();
    am_set_error("record view: count pass failed");
    return AM_ERR_HIP;
  }
  rc = AM_OK;
  void *rko = nullptr, *rke = nullptr, *rg = nullptr, *gp = nullptr, *ng = nullptr, *pr = nullptr;
  rc = am_dev_alloc(c, (d.n_keys + 1) * 8, &rko);
  if (!rc) st->allocs.push_back(rko);
  if (!rc && d.key_end) {
    rc = am_dev_alloc(c, (d.n_keys + 1) * 8, &rke);
    if (!rc) st->allocs.push_back(rke);
  }
  if (!rc) rc = am_dev_alloc(c, (n_rec + 4) * 4, &rg);
  if (!rc) st->allocs.push_back(rg), rc = am_dev_alloc(c, (n_rec + 4) * 16, &gp);
  if (!rc) st->allocs.push_back(gp), rc = am_dev_alloc(c, (d.n_keys + 1) * 4, &ng);
  if (!rc) st->allocs.push_back(ng), rc = am_dev_alloc(c, (n_rec + 4) * 16, &pr);
  if (!rc) st->allocs.push_back(pr);
  if (!rc) {
    hipLaunchKernelGGL(k_rec_key_off, dim3(grid_of(d.n_keys + 1)), dim3(256), 0, c->stream, d.key_off, d.key_end,
                       d.n_keys, cnt, (uint64_t *)rko, (uint64_t *)rke);
    am_op_log v = d;
    v.rec_key_off = (const uint64_t *)rko;
    v.rec_key_end = (const uint64_t *)rke;
    rc = am_launch_group_build(c, &v, cnt, (uint32_t *)rg, (uint64_t *)gp, (uint32_t *)ng, (uint64_t *)pr);
    if (!rc) rc = am_launch_group_build_big(c, &v, cnt, (uint32_t *)rg, (uint64_t *)gp, (uint32_t *)ng);
    if (!rc && (hipGetLastError() != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess)) {
      am_set_error("token-group view: build pass failed");
      rc = AM_ERR_HIP;
    }
  }
  void *gmk = nullptr;  // the group-mask view, over the store's padded op columns
  const size_t na = d.snap_stride ? d.snap_stride : d.n_ops;
  if (!rc && n_rec) {
    rc = am_dev_alloc(c, na * 8 + 32, &gmk);
    if (!rc) {
      st->allocs.push_back(gmk);
      am_op_log v = d;
      v.rec_key_off = (const uint64_t *)rko, v.rec_key_end = (const uint64_t *)rke;
      v.rec_g = (const uint32_t *)rg, v.key_ngrp = (const uint32_t *)ng;
      if (hipMemsetAsync(gmk, 0, na * 8 + 32, c->stream) != hipSuccess) rc = AM_ERR_HIP;
      if (!rc) {
        hipLaunchKernelGGL(k_gmask, dim3(grid_of(d.n_keys)), dim3(256), 0, c->stream, v, (uint64_t *)gmk);
        if (hipGetLastError() != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess) rc = AM_ERR_HIP;
      }
      if (rc) am_set_error("group-mask view: build pass failed");
    }
  }
  cleanup();
  if (rc) return rc;
  d.n_rec = n_rec;
  d.rec_key_off = (const uint64_t *)rko;
  d.rec_key_end = (const uint64_t *)rke;
  d.rec_g = (const uint32_t *)rg;
  d.grp = (const uint64_t *)gp;
  d.key_ngrp = (const uint32_t *)ng;
  d.prec = (const uint64_t *)pr;
  d.gmask = (const uint64_t *)gmk;
  return AM_OK;
}

// the key holding op slot p: the last k with key_off[k] <= p
__device__ __forceinline__ uint64_t key_of_slot(const am_op_log &L, uint64_t p) {
  uint64_t lo = 0, hi = L.n_keys;
  while (hi - lo > 1) {
    const uint64_t mid = (lo + hi) >> 1;
    if (L.key_off[mid] <= p) lo = mid;
    else hi = mid;
  }
  return lo;
}
// the first record of key k (records [rk0, rk1), op order) whose op is >= relative op `rel`
__device__ __forceinline__ uint64_t rec_lower(const am_op_log &L, uint64_t rk0, uint64_t rk1, uint64_t rel) {
  while (rk0 < rk1) {
    const uint64_t mid = (rk0 + rk1) >> 1;
    if (AM_REC_OP(L.rec_g[mid]) < rel) rk0 = mid + 1;
    else rk1 = mid;
  }
  return rk0;
}

// the summary capacity (words) of the blocks of key k: a vnode store (room for appends) sizes
// it for the key's groups to grow by a quarter + 32 before a rewrite no longer fits
__device__ __forceinline__ uint64_t zsum_cap_words(const am_op_log &L, uint32_t G) {
  uint32_t gc = G;
  if (L.key_end) {
    gc = G + G / 4 + 32;
    gc = gc > AM_GRP_MAX_REC ? AM_GRP_MAX_REC : gc;
  }
  return 2 * (uint64_t)((gc + 31) / 32);
}

// zone group summaries (include/antidote_mat.h zone_gsum), pass 1, one thread per zone: the
// block's summary slot (a block inside the op range, room included, of a grouped set key with
// <= AM_GRP_MAX_REC groups) into cnt[z]; an exact block's records begin / end into rows
// n_dc + 3 / n_dc + 2
__global__ void k_zsum_size(am_op_log L, uint64_t *zone, uint64_t nz, uint64_t *cnt) {
  for (uint64_t z = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; z < nz; z += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t words = 0, rend = 0, rbeg = 0;
    const uint64_t z0 = z * AM_ZONE_OPS;
    if (z0 < L.key_off[L.n_keys]) {
      const uint64_t k = key_of_slot(L, z0);
      const uint32_t ng = L.key_ngrp[k], G = am_ngrp_count(ng);
      const uint32_t t = L.key_type[k];
      if ((t == AM_AWSET || t == AM_MVREG) && !am_ngrp_big(ng) && G >= 1 && G <= AM_GRP_MAX_REC &&
          z0 + AM_ZONE_OPS <= L.key_off[k + 1]) {
        words = zsum_cap_words(L, G);
        if (zone[(uint64_t)L.n_dc * nz + z] == 1) {
          rend = rec_lower(L, L.rec_key_off[k], am_rkend(L, k), z0 + AM_ZONE_OPS - L.key_off[k]);
          rbeg = rec_lower(L, L.rec_key_off[k], am_rkend(L, k), z0 - L.key_off[k]);
        }
      }
    }
    cnt[z] = words;
    zone[(uint64_t)(L.n_dc + 2) * nz + z] = rend;
    zone[(uint64_t)(L.n_dc + 3) * nz + z] = rbeg;
  }
}

// pass 2, one wave per zone: row n_dc + 4 = the block's slot; an exact block's summary (the OR
// of its records into LDS bitmaps) written into it, row n_dc + 1 = its offset (else ~0)
__global__ void __launch_bounds__(256) k_zsum_fill(am_op_log L, uint64_t *zone, uint64_t nz, const uint64_t *off,
                                                   uint32_t *gsum) {
  __shared__ uint32_t bits[4][2 * (AM_GRP_MAX_REC / 32)];
  const uint32_t lane = threadIdx.x & (WAVE - 1), wv = threadIdx.x / WAVE;
  uint32_t *bw = bits[wv];
  const uint64_t waves = (uint64_t)gridDim.x * 4;
  for (uint64_t z = (uint64_t)blockIdx.x * 4 + wv; z < nz; z += waves) {
    const uint64_t o = off[z], cap = off[z + 1] - o;
    const bool exact = zone[(uint64_t)L.n_dc * nz + z] == 1;
    uint32_t gw = 0;
    uint64_t k = 0;
    if (cap && exact) {
      k = key_of_slot(L, z * AM_ZONE_OPS);
      gw = (am_ngrp_count(L.key_ngrp[k]) + 31) / 32;
    }
    const bool fill = cap && exact && 2 * (uint64_t)gw <= cap;
    if (lane == 0) {
      zone[(uint64_t)(L.n_dc + 4) * nz + z] = cap ? (cap << 48 | o) : 0ull;
      zone[(uint64_t)(L.n_dc + 1) * nz + z] = fill ? o : ~0ull;
    }
    if (!fill) continue;
    const uint64_t r0 = zone[(uint64_t)(L.n_dc + 3) * nz + z];
    const uint64_t r1 = zone[(uint64_t)(L.n_dc + 2) * nz + z];
    for (uint32_t w = lane; w < 2 * gw; w += WAVE) bw[w] = 0;
    wave_sync();
    for (uint64_t q = r0 + lane; q < r1; q += WAVE) {
      const uint32_t x = L.rec_g[q], g = AM_REC_GRP(x);
      if (x != 0xFFFFFFFFu) atomicOr(bw + ((x & AM_REC_KILL) ? gw : 0u) + (g >> 5), 1u << (g & 31));
    }
    wave_sync();
    for (uint32_t w = lane; w < 2 * gw; w += WAVE) gsum[o + w] = bw[w];
    wave_sync();
  }
}

// the zone index of a device store (every op column written) at `level` (AM_INDEX_*)
int build_zones(am_store *st, int level) {
  am_ctx *c = st->ctx;
  am_op_log &d = st->dev;
  st->zone_level = level;
  if (level <= AM_INDEX_NONE || !d.commit_time || !d.op_meta || !d.n_ops || (d.n_dc && !d.snap_vc)) return AM_OK;
  const uint64_t stride = d.snap_stride ? d.snap_stride : d.n_ops;
  const uint64_t nz = (stride + AM_ZONE_OPS - 1) / AM_ZONE_OPS;
  void *zb = nullptr;
  // rows: maxima, the exactness mark, the group-summary offset, the records end / begin, the
  // summary slot
  const size_t rows = (size_t)d.n_dc + AM_ZONE_EXTRA_ROWS;
  if (int rc = am_dev_alloc(c, rows * nz * 8 + 8, &zb)) return rc;
  st->allocs.push_back(zb);
  AM_HIP(hipMemsetAsync((char *)zb + (size_t)(d.n_dc + 1) * nz * 8, 0xFF, nz * 8, c->stream));
  AM_HIP(hipMemsetAsync((char *)zb + (size_t)(d.n_dc + 4) * nz * 8, 0, nz * 8, c->stream));
  const uint64_t blocks = (nz + 3) / 4 < 65536 ? (nz + 3) / 4 : 65536;
  hipLaunchKernelGGL(k_zone, dim3((unsigned)blocks), dim3(256), 0, c->stream, d, (uint64_t *)zb, nz,
                     level >= AM_INDEX_EXACT ? 1 : 0);
  AM_HIP(hipGetLastError());
  d.zone_vc = (const uint64_t *)zb;
  if (level < AM_INDEX_SUMMARIES || !d.rec_g || !d.key_ngrp || !d.rec_key_off || !d.pk_vc) {
    AM_HIP(hipStreamSynchronize(c->stream));
    return AM_OK;
  }
  // group summaries: slot sizes, exclusive scan, fill
  uint64_t *cnt = nullptr;
  void *tmp = nullptr;
  size_t tmp_b = 0;
  auto cleanup = [&]() {
    (void)hipStreamSynchronize(c->stream);
    am_dev_release(c, cnt);
    am_dev_release(c, tmp);
  };
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_b, cnt, cnt, nz + 1, c->stream) != hipSuccess) {
    am_set_error("zone summaries: scan sizing failed");
    return AM_ERR_HIP;
  }
  if (am_dev_alloc(c, (nz + 1) * 8, (void **)&cnt) || am_dev_alloc(c, tmp_b + 16, &tmp)) {
    cleanup();
    am_set_error("zone summaries: out of device memory");
    return AM_ERR_NOMEM;
  }
  uint64_t total = 0;
  bool ok = hipMemsetAsync(cnt + nz, 0, 8, c->stream) == hipSuccess;
  if (ok) {
    hipLaunchKernelGGL(k_zsum_size, dim3(grid_of(nz)), dim3(256), 0, c->stream, d, (uint64_t *)zb, nz, cnt);
    ok = hipGetLastError() == hipSuccess &&
         hipcub::DeviceScan::ExclusiveSum(tmp, tmp_b, cnt, cnt, nz + 1, c->stream) == hipSuccess &&
         hipMemcpyAsync(&total, cnt + nz, 8, hipMemcpyDeviceToHost, c->stream) == hipSuccess &&
         hipStreamSynchronize(c->stream) == hipSuccess;
  }
  void *gs = nullptr;
  if (ok && total) {
    ok = am_dev_alloc(c, total * 4 + 16, &gs) == AM_OK;
    if (ok) st->allocs.push_back(gs);
  }
  if (ok && total) {
    hipLaunchKernelGGL(k_zsum_fill, dim3((unsigned)blocks), dim3(256), 0, c->stream, d, (uint64_t *)zb, nz, cnt,
                       (uint32_t *)gs);
    ok = hipGetLastError() == hipSuccess;
  }
  cleanup();
  if (!ok) {
    am_set_error("zone summaries: build pass failed");
    return AM_ERR_HIP;
  }
  d.zone_gsum = total ? (const uint32_t *)gs : nullptr;
  return AM_OK;
}

}  // namespace

// the record view and zone map, for a store whose packed view was written by its builder
// (am_gc.hip)
int am_store_pack_records(am_store *st) {
  if (int rc = build_records(st)) return rc;
  if (int rc = build_esc_rows(st)) return rc;
  if (int rc = build_lag(st)) return rc;
  return build_zones(st, st->zone_level);
}

// drop the store's zone index and rebuild it at `level`
extern "C" int am_store_index(am_ctx *c, am_store *st, int level) {
  if (!c || !st || st->ctx != c || level < AM_INDEX_NONE || level > AM_INDEX_SUMMARIES) return AM_ERR_INVALID;
  AM_LOCK(c);
  AM_HIP(hipSetDevice(c->device));
  AM_HIP(hipStreamSynchronize(c->stream));
  am_op_log &d = st->dev;
  for (const void *p : {(const void *)d.zone_vc, (const void *)d.zone_gsum}) {
    if (!p) continue;
    for (size_t i = 0; i < st->allocs.size(); ++i)
      if (st->allocs[i] == p) {
        am_dev_release(c, st->allocs[i]);
        st->allocs.erase(st->allocs.begin() + (long)i);
        break;
      }
  }
  d.zone_vc = nullptr, d.zone_gsum = nullptr;
  if (int rc = build_zones(st, level)) return rc;
  AM_HIP(hipStreamSynchronize(c->stream));
  return AM_OK;
}

int am_store_pack(am_store *st) {
  am_ctx *c = st->ctx;
  am_op_log &d = st->dev;
  const uint64_t stride = d.snap_stride ? d.snap_stride : d.n_ops;
  // the packed view assumes full clocks (snap_pres NULL) and padded columns (16-byte loads);
  // the token-group view is built either way
  if (!d.commit_time || !d.op_meta || (d.n_ops && !d.snap_vc)) return AM_OK;
  if (stride % 4 || d.snap_pres) {
    if (int rc = build_records(st)) return rc;
    return build_zones(st, st->zone_level);
  }
  void *tb = nullptr, *pk = nullptr;
  int rc = am_dev_alloc(c, d.n_keys * 8 + 8, &tb);
  if (rc) return rc;
  st->allocs.push_back(tb);
  rc = am_dev_alloc(c, (size_t)d.n_dc * stride * 4, &pk);
  if (rc) return rc;
  st->allocs.push_back(pk);
  AM_HIP(hipMemsetAsync(pk, 0, (size_t)d.n_dc * stride * 4, c->stream));
  AM_HIP(hipMemsetAsync(tb, 0, d.n_keys * 8 + 8, c->stream));
  if (d.n_ops && d.n_keys) {
    const uint64_t blocks = (d.n_keys + 3) / 4 < 65536 ? (d.n_keys + 3) / 4 : 65536;
    hipLaunchKernelGGL(k_pack, dim3((unsigned)blocks), dim3(256), 0, c->stream, d, (uint64_t *)tb, (uint32_t *)pk);
    AM_HIP(hipGetLastError());
  }
  AM_HIP(hipStreamSynchronize(c->stream));
  d.key_tbase = (const uint64_t *)tb;
  d.pk_vc = (const uint32_t *)pk;
  if (int rc = build_records(st)) return rc;
  if (int rc = build_esc_rows(st)) return rc;  // after k_rec_count's escapes of invalid effects
  if (int rc = build_lag(st)) return rc;
  return build_zones(st, st->zone_level);
}
