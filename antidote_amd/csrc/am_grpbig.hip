// am_grpbig.hip -- the chunked token-group view of hot MV-register keys (include/antidote_mat.h,
// AM_NGRP_BIG).  k_grp_build (am_group.hip) sorts one key's births and kills in a workgroup's
// LDS, so it stops at AM_GRP_MAX_REC records; a Zipf-hot key with 2^20 ops is grouped here
// with device-wide segmented sorts instead (one segment per hot key):
//   k_bg_list      the hot keys (am_big_grp_key) and their record counts
//   k_bg_emit      one block per hot key: its births / kills into compact columns (token,
//                  value, op | kill << 31)
//   sort 1         records by token (the MV kill key) within the key -> raw groups = runs of
//                  one token (k_bg_starts + a scan), births per group (k_bg_groups): a token
//                  born twice leaves the key ungrouped, as k_grp_build does
//   sort 2         groups by the value of their birth (~0: none), stable, so within the key
//                  they end in (value, token) order = insert_sorted's (k_bg_final writes the
//                  pairs to grp)
//   k_bg_records   one u32 record per birth / effective kill at its place in the key's range
//   k_bg_table     the chunk table and key_ngrp
// A read of such a key (am_big.hip, grouped mode) then streams u32 records per 1024-op chunk
// and sets born / killed bits per group, with no hashing and no sort.
#include <hipcub/hipcub.hpp>

#include "am_block.h"

using namespace amk;

namespace {

unsigned grid_n(uint64_t n) { return (unsigned)((n + 255) / 256 < 65536 ? (n + 255) / 256 : 65536); }

// the hot keys: list[i] = key, nrec[i] = its record count (the range minus the chunk table)
__global__ void k_bg_list(am_op_log L, const uint64_t *rcnt, uint32_t *cnt, uint32_t *list, uint64_t *nrec) {
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < L.n_keys; k += (uint64_t)gridDim.x * blockDim.x) {
    if (!am_big_grp_key(L, k)) continue;
    const uint64_t o0 = L.key_off[k], o1 = am_kend(L, k);
    const uint32_t i = atomicAdd(cnt, 1u);
    list[i] = (uint32_t)k;
    nrec[i] = rcnt[o1] - rcnt[o0] - am_big_hdr(o1 - o0);
  }
}

struct BgCols {
  uint64_t *tok, *val;
  uint32_t *info, *kid, *pos;  // op | kill << 31; the record's hot-key index; iota (sort payload)
};

struct EmitSink {
  BgCols C;
  uint64_t o;
  uint32_t op, i;
  __device__ void put(uint64_t v, uint64_t t, uint32_t info) {
    C.tok[o] = t, C.val[o] = v, C.info[o] = info, C.kid[o] = i, C.pos[o] = (uint32_t)o;
    ++o;
  }
  __device__ void births(uint64_t e, const uint64_t *tk, uint32_t n, int32_t) {
    for (uint32_t j = 0; j < n; ++j) put(e, tk[j], op);
  }
  __device__ void birth(uint64_t a, uint64_t b, int32_t) { put(a, b, op); }
  __device__ void kills(const uint64_t *tk, uint32_t n, uint64_t e, int32_t) {
    for (uint32_t j = 0; j < n; ++j) put(e, tk[j], op | 0x80000000u);
  }
};

__global__ void k_bg_emit(am_op_log L, const uint64_t *rcnt, uint32_t nb, const uint32_t *list, const uint64_t *bo,
                          BgCols C) {
  for (uint32_t i = blockIdx.x; i < nb; i += gridDim.x) {
    const uint64_t k = list[i];
    const uint64_t o0 = L.key_off[k], o1 = am_kend(L, k);
    const uint64_t hdr = am_big_hdr(o1 - o0), base = rcnt[o0] + hdr;
    for (uint64_t p = o0 + threadIdx.x; p < o1; p += blockDim.x) {
      const uint32_t meta = L.op_meta[p];
      if (meta & AM_META_BAD) continue;  // no records (k_rec_count)
      const uint64_t a = rcnt[p] + (p == o0 ? hdr : 0);
      EmitSink sk{C, bo[i] + (a - base), (uint32_t)(p - o0), i};
      set_effects<AM_MVREG>(L, p, meta, 0, sk);
    }
  }
}

// a new raw group starts where the key or the token changes (sorted order)
__global__ void k_bg_starts(uint64_t n, const uint64_t *tok_s, const uint32_t *pos_s, const uint32_t *kid,
                            uint32_t *flag) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x)
    flag[j] = (j == 0 || kid[pos_s[j]] != kid[pos_s[j - 1]] || tok_s[j] != tok_s[j - 1]) ? 1u : 0u;
}

struct BgGroups {
  uint64_t *tok, *val;   // per group: token, value of its birth (~0: none)
  uint32_t *key, *nb, *bop, *idx;  // hot-key index, births, birth op, iota (sort payload)
  uint32_t *of;          // per record (compact position): its group
};

__global__ void k_bg_groups(uint64_t n, const uint64_t *tok_s, const uint32_t *pos_s, const uint32_t *gid,
                            const uint32_t *flag, BgCols C, BgGroups G) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t g = gid[j] - 1u, q = pos_s[j];
    G.of[q] = g;
    if (flag[j]) G.tok[g] = tok_s[j], G.key[g] = C.kid[q], G.idx[g] = g;
    if (!(C.info[q] & 0x80000000u)) {
      atomicAdd(&G.nb[g], 1u);
      G.val[g] = C.val[q];
      G.bop[g] = C.info[q];
    }
  }
}

// per hot key: first group and group count; a token born twice (or too many groups) -> bad
__global__ void k_bg_keys(uint32_t nb, const uint64_t *bo, const uint32_t *gid, uint64_t *gb, uint64_t *ge,
                          uint32_t *ng, uint8_t *bad) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += gridDim.x * blockDim.x) {
    const uint64_t a = bo[i], b = bo[i + 1];
    const uint32_t g0 = a < b ? gid[a] - 1u : 0u;
    const uint32_t cnt = a < b ? gid[b - 1] - g0 : 0u;
    gb[i] = g0, ge[i] = (uint64_t)g0 + cnt;
    ng[i] = cnt;
    if (cnt >= AM_BIG_MAX_GRP) bad[i] = 1;
  }
}
__global__ void k_bg_twice(uint64_t tg, BgGroups G, uint8_t *bad) {
  for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < tg; g += (uint64_t)gridDim.x * blockDim.x)
    if (G.nb[g] > 1) bad[G.key[g]] = 1;
}

// sorted group j -> its output position within the key, its pair into grp
__global__ void k_bg_final(uint64_t tg, const uint64_t *val_s, const uint32_t *idx_s, BgGroups G, const uint64_t *gb,
                           const uint8_t *bad, const uint32_t *list, const uint64_t *rko, uint64_t *grp, uint32_t *fin) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < tg; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t g = idx_s[j], i = G.key[g];
    if (bad[i]) continue;
    const uint64_t jj = j - gb[i];
    fin[g] = (uint32_t)jj;
    const uint64_t r0 = rko[list[i]];
    grp[2 * (r0 + jj)] = val_s[j];
    grp[2 * (r0 + jj) + 1] = G.tok[g];
  }
}

// one record per compact position, at its place in the key's range (after the chunk table)
__global__ void k_bg_records(am_op_log L, uint64_t n, BgCols C, BgGroups G, const uint32_t *fin, const uint8_t *bad,
                             const uint32_t *list, const uint64_t *bo, const uint64_t *rko, uint32_t *rec_g) {
  for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t i = C.kid[q];
    if (bad[i]) continue;
    const uint64_t k = list[i];
    const uint64_t hdr = am_big_hdr(am_kend(L, k) - L.key_off[k]);
    const uint32_t info = C.info[q], op = info & 0x7FFFFFFFu, g = G.of[q];
    const bool kill = (info & 0x80000000u) != 0;
    // a kill in the birth's own op or before it never removes the token (k_grp_build)
    const bool keep = !kill || G.nb[g] == 0 || op > (G.bop[g] & 0x7FFFFFFFu);
    rec_g[rko[k] + hdr + (q - bo[i])] =
        keep ? ((op & (AM_BIG_CHUNK - 1)) | (kill ? AM_BREC_KILL : 0u) | (fin[g] << 11)) : 0xFFFFFFFFu;
  }
}

// one block per hot key: the chunk table, then key_ngrp
__global__ void k_bg_table(am_op_log L, const uint64_t *rcnt, uint32_t nb, const uint32_t *list, const uint32_t *ng,
                           const uint8_t *bad, const uint64_t *rko, uint32_t *rec_g, uint32_t *ngrp) {
  for (uint32_t i = blockIdx.x; i < nb; i += gridDim.x) {
    const uint64_t k = list[i];
    const uint64_t o0 = L.key_off[k], o1 = am_kend(L, k);
    const uint64_t hdr = am_big_hdr(o1 - o0), nch = hdr - 1, r0 = rko[k];
    if (!bad[i])
      for (uint64_t c = threadIdx.x; c <= nch; c += blockDim.x)
        rec_g[r0 + c] = (uint32_t)(c == 0 ? hdr : (c < nch ? rcnt[o0 + c * AM_BIG_CHUNK] : rcnt[o1]) - r0);
    if (threadIdx.x == 0) ngrp[k] = bad[i] ? AM_NGRP_NONE : (ng[i] | AM_NGRP_BIG);
  }
}

}  // namespace

// the chunked view of every hot MV key of L (rec_key_off set; rcnt = per-op record offsets)
int am_launch_group_build_big(am_ctx *ctx, const am_op_log *L, const uint64_t *rcnt, uint32_t *rec_g, uint64_t *grp,
                              uint32_t *key_ngrp) {
  if (L->n_keys == 0 || L->n_keys > 0xFFFFFFFFull) return AM_OK;
  hipStream_t st = ctx->stream;
  std::vector<void *> tmp;
  auto alloc = [&](size_t b, void **p) -> bool {
    *p = nullptr;
    if (am_dev_alloc(ctx, b < 16 ? 16 : b, p)) return false;
    tmp.push_back(*p);
    return true;
  };
  auto done = [&](int rc) {
    (void)hipStreamSynchronize(st);
    for (void *p : tmp) am_dev_release(ctx, p);
    if (rc) am_set_error("chunked token-group view: build failed");
    return rc;
  };
  uint32_t *cnt = nullptr, *list = nullptr;
  uint64_t *nrec = nullptr;
  if (!alloc(16, (void **)&cnt) || !alloc(L->n_keys * 4, (void **)&list) || !alloc((L->n_keys + 1) * 8, (void **)&nrec))
    return done(AM_ERR_NOMEM);
  if (hipMemsetAsync(cnt, 0, 16, st) != hipSuccess) return done(AM_ERR_HIP);
  hipLaunchKernelGGL(k_bg_list, dim3(grid_n(L->n_keys)), dim3(256), 0, st, *L, rcnt, cnt, list, nrec);
  uint64_t h = 0;
  if (hipGetLastError() != hipSuccess || am_ctx_fetch(ctx, cnt, 1, &h)) return done(AM_ERR_HIP);
  const uint32_t nb = (uint32_t)(h & 0xFFFFFFFFu);
  if (nb == 0) return done(AM_OK);
  // compact record offsets bo[nb + 1]
  uint64_t *bo = nullptr;
  void *scan_tmp = nullptr;
  size_t scan_b = 0;
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, scan_b, nrec, bo, nb + 1, st) != hipSuccess) return done(AM_ERR_HIP);
  if (!alloc((nb + 1) * 8, (void **)&bo) || !alloc(scan_b + 16, &scan_tmp)) return done(AM_ERR_NOMEM);
  if (hipMemsetAsync(nrec + nb, 0, 8, st) != hipSuccess ||
      hipcub::DeviceScan::ExclusiveSum(scan_tmp, scan_b, nrec, bo, nb + 1, st) != hipSuccess)
    return done(AM_ERR_HIP);
  uint64_t n = 0;
  if (am_ctx_fetch(ctx, bo + nb, 1, &n)) return done(AM_ERR_HIP);
  if (n > 0x7FFFFFF0ull) return done(AM_OK);  // int item counts: the hot keys stay ungrouped (AM_NGRP_NONE)
  BgCols C;
  uint64_t *tok_s = nullptr;
  uint32_t *pos_s = nullptr, *flag = nullptr, *gid = nullptr;
  if (!alloc(n * 8, (void **)&C.tok) || !alloc(n * 8, (void **)&C.val) || !alloc(n * 4, (void **)&C.info) ||
      !alloc(n * 4, (void **)&C.kid) || !alloc(n * 4, (void **)&C.pos) || !alloc(n * 8, (void **)&tok_s) ||
      !alloc(n * 4, (void **)&pos_s) || !alloc(n * 4, (void **)&flag) || !alloc(n * 4 + 8, (void **)&gid))
    return done(AM_ERR_NOMEM);
  const unsigned eb = nb < 65536u ? nb : 65536u;
  hipLaunchKernelGGL(k_bg_emit, dim3(eb), dim3(256), 0, st, *L, rcnt, nb, list, bo, C);
  if (hipGetLastError() != hipSuccess) return done(AM_ERR_HIP);
  // sort 1: records by token within each hot key
  void *sort_tmp = nullptr;
  size_t sort_b = 0;
  if (hipcub::DeviceSegmentedRadixSort::SortPairs(nullptr, sort_b, C.tok, tok_s, C.pos, pos_s, (int)n, (int)nb, bo,
                                                  bo + 1, 0, 64, st) != hipSuccess)
    return done(AM_ERR_HIP);
  if (!alloc(sort_b + 16, &sort_tmp)) return done(AM_ERR_NOMEM);
  if (hipcub::DeviceSegmentedRadixSort::SortPairs(sort_tmp, sort_b, C.tok, tok_s, C.pos, pos_s, (int)n, (int)nb, bo,
                                                  bo + 1, 0, 64, st) != hipSuccess)
    return done(AM_ERR_HIP);
  hipLaunchKernelGGL(k_bg_starts, dim3(grid_n(n)), dim3(256), 0, st, n, tok_s, pos_s, C.kid, flag);
  size_t s2 = 0;
  if (hipcub::DeviceScan::InclusiveSum(nullptr, s2, flag, gid, (int)n, st) != hipSuccess) return done(AM_ERR_HIP);
  if (s2 > scan_b) {
    if (!alloc(s2 + 16, &scan_tmp)) return done(AM_ERR_NOMEM);
    scan_b = s2;
  }
  if (hipcub::DeviceScan::InclusiveSum(scan_tmp, scan_b, flag, gid, (int)n, st) != hipSuccess) return done(AM_ERR_HIP);
  uint64_t tg = 0;
  if (n && am_ctx_fetch(ctx, gid + n - 1, 1, &tg)) return done(AM_ERR_HIP);
  tg &= 0xFFFFFFFFull;
  BgGroups G;
  uint64_t *val_s = nullptr, *gb = nullptr, *ge = nullptr;
  uint32_t *idx_s = nullptr, *fin = nullptr, *ng = nullptr;
  uint8_t *bad = nullptr;
  const uint64_t tga = tg + 1;
  if (!alloc(tga * 8, (void **)&G.tok) || !alloc(tga * 8, (void **)&G.val) || !alloc(tga * 4, (void **)&G.key) ||
      !alloc(tga * 4, (void **)&G.nb) || !alloc(tga * 4, (void **)&G.bop) || !alloc(tga * 4, (void **)&G.idx) ||
      !alloc(n * 4 + 4, (void **)&G.of) || !alloc(tga * 8, (void **)&val_s) || !alloc(tga * 4, (void **)&idx_s) ||
      !alloc(tga * 4, (void **)&fin) || !alloc((nb + 1) * 8, (void **)&gb) || !alloc((nb + 1) * 8, (void **)&ge) || !alloc((nb + 1) * 4, (void **)&ng) ||
      !alloc(nb + 16, (void **)&bad))
    return done(AM_ERR_NOMEM);
  if (hipMemsetAsync(G.val, 0xFF, tga * 8, st) != hipSuccess || hipMemsetAsync(G.nb, 0, tga * 4, st) != hipSuccess ||
      hipMemsetAsync(G.bop, 0, tga * 4, st) != hipSuccess || hipMemsetAsync(bad, 0, nb + 16, st) != hipSuccess)
    return done(AM_ERR_HIP);
  hipLaunchKernelGGL(k_bg_groups, dim3(grid_n(n)), dim3(256), 0, st, n, tok_s, pos_s, gid, flag, C, G);
  hipLaunchKernelGGL(k_bg_keys, dim3(grid_n(nb)), dim3(256), 0, st, nb, bo, gid, gb, ge, ng, bad);
  hipLaunchKernelGGL(k_bg_twice, dim3(grid_n(tg)), dim3(256), 0, st, tg, G, bad);
  if (hipGetLastError() != hipSuccess) return done(AM_ERR_HIP);
  // sort 2: groups by the value of their birth, stable (the token order stays within a value)
  size_t sort2_b = 0;
  if (hipcub::DeviceSegmentedRadixSort::SortPairs(nullptr, sort2_b, G.val, val_s, G.idx, idx_s, (int)tg, (int)nb, gb,
                                                  ge, 0, 64, st) != hipSuccess)
    return done(AM_ERR_HIP);
  if (sort2_b > sort_b && !alloc(sort2_b + 16, &sort_tmp)) return done(AM_ERR_NOMEM);
  if (hipcub::DeviceSegmentedRadixSort::SortPairs(sort_tmp, sort2_b > sort_b ? sort2_b : sort_b, G.val, val_s, G.idx,
                                                  idx_s, (int)tg, (int)nb, gb, ge, 0, 64, st) != hipSuccess)
    return done(AM_ERR_HIP);
  hipLaunchKernelGGL(k_bg_final, dim3(grid_n(tg)), dim3(256), 0, st, tg, val_s, idx_s, G, gb, bad, list,
                     L->rec_key_off, grp, fin);
  hipLaunchKernelGGL(k_bg_records, dim3(grid_n(n)), dim3(256), 0, st, *L, n, C, G, fin, bad, list, bo,
                     L->rec_key_off, rec_g);
  hipLaunchKernelGGL(k_bg_table, dim3(eb), dim3(256), 0, st, *L, rcnt, nb, list, ng, bad, L->rec_key_off, rec_g,
                     key_ngrp);
  if (hipGetLastError() != hipSuccess) return done(AM_ERR_HIP);
  return done(AM_OK);
}
