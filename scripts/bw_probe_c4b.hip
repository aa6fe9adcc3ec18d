// bw_probe_c4b.hip -- the lane tier's whole memory pattern on C4, three ways (calibration probe,
// not part of the product).  8M keys x 16 ops, key k's type k % 5 -> PN PN LWW AW MV (40/20/20/20);
// per read: key_off[k], key_off[k+1] (the CSR), the 3 packed u32 columns of its ops, p0 (PN, LWW),
// p1 (LWW), and 7 output columns (55 B).  Sets read records instead of payload (here: nothing, to
// isolate the op columns).  Modes:
//   lane : lane = read, 16-byte loads of its own segments (the round-2 kernel's shape)
//   lds  : lane = read for the CSR / outputs; the wave's op span (64 consecutive keys) staged into
//          LDS with coalesced 16-byte loads (1 KiB per instruction), then each lane reads its ops
//          from LDS; p0 / p1 chunks loaded only where a PN / LWW key needs them
// Build: hipcc --offload-arch=gfx950 -O3 scripts/bw_probe_c4b.hip -o /tmp/bwc4b
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned long long u64;
typedef unsigned u32;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

constexpr int OPK = 16;

struct Cols {
  const u64 *key_off;
  const u32 *x[3];
  const u64 *p0, *p1;
  u32 *o_status, *o_count, *o_pres;
  u64 *o_nlo, *o_v0, *o_ct;
  unsigned char *o_flags;
  size_t n_keys;
};

__device__ __forceinline__ int ktype(size_t k) { return (int)(k % 5); }  // 0,1 PN  2 LWW  3,4 sets

__device__ __forceinline__ void outputs(const Cols &C, size_t r, u64 acc, u32 cnt) {
  C.o_status[r] = 0;
  C.o_count[r] = cnt;
  C.o_pres[r] = 7;
  C.o_flags[r] = 0;
  C.o_nlo[r] = acc;
  C.o_v0[r] = acc ^ 1;
#pragma unroll
  for (int d = 0; d < 3; ++d) C.o_ct[(size_t)d * C.n_keys + r] = acc + d;
}

__global__ void __launch_bounds__(256) lane(Cols C) {
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < C.n_keys; k += (size_t)gridDim.x * blockDim.x) {
    const u64 o0 = C.key_off[k], o1 = C.key_off[k + 1];
    const int t = ktype(k);
    u64 acc = 0;
    u32 cnt = 0;
    for (u64 g = o0; g < o1; g += 8) {
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        u32x4 a = *(const u32x4 *)(C.x[c] + g), b = *(const u32x4 *)(C.x[c] + g + 4);
        acc += a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w;
      }
      if (t < 3)
#pragma unroll
        for (int i = 0; i < 8; i += 2) {
          u64x2 a = *(const u64x2 *)(C.p0 + g + i);
          acc += a.x ^ a.y;
        }
      if (t == 2)
#pragma unroll
        for (int i = 0; i < 8; i += 2) {
          u64x2 a = *(const u64x2 *)(C.p1 + g + i);
          acc += a.x ^ a.y;
        }
      cnt += 8;
    }
    outputs(C, k, acc, cnt);
  }
}

// wave-cooperative staging: the wave's 64 consecutive keys' ops [s0, s1) into LDS
template <int SPAN>
__global__ void __launch_bounds__(256) lds(Cols C) {
  __shared__ u32 xs[4][3][SPAN];
  __shared__ u64 ps[4][2][SPAN];
  const u32 w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t nwaves = (size_t)gridDim.x * 4;
  for (size_t k0 = ((size_t)blockIdx.x * 4 + w) * 64; k0 < C.n_keys; k0 += nwaves * 64) {
    const size_t k = k0 + lane;
    const bool live = k < C.n_keys;
    const u64 o0 = live ? C.key_off[k] : 0, o1 = live ? C.key_off[k + 1] : 0;
    const u64 s0 = __shfl(o0, 0) & ~3ull;
    const u64 klast = k0 + 63 < C.n_keys ? 63 : (C.n_keys - 1 - k0);
    const u64 s1 = __shfl(o1, (int)klast);
    const int t = ktype(k);
    // 16-byte chunks of the span, coalesced: chunk q = lane + 64 i (4 u32 / 2 u64 per chunk)
    const u32 n4 = (u32)((s1 - s0 + 3) / 4);
#pragma unroll
    for (int c = 0; c < 3; ++c)
      for (u32 q = lane; q < n4; q += 64) *(u32x4 *)&xs[w][c][4 * q] = *(const u32x4 *)(C.x[c] + s0 + 4 * q);
    const u32 n2 = (u32)((s1 - s0 + 1) / 2);
    for (u32 q = lane; q < n2; q += 64) {
      const size_t kq = k0 + (2 * q) / OPK;  // uniform-length keys: the chunk's key
      const int tq = ktype(kq);
      if (tq < 3) *(u64x2 *)&ps[w][0][2 * q] = *(const u64x2 *)(C.p0 + s0 + 2 * q);
      if (tq == 2) *(u64x2 *)&ps[w][1][2 * q] = *(const u64x2 *)(C.p1 + s0 + 2 * q);
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    u64 acc = 0;
    u32 cnt = 0;
    for (u64 g = o0 - s0; live && g < o1 - s0; g += 4) {
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        u32x4 a = *(const u32x4 *)&xs[w][c][g];
        acc += a.x ^ a.y ^ a.z ^ a.w;
      }
      if (t < 3) {
        u64x2 a = *(const u64x2 *)&ps[w][0][g], b = *(const u64x2 *)&ps[w][0][g + 2];
        acc += a.x ^ a.y ^ b.x ^ b.y;
      }
      if (t == 2) {
        u64x2 a = *(const u64x2 *)&ps[w][1][g], b = *(const u64x2 *)&ps[w][1][g + 2];
        acc += a.x ^ a.y ^ b.x ^ b.y;
      }
      cnt += 4;
    }
    if (live) outputs(C, k, acc, cnt);
    __builtin_amdgcn_wave_barrier();
  }
}

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));      \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

int main() {
  const size_t n_keys = 8u << 20, n_ops = n_keys * OPK;
  Cols C{};
  C.n_keys = n_keys;
  u64 *key_off;
  CK(hipMalloc(&key_off, (n_keys + 1) * 8));
  u64 *h = (u64 *)malloc((n_keys + 1) * 8);
  for (size_t k = 0; k <= n_keys; ++k) h[k] = k * OPK;
  CK(hipMemcpy(key_off, h, (n_keys + 1) * 8, hipMemcpyHostToDevice));
  C.key_off = key_off;
  for (int c = 0; c < 3; ++c) {
    u32 *x;
    CK(hipMalloc(&x, n_ops * 4 + 4096));
    CK(hipMemset(x, 1, n_ops * 4));
    C.x[c] = x;
  }
  u64 *p0, *p1;
  CK(hipMalloc(&p0, n_ops * 8 + 4096));
  CK(hipMalloc(&p1, n_ops * 8 + 4096));
  C.p0 = p0, C.p1 = p1;
  CK(hipMalloc(&C.o_status, n_keys * 4));
  CK(hipMalloc(&C.o_count, n_keys * 4));
  CK(hipMalloc(&C.o_pres, n_keys * 4));
  CK(hipMalloc(&C.o_flags, n_keys));
  CK(hipMalloc(&C.o_nlo, n_keys * 8));
  CK(hipMalloc(&C.o_v0, n_keys * 8));
  CK(hipMalloc(&C.o_ct, n_keys * 24));
  // algorithmic bytes: key_off 8 + 12/op + p0 (60%) 8/op + p1 (20%) 8/op + 55 B out
  const double bytes = n_keys * (8.0 + 55.0) + n_ops * (12.0 + 0.6 * 8 + 0.2 * 8);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  for (int rep = 0; rep < 2; ++rep)
    for (int mode = 0; mode < 2; ++mode)
      for (int occ : {2, 4, 8}) {
        const int blocks = cus * occ;
        float best = 1e30f;
        for (int it = 0; it < 6; ++it) {
          CK(hipEventRecord(a));
          if (mode == 0) lane<<<blocks, 256>>>(C);
          else lds<1024 + 8><<<blocks, 256>>>(C);
          CK(hipGetLastError());
          CK(hipEventRecord(b));
          CK(hipEventSynchronize(b));
          float ms;
          CK(hipEventElapsedTime(&ms, a, b));
          if (it > 0 && ms < best) best = ms;
        }
        printf("{\"mode\": \"%s\", \"blocks_per_cu\": %d, \"ms\": %.4f, \"alg_GBps\": %.1f}\n", mode ? "lds" : "lane",
               occ, best, bytes / best / 1e6);
      }
  return 0;
}
