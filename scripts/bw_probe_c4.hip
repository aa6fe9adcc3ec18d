// bw_probe_c4.hip -- does the lane tier's load SHAPE cost bandwidth on C4?  (calibration
// probe, not part of the product).  C4-shaped columns: 3 u32 packed-commit-vector columns and
// two u64 payload columns, 16 ops per key, keys consecutive.  Same bytes, three shapes:
//   lane : lane i owns key i: 4 x 16-B loads per u32 column, 8 per u64 column, lanes 64 B /
//          128 B apart (the round-2 k_lane)
//   quad : 4 lanes per key: lane j of a quad loads ops [4j, 4j+4) of its key -- a quad's
//          loads are one contiguous 64 B, a wave instruction 1 KiB
//   flat : one grid-stride 16-B stream over the same bytes (the ceiling)
// Build: hipcc --offload-arch=gfx950 -O3 scripts/bw_probe_c4.hip -o scripts/bw_c4
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned long long u64;
typedef unsigned u32;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

constexpr int OPK = 16;

__global__ void __launch_bounds__(256) lane(const u32 *x0, const u32 *x1, const u32 *x2, const u64 *p0, const u64 *p1,
                                            size_t n_keys, u64 *out) {
  u64 acc = 0;
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < n_keys; k += (size_t)gridDim.x * blockDim.x) {
    const size_t g = k * OPK;
    const u32 *xs[3] = {x0, x1, x2};
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int i = 0; i < OPK; i += 4) {
        u32x4 a = *(const u32x4 *)(xs[c] + g + i);
        acc += a.x ^ a.y ^ a.z ^ a.w;
      }
#pragma unroll
    for (int i = 0; i < OPK; i += 2) {
      u64x2 a = *(const u64x2 *)(p0 + g + i), b = *(const u64x2 *)(p1 + g + i);
      acc += a.x ^ a.y ^ b.x ^ b.y;
    }
  }
  if (acc == 0x1234567) out[0] = acc;
}

__global__ void __launch_bounds__(256) quad(const u32 *x0, const u32 *x1, const u32 *x2, const u64 *p0, const u64 *p1,
                                            size_t n_keys, u64 *out) {
  u64 acc = 0;
  const u32 j = threadIdx.x & 3;
  for (size_t k = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 2; k < n_keys;
       k += ((size_t)gridDim.x * blockDim.x) >> 2) {
    const size_t g = k * OPK + 4 * j;
    const u32 *xs[3] = {x0, x1, x2};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      u32x4 a = *(const u32x4 *)(xs[c] + g);
      acc += a.x ^ a.y ^ a.z ^ a.w;
    }
#pragma unroll
    for (int i = 0; i < 4; i += 2) {
      u64x2 a = *(const u64x2 *)(p0 + g + i), b = *(const u64x2 *)(p1 + g + i);
      acc += a.x ^ a.y ^ b.x ^ b.y;
    }
  }
  if (acc == 0x1234567) out[0] = acc;
}

// quad2: as quad for the u32 columns; u64 columns as two 16-B loads per lane where lane j of
// a quad takes ops [2j + 8s, 2j + 8s + 2): every instruction reads whole 64-B segments
__global__ void __launch_bounds__(256) quad2(const u32 *x0, const u32 *x1, const u32 *x2, const u64 *p0, const u64 *p1,
                                             size_t n_keys, u64 *out) {
  u64 acc = 0;
  const u32 j = threadIdx.x & 3;
  for (size_t k = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 2; k < n_keys;
       k += ((size_t)gridDim.x * blockDim.x) >> 2) {
    const size_t g = k * OPK;
    const u32 *xs[3] = {x0, x1, x2};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      u32x4 a = *(const u32x4 *)(xs[c] + g + 4 * j);
      acc += a.x ^ a.y ^ a.z ^ a.w;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      u64x2 a = *(const u64x2 *)(p0 + g + 2 * j + 8 * s), b = *(const u64x2 *)(p1 + g + 2 * j + 8 * s);
      acc += a.x ^ a.y ^ b.x ^ b.y;
    }
  }
  if (acc == 0x1234567) out[0] = acc;
}

// blocked_pk: the 3 u32 columns of a key in one 192-byte block (column d at 64 d), p0 / p1
// separate; blocked_all: p0 and p1 in the block too (448 bytes per key); lane = key
__global__ void __launch_bounds__(256) blocked_pk(const u32 *blk, const u64 *p0, const u64 *p1, size_t n_keys, u64 *out) {
  u64 acc = 0;
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < n_keys; k += (size_t)gridDim.x * blockDim.x) {
    const u32 *b = blk + k * 48;
#pragma unroll
    for (int i = 0; i < 48; i += 4) {
      u32x4 a = *(const u32x4 *)(b + i);
      acc += a.x ^ a.y ^ a.z ^ a.w;
    }
    const size_t g = k * OPK;
#pragma unroll
    for (int i = 0; i < OPK; i += 2) {
      u64x2 a = *(const u64x2 *)(p0 + g + i), c = *(const u64x2 *)(p1 + g + i);
      acc += a.x ^ a.y ^ c.x ^ c.y;
    }
  }
  if (acc == 0x1234567) out[0] = acc;
}
__global__ void __launch_bounds__(256) blocked_all(const u32 *blk, size_t n_keys, u64 *out) {
  u64 acc = 0;
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < n_keys; k += (size_t)gridDim.x * blockDim.x) {
    const u32 *b = blk + k * 112;
#pragma unroll
    for (int i = 0; i < 112; i += 4) {
      u32x4 a = *(const u32x4 *)(b + i);
      acc += a.x ^ a.y ^ a.z ^ a.w;
    }
  }
  if (acc == 0x1234567) out[0] = acc;
}

__global__ void __launch_bounds__(256) flat(const u32x4 *a, size_t n4, u64 *out) {
  u64 acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    u32x4 v = a[i];
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x1234567) out[0] = acc;
}

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e = (x);                                               \
    if (e != hipSuccess) {                                            \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                        \
    }                                                                 \
  } while (0)

int main() {
  const size_t n_keys = 8u << 20, n_ops = n_keys * OPK;
  const size_t bytes = n_ops * (3 * 4 + 2 * 8);
  char *buf;
  CK(hipMalloc(&buf, bytes));
  CK(hipMemset(buf, 1, bytes));
  u64 *out;
  CK(hipMalloc(&out, 8));
  const u32 *x0 = (const u32 *)buf, *x1 = x0 + n_ops, *x2 = x1 + n_ops;
  const u64 *p0 = (const u64 *)(x2 + n_ops), *p1 = p0 + n_ops;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  int dev;
  hipDeviceProp_t prop;
  CK(hipGetDevice(&dev));
  CK(hipGetDeviceProperties(&prop, dev));
  const int cus = prop.multiProcessorCount;
  for (int rep = 0; rep < 2; ++rep)
    for (int mode = 0; mode < 6; ++mode)
      for (int occ : {2, 4, 8}) {
        const int blocks = cus * occ;
        float best = 1e30f;
        for (int it = 0; it < 6; ++it) {
          CK(hipEventRecord(a));
          if (mode == 0) lane<<<blocks, 256>>>(x0, x1, x2, p0, p1, n_keys, out);
          else if (mode == 1) quad<<<blocks, 256>>>(x0, x1, x2, p0, p1, n_keys, out);
          else if (mode == 3) quad2<<<blocks, 256>>>(x0, x1, x2, p0, p1, n_keys, out);
          else if (mode == 4) blocked_pk<<<blocks, 256>>>(x0, p0, p1, n_keys, out);
          else if (mode == 5) blocked_all<<<blocks, 256>>>(x0, n_keys, out);
          else flat<<<blocks, 256>>>((const u32x4 *)buf, bytes / 16, out);
          CK(hipEventRecord(b));
          CK(hipEventSynchronize(b));
          float ms;
          CK(hipEventElapsedTime(&ms, a, b));
          if (it > 0 && ms < best) best = ms;
        }
        printf("{\"mode\": \"%s\", \"blocks_per_cu\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n",
               mode == 0 ? "lane" : mode == 1 ? "quad" : mode == 3 ? "quad2" : mode == 4 ? "blocked_pk" : mode == 5 ? "blocked_all" : "flat", occ, best, bytes / best / 1e6);
      }
  return 0;
}
