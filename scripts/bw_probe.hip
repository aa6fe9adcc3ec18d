// bw_probe.hip -- achievable HBM read bandwidth for the materializer's access
// pattern (calibration for roofline.frac; not part of the product).
//   mode 0: one flat array, 16 B/lane, grid-stride
//   mode 1: 7 column arrays of the C2 LWW layout (u8 meta + 6 u64 columns), each
//           lane reads 4 consecutive ops of every column (exactly the kernel's loads)
//   mode 2: as mode 1 with non-temporal loads
// Build: hipcc --offload-arch=gfx950 -O3 scripts/bw_probe.hip -o /tmp/bw_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

__global__ void flat(const u64x2 *a, size_t n2, u64 *out) {
  u64 acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x) {
    u64x2 v = a[i];
    acc ^= v.x + v.y;
  }
  if (acc == 0x1234567) out[0] = acc;
}

__global__ void cols6(const u64 *c0, const u64 *c1, const u64 *c2, const u64 *c3, const u64 *c4, const u64 *c5,
                      size_t n_ops, u64 *out) {
  u64 acc = 0;
  const size_t n4 = n_ops / 4;
  for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += (size_t)gridDim.x * blockDim.x) {
    const size_t g = q * 4;
    const u64 *cs[6] = {c0, c1, c2, c3, c4, c5};
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      u64x2 a = *(const u64x2 *)(cs[c] + g), b = *(const u64x2 *)(cs[c] + g + 2);
      acc ^= a.x + a.y + b.x + b.y;
    }
  }
  if (acc == 0x1234567) out[0] = acc;
}

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
// 3 u64 columns + 3 u32 columns (compressed snapshot deltas)
__global__ void cols33(const u64 *c0, const u64 *c1, const u64 *c2, const unsigned *d0, const unsigned *d1,
                       const unsigned *d2, size_t n_ops, u64 *out) {
  u64 acc = 0;
  const size_t n4 = n_ops / 4;
  for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += (size_t)gridDim.x * blockDim.x) {
    const size_t g = q * 4;
    const u64 *cs[3] = {c0, c1, c2};
    const unsigned *ds[3] = {d0, d1, d2};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      u64x2 a = *(const u64x2 *)(cs[c] + g), b = *(const u64x2 *)(cs[c] + g + 2);
      acc ^= a.x + a.y + b.x + b.y;
      u32x4 v = *(const u32x4 *)(ds[c] + g);
      acc ^= v.x + v.y + v.z + v.w;
    }
  }
  if (acc == 0x1234567) out[0] = acc;
}

template <bool NT>
__global__ void cols(const unsigned *meta, const u64 *c0, const u64 *c1, const u64 *c2, const u64 *c3, const u64 *c4,
                     const u64 *c5, size_t n_ops, u64 *out) {
  u64 acc = 0;
  const size_t n4 = n_ops / 4;
  for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += (size_t)gridDim.x * blockDim.x) {
    const size_t g = q * 4;
    const u64 *cs[6] = {c0, c1, c2, c3, c4, c5};
    unsigned m;
    if (NT) m = __builtin_nontemporal_load(meta + q); else m = meta[q];
    acc ^= m;
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      u64x2 a, b;
      if (NT) {
        a = __builtin_nontemporal_load((const u64x2 *)(cs[c] + g));
        b = __builtin_nontemporal_load((const u64x2 *)(cs[c] + g + 2));
      } else {
        a = *(const u64x2 *)(cs[c] + g);
        b = *(const u64x2 *)(cs[c] + g + 2);
      }
      acc ^= a.x + a.y + b.x + b.y;
    }
  }
  if (acc == 0x1234567) out[0] = acc;
}

int main(int argc, char **argv) {
  const size_t n_ops = (size_t)1 << 28;  // 256M ops = C2
  const size_t bytes_col = n_ops * 8;
  u64 *cols_d[6];
  unsigned *meta;
  u64 *out;
  hipMalloc(&meta, n_ops);
  for (int c = 0; c < 6; ++c) hipMalloc(&cols_d[c], bytes_col);
  hipMalloc(&out, 64);
  hipMemset(meta, 1, n_ops);
  for (int c = 0; c < 6; ++c) hipMemset(cols_d[c], c + 1, bytes_col);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const size_t total = n_ops * (1 + 6 * 8);
  for (int blocks_per_cu : {4, 8, 16}) {
    const int grid = 256 * blocks_per_cu;
    for (int mode = 0; mode < 5; ++mode) {
      float best = 1e9;
      for (int it = 0; it < 6; ++it) {
        hipEventRecord(e0);
        if (mode == 0)
          hipLaunchKernelGGL(flat, dim3(grid), dim3(256), 0, 0, (const u64x2 *)cols_d[0], bytes_col * 6 / 16 > bytes_col / 16 ? bytes_col / 16 : 0, out);
        else if (mode == 1)
          hipLaunchKernelGGL(cols<false>, dim3(grid), dim3(256), 0, 0, meta, cols_d[0], cols_d[1], cols_d[2], cols_d[3],
                             cols_d[4], cols_d[5], n_ops, out);
        else if (mode == 3)
          hipLaunchKernelGGL(cols6, dim3(grid), dim3(256), 0, 0, cols_d[0], cols_d[1], cols_d[2], cols_d[3], cols_d[4],
                             cols_d[5], n_ops, out);
        else if (mode == 4)
          hipLaunchKernelGGL(cols33, dim3(grid), dim3(256), 0, 0, cols_d[0], cols_d[1], cols_d[2], (const unsigned *)cols_d[3],
                             (const unsigned *)cols_d[4], (const unsigned *)cols_d[5], n_ops, out);
        else
          hipLaunchKernelGGL(cols<true>, dim3(grid), dim3(256), 0, 0, meta, cols_d[0], cols_d[1], cols_d[2], cols_d[3],
                             cols_d[4], cols_d[5], n_ops, out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (it > 0 && ms < best) best = ms;
      }
      const double b = mode == 0 ? (double)bytes_col : mode == 3 ? (double)n_ops * 48 : mode == 4 ? (double)n_ops * 36 : (double)total;
      printf("blocks/CU %2d mode %d: %.3f ms  %.0f GB/s\n", blocks_per_cu, mode, best, b / (best * 1e-3) / 1e9);
    }
  }
  return 0;
}
