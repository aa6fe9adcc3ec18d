// bw_probe_c3s.hip -- HBM read rate of the C3 op stream (8 packed u32 commit-vector columns,
// 1024-op reads, one wave per read) under the wave kernel's shape, to size its pipelining.
// Not part of the product.   hipcc --offload-arch=gfx950 -O3 scripts/bw_probe_c3s.hip -o /tmp/bw_c3s
//   mode 0: SoA columns, 256-op tiles one at a time (the wave kernel's tile loop)
//   mode 1: SoA, two tiles in flight (double-buffered)
//   mode 2: SoA, the read's four tiles in flight together
//   mode 3: AoSoA (256-op blocks, the 8 columns of a block contiguous: 8 KB), one tile at a time
//   mode 4: AoSoA, two tiles in flight
//   mode 5: flat 16-byte reads of the same bytes (ceiling)
// LDS per block limits residency to W waves per CU (the wave kernel: 16).
#include <hip/hip_runtime.h>

#include <cstdio>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int D = 8;
constexpr size_t OPS = 1024;

template <int MODE>
__global__ void __launch_bounds__(256) probe(const unsigned *pk, size_t n, unsigned long long *out) {
  extern __shared__ unsigned sm[];
  const unsigned lane = threadIdx.x & 63;
  const size_t nreads = n / OPS;
  const size_t W = (size_t)gridDim.x * 4;
  unsigned acc = 0;
  auto soa = [&](size_t t, u32x4 *v) {
#pragma unroll
    for (int d = 0; d < D; ++d) v[d] = *(const u32x4 *)(pk + (size_t)d * n + t + 4 * lane);
  };
  auto aos = [&](size_t t, u32x4 *v) {
    const unsigned *b = pk + (t / 256) * 256 * D;
#pragma unroll
    for (int d = 0; d < D; ++d) v[d] = *(const u32x4 *)(b + d * 256 + 4 * lane);
  };
  auto use = [&](const u32x4 *v) {
#pragma unroll
    for (int d = 0; d < D; ++d) acc += v[d].x ^ v[d].y ^ v[d].z ^ v[d].w;
  };
  for (size_t r = (size_t)blockIdx.x * 4 + threadIdx.x / 64; r < nreads; r += W) {
    const size_t t0 = r * OPS;
    if (MODE == 0 || MODE == 3) {
      for (size_t t = t0; t < t0 + OPS; t += 256) {
        u32x4 v[D];
        if (MODE == 0) soa(t, v);
        else aos(t, v);
        use(v);
      }
    } else if (MODE == 1 || MODE == 4) {
      u32x4 a[D], b[D];
      if (MODE == 1) soa(t0, a), soa(t0 + 256, b);
      else aos(t0, a), aos(t0 + 256, b);
      use(a);
      if (MODE == 1) soa(t0 + 512, a);
      else aos(t0 + 512, a);
      use(b);
      if (MODE == 1) soa(t0 + 768, b);
      else aos(t0 + 768, b);
      use(a);
      use(b);
    } else if (MODE == 2) {
      u32x4 a[D], b[D], c[D], e[D];
      soa(t0, a), soa(t0 + 256, b), soa(t0 + 512, c), soa(t0 + 768, e);
      use(a), use(b), use(c), use(e);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const u32x4 v = *(const u32x4 *)(pk + t0 * D + (size_t)k * 1024 + 4 * lane);
        acc += v.x ^ v.y ^ v.z ^ v.w;
      }
    }
    sm[threadIdx.x] = acc;  // keep the LDS allocation live
  }
  if (acc == 0x1234567) out[0] = acc;
}

template <int MODE>
float run(const unsigned *pk, size_t n, unsigned long long *out, int wpc) {
  const size_t lds = 160 * 1024 / (wpc / 4) - 64;
  hipFuncSetAttribute((const void *)probe<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const unsigned blocks = 256 * (wpc / 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float best = 1e30f;
  for (int it = 0; it < 4; ++it) {
    hipEventRecord(e0);
    probe<MODE><<<blocks, 256, lds>>>(pk, n, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  return best;
}

int main() {
  const size_t n = (size_t)1 << 30;
  const double bytes = (double)n * 4 * D;
  unsigned *pk = nullptr;
  unsigned long long *out = nullptr;
  if (hipMalloc(&pk, (size_t)bytes + 4096) || hipMalloc(&out, 64)) {
    printf("alloc failed\n");
    return 1;
  }
  hipMemset(pk, 1, (size_t)bytes);
  for (int wpc : {16, 32}) {
    float ms[6] = {run<0>(pk, n, out, wpc), run<1>(pk, n, out, wpc), run<2>(pk, n, out, wpc),
                   run<3>(pk, n, out, wpc), run<4>(pk, n, out, wpc), run<5>(pk, n, out, wpc)};
    for (int m = 0; m < 6; ++m)
      printf("waves/CU %2d mode %d: %.3f ms  %.0f GB/s\n", wpc, m, ms[m], bytes / (ms[m] * 1e-3) / 1e9);
    fflush(stdout);
  }
  return 0;
}
