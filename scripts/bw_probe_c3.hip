// bw_probe_c3.hip -- achievable HBM read bandwidth for the C3 packed-view access pattern
// (ct_meta u64 + 8 int32 snapshot-delta columns per op), to decide the packed layout.
// Not part of the product.
//   mode 0: SoA columns (the current layout), grid-stride over 128-op tiles
//   mode 1: SoA columns, one wave walks one 1024-op read (8 tiles) then the next read
//   mode 2: AoSoA -- 256-op blocks [ct_meta x256 | delta0 x256 | ... | delta7 x256]
//           (10 KB contiguous per block), one wave walks one 1024-op read
//   mode 3: flat float4 read of the same bytes (the copy-kernel ceiling)
// Build: hipcc --offload-arch=gfx950 -O3 scripts/bw_probe_c3.hip -o /tmp/bw_c3
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int D = 8;

__global__ void soa_stride(const u64 *ct, const unsigned *dl, size_t n, size_t stride, u64 *out) {
  u64 acc = 0;
  const size_t lanes = (size_t)gridDim.x * blockDim.x;
  for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q * 2 < n; q += lanes) {
    const size_t g = q * 2;
    u64x2 c = *(const u64x2 *)(ct + g);
    acc ^= c.x + c.y;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      u32x2 v = *(const u32x2 *)(dl + (size_t)d * stride + g);
      acc += v.x ^ v.y;
    }
  }
  if (acc == 0x1234567) out[0] = acc;
}

// one wave per read of 1024 ops; reads visited in a scrambled order (like bench keys by wave)
__global__ void soa_reads(const u64 *ct, const unsigned *dl, size_t n, size_t stride, u64 *out) {
  u64 acc = 0;
  const unsigned lane = threadIdx.x & 63;
  const size_t nreads = n / 1024;
  const size_t W = (size_t)gridDim.x * (blockDim.x / 64);
  for (size_t r = (size_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64; r < nreads; r += W) {
    for (size_t t = r * 1024; t < (r + 1) * 1024; t += 128) {
      const size_t g = t + lane * 2;
      u64x2 c = *(const u64x2 *)(ct + g);
      acc ^= c.x + c.y;
#pragma unroll
      for (int d = 0; d < D; ++d) {
        u32x2 v = *(const u32x2 *)(dl + (size_t)d * stride + g);
        acc += v.x ^ v.y;
      }
    }
  }
  if (acc == 0x1234567) out[0] = acc;
}

// AoSoA blocks of 256 ops: block b at b * (256 * (2 + D)) dwords
__global__ void aosoa_reads(const unsigned *blk, size_t n, u64 *out) {
  u64 acc = 0;
  const unsigned lane = threadIdx.x & 63;
  const size_t nreads = n / 1024;
  const size_t W = (size_t)gridDim.x * (blockDim.x / 64);
  for (size_t r = (size_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64; r < nreads; r += W) {
    for (size_t t = r * 1024; t < (r + 1) * 1024; t += 128) {
      const size_t b = t / 256, o = (t % 256) + lane * 2;
      const unsigned *base = blk + b * (256 * (2 + D));
      u64x2 c = *(const u64x2 *)((const u64 *)base + o);
      acc ^= c.x + c.y;
#pragma unroll
      for (int d = 0; d < D; ++d) {
        u32x2 v = *(const u32x2 *)(base + 512 + d * 256 + o);
        acc += v.x ^ v.y;
      }
    }
  }
  if (acc == 0x1234567) out[0] = acc;
}

__global__ void flat(const u32x4 *a, size_t n4, u64 *out) {
  u64 acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    u32x4 v = a[i];
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x1234567) out[0] = acc;
}

int main(int argc, char **argv) {
  const size_t n = (size_t)1 << 30;  // ops
  const size_t stride = n;
  const double bytes = (double)n * (8 + 4 * D);
  // one allocation holds every layout: SoA = [ct_meta n x u64 | delta_d n x u32 ...],
  // AoSoA = the same bytes read as 256-op blocks
  unsigned *buf = nullptr;
  u64 *out = nullptr;
  if (hipMalloc(&buf, (size_t)bytes + 4096) || hipMalloc(&out, 64)) {
    printf("alloc failed\n");
    return 1;
  }
  hipMemset(buf, 1, (size_t)bytes);
  const u64 *ct = (const u64 *)buf;
  const unsigned *dl = buf + 2 * n;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int mode = 0; mode < 4; ++mode) {
    for (int bpc : {4, 8, 16}) {
      const unsigned blocks = 256 * bpc;
      float best = 1e30f;
      for (int it = 0; it < 5; ++it) {
        hipEventRecord(e0);
        if (mode == 0) soa_stride<<<blocks, 256>>>(ct, dl, n, stride, out);
        if (mode == 1) soa_reads<<<blocks, 256>>>(ct, dl, n, stride, out);
        if (mode == 2) aosoa_reads<<<blocks, 256>>>(buf, n, out);
        if (mode == 3) flat<<<blocks, 256>>>((const u32x4 *)buf, (size_t)(bytes / 16), out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }
      printf("mode %d blocks/CU %2d: %.3f ms  %.0f GB/s\n", mode, bpc, best, bytes / (best * 1e-3) / 1e9);
      fflush(stdout);
    }
  }
  return 0;
}
