// tools/claimprobe.hip -- calibration probe (not product): the latency of k_tail's inline claim
// flush (claims_flush) -- 8 claims, each one byte of the 64 rows of a chunk (lane = row), all
// loads in flight together, the next flush after the previous one's data arrived -- as a function
// of the row stride (config 2: 64 KiB) and of the load on the rest of the GPU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ __launch_bounds__(64) void flushes(const uint8_t *t, size_t stride, uint32_t nchunks,
                                              int nflush, uint32_t seed, uint32_t *out) {
  const int lane = threadIdx.x;
  uint32_t acc = 0, x = seed ^ (blockIdx.x * 0x9e3779b9u);
  for (int f = 0; f < nflush; f++) {
    uint32_t v[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      x = x * 1664525u + 1013904223u + (acc & 1u);  // depends on the previous flush's data
      const uint32_t chunk = (x >> 8) % nchunks;
      const uint32_t col = (x * 2654435761u) % (uint32_t)(stride > 65536 ? 65536 : stride);
      v[j] = t[((size_t)chunk * 64 + lane) * stride + col];
    }
#pragma unroll
    for (int j = 0; j < 8; j++) acc += v[j];
    acc = __shfl(acc, 0) + lane;  // wave-uniform dependency
  }
  out[blockIdx.x * 64 + lane] = acc;
}

int main() {
  const size_t rows = 65536;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  uint32_t *o;
  if (hipMalloc(&o, 4096 * 64 * 4) != hipSuccess) return 1;
  for (size_t stride : {(size_t)65536, (size_t)65536 + 256, (size_t)65536 + 4096}) {
    uint8_t *t;
    if (hipMalloc(&t, rows * stride) != hipSuccess) return 1;
    (void)hipMemset(t, 1, rows * stride);
    for (int waves : {1, 256, 2048}) {
      for (int rep = 0; rep < 2; rep++) {
        float ms;
        const int nf = 64;
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(flushes, dim3(waves), dim3(64), 0, 0, t, stride, (uint32_t)(rows / 64), nf,
                           (uint32_t)(rep * 7 + 1), o);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms, a, b);
        if (rep)
          printf("stride %6zu  waves %4d: %6.2f us per flush of 8 claims (%d flushes)\n", stride,
                 waves, ms * 1e3 / nf, nf);
      }
    }
    (void)hipFree(t);
  }
  return (int)hipDeviceSynchronize();
}
