// tools/patprobe.hip -- calibration probe for pass 1's access pattern: one chunk = 64 rows of
// a [n x M] row-major batch, streamed in tiles of TW bytes of every row, with D tiles of loads
// in flight per wave and W waves per chunk (rows split between waves).  No LDS, no compute:
// the loaded words are OR-reduced.  Not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int TW, int D, int W>
__global__ __launch_bounds__(64 * W) void pat(const unsigned char *base, size_t M, size_t S, unsigned *out) {
  constexpr int SLOTS = TW / 16, RPI = 64 / SLOTS, NLD = 64 / RPI / W;  // loads per lane per tile
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int lr = lane / SLOTS, ls = lane % SLOTS;
  const unsigned char *p = base + (size_t)blockIdx.x * 64 * S + ls * 16;
  const int ntiles = (int)(M / TW);
  u32x4 acc = {0, 0, 0, 0};
  u32x4 r[D][NLD];
#pragma unroll
  for (int d = 0; d < D; d++)
#pragma unroll
    for (int i = 0; i < NLD; i++) {
      const int row = (wave * NLD + i) * RPI + lr;
      r[d][i] = __builtin_nontemporal_load((const u32x4 *)(p + (size_t)row * S + (size_t)d * TW));
    }
  for (int t = 0; t < ntiles; t += D) {
#pragma unroll
    for (int d = 0; d < D; d++) {
#pragma unroll
      for (int i = 0; i < NLD; i++) acc |= r[d][i];
      const int tn = min(t + d + D, ntiles - 1);
#pragma unroll
      for (int i = 0; i < NLD; i++) {
        const int row = (wave * NLD + i) * RPI + lr;
        r[d][i] = __builtin_nontemporal_load((const u32x4 *)(p + (size_t)row * S + (size_t)tn * TW));
      }
    }
  }
  if ((acc.x | acc.y | acc.z | acc.w) == 0xdeadbeefu) out[0] = 1;
}

template <int TW, int D, int W>
void run(const unsigned char *p, size_t n, size_t M, size_t S, unsigned *o) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float best = 1e9;
  for (int r = 0; r < 5; r++) {
    (void)hipEventRecord(a);
    hipLaunchKernelGGL((pat<TW, D, W>), dim3(n / 64), dim3(64 * W), 0, 0, p, M, S, o);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    best = ms < best ? ms : best;
  }
  printf("stride %6zu TW %4d depth %d waves/chunk %d: %.3f ms %.1f GB/s\n", S, TW, D, W, best,
         n * M / (best * 1e-3) / 1e9);
}

int main(int argc, char **argv) {
  const size_t n = 65536, M = 65536;
  const size_t pads[] = {0, 256, 512, 4096 + 256};
  unsigned char *p;
  unsigned *o;
  if (hipMalloc(&p, n * (M + 4096 + 256)) || hipMalloc(&o, 4)) return 1;
  (void)hipMemset(p, 1, n * (M + 4096 + 256));
  for (size_t pad : pads) {
    const size_t S = M + pad;
    run<256, 2, 2>(p, n, M, S, o);
    run<256, 4, 2>(p, n, M, S, o);
    run<256, 2, 4>(p, n, M, S, o);
    run<512, 2, 2>(p, n, M, S, o);
    run<1024, 2, 2>(p, n, M, S, o);
  }
  run<256, 1, 1>(p, n, M, M, o);
  run<256, 2, 1>(p, n, M, M, o);
  run<256, 4, 1>(p, n, M, M, o);
  return 0;
}
