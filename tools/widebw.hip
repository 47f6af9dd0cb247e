// tools/widebw.hip -- calibration probe for k_pass1w's access pattern (BASELINE config 3: 16,384
// rows of 1 MiB, one 64-row chunk per CU): every chunk streams 256-B tiles of its 64 rows in
// step, W loader waves per chunk with D tiles of loads in flight each.  No LDS, no compute.
// Variants: row stride padded (channel mapping of the 1-MiB row stride), and a per-chunk phase
// (chunk c starts at tile (c * rot) mod ntiles and wraps, so chunks read different offsets at
// the same time).  Not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int D, int W>
__global__ __launch_bounds__(64 * W) void pat(const unsigned char *base, size_t M, size_t S,
                                               unsigned rot, unsigned *out) {
  constexpr int SLOTS = 16, RPI = 4, NLD = 64 / RPI / W;  // 256-B tiles
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int lr = lane / SLOTS, ls = lane % SLOTS;
  const unsigned char *p = base + (size_t)blockIdx.x * 64 * S + ls * 16;
  const int ntiles = (int)(M / 256);
  const int t0 = (int)((blockIdx.x * rot) % ntiles);
  u32x4 acc = {0, 0, 0, 0};
  u32x4 r[D][NLD];
  auto tile_of = [&](int t) { int x = t0 + t; return x >= ntiles ? x - ntiles : x; };
#pragma unroll
  for (int d = 0; d < D; d++)
#pragma unroll
    for (int i = 0; i < NLD; i++) {
      const int row = (wave * NLD + i) * RPI + lr;
      r[d][i] = __builtin_nontemporal_load((const u32x4 *)(p + (size_t)row * S + (size_t)tile_of(d) * 256));
    }
  for (int t = 0; t < ntiles; t += D) {
#pragma unroll
    for (int d = 0; d < D; d++) {
#pragma unroll
      for (int i = 0; i < NLD; i++) acc |= r[d][i];
      const int tn = tile_of(min(t + d + D, ntiles - 1));
#pragma unroll
      for (int i = 0; i < NLD; i++) {
        const int row = (wave * NLD + i) * RPI + lr;
        r[d][i] = __builtin_nontemporal_load((const u32x4 *)(p + (size_t)row * S + (size_t)tn * 256));
      }
    }
  }
  if ((acc.x | acc.y | acc.z | acc.w) == 0xdeadbeefu) out[0] = 1;
}

template <int D, int W>
void run(const unsigned char *p, size_t n, size_t M, size_t S, unsigned rot, unsigned *o) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float best = 1e9;
  for (int r = 0; r < 4; r++) {
    (void)hipEventRecord(a);
    hipLaunchKernelGGL((pat<D, W>), dim3(n / 64), dim3(64 * W), 0, 0, p, M, S, rot, o);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    best = ms < best ? ms : best;
  }
  printf("stride %8zu rot %5u depth %d waves/chunk %d: %.3f ms %.1f GB/s\n", S, rot, D, W, best,
         n * M / (best * 1e-3) / 1e9);
}

int main() {
  const size_t n = 16384, M = 1 << 20;
  unsigned char *p;
  unsigned *o;
  if (hipMalloc(&p, n * (M + 4096)) || hipMalloc(&o, 4)) return 1;
  (void)hipMemset(p, 1, n * (M + 4096));
  const size_t strides[] = {M, M + 256, M + 4096};
  for (size_t S : strides) {
    run<2, 2>(p, n, M, S, 0, o);
    run<4, 2>(p, n, M, S, 0, o);
    run<2, 4>(p, n, M, S, 0, o);
  }
  const unsigned rots[] = {1, 16, 17, 257, 1031};
  for (unsigned rot : rots) {
    run<2, 2>(p, n, M, M, rot, o);
    run<2, 4>(p, n, M, M, rot, o);
  }
  return 0;
}
