// tools/bwprobe.hip -- calibration probe: achievable HBM read bandwidth on this MI355X for the
// access pattern pass 1 uses (16 B per lane, coalesced 1 KiB wave-instructions, read once).
// Not part of the product; built and run by scripts/gpu_session.sh (step "probe").
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int UNROLL, bool NT>
__global__ __launch_bounds__(256) void rd(const u32x4 *p, size_t n16, unsigned *out) {
  u32x4 acc = {0, 0, 0, 0};
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (UNROLL - 1) * stride < n16; i += UNROLL * stride) {
    u32x4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; u++) v[u] = NT ? __builtin_nontemporal_load(p + i + u * stride) : p[i + u * stride];
#pragma unroll
    for (int u = 0; u < UNROLL; u++) acc |= v[u];
  }
  for (; i < n16; i += stride) acc |= p[i];
  if ((acc.x | acc.y | acc.z | acc.w) == 0xdeadbeef) out[0] = 1;
}

int main(int argc, char **argv) {
  size_t bytes = (argc > 1 ? atoll(argv[1]) : 4096) << 20;
  u32x4 *p;
  unsigned *o;
  if (hipMalloc(&p, bytes) || hipMalloc(&o, 4)) return 1;
  (void)hipMemset(p, 1, bytes);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  int grids[] = {1024, 2048, 4096, 8192};
  for (int nt = 0; nt < 2; nt++)
    for (int g : grids) {
      float best = 1e9;
      for (int r = 0; r < 5; r++) {
        (void)hipEventRecord(a);
        if (nt) hipLaunchKernelGGL((rd<8, true>), dim3(g), dim3(256), 0, 0, p, bytes / 16, o);
        else hipLaunchKernelGGL((rd<8, false>), dim3(g), dim3(256), 0, 0, p, bytes / 16, o);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
      }
      printf("read %s grid %5d x256: %.3f ms  %.1f GB/s\n", nt ? "nt  " : "plain", g, best,
             bytes / (best * 1e-3) / 1e9);
    }
  return 0;
}
