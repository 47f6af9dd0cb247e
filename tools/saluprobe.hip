// tools/saluprobe.hip -- calibration probe (not product): cycles per hash32 chain step of ONE
// trace, the latency that sets a DynamoRIO window of a few execs (the plugin at batch 1-16).
//   salu_pure  : the chain on the scalar unit, words generated in registers (no memory)
//   salu_load  : the same with the words read as uniform loads, 16 words double-buffered
//   salu_readlane: words mixed per lane, read into SGPRs by v_readlane, chained on the SALU
//   valu_pure  : the chain per lane (64 traces per wave), words in registers, as chainprobe
//   valu_load  : per lane, words loaded lane-coalesced 8 steps ahead
// v1 of this probe waited on each 8-word scalar load (135 cycles/step): the load latency, not
// the chain.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint64_t step(uint64_t h, uint64_t k) {
  h ^= k;
  h = (h << 27) | (h >> 37);
  return (h << 2) + h + 0x52dce729ull;
}

__device__ __forceinline__ uint64_t uni(uint64_t x) {
  return (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)x) |
         ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32)) << 32);
}

__global__ __launch_bounds__(64) void salu_pure(uint32_t nw, uint64_t *out) {
  uint64_t h = uni(0xa5b35705ull ^ nw ^ blockIdx.x);
  uint64_t k = uni(0x9e3779b97f4a7c15ull * (blockIdx.x + 1));
  for (uint32_t j = 0; j < nw; j++) {
    h = step(h, k);
    k += 0x9e3779b97f4a7c15ull;
  }
  if (threadIdx.x == 0) out[blockIdx.x] = h;
}

__global__ __launch_bounds__(64) void salu_load(const uint64_t *__restrict__ kb, uint32_t nw,
                                                uint64_t *out) {
  const uint64_t *p = kb + (size_t)blockIdx.x * nw;
  uint64_t h = uni(0xa5b35705ull ^ nw);
  uint64_t cur[16], nxt[16];
#pragma unroll
  for (int u = 0; u < 16; u++) cur[u] = p[u];
  for (uint32_t j = 16; j <= nw; j += 16) {
    const uint32_t jn = j < nw ? j : 0;
#pragma unroll
    for (int u = 0; u < 16; u++) nxt[u] = p[jn + u];
#pragma unroll
    for (int u = 0; u < 16; u++) h = step(h, cur[u]);
#pragma unroll
    for (int u = 0; u < 16; u++) cur[u] = nxt[u];
  }
  if (threadIdx.x == 0) out[blockIdx.x] = h;
}

// the words mixed per lane (one VALU instruction covers 64 words), then read into SGPRs one
// lane at a time (v_readlane, independent of the chain) and chained on the scalar unit
__global__ __launch_bounds__(64) void salu_readlane(const uint64_t *__restrict__ kb, uint32_t nw,
                                                    uint64_t *out) {
  const uint64_t *p = kb + (size_t)blockIdx.x * nw;
  uint64_t h = uni(0xa5b35705ull ^ nw);
  for (uint32_t j = 0; j < nw; j += 64) {
    const uint64_t kv = p[j + threadIdx.x] * 0x9e3779b97f4a7c15ull;
    const uint32_t lo = (uint32_t)kv, hi = (uint32_t)(kv >> 32);
#pragma unroll
    for (int l = 0; l < 64; l++)
      h = step(h, (uint64_t)__builtin_amdgcn_readlane(lo, l) |
                      ((uint64_t)__builtin_amdgcn_readlane(hi, l) << 32));
  }
  if (threadIdx.x == 0) out[blockIdx.x] = h;
}

__global__ __launch_bounds__(64) void valu_pure(uint32_t nw, uint64_t *out) {
  const uint32_t t = blockIdx.x * 64 + threadIdx.x;
  uint64_t h = 0xa5b35705ull ^ nw ^ t;
  uint64_t k = 0x9e3779b97f4a7c15ull * (t + 1);
  for (uint32_t j = 0; j < nw; j++) {
    h = step(h, k);
    k += 0x9e3779b97f4a7c15ull;
  }
  out[t] = h;
}

__global__ __launch_bounds__(64) void valu_load(const uint64_t *__restrict__ kb, uint32_t nw,
                                                uint64_t *out) {
  const uint32_t t = blockIdx.x * 64 + threadIdx.x, T = gridDim.x * 64;
  uint64_t h = 0xa5b35705ull ^ nw;
  uint64_t cur[8], nxt[8];
#pragma unroll
  for (int u = 0; u < 8; u++) cur[u] = kb[(size_t)u * T + t];
  for (uint32_t j = 8; j <= nw; j += 8) {
    const uint32_t jn = j < nw ? j : 0;
#pragma unroll
    for (int u = 0; u < 8; u++) nxt[u] = kb[(size_t)(jn + u) * T + t];
#pragma unroll
    for (int u = 0; u < 8; u++) h = step(h, cur[u]);
#pragma unroll
    for (int u = 0; u < 8; u++) cur[u] = nxt[u];
  }
  out[t] = h;
}

static float timed(void (*launch)(), hipEvent_t a, hipEvent_t b) {
  float ms = 0;
  (void)hipEventRecord(a);
  launch();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  (void)hipEventElapsedTime(&ms, a, b);
  return ms;
}

static const uint32_t NW = 8192;  // one 64 KiB map: 8,192 words
static uint64_t *K, *O;
static void l_sp() { hipLaunchKernelGGL(salu_pure, dim3(1), dim3(64), 0, 0, NW, O); }
static void l_sp256() { hipLaunchKernelGGL(salu_pure, dim3(256), dim3(64), 0, 0, NW, O); }
static void l_sl() { hipLaunchKernelGGL(salu_load, dim3(1), dim3(64), 0, 0, K, NW, O); }
static void l_sl256() { hipLaunchKernelGGL(salu_load, dim3(256), dim3(64), 0, 0, K, NW, O); }
static void l_srl() { hipLaunchKernelGGL(salu_readlane, dim3(1), dim3(64), 0, 0, K, NW, O); }
static void l_vp() { hipLaunchKernelGGL(valu_pure, dim3(1), dim3(64), 0, 0, NW, O); }
static void l_vl() { hipLaunchKernelGGL(valu_load, dim3(1), dim3(64), 0, 0, K, NW, O); }
static void l_empty() { hipLaunchKernelGGL(salu_pure, dim3(1), dim3(64), 0, 0, 0u, O); }

int main() {
  if (hipMalloc(&K, (size_t)256 * 64 * NW * 8) != hipSuccess ||
      hipMalloc(&O, 256 * 64 * 8) != hipSuccess)
    return 1;
  (void)hipMemset(K, 0x5a, (size_t)256 * 64 * NW * 8);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  struct { const char *name; void (*f)(); } runs[] = {
      {"empty launch (0 steps)", l_empty},
      {"salu_pure 1 wave", l_sp},
      {"salu_pure 256 waves", l_sp256},
      {"salu_load 1 wave", l_sl},
      {"salu_load 256 waves", l_sl256},
      {"salu_readlane 1 wave", l_srl},
      {"valu_pure 1 wave (64 traces)", l_vp},
      {"valu_load 1 wave (64 traces)", l_vl},
  };
  for (int rep = 0; rep < 3; rep++)
    for (auto &r : runs) {
      float ms = timed(r.f, a, b);
      printf("rep %d  %-30s %8.1f us  %6.1f cycles/step at 2.4 GHz\n", rep, r.name, ms * 1e3,
             ms * 1e-3 * 2.4e9 / NW);
    }
  return (int)hipDeviceSynchronize();
}
