// tools/chainprobe.hip -- latency of one hash32 chain step, h' = rotl(h ^ k, 27) * 5 + C
// (afl_progs/hash.h:51-53), in several instruction forms, measured as a long dependent chain
// in one wave per SIMD (the regime of pass 1 on large maps, where the per-trace chain is the
// critical path).  Not part of the product.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

__device__ __forceinline__ uint64_t step_default(uint64_t h, uint64_t k) {
  h ^= k;
  h = (h << 27) | (h >> 37);
  return h * 5 + 0x52dce729;
}
__device__ __forceinline__ uint64_t step_u64(uint64_t h, uint64_t k) {  // pass 1's form
  const uint32_t lo = (uint32_t)h ^ (uint32_t)k, hi = (uint32_t)(h >> 32) ^ (uint32_t)(k >> 32);
  const uint32_t rl = __builtin_amdgcn_alignbit(lo, hi, 5);
  const uint32_t rh = __builtin_amdgcn_alignbit(hi, lo, 5);
  uint64_t r = ((uint64_t)rh << 32) | rl, t;
  const uint64_t c = 0x52dce729ull;
  asm("v_lshl_add_u64 %0, %1, 2, %1" : "=v"(t) : "v"(r));
  asm("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(r) : "v"(t), "s"(c));
  return r;
}
__device__ __forceinline__ uint64_t step_u32(uint64_t h, uint64_t k) {  // 32-bit ops, carries
  const uint32_t lo = (uint32_t)h ^ (uint32_t)k, hi = (uint32_t)(h >> 32) ^ (uint32_t)(k >> 32);
  const uint32_t rl = __builtin_amdgcn_alignbit(lo, hi, 5);
  const uint32_t rh = __builtin_amdgcn_alignbit(hi, lo, 5);
  uint32_t o_lo, o_hi;
  asm("v_lshlrev_b32 %0, 2, %2\n\t"
      "v_alignbit_b32 %1, %3, %2, 30\n\t"
      "v_add_co_u32 %0, vcc, %2, %0\n\t"
      "v_addc_co_u32 %1, vcc, %3, %1, vcc\n\t"
      "v_add_co_u32 %0, vcc, 0x52dce729, %0\n\t"
      "v_addc_co_u32 %1, vcc, 0, %1, vcc"
      : "=&v"(o_lo), "=&v"(o_hi)
      : "v"(rl), "v"(rh)
      : "vcc");
  return ((uint64_t)o_hi << 32) | o_lo;
}
__device__ __forceinline__ uint64_t step_mad(uint64_t h, uint64_t k) {  // v_mad_u64_u32 + add
  const uint32_t lo = (uint32_t)h ^ (uint32_t)k, hi = (uint32_t)(h >> 32) ^ (uint32_t)(k >> 32);
  const uint32_t rl = __builtin_amdgcn_alignbit(lo, hi, 5);
  const uint32_t rh = __builtin_amdgcn_alignbit(hi, lo, 5);
  const uint64_t m = (uint64_t)rl * 5u + 0x52dce729ull;  // v_mad_u64_u32
  return m + ((uint64_t)(rh * 5u) << 32);
}

template <int V>
__global__ __launch_bounds__(64) void chain(const uint64_t *ks, uint64_t *out, int steps,
                                            unsigned long long *cyc) {
  uint64_t h = threadIdx.x + 1;
  const uint64_t k0 = ks[threadIdx.x], k1 = ks[threadIdx.x + 64];
  const unsigned long long t0 = clock64();
  for (int i = 0; i < steps; i += 2) {
    if (V == 0) { h = step_default(h, k0); h = step_default(h, k1); }
    if (V == 1) { h = step_u64(h, k0); h = step_u64(h, k1); }
    if (V == 2) { h = step_u32(h, k0); h = step_u32(h, k1); }
    if (V == 3) { h = step_mad(h, k0); h = step_mad(h, k1); }
  }
  const unsigned long long t1 = clock64();
  out[blockIdx.x * 64 + threadIdx.x] = h;
  if (threadIdx.x == 0 && blockIdx.x == 0) cyc[V] = t1 - t0;
}

int main() {
  const int steps = 1 << 16;
  uint64_t *ks, *out;
  unsigned long long *cyc;
  if (hipMalloc(&ks, 128 * 8) || hipMalloc(&out, 1024 * 64 * 8) || hipMalloc(&cyc, 4 * 8)) return 1;
  uint64_t hk[128];
  for (int i = 0; i < 128; i++) hk[i] = 0x9e3779b97f4a7c15ull * (i + 1);
  (void)hipMemcpy(ks, hk, sizeof(hk), hipMemcpyHostToDevice);
  uint64_t ref[4][64];
  const char *names[] = {"compiler default", "v_lshl_add_u64 x2 (pass 1)", "32-bit add/addc",
                         "v_mad_u64_u32"};
  for (int v = 0; v < 4; v++) {
    for (int rep = 0; rep < 2; rep++) {
      if (v == 0) hipLaunchKernelGGL(chain<0>, dim3(256), dim3(64), 0, 0, ks, out, steps, cyc);
      if (v == 1) hipLaunchKernelGGL(chain<1>, dim3(256), dim3(64), 0, 0, ks, out, steps, cyc);
      if (v == 2) hipLaunchKernelGGL(chain<2>, dim3(256), dim3(64), 0, 0, ks, out, steps, cyc);
      if (v == 3) hipLaunchKernelGGL(chain<3>, dim3(256), dim3(64), 0, 0, ks, out, steps, cyc);
    }
    (void)hipDeviceSynchronize();
    unsigned long long c[4];
    (void)hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    (void)hipMemcpy(ref[v], out, 64 * 8, hipMemcpyDeviceToHost);
    printf("%-28s %6.1f cycles per step%s\n", names[v], (double)c[v] / steps,
           (v && __builtin_memcmp(ref[v], ref[0], sizeof(ref[0]))) ? "  RESULT MISMATCH" : "");
  }
  // The config-3 floor: one 1 MiB trace is a chain of 131,072 steps; a batch of 16,384 traces
  // is 256 waves of 64 chains.  Wall time of exactly that (pass 1's step form, keys from
  // registers: no loads, no LDS), with 1 and 4 waves per CU.
  const int chain_steps = 131072;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int blocks : {256, 1024}) {
    hipLaunchKernelGGL(chain<1>, dim3(blocks), dim3(64), 0, 0, ks, out, chain_steps, cyc);
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(chain<1>, dim3(blocks), dim3(64), 0, 0, ks, out, chain_steps, cyc);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%d-step chains, %d waves of 64: %.3f ms\n", chain_steps, blocks, ms);
  }
  return 0;
}
