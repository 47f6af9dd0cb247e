// tools/xprobe.hip -- VALU throughput of k_pass1d's transform work (classify_counts of 16
// independent dwords, then the hash32 mix of the 8 words) against the number of waves per SIMD
// (1..4), timed by wall clock (HIP events) and by s_memtime / s_memrealtime (the shader clock).
// Decides whether more transform waves per SIMD buy issue throughput.  Not part of the product.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#include "../killerbeez_amd/csrc/kbz_device.h"

using namespace kbz;

// mix with the two 64-bit multiplies as three v_mad_u64_u32 each (no v_mul_lo / v_add3)
__device__ __forceinline__ uint64_t mul64_mad3(uint32_t lo, uint32_t hi, uint64_t c) {
  uint64_t p, q, r, cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(p), "=s"(cc) : "v"(lo), "s"((uint32_t)c));
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(q), "=s"(cc) : "v"(lo), "s"((uint32_t)(c >> 32)), "v"(p >> 32));
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cc) : "v"(hi), "s"((uint32_t)c), "v"(q));
  (void)cc;
  return (p & 0xffffffffull) | (r << 32);
}
__device__ __forceinline__ uint64_t mix_mad3(uint64_t k) {
  const uint64_t a = mul64_mad3((uint32_t)k, (uint32_t)(k >> 32), kH32C1);
  const uint32_t al = (uint32_t)a, ah = (uint32_t)(a >> 32);
  const uint32_t rl = __builtin_amdgcn_alignbit(al, ah, 1);
  const uint32_t rh = __builtin_amdgcn_alignbit(ah, al, 1);
  return mul64_mad3(rl, rh, kH32C2);
}

template <int V>
__global__ __launch_bounds__(1024) void probe(const uint32_t *in, uint32_t *out, int iters,
                                              unsigned long long *clk) {
  uint32_t a[16];
#pragma unroll
  for (int i = 0; i < 16; i++) a[i] = in[(threadIdx.x * 16 + i) & 4095];
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; it++) {
    if (V == 0 || V == 2) {
#pragma unroll
      for (int i = 0; i < 16; i++) a[i] = classify4(a[i]) ^ (uint32_t)it;
    }
    if (V == 1 || V == 2) {
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const uint64_t m = h32_mix_mad((uint64_t)a[2 * i] | ((uint64_t)a[2 * i + 1] << 32));
        a[2 * i] = (uint32_t)m ^ (uint32_t)it;
        a[2 * i + 1] = (uint32_t)(m >> 32);
      }
    }
    if (V == 3) {
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const uint64_t m = mix_mad3((uint64_t)a[2 * i] | ((uint64_t)a[2 * i + 1] << 32));
        a[2 * i] = (uint32_t)m ^ (uint32_t)it;
        a[2 * i + 1] = (uint32_t)(m >> 32);
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    clk[0] = t1 - t0;
    clk[1] = r1 - r0;
  }
}

typedef void (*kfn)(const uint32_t *, uint32_t *, int, unsigned long long *);

int main() {
  const int iters = 2048;
  uint32_t *in, *out;
  unsigned long long *clk;
  if (hipMalloc(&in, 4096 * 4) || hipMalloc(&out, 256 * 1024 * 4) || hipMalloc(&clk, 16)) return 1;
  uint32_t h[4096];
  for (int i = 0; i < 4096; i++) h[i] = 0x9e3779b9u * (i + 7);
  (void)hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  kfn ks[] = {probe<0>, probe<1>, probe<2>, probe<3>};
  const char *names[] = {"classify4 x16", "mix (v_mul_lo form) x8", "classify x16 + mix x8",
                         "mix (3 v_mad_u64_u32 per multiply) x8"};
  // VALU per iteration and lane, from the ISA of k_pass1d: classify 9 per dword, mix 10 per word
  const double valu[] = {16 * 9 + 16, 8 * 10 + 8, 16 * 9 + 8 * 10 + 16, 8 * 8 + 8};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int v = 0; v < 4; v++) {
    for (int w = 1; w <= 4; w++) {  // waves per SIMD: 4 * w waves per CU, one block per CU
      float ms = 0;
      for (int rep = 0; rep < 3; rep++) {
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(ks[v], dim3(256), dim3(256 * w), 0, 0, in, out, iters, clk);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
      }
      unsigned long long c[2];
      (void)hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
      const double ghz = (double)c[0] / ((double)c[1] / 100e6) / 1e9;
      const double instr = valu[v] * iters * w;  // VALU wave-instructions per SIMD
      printf("%-40s waves/SIMD %d: %.3f ms, clock %.2f GHz, %.2f SIMD-cycles per VALU (est.)\n",
             names[v], w, ms, ghz, (double)c[0] / instr);
    }
  }
  return 0;
}
