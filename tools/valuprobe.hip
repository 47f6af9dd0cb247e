// tools/valuprobe.hip -- VALU issue cost on gfx950 of the instructions pass 1's transform waves
// spend their time on (32-bit multiplies, v_mad_u64_u32, bit ops) and of whole per-word
// transform forms (classify_counts SWAR, hash32 mix), measured with 8 independent chains per
// lane and W waves per SIMD (the regime of k_pass1w's transform waves).  Not part of the
// product: it decides which instruction forms k_pass1w uses.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#include "../killerbeez_amd/csrc/kbz_device.h"

using namespace kbz;

// the round-1 form: smear, highest bit, double 4..63, fix c == 3 (16 instructions)
__device__ __forceinline__ uint32_t cls4_old(uint32_t x) {
  uint32_t s = x | ((x >> 1) & 0x7F7F7F7Fu);
  s |= (s >> 2) & 0x3F3F3F3Fu;
  s |= (s >> 4) & 0x0F0F0F0Fu;
  const uint32_t hb = s & ~((s >> 1) & 0x7F7F7F7Fu);
  const uint32_t e3 = x & (x >> 1) & (hb >> 1) & 0x01010101u;
  return hb + (hb & 0x3C3C3C3Cu) + (e3 << 1);
}
// the 13-instruction smear form (round 2 until the bit-reverse form replaced it)
__device__ __forceinline__ uint32_t cls4_smear(uint32_t x) {
  const uint32_t x1 = x << 1, x2 = x << 2;
  const uint32_t z = (x | (x1 & 0x78787878u)) | (x2 & x1 & 0x04040404u);
  uint32_t s = z | ((z >> 1) & 0x7F7F7F7Fu);
  s |= (s >> 2) & 0x3F3F3F3Fu;
  s |= (s >> 4) & 0x0F0F0F0Fu;
  return s ^ ((s >> 1) & 0x7F7F7F7Fu);
}
__device__ __forceinline__ uint64_t mix_default(uint64_t k) { return h32_mix(k); }
__device__ __forceinline__ uint64_t mix_mad(uint64_t k) { return h32_mix_mad(k); }

template <int V>
__global__ __launch_bounds__(512) void probe(const uint32_t *in, uint32_t *out, int iters,
                                             unsigned long long *cyc) {
  uint32_t a[8];
#pragma unroll
  for (int i = 0; i < 8; i++) a[i] = in[(threadIdx.x + i * 64) & 1023];
  const uint32_t s = in[1000];
  __syncthreads();
  const unsigned long long t0 = clock64();
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      if (V == 0) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "s"(s));
      if (V == 1) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "s"(s));
      if (V == 2) {
        uint32_t lo = a[i], hi = a[(i + 1) & 7];
        asm volatile("v_mad_u64_u32 v[0:1], vcc, %0, %1, 0" ::"v"(lo), "s"(s) : "v0", "v1", "vcc");
        (void)hi;
      }
      if (V == 3) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x6c" : "+v"(a[i]) : "s"(s));
      if (V == 4) asm volatile("v_lshl_add_u64 v[0:1], v[0:1], 2, v[0:1]" ::: "v0", "v1");
      if (V == 5) asm volatile("v_alignbit_b32 %0, %0, %0, 5" : "+v"(a[i]));
      if (V == 10) asm volatile("v_perm_b32 %0, %1, %0, %0" : "+v"(a[i]) : "s"(s));
      if (V == 11) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "s"(s));
      if (V == 12) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a[i]) : "s"(s));
      if (V == 13) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(a[i]) : "s"(s));
      if (V == 15) asm volatile("v_bfrev_b32 %0, %0" : "+v"(a[i]));
    }
    if (V == 6) {  // classify4, current SWAR form, 8 independent dwords
#pragma unroll
      for (int i = 0; i < 8; i++) a[i] = cls4_old(a[i]) ^ s;
    }
    if (V == 14) {
#pragma unroll
      for (int i = 0; i < 8; i++) a[i] = cls4_smear(a[i]) ^ s;
    }
    if (V == 7) {
#pragma unroll
      for (int i = 0; i < 8; i++) a[i] = classify4(a[i]) ^ s;
    }
    if (V == 8 || V == 9) {  // hash32 mix of 4 words
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const uint64_t k = (uint64_t)a[2 * i] | ((uint64_t)a[2 * i + 1] << 32);
        const uint64_t m = V == 8 ? mix_default(k) : mix_mad(k);
        a[2 * i] = (uint32_t)m ^ s;
        a[2 * i + 1] = (uint32_t)(m >> 32);
      }
    }
  }
  const unsigned long long t1 = clock64();
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
  if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
}

typedef void (*kfn)(const uint32_t *, uint32_t *, int, unsigned long long *);

int main() {
  const int iters = 4096;
  uint32_t *in, *out;
  unsigned long long *cyc;
  if (hipMalloc(&in, 4096 * 4) || hipMalloc(&out, 1024 * 512 * 4) || hipMalloc(&cyc, 8)) return 1;
  uint32_t h[4096];
  for (int i = 0; i < 4096; i++) h[i] = 0x9e3779b9u * (i + 7);
  (void)hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  kfn ks[] = {probe<0>, probe<1>, probe<2>, probe<3>, probe<4>, probe<5>, probe<6>, probe<7>,
              probe<8>, probe<9>, probe<10>, probe<11>, probe<12>, probe<13>, probe<14>, probe<15>};
  const char *names[] = {"v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64_u32", "v_bitop3_b32",
                         "v_lshl_add_u64", "v_alignbit_b32", "classify4 (round-1 form)",
                         "classify4 (bitrev form)", "h32_mix (compiler)", "h32_mix (mad form)",
                         "v_perm_b32", "v_mul_u32_u24", "v_xor_b32", "v_mad_u32_u24",
                         "classify4 (smear form)", "v_bfrev_b32"};
  // per-"unit": ops 0-5: one instruction of 8 chains; 6-7: one dword classified (8 per iter);
  // 8-9: one 64-bit word mixed (4 per iter)
  const int per_iter[] = {8, 8, 8, 8, 8, 8, 8, 8, 4, 4, 8, 8, 8, 8, 8, 8};
  for (int w = 1; w <= 2; w++) {  // waves per SIMD: block of 256*w threads, 1 block per CU
    for (int v = 0; v < 16; v++) {
      unsigned long long c = 0;
      for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(ks[v], dim3(256), dim3(256 * w), 0, 0, in, out, iters, cyc);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      }
      // cycles of one wave-instruction/unit per SIMD = measured cycles / (units per wave * w)
      const double units = (double)iters * per_iter[v] * w;
      printf("waves/SIMD %d  %-28s %7.2f SIMD-cycles per wave-unit\n", w, names[v], c / units);
    }
  }
  return 0;
}
