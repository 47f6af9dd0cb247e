// killerbeez_amd/csrc/kbz_device.h -- per-byte / per-word arithmetic shared by the gfx950
// kernels (and compiled for the host by tests/test_swar.py's exhaustive check).
//
// All of it is SWAR integer work on 32/64-bit registers; nothing here touches memory.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define KBZ_HD __host__ __device__ __forceinline__
#else
#define KBZ_HD static inline
#endif

namespace kbz {

constexpr uint32_t kHashConst = 0xa5b35705u;  // afl_progs/config.h:323
constexpr uint64_t kH32C1 = 0x87c37b91114253d5ULL, kH32C2 = 0x4cf5ad432745937fULL;
constexpr uint64_t kXP1 = 11400714785074694791ULL, kXP2 = 14029467366897019727ULL,
                   kXP3 = 1609587929392839161ULL, kXP4 = 9650029242287828579ULL,
                   kXP5 = 2870177450012600261ULL;  // xxhash.c:664-668
constexpr uint64_t kSimpleZero = 0x0101010101010101ULL;  // afl_instrumentation.c:688

KBZ_HD uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

KBZ_HD uint32_t bitrev32(uint32_t x) {
#if defined(__clang__)
  return __builtin_bitreverse32(x);  // v_bfrev_b32
#else
  x = ((x >> 1) & 0x55555555u) | ((x & 0x55555555u) << 1);
  x = ((x >> 2) & 0x33333333u) | ((x & 0x33333333u) << 2);
  x = ((x >> 4) & 0x0F0F0F0Fu) | ((x & 0x0F0F0F0Fu) << 4);
  x = ((x >> 8) & 0x00FF00FFu) | ((x & 0x00FF00FFu) << 8);
  return (x >> 16) | (x << 16);
#endif
}

// count_class bucket of every byte (dynamorio_instrumentation.c:246-255), branch-free in 9
// instructions on gfx950: the bucket is the highest set bit of z, where z moves bits 2-5 of the
// count c up by one (c in 4..63 -> doubled), gives c == 3 bit 2 (-> 4) and sets bit 0 of every
// byte (a sentinel: no byte of z is 0).  The highest set bit is the lowest set bit of the
// bit-reversed word, r & -r per byte; with every byte of r >= 0x80, -r per byte is one 32-bit
// subtraction with no borrow between bytes.  The sentinel alone (c == 0) is masked at the end.
// (The round-1 form, a 3-step smear of the highest bit, was 13 instructions:
// tools/valuprobe.hip.)
KBZ_HD uint32_t classify4(uint32_t x) {
  const uint32_t x1 = (x << 1) | 0x01010101u;                 // v_lshl_or_b32
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t m;  // one v_and_or_b32 (the compiler emits v_and + v_or); one SGPR operand at most
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(m) : "v"(x << 2), "s"(0x04040404u), "v"(0x79797979u));
#else
  const uint32_t m = ((x << 2) & 0x04040404u) | 0x79797979u;
#endif
  const uint32_t z = x | (x1 & m);                            // v_and_or_b32
  const uint32_t r = bitrev32(z);
  const uint32_t l = r & (0x01010100u - r);                   // v_sub, v_and
  return bitrev32(l) & (x | 0xFEFEFEFEu);                     // v_bfrev, v_bitop3
}
KBZ_HD uint64_t classify8(uint64_t x) {
  return (uint64_t)classify4((uint32_t)x) | ((uint64_t)classify4((uint32_t)(x >> 32)) << 32);
}

// simplify_lookup (afl_instrumentation.c:668-671): 0 -> 0x01, nonzero -> 0x80 per byte.
KBZ_HD uint32_t simplify4(uint32_t x) {
  const uint32_t nz = (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
  return nz | ((~nz >> 7) & 0x01010101u);
}
KBZ_HD uint64_t simplify8(uint64_t x) {
  return (uint64_t)simplify4((uint32_t)x) | ((uint64_t)simplify4((uint32_t)(x >> 32)) << 32);
}

// 0x80 in every byte of x that is nonzero, 0 elsewhere.
KBZ_HD uint64_t nonzero_hi8(uint64_t x) {
  return (((x & 0x7F7F7F7F7F7F7F7FULL) + 0x7F7F7F7F7F7F7F7FULL) | x) & 0x8080808080808080ULL;
}
// 0xff in every byte of x that is nonzero (0x80 - 0x01 = 0x7f borrows from no other byte; no
// multiply: a 32-bit v_mul_lo_u32 is a quarter-rate instruction).
KBZ_HD uint64_t nonzero_bytes8(uint64_t x) {
  const uint64_t nz = nonzero_hi8(x);
  return nz | (nz - (nz >> 7));
}

// hash32 pieces (afl_progs/hash.h:36-65): per-word mix, chain step, finalizer.
KBZ_HD uint64_t h32_mix(uint64_t k) {
  k *= kH32C1;
  k = rotl64(k, 31);
  return k * kH32C2;
}
#if defined(__HIPCC__)
// k * C mod 2^64 as one v_mad_u64_u32 (lo * C.lo, 64-bit) and two v_mul_lo_u32 for the cross
// terms; the compiler's own lowering spends a fourth multiply (v_mul_hi_u32) on some of them.
__device__ __forceinline__ uint64_t mul64_const(uint32_t lo, uint32_t hi, uint64_t c) {
  uint64_t p, cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(p), "=s"(cc) : "v"(lo), "s"((uint32_t)c));
  (void)cc;
  const uint32_t ph = (uint32_t)(p >> 32) + lo * (uint32_t)(c >> 32) + hi * (uint32_t)c;
  return (p & 0xffffffffull) | ((uint64_t)ph << 32);
}
// h32_mix with 6 multiplies and the rotation as two v_alignbit.
__device__ __forceinline__ uint64_t h32_mix_mad(uint64_t k) {
  const uint64_t a = mul64_const((uint32_t)k, (uint32_t)(k >> 32), kH32C1);
  const uint32_t al = (uint32_t)a, ah = (uint32_t)(a >> 32);
  const uint32_t rl = __builtin_amdgcn_alignbit(al, ah, 1);  // rotl 31 = rotr 33
  const uint32_t rh = __builtin_amdgcn_alignbit(ah, al, 1);
  return mul64_const(rl, rh, kH32C2);
}
#endif
KBZ_HD uint64_t h32_step(uint64_t h, uint64_t k) {
  h ^= k;
  h = rotl64(h, 27);
  return h * 5 + 0x52dce729;
}
KBZ_HD uint32_t h32_final(uint64_t h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdULL;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ULL;
  h ^= h >> 33;
  return (uint32_t)h;
}

// XXH64 pieces (xxhash.c:671-700).
KBZ_HD uint64_t xx_round(uint64_t acc, uint64_t in) {
  acc += in * kXP2;
  acc = rotl64(acc, 31);
  return acc * kXP1;
}
KBZ_HD uint64_t xx_merge(uint64_t acc, uint64_t v) {
  acc ^= xx_round(0, v);
  return acc * kXP1 + kXP4;
}
KBZ_HD uint64_t xx_avalanche(uint64_t h) {
  h ^= h >> 33;
  h *= kXP2;
  h ^= h >> 29;
  h *= kXP3;
  h ^= h >> 32;
  return h;
}

}  // namespace kbz
