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

// count_class bucket of every byte (dynamorio_instrumentation.c:246-255), branch-free:
// with hb = highest set bit of the byte, bucket = hb, doubled when 3 <= c <= 63
// (hb in {4,8,16,32}, or c == 3 where hb == 2).
KBZ_HD uint32_t classify4(uint32_t x) {
  uint32_t s = x | ((x >> 1) & 0x7F7F7F7Fu);
  s |= (s >> 2) & 0x3F3F3F3Fu;
  s |= (s >> 4) & 0x0F0F0F0Fu;
  const uint32_t hb = s & ~((s >> 1) & 0x7F7F7F7Fu);
  const uint32_t e3 = x & (x >> 1) & (hb >> 1) & 0x01010101u;
  return hb + (hb & 0x3C3C3C3Cu) + (e3 << 1);
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

// 0xff in every byte of x that is nonzero.
KBZ_HD uint64_t nonzero_bytes8(uint64_t x) {
  const uint64_t nz = (((x & 0x7F7F7F7F7F7F7F7FULL) + 0x7F7F7F7F7F7F7F7FULL) | x) &
                      0x8080808080808080ULL;
  return (nz >> 7) * 0xFFull;
}

// hash32 pieces (afl_progs/hash.h:36-65): per-word mix, chain step, finalizer.
KBZ_HD uint64_t h32_mix(uint64_t k) {
  k *= kH32C1;
  k = rotl64(k, 31);
  return k * kH32C2;
}
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
