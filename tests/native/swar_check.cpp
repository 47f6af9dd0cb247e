// Host-side exhaustive check of the SWAR byte transforms in killerbeez_amd/csrc/kbz_device.h
// against the byte lookup tables they replace (count_class_lookup,
// dynamorio_instrumentation.c:246-255; simplify_lookup, afl_instrumentation.c:668-671).
// Built and run by tests/test_swar.py.  Prints "OK" on success.
#include <cstdio>
#include <cstdint>
#include <random>
#include "kbz_device.h"

static uint8_t cls(uint8_t c) {
  if (c < 3) return c;
  if (c == 3) return 4;
  if (c < 8) return 8;
  if (c < 16) return 16;
  if (c < 32) return 32;
  if (c < 128) return 64;
  return 128;
}
static uint32_t ref4(uint32_t x, bool simp) {
  uint32_t r = 0;
  for (int b = 0; b < 4; b++) {
    uint8_t c = (x >> (8 * b)) & 0xff;
    uint8_t o = simp ? (c ? 0x80 : 0x01) : cls(c);
    r |= (uint32_t)o << (8 * b);
  }
  return r;
}
int main() {
  long bad = 0;
  // every pair of adjacent bytes in every position (covers cross-byte shifts/carries)
  for (int pos = 0; pos < 3; pos++)
    for (uint32_t v = 0; v < 65536; v++) {
      uint32_t x = v << (8 * pos);
      if (kbz::classify4(x) != ref4(x, false)) bad++;
      if (kbz::simplify4(x) != ref4(x, true)) bad++;
      uint32_t y = x | (0xA5u << ((8 * pos + 16) & 31));
      if (kbz::classify4(y) != ref4(y, false)) bad++;
    }
  std::mt19937_64 rng(42);
  for (int i = 0; i < 4000000; i++) {
    uint64_t x = rng();
    if (kbz::classify8(x) != ((uint64_t)ref4((uint32_t)x, false) | ((uint64_t)ref4(x >> 32, false) << 32))) bad++;
    if (kbz::simplify8(x) != ((uint64_t)ref4((uint32_t)x, true) | ((uint64_t)ref4(x >> 32, true) << 32))) bad++;
    uint64_t nz = 0;
    for (int b = 0; b < 8; b++) if ((x >> (8 * b)) & 0xff) nz |= 0xffull << (8 * b);
    if (kbz::nonzero_bytes8(x) != nz) bad++;
    uint64_t z = x & 0x00ff00ff00ff00ffull;
    nz = 0;
    for (int b = 0; b < 8; b++) if ((z >> (8 * b)) & 0xff) nz |= 0xffull << (8 * b);
    if (kbz::nonzero_bytes8(z) != nz) bad++;
  }
  if (bad) { printf("BAD %ld\n", bad); return 1; }
  printf("OK\n");
  return 0;
}
