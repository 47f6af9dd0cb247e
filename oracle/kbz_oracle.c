/*
 * oracle/kbz_oracle.c -- TEST INFRASTRUCTURE ONLY (see kbz_oracle.h).
 *
 * A clean-room restatement of the reference's CPU bitmap code.  Every function names the
 * reference lines whose behaviour it restates (paths relative to /root/reference).  The
 * word size of the reference loops (8-byte words on x86_64) is preserved where it is
 * observable (hash32, simplify's all-zero-word rule); elsewhere results are byte-exact.
 */
#include "kbz_oracle.h"

#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static inline uint64_t ld64(const uint8_t *p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return v;
}
static inline void st64(uint8_t *p, uint64_t v) { memcpy(p, &v, 8); }
static inline uint64_t rotl64(uint64_t x, unsigned r) { return (x << r) | (x >> (64 - r)); }

/* Hit-count buckets: instrumentation/dynamorio_instrumentation.c:246-255
 * (== afl_progs/afl-showmap.c:92-104 count_class_binary).
 * 0 ->0, 1 ->1, 2 ->2, 3 ->4, 4..7 ->8, 8..15 ->16, 16..31 ->32, 32..127 ->64, 128.. ->128 */
uint8_t kbzo_count_class(uint8_t c) {
  if (c < 3) return c;
  if (c == 3) return 4;
  if (c < 8) return 8;
  if (c < 16) return 16;
  if (c < 32) return 32;
  if (c < 128) return 64;
  return 128;
}

/* classify_counts: dynamorio_instrumentation.c:265-292.  All-zero 8-byte words are left
 * alone (bucket(0)==0 so that shortcut is not observable). */
void kbzo_classify_counts(uint8_t *trace, size_t map_size) {
  for (size_t i = 0; i < map_size; i++) trace[i] = kbzo_count_class(trace[i]);
}

/* simplify_trace (x86_64): afl_instrumentation.c:668-691.  Byte 0 -> 0x01, nonzero ->
 * 0x80; an all-zero 8-byte word becomes 0x0101010101010101, i.e. the same per-byte rule. */
void kbzo_simplify_trace(uint8_t *trace, size_t map_size) {
  for (size_t i = 0; i < map_size; i++) trace[i] = trace[i] ? 0x80 : 0x01;
}

/* has_new_bits: afl_instrumentation.c:600-662 (DynamoRIO twin dynamorio_instrumentation.c:
 * 95-174, identical results).  Per 8-byte word: if trace&virgin != 0 the result is at least 1,
 * and 2 when some byte has trace!=0 while virgin==0xff; then virgin &= ~trace. */
uint8_t kbzo_has_new_bits(uint8_t *virgin, const uint8_t *trace, size_t map_size) {
  uint8_t ret = 0;
  for (size_t w = 0; w < map_size; w += 8) {
    uint64_t cur = ld64(trace + w), vir = ld64(virgin + w);
    if (!(cur & vir)) continue;
    if (ret < 2) {
      uint8_t r = 1;
      for (int b = 0; b < 8; b++)
        if (trace[w + b] && virgin[w + b] == 0xff) r = 2;
      ret = r;
    }
    st64(virgin + w, vir & ~cur);
  }
  return ret;
}

/* has_new_bits_with_ignore: dynamorio_instrumentation.c:197-237.  Byte-wise, only bytes
 * whose ignore byte is ZERO are examined (note: the inverse of hash32_with_ignore's mask). */
uint8_t kbzo_has_new_bits_with_ignore(const uint8_t *trace, uint8_t *virgin,
                                      const uint8_t *ignore, size_t map_size) {
  uint8_t ret = 0;
  for (size_t i = 0; i < map_size; i++) {
    uint8_t t = trace[i], v = virgin[i];
    if (ignore[i] || !(t & v)) continue;
    if (ret < 2) ret = (t && v == 0xff) ? 2 : 1;
    virgin[i] = v & (uint8_t)~t;
  }
  return ret;
}

/* hash32 (x86_64): afl_progs/hash.h:36-65 == instrumentation/winafl_hash.h:49-78.
 * MurmurHash3-style chain over len/8 little-endian u64 words, fmix64, truncated to u32. */
#define KBZ_H32_C1 0x87c37b91114253d5ULL
#define KBZ_H32_C2 0x4cf5ad432745937fULL
static inline uint64_t h32_mix(uint64_t k) {
  k *= KBZ_H32_C1;
  k = rotl64(k, 31);
  return k * KBZ_H32_C2;
}
static inline uint64_t h32_step(uint64_t h, uint64_t k) {
  h ^= k;
  h = rotl64(h, 27);
  return h * 5 + 0x52dce729;
}
static inline uint32_t h32_final(uint64_t h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdULL;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ULL;
  h ^= h >> 33;
  return (uint32_t)h;
}
uint32_t kbzo_hash32(const void *key, uint32_t len, uint32_t seed) {
  const uint8_t *p = (const uint8_t *)key;
  uint64_t h = seed ^ len;
  for (uint32_t w = 0; w < len / 8; w++) h = h32_step(h, h32_mix(ld64(p + 8 * w)));
  return h32_final(h);
}
/* hash32_with_ignore (x86_64): winafl_hash.h:80-112 -- each word is ANDed with the ignore
 * word before mixing (so ignore byte 0x00 drops the byte, 0xff keeps it). */
uint32_t kbzo_hash32_with_ignore(const void *key, const void *ignore, uint32_t len,
                                 uint32_t seed) {
  const uint8_t *p = (const uint8_t *)key, *m = (const uint8_t *)ignore;
  uint64_t h = seed ^ len;
  for (uint32_t w = 0; w < len / 8; w++)
    h = h32_step(h, h32_mix(ld64(p + 8 * w) & ld64(m + 8 * w)));
  return h32_final(h);
}

/* XXH64 one-shot, xxHash v0.6.5 (instrumentation/xxhash.c:664-700 round/avalanche,
 * :760-853 endian_align + finalize, :855 entry point). */
#define P64_1 11400714785074694791ULL
#define P64_2 14029467366897019727ULL
#define P64_3 1609587929392839161ULL
#define P64_4 9650029242287828579ULL
#define P64_5 2870177450012600261ULL
static inline uint64_t xx_round(uint64_t acc, uint64_t in) {
  acc += in * P64_2;
  acc = rotl64(acc, 31);
  return acc * P64_1;
}
static inline uint64_t xx_merge(uint64_t acc, uint64_t v) {
  acc ^= xx_round(0, v);
  return acc * P64_1 + P64_4;
}
uint64_t kbzo_xxh64(const void *input, size_t len, uint64_t seed) {
  const uint8_t *p = (const uint8_t *)input, *end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t a = seed + P64_1 + P64_2, b = seed + P64_2, c = seed, d = seed - P64_1;
    const uint8_t *limit = end - 32;
    do {
      a = xx_round(a, ld64(p));
      b = xx_round(b, ld64(p + 8));
      c = xx_round(c, ld64(p + 16));
      d = xx_round(d, ld64(p + 24));
      p += 32;
    } while (p <= limit);
    h = rotl64(a, 1) + rotl64(b, 7) + rotl64(c, 12) + rotl64(d, 18);
    h = xx_merge(h, a);
    h = xx_merge(h, b);
    h = xx_merge(h, c);
    h = xx_merge(h, d);
  } else {
    h = seed + P64_5;
  }
  h += (uint64_t)len;
  while (p + 8 <= end) {
    h ^= xx_round(0, ld64(p));
    h = rotl64(h, 27) * P64_1 + P64_4;
    p += 8;
  }
  if (p + 4 <= end) {
    uint32_t v;
    memcpy(&v, p, 4);
    h ^= (uint64_t)v * P64_1;
    h = rotl64(h, 23) * P64_2 + P64_3;
    p += 4;
  }
  while (p < end) {
    h ^= (*p) * P64_5;
    h = rotl64(h, 11) * P64_1;
    p++;
  }
  h ^= h >> 33;
  h *= P64_2;
  h ^= h >> 29;
  h *= P64_3;
  h ^= h >> 32;
  return h;
}

/* merge_bitmaps: afl_instrumentation.c:116-121 (DR :334-339). */
void kbzo_merge_and(uint8_t *dest, const uint8_t *src, size_t n) {
  for (size_t i = 0; i < n; i++) dest[i] &= src[i];
}

/* ---- per-trace semantics -------------------------------------------------------------- */

/* Which virgin map (0 bits, 1 tmout, 2 crash) and which transform a trace gets.
 *   AFL           finish_fuzz_round afl_instrumentation.c:231-274: EXIT raw -> virgin_bits,
 *                 HANG simplify -> virgin_tmout, SIGNAL simplify -> virgin_crash.
 *   AFL_CLASSIFY  as AFL, but normal exits are bucketed first (classify_counts), the
 *                 afl-fuzz flavour the north_star names; simplify(classify(t)) == simplify(t).
 *   DYNAMORIO     has_new_coverage dynamorio_instrumentation.c:1428-1468: every outcome is
 *                 classified and checked against the single virgin_bits map. */
enum { XF_RAW = 0, XF_CLASSIFY = 1, XF_SIMPLIFY = 2 };
static int trace_xform(int mode, int outcome) {
  if (mode == KBZO_MODE_DYNAMORIO) return XF_CLASSIFY;
  if (outcome == KBZO_FUZZ_HANG || outcome == KBZO_FUZZ_CRASH) return XF_SIMPLIFY;
  return mode == KBZO_MODE_AFL_CLASSIFY ? XF_CLASSIFY : XF_RAW;
}
static int trace_map(int mode, int outcome) {
  if (mode == KBZO_MODE_DYNAMORIO) return 0;
  if (outcome == KBZO_FUZZ_HANG) return 1;
  if (outcome == KBZO_FUZZ_CRASH) return 2;
  return 0;
}
static void apply_xform(uint8_t *t, size_t m, int xf) {
  if (xf == XF_CLASSIFY) kbzo_classify_counts(t, m);
  else if (xf == XF_SIMPLIFY) kbzo_simplify_trace(t, m);
}

/* The same transforms, word at a time with a byte table (the multi-threaded path below; its
 * results are pinned to the byte loops above by tests/test_oracle_pin.py).  dst may be src. */
static uint8_t g_cls_lut[256];
static void init_lut(void) {
  for (int c = 0; c < 256; c++) g_cls_lut[c] = kbzo_count_class((uint8_t)c);
}
static void xform_words(uint8_t *dst, const uint8_t *src, size_t m, int xf) {
  for (size_t w = 0; w < m; w += 8) {
    uint64_t v = ld64(src + w);
    if (xf == XF_SIMPLIFY) {
      uint64_t r = 0;
      for (int b = 0; b < 8; b++) r |= (uint64_t)(((v >> (8 * b)) & 0xff) ? 0x80 : 0x01) << (8 * b);
      v = r;
    } else if (xf == XF_CLASSIFY && v) {
      uint64_t r = 0;
      for (int b = 0; b < 8; b++) r |= (uint64_t)g_cls_lut[(v >> (8 * b)) & 0xff] << (8 * b);
      v = r;
    }
    st64(dst + w, v);
  }
}
static void or_words(uint8_t *acc, const uint8_t *x, size_t m) {
  for (size_t w = 0; w < m; w += 8) st64(acc + w, ld64(acc + w) | ld64(x + w));
}

static int check_args(int mode, size_t stride, size_t map_size) {
  if (mode < 0 || mode > 2) return -1;
  if (map_size == 0 || (map_size & 7) || stride < map_size) return -1;
  if (map_size > 0xffffffffu) return -1;
  return 0;
}

int kbzo_triage_batch(int mode, const uint8_t *traces, size_t n, size_t stride,
                      size_t map_size, const int8_t *outcome, uint8_t *virgin,
                      const uint8_t *ignore, uint32_t *last_hash, int want,
                      uint8_t *hnb_out, uint32_t *h32_out, uint64_t *x64_out) {
  if (check_args(mode, stride, map_size)) return -1;
  if (mode != KBZO_MODE_DYNAMORIO) ignore = NULL; /* ignore_bytes is a DynamoRIO option */
  uint8_t *t = (uint8_t *)malloc(map_size);
  if (!t) return -1;
  uint32_t last = last_hash ? *last_hash : 0;
  for (size_t j = 0; j < n; j++) {
    int oc = outcome ? outcome[j] : KBZO_FUZZ_NONE;
    memcpy(t, traces + j * stride, map_size);
    apply_xform(t, map_size, trace_xform(mode, oc));
    uint8_t *vir = virgin + (size_t)trace_map(mode, oc) * map_size;
    uint32_t h = ignore ? kbzo_hash32_with_ignore(t, ignore, (uint32_t)map_size, 0xa5b35705u)
                        : kbzo_hash32(t, (uint32_t)map_size, 0xa5b35705u);
    uint8_t r;
    if (mode == KBZO_MODE_DYNAMORIO) {
      /* dynamorio_instrumentation.c:1450-1467: same hash as the last exec -> 0, virgin
       * untouched; otherwise remember the hash and run has_new_bits(_with_ignore). */
      if (h == last) {
        r = 0;
      } else {
        last = h;
        r = ignore ? kbzo_has_new_bits_with_ignore(t, vir, ignore, map_size)
                   : kbzo_has_new_bits(vir, t, map_size);
      }
    } else {
      r = kbzo_has_new_bits(vir, t, map_size);
    }
    if (hnb_out) hnb_out[j] = r;
    if (h32_out) h32_out[j] = h;
    if (x64_out && (want & KBZO_WANT_X64)) x64_out[j] = kbzo_xxh64(t, map_size, 0);
  }
  if (last_hash) *last_hash = last;
  free(t);
  return 0;
}

/* Multi-threaded exact variant (CPU baseline (ii)).  Decomposition, two reads
 * of every trace:
 *   A. parallel, per contiguous shard: transform + hash every trace (and XXH64), and OR the
 *      transformed traces into the shard's per-map aggregate -- except the shard's first trace,
 *      whose DYNAMORIO skip depends on the previous shard's last hash: it is kept aside;
 *   B. serial:   skip of every shard's first trace, its row OR'ed in unless skipped; exclusive
 *      prefix of the shard aggregates -> each shard's entry virgin V & ~prefix; V' = V & ~all;
 *   C. parallel: every shard replays the sequential rule from its entry virgin (second read).
 * Bytes hidden by ignore!=0 are never updated. */
int kbzo_triage_batch_mt(int mode, const uint8_t *traces, size_t n, size_t stride,
                         size_t map_size, const int8_t *outcome, uint8_t *virgin,
                         const uint8_t *ignore, uint32_t *last_hash, int want,
                         uint8_t *hnb_out, uint32_t *h32_out, uint64_t *x64_out, int threads) {
  if (check_args(mode, stride, map_size)) return -1;
  if (mode != KBZO_MODE_DYNAMORIO) ignore = NULL;
  if (threads < 1) threads = 1;
  if ((size_t)threads > n) threads = n ? (int)n : 1;
  const size_t m = map_size, nmaps = (mode == KBZO_MODE_DYNAMORIO) ? 1 : 3;
  const int dr = mode == KBZO_MODE_DYNAMORIO;
  uint32_t *h = (uint32_t *)malloc((n ? n : 1) * sizeof(uint32_t));
  uint8_t *skip = (uint8_t *)calloc(n ? n : 1, 1);
  uint8_t *aggr = (uint8_t *)calloc((size_t)threads * nmaps * m, 1);
  uint8_t *entry = (uint8_t *)malloc((size_t)threads * nmaps * m);
  uint8_t *first = (uint8_t *)malloc((size_t)threads * m);
  if (!h || !skip || !aggr || !entry || !first) {
    free(h); free(skip); free(aggr); free(entry); free(first);
    return -1;
  }
  const uint32_t seed = 0xa5b35705u;
  init_lut();
#pragma omp parallel num_threads(threads)
  {
#ifdef _OPENMP
    int s = omp_get_thread_num();
#else
    int s = 0;
#endif
    size_t lo = n * (size_t)s / threads, hi = n * (size_t)(s + 1) / threads;
    uint8_t *t = (uint8_t *)malloc(m);
    for (size_t j = lo; j < hi; j++) {
      int oc = outcome ? outcome[j] : KBZO_FUZZ_NONE;
      uint8_t *x = (j == lo) ? first + (size_t)s * m : t;
      xform_words(x, traces + j * stride, m, trace_xform(mode, oc));
      h[j] = ignore ? kbzo_hash32_with_ignore(x, ignore, (uint32_t)m, seed)
                    : kbzo_hash32(x, (uint32_t)m, seed);
      if (x64_out && (want & KBZO_WANT_X64)) x64_out[j] = kbzo_xxh64(x, m, 0);
      if (j == lo) continue;
      if (dr && (skip[j] = h[j] == h[j - 1])) continue;
      or_words(aggr + ((size_t)s * nmaps + trace_map(mode, oc)) * m, x, m);
    }
    free(t);
  }
  uint32_t last = last_hash ? *last_hash : 0;
  for (int s = 0; s < threads; s++) {
    const size_t lo = n * (size_t)s / threads, hi = n * (size_t)(s + 1) / threads;
    if (lo == hi) continue;
    if (dr) skip[lo] = h[lo] == (lo ? h[lo - 1] : last);
    if (skip[lo]) continue;
    int oc = outcome ? outcome[lo] : KBZO_FUZZ_NONE;
    uint8_t *a = aggr + ((size_t)s * nmaps + trace_map(mode, oc)) * m;
    const uint8_t *x = first + (size_t)s * m;
    for (size_t i = 0; i < m; i++) a[i] |= x[i];
  }
  if (dr && n) last = h[n - 1];
  for (size_t k = 0; k < nmaps; k++) {
    uint8_t *v = virgin + k * m;
    for (size_t i = 0; i < m; i++) {
      uint8_t pre = 0;
      for (int s = 0; s < threads; s++) {
        entry[((size_t)s * nmaps + k) * m + i] = v[i] & (uint8_t)~pre;
        pre |= aggr[((size_t)s * nmaps + k) * m + i];
      }
      if (!ignore || !ignore[i]) v[i] &= (uint8_t)~pre;
    }
  }
#pragma omp parallel num_threads(threads)
  {
#ifdef _OPENMP
    int s = omp_get_thread_num();
#else
    int s = 0;
#endif
    size_t lo = n * (size_t)s / threads, hi = n * (size_t)(s + 1) / threads;
    uint8_t *t = (uint8_t *)malloc(m);
    for (size_t j = lo; j < hi; j++) {
      int oc = outcome ? outcome[j] : KBZO_FUZZ_NONE;
      uint8_t r = 0;
      if (!skip[j]) {
        xform_words(t, traces + j * stride, m, trace_xform(mode, oc));
        uint8_t *v = entry + ((size_t)s * nmaps + trace_map(mode, oc)) * m;
        r = ignore ? kbzo_has_new_bits_with_ignore(t, v, ignore, m) : kbzo_has_new_bits(v, t, m);
      }
      if (hnb_out) hnb_out[j] = r;
      if (h32_out) h32_out[j] = h[j];
    }
    free(t);
  }
  if (last_hash) *last_hash = last;
  free(h); free(skip); free(aggr); free(entry); free(first);
  return 0;
}

void kbzo_merge_many(uint8_t *dest, const uint8_t *states, size_t n, size_t state_bytes) {
  memset(dest, 0xff, state_bytes);
  for (size_t s = 0; s < n; s++) kbzo_merge_and(dest, states + s * state_bytes, state_bytes);
}

/* Picker ignore-bytes diff (picker/main.c:240-262): for one module, runs[f][it][size] holds
 * the instrumentation data of iteration `it` of file `f`.  A byte is noisy (ignore 0x00) if
 * any two consecutive iterations of the same file differ there; every other byte stays 0xff.
 * pair_counts[f*(iters-1) + it-1] = bytes differing between iterations it-1 and it (the
 * reference's per-pair ignore_count, :246-258); returns the number of noisy bytes (its
 * total_ignore_count, :254-255). */
size_t kbzo_picker_ignore(const uint8_t *runs, size_t files, size_t iters, size_t size,
                          uint8_t *ignore, uint32_t *pair_counts) {
  size_t total = 0;
  memset(ignore, 0xff, size);
  for (size_t f = 0; f < files; f++) {
    for (size_t it = 1; it < iters; it++) {
      const uint8_t *prev = runs + (f * iters + it - 1) * size, *cur = prev + size;
      uint32_t cnt = 0;
      for (size_t i = 0; i < size; i++) {
        if (prev[i] == cur[i]) continue;
        total += ignore[i] != 0;
        ignore[i] = 0;
        cnt++;
      }
      if (pair_counts) pair_counts[f * (iters - 1) + it - 1] = cnt;
    }
  }
  return total;
}

/* Intel-PT path keys (linux_ipt_instrumentation.c:110-189 feeders, :238-243 reset, :409-416
 * digests), restated as two 8-byte word streams per exec hashed one-shot (XXH64's streaming and
 * one-shot forms agree on the concatenated input):
 *   TNT: packet bits are packed the reference's way -- bit i of a packet contributes
 *        (byte & (1 << i%8)) << k, k = bits already packed -- and every 8 packed bits (the
 *        `num_bits == sizeof(tnt_bits)` flush, :148) emit the word; at the end the partial word
 *        (if any) and the total bit count;
 *   TIP: every TIP address, ASLR-adjusted (:169-185): inside coverage library i ->
 *        (tip - start_i) | hash_i << 32; else, without libraries, inside the target ->
 *        tip - target_start; else unchanged.
 * Events as ref_ipt_keys: (0, bit bytes, num_bits) TNT, (1, tip, -) TIP, (2, -, -) end of exec.
 * keys_out[2e] = tip digest, [2e+1] = tnt digest.  Returns the number of execs. */
size_t kbzo_ipt_keys(const uint64_t *ev, size_t n_ev, size_t nlib, const uint64_t *lib_starts,
                     const uint64_t *lib_ends, const uint32_t *lib_hashes, uint64_t target_start,
                     uint64_t target_end, uint64_t *keys_out) {
  uint64_t *tnt = (uint64_t *)malloc((n_ev * 8 + 2) * sizeof(uint64_t));
  uint64_t *tip = (uint64_t *)malloc((n_ev + 1) * sizeof(uint64_t));
  size_t nt = 0, np = 0, execs = 0;
  uint64_t bits = 0, nb = 0, total = 0;
  for (size_t e = 0; e < n_ev; e++) {
    const uint64_t kind = ev[3 * e], a = ev[3 * e + 1], b = ev[3 * e + 2];
    if (kind == 0) {
      for (uint64_t i = 0; i < b; i++) {
        const unsigned byte = (unsigned)((a >> (8 * (i / 8))) & 0xff);
        bits |= (uint64_t)((byte & (1u << (i % 8))) << nb);
        if (++nb == 8) {
          tnt[nt++] = bits;
          bits = nb = 0;
        }
      }
      total += b;
    } else if (kind == 1) {
      uint64_t adj = a;
      if (nlib) {
        for (size_t i = 0; i < nlib; i++)
          if (lib_starts[i] <= a && a < lib_ends[i]) {
            adj = (a - lib_starts[i]) | ((uint64_t)lib_hashes[i] << 32);
            break;
          }
      } else if (target_start <= a && a < target_end) {
        adj = a - target_start;
      }
      tip[np++] = adj;
    } else {
      if (nb) tnt[nt++] = bits;
      tnt[nt++] = total;
      keys_out[2 * execs] = kbzo_xxh64(tip, np * 8, 0);
      keys_out[2 * execs + 1] = kbzo_xxh64(tnt, nt * 8, 0);
      execs++;
      nt = np = 0;
      bits = nb = total = 0;
    }
  }
  free(tnt);
  free(tip);
  return execs;
}

/* CPU parallelism probe for bench.py's all-core baseline (not a restatement of anything): every
 * one of `threads` OpenMP threads runs the same dependent hash32-step chain of `iters` steps
 * (registers only, no memory traffic).  Returns the wall time in seconds; with T real cores the
 * time equals the 1-thread time, so threads * t1 / tT is the number of cores actually granted. */
double kbzo_cpu_probe(int threads, long iters) {
  if (threads < 1) threads = 1;
  volatile uint64_t sink = 0;
  struct timespec a, b;
  clock_gettime(CLOCK_MONOTONIC, &a);
#pragma omp parallel num_threads(threads)
  {
    uint64_t h = 0x9e3779b97f4a7c15ull ^ (uint64_t)(size_t)&h;
    for (long i = 0; i < iters; i++) h = h32_step(h, (uint64_t)i);
    sink += h;
  }
  clock_gettime(CLOCK_MONOTONIC, &b);
  (void)sink;
  return (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
}

/* Host memory-stream probe for the same baseline: `threads` threads each read their own slice of
 * `buf` (n bytes, 8-byte words) `passes` times.  Returns wall seconds; bytes read = passes * n. */
double kbzo_mem_probe(int threads, const uint8_t *buf, size_t n, int passes) {
  if (threads < 1) threads = 1;
  volatile uint64_t sink = 0;
  struct timespec a, b;
  clock_gettime(CLOCK_MONOTONIC, &a);
#pragma omp parallel num_threads(threads)
  {
#ifdef _OPENMP
    const int t = omp_get_thread_num();
#else
    const int t = 0;
#endif
    const size_t words = n / 8, lo = words * (size_t)t / threads, hi = words * (size_t)(t + 1) / threads;
    uint64_t acc = 0;
    for (int p = 0; p < passes; p++)
      for (size_t i = lo; i < hi; i++) acc += ld64(buf + 8 * i);
    sink += acc;
  }
  clock_gettime(CLOCK_MONOTONIC, &b);
  (void)sink;
  return (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
}
