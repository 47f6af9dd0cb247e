/*
 * oracle/kbz_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Clean-room CPU restatement of the Killerbeez coverage-triage hot path.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only as the
 * checker / the timed CPU baseline; the product (libkbz_hip.so) never links or calls it.
 * Pinned against the reference's own code (oracle/_ref, built by oracle/Makefile) by
 * tests/test_oracle_pin.py and against the committed fixtures in tests/golden/.
 */
#ifndef KBZ_ORACLE_H
#define KBZ_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same numbering as include/kbz_triage.h (kept separate on purpose: the oracle must not
 * depend on product headers). */
enum { KBZO_MODE_AFL = 0, KBZO_MODE_DYNAMORIO = 1, KBZO_MODE_AFL_CLASSIFY = 2 };
enum { KBZO_FUZZ_NONE = 0, KBZO_FUZZ_HANG = 1, KBZO_FUZZ_CRASH = 2 };
enum { KBZO_WANT_H32 = 1, KBZO_WANT_X64 = 2 };

uint8_t kbzo_count_class(uint8_t c);
void kbzo_classify_counts(uint8_t *trace, size_t map_size);
void kbzo_simplify_trace(uint8_t *trace, size_t map_size);
uint8_t kbzo_has_new_bits(uint8_t *virgin, const uint8_t *trace, size_t map_size);
uint8_t kbzo_has_new_bits_with_ignore(const uint8_t *trace, uint8_t *virgin,
                                      const uint8_t *ignore, size_t map_size);
uint32_t kbzo_hash32(const void *key, uint32_t len, uint32_t seed);
uint32_t kbzo_hash32_with_ignore(const void *key, const void *ignore, uint32_t len,
                                 uint32_t seed);
uint64_t kbzo_xxh64(const void *input, size_t len, uint64_t seed);
void kbzo_merge_and(uint8_t *dest, const uint8_t *src, size_t n);

/* Sequential batch triage: the reference's per-exec semantics applied to traces[0..n) in
 * order.  traces is read-only (row j at traces + j*stride).  virgin = 3*map_size bytes
 * (bits | tmout | crash); DYNAMORIO mode uses only the first map.  ignore may be NULL.
 * last_hash (DYNAMORIO) is in/out.  Outputs may be NULL.  Returns 0, or -1 on bad args. */
int kbzo_triage_batch(int mode, const uint8_t *traces, size_t n, size_t stride,
                      size_t map_size, const int8_t *outcome, uint8_t *virgin,
                      const uint8_t *ignore, uint32_t *last_hash, int want,
                      uint8_t *hnb_out, uint32_t *h32_out, uint64_t *x64_out);

/* Same results as kbzo_triage_batch, computed with `threads` host threads by the exact
 * shard decomposition (per-shard OR aggregates, exclusive prefix, shard-local replay). */
int kbzo_triage_batch_mt(int mode, const uint8_t *traces, size_t n, size_t stride,
                         size_t map_size, const int8_t *outcome, uint8_t *virgin,
                         const uint8_t *ignore, uint32_t *last_hash, int want,
                         uint8_t *hnb_out, uint32_t *h32_out, uint64_t *x64_out, int threads);

/* bench.py's all-core baseline: wall seconds for `threads` threads each running an
 * `iters`-step register-only hash chain (t1 / tT x threads = cores actually granted). */
double kbzo_cpu_probe(int threads, long iters);
/* ... and a host memory-stream probe: `threads` threads read disjoint slices of buf (n bytes)
 * `passes` times; returns wall seconds. */
double kbzo_mem_probe(int threads, const uint8_t *buf, size_t n, int passes);

/* Merger fold (merger/merger.c:79-99): dest = AND of n states, each `state_bytes` long. */
void kbzo_merge_many(uint8_t *dest, const uint8_t *states, size_t n, size_t state_bytes);

/* Picker ignore-bytes diff (picker/main.c:240-262) over runs[files][iters][size]: ignore = 0x00
 * where consecutive iterations of a file differ, else 0xff; per-pair differing-byte counts;
 * returns the number of noisy bytes. */
size_t kbzo_picker_ignore(const uint8_t *runs, size_t files, size_t iters, size_t size,
                          uint8_t *ignore, uint32_t *pair_counts);
/* Intel-PT path keys {tip, tnt} per exec from an event list (see kbz_oracle.c). */
size_t kbzo_ipt_keys(const uint64_t *ev, size_t n_ev, size_t nlib, const uint64_t *lib_starts,
                     const uint64_t *lib_ends, const uint32_t *lib_hashes, uint64_t target_start,
                     uint64_t target_end, uint64_t *keys_out);

#ifdef __cplusplus
}
#endif
#endif
