/*
 * oracle/ref_harness.c -- TEST INFRASTRUCTURE ONLY (never shipped, never measured as the product).
 *
 * Exposes the reference's OWN bitmap code, compiled from the files under /root/reference,
 * through plain C entry points so the clean-room restatement (oracle/kbz_oracle.c) and the
 * committed golden fixtures can be pinned against it.  Built by oracle/Makefile into
 * oracle/_ref/libkbz_ref.so; nothing of the reference is copied into the repository: the
 * function bodies are pulled in at build time with #include / sed-extracted .inc files that
 * live only in a temporary build directory outside the repository (oracle/Makefile TMP).
 *
 * One translation unit per (source, MAP_SIZE) pair, selected with -D flags by the Makefile:
 *   REF_AFL   instrumentation/afl_instrumentation.c:116-121 (merge_bitmaps),
 *             :600-707 (has_new_bits, simplify_lookup, simplify_trace)   [x86_64 variants]
 *   REF_DR    instrumentation/dynamorio_instrumentation.c:79-339 (has_new_bits,
 *             has_new_bits_with_ignore, count_class_lookup, classify_counts, merge_bitmaps)
 *   REF_PICKER picker/main.c:240-262 (the ignore-bytes diff loop of the picker CLI, Win32 main()
 *             otherwise); its per-pair DEBUG_MSG (:260) is defined here to record the
 *             reference's own ignore_count / total_ignore_count instead of logging
 *   REF_HASH  afl_progs/hash.h:36-65 (hash32) and instrumentation/winafl_hash.h:80-112
 *             (hash32_with_ignore), instrumentation/xxhash.h + xxhash.c:855 (XXH64, v0.6.5)
 *   REF_IPT   instrumentation/linux_ipt_instrumentation.c:26-43 + :110-189 (the Intel-PT TNT /
 *             TIP streaming XXH64 feeders), over linux_ipt_instrumentation.h
 * MAP_SIZE is a compile-time constant in the reference (afl_progs/config.h:314-315); the
 * Makefile builds the 64 KiB and 1 MiB variants by defining it before the extracted code.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>

#ifndef REF_SUFFIX
#error "REF_SUFFIX must be defined (e.g. 64k)"
#endif
#define REF_CAT2(a, b) a##_##b
#define REF_CAT(a, b) REF_CAT2(a, b)
#define REF_NAME(n) REF_CAT(n, REF_SUFFIX)

#if defined(REF_AFL)
#include "types.h" /* /root/reference/afl_progs/types.h: u8.., likely/unlikely */
#define merge_bitmaps REF_NAME(afl_merge_bitmaps_impl) /* non-static in the reference: keep TUs apart */
#include "afl_merge.inc"
#include "afl_bitmap.inc"
uint8_t REF_NAME(ref_afl_has_new_bits)(uint8_t *virgin, uint8_t *trace) {
  return has_new_bits(virgin, trace);
}
void REF_NAME(ref_afl_simplify_trace)(uint8_t *trace) { simplify_trace((uint64_t *)trace); }
void REF_NAME(ref_afl_merge_bitmaps)(uint8_t *dest, const uint8_t *src) { merge_bitmaps(dest, src); }
size_t REF_NAME(ref_afl_map_size)(void) { return MAP_SIZE; }
/* The merger's fold (merger/merger.c:79-99 -> afl_merge afl_instrumentation.c:123-140) over n
 * in-memory states, each virgin_bits|virgin_tmout|virgin_crash (3*MAP_SIZE bytes), with the
 * reference's own merge_bitmaps; the JSON decode and per-state malloc of the CLI are left out
 * (their encoding lives in the absent killerbeez-utils).  acc: 3*MAP_SIZE, in/out.  The CPU
 * baseline of bench.py --workload merge ("kind": "reference"). */
void REF_NAME(ref_afl_merge_loop)(uint8_t *acc, const uint8_t *states, size_t n) {
  for (size_t s = 0; s < n; s++)
    for (int k = 0; k < 3; k++)
      merge_bitmaps(acc + (size_t)k * MAP_SIZE, states + (s * 3 + k) * (size_t)MAP_SIZE);
}
/* finish_fuzz_round's novelty step (afl_instrumentation.c:231-274) exec after exec: EXIT -> raw
 * trace vs virgin_bits; HANG / CRASH (outcome 1 / 2) -> simplify_trace, then virgin_tmout /
 * virgin_crash.  virgin: the 3 maps; scratch: MAP_SIZE bytes (the SHM trace_bits copy). */
void REF_NAME(ref_afl_triage_loop)(const uint8_t *traces, size_t n, size_t stride,
                                   const int8_t *outcome, uint8_t *virgin, uint8_t *hnb_out,
                                   uint8_t *scratch) {
  for (size_t j = 0; j < n; j++) {
    const int oc = outcome ? outcome[j] : 0;
    memcpy(scratch, traces + j * stride, MAP_SIZE);
    if (oc == 1 || oc == 2) simplify_trace((uint64_t *)scratch);
    hnb_out[j] = has_new_bits(virgin + (size_t)oc * MAP_SIZE, scratch);
  }
}

#elif defined(REF_DR)
#include "winafl_types.h" /* /root/reference/instrumentation/winafl_types.h */
#define merge_bitmaps REF_NAME(dr_merge_bitmaps_impl)
#include "dr_bitmap.inc"
uint8_t REF_NAME(ref_dr_has_new_bits)(uint8_t *trace, uint8_t *virgin) {
  return has_new_bits(trace, virgin);
}
uint8_t REF_NAME(ref_dr_has_new_bits_with_ignore)(uint8_t *trace, uint8_t *virgin, uint8_t *ignore) {
  return has_new_bits_with_ignore(trace, virgin, ignore);
}
void REF_NAME(ref_dr_classify_counts)(uint8_t *trace) { classify_counts((u64 *)trace); }
void REF_NAME(ref_dr_merge_bitmaps)(uint8_t *dest, const uint8_t *src) { merge_bitmaps(dest, src); }
uint8_t REF_NAME(ref_dr_count_class)(uint8_t c) { return count_class_lookup[c]; }

#include "winafl_hash.h" /* /root/reference/instrumentation/winafl_hash.h: hash32 (x86_64) */
/* The per-exec DynamoRIO novelty step as the reference runs it, exec after exec: the control
 * flow of has_new_coverage (dynamorio_instrumentation.c:1428-1468, without the Windows-only
 * debug dump) over the reference's own classify_counts / hash32 / has_new_bits.  This is the
 * CPU baseline bench.py times ("kind": "reference").  scratch: MAP_SIZE bytes (the SHM copy). */
void REF_NAME(ref_dr_triage_loop)(const uint8_t *traces, size_t n, size_t stride, uint8_t *virgin,
                                  uint32_t *last_hash, uint8_t *hnb_out, uint8_t *scratch) {
  uint32_t last = *last_hash;
  for (size_t j = 0; j < n; j++) {
    memcpy(scratch, traces + j * stride, MAP_SIZE);
    classify_counts((u64 *)scratch);
    uint32_t h = hash32(scratch, MAP_SIZE, 0xa5b35705u /* HASH_CONST winafl_config.h:330 */);
    if (h == last) {
      hnb_out[j] = 0;
      continue;
    }
    last = h;
    hnb_out[j] = has_new_bits(scratch, virgin);
  }
  *last_hash = last;
}

#elif defined(REF_PICKER)
/* One module's runs: module_infos[(file*num_iterations + iteration)*module_info_size], the
 * layout of picker/main.c:209.  pair_counts[file*(num_iterations-1) + iteration-1] receives the
 * reference's ignore_count of that pair; returns its final total_ignore_count. */
static unsigned *ref_pair_counts;
#define DEBUG_MSG(fmt, mod, file, prev_it, cur_it, ic, tic) \
  (ref_pair_counts ? (void)(ref_pair_counts[file_count * (num_iterations - 1) + iteration - 1] = (ic)) : (void)0)
int REF_NAME(ref_picker_ignore)(char *module_infos, int num_files, int num_iterations,
                               int module_info_size, char *ignore_bytes, unsigned *pair_counts) {
  int index = 0, file_count, iteration, i;
  ref_pair_counts = pair_counts;
#include "picker_diff.inc"
  ref_pair_counts = 0;
  return total_ignore_count;
}
#elif defined(REF_HASH)
#include "hash.h" /* /root/reference/afl_progs/hash.h (x86_64 hash32) */
uint32_t REF_NAME(ref_hash32)(const void *key, uint32_t len, uint32_t seed) {
  return hash32(key, len, seed);
}
#elif defined(REF_HASH_IGNORE)
#include "winafl_hash.h" /* /root/reference/instrumentation/winafl_hash.h */
uint32_t REF_NAME(ref_winafl_hash32)(const void *key, uint32_t len, uint32_t seed) {
  return hash32(key, len, seed);
}
uint32_t REF_NAME(ref_hash32_with_ignore)(const void *key, const void *ignore, uint32_t len,
                                          uint32_t seed) {
  return hash32_with_ignore(key, ignore, len, seed);
}
#elif defined(REF_XXH)
#include "xxhash.h" /* /root/reference/instrumentation/xxhash.h: XXH_INLINE_ALL pulls xxhash.c */
unsigned long long REF_NAME(ref_xxh64)(const void *input, size_t len, unsigned long long seed) {
  return XXH64(input, len, seed);
}
unsigned REF_NAME(ref_xxh_version)(void) { return XXH_versionNumber(); }
#elif defined(REF_IPT)
/* Intel-PT path hashing: the reference's own add_tnt_to_hash / add_tip_to_hash /
 * finish_tnt_hash (instrumentation/linux_ipt_instrumentation.c:110-189, its IPT_DEBUG and
 * BIT_TEST macros :26-43 with them), over its own state types (linux_ipt_instrumentation.h, which pulls in
 * forkserver_internal.h, uthash.h and xxhash.h from the reference tree).  WARNING_MSG is the
 * logging macro of the absent killerbeez-utils utils.h; its calls only report XXH_ERROR, which
 * XXH64_update never returns for a valid state. */
#define _GNU_SOURCE
#include <linux/perf_event.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/types.h>
#include "linux_ipt_instrumentation.h"
#define WARNING_MSG(...) ((void)0)
#include "ipt_hash.inc"
/* Events of one or more execs, as analyze_ipt (:212-425) feeds the hashes: kind 0 = TNT packet
 * bits (a = up to 8 bit bytes, little endian; b = num_bits), kind 1 = TIP address a (before the
 * ASLR adjustment), kind 2 = end of the exec -> keys_out[2e..2e+1] = {tip, tnt} digest, the
 * ipt_hashtable_key of :409-416.  Each exec starts from the reset of :238-243. */
size_t REF_NAME(ref_ipt_keys)(const uint64_t *ev, size_t n_ev, size_t nlib,
                              uint64_t *lib_starts, uint64_t *lib_ends, uint32_t *lib_hashes,
                              uint64_t target_start, uint64_t target_end, uint64_t *keys_out) {
  linux_ipt_state_t st;
  memset(&st, 0, sizeof(st));
  st.num_coverage_libraries = nlib;
  st.library_starts = lib_starts;
  st.library_ends = lib_ends;
  st.library_hashes = lib_hashes;
  st.target_start = target_start;
  st.target_end = target_end;
  st.ipt_hashes.tnt = XXH64_createState();
  st.ipt_hashes.tip = XXH64_createState();
  size_t execs = 0;
  int fresh = 1;
  for (size_t e = 0; e < n_ev; e++) {
    if (fresh) {  /* analyze_ipt :238-243 */
      st.ipt_hashes.tnt_bits = 0;
      st.ipt_hashes.num_bits = 0;
      st.ipt_hashes.total_num_bits = 0;
      XXH64_reset(st.ipt_hashes.tnt, 0);
      XXH64_reset(st.ipt_hashes.tip, 0);
      fresh = 0;
    }
    const uint64_t kind = ev[3 * e], a = ev[3 * e + 1], b = ev[3 * e + 2];
    if (kind == 0) {
      unsigned char bits[8];
      memcpy(bits, &a, 8);
      add_tnt_to_hash(&st.ipt_hashes, bits, (int)b);
    } else if (kind == 1) {
      add_tip_to_hash(&st, a);
    } else {  /* :409-416 */
      finish_tnt_hash(&st.ipt_hashes);
      keys_out[2 * execs] = XXH64_digest(st.ipt_hashes.tip);
      keys_out[2 * execs + 1] = XXH64_digest(st.ipt_hashes.tnt);
      execs++;
      fresh = 1;
    }
  }
  XXH64_freeState(st.ipt_hashes.tnt);
  XXH64_freeState(st.ipt_hashes.tip);
  return execs;
}
#else
#error "select one of REF_AFL / REF_DR / REF_PICKER / REF_HASH / REF_HASH_IGNORE / REF_XXH / REF_IPT"
#endif
