/*
 * include/kbz_plugin.h -- libkbz_plugin.so: Killerbeez instrumentation plugins whose bitmap
 * post-processing runs on the MI355X through libkbz_hip.so (include/kbz_triage.h).
 *
 * kbz_instrumentation_t has the member order of the reference's `struct instrumentation`
 * (instrumentation/instrumentation.h:40-62, Linux layout: enable takes a pid_t *), so a
 * reference caller can copy it into its own instrumentation_t, followed by two OPTIONAL members
 * appended after is_process_done: triage_batch and merge_many.  The
 * reference's instrumentation_factory memsets the struct before filling it
 * (instrumentation/instrumentation_factory.c:27-28), so callers that do not know the appended
 * members never read them.
 *
 * Two plugins, named as instrumentation_factory would bind them:
 *   "afl_gpu"       afl_instrumentation.c semantics per exec: EXIT -> has_new_bits(virgin_bits,
 *                   raw trace); HANG -> simplify_trace, has_new_bits(virgin_tmout); CRASH ->
 *                   simplify_trace, has_new_bits(virgin_crash) (finish_fuzz_round :231-274);
 *                   is_new_path folds 2 into 1 (afl_is_new_path :189-198).
 *   "dynamorio_gpu" dynamorio_instrumentation.c has_new_coverage semantics (:1428-1468):
 *                   classify_counts, hash32 (or hash32_with_ignore), skip when equal to the
 *                   previous exec's hash, has_new_bits (or _with_ignore) vs virgin_bits.
 *
 * Process control (fork server, SysV SHM, target launch) stays with the host plugin: these are
 * the bitmap half of the reference plugins.  The host hands each exec's RAW trace map to
 * kbz_*_gpu_record (the call that replaces has_new_bits in finish_fuzz_round; the GPU applies
 * simplify/classify itself), so enable() returns -1 and is_process_done() returns -1 here
 * (INTEGRATION.md shows the patch to afl_instrumentation.c).  Execs recorded between two result
 * queries are triaged as ONE ordered batch on the GPU; results are bit-exact with the per-exec
 * loop, since novelty depends only on the order, which the batch keeps.
 *
 * Options (create's JSON string; every key optional):
 *   {"map_size": 65536, "max_batch": 4096}; dynamorio_gpu also "ignore_bytes_file": "<path>",
 *   "per_module_coverage": 0/1, "coverage_modules": [names], "ignore_bytes_dir": "<dir>",
 *   "dump_map_dir": "<dir>" (dynamorio_instrumentation.c:1040-1051); both plugins "devices":
 *   "0,1,..." (GPU ordinals, repeats allowed) and "shard_min": 1024 -- windows / triage_batch
 *   chunks of at least shard_min execs are sharded over those GPUs (kbz_triage_batch_devices),
 *   smaller ones stay on the plugin's own GPU context (not with per_module_coverage)
 * State (get_state / set_state / create's state argument), keys as the reference's
 * afl_get_state :62-79 and dynamorio_get_state :1239-1281:
 *   afl_gpu       {"map_size": M, "virgin_bits": "<hex>", "virgin_tmout": "<hex>",
 *                  "virgin_crash": "<hex>"}
 *   dynamorio_gpu {"map_size": M, "virgin_bits": "<hex>", "last_shm_hash": H}
 * The reference encodes the maps with ADD_MEM/GET_MEM from the external killerbeez-utils
 * (jansson_helper.h, absent from the reference tree), so the blob ENCODING is parity-unpinned;
 * the map CONTENTS are exactly what the reference would store.
 *
 * Errors as in the reference: NULL from create/merge/merge_many/get_state, non-zero from
 * set_state, -1 from is_new_path / get_fuzz_result / record / result / triage_batch;
 * kbz_plugin_last_error() says why.  There is no CPU path: without a usable GPU every triage
 * and merge call fails.
 */
#ifndef KBZ_PLUGIN_H
#define KBZ_PLUGIN_H

#include <stddef.h>
#include <stdint.h>
#include <sys/types.h>

#ifdef __cplusplus
extern "C" {
#endif

/* FUZZ_* results of get_fuzz_result.  Their numeric values live in the external
 * killerbeez-utils; reference callers only rely on < 0 = error (fuzzer/main.c:376-383). */
#define KBZ_PLUGIN_FUZZ_NONE 0
#define KBZ_PLUGIN_FUZZ_HANG 1
#define KBZ_PLUGIN_FUZZ_CRASH 2
#define KBZ_PLUGIN_FUZZ_ERROR (-1)

/* instrumentation/instrumentation.h:17-37 (edge list of the optional get_edges).  The
 * reference selects 64-bit fields with MSVC's _M_X64 only, so its Linux build uses 32-bit ones;
 * this is that layout (tests/native/abi_layout.c checks it against the reference header). */
typedef struct kbz_instrumentation_edge {
  uint32_t from, to;
} kbz_instrumentation_edge_t;
typedef struct kbz_instrumentation_edges {
  uint32_t num_edges;
  kbz_instrumentation_edge_t edges[1];
} kbz_instrumentation_edges_t;

typedef struct kbz_instrumentation {
  void *(*create)(char *options, char *state);
  void (*cleanup)(void *instrumentation_state);
  void *(*merge)(void *instrumentation_state, void *other_instrumentation_state);
  char *(*get_state)(void *instrumentation_state);
  void (*free_state)(char *state);
  int (*set_state)(void *instrumentation_state, char *state);
  int (*enable)(void *instrumentation_state, pid_t *process, char *cmd_line, char *input,
                size_t input_length);
  int (*is_new_path)(void *instrumentation_state);
  int (*get_fuzz_result)(void *instrumentation_state);
  /* optional (instrumentation.h:58-61): NULL in afl_gpu (as in the afl plugin); dynamorio_gpu
   * binds both, as instrumentation_factory.c:53-54 does for the dynamorio plugin */
  int (*get_module_info)(void *instrumentation_state, int index, int *is_new, char **module_name,
                         char **info, int *size);
  kbz_instrumentation_edges_t *(*get_edges)(void *instrumentation_state, int index);
  int (*is_process_done)(void *instrumentation_state);
  /* appended: one ordered batch of n execs (host memory, row j at traces + j*stride, map_size
   * raw bytes each) with per-exec outcomes (FUZZ_* values; NULL = all FUZZ_NONE).  Writes the
   * per-exec has_new_bits result (0/1/2), hash32 and XXH64 of the transformed map (any output
   * may be NULL).  Execs queued with record() are triaged first. */
  int (*triage_batch)(void *instrumentation_state, const uint8_t *traces, size_t n, size_t stride,
                      const int8_t *outcome, uint8_t *hnb_out, uint32_t *h32_out,
                      uint64_t *x64_out);
  /* appended: AND-merge of n states into a new one (merger/merger.c:79-99 in one GPU call). */
  void *(*merge_many)(void **instrumentation_states, size_t n);
} kbz_instrumentation_t;

/* instrumentation_factory (instrumentation/instrumentation_factory.c:25-104) for the GPU
 * plugins: "afl_gpu" or "dynamorio_gpu".  Returns a malloc'd vtable (free() it), NULL for an
 * unknown name. */
kbz_instrumentation_t *kbz_instrumentation_factory(const char *name);
const char *kbz_plugin_last_error(void);

/* ---- afl_gpu ------------------------------------------------------------------------------ */
void *kbz_afl_gpu_create(char *options, char *state);
void kbz_afl_gpu_cleanup(void *state);
void *kbz_afl_gpu_merge(void *state, void *other);
char *kbz_afl_gpu_get_state(void *state);
void kbz_afl_gpu_free_state(char *state);
int kbz_afl_gpu_set_state(void *state, char *json);
int kbz_afl_gpu_enable(void *state, pid_t *process, char *cmd_line, char *input,
                       size_t input_length);
int kbz_afl_gpu_is_new_path(void *state);
int kbz_afl_gpu_get_fuzz_result(void *state);
int kbz_afl_gpu_is_process_done(void *state);
int kbz_afl_gpu_triage_batch(void *state, const uint8_t *traces, size_t n, size_t stride,
                             const int8_t *outcome, uint8_t *hnb_out, uint32_t *h32_out,
                             uint64_t *x64_out);
void *kbz_afl_gpu_merge_many(void **states, size_t n);
void *kbz_afl_gpu_merge_files(char *options, const char *const *paths, size_t n);
int kbz_afl_gpu_help(char **help_str);
/* Deferred per-exec path.  record: queue one exec's RAW trace map (map_size bytes, copied)
 * with its FUZZ_* result; returns the exec's ticket (>= 0) or -1.  The queue is triaged as one
 * batch when it reaches max_batch or at the next result query.  result: the has_new_bits value
 * (0/1/2) of a recorded exec, flushing the queue if needed; -1 if the ticket is older than the
 * last flushed window or on failure.  flush: triage everything queued now. */
long kbz_afl_gpu_record(void *state, const uint8_t *trace_bits, int fuzz_result);
int kbz_afl_gpu_result(void *state, long ticket);
int kbz_afl_gpu_flush(void *state);

/* ---- dynamorio_gpu ------------------------------------------------------------------------ */
void *kbz_dynamorio_gpu_create(char *options, char *state);
void kbz_dynamorio_gpu_cleanup(void *state);
void *kbz_dynamorio_gpu_merge(void *state, void *other);
char *kbz_dynamorio_gpu_get_state(void *state);
void kbz_dynamorio_gpu_free_state(char *state);
int kbz_dynamorio_gpu_set_state(void *state, char *json);
int kbz_dynamorio_gpu_enable(void *state, pid_t *process, char *cmd_line, char *input,
                             size_t input_length);
int kbz_dynamorio_gpu_is_new_path(void *state);
int kbz_dynamorio_gpu_get_fuzz_result(void *state);
int kbz_dynamorio_gpu_is_process_done(void *state);
int kbz_dynamorio_gpu_triage_batch(void *state, const uint8_t *traces, size_t n, size_t stride,
                                   const int8_t *outcome, uint8_t *hnb_out, uint32_t *h32_out,
                                   uint64_t *x64_out);
void *kbz_dynamorio_gpu_merge_many(void **states, size_t n);
void *kbz_dynamorio_gpu_merge_files(char *options, const char *const *paths, size_t n);
int kbz_dynamorio_gpu_help(char **help_str);
long kbz_dynamorio_gpu_record(void *state, const uint8_t *trace_bits, int fuzz_result);
int kbz_dynamorio_gpu_result(void *state, long ticket);
int kbz_dynamorio_gpu_flush(void *state);
/* dynamorio_get_module_info (dynamorio_instrumentation.c:1541-1573): module `index`'s
 * last_path_was_new for the last exec (is_new), its name, its trace map as has_new_coverage
 * left it (classified, map_size bytes, valid until the next exec) and map_size; asking for is_new
 * or info triages the queued execs first.  0 = found, 1 = no such module, -1 = error / no exec
 * yet.  Without per_module_coverage: the coverage_modules names, is_new 0, info NULL (as the
 * reference). */
int kbz_dynamorio_gpu_get_module_info(void *state, int index, int *is_new, char **module_name,
                                      char **info, int *size);
/* dynamorio_get_edges (:1582-1606): NULL (edge lists are not offered; the reference returns NULL
 * unless its "edges" option asked for them ahead of time). */
kbz_instrumentation_edges_t *kbz_dynamorio_gpu_get_edges(void *state, int index);

#ifdef __cplusplus
}
#endif
#endif /* KBZ_PLUGIN_H */
