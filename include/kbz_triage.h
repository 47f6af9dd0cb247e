/*
 * include/kbz_triage.h -- C ABI of libkbz_hip.so, the MI355X (gfx950) coverage-triage backend.
 *
 * Plain C types only (no torch, no HIP types): device pointers are `void *`/typed pointers to
 * device memory, streams are `void *` holding a hipStream_t (NULL = the null stream).
 *
 * What each entry point replaces in the reference (paths relative to ThePatrickStar/killerbeez):
 *
 *   kbz_triage_batch_device / kbz_triage_batch_host
 *       the per-exec novelty step, done for a whole ordered batch of traces:
 *         instrumentation/afl_instrumentation.c:231-274   finish_fuzz_round (raw/simplify +
 *                                                          has_new_bits vs 3 virgin maps)
 *         instrumentation/afl_instrumentation.c:189-198   afl_is_new_path   (hnb != 0)
 *         instrumentation/dynamorio_instrumentation.c:1428-1468 has_new_coverage (classify,
 *                                                          hash32[_with_ignore], last-hash skip,
 *                                                          has_new_bits[_with_ignore])
 *       Results are bit-exact with running those functions once per trace, in batch order.
 *   kbz_get_virgin / kbz_set_virgin
 *       the virgin-map part of afl_get_state / afl_set_state (afl_instrumentation.c:62-109)
 *   kbz_merge_and_device / kbz_merge_and_host
 *       the merger fold merger/merger.c:79-99 -> afl_merge afl_instrumentation.c:123-140
 *       (merge_bitmaps :116-121 == dynamorio_instrumentation.c:334-339)
 *   kbz_triage_modules_device
 *       has_new_coverage_per_module (dynamorio_instrumentation.c:1477-1493): per-module maps
 *   kbz_picker_ignore_device
 *       the picker CLI's ignore-bytes diff across repeated runs (picker/main.c:240-262)
 *   kbz_transform_rows_device / _host
 *       classify_counts (dynamorio_instrumentation.c:265-292) / simplify_trace
 *       (afl_instrumentation.c:674-706) over a batch of maps (get_module_info's info, dump_map_dir)
 *   kbz_hash32_device / kbz_xxh64_device
 *       afl_progs/hash.h:36-65 (hash32) and instrumentation/xxhash.c:855 (XXH64, v0.6.5)
 *       over every trace of a batch (crash/hang dedup keys).
 *
 * Conventions: every function returns 0 on success and -1 on failure (device errors are
 * mapped to -1; kbz_last_error() gives a message).  Buffers are caller-owned.  One context
 * per host thread; a context is bound to the device that was current at kbz_ctx_create.
 * Nothing here blocks the host unless its name ends in _host or it copies to host memory.
 */
#ifndef KBZ_TRIAGE_H
#define KBZ_TRIAGE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KBZ_ABI_VERSION 3

/* Triage semantics (which reference code path a batch reproduces). */
enum kbz_mode {
  KBZ_MODE_AFL = 0,          /* afl_instrumentation.c finish_fuzz_round: EXIT raw -> virgin_bits,
                                HANG simplify -> virgin_tmout, CRASH simplify -> virgin_crash,
                                result 0/1/2 (last_is_new_path) */
  KBZ_MODE_DYNAMORIO = 1,    /* dynamorio has_new_coverage: classify_counts, hash32 (or
                                hash32_with_ignore), skip if hash == last hash, has_new_bits
                                (or _with_ignore) vs virgin_bits; result 0/1/2, 0 when skipped */
  KBZ_MODE_AFL_CLASSIFY = 2  /* afl-fuzz flavour (north_star): EXIT classify_counts -> virgin_bits,
                                HANG/CRASH simplify -> virgin_tmout/virgin_crash */
};

/* Per-trace outcome, the FUZZ_* results of get_fuzz_result.  The numeric FUZZ_* values live
 * in the external killerbeez-utils (not in the reference tree); these are ours. */
enum kbz_outcome { KBZ_FUZZ_NONE = 0, KBZ_FUZZ_HANG = 1, KBZ_FUZZ_CRASH = 2 };

/* Which per-trace outputs to produce (hnb is always produced). */
enum kbz_want { KBZ_WANT_H32 = 1, KBZ_WANT_X64 = 2 };

typedef struct kbz_ctx kbz_ctx_t;

/* ---- context ------------------------------------------------------------------------------ */
/* map_size: bytes per trace map, a multiple of 256 (64 KiB = AFL MAP_SIZE, config.h:314-315;
 * 1 MiB = DynamoRIO/winafl-scale).  max_batch: largest n passed to a triage call.
 * Virgin maps start all-0xff (setup_shm, afl_instrumentation.c:555-559), last hash 0. */
kbz_ctx_t *kbz_ctx_create(size_t map_size, int mode, size_t max_batch);
void kbz_ctx_destroy(kbz_ctx_t *ctx);
const char *kbz_last_error(void);
int kbz_abi_version(void);
/* The preprocessor flags this library was built with: "" for the product library that
 * killerbeez_amd/build.py builds; experiment builds (build_variants/<name>/, timing A/Bs and
 * diagnostics, never for results) report their -D flags. */
const char *kbz_build_flags(void);

/* ignore_bytes for KBZ_MODE_DYNAMORIO (dynamorio_instrumentation.c:788-814): map_size bytes of
 * host memory, or NULL to clear.  Same conventions as the reference: hash32_with_ignore ANDs
 * each trace word with the ignore word, has_new_bits_with_ignore only looks at bytes whose
 * ignore byte is 0. */
int kbz_set_ignore(kbz_ctx_t *ctx, const uint8_t *host_ignore);

/* The three virgin maps, host memory, 3*map_size bytes: virgin_bits | virgin_tmout |
 * virgin_crash.  DYNAMORIO mode uses only virgin_bits.  Synchronous. */
int kbz_get_virgin(kbz_ctx_t *ctx, uint8_t *host_out);
int kbz_set_virgin(kbz_ctx_t *ctx, const uint8_t *host_in);
/* Stream-ordered reset of the three virgin maps to all-0xff, as a fresh afl_state_t or the
 * DynamoRIO plugin's first enable (dynamorio_instrumentation.c:496-497): no host sync; the next
 * batch enqueued on `stream` (or ordered after it) sees fresh maps. */
int kbz_reset_virgin(kbz_ctx_t *ctx, void *stream);
/* DynamoRIO last_shm_hash (dynamorio_instrumentation.c:1450-1461).  Synchronous.  The context
 * also keeps the previous batch's last trace (to tell a repeated exec from a hash collision);
 * kbz_set_last_hash forgets it, so a restored hash is handled without it (still exact). */
int kbz_get_last_hash(kbz_ctx_t *ctx, uint32_t *out);
int kbz_set_last_hash(kbz_ctx_t *ctx, uint32_t value);
/* Device pointer to the current virgin maps (3*map_size bytes); valid until the next triage
 * call (the context double-buffers them). */
uint8_t *kbz_virgin_device(kbz_ctx_t *ctx);

/* Which pass-1 kernel triages a batch: AUTO picks by batch shape (the wide-map variant when a
 * batch has fewer than 512 chunks of 64 traces, i.e. fewer than two per CU); NARROW / WIDE force
 * one (tests run every parity case through both; results are identical).  Default AUTO. */
enum kbz_pass1 { KBZ_PASS1_AUTO = 0, KBZ_PASS1_NARROW = 1, KBZ_PASS1_WIDE = 2 };
int kbz_ctx_set_pass1(kbz_ctx_t *ctx, int choice);
/* Work counters of the last finished batch, host uint32 out[3]: claim items resolved (new
 * coverage found), chunks recomputed by the DynamoRIO skip fix path, DynamoRIO skipped rows that
 * differ from their predecessor (hash collisions).  Synchronous; diagnostics only. */
int kbz_ctx_stats(kbz_ctx_t *ctx, uint32_t *out);
/* Timing of the dominant kernel (pass 1) with HIP events recorded around each of its launches on
 * the launch stream.  Returns the summed duration (ms) and count of the launches timed since
 * the previous call (waiting for them), then enables (enable != 0) or disables timing of later
 * launches.  Diagnostics only (bench.py's roofline). */
int kbz_ctx_time_pass1(kbz_ctx_t *ctx, int enable, double *total_ms, uint32_t *launches);
/* While pass-1 timing is on, time one pass-1 launch in `every` (1, the default: all of them).
 * Each timed launch carries start/stop events on its dispatch, which leave ~5 us of idle GPU
 * behind it; a benchmark samples the launches to keep that out of most steps.  No sync. */
int kbz_ctx_time_pass1_every(kbz_ctx_t *ctx, uint32_t every);
/* The same for the pipeline's other stages (k_skip, k_chain, k_total, k_scan, k_resolve,
 * k_pack): stage_ms[KBZ_NSTAGES] gets each stage's summed duration over the batches timed since
 * the previous call (index KBZ_STAGE_*; pass 1 stays with kbz_ctx_time_pass1, slot 0 is 0),
 * *batches how many batches finished (one KBZ_STAGE_SCAN record each; the fused one-shard tail,
 * k_tail, is recorded as KBZ_STAGE_SCAN).  Past 512 pending records the oldest are folded into
 * running sums (both calls), so timing left on without reads keeps a bounded event pool.
 * Diagnostics only (bench.py). */
enum kbz_stage { KBZ_STAGE_PASS1 = 0, KBZ_STAGE_SKIP = 1, KBZ_STAGE_LINK = 2, KBZ_STAGE_REDUCE = 3,
                 KBZ_STAGE_SCAN = 4, KBZ_STAGE_RESOLVE = 5, KBZ_STAGE_PACK = 6, KBZ_NSTAGES = 7 };
int kbz_ctx_time_stages(kbz_ctx_t *ctx, int enable, double *stage_ms, uint32_t *batches);

/* ---- batched triage ------------------------------------------------------------------------ */
/* traces:   device, n rows of map_size raw 8-bit hit counters, row j at traces + j*stride
 *           (stride a multiple of 16, base 16-byte aligned).  Not modified.
 * outcome:  device int8[n] of kbz_outcome, or NULL (= all KBZ_FUZZ_NONE).
 * hnb_out:  device uint8[n]: has_new_bits result of trace j given traces 0..j-1 (0/1/2).
 * h32_out:  device uint32[n] or NULL: hash32 (HASH_CONST seed) of the transformed trace
 *           (the value DynamoRIO compares with last_shm_hash).
 * x64_out:  device uint64[n] or NULL (needs KBZ_WANT_X64): XXH64(seed 0) of the transformed
 *           trace -- the crash/hang dedup key.
 * want:     KBZ_WANT_* bits.  DYNAMORIO mode always computes hash32 (its last-hash skip needs
 *           it).  The AFL modes hash only when asked (want & KBZ_WANT_H32, an XXH64 request, or
 *           a non-NULL h32_out), like the reference AFL plugin, which never hashes
 *           (afl_instrumentation.c:231-274): a batch with none of them runs a pass without the
 *           serial hash chains.
 * Stream-ordered; the virgin maps and last hash advance as if the n execs ran in order. */
int kbz_triage_batch_device(kbz_ctx_t *ctx, const uint8_t *traces, size_t n, size_t stride,
                            const int8_t *outcome, uint8_t *hnb_out, uint32_t *h32_out,
                            uint64_t *x64_out, int want, void *stream);

/* Host-memory variant: streams the batch through pinned staging slots with double-buffered
 * hipMemcpyAsync and overlaps copy-in with triage.  Blocks until results are in host memory. */
int kbz_triage_batch_host(kbz_ctx_t *ctx, const uint8_t *traces, size_t n, size_t stride,
                          const int8_t *outcome, uint8_t *hnb_out, uint32_t *h32_out,
                          uint64_t *x64_out, int want);

/* Pinned ingest ring (zero-copy producer path; SURVEY.md §8(b) kbz_ring_acquire/submit).  The
 * producer -- e.g. the fuzz loop copying each exec's trace_bits (fuzzer/main.c:370-418,
 * afl_instrumentation.c:153-180) -- writes rows straight into a pinned slot, so no staging copy
 * precedes the H2D transfer; two slots alternate, so filling one overlaps the GPU's work on the
 * other.  Batches are triaged in submission order against the carried virgin state.
 *   kbz_ring_acquire: waits until the next slot's previous batch is done (delivering its
 *     results), returns its rows (cap rows of map_size bytes, stride map_size) and outcome array.
 *   kbz_ring_submit: triages the slot's first n rows (outcome array used if have_outcome);
 *     returns at once.  hnb_out/h32_out/x64_out are host buffers (NULL = not wanted), filled
 *     when the slot is acquired again or at kbz_ring_flush.
 *   kbz_ring_commit (optional): rows [0, n_ready) of the acquired slot are written (and, if the
 *     producer used streaming stores, fenced): their host-to-device copy starts now, while the
 *     producer keeps filling the slot, and kbz_ring_submit copies only the rest.  Without it a
 *     batch's whole copy waits for the submit.  A slot with committed rows is always triaged
 *     from device memory (batches of <= 64 uncommitted rows are read from the pinned slot).
 *   kbz_ring_flush: waits for every submitted batch, delivers results, reports device errors.
 *   kbz_ring_release: hands the acquired slot back untriaged (its rows were consumed elsewhere,
 *     e.g. by kbz_triage_batch_devices, which reads pinned rows by DMA); the next acquire may
 *     return the same slot.
 * Do not interleave with kbz_triage_batch_host on the same context (they share the slots). */
int kbz_ring_acquire(kbz_ctx_t *ctx, uint8_t **rows, int8_t **outcome, size_t *cap);
int kbz_ring_commit(kbz_ctx_t *ctx, size_t n_ready);
int kbz_ring_submit(kbz_ctx_t *ctx, size_t n, int have_outcome, uint8_t *hnb_out,
                    uint32_t *h32_out, uint64_t *x64_out, int want);
int kbz_ring_flush(kbz_ctx_t *ctx);
int kbz_ring_release(kbz_ctx_t *ctx);

/* ---- sharded (multi-GPU) triage ------------------------------------------------------------ */
/* A batch split into contiguous shards, one per GPU (rank g holds traces [lo_g, hi_g)), gives
 * the same results as one kbz_triage_batch over the whole batch when each rank runs:
 *   1. kbz_shard_begin(ctx, shard, ...)                 -- local streaming pass
 *   2. (DYNAMORIO only) all-gather of kbz_shard_last_hash and kbz_shard_last_row, then
 *      kbz_shard_link(ctx, prev_last, prev_row, is_first_shard, global_last, global_row) with
 *      prev_* = pair / row of the nearest non-empty earlier rank and global_* = pair / row of
 *      the last non-empty rank (other modes: kbz_shard_link(ctx, NULL, NULL, 1, NULL, NULL))
 *   3. kbz_shard_reduce(ctx)                            -- local OR aggregates
 *   4. all-gather of kbz_shard_aggregate (nclass*map_size bytes per rank, device memory),
 *      OR of the ranks before this one -> prefix, OR of all ranks -> total
 *   5. kbz_shard_finish(ctx, prefix, total, hnb_out)    -- resolve + virgin update
 * RCCL has no bitwise reductions, so step 4 is an all-gather plus a local OR (kbz_or_reduce).
 * All pointers device memory, all calls stream-ordered on `stream`. */
int kbz_shard_begin(kbz_ctx_t *ctx, const uint8_t *traces, size_t n, size_t stride,
                    const int8_t *outcome, uint32_t *h32_out, uint64_t *x64_out, int want,
                    void *stream);
/* Copies {h32 of this shard's last trace, n != 0} into device uint32 d_out[2]. */
int kbz_shard_last_hash(kbz_ctx_t *ctx, uint32_t *d_out, void *stream);
/* Copies this shard's last raw trace (map_size bytes) into device d_out; nothing for an empty
 * shard. */
int kbz_shard_last_row(kbz_ctx_t *ctx, uint8_t *d_out, void *stream);
/* prev_last: device uint32[2] from the previous rank (ignored when is_first); prev_row: device
 * map_size bytes, that rank's last raw trace, or NULL (unknown: exact, slower if it repeats).
 * global_last: device uint32[2] from the last non-empty rank (becomes the context's last hash)
 * or NULL = this shard's own (a single-shard batch); global_row: that rank's last raw trace
 * (remembered as the next batch's row-0 predecessor) or NULL. */
int kbz_shard_link(kbz_ctx_t *ctx, const uint32_t *prev_last, const uint8_t *prev_row,
                   int is_first, const uint32_t *global_last, const uint8_t *global_row,
                   void *stream);
int kbz_shard_reduce(kbz_ctx_t *ctx, void *stream);
/* Copies this shard's OR aggregate (nclass*map_size bytes; nclass = 1 in DYNAMORIO mode,
 * 3 otherwise) into device memory d_out.  Only bits still virgin at batch entry are kept (the
 * OR of the transformed traces & V): all ranks hold the same V, and the protocol uses the
 * aggregates only under & V. */
int kbz_shard_aggregate(kbz_ctx_t *ctx, uint8_t *d_out, void *stream);
size_t kbz_shard_aggregate_bytes(kbz_ctx_t *ctx);
/* prefix/total: device, nclass*map_size bytes each (prefix may be NULL = all zero; total may be
 * NULL = this shard's own aggregate, i.e. a single-shard batch). */
int kbz_shard_finish(kbz_ctx_t *ctx, const uint8_t *prefix, const uint8_t *total,
                     uint8_t *hnb_out, void *stream);

/* The same protocol with fewer launches per step (round 6; killerbeez_amd/dist.py uses it):
 *   kbz_shard_exchange_row: the shard's last row and hash pair in ONE launch: d_out[0, M) = the
 *     last row (untouched for an empty shard), d_out[M, M + 8) = the pair, as kbz_shard_last_row
 *     + kbz_shard_last_hash write them (d_out 16-B aligned: a slot of the all-gather buffer).
 *   kbz_shard_reduce_into: in place of kbz_shard_reduce + kbz_shard_aggregate: the fix path and
 *     the shard's OR aggregate written straight into d_aggregate (nclass*map_size bytes, device,
 *     8-B aligned; e.g. this rank's slot of the all-gather buffer), the segment ORs kept.
 *   kbz_shard_finish_gathered: in place of kbz_or_prefix_total + kbz_shard_finish: the
 *     all-gathered aggregates d_gathered[world][nclass*map_size] (16-B aligned) give the prefix
 *     of ranks < rank and the batch total inside the fused tail (k_tail + k_fin, as a one-shard
 *     batch runs it).  A single shard passes its own aggregate with rank 0, world 1.
 * Order: begin, [DynamoRIO: exchange_row, all-gather, link], reduce_into, all-gather,
 * finish_gathered. */
int kbz_shard_exchange_row(kbz_ctx_t *ctx, uint8_t *d_out, void *stream);
int kbz_shard_reduce_into(kbz_ctx_t *ctx, uint8_t *d_aggregate, void *stream);
int kbz_shard_finish_gathered(kbz_ctx_t *ctx, const uint8_t *d_gathered, size_t rank,
                              size_t world, uint8_t *hnb_out, void *stream);

/* out[i] = OR of in[r*bytes + i] for r in [r_lo, r_hi).  Device, stream-ordered. */
int kbz_or_reduce(uint8_t *out, const uint8_t *in, size_t r_lo, size_t r_hi, size_t bytes,
                  void *stream);
/* Step 4 in one launch: prefix_out = OR of ranks [0, rank) (NULL: not wanted), total_out = OR of
 * all `world` rows of the all-gathered aggregates `in` (world x bytes).  Device, stream-ordered. */
int kbz_or_prefix_total(uint8_t *prefix_out, uint8_t *total_out, const uint8_t *in, size_t rank,
                        size_t world, size_t bytes, void *stream);

/* ---- merger -------------------------------------------------------------------------------- */
/* out = AND of n states (state_bytes each, typically 3*map_size), row s at states +
 * s*state_bytes.  n == 0 gives all-0xff.  Device, stream-ordered. */
int kbz_merge_and_device(uint8_t *out, const uint8_t *states, size_t n, size_t state_bytes,
                         void *stream);
/* Host variant: streams host states (pageable or pinned) through the device. Synchronous. */
int kbz_merge_and_host(uint8_t *out, const uint8_t *states, size_t n, size_t state_bytes);
/* The same fold with the states produced in place: the library calls fill(user, dst, first,
 * count) to write states [first, first + count) (state_bytes each, back to back) straight into
 * pinned staging memory dst, on the calling thread, while the GPU copies and folds the previous
 * slot (slots of up to 256 MiB).  fill returns 0, or non-zero to abort (the merge then fails).
 * The merger's file loop (merger/merger.c:79-99: read_file + create + merge per state file)
 * becomes one such call (kbz_*_gpu_merge_files in libkbz_plugin.so). */
typedef int (*kbz_merge_fill_fn)(void *user, uint8_t *dst, size_t first, size_t count);
int kbz_merge_and_fill(uint8_t *out, size_t n, size_t state_bytes, kbz_merge_fill_fn fill,
                       void *user);
/* The same fold with the result left in device memory d_out (state_bytes, the current device);
 * ordered after the work queued on `stream` so far, complete when the call returns. */
int kbz_merge_and_fill_device(uint8_t *d_out, size_t n, size_t state_bytes, kbz_merge_fill_fn fill,
                              void *user, void *stream);
/* The merger fold over several GPUs of one node (BASELINE config 4: merger/merger.c:79-104 with
 * the states sharded across the node's GPUs).  Worker w of ndev (device devices[w]; NULL = every
 * visible device, one worker each) folds the contiguous share [n*w/ndev, n*(w+1)/ndev) of the
 * states on its own host thread: fill(user, dst, first, count) is called with global indices,
 * concurrently from the workers for disjoint ranges (it must be thread-safe).  The partial folds
 * are then exchanged -- RCCL has no bitwise-AND reduction, so an all-gather over the workers'
 * GPUs (ncclCommInitAll + ncclAllGather, librccl loaded at run time) followed by a local AND on
 * every device, or peer / device-local copies of every partial to worker 0's device and one AND
 * there -- and the merged state is copied to host `out`.  exchange: KBZ_EXCHANGE_AUTO (RCCL when
 * the devices are distinct and more than one, else copies; copies also when any RCCL step fails:
 * the partial folds are intact), KBZ_EXCHANGE_COPY, KBZ_EXCHANGE_RCCL (fails if RCCL cannot be
 * used; one distinct device is a valid one-rank communicator).  A device may be listed several times (several workers on one
 * GPU: the copy path).  *used_out (or NULL) gets the exchange actually used.  Synchronous. */
enum kbz_exchange { KBZ_EXCHANGE_AUTO = 0, KBZ_EXCHANGE_COPY = 1, KBZ_EXCHANGE_RCCL = 2 };
int kbz_merge_and_fill_devices(uint8_t *out, size_t n, size_t state_bytes, kbz_merge_fill_fn fill,
                               void *user, const int *devices, size_t ndev, int exchange,
                               int *used_out);

/* ---- sharded triage over the GPUs of one node, from C ---------------------------------------- */
/* BASELINE north_star "Batches shard across the 8 GPUs of one node" for a C caller of the batched
 * loop (fuzzer/main.c:370-418 through INTEGRATION.md §2), in one process: the sharded protocol
 * above (kbz_shard_*) driven over ndev workers, worker w a context on device devices[w] (a device
 * may repeat: several workers on one GPU).  kbz_triage_batch_devices splits a HOST batch of n
 * traces (row i at traces + i*stride, stride >= map_size; outcome host int8[n] or NULL) into
 * contiguous shards [n*w/ndev, n*(w+1)/ndev), each at most max_batch; copies each to its
 * worker's device; runs pass 1 there; (DynamoRIO) gathers every shard's last row and hash pair on
 * every worker and links; gathers the shards' OR aggregates on every worker (peer copies, or
 * device-local copies for workers sharing a GPU: RCCL has no bitwise reduction, and one process
 * needs no communicator) and resolves with the prefix of the earlier shards.  hnb_out (host
 * uint8[n], or NULL) and h32_out (host uint32[n], or NULL; DynamoRIO always hashes) get the
 * results of one sequential pass over the whole batch -- the reference's per-exec
 * has_new_bits / has_new_coverage -- and every worker's virgin maps and last hash become that
 * pass's.  XXH64 is not offered here (KBZ_WANT_X64 fails).  Synchronous.
 * Host batches are staged per worker on the worker's own host thread through two pinned slots
 * (the host copy of one slot overlaps the DMA of the other), all workers at once; a batch that
 * already lies in pinned host memory (hipHostMalloc / hipHostRegister, e.g. a ring slot) goes to
 * each worker by DMA straight from there.
 * kbz_mctx_create enables peer access between every pair of the workers' distinct devices
 * (hipDeviceEnablePeerAccess) so the exchanges' peer copies run over xGMI;
 * kbz_mctx_peer_pairs returns how many ordered device pairs have it (0 on one GPU).
 * kbz_triage_batch_devices_resident: the same protocol on a batch already on the devices --
 * worker w's n[w] rows at traces[w] (device memory of devices[w], rows `stride` apart, stride
 * >= map_size and a multiple of 16), the batch being worker 0's rows, then worker 1's, ...;
 * outcome (array of W device int8 pointers, or NULL), hnb_out / h32_out (arrays of W device
 * pointers on the workers' devices; the array or an entry may be NULL).  Synchronous. */
typedef struct kbz_mctx kbz_mctx_t;
kbz_mctx_t *kbz_mctx_create(size_t map_size, int mode, size_t max_batch, const int *devices,
                            size_t ndev);
void kbz_mctx_destroy(kbz_mctx_t *m);
int kbz_mctx_workers(kbz_mctx_t *m);
kbz_ctx_t *kbz_mctx_worker(kbz_mctx_t *m, size_t w);  /* its context (ignore bytes, stats) */
int kbz_triage_batch_devices(kbz_mctx_t *m, const uint8_t *traces, size_t n, size_t stride,
                             const int8_t *outcome, uint8_t *hnb_out, uint32_t *h32_out,
                             int want);
int kbz_triage_batch_devices_resident(kbz_mctx_t *m, const uint8_t *const *traces,
                                      const size_t *n, size_t stride,
                                      const int8_t *const *outcome, uint8_t *const *hnb_out,
                                      uint32_t *const *h32_out, int want);
int kbz_mctx_peer_pairs(kbz_mctx_t *m);
/* Worker 0's virgin maps / last hash (every worker holds the same); set_virgin sets all. */
int kbz_mctx_get_virgin(kbz_mctx_t *m, uint8_t *host_out);
int kbz_mctx_set_virgin(kbz_mctx_t *m, const uint8_t *host_in);
int kbz_mctx_get_last_hash(kbz_mctx_t *m, uint32_t *out);

/* ---- DynamoRIO per-module coverage ----------------------------------------------------------- */
/* has_new_coverage_per_module (dynamorio_instrumentation.c:1477-1493) over an ordered batch: each
 * traced module m has its own context ctxs[m] (its virgin map, ignore bytes and last hash, as
 * target_module_t holds them, dynamorio_instrumentation.h:26-83) and its own map inside every
 * trace row, at traces + j*stride + module_offsets[m] (host size_t[k], 16-byte aligned).
 * hnb_out: device uint8[k*n], hnb_out[m*n + j] = module m's has_new_coverage result for exec j
 * (0/1/2; nonzero = last_path_was_new); any_out: device uint8[n] or NULL, the OR over modules
 * (the per-exec return value).  Stream-ordered. */
/* h32_out: device uint32[k*n] or NULL, h32_out[m*n + j] = module m's hash32 of exec j (what
 * has_new_coverage compares with last_shm_hash, :1441-1451; the dump_map_dir file name). */
int kbz_triage_modules_device(kbz_ctx_t *const *ctxs, size_t k, const uint8_t *traces, size_t n,
                              size_t stride, const size_t *module_offsets, const int8_t *outcome,
                              uint8_t *hnb_out, uint8_t *any_out, uint32_t *h32_out,
                              void *stream);

/* Host-memory variant (traces, module_offsets, outcome, hnb_out [k*n], any_out [n], h32_out
 * [k*n] all host memory).  Synchronous. */
int kbz_triage_modules_host(kbz_ctx_t *const *ctxs, size_t k, const uint8_t *traces, size_t n,
                            size_t stride, const size_t *module_offsets, const int8_t *outcome,
                            uint8_t *hnb_out, uint8_t *any_out, uint32_t *h32_out);

/* ---- transformed maps ------------------------------------------------------------------------ */
/* out row j = transform of row j (len bytes; out may equal rows with the same stride):
 * KBZ_XF_CLASSIFY = classify_counts (dynamorio_instrumentation.c:265-292, the map has_new_coverage
 * leaves in trace_bits: get_module_info's info, :1565, and the dump_map_dir files, :1453-1458),
 * KBZ_XF_SIMPLIFY = simplify_trace (afl_instrumentation.c:674-706), KBZ_XF_RAW = a copy.
 * len, strides and pointers 16-byte multiples / aligned.  Device, stream-ordered. */
enum kbz_xf { KBZ_XF_RAW = 0, KBZ_XF_CLASSIFY = 1, KBZ_XF_SIMPLIFY = 2 };
int kbz_transform_rows_device(const uint8_t *rows, size_t n, size_t stride, size_t len, int xf,
                              uint8_t *out, size_t out_stride, void *stream);
/* Host memory in and out (staged through the device).  Synchronous. */
int kbz_transform_rows_host(const uint8_t *rows, size_t n, size_t stride, size_t len, int xf,
                            uint8_t *out, size_t out_stride);

/* ---- picker: ignore bytes from repeated runs ------------------------------------------------ */
/* The picker's diff loop (picker/main.c:240-262) for one module: runs = device
 * [files][iters][size] bytes, the instrumentation data of iteration `it` of input file `f`
 * (picker/main.c:209 layout).  ignore_out (device, size bytes) = 0x00 where two consecutive
 * iterations of one file differ (a noisy byte), 0xff elsewhere -- the ignore_bytes file the
 * DynamoRIO plugin loads (kbz_set_ignore).  pair_counts_out (device uint32[files*(iters-1)] or
 * NULL): differing bytes of each (it-1, it) pair (the reference's ignore_count); total_out
 * (device uint64 or NULL): noisy bytes (total_ignore_count).  size and both pointers must be
 * multiples of 16 / 16-byte aligned.  Stream-ordered. */
int kbz_picker_ignore_device(const uint8_t *runs, size_t files, size_t iters, size_t size,
                             uint8_t *ignore_out, uint32_t *pair_counts_out, uint64_t *total_out,
                             void *stream);

/* ---- standalone hashes over a batch --------------------------------------------------------- */
/* h32_out[j] = hash32(row j, len, seed); x64_out[j] = XXH64(row j, len, seed).  len % 8 == 0
 * for hash32 (afl_progs/hash.h:38); any len for XXH64.  Device, stream-ordered. */
int kbz_hash32_device(const uint8_t *rows, size_t n, size_t stride, size_t len, uint32_t seed,
                      uint32_t *h32_out, void *stream);
int kbz_xxh64_device(const uint8_t *rows, size_t n, size_t stride, size_t len, uint64_t seed,
                     uint64_t *x64_out, void *stream);

/* Synchronise the context's work and report any device-side consistency error (-1). */
int kbz_sync(kbz_ctx_t *ctx, void *stream);

/* ---- unique crash/hang table: insert-if-absent set of 16-byte keys -------------------------- */
/* The reference's hash-set novelty (linux_ipt_instrumentation.c:412-424: HASH_FIND, HASH_ADD
 * when absent, new iff absent; insertion-ordered like uthash) applied to an ordered batch:
 * key j is new iff it is absent from the set and from keys 0..j-1 of the batch.  Keys are two
 * uint64 words like the IPT key {tip, tnt} (linux_ipt_instrumentation.h:19-22); for trace dedup
 * {XXH64 of the transformed trace (kbz_triage_batch_* x64_out), outcome class}. */
typedef struct kbz_set kbz_set_t;
/* capacity: most keys the set will hold (table = 2x, power of two). */
kbz_set_t *kbz_set_create(size_t capacity);
void kbz_set_destroy(kbz_set_t *set);
const char *kbz_set_last_error(void);
/* keys: device uint64[2*n]; mask: device uint8[n] or NULL (rows with mask 0 are neither
 * inserted nor new); is_new_out: device uint8[n] (1 = new, inserted).  Stream-ordered. */
int kbz_set_insert_device(kbz_set_t *set, const uint64_t *keys, const uint8_t *mask, size_t n,
                          uint8_t *is_new_out, void *stream);
/* Host variant: keys host uint64[2*n] inserted in order (e.g. a state's key list being loaded:
 * linux_ipt_set_state :1066-1075 adds each key not yet present); is_new_out host or NULL.
 * Synchronous. */
int kbz_set_insert_host(kbz_set_t *set, const uint64_t *keys, size_t n, uint8_t *is_new_out);
/* Number of keys in the set; -1 if the capacity was exceeded (keys dropped).  Synchronous. */
int kbz_set_size(kbz_set_t *set, size_t *out);
/* The first min(cap, size) keys in insertion order into host uint64[2*cap]; *n_out = size.
 * Synchronous. */
int kbz_set_keys(kbz_set_t *set, uint64_t *host_out, size_t cap, size_t *n_out);
/* A new set holding the union of two sets, replacing linux_ipt_merge
 * (linux_ipt_instrumentation.c:944-978): first's keys in first's insertion order, then the keys
 * of second absent from first, in second's insertion order.  Neither input is changed.  Runs on
 * the device, ordered on `stream`; NULL on failure (kbz_set_last_error). */
kbz_set_t *kbz_set_merge(kbz_set_t *first, kbz_set_t *second, void *stream);

/* ---- Intel-PT path keys (linux_ipt_instrumentation.c analyze_ipt :212-425) ------------------- */
/* The reference hashes every exec's IPT packets into two streaming XXH64s while parsing them:
 * TNT bits via add_tnt_to_hash (:132-156), TIP addresses via add_tip_to_hash (:163-189),
 * finish_tnt_hash (:115-124) at the end, and looks the digest pair {tip, tnt} up in its set
 * (:409-424).  Here the host-side parser (it stays on the CPU) feeds a batch of execs, each
 * call the counterpart of the reference function named; the digests of the whole batch are
 * computed on the GPU, and novelty is the unique set (kbz_set_*: insert-if-absent, insertion
 * order = the reference's uthash set; its state dump/load is kbz_set_keys / kbz_set_insert_host,
 * linux_ipt_merge is kbz_set_merge). */
typedef struct kbz_ipt_batch kbz_ipt_batch_t;
kbz_ipt_batch_t *kbz_ipt_batch_create(void);
void kbz_ipt_batch_destroy(kbz_ipt_batch_t *batch);
const char *kbz_ipt_last_error(void);
/* add_tip_to_hash's ASLR normalisation (:169-185): a TIP inside coverage library i (starts[i] <=
 * tip < ends[i]) becomes (tip - starts[i]) | library_hashes[i] << 32; without libraries, one
 * inside [target_start, target_end) becomes tip - target_start; others are kept. */
int kbz_ipt_set_ranges(kbz_ipt_batch_t *batch, size_t n_libraries, const uint64_t *starts,
                       const uint64_t *ends, const uint32_t *library_hashes,
                       uint64_t target_start, uint64_t target_end);
/* add_tnt_to_hash: num_bits TNT bits of one packet (tnt_bits[i / 8] bit i % 8). */
int kbz_ipt_add_tnt(kbz_ipt_batch_t *batch, const uint8_t *tnt_bits, int num_bits);
/* add_tip_to_hash: the IP of a TIP packet. */
int kbz_ipt_add_tip(kbz_ipt_batch_t *batch, uint64_t tip);
/* finish_tnt_hash: the current exec is complete (the next add starts a new one). */
int kbz_ipt_end_exec(kbz_ipt_batch_t *batch);
size_t kbz_ipt_execs(kbz_ipt_batch_t *batch);
/* keys_out: device uint64[2*n], {tip digest, tnt digest} per completed exec (the
 * ipt_hashtable_key of linux_ipt_instrumentation.h:19-22).  Uploads the batch, queues the
 * hashes on `stream` and empties the batch. */
int kbz_ipt_hash_device(kbz_ipt_batch_t *batch, uint64_t *keys_out, void *stream);
/* The whole novelty step for the batch: hashes, then insert into `set` in exec order;
 * keys_out (host uint64[2*n] or NULL) and is_new_out (host uint8[n] or NULL: 1 = the exec's path
 * was new, linux_ipt_is_new_path's result).  Synchronous; empties the batch. */
int kbz_ipt_triage(kbz_ipt_batch_t *batch, kbz_set_t *set, uint64_t *keys_out,
                   uint8_t *is_new_out);

#ifdef __cplusplus
}
#endif
#endif /* KBZ_TRIAGE_H */
