/*
 * tests/native/integration_harness.c -- INTEGRATION.md §1 and §2 as compiled C: the factory patch
 * (instrumentation/instrumentation_factory.c:72-84 gains an "afl_gpu" branch that copies the
 * plugin's vtable into the reference's own instrumentation_t) and the finish_fuzz_round /
 * afl_is_new_path patch of afl_instrumentation.c (:189-198, :231-274), driven like
 * fuzzer/main.c:370-418 -- one exec then is_new_path, or N execs then their results -- over
 * recorded traces.
 *
 * Built by tests/test_integration_c.py (and __graft_entry__.build()) against the REFERENCE's
 * instrumentation.h (-I /root/reference/instrumentation), so the factory code type-checks against
 * the real struct; where the reference tree is absent it is built with -DKBZ_NO_REFERENCE_HEADER
 * against kbz_plugin.h's layout-identical struct (tests/native/abi_layout.c checks the layout).
 *
 * usage: integration_harness <traces.bin> <n> <map_size> <batch>
 *   traces.bin: n rows of map_size raw hit counters, then n int8 outcomes (0 none, 1 hang,
 *   2 crash); batch 1 = the unmodified per-exec loop, batch > 1 = the batched loop of §2.
 *   Prints one line per exec: "<index> <is_new_path>", then "state <bytes of get_state>".
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/types.h>

#ifndef KBZ_NO_REFERENCE_HEADER
#define INSTRUMENTATION_NO_IMPORT
#include "instrumentation.h" /* the reference's struct instrumentation */
#endif
#include "kbz_plugin.h"
#ifdef KBZ_NO_REFERENCE_HEADER
typedef kbz_instrumentation_t instrumentation_t;
#endif

/* ---- instrumentation_factory with the GPU plugins registered ------------- */
static instrumentation_t *instrumentation_factory(const char *instrumentation_type) {
  instrumentation_t *ret = (instrumentation_t *)malloc(sizeof(instrumentation_t));
  if (!ret) return NULL;
  memset(ret, 0, sizeof(instrumentation_t)); /* instrumentation_factory.c:27-28 */
  if (!strcmp(instrumentation_type, "afl_gpu") || !strcmp(instrumentation_type, "dynamorio_gpu")) {
    kbz_instrumentation_t *k = kbz_instrumentation_factory(instrumentation_type);
    if (!k) {
      free(ret);
      return NULL; /* FACTORY_ERROR() */
    }
    /* kbz_instrumentation_t begins with struct instrumentation's members, in order */
    memcpy(ret, k, sizeof(instrumentation_t));
    free(k);
  } else {
    free(ret);
    return NULL;
  }
  return ret;
}

/* ---- the members of afl_state the patch adds or touches ------------------ */
typedef struct {
  void *gpu;        /* kbz_afl_gpu state (the vtable's create) */
  long gpu_ticket;  /* ticket of the last recorded exec */
  int fuzz_results_set;
  int last_fuzz_result;
  uint8_t *trace_bits;
  int outcome; /* what afl_is_process_done / WIFSIGNALED decide on the host (:241-256) */
} afl_state_t;

/* finish_fuzz_round (:231-274) patched: record the RAW map with the outcome; the GPU applies
 * simplify_trace for hangs / crashes and picks virgin_tmout / virgin_crash itself */
static int finish_fuzz_round(afl_state_t *state) {
  state->last_fuzz_result = state->outcome;
  state->gpu_ticket = kbz_afl_gpu_record(state->gpu, state->trace_bits, state->last_fuzz_result);
  if (state->gpu_ticket < 0) return KBZ_PLUGIN_FUZZ_ERROR;
  state->fuzz_results_set = 1;
  return state->last_fuzz_result;
}

/* afl_is_new_path (:189-198) patched */
static int afl_is_new_path(afl_state_t *state) {
  if (!state->fuzz_results_set) finish_fuzz_round(state);
  int r = kbz_afl_gpu_result(state->gpu, state->gpu_ticket);
  return r < 0 ? -1 : r != 0;
}

int main(int argc, char **argv) {
  if (argc != 5) {
    fprintf(stderr, "usage: %s traces.bin n map_size batch\n", argv[0]);
    return 2;
  }
  const size_t n = strtoul(argv[2], NULL, 10), m = strtoul(argv[3], NULL, 10);
  const size_t batch = strtoul(argv[4], NULL, 10);
  FILE *f = fopen(argv[1], "rb");
  uint8_t *rows = (uint8_t *)malloc(n * m);
  int8_t *oc = (int8_t *)malloc(n);
  if (!f || !rows || !oc || fread(rows, 1, n * m, f) != n * m || fread(oc, 1, n, f) != n) {
    fprintf(stderr, "cannot read %s\n", argv[1]);
    return 2;
  }
  fclose(f);
  instrumentation_t *instr = instrumentation_factory("afl_gpu");
  if (!instr) {
    fprintf(stderr, "factory: %s\n", kbz_plugin_last_error());
    return 1;
  }
  char options[128];
  snprintf(options, sizeof(options), "{\"map_size\": %zu, \"max_batch\": %zu}", m,
           batch > 64 ? batch : 64);
  afl_state_t state;
  memset(&state, 0, sizeof(state));
  state.gpu = instr->create(options, NULL); /* through the reference struct's member */
  if (!state.gpu) {
    fprintf(stderr, "create: %s\n", kbz_plugin_last_error());
    return 1;
  }
  long *tickets = (long *)malloc((batch ? batch : 1) * sizeof(long));
  size_t pending = 0, first = 0;
  for (size_t j = 0; j < n; j++) {
    state.trace_bits = rows + j * m; /* the target wrote its map here (SysV SHM) */
    state.outcome = oc[j];
    state.fuzz_results_set = 0;
    if (batch <= 1) { /* fuzzer/main.c:374-385: test_next_input, then is_new_path */
      if (finish_fuzz_round(&state) < 0) return 1;
      const int r = afl_is_new_path(&state);
      if (r < 0) {
        fprintf(stderr, "is_new_path: %s\n", kbz_plugin_last_error());
        return 1;
      }
      printf("%zu %d\n", j, r);
      continue;
    }
    /* INTEGRATION.md §2, batched: record N execs, then one GPU batch for all of them */
    if (finish_fuzz_round(&state) < 0) return 1;
    tickets[pending++] = state.gpu_ticket;
    if (pending == batch || j + 1 == n) {
      for (size_t i = 0; i < pending; i++) {
        const int r = kbz_afl_gpu_result(state.gpu, tickets[i]);
        if (r < 0) {
          fprintf(stderr, "result: %s\n", kbz_plugin_last_error());
          return 1;
        }
        printf("%zu %d\n", first + i, r > 0);
      }
      first += pending;
      pending = 0;
    }
  }
  char *st = instr->get_state(state.gpu);
  if (!st) return 1;
  printf("state %zu\n", strlen(st));
  instr->free_state(st);
  instr->cleanup(state.gpu);
  free(instr);
  free(tickets);
  free(rows);
  free(oc);
  return 0;
}
