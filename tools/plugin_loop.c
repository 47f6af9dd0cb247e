/* tools/plugin_loop.c -- the per-exec cost of the GPU plugins (libkbz_plugin.so) in the shape of
 * the reference's fuzz loop, from C, as a C fuzzer calls them (fuzzer/main.c:370-418 with the
 * batching of INTEGRATION.md §2).  Bench harness for `bench.py --workload plugin`; not product.
 *
 * Per exec:  memset(map, 0, M)            afl_enable's clear of trace_bits (afl_instrumentation.c:170)
 *            memcpy(map, pool[e % P], M)  the target's run writes its trace into the map
 *            ticket[e % B] = record(map, outcome)
 *            every B execs: result(ticket) for the B execs (is_new_path, fuzzer/main.c:385)
 * The map is a SysV shared-memory segment, as the reference's setup_shm makes it (:563-576).
 * The same loop without the two plugin calls is timed as `base` (what the host spends anyway);
 * the plugin's cost per exec is loop - base.
 *
 * usage: plugin_loop afl|dynamorio POOL_FILE OUTCOME_FILE MAP_SIZE POOL EXECS B1 [B2 ...]
 *   POOL_FILE: POOL rows of MAP_SIZE bytes; OUTCOME_FILE: POOL int8 FUZZ_* results.
 * Prints one JSON object: {"by_batch": {"B": {"us_per_exec": .., "base_us": .., "plugin_us": ..,
 * "new": ..}}}
 */
#define _GNU_SOURCE
#include <fcntl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/ipc.h>
#include <sys/mman.h>
#include <sys/shm.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "kbz_plugin.h"

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

static void *map_file(const char *path, size_t want) {
  int fd = open(path, O_RDONLY);
  struct stat st;
  if (fd < 0 || fstat(fd, &st) || (size_t)st.st_size < want) {
    fprintf(stderr, "plugin_loop: %s: missing or shorter than %zu bytes\n", path, want);
    exit(2);
  }
  void *p = mmap(NULL, want, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    perror("mmap");
    exit(2);
  }
  return p;
}

int main(int argc, char **argv) {
  if (argc < 8) {
    fprintf(stderr, "usage: %s afl|dynamorio POOL_FILE OUTCOME_FILE MAP_SIZE POOL EXECS B...\n",
            argv[0]);
    return 2;
  }
  const int dr = strcmp(argv[1], "dynamorio") == 0;
  const size_t M = strtoull(argv[4], NULL, 0), P = strtoull(argv[5], NULL, 0);
  const long execs = atol(argv[6]);
  const uint8_t *pool = (const uint8_t *)map_file(argv[2], P * M);
  const int8_t *oc = (const int8_t *)map_file(argv[3], P);
  void *(*create)(char *, char *) = dr ? kbz_dynamorio_gpu_create : kbz_afl_gpu_create;
  long (*record)(void *, const uint8_t *, int) = dr ? kbz_dynamorio_gpu_record : kbz_afl_gpu_record;
  int (*result)(void *, long) = dr ? kbz_dynamorio_gpu_result : kbz_afl_gpu_result;
  void (*cleanup)(void *) = dr ? kbz_dynamorio_gpu_cleanup : kbz_afl_gpu_cleanup;

  int id = shmget(IPC_PRIVATE, M, IPC_CREAT | IPC_EXCL | 0600);
  if (id < 0) {
    perror("shmget");
    return 1;
  }
  uint8_t *map = (uint8_t *)shmat(id, NULL, 0);
  shmctl(id, IPC_RMID, NULL);  /* freed when detached */
  if (map == (void *)-1) {
    perror("shmat");
    return 1;
  }

  printf("{\"execs\": %ld, \"map_size\": %zu, \"mode\": \"%s\", \"by_batch\": {", execs, M,
         argv[1]);
  double t0;
  long *tickets = NULL;
  for (int a = 7; a < argc; a++) {
    const long B = atol(argv[a]);
    char opt[128];
    snprintf(opt, sizeof opt, "{\"map_size\": %zu, \"max_batch\": %ld}", M, B);
    void *p = create(opt, NULL);
    if (!p) {
      fprintf(stderr, "create failed: %s\n", kbz_plugin_last_error());
      return 1;
    }
    tickets = (long *)realloc(tickets, (size_t)B * sizeof(long));
    /* warm: context, pinned ring slots, the first batch's allocations */
    const long warm = B < 64 ? 64 : B;
    for (long e = 0; e < warm; e++) {
      memset(map, 0, M);
      memcpy(map, pool + (size_t)(e % P) * M, M);
      tickets[e % B] = record(p, map, oc[e % P]);
      if ((e + 1) % B == 0)
        for (long j = 0; j < B; j++) (void)result(p, tickets[j]);
    }
    const long n = execs - execs % B;
    long fresh = 0;
    t0 = now_s();
    for (long e = 0; e < n; e++) {
      memset(map, 0, M);
      memcpy(map, pool + (size_t)(e % P) * M, M);
      tickets[e % B] = record(p, map, oc[e % P]);
      if (tickets[e % B] < 0) {
        fprintf(stderr, "record failed: %s\n", kbz_plugin_last_error());
        return 1;
      }
      if ((e + 1) % B == 0)
        for (long j = 0; j < B; j++) {
          const int r = result(p, tickets[j]);
          if (r < 0) {
            fprintf(stderr, "result failed: %s\n", kbz_plugin_last_error());
            return 1;
          }
          fresh += r > 0;
        }
    }
    const double per = (now_s() - t0) / n;
    /* base: the host's own per-exec work (clear + the target's writes), no plugin calls; timed
     * right after, three times, the fastest kept (the pool's DRAM state drifts) */
    double base = 1e9;
    for (int rep = 0; rep < 3; rep++) {
      t0 = now_s();
      for (long e = 0; e < n; e++) {
        memset(map, 0, M);
        memcpy(map, pool + (size_t)(e % P) * M, M);
        __asm__ volatile("" ::"r"(map) : "memory");
      }
      const double b = (now_s() - t0) / n;
      base = b < base ? b : base;
    }
    printf("%s\"%ld\": {\"us_per_exec\": %.4f, \"base_us\": %.4f, \"plugin_us\": %.4f, "
           "\"new\": %ld, \"execs\": %ld}",
           a > 7 ? ", " : "", B, 1e6 * per, 1e6 * base, 1e6 * (per - base), fresh, n);
    fflush(stdout);
    cleanup(p);
  }
  printf("}}\n");
  shmdt(map);
  return 0;
}
