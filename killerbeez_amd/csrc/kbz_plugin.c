/*
 * killerbeez_amd/csrc/kbz_plugin.c -- libkbz_plugin.so: the "afl_gpu" and "dynamorio_gpu"
 * instrumentation plugins of include/kbz_plugin.h.
 *
 * Every novelty result and every merge comes from libkbz_hip.so on the GPU; this file is the
 * host bookkeeping around it: options/state JSON, a host mirror of the virgin maps (so
 * get_state/set_state/merge work without replaying anything), the deferred per-exec queue that
 * turns the reference's one-exec-at-a-time calls into ordered GPU batches, and the vtable.
 * There is no CPU path: if the HIP library cannot reach a GPU, triage and merge calls fail
 * with the reference's error values.
 *
 * Reference behaviour mirrored (paths relative to ThePatrickStar/killerbeez):
 *   create/set_state      afl_create :23-35, afl_set_state :95-109 (3 maps), dynamorio_set_state
 *                         :1311-1372 (virgin_bits + last_shm_hash); fresh maps are all-0xff
 *                         (setup_shm afl_instrumentation.c:555-559)
 *   get_state             afl_get_state :62-79, dynamorio_get_state :1239-1281 (key names;
 *                         per_module_coverage: a "modules" array of {name, virgin_bits,
 *                         last_shm_hash, last_path_was_new})
 *   merge                 afl_merge :123-140 (AND of the 3 maps, everything else fresh),
 *                         dynamorio_merge :1180-1231 (AND of virgin_bits, last hash 0)
 *   is_new_path           afl_is_new_path :189-198 (last_is_new_path ? 1 : 0; -1 before the
 *                         first exec), dynamorio has_new_coverage :1465-1467 (hnb != 0)
 *   get_fuzz_result       afl_get_fuzz_result :208-216 (the recorded FUZZ_* of the last exec)
 *   ignore_bytes_file     load_ignore_bytes dynamorio_instrumentation.c:788-801 (exactly
 *                         map_size bytes); ignore_bytes_dir (per module: <dir>/<name>.dat, :802-814)
 *   per_module_coverage   dynamorio_instrumentation.c:1048-1063 options, has_new_coverage_per_
 *                         module :1477-1493 (own virgin map / ignore bytes / last hash per module,
 *                         the exec is new if any module is), dynamorio_merge :1180-1231 (modules
 *                         matched by name)
 */
#define _POSIX_C_SOURCE 200809L /* strdup under -std=c11 */
#include "kbz_plugin.h"

#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "kbz_triage.h"

static __thread char g_err[512];

static void set_err(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

const char *kbz_plugin_last_error(void) { return g_err; }

typedef struct kbz_plugin {
  int mode;                /* KBZ_MODE_AFL or KBZ_MODE_DYNAMORIO */
  size_t map_size, max_batch;
  uint8_t *ignore;         /* dynamorio_gpu ignore_bytes (map_size bytes) or NULL */
  uint8_t *virgin;         /* host mirror: virgin_bits | virgin_tmout | virgin_crash */
  uint32_t last_hash;      /* dynamorio last_shm_hash */
  int mirror_stale;        /* the GPU copy is newer than the mirror */
  kbz_ctx_t *ctx;          /* GPU context, created on the first triage */
  uint8_t *q_rows;         /* deferred execs: the acquired pinned ring slot (kbz_ring_acquire) */
  int8_t *q_outcome;
  size_t q_cap;            /* its rows (<= max_batch) */
  size_t q_n;
  long q_base;             /* ticket of q_rows[0] */
  uint8_t *r_hnb;          /* results of the last flushed window */
  size_t r_n;
  long r_base;
  long last_ticket;        /* -1 until the first record */
  int last_fuzz_result;
  int last_path_was_new;   /* has_new_coverage result of the last triaged exec (DR state key) */
  /* dynamorio_gpu per_module_coverage (dynamorio_instrumentation.c:1048-1063): nmod module maps
   * per exec, each with its own context (virgin map, ignore bytes, last hash).  The queue is a
   * host buffer of max_batch rows of nmod*map_size bytes (module m at offset m*map_size). */
  int per_module;
  size_t nmod;
  char **mod_names;
  kbz_ctx_t **mctx;
  uint8_t *mvirgin;        /* [nmod][map_size] host mirror */
  uint32_t *mlast;         /* [nmod] last_shm_hash */
  uint8_t *mnew;           /* [nmod] last_path_was_new */
  uint8_t **mignore;       /* [nmod] ignore bytes or NULL */
  uint8_t *mq;             /* queued execs, max_batch rows */
  int8_t *mq_outcome;
  uint8_t *r_mhnb;         /* [nmod][max_batch] per-module results of the last window */
} kbz_plugin_t;

static size_t nmaps(const kbz_plugin_t *p) { return p->mode == KBZ_MODE_DYNAMORIO ? 1 : 3; }

/* ---- minimal JSON: flat objects with number / string values (the formats of this file) ---- */
static const char *json_value(const char *json, const char *key) {
  char pat[96];
  snprintf(pat, sizeof(pat), "\"%s\"", key);
  for (const char *p = json; (p = strstr(p, pat)); p++) {
    const char *q = p + strlen(pat);
    while (*q == ' ' || *q == '\t' || *q == '\n' || *q == '\r') q++;
    if (*q != ':') continue;
    q++;
    while (*q == ' ' || *q == '\t' || *q == '\n' || *q == '\r') q++;
    return q;
  }
  return NULL;
}

/* 1 found, 0 absent, -1 malformed */
static int json_u64(const char *json, const char *key, unsigned long long *out) {
  const char *v = json ? json_value(json, key) : NULL;
  if (!v) return 0;
  char *end;
  unsigned long long x = strtoull(v, &end, 10);
  if (end == v) return -1;
  *out = x;
  return 1;
}

static char *json_str(const char *json, const char *key) {
  const char *v = json ? json_value(json, key) : NULL;
  if (!v || *v != '"') return NULL;
  v++;
  char *s = (char *)malloc(strlen(v) + 1);
  if (!s) return NULL;
  size_t n = 0;
  for (; *v && *v != '"'; v++) {
    if (*v == '\\' && v[1]) v++;
    s[n++] = *v;
  }
  s[n] = 0;
  return s;
}

/* The raw text of a JSON array value ("[...]") -> its top-level elements as malloc'd strings
 * (quotes kept for strings, braces for objects); NULL + *n = 0 when the key is absent. */
static char **json_array(const char *json, const char *key, size_t *n, int *bad) {
  *n = 0;
  *bad = 0;
  const char *v = json ? json_value(json, key) : NULL;
  if (!v) return NULL;
  if (*v != '[') {
    *bad = 1;
    return NULL;
  }
  char **items = NULL;
  const char *q = v + 1;
  for (;;) {
    while (*q == ' ' || *q == '\t' || *q == '\n' || *q == '\r' || *q == ',') q++;
    if (*q == ']') return items;
    if (!*q) break;
    const char *b = q;
    int depth = 0, in_str = 0;
    for (; *q; q++) {
      if (in_str) {
        if (*q == '\\' && q[1]) q++;
        else if (*q == '"') in_str = 0;
        if (!in_str && !depth) {
          q++;
          break;
        }
        continue;
      }
      if (*q == '"') in_str = 1;
      else if (*q == '{' || *q == '[') depth++;
      else if (*q == '}' || *q == ']') {
        if (!depth) break;
        if (!--depth) {
          q++;
          break;
        }
      } else if (*q == ',' && !depth) break;
    }
    char **grown = (char **)realloc(items, (*n + 1) * sizeof(char *));
    if (!grown) break;
    items = grown;
    items[*n] = strndup(b, (size_t)(q - b));
    if (!items[*n]) break;
    (*n)++;
  }
  *bad = 1;
  for (size_t i = 0; i < *n; i++) free(items[i]);
  free(items);
  *n = 0;
  return NULL;
}
static void free_strings(char **v, size_t n) {
  if (!v) return;
  for (size_t i = 0; i < n; i++) free(v[i]);
  free(v);
}
/* a JSON string element ("...") -> malloc'd unescaped text */
static char *json_unquote(const char *s) {
  if (!s || *s != '"') return NULL;
  char *o = (char *)malloc(strlen(s));
  if (!o) return NULL;
  size_t n = 0;
  for (s++; *s && *s != '"'; s++) {
    if (*s == '\\' && s[1]) s++;
    o[n++] = *s;
  }
  o[n] = 0;
  return o;
}

static int hexval(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

static int json_hex(const char *json, const char *key, uint8_t *out, size_t n) {
  const char *v = json_value(json, key);
  if (!v || *v != '"') return -1;
  v++;
  for (size_t i = 0; i < n; i++) {
    const int hi = hexval(v[2 * i]);
    const int lo = hi < 0 ? -1 : hexval(v[2 * i + 1]);
    if (hi < 0 || lo < 0) return -1;
    out[i] = (uint8_t)(hi << 4 | lo);
  }
  return v[2 * n] == '"' ? 0 : -1;
}

static char *put_hex(char *o, const uint8_t *b, size_t n) {
  static const char digits[] = "0123456789abcdef";
  for (size_t i = 0; i < n; i++) {
    *o++ = digits[b[i] >> 4];
    *o++ = digits[b[i] & 15];
  }
  return o;
}

/* ---- lifetime ------------------------------------------------------------------------------ */
static void plugin_free(kbz_plugin_t *p) {
  if (!p) return;
  if (p->ctx) kbz_ctx_destroy(p->ctx);
  for (size_t m = 0; m < p->nmod; m++) {
    if (p->mctx && p->mctx[m]) kbz_ctx_destroy(p->mctx[m]);
    if (p->mignore) free(p->mignore[m]);
  }
  free_strings(p->mod_names, p->nmod);
  free(p->mctx);
  free(p->mignore);
  free(p->mvirgin);
  free(p->mlast);
  free(p->mnew);
  free(p->mq);
  free(p->mq_outcome);
  free(p->r_mhnb);
  free(p->ignore);
  free(p->virgin);
  free(p->r_hnb);
  free(p);
}

/* per_module_coverage: module tables for the given names (taken over) */
static int plugin_modules(kbz_plugin_t *p, char **names, size_t n) {
  p->per_module = 1;
  p->nmod = n;
  p->mod_names = names;
  const size_t m = p->map_size;
  p->mctx = (kbz_ctx_t **)calloc(n, sizeof(kbz_ctx_t *));
  p->mignore = (uint8_t **)calloc(n, sizeof(uint8_t *));
  p->mvirgin = (uint8_t *)malloc(n * m);
  p->mlast = (uint32_t *)calloc(n, sizeof(uint32_t));
  p->mnew = (uint8_t *)calloc(n, 1);
  p->mq = (uint8_t *)malloc(p->max_batch * n * m);
  p->mq_outcome = (int8_t *)malloc(p->max_batch);
  p->r_mhnb = (uint8_t *)malloc(n * p->max_batch);
  if (!p->mctx || !p->mignore || !p->mvirgin || !p->mlast || !p->mnew || !p->mq ||
      !p->mq_outcome || !p->r_mhnb) {
    set_err("out of host memory");
    return -1;
  }
  memset(p->mvirgin, 0xff, n * m);
  return 0;
}
static long module_index(const kbz_plugin_t *p, const char *name) {
  for (size_t i = 0; i < p->nmod; i++)
    if (!strcmp(p->mod_names[i], name)) return (long)i;
  return -1;
}

static kbz_plugin_t *plugin_alloc(int mode, size_t map_size, size_t max_batch) {
  kbz_plugin_t *p = (kbz_plugin_t *)calloc(1, sizeof(*p));
  if (!p) return NULL;
  p->mode = mode;
  p->map_size = map_size;
  p->max_batch = max_batch;
  p->last_ticket = -1;
  p->last_fuzz_result = KBZ_PLUGIN_FUZZ_ERROR;
  p->virgin = (uint8_t *)malloc(3 * map_size);
  p->r_hnb = (uint8_t *)malloc(max_batch);
  if (!p->virgin || !p->r_hnb) {
    plugin_free(p);
    set_err("out of host memory");
    return NULL;
  }
  memset(p->virgin, 0xff, 3 * map_size);
  return p;
}

static uint8_t *load_ignore_file(const char *path, size_t map_size) {
  FILE *f = fopen(path, "rb");
  if (!f) {
    set_err("Could not open ignore bytes file %s", path);
    return NULL;
  }
  uint8_t *b = (uint8_t *)malloc(map_size);
  size_t got = b ? fread(b, 1, map_size, f) : 0;
  const int extra = fgetc(f) != EOF;
  fclose(f);
  if (got != map_size || extra) {
    set_err("Incorrect size of ignore bytes file %s (need exactly %zu bytes)", path, map_size);
    free(b);
    return NULL;
  }
  return b;
}
static int load_ignore(kbz_plugin_t *p, const char *path) {
  p->ignore = load_ignore_file(path, p->map_size);
  return p->ignore ? 0 : -1;
}

static kbz_plugin_t *plugin_from_options(int mode, const char *options) {
  unsigned long long m = 65536, mb = 4096;
  if (json_u64(options, "map_size", &m) < 0 || json_u64(options, "max_batch", &mb) < 0) {
    set_err("bad options (map_size / max_batch must be integers)");
    return NULL;
  }
  if (m < 256 || m % 256 || m > (1ull << 24)) {
    set_err("map_size must be a multiple of 256 in [256, 16 MiB]");
    return NULL;
  }
  if (mb < 1 || mb * m > (1ull << 34)) {
    set_err("max_batch must be >= 1 and max_batch * map_size <= 16 GiB");
    return NULL;
  }
  kbz_plugin_t *p = plugin_alloc(mode, (size_t)m, (size_t)mb);
  if (!p) return NULL;
  unsigned long long pm = 0;
  if (mode == KBZ_MODE_DYNAMORIO && json_u64(options, "per_module_coverage", &pm) < 0) {
    set_err("bad options (per_module_coverage must be an integer)");
    plugin_free(p);
    return NULL;
  }
  if (pm) {  /* dynamorio_instrumentation.c:1048-1063 */
    size_t n = 0;
    int bad = 0;
    char **raw = json_array(options, "coverage_modules", &n, &bad);
    if (bad || !n) {
      free_strings(raw, n);
      set_err("No Coverage Module selected, please specify one with the coverage_modules option.");
      plugin_free(p);
      return NULL;
    }
    char **names = (char **)calloc(n, sizeof(char *));
    for (size_t i = 0; names && i < n; i++) names[i] = json_unquote(raw[i]);
    free_strings(raw, n);
    int ok = names != NULL;
    for (size_t i = 0; ok && i < n; i++) ok = names[i] && *names[i];
    if (!ok) {
      free_strings(names, n);
      set_err("coverage_modules must be an array of module names");
      plugin_free(p);
      return NULL;
    }
    if (plugin_modules(p, names, n)) {
      plugin_free(p);
      return NULL;
    }
    char *dir = json_str(options, "ignore_bytes_dir");  /* :802-814: <dir>/<module>.dat */
    for (size_t i = 0; dir && i < n; i++) {
      char path[4096];
      snprintf(path, sizeof(path), "%s/%s.dat", dir, names[i]);
      FILE *f = fopen(path, "rb");
      if (!f) continue;  /* a module without a file has no ignore bytes */
      fclose(f);
      if (!(p->mignore[i] = load_ignore_file(path, p->map_size))) {
        free(dir);
        plugin_free(p);
        return NULL;
      }
    }
    free(dir);
    return p;
  }
  char *ign = mode == KBZ_MODE_DYNAMORIO ? json_str(options, "ignore_bytes_file") : NULL;
  if (ign) {
    const int rc = load_ignore(p, ign);
    free(ign);
    if (rc) {
      plugin_free(p);
      return NULL;
    }
  }
  return p;
}

/* a fresh state with the same configuration (merge results) */
static kbz_plugin_t *plugin_clone_config(const kbz_plugin_t *src) {
  kbz_plugin_t *p = plugin_alloc(src->mode, src->map_size, src->max_batch);
  if (p && src->per_module) {
    char **names = (char **)calloc(src->nmod, sizeof(char *));
    for (size_t i = 0; names && i < src->nmod; i++) names[i] = strdup(src->mod_names[i]);
    int ok = names && !plugin_modules(p, names, src->nmod);
    for (size_t i = 0; ok && i < src->nmod; i++) {
      ok = names[i] != NULL;
      if (ok && src->mignore[i]) {
        ok = (p->mignore[i] = (uint8_t *)malloc(src->map_size)) != NULL;
        if (ok) memcpy(p->mignore[i], src->mignore[i], src->map_size);
      }
    }
    if (!ok) {
      if (names && !p->mod_names) free_strings(names, src->nmod);
      plugin_free(p);
      set_err("out of host memory");
      return NULL;
    }
    return p;
  }
  if (p && src->ignore) {
    p->ignore = (uint8_t *)malloc(src->map_size);
    if (!p->ignore) {
      plugin_free(p);
      set_err("out of host memory");
      return NULL;
    }
    memcpy(p->ignore, src->ignore, src->map_size);
  }
  return p;
}

/* ---- GPU side ------------------------------------------------------------------------------ */
static int ensure_module_ctxs(kbz_plugin_t *p) {
  const size_t m = p->map_size;
  uint8_t *v3 = (uint8_t *)malloc(3 * m);
  if (!v3) {
    set_err("out of host memory");
    return -1;
  }
  memset(v3, 0xff, 3 * m);
  for (size_t i = 0; i < p->nmod; i++) {
    if (p->mctx[i]) continue;
    p->mctx[i] = kbz_ctx_create(m, KBZ_MODE_DYNAMORIO, p->max_batch);
    memcpy(v3, p->mvirgin + i * m, m);
    if (!p->mctx[i] || kbz_set_virgin(p->mctx[i], v3) ||
        kbz_set_last_hash(p->mctx[i], p->mlast[i]) ||
        (p->mignore[i] && kbz_set_ignore(p->mctx[i], p->mignore[i]))) {
      set_err("GPU context (module %s): %s", p->mod_names[i], kbz_last_error());
      if (p->mctx[i]) kbz_ctx_destroy(p->mctx[i]);
      p->mctx[i] = NULL;
      free(v3);
      return -1;
    }
  }
  free(v3);
  return 0;
}

static int ensure_ctx(kbz_plugin_t *p) {
  if (p->per_module) return ensure_module_ctxs(p);
  if (p->ctx) return 0;
  p->ctx = kbz_ctx_create(p->map_size, p->mode, p->max_batch);
  if (!p->ctx) {
    set_err("GPU context: %s", kbz_last_error());
    return -1;
  }
  if (kbz_set_virgin(p->ctx, p->virgin) || kbz_set_last_hash(p->ctx, p->last_hash) ||
      (p->ignore && kbz_set_ignore(p->ctx, p->ignore))) {
    set_err("GPU state upload: %s", kbz_last_error());
    kbz_ctx_destroy(p->ctx);
    p->ctx = NULL;
    return -1;
  }
  return 0;
}

static int sync_mirror(kbz_plugin_t *p) {
  if (!p->mirror_stale) return 0;
  if (p->per_module) {
    const size_t m = p->map_size;
    uint8_t *v3 = (uint8_t *)malloc(3 * m);
    if (!v3) {
      set_err("out of host memory");
      return -1;
    }
    for (size_t i = 0; i < p->nmod; i++) {
      if (!p->mctx[i]) continue;
      if (kbz_get_virgin(p->mctx[i], v3) || kbz_get_last_hash(p->mctx[i], &p->mlast[i])) {
        set_err("GPU state download: %s", kbz_last_error());
        free(v3);
        return -1;
      }
      memcpy(p->mvirgin + i * m, v3, m);
    }
    free(v3);
    p->mirror_stale = 0;
    return 0;
  }
  if (!p->ctx) return 0;
  if (kbz_get_virgin(p->ctx, p->virgin) || kbz_get_last_hash(p->ctx, &p->last_hash)) {
    set_err("GPU state download: %s", kbz_last_error());
    return -1;
  }
  p->mirror_stale = 0;
  return 0;
}

/* Triage the queued execs (the acquired ring slot) as one ordered batch and wait for it.  A
 * batch of at most 64 execs is read by the GPU straight from the pinned slot (no DMA). */
static int plugin_flush(kbz_plugin_t *p) {
  if (!p->q_rows) return 0;
  p->mirror_stale = 1;
  const size_t n = p->q_n;
  p->q_rows = NULL;
  p->q_n = 0;
  if (p->per_module) {  /* has_new_coverage_per_module over the batch */
    size_t offs[p->nmod];
    for (size_t i = 0; i < p->nmod; i++) offs[i] = i * p->map_size;
    if (kbz_triage_modules_host(p->mctx, p->nmod, p->mq, n, p->nmod * p->map_size, offs,
                                p->mq_outcome, p->r_mhnb, p->r_hnb)) {
      set_err("GPU triage: %s", kbz_last_error());
      return -1;
    }
    for (size_t i = 0; i < p->nmod; i++) p->mnew[i] = p->r_mhnb[i * n + n - 1] != 0;
  } else if (kbz_ring_submit(p->ctx, n, 1, p->r_hnb, NULL, NULL, 0) || kbz_ring_flush(p->ctx)) {
    set_err("GPU triage: %s", kbz_last_error());
    return -1;
  }
  p->last_path_was_new = p->r_hnb[n - 1] != 0;
  p->r_base = p->q_base;
  p->r_n = n;
  p->q_base += (long)n;
  return 0;
}

static long plugin_record(kbz_plugin_t *p, const uint8_t *trace, int fuzz_result) {
  if (!p || !trace) {
    set_err("null argument");
    return -1;
  }
  if (fuzz_result != KBZ_PLUGIN_FUZZ_NONE && fuzz_result != KBZ_PLUGIN_FUZZ_HANG &&
      fuzz_result != KBZ_PLUGIN_FUZZ_CRASH) {
    set_err("fuzz_result must be FUZZ_NONE, FUZZ_HANG or FUZZ_CRASH");
    return -1;
  }
  if (p->q_rows && p->q_n == p->q_cap && plugin_flush(p)) return -1;
  if (p->per_module && !p->q_rows) {  /* module maps back to back: nmod * map_size bytes */
    if (ensure_ctx(p)) return -1;
    p->q_rows = p->mq;
    p->q_outcome = p->mq_outcome;
    p->q_cap = p->max_batch;
  }
  if (!p->q_rows) {  /* the exec's trace goes straight into pinned memory */
    if (ensure_ctx(p)) return -1;
    if (kbz_ring_acquire(p->ctx, &p->q_rows, &p->q_outcome, &p->q_cap)) {
      p->q_rows = NULL;
      set_err("GPU ring: %s", kbz_last_error());
      return -1;
    }
    if (p->q_cap > p->max_batch) p->q_cap = p->max_batch;
  }
  const size_t row = (p->per_module ? p->nmod : 1) * p->map_size;
  memcpy(p->q_rows + p->q_n * row, trace, row);
  /* the KBZ_FUZZ_* outcomes of kbz_triage.h use the same numbering */
  p->q_outcome[p->q_n] = (int8_t)fuzz_result;
  p->last_ticket = p->q_base + (long)p->q_n++;
  p->last_fuzz_result = fuzz_result;
  return p->last_ticket;
}

static int plugin_result(kbz_plugin_t *p, long ticket) {
  if (!p || ticket < 0) {
    set_err("no exec recorded");
    return -1;
  }
  if (ticket >= p->q_base && plugin_flush(p)) return -1;
  if (ticket < p->r_base || ticket >= p->r_base + (long)p->r_n) {
    set_err("exec %ld is outside the last triaged window [%ld, %ld)", ticket, p->r_base,
            p->r_base + (long)p->r_n);
    return -1;
  }
  return p->r_hnb[ticket - p->r_base];
}

static int plugin_triage_batch(kbz_plugin_t *p, const uint8_t *traces, size_t n, size_t stride,
                               const int8_t *outcome, uint8_t *hnb, uint32_t *h32,
                               uint64_t *x64) {
  const size_t row = p ? (p->per_module ? p->nmod : 1) * p->map_size : 0;
  if (!p || (n && !traces) || stride < row) {
    set_err("bad arguments (null traces or stride < the exec's map bytes)");
    return -1;
  }
  if (plugin_flush(p) || ensure_ctx(p)) return -1; /* queued execs come first */
  p->mirror_stale = 1;
  if (p->per_module) {  /* hnb = the exec's result over all modules (0/1) */
    if (h32 || x64) {
      set_err("per_module_coverage: hashes are per module, not per exec");
      return -1;
    }
    size_t offs[p->nmod];
    for (size_t i = 0; i < p->nmod; i++) offs[i] = i * p->map_size;
    for (size_t lo = 0; lo < n; lo += p->max_batch) {
      const size_t cnt = n - lo < p->max_batch ? n - lo : p->max_batch;
      if (kbz_triage_modules_host(p->mctx, p->nmod, traces + lo * stride, cnt, stride, offs,
                                  outcome ? outcome + lo : NULL, p->r_mhnb,
                                  hnb ? hnb + lo : p->r_hnb)) {
        set_err("GPU triage: %s", kbz_last_error());
        return -1;
      }
      for (size_t i = 0; i < p->nmod; i++) p->mnew[i] = p->r_mhnb[i * cnt + cnt - 1] != 0;
    }
    return 0;
  }
  const int want = (h32 ? KBZ_WANT_H32 : 0) | (x64 ? KBZ_WANT_X64 : 0);
  for (size_t lo = 0; lo < n; lo += p->max_batch) {
    const size_t cnt = n - lo < p->max_batch ? n - lo : p->max_batch;
    if (kbz_triage_batch_host(p->ctx, traces + lo * stride, cnt, stride,
                              outcome ? outcome + lo : NULL, hnb ? hnb + lo : NULL,
                              h32 ? h32 + lo : NULL, x64 ? x64 + lo : NULL, want)) {
      set_err("GPU triage: %s", kbz_last_error());
      return -1;
    }
  }
  return 0;
}

/* ---- state --------------------------------------------------------------------------------- */
static const char *const kMapNames[3] = {"virgin_bits", "virgin_tmout", "virgin_crash"};

static char *plugin_get_state(kbz_plugin_t *p) {
  if (!p) {
    set_err("null state");
    return NULL;
  }
  if (plugin_flush(p) || sync_mirror(p)) return NULL;
  const size_t m = p->map_size, k = p->per_module ? p->nmod : nmaps(p);
  size_t extra = 0;
  for (size_t i = 0; p->per_module && i < p->nmod; i++) extra += 2 * strlen(p->mod_names[i]) + 128;
  char *s = (char *)malloc(256 + k * (2 * m + 64) + extra);
  if (!s) {
    set_err("out of host memory");
    return NULL;
  }
  /* last_process_status: the FUZZ_* result of the last exec (dynamorio_get_state :1249) */
  char *o = s + sprintf(s, "{\"map_size\":%zu", m);
  if (p->mode == KBZ_MODE_DYNAMORIO)
    o += sprintf(o, ",\"last_process_status\":%d", p->last_ticket >= 0 ? p->last_fuzz_result : 0);
  if (p->per_module) {  /* dynamorio_get_state :1260-1275 */
    o += sprintf(o, ",\"modules\":[");
    for (size_t i = 0; i < p->nmod; i++) {
      o += sprintf(o, "%s{\"name\":\"", i ? "," : "");
      for (const char *c = p->mod_names[i]; *c; c++) {
        if (*c == '"' || *c == '\\') *o++ = '\\';
        *o++ = *c;
      }
      o += sprintf(o, "\",\"virgin_bits\":\"");
      o = put_hex(o, p->mvirgin + i * m, m);
      o += sprintf(o, "\",\"last_shm_hash\":%u,\"last_path_was_new\":%d}", p->mlast[i],
                   p->mnew[i]);
    }
    *o++ = ']';
  } else {
    for (size_t i = 0; i < k; i++) {
      o += sprintf(o, ",\"%s\":\"", kMapNames[i]);
      o = put_hex(o, p->virgin + i * m, m);
      *o++ = '"';
    }
    if (p->mode == KBZ_MODE_DYNAMORIO)
      o += sprintf(o, ",\"last_shm_hash\":%u,\"last_path_was_new\":%d", p->last_hash,
                   p->last_path_was_new);
  }
  *o++ = '}';
  *o = 0;
  return s;
}

static int set_state_modules(kbz_plugin_t *p, const char *json) {
  size_t n = 0;
  int bad = 0;
  char **objs = json_array(json, "modules", &n, &bad);
  if (bad || !objs) {
    free_strings(objs, n);
    set_err("state lacks a valid \"modules\" array");
    return 1;
  }
  const size_t m = p->map_size;
  uint8_t *v = (uint8_t *)malloc(p->nmod * m);
  uint32_t *last = (uint32_t *)malloc(p->nmod * sizeof(uint32_t));
  uint8_t *nw = (uint8_t *)malloc(p->nmod);
  int rc = (!v || !last || !nw) ? (set_err("out of host memory"), 1) : 0;
  if (!rc) {
    memcpy(v, p->mvirgin, p->nmod * m);
    memcpy(last, p->mlast, p->nmod * sizeof(uint32_t));
    memcpy(nw, p->mnew, p->nmod);
  }
  for (size_t j = 0; !rc && j < n; j++) {  /* dynamorio_set_state :1330-1349: match by name */
    char *name = json_str(objs[j], "name");
    const long i = name ? module_index(p, name) : -1;
    unsigned long long h = 0, lw = 0;
    if (i < 0) {
      set_err("state module %s is not a coverage module", name ? name : "(unnamed)");
      rc = 1;
    } else if (json_hex(objs[j], "virgin_bits", v + (size_t)i * m, m) ||
               json_u64(objs[j], "last_shm_hash", &h) < 0 ||
               json_u64(objs[j], "last_path_was_new", &lw) < 0) {
      set_err("state module %s lacks valid virgin_bits / last_shm_hash", name);
      rc = 1;
    } else {
      last[i] = (uint32_t)h;
      nw[i] = lw != 0;
    }
    free(name);
  }
  uint8_t *v3 = rc ? NULL : (uint8_t *)malloc(3 * m);
  if (!rc && !v3) rc = (set_err("out of host memory"), 1);
  for (size_t i = 0; !rc && i < p->nmod; i++) {
    if (!p->mctx[i]) continue;
    memset(v3, 0xff, 3 * m);
    memcpy(v3, v + i * m, m);
    if (kbz_set_virgin(p->mctx[i], v3) || kbz_set_last_hash(p->mctx[i], last[i])) {
      set_err("GPU state upload: %s", kbz_last_error());
      rc = 1;
    }
  }
  free(v3);
  if (!rc) {
    memcpy(p->mvirgin, v, p->nmod * m);
    memcpy(p->mlast, last, p->nmod * sizeof(uint32_t));
    memcpy(p->mnew, nw, p->nmod);
    p->mirror_stale = 0;
  }
  free(v);
  free(last);
  free(nw);
  free_strings(objs, n);
  return rc;
}

static int plugin_set_state(kbz_plugin_t *p, const char *json) {
  if (!p || !json) {
    set_err("null argument");
    return 1;
  }
  unsigned long long m = 0, h = 0, lw = 0, ls = 0;
  if (json_u64(json, "map_size", &m) == 1 && m != p->map_size) {
    set_err("state map_size %llu does not match the plugin's %zu", m, p->map_size);
    return 1;
  }
  /* execs recorded before the new state was loaded belong to the old one */
  if (plugin_flush(p)) return 1;
  if (json_u64(json, "last_process_status", &ls) < 0) {
    set_err("bad last_process_status");
    return 1;
  }
  if (p->per_module) return set_state_modules(p, json);
  const size_t ms = p->map_size, k = nmaps(p);
  uint8_t *v = (uint8_t *)malloc(3 * ms);
  if (!v) {
    set_err("out of host memory");
    return 1;
  }
  memset(v, 0xff, 3 * ms);
  for (size_t i = 0; i < k; i++) {
    if (json_hex(json, kMapNames[i], v + i * ms, ms)) {
      set_err("state lacks a valid \"%s\" (%zu bytes as hex)", kMapNames[i], ms);
      free(v);
      return 1;
    }
  }
  if (p->mode == KBZ_MODE_DYNAMORIO && (json_u64(json, "last_shm_hash", &h) < 0 ||
                                        json_u64(json, "last_path_was_new", &lw) < 0)) {
    set_err("bad last_shm_hash / last_path_was_new");
    free(v);
    return 1;
  }
  if (p->ctx && (kbz_set_virgin(p->ctx, v) || kbz_set_last_hash(p->ctx, (uint32_t)h))) {
    set_err("GPU state upload: %s", kbz_last_error());
    free(v);
    return 1;
  }
  memcpy(p->virgin, v, 3 * ms);
  free(v);
  p->last_hash = (uint32_t)h;
  p->last_path_was_new = lw != 0;
  p->mirror_stale = 0;
  return 0;
}

static kbz_plugin_t *plugin_create(int mode, const char *options, const char *state) {
  kbz_plugin_t *p = plugin_from_options(mode, options);
  if (p && state && plugin_set_state(p, state)) {
    plugin_free(p);
    return NULL;
  }
  return p;
}

/* ---- merge --------------------------------------------------------------------------------- */
static kbz_plugin_t *plugin_merge_many(kbz_plugin_t **ps, size_t n) {
  if (!ps || !n || !ps[0]) {
    set_err("nothing to merge");
    return NULL;
  }
  for (size_t i = 0; i < n; i++) {
    int ok = ps[i] && ps[i]->mode == ps[0]->mode && ps[i]->map_size == ps[0]->map_size &&
             ps[i]->per_module == ps[0]->per_module && ps[i]->nmod == ps[0]->nmod;
    for (size_t j = 0; ok && j < ps[0]->nmod; j++)  /* dynamorio_merge :1190-1203 */
      ok = module_index(ps[i], ps[0]->mod_names[j]) >= 0;
    if (!ok) {
      set_err("states to merge must come from the same plugin with the same map_size and "
              "coverage modules");
      return NULL;
    }
    if (plugin_flush(ps[i]) || sync_mirror(ps[i])) return NULL;
  }
  const size_t m = ps[0]->map_size;
  const size_t row = ps[0]->per_module ? m : nmaps(ps[0]) * m;
  const size_t parts = ps[0]->per_module ? ps[0]->nmod : 1;
  uint8_t *rows = (uint8_t *)malloc(n * row);
  kbz_plugin_t *r = rows ? plugin_clone_config(ps[0]) : NULL;
  if (!r) {
    free(rows);
    if (!rows) set_err("out of host memory");
    return NULL;
  }
  for (size_t q = 0; q < parts; q++) {  /* one AND-fold per module (matched by name) */
    for (size_t i = 0; i < n; i++) {
      const uint8_t *src = ps[0]->per_module
                               ? ps[i]->mvirgin + (size_t)module_index(ps[i], r->mod_names[q]) * m
                               : ps[i]->virgin;
      memcpy(rows + i * row, src, row);
    }
    uint8_t *dst = r->per_module ? r->mvirgin + q * m : r->virgin;
    if (kbz_merge_and_host(dst, rows, n, row)) {
      set_err("GPU merge: %s", kbz_last_error());
      free(rows);
      plugin_free(r);
      return NULL;
    }
  }
  free(rows);
  r->last_hash = 0; /* dynamorio_merge :1215-1228; afl_merge starts all but the maps fresh */
  return r;
}

/* ---- merge of state files: the merger's file loop (merger/merger.c:79-99) as one GPU fold ---
 * Each file holds one state as get_state writes it.  Worker threads read and hex-decode the
 * files straight into the library's pinned staging slots (kbz_merge_and_fill), k maps of
 * map_size bytes per state back to back (k = 3 for afl_gpu, 1 for dynamorio_gpu, the number of
 * coverage modules with per_module_coverage, in coverage_modules order); the GPU folds one slot
 * while the next is decoded.  The result is what merging the created states pairwise gives:
 * the AND of the maps, everything else fresh (afl_merge :123-140, dynamorio_merge :1180-1231). */
static int8_t g_hexv[256];
static pthread_once_t g_hex_once = PTHREAD_ONCE_INIT;
static void hex_table_init(void) {
  for (int c = 0; c < 256; c++) g_hexv[c] = (int8_t)hexval((char)c);
}
/* n bytes from the 2n hex digits of the JSON string value at v (just past its opening quote) */
static int hex_decode(const char *v, uint8_t *out, size_t n) {
  for (size_t i = 0; i < n; i++) {
    const int hi = g_hexv[(uint8_t)v[2 * i]];  /* -1 for a non-digit, the NUL included */
    if (hi < 0) return -1;
    const int lo = g_hexv[(uint8_t)v[2 * i + 1]];
    if (lo < 0) return -1;
    out[i] = (uint8_t)(hi << 4 | lo);
  }
  return v[2 * n] == '"' ? 0 : -1;
}
static int json_hex_fast(const char *json, const char *key, uint8_t *out, size_t n) {
  const char *v = json_value(json, key);
  if (!v || *v != '"') return -1;
  return hex_decode(v + 1, out, n);
}

typedef struct {
  const kbz_plugin_t *cfg;   /* options of the merge (mode, map_size, modules) */
  const char *const *paths;
  size_t row;                /* bytes per state row */
  uint8_t *dst;              /* current slot */
  size_t first, count, next;
  pthread_mutex_t mu;
  int failed;
  char err[512];
} files_job_t;

static char *read_text_file(const char *path) {
  FILE *f = fopen(path, "rb");
  if (!f) return NULL;
  char *buf = NULL;
  if (fseek(f, 0, SEEK_END) == 0) {
    const long len = ftell(f);
    if (len > 0 && fseek(f, 0, SEEK_SET) == 0 && (buf = (char *)malloc((size_t)len + 1))) {
      if (fread(buf, 1, (size_t)len, f) != (size_t)len) {
        free(buf);
        buf = NULL;
      } else {
        buf[len] = 0;
      }
    }
  }
  fclose(f);
  return buf;
}

/* one file -> one row; returns 0 or writes a message to err */
static int decode_state_file(const files_job_t *j, const char *path, uint8_t *row, char *err,
                             size_t errn) {
  const kbz_plugin_t *c = j->cfg;
  const size_t m = c->map_size;
  char *text = read_text_file(path);
  if (!text) {
    snprintf(err, errn, "Could not read instrumentation file or empty instrumentation file: %s",
             path);
    return -1;
  }
  unsigned long long ms = 0;
  int rc = 0;
  if (json_u64(text, "map_size", &ms) == 1 && ms != m) {
    snprintf(err, errn, "%s: map_size %llu differs from the options' %zu", path, ms, m);
    rc = -1;
  } else if (c->per_module) {  /* dynamorio_set_state :1330-1349: modules matched by name */
    size_t n = 0;
    int bad = 0;
    char **objs = json_array(text, "modules", &n, &bad);
    uint8_t *seen = (uint8_t *)calloc(c->nmod, 1);
    if (bad || !objs || !seen) {
      snprintf(err, errn, "%s: state lacks a valid \"modules\" array", path);
      rc = -1;
    }
    for (size_t q = 0; !rc && q < n; q++) {
      char *name = json_str(objs[q], "name");
      const long i = name ? module_index(c, name) : -1;
      if (i < 0 || json_hex_fast(objs[q], "virgin_bits", row + (size_t)i * m, m)) {
        snprintf(err, errn, "%s: module %s is not a coverage module or lacks virgin_bits", path,
                 name ? name : "(unnamed)");
        rc = -1;
      } else {
        seen[i] = 1;
      }
      free(name);
    }
    for (size_t i = 0; !rc && i < c->nmod; i++)
      if (!seen[i]) {  /* dynamorio_merge :1190-1203 needs the same modules in every state */
        snprintf(err, errn, "%s: state lacks coverage module %s", path, c->mod_names[i]);
        rc = -1;
      }
    free(seen);
    free_strings(objs, n);
  } else {
    for (size_t i = 0; !rc && i < nmaps(c); i++)
      if (json_hex_fast(text, kMapNames[i], row + i * m, m)) {
        snprintf(err, errn, "%s: state lacks a valid \"%s\" (%zu bytes as hex)", path,
                 kMapNames[i], m);
        rc = -1;
      }
  }
  free(text);
  return rc;
}

static void *files_worker(void *arg) {
  files_job_t *j = (files_job_t *)arg;
  char err[512];
  for (;;) {
    pthread_mutex_lock(&j->mu);
    const size_t i = j->failed ? j->count : j->next++;
    pthread_mutex_unlock(&j->mu);
    if (i >= j->count) return NULL;
    if (decode_state_file(j, j->paths[j->first + i], j->dst + i * j->row, err, sizeof(err))) {
      pthread_mutex_lock(&j->mu);
      if (!j->failed) memcpy(j->err, err, sizeof(err));
      j->failed = 1;
      pthread_mutex_unlock(&j->mu);
      return NULL;
    }
  }
}

static int fill_from_files(void *user, uint8_t *dst, size_t first, size_t count) {
  files_job_t *j = (files_job_t *)user;
  j->dst = dst;
  j->first = first;
  j->count = count;
  j->next = 0;
  enum { kMaxThreads = 16 };
  pthread_t th[kMaxThreads];
  size_t nt = count < kMaxThreads ? count : kMaxThreads, started = 0;
  for (; started < nt; started++)
    if (pthread_create(&th[started], NULL, files_worker, j)) break;
  if (started == 0) files_worker(j);  /* no threads available: decode on the caller */
  for (size_t t = 0; t < started; t++) pthread_join(th[t], NULL);
  return j->failed;
}

static kbz_plugin_t *plugin_merge_files(int mode, const char *options, const char *const *paths,
                                        size_t n) {
  if (!paths || !n) {
    set_err("nothing to merge");
    return NULL;
  }
  for (size_t i = 0; i < n; i++)
    if (!paths[i]) {
      set_err("null path");
      return NULL;
    }
  kbz_plugin_t *r = plugin_from_options(mode, options);
  if (!r) return NULL;
  pthread_once(&g_hex_once, hex_table_init);
  const size_t k = r->per_module ? r->nmod : nmaps(r);
  files_job_t j;
  memset(&j, 0, sizeof(j));
  j.cfg = r;
  j.paths = paths;
  j.row = k * r->map_size;
  pthread_mutex_init(&j.mu, NULL);
  uint8_t *out = (uint8_t *)malloc(j.row);
  int rc = out ? kbz_merge_and_fill(out, n, j.row, fill_from_files, &j) : -1;
  pthread_mutex_destroy(&j.mu);
  if (rc) {
    if (!out) set_err("out of host memory");
    else if (j.failed) set_err("%s", j.err);
    else set_err("GPU merge: %s", kbz_last_error());
    free(out);
    plugin_free(r);
    return NULL;
  }
  memcpy(r->per_module ? r->mvirgin : r->virgin, out, j.row);
  free(out);
  return r;  /* last hashes 0, nothing queued: a fresh state with the merged maps */
}

static const char kHelpAfl[] =
    "afl_gpu - AFL bitmap triage (has_new_bits vs virgin_bits/tmout/crash) on the GPU\n"
    "Options:\n"
    "  map_size              Trace map size in bytes (default 65536)\n"
    "  max_batch             Execs triaged per GPU batch (default 4096)\n";
static const char kHelpDr[] =
    "dynamorio_gpu - DynamoRIO/winafl triage (classify_counts, hash32, last-hash skip,\n"
    "                has_new_bits) on the GPU\n"
    "Options:\n"
    "  map_size              Trace map size in bytes (default 65536)\n"
    "  max_batch             Execs triaged per GPU batch (default 4096)\n"
    "  ignore_bytes_file     File of map_size bytes: nonzero bytes are ignored\n"
    "  per_module_coverage   1: one map per coverage module (record() takes the modules'\n"
    "                        maps back to back, in coverage_modules order)\n"
    "  coverage_modules      Array of module names (per_module_coverage)\n"
    "  ignore_bytes_dir      Directory of <module>.dat ignore bytes files (per_module_coverage)\n";

static int plugin_help(int mode, char **help_str) {
  if (!help_str) return -1;
  *help_str = strdup(mode == KBZ_MODE_DYNAMORIO ? kHelpDr : kHelpAfl);
  return *help_str ? 0 : -1;
}

/* ---- exported entry points ------------------------------------------------------------------ */
#define KBZ_PLUGIN_ENTRY_POINTS(P, MODE, NAME)                                                   \
  void *P##_create(char *options, char *state) { return plugin_create(MODE, options, state); } \
  void P##_cleanup(void *s) { plugin_free((kbz_plugin_t *)s); }                                \
  void *P##_merge(void *a, void *b) {                                                          \
    kbz_plugin_t *v[2] = {(kbz_plugin_t *)a, (kbz_plugin_t *)b};                               \
    return (a && b) ? plugin_merge_many(v, 2) : (set_err("null state"), (void *)NULL);         \
  }                                                                                            \
  void *P##_merge_many(void **s, size_t n) { return plugin_merge_many((kbz_plugin_t **)s, n); } \
  void *P##_merge_files(char *options, const char *const *paths, size_t n) {                   \
    return plugin_merge_files(MODE, options, paths, n);                                        \
  }                                                                                            \
  char *P##_get_state(void *s) { return plugin_get_state((kbz_plugin_t *)s); }                 \
  void P##_free_state(char *s) { free(s); }                                                    \
  int P##_set_state(void *s, char *json) { return plugin_set_state((kbz_plugin_t *)s, json); } \
  int P##_enable(void *s, pid_t *process, char *cmd_line, char *input, size_t input_length) {  \
    (void)s, (void)process, (void)cmd_line, (void)input, (void)input_length;                   \
    set_err(NAME ": process control stays with the host instrumentation; hand each exec's "    \
                 "trace to " #P "_record (INTEGRATION.md)");                                   \
    return -1;                                                                                 \
  }                                                                                            \
  int P##_is_process_done(void *s) {                                                           \
    (void)s;                                                                                   \
    set_err(NAME ": no target process is run by this plugin");                                 \
    return -1;                                                                                 \
  }                                                                                            \
  int P##_get_fuzz_result(void *s) {                                                           \
    kbz_plugin_t *p = (kbz_plugin_t *)s;                                                       \
    return (p && p->last_ticket >= 0) ? p->last_fuzz_result : KBZ_PLUGIN_FUZZ_ERROR;           \
  }                                                                                            \
  int P##_is_new_path(void *s) {                                                               \
    kbz_plugin_t *p = (kbz_plugin_t *)s;                                                       \
    const int r = p ? plugin_result(p, p->last_ticket) : -1;                                   \
    return r < 0 ? -1 : (r ? 1 : 0);                                                           \
  }                                                                                            \
  int P##_triage_batch(void *s, const uint8_t *t, size_t n, size_t stride, const int8_t *oc,   \
                       uint8_t *hnb, uint32_t *h32, uint64_t *x64) {                           \
    return plugin_triage_batch((kbz_plugin_t *)s, t, n, stride, oc, hnb, h32, x64);            \
  }                                                                                            \
  int P##_help(char **help_str) { return plugin_help(MODE, help_str); }                        \
  long P##_record(void *s, const uint8_t *t, int fuzz_result) {                                \
    return plugin_record((kbz_plugin_t *)s, t, fuzz_result);                                   \
  }                                                                                            \
  int P##_result(void *s, long ticket) { return plugin_result((kbz_plugin_t *)s, ticket); }    \
  int P##_flush(void *s) { return s ? plugin_flush((kbz_plugin_t *)s) : -1; }

KBZ_PLUGIN_ENTRY_POINTS(kbz_afl_gpu, KBZ_MODE_AFL, "afl_gpu")
KBZ_PLUGIN_ENTRY_POINTS(kbz_dynamorio_gpu, KBZ_MODE_DYNAMORIO, "dynamorio_gpu")

#define KBZ_FILL_VTABLE(r, P)          \
  do {                                 \
    (r)->create = P##_create;          \
    (r)->cleanup = P##_cleanup;        \
    (r)->merge = P##_merge;            \
    (r)->get_state = P##_get_state;    \
    (r)->free_state = P##_free_state;  \
    (r)->set_state = P##_set_state;    \
    (r)->enable = P##_enable;          \
    (r)->is_new_path = P##_is_new_path; \
    (r)->get_fuzz_result = P##_get_fuzz_result; \
    (r)->is_process_done = P##_is_process_done; \
    (r)->triage_batch = P##_triage_batch; \
    (r)->merge_many = P##_merge_many;  \
  } while (0)

kbz_instrumentation_t *kbz_instrumentation_factory(const char *name) {
  if (!name) {
    set_err("null instrumentation name");
    return NULL;
  }
  kbz_instrumentation_t *r = (kbz_instrumentation_t *)calloc(1, sizeof(*r));
  if (!r) return NULL;
  if (!strcmp(name, "afl_gpu")) {
    KBZ_FILL_VTABLE(r, kbz_afl_gpu);
  } else if (!strcmp(name, "dynamorio_gpu")) {
    KBZ_FILL_VTABLE(r, kbz_dynamorio_gpu);
  } else {
    free(r);
    set_err("unknown instrumentation %s", name);
    return NULL;
  }
  return r;
}
