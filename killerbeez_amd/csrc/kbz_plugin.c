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

#if defined(__SSE2__)
#include <emmintrin.h>
#endif

/* An exec's trace into its pinned ring slot.  The CPU does not read the slot again before the GPU
 * does, so a cached copy's read-for-ownership of every destination line is wasted traffic (64 KiB
 * per exec): streaming stores skip it (plugin_flush fences them before the batch is submitted). */
static void copy_to_slot(uint8_t *dst, const uint8_t *src, size_t n) {
#if defined(__SSE2__)
  if (((uintptr_t)dst & 15) == 0 && n % 64 == 0) {
    for (size_t i = 0; i < n; i += 64) {
      const __m128i a = _mm_loadu_si128((const __m128i *)(src + i));
      const __m128i b = _mm_loadu_si128((const __m128i *)(src + i + 16));
      const __m128i c = _mm_loadu_si128((const __m128i *)(src + i + 32));
      const __m128i d = _mm_loadu_si128((const __m128i *)(src + i + 48));
      _mm_stream_si128((__m128i *)(dst + i), a);
      _mm_stream_si128((__m128i *)(dst + i + 16), b);
      _mm_stream_si128((__m128i *)(dst + i + 32), c);
      _mm_stream_si128((__m128i *)(dst + i + 48), d);
    }
    return;
  }
#endif
  memcpy(dst, src, n);
}
static void slot_copies_done(void) {
#if defined(__SSE2__)
  _mm_sfence();  /* the streaming stores are globally visible before the GPU is told to read */
#endif
}

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
  uint8_t *w_hnb;          /* results of the window being recorded (its submitted parts) */
  size_t q_off;            /* execs of this window already submitted as sub-batches */
  size_t sub_k;            /* afl_gpu: submit every sub_k execs of a small window (0: off) */
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
  /* get_module_info (dynamorio_instrumentation.c:1541-1573): the last triaged exec's raw maps
   * (all modules, back to back) and, computed on the GPU when first asked, its classified maps
   * (has_new_coverage leaves trace_bits classified, :1434) */
  uint8_t *last_raw, *last_cls;
  unsigned long gen, cls_gen;  /* windows triaged so far / window last_cls was computed for */
  int have_exec;           /* an exec was triaged (the reference's enable_called) */
  char **cov_names;        /* coverage_modules without per_module_coverage: names only */
  size_t ncov;
  /* dump_map_dir (dynamorio_instrumentation.c:1043, :1453-1458): every exec that is not a
   * last-hash skip writes its classified map to <dir>/<%08x hash>; dprev[m] = module m's last
   * hash before the next window */
  char *dump_dir;
  uint32_t *dprev;
  uint32_t *r_h32;         /* [nmod or 1][max_batch] hashes of the last window (dump_map_dir) */
  int restored_status;     /* last_process_status of a loaded state, until the next exec */
  /* dynamorio_gpu: the first exec stands for the reference's first dynamorio_enable, whose
   * setup_shm_and_pick_fuzzer_id(state, 1) resets the virgin maps (see dr_first_enable) */
  int dr_enabled;
  unsigned long dump_failures;  /* dump_map_dir / get_module_info bookkeeping that failed */
  int early_copy;          /* start large windows' host-to-device copy while recording (default
                            * 1; KBZ_PLUGIN_EARLY_COPY=0 for A/B runs) */
  /* option "devices" ("0,1,2,3"): windows and batches of at least shard_min execs (option
   * "shard_min", default 1024) are triaged sharded over these GPUs (kbz_triage_batch_devices,
   * one host thread per GPU); the plugin's own context keeps the smaller ones.  The state moves
   * through the host mirror around every sharded batch, so both always agree. */
  int *shard_dev;
  size_t shard_ndev, shard_min;
  kbz_mctx_t *shard;
} kbz_plugin_t;

static size_t nmaps(const kbz_plugin_t *p) { return p->mode == KBZ_MODE_DYNAMORIO ? 1 : 3; }

/* ---- JSON: the state / option formats of this file ------------------------------------------
 * A small validating reader: a key is looked up among the TOP-LEVEL members of an object only
 * (state objects nest module objects whose keys repeat the top-level names), values are skipped
 * with full syntax checks (strings with escapes, numbers, literals, nested objects / arrays up to
 * a depth limit), and strings are decoded (\" \\ \/ \b \f \n \r \t \uXXXX, surrogate pairs to
 * UTF-8).  Malformed text is "not found" / an error, never a read past the terminating NUL. */
enum { kJsonMaxDepth = 64 };
static const char *js_ws(const char *p) {
  while (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r') p++;
  return p;
}
static int js_hex4(const char *p, unsigned *out) {
  unsigned v = 0;
  for (int i = 0; i < 4; i++) {
    const char c = p[i];
    const int d = (c >= '0' && c <= '9') ? c - '0' : (c >= 'a' && c <= 'f') ? c - 'a' + 10
                  : (c >= 'A' && c <= 'F') ? c - 'A' + 10 : -1;
    if (d < 0) return -1;
    v = v << 4 | (unsigned)d;
  }
  *out = v;
  return 0;
}
/* past the closing quote of the string at p (*p == '"'), or NULL */
static const char *js_skip_string(const char *p) {
  for (p++; *p != '"'; p++) {
    if (!*p || (unsigned char)*p < 0x20) return NULL;
    if (*p == '\\') {
      p++;
      if (*p == 'u') {
        unsigned u;
        if (js_hex4(p + 1, &u)) return NULL;
        p += 4;
      } else if (!strchr("\"\\/bfnrt", *p) || !*p) {
        return NULL;
      }
    }
  }
  return p + 1;
}
/* past the JSON value at p, or NULL if it is malformed */
static const char *js_skip(const char *p, int depth) {
  p = js_ws(p);
  if (depth > kJsonMaxDepth) return NULL;
  if (*p == '"') return js_skip_string(p);
  if (*p == '{' || *p == '[') {
    const char close = *p == '{' ? '}' : ']';
    p = js_ws(p + 1);
    if (*p == close) return p + 1;
    for (;;) {
      if (close == '}') {
        if (*p != '"' || !(p = js_skip_string(p))) return NULL;
        p = js_ws(p);
        if (*p != ':') return NULL;
        p++;
      }
      if (!(p = js_skip(p, depth + 1))) return NULL;
      p = js_ws(p);
      if (*p == ',') {
        p = js_ws(p + 1);
        continue;
      }
      return *p == close ? p + 1 : NULL;
    }
  }
  if (!strncmp(p, "true", 4)) return p + 4;
  if (!strncmp(p, "false", 5)) return p + 5;
  if (!strncmp(p, "null", 4)) return p + 4;
  const char *q = p;
  if (*q == '-') q++;
  if (*q < '0' || *q > '9') return NULL;
  while (*q >= '0' && *q <= '9') q++;
  if (*q == '.') {
    q++;
    if (*q < '0' || *q > '9') return NULL;
    while (*q >= '0' && *q <= '9') q++;
  }
  if (*q == 'e' || *q == 'E') {
    q++;
    if (*q == '+' || *q == '-') q++;
    if (*q < '0' || *q > '9') return NULL;
    while (*q >= '0' && *q <= '9') q++;
  }
  return q;
}
/* the whole text is one well-formed JSON object (and nothing else but whitespace) */
static int json_valid_object(const char *json) {
  if (!json) return 0;
  const char *p = js_ws(json);
  if (*p != '{' || !(p = js_skip(p, 0))) return 0;
  return *js_ws(p) == 0;
}

/* the value of top-level member `key` of the object `json`, or NULL (absent or malformed).  Keys
 * are compared as written (the formats here never escape key characters). */
static const char *json_value(const char *json, const char *key) {
  if (!json) return NULL;
  const size_t kl = strlen(key);
  const char *p = js_ws(json);
  if (*p != '{') return NULL;
  p = js_ws(p + 1);
  if (*p == '}') return NULL;
  for (;;) {
    if (*p != '"') return NULL;
    const char *ks = p + 1, *ke = js_skip_string(p);
    if (!ke) return NULL;
    p = js_ws(ke);
    if (*p != ':') return NULL;
    const char *v = js_ws(p + 1);
    if ((size_t)(ke - 1 - ks) == kl && !memcmp(ks, key, kl)) return v;
    if (!(p = js_skip(v, 1))) return NULL;
    p = js_ws(p);
    if (*p != ',') return NULL;
    p = js_ws(p + 1);
  }
}

/* 1 found, 0 absent, -1 malformed (not a non-negative integer that fits) */
static int json_u64(const char *json, const char *key, unsigned long long *out) {
  const char *v = json ? json_value(json, key) : NULL;
  if (!v) return 0;
  if (*v < '0' || *v > '9') return -1;
  unsigned long long x = 0;
  for (; *v >= '0' && *v <= '9'; v++) {
    if (x > (~0ull - (unsigned)(*v - '0')) / 10) return -1;
    x = x * 10 + (unsigned)(*v - '0');
  }
  const char *e = js_ws(v);
  if (*e != ',' && *e != '}') return -1;
  *out = x;
  return 1;
}

/* the JSON string at s (*s == '"') -> malloc'd decoded UTF-8 text, NULL if malformed */
static char *json_unquote(const char *s) {
  if (!s || *s != '"') return NULL;
  const char *end = js_skip_string(s);
  if (!end) return NULL;
  char *o = (char *)malloc((size_t)(end - s) * 2 + 1);  /* \uXXXX -> at most 3 bytes */
  if (!o) return NULL;
  size_t n = 0;
  for (s++; s < end - 1; s++) {
    if (*s != '\\') {
      o[n++] = *s;
      continue;
    }
    s++;
    switch (*s) {
      case 'b': o[n++] = '\b'; break;
      case 'f': o[n++] = '\f'; break;
      case 'n': o[n++] = '\n'; break;
      case 'r': o[n++] = '\r'; break;
      case 't': o[n++] = '\t'; break;
      case 'u': {
        unsigned u, lo;
        js_hex4(s + 1, &u);
        s += 4;
        if (u >= 0xd800 && u < 0xdc00 && s[1] == '\\' && s[2] == 'u' && !js_hex4(s + 3, &lo) &&
            lo >= 0xdc00 && lo < 0xe000) {
          u = 0x10000 + ((u - 0xd800) << 10) + (lo - 0xdc00);
          s += 6;
        }
        if (!u || (u >= 0xd800 && u < 0xe000)) {  /* NUL or a lone surrogate: reject */
          free(o);
          return NULL;
        }
        if (u < 0x80) {
          o[n++] = (char)u;
        } else if (u < 0x800) {
          o[n++] = (char)(0xc0 | u >> 6);
          o[n++] = (char)(0x80 | (u & 0x3f));
        } else if (u < 0x10000) {
          o[n++] = (char)(0xe0 | u >> 12);
          o[n++] = (char)(0x80 | ((u >> 6) & 0x3f));
          o[n++] = (char)(0x80 | (u & 0x3f));
        } else {
          o[n++] = (char)(0xf0 | u >> 18);
          o[n++] = (char)(0x80 | ((u >> 12) & 0x3f));
          o[n++] = (char)(0x80 | ((u >> 6) & 0x3f));
          o[n++] = (char)(0x80 | (u & 0x3f));
        }
        break;
      }
      default: o[n++] = *s;  /* \" \\ \/ */
    }
  }
  o[n] = 0;
  return o;
}

static char *json_str(const char *json, const char *key) {
  return json_unquote(json ? json_value(json, key) : NULL);
}

/* The elements of top-level array member `key` as malloc'd strings of their raw JSON text
 * (quotes kept for strings, braces for objects); NULL + *n = 0 when the key is absent; *bad = 1
 * when it is not a well-formed array. */
static char **json_array(const char *json, const char *key, size_t *n, int *bad) {
  *n = 0;
  *bad = 0;
  const char *v = json ? json_value(json, key) : NULL;
  if (!v) return NULL;
  if (*v != '[' || !js_skip(v, 1)) {
    *bad = 1;
    return NULL;
  }
  char **items = NULL;
  const char *q = js_ws(v + 1);
  if (*q == ']') return (char **)calloc(1, sizeof(char *));  /* empty: non-NULL, n = 0 */
  for (;;) {
    const char *e = js_skip(q, 2);  /* well-formed: checked above */
    char **grown = (char **)realloc(items, (*n + 1) * sizeof(char *));
    if (!grown) break;
    items = grown;
    if (!(items[*n] = strndup(q, (size_t)(e - q)))) break;
    (*n)++;
    q = js_ws(e);
    if (*q == ']') return items;
    q = js_ws(q + 1);  /* ',' */
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
  if (p->shard) kbz_mctx_destroy(p->shard);
  free(p->shard_dev);
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
  free(p->last_raw);
  free(p->last_cls);
  free_strings(p->cov_names, p->ncov);
  free(p->dump_dir);
  free(p->dprev);
  free(p->r_h32);
  free(p->ignore);
  free(p->virgin);
  free(p->r_hnb);
  free(p->w_hnb);
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
  p->restored_status = 0;
  const char *ec = getenv("KBZ_PLUGIN_EARLY_COPY");
  p->early_copy = !ec || atoi(ec) != 0;
  p->virgin = (uint8_t *)malloc(3 * map_size);
  p->r_hnb = (uint8_t *)malloc(max_batch);
  p->w_hnb = (uint8_t *)malloc(max_batch);
  /* afl_gpu: parts of 8 execs (same-box A/B, profiles/r06/plugin/ab_subbatch.txt: windows of 16
   * and 64 -0.45 us per exec; parts of 4 were slower); KBZ_PLUGIN_SUBBATCH=0 turns it off */
  const char *sk = getenv("KBZ_PLUGIN_SUBBATCH");
  p->sub_k = sk ? (size_t)strtoul(sk, NULL, 0) : 8;
  if (p->sub_k > 64) p->sub_k = 64;  /* a sub-batch is read from the pinned slot (<= 64 rows) */
  if (!p->virgin || !p->r_hnb || !p->w_hnb) {
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

/* dump_map_dir: per-map last hashes and the window's hash buffer (frees p on failure) */
static kbz_plugin_t *plugin_dump_alloc(kbz_plugin_t *p) {
  if (!p->dump_dir) return p;
  const size_t k = p->per_module ? p->nmod : 1;
  p->dprev = (uint32_t *)calloc(k, sizeof(uint32_t));
  p->r_h32 = (uint32_t *)malloc(k * p->max_batch * sizeof(uint32_t));
  if (!p->dprev || !p->r_h32) {
    set_err("out of host memory");
    plugin_free(p);
    return NULL;
  }
  return p;
}

/* "devices": comma-separated GPU ordinals (repeats allowed: workers sharing a GPU),
 * "shard_min": the smallest batch that is sharded (>= 1).  Sharded windows are never split into
 * afl_gpu's early sub-batches, and their rows are not copied early: the whole window goes to the
 * workers at once. */
static int plugin_shard_options(kbz_plugin_t *p, const char *options) {
  unsigned long long smin = 1024;
  if (json_u64(options, "shard_min", &smin) < 0 || smin < 1) {
    set_err("bad options (shard_min must be an integer >= 1)");
    return -1;
  }
  p->shard_min = (size_t)smin;
  const int given = options && json_value(options, "devices");
  char *devs = given ? json_str(options, "devices") : NULL;
  if (given && !devs) {
    set_err("devices must be a string of comma-separated GPU ordinals");
    return -1;
  }
  if (!devs) return 0;
  size_t n = 1;
  for (const char *c = devs; *c; c++) n += *c == ',';
  p->shard_dev = (int *)calloc(n, sizeof(int));
  if (!p->shard_dev) {
    free(devs);
    set_err("out of host memory");
    return -1;
  }
  const char *c = devs;
  for (size_t i = 0; i < n; i++) {
    char *end = NULL;
    const long d = strtol(c, &end, 10);
    if (end == c || d < 0 || (*end && *end != ',')) {
      free(devs);
      set_err("devices must be a string of comma-separated GPU ordinals");
      return -1;
    }
    p->shard_dev[i] = (int)d;
    c = *end ? end + 1 : end;
  }
  free(devs);
  p->shard_ndev = n;
  p->sub_k = 0;
  p->early_copy = 0;
  return 0;
}

static kbz_plugin_t *plugin_from_options(int mode, const char *options) {
  unsigned long long m = 65536, mb = 4096;
  if (options && !json_valid_object(options)) {
    set_err("options are not a well-formed JSON object");
    return NULL;
  }
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
  char **names = NULL;
  size_t n = 0;
  if (mode == KBZ_MODE_DYNAMORIO) {  /* coverage_modules, dump_map_dir (:1043, :1050) */
    int bad = 0;
    char **raw = json_array(options, "coverage_modules", &n, &bad);
    names = bad ? NULL : (char **)calloc(n ? n : 1, sizeof(char *));
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
    if (json_value(options, "dump_map_dir") && !(p->dump_dir = json_str(options, "dump_map_dir"))) {
      free_strings(names, n);
      set_err("dump_map_dir must be a string");
      plugin_free(p);
      return NULL;
    }
  }
  if (pm && !n) {
    free_strings(names, n);
    set_err("No Coverage Module selected, please specify one with the coverage_modules option.");
    plugin_free(p);
    return NULL;
  }
  if (!pm) {  /* names only: get_module_info reports them (no per-module maps) */
    p->cov_names = names;
    p->ncov = n;
  }
  if (pm) {  /* dynamorio_instrumentation.c:1048-1063 */
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
    return plugin_dump_alloc(p);
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
  if (plugin_shard_options(p, options)) {
    plugin_free(p);
    return NULL;
  }
  return plugin_dump_alloc(p);
}

/* a fresh state with the same configuration (merge results) */
static kbz_plugin_t *plugin_clone_config(const kbz_plugin_t *src) {
  kbz_plugin_t *p = plugin_alloc(src->mode, src->map_size, src->max_batch);
  if (p && src->ncov) {
    p->cov_names = (char **)calloc(src->ncov, sizeof(char *));
    for (size_t i = 0; p->cov_names && i < src->ncov; i++) {
      if (!(p->cov_names[i] = strdup(src->cov_names[i]))) {
        free_strings(p->cov_names, i);
        p->cov_names = NULL;
        break;
      }
    }
    if (!p->cov_names) {
      plugin_free(p);
      set_err("out of host memory");
      return NULL;
    }
    p->ncov = src->ncov;
  }
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

/* A batch of the plugin's own execs sharded over the "devices" GPUs: the state goes to every
 * worker from the host mirror (the plugin's context is synced into it first), the sharded
 * protocol runs (kbz_triage_batch_devices: synchronous), and the resulting state comes back into
 * the mirror and the plugin's context.  Rows in pinned memory (the ring slot) go to the workers
 * by DMA straight from there. */
static int shard_batch(kbz_plugin_t *p, const uint8_t *rows, size_t n, size_t stride,
                       const int8_t *outcome, uint8_t *hnb, uint32_t *h32) {
  if (!p->shard) {
    p->shard = kbz_mctx_create(p->map_size, p->mode, p->max_batch, p->shard_dev, p->shard_ndev);
    if (!p->shard) {
      set_err("GPU shards: %s", kbz_last_error());
      return -1;
    }
    for (size_t w = 0; p->ignore && w < p->shard_ndev; w++)
      if (kbz_set_ignore(kbz_mctx_worker(p->shard, w), p->ignore)) {
        set_err("GPU shards (ignore bytes): %s", kbz_last_error());
        return -1;
      }
  }
  if (sync_mirror(p)) return -1;
  for (size_t w = 0; w < p->shard_ndev; w++) {
    kbz_ctx_t *c = kbz_mctx_worker(p->shard, w);
    if (kbz_set_virgin(c, p->virgin) || kbz_set_last_hash(c, p->last_hash)) {
      set_err("GPU shards (state upload): %s", kbz_last_error());
      return -1;
    }
  }
  const int want = h32 ? KBZ_WANT_H32 : 0;
  if (kbz_triage_batch_devices(p->shard, rows, n, stride, outcome, hnb, h32, want) ||
      kbz_mctx_get_virgin(p->shard, p->virgin) || kbz_mctx_get_last_hash(p->shard, &p->last_hash) ||
      kbz_set_virgin(p->ctx, p->virgin) || kbz_set_last_hash(p->ctx, p->last_hash)) {
    set_err("GPU shards: %s", kbz_last_error());
    p->mirror_stale = 1;
    return -1;
  }
  p->mirror_stale = 0;
  return 0;
}
static int shard_eligible(const kbz_plugin_t *p, size_t n, int want_x64) {
  return p->shard_ndev && !p->per_module && !want_x64 && n >= p->shard_min;
}

/* classify_counts (dynamorio_instrumentation.c:246-292: count_class_lookup8 over each byte) for
 * the side outputs that need one classified map at a time -- a dump_map_dir file, get_module_info's
 * info -- on the host: the novelty path itself never runs here. */
static uint8_t g_cls8[256];
static pthread_once_t g_cls_once = PTHREAD_ONCE_INIT;
static void cls_table_init(void) {
  for (int b = 0; b < 256; b++)
    g_cls8[b] = b == 0 ? 0 : b == 1 ? 1 : b == 2 ? 2 : b == 3 ? 4 : b <= 7 ? 8 : b <= 15 ? 16
                : b <= 31 ? 32 : b <= 127 ? 64 : 128;
}
static void classify_host(const uint8_t *in, uint8_t *out, size_t n) {
  pthread_once(&g_cls_once, cls_table_init);
  for (size_t i = 0; i < n; i++) out[i] = g_cls8[in[i]];
}

/* After a triaged window of n execs (rows of the k module maps back to back, `stride` apart):
 * remember the last exec's raw maps for get_module_info (dynamorio_instrumentation.c:1541-1573)
 * and, with dump_map_dir, write the classified map (has_new_coverage classifies trace_bits in
 * place, :1434) of every exec whose hash differs from the previous exec's -- the execs
 * has_new_coverage does not skip (:1450-1451) -- to <dir>/<%08x hash> (:1453-1458), in exec
 * order (a later exec with the same hash overwrites the file, as the reference's writes do).
 * p->r_h32 holds the window's hashes ([k][n]); each dumped map is classified as it is written.
 * Side outputs only: the window's results and tickets are already final when this runs, and a
 * failure here (a full disk, host memory) is counted, never reported as a triage failure -- the
 * reference ignores a failed write too. */
static void plugin_window_done(kbz_plugin_t *p, const uint8_t *rows, size_t n, size_t stride) {
  const size_t k = p->per_module ? p->nmod : 1, m = p->map_size, row = k * m;
  if (!n) return;
  p->have_exec = 1;
  p->gen++;
  if (p->per_module) {
    if (!p->last_raw && !(p->last_raw = (uint8_t *)malloc(row))) {
      p->dump_failures++;
      return;
    }
    memcpy(p->last_raw, rows + (n - 1) * stride, row);
  }
  if (!p->dump_dir) return;
  uint8_t *cls = (uint8_t *)malloc(m);
  if (!cls) {
    p->dump_failures++;
    return;
  }
  for (size_t q = 0; q < k; q++) {
    uint32_t prev = p->dprev[q];
    for (size_t j = 0; j < n; j++) {
      const uint32_t h = p->r_h32[q * n + j];
      if (h == prev) continue;  /* a last-hash skip: nothing is written */
      prev = h;
      char path[4096];
      snprintf(path, sizeof(path), "%s/%08x", p->dump_dir, h);
      classify_host(rows + j * stride + q * m, cls, m);
      FILE *f = fopen(path, "wb");
      if (!f || fwrite(cls, 1, m, f) != m) p->dump_failures++;
      if (f) fclose(f);
    }
    p->dprev[q] = prev;
  }
  free(cls);
}

/* The reference's first dynamorio_enable calls setup_shm_and_pick_fuzzer_id(state, 1)
 * (dynamorio_instrumentation.c:1380-1382), which resets virgin_bits to 0xff (:496-497) -- and,
 * with per_module_coverage, every module's map (:458-459, :474-475) -- even when create(options,
 * state) or set_state loaded them; last_shm_hash (and last_path_was_new) are kept.  Here the first
 * exec an instance records or triages stands for that enable.  A set_state after it keeps the
 * loaded maps (fuzzer_id is set by then), and a create + merge with no exec never resets.  The AFL
 * plugin keeps loaded maps: its setup_shm only fills maps it allocates (afl_instrumentation.c:
 * 553-559). */
static int dr_first_enable(kbz_plugin_t *p) {
  if (p->mode != KBZ_MODE_DYNAMORIO || p->dr_enabled) return 0;
  const size_t m = p->map_size;
  if (p->per_module) {
    memset(p->mvirgin, 0xff, p->nmod * m);
    uint8_t *v3 = (uint8_t *)malloc(3 * m);
    if (!v3) {
      set_err("out of host memory");
      return -1;
    }
    memset(v3, 0xff, 3 * m);
    for (size_t i = 0; i < p->nmod; i++) {
      if (p->mctx[i] && kbz_set_virgin(p->mctx[i], v3)) {
        set_err("GPU state upload: %s", kbz_last_error());
        free(v3);
        return -1;
      }
    }
    free(v3);
  } else {
    memset(p->virgin, 0xff, 3 * m);
    if (p->ctx && kbz_set_virgin(p->ctx, p->virgin)) {
      set_err("GPU state upload: %s", kbz_last_error());
      return -1;
    }
  }
  p->dr_enabled = 1;
  return 0;
}

/* Triage the queued execs (the acquired ring slot) as one ordered batch and wait for it.  A
 * batch of at most 64 execs is read by the GPU straight from the pinned slot (no DMA). */
static int plugin_flush(kbz_plugin_t *p) {
  if (!p->q_rows && !p->q_off) return 0;
  slot_copies_done();
  p->mirror_stale = 1;
  const size_t n = p->q_off + p->q_n;  /* the window: submitted sub-batches + the slot's rows */
  const size_t nq = p->q_n, off = p->q_off;
  const uint8_t *rows = p->q_rows;  /* the slot stays valid until the next record */
  p->q_rows = NULL;
  p->q_n = 0;
  p->q_off = 0;
  if (p->per_module) {  /* has_new_coverage_per_module over the batch */
    size_t offs[p->nmod];
    for (size_t i = 0; i < p->nmod; i++) offs[i] = i * p->map_size;
    if (kbz_triage_modules_host(p->mctx, p->nmod, p->mq, n, p->nmod * p->map_size, offs,
                                p->mq_outcome, p->r_mhnb, p->r_hnb, p->dump_dir ? p->r_h32 : NULL)) {
      set_err("GPU triage: %s", kbz_last_error());
      return -1;
    }
    for (size_t i = 0; i < p->nmod; i++) p->mnew[i] = p->r_mhnb[i * n + n - 1] != 0;
  } else if (!off && shard_eligible(p, nq, 0)) {
    /* the window sharded over the "devices" GPUs, read from the pinned slot; the slot is handed
     * back to the ring empty */
    if (shard_batch(p, rows, nq, p->map_size, p->q_outcome, p->w_hnb,
                    p->dump_dir ? p->r_h32 : NULL))
      return -1;
    if (kbz_ring_release(p->ctx) || kbz_ring_flush(p->ctx)) {
      set_err("GPU ring: %s", kbz_last_error());
      return -1;
    }
    uint8_t *t = p->r_hnb;
    p->r_hnb = p->w_hnb;
    p->w_hnb = t;
  } else {
    /* the slot's rows (after any sub-batches: AFL, no hashes), results into the window's buffer;
     * the flush delivers every part, then the window's buffer becomes the queryable one */
    if ((nq && kbz_ring_submit(p->ctx, nq, 1, p->w_hnb + off,
                               p->dump_dir ? p->r_h32 + off : NULL, NULL,
                               p->dump_dir ? KBZ_WANT_H32 : 0)) ||
        kbz_ring_flush(p->ctx)) {
      set_err("GPU triage: %s", kbz_last_error());
      return -1;
    }
    uint8_t *t = p->r_hnb;
    p->r_hnb = p->w_hnb;
    p->w_hnb = t;
  }
  /* the window's results and tickets first: the side outputs below cannot undo them */
  p->last_path_was_new = p->r_hnb[n - 1] != 0;
  p->r_base = p->q_base;
  p->r_n = n;
  p->q_base += (long)n;
  /* (sub-batched windows are AFL windows: plugin_window_done reads no rows for them) */
  plugin_window_done(p, off ? NULL : rows, n, (p->per_module ? p->nmod : 1) * p->map_size);
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
  if (((p->q_rows && p->q_n == p->q_cap) || p->q_off == p->max_batch) && plugin_flush(p))
    return -1;
  if (dr_first_enable(p)) return -1;
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
    if (p->q_cap > p->max_batch - p->q_off) p->q_cap = p->max_batch - p->q_off;
  }
  const size_t row = (p->per_module ? p->nmod : 1) * p->map_size;
  copy_to_slot(p->q_rows + p->q_n * row, trace, row);
  /* the KBZ_FUZZ_* outcomes of kbz_triage.h use the same numbering */
  p->q_outcome[p->q_n] = (int8_t)fuzz_result;
  p->last_ticket = p->q_base + (long)(p->q_off + p->q_n++);
  p->last_fuzz_result = fuzz_result;
  /* afl_gpu, small windows: every sub_k execs the slot's rows go to the GPU as their own batch
   * (one k_small launch reading them from the pinned slot) while the next execs are recorded in
   * the other slot; the result query then waits for the last part only */
  if (p->sub_k && p->q_n == p->sub_k && p->q_off + p->q_n <= 64 && p->mode == KBZ_MODE_AFL &&
      !p->per_module && !p->dump_dir) {
    slot_copies_done();
    if (kbz_ring_submit(p->ctx, p->q_n, 1, p->w_hnb + p->q_off, NULL, NULL, 0)) {
      set_err("GPU triage: %s", kbz_last_error());
      return -1;
    }
    p->q_off += p->q_n;
    p->q_n = 0;
    p->q_rows = NULL;
    return p->last_ticket;
  }
  /* every 64 execs past the first 128 (a window that will not fit the pinned-read path of
   * <= 64 rows): the rows recorded so far start their copy to the GPU now, overlapped with the
   * execs still to come, instead of all at the result query.  The copy is only started early;
   * if it cannot be, the flush copies those rows itself. */
  if (p->early_copy && !p->per_module && p->q_n >= 128 && (p->q_n & 63) == 0) {
    slot_copies_done();
    (void)kbz_ring_commit(p->ctx, p->q_n);
  }
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
  if (plugin_flush(p)) return -1; /* queued execs come first */
  if (n && dr_first_enable(p)) return -1;
  if (ensure_ctx(p)) return -1;
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
                                  hnb ? hnb + lo : p->r_hnb, p->dump_dir ? p->r_h32 : NULL)) {
        set_err("GPU triage: %s", kbz_last_error());
        return -1;
      }
      for (size_t i = 0; i < p->nmod; i++) p->mnew[i] = p->r_mhnb[i * cnt + cnt - 1] != 0;
      plugin_window_done(p, traces + lo * stride, cnt, stride);
    }
    return 0;
  }
  const int want = (h32 || p->dump_dir ? KBZ_WANT_H32 : 0) | (x64 ? KBZ_WANT_X64 : 0);
  for (size_t lo = 0; lo < n; lo += p->max_batch) {
    const size_t cnt = n - lo < p->max_batch ? n - lo : p->max_batch;
    uint32_t *hb = h32 ? h32 + lo : p->dump_dir ? p->r_h32 : NULL;
    if (shard_eligible(p, cnt, x64 != NULL)) {
      if (shard_batch(p, traces + lo * stride, cnt, stride, outcome ? outcome + lo : NULL,
                      hnb ? hnb + lo : p->r_hnb, hb))
        return -1;
    } else {
      p->mirror_stale = 1;  /* (a sharded chunk before this one left the mirror current) */
      if (kbz_triage_batch_host(p->ctx, traces + lo * stride, cnt, stride,
                                outcome ? outcome + lo : NULL, hnb ? hnb + lo : NULL, hb,
                                x64 ? x64 + lo : NULL, want)) {
        set_err("GPU triage: %s", kbz_last_error());
        return -1;
      }
    }
    if (p->dump_dir && hb != p->r_h32) memcpy(p->r_h32, hb, cnt * sizeof(uint32_t));
    plugin_window_done(p, traces + lo * stride, cnt, stride);
  }
  return 0;
}

/* get_module_info (dynamorio_instrumentation.c:1541-1573): asking for is_new or info finishes the
 * round first (finish_fuzz_round: here, triage the queued execs); -1 before any exec.  With
 * per_module_coverage: the module's last_path_was_new for the last exec, its name, its trace map
 * as has_new_coverage left it (classified, :1434; classified on the GPU when first asked, kept
 * until the next triaged exec) and map_size; 1 for an index past the modules.  Without it the
 * coverage_modules are reported with is_new 0 and no map, as the reference does (per-module
 * trace maps and last_path_was_new exist only with per_module_coverage, :453-470, :1488). */
static int plugin_module_info(kbz_plugin_t *p, int index, int *is_new, char **module_name,
                              char **info, int *size) {
  if (!p) {
    set_err("null state");
    return -1;
  }
  if (info || is_new) {
    if (plugin_flush(p)) return -1;
    if (!p->have_exec) {
      set_err("no exec has been triaged yet");
      return -1;
    }
  }
  const size_t m = p->map_size;
  if (p->per_module) {
    if (index < 0 || (size_t)index >= p->nmod) return 1;
    if (is_new) *is_new = p->mnew[index];
    if (module_name) *module_name = p->mod_names[index];
    if (info) {
      const size_t row = p->nmod * m;
      if (p->cls_gen != p->gen || !p->last_cls) {
        if (!p->last_raw || (!p->last_cls && !(p->last_cls = (uint8_t *)malloc(row)))) {
          set_err("out of host memory");
          return -1;
        }
        classify_host(p->last_raw, p->last_cls, row);  /* one exec's maps: no GPU round trip */
        p->cls_gen = p->gen;
      }
      *info = (char *)p->last_cls + (size_t)index * m;
    }
    if (size) *size = (int)m;
    return 0;
  }
  if (index < 0 || (size_t)index >= p->ncov) return 1;
  if (is_new) *is_new = 0;
  if (module_name) *module_name = p->cov_names[index];
  if (info) *info = NULL;
  if (size) *size = (int)m;
  return 0;
}

/* get_edges (dynamorio_instrumentation.c:1582-1606): edge lists exist only when the "edges"
 * option asked for them ahead of time, which this plugin does not offer: NULL, as the reference
 * returns without it. */
static kbz_instrumentation_edges_t *plugin_edges(kbz_plugin_t *p, int index) {
  (void)p, (void)index;
  set_err("no edge list: the edges option is not supported (trace maps only)");
  return NULL;
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
  for (size_t i = 0; p->per_module && i < p->nmod; i++) extra += 6 * strlen(p->mod_names[i]) + 128;
  char *s = (char *)malloc(256 + k * (2 * m + 64) + extra);
  if (!s) {
    set_err("out of host memory");
    return NULL;
  }
  /* last_process_status: the FUZZ_* result of the last exec (dynamorio_get_state :1249) */
  char *o = s + sprintf(s, "{\"map_size\":%zu", m);
  if (p->mode == KBZ_MODE_DYNAMORIO)
    o += sprintf(o, ",\"last_process_status\":%d",
                 p->last_ticket >= 0 ? p->last_fuzz_result : p->restored_status);
  if (p->per_module) {  /* dynamorio_get_state :1260-1275 */
    o += sprintf(o, ",\"modules\":[");
    for (size_t i = 0; i < p->nmod; i++) {
      o += sprintf(o, "%s{\"name\":\"", i ? "," : "");
      for (const char *c = p->mod_names[i]; *c; c++) {  /* JSON string escapes */
        if ((unsigned char)*c < 0x20) {
          o += sprintf(o, "\\u%04x", (unsigned char)*c);
          continue;
        }
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
  if (!json_valid_object(json)) {
    set_err("state is not a well-formed JSON object");
    return 1;
  }
  unsigned long long m = 0, h = 0, lw = 0, ls = 0;
  const int hm = json_u64(json, "map_size", &m);
  if (hm < 0 || (hm == 1 && m != p->map_size)) {
    set_err("state map_size does not match the plugin's %zu", p->map_size);
    return 1;
  }
  /* execs recorded before the new state was loaded belong to the old one */
  if (plugin_flush(p)) return 1;
  if (json_u64(json, "last_process_status", &ls) < 0 || ls > 0x7fffffff) {
    set_err("bad last_process_status");
    return 1;
  }
  if (p->per_module) {
    if (set_state_modules(p, json)) return 1;
    p->restored_status = (int)ls;  /* dynamorio_set_state :1325 */
    if (p->dprev) memcpy(p->dprev, p->mlast, p->nmod * sizeof(uint32_t));
    return 0;
  }
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
  p->restored_status = (int)ls;  /* dynamorio_set_state :1325 (reported until the next exec) */
  if (p->dprev) p->dprev[0] = p->last_hash;
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

typedef struct {             /* one merge_files call */
  const kbz_plugin_t *cfg;   /* options of the merge (mode, map_size, modules) */
  const char *const *paths;
  size_t row;                /* bytes per state row */
  size_t threads;            /* decoding threads per fill call */
  pthread_mutex_t mu;
  int failed;
  char err[512];
} files_ctx_t;
typedef struct {             /* one fill call: a slot of states [first, first + count) */
  files_ctx_t *ctx;
  uint8_t *dst;
  size_t first, count, next;
  pthread_mutex_t mu;
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
static int decode_state_file(const files_ctx_t *j, const char *path, uint8_t *row, char *err,
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
  if (!json_valid_object(text)) {
    snprintf(err, errn, "%s: not a well-formed JSON object", path);
    rc = -1;
  } else if (json_u64(text, "map_size", &ms) == 1 && ms != m) {
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
  files_ctx_t *c = j->ctx;
  char err[512];
  for (;;) {
    pthread_mutex_lock(&j->mu);
    const size_t i = j->next++;
    pthread_mutex_unlock(&j->mu);
    pthread_mutex_lock(&c->mu);
    const int failed = c->failed;
    pthread_mutex_unlock(&c->mu);
    if (i >= j->count || failed) return NULL;
    if (decode_state_file(c, c->paths[j->first + i], j->dst + i * c->row, err, sizeof(err))) {
      pthread_mutex_lock(&c->mu);
      if (!c->failed) memcpy(c->err, err, sizeof(err));
      c->failed = 1;
      pthread_mutex_unlock(&c->mu);
      return NULL;
    }
  }
}

/* kbz_merge_and_fill(_devices) callback: decode states [first, first + count) into dst.  With
 * several GPUs the workers call it concurrently for disjoint ranges: everything it changes is per
 * call, except the shared failure record (under ctx->mu). */
static int fill_from_files(void *user, uint8_t *dst, size_t first, size_t count) {
  files_job_t j;
  j.ctx = (files_ctx_t *)user;
  j.dst = dst;
  j.first = first;
  j.count = count;
  j.next = 0;
  pthread_mutex_init(&j.mu, NULL);
  enum { kMaxThreads = 16 };
  pthread_t th[kMaxThreads];
  size_t nt = j.ctx->threads < kMaxThreads ? j.ctx->threads : kMaxThreads, started = 0;
  if (nt > count) nt = count;
  for (; started < nt; started++)
    if (pthread_create(&th[started], NULL, files_worker, &j)) break;
  if (started == 0) files_worker(&j);  /* no threads available: decode on the caller */
  for (size_t t = 0; t < started; t++) pthread_join(th[t], NULL);
  pthread_mutex_destroy(&j.mu);
  pthread_mutex_lock(&j.ctx->mu);
  const int failed = j.ctx->failed;
  pthread_mutex_unlock(&j.ctx->mu);
  return failed;
}

/* merge_devices option: absent = the current GPU (one fold); an array of device ordinals (a device
 * may repeat) or "all" = every visible GPU: kbz_merge_and_fill_devices.  0 ok (*ndev 0 = absent),
 * -1 malformed. */
static int parse_merge_devices(const char *options, int **devs, size_t *ndev, int *all) {
  *devs = NULL;
  *ndev = 0;
  *all = 0;
  const char *v = options ? json_value(options, "merge_devices") : NULL;
  if (!v) return 0;
  if (*v == '"') {
    char *sv = json_unquote(v);
    const int ok = sv && !strcmp(sv, "all");
    free(sv);
    if (!ok) return -1;
    *all = 1;
    return 0;
  }
  size_t n = 0;
  int bad = 0;
  char **items = json_array(options, "merge_devices", &n, &bad);
  if (bad || !items || !n || n > 64) {
    free_strings(items, n);
    return -1;
  }
  int *d = (int *)malloc(n * sizeof(int));
  for (size_t i = 0; d && i < n; i++) {
    char *e = NULL;
    const long x = strtol(items[i], &e, 10);
    if (!e || *e || e == items[i] || x < 0 || x > 1024) {
      free(d);
      d = NULL;
    } else {
      d[i] = (int)x;
    }
  }
  free_strings(items, n);
  if (!d) return -1;
  *devs = d;
  *ndev = n;
  return 0;
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
  int *devs = NULL, all = 0;
  size_t ndev = 0;
  if (parse_merge_devices(options, &devs, &ndev, &all)) {
    set_err("merge_devices must be \"all\" or an array of GPU ordinals");
    plugin_free(r);
    return NULL;
  }
  pthread_once(&g_hex_once, hex_table_init);
  const size_t k = r->per_module ? r->nmod : nmaps(r);
  files_ctx_t j;
  memset(&j, 0, sizeof(j));
  j.cfg = r;
  j.paths = paths;
  j.row = k * r->map_size;
  /* 16 decoding threads in all, shared by the GPU workers */
  const size_t workers = all ? 8 : ndev ? ndev : 1;
  j.threads = workers >= 8 ? 2 : 16 / workers;
  pthread_mutex_init(&j.mu, NULL);
  uint8_t *out = (uint8_t *)malloc(j.row);
  int rc = -1;
  if (out && (all || ndev))  /* the node's GPUs: merger/merger.c's fold sharded across them */
    rc = kbz_merge_and_fill_devices(out, n, j.row, fill_from_files, &j, all ? NULL : devs,
                                    ndev, KBZ_EXCHANGE_AUTO, NULL);
  else if (out)
    rc = kbz_merge_and_fill(out, n, j.row, fill_from_files, &j);
  free(devs);
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
    "  max_batch             Execs triaged per GPU batch (default 4096)\n"
    "  merge_devices         merge_files: \"all\" or an array of GPU ordinals to shard the\n"
    "                        fold over (default: the current GPU)\n";
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
    "  ignore_bytes_dir      Directory of <module>.dat ignore bytes files (per_module_coverage)\n"
    "  dump_map_dir          Directory: every exec that is not a last-hash skip writes its\n"
    "                        classified map to <dir>/<hash32 as %08x>\n"
    "  merge_devices         merge_files: \"all\" or an array of GPU ordinals to shard the\n"
    "                        fold over (default: the current GPU)\n";

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

/* the DynamoRIO plugin's optional members (instrumentation_factory.c:53-54 binds them) */
int kbz_dynamorio_gpu_get_module_info(void *s, int index, int *is_new, char **module_name,
                                      char **info, int *size) {
  return plugin_module_info((kbz_plugin_t *)s, index, is_new, module_name, info, size);
}
kbz_instrumentation_edges_t *kbz_dynamorio_gpu_get_edges(void *s, int index) {
  return plugin_edges((kbz_plugin_t *)s, index);
}

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
    r->get_module_info = kbz_dynamorio_gpu_get_module_info;
    r->get_edges = kbz_dynamorio_gpu_get_edges;
  } else {
    free(r);
    set_err("unknown instrumentation %s", name);
    return NULL;
  }
  return r;
}
