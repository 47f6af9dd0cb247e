// killerbeez_amd/csrc/kbz_set.hip -- GPU insert-if-absent set of 16-byte keys (kbz_set_* in
// include/kbz_triage.h): the unique crash/hang table of BASELINE config 5.
//
// Semantics are the reference's hash-set novelty (linux_ipt_instrumentation.c:412-424:
// HASH_FIND, HASH_ADD when absent, "new" iff it was absent; entries iterate in insertion order,
// uthash 2.0.2), applied to an ordered batch: key j is new iff it is absent from the set AND
// from keys 0..j-1 of the batch; every new key is inserted with sequence number (batch base + j).
// Keys are 16 bytes like the IPT key {tip, tnt} (linux_ipt_instrumentation.h:19-22); for trace
// dedup the key is {XXH64 of the transformed trace, outcome class}.
//
// Per batch (stream-ordered, no host sync):
//   1. k_set_probe   every masked-in key probes the table (open addressing, linear probing;
//                    the table is only read in this launch): absent keys are candidates
//                    (is_new = 2), sort key = low word; other rows sort key = ~0;
//   2. radix sort    (hipcub, stable) of (low word, batch index) over all n rows, so equal low
//                    words keep batch order;
//   3. k_set_first   a candidate is the first occurrence of its key iff no earlier candidate in
//                    its equal-low-word run has the same high word (runs are 1 long except for
//                    repeated keys or 64-bit collisions) -> is_new = 1;
//   4. k_set_insert  first occurrences claim a free slot with one CAS on the slot's sequence
//                    word, then write the key; other candidates get is_new = 0.  All keys one
//                    launch inserts are distinct and absent, so no thread ever waits for another
//                    thread's key to land (a spin-wait between lanes of one wave would deadlock
//                    under SIMT divergence).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "kbz_triage.h"

namespace {

constexpr unsigned long long kEmpty = ~0ull;

struct Slot {
  unsigned long long seq;  // kEmpty = free, else insertion sequence number
  unsigned long long lo, hi;
};

__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}
__device__ __forceinline__ size_t home(unsigned long long lo, unsigned long long hi, size_t mask) {
  return (size_t)(mix64(lo ^ mix64(hi + 0x9e3779b97f4a7c15ULL)) & mask);
}

__global__ void k_set_probe(const Slot *tab, size_t mask, const unsigned long long *keys,
                            const uint8_t *in_mask, uint32_t n, unsigned long long *sort_lo,
                            uint32_t *sort_idx, uint8_t *is_new, uint32_t *overflow) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  sort_idx[j] = j;
  sort_lo[j] = kEmpty;
  is_new[j] = 0;
  if (in_mask && !in_mask[j]) return;
  const unsigned long long lo = keys[2 * j], hi = keys[2 * j + 1];
  for (size_t i = home(lo, hi, mask), step = 0; step <= mask; i = (i + 1) & mask, step++) {
    const Slot s = tab[i];
    if (s.seq == kEmpty) {  // absent: a candidate
      sort_lo[j] = lo;
      is_new[j] = 2;
      return;
    }
    if (s.lo == lo && s.hi == hi) return;  // already in the set
  }
  // every slot taken and none holds the key: it is new but cannot be inserted -- report it
  // (kbz_set_size fails) rather than calling it already seen
  atomicOr(overflow, 1u);
}

__global__ void k_set_first(const unsigned long long *s_lo, const uint32_t *s_idx, uint32_t n,
                            const unsigned long long *keys, uint8_t *is_new) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const uint32_t j = s_idx[p];
  if (!is_new[j]) return;  // not a candidate (reads 2 or 1: both mean candidate)
  const unsigned long long lo = s_lo[p], hi = keys[2 * j + 1];
  for (uint32_t q = p; q > 0 && s_lo[q - 1] == lo; q--) {
    const uint32_t i = s_idx[q - 1];
    if (is_new[i] && keys[2 * i + 1] == hi) return;  // an earlier occurrence of the key
  }
  is_new[j] = 1;
}

__global__ void k_set_insert(Slot *tab, size_t mask, const unsigned long long *keys, uint32_t n,
                             uint8_t *is_new, unsigned long long seq_base,
                             unsigned long long *count, uint32_t *overflow) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint8_t v = is_new[j];
  if (v == 2) is_new[j] = 0;  // a repeat of an earlier key of this batch
  if (v != 1) return;
  const unsigned long long lo = keys[2 * j], hi = keys[2 * j + 1];
  for (size_t i = home(lo, hi, mask), step = 0; step <= mask; i = (i + 1) & mask, step++) {
    if (atomicCAS(&tab[i].seq, kEmpty, seq_base + j) == kEmpty) {
      tab[i].lo = lo;
      tab[i].hi = hi;
      atomicAdd(count, 1ull);
      return;
    }
  }
  atomicOr(overflow, 1u);
}

// Merge support: a table's slots in insertion order.  Sorting (seq, slot) puts occupied slots
// first in the order they were inserted (free slots carry seq = kEmpty and sort last).
__global__ void k_slot_seq(const Slot *tab, uint32_t nslots, unsigned long long *seq_out,
                           uint32_t *idx_out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nslots) return;
  seq_out[i] = tab[i].seq;
  idx_out[i] = i;
}

__global__ void k_slot_gather(const Slot *tab, const uint32_t *idx, uint32_t nslots,
                              unsigned long long *keys_out, uint8_t *mask_out) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= nslots) return;
  const Slot s = tab[idx[p]];
  keys_out[2 * p] = s.lo;
  keys_out[2 * p + 1] = s.hi;
  mask_out[p] = s.seq != kEmpty;
}

thread_local std::string g_set_err;
int set_fail(const std::string &m) {
  g_set_err = m;
  return -1;
}
#define SET_TRY(expr)                                                                          \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess) return set_fail(std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

}  // namespace

struct kbz_set {
  int device = 0;
  Slot *tab = nullptr;
  size_t mask = 0;
  unsigned long long *count = nullptr;  // device
  uint32_t *overflow = nullptr;         // device
  unsigned long long next_seq = 0;      // host: sequence number of the next batch's row 0
};

extern "C" {

const char *kbz_set_last_error(void) { return g_set_err.c_str(); }

kbz_set_t *kbz_set_create(size_t capacity) {
  if (capacity == 0 || capacity > (1ull << 31)) {
    set_fail("capacity must be in [1, 2^31]");
    return nullptr;
  }
  size_t slots = 16;
  while (slots < 2 * capacity) slots <<= 1;  // load factor <= 1/2
  kbz_set *s = new kbz_set();
  (void)hipGetDevice(&s->device);
  s->mask = slots - 1;
  if (hipMalloc((void **)&s->tab, slots * sizeof(Slot)) != hipSuccess ||
      hipMalloc((void **)&s->count, sizeof(unsigned long long)) != hipSuccess ||
      hipMalloc((void **)&s->overflow, sizeof(uint32_t)) != hipSuccess ||
      hipMemset(s->tab, 0xff, slots * sizeof(Slot)) != hipSuccess ||
      hipMemset(s->count, 0, sizeof(unsigned long long)) != hipSuccess ||
      hipMemset(s->overflow, 0, sizeof(uint32_t)) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess) {
    set_fail("kbz_set_create: device allocation failed");
    kbz_set_destroy(s);
    return nullptr;
  }
  return s;
}

void kbz_set_destroy(kbz_set_t *s) {
  if (!s) return;
  if (s->tab) (void)hipFree(s->tab);
  if (s->count) (void)hipFree(s->count);
  if (s->overflow) (void)hipFree(s->overflow);
  delete s;
}

int kbz_set_insert_device(kbz_set_t *s, const uint64_t *keys, const uint8_t *mask, size_t n,
                          uint8_t *is_new_out, void *stream) {
  if (!s || (n && (!keys || !is_new_out))) return set_fail("null argument");
  if (n == 0) return 0;
  if (n > 0x7fffffffu) return set_fail("n must be < 2^31");
  hipStream_t st = (hipStream_t)stream;
  const unsigned long long *k = (const unsigned long long *)keys;
  const unsigned blocks = (unsigned)((n + 255) / 256);
  unsigned long long *lo_in = nullptr, *lo_out = nullptr;
  uint32_t *idx_in = nullptr, *idx_out = nullptr;
  void *tmp = nullptr;
  size_t tmp_bytes = 0;
  SET_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, lo_in, lo_out, idx_in, idx_out,
                                             (int)n, 0, 64, st));
  SET_TRY(hipMallocAsync((void **)&lo_in, n * 8, st));
  SET_TRY(hipMallocAsync((void **)&lo_out, n * 8, st));
  SET_TRY(hipMallocAsync((void **)&idx_in, n * 4, st));
  SET_TRY(hipMallocAsync((void **)&idx_out, n * 4, st));
  SET_TRY(hipMallocAsync(&tmp, tmp_bytes ? tmp_bytes : 1, st));
  hipLaunchKernelGGL(k_set_probe, dim3(blocks), dim3(256), 0, st, s->tab, s->mask, k, mask,
                     (uint32_t)n, lo_in, idx_in, is_new_out, s->overflow);
  SET_TRY(hipGetLastError());
  SET_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, lo_in, lo_out, idx_in, idx_out,
                                             (int)n, 0, 64, st));
  hipLaunchKernelGGL(k_set_first, dim3(blocks), dim3(256), 0, st, lo_out, idx_out, (uint32_t)n,
                     k, is_new_out);
  SET_TRY(hipGetLastError());
  hipLaunchKernelGGL(k_set_insert, dim3(blocks), dim3(256), 0, st, s->tab, s->mask, k,
                     (uint32_t)n, is_new_out, s->next_seq, s->count, s->overflow);
  SET_TRY(hipGetLastError());
  s->next_seq += n;
  SET_TRY(hipFreeAsync(lo_in, st));
  SET_TRY(hipFreeAsync(lo_out, st));
  SET_TRY(hipFreeAsync(idx_in, st));
  SET_TRY(hipFreeAsync(idx_out, st));
  SET_TRY(hipFreeAsync(tmp, st));
  return 0;
}

int kbz_set_insert_host(kbz_set_t *s, const uint64_t *keys, size_t n, uint8_t *is_new_out) {
  if (!s || (n && !keys)) return set_fail("null argument");
  if (n == 0) return 0;
  uint64_t *d_keys = nullptr;
  uint8_t *d_new = nullptr;
  int rc = set_fail("kbz_set_insert_host: device staging");
  if (hipMalloc((void **)&d_keys, n * 16) == hipSuccess &&
      hipMalloc((void **)&d_new, n) == hipSuccess &&
      hipMemcpy(d_keys, keys, n * 16, hipMemcpyHostToDevice) == hipSuccess) {
    rc = kbz_set_insert_device(s, d_keys, nullptr, n, d_new, nullptr);
    if (!rc && (hipDeviceSynchronize() != hipSuccess ||
                (is_new_out && hipMemcpy(is_new_out, d_new, n, hipMemcpyDeviceToHost) != hipSuccess)))
      rc = set_fail("kbz_set_insert_host: copy out");
  }
  if (d_keys) (void)hipFree(d_keys);
  if (d_new) (void)hipFree(d_new);
  return rc;
}

// Insert every key of src into dst, in src's insertion order (device-only, stream-ordered).
static int append_set(kbz_set_t *dst, const kbz_set_t *src, hipStream_t st) {
  const size_t nslots = src->mask + 1;
  if (nslots > 0x7fffffffu) return set_fail("source table too large");
  const unsigned blocks = (unsigned)((nslots + 255) / 256);
  unsigned long long *seq_in = nullptr, *seq_out = nullptr, *keys = nullptr;
  uint32_t *idx_in = nullptr, *idx_out = nullptr;
  uint8_t *occupied = nullptr, *is_new = nullptr;
  void *tmp = nullptr;
  size_t tmp_bytes = 0;
  SET_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, seq_in, seq_out, idx_in, idx_out,
                                             (int)nslots, 0, 64, st));
  SET_TRY(hipMallocAsync((void **)&seq_in, nslots * 8, st));
  SET_TRY(hipMallocAsync((void **)&seq_out, nslots * 8, st));
  SET_TRY(hipMallocAsync((void **)&idx_in, nslots * 4, st));
  SET_TRY(hipMallocAsync((void **)&idx_out, nslots * 4, st));
  SET_TRY(hipMallocAsync((void **)&keys, nslots * 16, st));
  SET_TRY(hipMallocAsync((void **)&occupied, nslots, st));
  SET_TRY(hipMallocAsync((void **)&is_new, nslots, st));
  SET_TRY(hipMallocAsync(&tmp, tmp_bytes ? tmp_bytes : 1, st));
  hipLaunchKernelGGL(k_slot_seq, dim3(blocks), dim3(256), 0, st, src->tab, (uint32_t)nslots,
                     seq_in, idx_in);
  SET_TRY(hipGetLastError());
  SET_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, seq_in, seq_out, idx_in, idx_out,
                                             (int)nslots, 0, 64, st));
  hipLaunchKernelGGL(k_slot_gather, dim3(blocks), dim3(256), 0, st, src->tab, idx_out,
                     (uint32_t)nslots, keys, occupied);
  SET_TRY(hipGetLastError());
  if (kbz_set_insert_device(dst, (const uint64_t *)keys, occupied, nslots, is_new, st)) return -1;
  SET_TRY(hipFreeAsync(seq_in, st));
  SET_TRY(hipFreeAsync(seq_out, st));
  SET_TRY(hipFreeAsync(idx_in, st));
  SET_TRY(hipFreeAsync(idx_out, st));
  SET_TRY(hipFreeAsync(keys, st));
  SET_TRY(hipFreeAsync(occupied, st));
  SET_TRY(hipFreeAsync(is_new, st));
  SET_TRY(hipFreeAsync(tmp, st));
  return 0;
}

kbz_set_t *kbz_set_merge(kbz_set_t *first, kbz_set_t *second, void *stream) {
  if (!first || !second) {
    set_fail("null argument");
    return nullptr;
  }
  // Each input holds at most slots/2 keys (kbz_set_create's load factor), so this fits both.
  kbz_set_t *m = kbz_set_create((first->mask + 1 + second->mask + 1) / 2);
  if (!m) return nullptr;
  hipStream_t st = (hipStream_t)stream;
  if (append_set(m, first, st) || append_set(m, second, st)) {
    std::string err = g_set_err;
    (void)hipStreamSynchronize(st);
    kbz_set_destroy(m);
    set_fail("kbz_set_merge: " + err);
    return nullptr;
  }
  return m;
}

int kbz_set_size(kbz_set_t *s, size_t *out) {
  if (!s || !out) return set_fail("null argument");
  SET_TRY(hipDeviceSynchronize());
  unsigned long long c = 0;
  uint32_t ov = 0;
  SET_TRY(hipMemcpy(&c, s->count, sizeof(c), hipMemcpyDeviceToHost));
  SET_TRY(hipMemcpy(&ov, s->overflow, sizeof(ov), hipMemcpyDeviceToHost));
  if (ov) return set_fail("set capacity exceeded: keys were dropped");
  *out = (size_t)c;
  return 0;
}

int kbz_set_keys(kbz_set_t *s, uint64_t *host_out, size_t cap, size_t *n_out) {
  if (!s || !n_out || (cap && !host_out)) return set_fail("null argument");
  size_t cnt = 0;
  if (kbz_set_size(s, &cnt)) return -1;
  std::vector<Slot> tab(s->mask + 1);
  SET_TRY(hipMemcpy(tab.data(), s->tab, tab.size() * sizeof(Slot), hipMemcpyDeviceToHost));
  std::vector<std::pair<unsigned long long, size_t>> order;
  order.reserve(cnt);
  for (size_t i = 0; i < tab.size(); i++)
    if (tab[i].seq != kEmpty) order.emplace_back(tab[i].seq, i);
  std::sort(order.begin(), order.end());
  const size_t m = std::min(cap, order.size());
  for (size_t r = 0; r < m; r++) {
    host_out[2 * r] = tab[order[r].second].lo;
    host_out[2 * r + 1] = tab[order[r].second].hi;
  }
  *n_out = order.size();
  return 0;
}

}  // extern "C"
