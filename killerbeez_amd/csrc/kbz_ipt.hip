// killerbeez_amd/csrc/kbz_ipt.hip -- Intel-PT path keys on the GPU (kbz_ipt_* in
// include/kbz_triage.h): the hashing half of the reference's IPT novelty, batched.
//
// The reference hashes every exec's IPT packets while parsing them on the CPU
// (linux_ipt_instrumentation.c analyze_ipt :212-425): TNT bits go through add_tnt_to_hash
// (:132-156) into one streaming XXH64, TIP addresses through add_tip_to_hash (:163-189) into a
// second one, finish_tnt_hash (:115-124) closes the TNT stream, and the pair of digests
// {tip, tnt} (:409-416) is looked up / added in a uthash set (:418-424).  The packet parse stays
// on the CPU (it needs the perf IPT buffer and is sequential); what moves here:
//   host   the feeders, restated as appends to two 8-byte word streams per exec (XXH64's
//          streaming and one-shot forms agree on the concatenated input): TNT bits packed the
//          reference's way -- bit i of a packet byte contributes (byte & (1 << i%8)) << k, k =
//          bits already packed -- a word every 8 bits (the `num_bits == sizeof(tnt_bits)` flush,
//          :148), then the partial word and the total bit count; TIP addresses ASLR-adjusted
//          (:169-185);
//   device one XXH64 (seed 0, v0.6.5: xxhash.c:855) per stream for a whole batch of execs,
//          4 lanes per stream (one per accumulator lane of the 32-byte stripes), then the
//          set insert (kbz_set_insert_device: insert-if-absent in exec order, like :418-424).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "kbz_device.h"
#include "kbz_triage.h"

using namespace kbz;

namespace {

thread_local std::string g_ipt_err;
int ipt_fail(const std::string &m) {
  g_ipt_err = m;
  return -1;
}
#define IPT_TRY(expr)                                                                          \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess) return ipt_fail(std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

// XXH64 (seed 0) of every word stream r = words[off[r] .. off[r+1]) into out[2 r + slot]:
// 4 lanes per stream, lane a runs accumulator a over words 4 s + a of the full 32-byte stripes,
// lane 0 then merges the four and hashes the tail words (xxhash.c:760-853 without the 4- and
// 1-byte tails: every input is whole 8-byte words).
__global__ __launch_bounds__(256) void k_ipt_xxh64(const uint64_t *words, const uint64_t *off,
                                                   uint32_t n, uint64_t *out, int slot) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t r = t >> 2, a = t & 3;
  const bool live = r < n;
  const uint64_t lo = live ? off[r] : 0, nw = live ? off[r + 1] - lo : 0;
  const uint64_t stripes = nw >= 4 ? nw / 4 : 0;
  const uint64_t init[4] = {kXP1 + kXP2, kXP2, 0, 0 - kXP1};
  uint64_t acc = init[a];
  const uint64_t *w = words + lo + a;
  for (uint64_t s = 0; s < stripes; s++) acc = xx_round(acc, w[4 * s]);
  // the row's 4 lanes are 4 consecutive lanes of this wave
  const uint64_t v1 = __shfl(acc, (threadIdx.x & ~3u) + 0), v2 = __shfl(acc, (threadIdx.x & ~3u) + 1);
  const uint64_t v3 = __shfl(acc, (threadIdx.x & ~3u) + 2), v4 = __shfl(acc, (threadIdx.x & ~3u) + 3);
  if (!live || a) return;
  uint64_t h;
  if (stripes) {
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h = xx_merge(h, v1);
    h = xx_merge(h, v2);
    h = xx_merge(h, v3);
    h = xx_merge(h, v4);
  } else {
    h = kXP5;
  }
  h += nw * 8;
  for (uint64_t i = 4 * stripes; i < nw; i++) {
    h ^= xx_round(0, words[lo + i]);
    h = rotl64(h, 27) * kXP1 + kXP4;
  }
  out[2 * (size_t)r + slot] = xx_avalanche(h);
}

}  // namespace

struct kbz_ipt_batch {
  // the two word streams of every closed exec (CSR) and of the exec being fed
  std::vector<uint64_t> tnt, tip, tnt_off{0}, tip_off{0};
  uint64_t bits = 0, nb = 0, total = 0;  // struct ipt_hash_state (linux_ipt_instrumentation.h)
  // ASLR normalisation (add_tip_to_hash :169-185)
  std::vector<uint64_t> lib_starts, lib_ends;
  std::vector<uint32_t> lib_hashes;
  uint64_t target_start = 0, target_end = 0;
  // device staging, grown on demand
  uint64_t *d_words = nullptr, *d_off = nullptr;
  size_t cap_words = 0, cap_off = 0;
  int device = 0;
};

extern "C" {

const char *kbz_ipt_last_error(void) { return g_ipt_err.c_str(); }

kbz_ipt_batch_t *kbz_ipt_batch_create(void) {
  kbz_ipt_batch *b = new kbz_ipt_batch();
  (void)hipGetDevice(&b->device);
  return b;
}

void kbz_ipt_batch_destroy(kbz_ipt_batch_t *b) {
  if (!b) return;
  if (b->d_words) (void)hipFree(b->d_words);
  if (b->d_off) (void)hipFree(b->d_off);
  delete b;
}

int kbz_ipt_set_ranges(kbz_ipt_batch_t *b, size_t n_libraries, const uint64_t *starts,
                       const uint64_t *ends, const uint32_t *library_hashes,
                       uint64_t target_start, uint64_t target_end) {
  if (!b || (n_libraries && (!starts || !ends || !library_hashes))) return ipt_fail("null argument");
  b->lib_starts.assign(starts, starts + n_libraries);
  b->lib_ends.assign(ends, ends + n_libraries);
  b->lib_hashes.assign(library_hashes, library_hashes + n_libraries);
  b->target_start = target_start;
  b->target_end = target_end;
  return 0;
}

int kbz_ipt_add_tnt(kbz_ipt_batch_t *b, const uint8_t *tnt_bits, int num_bits) {
  if (!b || (num_bits > 0 && !tnt_bits)) return ipt_fail("null argument");
  if (num_bits < 0) return ipt_fail("kbz_ipt_add_tnt: num_bits < 0 (no stop bit in the packet)");
  for (int i = 0; i < num_bits; i++) {
    b->bits |= (uint64_t)((tnt_bits[i / 8] & (1u << (i % 8))) << b->nb);
    if (++b->nb == 8) {  // :148 -- sizeof(uint64_t) bits, i.e. every 8
      b->tnt.push_back(b->bits);
      b->bits = b->nb = 0;
    }
  }
  b->total += (uint64_t)num_bits;
  return 0;
}

int kbz_ipt_add_tip(kbz_ipt_batch_t *b, uint64_t tip) {
  if (!b) return ipt_fail("null argument");
  uint64_t adj = tip;
  if (!b->lib_starts.empty()) {
    for (size_t i = 0; i < b->lib_starts.size(); i++)
      if (b->lib_starts[i] <= tip && tip < b->lib_ends[i]) {
        adj = (tip - b->lib_starts[i]) | ((uint64_t)b->lib_hashes[i] << 32);
        break;
      }
  } else if (b->target_start <= tip && tip < b->target_end) {
    adj = tip - b->target_start;
  }
  b->tip.push_back(adj);
  return 0;
}

int kbz_ipt_end_exec(kbz_ipt_batch_t *b) {
  if (!b) return ipt_fail("null argument");
  if (b->nb) b->tnt.push_back(b->bits);  // finish_tnt_hash :117-121
  b->tnt.push_back(b->total);            // :122-123
  b->tnt_off.push_back(b->tnt.size());
  b->tip_off.push_back(b->tip.size());
  b->bits = b->nb = b->total = 0;        // the next exec starts from analyze_ipt's reset
  return 0;
}

size_t kbz_ipt_execs(kbz_ipt_batch_t *b) { return b ? b->tnt_off.size() - 1 : 0; }

int kbz_ipt_hash_device(kbz_ipt_batch_t *b, uint64_t *keys_out, void *stream) {
  if (!b) return ipt_fail("null argument");
  const size_t n = b->tnt_off.size() - 1;
  if (!n) return 0;
  if (!keys_out) return ipt_fail("null argument");
  if (n > 0x3fffffffu) return ipt_fail("kbz_ipt_hash_device: too many execs in one batch");
  int cur = 0;
  (void)hipGetDevice(&cur);
  if (cur != b->device) IPT_TRY(hipSetDevice(b->device));
  hipStream_t s = (hipStream_t)stream;
  const size_t nw = std::max(b->tnt.size(), b->tip.size()), no = n + 1;
  if (nw > b->cap_words) {
    if (b->d_words) IPT_TRY(hipFree(b->d_words));
    b->d_words = nullptr;
    IPT_TRY(hipMalloc((void **)&b->d_words, 2 * nw * sizeof(uint64_t)));
    b->cap_words = nw;
  }
  if (no > b->cap_off) {
    if (b->d_off) IPT_TRY(hipFree(b->d_off));
    b->d_off = nullptr;
    IPT_TRY(hipMalloc((void **)&b->d_off, 2 * no * sizeof(uint64_t)));
    b->cap_off = no;
  }
  uint64_t *dw_tip = b->d_words, *dw_tnt = b->d_words + b->cap_words;
  uint64_t *do_tip = b->d_off, *do_tnt = b->d_off + b->cap_off;
  IPT_TRY(hipMemcpyAsync(dw_tip, b->tip.data(), b->tip.size() * 8, hipMemcpyHostToDevice, s));
  IPT_TRY(hipMemcpyAsync(dw_tnt, b->tnt.data(), b->tnt.size() * 8, hipMemcpyHostToDevice, s));
  IPT_TRY(hipMemcpyAsync(do_tip, b->tip_off.data(), no * 8, hipMemcpyHostToDevice, s));
  IPT_TRY(hipMemcpyAsync(do_tnt, b->tnt_off.data(), no * 8, hipMemcpyHostToDevice, s));
  IPT_TRY(hipStreamSynchronize(s));  // the host streams may be reused once this returns
  const unsigned blocks = (unsigned)((4 * n + 255) / 256);
  hipLaunchKernelGGL(k_ipt_xxh64, dim3(blocks), dim3(256), 0, s, dw_tip, do_tip, (uint32_t)n,
                     keys_out, 0);
  hipLaunchKernelGGL(k_ipt_xxh64, dim3(blocks), dim3(256), 0, s, dw_tnt, do_tnt, (uint32_t)n,
                     keys_out, 1);
  IPT_TRY(hipGetLastError());
  b->tnt.clear();
  b->tip.clear();
  b->tnt_off.assign(1, 0);
  b->tip_off.assign(1, 0);
  if (cur != b->device) (void)hipSetDevice(cur);
  return 0;
}

int kbz_ipt_triage(kbz_ipt_batch_t *b, kbz_set_t *set, uint64_t *keys_out, uint8_t *is_new_out) {
  if (!b || !set) return ipt_fail("null argument");
  const size_t n = b->tnt_off.size() - 1;
  if (!n) return 0;
  hipStream_t s = nullptr;
  uint64_t *d_keys = nullptr;
  uint8_t *d_new = nullptr;
  int rc = -1;
  do {
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc((void **)&d_keys, n * 16) != hipSuccess ||
        hipMalloc((void **)&d_new, n) != hipSuccess) {
      ipt_fail("kbz_ipt_triage: device staging");
      break;
    }
    if (kbz_ipt_hash_device(b, d_keys, s)) break;
    if (kbz_set_insert_device(set, d_keys, nullptr, n, d_new, s)) {
      ipt_fail(std::string("kbz_ipt_triage: ") + kbz_set_last_error());
      break;
    }
    if ((keys_out && hipMemcpyAsync(keys_out, d_keys, n * 16, hipMemcpyDeviceToHost, s)) ||
        (is_new_out && hipMemcpyAsync(is_new_out, d_new, n, hipMemcpyDeviceToHost, s)) ||
        hipStreamSynchronize(s) != hipSuccess) {
      ipt_fail("kbz_ipt_triage: copy out");
      break;
    }
    rc = 0;
  } while (0);
  if (s) (void)hipStreamSynchronize(s);
  if (d_keys) (void)hipFree(d_keys);
  if (d_new) (void)hipFree(d_new);
  if (s) (void)hipStreamDestroy(s);
  return rc;
}

}  // extern "C"
