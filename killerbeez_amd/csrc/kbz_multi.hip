// killerbeez_amd/csrc/kbz_multi.hip -- the merger fold over several GPUs of one node, from C.
//
// The reference merger is one C process folding client states pairwise (merger/merger.c:79-99:
// read_file + create + merge per state file, merge = afl_merge, afl_instrumentation.c:123-140,
// a byte-wise AND of the three virgin maps, merge_bitmaps :116-121).  BASELINE config 4 shards
// that fold across the GPUs of a node.  kbz_merge_and_fill_devices does it inside the caller's
// process, one host thread per worker:
//   1. worker w (device devices[w]) folds its contiguous share of the states with
//      kbz_merge_and_fill_device: the fill callback decodes states straight into pinned staging
//      slots on the worker's thread while the worker's GPU copies and AND-folds the previous slot,
//      so the host-side decoding of state files runs on ndev threads at once;
//   2. exchange of the partial folds.  RCCL has no bitwise-AND reduction, so either
//      RCCL:  one ncclAllGather of state_bytes per worker over comms from ncclCommInitAll (one
//             rank per distinct GPU), then a local AND of the ndev gathered rows on every device;
//      COPY:  peer (or, for workers sharing a GPU, device-local) copies of every partial into a
//             buffer on worker 0's device and one AND there;
//   3. worker 0's merged state goes to host memory.
// AND is commutative and associative, so any sharding gives the reference's result.
// librccl is loaded with dlopen the first time it is needed: the library has no link-time
// dependency on it, and an RCCL request fails loudly when it is absent.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "kbz_triage.h"

extern "C" void kbz__set_error(const char *msg);  // kbz_triage.hip

namespace {

int fail_multi(const std::string &msg) {
  kbz__set_error(msg.c_str());
  return -1;
}

struct Rccl {
  bool tried = false, ok = false;
  std::string why;
  decltype(&ncclCommInitAll) init_all = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclGetErrorString) err_str = nullptr;
};

Rccl &rccl() {
  static Rccl r;
  static std::mutex mu;
  std::lock_guard<std::mutex> g(mu);
  if (r.tried) return r;
  r.tried = true;
  void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    const char *e = dlerror();
    r.why = std::string("librccl not loadable: ") + (e ? e : "?");
    return r;
  }
  r.init_all = (decltype(r.init_all))dlsym(h, "ncclCommInitAll");
  r.all_gather = (decltype(r.all_gather))dlsym(h, "ncclAllGather");
  r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
  r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
  r.destroy = (decltype(r.destroy))dlsym(h, "ncclCommDestroy");
  r.err_str = (decltype(r.err_str))dlsym(h, "ncclGetErrorString");
  r.ok = r.init_all && r.all_gather && r.group_start && r.group_end && r.destroy && r.err_str;
  if (!r.ok) r.why = "librccl lacks a needed symbol";
  return r;
}

// Per-worker resources, released on every exit path.
struct Worker {
  int dev = 0;
  size_t lo = 0, hi = 0;
  hipStream_t s = nullptr;
  uint8_t *part = nullptr;    // this worker's fold (state_bytes)
  uint8_t *gather = nullptr;  // RCCL: ndev x state_bytes; COPY (worker 0): the same
  uint8_t *merged = nullptr;  // AND of the gathered rows
  int rc = 0;
  std::string err;
  ~Worker() {
    if (s) (void)hipStreamSynchronize(s);
    int cur = -1;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(dev);
    for (uint8_t *p : {part, gather, merged})
      if (p) (void)hipFree(p);
    if (s) (void)hipStreamDestroy(s);
    if (cur >= 0) (void)hipSetDevice(cur);
  }
};

#define MHIP(expr)                                                                      \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) return fail_multi(std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

struct DevScope {  // restore the calling thread's device
  int old = -1;
  DevScope() { (void)hipGetDevice(&old); }
  ~DevScope() {
    if (old >= 0) (void)hipSetDevice(old);
  }
};

// RCCL exchange: one ncclAllGather of every worker's fold over comms from ncclCommInitAll (one
// rank per distinct GPU), then a local AND of the gathered rows on every device.  Every stream
// is synchronised before the communicators are destroyed (no collective or AND still queued on
// a comm being torn down).  Returns 0, or -1 with *why set; the partial folds are left intact,
// so a caller may still exchange them by copies.
int rccl_exchange(std::vector<Worker> &ws, const std::vector<int> &devs, size_t state_bytes,
                  std::string *why) {
  Rccl &r = rccl();
  const size_t W = ws.size();
  std::vector<ncclComm_t> comms(W, nullptr);
  ncclResult_t e = r.init_all(comms.data(), (int)W, devs.data());
  if (e != ncclSuccess) {
    *why = std::string("ncclCommInitAll: ") + r.err_str(e);
    return -1;
  }
  int rc = 0;
  e = r.group_start();
  for (size_t w = 0; w < W && e == ncclSuccess; w++) {
    (void)hipSetDevice(ws[w].dev);
    e = r.all_gather(ws[w].part, ws[w].gather, state_bytes, ncclUint8, comms[w], ws[w].s);
  }
  const ncclResult_t eg = r.group_end();
  if (e == ncclSuccess) e = eg;
  if (e != ncclSuccess) {
    *why = std::string("ncclAllGather: ") + r.err_str(e);
    rc = -1;
  }
  for (size_t w = 0; w < W && rc == 0; w++) {  // every device ANDs the gathered rows locally
    if (hipSetDevice(ws[w].dev) != hipSuccess ||
        kbz_merge_and_device(ws[w].merged, ws[w].gather, W, state_bytes, ws[w].s)) {
      *why = std::string("local AND after the all-gather: ") + kbz_last_error();
      rc = -1;
    }
  }
  for (size_t w = 0; w < W; w++) {  // drain before the comms go away
    (void)hipSetDevice(ws[w].dev);
    if (hipStreamSynchronize(ws[w].s) != hipSuccess && rc == 0) {
      *why = "stream synchronise after the all-gather failed";
      rc = -1;
    }
  }
  for (auto c : comms)
    if (c) (void)r.destroy(c);
  return rc;
}

}  // namespace

extern "C" int kbz_merge_and_fill_devices(uint8_t *out, size_t n, size_t state_bytes,
                                          kbz_merge_fill_fn fill, void *user, const int *devices,
                                          size_t ndev, int exchange, int *used_out) {
  if (!out || (!fill && n)) return fail_multi("null argument");
  if (exchange < KBZ_EXCHANGE_AUTO || exchange > KBZ_EXCHANGE_RCCL)
    return fail_multi("bad exchange");
  DevScope keep;
  std::vector<int> devs;
  int count = 0;
  MHIP(hipGetDeviceCount(&count));
  if (devices) {
    if (ndev == 0) return fail_multi("ndev must be >= 1");
    devs.assign(devices, devices + ndev);
  } else {
    for (int d = 0; d < count; d++) devs.push_back(d);
  }
  for (int d : devs)
    if (d < 0 || d >= count) return fail_multi("device ordinal out of range");
  const size_t W = devs.size();
  if (W == 0) return fail_multi("no device");
  std::vector<int> sorted = devs;
  std::sort(sorted.begin(), sorted.end());
  const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
  bool use_rccl = false;
  if (exchange == KBZ_EXCHANGE_RCCL) {
    if (!distinct) return fail_multi("RCCL exchange needs distinct devices (one rank per GPU)");
    if (!rccl().ok) return fail_multi(rccl().why);
    use_rccl = true;
  } else if (exchange == KBZ_EXCHANGE_AUTO) {
    use_rccl = W > 1 && distinct && rccl().ok;
  }
  if (used_out) *used_out = use_rccl ? KBZ_EXCHANGE_RCCL : KBZ_EXCHANGE_COPY;
  if (state_bytes == 0) return 0;
  if (n == 0) {
    memset(out, 0xff, state_bytes);
    return 0;
  }
  std::vector<Worker> ws(W);
  for (size_t w = 0; w < W; w++) {
    ws[w].dev = devs[w];
    ws[w].lo = n * w / W;
    ws[w].hi = n * (w + 1) / W;
    MHIP(hipSetDevice(devs[w]));
    MHIP(hipStreamCreateWithFlags(&ws[w].s, hipStreamNonBlocking));
    MHIP(hipMalloc((void **)&ws[w].part, state_bytes));
    if (use_rccl || w == 0) {
      MHIP(hipMalloc((void **)&ws[w].gather, W * state_bytes));
      MHIP(hipMalloc((void **)&ws[w].merged, state_bytes));
    }
  }
  // 1. the folds, one host thread per worker (fill is called with global state indices)
  struct Shifted {
    kbz_merge_fill_fn fill;
    void *user;
    size_t base;
    static int call(void *u, uint8_t *dst, size_t first, size_t cnt) {
      const Shifted *sh = (const Shifted *)u;
      return sh->fill(sh->user, dst, sh->base + first, cnt);
    }
  };
  std::vector<std::thread> threads;
  for (size_t w = 0; w < W; w++) {
    threads.emplace_back([&, w] {
      Worker &k = ws[w];
      if (hipSetDevice(k.dev) != hipSuccess) {
        k.rc = -1;
        k.err = "hipSetDevice failed";
        return;
      }
      Shifted sh{fill, user, k.lo};
      k.rc = kbz_merge_and_fill_device(k.part, k.hi - k.lo, state_bytes, Shifted::call, &sh, k.s);
      if (k.rc) k.err = kbz_last_error();
    });
  }
  for (auto &t : threads) t.join();
  for (size_t w = 0; w < W; w++)
    if (ws[w].rc) return fail_multi("worker " + std::to_string(w) + " (device " +
                                    std::to_string(ws[w].dev) + "): " + ws[w].err);
  // 2. exchange the partial folds.  AUTO falls back to copies when any RCCL step fails (the
  //    folds are intact); an explicit RCCL request fails loudly instead.
  bool copied = !use_rccl;
  if (use_rccl) {
    std::string why;
    if (rccl_exchange(ws, devs, state_bytes, &why)) {
      if (exchange == KBZ_EXCHANGE_RCCL) return fail_multi(why);
      copied = true;
      if (used_out) *used_out = KBZ_EXCHANGE_COPY;
    }
  }
  if (copied) {
    Worker &k0 = ws[0];
    MHIP(hipSetDevice(k0.dev));
    for (size_t w = 0; w < W; w++) {
      // worker w's fold is complete (its stream was synchronised by the fold); copy it over
      if (ws[w].dev == k0.dev)
        MHIP(hipMemcpyAsync(k0.gather + w * state_bytes, ws[w].part, state_bytes,
                            hipMemcpyDeviceToDevice, k0.s));
      else
        MHIP(hipMemcpyPeerAsync(k0.gather + w * state_bytes, k0.dev, ws[w].part, ws[w].dev,
                                state_bytes, k0.s));
    }
    if (kbz_merge_and_device(k0.merged, k0.gather, W, state_bytes, k0.s)) return -1;
  }
  // 3. worker 0's merged state to the host
  MHIP(hipSetDevice(ws[0].dev));
  MHIP(hipMemcpyAsync(out, ws[0].merged, state_bytes, hipMemcpyDeviceToHost, ws[0].s));
  for (size_t w = 0; w < W; w++) {
    MHIP(hipSetDevice(ws[w].dev));
    MHIP(hipStreamSynchronize(ws[w].s));
  }
  return 0;
}
