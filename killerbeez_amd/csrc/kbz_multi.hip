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

// Peer access between every pair of distinct devices in devs (both directions), so peer copies
// (hipMemcpyPeerAsync) go GPU to GPU over xGMI instead of staging through host memory.  Pairs
// the platform cannot connect are left alone (their copies still work, staged by the runtime).
// Returns the number of ordered pairs with peer access enabled.
int enable_peers(const std::vector<int> &devs) {
  std::vector<int> d = devs;
  std::sort(d.begin(), d.end());
  d.erase(std::unique(d.begin(), d.end()), d.end());
  int pairs = 0;
  for (int a : d)
    for (int b : d) {
      if (a == b) continue;
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, a, b) != hipSuccess || !can) continue;
      if (hipSetDevice(a) != hipSuccess) continue;
      const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
      if (e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled) pairs++;
      (void)hipGetLastError();  // an "already enabled" is not an error of a later call
    }
  return pairs;
}

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
  if (!use_rccl) (void)enable_peers(devs);  // the copy exchange's peer copies over xGMI
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

// ---- sharded triage over several GPUs of one node, from C -----------------------------------
// The protocol of killerbeez_amd/dist.py (include/kbz_triage.h "sharded
// triage") driven by one host thread over W workers, each a kbz_ctx on its device with its own
// stream: contiguous shards of a host batch, the DynamoRIO link rows and the OR aggregates
// exchanged by peer copies (device-local copies for workers sharing a GPU) into a gather buffer
// on every worker (each worker's own aggregate written into its slot by kbz_shard_reduce_into),
// prefix and total taken inside kbz_shard_finish_gathered.  Cross-stream order by events only:
// no host sync until the results are copied back.
struct kbz_mctx {
  size_t M = 0, max_batch = 0, W = 0, ab = 0;  // ab = aggregate bytes per worker
  int mode = 0;
  int peer_pairs = 0;  // ordered pairs of the workers' distinct devices with peer access on
  size_t stage_rows = 0;  // host batches: rows per pinned staging slot (2 slots per worker)
  std::vector<int> dev;
  std::vector<uint8_t *> pin[2];   // per worker: pinned staging slots (host batches)
  std::vector<int8_t *> pin_oc;    // per worker: pinned outcome staging (max_batch)
  std::vector<hipEvent_t> ev_slot[2];
  std::vector<kbz_ctx_t *> ctx;
  std::vector<hipStream_t> s;
  std::vector<hipEvent_t> ev_link, ev_agg;
  std::vector<uint8_t *> traces, hnb, mine, gather, agg_all;
  std::vector<int8_t *> oc;
  std::vector<uint32_t *> h32;
};

namespace {
void mctx_free(kbz_mctx *m) {
  for (size_t w = 0; w < m->W; w++) {
    if (w < m->dev.size()) (void)hipSetDevice(m->dev[w]);
    if (w < m->s.size() && m->s[w]) (void)hipStreamSynchronize(m->s[w]);
    for (auto *v : {&m->traces, &m->hnb, &m->mine, &m->gather, &m->agg_all})
      if (w < v->size() && (*v)[w]) (void)hipFree((*v)[w]);
    if (w < m->oc.size() && m->oc[w]) (void)hipFree(m->oc[w]);
    if (w < m->h32.size() && m->h32[w]) (void)hipFree(m->h32[w]);
    if (w < m->ev_link.size() && m->ev_link[w]) (void)hipEventDestroy(m->ev_link[w]);
    if (w < m->ev_agg.size() && m->ev_agg[w]) (void)hipEventDestroy(m->ev_agg[w]);
    for (int i = 0; i < 2; i++) {
      if (w < m->pin[i].size() && m->pin[i][w]) (void)hipHostFree(m->pin[i][w]);
      if (w < m->ev_slot[i].size() && m->ev_slot[i][w]) (void)hipEventDestroy(m->ev_slot[i][w]);
    }
    if (w < m->pin_oc.size() && m->pin_oc[w]) (void)hipHostFree(m->pin_oc[w]);
    if (w < m->ctx.size() && m->ctx[w]) kbz_ctx_destroy(m->ctx[w]);
    if (w < m->s.size() && m->s[w]) (void)hipStreamDestroy(m->s[w]);
  }
  delete m;
}
// dst (on device dd) <- src (on device sd), n bytes, on stream st (dd's)
hipError_t xcopy(void *dst, int dd, const void *src, int sd, size_t n, hipStream_t st) {
  if (dd == sd) return hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, st);
  return hipMemcpyPeerAsync(dst, dd, src, sd, n, st);
}
}  // namespace

extern "C" kbz_mctx_t *kbz_mctx_create(size_t map_size, int mode, size_t max_batch,
                                       const int *devices, size_t ndev) {
  if (!devices || ndev == 0) {
    fail_multi("kbz_mctx_create: devices[] and ndev >= 1 are required");
    return nullptr;
  }
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess) {
    fail_multi("kbz_mctx_create: no device");
    return nullptr;
  }
  for (size_t w = 0; w < ndev; w++)
    if (devices[w] < 0 || devices[w] >= count) {
      fail_multi("kbz_mctx_create: device ordinal out of range");
      return nullptr;
    }
  DevScope keep;
  kbz_mctx *m = new kbz_mctx;
  m->M = map_size;
  m->mode = mode;
  m->max_batch = max_batch;
  m->W = ndev;
  m->dev.assign(devices, devices + ndev);
  const size_t W = ndev, row = map_size + 16;  // gathered link rows: [row | hash pair | pad]
  for (auto *v : {&m->traces, &m->hnb, &m->mine, &m->gather, &m->agg_all}) v->assign(W, nullptr);
  m->oc.assign(W, nullptr);
  m->h32.assign(W, nullptr);
  m->ctx.assign(W, nullptr);
  m->s.assign(W, nullptr);
  m->ev_link.assign(W, nullptr);
  m->ev_agg.assign(W, nullptr);
  for (int i = 0; i < 2; i++) {
    m->pin[i].assign(W, nullptr);
    m->ev_slot[i].assign(W, nullptr);
  }
  m->pin_oc.assign(W, nullptr);
  // staging slots of up to 32 MiB (at least one row, at most a shard)
  m->stage_rows = std::max<size_t>(1, std::min(max_batch, (size_t)(32u << 20) / map_size));
  auto bad = [&](const char *what) {
    std::string msg = std::string("kbz_mctx_create: ") + what;
    mctx_free(m);
    fail_multi(msg);
    return (kbz_mctx_t *)nullptr;
  };
  for (size_t w = 0; w < W; w++) {
    if (hipSetDevice(m->dev[w]) != hipSuccess) return bad("hipSetDevice");
    m->ctx[w] = kbz_ctx_create(map_size, mode, max_batch);
    if (!m->ctx[w]) return bad(kbz_last_error());
    if (w == 0) m->ab = kbz_shard_aggregate_bytes(m->ctx[0]);
    if (hipStreamCreateWithFlags(&m->s[w], hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&m->ev_link[w], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&m->ev_agg[w], hipEventDisableTiming) != hipSuccess ||
        hipMalloc((void **)&m->traces[w], max_batch * map_size + 16) != hipSuccess ||
        hipMalloc((void **)&m->oc[w], max_batch + 16) != hipSuccess ||
        hipMalloc((void **)&m->h32[w], max_batch * 4 + 16) != hipSuccess ||
        hipMalloc((void **)&m->hnb[w], max_batch + 16) != hipSuccess ||
        hipMalloc((void **)&m->mine[w], row) != hipSuccess ||
        hipMalloc((void **)&m->gather[w], W * row) != hipSuccess ||
        hipMalloc((void **)&m->agg_all[w], W * m->ab) != hipSuccess)
      return bad("out of device memory");
    if (hipMemset(m->mine[w], 0, row) != hipSuccess) return bad("hipMemset");
    for (int i = 0; i < 2; i++)
      if (hipHostMalloc((void **)&m->pin[i][w], m->stage_rows * map_size, 0) != hipSuccess ||
          hipEventCreateWithFlags(&m->ev_slot[i][w], hipEventDisableTiming) != hipSuccess)
        return bad("out of pinned host memory");
    if (hipHostMalloc((void **)&m->pin_oc[w], max_batch + 16, 0) != hipSuccess)
      return bad("out of pinned host memory");
  }
  m->peer_pairs = enable_peers(m->dev);
  return m;
}

extern "C" void kbz_mctx_destroy(kbz_mctx_t *m) {
  if (!m) return;
  DevScope keep;
  mctx_free(m);
}

extern "C" int kbz_mctx_workers(kbz_mctx_t *m) { return m ? (int)m->W : -1; }
extern "C" kbz_ctx_t *kbz_mctx_worker(kbz_mctx_t *m, size_t w) {
  return (m && w < m->W) ? m->ctx[w] : nullptr;
}

extern "C" int kbz_mctx_peer_pairs(kbz_mctx_t *m) { return m ? m->peer_pairs : -1; }

namespace {
// Rows [r0, r1) of a host shard (stride apart) into a pinned slot, split over up to `nt` threads
// (one thread's copy out of pageable memory runs well below the PCIe rate).
void fill_rows(uint8_t *dst, const uint8_t *src, size_t rows, size_t stride, size_t M, int nt) {
  auto part = [=](size_t a, size_t b) {
    if (stride == M) memcpy(dst + a * M, src + a * M, (b - a) * M);
    else
      for (size_t r = a; r < b; r++) memcpy(dst + r * M, src + r * stride, M);
  };
  const size_t T = std::min<size_t>(nt, std::max<size_t>(1, rows * M >> 22));  // >= 4 MiB each
  if (T <= 1) return part(0, rows);
  std::vector<std::thread> th;
  for (size_t i = 1; i < T; i++) th.emplace_back(part, rows * i / T, rows * (i + 1) / T);
  part(0, rows / T);
  for (auto &t : th) t.join();
}

// Host memory the runtime pinned (hipHostMalloc / hipHostRegister): its DMA needs no staging.
bool pinned_host(const void *p) {
  hipPointerAttribute_t at;
  const bool ok = hipPointerGetAttributes(&at, p) == hipSuccess && at.type == hipMemoryTypeHost;
  (void)hipGetLastError();  // pageable memory: an "invalid value" that is no error here
  return ok;
}

// Worker w's host shard (nw rows) to its device rows m->traces[w] through its two pinned slots:
// the host copy of slot i overlaps the DMA of slot i ^ 1.  Runs on the worker's own thread.  A
// shard already in pinned memory (e.g. the plugin's ring slot) is copied by the DMA engine
// straight from there.
int stage_shard(kbz_mctx *m, size_t w, const uint8_t *src, size_t nw, size_t stride,
                const int8_t *oc, int threads, bool pinned) {
  const size_t M = m->M, R = m->stage_rows;
  MHIP(hipSetDevice(m->dev[w]));
  if (pinned && nw)
    MHIP(hipMemcpy2DAsync(m->traces[w], M, src, stride, M, nw, hipMemcpyHostToDevice, m->s[w]));
  for (size_t r0 = 0, i = 0; !pinned && r0 < nw; r0 += R, i++) {
    const int sl = (int)(i & 1);
    const size_t cnt = std::min(R, nw - r0);
    MHIP(hipEventSynchronize(m->ev_slot[sl][w]));  // the slot's previous DMA is done
    fill_rows(m->pin[sl][w], src + r0 * stride, cnt, stride, M, threads);
    MHIP(hipMemcpyAsync(m->traces[w] + r0 * M, m->pin[sl][w], cnt * M, hipMemcpyHostToDevice,
                        m->s[w]));
    MHIP(hipEventRecord(m->ev_slot[sl][w], m->s[w]));
  }
  if (oc && nw) {
    memcpy(m->pin_oc[w], oc, nw);
    MHIP(hipMemcpyAsync(m->oc[w], m->pin_oc[w], nw, hipMemcpyHostToDevice, m->s[w]));
  }
  return 0;
}

// The sharded protocol over the workers, on batches already on their devices: worker w holds
// n[w] rows at traces[w] (stride apart); the batch is worker 0's rows, then worker 1's, ...
// Results into hnb[w] / h32[w] (device, or null); m->h32[w] stands in when a hash is needed.
// Ends with each worker's stream and sticky error flags checked.
int run_protocol(kbz_mctx *m, const uint8_t *const *traces, const size_t *n, size_t stride,
                 const int8_t *const *outcome, uint8_t *const *hnb, uint32_t *const *h32,
                 int want) {
  const size_t W = m->W, M = m->M, row = M + 16;
  const bool dr = m->mode == KBZ_MODE_DYNAMORIO;
  const bool hashed = dr || (want & KBZ_WANT_H32);
  std::vector<size_t> nonempty;
  for (size_t w = 0; w < W; w++)
    if (n[w]) nonempty.push_back(w);
  // 1. pass 1 (+ k_skip) per shard; DynamoRIO: each shard's link row and hash pair
  for (size_t w = 0; w < W; w++) {
    MHIP(hipSetDevice(m->dev[w]));
    uint32_t *hw = (h32 && h32[w]) ? h32[w] : m->h32[w];
    if (kbz_shard_begin(m->ctx[w], n[w] ? traces[w] : nullptr, n[w], stride,
                        (outcome && n[w]) ? outcome[w] : nullptr, hashed ? hw : nullptr, nullptr,
                        want, m->s[w]))
      return -1;
    if (dr) {
      if (kbz_shard_exchange_row(m->ctx[w], m->mine[w], m->s[w])) return -1;
      MHIP(hipEventRecord(m->ev_link[w], m->s[w]));
    }
  }
  // 2. DynamoRIO: every worker gathers the link rows, then links to the nearest non-empty earlier
  //    shard and to the last non-empty one (the batch's last exec)
  for (size_t v = 0; v < W; v++) {
    MHIP(hipSetDevice(m->dev[v]));
    if (dr) {
      for (size_t w : nonempty) {
        MHIP(hipStreamWaitEvent(m->s[v], m->ev_link[w], 0));
        MHIP(xcopy(m->gather[v] + w * row, m->dev[v], m->mine[w], m->dev[w], row, m->s[v]));
      }
      long p = -1;
      for (size_t w : nonempty)
        if (w < v) p = (long)w;
      const long g = nonempty.empty() ? -1 : (long)nonempty.back();
      const uint8_t *gp = m->gather[v];
      if (kbz_shard_link(m->ctx[v], p < 0 ? nullptr : (const uint32_t *)(gp + p * row + M),
                         p < 0 ? nullptr : gp + p * row, p < 0 ? 1 : 0,
                         g < 0 ? nullptr : (const uint32_t *)(gp + g * row + M),
                         g < 0 ? nullptr : gp + g * row, m->s[v]))
        return -1;
    } else if (kbz_shard_link(m->ctx[v], nullptr, nullptr, 1, nullptr, nullptr, m->s[v])) {
      return -1;
    }
    // the aggregate goes straight into this worker's own slot of its gather buffer
    if (kbz_shard_reduce_into(m->ctx[v], m->agg_all[v] + v * m->ab, m->s[v])) return -1;
    MHIP(hipEventRecord(m->ev_agg[v], m->s[v]));
  }
  // 3. every worker gathers the other aggregates, then resolves with the prefix (earlier shards)
  //    and the total taken from the gathered rows inside the fused tail
  for (size_t v = 0; v < W; v++) {
    MHIP(hipSetDevice(m->dev[v]));
    for (size_t w = 0; w < W; w++) {
      if (w == v) continue;
      MHIP(hipStreamWaitEvent(m->s[v], m->ev_agg[w], 0));
      MHIP(xcopy(m->agg_all[v] + w * m->ab, m->dev[v], m->agg_all[w] + w * m->ab, m->dev[w], m->ab,
                 m->s[v]));
    }
    if (kbz_shard_finish_gathered(m->ctx[v], m->agg_all[v], v, W,
                                  (hnb && hnb[v]) ? hnb[v] : m->hnb[v], m->s[v]))
      return -1;
  }
  return 0;
}

int check_errors(kbz_mctx *m) {
  for (size_t v = 0; v < m->W; v++) {
    MHIP(hipSetDevice(m->dev[v]));
    if (kbz_sync(m->ctx[v], m->s[v])) return -1;  // the stream, then the sticky error flags
  }
  return 0;
}
}  // namespace

extern "C" int kbz_triage_batch_devices(kbz_mctx_t *m, const uint8_t *traces, size_t n,
                                        size_t stride, const int8_t *outcome, uint8_t *hnb_out,
                                        uint32_t *h32_out, int want) {
  if (!m) return fail_multi("null mctx");
  if (n && (!traces || stride < m->M)) return fail_multi("bad traces / stride");
  if (want & KBZ_WANT_X64) return fail_multi("kbz_triage_batch_devices: XXH64 is not gathered");
  const size_t W = m->W, M = m->M;
  std::vector<size_t> lo(W + 1), cnt(W);
  for (size_t w = 0; w <= W; w++) lo[w] = n * w / W;
  for (size_t w = 0; w < W; w++) {
    cnt[w] = lo[w + 1] - lo[w];
    if (cnt[w] > m->max_batch) return fail_multi("a shard exceeds max_batch");
  }
  DevScope keep;
  const bool hashed = m->mode == KBZ_MODE_DYNAMORIO || (want & KBZ_WANT_H32);
  // 1. every worker stages its shard on its own host thread (pinned slots, DMA overlapped with the
  //    next slot's host copy); the copy threads of a slot are shared out over the workers
  const int per = std::max(1, 8 / (int)W);
  std::vector<int> rc(W, 0);
  std::vector<std::string> err(W);
  const bool pinned = n && pinned_host(traces);
  auto job = [&](size_t w) {
    if (stage_shard(m, w, traces + lo[w] * stride, cnt[w], stride, outcome ? outcome + lo[w] : nullptr,
                    per, pinned)) {
      rc[w] = -1;
      err[w] = kbz_last_error();
    }
  };
  if (W == 1) {
    job(0);
  } else {
    std::vector<std::thread> th;
    for (size_t w = 0; w < W; w++) th.emplace_back(job, w);
    for (auto &t : th) t.join();
  }
  for (size_t w = 0; w < W; w++)
    if (rc[w]) return fail_multi("staging shard " + std::to_string(w) + ": " + err[w]);
  std::vector<const uint8_t *> tp(W);
  std::vector<const int8_t *> op(W);
  for (size_t w = 0; w < W; w++) {
    tp[w] = m->traces[w];
    op[w] = outcome ? m->oc[w] : nullptr;
  }
  if (run_protocol(m, tp.data(), cnt.data(), M, outcome ? op.data() : nullptr, nullptr, nullptr,
                   want))
    return -1;
  // 2. results to the host, per worker on its stream
  for (size_t v = 0; v < W; v++) {
    MHIP(hipSetDevice(m->dev[v]));
    if (cnt[v] && hnb_out)
      MHIP(hipMemcpyAsync(hnb_out + lo[v], m->hnb[v], cnt[v], hipMemcpyDeviceToHost, m->s[v]));
    if (cnt[v] && h32_out && hashed)
      MHIP(hipMemcpyAsync(h32_out + lo[v], m->h32[v], cnt[v] * 4, hipMemcpyDeviceToHost, m->s[v]));
  }
  return check_errors(m);
}

extern "C" int kbz_triage_batch_devices_resident(kbz_mctx_t *m, const uint8_t *const *traces,
                                                 const size_t *n, size_t stride,
                                                 const int8_t *const *outcome,
                                                 uint8_t *const *hnb_out, uint32_t *const *h32_out,
                                                 int want) {
  if (!m || !n) return fail_multi("null argument");
  if (want & KBZ_WANT_X64) return fail_multi("kbz_triage_batch_devices: XXH64 is not gathered");
  if (stride < m->M || stride % 16) return fail_multi("stride must be >= map_size and a multiple of 16");
  for (size_t w = 0; w < m->W; w++) {
    if (n[w] > m->max_batch) return fail_multi("a shard exceeds max_batch");
    if (n[w] && (!traces || !traces[w])) return fail_multi("null traces for a non-empty shard");
  }
  DevScope keep;
  if (run_protocol(m, traces, n, stride, outcome, hnb_out, h32_out, want)) return -1;
  return check_errors(m);
}

extern "C" int kbz_mctx_get_virgin(kbz_mctx_t *m, uint8_t *host_out) {
  if (!m || !host_out) return fail_multi("null argument");
  DevScope keep;
  MHIP(hipSetDevice(m->dev[0]));
  return kbz_get_virgin(m->ctx[0], host_out);
}

extern "C" int kbz_mctx_set_virgin(kbz_mctx_t *m, const uint8_t *host_in) {
  if (!m || !host_in) return fail_multi("null argument");
  DevScope keep;
  for (size_t w = 0; w < m->W; w++) {
    MHIP(hipSetDevice(m->dev[w]));
    if (kbz_set_virgin(m->ctx[w], host_in)) return -1;
  }
  return 0;
}

extern "C" int kbz_mctx_get_last_hash(kbz_mctx_t *m, uint32_t *out) {
  if (!m || !out) return fail_multi("null argument");
  DevScope keep;
  MHIP(hipSetDevice(m->dev[0]));
  return kbz_get_last_hash(m->ctx[0], out);
}
