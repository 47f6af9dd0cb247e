// Diagnostic (not the product): does an in-launch hand-off read stale data when the READER's
// XCD L2 already holds an older copy of the line?  This is the situation of round 4's removed
// in-launch helpers: a column window of chunk_or written by pass 1 (plain stores, an earlier
// launch) was overwritten in k_tail with sc1 stores (write-through), drained, published, and
// read by a helper with sc1 loads after an agent-scope acquire.
//
// K1: block b writes region b (plain stores, value 1) and records its XCD.
// K2: producer block b (blocks 0..R-1, dispatched first) overwrites region b with the agent
//     sc1 stores, s_waitcnt vmcnt(0), then sets flag b with an sc1 store; consumer block R + b
//     (optionally after warming its L2 with a plain read of region b) polls flag b with sc1
//     loads, runs an agent acquire fence + vmcnt(0), and reads region b with LOAD_KIND:
//       0: sc1 loads, 1: plain loads, 2: sc0 sc1 loads (system scope), 3: nt loads
//     and counts words that are not the producer's value.
// Output per consumer: stale words, its XCD, K1's writer XCD, the producer's XCD, spin timeout.
// With a third argument S, K2 also runs S load blocks beside the hand-offs (see stream_block).
// Build: hipcc --offload-arch=gfx950 -O3 tools/l2_handoff_probe.hip -o tools/l2_handoff_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                     \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

constexpr int kWords = 256;  // uint64 words per region: 2 KiB (16 lines), 4 per lane
__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xf;
}
__global__ void k1(uint64_t *d, uint32_t *wx) {
  const uint32_t b = blockIdx.x;
  for (int i = threadIdx.x; i < kWords; i += 64) d[(size_t)b * kWords + i] = 1;
  if (threadIdx.x == 0) wx[b] = xcc_id();
}
template <int KIND>
__device__ __forceinline__ uint64_t ld(const uint64_t *p) {
  if (KIND == 0) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (KIND == 2) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (KIND == 3) return __builtin_nontemporal_load(p);
  return *(volatile const uint64_t *)p;
}
// Load: blocks 2R.. of K2 stream kStreamBytes each of another buffer (16-B nt loads, 8 in flight
// per lane) and atomicMax a hash of what they read into a 64 Ki-entry score array -- what every
// k_tail workgroup does beside a hand-off (the failing in-launch helpers ran under that load).
constexpr size_t kStreamBytes = 4u << 20;
__device__ __forceinline__ void stream_block(const uint4 *src, uint32_t *score) {
  const int lane = threadIdx.x & 63;
  uint32_t acc = 0;
  for (size_t i = 0; i < kStreamBytes / 16; i += 64 * 8) {
    uint4 v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) v[u] = src[i + u * 64 + lane];
#pragma unroll
    for (int u = 0; u < 8; u++) acc += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    atomicMax(&score[(acc * 2654435761u) >> 16], acc);
  }
}
template <int KIND>
__global__ void k2(uint64_t *d, uint32_t *flag, uint32_t R, uint64_t val, int warm,
                   uint32_t *out, uint32_t ps, uint32_t cs, const uint4 *sbuf, uint32_t *score) {
  if (blockIdx.x >= 2 * R) {  // load blocks (dispatched after every producer and consumer)
    stream_block(sbuf + (size_t)(blockIdx.x - 2 * R) * (kStreamBytes / 16), score);
    return;
  }
  // producer block p serves region (p + ps) % R, consumer block R + j region (j + cs) % R:
  // shifting the regions moves each role to other XCDs (blocks b and b + 8 share one)
  const uint32_t b = blockIdx.x < R ? (blockIdx.x + ps) % R : R + (blockIdx.x - R + cs) % R;
  if (blockIdx.x < R) {  // producer
    for (int i = threadIdx.x; i < kWords; i += 64)
      __hip_atomic_store(&d[(size_t)b * kWords + i], val, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __hip_atomic_store(&flag[b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      out[(size_t)b * 4 + 2] = xcc_id();
    }
    return;
  }
  const uint32_t c = b - R;
  uint64_t acc = 0;
  if (warm)
    for (int i = threadIdx.x; i < kWords; i += 64) acc += ((volatile uint64_t *)d)[(size_t)c * kWords + i];
  __shared__ int ok;
  if (threadIdx.x == 0) {
    int it = 0;
    while (__hip_atomic_load(&flag[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 1u &&
           it < (1 << 22)) {
      __builtin_amdgcn_s_sleep(2);
      it++;
    }
    ok = it < (1 << 22);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  uint32_t stale = 0;
  for (int i = threadIdx.x; i < kWords; i += 64)
    stale += ld<KIND>(&d[(size_t)c * kWords + i]) != val;
  for (int o = 32; o; o >>= 1) stale += __shfl_xor(stale, o);
  if (threadIdx.x == 0) {
    out[(size_t)c * 4 + 0] = stale + (acc == 12345 ? 1 : 0);
    out[(size_t)c * 4 + 1] = xcc_id();
    out[(size_t)c * 4 + 3] = ok ? 0 : 1;
  }
}

int main(int argc, char **argv) {
  const uint32_t R = argc > 1 ? atoi(argv[1]) : 1024;  // regions (producer / consumer pairs)
  const int reps = argc > 2 ? atoi(argv[2]) : 64;  // every (producer, consumer) shift pair
  const uint32_t S = argc > 3 ? atoi(argv[3]) : 0;  // load blocks (each streams 4 MiB)
  uint64_t *d;
  uint32_t *flag, *wx, *out, *score;
  uint4 *sbuf = nullptr;
  CHECK(hipMalloc(&score, 65536 * 4));
  if (S) {
    CHECK(hipMalloc(&sbuf, (size_t)S * kStreamBytes));
    CHECK(hipMemset(sbuf, 1, (size_t)S * kStreamBytes));
  }
  CHECK(hipMalloc(&d, (size_t)R * kWords * 8));
  CHECK(hipMalloc(&flag, R * 4));
  CHECK(hipMalloc(&wx, R * 4));
  CHECK(hipMalloc(&out, (size_t)R * 16));
  std::vector<uint32_t> h(R * 4), hw(R);
  for (int kind = 0; kind < 4; kind++)
    for (int warm = 0; warm < 2; warm++) {
      // stale words: [same XCD as K1's writer][consumer same XCD as producer]
      unsigned long long st[2][2] = {{0, 0}, {0, 0}}, cnt[2][2] = {{0, 0}, {0, 0}};
      unsigned long long timeouts = 0, blocks_stale = 0;
      for (int r = 0; r < reps; r++) {
        hipLaunchKernelGGL(k1, dim3(R), dim3(64), 0, 0, d, wx);
        CHECK(hipMemset(flag, 0, R * 4));
        const uint64_t val = 2 + r;
        if (kind == 0) hipLaunchKernelGGL(k2<0>, dim3(2 * R + S), dim3(64), 0, 0, d, flag, R, val, warm, out, r % 8, (r / 8) % 8, sbuf, score);
        if (kind == 1) hipLaunchKernelGGL(k2<1>, dim3(2 * R + S), dim3(64), 0, 0, d, flag, R, val, warm, out, r % 8, (r / 8) % 8, sbuf, score);
        if (kind == 2) hipLaunchKernelGGL(k2<2>, dim3(2 * R + S), dim3(64), 0, 0, d, flag, R, val, warm, out, r % 8, (r / 8) % 8, sbuf, score);
        if (kind == 3) hipLaunchKernelGGL(k2<3>, dim3(2 * R + S), dim3(64), 0, 0, d, flag, R, val, warm, out, r % 8, (r / 8) % 8, sbuf, score);
        CHECK(hipDeviceSynchronize());
        CHECK(hipMemcpy(h.data(), out, R * 16, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(hw.data(), wx, R * 4, hipMemcpyDeviceToHost));
        for (uint32_t c = 0; c < R; c++) {
          const int a = h[c * 4 + 1] == hw[c], p = h[c * 4 + 1] == h[c * 4 + 2];
          st[a][p] += h[c * 4];
          cnt[a][p] += 1;
          timeouts += h[c * 4 + 3];
          blocks_stale += h[c * 4] != 0;
        }
      }
      static const char *names[4] = {"sc1", "plain", "sc0sc1", "nt"};
      printf("S=%u load=%-6s warm=%d  stale blocks %llu / %llu  timeouts %llu | stale words by "
             "(consumer on K1-writer XCD, consumer on producer XCD): "
             "(n,n) %llu/%llu (n,y) %llu/%llu (y,n) %llu/%llu (y,y) %llu/%llu\n",
             S, names[kind], warm, blocks_stale, (unsigned long long)R * reps, timeouts,
             st[0][0], cnt[0][0] * kWords, st[0][1], cnt[0][1] * kWords, st[1][0],
             cnt[1][0] * kWords, st[1][1], cnt[1][1] * kWords);
    }
  return 0;
}
