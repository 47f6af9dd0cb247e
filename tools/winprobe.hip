// tools/winprobe.hip -- calibration probe (not product): the access pattern of k_fin's window
// items on config 3 (16,384 rows x 1 MiB): a wave reads one 1-KiB column window of a chunk's 64
// rows (16 B per lane, KBZ_WIN_ROWS = 16 rows in flight), items dealt round-robin over 2,048
// waves.  Orders of the ~14,000 items of a novelty-heavy batch:
//   chunk-major : items i .. i + 2047 in flight together cover 2 chunks (128 rows)
//   runs        : k_tail's order -- each column group's run of consecutive chunks (0..13)
//   random      : any chunk of the batch, any column
//   contiguous  : control -- 64 KiB of one row per item (no 1-MiB stride)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr uint32_t kRows = 16384, kRowBytes = 1u << 20, kChunk = 64, kWin = 1024;

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

// item -> (first row, byte offset of the window in the row)
__device__ __forceinline__ void item_of(int order, uint32_t i, uint32_t nitems, uint64_t &row0,
                                        uint32_t &col) {
  if (order == 0) {  // chunk-major
    row0 = (uint64_t)(i / (kRowBytes / kWin)) * kChunk;
    col = (i % (kRowBytes / kWin)) * kWin;
  } else if (order == 1) {  // runs of 14 consecutive chunks per column window
    const uint32_t run = i / 14;
    row0 = (uint64_t)(i % 14) * kChunk;
    col = (mix32(run) % (kRowBytes / kWin)) * kWin;
  } else {  // random chunk, random window
    row0 = (uint64_t)(mix32(i * 2 + 1) % (kRows / kChunk)) * kChunk;
    col = (mix32(i * 2 + 2) % (kRowBytes / kWin)) * kWin;
  }
}

template <int WR>
__global__ __launch_bounds__(256) void windows(const uint8_t *t, uint32_t nitems, int order,
                                               uint4 *out) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (uint32_t it = wave; it < nitems; it += nwaves) {
    uint64_t row0;
    uint32_t col;
    item_of(order < 3 ? order : 0, it, nitems, row0, col);
    for (int r0 = 0; r0 < (int)kChunk; r0 += WR) {
      uint4 v[WR];
#pragma unroll
      for (int u = 0; u < WR; u++) {
        const size_t off = order == 3 ? (size_t)row0 * kRowBytes + (size_t)(r0 + u) * kWin + col / 64 + lane * 16
                                      : (size_t)(row0 + r0 + u) * kRowBytes + col + lane * 16;
        v[u] = *(const uint4 *)(t + off);
      }
#pragma unroll
      for (int u = 0; u < WR; u++) {
        acc.x |= v[u].x; acc.y ^= v[u].y; acc.z += v[u].z; acc.w |= v[u].w;
      }
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
  uint8_t *t;
  uint4 *o;
  const size_t bytes = (size_t)kRows * kRowBytes;
  if (hipMalloc(&t, bytes) != hipSuccess || hipMalloc(&o, 512 * 256 * sizeof(uint4)) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  (void)hipMemset(t, 1, bytes);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const uint32_t nitems = 14336;
  const char *names[] = {"chunk-major", "runs", "random", "contiguous"};
  for (int rep = 0; rep < 3; rep++)
    for (int order = 0; order < 4; order++) {
      float ms;
      (void)hipEventRecord(a);
      hipLaunchKernelGGL(windows<16>, dim3(512), dim3(256), 0, 0, t, nitems, order, o);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      (void)hipEventElapsedTime(&ms, a, b);
      printf("rep %d %-12s %u windows x 64 KiB: %8.1f us = %6.2f TB/s\n", rep, names[order], nitems,
             ms * 1e3, (double)nitems * 65536 / (ms * 1e-3) / 1e12);
    }
  return (int)hipDeviceSynchronize();
}
