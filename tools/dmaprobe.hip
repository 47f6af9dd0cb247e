// tools/dmaprobe.hip -- what it costs, per exec, to move one exec's trace map out of the target's
// SysV shared-memory segment (afl_instrumentation.c:563-576 creates and attaches it) into a GPU
// batch row, so that the next exec's memset (:170) may overwrite it.  Not part of the product.
//
// Each loop runs `execs` execs.  An "exec" is simulated by the host writing the exec's sparse
// trace into the shm map (a config-2-like trace: ~2 % nonzero bytes at fixed positions, the values
// changing per exec) after the reference's memset of the map; then the variant moves the map:
//   base         nothing (the target's writes + the reference's memset alone)
//   cpu          the plugin's copy today: 16-B streaming stores into a pinned ring slot
//   dma_event    hipMemcpyAsync(device row <- registered map) + event record + event sync
//   dma_flag     hipMemcpyAsync + hipStreamWriteValue32(host flag) + host spin on the flag
//   dma_zero     as dma_flag, and the GPU also zeroes the map (hipMemsetAsync on the registered
//                map): the host skips its memset
//   kern_flag    one kernel reads the registered map (zero-copy), writes the device row and zeroes
//                the map; hipStreamWriteValue32 + spin
//   dma_nowait   hipMemcpyAsync per exec with no wait (NOT a valid protocol: the map is reused;
//                measures the enqueue cost alone)
// Reported: us per exec, and that minus `base`.
#include <hip/hip_runtime.h>
#include <sys/ipc.h>
#include <sys/shm.h>
#include <time.h>
#include <emmintrin.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

static double now_us() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_copy_zero(const u32x4 *src, u32x4 *dst, u32x4 *zsrc, int n16) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n16) {
    dst[i] = __builtin_nontemporal_load(src + i);
    zsrc[i] = u32x4{0, 0, 0, 0};
  }
}

static void stream_copy(uint8_t *dst, const uint8_t *src, size_t n) {
  for (size_t i = 0; i < n; i += 64) {
    __m128i a = _mm_loadu_si128((const __m128i *)(src + i));
    __m128i b = _mm_loadu_si128((const __m128i *)(src + i + 16));
    __m128i c = _mm_loadu_si128((const __m128i *)(src + i + 32));
    __m128i d = _mm_loadu_si128((const __m128i *)(src + i + 48));
    _mm_stream_si128((__m128i *)(dst + i), a);
    _mm_stream_si128((__m128i *)(dst + i + 16), b);
    _mm_stream_si128((__m128i *)(dst + i + 32), c);
    _mm_stream_si128((__m128i *)(dst + i + 48), d);
  }
}

int main(int argc, char **argv) {
  const size_t M = argc > 1 ? strtoull(argv[1], 0, 0) : 65536;
  const int execs = argc > 2 ? atoi(argv[2]) : 4096;
  const int spin = argc > 3 ? atoi(argv[3]) : 1;
  if (spin) CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
  CK(hipSetDevice(0));
  const int ring = 256;
  // the target's map: a SysV segment, as the reference's setup_shm makes it
  int id = shmget(IPC_PRIVATE, M, IPC_CREAT | IPC_EXCL | 0600);
  if (id < 0) { perror("shmget"); return 1; }
  uint8_t *map = (uint8_t *)shmat(id, NULL, 0);
  shmctl(id, IPC_RMID, NULL);
  if (map == (void *)-1) { perror("shmat"); return 1; }
  memset(map, 0, M);
  double t0 = now_us();
  CK(hipHostRegister(map, M, hipHostRegisterMapped));
  printf("hipHostRegister(%zu B SysV shm): %.1f us\n", M, now_us() - t0);
  uint8_t *map_d;
  CK(hipHostGetDevicePointer((void **)&map_d, map, 0));
  uint8_t *rows_d, *slot_h;
  CK(hipMalloc(&rows_d, ring * M));
  CK(hipHostMalloc(&slot_h, ring * M, hipHostMallocDefault));
  volatile uint32_t *flag_h;
  CK(hipHostMalloc((void **)&flag_h, 64, hipHostMallocCoherent | hipHostMallocMapped));
  uint32_t *flag_d;
  CK(hipHostGetDevicePointer((void **)&flag_d, (void *)flag_h, 0));
  *flag_h = 0;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  // sparse positions: 2 % of the map
  std::vector<uint32_t> pos;
  uint64_t x = 88172645463325252ull;
  for (size_t i = 0; i < M / 50; i++) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    pos.push_back((uint32_t)(x % M));
  }
  const char *names[] = {"base", "cpu", "dma_event", "dma_flag", "dma_zero", "kern_flag", "dma_nowait"};
  double base_us = 0;
  uint32_t seq = 0;
  for (int rep = 0; rep < 2; rep++)
    for (int v = 0; v < 7; v++) {
      const double t = now_us();
      for (int e = 0; e < execs; e++) {
        // the reference's enable: memset (:170) -- skipped when the GPU zeroed the map
        if (v != 4 && v != 5) memset(map, 0, M);
        // the target's exec writes its trace
        const uint8_t val = (uint8_t)(e * 7 + 1);
        for (uint32_t p : pos) map[p] += val;
        const size_t r = (size_t)(e % ring) * M;
        switch (v) {
          case 0: break;
          case 1: stream_copy(slot_h + r, map, M); break;
          case 2:
            CK(hipMemcpyAsync(rows_d + r, map, M, hipMemcpyHostToDevice, s));
            CK(hipEventRecord(ev, s));
            CK(hipEventSynchronize(ev));
            break;
          case 3:
          case 4:
          case 5:
            ++seq;
            if (v == 5) {
              k_copy_zero<<<(int)((M / 16 + 255) / 256), 256, 0, s>>>((const u32x4 *)map_d, (u32x4 *)(rows_d + r), (u32x4 *)map_d, (int)(M / 16));
            } else {
              CK(hipMemcpyAsync(rows_d + r, map, M, hipMemcpyHostToDevice, s));
              if (v == 4) CK(hipMemsetAsync(map_d, 0, M, s));
            }
            CK(hipStreamWriteValue32(s, flag_d, seq, 0));
            while (*flag_h != seq) _mm_pause();
            break;
          case 6:
            CK(hipMemcpyAsync(rows_d + r, map, M, hipMemcpyHostToDevice, s));
            if (e % ring == ring - 1) CK(hipStreamSynchronize(s));
            break;
        }
      }
      if (v == 1) _mm_sfence();
      CK(hipStreamSynchronize(s));
      const double per = (now_us() - t) / execs;
      if (v == 0) base_us = per;
      if (rep == 1) printf("%-11s %8.3f us/exec  (+%.3f over base)\n", names[v], per, per - base_us);
      if (v == 4 || v == 5) {  // the GPU zeroed the map after the last exec's move
        size_t nz = 0;
        for (size_t i = 0; i < M; i++) nz += map[i] != 0;
        if (nz) printf("%s: %zu nonzero map bytes after the last move (expect 0)\n", names[v], nz);
      }
    }
  CK(hipHostUnregister(map));
  shmdt(map);
  return 0;
}
