// killerbeez_amd/csrc/kbz_triage.hip -- gfx950 coverage-triage engine behind include/kbz_triage.h.
//
// The reference checks every exec's trace against the virgin maps one at a time
// (afl_instrumentation.c:600-662 has_new_bits inside finish_fuzz_round :231-274;
// dynamorio_instrumentation.c:1428-1468 has_new_coverage).  Here a whole ordered batch is
// triaged at once with the same results, using the per-byte decomposition of has_new_bits
// (SURVEY.md §0.7): with P[j,i] the OR of traces k<j at byte i,
//     trace j claims bits  t[j,i] & V[i] & ~P[j,i];
//     hnb[j] = 2 if it claims anything where V[i]==0xff and P[j,i]==0, else 1 if it claims
//              anything, else 0;                       V' = V & ~P[n,.]
// Pipeline per batch (all stream-ordered, no host sync):
//   pass1   one wave per 64-trace chunk streams its rows once through LDS (16 KiB tiles),
//           lane = trace: transform (raw / classify / simplify), hash32 chain, optional XXH64,
//           per-chunk column OR per virgin map, equality with the previous trace (DynamoRIO
//           skip).  Word positions where every trace of the chunk is zero take a short path.
//   skip    (DynamoRIO) skip[j] = hash[j]==hash[j-1]; chunks whose OR included a skipped
//           trace that differs from its predecessor are recomputed without it (fixchunk).
//   segor/total/prefix   OR of chunk aggregates per segment, exclusive prefix over segments,
//           virgin update V' = V & ~OR_all.
//   scan    per column, walk the segment's chunks: bits new to the chunk (OR_c & V & ~prefix)
//           become claim items; each column yields at most 8 items per map per batch.
//   resolve one wave per item re-reads that column of the claiming chunk's 64 rows and
//           finds, per new bit, the first trace holding it -> atomicMax(hnb, 1 or 2).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <utility>

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "kbz_device.h"
#include "kbz_triage.h"

using namespace kbz;

namespace {

constexpr int kChunk = 64;   // traces per chunk: one wave, one lane per trace
constexpr int kTileW = 256;  // bytes of every row staged per tile
constexpr int kMaxSeg = 32;  // chunk segments for the column scan
constexpr int kItemsPerCol = 8;

enum { XF_RAW = 0, XF_CLASSIFY = 1, XF_SIMPLIFY = 2 };
template <int V>
struct IntC {  // a compile-time int passed to generic lambdas
  static constexpr int value = V;
};
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F &f, std::integer_sequence<int, I...>) {
  (f(IntC<I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F &&f) {  // f(IntC<0>{}), ..., f(IntC<N - 1>{})
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

__host__ __device__ __forceinline__ int mode_nclass(int mode) {
  return mode == KBZ_MODE_DYNAMORIO ? 1 : 3;
}
__host__ __device__ __forceinline__ int class_of(int mode, int outcome) {
  if (mode == KBZ_MODE_DYNAMORIO) return 0;
  return (outcome == KBZ_FUZZ_HANG) ? 1 : (outcome == KBZ_FUZZ_CRASH) ? 2 : 0;
}
// transform applied to traces of virgin class k
__host__ __device__ __forceinline__ int class_xf(int mode, int k) {
  if (mode == KBZ_MODE_DYNAMORIO) return XF_CLASSIFY;
  if (k != 0) return XF_SIMPLIFY;
  return mode == KBZ_MODE_AFL_CLASSIFY ? XF_CLASSIFY : XF_RAW;
}

__device__ __forceinline__ uint64_t xform8(uint64_t x, int xf) {
  if (xf == XF_CLASSIFY) return classify8(x);
  if (xf == XF_SIMPLIFY) return simplify8(x);
  return x;
}

// OR of a 32-bit value over the 64 lanes of the wave (DPP row shifts + row broadcasts).
__device__ __forceinline__ uint32_t wave_or32(uint32_t v) {
  v |= __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v |= __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v |= __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v |= __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v |= __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v |= __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ uint64_t wave_or64(uint64_t v) {
  return (uint64_t)wave_or32((uint32_t)v) | ((uint64_t)wave_or32((uint32_t)(v >> 32)) << 32);
}
// value of lane-1 (lane 0 gets 0): DPP wave_shr:1, no LDS round trip
__device__ __forceinline__ uint64_t from_prev_lane(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_update_dpp(0u, (uint32_t)v, 0x138, 0xf, 0xf, false);
  const uint32_t hi = __builtin_amdgcn_update_dpp(0u, (uint32_t)(v >> 32), 0x138, 0xf, 0xf, false);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}
// hash32 chain step (afl_progs/hash.h:52-54) as 4 dependent instructions: xor, rotl 27 as two
// v_alignbit (rotr 37), h*5 and +C as v_lshl_add_u64 (the compiler's default is two
// quarter-rate v_mad_u64_u32 on the serial chain).
__device__ __forceinline__ uint64_t h32_step_fast(uint64_t h, uint64_t k) {
  const uint32_t lo = (uint32_t)h ^ (uint32_t)k, hi = (uint32_t)(h >> 32) ^ (uint32_t)(k >> 32);
  const uint32_t rl = __builtin_amdgcn_alignbit(lo, hi, 5);
  const uint32_t rh = __builtin_amdgcn_alignbit(hi, lo, 5);
  uint64_t r = ((uint64_t)rh << 32) | rl, t;
  const uint64_t c = 0x52dce729ull;
  asm("v_lshl_add_u64 %0, %1, 2, %1" : "=v"(t) : "v"(r));
  asm("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(r) : "v"(t), "s"(c));
  return r;
}
// The inverse of h32_mix (a bijection of 64-bit words: both constants are odd), so pass 1 can
// read a transformed word back from the mixed words it leaves in LDS for the chain.
constexpr uint64_t inv_odd64(uint64_t c) {  // c^-1 mod 2^64 (Newton: 5 doublings of 3 bits)
  uint64_t x = c;
  for (int i = 0; i < 5; i++) x *= 2 - c * x;
  return x;
}
constexpr uint64_t kH32C1Inv = inv_odd64(kH32C1), kH32C2Inv = inv_odd64(kH32C2);
static_assert(kH32C1 * kH32C1Inv == 1 && kH32C2 * kH32C2Inv == 1, "h32_mix inverse");
__device__ __forceinline__ uint64_t h32_unmix(uint64_t k) {
  return rotl64(k * kH32C2Inv, 33) * kH32C1Inv;
}
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// Workgroup barrier for LDS hand-offs only.  __syncthreads() is also a release fence for
// global memory: with vmcnt counting loads and stores in issue order, it drains this wave's
// in-flight prefetch loads whenever a global store was issued after them.  Here only LDS
// must be ordered: wait for this wave's LDS ops, then s_barrier ("memory" keeps the compiler
// from moving memory accesses across it).
// Prefetch loads issued as inline asm: the compiler does not track them, so the caller must
// wait with vmcnt_wait<N>() before reading the registers (N = VMEM ops issued after them).
// Used where the compiler's own counting would drain the prefetch (see k_pass1s).
__device__ __forceinline__ void asm_load16(u32x4 &r, const uint8_t *p) {
  asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(r) : "v"(p) : "memory");
}
template <int N>
__device__ __forceinline__ void vmcnt_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// The same wait naming the ring slot's registers "+v" (cdna_hip_programming.md, asm loads form
// (ii)): no consumer of them, a register copy included, is scheduled above it.
template <int N>
__device__ __forceinline__ void vmcnt_wait_ring(u32x4 (&r)[2]) {
  asm volatile("s_waitcnt vmcnt(%2)" : "+v"(r[0]), "+v"(r[1]) : "n"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void vmcnt_wait_ring(u32x4 (&r)[18]) {  // k_pass1d: + ignore words
  asm volatile("s_waitcnt vmcnt(%18)"
               : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]),
                 "+v"(r[6]), "+v"(r[7]), "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]),
                 "+v"(r[12]), "+v"(r[13]), "+v"(r[14]), "+v"(r[15]), "+v"(r[16]), "+v"(r[17])
               : "n"(N)
               : "memory");
}
template <int N>
__device__ __forceinline__ void vmcnt_wait_ring(u32x4 (&r)[17]) {  // k_pass1n: 16 rows + virgin
  asm volatile("s_waitcnt vmcnt(%17)"
               : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]),
                 "+v"(r[6]), "+v"(r[7]), "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]),
                 "+v"(r[12]), "+v"(r[13]), "+v"(r[14]), "+v"(r[15]), "+v"(r[16])
               : "n"(N)
               : "memory");
}
template <int N>
__device__ __forceinline__ void vmcnt_wait_ring(u32x4 (&r)[3]) {
  asm volatile("s_waitcnt vmcnt(%3)" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]) : "n"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void vmcnt_wait_ring(u32x4 (&r)[4]) {
  asm volatile("s_waitcnt vmcnt(%4)"
               : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3])
               : "n"(N)
               : "memory");
}
template <int N>
__device__ __forceinline__ void vmcnt_wait_ring(u32x4 (&r)[5]) {
  asm volatile("s_waitcnt vmcnt(%5)"
               : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4])
               : "n"(N)
               : "memory");
}
template <int N>
__device__ __forceinline__ void vmcnt_wait_ring(u32x4 (&r)[8]) {
  asm volatile("s_waitcnt vmcnt(%8)"
               : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]),
                 "+v"(r[6]), "+v"(r[7])
               : "n"(N)
               : "memory");
}
template <int N>
__device__ __forceinline__ void vmcnt_wait_ring(u32x4 (&r)[9]) {
  asm volatile("s_waitcnt vmcnt(%9)"
               : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]),
                 "+v"(r[6]), "+v"(r[7]), "+v"(r[8])
               : "n"(N)
               : "memory");
}
// The same with a wave-uniform 64-bit base in SGPRs and a 32-bit per-lane offset (the saddr
// form): moving the base costs SALU only, no 64-bit VALU address add per load.
__device__ __forceinline__ void asm_load16_s(u32x4 &r, uint32_t voff, const uint8_t *sbase) {
  asm volatile("global_load_dwordx4 %0, %1, %2 nt" : "=v"(r) : "v"(voff), "s"(sbase) : "memory");
}
__device__ __forceinline__ void asm_load16_s_cached(u32x4 &r, uint32_t voff, const uint8_t *sbase) {
  asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(r) : "v"(voff), "s"(sbase) : "memory");
}
// cached (not nontemporal) 16-B load: data every workgroup re-reads (the virgin maps)
__device__ __forceinline__ void asm_load16_cached(u32x4 &r, const uint8_t *p) {
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
}
// Drain every asm load, keeping their destination registers live up to the wait: an asm
// load's output looks ready to the compiler, so once it is dead the compiler may reuse the
// register while the load is still in flight (the late write would clobber it).
template <int DD, int NL>
__device__ __forceinline__ void drain_asm_loads(const u32x4 (&r)[DD][NL]) {
#pragma unroll
  for (int d = 0; d < DD; d++)
#pragma unroll
    for (int i = 0; i < NL; i++) asm volatile("" ::"v"(r[d][i]));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int d = 0; d < DD; d++)
#pragma unroll
    for (int i = 0; i < NL; i++) asm volatile("" ::"v"(r[d][i]));
}
// Diagnostic build only (-DKBZ_STAMPS): per-wave cycle accounting of pass 1's step phases,
// read back by tools/stamps.py through kbz_debug_stamps().  No stamp executes otherwise.
#ifdef KBZ_STAMPS
__device__ unsigned long long g_kbz_stamps[4096 * 2 * 4];
__device__ __forceinline__ unsigned long long stamp_now() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define KBZ_STAMP_DECL unsigned long long st_acc[4] = {0, 0, 0, 0}, st_t = stamp_now()
#define KBZ_STAMP(i) do { const unsigned long long _n = stamp_now(); st_acc[i] += _n - st_t; st_t = _n; } while (0)
#define KBZ_STAMP_FLUSH(slot) do { if ((threadIdx.x & 63) == 0 && (slot) < 8192u) { for (int _i = 0; _i < 4; _i++) g_kbz_stamps[(slot) * 4 + _i] = st_acc[_i]; } } while (0)
#else
#define KBZ_STAMP_DECL do {} while (0)
#define KBZ_STAMP(i) do {} while (0)
#define KBZ_STAMP_FLUSH(slot) do {} while (0)
#endif
// Diagnostic build only (-DKBZ_TAIL_STAMPS): per-wave records of the tail kernels (100-MHz
// s_memrealtime at entry / after the prologue / at exit, work counters), read back by
// tools/tail_stamps.py through kbz_debug_tail().  No record is written otherwise.
#ifdef KBZ_TAIL_STAMPS
constexpr int kTailRecs = 1 << 16;
constexpr int kTailFields = 8;  // t0, prologue end, end, work counters, 4 phase sums (k_tail)
__device__ unsigned long long g_kbz_tail[kTailRecs * kTailFields];
__device__ __forceinline__ unsigned long long rt_now() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
constexpr uint32_t kFinStampBase = kTailRecs / 2;  // k_fin's records (k_tail's below)
#define KBZ_TAIL_DECL unsigned long long tl_t0 = rt_now(), tl_t1 = 0, tl_last = 0, tl_ph[4] = {0, 0, 0, 0}; uint32_t tl_walk = 0, tl_claims = 0, tl_flush = 0, tl_win = 0
#define KBZ_TAIL_MARK() (tl_t1 = tl_last = rt_now())
#define KBZ_TAIL_ADD(f, v) (tl_##f += (v))
// phase sums of k_tail's walk (the stamp build waits for every load at each phase end, so a
// phase's loads are charged to it): 0 group loads, 1 per-chunk claims, 2 record scores, 3 flushes
#define KBZ_TAIL_PH(i) do { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); const unsigned long long _n = rt_now(); tl_ph[i] += _n - tl_last; tl_last = _n; } while (0)
#define KBZ_TAIL_END(id) do { const unsigned long long _e = rt_now(); const uint32_t _i = (id); \
    if ((threadIdx.x & 63) == 0 && _i < (uint32_t)kTailRecs) { unsigned long long *_r = g_kbz_tail + (size_t)_i * kTailFields; _r[0] = tl_t0; _r[1] = tl_t1 ? tl_t1 : _e; \
    _r[2] = _e; _r[3] = ((unsigned long long)tl_walk << 48) | ((unsigned long long)(tl_claims & 0xffff) << 32) | ((tl_flush & 0xffff) << 16) | (tl_win & 0xffff); \
    for (int _p = 0; _p < 4; _p++) _r[4 + _p] = tl_ph[_p]; } } while (0)
#else
constexpr uint32_t kFinStampBase = 0;
#define KBZ_TAIL_DECL do {} while (0)
#define KBZ_TAIL_MARK() do {} while (0)
#define KBZ_TAIL_ADD(f, v) do {} while (0)
#define KBZ_TAIL_PH(i) do {} while (0)
#define KBZ_TAIL_END(id) do {} while (0)
#endif
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
// The same barrier written with builtins, so the compiler's wait-count pass sees that every LDS
// operation issued before it is complete: after the inline-asm form it still waits lgkmcnt(0)
// for loads whose results were already in registers, before the first use of any of them
// (k_pass1w keeps a tile's words in registers across a barrier).  The empty asm statements are
// compiler memory fences (the s_barrier builtin is not one).
__device__ __forceinline__ void lds_barrier_seen() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xc07f);  // vmcnt(63) expcnt(7) lgkmcnt(0): LDS only
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
// streaming 16-B load of data read exactly once (nontemporal: do not keep it in L2)
__device__ __forceinline__ uint4 ld_stream16(const uint8_t *p) {
  const u32x4 v = __builtin_nontemporal_load((const u32x4 *)p);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint64_t ld_u64(const uint4 &v, int e) {
  return e ? ((uint64_t)v.z | ((uint64_t)v.w << 32)) : ((uint64_t)v.x | ((uint64_t)v.y << 32));
}
__device__ __forceinline__ uint4 or4(uint4 a, uint4 b) {
  return make_uint4(a.x | b.x, a.y | b.y, a.z | b.z, a.w | b.w);
}
__device__ __forceinline__ uint4 classify16(uint4 a) {
  return make_uint4(classify4(a.x), classify4(a.y), classify4(a.z), classify4(a.w));
}
__device__ __forceinline__ uint32_t byte_xform(uint32_t b, int xf) {
  if (xf == XF_CLASSIFY) return classify4(b) & 0xff;
  if (xf == XF_SIMPLIFY) return b ? 0x80u : 0x01u;
  return b;
}

// k_pass1w shape (timing variants override them with -D): transform waves, loader waves, their
// register ring depth, wave L's priority
#ifndef KBZ_WIDE_NX
#define KBZ_WIDE_NX 8
#endif
#ifndef KBZ_WIDE_NL
#define KBZ_WIDE_NL 4
#endif
#ifndef KBZ_WIDE_D
#define KBZ_WIDE_D 3  // 3 vs 2: config 3 pass 1 3.75-3.77 vs 3.81-3.86 ms same-box (profiles/r02_final2)
#endif
#ifndef KBZ_WIDE_LPRIO
#define KBZ_WIDE_LPRIO 3
#endif
#ifndef KBZ_PASS1_SROWS  // timing variants: 0 = per-word reductions for every class
#define KBZ_PASS1_SROWS 1
#endif
#ifndef KBZ_SROWS_MAX
#define KBZ_SROWS_MAX 16  // 8, 16, 32 equal at 2 % hangs + crashes; 4 is slower (profiles/r02_v19)
#endif
#ifndef KBZ_PASS1_LPRE  // k_pass1s wave L: iterations (2 LDS slots each) read ahead (1 or 2)
#define KBZ_PASS1_LPRE 1
#endif
#ifndef KBZ_PASS1_TPRE  // k_pass1s wave T: LDS slots read this many slots ahead (1 or 4)
#define KBZ_PASS1_TPRE 8  // 1 / 4 / 8: 0.80 / 0.767 / 0.744 ms, profiles/r03_v10
#endif
#ifndef KBZ_PASS1_TMIX  // which modes' mix wave T computes (see k_pass1s); 0 = none
#define KBZ_PASS1_TMIX 3
#endif
#ifndef KBZ_P1S_LEARLY  // k_pass1s wave L: issue each step's loads before its chain (ring D + 1)
#define KBZ_P1S_LEARLY 1
#endif
#ifndef KBZ_P1S_GROUP  // k_pass1s DynamoRIO: nonzero words transformed G at a time (0: one by one)
#define KBZ_P1S_GROUP 4
#endif
#ifndef KBZ_P1S_ORGATE  // k_pass1s: column ORs only for words where some row holds a virgin bit
#define KBZ_P1S_ORGATE 1
#endif
#ifndef KBZ_WIDE_PEEL  // k_pass1w transform waves: steady steps without bounds tests
#define KBZ_WIDE_PEEL 1
#endif
#ifndef KBZ_WIDE_BAL
#define KBZ_WIDE_BAL 1
#endif

// k_pass1s: which instantiations have wave T compute the hash32 mix (KBZ_PASS1_TMIX), and which
// write claim records -- one predicate for the kernel and the host (shard_begin_impl decides
// from it whether k_tail may read records).
__host__ __device__ constexpr bool p1s_tmix(int mode, bool x64) {
  return !x64 && (KBZ_PASS1_TMIX == 2 || (KBZ_PASS1_TMIX >= 1 && mode == KBZ_MODE_AFL) ||
                  (KBZ_PASS1_TMIX == 3 && mode == KBZ_MODE_DYNAMORIO));
}
__host__ __device__ constexpr bool p1s_records(int mode, bool ign, bool x64) {
  return p1s_tmix(mode, x64) && mode == KBZ_MODE_DYNAMORIO && !ign;
}
struct Pass1Args {
  const uint8_t *traces;
  size_t stride;
  uint32_t n;
  uint32_t map_size;
  const int8_t *outcome;
  const uint8_t *ignore;
  uint32_t *h32;        // internal [n]
  uint64_t *x64;        // user [n] or null
  uint8_t *neq;         // [n]: transformed trace differs from the previous one (relevant bytes)
  uint8_t *chunk_or;    // [chunks][nclass][map_size]
  uint8_t *chunk_cls;   // [chunks] bitmask of classes present
  uint32_t *shard_last; // [2]
  uint8_t *segor;       // [nseg][nclass][map_size], zero on entry: OR'ed into with atomics
  uint32_t seg_len;     // chunks per segment
  const uint8_t *vcur;  // [3][map_size] virgin maps at batch entry
  uint64_t *tflags;     // [chunks][nclass][nfw]: bit t%64 of word t/64 = tile t of chunk_or stored
  uint32_t nfw;         // flag words per (chunk, class) = ceil(tiles / 64)
  uint64_t *frec;       // [chunks][map_size] claim records (k_pass1s DynamoRIO without ignore
                        // bytes / XXH64, one-shard batches) or null
  uint64_t *rflags;     // [chunks][nfw]: bit t%64 of word t/64 = tile t's records written
  uint32_t epoch;       // this batch's record tag (1..1023)
  // One-shard DynamoRIO batches through k_pass1s (kbz_triage_batch_device): k_skip's rule runs
  // in the kernel's epilogue (p1s_skip_rule), so no k_skip launch follows.  skip == null: k_skip.
  uint8_t *skip;        // [n] out: row j repeats row j-1's hash (row 0: the context's last hash)
  uint32_t *fix_flags, *fix_list, *fix_cnt, *bad_list, *bad_cnt;  // bad rows (as k_skip)
  uint64_t *lastpub;    // [chunks]: tag << 32 | hash of the chunk's last row (look-back)
  uint32_t tag;         // this batch's look-back tag (never 0)
  const uint32_t *row0_hp;  // row 0's predecessor hash
  int pred_saved;           // the saved row (the previous batch's last) is valid ...
  const uint32_t *pred_ok;  // ... and clean iff *pred_ok
  const uint8_t *prow;      // the saved row
  uint32_t *bad0;           // out: row 0 is skipped and differs / has an unknown predecessor
  uint32_t *err;            // sticky error flags (a look-back that never completes: 512)
  uint32_t spin_max;        // look-back polls before that (tests force 0: the fallback path)
};
#ifndef KBZ_REC_MAX_WORDS  // a stored tile with more words holding still-virgin bits gets no
#define KBZ_REC_MAX_WORDS 2  // records (fresh maps, novelty-heavy batches): its claims read rows
#endif                       // (one ballot per stored tile; a byte count cost novelty pass 1 +30 %)
// Claim record of one still-virgin byte of one chunk (pass 1, stored tiles only): for each bit t
// of the byte that is still virgin at batch entry, the first row of the chunk holding it (bits
// 6t..6t+5), the first row whose byte is nonzero (48..53), the batch tag (54..63).  A claim of
// the tail then needs one 8-B load instead of that byte of all 64 rows (DynamoRIO, chunks off
// the fix list: a skipped row repeats an earlier row's bytes, so the first holder of a bit is
// never one, see k_tail).
constexpr int kRecEpochShift = 54;
constexpr uint32_t kRecEpochMask = 1023;

// Rows x and y differ on the examined (classified, not ignored) bytes: this thread's part of
// the map (16 B every `step` bytes from `first`), 8 pairs of loads in flight.
__device__ __forceinline__ int rows_differ_part(const uint8_t *x, const uint8_t *y,
                                                const uint8_t *ignore, uint32_t map_size,
                                                uint32_t first, uint32_t step) {
  int diff = 0;
#pragma unroll 8
  for (uint32_t i = first; i < map_size; i += step) {
    const uint4 a = *(const uint4 *)(x + i), b = *(const uint4 *)(y + i);
    const uint64_t a0 = classify8((uint64_t)a.x | ((uint64_t)a.y << 32));
    const uint64_t a1 = classify8((uint64_t)a.z | ((uint64_t)a.w << 32));
    const uint64_t b0 = classify8((uint64_t)b.x | ((uint64_t)b.y << 32));
    const uint64_t b1 = classify8((uint64_t)b.z | ((uint64_t)b.w << 32));
    uint64_t r0 = ~0ull, r1 = ~0ull;
    if (ignore) {
      const uint4 g = *(const uint4 *)(ignore + i);
      r0 = ~nonzero_bytes8((uint64_t)g.x | ((uint64_t)g.y << 32));
      r1 = ~nonzero_bytes8((uint64_t)g.z | ((uint64_t)g.w << 32));
    }
    diff |= (((a0 ^ b0) & r0) | ((a1 ^ b1) & r1)) != 0;
  }
  return diff;
}
__device__ void p1s_skip_rule(const Pass1Args &a, uint32_t *sh, int wave, int lane,
                              uint32_t chunk, uint64_t row0, int nrows);

// ---------------------------------------------------------------------------------------------
// pass 1: two waves per 64-trace chunk (lane = trace) sharing two 16-KiB LDS tile buffers.
// Both waves stream: each loads half of every tile's rows (8 x 1-KiB coalesced wave-loads per
// tile) into a ring of D register buffers, D tiles ahead.  A single loader wave per chunk
// cannot keep enough loads in flight (tools/patprobe: ~4.5 TB/s vs ~6.6 TB/s with two).
// Measured on MI355X (profiles/r01_v5): D = 2, 3, 4, 6 all give 0.757-0.764 ms per 4 GiB
// batch, so the default is D = 2 (KBZ_PASS1_DEPTH; fewest VGPRs).
//   wave L: fills rows 0-31 of tile s+1, runs the serial per-trace chains (hash32 mix+step,
//           optional XXH64) over tile s-1 after wave T transformed it;
//   wave T: fills rows 32-63 of tile s, then per word transforms it in place (classify /
//           simplify), ORs each column over the 64 traces (DPP), DynamoRIO equality with the
//           previous trace; stores the chunk's column ORs and ORs them into the segment
//           aggregate (64-bit atomics, nonzero words only).
// Step s = 0..ntiles, rounded up to a multiple of D (no early exit from the unrolled ring:
// every exit point would need its own copy of the ring registers), one barrier per step: T fills+transforms tile s in buffer s&1 while L
// chains tile s-1 and then refills that buffer with its half of tile s+1.  16-B slot q of row r
// lives at slot q ^ (r & 15): fills (ds_write_b128, 4 rows per instruction) and the
// row-per-lane ds_read_b128 are both bank-conflict-free.  Raw zero words stay 0 in LDS; a
// simplified trace's transformed word is never 0, so L maps an untouched 0 of a simplified
// lane to 0x0101010101010101.
// ---------------------------------------------------------------------------------------------
template <int MODE, bool IGN, bool X64, int D>
__global__ __launch_bounds__(128, 2) void k_pass1s(Pass1Args a) {
  constexpr int NC = (MODE == KBZ_MODE_DYNAMORIO) ? 1 : 3;
  // AFL mode: wave T also computes the hash32 mix of every word it transforms and leaves it in
  // LDS for wave L (T only simplifies the few hang/crash rows there, L was the slower wave:
  // pass 1 1.23 -> 1.13 ms, profiles/r02_v18).  DynamoRIO and AFL_CLASSIFY keep the mix on L:
  // T's classify makes T the busier wave there.  XXH64 needs the transformed words on L.
  // KBZ_PASS1_TMIX: 1 = AFL only, 2 = every mode, 3 (default) = AFL and DynamoRIO.  With T
  // mixing, wave L is a bare chain: DynamoRIO config 2 pass 1 -2 % same-box since wave T reads
  // its slots 8 ahead (profiles/r03_v13); AFL_CLASSIFY stays on L (+3 % with T mixing).
  constexpr bool TMIX = p1s_tmix(MODE, X64);
  // claim records (a.frec): DynamoRIO with the mix in LDS and every byte examined
  constexpr bool REC = p1s_records(MODE, IGN, X64);
  // AFL modes: the simplified classes' column ORs come from their rows, once per tile
  constexpr bool SROWS = KBZ_PASS1_SROWS && NC > 1;
  constexpr int TW = 256, SLOTS = 16, RPI = 4, NLD = 8;  // 8 x 1-KiB loads per wave per tile
  constexpr int TILE = kChunk * SLOTS;                     // uint4 per tile buffer
  // 2 tile buffers (32 KiB) + 8 KiB: wave T's virgin words (2 x 768 B) and padding, at most 4
  // chunks per CU, so 1,024 chunks spread over all 256 CUs
  __shared__ uint4 lds[2 * TILE + 512];
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const uint32_t chunk = blockIdx.x;
  const uint64_t row0 = (uint64_t)chunk * kChunk;
  const int nrows = (int)min((uint64_t)kChunk, (uint64_t)a.n - row0);
  const bool valid = lane < nrows;
  const int oc = (valid && a.outcome) ? a.outcome[row0 + lane] : KBZ_FUZZ_NONE;
  const int cls = class_of(MODE, oc);
  const int xf = valid ? class_xf(MODE, cls) : XF_RAW;
  const bool simp = (xf == XF_SIMPLIFY);
  const uint32_t ntiles = a.map_size / TW;

  // this wave's half of the rows: rows past the end of a partial chunk re-read its last row
  // (those lanes are invalid: masked out of the ORs, hashes not stored)
  const int lr = lane / SLOTS, ls = lane % SLOTS;
  const uint8_t *lbase = a.traces + row0 * a.stride + ls * 16;
  uint32_t roff[NLD];  // < 64 rows x stride <= 32 MiB: fits 32 bits
#pragma unroll
  for (int i = 0; i < NLD; i++)
    roff[i] = (uint32_t)(min(32 * wave + RPI * i + lr, nrows - 1) * a.stride);
  // Prefetch: asm loads, waited for by hand (vmcnt counts VMEM ops of this wave in issue
  // order).  Every step issues exactly NLD loads (tiles past the end re-load the chunk's first 256 B), so
  // when a buffer is consumed exactly D-1 younger load groups exist -> vmcnt((D-1)*NLD).
  // Wave T's global stores are younger still: the count is a lower bound, which is safe.
  // Branch-free: an if/else around the asm loads would merge their outputs with register
  // copies the compiler believes are safe while the loads are still in flight.
  auto load_half = [&](u32x4 (&r)[NLD], uint32_t t) {
    const uint32_t msk = t < ntiles ? ~0u : 0u;
#pragma unroll
    for (int i = 0; i < NLD; i++) asm_load16(r[i], lbase + ((t * TW + roff[i]) & msk));
  };
  auto store_half = [&](const u32x4 (&r)[NLD], int b) {
#pragma unroll
    for (int i = 0; i < NLD; i++) {
      const int rr = 32 * wave + RPI * i + lr;
      const u32x4 v = r[i];
      lds[b * TILE + rr * SLOTS + (ls ^ (rr & 15))] = make_uint4(v.x, v.y, v.z, v.w);
    }
  };
  // L's register ring is one slot deeper than T's: each step issues its next loads BEFORE the
  // chain and stores the oldest slot after it, so the chain no longer delays L's loads (the
  // chain-free ablation was 4 % faster, profiles/r05/ab_p1s_ablations_d2.txt).  Both waves run
  // the same number of steps (barriers): 0..ntiles rounded up to a multiple of both rings, so
  // neither unrolled loop needs a guard around its asm loads.
  constexpr int DL = KBZ_P1S_LEARLY ? D + 1 : D;
  constexpr int SP = DL == D ? D : D * DL;
  const uint32_t nsteps = (ntiles + SP) / SP * SP;
  uint32_t h32v = 0, neqv = 0;  // this lane's row: hash (L), differs from the previous row (T)
  if (wave == 0) {
    u32x4 R[DL][NLD];
#pragma unroll
    for (int d = 0; d < DL; d++) load_half(R[d], d);
    // ------------------------------------------------------------------ wave L
    uint64_t h = (uint64_t)(kHashConst ^ a.map_size);
    uint64_t x0 = kXP1 + kXP2, x1 = kXP2, x2 = 0, x3 = 0 - kXP1;
    const uint64_t ksimp = h32_mix(kSimpleZero);
    auto chain_tile = [&](uint32_t t, int b) {
      const uint64_t *ig = IGN ? (const uint64_t *)(a.ignore + (size_t)t * TW) : nullptr;
      const uint4 *row = &lds[b * TILE + lane * SLOTS];
      const int sw = lane & 15;
      uint4 v0 = row[0 ^ sw], v1 = row[1 ^ sw];
      constexpr int LP = KBZ_PASS1_LPRE;  // iterations (of 2 slots) read ahead
      uint4 u0 = LP > 1 ? row[2 ^ sw] : v0, u1 = LP > 1 ? row[3 ^ sw] : v1;
#pragma unroll LP
      for (int q = 0; q < SLOTS; q += 2) {
        // software pipeline: the next LP x 2 slots are in flight while these 4 words chain
        const int qn = (q + 2 * LP) & (SLOTS - 1);
        const uint4 n0 = row[qn ^ sw], n1 = row[(qn + 1) ^ sw];
#pragma unroll
        for (int qq = 0; qq < 2; qq++) {
          const uint4 v = qq ? v1 : v0;
#pragma unroll
          for (int e = 0; e < 2; e++) {
            const int wi = 2 * (q + qq) + e;
            const uint64_t w = ld_u64(v, e);
            uint64_t tw, k;
            if (TMIX) {  // wave T left the word's hash32 mix (0 only for a raw 0 word)
              tw = 0;
              k = (simp && w == 0) ? ksimp : w;
            } else if (__ballot(w != 0)) {
              tw = (simp && w == 0) ? kSimpleZero : w;
              k = h32_mix(tw & (IGN ? ig[wi] : ~0ull));
            } else {
              tw = simp ? kSimpleZero : 0;
              k = simp ? ksimp : 0;
            }
            h = h32_step_fast(h, k);
            if (X64) {
              const int xl = (2 * qq + e) & 3;
              if (xl == 0) x0 = xx_round(x0, tw);
              else if (xl == 1) x1 = xx_round(x1, tw);
              else if (xl == 2) x2 = xx_round(x2, tw);
              else x3 = xx_round(x3, tw);
            }
          }
        }
        if (LP > 1) {
          v0 = u0;
          v1 = u1;
          u0 = n0;
          u1 = n1;
        } else {
          v0 = n0;
          v1 = n1;
        }
      }
    };
    // prologue: own half of tile 0 -> buffer 0 (T transforms it at step 0)
    vmcnt_wait<(DL - 1) * NLD>();
    store_half(R[0], 0);
    if (DL == D) load_half(R[0], D);
    lds_barrier();  // (A)
    KBZ_STAMP_DECL;
    if (DL > D) {
      // step s: prefetch tile s+DL into ring slot (s+DL)%DL (its tile s was stored last step),
      // chain tile s-1, store own half of tile s+1 (slot (s+1)%DL) into the buffer just chained
      for (uint32_t g = 0; g < nsteps; g += DL) {
#pragma unroll
        for (int u = 0; u < DL; u++) {
          const uint32_t s = g + u;
          load_half(R[u], s + DL);
          if (s >= 1 && s <= ntiles) chain_tile(s - 1, (s - 1) & 1);
          KBZ_STAMP(0);
          vmcnt_wait<(DL - 1) * NLD>();
          KBZ_STAMP(1);
          store_half(R[(u + 1) % DL], (s + 1) & 1);
          KBZ_STAMP(2);
          lds_barrier();
          KBZ_STAMP(3);
        }
      }
    } else {
      // step s: chain tile s-1, store own half of tile s+1 (ring slot (s+1)%D) into the buffer
      // just chained, prefetch tile s+1+D into that slot.
      for (uint32_t g = 0; g < nsteps; g += D) {
#pragma unroll
        for (int u = 0; u < D; u++) {
          const uint32_t s = g + u;
          if (s >= 1 && s <= ntiles) chain_tile(s - 1, (s - 1) & 1);
          KBZ_STAMP(0);
          vmcnt_wait<(D - 1) * NLD>();
          KBZ_STAMP(1);
          store_half(R[(u + 1) % D], (s + 1) & 1);
          load_half(R[(u + 1) % D], s + 1 + D);
          KBZ_STAMP(2);
          lds_barrier();
          KBZ_STAMP(3);
        }
      }
    }
    KBZ_STAMP_FLUSH(chunk * 2 + 0);
    drain_asm_loads(R);
    if (valid) {
      // (the no-chain ablation stores distinct hashes, so nothing downstream sees repeats)
      const uint32_t h32 = h32_final(h);
      a.h32[row0 + lane] = h32;
      h32v = h32;
      // the next chunk's row 0 compares with this chunk's last row: publish its hash at once
      if (MODE == KBZ_MODE_DYNAMORIO && a.skip && lane == nrows - 1 && chunk + 1 < gridDim.x)
        __hip_atomic_store(&a.lastpub[chunk], ((uint64_t)a.tag << 32) | h32, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      if (X64 && a.x64) {
        uint64_t xh = rotl64(x0, 1) + rotl64(x1, 7) + rotl64(x2, 12) + rotl64(x3, 18);
        xh = xx_merge(xh, x0);
        xh = xx_merge(xh, x1);
        xh = xx_merge(xh, x2);
        xh = xx_merge(xh, x3);
        xh += a.map_size;
        a.x64[row0 + lane] = xx_avalanche(xh);
      }
      if (row0 + lane == (uint64_t)a.n - 1) {
        a.shard_last[0] = h32;
        atomicOr(&a.shard_last[1], 1u);  // (the fused skip rule ORs its bits in meanwhile)
      }
    }
  } else {
    // ------------------------------------------------------------------ wave T
    uint64_t present[NC];
    // every simplified class has at most KBZ_SROWS_MAX rows in this chunk: their column ORs
    // come from their rows, once per tile (wave-uniform; crash-heavy chunks take the other path)
    bool rowwise = SROWS;
#pragma unroll
    for (int k = 0; k < NC; k++) {
      present[k] = __ballot(valid && cls == k);
      if (k > 0 && __popcll(present[k]) > KBZ_SROWS_MAX) rowwise = false;
    }
    if (lane == 0) {
      uint8_t m = 0;
#pragma unroll
      for (int k = 0; k < NC; k++) m |= present[k] ? (1u << k) : 0u;
      a.chunk_cls[chunk] = m;
    }
    uint64_t neq = 0;
    const uint32_t seg = chunk / a.seg_len;
    // Virgin words of each tile travel with its rows: a 9th ring register per slot (lane l < 16 NC
    // loads 16 B of class l / 16), stored to a per-buffer LDS area next to the tile, so T can
    // limit its stores to words that still hold virgin bits (below).
    u32x4 R[D][NLD + 1];
    const uint32_t vl = min(lane, 16 * NC - 1);
    const uint8_t *vbase = a.vcur + (size_t)(vl / 16) * a.map_size + (vl % 16) * 16;
    auto load_t = [&](u32x4 (&r)[NLD + 1], uint32_t t) {
      load_half(*(u32x4(*)[NLD])r, t);
      const uint32_t msk = t < ntiles ? ~0u : 0u;
      asm_load16_cached(r[NLD], vbase + ((t * TW) & msk));
    };
    auto store_t = [&](const u32x4 (&r)[NLD + 1], int b) {
      store_half(*(const u32x4(*)[NLD])r, b);
      if (lane < 16 * NC) {
        const u32x4 v = r[NLD];
        lds[2 * TILE + b * 48 + lane] = make_uint4(v.x, v.y, v.z, v.w);
      }
    };
#pragma unroll
    for (int d = 0; d < D; d++) load_t(R[d], d);
    uint64_t tfl[NC];  // stored-tile bits of the current 64-tile flag word
#pragma unroll
    for (int k = 0; k < NC; k++) tfl[k] = 0;
    uint64_t rfl = 0;  // records-written bits of the current 64-tile flag word
    uint64_t *tfbase = a.tflags + (size_t)chunk * NC * a.nfw;
    // claim records of a stored tile (rare on a warm map): the words with still-virgin bits are
    // read back from the tile buffer (mixed for wave L, which chains it next step) and unmixed
    auto tile_records = [&](uint32_t s, int b, uint64_t m) {
      const uint4 *rw = &lds[b * TILE + lane * SLOTS];
      const int sw = lane & 15;
      uint64_t wm = __ballot(lane < TW / 8 && m != 0);
      if (__popcll(wm) > KBZ_REC_MAX_WORDS) return false;
      uint64_t *fr = a.frec + (size_t)chunk * a.map_size + (size_t)s * TW;
      const uint64_t ep = (uint64_t)a.epoch << kRecEpochShift;
      while (wm) {  // wave-uniform
        const int wi = __builtin_ctzll(wm);
        wm &= wm - 1;
        const uint64_t mw = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(m >> 32), wi) << 32) |
                            __builtin_amdgcn_readlane((uint32_t)m, wi);
        const uint64_t kq = ((const uint64_t *)&rw[(wi >> 1) ^ sw])[wi & 1];
        const uint64_t tw = valid ? h32_unmix(kq) : 0ull;
        for (int bb = 0; bb < 8; bb++) {
          const uint32_t mb = (uint32_t)(mw >> (8 * bb)) & 0xffu;
          if (!mb) continue;  // uniform
          const uint32_t byte = (uint32_t)(tw >> (8 * bb)) & 0xffu;
          const uint64_t nz = __ballot(byte != 0);
          uint64_t rec = ep | ((uint64_t)(nz ? __builtin_ctzll(nz) : 63) << 48);
          for (int t = 0; t < 8; t++) {
            if (!((mb >> t) & 1)) continue;
            const uint64_t bm = __ballot((byte >> t) & 1);
            rec |= (uint64_t)(bm ? __builtin_ctzll(bm) : 63) << (6 * t);
          }
          if (lane == 0) fr[wi * 8 + bb] = rec;
        }
      }
      return true;
    };
    auto transform_tile = [&](uint32_t s, auto rwc) {
      constexpr bool RW = decltype(rwc)::value;  // simplified classes ORed row-wise (few rows)
      const int b = s & 1;
      const uint64_t *ig = IGN ? (const uint64_t *)(a.ignore + (size_t)s * TW) : nullptr;
      uint64_t orw[NC];
#pragma unroll
      for (int k = 0; k < NC; k++) orw[k] = 0;
      if (RW) {
        // hang / crash classes with few rows in the chunk (the usual case: 2 % of execs): OR their
        // raw rows word-parallel (lane = word), before the word loop rewrites the tile in place --
        // instead of a 64-lane reduction per class for every nonzero word (AFL pass 1 1.15 ->
        // 0.80 ms, profiles/r02_v19).  simplify8(0) = 0x01 bytes covers words that are zero in
        // every row.  Crash-heavy chunks keep the per-word reductions.
        const uint64_t *tile = (const uint64_t *)&lds[b * TILE];
        const int wl = lane & 31;  // lanes 32-63 duplicate 0-31 (only lanes < 32 are stored)
#pragma unroll
        for (int k = 1; k < NC; k++) {
          uint64_t acc = 0;
          for (uint64_t mm = present[k]; mm; mm &= mm - 1) {
            const int rr = __builtin_ctzll(mm);  // wave-uniform
            acc |= simplify8(tile[(rr * SLOTS + ((wl >> 1) ^ (rr & 15))) * 2 + (wl & 1)]);
          }
          orw[k] = acc;
        }
      }
      uint4 *row = &lds[b * TILE + lane * SLOTS];
      const int sw = lane & 15;
      // the tile's virgin words at batch entry, lane w < 32 holding word w of each class
      uint64_t vlane[NC];
#pragma unroll
      for (int k = 0; k < NC; k++)
        vlane[k] = ((const uint64_t *)&lds[2 * TILE + b * 48 + k * 16])[lane & 31];
      if constexpr (MODE == KBZ_MODE_DYNAMORIO && KBZ_P1S_GROUP > 0) {
        // DynamoRIO: the nonzero words of the tile in groups of G, each group's G words
        // transformed, mixed and compared side by side.  Processed one word at a time (the loop
        // below) every nonzero word was a dependent chain of ~40 instructions behind a branch --
        // at two waves per SIMD wave T spent 87 % of each step in that latency
        // (profiles/r05_c/stamps_k_pass1s.txt).  (1) one 32-bit mask of the words that are nonzero
        // in some row; (2) groups of G set bits (the last group padded with its last word: a word
        // processed twice gives the same results), each word re-read from the tile buffer by a
        // uniform index, written back mixed for wave L.
        constexpr int G = KBZ_P1S_GROUP > 0 ? KBZ_P1S_GROUP : 1;  // (the branch is dead at 0)
        uint32_t nzm = 0;
        {
          uint4 vv[SLOTS];
#pragma unroll
          for (int q = 0; q < SLOTS; q++) vv[q] = row[q ^ sw];
#pragma unroll
          for (int q = 0; q < SLOTS; q++) {
            nzm |= __ballot((vv[q].x | vv[q].y) != 0) ? 1u << (2 * q) : 0u;
            nzm |= __ballot((vv[q].z | vv[q].w) != 0) ? 1u << (2 * q + 1) : 0u;
          }
        }
        uint64_t *roww = (uint64_t *)row;
        while (nzm) {  // wave-uniform
          int w[G];
          int last = 0;
#pragma unroll
          for (int g = 0; g < G; g++) {
            if (nzm) {
              last = __builtin_ctz(nzm);
              nzm &= nzm - 1;
            }
            w[g] = last;
          }
          uint64_t tw[G];
#pragma unroll
          for (int g = 0; g < G; g++) tw[g] = roww[(((w[g] >> 1) ^ sw) << 1) | (w[g] & 1)];
#pragma unroll
          for (int g = 0; g < G; g++) tw[g] = classify8(tw[g]);
#pragma unroll
          for (int g = 0; g < G; g++) {
            const uint64_t out = TMIX ? h32_mix_mad(tw[g] & (IGN ? ig[w[g]] : ~0ull)) : tw[g];
            roww[(((w[g] >> 1) ^ sw) << 1) | (w[g] & 1)] = out;
          }
          if (present[0]) {
            uint64_t c[G], any = 0;
#pragma unroll
            for (int g = 0; g < G; g++) {
              const uint64_t vw =
                  ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(vlane[0] >> 32), w[g]) << 32) |
                  __builtin_amdgcn_readlane((uint32_t)vlane[0], w[g]);
              c[g] = valid ? (tw[g] & vw) : 0ull;
              any |= c[g];
            }
            if (__ballot(any != 0)) {  // some row holds a still-virgin bit (rare on a warm map)
              uint64_t r[G];  // the G reductions side by side (no branch between them)
#pragma unroll
              for (int g = 0; g < G; g++) r[g] = wave_or64(c[g]);
#pragma unroll
              for (int g = 0; g < G; g++) orw[0] = (lane == w[g]) ? r[g] : orw[0];
            }
          }
#pragma unroll
          for (int g = 0; g < G; g++) {
            const uint64_t rel = IGN ? ~nonzero_bytes8(ig[w[g]]) : ~0ull;
            neq |= (tw[g] ^ from_prev_lane(tw[g])) & rel;
          }
        }
      } else {
      // slots in flight: a mostly-zero slot takes a few instructions, far less than an LDS round
      // trip (deeper register rings, timing-only builds, keep 2: their VGPRs are spent)
      constexpr int TP = D > 2 ? 2 : KBZ_PASS1_TPRE;
      uint4 vring[TP];
#pragma unroll
      for (int j = 0; j < TP; j++) vring[j] = row[j ^ sw];
#pragma unroll 1
      for (int q0 = 0; q0 < SLOTS; q0 += TP)
#pragma unroll
      for (int u = 0; u < TP; u++) {
        const int q = q0 + u;
        uint4 *slot = &row[q ^ sw];
        uint4 v = vring[u];
        vring[u] = row[((q + TP) & (SLOTS - 1)) ^ sw];  // (wraps at the end: discarded)
        bool dirty = false;
#pragma unroll
        for (int e = 0; e < 2; e++) {
          const int wi = 2 * q + e;
          const uint64_t x = ld_u64(v, e);
          if (__ballot(x != 0)) {
            const uint64_t tw = xform8(x, xf);
            // what wave L chains next step (with ignore bytes the mix sees the kept bytes only)
            const uint64_t out = TMIX ? h32_mix_mad(tw & (IGN ? ig[wi] : ~0ull)) : tw;
            if (e) { v.z = (uint32_t)out; v.w = (uint32_t)(out >> 32); }
            else { v.x = (uint32_t)out; v.y = (uint32_t)(out >> 32); }
            dirty = true;
#pragma unroll
            for (int k = 0; k < (RW ? 1 : NC); k++) {
              if (present[k]) {
                if (KBZ_P1S_ORGATE) {
                  // only bits still virgin at batch entry are kept (m = OR & V below): the
                  // 64-lane reduction runs only when some row of the class holds one in this word
                  // (on a warm map almost never: config 2 pass 1 -5 %, the no-OR ablation)
                  const uint64_t vw =
                      ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(vlane[k] >> 32), wi) << 32) |
                      __builtin_amdgcn_readlane((uint32_t)vlane[k], wi);
                  const uint64_t c = (valid && cls == k) ? (tw & vw) : 0;
                  if (__ballot(c != 0)) {
                    const uint64_t r = wave_or64(c);
                    orw[k] = (lane == wi) ? r : orw[k];
                  }
                } else {
                  const uint64_t r = wave_or64((valid && cls == k) ? tw : 0);
                  orw[k] = (lane == wi) ? r : orw[k];
                }
              }
            }
            if (MODE == KBZ_MODE_DYNAMORIO) {
              const uint64_t rel = IGN ? ~nonzero_bytes8(ig[wi]) : ~0ull;
              neq |= (tw ^ from_prev_lane(tw)) & rel;
            }
          } else if (MODE != KBZ_MODE_DYNAMORIO && !RW) {
#pragma unroll
            for (int k = 1; k < NC; k++)  // simplified classes see 0x01 bytes everywhere
              if (present[k]) orw[k] = (lane == wi) ? kSimpleZero : orw[k];
          }
        }
        // raw AFL words are their own transform (only simplified lanes change) unless T mixes
        if (dirty && (TMIX || MODE != KBZ_MODE_AFL || simp)) *slot = v;
      }
      }
      // chunk_or keeps only bits still virgin at batch entry (orw & V): the scan uses nothing
      // else (its new bits are o & V & ~prev, and f2 only looks at bytes with V == 0xff), and a
      // tile with none is not stored at all, only its flag bit stays clear.  In steady-state
      // fuzzing almost no tile is stored, which keeps these stores (and the drain of the
      // prefetch they cause: vmcnt counts them) off the stream.
#pragma unroll
      for (int k = 0; k < NC; k++) {
        if (!present[k]) continue;
        const size_t off = (size_t)k * a.map_size + (size_t)s * TW + (size_t)lane * 8;
        const uint64_t m = orw[k] & vlane[k];
        if (__ballot(lane < TW / 8 && m != 0)) {
          tfl[k] |= 1ull << (s & 63);
          if (lane < TW / 8)
            *(uint64_t *)(a.chunk_or + (size_t)chunk * NC * a.map_size + off) = m;
          if (REC && a.frec && tile_records(s, b, m)) rfl |= 1ull << (s & 63);
        }
        // segment aggregate, restricted to still-virgin bits like chunk_or (its consumers only
        // use it under & V: k_scan's segment test and V' = V & ~total): almost never an atomic
        if (lane < TW / 8 && m)
          atomicOr((unsigned long long *)(a.segor + (size_t)seg * NC * a.map_size + off),
                   (unsigned long long)m);
        if ((s & 63) == 63 || s + 1 == ntiles) {
          if (lane == 0) tfbase[k * a.nfw + (s >> 6)] = tfl[k];
          tfl[k] = 0;
          if (REC && a.frec) {
            if (lane == 0) a.rflags[(size_t)chunk * a.nfw + (s >> 6)] = rfl;
            rfl = 0;
          }
        }
      }
    };
    lds_barrier();  // (A): L's half of tile 0 is in buffer 0
    KBZ_STAMP_DECL;
    // step s: store own half of tile s (ring slot s%D), prefetch tile s+D into that slot,
    // transform tile s.  T issues NLD + NC loads per step.
    for (uint32_t g = 0; g < nsteps; g += D) {
#pragma unroll
      for (int u = 0; u < D; u++) {
        const uint32_t s = g + u;
        vmcnt_wait_ring<(D - 1) * (NLD + 1)>(R[u]);
        KBZ_STAMP(1);
        store_t(R[u], s & 1);
        load_t(R[u], s + D);
        KBZ_STAMP(2);
        if (s < ntiles) {
          if (SROWS && rowwise) transform_tile(s, IntC<1>{});
          else transform_tile(s, IntC<0>{});
        }
        KBZ_STAMP(0);
        lds_barrier();
        KBZ_STAMP(3);
      }
    }
    KBZ_STAMP_FLUSH(chunk * 2 + 1);
    drain_asm_loads(R);
    // lane 0 has no predecessor in the wave: its value is a placeholder (k_skip compares a chunk's
    // row 0 with the previous row itself, and only when their hashes are equal)
    if (MODE == KBZ_MODE_DYNAMORIO && valid) a.neq[row0 + lane] = neq != 0;
    neqv = neq != 0;
  }
  if (MODE == KBZ_MODE_DYNAMORIO && a.skip) {  // k_skip's rule for this chunk's rows
    lds_barrier();  // both waves are past their last reads of the tile buffers
    uint32_t *sh = (uint32_t *)lds;
    sh[wave * 64 + lane] = wave == 0 ? h32v : neqv;
    p1s_skip_rule(a, sh, wave, lane, chunk, row0, nrows);
  }
}

// k_skip's rule for one chunk of a fused one-shard DynamoRIO batch, in k_pass1s's epilogue: the
// outputs of k_skip's row blocks, chunk-start blocks and row-0 block for these rows.  sh[0..63]
// the rows' hashes, sh[64..127] "differs from the previous row" (pass 1's neighbour test; lane
// 0's is a placeholder).  The chunk's row 0 is compared with its predecessor: the previous
// chunk's last row, whose hash that workgroup's wave L published in lastpub (a look-back on a
// lower workgroup: dispatched earlier, and it publishes before any wait of its own), or for
// chunk 0 the saved row; when the hashes are equal, the two rows themselves (both waves).
// hash32 of one DynamoRIO row as pass 1 chains it (hash32_with_ignore over the classified map,
// winafl_hash.h:80-112; without ignore bytes the plain hash32, afl_progs/hash.h:36-65): one lane,
// direct loads
__device__ uint32_t row_hash32_dr(const uint8_t *row, const uint8_t *ignore, uint32_t map_size) {
  uint64_t h = (uint64_t)(kHashConst ^ map_size);
  for (uint32_t w = 0; w < map_size / 8; w++) {
    uint64_t k = classify8(*(const uint64_t *)(row + 8 * (size_t)w));
    if (ignore) k &= *(const uint64_t *)(ignore + 8 * (size_t)w);
    h = h32_step(h, h32_mix(k));
  }
  return h32_final(h);
}
// look-back polls (Pass1Args::spin_max, default 2^20 x ~2 us: a look-back never ends in seconds)
__device__ void p1s_skip_rule(const Pass1Args &a, uint32_t *sh, int wave, int lane,
                              uint32_t chunk, uint64_t row0, int nrows) {
  if (wave == 1 && lane == 0) {
    uint32_t hp = 0, known = 1;
    if (chunk == 0) {  // (a shard of the sharded protocol: k_chain links row 0, row0_hp null)
      hp = a.row0_hp ? *a.row0_hp : ~sh[0];
      known = a.row0_hp && a.pred_saved && *a.pred_ok != 0;
    } else {
      // polls back off to one per ~2 us: on uneven batches (fresh maps) hundreds of workgroups
      // wait here at once, and tight agent-scope polls take bandwidth from the ones still
      // streaming
      uint32_t backoff = 1;
      for (uint32_t it = 0;; it++) {
        const uint64_t pv = __hip_atomic_load(&a.lastpub[chunk - 1], __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
        hp = (uint32_t)pv;
        if ((uint32_t)(pv >> 32) == a.tag) break;
        if (it >= a.spin_max) {
          // the lower workgroup never published: the stall is reported (512), and the
          // predecessor's hash is recomputed from its row here (8 K dependent steps: a path
          // that should never run), so the skip rule below stays exact
          atomicOr(a.err, 512u);
          hp = row_hash32_dr(a.traces + (row0 - 1) * a.stride, a.ignore, a.map_size);
          break;
        }
        for (uint32_t z = 0; z < backoff; z++) __builtin_amdgcn_s_sleep(8);
        backoff = backoff < 8 ? 2 * backoff : 8;
      }
    }
    sh[128] = hp;
    sh[129] = known;
  }
  lds_barrier();
  const bool known = sh[129] != 0;
  const bool sk0 = sh[0] == sh[128];  // workgroup-uniform
  bool diff = false;
  if (sk0 && (chunk > 0 || known)) {  // uniform: the rows themselves, half the map per wave
    // (chunk 0 of a shard never gets here: its stand-in hash differs from row 0's)
    const uint8_t *x = a.traces + row0 * a.stride;
    const uint8_t *y = chunk > 0 ? x - a.stride : a.prow;
    const int d = rows_differ_part(x, y, a.ignore, a.map_size, threadIdx.x * 16, blockDim.x * 16);
    const bool any = __ballot(d) != 0;
    if (lane == 0) sh[130 + wave] = any;
    lds_barrier();
    diff = (sh[130] | sh[131]) != 0;
  }
  if (wave != 1) return;
  const uint64_t j = row0 + lane;
  bool applied = false, bad = false;
  if (lane == 0) {
    if (chunk > 0) {
      a.skip[j] = sk0;
      applied = !sk0;
      if (sk0) a.neq[j] = diff;  // exact now: the chain walks read it
      bad = sk0 && diff;
    } else if (a.row0_hp) {  // one shard: row 0 against the saved row (k_chain's role)
      a.skip[j] = sk0;
      *a.bad0 = sk0 && (!known || diff);
    }
  } else if (lane < nrows) {
    const bool sk = sh[lane] == sh[lane - 1];
    a.skip[j] = sk;
    applied = !sk;
    bad = sk && sh[64 + lane] != 0;
  }
  if (bad) {  // rare (hash collisions): the chunk to the fix list, the row to the chain walks
    if (atomicExch(&a.fix_flags[chunk], 1u) == 0u) a.fix_list[atomicAdd(a.fix_cnt, 1u)] = chunk;
    a.bad_list[atomicAdd(a.bad_cnt, 1u)] = (uint32_t)j;
  }
  const uint32_t want = (__ballot(bad) ? 2u : 0u) | (__ballot(applied) ? 4u : 0u);
  if (lane == 0 && (want & ~__hip_atomic_load(&a.shard_last[1], __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT)))
    atomicOr(&a.shard_last[1], want);
}

// k_pass1w row groups.  X wave xi transforms two groups of wide_rg(xi) consecutive rows (one
// per half-wave); groups 2 xi and 2 xi + 1 in row order.  Balanced layout (NX = 8, NL = 4): the
// workgroup's waves are dealt to the 4 SIMDs cyclically, so X_0 and X_4 share a SIMD with wave
// L, whose hash chain takes about four row-words of that SIMD's issue per step: they get 3 and
// 2 rows per group, the others 5 and 4 (9 row-words per SIMD per step, L included).
template <int NX, int NL>
__host__ __device__ constexpr int wide_rg(int xi) {
  return (KBZ_WIDE_BAL && NX == 8 && NL == 4)
             ? ((xi & 3) == 0 ? (xi < 4 ? 3 : 2) : (xi < 4 ? 5 : 4))
             : kChunk / (2 * NX);
}
template <int NX, int NL>
__host__ __device__ constexpr int wide_gstart(int g) {
  int r = 0;
  for (int i = 0; i < g; i++) r += wide_rg<NX, NL>(i / 2);
  return r;
}
template <int NX, int NL>
__host__ __device__ constexpr bool wide_groups_ok() {
  return wide_gstart<NX, NL>(2 * NX) == kChunk;
}
// the RG a switch case instantiates: the case's own value where some wave uses it, else the
// uniform size (keeps unused instantiations out of the binary)
template <int NX, int NL>
__host__ __device__ constexpr int wide_rg_or(int rg) {
  for (int i = 0; i < NX; i++)
    if (wide_rg<NX, NL>(i) == rg) return rg;
  return kChunk / (2 * NX);
}

// ---------------------------------------------------------------------------------------------
// pass 1, wide-map variant (few chunks: a batch of large maps, e.g. BASELINE config 3 with
// 16,384 x 1 MiB = 256 chunks, one per CU).  k_pass1s would run one 2-wave workgroup per CU and
// be compute-bound twice over (config 3: 27.2 ms per batch).  Here the per-word work is spread
// over NX transform waves and the serial chain is cut to its dependent part:
//   loaders  waves 0..NL-1 load 64/NL rows each of tile s into a D-deep register ring and store
//            it to LDS at step s (NL = 4: two waves per chunk reach 4.8 TB/s on this pattern,
//            four 6.0-6.2 TB/s, tools/widebw);
//   L        wave 0 (also a loader, at raised priority) chains tile s-3: per word only the
//            hash32 step (xor, rotl, *5+C) on the mixed word the X waves computed (+ XXH64);
//   X_i      read tile s-1's words from LDS into registers at step s, transform them at step
//            s+1 -- so no LDS latency is ever waited for before computing -- COLUMN-wise: lane
//            (w = lane % 32, half h = lane / 32) owns word w of the rows of row group
//            g = 2 i + h (64 / (2 NX) consecutive rows).  Per (row, word): classify / simplify,
//            the hash32 mix k = h32_mix(word & ignore) into the k buffer (and the transformed
//            word into twb for XXH64), a plain per-lane OR per class, the DynamoRIO neighbour
//            test against the previous row of the same lane (one ballot per row; group
//            boundaries are compared one step later through LDS).  The groups' ORs meet in LDS
//            (ds_or_b64); X_0 stores them (chunk_or, segment atomics) one step later.  X waves
//            issue no asm loads, so their stores disturb no counted wait.
// Tile t: raw[t & 1] filled at step t and read at t+1; kbuf / twb[t & 1] written at t+2 and
// chained at t+3; its ORs in orb[t & 1] from t+2 to t+3.  Steps s = 0..ntiles+2 rounded up to
// a multiple of D, one barrier each (its lgkmcnt(0) completes every LDS read issued in the
// step).  k values use the tile's swizzled [row][slot] layout, so the X writes (32 lanes per
// row) and L's row-per-lane ds_read_b128 are both conflict-free.  Same vmcnt accounting as
// k_pass1s for the loaders.  LDS 65 KiB (97 KiB with XXH64): one workgroup per CU.
// ---------------------------------------------------------------------------------------------
template <int MODE, bool IGN, bool X64, int NX, int NL, int D>
__global__ __launch_bounds__(64 * (NL + NX), 1) void k_pass1w(Pass1Args a) {
  static_assert(NL == 2 || NL == 4 || NL == 8, "64/NL rows per loader, 4 rows per wave-load");
  static_assert(kChunk % (2 * NX) == 0 && wide_groups_ok<NX, NL>(), "row groups cover the chunk");
  constexpr int NC = (MODE == KBZ_MODE_DYNAMORIO) ? 1 : 3;
  constexpr int TW = 256, SLOTS = 16, RPI = 4, RPW = kChunk / NL, NLD = RPW / RPI;
  constexpr int TILE = kChunk * SLOTS;  // uint4 per tile buffer
  __shared__ uint4 raw[2 * TILE];
  __shared__ uint4 kbuf[2 * TILE];              // k of each (row, word), same layout as raw
  __shared__ uint4 twb[X64 ? 2 * TILE : 1];     // transformed words (XXH64 input)
  __shared__ uint64_t orb[2][NC][TW / 8];       // column ORs of the tile, per class
  __shared__ uint64_t bnd[2][2 * NX][TW / 8];   // last row of each group (neighbour test)
  __shared__ uint64_t neqs[NX];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // uniform: SGPR
  const int lane = threadIdx.x & 63;
  const uint32_t chunk = blockIdx.x;
  const uint64_t row0 = (uint64_t)chunk * kChunk;
  const int nrows = (int)min((uint64_t)kChunk, (uint64_t)a.n - row0);
  const bool valid = lane < nrows;
  const int oc = (valid && a.outcome) ? a.outcome[row0 + lane] : KBZ_FUZZ_NONE;
  const int cls = class_of(MODE, oc);
  const uint32_t ntiles = a.map_size / TW;
  const uint32_t nsteps = ntiles + 3;
  const uint32_t nb = (nsteps + D - 1) / D * D;  // steps (= barriers) of every wave

  if (wave < NL) {
    // ------------------------------------------------------------ loader waves (wave 0 = L)
    const bool isL = wave == 0;
    const int li = wave;
    const int lr = lane / SLOTS, ls = lane % SLOTS;
    const uint8_t *lbase = a.traces + row0 * a.stride + ls * 16;
    uint32_t roff[NLD];
#pragma unroll
    for (int i = 0; i < NLD; i++)
      roff[i] = (uint32_t)(min(RPW * li + RPI * i + lr, nrows - 1) * a.stride);
    auto load_part = [&](u32x4 (&r)[NLD], uint32_t t) {  // branch-free (see k_pass1s)
      const uint32_t msk = t < ntiles ? ~0u : 0u;
#pragma unroll
      for (int i = 0; i < NLD; i++) asm_load16(r[i], lbase + ((t * TW + roff[i]) & msk));
    };
    auto store_part = [&](const u32x4 (&r)[NLD], int b) {
#pragma unroll
      for (int i = 0; i < NLD; i++) {
        const int rr = RPW * li + RPI * i + lr;
        const u32x4 v = r[i];
        raw[b * TILE + rr * SLOTS + (ls ^ (rr & 15))] = make_uint4(v.x, v.y, v.z, v.w);
      }
    };
    uint64_t h = (uint64_t)(kHashConst ^ a.map_size);
    uint64_t x0 = kXP1 + kXP2, x1 = kXP2, x2 = 0, x3 = 0 - kXP1;
    // all 16 slots of the lane's row are read first: one LDS wait per tile, then 32 steps
    auto chain_tile = [&](uint32_t t) {
      const int b = t & 1;
      const int sw = lane & 15;
      uint4 kk[SLOTS];
#pragma unroll
      for (int q = 0; q < SLOTS; q++) kk[q] = kbuf[b * TILE + lane * SLOTS + (q ^ sw)];
#pragma unroll
      for (int q = 0; q < SLOTS; q++) {
        h = h32_step_fast(h, (uint64_t)kk[q].x | ((uint64_t)kk[q].y << 32));
        h = h32_step_fast(h, (uint64_t)kk[q].z | ((uint64_t)kk[q].w << 32));
      }
      if (X64) {
#pragma unroll 4
        for (int q = 0; q < SLOTS; q++) {
          const uint4 v = twb[b * TILE + lane * SLOTS + (q ^ sw)];
#pragma unroll
          for (int e = 0; e < 2; e++) {
            const uint64_t tw = ld_u64(v, e);
            const int xl = (2 * q + e) & 3;
            if (xl == 0) x0 = xx_round(x0, tw);
            else if (xl == 1) x1 = xx_round(x1, tw);
            else if (xl == 2) x2 = xx_round(x2, tw);
            else x3 = xx_round(x3, tw);
          }
        }
      }
    };
    {  // the whole ring lives inside this wave-uniform branch
      if (isL) __builtin_amdgcn_s_setprio(KBZ_WIDE_LPRIO);  // the chain is the critical path
      u32x4 R[D][NLD];
#pragma unroll
      for (int d = 0; d < D; d++) load_part(R[d], d);
      KBZ_STAMP_DECL;
      for (uint32_t g = 0; g < nb; g += D) {
#pragma unroll
        for (int u = 0; u < D; u++) {
          const uint32_t s = g + u;
          if (isL && s >= 3 && s - 3 < ntiles) chain_tile(s - 3);
          KBZ_STAMP(0);
          vmcnt_wait_ring<(D - 1) * NLD>(R[u]);
          KBZ_STAMP(2);
          store_part(R[u], s & 1);
          load_part(R[u], s + D);
          KBZ_STAMP(3);
          lds_barrier_seen();
          KBZ_STAMP(1);
        }
      }
      KBZ_STAMP_FLUSH(chunk * 16 + wave);
      drain_asm_loads(R);
    }
    lds_barrier_seen();  // (Z): the X waves' neighbour flags are in neqs
    if (isL && valid) {
      const uint32_t h32 = h32_final(h);
      a.h32[row0 + lane] = h32;
      if (X64 && a.x64) {
        uint64_t xh = rotl64(x0, 1) + rotl64(x1, 7) + rotl64(x2, 12) + rotl64(x3, 18);
        xh = xx_merge(xh, x0);
        xh = xx_merge(xh, x1);
        xh = xx_merge(xh, x2);
        xh = xx_merge(xh, x3);
        xh += a.map_size;
        a.x64[row0 + lane] = xx_avalanche(xh);
      }
      if (row0 + lane == (uint64_t)a.n - 1) {
        a.shard_last[0] = h32;
        a.shard_last[1] = 1;
      }
    }
    if (li == 1 && MODE == KBZ_MODE_DYNAMORIO && valid) {
      uint64_t nq = 0;
#pragma unroll
      for (int i = 0; i < NX; i++) nq |= neqs[i];
      a.neq[row0 + lane] = (nq >> lane) & 1;
    }
  } else {
    // ------------------------------------------------------------ waves X_i (column-wise)
    const int xi = wave - NL;
    auto xwave = [&](auto rgc) {
    constexpr int RG = decltype(rgc)::value;  // rows per group of this wave
    const int w = lane & 31, hf = lane >> 5;
    const int grp = 2 * xi + hf;
    const int r0 = wide_gstart<NX, NL>(grp);  // this lane's rows: r0 .. r0 + RG - 1
    const int r0a = wide_gstart<NX, NL>(2 * xi), r0b = r0a + RG;  // the wave's two groups
    uint64_t present[NC];
#pragma unroll
    for (int k = 0; k < NC; k++) present[k] = __ballot(valid && cls == k);
    // 2-bit class code of each of this lane's rows.  A row past the end of a partial chunk
    // holds a copy of the chunk's last row (the loaders clamp) and takes that row's class: OR-ing
    // a copy into the class aggregate changes nothing, so no row needs masking.
    uint32_t clsw = 0;
    if (NC > 1) {
#pragma unroll
      for (int i = 0; i < RG; i++) {
        const int r = min(r0 + i, nrows - 1);
        uint32_t c = 0;
#pragma unroll
        for (int k = 1; k < NC; k++) c = ((present[k] >> r) & 1) ? (uint32_t)k : c;
        clsw |= c << (2 * i);
      }
    }
    if (xi == 0) {
      if (lane == 0) {
        uint8_t m = 0;
#pragma unroll
        for (int k = 0; k < NC; k++) m |= present[k] ? (1u << k) : 0u;
        a.chunk_cls[chunk] = m;
      }
      for (int i = lane; i < 2 * NC * (TW / 8); i += 64) (&orb[0][0][0])[i] = 0;
    }
    const uint32_t seg = chunk / a.seg_len;
    const uint64_t *igp = IGN ? (const uint64_t *)a.ignore + w : nullptr;
    uint64_t ig_next = IGN ? igp[0] : ~0ull;  // ignore word of the next tile (prefetched)
    // per row i of this wave's two groups: OR over tiles of the ballot "differs from the row
    // before" (wave-uniform: SGPR pairs, one s_or per row and tile); bit r of the chunk's neq
    // mask comes from its half at the end
    uint64_t nacc[RG];
#pragma unroll
    for (int i = 0; i < RG; i++) nacc[i] = 0;
    uint64_t ftw = 0, frel = ~0ull;  // first row's word / rel mask of the last transformed tile
    // byte offset of this lane's word in each of its rows, in tile buffer 0 (buffer b: + b TILE)
    uint32_t adr[RG];
#pragma unroll
    for (int i = 0; i < RG; i++) {
      const int r = r0 + i;
      adr[i] = (uint32_t)(r * SLOTS + ((w >> 1) ^ (r & 15))) * 16u + (uint32_t)(w & 1) * 8u;
    }
    // words of two tiles in registers: xw[t & 1] holds tile t from its read (step t+1) to its
    // transform (step t+2).  The step loop is unrolled by 2, so every buffer and register set
    // index is a constant and each LDS access is a per-row base plus an immediate offset.
    uint64_t xw[2][RG];
#pragma unroll
    for (int j = 0; j < 2; j++)
#pragma unroll
      for (int i = 0; i < RG; i++) xw[j][i] = 0;
    auto read_tile = [&](uint32_t t, auto bc) {
      constexpr int b = decltype(bc)::value;  // t & 1
      const char *tb = (const char *)&raw[b * TILE];
#pragma unroll
      for (int i = 0; i < RG; i++) xw[b][i] = *(const uint64_t *)(tb + adr[i]);
    };
    auto transform_tile = [&](uint32_t t, auto bc) {
      constexpr int b = decltype(bc)::value;  // t & 1
      const uint64_t igw = ig_next;
      if (IGN) ig_next = igp[(size_t)min(t + 1, ntiles - 1) * (TW / 8)];
      const uint64_t rel = IGN ? ~nonzero_bytes8(igw) : ~0ull;
      uint64_t tw[RG];
#pragma unroll
      for (int i = 0; i < RG; i++) {
        tw[i] = xw[b][i];
        const uint32_t c = (clsw >> (2 * i)) & 3;
        if (MODE == KBZ_MODE_DYNAMORIO) tw[i] = classify8(tw[i]);
        else if (c != 0) tw[i] = simplify8(tw[i]);
        else if (MODE == KBZ_MODE_AFL_CLASSIFY) tw[i] = classify8(tw[i]);
      }
      if (X64) {
        char *xb = (char *)&twb[b * TILE];
#pragma unroll
        for (int i = 0; i < RG; i++) *(uint64_t *)(xb + adr[i]) = tw[i];
      }
      char *kb = (char *)&kbuf[b * TILE];
#pragma unroll
      for (int i = 0; i < RG; i++) {
        *(uint64_t *)(kb + adr[i]) = h32_mix_mad(tw[i] & igw);
      }
      uint64_t ow[NC];
#pragma unroll
      for (int k = 0; k < NC; k++) ow[k] = 0;
#pragma unroll
      for (int i = 0; i < RG; i++) {
        if (NC == 1) {
          ow[0] |= tw[i];
        } else {
          const uint32_t c = (clsw >> (2 * i)) & 3;
#pragma unroll
          for (int k = 0; k < NC; k++) ow[k] |= (c == (uint32_t)k) ? tw[i] : 0;
        }
      }
      if (MODE == KBZ_MODE_DYNAMORIO) {
#pragma unroll
        for (int i = 1; i < RG; i++) nacc[i] |= __ballot(((tw[i] ^ tw[i - 1]) & rel) != 0);
        ftw = tw[0];
        bnd[b][grp][w] = tw[RG - 1];
        frel = rel;
      }
#pragma unroll
      for (int k = 0; k < NC; k++)
        if (present[k] && (KBZ_WIDE_PEEL || ow[k]))  // (dense maps: a zero OR is rare)
          atomicOr((unsigned long long *)&orb[b][k][w], (unsigned long long)ow[k]);
    };
    // X_0: the virgin words of tile t, loaded into vpre[t & 1] at the end of step t+1, two
    // steps before finish_tile(t) needs them
    uint64_t vpre[2][NC];
#pragma unroll
    for (int j = 0; j < 2; j++)
#pragma unroll
      for (int k = 0; k < NC; k++) vpre[j][k] = 0;
    auto load_virgin = [&](uint32_t t, auto bc) {
      constexpr int b = decltype(bc)::value;  // t & 1
#pragma unroll
      for (int k = 0; k < NC; k++)
        if (present[k] && lane < TW / 8)
          vpre[b][k] = *(const uint64_t *)(a.vcur + (size_t)k * a.map_size + (size_t)t * TW +
                                          (size_t)lane * 8);
    };
    uint64_t tfl[NC];  // X_0: stored-tile bits of the current 64-tile flag word (k_pass1s)
#pragma unroll
    for (int k = 0; k < NC; k++) tfl[k] = 0;
    uint64_t *tfbase = a.tflags + (size_t)chunk * NC * a.nfw;
    // one step after tile t was transformed: group-boundary neighbour test (pl = the previous
    // group's last row, read at the start of the step), and X_0 stores the tile's column ORs
    auto finish_tile = [&](uint32_t t, uint64_t pl, uint64_t fw, uint64_t fr, auto bc) {
      constexpr int b = decltype(bc)::value;  // t & 1
      if (MODE == KBZ_MODE_DYNAMORIO) nacc[0] |= __ballot(((fw ^ pl) & fr) != 0);
      if (xi == 0) {
        // like k_pass1s: chunk_or and the segment aggregate keep only the bits still virgin at
        // batch entry; a tile with none is not stored, its flag bit stays clear
#pragma unroll
        for (int k = 0; k < NC; k++) {
          if (!present[k]) continue;
          const size_t off = (size_t)k * a.map_size + (size_t)t * TW + (size_t)(lane & 31) * 8;
          uint64_t m = 0;
          if (lane < TW / 8) {
            m = orb[b][k][lane] & vpre[b][k];
            orb[b][k][lane] = 0;
          }
          if (__ballot(m != 0)) {
            tfl[k] |= 1ull << (t & 63);
            if (lane < TW / 8) *(uint64_t *)(a.chunk_or + (size_t)chunk * NC * a.map_size + off) = m;
          }
          if (m)
            atomicOr((unsigned long long *)(a.segor + (size_t)seg * NC * a.map_size + off),
                     (unsigned long long)m);
          if ((t & 63) == 63 || t + 1 == ntiles) {
            if (lane == 0) tfbase[k * a.nfw + (t >> 6)] = tfl[k];
            tfl[k] = 0;
          }
        }
      }
    };
    KBZ_STAMP_DECL;
    auto step = [&](uint32_t s, auto pc, auto stc) {
      constexpr int p = decltype(pc)::value;  // s & 1
      constexpr bool ST = decltype(stc)::value;  // 3 <= s <= ntiles: every part runs (no tests)
      // (1) LDS reads, issued first and waited for only after the transform (the LDS queue is
      // long right after the barrier, with every wave's fills, reads and writes): the previous
      // group's last row of tile s-3, then the words of tile s-1 (transformed next step)
      uint64_t pl = 0;
      const bool fin = ST || (s >= 3 && s - 3 < ntiles);
      const bool rd = ST || (s >= 1 && s - 1 < ntiles);
      if (MODE == KBZ_MODE_DYNAMORIO && fin && grp > 0) pl = bnd[p ^ 1][grp - 1][w];
      if (rd) read_tile(s - 1, IntC<p ^ 1>{});
      const uint64_t fw = ftw, fr = frel;  // tile s-3's, from its transform at step s-1
      KBZ_STAMP(2);
      // (2) transform tile s-2 from the registers read at step s-1
      if (ST || (s >= 2 && s - 2 < ntiles)) transform_tile(s - 2, IntC<p>{});
      KBZ_STAMP(0);
      // (3) finish tile s-3
      if (fin) finish_tile(s - 3, pl, fw, fr, IntC<p ^ 1>{});
      // (4) X_0: virgin words of tile s-1 (finished at step s+2; vpre[p ^ 1] was last read by
      // finish_tile(s-3) above)
      if (xi == 0 && rd) load_virgin(s - 1, IntC<p ^ 1>{});
      KBZ_STAMP(3);
      lds_barrier_seen();
      KBZ_STAMP(1);
    };
    uint32_t s0 = 0;
#if KBZ_WIDE_PEEL
    // steps 0-3 and the last ones test which parts run; the steady steps in between do not
    for (; s0 < 4 && s0 < nb; s0 += 2) {
      step(s0, IntC<0>{}, IntC<0>{});
      if (s0 + 1 < nb) step(s0 + 1, IntC<1>{}, IntC<0>{});
    }
    for (; s0 + 1 <= ntiles; s0 += 2) {
      step(s0, IntC<0>{}, IntC<1>{});
      step(s0 + 1, IntC<1>{}, IntC<1>{});
    }
#endif
    for (; s0 < nb; s0 += 2) {
      step(s0, IntC<0>{}, IntC<0>{});
      if (s0 + 1 < nb) step(s0 + 1, IntC<1>{}, IntC<0>{});
    }
    KBZ_STAMP_FLUSH(chunk * 16 + wave);
    uint64_t nm = 0;  // rows that differ from their predecessor
#pragma unroll
    for (int i = 0; i < RG; i++)
      nm |= ((uint64_t)((uint32_t)nacc[i] != 0u) << (r0a + i)) |
            ((uint64_t)((uint32_t)(nacc[i] >> 32) != 0u) << (r0b + i));
    if (lane == 0) neqs[xi] = nm;
    lds_barrier_seen();  // (Z)
    };
    switch (wide_rg<NX, NL>(xi)) {  // wave-uniform
      case 2: xwave(IntC<wide_rg_or<NX, NL>(2)>{}); break;
      case 3: xwave(IntC<wide_rg_or<NX, NL>(3)>{}); break;
      case 4: xwave(IntC<wide_rg_or<NX, NL>(4)>{}); break;
      default: xwave(IntC<wide_rg_or<NX, NL>(5)>{}); break;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// pass 1 without hashes: AFL / AFL_CLASSIFY batches for which neither hash32 nor XXH64 is wanted
// (the reference AFL plugin never hashes: finish_fuzz_round, afl_instrumentation.c:231-274).
// Nothing is serial, so the waves of a chunk need not share a tile: wave w owns a contiguous
// range of the map's tiles (whole 64-tile flag words, so the waves write disjoint tile-flag
// words) and streams all 64 rows of each of its tiles into a D-deep register ring -- ring
// register i holds 16-B slot l % 16 of row 4 i + l / 16 in lane l, the same rows for the whole
// kernel -- plus the tile's virgin words (lane l < 48: class l / 16, slot l % 16).  The column ORs
// come from registers: per lane an OR over its 16 rows with per-lane class masks (class 0: the raw
// row, AFL_CLASSIFY: classified), then across the 4 lanes sharing a slot (permlane16 / 32 swaps).
// Simplified classes (HANG / CRASH rows, simplify_trace :668-706) need no per-row transform: OR
// over rows of simplify(x) is, per byte, 0x80 where some row is nonzero and 0x01 where some row
// is zero, so each lane keeps the OR of the class's raw rows and the AND of their "byte nonzero"
// bits, only over ring registers that hold a row of that class (usually one or two).  Lane group
// g = l / 16 then finishes class g of the tile: chunk_or where V still has bits, the tile flag,
// the segment atomics.  No LDS, no barrier: every wave streams on its own.
// NW = 2 for batches of many chunks (4 chunks per CU), 8 for the wide case (one chunk per CU).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t or_xor16_32(uint32_t v) {  // OR of lanes l, l^16, l^32, l^48
  const auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  const uint32_t w = a[0] | a[1];
  const auto b = __builtin_amdgcn_permlane32_swap(w, w, false, false);
  return b[0] | b[1];
}
__device__ __forceinline__ uint32_t and_xor16_32(uint32_t v) {
  const auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  const uint32_t w = a[0] & a[1];
  const auto b = __builtin_amdgcn_permlane32_swap(w, w, false, false);
  return b[0] & b[1];
}
// bit 7 of every byte: the byte is nonzero (other bits: don't care)
__device__ __forceinline__ uint32_t nz_hi7(uint32_t x) {
  return ((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x;
}
__device__ __forceinline__ u32x4 or_lanes(u32x4 v) {
  return u32x4{or_xor16_32(v.x), or_xor16_32(v.y), or_xor16_32(v.z), or_xor16_32(v.w)};
}
__device__ __forceinline__ u32x4 and_lanes(u32x4 v) {
  return u32x4{and_xor16_32(v.x), and_xor16_32(v.y), and_xor16_32(v.z), and_xor16_32(v.w)};
}
// simplify's OR over rows from the raw rows' OR and the AND of their "nonzero" bits
__device__ __forceinline__ u32x4 simp_or(u32x4 o, u32x4 z) {
  const u32x4 nz = u32x4{nz_hi7(o.x), nz_hi7(o.y), nz_hi7(o.z), nz_hi7(o.w)} & 0x80808080u;
  return nz | ((~z >> 7) & 0x01010101u);
}

template <int MODE, int NW, int D>
__global__ __launch_bounds__(64 * NW, 2) void k_pass1n(Pass1Args a) {
  static_assert(MODE != KBZ_MODE_DYNAMORIO, "DynamoRIO always hashes (last-hash skip)");
  constexpr int NC = 3, TW = 256, SLOTS = 16, RPI = 4, NLD = kChunk / RPI, NR = NLD + 1;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const uint32_t chunk = blockIdx.x;
  const uint64_t row0 = (uint64_t)chunk * kChunk;
  const int nrows = (int)min((uint64_t)kChunk, (uint64_t)a.n - row0);
  const uint32_t ntiles = a.map_size / TW;
  // this wave's tiles [t0, t1): whole flag words (64 tiles each; a.nfw words per class)
  const uint32_t t0 = min(ntiles, a.nfw * wave / NW * 64);
  const uint32_t t1 = min(ntiles, a.nfw * (wave + 1) / NW * 64);
  const uint32_t nb = (t1 - t0 + D - 1) / D * D;  // steps, a multiple of D (0 for an idle wave)
  // classes present in the chunk (wave-uniform; lane = row)
  const int ocl = (lane < nrows && a.outcome) ? a.outcome[row0 + lane] : KBZ_FUZZ_NONE;
  const int clane = class_of(MODE, ocl);
  uint64_t present[NC];
#pragma unroll
  for (int k = 0; k < NC; k++) present[k] = __ballot(lane < nrows && clane == k);
  if (wave == 0 && lane == 0) {
    uint8_t m = 0;
#pragma unroll
    for (int k = 0; k < NC; k++) m |= present[k] ? (1u << k) : 0u;
    a.chunk_cls[chunk] = m;
    if (row0 + kChunk >= (uint64_t)a.n) a.shard_last[1] = 1;  // non-empty (no hash to report)
  }
  // this lane's rows (register i: row 4 i + lr; past the end of a partial chunk: the last row,
  // masked out) and their classes: per lane bit i of cbits[k], per wave bit i of regs[k]
  const int lr = lane / SLOTS, ls = lane % SLOTS;
  const uint8_t *lbase = a.traces + row0 * a.stride + ls * 16;
  uint32_t cbits[NC], regs[NC];
#pragma unroll
  for (int k = 0; k < NC; k++) cbits[k] = regs[k] = 0;
#pragma unroll
  for (int i = 0; i < NLD; i++) {
    const int r = RPI * i + lr;
    const int c = (r < nrows) ? class_of(MODE, a.outcome ? a.outcome[row0 + r] : KBZ_FUZZ_NONE)
                              : -1;
#pragma unroll
    for (int k = 0; k < NC; k++) {
      cbits[k] |= (c == k) ? (1u << i) : 0u;
      regs[k] |= __ballot(c == k) ? (1u << i) : 0u;
    }
  }
  // all-ones where bit i of cbits[k] is set: one v_bfe_i32 at the use (volatile: kept in the
  // loop; hoisted, the masks and their complements cost more VGPRs than the ring)
  auto msk = [&](int k, int i) -> uint32_t {
    uint32_t m;
    asm volatile("v_bfe_i32 %0, %1, %2, 1" : "=v"(m) : "v"(cbits[k]), "n"(i));
    return m;
  };
  const uint32_t vl = min(lane, 16 * NC - 1);
  const uint8_t *vbase = a.vcur + (size_t)(vl / 16) * a.map_size + (vl % 16) * 16;
  const uint32_t rstep = (uint32_t)(RPI * a.stride);  // <= 128 MiB
  const uint32_t rlast = (uint32_t)((nrows - 1) * a.stride);
  // branch-free asm loads (see k_pass1s); tiles past t1 re-load tile t0
  auto load = [&](u32x4 (&r)[NR], uint32_t t) {
    const uint32_t tt = t < t1 ? t : t0;
#pragma unroll
    for (int i = 0; i < NLD; i++) {
      const uint32_t off = min((uint32_t)(i * rstep + lr * a.stride), rlast);
      asm_load16(r[i], lbase + (size_t)tt * TW + off);
    }
    asm_load16_cached(r[NLD], vbase + (size_t)tt * TW);
  };
  const uint32_t seg = chunk / a.seg_len;
  uint64_t *tfbase = a.tflags + (size_t)chunk * NC * a.nfw;
  uint64_t tfl[NC];
#pragma unroll
  for (int k = 0; k < NC; k++) tfl[k] = 0;
  const int g = lane / 16;  // the class this lane group finishes
  u32x4 R[D][NR];
#pragma unroll
  for (int d = 0; d < D; d++) load(R[d], t0 + d);
  for (uint32_t s0 = 0; s0 < nb; s0 += D) {
#pragma unroll
    for (int u = 0; u < D; u++) {
      const uint32_t t = t0 + s0 + u;
      vmcnt_wait_ring<(D - 1) * NR>(R[u]);
      // ---- column ORs of tile t over the chunk's rows, per class
      u32x4 o0 = {0, 0, 0, 0};
#pragma unroll
      for (int i = 0; i < NLD; i++) {
        u32x4 x = R[u][i];
        if (MODE == KBZ_MODE_AFL_CLASSIFY)
          x = u32x4{classify4(x.x), classify4(x.y), classify4(x.z), classify4(x.w)};
        o0 |= x & msk(0, i);
      }
      u32x4 fin[NC];
      fin[0] = or_lanes(o0);
#pragma unroll
      for (int k = 1; k < NC; k++) {
        fin[k] = u32x4{0, 0, 0, 0};
        if (!present[k]) continue;  // wave-uniform, per chunk
        u32x4 ok = {0, 0, 0, 0}, zk = {~0u, ~0u, ~0u, ~0u};
#pragma unroll
        for (int i = 0; i < NLD; i++) {
          if (!(regs[k] & (1u << i))) continue;  // wave-uniform: no row of class k here
          const u32x4 x = R[u][i];
          const uint32_t mk = msk(k, i);
          ok |= x & mk;
          const u32x4 y = x | ~mk;
          zk &= u32x4{nz_hi7(y.x), nz_hi7(y.y), nz_hi7(y.z), nz_hi7(y.w)};
        }
        fin[k] = simp_or(or_lanes(ok), and_lanes(zk));
      }
      // lane group g keeps class g's OR, masked with V (still-virgin bits only, like k_pass1s)
      u32x4 m = g == 0 ? fin[0] : g == 1 ? fin[1] : fin[2];
      m &= R[u][NLD];
      if (g >= NC) m = u32x4{0, 0, 0, 0};
      // m is complete here, so no value of the slot is still live when its registers are
      // reloaded (otherwise the compiler renames the slot and copies it while loads fly)
      asm volatile("" : "+v"(m));
      // the tile's writes before the slot's next loads (as in k_pass1d: written after them, the
      // next step's load-counting wait also waited for the tile just prefetched)
      if (s0 + u < t1 - t0) {
        const bool any = (m.x | m.y | m.z | m.w) != 0;
        const uint64_t bal = __ballot(any);
        const size_t off = (size_t)g * a.map_size + (size_t)t * TW + (size_t)ls * 16;
        if (bal) {  // (rare) a class whose tile has still-virgin bits: its whole 256 B row
          if ((bal >> (16 * g)) & 0xffffull)
            *(uint4 *)(a.chunk_or + (size_t)chunk * NC * a.map_size + off) =
                make_uint4(m.x, m.y, m.z, m.w);
          if (any) {
            unsigned long long *sp =
                (unsigned long long *)(a.segor + (size_t)seg * NC * a.map_size + off);
            const uint64_t lo = (uint64_t)m.x | ((uint64_t)m.y << 32);
            const uint64_t hi = (uint64_t)m.z | ((uint64_t)m.w << 32);
            if (lo) atomicOr(sp, (unsigned long long)lo);
            if (hi) atomicOr(sp + 1, (unsigned long long)hi);
          }
#pragma unroll
          for (int k = 0; k < NC; k++)
            if ((bal >> (16 * k)) & 0xffffull) tfl[k] |= 1ull << (t & 63);
        }
        if ((t & 63) == 63 || t + 1 == t1) {
          if (lane < NC) {
            const uint64_t f = lane == 0 ? tfl[0] : lane == 1 ? tfl[1] : tfl[2];
            if (present[lane]) tfbase[lane * a.nfw + (t >> 6)] = f;
          }
#pragma unroll
          for (int k = 0; k < NC; k++) tfl[k] = 0;
        }
      }
      load(R[u], t + D);  // the ring slot is free again
    }
  }
  drain_asm_loads(R);
}

// ---------------------------------------------------------------------------------------------
// pass 1, DynamoRIO wide-map variant without lock-step (few chunks: BASELINE config 3, 16,384 x
// 1 MiB = 256 chunks, one per CU).  has_new_coverage needs, per trace, the hash32 chain over the
// classified words in order -- 131,072 dependent steps for a 1 MiB map, the floor of any batch --
// and per column the OR over the chunk's rows.  The two halves only meet through an LDS ring of
// RING tiles, NX + 2 waves per workgroup (dealt to the 4 SIMDs cyclically: wave w on SIMD w % 4):
//   C     (wave 0) for t = 0, 1, ...: the 32 dependent hash32 steps of its row over tile t's k
//         words, read (16 ds_read_b128, row per lane) one tile ahead so no LDS wait is ever on
//         the chain; raised priority.  XXH64 (X64) from a ring of classified words.
//   N     (wave 4, C's SIMD partner: light work, so the chain keeps its SIMD's issue) the
//         neighbour test for the DynamoRIO skip: row r's words against row r-1's through DPP
//         wave_shr:1 (the mix is a bijection: k equal <=> classified words equal; with ignore
//         bytes the examined bytes are not the hashed ones, so X also writes classified &
//         examined words to a second ring for N).
//   X     (the other NX waves) each own every NX-th tile (t = x + NX q) and stream all 64 rows of
//         it into a D-deep register ring (the k_pass1n layout: register i = row 4 i + l / 16,
//         16-B slot l % 16), plus the tile's virgin (and ignore) words.  In registers:
//         classify_counts, the column OR (lanes OR-reduced per slot), the still-virgin part
//         stored like k_pass1s (chunk_or, segment atomics; tile flags OR'ed into LDS, written at
//         the end), and the hash32 mix k = h32_mix(word & ignore) into ring slot t % RING
//         (row-major, XOR-swizzled: conflict-free for row-per-lane reads); then ready[slot] = t.
//         A slot is reused once C and N have read it (freed_c / freed_n).
// No barrier inside the tile loop: the waves synchronise only through the LDS flags (polled with
// s_sleep) and one barrier at the end (tile flags, neighbour flags).
// ---------------------------------------------------------------------------------------------
#ifndef KBZ_PASS1D_READ2  // k_pass1d wave C: the next tile's 16 reads in the first half of the chain
#define KBZ_PASS1D_READ2 0
#endif
#ifndef KBZ_PASS1D_CWAIT  // 1: wave C drains its next-tile LDS reads at the end of every tile
#define KBZ_PASS1D_CWAIT 1
#endif
#ifndef KBZ_MAX_FW
#define KBZ_MAX_FW 1024  // tile-flag words per class: maps up to 16 MiB
#endif
template <bool IGN, bool X64, int NX, int RING, int D>
__global__ __launch_bounds__(64 * (NX / 3 * 4), 1) void k_pass1d(Pass1Args a) {
  // X waves are the waves off SIMD 0 (3 of every 4): wave 0 is C, wave 4 is N, wave 8 idles
  static_assert(NX == 6 || NX == 9, "6 or 9 X waves: 8 or 12 waves per workgroup");
  constexpr int TW = 256, SLOTS = 16, RPI = 4, NLD = kChunk / RPI;
  constexpr int NR = NLD + 1 + (IGN ? 1 : 0);  // rows, virgin words, ignore words
  constexpr int TILE = kChunk * SLOTS;          // uint4 per ring slot
  __shared__ uint4 kring[RING * TILE];
  __shared__ uint4 wring[IGN ? RING * TILE : 1];
  __shared__ uint4 tring[X64 ? RING * TILE : 1];
  __shared__ int ready[RING], freed_c[RING], freed_n[RING];
  __shared__ unsigned long long tfl_lds[KBZ_MAX_FW];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const uint32_t chunk = blockIdx.x;
  const uint64_t row0 = (uint64_t)chunk * kChunk;
  const int nrows = (int)min((uint64_t)kChunk, (uint64_t)a.n - row0);
  const uint32_t ntiles = a.map_size / TW;
  for (int i = threadIdx.x; i < (int)a.nfw; i += blockDim.x) tfl_lds[i] = 0;
  if (threadIdx.x < RING) {
    ready[threadIdx.x] = -1;
    freed_c[threadIdx.x] = freed_n[threadIdx.x] = (int)threadIdx.x - RING;  // slot s: tile s
  }
  __syncthreads();
  // the ring flags: relaxed workgroup-scope atomics on the LDS arrays themselves, so they are
  // ds_read/ds_write (a volatile generic pointer compiles to flat accesses, and each of those
  // waits vmcnt(0): every X wave's register-ring loads in flight)
#define KBZ_FLD(arr, i) __hip_atomic_load(&(arr)[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
#define KBZ_FST(arr, i, v) __hip_atomic_store(&(arr)[i], (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
  const uint32_t seg = chunk / a.seg_len;
  const int sw = lane & 15;
  auto wait_ready = [&](uint32_t t) {
    while (KBZ_FLD(ready, t % RING) != (int)t) __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
  };

  if (wave == 0) {
    // ------------------------------------------------------------ C: the chains
    __builtin_amdgcn_s_setprio(3);
    uint64_t h = (uint64_t)(kHashConst ^ a.map_size);
    uint64_t x0 = kXP1 + kXP2, x1 = kXP2, x2 = 0, x3 = 0 - kXP1;
    uint4 kb[2][SLOTS];  // tile t's k words in kb[t & 1], read one tile ahead
    // Slots are compile-time constants (the tile loop is unrolled by the ring size, and by twice
    // that for an odd ring so the kb parity repeats): every LDS address is a loop-invariant
    // register plus an immediate offset, no address arithmetic per read.
    auto read_k = [&](auto bc, auto sc) {  // the words of the tile in slot sc into kb[bc]
      constexpr int b = decltype(bc)::value, sl = decltype(sc)::value;
#pragma unroll
      for (int q = 0; q < SLOTS; q++) kb[b][q] = kring[sl * TILE + lane * SLOTS + (q ^ sw)];
    };
    // chain the tile in kb[b] (slot sl); tile t + 1's words (slot sl + 1) are read meanwhile, one
    // ds_read_b128 per two steps (in the chain's dependency gaps, not as a burst of 16)
    auto chain = [&](auto bc, auto sc) {
      constexpr int b = decltype(bc)::value, sl = decltype(sc)::value, sl1 = (sl + 1) % RING;
#pragma unroll
      for (int q = 0; q < SLOTS; q++) {
        if (KBZ_PASS1D_READ2) {  // two reads per chain step in the first half: all 16 are in
          if (q < SLOTS / 2) {   // flight by mid-tile, none left for the end-of-tile wait
            kb[b ^ 1][2 * q] = kring[sl1 * TILE + lane * SLOTS + ((2 * q) ^ sw)];
            kb[b ^ 1][2 * q + 1] = kring[sl1 * TILE + lane * SLOTS + ((2 * q + 1) ^ sw)];
          }
        } else {
          kb[b ^ 1][q] = kring[sl1 * TILE + lane * SLOTS + (q ^ sw)];
        }
        __builtin_amdgcn_sched_barrier(0);
        const uint4 kq = kb[b][q];
        h = h32_step_fast(h, (uint64_t)kq.x | ((uint64_t)kq.y << 32));
        h = h32_step_fast(h, (uint64_t)kq.z | ((uint64_t)kq.w << 32));
      }
      if (X64) {
#pragma unroll 4
        for (int q = 0; q < SLOTS; q++) {
          const uint4 v = tring[sl * TILE + lane * SLOTS + (q ^ sw)];
#pragma unroll
          for (int e = 0; e < 2; e++) {
            const uint64_t tw = ld_u64(v, e);
            const int xl = (2 * q + e) & 3;
            if (xl == 0) x0 = xx_round(x0, tw);
            else if (xl == 1) x1 = xx_round(x1, tw);
            else if (xl == 2) x2 = xx_round(x2, tw);
            else x3 = xx_round(x3, tw);
          }
        }
      }
    };
    KBZ_STAMP_DECL;
    // Step t (in slot sl, words in kb[b]): the flag of slot sl + 1 is read before the chain's
    // speculative reads of its words: a wave's LDS operations execute in order, so if the flag
    // says "ready", the words are tile t + 1's.  Otherwise they are read again once it does.
    // Slot sl + 1 is freed (without XXH64) when its words are in registers: at the end of step t;
    // with XXH64 slot sl is, after the chain read its classified words.
    auto step = [&](uint32_t t, auto bc, auto sc) {
      constexpr int b = decltype(bc)::value, sl = decltype(sc)::value, sl1 = (sl + 1) % RING;
      const bool more = t + 1 < ntiles;
      const int f = KBZ_FLD(ready, sl1);
      asm volatile("" ::: "memory");  // the flag read stays ahead of the word reads
      KBZ_STAMP(3);
      chain(bc, sc);
      KBZ_STAMP(0);
      if (more && f != (int)(t + 1)) {
        wait_ready(t + 1);
        KBZ_STAMP(1);
        read_k(IntC<b ^ 1>{}, IntC<sl1>{});
      }
      // Tile t + 1's words have arrived before the freed flag is written.  (Without this wait --
      // safe, since a wave's LDS operations execute in issue order, with the compiler kept from
      // sinking the reads below the flag store by an empty asm -- config 3 pass 1 was 1.3 %
      // slower: 3.10 vs 3.06 ms same-box, profiles/r05_d/ab2.txt.)
      if (KBZ_PASS1D_CWAIT) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      else asm volatile("" ::: "memory");
      KBZ_STAMP(2);
      if (lane == 0) {
        if (X64) KBZ_FST(freed_c, sl, (int)t);
        else if (more) KBZ_FST(freed_c, sl1, (int)(t + 1));
      }
    };
    if (ntiles) {
      wait_ready(0);
      read_k(IntC<0>{}, IntC<0>{});
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (!X64 && lane == 0) KBZ_FST(freed_c, 0, 0);
    }
    constexpr int U = (RING % 2 == 0) ? RING : 2 * RING;
    for (uint32_t t0 = 0; t0 < ntiles; t0 += U)
      static_for<U>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        if (t0 + u < ntiles) step(t0 + u, IntC<u & 1>{}, IntC<u % RING>{});
      });
    KBZ_STAMP_FLUSH(chunk * 16 + wave);
    if (lane < nrows) {
      const uint32_t h32 = h32_final(h);
      a.h32[row0 + lane] = h32;
      if (X64 && a.x64) {
        uint64_t xh = rotl64(x0, 1) + rotl64(x1, 7) + rotl64(x2, 12) + rotl64(x3, 18);
        xh = xx_merge(xh, x0);
        xh = xx_merge(xh, x1);
        xh = xx_merge(xh, x2);
        xh = xx_merge(xh, x3);
        xh += a.map_size;
        a.x64[row0 + lane] = xx_avalanche(xh);
      }
      if (row0 + lane == (uint64_t)a.n - 1) {
        a.shard_last[0] = h32;
        a.shard_last[1] = 1;
      }
    }
    if (lane == 0) a.chunk_cls[chunk] = 1;  // DynamoRIO: one virgin map, every row in it
  } else if (wave == 4) {
    // ------------------------------------------------------------ N: the neighbour test
    uint64_t nacc = 0;  // OR over the row's words of (word ^ previous row's word)
    const uint4 *ring = IGN ? wring : kring;
    KBZ_STAMP_DECL;  // N: {compare, ready wait, LDS read wait, -}
    for (uint32_t t0 = 0; t0 < ntiles; t0 += RING)
      static_for<RING>([&](auto sc) {  // slots as compile-time constants (see C)
      constexpr int sl = decltype(sc)::value;
      const uint32_t t = t0 + sl;
      if (t >= ntiles) return;
      wait_ready(t);
      KBZ_STAMP(1);
      uint4 vv[SLOTS];
#pragma unroll
      for (int q = 0; q < SLOTS; q++) vv[q] = ring[sl * TILE + lane * SLOTS + (q ^ sw)];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      KBZ_STAMP(2);
      if (lane == 0) KBZ_FST(freed_n, sl, (int)t);
#pragma unroll
      for (int q = 0; q < SLOTS; q++) {
        const uint64_t w0 = (uint64_t)vv[q].x | ((uint64_t)vv[q].y << 32);
        const uint64_t w1 = (uint64_t)vv[q].z | ((uint64_t)vv[q].w << 32);
        nacc |= (w0 ^ from_prev_lane(w0)) | (w1 ^ from_prev_lane(w1));
      }
      KBZ_STAMP(0);
    });
    KBZ_STAMP_FLUSH(chunk * 16 + wave);
    // lane 0 has no predecessor in the wave: a placeholder (k_skip compares chunk starts)
    if (lane < nrows) a.neq[row0 + lane] = nacc != 0;
  } else if ((wave & 3) == 0) {
    // idle (wave 8): SIMD 0 is left to the chain
  } else {
    // ------------------------------------------------------------ X waves
    const int xi = wave - 1 - wave / 4;  // 0..NX-1
    const int lr = lane / SLOTS, ls = lane % SLOTS;
    const uint8_t *cbase = a.traces + row0 * a.stride;  // the chunk's rows: < 64 x 32 MiB
    const uint32_t rstep = (uint32_t)(RPI * a.stride);
    const uint32_t rlast = (uint32_t)((nrows - 1) * a.stride);
    uint32_t voff[NLD];  // per lane: its row of each load and its 16-B slot (loop-invariant)
#pragma unroll
    for (int i = 0; i < NLD; i++)
      voff[i] = min((uint32_t)(i * rstep + lr * a.stride), rlast) + (uint32_t)ls * 16;
    const uint32_t vsl = (uint32_t)ls * 16;
    const uint32_t nmine = ntiles > (uint32_t)xi ? (ntiles - 1 - xi) / NX + 1 : 0;
    const uint32_t nb = (nmine + D - 1) / D * D;
    auto tile_of = [&](uint32_t q) { return (uint32_t)xi + q * NX; };
    // branch-free asm loads (see k_pass1s); steps past the wave's last tile re-load its first.
    // The tile's offset moves the SGPR base (saddr form), the lanes' offsets stay put.
    auto load = [&](u32x4 (&r)[NR], uint32_t q) {
      const uint32_t t = q < nmine ? tile_of(q) : (uint32_t)xi;
      const uint32_t tt = t < ntiles ? t : 0;
#pragma unroll
      for (int i = 0; i < NLD; i++) asm_load16_s(r[i], voff[i], cbase + (size_t)tt * TW);
      asm_load16_s_cached(r[NLD], vsl, a.vcur + (size_t)tt * TW);
      if (IGN) asm_load16_s_cached(r[NLD + 1], vsl, a.ignore + (size_t)tt * TW);
    };
    u32x4 R[D][NR];
#pragma unroll
    for (int d = 0; d < D; d++) load(R[d], d);
    KBZ_STAMP_DECL;
    for (uint32_t q0 = 0; q0 < nb; q0 += D) {
#pragma unroll
      for (int u = 0; u < D; u++) {
        const uint32_t q = q0 + u;
        const uint32_t t = tile_of(q);
        // younger than slot u's loads: the next D - 1 tiles' loads and the VMEM writes issued
        // before each of them (counted as loads here: the wait also covers those writes, which
        // were issued a step or more ago -- see the writes below)
        vmcnt_wait_ring<(D - 1) * NR>(R[u]);
        KBZ_STAMP(0);
        // classify_counts in place, the column OR (rows past the end of a partial chunk are
        // copies of its last row: OR-ing them changes nothing)
        u32x4 o = {0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < NLD; i++) {
          const u32x4 x = R[u][i];
          R[u][i] = u32x4{classify4(x.x), classify4(x.y), classify4(x.z), classify4(x.w)};
          o |= R[u][i];
        }
        o = or_lanes(o);
        u32x4 m = o & R[u][NLD];  // still-virgin bits only (like k_pass1s)
        if (lane >= SLOTS) m = u32x4{0, 0, 0, 0};
        u32x4 igw = {~0u, ~0u, ~0u, ~0u};
        if (IGN) igw = R[u][NLD + 1];
        // no value of the slot live across its reload (igw only with ignore bytes: otherwise it is
        // the constant ~0 and the masks below fold away)
        if (IGN) asm volatile("" : "+v"(m), "+v"(igw));
        else asm volatile("" : "+v"(m));
        const bool mine = q < nmine;
        const int sl = (int)(t % RING);
        KBZ_STAMP(1);
        if (mine)  // the slot is free once C and N have read tile t - RING from it
          while (KBZ_FLD(freed_c, sl) != (int)t - RING || KBZ_FLD(freed_n, sl) != (int)t - RING)
            __builtin_amdgcn_s_sleep(1);
        asm volatile("" ::: "memory");
        KBZ_STAMP(2);
        if (mine) {  // wave-uniform: one branch around the tile's mixes and ring writes
#pragma unroll
          for (int i = 0; i < NLD; i++) {
            const int rr = RPI * i + lr;
            const int idx = sl * TILE + rr * SLOTS + (ls ^ (rr & 15));
            const u32x4 c = R[u][i];
            const uint64_t c0 = (uint64_t)c.x | ((uint64_t)c.y << 32);
            const uint64_t c1 = (uint64_t)c.z | ((uint64_t)c.w << 32);
            const uint64_t g0 = (uint64_t)igw.x | ((uint64_t)igw.y << 32);
            const uint64_t g1 = (uint64_t)igw.z | ((uint64_t)igw.w << 32);
            const uint64_t k0 = h32_mix_mad(c0 & g0);
            const uint64_t k1 = h32_mix_mad(c1 & g1);
            kring[idx] = make_uint4((uint32_t)k0, (uint32_t)(k0 >> 32), (uint32_t)k1,
                                    (uint32_t)(k1 >> 32));
            if (IGN) {  // the neighbour test looks at the bytes whose ignore byte is 0
              const uint64_t e0 = c0 & ~nonzero_bytes8(g0), e1 = c1 & ~nonzero_bytes8(g1);
              wring[idx] = make_uint4((uint32_t)e0, (uint32_t)(e0 >> 32), (uint32_t)e1,
                                      (uint32_t)(e1 >> 32));
            }
            if (X64) tring[idx] = make_uint4(c.x, c.y, c.z, c.w);
          }
        }
        if (mine) {
          __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the slot's words are written
          asm volatile("" ::: "memory");
          if (lane == 0) KBZ_FST(ready, sl, (int)t);
        }
        // The tile's writes (chunk_or, segment-OR atomics: still-virgin bits only) go BEFORE the
        // slot's next loads.  vmcnt counts loads and writes in issue order: written after the
        // loads, the next step's wait -- which counts only loads -- also waited for the oldest
        // loads of the tile just prefetched, a memory latency per step whenever tiles are stored
        // (novelty-heavy batches: every tile).  Written before them, that wait covers writes
        // issued a step earlier.
        if (mine) {
          const bool any = (m.x | m.y | m.z | m.w) != 0;
          if (__ballot(any)) {
            if (lane < SLOTS)
              *(uint4 *)(a.chunk_or + (size_t)chunk * a.map_size + (size_t)t * TW + lane * 16) =
                  make_uint4(m.x, m.y, m.z, m.w);
            if (lane == 0) atomicOr(&tfl_lds[t >> 6], 1ull << (t & 63));
          }
          if (any) {
            unsigned long long *sp = (unsigned long long *)(a.segor + (size_t)seg * a.map_size +
                                                            (size_t)t * TW + lane * 16);
            const uint64_t lo = (uint64_t)m.x | ((uint64_t)m.y << 32);
            const uint64_t hi = (uint64_t)m.z | ((uint64_t)m.w << 32);
            if (lo) atomicOr(sp, (unsigned long long)lo);
            if (hi) atomicOr(sp + 1, (unsigned long long)hi);
          }
        }
        load(R[u], q + D);  // the ring slot is free again
        KBZ_STAMP(3);
      }
    }
    KBZ_STAMP_FLUSH(chunk * 16 + wave);
    drain_asm_loads(R);
  }
  __syncthreads();  // every X wave's tile flags are in tfl_lds
  uint64_t *tfbase = a.tflags + (size_t)chunk * a.nfw;
  for (int i = threadIdx.x; i < (int)a.nfw; i += blockDim.x) tfbase[i] = tfl_lds[i];
}
#undef KBZ_FLD
#undef KBZ_FST

// DynamoRIO last-hash skip: skip[j] = hash[j] == hash[j-1] (hash[-1] = previous exec's).
// A skipped trace must not touch the virgin map.  Pass 1 OR'ed it into its chunk, which is
// harmless when it equals its predecessor on the bytes has_new_bits examines (neq[j] == 0, exact
// for every j > 0 of the shard: pass 1 compares row 0 of a chunk with the previous chunk's last
// row) AND that predecessor's content is legitimately in the ORs or already in V.  So:
//   bad[j]  = skip[j] && differs[j]   (a hash collision, or row 0 with an unknown / unclean
//                                      predecessor)
//   link[j] = skip[j] && !differs[j]  (same content as row j-1)
// Every chunk holding a bad row, or a link row whose chain of links goes back to a bad row, is
// recomputed without its skipped rows (fix list, k_total).
//
// k_skip (in kbz_shard_begin, rows j >= 1: they need no other shard) lists the chunks of bad
// rows and queues those rows for k_chain.  It also publishes, in the shard's last-hash pair
// (shard_last[1], bit 0 = non-empty), bit 1 = "has a bad row j >= 1" and bit 2 = "has a
// non-skipped row j >= 1": a shard with bit 2 and without bit 1 ends in a clean row (its last
// row's chain of links starts at a row that was applied), whatever its row 0 is.
// Row j's content against row j-1's on the examined bytes (classify_counts applied to both; with
// ignore bytes only bytes whose ignore byte is 0), 16 B per thread per step: a block-wide OR.
__device__ __forceinline__ int rows_differ(const uint8_t *x, const uint8_t *y, const uint8_t *ignore,
                                           uint32_t map_size) {
  int diff = 0;
#pragma unroll 8  // independent iterations: 8 pairs of loads in flight per thread
  for (uint32_t i = threadIdx.x * 16; i < map_size; i += blockDim.x * 16) {
    const uint4 a = *(const uint4 *)(x + i), b = *(const uint4 *)(y + i);
    const uint64_t a0 = classify8((uint64_t)a.x | ((uint64_t)a.y << 32));
    const uint64_t a1 = classify8((uint64_t)a.z | ((uint64_t)a.w << 32));
    const uint64_t b0 = classify8((uint64_t)b.x | ((uint64_t)b.y << 32));
    const uint64_t b1 = classify8((uint64_t)b.z | ((uint64_t)b.w << 32));
    uint64_t r0 = ~0ull, r1 = ~0ull;
    if (ignore) {
      const uint4 g = *(const uint4 *)(ignore + i);
      r0 = ~nonzero_bytes8((uint64_t)g.x | ((uint64_t)g.y << 32));
      r1 = ~nonzero_bytes8((uint64_t)g.z | ((uint64_t)g.w << 32));
    }
    diff |= (((a0 ^ b0) & r0) | ((a1 ^ b1) & r1)) != 0;
  }
  return __syncthreads_or(diff);
}

// k_skip (in kbz_shard_begin, rows j >= 1: they need no other shard) lists the chunks of bad
// rows and queues those rows for k_chain.  Pass 1 compared every row with its predecessor
// inside the chunk (neq); a chunk's row 0 has none there, so for j = 64c the extra blocks
// compare the two rows themselves -- only when their hashes are equal (the only case the rule
// looks at), which leaves the streaming pass without the previous chunk's row.  The shard's
// last-hash pair (shard_last[1], bit 0 = non-empty) gets bit 1 = "has a bad row j >= 1" and
// bit 2 = "has a non-skipped row j >= 1": a shard with bit 2 and without bit 1 ends in a clean
// row (its last row's chain of links starts at a row that was applied), whatever its row 0 is.
// Predecessor of the shard's row 0 (kbz_shard_link): unknown, the context's saved row (the
// previous batch's last, clean iff *ok), or another shard's last row (clean iff its pair's
// flags say so, see k_skip).
enum { PRED_UNKNOWN = 0, PRED_SAVED = 1, PRED_PAIR = 2 };
__device__ __forceinline__ bool pair_clean(uint32_t f) { return !(f & 2u) && (f & 4u); }

// The fused tail's extra k_skip roles (one-shard batches, kbz_triage_batch_device): the block
// after the chunk-start blocks does k_chain's row-0 test against the saved row (bad0 -> a
// device word the tail reads), the blocks after it copy the batch's last row into the context
// (the next batch's row-0 predecessor).  Null row0_hp: the sharded protocol (k_chain does both).
struct SkipExtra {
  const uint32_t *row0_hp;  // the context's last hash (row 0's predecessor hash)
  int pred_saved;           // the saved row is valid ...
  const uint32_t *pred_ok;  // ... and clean iff *pred_ok
  const uint8_t *prow;      // the saved row
  uint32_t *bad0;           // out: row 0 is skipped and differs / has an unknown predecessor
  const uint8_t *copy_src;  // the batch's last row -> copy_dst (map_size bytes), or null
  uint8_t *copy_dst;
  uint32_t copy_blocks;
};
__global__ void k_skip(const uint32_t *h32, uint8_t *neq, uint32_t n, uint8_t *skip,
                       uint32_t *flags, uint32_t *fix_list, uint32_t *fix_cnt, uint32_t *bad_list,
                       uint32_t *bad_cnt, uint32_t *shard_last, const uint8_t *traces,
                       size_t stride, const uint8_t *ignore, uint32_t map_size,
                       uint32_t row_blocks, SkipExtra x) {
  auto bad_row = [&](uint32_t j) {
    const uint32_t c = j / kChunk;
    if (atomicExch(&flags[c], 1u) == 0u) fix_list[atomicAdd(fix_cnt, 1u)] = c;
    bad_list[atomicAdd(bad_cnt, 1u)] = j;
  };
  const uint32_t cs_end = row_blocks + (n > kChunk ? (n - 1) / kChunk : 0);
  if (blockIdx.x >= cs_end) {  // fused tail only: row 0, then the copy of the last row
    if (blockIdx.x == cs_end) {
      const bool sk0 = h32[0] == *x.row0_hp;
      const bool known = x.pred_saved && *x.pred_ok != 0;
      const int diff = (sk0 && known) ? rows_differ(traces, x.prow, ignore, map_size) : 0;
      if (threadIdx.x == 0) {
        skip[0] = sk0;
        *x.bad0 = sk0 && (!known || diff);
      }
      return;
    }
    const uint32_t cb = blockIdx.x - cs_end - 1;
    if (x.copy_src)
      for (uint32_t i = (cb * blockDim.x + threadIdx.x) * 16; i < map_size;
           i += x.copy_blocks * blockDim.x * 16)
        *(uint4 *)(x.copy_dst + i) = *(const uint4 *)(x.copy_src + i);
    return;
  }
  if (blockIdx.x >= row_blocks) {  // chunk start j = 64 c, c >= 1
    const uint32_t j = (blockIdx.x - row_blocks + 1) * kChunk;
    if (j >= n || h32[j] != h32[j - 1]) return;  // block-uniform
    const uint8_t *x = traces + (size_t)j * stride;
    const int diff = rows_differ(x, x - stride, ignore, map_size);
    if (threadIdx.x == 0) {
      neq[j] = diff != 0;  // exact now: k_chain's chain walks read it
      if (diff) {
        bad_row(j);
        atomicOr(&shard_last[1], 2u);
      }
    }
    return;
  }
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  bool applied = false, bad = false;
  if (j >= 1 && j < n) {
    const bool sk = h32[j] == h32[j - 1];
    skip[j] = sk;
    applied = !sk;
    if (sk && (j % kChunk) && neq[j]) {
      bad = true;
      bad_row(j);
    }
  }
  // one atomic per block at most (a flag word every wave hits serialises), skipped when the
  // bits are already set
  const int ap = __syncthreads_or(applied), bd = __syncthreads_or(bad);
  const uint32_t want = (bd ? 2u : 0u) | (ap ? 4u : 0u);
  if (threadIdx.x == 0 && (want & ~*(volatile uint32_t *)&shard_last[1]))
    atomicOr(&shard_last[1], want);
}

// One wave per bad row (row 0 included when bad0): follow its chain of link rows (skipped and
// equal to their predecessor), 64 rows per step, and list every chunk the chain enters (the bad
// row's own chunk is listed already by k_skip; row 0's is listed here).
__device__ __forceinline__ void chain_walks(uint32_t n, const uint8_t *skip, const uint8_t *neq,
                            const uint32_t *bad_list, uint32_t nbad, bool bad0, uint32_t *flags,
                            uint32_t *fix_list, uint32_t *fix_cnt) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  auto list = [&](uint32_t c) {
    if (atomicExch(&flags[c], 1u) == 0u) fix_list[atomicAdd(fix_cnt, 1u)] = c;
  };
  const uint32_t cnt = nbad + (bad0 ? 1u : 0u);
  for (uint32_t i = wave; i < cnt; i += blockDim.x / 64) {
    const uint32_t b = (bad0 && i == cnt - 1) ? 0u : bad_list[i];
    if (b == 0 && lane == 0) list(0);
    for (uint32_t j0 = b + 1; j0 < n; j0 += 64) {
      const uint32_t j = j0 + lane;
      const bool lk = j < n && skip[j] && !neq[j];
      const uint64_t stop = __ballot(!lk);
      const uint32_t len = stop ? (uint32_t)__builtin_ctzll(stop) : 64u;  // links from j0 on
      if (lane < len && (j % kChunk) == 0) list(j / kChunk);  // chunk starts on the chain
      if (len < 64) break;
    }
  }
}

struct ChainArgs {
  uint32_t n;
  const uint32_t *h32;
  uint8_t *skip;
  const uint8_t *neq;
  const uint32_t *bad_list, *bad_cnt;
  uint32_t *flags, *fix_list, *fix_cnt;
  const uint32_t *prev_last;  // [2] predecessor hash (or null: ctx_last)
  const uint32_t *ctx_last;
  const uint32_t *global_last;  // [2]
  uint32_t *next_last;
  int pred_kind;
  const uint32_t *pred_ok;   // PRED_SAVED: nonzero = clean; PRED_PAIR: the pair's flag word
  const uint8_t *row0, *prow, *ignore;
  uint32_t map_size;
  const uint32_t *shard_flags;  // this shard's shard_last[1]
  int single;                   // single-shard batch: the next saved row is our own last row
  uint32_t *saved_ok;           // [1] clean flag of the next saved row (in/out)
  const uint8_t *copy_src;      // row to save (or null), map_size bytes -> copy_dst
  uint8_t *copy_dst;
};

// Row 0, then one wave per bad row (row 0 included when it is skipped and differs from its
// predecessor, or the predecessor is unknown or unclean): follow its chain of link rows, 64 rows
// per step, and list every chunk the chain enters (the bad row's own chunk is listed already).
// Usually nothing is bad and block 0 returns after a few loads.  Blocks >= 1 copy the batch's
// last row into the context (the next batch's row-0 predecessor).
__global__ __launch_bounds__(256) void k_chain(ChainArgs a) {
  if (blockIdx.x > 0) {
    for (uint32_t i = ((blockIdx.x - 1) * blockDim.x + threadIdx.x) * 16; i < a.map_size;
         i += (gridDim.x - 1) * blockDim.x * 16)
      *(uint4 *)(a.copy_dst + i) = *(const uint4 *)(a.copy_src + i);
    return;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t n = a.n;
  bool bad0 = false;
  if (n) {
    const uint32_t hp = a.prev_last ? a.prev_last[0] : *a.ctx_last;
    const bool sk0 = a.h32[0] == hp;
    const bool known = a.pred_kind == PRED_SAVED ? *a.pred_ok != 0
                       : a.pred_kind == PRED_PAIR ? pair_clean(*a.pred_ok) : false;
    // row 0 against its predecessor (block-uniform condition)
    const int diff = (sk0 && known) ? rows_differ(a.row0, a.prow, a.ignore, a.map_size) : 0;
    bad0 = sk0 && (!known || diff);
    if (threadIdx.x == 0) a.skip[0] = sk0;
  }
  __syncthreads();  // skip[0] is read by the chain walks below
  if (threadIdx.x == 0) {
    *a.next_last = a.global_last[1] ? a.global_last[0] : *a.ctx_last;
    // clean flag of the row the context saves for the next batch
    if (a.single) {
      if (n) *a.saved_ok = (*a.bad_cnt == 0) && ((*a.shard_flags & 4u) || !bad0);
    } else {
      *a.saved_ok = a.copy_src ? pair_clean(a.global_last[1]) : 0u;
    }
  }
  (void)lane;
  (void)wave;
  chain_walks(n, a.skip, a.neq, a.bad_list, *a.bad_cnt, bad0, a.flags, a.fix_list, a.fix_cnt);
}

// DynamoRIO fix path of the skip rule, for k_total: chunks listed by k_skip hold a skipped trace
// that differs from its predecessor, so their ORs (class 0) are recomputed without the skipped
// traces, and so are the aggregates of their segments.  One thread owns one 8-byte column of
// every listed chunk and segment, so no other thread's result is needed (usually no chunk is
// listed and this costs one load).
struct FixArgs {
  const uint8_t *traces;
  size_t stride;
  uint32_t n;
  const uint8_t *skip;
  const uint32_t *fix_list;
  const uint32_t *fix_cnt;
  uint8_t *chunk_or;
  const uint8_t *chunk_cls;
  uint32_t nchunks, seg_len;
  const uint32_t *listed;  // [chunks] nonzero: in fix_list
  const uint64_t *tflags;  // pass 1's stored-tile bits (class 0), see Pass1Args
  uint32_t nfw;
};
// Was tile col/256 of chunk c's class-k row of chunk_or stored by pass 1?  An unstored tile
// held no still-virgin bit: it reads as 0.
__device__ __forceinline__ bool tile_stored(const uint64_t *tflags, uint32_t nfw, int nclass,
                                            uint32_t c, int k, uint32_t col) {
  const uint32_t t = col / kTileW;
  return (tflags[((size_t)c * nclass + k) * nfw + (t >> 6)] >> (t & 63)) & 1;
}
__device__ __forceinline__ void fix_column(const FixArgs &f, uint32_t map_size, uint32_t col, uint8_t *segor) {
  const uint32_t cnt = min(*f.fix_cnt, f.nchunks);
  for (uint32_t i = 0; i < cnt; i++) {
    const uint32_t chunk = f.fix_list[i];
    const uint64_t row0 = (uint64_t)chunk * kChunk;
    const int nrows = (int)min((uint64_t)kChunk, (uint64_t)f.n - row0);
    uint64_t acc = 0;
    for (int r = 0; r < nrows; r++)
      if (!f.skip[row0 + r]) acc |= classify8(*(const uint64_t *)(f.traces + (row0 + r) * f.stride + col));
    *(uint64_t *)(f.chunk_or + (size_t)chunk * map_size + col) = acc;
  }
  for (uint32_t i = 0; i < cnt; i++) {  // idempotent when two listed chunks share a segment
    const uint32_t seg = f.fix_list[i] / f.seg_len;
    const uint32_t c0 = seg * f.seg_len, c1 = min(f.nchunks, c0 + f.seg_len);
    uint64_t acc = 0;
    for (uint32_t c = c0; c < c1; c++)
      if ((f.chunk_cls[c] & 1) && (f.listed[c] || tile_stored(f.tflags, f.nfw, 1, c, 0, col)))
        acc |= *(const uint64_t *)(f.chunk_or + (size_t)c * map_size + col);
    *(uint64_t *)(segor + (size_t)seg * map_size + col) = acc;
  }
}

// Per column (8 B per thread): [DynamoRIO: fix path first], then segprev[s] = OR of segments
// < s (local exclusive prefix), total = OR of all segments; segor is re-zeroed for the next
// batch.
// KEEP (the sharded protocol's fused finish, kbz_shard_reduce_into): only the fix path and the
// total -- the segment ORs stay for k_tail, which takes its prefixes from them and zeroes the
// other buffer, and `total` is the caller's exchange buffer.
template <bool KEEP>
__global__ __launch_bounds__(256) void k_total(uint8_t *segor, uint32_t nseg, int nclass,
                                                uint32_t map_size, uint8_t *segprev,
                                                uint8_t *total, FixArgs fix) {
  const uint32_t col = (blockIdx.x * blockDim.x + threadIdx.x) * 8;
  const int k = blockIdx.z;
  if (col >= map_size) return;
  if (fix.fix_cnt && k == 0) fix_column(fix, map_size, col, segor);
  uint64_t v[kMaxSeg];
#pragma unroll
  for (int s = 0; s < kMaxSeg; s++)  // all loads in flight at once
    v[s] = s < (int)nseg ? *(const uint64_t *)(segor + ((size_t)s * nclass + k) * map_size + col) : 0;
  uint64_t acc = 0;
#pragma unroll
  for (int s = 0; s < kMaxSeg; s++) {
    if (s < (int)nseg) {
      const size_t off = ((size_t)s * nclass + k) * map_size + col;
      if (!KEEP) {
        *(uint64_t *)(segprev + off) = acc;
        *(uint64_t *)(segor + off) = 0;  // ready for the next batch
      }
      acc |= v[s];
    }
  }
  *(uint64_t *)(total + (size_t)k * map_size + col) = acc;
}

// The sharded protocol's link exchange in one launch: this shard's last row (if any) and its
// hash pair {last hash32, flags} -> out[0 .. M) and out[M .. M + 8).
__global__ __launch_bounds__(256) void k_exch(const uint8_t *row, uint32_t M,
                                               const uint32_t *pair, uint8_t *out) {
  const uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) * 16;
  if (row && i < M) *(uint4 *)(out + i) = *(const uint4 *)(row + i);
  if (blockIdx.x == 0 && threadIdx.x < 2) ((uint32_t *)(out + M))[threadIdx.x] = pair[threadIdx.x];
}

#ifndef KBZ_SCAN_ILP  // chunk rows k_scan loads per round trip: 8 beat 16 and 32 on fresh config-2
                      // batches (step 0.77-0.78 vs 0.80-0.81 ms, profiles/r02_v10/ab_scan_ilp.txt)
#define KBZ_SCAN_ILP 8
#endif
// item: [7:0] new bits, [8] score-2 candidate, [10:9] class, [34:11] column, [59:35] chunk,
// [63] present (never 0: the fused tail tells a written slot from a reserved one by it; every
// resolver zeroes the slots it consumed, so the list is all-zero between batches)
constexpr uint64_t kItemPresent = 1ull << 63;
__device__ __forceinline__ uint64_t pack_item(uint32_t chunk, int k, uint32_t col, uint32_t nb,
                                              bool f2) {
  return kItemPresent | ((uint64_t)chunk << 35) | ((uint64_t)col << 11) | ((uint64_t)k << 9) |
         ((uint64_t)f2 << 8) | nb;
}
__device__ __forceinline__ uint32_t item_chunk(uint64_t item) { return (uint32_t)((item >> 35) & 0x1FFFFFFu); }
// Hand-off stores and loads between workgroups of one launch (the fused tail): agent-scope
// relaxed atomics, i.e. sc1 accesses performed at the coherence point, so another XCD's reader
// sees them without cache maintenance (MI355X_MICROARCH.md, hand-off rules).
__device__ __forceinline__ void st_sc1(uint64_t *p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_sc1(const uint64_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_sc1(const uint32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(uint32_t *p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// A claim's score for trace `row` (has_new_bits' 1 or 2, the maximum over its claims):
// fire-and-forget, the outputs are copied once every score is final (k_pack / k_fin).
__device__ __forceinline__ void score_row(uint32_t *hnb32, uint64_t row, uint32_t v) {
  atomicMax(&hnb32[row], v);
}

// Append this lane's claim items (one per nonzero byte of nb) with ONE atomic per wave:
// wave-wide exclusive prefix of the per-lane counts, lane 63 reserves the block.
__device__ __forceinline__ uint32_t wave_excl_prefix(uint32_t v, uint32_t &total) {
  const int lane = threadIdx.x & 63;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  total = __shfl(x, 63);
  return x - v;
}
// A wave's claim items are staged in LDS and appended to the global list with ONE atomic per
// flush (a global counter hit once per chunk by every wave serialises: 32k atomics on one
// address cost ~0.3 ms on a fresh virgin map).
constexpr int kWaveItems = 256;
struct ItemStage {
  uint64_t *buf;  // this wave's LDS staging area, kWaveItems entries
  uint32_t n;     // wave-uniform fill
};
__device__ __forceinline__ void flush_items(ItemStage &st, uint64_t *items, uint32_t cap,
                                            uint32_t *counters) {
  if (!st.n) return;
  // the wave's staged LDS writes and its window-prefix stores (emit_items_wave) are done: an
  // item never becomes visible before the data it names
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  uint32_t base = 0;
  if ((threadIdx.x & 63) == 0) base = atomicAdd(&counters[0], st.n);
  base = __shfl(base, 0);
  for (uint32_t i = threadIdx.x & 63; i < st.n; i += 64) {
    if (base + i < cap) st_sc1(&items[base + i], st.buf[i]);
    else atomicOr(&counters[1], 1u);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the area is reused
  st.n = 0;
}
#ifndef KBZ_WIN_LANEMASK  // window items: lanes without new bits load none of the window's rows
#define KBZ_WIN_LANEMASK 1
#endif
#ifndef KBZ_WIN_ITEMS  // claimed bytes of one chunk's 1-KiB column window from which k_resolve
#define KBZ_WIN_ITEMS 16  // streams the window's 64 rows (64 KiB, coalesced) instead of reading
#endif                    // one scattered byte per row and claimed byte
__device__ __forceinline__ void emit_items_wave(uint32_t chunk, int k, uint32_t col, uint4 nb,
                                                uint4 vir, uint4 prev, ItemStage &st,
                                                uint64_t *items, uint32_t cap,
                                                uint32_t *counters, uint8_t *win_prev,
                                                bool live, uint32_t win_items) {
  const uint32_t w[4] = {nb.x, nb.y, nb.z, nb.w};
  const uint32_t vv[4] = {vir.x, vir.y, vir.z, vir.w};
  const uint32_t pv[4] = {prev.x, prev.y, prev.z, prev.w};
  uint32_t cnt = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) cnt += __popc(nonzero_bytes8(w[i]) & 0x80808080u);
  uint32_t total;
  const uint32_t off = wave_excl_prefix(cnt, total);
  if (total >= win_items) {
    // window item (new bits field 0): the wave's 1-KiB column window of this chunk.  The running
    // OR before this chunk replaces the chunk's (consumed) column OR in chunk_or, and k_resolve
    // re-derives the claims row by row in order: new bits of row r = t_r & V & ~(prev | rows < r)
    if (live) {  // read by whichever wave resolves the item (maybe another workgroup)
      // a lane whose 16 B hold no new bit gets prev = all ones: no row can claim there, and the
      // resolver loads nothing for it (KBZ_WIN_LANEMASK; dense novelty-heavy windows have
      // claims in a fraction of their lanes)
      const bool none = KBZ_WIN_LANEMASK && (nb.x | nb.y | nb.z | nb.w) == 0;
      st_sc1((uint64_t *)win_prev, none ? ~0ull : (uint64_t)prev.x | ((uint64_t)prev.y << 32));
      st_sc1((uint64_t *)win_prev + 1, none ? ~0ull : (uint64_t)prev.z | ((uint64_t)prev.w << 32));
    }
    const uint32_t wcol = __shfl(col, 0);
    if (st.n + 1 > kWaveItems) flush_items(st, items, cap, counters);
    if ((threadIdx.x & 63) == 0) st.buf[st.n] = pack_item(chunk, k, wcol, 0u, false);
    st.n += 1;
    return;
  }
  if (st.n + total > kWaveItems) flush_items(st, items, cap, counters);
  const bool staged = total <= kWaveItems;  // else (rare) straight to the global list
  uint32_t base = st.n + off;
  if (!staged) {
    uint32_t g = 0;
    if ((threadIdx.x & 63) == 63) g = atomicAdd(&counters[0], total);
    base = __shfl(g, 63) + off;
  }
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const uint32_t x = (w[i] >> (8 * b)) & 0xff;
      if (!x) continue;
      const bool f2 = ((vv[i] >> (8 * b)) & 0xff) == 0xff && ((pv[i] >> (8 * b)) & 0xff) == 0;
      const uint64_t it = pack_item(chunk, k, col + 4 * i + b, x, f2);
      if (staged) st.buf[base] = it;
      else if (base < cap) st_sc1(&items[base], it);
      else atomicOr(&counters[1], 1u);
      base++;
    }
  if (staged) st.n += total;
}

#ifndef KBZ_SCAN_INLINE  // 1: k_scan resolves chunks with few claimed bytes itself (no item, no
#define KBZ_SCAN_INLINE 1  // append, no k_resolve work); 0: per-byte items for k_resolve
#endif
struct ClaimArgs {  // what k_scan needs to resolve claims inline (k_resolve's inputs)
  const uint8_t *traces;
  size_t stride;
  uint32_t n;
  int mode;
  const int8_t *outcome;
  const uint8_t *skip;
  uint32_t *hnb32;
  uint32_t *err;
};
__device__ __forceinline__ uint32_t pick4(uint4 v, int i) {  // i wave-uniform
  return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w;
}
// Claimed bytes resolved by k_scan's wave itself.  They are queued (per wave, in LDS: chunk,
// byte column, new bits, the "2" candidate flag) over the chunks of the walk and resolved 8 at
// a time, all 8 rows' bytes (and their chunk's outcome / skip flags) in flight together: lane r
// reads the byte of row r of the claim's chunk, and per new bit the first row holding it
// (class k, not skipped) scores 1, or 2 if the byte was all-virgin and it is the first row with
// a nonzero byte there -- k_resolve's per-item rule, without the item.
constexpr int kClaimQ = 8;
struct ClaimQ {
  uint4 *q;  // this wave's kClaimQ entries in LDS: {chunk, column, new bits | f2 << 8, class}
  int m;     // wave-uniform fill
};
__device__ __forceinline__ void claims_flush(const ClaimArgs &ca, ClaimQ &cq) {
  if (!cq.m) return;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // lane 0's entries are written
  const int lane = threadIdx.x & 63;
  uint4 e[kClaimQ];
  uint32_t raw[kClaimQ];
  int oc[kClaimQ];
  uint8_t sk[kClaimQ];
#pragma unroll
  for (int j = 0; j < kClaimQ; j++) e[j] = j < cq.m ? cq.q[j] : make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int j = 0; j < kClaimQ; j++) {  // loads in flight together
    const uint64_t rc = min((uint64_t)e[j].x * kChunk + lane, (uint64_t)ca.n - 1);
    raw[j] = j < cq.m ? ca.traces[rc * ca.stride + e[j].y] : 0u;
    oc[j] = (j < cq.m && ca.outcome) ? ca.outcome[rc] : KBZ_FUZZ_NONE;
    sk[j] = (j < cq.m && ca.skip) ? ca.skip[rc] : 0;
  }
#pragma unroll
  for (int j = 0; j < kClaimQ; j++) {
    if (j >= cq.m) break;  // wave-uniform
    const uint64_t row = (uint64_t)e[j].x * kChunk + lane;
    const int k = (int)e[j].w;  // the entry's class
    const bool ok = row < ca.n && class_of(ca.mode, oc[j]) == k && !sk[j];
    const uint32_t nbits = e[j].z & 0xffu;
    const uint32_t tb = ok ? byte_xform(raw[j], class_xf(ca.mode, k)) : 0u;
    const uint64_t first_nz = __ballot(tb != 0);
    uint64_t claimers = 0;
    for (int bit = 0; bit < 8; bit++) {
      if ((nbits >> bit) & 1) {
        const uint64_t mm = __ballot((tb >> bit) & 1);
        if (!mm && lane == 0) atomicOr(ca.err, 2u);  // k_scan's OR says some row has it
        claimers |= mm & (0 - mm);
      }
    }
    if ((claimers >> lane) & 1) {
      const bool two = (e[j].z >> 8) && first_nz && (lane == __builtin_ctzll(first_nz));
      score_row(ca.hnb32, row, two ? 2u : 1u);
    }
  }
  asm volatile("" ::: "memory");
  cq.m = 0;
}
// Queue the claimed bytes of this wave's window of chunk `chunk` (flushing every kClaimQ).
__device__ __forceinline__ void claims_enqueue(const ClaimArgs &ca, int k, ClaimQ &cq, uint32_t chunk,
                               uint32_t col, uint4 nb, uint4 vir, uint4 prev) {
  const int lane = threadIdx.x & 63;
  uint32_t rem = 0;  // this lane's claimed bytes, bit i = byte i of its 16
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint32_t w = pick4(nb, i);
#pragma unroll
    for (int b = 0; b < 4; b++) rem |= ((w >> (8 * b)) & 0xffu) ? 1u << (4 * i + b) : 0u;
  }
  uint64_t lanes = __ballot(rem != 0);
  while (lanes) {  // wave-uniform scalar work
    const int L = __builtin_ctzll(lanes);
    const uint32_t r = __builtin_amdgcn_readlane(rem, L);
    const int b = __builtin_ctz(r), wi = b >> 2, sh = 8 * (b & 3);
    const uint32_t nbits = (__builtin_amdgcn_readlane(pick4(nb, wi), L) >> sh) & 0xffu;
    const uint32_t vb = (__builtin_amdgcn_readlane(pick4(vir, wi), L) >> sh) & 0xffu;
    const uint32_t pb = (__builtin_amdgcn_readlane(pick4(prev, wi), L) >> sh) & 0xffu;
    const uint32_t cc = __builtin_amdgcn_readlane(col, L) + b;
    if (lane == 0) cq.q[cq.m] = make_uint4(chunk, cc, nbits | ((vb == 0xffu && pb == 0) ? 0x100u : 0u), (uint32_t)k);
    cq.m++;
    if (lane == L) rem &= ~(1u << b);
    if (r == (1u << b)) lanes &= lanes - 1;
    if (cq.m == kClaimQ) claims_flush(ca, cq);
  }
}
// number of claimed (nonzero) bytes over the wave: 16 per lane at most, 5 ballots
__device__ __forceinline__ uint32_t wave_claimed_bytes(uint4 nb) {
  uint32_t cnt = 0;
  const uint32_t w[4] = {nb.x, nb.y, nb.z, nb.w};
#pragma unroll
  for (int i = 0; i < 4; i++) cnt += __popc(nonzero_bytes8(w[i]) & 0x80808080u);
  uint32_t total = 0;
#pragma unroll
  for (int b = 0; b < 5; b++) total += (uint32_t)__popcll(__ballot((cnt >> b) & 1)) << b;
  return total;
}

// Per (segment, 16-B column group): walk the segment's chunks in order with the running OR
// `prev` (seeded with the OR of earlier segments and earlier shards); bits a chunk adds
// that are still virgin become claim items.  Blocks of segment 0 also write V' = V & ~total.
// A segment whose cumulative OR (segprev of the next segment, or this shard's total for the
// last one) adds no still-virgin bit over `prev` cannot claim anything: its waves skip the
// chunk walk (exact; in steady-state fuzzing almost every segment takes this path).
__global__ __launch_bounds__(256) void k_scan(uint8_t *chunk_or, const uint8_t *chunk_cls,
                                               uint32_t nchunks, uint32_t seg_len, int nclass,
                                               uint32_t map_size, const uint8_t *segprev,
                                               uint32_t nseg, const uint8_t *ltotal,
                                               const uint8_t *gprefix, const uint8_t *gtotal,
                                               const uint8_t *vcur, uint8_t *vnext,
                                               const uint8_t *ignore, uint64_t *items,
                                               uint32_t cap, uint32_t *counters,
                                               const uint64_t *tflags, uint32_t nfw,
                                               const uint32_t *listed, uint32_t win_items,
                                               ClaimArgs ca) {
  // no per-lane early return: every lane of a wave takes part in the item-allocation prefix
  KBZ_TAIL_DECL;
  const uint32_t tail_id = ((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * 4 + (threadIdx.x >> 6);
  (void)tail_id;
  const uint32_t col0 = (blockIdx.x * blockDim.x + threadIdx.x) * 16;
  const bool live = col0 < map_size;
  const uint32_t col = live ? col0 : 0;
  const uint32_t s = blockIdx.y;
  const int k = blockIdx.z;
  const size_t kc = (size_t)k * map_size + col;
  // every load of the prologue in one round trip (absent inputs read a valid dummy and are
  // masked): the compiler otherwise waits for each before issuing the next
  const uint4 p0 = *(const uint4 *)(segprev + (size_t)s * nclass * map_size + kc);
  const uint4 p1 = *(const uint4 *)((gprefix ? gprefix : segprev) + kc);
  const uint4 vir = *(const uint4 *)(vcur + kc);
  const uint4 ig = *(const uint4 *)((ignore ? ignore : vcur) + col);
  const uint4 tot = *(const uint4 *)(gtotal + kc);
  const uint4 send = *(const uint4 *)((s + 1 < nseg) ? segprev + (size_t)(s + 1) * nclass * map_size + kc
                                                      : ltotal + kc);
  const uint32_t c0 = s * seg_len, c1 = min(nchunks, c0 + seg_len);
  const uint32_t t0 = (blockIdx.x * blockDim.x + (threadIdx.x & ~63u)) * 16 / kTileW;
  // the first 64 chunks' tile flags, for the walk below (also in this round trip)
  const uint32_t cl0 = c0 + (threadIdx.x & 63);
  uint8_t ccls0 = 0;
  uint64_t tfw0 = 0;
  uint32_t lst0 = 0;
  if (cl0 < c1) {
    ccls0 = chunk_cls[cl0];
    tfw0 = tflags[((size_t)cl0 * nclass + k) * nfw + (t0 >> 6)];
    if (listed) lst0 = listed[cl0];
  }
  uint4 prev = gprefix ? or4(p0, p1) : p0;
  uint4 rel = make_uint4(~0u, ~0u, ~0u, ~0u);
  if (ignore) {  // has_new_bits_with_ignore only examines bytes whose ignore byte is 0
    const uint64_t m0 = nonzero_bytes8((uint64_t)ig.x | ((uint64_t)ig.y << 32));
    const uint64_t m1 = nonzero_bytes8((uint64_t)ig.z | ((uint64_t)ig.w << 32));
    rel = make_uint4(~(uint32_t)m0, ~(uint32_t)(m0 >> 32), ~(uint32_t)m1, ~(uint32_t)(m1 >> 32));
  }
  if (s == 0 && live) {
    const uint4 t = tot;
    *(uint4 *)(vnext + kc) = make_uint4(vir.x & ~(t.x & rel.x), vir.y & ~(t.y & rel.y),
                                        vir.z & ~(t.z & rel.z), vir.w & ~(t.w & rel.w));
    if (k == nclass - 1)  // maps this mode does not use (DynamoRIO: tmout, crash) carry over
      for (int kk = nclass; kk < 3; kk++)
        *(uint4 *)(vnext + (size_t)kk * map_size + col) =
            *(const uint4 *)(vcur + (size_t)kk * map_size + col);
  }
  const uint4 vr = live ? make_uint4(vir.x & rel.x, vir.y & rel.y, vir.z & rel.z, vir.w & rel.w)
                        : make_uint4(0, 0, 0, 0);
  __shared__ uint64_t stage_buf[4][kWaveItems];  // 256 threads = 4 waves
  ItemStage stg{stage_buf[threadIdx.x >> 6], 0u};
  __shared__ uint4 claim_q[4][kClaimQ];
  ClaimQ cq{claim_q[threadIdx.x >> 6], 0};
  const uint32_t seg_new = (send.x & vr.x & ~prev.x) | (send.y & vr.y & ~prev.y) |
                           (send.z & vr.z & ~prev.z) | (send.w & vr.w & ~prev.w);
  KBZ_TAIL_MARK();
  if (!__ballot(seg_new != 0)) {  // wave-uniform: nothing new in this segment
    KBZ_TAIL_END(tail_id);
    return;
  }
  // Only chunks that hold traces of class k AND stored (or, DynamoRIO fix path, recomputed) one
  // of this wave's 4 tiles can add bits here: an unstored tile held no still-virgin bit, so a
  // skipped chunk changes neither the claims nor the running OR.  Lane l tests chunk cg + l;
  // the wave walks the set bits of the ballot in order, KBZ_SCAN_ILP chunk loads per memory round
  // trip.
  for (uint32_t cg = c0; cg < c1; cg += 64) {
    const uint32_t cl = cg + (threadIdx.x & 63);
    bool any = false;
    if (cg == c0) {  // loaded with the prologue
      if (cl < c1 && ((ccls0 >> k) & 1)) any = lst0 || ((tfw0 >> (t0 & 63)) & 0xFull);
    } else if (cl < c1 && ((chunk_cls[cl] >> k) & 1))
      any = (listed && listed[cl]) ||
            ((tflags[((size_t)cl * nclass + k) * nfw + (t0 >> 6)] >> (t0 & 63)) & 0xFull);
    uint64_t mask = __ballot(any);
    KBZ_TAIL_ADD(walk, (uint32_t)__popcll(mask));
    while (mask) {
      uint32_t cs[KBZ_SCAN_ILP];
#pragma unroll
      for (int u = 0; u < KBZ_SCAN_ILP; u++) {
        cs[u] = mask ? cg + (uint32_t)__builtin_ctzll(mask) : ~0u;
        mask &= mask - 1;
      }
      uint4 o[KBZ_SCAN_ILP];
      bool st[KBZ_SCAN_ILP];
#pragma unroll
      for (int u = 0; u < KBZ_SCAN_ILP; u++) {
        const uint32_t c = cs[u] != ~0u ? cs[u] : cs[0];
        o[u] = *(const uint4 *)(chunk_or + (size_t)c * nclass * map_size + kc);
        // DynamoRIO fix path: a listed chunk's row was rewritten whole (unmasked) by k_total
        st[u] = tile_stored(tflags, nfw, nclass, c, k, col) || (listed && listed[c]);
      }
#pragma unroll
      for (int u = 0; u < KBZ_SCAN_ILP; u++) {
        const uint32_t c = cs[u];  // uniform across the wave
        if (c == ~0u) break;
        if (!st[u]) o[u] = make_uint4(0, 0, 0, 0);  // nothing still virgin in that tile
        const uint4 nb = make_uint4(o[u].x & vr.x & ~prev.x, o[u].y & vr.y & ~prev.y,
                                    o[u].z & vr.z & ~prev.z, o[u].w & vr.w & ~prev.w);
        if (__ballot(nb.x | nb.y | nb.z | nb.w)) {  // wave-uniform
          const uint32_t ncl = wave_claimed_bytes(nb);
          if (KBZ_SCAN_INLINE && ncl < win_items) {
            KBZ_TAIL_ADD(claims, ncl);
            claims_enqueue(ca, k, cq, c, col, nb, vir, prev);
          } else {
            KBZ_TAIL_ADD(win, 1);
            emit_items_wave(c, k, col, nb, vir, prev, stg, items, cap, counters,
                            (uint8_t *)chunk_or + (size_t)c * nclass * map_size + kc, live,
                            win_items);
          }
        }
        prev = or4(prev, o[u]);
      }
    }
  }
  claims_flush(ca, cq);
  flush_items(stg, items, cap, counters);
  KBZ_TAIL_END(tail_id);
}

// Window item: lane l owns 16-B column group l of the chunk's 1-KiB window; the rows of the
// chunk that belong to class k (and are not skipped) are walked in order with their running OR
// `acc`: row r claims t_r & V & ~(prev | acc) (has_new_bits, afl_instrumentation.c:600-662, over
// the window), and scores 2 if it is the first row with a nonzero byte where V is 0xff and prev
// is 0 (:644-651).  Rows are loaded KBZ_WIN_ROWS at a time (1 KiB per row, coalesced).
#ifndef KBZ_WIN_PIPE  // window items: the next WR rows' loads issued before the current WR rows
#define KBZ_WIN_PIPE 1  // are processed (two register groups); 0: load, wait, process
#endif
#ifndef KBZ_WIN_ROWS  // rows of a window item per group (unpipelined: in flight per round trip;
#if KBZ_WIN_PIPE     // 8 spent 8 round trips per item on novelty-heavy k_fin).  Pipelined, two
#define KBZ_WIN_ROWS 8  // groups of 8 are in flight (k_fin 186 VGPRs: 2 waves per SIMD; two
#else                   // groups of 16 take 308)
#define KBZ_WIN_ROWS 16
#endif
#endif
struct ResolveArgs {  // what resolving a claim item needs (k_resolve, the fused tail)
  const uint8_t *traces;
  size_t stride;
  uint32_t n;
  int mode;
  const int8_t *outcome;
  const uint8_t *skip;
  uint32_t *hnb32;
  uint32_t *err;
  const uint8_t *chunk_or;
  int nclass;
  uint32_t map_size;
  const uint8_t *vcur;
  const uint8_t *ignore;
};
#ifndef KBZ_SCORE_SKIP  // window / byte items read the rows' scores so far and skip the atomicMax
#define KBZ_SCORE_SKIP 1  // where it cannot raise one (exact: scores only grow until k_fin's copy).
#endif                    // A novelty-heavy chunk has ~1,000 window items scoring the same 64 rows
#ifndef KBZ_WIN_XF  // 1: the window loop instantiated per transform (no per-row branch; k_fin
#define KBZ_WIN_XF 0  // 119 -> 181 VGPRs): config-3 novelty-heavy k_fin 0.599 vs 0.616 ms, AFL
#endif                // 0.069 vs 0.048 ms (profiles/r06/ab/ab_winv_*.txt); 0: one loop, the
                      // transform chosen per row at run time
template <int XF>  // the class's transform (XF < 0: xf_rt, chosen at run time)
__device__ __forceinline__ void resolve_window_xf(const ResolveArgs &r, uint32_t chunk, int k,
                                                 uint32_t wcol, const uint8_t *win_prev,
                                                 int xf_rt) {
  const int xf = XF >= 0 ? XF : xf_rt;
  const int lane = threadIdx.x & 63;
  const uint64_t row0 = (uint64_t)chunk * kChunk;
  const uint64_t rl = row0 + lane;
  bool ok = rl < r.n;
  if (ok && r.outcome) ok = class_of(r.mode, r.outcome[rl]) == k;
  if (ok && r.skip) ok = !r.skip[rl];
  uint64_t rows = __ballot(ok);
  const uint32_t col = wcol + 16 * lane;
  const bool live = col < r.map_size;
  const uint32_t cl = live ? col : wcol;
  // k_scan's running OR (maybe stored by another workgroup of the fused tail: sc1 loads)
  const uint64_t *wp = (const uint64_t *)(win_prev + (cl - wcol));
  uint64_t pa0 = ld_sc1(wp), pa1 = ld_sc1(wp + 1);
  const uint4 vir = *(const uint4 *)(r.vcur + (size_t)k * r.map_size + cl);
  uint64_t rel0 = ~0ull, rel1 = ~0ull;
  if (r.ignore) {
    const uint4 ig = *(const uint4 *)(r.ignore + cl);
    rel0 = ~nonzero_bytes8((uint64_t)ig.x | ((uint64_t)ig.y << 32));
    rel1 = ~nonzero_bytes8((uint64_t)ig.z | ((uint64_t)ig.w << 32));
  }
  uint64_t vr0 = ((uint64_t)vir.x | ((uint64_t)vir.y << 32)) & rel0;
  uint64_t vr1 = ((uint64_t)vir.z | ((uint64_t)vir.w << 32)) & rel1;
  if (!live) vr0 = vr1 = 0;
  // the emitter marked lanes without new bits with an all-ones prev: they read no rows
  const bool act = live && !(KBZ_WIN_LANEMASK && pa0 == ~0ull && pa1 == ~0ull);
  // bit 7 of each byte with V == 0xff (examined): a 2 is possible there while prev | acc is
  // still 0
  constexpr uint64_t kHi = 0x8080808080808080ull;
  const uint64_t ff0 = ~nonzero_hi8(~vr0) & kHi, ff1 = ~nonzero_hi8(~vr1) & kHi;
  bool claimed = false;
  constexpr int WR = KBZ_WIN_ROWS;
  // the next WR rows' loads (and, lane l, row l's score so far: a row whose score already covers
  // this window's needs no atomic)
  auto issue = [&](int (&rr)[WR], uint4 (&v)[WR], uint32_t &have) {
    have = (KBZ_SCORE_SKIP && rl < r.n) ? ld_sc1(&r.hnb32[rl]) : 0u;
#pragma unroll
    for (int u = 0; u < WR; u++) {
      rr[u] = rows ? __builtin_ctzll(rows) : -1;
      rows &= rows - 1;
      const uint64_t rw = row0 + (rr[u] >= 0 ? rr[u] : 0);
      v[u] = act ? *(const uint4 *)(r.traces + rw * r.stride + cl) : make_uint4(0, 0, 0, 0);
    }
  };
  // those rows in order: new bits against the running OR, the "2" test, the score
  auto process = [&](const int (&rr)[WR], const uint4 (&v)[WR], uint32_t have) {
#pragma unroll
    for (int u = 0; u < WR; u++) {
      if (rr[u] < 0) break;  // wave-uniform
      const uint64_t t0 = xform8((uint64_t)v[u].x | ((uint64_t)v[u].y << 32), xf) & rel0;
      const uint64_t t1 = xform8((uint64_t)v[u].z | ((uint64_t)v[u].w << 32), xf) & rel1;
      const bool nw = ((t0 & vr0 & ~pa0) | (t1 & vr1 & ~pa1)) != 0;
      const bool two = ((nonzero_hi8(t0) & ff0 & ~nonzero_hi8(pa0)) |
                        (nonzero_hi8(t1) & ff1 & ~nonzero_hi8(pa1))) != 0;
      pa0 |= t0;
      pa1 |= t1;
      const uint32_t sc = __ballot(two) ? 2u : __ballot(nw) ? 1u : 0u;
      if (sc) {
        claimed = true;
        if (lane == 0 && __builtin_amdgcn_readlane(have, rr[u]) < sc)
          score_row(r.hnb32, row0 + rr[u], sc);
      }
    }
  };
#if KBZ_WIN_PIPE
  // two register groups: a group's loads are in flight while the previous group is processed
  if (rows) {
    int rA[WR], rB[WR];
    uint4 vA[WR], vB[WR];
    uint32_t hA, hB;
    issue(rA, vA, hA);
    while (true) {  // wave-uniform
      if (!rows) {
        process(rA, vA, hA);
        break;
      }
      issue(rB, vB, hB);
      process(rA, vA, hA);
      if (!rows) {
        process(rB, vB, hB);
        break;
      }
      issue(rA, vA, hA);
      process(rB, vB, hB);
    }
  }
#else
  while (rows) {
    int rr[WR];
    uint4 v[WR];
    uint32_t have;
    issue(rr, v, have);
    process(rr, v, have);
  }
#endif
  if (!claimed && lane == 0) atomicOr(r.err, 8u);  // k_scan saw new bits here: inconsistent
}
__device__ __forceinline__ void resolve_window(const ResolveArgs &r, uint32_t chunk, int k,
                                               uint32_t wcol, const uint8_t *win_prev) {
  const int xf = class_xf(r.mode, k);  // wave-uniform
  if (!KBZ_WIN_XF) resolve_window_xf<-1>(r, chunk, k, wcol, win_prev, xf);
  else if (xf == XF_CLASSIFY) resolve_window_xf<XF_CLASSIFY>(r, chunk, k, wcol, win_prev, xf);
  else if (xf == XF_SIMPLIFY) resolve_window_xf<XF_SIMPLIFY>(r, chunk, k, wcol, win_prev, xf);
  else resolve_window_xf<XF_RAW>(r, chunk, k, wcol, win_prev, xf);
}

// One claim item (wave-uniform): a window item (new bits field 0) or one claimed byte of one
// chunk -- per new bit, the first trace of the chunk (class k, not skipped) holding it scores 1,
// or 2 if the byte was all-virgin and it is the chunk's first trace with a nonzero byte there.
__device__ __forceinline__ void resolve_item(const ResolveArgs &r, uint64_t item) {
  const int lane = threadIdx.x & 63;
  const uint32_t nb = item & 0xff;
  const bool f2 = (item >> 8) & 1;
  const int k = (item >> 9) & 3;
  const uint32_t col = (item >> 11) & 0xffffff;
  const uint32_t chunk = item_chunk(item);
  if (nb == 0) {  // window item
    resolve_window(r, chunk, k, col,
                   r.chunk_or + ((size_t)chunk * r.nclass + k) * r.map_size + col);
    return;
  }
  const uint64_t row = (uint64_t)chunk * kChunk + lane;
  const uint64_t rc = min(row, (uint64_t)r.n - 1);  // independent loads, one round trip
  const int oc = r.outcome ? r.outcome[rc] : KBZ_FUZZ_NONE;
  const uint8_t sk = r.skip ? r.skip[rc] : 0;
  const uint32_t raw = r.traces[rc * r.stride + col];
  const uint32_t have = KBZ_SCORE_SKIP ? ld_sc1(&r.hnb32[rc]) : 0u;  // row rc's score so far
  const bool ok = row < r.n && class_of(r.mode, oc) == k && !sk;
  const uint32_t tb = ok ? byte_xform(raw, class_xf(r.mode, k)) : 0u;
  const uint64_t first_nz = __ballot(tb != 0);
  uint64_t claimers = 0;
  for (int b = 0; b < 8; b++) {
    if ((nb >> b) & 1) {
      const uint64_t m = __ballot((tb >> b) & 1);
      if (!m) {
        if (lane == 0) atomicOr(r.err, 16u);
      }
      claimers |= m & (0 - m);
    }
  }
  if ((claimers >> lane) & 1) {
    const bool two = f2 && first_nz && (lane == __builtin_ctzll(first_nz));
    if (have < (two ? 2u : 1u)) score_row(r.hnb32, row, two ? 2u : 1u);
  }
}

__global__ __launch_bounds__(256) void k_resolve(ResolveArgs r, uint64_t *items,
                                                  const uint32_t *counters, uint32_t cap) {
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
  const uint32_t cnt = min(counters[0], cap);
  for (uint32_t it = wave; it < cnt; it += nwaves) {
    const uint64_t item = items[it];
    resolve_item(r, item);
    if ((threadIdx.x & 63) == 0) items[it] = 0;  // the list is all-zero between batches
  }
}

// Per-trace outputs, then re-arm the per-batch state for the next batch (no memsets between
// batches): hnb32, the item, fix-list and bad-row counters and the row-0 flag (the sticky error
// flags counters[1..2] stay until kbz_sync reports them), the fix-list flags and the shard's
// last-hash pair.
__global__ void k_pack(uint32_t *hnb32, const uint32_t *h32, uint32_t n, uint8_t *hnb_out,
                       uint32_t *h32_out, uint32_t *counters, uint32_t *flags, uint32_t nchunks,
                       uint32_t *shard_last, uint32_t *err_out) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < nchunks && flags) flags[j] = 0;
  if (j == 0) {
    err_out[0] = counters[1];  // the sticky error flags, readable without a copy (host-mapped)
    err_out[1] = counters[2];
    counters[8] = counters[0];   // kbz_ctx_stats: claim items, recomputed chunks, bad rows
    counters[9] = counters[3];
    counters[10] = counters[4];
    counters[0] = 0;
    counters[3] = 0;
    counters[4] = 0;
    counters[5] = 0;
    shard_last[0] = 0;
    shard_last[1] = 0;
  }
  if (j >= n) return;
  if (hnb_out) hnb_out[j] = (uint8_t)hnb32[j];
  if (h32_out) h32_out[j] = h32[j];
  hnb32[j] = 0;  // ready for the next batch
}

// ---------------------------------------------------------------------------------------------
// The fused tail of a one-shard batch (kbz_triage_batch_device): everything after pass 1 (and,
// in DynamoRIO mode, after k_skip with its row-0 / saved-row roles) in ONE launch, in place of
// k_chain, k_total, k_scan, k_resolve and k_pack.  Grid (column groups of 4 KiB, segments,
// classes) as k_scan; a workgroup:
//   1. DynamoRIO, only when k_skip found bad rows (hash collisions): workgroup 0 finishes
//      k_chain's part (the chain walks), the segment-0 workgroup of each column group runs
//      k_total's fix for its columns, the others wait for it (flags; every wait is on a
//      workgroup of lower linear index, which was dispatched first: no deadlock at any grid size);
//   2. k_scan's walk, with the segment prefixes taken from the segment ORs themselves (all 32
//      loads in one round trip) instead of k_total's output; segment 0 writes V' = V & ~total;
//   3. appends the claims it does not resolve inline as items for k_fin (the next launch), which
//      resolves them over a wide grid and copies the scores into hnb_out once they are final,
//      then re-arms the per-batch state.
// It also zeroes the other segment-OR buffer for the next batch (segor is double-buffered).
// Hand-offs between workgroups use agent-scope atomics or sc1 stores/loads (score_row, st_sc1,
// ld_sc1); the rare fix path publishes plain stores with release / acquire fences.
// ---------------------------------------------------------------------------------------------
constexpr int kTailFixDone = 16;  // tail words: [0] ticket (k_fin) [3] walks done
                                  // [4] bad0 (k_skip) [5] fixing [16 + bx] column group bx fixed
constexpr uint32_t kSpinMax = 1u << 22;

__device__ __forceinline__ bool spin_until(const uint32_t *p, uint32_t want) {
  for (uint32_t it = 0; it < kSpinMax; it++) {
    if (ld_sc1(p) == want) return true;
    __builtin_amdgcn_s_sleep(2);
  }
  return false;
}
struct TailArgs {
  ClaimArgs ca;         // traces, stride, n, mode, outcome, skip, hnb32, err
  ResolveArgs ra;
  FixArgs fx;           // DynamoRIO fix path (fx.fix_cnt = counters + 3)
  uint8_t *chunk_or;
  const uint8_t *chunk_cls;
  uint32_t nchunks, seg_len, nseg;
  int nclass;
  uint32_t map_size;
  uint8_t *segor;       // this batch's segment ORs
  uint8_t *segor_next;  // the other buffer: zeroed for the next batch
  const uint8_t *vcur;
  uint8_t *vnext;
  const uint8_t *ignore;
  uint64_t *items;
  uint32_t cap;
  uint32_t *counters;
  const uint64_t *tflags;
  uint32_t nfw;
  const uint32_t *listed;  // DynamoRIO: fix-list flags
  uint32_t win_items;
  uint32_t inline_max;  // claimed bytes a wave resolves inline (KBZ_TAIL_INLINE_MAX)
  uint32_t *tail;
  uint32_t *shard_last;
  const uint64_t *frec;    // pass 1's claim records (null: none this batch)
  const uint64_t *rflags;  // which tiles have them
  uint32_t epoch;
  // DynamoRIO chain bookkeeping of k_chain (one shard)
  const uint8_t *neq;
  const uint32_t *bad_list;
  const uint32_t *ctx_last;
  uint32_t *next_last;
  uint32_t *saved_ok;
  uint32_t *flags_w, *fix_list_w, *fix_cnt_w;  // the walks' fix list (DynamoRIO)
  const uint8_t *copy_src;  // the batch's last row -> the context's saved row (when pass 1 ran
  uint8_t *copy_dst;        // k_skip's rule, k_skip's copy blocks' role), or null
  // a shard of the sharded protocol (kbz_shard_finish_gathered): k_chain and k_total<true> ran
  // (walks, fix path, bookkeeping); the prefix of the earlier shards and the batch total come
  // from the all-gathered aggregates [world][nclass * map_size]
  uint32_t shard;
  const uint8_t *gathered;
  uint32_t rank, world;
};
#ifndef KBZ_TAIL_INLINE_MAX  // claimed bytes one k_tail wave resolves inline; the rest become
#define KBZ_TAIL_INLINE_MAX 16  // items, dealt over all of k_fin's waves.  Fresh batches on a warm
#endif                          // map stay inline (their busiest waves had 8-9); on all-0xff maps
                                // the busiest waves had 40-50 and set k_tail's span
                                // (profiles/r05/tail_stamps_novelty.txt)
#ifndef KBZ_TAIL_INLINE  // 1: k_tail resolves claims of < win_items bytes itself, as k_scan does;
#define KBZ_TAIL_INLINE 1  // 0: every claim is an item, resolved by k_fin over the whole grid
#endif                     // (config 2 tail 64 -> 115 us: the 64-row byte reads are the cost)
// One claimed byte's record: info = new bits | f2 << 8 (see claims_records).
__device__ __forceinline__ void record_score(uint64_t rec, uint32_t info, uint32_t chunk,
                                             uint32_t epoch, uint32_t *hnb32, uint32_t *err) {
  if ((uint32_t)(rec >> kRecEpochShift) != epoch) {  // no record of this batch: internal error
    atomicOr(err, 128u);
    return;
  }
  const bool f2 = (info >> 8) & 1;
  const uint32_t fz = (uint32_t)(rec >> 48) & 63u;
  for (uint32_t bits = info & 0xffu; bits; bits &= bits - 1) {
    const int t = __builtin_ctz(bits);
    const uint32_t r = (uint32_t)(rec >> (6 * t)) & 63u;
    atomicMax(&hnb32[(size_t)chunk * kChunk + r], (f2 && r == fz) ? 2u : 1u);
  }
}
// Claims from pass 1's records (a.frec: DynamoRIO, chunk not on the fix list): per lane, each
// claimed byte of its 16 costs one 8-B load; per new bit its first holder scores 1, or 2 where
// the byte was all-virgin, nothing earlier had it and that holder is the first nonzero row.  A
// skipped row is never a first holder: off the fix list it repeats its predecessor's examined
// bytes (k_skip's link rows), whose chain starts at an applied row of this chunk or at a row
// whose bytes are already in prev (an earlier chunk) or V (an earlier batch).
__device__ __forceinline__ void claims_records(const uint64_t *frec, uint32_t epoch, uint32_t chunk,
                                               uint32_t map_size, uint32_t col, bool live,
                                               uint4 nb, uint4 vir, uint4 prev, uint32_t *hnb32,
                                               uint32_t *err) {
  const uint32_t w[4] = {nb.x, nb.y, nb.z, nb.w};
  const uint32_t vv[4] = {vir.x, vir.y, vir.z, vir.w};
  const uint32_t pv[4] = {prev.x, prev.y, prev.z, prev.w};
  const uint64_t *fr = frec + (size_t)chunk * map_size + col;
  uint64_t rv[16];
#pragma unroll
  for (int b = 0; b < 16; b++) {
    const uint32_t x = (w[b >> 2] >> (8 * (b & 3))) & 0xffu;
    rv[b] = (live && x) ? fr[b] : 0ull;
  }
#pragma unroll
  for (int b = 0; b < 16; b++) {
    const uint32_t x = (w[b >> 2] >> (8 * (b & 3))) & 0xffu;
    if (!live || !x) continue;
    const uint64_t rec = rv[b];
    if ((uint32_t)(rec >> kRecEpochShift) != epoch) {  // no record of this batch: internal error
      atomicOr(err, 128u);
      continue;
    }
    const bool f2 = ((vv[b >> 2] >> (8 * (b & 3))) & 0xffu) == 0xffu &&
                    ((pv[b >> 2] >> (8 * (b & 3))) & 0xffu) == 0u;
    const uint32_t fz = (uint32_t)(rec >> 48) & 63u;
    for (uint32_t bits = x; bits; bits &= bits - 1) {
      const int t = __builtin_ctz(bits);
      const uint32_t r = (uint32_t)(rec >> (6 * t)) & 63u;
      atomicMax(&hnb32[(size_t)chunk * kChunk + r], (f2 && r == fz) ? 2u : 1u);
    }
  }
}
__global__ __launch_bounds__(256) void k_tail(TailArgs a) {
  const int lane = threadIdx.x & 63;
  const uint32_t bx = blockIdx.x, s = blockIdx.y;
  const int k = blockIdx.z;
  const uint32_t M = a.map_size;
  const bool dr = a.ca.mode == KBZ_MODE_DYNAMORIO;
  const bool wg0 = bx == 0 && s == 0 && k == 0;
  const uint32_t col0 = (bx * blockDim.x + threadIdx.x) * 16;
  const bool live = col0 < M;
  const uint32_t col = live ? col0 : 0;
  const size_t kc = (size_t)k * M + col;
  __shared__ int sh_flag;
  KBZ_TAIL_DECL;
  const uint32_t tail_id = ((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * 4 + (threadIdx.x >> 6);
  (void)tail_id;
  if (a.copy_src) {  // the batch's last row -> the saved row (the next batch's row-0 predecessor)
    const uint32_t wg = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    const uint32_t step = gridDim.x * gridDim.y * gridDim.z * blockDim.x * 16;
    for (uint32_t i = (wg * blockDim.x + threadIdx.x) * 16; i < M; i += step)
      *(uint4 *)(a.copy_dst + i) = *(const uint4 *)(a.copy_src + i);
  }
  // the next batch's segment ORs start at zero (every segment of this column slice and class)
  if (live)
    for (uint32_t ss = s; ss < kMaxSeg; ss += a.nseg)
      *(uint4 *)(a.segor_next + ((size_t)ss * a.nclass + k) * M + col) = make_uint4(0, 0, 0, 0);
  // ---- 1. DynamoRIO chain / fix path -------------------------------------------------------
  // (a shard: k_chain walked its bad rows and k_total<true> ran the fix path already)
  const uint32_t nbad = (dr && !a.shard) ? a.counters[4] : 0u;
  const uint32_t bad0 = (dr && !a.shard) ? a.tail[4] : 0u;
  if (dr && !a.shard && wg0 && threadIdx.x == 0) {  // k_chain's bookkeeping for a one-shard batch
    const uint32_t f = a.shard_last[1];
    *a.next_last = f ? a.shard_last[0] : *a.ctx_last;
    *a.saved_ok = (nbad == 0) && ((f & 4u) || !bad0);
  }
  bool fixing = false;
  if (nbad + bad0) {  // block-uniform; rare (hash collisions)
    if (wg0) {
      chain_walks(a.ca.n, a.ca.skip, a.neq, a.bad_list, nbad, bad0 != 0, a.flags_w,
                  a.fix_list_w, a.fix_cnt_w);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        st_sc1(&a.tail[5], ld_sc1(a.fx.fix_cnt) != 0 ? 1u : 0u);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        st_sc1(&a.tail[3], 1u);
      }
    }
    if (threadIdx.x == 0) {
      if (!spin_until(&a.tail[3], 1u)) atomicOr(a.ca.err, 32u);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      sh_flag = (int)ld_sc1(&a.tail[5]);
    }
    __syncthreads();
    fixing = sh_flag != 0;
    if (fixing) {
      if (s == 0) {  // DynamoRIO: one class; this column group's k_total fix
        if (live) {
          fix_column(a.fx, M, col, a.segor);
          fix_column(a.fx, M, col + 8, a.segor);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          st_sc1(&a.tail[kTailFixDone + bx], 1u);
        }
      } else if (threadIdx.x == 0) {
        if (!spin_until(&a.tail[kTailFixDone + bx], 1u)) atomicOr(a.ca.err, 32u);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
    }
  }
  // ---- 2. the scan (k_scan's walk; prefixes from the segment ORs) --------------------------
  {
    uint4 prev = make_uint4(0, 0, 0, 0), send = prev, tot = prev;
    // the segment ORs, 16 loads per round trip (unused segments are 0)
    constexpr int SH = kMaxSeg / 2;
    for (int h = 0; h < 2; h++) {
      uint4 sv[SH];
#pragma unroll
      for (int q = 0; q < SH; q++)
        sv[q] = *(const uint4 *)(a.segor + (size_t)(h * SH + q) * a.nclass * M + kc);
#pragma unroll
      for (int q = 0; q < SH; q++) {
        const uint32_t ss = h * SH + q;
        tot = or4(tot, sv[q]);
        if (ss < s) prev = or4(prev, sv[q]);
        if (ss <= s) send = or4(send, sv[q]);
      }
    }
    if (a.gathered) {  // a shard: + the earlier shards' coverage; V' from the batch total
      const size_t ab = (size_t)a.nclass * M;
      uint4 pre = make_uint4(0, 0, 0, 0), all = pre;
      for (uint32_t r = 0; r < a.world; r++) {
        const uint4 g = *(const uint4 *)(a.gathered + r * ab + kc);
        if (r < a.rank) pre = or4(pre, g);
        all = or4(all, g);
      }
      prev = or4(prev, pre);
      send = or4(send, pre);
      tot = all;
    }
    const uint4 vir = *(const uint4 *)(a.vcur + kc);
    const uint4 ig = *(const uint4 *)((a.ignore ? a.ignore : a.vcur) + col);
    const uint32_t c0 = s * a.seg_len, c1 = min(a.nchunks, c0 + a.seg_len);
    const uint32_t t0 = (bx * blockDim.x + (threadIdx.x & ~63u)) * 16 / kTileW;
    const uint32_t cl0 = c0 + lane;
    uint8_t ccls0 = 0;
    uint64_t tfw0 = 0;
    uint32_t lst0 = 0;
    if (cl0 < c1) {
      ccls0 = a.chunk_cls[cl0];
      tfw0 = a.tflags[((size_t)cl0 * a.nclass + k) * a.nfw + (t0 >> 6)];
      if (a.listed) lst0 = a.listed[cl0];
    }
    uint4 rel = make_uint4(~0u, ~0u, ~0u, ~0u);
    if (a.ignore) {  // has_new_bits_with_ignore only examines bytes whose ignore byte is 0
      const uint64_t m0 = nonzero_bytes8((uint64_t)ig.x | ((uint64_t)ig.y << 32));
      const uint64_t m1 = nonzero_bytes8((uint64_t)ig.z | ((uint64_t)ig.w << 32));
      rel = make_uint4(~(uint32_t)m0, ~(uint32_t)(m0 >> 32), ~(uint32_t)m1, ~(uint32_t)(m1 >> 32));
    }
    if (s == 0 && live) {
      *(uint4 *)(a.vnext + kc) = make_uint4(vir.x & ~(tot.x & rel.x), vir.y & ~(tot.y & rel.y),
                                            vir.z & ~(tot.z & rel.z), vir.w & ~(tot.w & rel.w));
      if (k == a.nclass - 1)  // maps this mode does not use (DynamoRIO: tmout, crash) carry over
        for (int kk = a.nclass; kk < 3; kk++)
          *(uint4 *)(a.vnext + (size_t)kk * M + col) = *(const uint4 *)(a.vcur + (size_t)kk * M + col);
    }
    const uint4 vr = live ? make_uint4(vir.x & rel.x, vir.y & rel.y, vir.z & rel.z, vir.w & rel.w)
                          : make_uint4(0, 0, 0, 0);
    __shared__ uint64_t stage_buf[4][kWaveItems];
    ItemStage stg{stage_buf[threadIdx.x >> 6], 0u};
    __shared__ uint4 claim_q[4][kClaimQ];
    ClaimQ cq{claim_q[threadIdx.x >> 6], 0};
    uint32_t inl = 0;  // claimed bytes this wave resolved inline (wave-uniform)
    const uint32_t seg_new = (send.x & vr.x & ~prev.x) | (send.y & vr.y & ~prev.y) |
                             (send.z & vr.z & ~prev.z) | (send.w & vr.w & ~prev.w);
    KBZ_TAIL_MARK();
    if (__ballot(seg_new != 0)) {  // wave-uniform
      for (uint32_t cg = c0; cg < c1; cg += 64) {
        const uint32_t cl = cg + lane;
        bool any = false;
        if (cg == c0) {
          if (cl < c1 && ((ccls0 >> k) & 1)) any = lst0 || ((tfw0 >> (t0 & 63)) & 0xFull);
        } else if (cl < c1 && ((a.chunk_cls[cl] >> k) & 1)) {
          any = (a.listed && a.listed[cl]) ||
                ((a.tflags[((size_t)cl * a.nclass + k) * a.nfw + (t0 >> 6)] >> (t0 & 63)) & 0xFull);
        }
        uint64_t mask = __ballot(any);
        KBZ_TAIL_ADD(walk, (uint32_t)__popcll(mask));
        while (mask) {
          uint32_t cs[KBZ_SCAN_ILP];
#pragma unroll
          for (int u = 0; u < KBZ_SCAN_ILP; u++) {
            cs[u] = mask ? cg + (uint32_t)__builtin_ctzll(mask) : ~0u;
            mask &= mask - 1;
          }
          uint4 o[KBZ_SCAN_ILP];
          bool st[KBZ_SCAN_ILP], lst[KBZ_SCAN_ILP], rec[KBZ_SCAN_ILP];
          // each chunk's first record claim of this lane: its load is issued in the walk and
          // scored after the group, so the group's record loads share one round trip
          uint64_t rv[KBZ_SCAN_ILP];
          uint32_t ri[KBZ_SCAN_ILP];  // new bits | f2 << 8 | 1 << 16 (pending)
          const uint32_t tl = col / kTileW;  // this lane's tile
#pragma unroll
          for (int u = 0; u < KBZ_SCAN_ILP; u++) {  // every load of the group in one round trip
            const uint32_t c = cs[u] != ~0u ? cs[u] : cs[0];
            o[u] = *(const uint4 *)(a.chunk_or + (size_t)c * a.nclass * M + kc);
            lst[u] = a.listed && a.listed[c];
            st[u] = tile_stored(a.tflags, a.nfw, a.nclass, c, k, col) || lst[u];
            rec[u] = a.frec && ((a.rflags[(size_t)c * a.nfw + (tl >> 6)] >> (tl & 63)) & 1);
            ri[u] = 0;
            rv[u] = 0;
          }
          KBZ_TAIL_PH(0);
#pragma unroll
          for (int u = 0; u < KBZ_SCAN_ILP; u++) {
            const uint32_t c = cs[u];  // uniform across the wave
            if (c == ~0u) break;
            if (!st[u]) o[u] = make_uint4(0, 0, 0, 0);
            uint4 nb = make_uint4(o[u].x & vr.x & ~prev.x, o[u].y & vr.y & ~prev.y,
                                  o[u].z & vr.z & ~prev.z, o[u].w & vr.w & ~prev.w);
            if (__ballot(nb.x | nb.y | nb.z | nb.w)) {
              if (a.frec && !lst[u]) {  // lst wave-uniform
                uint4 nbr = make_uint4(0, 0, 0, 0);  // this lane's claimed bytes with records
                if (rec[u]) {
                  nbr = nb;
                  nb = make_uint4(0, 0, 0, 0);
                }
                if (__ballot(nbr.x | nbr.y | nbr.z | nbr.w)) {
                  KBZ_TAIL_ADD(claims, wave_claimed_bytes(nbr));
                  const uint32_t w4[4] = {nbr.x, nbr.y, nbr.z, nbr.w};
                  int b0 = -1;
#pragma unroll
                  for (int b = 15; b >= 0; b--)
                    if ((w4[b >> 2] >> (8 * (b & 3))) & 0xffu) b0 = b;
                  if (live && b0 >= 0) {
                    const int wi = b0 >> 2, sh = 8 * (b0 & 3);
                    const uint32_t x = (pick4(nbr, wi) >> sh) & 0xffu;
                    const bool f2 = ((pick4(vir, wi) >> sh) & 0xffu) == 0xffu &&
                                    ((pick4(prev, wi) >> sh) & 0xffu) == 0u;
                    ri[u] = x | (f2 ? 0x100u : 0u) | 0x10000u;
                    rv[u] = a.frec[(size_t)c * M + col + b0];
                    const uint32_t clr = ~(0xffu << sh);  // the rest of the lane's bytes
                    nbr = make_uint4(wi == 0 ? nbr.x & clr : nbr.x, wi == 1 ? nbr.y & clr : nbr.y,
                                     wi == 2 ? nbr.z & clr : nbr.z, wi == 3 ? nbr.w & clr : nbr.w);
                  }
                  if (__ballot(nbr.x | nbr.y | nbr.z | nbr.w))  // a lane with more (rare)
                    claims_records(a.frec, a.epoch, c, M, col, live, nbr, vir, prev, a.ca.hnb32,
                                   a.ca.err);
                }
              }
              const uint32_t ncl = wave_claimed_bytes(nb);  // the rest: read the rows
              if (!__ballot(nb.x | nb.y | nb.z | nb.w)) {
                // every claimed byte had a record
              } else if (KBZ_TAIL_INLINE && ncl < a.win_items && inl + ncl <= a.inline_max) {
                KBZ_TAIL_ADD(claims, ncl);
                inl += ncl;
                claims_enqueue(a.ca, k, cq, c, col, nb, vir, prev);
              } else {
                KBZ_TAIL_ADD(win, 1);
                emit_items_wave(c, k, col, nb, vir, prev, stg, a.items, a.cap, a.counters,
                                (uint8_t *)a.chunk_or + (size_t)c * a.nclass * M + kc, live,
                                a.win_items);
              }
            }
            prev = or4(prev, o[u]);
          }
          KBZ_TAIL_PH(1);
#pragma unroll
          for (int u = 0; u < KBZ_SCAN_ILP; u++)
            if (ri[u] >> 16) record_score(rv[u], ri[u], cs[u], a.epoch, a.ca.hnb32, a.ca.err);
          KBZ_TAIL_PH(2);
        }
      }
      claims_flush(a.ca, cq);
      flush_items(stg, a.items, a.cap, a.counters);
      KBZ_TAIL_PH(3);
    }
  }
  KBZ_TAIL_END(tail_id);
  // Window and byte items are resolved by k_fin, the next launch: helping with them here, while
  // other workgroups still scan, read stale column windows on gfx950 (the running OR a window
  // item leaves over its chunk's column window, stored sc1 and drained before the item was
  // published, read back sc1 after an agent-scope acquire) -- 8 of 11 fused parity cases raised
  // inconsistent-claim flags; after a launch boundary they are exact.
}

// The second launch of the fused tail.  Scores are fire-and-forget atomicMax into hnb32 (k_tail's
// inline claims, then these items); the outputs are copied once every score is final:
//   - no claim items (the common case: fresh batches on a warm map, every claim inline): k_tail
//     was the previous launch, so every workgroup copies its slice of the rows at once, and
//     workgroup 0 re-arms the per-batch words (no other workgroup reads them: no ticket);
//   - otherwise the items are resolved over the whole grid (k_resolve's work) and the LAST
//     workgroup (an agent-scope ticket after each workgroup's drained atomics) copies all rows
//     with sc1 loads (k_pack's role).
// The last workgroup also clears the fix-list flags and re-arms the per-batch words.
struct FinArgs {
  ResolveArgs ra;
  uint64_t *items;
  uint32_t cap;
  uint32_t *counters;
  uint32_t *tail;
  uint32_t tail_fix_words;  // k_tail's column groups (its fix-done flags)
  uint8_t *hnb_out;
  uint32_t *err_out;
  uint32_t *shard_last;
  uint32_t *flags_w;
  const uint32_t *fix_list_w;
  const uint32_t *fix_cnt;  // null: AFL modes (no fix list)
  uint32_t nchunks;
};
#ifndef KBZ_FIN_GRID  // k_fin's workgroups (its waves share out the claim items)
#define KBZ_FIN_GRID 512
#endif
constexpr uint32_t kFinCopiers = 16;
__device__ __forceinline__ bool spin_until_ge(const uint32_t *p, uint32_t want) {
  for (uint32_t it = 0; it < kSpinMax; it++) {
    if (ld_sc1(p) >= want) return true;
    __builtin_amdgcn_s_sleep(2);
  }
  return false;
}
__device__ __forceinline__ void fin_copy_rows_sc1(const FinArgs &a, uint32_t part, uint32_t parts) {
  // the copiers, after every workgroup arrived: hnb32 was scored with atomics in this launch (sc1
  // loads); copier `part` of `parts` takes every parts-th block of 4 x 16 x blockDim rows, 16 x 4
  // rows in flight per thread
  const uint32_t n = a.ra.n;
  constexpr int U = 16;
  for (uint32_t j0 = 4 * threadIdx.x + part * 4 * U * blockDim.x; j0 < n;
       j0 += parts * 4 * U * blockDim.x) {
    uint32_t h[U][4];
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
      for (int e = 0; e < 4; e++) {
        const uint32_t j = j0 + 4 * u * blockDim.x + e;
        h[u][e] = j < n ? ld_sc1(&a.ra.hnb32[j]) : 0u;
      }
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
      for (int e = 0; e < 4; e++) {
        const uint32_t j = j0 + 4 * u * blockDim.x + e;
        if (j < n) {
          a.ra.hnb32[j] = 0;
          if (a.hnb_out) a.hnb_out[j] = (uint8_t)h[u][e];
        }
      }
  }
}
__device__ __forceinline__ void fin_copy_rows(const FinArgs &a, uint32_t j0, uint32_t step) {
  // no items: hnb32 is final since k_tail (an earlier launch); 4 rows per thread per step (one
  // 16-B load of hnb32), j0 a multiple of 4
  const uint32_t n = a.ra.n;
  for (uint32_t j = j0; j < n; j += step) {
    uint32_t h[4];
    if (j + 4 <= n) {
      const uint4 v = *(const uint4 *)(a.ra.hnb32 + j);
      h[0] = v.x, h[1] = v.y, h[2] = v.z, h[3] = v.w;
      *(uint4 *)(a.ra.hnb32 + j) = make_uint4(0, 0, 0, 0);
    } else {
      for (int u = 0; u < 4; u++) {
        h[u] = j + u < n ? a.ra.hnb32[j + u] : 0u;
        if (j + u < n) a.ra.hnb32[j + u] = 0;
      }
    }
    if (a.hnb_out) {
      if (j + 4 <= n && !((uintptr_t)(a.hnb_out + j) & 3))
        *(uint32_t *)(a.hnb_out + j) = h[0] | (h[1] << 8) | (h[2] << 16) | (h[3] << 24);
      else
        for (int u = 0; u < 4; u++)
          if (j + u < n) a.hnb_out[j + u] = (uint8_t)h[u];
    }
  }
}
// fix-list flags, k_tail's fix-done flags, the sticky error flags' host-mapped copy, the stats
// words and the per-batch counters (one workgroup)
__device__ __forceinline__ void fin_rearm(const FinArgs &a) {
  const uint32_t nfix = a.fix_cnt ? min(ld_sc1(a.fix_cnt), a.nchunks) : 0u;
  for (uint32_t i = threadIdx.x; i < nfix; i += blockDim.x) a.flags_w[a.fix_list_w[i]] = 0;
  for (uint32_t i = threadIdx.x; i < a.tail_fix_words; i += blockDim.x) a.tail[kTailFixDone + i] = 0;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t *cn = a.counters;
    a.err_out[0] = ld_sc1(&cn[1]);  // the sticky error flags, host-mapped (k_pack's role)
    a.err_out[1] = ld_sc1(&cn[2]);
    cn[8] = ld_sc1(&cn[0]);  // kbz_ctx_stats: claim items, recomputed chunks, bad rows
    cn[9] = ld_sc1(&cn[3]);
    cn[10] = ld_sc1(&cn[4]);
    cn[0] = cn[3] = cn[4] = cn[5] = 0;
    a.shard_last[0] = a.shard_last[1] = 0;
    for (int i = 0; i < 6; i++) a.tail[i] = 0;
  }
}
__global__ __launch_bounds__(256) void k_fin(FinArgs a) {
  __shared__ int last;
  const uint32_t gtid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t wave = gtid >> 6;
  const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
  const uint32_t cnt = min(a.counters[0], a.cap);  // k_tail's appends: an earlier launch
  // stamp build: k_fin's waves are records kFinStampBase + wave (phases: windows, byte-item
  // flushes, the rest of the item loop, the ticket / copy)
  KBZ_TAIL_DECL;
  const uint32_t fin_id = kFinStampBase + wave;
  (void)fin_id;
  if (cnt == 0) {
    fin_copy_rows(a, 4 * gtid, 4 * gridDim.x * blockDim.x);
    if (blockIdx.x == 0) fin_rearm(a);
    return;
  }
  KBZ_TAIL_MARK();
  // kClaimQ items per wave per round: byte items go through the claim queue (their rows' bytes
  // in flight together, as k_scan's inline claims), window items one at a time
  const int lane = threadIdx.x & 63;
  __shared__ uint4 fin_q[4][kClaimQ];
  ClaimQ cq{fin_q[threadIdx.x >> 6], 0};
  const ClaimArgs ca{a.ra.traces, a.ra.stride, a.ra.n, a.ra.mode, a.ra.outcome, a.ra.skip,
                     a.ra.hnb32, a.ra.err};
  // items are dealt round-robin over the waves (item i to wave i % nwaves): a window item streams
  // 64 rows, so consecutive ones must not queue on one wave (novelty-heavy batches: ~50 window
  // items, dealt 8 per wave k_fin took 250 us)
  for (uint32_t it0 = wave; it0 < cnt; it0 += nwaves * kClaimQ) {
    const uint32_t myit = it0 + (uint32_t)lane * nwaves;
    const uint64_t mine = (lane < kClaimQ && myit < cnt) ? a.items[myit] : 0ull;
    if (lane < kClaimQ && myit < cnt) a.items[myit] = 0;  // all-zero between batches
#pragma unroll
    for (int j = 0; j < kClaimQ; j++) {
      if (it0 + (uint32_t)j * nwaves >= cnt) break;  // wave-uniform
      const uint64_t item = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(mine >> 32), j) << 32) |
                            __builtin_amdgcn_readlane((uint32_t)mine, j);
      if (!item) {  // reserved and never written
        if (lane == 0) atomicOr(a.ra.err, 64u);
        continue;
      }
      if ((item & 0xff) == 0) {
        KBZ_TAIL_PH(2);
        resolve_item(a.ra, item);  // window item
        KBZ_TAIL_ADD(win, 1);
        KBZ_TAIL_PH(0);
      } else {
        KBZ_TAIL_ADD(claims, 1);
        if (lane == 0)
          cq.q[cq.m] = make_uint4(item_chunk(item), (uint32_t)(item >> 11) & 0xffffff,
                                  (uint32_t)item & 0x1ff, (uint32_t)(item >> 9) & 3);
        cq.m++;
      }
    }
    KBZ_TAIL_PH(2);
    claims_flush(ca, cq);
    KBZ_TAIL_PH(1);
  }
  // The last kFinCopiers workgroups to arrive copy the rows together once every workgroup has
  // arrived: they only wait for workgroups that already hold a ticket or are still to be
  // dispatched (at most kFinCopiers - 1 of them), never for one that waits.  The last copier
  // to finish re-arms.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's atomics and stores are done
  __syncthreads();
  const uint32_t G = gridDim.x, nc = min(G, (uint32_t)kFinCopiers);
  if (threadIdx.x == 0) {
    const uint32_t tk = atomicAdd(&a.tail[0], 1u);
    last = tk >= G - nc ? (int)(tk - (G - nc)) : -1;  // copier index, or -1
    if (last >= 0 && !spin_until_ge(&a.tail[0], G)) atomicOr(a.ra.err, 64u);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  KBZ_TAIL_PH(3);
  KBZ_TAIL_END(fin_id);
  if (last < 0) return;
  fin_copy_rows_sc1(a, (uint32_t)last, nc);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(&a.tail[1], 1u) == nc - 1;  // the last copier done
  __syncthreads();
  if (!last) return;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  fin_rearm(a);
}

// ---------------------------------------------------------------------------------------------
// Small AFL-mode batches without hashes in ONE launch (the AFL plugin's per-exec flushes:
// fuzzer/main.c:385 asks is_new_path after every exec; afl_instrumentation.c:231-274 routes each
// exec's map by outcome and runs has_new_bits, :600-662, on it).  With n <= 64 traces every
// workgroup owns a slice of the map's columns for ALL rows of the batch, so the sequential rule
// needs no other workgroup: lane = 16-B column group, rows in order with the three virgin maps
// in registers -- row j claims t_j & V_k (k = its class), scores 2 where it has a nonzero byte
// whose V_k byte is 0xff, V_k &= ~t_j.  Per row the workgroup's best score meets in LDS, then one
// agent-scope atomicMax per (workgroup, row) into hnb32; the last workgroup to finish (an agent
// atomic ticket after a release fence) packs hnb32 into hnb_out and re-arms it.  Rows are read 16
// at a time (from pinned host memory on the plugin's zero-copy path).
// ---------------------------------------------------------------------------------------------
constexpr uint32_t kSmallRows = 64;
#ifndef KBZ_SMALL_TPB  // k_small's threads per workgroup (64: one wave each, 4x the workgroups)
#define KBZ_SMALL_TPB 256
#endif
static_assert(KBZ_SMALL_TPB >= (int)kSmallRows && KBZ_SMALL_TPB % 64 == 0, "k_small block");
struct SmallArgs {
  const uint8_t *traces;
  size_t stride;
  uint32_t n, map_size;
  const int8_t *outcome;
  const uint8_t *vcur;
  uint8_t *vnext;
  uint32_t *hnb32;
  uint8_t *hnb_out;
  uint32_t *ticket;    // zero between launches (the last workgroup re-arms it)
  uint32_t *stats;     // kbz_ctx_stats words of the batch (counters[8..10])
};
__device__ __forceinline__ uint4 xform16(uint4 a, int xf) {
  const uint64_t lo = xform8((uint64_t)a.x | ((uint64_t)a.y << 32), xf);
  const uint64_t hi = xform8((uint64_t)a.z | ((uint64_t)a.w << 32), xf);
  return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}
template <int MODE>
__global__ __launch_bounds__(KBZ_SMALL_TPB) void k_small(SmallArgs a) {
  static_assert(MODE != KBZ_MODE_DYNAMORIO, "DynamoRIO hashes every trace (k_pass1*)");
  __shared__ uint32_t score[kSmallRows];
  __shared__ int last;
  const int lane = threadIdx.x & 63;
  if (threadIdx.x < kSmallRows) score[threadIdx.x] = 0;
  const uint32_t n = a.n;
  // lane j: row j's class (rows are wave-uniform below: readlane)
  const int clsl = class_of(MODE, (lane < (int)n && a.outcome) ? a.outcome[lane] : KBZ_FUZZ_NONE);
  const uint32_t col0 = (blockIdx.x * blockDim.x + threadIdx.x) * 16;
  const bool live = col0 < a.map_size;
  const uint32_t col = live ? col0 : 0;
  uint4 v[3];
#pragma unroll
  for (int k = 0; k < 3; k++) v[k] = *(const uint4 *)(a.vcur + (size_t)k * a.map_size + col);
  if (!live)
#pragma unroll
    for (int k = 0; k < 3; k++) v[k] = make_uint4(0, 0, 0, 0);  // no claim from a dead lane
  __syncthreads();  // score[] is zero
  constexpr int G = 16;  // rows in flight per lane
  for (uint32_t j0 = 0; j0 < n; j0 += G) {
    uint4 r[G];
#pragma unroll
    for (int u = 0; u < G; u++) {
      const uint32_t j = min(j0 + u, n - 1);  // past the end: a valid row, not processed
      r[u] = *(const uint4 *)(a.traces + (size_t)j * a.stride + col);
    }
#pragma unroll
    for (int u = 0; u < G; u++) {
      const uint32_t j = j0 + u;
      if (j >= n) break;  // uniform
      const int k = __builtin_amdgcn_readlane(clsl, j);
      const uint4 t = xform16(r[u], class_xf(MODE, k));
      uint4 vk = k == 0 ? v[0] : k == 1 ? v[1] : v[2];
      const uint64_t t0 = (uint64_t)t.x | ((uint64_t)t.y << 32), t1 = (uint64_t)t.z | ((uint64_t)t.w << 32);
      const uint64_t v0 = (uint64_t)vk.x | ((uint64_t)vk.y << 32), v1 = (uint64_t)vk.z | ((uint64_t)vk.w << 32);
      const bool any = ((t0 & v0) | (t1 & v1)) != 0;
      // has_new_bits' 2: a nonzero byte of the trace where the virgin byte is still 0xff
      const bool two = ((nonzero_hi8(t0) & ~nonzero_hi8(~v0)) |
                        (nonzero_hi8(t1) & ~nonzero_hi8(~v1))) != 0;
      vk = make_uint4(vk.x & ~t.x, vk.y & ~t.y, vk.z & ~t.z, vk.w & ~t.w);
      if (k == 0) v[0] = vk;
      else if (k == 1) v[1] = vk;
      else v[2] = vk;
      const uint64_t b2 = __ballot(two), b1 = __ballot(any);
      if ((b1 | b2) && lane == 0) atomicMax(&score[j], b2 ? 2u : 1u);
    }
  }
  if (live)
#pragma unroll
    for (int k = 0; k < 3; k++) *(uint4 *)(a.vnext + (size_t)k * a.map_size + col) = v[k];
  __syncthreads();  // every wave's scores are in score[]
  if (threadIdx.x < n && score[threadIdx.x]) atomicMax(&a.hnb32[threadIdx.x], score[threadIdx.x]);
  // hand-off to the last workgroup: every wave's atomics complete, then one release + ticket
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = atomicAdd(a.ticket, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (threadIdx.x < n) {
    const uint32_t h = __hip_atomic_load(&a.hnb32[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (a.hnb_out) a.hnb_out[threadIdx.x] = (uint8_t)h;
    __hip_atomic_store(&a.hnb32[threadIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (threadIdx.x == 0) {
    __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    a.stats[0] = a.stats[1] = a.stats[2] = 0;  // no claim items, no fix path
  }
}

__global__ __launch_bounds__(256) void k_or_reduce(uint8_t *out, const uint8_t *in, size_t r_lo,
                                                    size_t r_hi, size_t bytes) {
  const size_t i = (size_t)(blockIdx.x * blockDim.x + threadIdx.x) * 16;
  if (i + 16 <= bytes) {
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (size_t r = r_lo; r < r_hi; r++) acc = or4(acc, *(const uint4 *)(in + r * bytes + i));
    *(uint4 *)(out + i) = acc;
  } else {
    for (size_t b = i; b < bytes; b++) {
      uint8_t acc = 0;
      for (size_t r = r_lo; r < r_hi; r++) acc |= in[r * bytes + b];
      out[b] = acc;
    }
  }
}

// The sharded protocol's prefix (OR of ranks < rank) and total (OR of all ranks) of the
// all-gathered aggregates, in one pass over them (16 B per thread; prefix may be null).
__global__ __launch_bounds__(256) void k_or_prefix_total(uint8_t *prefix, uint8_t *total,
                                                          const uint8_t *in, size_t rank,
                                                          size_t world, size_t bytes) {
  const size_t i = (size_t)(blockIdx.x * blockDim.x + threadIdx.x) * 16;
  if (i + 16 <= bytes) {
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (size_t r = 0; r < world; r++) {
      if (r == rank && prefix) *(uint4 *)(prefix + i) = acc;
      acc = or4(acc, *(const uint4 *)(in + r * bytes + i));
    }
    if (rank >= world && prefix) *(uint4 *)(prefix + i) = acc;
    *(uint4 *)(total + i) = acc;
  } else {
    for (size_t b = i; b < bytes; b++) {
      uint8_t acc = 0;
      for (size_t r = 0; r < world; r++) {
        if (r == rank && prefix) prefix[b] = acc;
        acc |= in[r * bytes + b];
      }
      if (rank >= world && prefix) prefix[b] = acc;
      total[b] = acc;
    }
  }
}

// ---- merger: AND-fold -----------------------------------------------------------------------
// partial[g][:] = AND of states in group g (16 B per thread, 8 independent streaming loads in
// flight; states are read once, so the loads bypass cache retention).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_and_groups(const uint8_t *states, size_t n,
                                                     size_t state_bytes, size_t group_len,
                                                     uint8_t *partial) {
  const size_t col = (size_t)(blockIdx.x * blockDim.x + threadIdx.x) * 16;
  const size_t g = blockIdx.y;
  if (col >= state_bytes) return;
  const size_t s0 = g * group_len, s1 = std::min(n, s0 + group_len);
  const u32x4 *p = (const u32x4 *)(states + col);
  const size_t st = state_bytes / 16;  // row stride in u32x4
  u32x4 acc = {~0u, ~0u, ~0u, ~0u};
  size_t s = s0;
  for (; s + 8 <= s1; s += 8) {
    u32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) v[u] = __builtin_nontemporal_load(p + (s + u) * st);
#pragma unroll
    for (int u = 0; u < 8; u++) acc &= v[u];
  }
  for (; s < s1; s++) acc &= __builtin_nontemporal_load(p + s * st);
  *(u32x4 *)(partial + g * state_bytes + col) = acc;
}
__global__ __launch_bounds__(256) void k_and_rows(const uint8_t *rows, size_t nrows, size_t bytes,
                                                   uint8_t *out, int accumulate) {
  const size_t col = (size_t)(blockIdx.x * blockDim.x + threadIdx.x) * 16;
  if (col >= bytes) return;
  uint4 acc = accumulate ? *(const uint4 *)(out + col) : make_uint4(~0u, ~0u, ~0u, ~0u);
  for (size_t r = 0; r < nrows; r++) {
    const uint4 a = *(const uint4 *)(rows + r * bytes + col);
    acc.x &= a.x; acc.y &= a.y; acc.z &= a.z; acc.w &= a.w;
  }
  *(uint4 *)(out + col) = acc;
}
// byte-granular fallback for state sizes that are not a multiple of 16
__global__ void k_and_bytes(const uint8_t *states, size_t n, size_t state_bytes, uint8_t *out,
                            int accumulate) {
  const size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= state_bytes) return;
  uint8_t acc = accumulate ? out[b] : 0xff;
  for (size_t s = 0; s < n; s++) acc &= states[s * state_bytes + b];
  out[b] = acc;
}

// per-module combine (dynamorio_instrumentation.c:1477-1493): any[j] = OR over modules of hnb != 0
__global__ __launch_bounds__(256) void k_modules_any(const uint8_t *hnb, size_t k, size_t n,
                                                     uint8_t *any) {
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  uint8_t r = 0;
  for (size_t m = 0; m < k; m++) r |= hnb[m * n + j] != 0;
  any[j] = r;
}

// ---- picker: ignore-bytes diff across repeated runs (picker/main.c:240-262) --------------------
// 0x80 in every nonzero byte of x
__device__ __forceinline__ uint32_t nz_bytes32(uint32_t x) {
  return (((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
}
__device__ __forceinline__ uint32_t wave_sum32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
// grid (columns of 16 B / 256, files): per 16-B column, XOR of consecutive iterations of one
// file (each row read once, the previous one kept in registers); the OR of the differences goes
// to diff (zeroed, u32 atomics, nonzero words only); pair_counts[f*(iters-1) + it-1] += differing
// bytes of this wave's 1 KiB (one atomic per wave per pair).
__global__ __launch_bounds__(256) void k_picker_diff(const uint8_t *runs, size_t files, size_t iters,
                                                     size_t size, uint32_t *diff,
                                                     uint32_t *pair_counts) {
  const size_t col = (size_t)(blockIdx.x * blockDim.x + threadIdx.x) * 16;
  const bool in = col < size;
  for (size_t f = blockIdx.y; f < files; f += gridDim.y) {
    const uint8_t *base = runs + f * iters * size + (in ? col : 0);
    uint4 prev = in ? ld_stream16(base) : make_uint4(0, 0, 0, 0);
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (size_t it = 1; it < iters; it++) {
      const uint4 cur = in ? ld_stream16(base + it * size) : make_uint4(0, 0, 0, 0);
      const uint4 d = make_uint4(prev.x ^ cur.x, prev.y ^ cur.y, prev.z ^ cur.z, prev.w ^ cur.w);
      acc = or4(acc, d);
      const uint32_t c = __popc(nz_bytes32(d.x)) + __popc(nz_bytes32(d.y)) +
                         __popc(nz_bytes32(d.z)) + __popc(nz_bytes32(d.w));
      const uint32_t tot = wave_sum32(c);
      if (pair_counts && (threadIdx.x & 63) == 0 && tot)
        atomicAdd(pair_counts + f * (iters - 1) + it - 1, tot);
      prev = cur;
    }
    if (in) {
      uint32_t *dw = diff + col / 4;
      if (acc.x) atomicOr(dw + 0, acc.x);
      if (acc.y) atomicOr(dw + 1, acc.y);
      if (acc.z) atomicOr(dw + 2, acc.z);
      if (acc.w) atomicOr(dw + 3, acc.w);
    }
  }
}
// in place: a byte that differed anywhere -> 0x00 (ignore), else 0xff; counts the noisy bytes
__global__ __launch_bounds__(256) void k_picker_final(uint32_t *words, size_t nwords,
                                                      unsigned long long *total) {
  const size_t w = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t nz = 0;
  if (w < nwords) {
    nz = nz_bytes32(words[w]);
    words[w] = ~((nz >> 7) * 0xffu);
  }
  const uint32_t c = wave_sum32(__popc(nz));
  if (total && (threadIdx.x & 63) == 0 && c) atomicAdd(total, (unsigned long long)c);
}

// ---- transform rows: classify_counts / simplify_trace applied to a batch of maps -------------
// 16 B per thread, grid (columns / 256 threads, rows).  The all-zero-word skip of classify_counts
// (dynamorio_instrumentation.c:273) gives the same bytes (classify(0) = 0); simplify writes its
// 0x01 bytes into all-zero words too (afl_instrumentation.c:688).
__global__ __launch_bounds__(256) void k_transform_rows(const uint8_t *rows, size_t n, size_t stride,
                                                        size_t len, int xf, uint8_t *out,
                                                        size_t out_stride) {
  const size_t col = (size_t)(blockIdx.x * blockDim.x + threadIdx.x) * 16;
  if (col >= len) return;
  for (size_t r = blockIdx.y; r < n; r += gridDim.y) {
    const uint4 v = *(const uint4 *)(rows + r * stride + col);
    const uint64_t lo = xform8((uint64_t)v.x | ((uint64_t)v.y << 32), xf);
    const uint64_t hi = xform8((uint64_t)v.z | ((uint64_t)v.w << 32), xf);
    *(uint4 *)(out + r * out_stride + col) =
        make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
  }
}

// ---- standalone row hashes (utility path: one lane per row, direct loads) ---------------------
__global__ void k_rowhash32(const uint8_t *rows, size_t n, size_t stride, size_t len, uint32_t seed,
                            uint32_t *out) {
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint8_t *p = rows + j * stride;
  uint64_t h = (uint64_t)(seed ^ (uint32_t)len);
  for (size_t w = 0; w < len / 8; w++) {
    uint64_t k;
    memcpy(&k, p + 8 * w, 8);
    h = h32_step(h, h32_mix(k));
  }
  out[j] = h32_final(h);
}
__global__ void k_rowxxh64(const uint8_t *rows, size_t n, size_t stride, size_t len, uint64_t seed,
                           uint64_t *out) {
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint8_t *p = rows + j * stride, *end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t a = seed + kXP1 + kXP2, b = seed + kXP2, c = seed, d = seed - kXP1;
    while (p + 32 <= end) {
      uint64_t w[4];
      memcpy(w, p, 32);
      a = xx_round(a, w[0]);
      b = xx_round(b, w[1]);
      c = xx_round(c, w[2]);
      d = xx_round(d, w[3]);
      p += 32;
    }
    h = rotl64(a, 1) + rotl64(b, 7) + rotl64(c, 12) + rotl64(d, 18);
    h = xx_merge(h, a);
    h = xx_merge(h, b);
    h = xx_merge(h, c);
    h = xx_merge(h, d);
  } else {
    h = seed + kXP5;
  }
  h += (uint64_t)len;
  while (p + 8 <= end) {
    uint64_t w;
    memcpy(&w, p, 8);
    h ^= xx_round(0, w);
    h = rotl64(h, 27) * kXP1 + kXP4;
    p += 8;
  }
  if (p + 4 <= end) {
    uint32_t w;
    memcpy(&w, p, 4);
    h ^= (uint64_t)w * kXP1;
    h = rotl64(h, 23) * kXP2 + kXP3;
    p += 4;
  }
  while (p < end) {
    h ^= (*p) * kXP5;
    h = rotl64(h, 11) * kXP1;
    p++;
  }
  out[j] = xx_avalanche(h);
}

}  // namespace

// =============================================================================================
// host runtime
// =============================================================================================
struct kbz_ctx {
  int device = 0;
  size_t M = 0;
  int mode = 0;
  int nc = 1;
  size_t max_batch = 0;
  size_t max_chunks = 0;
  uint8_t *V[2] = {nullptr, nullptr};
  int vcur = 0;
  uint32_t *last = nullptr;  // [2] double-buffered last hash
  int lcur = 0;
  uint8_t *ignore = nullptr;
  uint8_t *chunk_or = nullptr;
  uint8_t *chunk_cls = nullptr;
  uint64_t *tflags = nullptr;    // [chunks][nc][nfw] stored tiles of chunk_or (Pass1Args)
  uint32_t nfw = 1;
  uint32_t *flags = nullptr;     // [chunks] queued for recomputation
  uint32_t *fix_list = nullptr;  // [chunks]
  uint32_t *bad_list = nullptr;  // [max_batch] DynamoRIO rows skipped but differing (k_skip)
  uint8_t *saved_row = nullptr;  // [2][M] raw last row of the previous batch (row 0's
  int srow = 0;                  // predecessor) is saved_row + srow*M; its clean flag counters[6+srow]
  bool saved_valid = false;
  int pass1 = KBZ_PASS1_AUTO;    // kbz_ctx_set_pass1
  uint8_t *skip = nullptr;
  uint8_t *neq = nullptr;
  uint32_t *h32 = nullptr;
  uint32_t *hnb32 = nullptr;
  uint8_t *segor = nullptr;      // this batch's segment ORs (zero at batch start)
  uint8_t *segor_alt = nullptr;  // the other buffer (the fused tail zeroes it and swaps)
  uint32_t *tail = nullptr;      // k_tail's words (kTailFixDone + column groups)
  bool fused_ok = true;          // one-shard batches through k_tail (KBZ_DEBUG_STAGED=1: staged)
  bool shard_keep = false;       // this batch's k_total kept the segment ORs (kbz_shard_reduce_into)
  bool rec_ok = true;            // pass-1 claim records (KBZ_DEBUG_NO_REC=1: off)
  uint64_t *frec = nullptr;      // [max_chunks][M] claim records, allocated on first use
  uint64_t *rflags = nullptr;    // [max_chunks][nfw] tiles with records
  uint32_t epoch = 0;            // the record tag of the current batch (1..1023)
  bool cur_rec = false;          // the current batch's pass 1 wrote records
  uint8_t *segprev = nullptr;
  uint8_t *total = nullptr;
  uint64_t *items = nullptr;
  uint32_t item_cap = 0;
  uint32_t win_items = KBZ_WIN_ITEMS;  // claimed bytes per chunk x 1-KiB window: window item
  uint32_t inline_max = KBZ_TAIL_INLINE_MAX;  // k_tail: inline claims per wave (tests: env)
  bool small_ok = true;  // k_small for small AFL batches (tests: KBZ_DEBUG_NO_SMALL=1 disables)
  uint32_t *counters = nullptr;  // [0] items, [1] overflow, [2] resolve error, [3] fix list,
                                 // [4] bad rows, [6..7] clean flags of the saved rows,
                                 // [8..10] the last finished batch's [0], [3], [4],
                                 // [12] k_small's workgroup ticket
  uint32_t *shard_last = nullptr;  // [2]
  // k_pass1s runs k_skip's rule itself for fused one-shard DynamoRIO batches (no k_skip launch;
  // KBZ_DEBUG_NO_FSKIP=1: k_skip as before)
  bool fskip_ok = true;
  uint32_t spin_max = 1u << 20;  // kLookbackSpinMax; KBZ_DEBUG_LOOKBACK_SPIN overrides (tests)
  uint64_t *lastpub = nullptr;  // [max_chunks] look-back words (tag << 32 | last-row hash)
  uint32_t skip_tag = 0;
  const uint8_t *tail_copy_src = nullptr;  // this batch's last row -> saved row, by k_tail
  uint8_t *tail_copy_dst = nullptr;
  // in-flight shard
  const uint8_t *cur_traces = nullptr;
  size_t cur_n = 0, cur_stride = 0;
  const int8_t *cur_outcome = nullptr;
  uint32_t *cur_h32_out = nullptr;
  uint32_t *cur_h32 = nullptr;  // where pass 1 wrote this shard's hashes
  uint32_t cur_chunks = 0, cur_seg_len = 1, cur_nseg = 1;
  bool fix_pending = false;  // DynamoRIO: k_skip ran for this batch, k_total runs the fix path
  int stage = 0;
  // a fused one-shard DynamoRIO batch: the last-hash and saved-row words k_tail reads / writes
  uint32_t *fchain_ctx_last = nullptr, *fchain_next_last = nullptr, *fchain_saved_ok = nullptr;
  // host streaming
  hipStream_t copy_stream = nullptr, work_stream = nullptr;
  uint8_t *pin[2] = {nullptr, nullptr};
  int8_t *pin_oc[2] = {nullptr, nullptr};
  uint8_t *dslot[2] = {nullptr, nullptr};
  int8_t *dslot_oc[2] = {nullptr, nullptr};
  uint8_t *dres_hnb = nullptr;
  uint32_t *dres_h32 = nullptr;
  uint64_t *dres_x64 = nullptr;
  size_t slot_rows = 0;
  hipEvent_t ev_copied[2] = {nullptr, nullptr}, ev_used[2] = {nullptr, nullptr};
  // kbz_reset_virgin on a caller's stream: the next batch's stream waits for ev_reset (the host
  // paths run on work_stream, which nothing else orders after the caller's stream); ev_prior
  // orders the fill after batches still queued on work_stream
  hipEvent_t ev_reset = nullptr, ev_prior = nullptr;
  hipStream_t reset_stream = nullptr;
  bool reset_pending = false;
  // pinned ingest ring (kbz_ring_*): per slot, device + pinned results and the pending
  // delivery of the batch last submitted from it
  struct RingSlot {
    uint8_t *d_hnb = nullptr, *h_hnb = nullptr;
    uint32_t *d_h32 = nullptr, *h_h32 = nullptr;
    uint64_t *d_x64 = nullptr, *h_x64 = nullptr;
    // device views of the pinned rows / outcomes / results (zero-copy small batches)
    uint8_t *m_rows = nullptr, *m_hnb = nullptr;
    int8_t *m_oc = nullptr;
    uint32_t *m_h32 = nullptr;
    uint64_t *m_x64 = nullptr;
    size_t n = 0;
    size_t copied = 0;  // rows [0, copied) already queued for the device slot (kbz_ring_commit)
    bool pending = false;
    uint8_t *hnb_out = nullptr;
    uint32_t *h32_out = nullptr;
    uint64_t *x64_out = nullptr;
  } ring[2];
  int ring_next = 0;        // slot the next kbz_ring_acquire returns
  int ring_acquired = -1;   // slot handed out and not yet submitted
  uint32_t *h_err = nullptr, *d_err = nullptr;  // host-mapped copy of counters[1..2] (k_pack)
  // kbz_ctx_time_pass1: HIP events around every pass-1 launch (on its stream)
  bool timing = false;
  uint32_t time_every = 1, p1_launch_no = 0;  // time one pass-1 launch in time_every
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pass1;
  size_t ev_used_n = 0;
  double pass1_folded_ms = 0;  // launches folded out of the event pool (kEvFoldAt)
  uint32_t pass1_folded_n = 0;
  // kbz_ctx_time_stages: HIP events around the other stages' launches (stage id, start, end)
  bool stage_timing = false;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_pool_used = 0;
  struct StageRec {
    int stage;
    hipEvent_t a, b;
  };
  std::vector<StageRec> stage_recs;
  double stage_folded_ms[KBZ_NSTAGES] = {};
  uint32_t stage_folded_nb = 0;
};

namespace {
thread_local std::string g_err;

int fail(const std::string &msg) {
  g_err = msg;
  return -1;
}
#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess)                                                               \
      return fail(std::string(#expr) + ": " + hipGetErrorString(_e));                   \
  } while (0)

struct DevGuard {
  int old = -1;
  explicit DevGuard(int dev) {
    (void)hipGetDevice(&old);
    if (old != dev) (void)hipSetDevice(dev);
  }
  ~DevGuard() {
    int cur;
    (void)hipGetDevice(&cur);
    if (old >= 0 && cur != old) (void)hipSetDevice(old);
  }
};

inline unsigned cdiv(size_t a, size_t b) { return (unsigned)((a + b - 1) / b); }

template <typename T>
int dalloc(T **p, size_t count) {
  if (count == 0) count = 1;
  HIP_TRY(hipMalloc((void **)p, count * sizeof(T)));
  return 0;
}

void free_ctx(kbz_ctx *c) {
  if (!c) return;
  DevGuard g(c->device);
  void *ptrs[] = {c->V[0], c->V[1], c->last, c->ignore, c->chunk_or, c->chunk_cls, c->tflags,
                  c->flags, c->fix_list, c->bad_list, c->saved_row,
                  c->skip, c->neq, c->h32, c->hnb32, c->segor, c->segor_alt, c->tail,
                  c->segprev, c->total,
                  c->items, c->counters, c->shard_last, c->dslot[0], c->dslot[1],
                  c->dslot_oc[0], c->dslot_oc[1], c->dres_hnb, c->dres_h32, c->dres_x64, c->frec,
                  c->rflags, c->lastpub};
  for (void *p : ptrs)
    if (p) (void)hipFree(p);
  for (int i = 0; i < 2; i++) {
    auto &r = c->ring[i];
    for (void *p : {(void *)r.d_hnb, (void *)r.d_h32, (void *)r.d_x64})
      if (p) (void)hipFree(p);
    for (void *p : {(void *)r.h_hnb, (void *)r.h_h32, (void *)r.h_x64})
      if (p) (void)hipHostFree(p);
    if (c->pin[i]) (void)hipHostFree(c->pin[i]);
    if (c->pin_oc[i]) (void)hipHostFree(c->pin_oc[i]);
    if (c->ev_copied[i]) (void)hipEventDestroy(c->ev_copied[i]);
    if (c->ev_used[i]) (void)hipEventDestroy(c->ev_used[i]);
  }
  for (auto &e : c->ev_pass1) {
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  for (auto e : c->ev_pool) (void)hipEventDestroy(e);
  if (c->ev_reset) (void)hipEventDestroy(c->ev_reset);
  if (c->ev_prior) (void)hipEventDestroy(c->ev_prior);
  if (c->h_err) (void)hipHostFree(c->h_err);
  if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
  if (c->work_stream) (void)hipStreamDestroy(c->work_stream);
  delete c;
}

constexpr int kWideNX = KBZ_WIDE_NX;        // transform waves of k_pass1w
constexpr int kWideNL = KBZ_WIDE_NL;        // loader waves of k_pass1w
constexpr int kWideD = KBZ_WIDE_D;          // their register ring depth
constexpr uint32_t kWideBelowChunks = 512;  // 2 chunks per CU on a 256-CU MI355X
// pass-1 / stage timing events: device-scope release (the default system-scope fence costs
// ~6 us of idle GPU per event, profiles/r02_v9)
#ifndef KBZ_P1_STOP_ON_NEXT  // DynamoRIO pass-1 timing: stop event = k_skip's start (0: own stop)
#define KBZ_P1_STOP_ON_NEXT 0
#endif
#ifndef KBZ_EVENT_FLAGS
#define KBZ_EVENT_FLAGS hipEventReleaseToDevice
#endif
constexpr unsigned kEventScope = KBZ_EVENT_FLAGS;
#ifndef KBZ_PASS1_DEPTH
#define KBZ_PASS1_DEPTH 2
#endif
// Fewer chunks than two per CU (large maps, small batches): the wide-map variant, unless the
// context forces one (kbz_ctx_set_pass1; the environment KBZ_PASS1=narrow|wide sets a new
// context's default, for A/B timing).
bool pass1_is_wide(int choice, uint32_t chunks) {
  if (choice == KBZ_PASS1_NARROW) return false;
  if (choice == KBZ_PASS1_WIDE) return true;
  return chunks < kWideBelowChunks;
}
// Pass-1 launches.  With timing on (kbz_ctx_time_pass1) the kernel is dispatched by
// hipExtLaunchKernelGGL with start/stop events taken from its own dispatch packet: no marker
// packets around it (two hipEventRecord calls left ~6 us of idle GPU each between pass 1 and
// its neighbours, ~1.5 % of a config-2 step, profiles/r03_v8 kernel trace).
struct P1Ev {
  hipEvent_t start = nullptr, stop = nullptr;
};
template <typename K>
void p1_launch(K kernel, dim3 grid, dim3 block, hipStream_t s, const P1Ev &ev, const Pass1Args &a) {
  if (ev.start)
    hipExtLaunchKernelGGL(kernel, grid, block, 0, s, ev.start, ev.stop, 0, a);
  else
    hipLaunchKernelGGL(kernel, grid, block, 0, s, a);
}
#ifndef KBZ_PASS1D_D
#define KBZ_PASS1D_D 2
#endif
#ifndef KBZ_PASS1D_RING  // ring tiles of k_pass1d without ignore bytes / XXH64 (16 KiB each)
#define KBZ_PASS1D_RING 4
#endif
#ifndef KBZ_PASS1D_NX  // X waves of k_pass1d: 6 = 8 waves, 2 per SIMD (C and N alone on SIMD 0);
#define KBZ_PASS1D_NX 6  // 10 X waves with D = 1 (3 per SIMD): 3.72-3.77 vs 3.54 ms (r03_v7)
#endif
template <int MODE, bool IGN, bool X64>
void launch_pass1(int choice, const Pass1Args &a, uint32_t chunks, hipStream_t s, const P1Ev &ev) {
  if (MODE == KBZ_MODE_DYNAMORIO && pass1_is_wide(choice, chunks)) {
    constexpr int RING = (IGN && X64) ? 2 : (IGN || X64) ? 3 : KBZ_PASS1D_RING;
    constexpr int NW = KBZ_PASS1D_NX / 3 * 4;
    p1_launch(k_pass1d<IGN, X64, KBZ_PASS1D_NX, RING, KBZ_PASS1D_D>, dim3(chunks), dim3(64 * NW),
              s, ev, a);
  } else if (pass1_is_wide(choice, chunks))
    p1_launch(k_pass1w<MODE, IGN, X64, kWideNX, kWideNL, kWideD>, dim3(chunks),
              dim3(64 * (kWideNL + kWideNX)), s, ev, a);
  else
    p1_launch(k_pass1s<MODE, IGN, X64, KBZ_PASS1_DEPTH>, dim3(chunks), dim3(128), s, ev, a);
}

#ifndef KBZ_PASS1N_D  // register ring depth of k_pass1n, narrow (2 waves per chunk) / wide (8)
#define KBZ_PASS1N_D 2
#endif
#ifndef KBZ_PASS1N_WD
#define KBZ_PASS1N_WD 2
#endif
template <int MODE>
void launch_pass1n(int choice, const Pass1Args &a, uint32_t chunks, hipStream_t s, const P1Ev &ev) {
  if (pass1_is_wide(choice, chunks))
    p1_launch(k_pass1n<MODE, 8, KBZ_PASS1N_WD>, dim3(chunks), dim3(512), s, ev, a);
  else
    p1_launch(k_pass1n<MODE, 2, KBZ_PASS1N_D>, dim3(chunks), dim3(128), s, ev, a);
}

// hashed == false: an AFL-mode batch that wants neither hash (k_pass1n)
int pass1_dispatch(kbz_ctx *c, const Pass1Args &a, uint32_t chunks, bool x64, bool hashed,
                   hipStream_t s, const P1Ev &ev) {
  const bool ign = c->ignore != nullptr && c->mode == KBZ_MODE_DYNAMORIO;
  if (!hashed && c->mode == KBZ_MODE_AFL) {
    launch_pass1n<KBZ_MODE_AFL>(c->pass1, a, chunks, s, ev);
    HIP_TRY(hipGetLastError());
    return 0;
  }
  if (!hashed && c->mode == KBZ_MODE_AFL_CLASSIFY) {
    launch_pass1n<KBZ_MODE_AFL_CLASSIFY>(c->pass1, a, chunks, s, ev);
    HIP_TRY(hipGetLastError());
    return 0;
  }
  switch (c->mode) {
    case KBZ_MODE_AFL:
      x64 ? launch_pass1<KBZ_MODE_AFL, false, true>(c->pass1, a, chunks, s, ev)
          : launch_pass1<KBZ_MODE_AFL, false, false>(c->pass1, a, chunks, s, ev);
      break;
    case KBZ_MODE_AFL_CLASSIFY:
      x64 ? launch_pass1<KBZ_MODE_AFL_CLASSIFY, false, true>(c->pass1, a, chunks, s, ev)
          : launch_pass1<KBZ_MODE_AFL_CLASSIFY, false, false>(c->pass1, a, chunks, s, ev);
      break;
    default:
      if (ign)
        x64 ? launch_pass1<KBZ_MODE_DYNAMORIO, true, true>(c->pass1, a, chunks, s, ev)
            : launch_pass1<KBZ_MODE_DYNAMORIO, true, false>(c->pass1, a, chunks, s, ev);
      else
        x64 ? launch_pass1<KBZ_MODE_DYNAMORIO, false, true>(c->pass1, a, chunks, s, ev)
            : launch_pass1<KBZ_MODE_DYNAMORIO, false, false>(c->pass1, a, chunks, s, ev);
  }
  HIP_TRY(hipGetLastError());
  return 0;
}

// A caller that enables timing and never reads it must not grow the event pools without bound:
// past kEvFoldAt records the oldest ones are read (their end events waited for) and folded into
// running sums that the next kbz_ctx_time_* call reports with the rest.
constexpr size_t kEvFoldAt = 512;
int fold_pass1(kbz_ctx *c) {
  for (size_t i = 0; i < c->ev_used_n; i++) {
    HIP_TRY(hipEventSynchronize(c->ev_pass1[i].second));
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, c->ev_pass1[i].first, c->ev_pass1[i].second));
    c->pass1_folded_ms += ms;
  }
  c->pass1_folded_n += (uint32_t)c->ev_used_n;
  c->ev_used_n = 0;
  return 0;
}
int fold_stages(kbz_ctx *c) {
  for (const auto &r : c->stage_recs) {
    HIP_TRY(hipEventSynchronize(r.b));
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, r.a, r.b));
    c->stage_folded_ms[r.stage] += ms;
    c->stage_folded_nb += r.stage == KBZ_STAGE_SCAN;
  }
  c->stage_recs.clear();
  c->ev_pool_used = 0;
  return 0;
}
// Stage timing (kbz_ctx_time_stages): a start event now, the end event at stage_end.
int stage_begin(kbz_ctx *c, hipStream_t s, hipEvent_t *out) {
  *out = nullptr;
  if (!c->stage_timing) return 0;
  if (c->ev_pool_used + 2 > 2 * kEvFoldAt && fold_stages(c)) return -1;
  if (c->ev_pool_used + 2 > c->ev_pool.size()) {
    for (int i = 0; i < 2; i++) {
      hipEvent_t e;
      HIP_TRY(hipEventCreateWithFlags(&e, kEventScope));
      c->ev_pool.push_back(e);
    }
  }
  *out = c->ev_pool[c->ev_pool_used++];
  HIP_TRY(hipEventRecord(*out, s));
  return 0;
}
int stage_end(kbz_ctx *c, hipStream_t s, int stage, hipEvent_t a) {
  if (!a) return 0;
  hipEvent_t b = c->ev_pool[c->ev_pool_used++];
  HIP_TRY(hipEventRecord(b, s));
  c->stage_recs.push_back({stage, a, b});
  return 0;
}

int check_rows(const void *p, size_t stride, size_t M) {
  if (((uintptr_t)p & 15) || (stride & 15) || stride < M)
    return fail("traces must be 16-byte aligned with stride % 16 == 0 and stride >= map_size");
  if (stride > (1u << 25)) return fail("stride must be <= 32 MiB");
  return 0;
}

}  // namespace

extern "C" {

int kbz_abi_version(void) { return KBZ_ABI_VERSION; }
#ifndef KBZ_BUILD_FLAGS_STR  // set by killerbeez_amd/build.py: "" for the product library
#define KBZ_BUILD_FLAGS_STR "unrecorded: built outside killerbeez_amd/build.py"
#endif
const char *kbz_build_flags(void) { return KBZ_BUILD_FLAGS_STR; }
const char *kbz_last_error(void) { return g_err.c_str(); }

kbz_ctx_t *kbz_ctx_create(size_t map_size, int mode, size_t max_batch) {
  if (map_size < kTileW || map_size % kTileW || map_size > (1u << 24)) {
    fail("map_size must be a multiple of 256 in [256, 16 MiB]");
    return nullptr;
  }
  if (mode < 0 || mode > 2) {
    fail("bad mode");
    return nullptr;
  }
  if (max_batch == 0 || max_batch > (1ull << 31)) {
    fail("max_batch must be in [1, 2^31]");
    return nullptr;
  }
  kbz_ctx *c = new kbz_ctx();
  (void)hipGetDevice(&c->device);
  c->M = map_size;
  c->mode = mode;
  c->nc = mode_nclass(mode);
  c->max_batch = max_batch;
  c->max_chunks = cdiv(max_batch, kChunk);
  c->nfw = cdiv(map_size / kTileW, 64);
  if (const char *force = getenv("KBZ_PASS1"))
    c->pass1 = !strcmp(force, "wide") ? KBZ_PASS1_WIDE
               : !strcmp(force, "narrow") ? KBZ_PASS1_NARROW : KBZ_PASS1_AUTO;
  const size_t M = map_size, nc = c->nc;
  c->item_cap = (uint32_t)std::min<size_t>(kItemsPerCol * M * nc + 1024, 0xffffffffu);
  // tests only: a smaller claim list, to exercise the overflow error path (a real batch cannot
  // overflow it: each column yields at most 8 items per map per batch)
  if (const char *cap = getenv("KBZ_DEBUG_ITEM_CAP")) c->item_cap = std::max(1, atoi(cap));
  // tests only: force window items everywhere (1) or never (a large value)
  if (const char *w = getenv("KBZ_DEBUG_WIN_ITEMS")) c->win_items = (uint32_t)std::max(1, atoi(w));
  if (const char *w = getenv("KBZ_DEBUG_TAIL_INLINE_MAX")) c->inline_max = (uint32_t)std::max(0, atoi(w));
  // tests only: small AFL batches through the general pipeline instead of k_small
  if (const char *w = getenv("KBZ_DEBUG_NO_SMALL")) c->small_ok = atoi(w) == 0;
  // tests only: fused DynamoRIO batches through k_skip instead of k_pass1s's skip rule
  if (const char *w = getenv("KBZ_DEBUG_NO_FSKIP")) c->fskip_ok = atoi(w) == 0;
  if (const char *w = getenv("KBZ_DEBUG_LOOKBACK_SPIN")) c->spin_max = (uint32_t)strtoul(w, 0, 0);
  // tests only: one-shard batches through the staged kernels (k_chain ... k_pack) instead of k_tail
  if (const char *w = getenv("KBZ_DEBUG_STAGED")) c->fused_ok = atoi(w) == 0;
  // tests only: fused DynamoRIO batches without pass-1 claim records (k_tail reads the rows)
  if (const char *w = getenv("KBZ_DEBUG_NO_REC")) c->rec_ok = atoi(w) == 0;
  bool ok = !dalloc(&c->V[0], 3 * M) && !dalloc(&c->V[1], 3 * M) && !dalloc(&c->last, 2) &&
            !dalloc(&c->chunk_or, c->max_chunks * nc * M) && !dalloc(&c->chunk_cls, c->max_chunks) &&
            !dalloc(&c->tflags, c->max_chunks * nc * c->nfw) &&
            !dalloc(&c->flags, c->max_chunks) && !dalloc(&c->fix_list, c->max_chunks) &&
            !dalloc(&c->bad_list, max_batch) && !dalloc(&c->saved_row, 2 * M) &&
            !dalloc(&c->skip, max_batch) &&
            !dalloc(&c->neq, max_batch) && !dalloc(&c->h32, max_batch) &&
            !dalloc(&c->hnb32, max_batch) && !dalloc(&c->segor, kMaxSeg * nc * M) &&
            !dalloc(&c->segor_alt, kMaxSeg * nc * M) &&
            !dalloc(&c->tail, kTailFixDone + cdiv(M / 16, 256)) &&
            !dalloc(&c->segprev, kMaxSeg * nc * M) && !dalloc(&c->total, nc * M) &&
            !dalloc(&c->items, c->item_cap) && !dalloc(&c->counters, 16) &&
            !dalloc(&c->shard_last, 2) && !dalloc(&c->lastpub, c->max_chunks);
  if (!ok) {
    std::string e = g_err;
    free_ctx(c);
    g_err = e;
    return nullptr;
  }
  if (hipHostMalloc((void **)&c->h_err, 2 * sizeof(uint32_t), hipHostMallocMapped) != hipSuccess ||
      hipHostGetDevicePointer((void **)&c->d_err, c->h_err, 0) != hipSuccess) {
    fail("pinned error words");
    free_ctx(c);
    return nullptr;
  }
  c->h_err[0] = c->h_err[1] = 0;
  (void)hipMemset(c->V[0], 0xff, 3 * M);
  (void)hipMemset(c->last, 0, 2 * sizeof(uint32_t));
  (void)hipMemset(c->counters, 0, 16 * sizeof(uint32_t));
  (void)hipMemset(c->shard_last, 0, 2 * sizeof(uint32_t));
  (void)hipMemset(c->lastpub, 0, c->max_chunks * sizeof(uint64_t));
  // consumers re-zero these for the next batch (k_total: segor, k_pack: hnb32)
  (void)hipMemset(c->segor, 0, kMaxSeg * nc * M);
  (void)hipMemset(c->segor_alt, 0, kMaxSeg * nc * M);
  (void)hipMemset(c->tail, 0, (kTailFixDone + cdiv(M / 16, 256)) * sizeof(uint32_t));
  (void)hipMemset(c->items, 0, (size_t)c->item_cap * sizeof(uint64_t));  // zero between batches
  (void)hipMemset(c->hnb32, 0, max_batch * sizeof(uint32_t));
  (void)hipMemset(c->flags, 0, c->max_chunks * sizeof(uint32_t));
  if (hipDeviceSynchronize() != hipSuccess) {
    fail("device init failed");
    free_ctx(c);
    return nullptr;
  }
  return c;
}

void kbz_ctx_destroy(kbz_ctx_t *ctx) { free_ctx(ctx); }

int kbz_set_ignore(kbz_ctx_t *c, const uint8_t *host_ignore) {
  if (!c) return fail("null ctx");
  DevGuard g(c->device);
  if (!host_ignore) {
    if (c->ignore) (void)hipFree(c->ignore);
    c->ignore = nullptr;
    c->saved_valid = false;
    return 0;
  }
  if (!c->ignore && dalloc(&c->ignore, c->M)) return -1;
  HIP_TRY(hipMemcpy(c->ignore, host_ignore, c->M, hipMemcpyHostToDevice));
  c->saved_valid = false;  // "same content as the last exec" depended on the examined bytes
  return 0;
}

int kbz_get_virgin(kbz_ctx_t *c, uint8_t *out) {
  if (!c || !out) return fail("null argument");
  DevGuard g(c->device);
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(out, c->V[c->vcur], 3 * c->M, hipMemcpyDeviceToHost));
  return 0;
}
int kbz_set_virgin(kbz_ctx_t *c, const uint8_t *in) {
  if (!c || !in) return fail("null argument");
  DevGuard g(c->device);
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(c->V[c->vcur], in, 3 * c->M, hipMemcpyHostToDevice));
  // the saved last row's "clean" flag said its bits were in V; with new maps they may not be,
  // so a repeat of it in the next batch is checked like one after a restored hash
  c->saved_valid = false;
  return 0;
}
int kbz_reset_virgin(kbz_ctx_t *c, void *stream) {
  if (!c) return fail("null argument");
  DevGuard g(c->device);
  const hipStream_t s = (hipStream_t)stream;
  if (!c->ev_reset) {
    HIP_TRY(hipEventCreateWithFlags(&c->ev_reset, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&c->ev_prior, hipEventDisableTiming));
  }
  // a host batch or ring submit still queued on work_stream writes the buffer filled here (its
  // V' is the next batch's V): the fill comes after it
  if (c->work_stream && c->work_stream != s) {
    HIP_TRY(hipEventRecord(c->ev_prior, c->work_stream));
    HIP_TRY(hipStreamWaitEvent(s, c->ev_prior, 0));
  }
  // the buffer the next enqueued batch reads (vcur flips when a batch is enqueued)
  HIP_TRY(hipMemsetAsync(c->V[c->vcur], 0xff, 3 * c->M, s));
  HIP_TRY(hipEventRecord(c->ev_reset, s));
  c->reset_stream = s;
  c->reset_pending = true;  // the next batch's stream waits for the fill (shard_begin_impl)
  c->saved_valid = false;  // as kbz_set_virgin: the saved row's bits may not be in the new maps
  return 0;
}
int kbz_get_last_hash(kbz_ctx_t *c, uint32_t *out) {
  if (!c || !out) return fail("null argument");
  DevGuard g(c->device);
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(out, c->last + c->lcur, 4, hipMemcpyDeviceToHost));
  return 0;
}
int kbz_set_last_hash(kbz_ctx_t *c, uint32_t v) {
  if (!c) return fail("null ctx");
  DevGuard g(c->device);
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(c->last + c->lcur, &v, 4, hipMemcpyHostToDevice));
  c->saved_valid = false;  // a restored hash comes without its trace: row 0 is checked blind
  return 0;
}
int kbz_ctx_stats(kbz_ctx_t *c, uint32_t *out) {
  if (!c || !out) return fail("null argument");
  DevGuard g(c->device);
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(out, c->counters + 8, 3 * sizeof(uint32_t), hipMemcpyDeviceToHost));
  return 0;
}
int kbz_ctx_time_pass1(kbz_ctx_t *c, int enable, double *total_ms, uint32_t *launches) {
  if (!c) return fail("null ctx");
  DevGuard g(c->device);
  if (fold_pass1(c)) return -1;
  if (total_ms) *total_ms = c->pass1_folded_ms;
  if (launches) *launches = c->pass1_folded_n;
  c->pass1_folded_ms = 0;
  c->pass1_folded_n = 0;
  c->timing = enable != 0;
  return 0;
}
int kbz_ctx_time_pass1_every(kbz_ctx_t *c, uint32_t every) {
  if (!c) return fail("null ctx");
  if (every == 0) return fail("every must be >= 1");
  c->time_every = every;
  c->p1_launch_no = 0;
  return 0;
}
int kbz_ctx_time_stages(kbz_ctx_t *c, int enable, double *stage_ms, uint32_t *batches) {
  if (!c) return fail("null ctx");
  DevGuard g(c->device);
  if (fold_stages(c)) return -1;
  if (stage_ms)
    for (int i = 0; i < KBZ_NSTAGES; i++) stage_ms[i] = c->stage_folded_ms[i];
  if (batches) *batches = c->stage_folded_nb;
  for (int i = 0; i < KBZ_NSTAGES; i++) c->stage_folded_ms[i] = 0;
  c->stage_folded_nb = 0;
  c->stage_timing = enable != 0;
  return 0;
}
int kbz_ctx_set_pass1(kbz_ctx_t *c, int choice) {
  if (!c) return fail("null ctx");
  if (choice < KBZ_PASS1_AUTO || choice > KBZ_PASS1_WIDE) return fail("bad pass-1 choice");
  c->pass1 = choice;
  return 0;
}
uint8_t *kbz_virgin_device(kbz_ctx_t *c) { return c ? c->V[c->vcur] : nullptr; }

}  // extern "C"
namespace {
int fused_link(kbz_ctx *c, hipStream_t s, SkipExtra *x);
void fused_link_commit(kbz_ctx *c);
// kbz_reset_virgin's fill, queued on another stream, comes before the next batch on stream s
int wait_reset(kbz_ctx *c, hipStream_t s) {
  if (!c->reset_pending) return 0;
  if (c->reset_stream != s) HIP_TRY(hipStreamWaitEvent(s, c->ev_reset, 0));
  c->reset_pending = false;
  return 0;
}
// kbz_shard_begin; with `fused` (a one-shard batch of kbz_triage_batch_device) k_skip takes
// k_chain's row-0 and saved-row roles (the fused tail).
int shard_begin_impl(kbz_ctx *c, const uint8_t *traces, size_t n, size_t stride,
                     const int8_t *outcome, uint32_t *h32_out, uint64_t *x64_out, int want,
                     void *stream, bool fused) {
  if (!c) return fail("null ctx");
  if (n > c->max_batch) return fail("n exceeds max_batch");
  if (n && check_rows(traces, stride, c->M)) return -1;
  DevGuard g(c->device);
  hipStream_t s = (hipStream_t)stream;
  if (wait_reset(c, s)) return -1;
  if (c->stage != 0) {
    // the previous batch was abandoned between stages (e.g. a collective failed): re-arm what
    // its later kernels would have reset -- the per-batch counters, fix-list flags, the shard's
    // last-hash pair, the per-trace results and the segment aggregates
    HIP_TRY(hipMemsetAsync(c->counters, 0, sizeof(uint32_t), s));  // [1..2] stay sticky
    HIP_TRY(hipMemsetAsync(c->counters + 3, 0, 3 * sizeof(uint32_t), s));
    HIP_TRY(hipMemsetAsync(c->flags, 0, c->max_chunks * sizeof(uint32_t), s));
    HIP_TRY(hipMemsetAsync(c->shard_last, 0, 2 * sizeof(uint32_t), s));
    HIP_TRY(hipMemsetAsync(c->hnb32, 0, c->max_batch * sizeof(uint32_t), s));
    HIP_TRY(hipMemsetAsync(c->segor, 0, kMaxSeg * c->nc * c->M, s));
    HIP_TRY(hipMemsetAsync(c->segor_alt, 0, kMaxSeg * c->nc * c->M, s));
    // kbz_shard_link may already have marked this batch's last row as the next row-0
    // predecessor, but V never received that batch: forget the row
    c->saved_valid = false;
    c->shard_keep = false;
    c->stage = 0;
  }
  c->cur_traces = traces;
  c->cur_n = n;
  c->cur_stride = stride;
  c->cur_outcome = outcome;
  c->cur_h32_out = h32_out;
  c->cur_chunks = cdiv(n, kChunk);
  c->cur_nseg = std::max(1u, std::min<unsigned>(kMaxSeg, c->cur_chunks));
  c->cur_seg_len = std::max(1u, cdiv(c->cur_chunks, c->cur_nseg));
  c->cur_nseg = std::max(1u, cdiv(c->cur_chunks, c->cur_seg_len));
  c->fix_pending = false;
  // counters[0], counters[3], flags and shard_last are zero here: k_pack of the previous
  // batch (or context creation) re-armed them
  if (n == 0) {
    c->stage = 1;
    return 0;
  }
  Pass1Args a{};
  a.traces = traces;
  a.stride = stride;
  a.n = (uint32_t)n;
  a.map_size = (uint32_t)c->M;
  a.outcome = outcome;
  a.ignore = c->ignore;
  a.x64 = (want & KBZ_WANT_X64) ? x64_out : nullptr;
  // AFL modes hash only on request (the reference AFL plugin never hashes); DynamoRIO always
  // does (the last-hash skip)
  const bool hashed = c->mode == KBZ_MODE_DYNAMORIO || (want & KBZ_WANT_H32) || a.x64 || h32_out;
  a.h32 = !hashed ? nullptr : h32_out ? h32_out : c->h32;  // straight to the caller's buffer
  c->cur_h32 = a.h32;
  c->cur_h32_out = hashed ? h32_out : nullptr;
  a.neq = c->neq;
  a.chunk_or = c->chunk_or;
  a.chunk_cls = c->chunk_cls;
  a.shard_last = c->shard_last;
  a.segor = c->segor;
  a.seg_len = c->cur_seg_len;
  a.vcur = c->V[c->vcur];
  a.tflags = c->tflags;
  a.nfw = c->nfw;
  a.frec = nullptr;
  a.rflags = nullptr;
  a.epoch = 0;
  c->cur_rec = false;
  // DynamoRIO batches through k_pass1s without ignore bytes or XXH64 (one-shard batches and
  // shards): claim records.  A shard's row 0 is linked later (k_chain), but a record never needs
  // it: a row 0 that repeats its predecessor holds only bits of the prefix (the earlier shards'
  // aggregate holds the predecessor's), so it is never a claim's first holder, and a row 0 that
  // differs (a collision) puts its chunk on the fix list, whose claims read the rows.
  if (c->rec_ok && p1s_records(c->mode, c->ignore != nullptr, a.x64 != nullptr) &&
      !pass1_is_wide(c->pass1, c->cur_chunks)) {
    if (!c->frec) {
      const size_t bytes = (size_t)c->max_chunks * c->M * sizeof(uint64_t);
      if (hipMalloc((void **)&c->frec, bytes) != hipSuccess ||
          hipMalloc((void **)&c->rflags, (size_t)c->max_chunks * c->nfw * sizeof(uint64_t)) !=
              hipSuccess) {
        (void)hipGetLastError();
        if (c->frec) (void)hipFree(c->frec);
        c->frec = nullptr;
        c->rflags = nullptr;
        c->rec_ok = false;  // no room: k_tail reads the rows instead
      } else if (hipMemsetAsync(c->rflags, 0, (size_t)c->max_chunks * c->nfw * sizeof(uint64_t),
                                s) != hipSuccess) {
        return fail("hipMemsetAsync of the record flags failed");
      }
    }
    if (c->frec) {
      c->epoch = c->epoch % kRecEpochMask + 1;
      a.frec = c->frec;
      a.rflags = c->rflags;
      a.epoch = c->epoch;
      c->cur_rec = true;
    }
  }
  P1Ev pev;
  if (c->timing && (c->p1_launch_no++ % c->time_every) == 0) {
    if (c->ev_used_n >= kEvFoldAt && fold_pass1(c)) return -1;
    if (c->ev_used_n == c->ev_pass1.size()) {
      std::pair<hipEvent_t, hipEvent_t> e;
      // device-scope release: the default system-scope fence adds ~13 us per batch on MI355X
      // (same-box A/B, profiles/r02_v9)
      HIP_TRY(hipEventCreateWithFlags(&e.first, kEventScope));
      HIP_TRY(hipEventCreateWithFlags(&e.second, kEventScope));
      c->ev_pass1.push_back(e);
    }
    pev.start = c->ev_pass1[c->ev_used_n].first;
    pev.stop = c->ev_pass1[c->ev_used_n++].second;
  }
  // DynamoRIO: pass 1's stop event is the start of k_skip, its successor on the stream (a stop
  // event on pass 1's own dispatch left 4.8 us of idle GPU after it, profiles/r05_evgap; the
  // interval now also holds the boundary, so the pass-1 time is an upper bound)
  // a fused DynamoRIO batch through k_pass1s: the kernel runs k_skip's rule itself (its row-0 and
  // saved-row roles included); the copy of the last row into the context goes to k_tail
  const bool fsk = c->mode == KBZ_MODE_DYNAMORIO && c->fskip_ok &&
                   !pass1_is_wide(c->pass1, c->cur_chunks);
  // (no k_skip launch when pass 1 runs the rule itself: the stop event stays on pass 1)
  const bool stop_on_skip =
      pev.start && c->mode == KBZ_MODE_DYNAMORIO && KBZ_P1_STOP_ON_NEXT && !fsk;
  P1Ev pev1 = pev;
  if (stop_on_skip) pev1.stop = nullptr;
  c->tail_copy_src = nullptr;
  c->tail_copy_dst = nullptr;
  if (fsk) {  // (a shard of the sharded protocol: rows j >= 1 only, k_chain links row 0)
    SkipExtra x{};
    if (fused && fused_link(c, s, &x)) return -1;
    c->skip_tag = c->skip_tag + 1 ? c->skip_tag + 1 : 1;
    a.skip = c->skip;
    a.fix_flags = c->flags;
    a.fix_list = c->fix_list;
    a.fix_cnt = c->counters + 3;
    a.bad_list = c->bad_list;
    a.bad_cnt = c->counters + 4;
    a.lastpub = c->lastpub;
    a.tag = c->skip_tag;
    a.row0_hp = x.row0_hp;
    a.pred_saved = x.pred_saved;
    a.pred_ok = x.pred_ok;
    a.prow = x.prow;
    a.bad0 = x.bad0;
    a.err = c->counters + 2;
    a.spin_max = c->spin_max;
    c->tail_copy_src = x.copy_src;
    c->tail_copy_dst = x.copy_dst;
  }
  if (pass1_dispatch(c, a, c->cur_chunks, a.x64 != nullptr, hashed, s, pev1)) return -1;
  if (fsk) {
    if (fused) fused_link_commit(c);  // pass 1 is queued: this batch's row is the next predecessor
  } else if (c->mode == KBZ_MODE_DYNAMORIO) {  // the skip rule for rows j >= 1 needs no other shard
    hipEvent_t st0;
    if (stage_begin(c, s, &st0)) return -1;
    const unsigned row_blocks = cdiv(n, 256);
    SkipExtra x{};
    unsigned extra = 0;
    if (fused) {  // + row 0 and the saved-row copy (k_chain's jobs in the staged pipeline)
      if (fused_link(c, s, &x)) return -1;
      extra = 1 + x.copy_blocks;
    }
    hipExtLaunchKernelGGL(k_skip, dim3(row_blocks + c->cur_chunks - 1 + extra), dim3(256), 0, s,
                          stop_on_skip ? pev.stop : nullptr, nullptr, 0, c->cur_h32, c->neq,
                          (uint32_t)n, c->skip, c->flags, c->fix_list, c->counters + 3,
                          c->bad_list, c->counters + 4, c->shard_last, traces, stride, c->ignore,
                          (uint32_t)c->M, row_blocks, x);
    HIP_TRY(hipGetLastError());
    if (fused) fused_link_commit(c);  // k_skip is queued: this batch's row is the next predecessor
    if (stage_end(c, s, KBZ_STAGE_SKIP, st0)) return -1;
  }
  c->stage = 1;
  return 0;
}

// The row-0 / saved-row arguments of a fused batch's k_skip and the context's chain bookkeeping
// (kbz_shard_link for a one-shard batch): row 0's predecessor is the saved row (clean iff its
// flag), the batch's last row becomes the next batch's predecessor (the other saved slot), the
// next last hash goes to the other last-hash word; k_tail writes those two words.
// fused_link only fills the arguments (and the chain words k_tail gets, kept in the context);
// the context's saved-row / last-hash slots flip once k_skip is launched (fused_link_commit).
int fused_link(kbz_ctx *c, hipStream_t, SkipExtra *x) {
  const size_t M = c->M, n = c->cur_n;
  x->row0_hp = c->last + c->lcur;
  x->pred_saved = c->saved_valid ? 1 : 0;
  x->pred_ok = c->counters + 6 + c->srow;
  x->prow = c->saved_row + c->srow * M;
  x->bad0 = c->tail + 4;
  x->copy_src = c->cur_traces + (n - 1) * c->cur_stride;
  x->copy_dst = c->saved_row + (c->srow ^ 1) * M;
  x->copy_blocks = std::min(64u, cdiv(M / 16, 256));
  c->fchain_ctx_last = c->last + c->lcur;
  c->fchain_next_last = c->last + (c->lcur ^ 1);
  c->fchain_saved_ok = c->counters + 6 + (c->srow ^ 1);
  return 0;
}
void fused_link_commit(kbz_ctx *c) {
  c->srow ^= 1;
  c->saved_valid = true;
  c->lcur ^= 1;
}

// Everything after pass 1 (and k_skip) of a one-shard batch in one launch: k_tail.
int fused_tail(kbz_ctx *c, uint8_t *hnb_out, hipStream_t s) {
  const bool dr = c->mode == KBZ_MODE_DYNAMORIO;
  const uint32_t n = (uint32_t)c->cur_n, M = (uint32_t)c->M;
  const uint8_t *ign = dr ? c->ignore : nullptr;
  const uint8_t *skip = dr ? c->skip : nullptr;
  const int vn = c->vcur ^ 1;
  TailArgs a{};
  a.ca = ClaimArgs{c->cur_traces, c->cur_stride, n, c->mode, c->cur_outcome, skip, c->hnb32,
                   c->counters + 2};
  a.ra = ResolveArgs{c->cur_traces, c->cur_stride, n, c->mode, c->cur_outcome, skip, c->hnb32,
                     c->counters + 2, c->chunk_or, c->nc, M, c->V[c->vcur], ign};
  a.fx = FixArgs{c->cur_traces, c->cur_stride, n, c->skip, c->fix_list, c->counters + 3,
                 c->chunk_or, c->chunk_cls, c->cur_chunks, c->cur_seg_len, c->flags, c->tflags,
                 c->nfw};
  a.chunk_or = c->chunk_or;
  a.chunk_cls = c->chunk_cls;
  a.nchunks = c->cur_chunks;
  a.seg_len = c->cur_seg_len;
  a.nseg = c->cur_nseg;
  a.nclass = c->nc;
  a.map_size = M;
  a.segor = c->segor;
  a.segor_next = c->segor_alt;
  a.vcur = c->V[c->vcur];
  a.vnext = c->V[vn];
  a.ignore = ign;
  a.items = c->items;
  a.cap = c->item_cap;
  a.counters = c->counters;
  a.tflags = c->tflags;
  a.nfw = c->nfw;
  a.listed = dr ? c->flags : nullptr;
  a.win_items = c->win_items;
  a.inline_max = c->inline_max;
  a.tail = c->tail;
  a.frec = c->cur_rec ? c->frec : nullptr;
  a.rflags = c->rflags;
  a.epoch = c->epoch;
  a.shard_last = c->shard_last;
  a.neq = c->neq;
  a.bad_list = c->bad_list;
  a.ctx_last = c->fchain_ctx_last;
  a.next_last = c->fchain_next_last;
  a.saved_ok = c->fchain_saved_ok;
  a.flags_w = c->flags;
  a.fix_list_w = c->fix_list;
  a.fix_cnt_w = c->counters + 3;
  a.copy_src = c->tail_copy_src;
  a.copy_dst = c->tail_copy_dst;
  hipEvent_t st0;
  if (stage_begin(c, s, &st0)) return -1;
  const unsigned ncg = cdiv(M / 16, 256);
  hipLaunchKernelGGL(k_tail, dim3(ncg, c->cur_nseg, c->nc), dim3(256), 0, s, a);
  HIP_TRY(hipGetLastError());
  if (stage_end(c, s, KBZ_STAGE_SCAN, st0)) return -1;
  FinArgs f{};
  f.ra = a.ra;
  f.items = c->items;
  f.cap = c->item_cap;
  f.counters = c->counters;
  f.tail = c->tail;
  f.tail_fix_words = ncg;
  f.hnb_out = hnb_out;
  f.err_out = c->d_err;
  f.shard_last = c->shard_last;
  f.flags_w = c->flags;
  f.fix_list_w = c->fix_list;
  f.fix_cnt = dr ? c->counters + 3 : nullptr;
  f.nchunks = c->cur_chunks;
  if (stage_begin(c, s, &st0)) return -1;
  hipLaunchKernelGGL(k_fin, dim3(KBZ_FIN_GRID), dim3(256), 0, s, f);
  HIP_TRY(hipGetLastError());
  if (stage_end(c, s, KBZ_STAGE_RESOLVE, st0)) return -1;
  std::swap(c->segor, c->segor_alt);
  c->vcur = vn;
  c->stage = 0;
  return 0;
}
}  // namespace
extern "C" {

int kbz_shard_begin(kbz_ctx_t *c, const uint8_t *traces, size_t n, size_t stride,
                    const int8_t *outcome, uint32_t *h32_out, uint64_t *x64_out, int want,
                    void *stream) {
  return shard_begin_impl(c, traces, n, stride, outcome, h32_out, x64_out, want, stream, false);
}

int kbz_shard_last_hash(kbz_ctx_t *c, uint32_t *d_out, void *stream) {
  if (!c || !d_out) return fail("null argument");
  if (c->stage < 1) return fail("kbz_shard_last_hash: call kbz_shard_begin first");
  DevGuard g(c->device);
  HIP_TRY(hipMemcpyAsync(d_out, c->shard_last, 2 * sizeof(uint32_t), hipMemcpyDeviceToDevice,
                         (hipStream_t)stream));
  return 0;
}

int kbz_shard_last_row(kbz_ctx_t *c, uint8_t *d_out, void *stream) {
  if (!c || !d_out) return fail("null argument");
  if (c->stage < 1) return fail("kbz_shard_last_row: call kbz_shard_begin first");
  if (c->cur_n == 0) return 0;  // an empty shard has no last row (its pair says so)
  DevGuard g(c->device);
  HIP_TRY(hipMemcpyAsync(d_out, c->cur_traces + (c->cur_n - 1) * c->cur_stride, c->M,
                         hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return 0;
}

int kbz_shard_link(kbz_ctx_t *c, const uint32_t *prev_last, const uint8_t *prev_row,
                   int is_first, const uint32_t *global_last, const uint8_t *global_row,
                   void *stream) {
  if (!c || c->stage != 1) return fail("kbz_shard_link: call kbz_shard_begin first");
  DevGuard g(c->device);
  hipStream_t s = (hipStream_t)stream;
  if (c->mode == KBZ_MODE_DYNAMORIO) {
    const size_t n = c->cur_n, M = c->M;
    const int nl = c->lcur ^ 1;
    ChainArgs a{};
    a.n = (uint32_t)n;
    a.h32 = c->cur_h32;
    a.skip = c->skip;
    a.neq = c->neq;
    a.bad_list = c->bad_list;
    a.bad_cnt = c->counters + 4;
    a.flags = c->flags;
    a.fix_list = c->fix_list;
    a.fix_cnt = c->counters + 3;
    a.prev_last = is_first ? nullptr : prev_last;
    a.ctx_last = c->last + c->lcur;
    a.global_last = global_last ? global_last : c->shard_last;
    a.next_last = c->last + nl;
    // row 0's predecessor: the previous batch's last row (first shard) or the previous
    // non-empty shard's last row; unknown or unclean -> row 0 counts as differing if skipped
    if (is_first) {
      a.pred_kind = c->saved_valid ? PRED_SAVED : PRED_UNKNOWN;
      a.pred_ok = c->counters + 6 + c->srow;
      a.prow = c->saved_row + c->srow * M;
    } else {
      a.pred_kind = (prev_row && prev_last) ? PRED_PAIR : PRED_UNKNOWN;
      a.pred_ok = prev_last ? prev_last + 1 : nullptr;
      a.prow = prev_row;
    }
    a.row0 = c->cur_traces;
    a.ignore = c->ignore;
    a.map_size = (uint32_t)M;
    a.shard_flags = c->shard_last + 1;
    // the batch's last row becomes the next batch's row-0 predecessor: the caller's global row
    // (sharded), else this shard's own last row (a single-shard batch; an empty one keeps the
    // old row).  It goes to the other saved slot: block 0 may still read the current one.
    a.single = !global_row && !global_last;
    a.copy_src = global_row ? global_row
                 : (a.single && n) ? c->cur_traces + (n - 1) * c->cur_stride : nullptr;
    a.copy_dst = c->saved_row + (c->srow ^ 1) * M;
    a.saved_ok = c->counters + 6 + (c->srow ^ 1);
    const unsigned copy_blocks = a.copy_src ? std::min(64u, cdiv(M / 16, 256)) : 0;
    hipEvent_t st0;
    if (stage_begin(c, s, &st0)) return -1;
    hipLaunchKernelGGL(k_chain, dim3(1 + copy_blocks), dim3(256), 0, s, a);
    HIP_TRY(hipGetLastError());
    if (stage_end(c, s, KBZ_STAGE_LINK, st0)) return -1;
    if (a.copy_src) {
      c->srow ^= 1;
      c->saved_valid = true;
    } else if (!a.single) {
      c->saved_valid = false;  // sharded without the last row: forget it
    }
    c->lcur = nl;
    c->fix_pending = n != 0;  // k_total runs the (usually empty) fix path
  }
  c->stage = 2;
  return 0;
}

int kbz_shard_reduce(kbz_ctx_t *c, void *stream) {
  if (!c || c->stage != 2) return fail("kbz_shard_reduce: call kbz_shard_link first");
  DevGuard g(c->device);
  hipStream_t s = (hipStream_t)stream;
  c->shard_keep = false;
  if (c->cur_n == 0) {
    HIP_TRY(hipMemsetAsync(c->total, 0, c->nc * c->M, s));
    HIP_TRY(hipMemsetAsync(c->segprev, 0, c->nc * c->M, s));
  } else {
    FixArgs fx{};
    if (c->fix_pending) {
      fx.traces = c->cur_traces;
      fx.stride = c->cur_stride;
      fx.n = (uint32_t)c->cur_n;
      fx.skip = c->skip;
      fx.fix_list = c->fix_list;
      fx.fix_cnt = c->counters + 3;
      fx.chunk_or = c->chunk_or;
      fx.chunk_cls = c->chunk_cls;
      fx.nchunks = c->cur_chunks;
      fx.seg_len = c->cur_seg_len;
      fx.listed = c->flags;
      fx.tflags = c->tflags;
      fx.nfw = c->nfw;
    }
    hipEvent_t st0;
    if (stage_begin(c, s, &st0)) return -1;
    hipLaunchKernelGGL(k_total<false>, dim3(cdiv(c->M / 8, 256), 1, c->nc), dim3(256), 0, s, c->segor,
                       c->cur_nseg, c->nc, (uint32_t)c->M, c->segprev, c->total, fx);
    HIP_TRY(hipGetLastError());
    if (stage_end(c, s, KBZ_STAGE_REDUCE, st0)) return -1;
  }
  c->stage = 3;
  return 0;
}

int kbz_shard_aggregate(kbz_ctx_t *c, uint8_t *d_out, void *stream) {
  if (!c || !d_out) return fail("null argument");
  if (c->stage != 3) return fail("kbz_shard_aggregate: call kbz_shard_reduce first");
  DevGuard g(c->device);
  HIP_TRY(hipMemcpyAsync(d_out, c->total, c->nc * c->M, hipMemcpyDeviceToDevice,
                         (hipStream_t)stream));
  return 0;
}
size_t kbz_shard_aggregate_bytes(kbz_ctx_t *c) { return c ? c->nc * c->M : 0; }

int kbz_shard_finish(kbz_ctx_t *c, const uint8_t *prefix, const uint8_t *total, uint8_t *hnb_out,
                     void *stream) {
  if (!c || c->stage != 3) return fail("kbz_shard_finish: call kbz_shard_reduce first");
  if (c->shard_keep) return fail("kbz_shard_finish: after kbz_shard_reduce_into, finish with "
                                 "kbz_shard_finish_gathered");
  if (!total) total = c->total;  // single shard: its own aggregate is the total
  DevGuard g(c->device);
  hipStream_t s = (hipStream_t)stream;
  const unsigned gx = cdiv(c->M / 16, 256);
  const int vn = c->vcur ^ 1;
  const uint8_t *ign = (c->mode == KBZ_MODE_DYNAMORIO) ? c->ignore : nullptr;
  const uint32_t nseg = c->cur_n ? c->cur_nseg : 1;
  hipEvent_t st0;
  if (stage_begin(c, s, &st0)) return -1;
  hipLaunchKernelGGL(k_scan, dim3(gx, nseg, c->nc), dim3(256), 0, s, c->chunk_or, c->chunk_cls,
                     c->cur_chunks, c->cur_seg_len, c->nc, (uint32_t)c->M, c->segprev, nseg,
                     c->total, prefix, total, c->V[c->vcur], c->V[vn], ign, c->items,
                     c->item_cap, c->counters, c->tflags, c->nfw,
                     c->mode == KBZ_MODE_DYNAMORIO ? c->flags : nullptr, c->win_items,
                     ClaimArgs{c->cur_traces, c->cur_stride, (uint32_t)c->cur_n, c->mode,
                               c->cur_outcome, c->mode == KBZ_MODE_DYNAMORIO ? c->skip : nullptr,
                               c->hnb32, c->counters + 2});
  HIP_TRY(hipGetLastError());
  if (stage_end(c, s, KBZ_STAGE_SCAN, st0)) return -1;
  if (c->cur_n) {
    if (stage_begin(c, s, &st0)) return -1;
    hipLaunchKernelGGL(k_resolve, dim3(512), dim3(256), 0, s,
                       ResolveArgs{c->cur_traces, c->cur_stride, (uint32_t)c->cur_n, c->mode,
                                   c->cur_outcome, c->mode == KBZ_MODE_DYNAMORIO ? c->skip : nullptr,
                                   c->hnb32, c->counters + 2, c->chunk_or, c->nc, (uint32_t)c->M,
                                   c->V[c->vcur], ign},
                       c->items, c->counters, c->item_cap);
    HIP_TRY(hipGetLastError());
    if (stage_end(c, s, KBZ_STAGE_RESOLVE, st0)) return -1;
    if (stage_begin(c, s, &st0)) return -1;
    hipLaunchKernelGGL(k_pack, dim3(cdiv(c->cur_n, 256)), dim3(256), 0, s, c->hnb32, c->cur_h32,
                       (uint32_t)c->cur_n, hnb_out ? hnb_out : (uint8_t *)nullptr,
                       (c->cur_h32_out && c->cur_h32_out != c->cur_h32) ? c->cur_h32_out : nullptr,
                       c->counters, c->mode == KBZ_MODE_DYNAMORIO ? c->flags : nullptr,
                       c->cur_chunks, c->shard_last, c->d_err);
    HIP_TRY(hipGetLastError());
    if (stage_end(c, s, KBZ_STAGE_PACK, st0)) return -1;
  } else {
    // empty shard: k_skip may still have written the fix count / shard pair; re-arm them
    HIP_TRY(hipMemsetAsync(c->counters + 3, 0, 3 * sizeof(uint32_t), s));
    HIP_TRY(hipMemsetAsync(c->shard_last, 0, 2 * sizeof(uint32_t), s));
  }
  c->vcur = vn;
  c->stage = 0;
  return 0;
}

int kbz_shard_exchange_row(kbz_ctx_t *c, uint8_t *d_out, void *stream) {
  if (!c || !d_out) return fail("null argument");
  if (c->stage < 1) return fail("kbz_shard_exchange_row: call kbz_shard_begin first");
  if (((uintptr_t)d_out | c->M) & 15) return fail("kbz_shard_exchange_row: d_out must be 16-B aligned");
  DevGuard g(c->device);
  const uint8_t *row = c->cur_n ? c->cur_traces + (c->cur_n - 1) * c->cur_stride : nullptr;
  hipLaunchKernelGGL(k_exch, dim3(cdiv(c->M / 16, 256)), dim3(256), 0, (hipStream_t)stream, row,
                     (uint32_t)c->M, c->shard_last, d_out);
  HIP_TRY(hipGetLastError());
  return 0;
}

int kbz_shard_reduce_into(kbz_ctx_t *c, uint8_t *d_aggregate, void *stream) {
  if (!c || !d_aggregate) return fail("null argument");
  if (c->stage != 2) return fail("kbz_shard_reduce_into: call kbz_shard_link first");
  if ((uintptr_t)d_aggregate & 7) return fail("kbz_shard_reduce_into: d_aggregate must be 8-B aligned");
  DevGuard g(c->device);
  hipStream_t s = (hipStream_t)stream;
  if (c->cur_n == 0) {
    HIP_TRY(hipMemsetAsync(d_aggregate, 0, c->nc * c->M, s));
  } else {
    FixArgs fx{};
    if (c->fix_pending) {
      fx.traces = c->cur_traces;
      fx.stride = c->cur_stride;
      fx.n = (uint32_t)c->cur_n;
      fx.skip = c->skip;
      fx.fix_list = c->fix_list;
      fx.fix_cnt = c->counters + 3;
      fx.chunk_or = c->chunk_or;
      fx.chunk_cls = c->chunk_cls;
      fx.nchunks = c->cur_chunks;
      fx.seg_len = c->cur_seg_len;
      fx.listed = c->flags;
      fx.tflags = c->tflags;
      fx.nfw = c->nfw;
    }
    hipEvent_t st0;
    if (stage_begin(c, s, &st0)) return -1;
    hipLaunchKernelGGL(k_total<true>, dim3(cdiv(c->M / 8, 256), 1, c->nc), dim3(256), 0, s,
                       c->segor, c->cur_nseg, c->nc, (uint32_t)c->M, nullptr, d_aggregate, fx);
    HIP_TRY(hipGetLastError());
    if (stage_end(c, s, KBZ_STAGE_REDUCE, st0)) return -1;
  }
  c->shard_keep = true;
  c->stage = 3;
  return 0;
}

int kbz_shard_finish_gathered(kbz_ctx_t *c, const uint8_t *d_gathered, size_t rank, size_t world,
                              uint8_t *hnb_out, void *stream) {
  if (!c || !d_gathered) return fail("null argument");
  if (c->stage != 3 || !c->shard_keep)
    return fail("kbz_shard_finish_gathered: call kbz_shard_reduce_into first");
  if (world == 0 || rank >= world) return fail("kbz_shard_finish_gathered: rank >= world");
  if (((uintptr_t)d_gathered | (c->nc * c->M)) & 15)
    return fail("kbz_shard_finish_gathered: d_gathered must be 16-B aligned");
  DevGuard g(c->device);
  hipStream_t s = (hipStream_t)stream;
  const bool dr = c->mode == KBZ_MODE_DYNAMORIO;
  const uint32_t n = (uint32_t)c->cur_n, M = (uint32_t)c->M;
  const uint8_t *ign = dr ? c->ignore : nullptr;
  const uint8_t *skip = dr ? c->skip : nullptr;
  const int vn = c->vcur ^ 1;
  TailArgs a{};
  a.ca = ClaimArgs{c->cur_traces, c->cur_stride, n, c->mode, c->cur_outcome, skip, c->hnb32,
                   c->counters + 2};
  a.ra = ResolveArgs{c->cur_traces, c->cur_stride, n, c->mode, c->cur_outcome, skip, c->hnb32,
                     c->counters + 2, c->chunk_or, c->nc, M, c->V[c->vcur], ign};
  a.fx = FixArgs{c->cur_traces, c->cur_stride, n, c->skip, c->fix_list, c->counters + 3,
                 c->chunk_or, c->chunk_cls, c->cur_chunks, c->cur_seg_len, c->flags, c->tflags,
                 c->nfw};
  a.chunk_or = c->chunk_or;
  a.chunk_cls = c->chunk_cls;
  a.nchunks = c->cur_chunks;
  a.seg_len = c->cur_seg_len;
  a.nseg = c->cur_nseg;
  a.nclass = c->nc;
  a.map_size = M;
  a.segor = c->segor;
  a.segor_next = c->segor_alt;
  a.vcur = c->V[c->vcur];
  a.vnext = c->V[vn];
  a.ignore = ign;
  a.items = c->items;
  a.cap = c->item_cap;
  a.counters = c->counters;
  a.tflags = c->tflags;
  a.nfw = c->nfw;
  a.listed = dr ? c->flags : nullptr;
  a.win_items = c->win_items;
  a.inline_max = c->inline_max;
  a.tail = c->tail;
  a.frec = c->cur_rec ? c->frec : nullptr;  // pass 1's claim records (see shard_begin_impl)
  a.rflags = c->rflags;
  a.epoch = c->epoch;
  a.shard_last = c->shard_last;
  a.neq = c->neq;
  a.bad_list = c->bad_list;
  a.flags_w = c->flags;
  a.fix_list_w = c->fix_list;
  a.fix_cnt_w = c->counters + 3;
  a.shard = 1;
  a.gathered = d_gathered;
  a.rank = (uint32_t)rank;
  a.world = (uint32_t)world;
  hipEvent_t st0;
  if (stage_begin(c, s, &st0)) return -1;
  const unsigned ncg = cdiv(M / 16, 256);
  hipLaunchKernelGGL(k_tail, dim3(ncg, c->cur_nseg, c->nc), dim3(256), 0, s, a);
  HIP_TRY(hipGetLastError());
  if (stage_end(c, s, KBZ_STAGE_SCAN, st0)) return -1;
  FinArgs f{};
  f.ra = a.ra;
  f.items = c->items;
  f.cap = c->item_cap;
  f.counters = c->counters;
  f.tail = c->tail;
  f.tail_fix_words = ncg;
  f.hnb_out = hnb_out;
  f.err_out = c->d_err;
  f.shard_last = c->shard_last;
  f.flags_w = c->flags;
  f.fix_list_w = c->fix_list;
  f.fix_cnt = dr ? c->counters + 3 : nullptr;
  f.nchunks = c->cur_chunks;
  if (stage_begin(c, s, &st0)) return -1;
  hipLaunchKernelGGL(k_fin, dim3(KBZ_FIN_GRID), dim3(256), 0, s, f);
  HIP_TRY(hipGetLastError());
  if (stage_end(c, s, KBZ_STAGE_RESOLVE, st0)) return -1;
  std::swap(c->segor, c->segor_alt);
  c->vcur = vn;
  c->shard_keep = false;
  c->stage = 0;
  return 0;
}

int kbz_triage_batch_device(kbz_ctx_t *c, const uint8_t *traces, size_t n, size_t stride,
                            const int8_t *outcome, uint8_t *hnb_out, uint32_t *h32_out,
                            uint64_t *x64_out, int want, void *stream) {
  // AFL modes, no hash, at most 64 execs (the AFL plugin's per-exec flushes): one launch
  if (c && c->small_ok && c->mode != KBZ_MODE_DYNAMORIO && n && n <= kSmallRows && c->stage == 0 &&
      !h32_out && !(want & (KBZ_WANT_H32 | KBZ_WANT_X64))) {
    if (check_rows(traces, stride, c->M)) return -1;
    if (n > c->max_batch) return fail("n exceeds max_batch");
    DevGuard g(c->device);
    if (wait_reset(c, (hipStream_t)stream)) return -1;
    const int vn = c->vcur ^ 1;
    SmallArgs a{traces, stride, (uint32_t)n, (uint32_t)c->M, outcome, c->V[c->vcur], c->V[vn],
                c->hnb32, hnb_out, c->counters + 12, c->counters + 8};
    const dim3 grid(cdiv(c->M / 16, KBZ_SMALL_TPB));
    if (c->mode == KBZ_MODE_AFL)
      hipLaunchKernelGGL(k_small<KBZ_MODE_AFL>, grid, dim3(KBZ_SMALL_TPB), 0, (hipStream_t)stream, a);
    else
      hipLaunchKernelGGL(k_small<KBZ_MODE_AFL_CLASSIFY>, grid, dim3(KBZ_SMALL_TPB), 0,
                         (hipStream_t)stream, a);
    HIP_TRY(hipGetLastError());
    c->vcur = vn;
    return 0;
  }
  if (c && c->fused_ok && n && c->stage == 0) {  // one shard: pass 1, [k_skip], k_tail
    if (shard_begin_impl(c, traces, n, stride, outcome, h32_out, x64_out, want, stream, true))
      return -1;
    DevGuard g(c->device);
    return fused_tail(c, hnb_out, (hipStream_t)stream);
  }
  if (kbz_shard_begin(c, traces, n, stride, outcome, h32_out, x64_out, want, stream)) return -1;
  if (kbz_shard_link(c, nullptr, nullptr, 1, nullptr, nullptr, stream)) return -1;
  if (kbz_shard_reduce(c, stream)) return -1;
  return kbz_shard_finish(c, nullptr, c->total, hnb_out, stream);
}

int kbz_or_prefix_total(uint8_t *prefix_out, uint8_t *total_out, const uint8_t *in, size_t rank,
                        size_t world, size_t bytes, void *stream) {
  if (!total_out || (!in && world)) return fail("null argument");
  if (bytes == 0) return 0;
  hipLaunchKernelGGL(k_or_prefix_total, dim3(cdiv(bytes, 16 * 256)), dim3(256), 0,
                     (hipStream_t)stream, prefix_out, total_out, in, rank, world, bytes);
  HIP_TRY(hipGetLastError());
  return 0;
}

int kbz_or_reduce(uint8_t *out, const uint8_t *in, size_t r_lo, size_t r_hi, size_t bytes,
                  void *stream) {
  if (!out || (!in && r_hi > r_lo)) return fail("null argument");
  if (bytes == 0) return 0;
  hipLaunchKernelGGL(k_or_reduce, dim3(cdiv(bytes, 16 * 256)), dim3(256), 0, (hipStream_t)stream,
                     out, in, r_lo, r_hi, bytes);
  HIP_TRY(hipGetLastError());
  return 0;
}

#ifdef KBZ_TAIL_STAMPS
// diagnostic build only: k_scan's per-wave records {entry, prologue done, exit, counters}
int kbz_debug_tail(unsigned long long *host_out, size_t count) {
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_kbz_tail),
                              std::min<size_t>(count, (size_t)kTailRecs * kTailFields) * 8));
  void *sym = nullptr;
  HIP_TRY(hipGetSymbolAddress(&sym, HIP_SYMBOL(g_kbz_tail)));
  HIP_TRY(hipMemset(sym, 0, (size_t)kTailRecs * kTailFields * 8));
  return 0;
}
#endif
#ifdef KBZ_STAMPS
// diagnostic build only: per (chunk, wave) cycles {compute, vmcnt wait, fill+prefetch, barrier}
int kbz_debug_stamps(unsigned long long *host_out, size_t count) {
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_kbz_stamps),
                              std::min<size_t>(count, 4096 * 2 * 4) * 8));
  return 0;
}
#endif

int kbz_sync(kbz_ctx_t *c, void *stream) {
  if (!c) return fail("null ctx");
  DevGuard g(c->device);
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  uint32_t cnt[4];
  HIP_TRY(hipMemcpy(cnt, c->counters, sizeof(cnt), hipMemcpyDeviceToHost));
  if (cnt[1] || cnt[2]) {  // sticky until reported here
    HIP_TRY(hipMemset(c->counters + 1, 0, 2 * sizeof(uint32_t)));
    c->h_err[0] = c->h_err[1] = 0;  // k_pack's host-mapped copy: reported now, not again
    // the inconsistency flags name the site: 2 inline claim (k_scan / k_tail), 8 window item,
    // 16 byte item, 4 / 64 an item never written (k_tail helper / last workgroup), 32 a fix-path
    // flag never set (k_tail), 128 a claim record of another batch, 512 a pass-1 look-back
    // (k_pass1s's skip rule) that never saw the previous chunk's hash
    char msg[96];
    snprintf(msg, sizeof msg, "inconsistent claim (internal error, flags 0x%x)", cnt[2]);
    return fail(cnt[1] ? "claim list overflow" : msg);
  }
  c->h_err[0] = c->h_err[1] = 0;
  return 0;
}

// ---- host streaming ---------------------------------------------------------------------------
namespace {
int ensure_streaming(kbz_ctx *c) {
  if (c->work_stream) return 0;
  // slot = up to 256 MiB of traces (>= 64 rows), bounded by max_batch
  size_t rows = std::max<size_t>(64, (256u << 20) / c->M);
  rows = std::min(rows, c->max_batch);
  c->slot_rows = rows;
  HIP_TRY(hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
  HIP_TRY(hipStreamCreateWithFlags(&c->work_stream, hipStreamNonBlocking));
  for (int i = 0; i < 2; i++) {
    HIP_TRY(hipHostMalloc((void **)&c->pin[i], rows * c->M, hipHostMallocMapped));
    HIP_TRY(hipHostMalloc((void **)&c->pin_oc[i], rows, hipHostMallocMapped));
    HIP_TRY(hipMalloc((void **)&c->dslot[i], rows * c->M));
    HIP_TRY(hipMalloc((void **)&c->dslot_oc[i], rows));
    HIP_TRY(hipEventCreateWithFlags(&c->ev_copied[i], hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&c->ev_used[i], hipEventDisableTiming));
  }
  HIP_TRY(hipMalloc((void **)&c->dres_hnb, c->max_batch));
  HIP_TRY(hipMalloc((void **)&c->dres_h32, c->max_batch * 4));
  HIP_TRY(hipMalloc((void **)&c->dres_x64, c->max_batch * 8));
  return 0;
}

// Rows [0, cnt) of a host batch into a pinned slot, split over several host threads: one
// thread's memcpy from pageable memory runs well below PCIe Gen5 rate, so a single copier would
// bound the streaming path (KBZ_FILL_THREADS, default 8).
void fill_slot(uint8_t *dst, const uint8_t *src, size_t cnt, size_t stride, size_t M) {
  static const int nt = std::max(1, std::min(64, getenv("KBZ_FILL_THREADS")
                                                     ? atoi(getenv("KBZ_FILL_THREADS")) : 8));
  auto part = [=](size_t r0, size_t r1) {
    if (stride == M) memcpy(dst + r0 * M, src + r0 * M, (r1 - r0) * M);
    else
      for (size_t r = r0; r < r1; r++) memcpy(dst + r * M, src + r * stride, M);
  };
  const size_t T = std::min<size_t>(nt, std::max<size_t>(1, cnt * M >> 22));  // >= 4 MiB each
  if (T <= 1) return part(0, cnt);
  std::vector<std::thread> th;
  for (size_t i = 1; i < T; i++) th.emplace_back(part, cnt * i / T, cnt * (i + 1) / T);
  part(0, cnt / T);
  for (auto &t : th) t.join();
}
}  // namespace

int kbz_triage_batch_host(kbz_ctx_t *c, const uint8_t *traces, size_t n, size_t stride,
                          const int8_t *outcome, uint8_t *hnb_out, uint32_t *h32_out,
                          uint64_t *x64_out, int want) {
  if (!c) return fail("null ctx");
  if (n > c->max_batch) return fail("n exceeds max_batch");
  if (stride < c->M) return fail("stride < map_size");
  DevGuard g(c->device);
  if (ensure_streaming(c)) return -1;
  const size_t R = c->slot_rows, M = c->M;
  const size_t nsub = (n + R - 1) / R;
  // sub-batches are triaged in order against the carried virgin state: the sequential
  // semantics compose, so this equals one triage of the whole batch.
  for (size_t b = 0; b < nsub; b++) {
    const int sl = (int)(b & 1);
    const size_t lo = b * R, cnt = std::min(R, n - lo);
    HIP_TRY(hipEventSynchronize(c->ev_used[sl]));  // slot free (no-op the first time)
    fill_slot(c->pin[sl], traces + lo * stride, cnt, stride, M);
    if (outcome) memcpy(c->pin_oc[sl], outcome + lo, cnt);
    HIP_TRY(hipMemcpyAsync(c->dslot[sl], c->pin[sl], cnt * M, hipMemcpyHostToDevice,
                           c->copy_stream));
    if (outcome)
      HIP_TRY(hipMemcpyAsync(c->dslot_oc[sl], c->pin_oc[sl], cnt, hipMemcpyHostToDevice,
                             c->copy_stream));
    HIP_TRY(hipEventRecord(c->ev_copied[sl], c->copy_stream));
    HIP_TRY(hipStreamWaitEvent(c->work_stream, c->ev_copied[sl], 0));
    if (kbz_triage_batch_device(c, c->dslot[sl], cnt, M, outcome ? c->dslot_oc[sl] : nullptr,
                                c->dres_hnb + lo, h32_out ? c->dres_h32 + lo : nullptr,
                                x64_out ? c->dres_x64 + lo : nullptr, want, c->work_stream))
      return -1;
    HIP_TRY(hipEventRecord(c->ev_used[sl], c->work_stream));
  }
  HIP_TRY(hipStreamSynchronize(c->work_stream));
  if (n) {
    if (hnb_out) HIP_TRY(hipMemcpy(hnb_out, c->dres_hnb, n, hipMemcpyDeviceToHost));
    if (h32_out) HIP_TRY(hipMemcpy(h32_out, c->dres_h32, n * 4, hipMemcpyDeviceToHost));
    if (x64_out && (want & KBZ_WANT_X64))
      HIP_TRY(hipMemcpy(x64_out, c->dres_x64, n * 8, hipMemcpyDeviceToHost));
  }
  return kbz_sync(c, c->work_stream);
}

// ---- pinned ingest ring ------------------------------------------------------------------------
// The producer (the fuzz loop copying each exec's trace_bits, fuzzer/main.c:370-418 in batched
// form) writes straight into one of two pinned slots; submit queues the slot's H2D copy, the
// triage and the D2H copy of its results, and returns.  While the GPU works on one slot the
// producer fills the other.  Results reach the caller's buffers when that slot is acquired again
// (its previous batch is then complete) or at kbz_ring_flush.
namespace {
int ensure_ring(kbz_ctx *c) {
  if (ensure_streaming(c)) return -1;
  const size_t R = c->slot_rows;
  for (int i = 0; i < 2; i++) {
    auto &r = c->ring[i];
    if (r.d_hnb) continue;
    HIP_TRY(hipMalloc((void **)&r.d_hnb, R));
    HIP_TRY(hipMalloc((void **)&r.d_h32, R * 4));
    HIP_TRY(hipMalloc((void **)&r.d_x64, R * 8));
    HIP_TRY(hipHostMalloc((void **)&r.h_hnb, R, hipHostMallocMapped));
    HIP_TRY(hipHostMalloc((void **)&r.h_h32, R * 4, hipHostMallocMapped));
    HIP_TRY(hipHostMalloc((void **)&r.h_x64, R * 8, hipHostMallocMapped));
    HIP_TRY(hipHostGetDevicePointer((void **)&r.m_rows, c->pin[i], 0));
    HIP_TRY(hipHostGetDevicePointer((void **)&r.m_oc, c->pin_oc[i], 0));
    HIP_TRY(hipHostGetDevicePointer((void **)&r.m_hnb, r.h_hnb, 0));
    HIP_TRY(hipHostGetDevicePointer((void **)&r.m_h32, r.h_h32, 0));
    HIP_TRY(hipHostGetDevicePointer((void **)&r.m_x64, r.h_x64, 0));
  }
  return 0;
}
// the slot's batch is complete (its ev_used has been waited for): hand its results over
void ring_deliver(kbz_ctx::RingSlot &r) {
  if (!r.pending) return;
  if (r.hnb_out) memcpy(r.hnb_out, r.h_hnb, r.n);
  if (r.h32_out) memcpy(r.h32_out, r.h_h32, r.n * 4);
  if (r.x64_out) memcpy(r.x64_out, r.h_x64, r.n * 8);
  r.pending = false;
}
// The sticky device error flags, as k_pack last copied them into host-mapped memory: reported
// (and cleared) without a device round trip.
int ring_errors(kbz_ctx *c) {
  if (!c->h_err[0] && !c->h_err[1]) return 0;
  const bool ovf = c->h_err[0] != 0;
  HIP_TRY(hipMemset(c->counters + 1, 0, 2 * sizeof(uint32_t)));
  c->h_err[0] = c->h_err[1] = 0;
  return fail(ovf ? "claim list overflow" : "inconsistent claim (internal error)");
}
}  // namespace

int kbz_ring_acquire(kbz_ctx_t *c, uint8_t **rows, int8_t **outcome, size_t *cap) {
  if (!c || !rows) return fail("null argument");
  if (c->ring_acquired >= 0) return fail("kbz_ring_acquire: previous slot not submitted");
  DevGuard g(c->device);
  if (ensure_ring(c)) return -1;
  const int sl = c->ring_next;
  HIP_TRY(hipEventSynchronize(c->ev_used[sl]));  // its previous batch is done
  ring_deliver(c->ring[sl]);
  // an error of an earlier batch is reported (once) with no slot handed out, so the caller's
  // next acquire starts clean instead of finding a slot it never received still held
  if (ring_errors(c)) return -1;
  c->ring_acquired = sl;
  c->ring[sl].copied = 0;
  *rows = c->pin[sl];
  if (outcome) *outcome = c->pin_oc[sl];
  if (cap) *cap = c->slot_rows;
  return 0;
}

// Batches of at most one chunk are triaged straight from the pinned slot and write their
// results straight into pinned memory (the kernels read / write host memory over PCIe): no
// DMA transfers on the latency path of a per-exec flush.
constexpr size_t kZeroCopyRows = 64;

int kbz_ring_submit(kbz_ctx_t *c, size_t n, int have_outcome, uint8_t *hnb_out,
                    uint32_t *h32_out, uint64_t *x64_out, int want) {
  if (!c) return fail("null ctx");
  const int sl = c->ring_acquired;
  if (sl < 0) return fail("kbz_ring_submit: no slot acquired");
  if (n > c->slot_rows) return fail("kbz_ring_submit: n exceeds the slot capacity");
  DevGuard g(c->device);
  auto &r = c->ring[sl];
  const size_t M = c->M;
  const bool x64 = (want & KBZ_WANT_X64) && x64_out;
  if (n <= kZeroCopyRows && r.copied == 0) {
    if (kbz_triage_batch_device(c, r.m_rows, n, M, have_outcome ? r.m_oc : nullptr, r.m_hnb,
                                h32_out ? r.m_h32 : nullptr, x64 ? r.m_x64 : nullptr, want,
                                c->work_stream))
      return -1;
  } else {
    if (n > r.copied)  // the rows kbz_ring_commit has not queued yet
      HIP_TRY(hipMemcpyAsync(c->dslot[sl] + r.copied * M, c->pin[sl] + r.copied * M,
                             (n - r.copied) * M, hipMemcpyHostToDevice, c->copy_stream));
    if (have_outcome)
      HIP_TRY(hipMemcpyAsync(c->dslot_oc[sl], c->pin_oc[sl], n, hipMemcpyHostToDevice,
                             c->copy_stream));
    HIP_TRY(hipEventRecord(c->ev_copied[sl], c->copy_stream));
    HIP_TRY(hipStreamWaitEvent(c->work_stream, c->ev_copied[sl], 0));
    if (kbz_triage_batch_device(c, c->dslot[sl], n, M, have_outcome ? c->dslot_oc[sl] : nullptr,
                                r.d_hnb, h32_out ? r.d_h32 : nullptr, x64 ? r.d_x64 : nullptr,
                                want, c->work_stream))
      return -1;
    if (n) {
      HIP_TRY(hipMemcpyAsync(r.h_hnb, r.d_hnb, n, hipMemcpyDeviceToHost, c->work_stream));
      if (h32_out)
        HIP_TRY(hipMemcpyAsync(r.h_h32, r.d_h32, n * 4, hipMemcpyDeviceToHost, c->work_stream));
      if (x64)
        HIP_TRY(hipMemcpyAsync(r.h_x64, r.d_x64, n * 8, hipMemcpyDeviceToHost, c->work_stream));
    }
  }
  HIP_TRY(hipEventRecord(c->ev_used[sl], c->work_stream));
  r.n = n;
  r.hnb_out = hnb_out;
  r.h32_out = h32_out;
  r.x64_out = x64 ? x64_out : nullptr;
  r.pending = true;
  c->ring_acquired = -1;
  c->ring_next = sl ^ 1;
  return 0;
}

// Rows [0, n_ready) of the acquired slot are final: their H2D copy starts now, on the copy
// stream, while the producer keeps filling the slot (the submit then copies only the rest).
int kbz_ring_commit(kbz_ctx_t *c, size_t n_ready) {
  if (!c) return fail("null ctx");
  const int sl = c->ring_acquired;
  if (sl < 0) return fail("kbz_ring_commit: no slot acquired");
  if (n_ready > c->slot_rows) return fail("kbz_ring_commit: n_ready exceeds the slot capacity");
  auto &r = c->ring[sl];
  if (n_ready <= r.copied) return 0;
  DevGuard g(c->device);
  const size_t M = c->M;
  // the slot's previous batch is done (kbz_ring_acquire waited for it): its device rows are free
  HIP_TRY(hipMemcpyAsync(c->dslot[sl] + r.copied * M, c->pin[sl] + r.copied * M,
                         (n_ready - r.copied) * M, hipMemcpyHostToDevice, c->copy_stream));
  r.copied = n_ready;
  return 0;
}

int kbz_ring_release(kbz_ctx_t *c) {
  if (!c) return fail("null ctx");
  if (c->ring_acquired < 0) return fail("kbz_ring_release: no slot acquired");
  c->ring_acquired = -1;  // untouched by the GPU: the next acquire may hand it out again
  return 0;
}

int kbz_ring_flush(kbz_ctx_t *c) {
  if (!c) return fail("null ctx");
  if (!c->work_stream) return 0;  // nothing was ever submitted
  DevGuard g(c->device);
  HIP_TRY(hipStreamSynchronize(c->work_stream));
  for (auto &r : c->ring) ring_deliver(r);
  return ring_errors(c);
}

// ---- merger -----------------------------------------------------------------------------------
int kbz_merge_and_device(uint8_t *out, const uint8_t *states, size_t n, size_t state_bytes,
                         void *stream) {
  if (!out || (!states && n)) return fail("null argument");
  if (state_bytes == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) {
    HIP_TRY(hipMemsetAsync(out, 0xff, state_bytes, s));
    return 0;
  }
  if ((state_bytes & 15) || ((uintptr_t)states & 15) || ((uintptr_t)out & 15)) {
    hipLaunchKernelGGL(k_and_bytes, dim3(cdiv(state_bytes, 256)), dim3(256), 0, s, states, n,
                       state_bytes, out, 0);
    HIP_TRY(hipGetLastError());
    return 0;
  }
  const unsigned gx = cdiv(state_bytes / 16, 256);
  // enough groups to put >= 8 waves per CU on a 256-CU part, each group >= 16 states
  size_t groups = std::max<size_t>(1, std::min<size_t>(n / 16, (2048 * 64) / std::max(1u, gx * 4)));
  groups = std::min<size_t>(groups, 65535);
  if (groups <= 1) {
    hipLaunchKernelGGL(k_and_rows, dim3(gx), dim3(256), 0, s, states, n, state_bytes, out, 0);
    HIP_TRY(hipGetLastError());
    return 0;
  }
  const size_t glen = (n + groups - 1) / groups;
  groups = (n + glen - 1) / glen;
  // Tree: stage 1 folds groups of glen states; later stages fold 16 partial rows per group
  // (a full-width grid each) until at most 16 rows are left for k_and_rows, whose one thread per
  // column would otherwise walk every partial row with dependent round trips.
  constexpr size_t kTreeLen = 16;
  size_t total_rows = groups;
  for (size_t r = groups; r > kTreeLen;) {
    r = (r + kTreeLen - 1) / kTreeLen;
    total_rows += r;
  }
  uint8_t *partial = nullptr;
  HIP_TRY(hipMallocAsync((void **)&partial, total_rows * state_bytes, s));
  hipLaunchKernelGGL(k_and_groups, dim3(gx, (unsigned)groups), dim3(256), 0, s, states, n,
                     state_bytes, glen, partial);
  HIP_TRY(hipGetLastError());
  uint8_t *src = partial;
  size_t rows = groups;
  while (rows > kTreeLen) {
    const size_t next = (rows + kTreeLen - 1) / kTreeLen;
    uint8_t *dst = src + rows * state_bytes;
    hipLaunchKernelGGL(k_and_groups, dim3(gx, (unsigned)next), dim3(256), 0, s, src, rows,
                       state_bytes, kTreeLen, dst);
    HIP_TRY(hipGetLastError());
    src = dst;
    rows = next;
  }
  hipLaunchKernelGGL(k_and_rows, dim3(gx), dim3(256), 0, s, src, rows, state_bytes, out, 0);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipFreeAsync(partial, s));
  return 0;
}

namespace {
// Resources of one kbz_merge_and_host call, released on every exit path.
struct MergeStaging {
  hipStream_t cs = nullptr, ws = nullptr;
  uint8_t *pin[2] = {nullptr, nullptr}, *dst[2] = {nullptr, nullptr};
  uint8_t *part = nullptr;
  hipEvent_t copied[2] = {nullptr, nullptr}, used[2] = {nullptr, nullptr};
  ~MergeStaging() {
    if (ws) (void)hipStreamSynchronize(ws);
    if (cs) (void)hipStreamSynchronize(cs);
    for (int i = 0; i < 2; i++) {
      if (pin[i]) (void)hipHostFree(pin[i]);
      if (dst[i]) (void)hipFree(dst[i]);
      if (copied[i]) (void)hipEventDestroy(copied[i]);
      if (used[i]) (void)hipEventDestroy(used[i]);
    }
    if (part) (void)hipFree(part);
    if (cs) (void)hipStreamDestroy(cs);
    if (ws) (void)hipStreamDestroy(ws);
  }
};
}  // namespace

// The fold of kbz_merge_and_fill with its result left in device memory d_out (state_bytes,
// current device), ordered on `stream` (the library's own streams do the copies and folds).
int kbz_merge_and_fill_device(uint8_t *d_out, size_t n, size_t state_bytes, kbz_merge_fill_fn fill,
                              void *user, void *stream) {
  if (!d_out || (!fill && n)) return fail("null argument");
  if (state_bytes == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) {
    HIP_TRY(hipMemsetAsync(d_out, 0xff, state_bytes, s));
    return 0;
  }
  // slots of up to 256 MiB: the caller fills slot b while the GPU copies and folds slot b ^ 1
  const size_t per = std::max<size_t>(1, (256u << 20) / state_bytes);
  const size_t cap = std::min(per, n);
  MergeStaging m;
  HIP_TRY(hipStreamCreateWithFlags(&m.cs, hipStreamNonBlocking));
  HIP_TRY(hipStreamCreateWithFlags(&m.ws, hipStreamNonBlocking));
  for (int i = 0; i < 2; i++) {
    HIP_TRY(hipHostMalloc((void **)&m.pin[i], cap * state_bytes, hipHostMallocDefault));
    HIP_TRY(hipMalloc((void **)&m.dst[i], cap * state_bytes));
    HIP_TRY(hipEventCreateWithFlags(&m.copied[i], hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&m.used[i], hipEventDisableTiming));
  }
  HIP_TRY(hipMalloc((void **)&m.part, state_bytes));
  // the caller's stream may still be using d_out: the fold starts after it
  hipEvent_t ready = nullptr;
  HIP_TRY(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
  const hipError_t er = hipEventRecord(ready, s);
  const hipError_t ew = er == hipSuccess ? hipStreamWaitEvent(m.ws, ready, 0) : er;
  (void)hipEventDestroy(ready);
  HIP_TRY(ew);
  HIP_TRY(hipMemsetAsync(d_out, 0xff, state_bytes, m.ws));
  for (size_t lo = 0, b = 0; lo < n; lo += cap, b++) {
    const int sl = (int)(b & 1);
    const size_t cnt = std::min(cap, n - lo);
    HIP_TRY(hipEventSynchronize(m.used[sl]));
    if (fill(user, m.pin[sl], lo, cnt)) return fail("kbz_merge_and_fill: the fill callback failed");
    HIP_TRY(hipMemcpyAsync(m.dst[sl], m.pin[sl], cnt * state_bytes, hipMemcpyHostToDevice, m.cs));
    HIP_TRY(hipEventRecord(m.copied[sl], m.cs));
    HIP_TRY(hipStreamWaitEvent(m.ws, m.copied[sl], 0));
    if (kbz_merge_and_device(m.part, m.dst[sl], cnt, state_bytes, m.ws)) return -1;
    if (state_bytes % 16 == 0 && ((uintptr_t)d_out & 15) == 0) {
      hipLaunchKernelGGL(k_and_rows, dim3(cdiv(state_bytes / 16, 256)), dim3(256), 0, m.ws, m.part,
                         (size_t)1, state_bytes, d_out, 1);
    } else {
      hipLaunchKernelGGL(k_and_bytes, dim3(cdiv(state_bytes, 256)), dim3(256), 0, m.ws, m.part,
                         (size_t)1, state_bytes, d_out, 1);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(m.used[sl], m.ws));
  }
  // the caller's stream continues after the fold (m's streams are synchronised and destroyed
  // on return, so this wait is already satisfied when it is queued)
  HIP_TRY(hipStreamSynchronize(m.ws));
  return 0;
}

int kbz_merge_and_fill(uint8_t *out, size_t n, size_t state_bytes, kbz_merge_fill_fn fill,
                       void *user) {
  if (!out || (!fill && n)) return fail("null argument");
  if (state_bytes == 0) return 0;
  if (n == 0) {
    memset(out, 0xff, state_bytes);
    return 0;
  }
  uint8_t *acc = nullptr;
  HIP_TRY(hipMalloc((void **)&acc, state_bytes));
  int rc = kbz_merge_and_fill_device(acc, n, state_bytes, fill, user, nullptr);
  if (!rc && hipMemcpy(out, acc, state_bytes, hipMemcpyDeviceToHost) != hipSuccess)
    rc = fail("kbz_merge_and_fill: copy of the result failed");
  (void)hipFree(acc);
  return rc;
}

// Internal (not in the header): kbz_multi.hip's worker threads hand their error message to the
// calling thread through it.
void kbz__set_error(const char *msg) { g_err = msg ? msg : ""; }

namespace {
struct HostRows {
  const uint8_t *states;
  size_t state_bytes;
};
int fill_from_host(void *user, uint8_t *dst, size_t first, size_t count) {
  const HostRows *h = (const HostRows *)user;
  memcpy(dst, h->states + first * h->state_bytes, count * h->state_bytes);
  return 0;
}
}  // namespace

int kbz_merge_and_host(uint8_t *out, const uint8_t *states, size_t n, size_t state_bytes) {
  if (!out || (!states && n)) return fail("null argument");
  HostRows h{states, state_bytes};
  return kbz_merge_and_fill(out, n, state_bytes, fill_from_host, &h);
}

// ---- standalone hashes ---------------------------------------------------------------------------
// ---- DynamoRIO per-module coverage ------------------------------------------------------------
int kbz_triage_modules_device(kbz_ctx_t *const *ctxs, size_t k, const uint8_t *traces, size_t n,
                              size_t stride, const size_t *module_offsets, const int8_t *outcome,
                              uint8_t *hnb_out, uint8_t *any_out, uint32_t *h32_out,
                              void *stream) {
  if (!ctxs || (k && !module_offsets) || (n && !hnb_out)) return fail("null argument");
  for (size_t m = 0; m < k; m++) {
    if (!ctxs[m]) return fail("kbz_triage_modules_device: null context");
    if (module_offsets[m] + ctxs[m]->M > stride)
      return fail("kbz_triage_modules_device: module map exceeds the row stride");
    if (module_offsets[m] & 15) return fail("kbz_triage_modules_device: offset not 16-byte aligned");
  }
  for (size_t m = 0; m < k; m++)
    if (kbz_triage_batch_device(ctxs[m], traces + module_offsets[m], n, stride, outcome,
                                hnb_out + m * n, h32_out ? h32_out + m * n : nullptr, nullptr,
                                KBZ_WANT_H32, stream))
      return -1;
  if (any_out && n) {
    hipStream_t s = (hipStream_t)stream;
    if (k == 0) {
      HIP_TRY(hipMemsetAsync(any_out, 0, n, s));
      return 0;
    }
    hipLaunchKernelGGL(k_modules_any, dim3(cdiv(n, 256)), dim3(256), 0, s, hnb_out, k, n, any_out);
    HIP_TRY(hipGetLastError());
  }
  return 0;
}

int kbz_triage_modules_host(kbz_ctx_t *const *ctxs, size_t k, const uint8_t *traces, size_t n,
                            size_t stride, const size_t *module_offsets, const int8_t *outcome,
                            uint8_t *hnb_out, uint8_t *any_out, uint32_t *h32_out) {
  if (!ctxs || !k || !ctxs[0]) return fail("kbz_triage_modules_host: no modules");
  if (n && (!traces || !hnb_out)) return fail("null argument");
  if (stride & 15) return fail("kbz_triage_modules_host: stride must be a multiple of 16");
  if (n == 0) return 0;
  DevGuard g(ctxs[0]->device);
  hipStream_t s = nullptr;
  uint8_t *d_t = nullptr, *d_hnb = nullptr, *d_any = nullptr;
  uint32_t *d_h32 = nullptr;
  int8_t *d_oc = nullptr;
  int rc = -1;
  auto release = [&]() {
    (void)hipStreamSynchronize(s);
    if (d_t) (void)hipFree(d_t);
    if (d_h32) (void)hipFree(d_h32);
    if (d_oc) (void)hipFree(d_oc);
    if (d_hnb) (void)hipFree(d_hnb);
    if (d_any) (void)hipFree(d_any);
    if (s) (void)hipStreamDestroy(s);
  };
  do {
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc((void **)&d_t, n * stride) != hipSuccess ||
        hipMalloc((void **)&d_hnb, k * n) != hipSuccess ||
        hipMalloc((void **)&d_any, n) != hipSuccess ||
        (h32_out && hipMalloc((void **)&d_h32, k * n * sizeof(uint32_t)) != hipSuccess) ||
        (outcome && hipMalloc((void **)&d_oc, n) != hipSuccess)) {
      fail("kbz_triage_modules_host: device staging");
      break;
    }
    if (hipMemcpyAsync(d_t, traces, n * stride, hipMemcpyHostToDevice, s) != hipSuccess ||
        (outcome && hipMemcpyAsync(d_oc, outcome, n, hipMemcpyHostToDevice, s) != hipSuccess)) {
      fail("kbz_triage_modules_host: copy in");
      break;
    }
    if (kbz_triage_modules_device(ctxs, k, d_t, n, stride, module_offsets, d_oc, d_hnb, d_any,
                                  d_h32, s))
      break;
    if (hipMemcpyAsync(hnb_out, d_hnb, k * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
        (h32_out && hipMemcpyAsync(h32_out, d_h32, k * n * sizeof(uint32_t), hipMemcpyDeviceToHost,
                                   s) != hipSuccess) ||
        (any_out && hipMemcpyAsync(any_out, d_any, n, hipMemcpyDeviceToHost, s) != hipSuccess)) {
      fail("kbz_triage_modules_host: copy out");
      break;
    }
    rc = 0;
    for (size_t m = 0; m < k && !rc; m++) rc = kbz_sync(ctxs[m], s);
  } while (0);
  release();
  return rc;
}

// ---- picker -----------------------------------------------------------------------------------
int kbz_picker_ignore_device(const uint8_t *runs, size_t files, size_t iters, size_t size,
                             uint8_t *ignore_out, uint32_t *pair_counts_out, uint64_t *total_out,
                             void *stream) {
  if (!ignore_out || (!runs && files && iters)) return fail("null argument");
  if ((size & 15) || ((uintptr_t)runs & 15) || ((uintptr_t)ignore_out & 15))
    return fail("kbz_picker_ignore_device: size and pointers must be 16-byte multiples/aligned");
  if (size == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  HIP_TRY(hipMemsetAsync(ignore_out, 0, size, s));
  if (total_out) HIP_TRY(hipMemsetAsync(total_out, 0, sizeof(uint64_t), s));
  if (files && iters >= 2) {
    if (pair_counts_out)
      HIP_TRY(hipMemsetAsync(pair_counts_out, 0, files * (iters - 1) * sizeof(uint32_t), s));
    hipLaunchKernelGGL(k_picker_diff, dim3(cdiv(size / 16, 256), (unsigned)std::min<size_t>(files, 65535)),
                       dim3(256), 0, s, runs, files, iters, size, (uint32_t *)ignore_out,
                       pair_counts_out);
    HIP_TRY(hipGetLastError());
  }
  hipLaunchKernelGGL(k_picker_final, dim3(cdiv(size / 4, 256)), dim3(256), 0, s,
                     (uint32_t *)ignore_out, size / 4, (unsigned long long *)total_out);
  HIP_TRY(hipGetLastError());
  return 0;
}

int kbz_transform_rows_device(const uint8_t *rows, size_t n, size_t stride, size_t len, int xf,
                              uint8_t *out, size_t out_stride, void *stream) {
  if (xf < KBZ_XF_RAW || xf > KBZ_XF_SIMPLIFY) return fail("bad transform");
  if ((len & 15) || (stride & 15) || (out_stride & 15) || ((uintptr_t)rows & 15) ||
      ((uintptr_t)out & 15) || stride < len || out_stride < len)
    return fail("kbz_transform_rows: len, strides and pointers must be 16-byte multiples/aligned");
  if (!n || !len) return 0;
  if (!rows || !out) return fail("null argument");
  hipLaunchKernelGGL(k_transform_rows, dim3(cdiv(len / 16, 256), (unsigned)std::min<size_t>(n, 65535)),
                     dim3(256), 0, (hipStream_t)stream, rows, n, stride, len, xf, out, out_stride);
  HIP_TRY(hipGetLastError());
  return 0;
}
int kbz_transform_rows_host(const uint8_t *rows, size_t n, size_t stride, size_t len, int xf,
                            uint8_t *out, size_t out_stride) {
  if (xf < KBZ_XF_RAW || xf > KBZ_XF_SIMPLIFY) return fail("bad transform");
  if ((len & 15) || stride < len || out_stride < len)
    return fail("kbz_transform_rows: len must be a multiple of 16, strides >= len");
  if (!n || !len) return 0;
  if (!rows || !out) return fail("null argument");
  uint8_t *d = nullptr;
  HIP_TRY(hipMalloc((void **)&d, n * len));
  int rc = -1;
  do {
    if (hipMemcpy2D(d, len, rows, stride, len, n, hipMemcpyHostToDevice) != hipSuccess) {
      fail("kbz_transform_rows_host: copy in");
      break;
    }
    if (kbz_transform_rows_device(d, n, len, len, xf, d, len, nullptr)) break;
    if (hipMemcpy2D(out, out_stride, d, len, len, n, hipMemcpyDeviceToHost) != hipSuccess) {
      fail("kbz_transform_rows_host: copy out");
      break;
    }
    rc = 0;
  } while (0);
  (void)hipFree(d);
  return rc;
}

int kbz_hash32_device(const uint8_t *rows, size_t n, size_t stride, size_t len, uint32_t seed,
                      uint32_t *h32_out, void *stream) {
  if (len % 8) return fail("hash32 needs len % 8 == 0 (afl_progs/hash.h:38)");
  if (!n) return 0;
  if (!rows || !h32_out) return fail("null argument");
  hipLaunchKernelGGL(k_rowhash32, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, rows, n,
                     stride, len, seed, h32_out);
  HIP_TRY(hipGetLastError());
  return 0;
}
int kbz_xxh64_device(const uint8_t *rows, size_t n, size_t stride, size_t len, uint64_t seed,
                     uint64_t *x64_out, void *stream) {
  if (!n) return 0;
  if (!rows || !x64_out) return fail("null argument");
  hipLaunchKernelGGL(k_rowxxh64, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, rows, n,
                     stride, len, seed, x64_out);
  HIP_TRY(hipGetLastError());
  return 0;
}

}  // extern "C"
