// g2n_scan.hip — single-pass device-wide exclusive scan (decoupled look-back), gfx950.
//
// Replaces the library scans of the pipeline (tile counts, first-touch ranks, name offsets,
// CSR row offsets, export line offsets): each is an exclusive prefix sum of a u8/u32/u64 count
// array into a u32/u64/i64 offset array (builders.py:284-288 node_list order -> blob offsets,
// scipy csr indptr = cumsum of row counts, ...).
//
// One 256-thread block scans kScanPer * 256 consecutive items.  Blocks take their tile index
// from an atomic ticket, so every tile before a block's own is resident or done when it looks
// back (forward progress without relying on launch order).  Each tile publishes a 64-bit status
// word per tile: bits 63..62 = 1 (aggregate of the tile) or 2 (inclusive prefix through the
// tile), bits 61..50 the launch's epoch, bits 49..0 the value — one atomic store, so value and
// flag are never seen torn.  The look-back is done by the first wave, 64 predecessors per step.
// The epoch and a ticket that only grows (tile = ticket - the launch's base) let launches reuse
// one status buffer without clearing it: a word of another epoch reads as unpublished (the host
// clears the buffer once per 4095 launches, and whenever it is reallocated).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace g2n {

constexpr uint32_t kScanPer = 16;                 // items per thread
constexpr uint32_t kScanTile = kScanPer * 256;    // items per block
constexpr unsigned long long kStAgg = 1ull << 62, kStInc = 2ull << 62, kStVal = (1ull << 50) - 1;
constexpr uint32_t kStEpochs = 4095;  // epochs 1 .. 4095 (0 = cleared memory)

__device__ inline unsigned long long status_load(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void status_store(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Decoupled look-back for tile `tile` whose own sum is `agg` (called by every lane of wave 0):
// publishes the aggregate, walks back over the predecessors' status words and returns the
// exclusive prefix of the tile (the inclusive prefix is published before returning).
__device__ inline unsigned long long lookback(unsigned long long* __restrict__ status, uint64_t tile,
                                              unsigned long long agg, uint32_t epoch) {
  const int lane = threadIdx.x & 63;
  const unsigned long long tag = (unsigned long long)epoch << 50;
  if (tile == 0) {
    if (lane == 0) status_store(&status[0], kStInc | tag | agg);
    return 0;
  }
  if (lane == 0) status_store(&status[tile], kStAgg | tag | agg);
  // a word of another launch (epoch) is not published yet
  auto load = [&](int64_t q) {
    const unsigned long long v = status_load(&status[q]);
    return ((v >> 50) & 0xFFFu) == epoch ? v : 0ull;
  };
  unsigned long long excl = 0;
  int64_t w = (int64_t)tile - 1;  // highest predecessor of the current window
  while (true) {
    const int64_t q = w - lane;
    unsigned long long s = q >= 0 ? load(q) : kStInc;  // before tile 0: prefix 0
    // wait until every lane of the window sees a published word
    while (__ballot((s >> 62) == 0)) {
      if ((s >> 62) == 0) s = load(q);
      __builtin_amdgcn_s_sleep(1);
    }
    const unsigned long long inc = __ballot((s >> 62) == 2);
    const int stop = inc ? __builtin_ctzll(inc) : 64;  // closest predecessor with an inclusive prefix
    unsigned long long v = lane <= stop ? (s & kStVal) : 0ull;
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    excl += v;
    if (inc) break;
    w -= 64;
  }
  if (lane == 0) status_store(&status[tile], kStInc | tag | (excl + agg));
  return excl;
}

// Exclusive scan of n items of TIn into TOut; *total (optional) = the sum of all items.
// status: one u64 per tile, no word of this epoch in it (1 <= epoch <= kStEpochs); ticket: the
// launch's first ticket is t_base.
template <class TIn, class TOut>
__global__ void __launch_bounds__(256) k_scan_excl(const TIn* __restrict__ in, TOut* __restrict__ out, uint64_t n,
                                                   unsigned long long* __restrict__ status,
                                                   unsigned long long* __restrict__ ticket, TOut* __restrict__ total,
                                                   uint32_t epoch, unsigned long long t_base) {
  __shared__ uint32_t s_tile;
  __shared__ unsigned long long s_wave[4], s_base;
  if (threadIdx.x == 0) s_tile = (uint32_t)(atomicAdd(ticket, 1ull) - t_base);
  __syncthreads();
  const uint64_t tile = s_tile;
  const uint64_t i0 = tile * kScanTile + (uint64_t)threadIdx.x * kScanPer;
  unsigned long long v[kScanPer];
  unsigned long long sum = 0;
  const bool full = i0 + kScanPer <= n;
  if (full && ((uintptr_t)in & 15) == 0) {  // 16-byte vector loads of the thread's items
    constexpr uint32_t kV = (uint32_t)(sizeof(TIn) * kScanPer / 16);
    uint4 r[kV];
#pragma unroll
    for (uint32_t j = 0; j < kV; j++) r[j] = ((const uint4*)(in + i0))[j];
    TIn t[kScanPer];
    __builtin_memcpy(t, r, sizeof(t));
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; k++) v[k] = (unsigned long long)t[k];
  } else {
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; k++) {
      const uint64_t i = i0 + k;
      v[k] = i < n ? (unsigned long long)in[i] : 0ull;
    }
  }
#pragma unroll
  for (uint32_t k = 0; k < kScanPer; k++) sum += v[k];
  // block scan of the per-thread sums
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  unsigned long long x = sum;
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_wave[wid] = x;
  __syncthreads();
  unsigned long long wbase = 0, agg = 0;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    if (q < wid) wbase += s_wave[q];
    agg += s_wave[q];
  }
  if (wid == 0) {
    const unsigned long long b = lookback(status, tile, agg, epoch);
    if (lane == 0) s_base = b;
  }
  __syncthreads();
  unsigned long long run = s_base + wbase + x - sum;
  if (full && ((uintptr_t)out & 15) == 0) {
    TOut t[kScanPer];
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; k++) {
      t[k] = (TOut)run;
      run += v[k];
    }
    constexpr uint32_t kV = (uint32_t)(sizeof(TOut) * kScanPer / 16);
    uint4 r[kV];
    __builtin_memcpy(r, t, sizeof(t));
#pragma unroll
    for (uint32_t j = 0; j < kV; j++) ((uint4*)(out + i0))[j] = r[j];
  } else {
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; k++) {
      const uint64_t i = i0 + k;
      if (i < n) out[i] = (TOut)run;
      run += v[k];
    }
  }
  if (total && i0 <= n && n <= i0 + kScanPer) *total = (TOut)run;  // the thread holding the last item
  if (total && n == 0 && tile == 0 && threadIdx.x == 0) *total = (TOut)0;
}

inline uint64_t scan_tiles(uint64_t n) { return n ? (n + kScanTile - 1) / kScanTile : 1; }

// Exclusive scan of an array of a multi-field count struct T (T + T; T{} = 0) by reduce-then-
// scan (its sums do not fit one 62-bit look-back word): k_struct_reduce sums each kStructChunk
// run, k_struct_scan_parts (one block) scans those sums, k_struct_scan_chunks scans every run from
// its base.  For the front end's per-tile counts (~200K x 48 B on C4).
constexpr uint32_t kStructChunk = 1024;  // 4 items per thread of a 256-thread block

template <class T>
__device__ inline T block_incl_scan_struct(T v, T* buf /* 256 */) {  // Hillis-Steele in LDS
  buf[threadIdx.x] = v;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {
    const T y = (int)threadIdx.x >= o ? buf[threadIdx.x - o] : T{};
    __syncthreads();
    v = v + y;
    buf[threadIdx.x] = v;
    __syncthreads();
  }
  return v;
}

template <class T>
__global__ void __launch_bounds__(256) k_struct_reduce(const T* __restrict__ in, uint64_t n, T* __restrict__ part) {
  __shared__ T buf[256];
  const uint64_t i0 = (uint64_t)blockIdx.x * kStructChunk + 4 * threadIdx.x;
  T s{};
  for (uint32_t k = 0; k < 4; k++)
    if (i0 + k < n) s = s + in[i0 + k];
  const T inc = block_incl_scan_struct(s, buf);
  if (threadIdx.x == 255) part[blockIdx.x] = inc;
}

template <class T>
__global__ void __launch_bounds__(256) k_struct_scan_parts(T* __restrict__ part, uint64_t n_parts, T* __restrict__ total) {
  __shared__ T buf[256];
  __shared__ T carry;
  if (threadIdx.x == 0) carry = T{};
  __syncthreads();
  for (uint64_t b0 = 0; b0 < n_parts; b0 += 256) {
    const uint64_t k = b0 + threadIdx.x;
    const T v = k < n_parts ? part[k] : T{};
    const T inc = block_incl_scan_struct(v, buf);
    const T c = carry;
    const T excl = threadIdx.x ? buf[threadIdx.x - 1] : T{};
    __syncthreads();
    if (k < n_parts) part[k] = c + excl;
    if (threadIdx.x == 255) carry = c + inc;
    __syncthreads();
  }
  if (threadIdx.x == 0 && total) *total = carry;
}

template <class T>
__global__ void __launch_bounds__(256) k_struct_scan_chunks(const T* __restrict__ in, uint64_t n,
                                                            const T* __restrict__ part, T* __restrict__ out) {
  __shared__ T buf[256];
  const uint64_t i0 = (uint64_t)blockIdx.x * kStructChunk + 4 * threadIdx.x;
  T v[4], s{};
  for (uint32_t k = 0; k < 4; k++) {
    v[k] = i0 + k < n ? in[i0 + k] : T{};
    s = s + v[k];
  }
  block_incl_scan_struct(s, buf);
  T run = part[blockIdx.x] + (threadIdx.x ? buf[threadIdx.x - 1] : T{});
  for (uint32_t k = 0; k < 4; k++) {
    if (i0 + k < n) out[i0 + k] = run;
    run = run + v[k];
  }
}

}  // namespace g2n
