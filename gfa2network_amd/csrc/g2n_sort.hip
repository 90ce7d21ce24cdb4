// g2n_sort.hip — stable LSD radix sort of (u32 key, payload) pairs on gfx950, hand-written.
//
// Replaces the library sort under scipy's `coo_matrix.tocsr()` for weighted / float builds
// (builders.py:281-283 -> scipy coo_tocsr + csr_sort_indices; utils.py:55 convert_format):
// the triplets are ordered by row with the stream order kept inside each row, which is what
// k_row_sum / k_row_emulate (g2n_kernels.hip) need to reproduce scipy's duplicate summation
// order.  Also the owner sort of the sharded key / triplet exchange when more ranks than the
// stable owner partition handles.
//
// One pass per digit (<= 8 bits; a w-bit key takes ceil(w / 8) passes of equal width), each
// three launches, reduce-then-scan:
//   H  k_rsort_hist:    one 256-thread block per 4096-item tile, LDS digit histogram ->
//                       digit-major count matrix [digit][tile];
//      k_scan_excl:     one device scan of the matrix (g2n_scan.hip) = every (digit, tile)
//                       run's output position;
//   S  k_rsort_scatter: the same tile re-read; each wave ranks its 16 x 64 items in order with
//                       a ballot match on the digit bits (peers = lanes holding the same digit)
//                       and per-wave LDS digit cursors, so ranks follow (wave, step, lane) =
//                       input order: STABLE.  Keys and 12-bit source indices are staged in LDS
//                       in digit order and written as contiguous runs; each payload is gathered
//                       from the tile's own input range (L2-resident) at its staged index.
// Algorithmic bytes per pass: (4 + sizeof(V)) in + (4 + sizeof(V)) out + 4 B (histogram read).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace g2n {

constexpr uint32_t kRsTPB = 256;                  // 4 waves
constexpr uint32_t kRsPer = 16;                   // items per thread (per wave: 16 steps of 64)
constexpr uint32_t kRsWaveItems = kRsPer * 64;    // 1024 consecutive items per wave
constexpr uint32_t kRsTile = kRsPer * kRsTPB;     // 4096 items per block
constexpr uint32_t kRsMaxBits = 8;                // digit width
constexpr uint32_t kRsMaxDig = 1u << kRsMaxBits;  // = kRsTPB: one digit per thread in the scans
static_assert(kRsMaxDig == kRsTPB, "digit scans assume one digit per thread");
static_assert(kRsTile <= 65536, "staged source indices are u16");

__global__ void __launch_bounds__(kRsTPB) k_rsort_hist(const uint32_t* __restrict__ key, uint64_t n, uint32_t shift,
                                                       uint32_t n_dig, uint32_t* __restrict__ counts, uint64_t n_blk) {
  __shared__ uint32_t hist[kRsMaxDig];
  hist[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t t0 = (uint64_t)blockIdx.x * kRsTile;
  const uint32_t dmask = n_dig - 1;
  // 16-byte loads: thread t takes keys 4t..4t+3 of each 1024-key quarter
  if (t0 + kRsTile <= n && ((uintptr_t)key & 15) == 0) {
    uint4 v[kRsPer / 4];
#pragma unroll
    for (uint32_t q = 0; q < kRsPer / 4; q++) v[q] = ((const uint4*)(key + t0))[q * kRsTPB + threadIdx.x];
#pragma unroll
    for (uint32_t q = 0; q < kRsPer / 4; q++) {
      atomicAdd(&hist[(v[q].x >> shift) & dmask], 1u);
      atomicAdd(&hist[(v[q].y >> shift) & dmask], 1u);
      atomicAdd(&hist[(v[q].z >> shift) & dmask], 1u);
      atomicAdd(&hist[(v[q].w >> shift) & dmask], 1u);
    }
  } else {
    for (uint32_t k = 0; k < kRsPer; k++) {
      const uint64_t i = t0 + (uint64_t)k * kRsTPB + threadIdx.x;
      if (i < n) atomicAdd(&hist[(key[i] >> shift) & dmask], 1u);
    }
  }
  __syncthreads();
  if (threadIdx.x < n_dig) counts[(uint64_t)threadIdx.x * n_blk + blockIdx.x] = hist[threadIdx.x];
}

template <class V>
__global__ void __launch_bounds__(kRsTPB) k_rsort_scatter(const uint32_t* __restrict__ kin, const V* __restrict__ vin,
                                                          uint32_t* __restrict__ kout, V* __restrict__ vout, uint64_t n,
                                                          uint32_t shift, uint32_t dbits,
                                                          const uint32_t* __restrict__ offs, uint64_t n_blk) {
  __shared__ uint32_t wcur[kRsTPB / 64][kRsMaxDig];  // per-wave digit cursors, then the waves' bases
  __shared__ uint32_t dstart[kRsMaxDig];             // block-local start of each digit's run
  __shared__ uint32_t gbase[kRsMaxDig];              // output position of each digit's run
  __shared__ uint32_t skey[kRsTile];
  __shared__ uint16_t sidx[kRsTile];
  __shared__ uint32_t red[kRsTPB / 64];
  const uint32_t n_dig = 1u << dbits, dmask = n_dig - 1;
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (uint32_t q = 0; q < kRsTPB / 64; q++) wcur[q][threadIdx.x] = 0;
  if (threadIdx.x < n_dig) gbase[threadIdx.x] = offs[(uint64_t)threadIdx.x * n_blk + blockIdx.x];
  const uint64_t t0 = (uint64_t)blockIdx.x * kRsTile;
  const uint64_t w0 = t0 + (uint64_t)w * kRsWaveItems;
  uint32_t key[kRsPer];
#pragma unroll
  for (uint32_t k = 0; k < kRsPer; k++) {
    const uint64_t i = w0 + (uint64_t)k * 64 + lane;
    key[k] = i < n ? kin[i] : 0u;
  }
  __syncthreads();
  const uint64_t lt = (1ull << lane) - 1ull;  // lanes below this one
  uint32_t rank[kRsPer];
#pragma unroll
  for (uint32_t k = 0; k < kRsPer; k++) {
    const uint64_t i = w0 + (uint64_t)k * 64 + lane;
    const uint32_t d = (key[k] >> shift) & dmask;
    uint64_t peers = __ballot(i < n);
    for (uint32_t b = 0; b < dbits; b++) {
      const bool bit = (d >> b) & 1u;
      const uint64_t m = __ballot(bit);
      peers &= bit ? m : ~m;
    }
    const uint32_t before = (uint32_t)__popcll(peers & lt);
    const uint32_t base = wcur[w][d];  // every lane reads before any lane of the wave writes
    if (i < n && before == 0) wcur[w][d] = base + (uint32_t)__popcll(peers);
    rank[k] = base + before;
  }
  __syncthreads();
  // per digit (thread = digit): the waves' exclusive bases, then the block's digit starts
  uint32_t tot = 0;
#pragma unroll
  for (uint32_t q = 0; q < kRsTPB / 64; q++) {
    const uint32_t c = wcur[q][threadIdx.x];
    wcur[q][threadIdx.x] = tot;
    tot += c;
  }
  uint32_t ex;
  const uint32_t tile_n = block_excl_scan_u32(tot, &ex, red);
  dstart[threadIdx.x] = ex;
  __syncthreads();
#pragma unroll
  for (uint32_t k = 0; k < kRsPer; k++) {
    const uint64_t i = w0 + (uint64_t)k * 64 + lane;
    if (i < n) {
      const uint32_t d = (key[k] >> shift) & dmask;
      const uint32_t p = dstart[d] + wcur[w][d] + rank[k];
      skey[p] = key[k];
      sidx[p] = (uint16_t)(w * kRsWaveItems + k * 64 + lane);
    }
  }
  __syncthreads();
  for (uint32_t p = threadIdx.x; p < tile_n; p += kRsTPB) {
    const uint32_t x = skey[p];
    const uint32_t d = (x >> shift) & dmask;
    const uint32_t o = gbase[d] + (p - dstart[d]);
    kout[o] = x;
    vout[o] = vin[t0 + sidx[p]];
  }
}

}  // namespace g2n
