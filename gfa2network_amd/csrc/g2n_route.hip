// g2n_route.hip — triplets to the ranks that own their rows (step 5 of the sharded build,
// gfa2network_amd/shard.py), a stable partition by owner on gfx950.
//
// Owner of a (mapped) row x = floor(x * n_ranks / n_global): rank k owns rows
// [ceil(k n / G), ceil((k + 1) n / G)) — the bounds are precomputed, so a block finds an owner by
// binary search over them in LDS instead of a 64-bit division.  Two launches over 16384-element
// tiles (1024 threads x 16 rounds, element base + 1024 r + t, i.e. rounds in stream order):
//   C  per tile, the count of each owner (wave ballots: the lanes holding the same owner are
//      found with log2(R) ballots, the lowest of them adds the group's size to an LDS counter),
//      written owner-major into a count matrix; one device scan (g2n_scan.hip) gives every
//      (owner, tile) its output offset.
//   S  the same tile again: per round, each wave's per-owner group sizes go to LDS, one thread
//      per owner turns them into wave bases (in wave order) and advances the owner's running
//      offset, and each lane writes its triplet at base + its rank inside its wave group — so
//      the output keeps stream order within every owner (scipy's duplicate-summation order).
// Replaces a radix sort of (owner, index) pairs plus a gather by the sorted index (one random
// 4-byte read per coordinate).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "g2n_kernels.h"

namespace g2n {

constexpr uint32_t kRouteTPB = 1024;
constexpr uint32_t kRouteRounds = 16;
constexpr uint32_t kRouteTile = kRouteTPB * kRouteRounds;  // 16384 elements per block
constexpr uint32_t kRouteMaxRanks = 256;                     // larger groups take the sort path
constexpr uint32_t kRouteWaves = kRouteTPB / 64;

struct RouteSrc {
  const int32_t* rows;
  const int32_t* cols;
  const uint32_t* map;  // nullptr: identity
  uint64_t n;
  uint32_t n_ranks;
  int transposed;
  const uint64_t* bounds;  // n_ranks + 1 row bounds (device)
  // group slots (a tile-local parse's COO, G2N_RANGE_SLOTS): group g's entries are [g gcap, g gcap +
  // gcount[g]); block b takes tile b % tpg of group b / tpg.  gcount null: entries [0, n)
  const uint32_t* gcount = nullptr;
  uint64_t gcap = 0;
  uint32_t tpg = 1;
};

// block b's elements [e0, e1)
__device__ __forceinline__ void route_range(const RouteSrc& s, uint64_t b, uint64_t& e0, uint64_t& e1) {
  if (s.gcount) {
    const uint64_t g = b / s.tpg, t = b % s.tpg;
    const uint64_t end = g * s.gcap + s.gcount[g];
    e0 = g * s.gcap + t * kRouteTile;
    e1 = e0 + kRouteTile < end ? e0 + kRouteTile : end;
  } else {
    e0 = b * kRouteTile;
    e1 = e0 + kRouteTile < s.n ? e0 + kRouteTile : s.n;
  }
}

// owner of row x: the k with bounds[k] <= x < bounds[k + 1] (bounds in LDS)
__device__ __forceinline__ uint32_t route_owner(const uint64_t* sb, uint32_t n_ranks, uint64_t x) {
  uint32_t lo = 0, hi = n_ranks;  // invariant: bounds[lo] <= x < bounds[hi]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (sb[mid] <= x) lo = mid;
    else hi = mid;
  }
  return lo;
}

// lanes of this wave whose owner equals this lane's (log2(R) ballots)
__device__ __forceinline__ uint64_t route_match(uint32_t o, uint32_t bits, bool valid) {
  uint64_t m = __ballot(valid);
  for (uint32_t b = 0; b < bits; b++) {
    const bool set = (o >> b) & 1u;
    const uint64_t bal = __ballot(valid && set);
    m &= set ? bal : ~bal;
  }
  return valid ? m : 0ull;
}

__device__ __forceinline__ uint32_t route_row(const RouteSrc& s, uint64_t i) {
  const uint32_t x = (uint32_t)(s.transposed ? s.cols[i] : s.rows[i]);
  return s.map ? s.map[x] : x;
}

__global__ void __launch_bounds__(kRouteTPB) k_route_count(RouteSrc s, uint32_t bits, uint64_t n_blk,
                                                           uint32_t* __restrict__ cnt) {
  __shared__ uint64_t sb[kRouteMaxRanks + 1];
  __shared__ uint32_t hist[kRouteMaxRanks];
  const uint32_t t = threadIdx.x, lane = t & 63;
  for (uint32_t k = t; k <= s.n_ranks; k += kRouteTPB) sb[k] = s.bounds[k];
  for (uint32_t k = t; k < s.n_ranks; k += kRouteTPB) hist[k] = 0;
  __syncthreads();
  uint64_t base, end;
  route_range(s, blockIdx.x, base, end);
  uint32_t own[kRouteRounds];
#pragma unroll
  for (uint32_t r = 0; r < kRouteRounds; r++) {  // all loads in flight first
    const uint64_t i = base + r * kRouteTPB + t;
    own[r] = i < end ? route_row(s, i) : 0u;
  }
#pragma unroll
  for (uint32_t r = 0; r < kRouteRounds; r++) {
    const uint64_t i = base + r * kRouteTPB + t;
    const bool valid = i < end;
    const uint32_t o = valid ? route_owner(sb, s.n_ranks, own[r]) : 0u;
    const uint64_t m = route_match(o, bits, valid);
    if (valid && (m & ((1ull << lane) - 1)) == 0) atomicAdd(&hist[o], (uint32_t)__popcll(m));
  }
  __syncthreads();
  for (uint32_t k = t; k < s.n_ranks; k += kRouteTPB) cnt[(uint64_t)k * n_blk + blockIdx.x] = hist[k];
}

template <class W>  // an unsigned type of the value's size; data == nullptr: coordinates only
__global__ void __launch_bounds__(kRouteTPB) k_route_scatter(RouteSrc s, uint32_t bits, uint64_t n_blk,
                                                             const uint32_t* __restrict__ off,
                                                             const W* __restrict__ data,
                                                             int32_t* __restrict__ orows, int32_t* __restrict__ ocols,
                                                             W* __restrict__ odata) {
  __shared__ uint64_t sb[kRouteMaxRanks + 1];
  __shared__ uint32_t run[kRouteMaxRanks];                 // next output position of each owner
  __shared__ uint32_t wcnt[kRouteWaves][kRouteMaxRanks];   // per round: group sizes, then wave bases
  const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
  for (uint32_t k = t; k <= s.n_ranks; k += kRouteTPB) sb[k] = s.bounds[k];
  for (uint32_t k = t; k < s.n_ranks; k += kRouteTPB) run[k] = off[(uint64_t)k * n_blk + blockIdx.x];
  __syncthreads();
  uint64_t base, end;
  route_range(s, blockIdx.x, base, end);
  int32_t ra[kRouteRounds], rb[kRouteRounds];
#pragma unroll
  for (uint32_t r = 0; r < kRouteRounds; r++) {  // the tile's coordinates, all loads in flight first
    const uint64_t i = base + r * kRouteTPB + t;
    ra[r] = rb[r] = 0;
    if (i < end) {
      ra[r] = s.rows[i];
      rb[r] = s.cols[i];
    }
  }
#pragma unroll
  for (uint32_t r = 0; r < kRouteRounds; r++) {
    const uint64_t i = base + r * kRouteTPB + t;
    const bool valid = i < end;
    int32_t a = ra[r], b = rb[r];
    if (valid) {
      if (s.map) {
        a = (int32_t)s.map[(uint32_t)a];
        b = (int32_t)s.map[(uint32_t)b];
      }
      if (s.transposed) {
        const int32_t x = a;
        a = b;
        b = x;
      }
    }
    const uint32_t o = valid ? route_owner(sb, s.n_ranks, (uint32_t)a) : 0u;
    const uint64_t m = route_match(o, bits, valid);
    const uint32_t below = (uint32_t)__popcll(m & ((1ull << lane) - 1));
    for (uint32_t k = lane; k < s.n_ranks; k += 64) wcnt[w][k] = 0;
    __syncthreads();  // also orders the previous round's base reads before these writes
    if (valid && below == 0) wcnt[w][o] = (uint32_t)__popcll(m);
    __syncthreads();
    for (uint32_t k = t; k < s.n_ranks; k += kRouteTPB) {  // wave bases, in wave (= stream) order
      uint32_t p = run[k];
#pragma unroll
      for (uint32_t v = 0; v < kRouteWaves; v++) {
        const uint32_t c = wcnt[v][k];
        wcnt[v][k] = p;
        p += c;
      }
      run[k] = p;
    }
    __syncthreads();
    if (valid) {
      const uint32_t pos = wcnt[w][o] + below;
      orows[pos] = a;
      ocols[pos] = b;
      if (data) odata[pos] = data[i];
    }
  }
}

// starts[k] = first output of owner k (off[k * n_blk]), starts[n_ranks] = n (the elements routed)
__global__ void k_route_starts(const uint32_t* __restrict__ off, uint64_t n_blk, uint32_t n_ranks, uint64_t n,
                               uint32_t* __restrict__ starts) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n_ranks) starts[k] = off[(uint64_t)k * n_blk];
  else if (k == n_ranks) starts[k] = (uint32_t)n;
}

// ---- the general protocol's global ids (shard.py step 4), one thread per distinct key -------------
// Order key of an owner's distinct key j: (source rank, the key's local id there) of its first
// arrival f = first_of[j]; the source is the one whose arrival range [ends[s - 1], ends[s]) holds f.
// Ranges are contiguous and every source's keys arrive in its local-id order, so these keys ascend
// with j and sort the owner's keys by global first touch (builders.py:194-198 across byte ranges).
__global__ void __launch_bounds__(kTPB) k_order_keys(const uint32_t* __restrict__ first_of,
                                                     const int64_t* __restrict__ src_idx, uint64_t nd,
                                                     const uint64_t* __restrict__ ends, uint32_t n_src,
                                                     uint64_t* __restrict__ out) {
  const uint64_t j = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  if (j >= nd) return;
  const uint64_t f = first_of[j];
  uint32_t lo = 0, hi = n_src;  // first s with ends[s] > f
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (ends[mid] <= f) lo = mid + 1;
    else hi = mid;
  }
  out[j] = ((uint64_t)lo << 32) | (uint64_t)(uint32_t)src_idx[f];
}

// Global id of distinct key j of owner `self`: j + the number of smaller order keys every other owner
// holds (each owner's keys ascend; all owners' keys are distinct) — the rank in the merged order.
__global__ void __launch_bounds__(kTPB) k_rank_keys(const uint64_t* __restrict__ keys, uint64_t n,
                                                    const uint64_t* __restrict__ all,
                                                    const uint64_t* __restrict__ all_off, uint32_t n_ranks,
                                                    uint32_t self, int64_t* __restrict__ out) {
  const uint64_t j = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  if (j >= n) return;
  const uint64_t x = keys[j];
  uint64_t g = j;
  for (uint32_t o = 0; o < n_ranks; o++) {
    if (o == self) continue;
    uint64_t lo = all_off[o], hi = all_off[o + 1];  // lower bound of x in all[lo, hi)
    const uint64_t b = lo;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (all[mid] < x) lo = mid + 1;
      else hi = mid;
    }
    g += lo - b;
  }
  out[j] = (int64_t)g;
}

}  // namespace g2n
