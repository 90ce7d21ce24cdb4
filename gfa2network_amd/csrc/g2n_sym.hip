// g2n_sym.hip — A.maximum(A.T) of an unweighted build on gfx950: bucket partition + bucket finish.
//
// Replaces scipy's `coo_matrix.maximum(A.T)` of the matrix branch (builders.py:282-283:
// coo -> csr for A and for A.T, csr_sort_indices, csr_sum_duplicates, csr_maximum_csr) for
// builds whose every value is dtype(1) (no weight tag).  Each entry of A (stream-order COO from
// the parse) is one element of row a (side 0, column b) and one of row b (side 1: the A.T entry,
// column a).  Because every value is 1, a row's result is a function of the MULTISET of its
// (column, side) pairs: out[r, c] = max(sum of the side-0 copies, sum of the side-1 copies)
// (dtype arithmetic, zeros dropped).  The order inside a bucket is therefore free, and the
// partition need not be stable.
//
//   P1 (one or two passes, MSD): elements are partitioned by the high bits of their row into
//      buckets of 2^low rows — per 1024-thread block, an LDS histogram (written to a digit-major
//      count matrix), a device scan of that matrix (g2n_scan.hip), then the same block re-ranks
//      each sub-tile with per-digit cursors in LDS and writes each digit's run contiguously.
//      Pass 1 reads the COO coordinates themselves (both sides generated on the fly; an entry
//      whose two rows share a bucket is ONE kElPair element); pass 2 works inside each pass-1
//      group, blocks mapped to (group, chunk) on the device.  The SUM CSR (coo.tocsr of an
//      unweighted undirected build: adjacent (a, b), (b, a) twins in one bucket are one kElPair
//      element) and a sharded rank's row slice (pair streams, row base) use the same partition.
//   F1 one block per bucket (<= kSymCap entries): count rows in LDS (kElPair elements expanded),
//      scatter by row, sort each row (registers, a whole wave, or a lane's Shell sort), merge the
//      two sides per column, stage the merged entries in LDS and write them, coalesced, at twice
//      the bucket's input offset;
//   F2 after a scan of the buckets' entry counts, one block per bucket copies them to their CSR
//      place (indices, data) and rebases the bucket's indptr.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "g2n_kernels.h"
#include "g2n_scan.hip"

namespace g2n {

#ifndef G2N_PART_TPB  // experiment builds vary the partition block shape
#define G2N_PART_TPB 1024
#endif
#ifndef G2N_PART_PREFETCH
#define G2N_PART_PREFETCH 1
#endif
#ifndef G2N_SYM_DPP  // experiment builds: 1 = the partition / finish scans by DPP (g2n_kernels.hip) — measured
#define G2N_SYM_DPP 0  // slower for the finish (maxsym 2.44 -> 2.54 ms on C4, same box): shuffles kept here
#endif
constexpr uint32_t kPartTPB = G2N_PART_TPB;       // threads of a partition block
constexpr uint32_t kSubPer = 8;                    // elements per thread in one sub-tile
constexpr uint32_t kSub = kSubPer * kPartTPB;      // 8192 elements per sub-tile
constexpr uint32_t kChunkSubs = 8 * 1024 / kPartTPB;  // sub-tiles per block (65536 elements)
constexpr uint32_t kPartTile = kSub * kChunkSubs;  // 65536 elements per partition block
constexpr uint32_t kMaxDigitBits = 10;             // LDS histogram of at most 1024 digits (the tuned shape)
constexpr uint32_t kWideDigitBits = 11;            // pass 2 of a partition past 2^20 buckets (> 2^31 elements)
#ifndef G2N_FIN_TPB  // experiment builds vary the finish block (one row per thread)
#define G2N_FIN_TPB 256
#endif
// F1 at 8 waves per SIMD: its 106 SGPRs held it to 7; capped, 34 of them spill to VGPR lanes (VGPRs
// stay at 62) and the C4 build gains 0.08-0.13 ms (same box, tools/gpu_r4fw8.sh).  0: uncapped.
#ifndef G2N_FIN_W8
#define G2N_FIN_W8 1
#endif
#if G2N_FIN_W8
#define G2N_FIN_WAVES __attribute__((amdgpu_waves_per_eu(8, 8)))
#else
#define G2N_FIN_WAVES
#endif
constexpr uint32_t kFinTPB = G2N_FIN_TPB;          // threads (= rows) of a finish block
constexpr uint32_t kSymCap = 16 * kFinTPB;         // elements one finish block holds
constexpr uint32_t kSymPer = kSymCap / kFinTPB;    // 16 per thread
#ifndef G2N_FIN_REG
#define G2N_FIN_REG 8
#endif
constexpr uint32_t kSymReg = G2N_FIN_REG;         // stored elements per thread kept in registers
// F1 rows at 4-word starts (a bucket whose padded rows fit kSymCap): a short row is read with four
// ds_read_b128 instead of up to 16 lane-irregular ds_read_b32 — measured neutral on C4 (maxsym 2.427-2.441
// against 2.442-2.444 ms, same box, round 6): the short-row reads are not what holds F1
#ifndef G2N_F1_PAD
#define G2N_F1_PAD 0
#endif

// exclusive scan of one u32 per thread over a kN-thread block; returns the block total
template <uint32_t kN>
__device__ inline uint32_t block_excl_scan_n(uint32_t v, uint32_t* excl, uint32_t* lds /* >= kN / 64 */) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#if G2N_DPP_SCAN && G2N_SYM_DPP  // (g2n_kernels.hip: DPP row_shr / row_bcast, no ds_bpermute round trips)
  const uint32_t x = wave_dpp_incl(v, 0u, dpp_add);
#else
  uint32_t x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
#endif
  if (lane == 63) lds[wid] = x;
  __syncthreads();
  uint32_t wbase = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < (int)(kN / 64); w++) {
    const uint32_t y = lds[w];
    if (w < wid) wbase += y;
    tot += y;
  }
  __syncthreads();
  *excl = wbase + x - v;
  return tot;
}

// element: x = row, y = column << 2 | kind (columns < 2^30).  kind 0: the A entry (row, column);
// 1: the A.T entry of A's (column, row); 2: BOTH entries of A's (row, column), whose two rows share a
// bucket — P1 emits one such element instead of two when the entry's rows fall in the same bucket
// (graphs whose edges join nearby ids: half the partition and finish traffic), F1 expands it.
constexpr uint32_t kElSide1 = 1, kElPair = 2;
__device__ inline uint2 sym_elem(uint32_t row, uint32_t col, uint32_t kind) { return make_uint2(row, (col << 2) | kind); }

// Where a partition block's elements come from.  Pass 1: the COO entries, each giving two
// elements (row a, side 0) and (row b, side 1) for A.maximum(A.T), or one (row a, side 0) for the
// SUM CSR (coo.tocsr).  Pass 2: the pass-1 output of one group g (block -> (group, chunk j)).
struct PartSrc {
  const uint32_t* rows;   // pass 1: stream A
  const uint32_t* cols;
  uint64_t n_entries;
  uint32_t one_side;      // pass 1: 1 = one element per entry (A side 0, then T side 1), 0 = two per A entry
  const uint32_t* rows_t; // pass 1, one_side: stream T (a sharded MAX-SYM slice's A.T entries), side 1
  const uint32_t* cols_t;
  uint64_t n_t;
  uint32_t row_base;      // pass 1: rows are global ids; elements carry row - row_base (a slice's rows)
  const uint2* in;        // pass 2
  const uint32_t* gstart; // n_groups + 1 element offsets of the groups
  const uint32_t* bstart; // n_groups + 1 first block of each group
  uint32_t n_groups;
  const uint32_t* gcount; // pass 1 over group slots (GroupedCoo): block b = slot b, gcount[b] entries
  uint64_t gcap;          //   from entry b * gcap
  uint32_t pair_bits;     // pass 1, two per entry: 0, or low + 1 — an entry whose rows agree above bit
                          //   low (one bucket) is one kElPair element
  const uint32_t* vals = nullptr;  // weighted SUM (passes 5 / 6): the entries' values as exact int32
  const uint32_t* in_w = nullptr;  //   pass 6: the values beside `in`; pass 7: the pair words
  uint32_t tile = kPartTile;       // elements per block (a quarter for small inputs: more blocks than CUs)
  // a count matrix scanned together with the one before it (one scan launch for passes 2 and 7): the
  // device word holding that scan's value at this matrix's start, subtracted from every offset read
  const uint32_t* obase = nullptr;
};

// Passes 5 / 6: passes 4 / 2 of the weighted SUM CSR (coo.tocsr of a weighted COO whose duplicate
// sums cannot depend on their order — k_weight_encode checked): each element carries its value, a
// u32 in a parallel array, and two twins pair only when their values are equal.
template <int kPass>
constexpr int kBase = kPass == 5 ? 4 : (kPass == 6 || kPass == 7) ? 2 : kPass;
template <int kPass>
constexpr bool kHasW = kPass == 5 || kPass == 6;
// Pair words.  Pass 1 writes its kElPair elements — nearly every entry of a graph whose edges join
// nearby ids — as ONE 4-byte word into a second stream (A) beside the 8-byte elements (B): both rows
// share the bucket, so the word holds a's bits below pass 1's digit and b's bits below `low`:
// word = (a mod 2^shift1) << low | (b mod 2^low) (shift1 + low <= 26 bits).  Pass 7 is pass 2 over
// stream A (words in, words out; digit = word >> 2 low = bits of a >> low); F1 rebuilds (a, b) from the
// bucket id.
// Half the bytes of those elements through the rest of the partition and into F1.
template <int kPass>
constexpr bool kSplit = kPass == 1 || kPass == 4;  // MAX-SYM pass 1, and the SUM CSR's twins (pass 4)
template <int kPass>
constexpr bool kWords = kPass == 7;
// (a sharded SUM slice: rows are slice rows, columns global — b's slice row is column - row_base)
__device__ inline uint32_t pair_word(uint2 y, uint32_t shift1, uint32_t low, uint32_t row_base) {
  return ((y.x & ((1u << shift1) - 1u)) << low) | (((y.y >> 2) - row_base) & ((1u << low) - 1u));
}

struct PartBlock {  // this block's range: elements [e0, e1) (pass 1: entries [e0/2, e1/2))
  uint64_t e0, e1;
  uint32_t g, j, nb;
};

// kPass: 1 = pass 1 over A entries, two elements each (or one kElPair); 3 = pass 1 with one element
// per entry (a sharded MAX-SYM slice's two streams); 4 = pass 1 of the SUM CSR (coo.tocsr of an
// undirected build, one stream): one element per entry, or one kElPair for two adjacent entries
// that are each other's transpose in one bucket (the (a, b), (b, a) twins an undirected build writes
// for every edge); 2 = pass 2 over pass-1 groups
template <int kPass>
__device__ inline bool part_block(const PartSrc& S, uint32_t blk, PartBlock& B) {
  if (kBase<kPass> != 2 && S.gcount) {
    const uint64_t per = kPass == 1 ? 2 : 1;  // element slots per entry
    B.g = 0;
    B.j = blk;
    B.nb = 0;
    B.e0 = (uint64_t)blk * S.gcap * per;
    B.e1 = B.e0 + (uint64_t)S.gcount[blk] * per;
    return true;
  }
  if (kBase<kPass> != 2) {
    B.g = 0;
    B.j = blk;
    B.nb = 0;
    B.e0 = (uint64_t)blk * S.tile;
    const uint64_t n_el = kPass == 1 ? 2 * S.n_entries : S.n_entries + S.n_t;
    B.e1 = B.e0 + S.tile < n_el ? B.e0 + S.tile : n_el;
    return true;
  }
  if (blk >= S.bstart[S.n_groups]) return false;
  uint32_t lo = 0, hi = S.n_groups;  // last g with bstart[g] <= blk
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (S.bstart[mid] <= blk) lo = mid;
    else hi = mid;
  }
  B.g = lo;
  B.j = blk - S.bstart[lo];
  B.nb = S.bstart[lo + 1] - S.bstart[lo];
  B.e0 = (uint64_t)S.gstart[lo] + (uint64_t)B.j * S.tile;
  const uint64_t ge = S.gstart[lo + 1];
  B.e1 = B.e0 + S.tile < ge ? B.e0 + S.tile : ge;
  return true;
}

// Element slots per thread in one sub-tile: pass 1 loads kSubPer entries (a, b), each one or two
// elements (kElPair) — up to 16 K elements per sub-tile, staged in 128 KB of LDS (pass 1 runs one
// block per CU) — and expands them only when ranked, so the next sub-tile's prefetch holds the
// entries, not the elements; the other passes load G2N_PART_EL2 elements per thread.
#ifndef G2N_PART_EL2
#define G2N_PART_EL2 16
#endif
#ifndef G2N_PART_EL4  // pass 4 (SUM twins): 16 per thread spills 124 B per lane
#define G2N_PART_EL4 8
#endif
template <int kPass>
constexpr uint32_t kElPer = kPass == 1 ? 2 * kSubPer : kBase<kPass> == 4 ? G2N_PART_EL4 : kPass == 6 ? 8 : G2N_PART_EL2;
template <int kPass>
constexpr uint32_t kSubEl = kElPer<kPass> * kPartTPB;  // element slots per sub-tile

template <int kPass>
struct PartRaw {
  static constexpr uint32_t kN = kPass == 1 ? kSubPer : kElPer<kPass>;
  uint2 v[kN];
  uint32_t w[kHasW<kPass> ? kN : 1];  // weighted passes: the values
  uint32_t valid;  // bit k: v[k] holds an entry / element
};

// Sub-tile at element slot e (a multiple of kSubEl within the block's range): thread t's entries
// or elements.  Pass 1: entries e/2 + t + kPartTPB k (k < 8), coalesced u32 loads of rows and cols;
// otherwise elements e + t + kPartTPB k (k < 8).
template <int kPass>
__device__ inline void part_fetch(const PartSrc& S, uint64_t e, uint64_t e1, PartRaw<kPass>& r) {
  r.valid = 0;
#pragma unroll
  for (uint32_t k = 0; k < PartRaw<kPass>::kN; k++) {
    r.v[k] = make_uint2(0, 0);
    if constexpr (kHasW<kPass>) r.w[k] = 0;
    if (kPass == 1) {
      const uint64_t i = e / 2 + threadIdx.x + (uint64_t)k * kPartTPB;
      if (2 * i < e1) {
        r.v[k] = make_uint2(S.rows[i], S.cols[i]);
        r.valid |= 1u << k;
      }
    } else if (kBase<kPass> == 4) {  // adjacent entries per thread: item k / 2 = entries i0, i0 + 1
      const uint64_t i = e + 2 * (threadIdx.x + (uint64_t)(k / 2) * kPartTPB) + (k & 1);
      if (i < e1) {
        r.v[k] = make_uint2(S.rows[i] - S.row_base, S.cols[i]);
        if constexpr (kHasW<kPass>) r.w[k] = S.vals[i];
        r.valid |= 1u << k;
      }
    } else if (kPass == 7) {  // pair words: the word is the "row" (its digit: shift = 2 low), nothing beside
      const uint64_t i = e + threadIdx.x + (uint64_t)k * kPartTPB;
      if (i < e1) {
        r.v[k] = make_uint2(S.in_w[i], 0u);
        r.valid |= 1u << k;
      }
    } else if (kPass == 3) {
      const uint64_t i = e + threadIdx.x + (uint64_t)k * kPartTPB;
      if (i < e1) {
        const bool t = i >= S.n_entries;
        const uint64_t j = t ? i - S.n_entries : i;
        r.v[k] = sym_elem((t ? S.rows_t[j] : S.rows[j]) - S.row_base, t ? S.cols_t[j] : S.cols[j], t ? 1u : 0u);
        r.valid |= 1u << k;
      }
    } else {
      const uint64_t i = e + threadIdx.x + (uint64_t)k * kPartTPB;
      if (i < e1) {
        r.v[k] = S.in[i];
        if constexpr (kHasW<kPass>) r.w[k] = S.in_w[i];
        r.valid |= 1u << k;
      }
    }
  }
}

// The sub-tile's elements, derived from what was loaded (no second copy in registers): pass 1
// turns entry (a, b) into (a, b, side 0) and (b, a, side 1), or one (a, b, kElPair) when both rows
// fall in one bucket.
template <int kPass>
__device__ inline bool part_pair(const PartSrc& S, uint2 v) {
  return S.pair_bits && ((v.x ^ v.y) >> (S.pair_bits - 1)) == 0;
}
// kPass 4: entries u = (row - row_base, col) and w, adjacent, are one kElPair element
__device__ inline bool part_twins(const PartSrc& S, uint2 u, uint2 w) {
  const uint32_t b = u.y - S.row_base;  // u's column as a slice row
  return S.pair_bits && w.x == b && w.y == u.x + S.row_base && ((u.x ^ b) >> (S.pair_bits - 1)) == 0;
}
template <int kPass>
__device__ inline uint32_t part_valid(const PartSrc& S, const PartRaw<kPass>& r) {
  if constexpr (kPass == 1) {
    uint32_t valid = 0;
#pragma unroll
    for (uint32_t k = 0; k < kSubPer; k++)
      valid |= (r.valid >> k & 1u) ? (part_pair<kPass>(S, r.v[k]) ? 1u : 3u) << (2 * k) : 0u;
    return valid;
  } else if constexpr (kBase<kPass> == 4) {
    uint32_t valid = r.valid;
#pragma unroll
    for (uint32_t k = 0; k < kElPer<kPass>; k += 2)
      if ((r.valid >> k & 3u) == 3u && part_twins(S, r.v[k], r.v[k + 1]) && (!kHasW<kPass> || r.w[k] == r.w[k + 1]))
        valid &= ~(2u << k);
    return valid;
  } else {
    return r.valid;
  }
}
template <int kPass>
__device__ inline uint2 part_elem(const PartSrc& S, const PartRaw<kPass>& r, uint32_t k) {
  if constexpr (kPass == 1) {
    const uint2 v = r.v[k / 2];
    return (k & 1) ? sym_elem(v.y, v.x, kElSide1) : sym_elem(v.x, v.y, part_pair<kPass>(S, v) ? kElPair : 0u);
  } else if constexpr (kBase<kPass> == 4) {
    const bool tw = !(k & 1) && (r.valid >> k & 3u) == 3u && part_twins(S, r.v[k], r.v[k + 1]) &&
                    (!kHasW<kPass> || r.w[k] == r.w[k + 1]);
    return sym_elem(r.v[k].x, r.v[k].y, tw ? kElPair : 0u);
  } else {
    return r.v[k];
  }
}
template <int kPass>
__device__ inline uint32_t part_row(const PartRaw<kPass>& r, uint32_t k) {
  if constexpr (kPass == 1) return (k & 1) ? r.v[k / 2].y : r.v[k / 2].x;
  else return r.v[k].x;
}

// index of the block's count for digit d in the count matrix: pass 1 digit-major over blocks,
// pass 2 group by group, digit-major over the group's blocks (so one device scan of the matrix
// gives every (block, digit) run its output position)
// element k's digit; pass 1: the pair elements' digits follow the others' (n_dig + d: stream A)
template <int kPass>
__device__ inline uint32_t part_digit(const PartSrc& S, const PartRaw<kPass>& r, uint32_t k, uint32_t shift,
                                      uint32_t dmask, uint32_t n_dig) {
  const uint32_t d = (part_row<kPass>(r, k) >> shift) & dmask;
  if constexpr (kPass == 1) return d + ((!(k & 1) && part_pair<kPass>(S, r.v[k / 2])) ? n_dig : 0u);
  else if constexpr (kPass == 4)
    return d + ((!(k & 1) && (r.valid >> k & 3u) == 3u && part_twins(S, r.v[k], r.v[k + 1])) ? n_dig : 0u);
  else return d;
}

template <int kPass>
__device__ inline uint64_t part_slot(const PartSrc& S, const PartBlock& B, uint32_t d, uint32_t n_dig, uint64_t n_blk) {
  if (kBase<kPass> != 2) return (uint64_t)d * n_blk + B.j;
  return (uint64_t)S.bstart[B.g] * n_dig + (uint64_t)d * B.nb + B.j;
}

// Histogram of the block's digits (row >> shift) & (n_dig - 1) over its whole range.
template <int kPass, uint32_t kDB = kMaxDigitBits>
__global__ void __launch_bounds__(kPartTPB) k_part_hist(PartSrc S, uint32_t shift, uint32_t n_dig,
                                                    uint32_t* __restrict__ counts, uint64_t n_blk) {
  constexpr uint32_t kStreams = kSplit<kPass> ? 2 : 1;
  __shared__ uint32_t hist[kStreams << kDB];
  const uint32_t nd = kStreams * n_dig;  // pass 1: stream B's digits, then stream A's
  for (uint32_t d = threadIdx.x; d < nd; d += kPartTPB) hist[d] = 0;
  PartBlock B;
  if (!part_block<kPass>(S, blockIdx.x, B)) {  // block-uniform: past the last group's blocks
    for (uint32_t d = threadIdx.x; d < n_dig; d += kPartTPB) counts[(uint64_t)blockIdx.x * n_dig + d] = 0;
    return;
  }
  __syncthreads();
  const uint32_t dmask = n_dig - 1;
#pragma unroll 2
  for (uint64_t e = B.e0; e < B.e1; e += kSubEl<kPass>) {
    PartRaw<kPass> r;
    part_fetch<kPass>(S, e, B.e1, r);
    const uint32_t valid = part_valid<kPass>(S, r);
#pragma unroll
    for (uint32_t k = 0; k < kElPer<kPass>; k++)
      if (valid >> k & 1) atomicAdd(&hist[part_digit<kPass>(S, r, k, shift, dmask, n_dig)], 1u);
  }
  __syncthreads();
  for (uint32_t d = threadIdx.x; d < nd; d += kPartTPB) counts[part_slot<kPass>(S, B, d, n_dig, n_blk)] = hist[d];
}

// Scatter: per sub-tile, elements ranked in LDS (unstable), staged in digit order and written
// as runs at each digit's cursor; the cursors advance sub-tile by sub-tile, so one block fills
// each of its runs front to back (whole cache lines from one L2).
// waves per SIMD the scatter is compiled for: one 1024-thread block per CU (pass 1's stage is 128 KB;
// two blocks per CU at 64 VGPRs spill and measured slower: 10.0 vs 9.6 ms per C4 build)
#ifndef G2N_PART1_WAVES
#define G2N_PART1_WAVES 4
#endif
#ifndef G2N_PART2_WAVES
#define G2N_PART2_WAVES 4
#endif
template <int kPass, uint32_t kDB = kMaxDigitBits>
__global__ void __launch_bounds__(kPartTPB)
    __attribute__((amdgpu_waves_per_eu(kPass == 1 ? G2N_PART1_WAVES : G2N_PART2_WAVES)))
    k_part_scatter(PartSrc S, uint32_t shift, uint32_t n_dig,
                                                       const uint32_t* __restrict__ offs, uint64_t n_blk,
                                                       uint2* __restrict__ out, uint32_t* __restrict__ wout = nullptr) {
  constexpr uint32_t kStreams = kSplit<kPass> ? 2 : 1;
  __shared__ uint32_t hist[kStreams << kDB];  // sub-tile counts, then its digit starts
  __shared__ uint32_t cur[kStreams << kDB];   // output position of the next element of digit d
  __shared__ uint2 stage[kSubEl<kPass>];
  __shared__ uint32_t wstage[kHasW<kPass> ? kSubEl<kPass> : 1];  // weighted passes: the values beside
  __shared__ uint32_t red[kPartTPB / 64];
  PartBlock B;
  if (!part_block<kPass>(S, blockIdx.x, B)) return;
  const uint32_t nd = kStreams * n_dig;  // pass 1: stream A's cursors after B's
  // one scan covers both streams' matrices (round 6: one launch): stream A's offsets start at B's total,
  // the scan's value at A's first count; a matrix scanned after another one subtracts S.obase's value
  const uint32_t ob = S.obase ? *S.obase : 0u;
  const uint32_t obA = kSplit<kPass> ? offs[(uint64_t)n_dig * n_blk] : 0u;
  for (uint32_t d = threadIdx.x; d < nd; d += kPartTPB)
    cur[d] = offs[part_slot<kPass>(S, B, d, n_dig, n_blk)] - (kSplit<kPass> && d >= n_dig ? obA : ob);
  const uint32_t dmask = n_dig - 1;
  const uint32_t low = S.pair_bits - 1;  // pass 1: the pair words' b bits
  PartRaw<kPass> raw, nraw;
  part_fetch<kPass>(S, B.e0, B.e1, raw);
  constexpr uint64_t kStep = kSubEl<kPass>;
  for (uint64_t e = B.e0; e < B.e1; e += kStep) {
    for (uint32_t d = threadIdx.x; d < nd; d += kPartTPB) hist[d] = 0;
    if (G2N_PART_PREFETCH && e + kStep < B.e1) part_fetch<kPass>(S, e + kStep, B.e1, nraw);  // next sub-tile in flight
    const uint32_t valid = part_valid<kPass>(S, raw);
    __syncthreads();
    uint32_t rk[kElPer<kPass>];
#pragma unroll
    for (uint32_t k = 0; k < kElPer<kPass>; k++)
      rk[k] = (valid >> k & 1) ? atomicAdd(&hist[part_digit<kPass>(S, raw, k, shift, dmask, n_dig)], 1u) : 0u;
    __syncthreads();
    // digit starts: kDigPer consecutive digits per thread (nd <= kStreams * 1024)
    constexpr uint32_t kDigPer = (kStreams << kDB) / kPartTPB;
    uint32_t hv[kDigPer], hsum = 0;
#pragma unroll
    for (uint32_t q = 0; q < kDigPer; q++) {
      const uint32_t d = threadIdx.x * kDigPer + q;
      hv[q] = d < nd ? hist[d] : 0u;
      hsum += hv[q];
    }
    uint32_t ex;
    const uint32_t tot = block_excl_scan_n<kPartTPB>(hsum, &ex, red);
#pragma unroll
    for (uint32_t q = 0; q < kDigPer; q++) {
      const uint32_t d = threadIdx.x * kDigPer + q;
      if (d < nd) hist[d] = ex;
      ex += hv[q];
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kElPer<kPass>; k++)
      if (valid >> k & 1) {
        const uint32_t at = hist[part_digit<kPass>(S, raw, k, shift, dmask, n_dig)] + rk[k];
        stage[at] = part_elem<kPass>(S, raw, k);
        if constexpr (kHasW<kPass>) wstage[at] = raw.w[k];
      }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < tot; i += kPartTPB) {
      const uint2 y = stage[i];
      uint32_t d = (y.x >> shift) & dmask;
      if constexpr (kSplit<kPass>) {
        if ((y.y & 3u) == kElPair) {  // stream A: the pair word
          d += n_dig;
          wout[cur[d] + (i - hist[d])] = pair_word(y, shift, low, S.row_base);
          continue;
        }
      }
      if constexpr (kWords<kPass>) {
        wout[cur[d] + (i - hist[d])] = y.x;
      } else {
        out[cur[d] + (i - hist[d])] = y;
        if constexpr (kHasW<kPass>) wout[cur[d] + (i - hist[d])] = wstage[i];
      }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < kDigPer; q++) {
      const uint32_t d = threadIdx.x * kDigPer + q;
      if (d < nd) cur[d] += hv[q];
    }
    if (G2N_PART_PREFETCH) raw = nraw;
    else if (e + kStep < B.e1) part_fetch<kPass>(S, e + kStep, B.e1, raw);
  }
}

// the elements pass 1 wrote (kElPair elements make it data-dependent): the end of the scanned count matrix
__device__ inline uint32_t part_total(const uint32_t* offs, const uint32_t* counts, uint64_t n) {
  return n ? offs[n - 1] + counts[n - 1] : 0u;
}

// pass-1 groups -> pass-2 block map: gstart[g] = offs[g * n_blk1] (the scan at digit g, block 0),
// bstart = scan of the groups' block counts.  One block of 1024 threads (n_groups <= 1024) per stream:
// block s takes the s-th count matrix (stream A's after B's, both in one scan: its offsets less the
// scan's value at its start) and writes gstart / bstart at gstart + 2 s (n_groups + 1).
__global__ void __launch_bounds__(1024) k_part_groups(const uint32_t* __restrict__ offs_all,
                                                      const uint32_t* __restrict__ cnt_all, uint64_t n_blk1,
                                                      uint32_t n_groups, uint32_t* __restrict__ gstart_all,
                                                      uint32_t tile) {
  __shared__ uint32_t red[16];
  const uint64_t nm = (uint64_t)n_groups * n_blk1;
  const uint32_t* offs1 = offs_all + blockIdx.x * nm;
  const uint32_t* cnt1 = cnt_all + blockIdx.x * nm;
  uint32_t* gstart = gstart_all + 2 * (uint64_t)blockIdx.x * (n_groups + 1);
  uint32_t* bstart = gstart + n_groups + 1;
  const uint32_t sub = blockIdx.x ? offs1[0] : 0u;
  const uint32_t g = threadIdx.x;
  const uint32_t total = part_total(offs1, cnt1, nm) - sub;
  const uint32_t s = g < n_groups ? offs1[(uint64_t)g * n_blk1] - sub : total;
  const uint32_t e = g + 1 < n_groups ? offs1[(uint64_t)(g + 1) * n_blk1] - sub : total;
  const uint32_t nb = g < n_groups ? (e - s + tile - 1) / tile : 0u;
  // block scan over 1024 threads (16 waves)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t x = nb;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) red[wid] = x;
  __syncthreads();
  uint32_t base = 0, all = 0;
  for (int q = 0; q < 16; q++) {
    if (q < wid) base += red[q];
    all += red[q];
  }
  if (g < n_groups) {
    gstart[g] = s;
    bstart[g] = base + x - nb;
  }
  if (g == 0) {
    gstart[n_groups] = total;
    bstart[n_groups] = all;
  }
}

// bucket starts after the last pass: bucket q = (g << bits2) | d
__global__ void __launch_bounds__(kTPB) k_part_bucket_starts(const uint32_t* __restrict__ offs2, PartSrc m,
                                                             uint32_t n_dig2, uint64_t n_buckets,
                                                             uint32_t* __restrict__ bstart_out) {
  const uint64_t q = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  if (q > n_buckets) return;
  if (q == n_buckets) {
    bstart_out[q] = m.gstart[m.n_groups];  // the total
    return;
  }
  const uint32_t g = (uint32_t)(q / n_dig2), d = (uint32_t)(q % n_dig2);
  const uint32_t nb = m.bstart[g + 1] - m.bstart[g];
  bstart_out[q] = nb ? offs2[(uint64_t)m.bstart[g] * n_dig2 + (uint64_t)d * nb] - (m.obase ? *m.obase : 0u)
                     : m.gstart[g];
}

// single pass: bucket q = digit q, start = offs1[q * n_blk1]
// (sub: stream A's matrix, scanned after B's: the scan's value at its start, subtracted)
__global__ void __launch_bounds__(kTPB) k_part_bucket_starts1(const uint32_t* __restrict__ offs1,
                                                              const uint32_t* __restrict__ cnt1, uint64_t n_blk1,
                                                              uint64_t n_buckets, uint32_t* __restrict__ bstart_out,
                                                              const uint32_t* __restrict__ sub) {
  const uint64_t q = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  if (q > n_buckets) return;
  bstart_out[q] = (q == n_buckets ? part_total(offs1, cnt1, n_buckets * n_blk1) : offs1[q * n_blk1]) - (sub ? *sub : 0u);
}

// ---- F: bucket finish --------------------------------------------------------------------
// sorts the n values at seg (LDS) ascending: registers for n <= 16, else Shell sort
__device__ inline void sym_sort_row(uint32_t* seg, uint32_t n) {
  if (n <= 1) return;
  if (n <= 16) {
    uint32_t k[16];
#pragma unroll
    for (uint32_t q = 0; q < 16; q++) k[q] = q < n ? seg[q] : 0xFFFFFFFFu;
    if (n <= 4) net_sort<4>(k);
    else if (n <= 8) net_sort<8>(k);
    else net_sort<16>(k);
#pragma unroll
    for (uint32_t q = 0; q < 16; q++)
      if (q < n) seg[q] = k[q];
    return;
  }
  constexpr uint32_t gaps[8] = {701, 301, 132, 57, 23, 10, 4, 1};  // Ciura
  for (uint32_t gp : gaps) {
    if (gp >= n) continue;
    for (uint32_t i = gp; i < n; i++) {
      const uint32_t v = seg[i];
      uint32_t jj = i;
      while (jj >= gp && seg[jj - gp] > v) {
        seg[jj] = seg[jj - gp];
        jj -= gp;
      }
      seg[jj] = v;
    }
  }
}

// One block per bucket of 2^low <= 256 rows.  F1 (k_sym_finish) merges the bucket and writes its
// entries, coalesced through LDS, at the bucket's INPUT offset in `tmp` (a bucket's output never
// outgrows its input), its rows' local offsets in indptr and its entry count in btot; after one
// scan of btot, F2 (k_sym_place) copies each bucket to its CSR place and rebases its indptr.
// (A single kernel that found each bucket's offset by a look-back over its predecessors in block
// order measured 4.32 ms on C4 against 3.94 ms for F1 + scan + F2: the cross-XCD status polling
// costs more than the extra 4.6 GB of staging traffic.)  A bucket over kSymCap elements sets
// ctl->bucket_overflow (the host then takes the general path).
constexpr uint32_t kShortRow = 16;
constexpr uint32_t kMidRow = 64;  // rows of kShortRow + 1 .. kMidRow entries: sorted and merged by a whole wave
constexpr uint32_t kStagedSkip = 0xFFFFFFFFu;
constexpr uint32_t kMultiCopy = 0x80000000u;  // staged entry flag: its copies are in tcn

// ascending bitonic sort of one u32 per lane across the wave
__device__ inline uint32_t wave_sort64(uint32_t x) {
  const uint32_t lane = threadIdx.x & 63;
#pragma unroll
  for (uint32_t k = 2; k <= 64; k <<= 1)
#pragma unroll
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      const uint32_t y = (uint32_t)__shfl_xor((int)x, (int)j, 64);
      const bool up = (lane & k) == 0;
      const bool lower = (lane & j) == 0;
      x = (lower == up) ? min(x, y) : max(x, y);
    }
  return x;
}

// One row of nr <= 64 sorted values (column << 1 | side), lane l holding entry l: for each column
// run, the side-0 copies kx and side-1 copies ky; keep(kx, ky, kk) decides the entry.  Returns the
// entries kept; emit(j, column, kk) for the j-th (lanes in order).
template <class Keep, class Emit>
__device__ inline uint32_t wave_merge(uint32_t x, uint32_t nr, Keep keep, Emit emit) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t col = x >> 1, sd = x & 1u;
  const bool valid = lane < nr;
  const uint32_t pcol = (uint32_t)__shfl_up((int)col, 1, 64), ncol = (uint32_t)__shfl_down((int)col, 1, 64);
  const bool start = valid && (lane == 0 || pcol != col);
  const bool last = valid && (lane + 1 == nr || ncol != col);
  const unsigned long long smask = __ballot(start), s1 = __ballot(valid && sd);
  const unsigned long long upto = (2ull << lane) - 1ull;  // lanes 0..lane (all 64 for lane 63)
  const uint32_t sl = 63u - (uint32_t)__clzll((smask & upto) | 1ull);  // this lane's run start
  const unsigned long long run = upto & ~((1ull << sl) - 1ull);
  const uint32_t ky = (uint32_t)__popcll(s1 & run), kx = lane - sl + 1 - ky;
  uint32_t kk = 0;
  const bool kept = last && keep(kx, ky, kk);
  const unsigned long long km = __ballot(kept);
  if (kept) emit((uint32_t)__popcll(km & ((1ull << lane) - 1ull)), col, kk);
  return (uint32_t)__popcll(km);
}

// Diagnostics build only (-DG2N_F1_STAMPS, tools/k2_stamps.py ... f1): per bucket, the wall clock
// at F1's phase boundaries (thread 0) and the hardware id of the CU it ran on.
#ifdef G2N_F1_STAMPS
constexpr int kF1Stamps = 10;
__device__ unsigned long long* g2n_f1_stamps;
#define F1_STAMP(k)                                                                          \
  do {                                                                                       \
    if (threadIdx.x == 0) g2n_f1_stamps[blockIdx.x * kF1Stamps + (k)] = wall_clock64();      \
  } while (0)
#else
#define F1_STAMP(k) \
  do {              \
  } while (0)
#endif

// Decoupled look-back over the buckets' status words (kDirect F1): a word holds the bucket's merged
// entry count (kLbAgg) or the inclusive prefix through it (kLbIncl).  Written with one relaxed
// agent-scope 8-byte store, polled with relaxed agent-scope loads (sc1: L2-served, the store drops
// the line from its XCD's L2 — MI355X_MICROARCH.md's flag hand-off).  Every thread of the block
// reads one predecessor per round, so a round covers kFinTPB buckets: the inclusive frontier moves
// faster than blocks are dispatched, and a block rarely needs a second round.
constexpr uint64_t kLbAgg = 1ull << 62, kLbIncl = 2ull << 62, kLbVal = (1ull << 62) - 1;

__device__ inline uint64_t fin_lookback(uint64_t* lbst, uint64_t b, uint32_t* lb /* 4 */, uint64_t* red64 /* kFinTPB / 64 */) {
  uint64_t acc = 0;
  int64_t hi = (int64_t)b;
  for (uint32_t it = 0;; it++) {
    uint32_t* w = lb + 2 * (it & 1);  // parity-double-buffered: a thread may still read the other pair
    if (threadIdx.x == 0) w[0] = w[1] = kFinTPB;
    __syncthreads();
    const int64_t j = hi - 1 - (int64_t)threadIdx.x;
    const uint64_t st = j >= 0 ? __hip_atomic_load(lbst + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kLbIncl;
    const uint64_t f = st >> 62;
    if (f == 2) atomicMin(&w[0], threadIdx.x);
    if (f == 0) atomicMin(&w[1], threadIdx.x);
    __syncthreads();
    const uint32_t p = w[0], z = w[1];  // nearest inclusive predecessor, nearest unpublished one
    if (z < p) {  // block-uniform: a needed predecessor has not published yet
      __builtin_amdgcn_s_sleep(4);
      continue;
    }
    uint64_t v = threadIdx.x <= p ? (st & kLbVal) : 0ull;
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0) red64[threadIdx.x >> 6] = v;
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < kFinTPB / 64; q++) acc += red64[q];
    __syncthreads();  // red64 is reused by the next round
    if (p < kFinTPB) return acc;
    hi -= kFinTPB;
  }
}

// kDirect: the bucket's offset comes from the look-back above, and F1 writes indptr / indices /
// data at their final place (no staging, no F2).  Otherwise F1 stages (tcol / tcn) and F2 places.
// Measured on C4 (G2N_FIN_DIRECT, F1 stamps): the look-back costs ~10 us per block (merge + offsets
// 1.8 -> 11.9 us: a block's window waits on predecessors dispatched to other XCDs), F1 3.56 ms
// against 1.94 + 1.12 ms for F1 + F2 — so the staged form is the default.
template <class T, bool kSum, bool kDirect>
__global__ void __launch_bounds__(kFinTPB) G2N_FIN_WAVES k_sym_finish(const uint2* __restrict__ el, const uint32_t* __restrict__ bstart,
                                                     uint32_t low, uint64_t n_rows, T one, uint32_t* __restrict__ btot,
                                                     uint32_t* __restrict__ tcol, uint16_t* __restrict__ tcn,
                                                     int32_t* __restrict__ indptr, Ctl* ctl, uint64_t* __restrict__ lbst,
                                                     int32_t* __restrict__ indices, T* __restrict__ data,
                                                     uint32_t row_base, const uint32_t* __restrict__ wa,
                                                     const uint32_t* __restrict__ bstA, uint32_t b0) {
  __shared__ __attribute__((aligned(16))) uint32_t seg[kSymCap];  // values (column << 1 | side) grouped by row; then merged columns
  __shared__ uint32_t cnt[kFinTPB];
  __shared__ uint32_t cur[kFinTPB];    // placement cursors
  __shared__ uint32_t red[kFinTPB / 64];
  __shared__ uint16_t mlist[kFinTPB];  // the bucket's rows of kShortRow + 1 .. kMidRow entries
  __shared__ uint32_t mval[kFinTPB];   // per such row: its entries kept, then its output offset
  __shared__ uint32_t mcount;
  __shared__ uint32_t lb[4];
  __shared__ uint64_t red64[kFinTPB / 64];
  F1_STAMP(0);
  cnt[threadIdx.x] = 0;
  if (threadIdx.x == 0) mcount = 0;
  const uint64_t b = b0 + blockIdx.x;  // b0: the first bucket of this launch (F1 / F2 overlapped by ranges)
  // stored elements (a kElPair one is two entries): stream B's (8-byte elements) and stream A's (pair
  // words, bstA non-null); the bucket stages its entries at twice its offset in both streams together
  const uint32_t eB = bstart[b], nB = bstart[b + 1] - eB;
  const uint32_t eA = bstA ? bstA[b] : 0u, nA = bstA ? bstA[b + 1] - eA : 0u;
  const uint32_t e0 = eB + eA, n = nB + nA;
  auto overflow = [&]() {  // the build's sums go through the general path
    if (threadIdx.x == 0) {
      ctl->bucket_overflow = 1;
      if constexpr (kDirect) __hip_atomic_store(lbst + b, kLbIncl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else btot[b] = 0;
    }
  };
  if (n > kSymCap) {  // block-uniform
    overflow();
    return;
  }
  __syncthreads();
  const uint32_t rmask = (1u << low) - 1u;
  uint32_t my, rs, nx;  // nx: the bucket's entries, kElPair elements expanded
  bool padded = false;  // (G2N_F1_PAD) rows at 4-word starts; block-uniform
  {
    // the first kSymReg elements per thread stay in registers from the count to the placement;
    // a bucket of more stored elements (rare: a skewed bucket) reads the rest again, so F1 keeps
    // to 64 VGPRs — 4 blocks per CU
    // the registers hold stream A's words (most of a bucket) or, without stream A, B's elements
    const uint32_t hi = (uint32_t)b << low;  // a pair word's row bits above low
    auto word = [&](uint32_t w) {
      return make_uint2(hi | ((w >> low) & rmask), (((hi | (w & rmask)) + row_base) << 2) | kElPair);
    };
    const uint32_t nr = bstA ? nA : nB;
    uint2 xs[kSymReg];
    uint2 xb = make_uint2(0, 0);  // with stream A: one of stream B's elements (a bucket holds a few dozen)
    if (bstA) {  // (the stream choice hoisted out of the loads: a per-load select serializes them)
      uint32_t ws[kSymReg];
#pragma unroll
      for (uint32_t k = 0; k < kSymReg; k++) {  // every load in flight before the first count
        const uint32_t i = threadIdx.x + k * kFinTPB;
        ws[k] = i < nr ? wa[eA + i] : 0u;
      }
      if (threadIdx.x < nB) xb = el[eB + threadIdx.x];
#pragma unroll
      for (uint32_t k = 0; k < kSymReg; k++) xs[k] = word(ws[k]);
    } else {
#pragma unroll
      for (uint32_t k = 0; k < kSymReg; k++) {
        const uint32_t i = threadIdx.x + k * kFinTPB;
        if (i < nr) xs[k] = el[eB + i];
      }
    }
    // a kElPair element (x.x, column b) is also the entry (b, x.x): the A.T entry of MAX-SYM (side
    // 1), or the SUM CSR's twin (side 0); rows are slice rows (row - row_base), columns global
    auto count = [&](uint2 x) {
      atomicAdd(&cnt[x.x & rmask], 1u);
      if ((x.y & 3u) == kElPair) atomicAdd(&cnt[((x.y >> 2) - row_base) & rmask], 1u);
    };
    auto place = [&](uint2 x) {
      const uint32_t kind = x.y & 3u, col = x.y >> 2;
      seg[atomicAdd(&cur[x.x & rmask], 1u)] = (col << 1) | (kind & 1u);
      if (kind == kElPair)
        seg[atomicAdd(&cur[(col - row_base) & rmask], 1u)] = ((x.x + row_base) << 1) | (kSum ? 0u : 1u);
    };
#pragma unroll
    for (uint32_t k = 0; k < kSymReg; k++)
      if (threadIdx.x + k * kFinTPB < nr) count(xs[k]);
    for (uint32_t i = threadIdx.x + kSymReg * kFinTPB; i < nr; i += kFinTPB) count(bstA ? word(wa[eA + i]) : el[eB + i]);
    if (bstA) {
      if (threadIdx.x < nB) count(xb);
      for (uint32_t i = threadIdx.x + kFinTPB; i < nB; i += kFinTPB) count(el[eB + i]);
    }
    __syncthreads();
    F1_STAMP(1);
    my = cnt[threadIdx.x];
    if constexpr (G2N_F1_PAD && !kDirect) {
      // one scan of both layouts: the entries (low 16 bits, nx <= 2 kSymCap) and the rows rounded up
      // to 4 words (high 16 bits); the padded layout when it fits
      const uint32_t pm = (my + 3u) & ~3u;
      uint32_t ex;
      const uint32_t both = block_excl_scan_n<kFinTPB>(my | (pm << 16), &ex, red);
      nx = both & 0xFFFFu;
      padded = (both >> 16) <= kSymCap;
      rs = padded ? ex >> 16 : ex & 0xFFFFu;
    } else {
      nx = block_excl_scan_n<kFinTPB>(my, &rs, red);
    }
    if (nx > kSymCap) {  // block-uniform
      overflow();
      return;
    }
    cnt[threadIdx.x] = rs;  // row starts
    cur[threadIdx.x] = rs;
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kSymReg; k++)
      if (threadIdx.x + k * kFinTPB < nr) place(xs[k]);
    for (uint32_t i = threadIdx.x + kSymReg * kFinTPB; i < nr; i += kFinTPB) place(bstA ? word(wa[eA + i]) : el[eB + i]);
    if (bstA) {
      if (threadIdx.x < nB) place(xb);
      for (uint32_t i = threadIdx.x + kFinTPB; i < nB; i += kFinTPB) place(el[eB + i]);
    }
    __syncthreads();
    F1_STAMP(2);
  }
  const uint64_t row = (b << low) + threadIdx.x;
  const bool live = threadIdx.x <= rmask && row < n_rows;
  const bool shortrow = my <= kShortRow;
  const bool midrow = live && !shortrow && my <= kMidRow;
  const bool longrow = live && my > kMidRow;
  uint32_t* sg = seg + rs;
  // the rows of kShortRow + 1 .. kMidRow entries (about one per bucket): a whole wave sorts each
  // (bitonic across lanes, in place in LDS) and counts its kept entries; a longer row is sorted by
  // its own lane (Shell sort) — one row's lane-serial sort would hold its wave for microseconds
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (midrow) mlist[atomicAdd(&mcount, 1u)] = (uint16_t)threadIdx.x;
  __syncthreads();
  const uint32_t n_mid = mcount;  // block-uniform
  // short rows: registers; sorted ascending, padding sorts last
  uint32_t k[kShortRow];
  if constexpr (G2N_F1_PAD && !kDirect) {
    if (padded) {
#pragma unroll
      for (uint32_t q4 = 0; q4 < kShortRow / 4; q4++) {
        uint4 v = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
        if (live && shortrow && 4 * q4 < my) v = *reinterpret_cast<const uint4*>(sg + 4 * q4);
        k[4 * q4] = v.x;
        k[4 * q4 + 1] = v.y;
        k[4 * q4 + 2] = v.z;
        k[4 * q4 + 3] = v.w;
      }
#pragma unroll
      for (uint32_t q = 0; q < kShortRow; q++)
        if (!(live && shortrow && q < my)) k[q] = 0xFFFFFFFFu;
    } else {
#pragma unroll
      for (uint32_t q = 0; q < kShortRow; q++) k[q] = (live && shortrow && q < my) ? sg[q] : 0xFFFFFFFFu;
    }
  } else {
#pragma unroll
    for (uint32_t q = 0; q < kShortRow; q++) k[q] = (live && shortrow && q < my) ? sg[q] : 0xFFFFFFFFu;
  }
  {  // one network per wave: the longest short row of the wave picks it (no divergent sorts)
    uint32_t wm = (live && shortrow) ? my : 0u;
#if G2N_DPP_SCAN && G2N_SYM_DPP
    wm = wave_dpp_reduce(wm, 0u, dpp_max);
#else
    for (int o = 32; o > 0; o >>= 1) wm = max(wm, (uint32_t)__shfl_xor(wm, o, 64));
#endif
    if (wm > 8) net_sort<16>(k);
    else if (wm > 4) net_sort<8>(k);
    else if (wm > 1) net_sort<4>(k);
  }
  if (longrow) sym_sort_row(sg, my);
  // merged entries: per column the side-0 copies (x) and side-1 copies (y); the value is
  // max(sum of x ones, sum of y ones) in dtype arithmetic, zeros dropped (csr_maximum_csr)
  auto keep = [&](uint32_t kx, uint32_t ky, uint32_t& kk) -> bool {
    if constexpr (kSum) {  // coo.tocsr: the run's sum, explicit zeros kept (csr_sum_duplicates)
      kk = kx;
      return true;
    } else if constexpr (std::is_same<T, int8_t>::value) {  // int8 sums wrap: compare the dtype values
      const T x = kx ? sum_copies<T>(one, kx) : (T)0, y = ky ? sum_copies<T>(one, ky) : (T)0;
      kk = (x < y) ? ky : kx;
      return ((x < y) ? y : x) != (T)0;
    } else {  // bool / int32 / float32 / float64: the sum of k >= 1 ones is non-zero and
              // non-decreasing in k (k <= kSymCap), so the max is the larger count's sum
      kk = kx > ky ? kx : ky;
      return kk != 0;
    }
  };
  // short row, unrolled and branch-free: the kept columns' positions (bit q: k[q] ends a kept
  // column run) and copies (byte q of kq: <= kShortRow) in registers, emitted after the offsets
  // are known (padding 0xFFFFFFFF never ends a run of a real column: columns < 2^31 - 1)
  uint32_t kmask = 0;
  uint64_t kq[kShortRow / 8] = {};
  auto short_merge = [&]() -> uint32_t {
    uint32_t kx = 0, ky = 0;
#pragma unroll
    for (uint32_t q = 0; q < kShortRow; q++) {
      const bool valid = q < my;
      const uint32_t sd = k[q] & 1u;
      kx += (valid && !sd) ? 1u : 0u;
      ky += (valid && sd) ? 1u : 0u;
      const bool last = valid && (q + 1 == kShortRow || (k[q + 1] >> 1) != (k[q] >> 1));
      uint32_t kk;
      const bool kept = keep(kx, ky, kk);
      kmask |= (last && kept) ? 1u << q : 0u;
      kq[q / 8] |= (uint64_t)(kk & 0xFFu) << (8 * (q % 8));
      kx = last ? 0u : kx;
      ky = last ? 0u : ky;
    }
    return (uint32_t)__builtin_popcount(kmask);
  };
  auto long_merge = [&](auto emit) -> uint32_t {
    uint32_t i = 0, m = 0;
    while (i < my) {
      const uint32_t c = sg[i] >> 1;
      uint32_t kx = 0, ky = 0;
      while (i < my && (sg[i] >> 1) == c) {
        if (sg[i] & 1) ky++;
        else kx++;
        i++;
      }
      uint32_t kk;
      if (keep(kx, ky, kk)) emit(m++, c, kk);
    }
    return m;
  };
  auto none = [](uint32_t, uint32_t, uint32_t) {};
  if (n_mid) {
    for (uint32_t i = wv; i < n_mid; i += kFinTPB / 64) {
      const uint32_t r = mlist[i], s0 = cnt[r], nr = cur[r] - s0;  // (cur: the row's end after placement)
      uint32_t x = lane < nr ? seg[s0 + lane] : 0xFFFFFFFFu;
      x = wave_sort64(x);
      if (lane < nr) seg[s0 + lane] = x;
      const uint32_t mm = wave_merge(x, nr, keep, none);
      if (lane == 0) mval[r] = mm;
    }
    __syncthreads();
  }
  F1_STAMP(3);
  const uint32_t m = !live ? 0u : (shortrow ? short_merge() : midrow ? mval[threadIdx.x] : long_merge(none));
  // kDirect: a short row's sorted values go back to its own segment (nobody else reads or writes it
  // before the staging below), so k[] need not stay in registers across the look-back
  if (kDirect && live && shortrow) {
#pragma unroll
    for (uint32_t q = 0; q < kShortRow; q++)
      if (q < my) sg[q] = k[q];
  }
  uint32_t off;
  const uint32_t tot = block_excl_scan_n<kFinTPB>(m, &off, red);
  uint64_t base = 0;  // kDirect: the bucket's first CSR entry
  if constexpr (kDirect) {
    if (threadIdx.x == 0) __hip_atomic_store(lbst + b, kLbAgg | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    base = fin_lookback(lbst, b, lb, red64);
    if (threadIdx.x == 0) __hip_atomic_store(lbst + b, kLbIncl | (base + tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    if (threadIdx.x == 0) btot[b] = tot;
  }
  F1_STAMP(4);
  // tot <= nx <= 2 n: the bucket's staged entries stay inside [2 e0, 2 e0 + 2 n).  A staged entry is
  // its column with bit 31 set when its value sums more than one copy (columns < 2^30); only then
  // are the copies written (ocn), so the common single copy costs no bytes
  uint32_t* ocol = tcol + 2 * (uint64_t)e0;
  uint16_t* ocn = tcn + 2 * (uint64_t)e0;
  auto stage = [&](uint32_t j, uint32_t c, uint32_t kk) -> uint32_t {  // entry j of the bucket, staged
    if (kk > 1u) {
      if constexpr (kDirect) data[base + j] = sum_copies<T>(one, kk);
      else ocn[j] = (uint16_t)kk;
    }
    return kk > 1u ? (c | kMultiCopy) : c;
  };
  auto out = [&](uint32_t j, uint32_t c, uint32_t kk) {  // entry j of the bucket, straight out
    if constexpr (kDirect) {
      indices[base + j] = (int32_t)c;
      data[base + j] = sum_copies<T>(one, kk);
    } else {
      ocol[j] = stage(j, c, kk);
    }
  };
  if (live) {
    indptr[row] = (int32_t)(base + off);  // !kDirect: local, k_sym_place adds the bucket's offset
    if (row == n_rows - 1) indptr[n_rows] = (int32_t)(base + off + m);
    if (longrow)  // straight out, before the staging below reuses the segments
      long_merge([&](uint32_t j, uint32_t c, uint32_t kk) { out(off + j, c, kk); });
    if (midrow) mval[threadIdx.x] = off;
  }
  if constexpr (kDirect) {
#pragma unroll
    for (uint32_t q = 0; q < kShortRow; q++) k[q] = (live && shortrow && q < my) ? sg[q] : 0xFFFFFFFFu;
  }
  __syncthreads();  // every segment read before the staging below overwrites them
  if (n_mid) {  // the wave-sorted rows, straight out (consecutive lanes write consecutive entries)
    for (uint32_t i = wv; i < n_mid; i += kFinTPB / 64) {
      const uint32_t r = mlist[i], s0 = cnt[r], nr = cur[r] - s0, o = mval[r];
      const uint32_t x = lane < nr ? seg[s0 + lane] : 0xFFFFFFFFu;
      wave_merge(x, nr, keep, [&](uint32_t j, uint32_t c, uint32_t kk) { out(o + j, c, kk); });
    }
    __syncthreads();
  }
  if (live) {
    if (shortrow) {
      uint32_t j = off;
#pragma unroll
      for (uint32_t q = 0; q < kShortRow; q++)
        if (kmask >> q & 1u) {
          seg[j] = stage(j, k[q] >> 1, (uint32_t)(kq[q / 8] >> (8 * (q % 8))) & 0xFFu);
          j++;
        }
    } else {
      for (uint32_t j = 0; j < m; j++) seg[off + j] = kStagedSkip;
    }
  }
  __syncthreads();
  F1_STAMP(5);
  for (uint32_t i = threadIdx.x; i < tot; i += kFinTPB) {
    const uint32_t c = seg[i];
    if (c == kStagedSkip) continue;
    if constexpr (kDirect) {
      indices[base + i] = (int32_t)(c & ~kMultiCopy);
      if (!(c & kMultiCopy)) data[base + i] = sum_copies<T>(one, 1u);
    } else {
      ocol[i] = c;
    }
  }
#ifdef G2N_F1_STAMPS
  F1_STAMP(6);
  if (threadIdx.x == 0) {
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    g2n_f1_stamps[blockIdx.x * kF1Stamps + 9] = ((unsigned long long)xcc << 32) | hw;
  }
#endif
}

// F2: bucket b's staged entries to their CSR place (boff = exclusive scan of btot), indptr rebased.
// I = int64_t: scipy's int64 index arrays (more than 2^31 - 1 entries): indices widened, and indptr64
// = base + F1's local offsets (indptr holds those; every offset stays below 2^32 — elements < 2^32).
template <class T, class I>
__global__ void __launch_bounds__(kFinTPB) k_sym_place(const uint32_t* __restrict__ bstart, const uint32_t* __restrict__ btot,
                                                    const uint32_t* __restrict__ boff, uint32_t low, uint64_t n_rows,
                                                    T one, const uint32_t* __restrict__ tcol,
                                                    const uint16_t* __restrict__ tcn, int32_t* __restrict__ indptr,
                                                    I* __restrict__ indices, T* __restrict__ data,
                                                    int64_t* __restrict__ indptr64, const uint32_t* __restrict__ bstA,
                                                    uint32_t b0, const uint32_t* __restrict__ rtot, uint32_t rk) {
  // b0: the first bucket of this launch; rtot[0 .. rk): the entries of the bucket ranges before it
  // (boff then holds offsets relative to the range: F1 / F2 overlapped by ranges), or rtot null
  const uint32_t b = b0 + blockIdx.x;
  uint32_t rbase = 0;
  for (uint32_t j = 0; rtot && j < rk; j++) rbase += rtot[j];
  const uint32_t e0 = bstart[b] + (bstA ? bstA[b] : 0u), tot = btot[b], base = boff[b] + rbase;
  const uint32_t* src = tcol + 2 * (uint64_t)e0;
  const uint16_t* scn = tcn + 2 * (uint64_t)e0;
#ifndef G2N_PLACE_U
#define G2N_PLACE_U 8
#endif
  constexpr uint32_t kU = G2N_PLACE_U;  // loads in flight per thread (a bucket averages ~1500 entries)
  for (uint32_t i0 = threadIdx.x; i0 < tot; i0 += kU * kFinTPB) {
    uint32_t c[kU];
#pragma unroll
    for (uint32_t u = 0; u < kU; u++) c[u] = i0 + u * kFinTPB < tot ? src[i0 + u * kFinTPB] : 0u;
#pragma unroll
    for (uint32_t u = 0; u < kU; u++) {
      const uint32_t i = i0 + u * kFinTPB;
      if (i < tot) {
        indices[(uint64_t)base + i] = (I)(c[u] & ~kMultiCopy);
        data[(uint64_t)base + i] = sum_copies<T>(one, (c[u] & kMultiCopy) ? (uint32_t)scn[i] : 1u);
      }
    }
  }
  const uint64_t row = ((uint64_t)b << low) + threadIdx.x;
  if (threadIdx.x < (1u << low) && row < n_rows) {
    if constexpr (sizeof(I) == 8) {
      indptr64[row] = (int64_t)base + (int64_t)(uint32_t)indptr[row];
      if (row == n_rows - 1) indptr64[n_rows] = (int64_t)base + (int64_t)(uint32_t)indptr[n_rows];
    } else {
      indptr[row] += (int32_t)base;
      if (row == n_rows - 1) indptr[n_rows] += (int32_t)base;
    }
  }
}

// ---- weighted SUM CSR (coo.tocsr of a weighted COO, utils.py:55, builders.py:281) --------------
// When every duplicate sum is order-independent — integer dtypes (wrapping sums), bool (logical or),
// float dtypes whose values are all integers below 2^31 in magnitude (not -0.0) and whose per-entry
// sums of magnitudes stay below 2^24 (float32) / 2^53 (float64), so every partial sum is exact — the
// result does not depend on scipy's std::sort order: the bucket partition (passes 5 / 6 carry the
// values) and a finish that sums in any order replace the stable LSD sort + row sums.

// the values as exact int32 (weight_enc, g2n_kernels.hip): when k_values did not write them
template <class T>
__global__ void __launch_bounds__(kTPB) k_weight_encode(const T* __restrict__ data, uint64_t n,
                                                        uint32_t* __restrict__ enc, Ctl* ctl) {
  const uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  bool bad = false;
  if (i < n) enc[i] = weight_enc<T>(data[i], bad);
  if (__ballot(bad) && (threadIdx.x & 63) == 0) ctl->w_inexact = 1;
}

// A run's sum in T's arithmetic (any order): wrapping for the integer dtypes, or for bool, a plain
// integer sum for the floats (exact under k_weight_encode's bounds; `mag` collects the magnitudes).
template <class T>
struct WSum {
  int64_t s = 0;
  uint64_t mag = 0;
  __device__ void add(uint32_t e) {
    if constexpr (std::is_same<T, uint8_t>::value) s |= (int64_t)e;
    else {
      const int32_t x = (int32_t)e;
      s += x;
      mag += (uint64_t)(x < 0 ? -(int64_t)x : (int64_t)x);
    }
  }
  __device__ T value() const {
    if constexpr (std::is_same<T, uint8_t>::value) return (T)(s != 0);
    else if constexpr (std::is_same<T, int8_t>::value) return (T)(int8_t)(uint8_t)(uint64_t)s;
    else if constexpr (std::is_same<T, int32_t>::value) return (T)(int32_t)(uint32_t)(uint64_t)s;
    else return (T)s;
  }
  __device__ bool exact() const {
    if constexpr (std::is_same<T, float>::value) return mag < (1ull << 24);
    else if constexpr (std::is_same<T, double>::value) return mag < (1ull << 53);
    else return true;
  }
};

// ascending bitonic network over r[0, kN) (kN a power of two; every index compile-time)
template <int kN, int kM>
__device__ inline void sumw_sort_net(unsigned long long (&r)[kM]) {
#pragma unroll
  for (int k = 2; k <= kN; k <<= 1)
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1)
#pragma unroll
      for (int i = 0; i < kN; i++) {
        const int l = i ^ j;
        if (l > i) {
          const unsigned long long a = r[i], b = r[l];
          const bool sw = ((i & k) == 0) ? a > b : a < b;
          r[i] = sw ? b : a;
          r[l] = sw ? a : b;
        }
      }
}

// sorts n u64 keys at seg (LDS) ascending: insertion for short rows, Shell sort beyond
__device__ inline void sumw_sort_row(unsigned long long* seg, uint32_t n) {
  if (n <= 1) return;
  constexpr uint32_t gaps[8] = {701, 301, 132, 57, 23, 10, 4, 1};  // Ciura
  for (uint32_t gp : gaps) {
    if (gp >= n) continue;
    for (uint32_t i = gp; i < n; i++) {
      const unsigned long long v = seg[i];
      uint32_t jj = i;
      while (jj >= gp && seg[jj - gp] > v) {
        seg[jj] = seg[jj - gp];
        jj -= gp;
      }
      seg[jj] = v;
    }
  }
}

#ifndef G2N_F1W_MID  // experiment builds: the longest row F1w sorts by a whole wave (16: none)
#define G2N_F1W_MID 64
#endif
// F1w: one block per bucket of 2^low <= kFinTPB rows (thread = row): the bucket's entries (a kElPair
// element is the twins (a, b) and (b, a) of one value) grouped by row as (column << 32 | value) in
// LDS, each row sorted by its lane, its column runs summed; the merged entries staged at twice the
// bucket's input offset (columns in tcol, values in tval), local row offsets in indptr, the count
// in btot.  ctl->bucket_overflow: a bucket past kSymCap entries; ctl->w_inexact: a float run past
// its exact bound — the caller then takes the stable row-sum path.
template <class T>
__global__ void __launch_bounds__(kFinTPB) k_sumw_finish(const uint2* __restrict__ el, const uint32_t* __restrict__ ew,
                                                       const uint32_t* __restrict__ bstart, uint32_t low,
                                                       uint64_t n_rows, uint32_t* __restrict__ btot,
                                                       uint32_t* __restrict__ tcol, T* __restrict__ tval,
                                                       int32_t* __restrict__ indptr, Ctl* ctl) {
  __shared__ unsigned long long seg[kSymCap];
  __shared__ uint32_t cnt[kFinTPB];
  __shared__ uint32_t cur[kFinTPB];
  __shared__ uint32_t red[kFinTPB / 64];
  __shared__ uint16_t mlist[kFinTPB];  // the bucket's rows of kR + 1 .. kMidRow entries
  __shared__ uint32_t mval[kFinTPB];   // per such row: its entries kept, then its output offset
  __shared__ uint32_t mcount;
  F1_STAMP(0);
  if (threadIdx.x == 0) mcount = 0;
  const uint64_t b = blockIdx.x;
  const uint32_t e0 = bstart[b], n = bstart[b + 1] - e0;
  if (n > kSymCap) {  // block-uniform
    if (threadIdx.x == 0) {
      ctl->bucket_overflow = 1;
      btot[b] = 0;
    }
    return;
  }
  // the bucket's elements into registers first (kSymPer per thread, all loads in flight at once),
  // then counted and placed from there
  uint2 xe[kSymPer];
  uint32_t xw[kSymPer];
#pragma unroll
  for (uint32_t k = 0; k < kSymPer; k++) {
    const uint32_t i = threadIdx.x + k * kFinTPB;
    if (i < n) {
      xe[k] = el[e0 + i];
      xw[k] = ew[e0 + i];
    }
  }
  cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t rmask = (1u << low) - 1u;
#pragma unroll
  for (uint32_t k = 0; k < kSymPer; k++) {
    if (threadIdx.x + k * kFinTPB < n) {
      atomicAdd(&cnt[xe[k].x & rmask], 1u);
      if ((xe[k].y & 3u) == kElPair) atomicAdd(&cnt[(xe[k].y >> 2) & rmask], 1u);
    }
  }
  __syncthreads();
  F1_STAMP(1);
  const uint32_t my = cnt[threadIdx.x];
  uint32_t rs;
  const uint32_t nx = block_excl_scan_n<kFinTPB>(my, &rs, red);
  if (nx > kSymCap) {  // block-uniform
    if (threadIdx.x == 0) {
      ctl->bucket_overflow = 1;
      btot[b] = 0;
    }
    return;
  }
  cnt[threadIdx.x] = rs;  // row starts (the mid rows' waves read them)
  cur[threadIdx.x] = rs;
  __syncthreads();
#pragma unroll
  for (uint32_t k = 0; k < kSymPer; k++) {
    if (threadIdx.x + k * kFinTPB < n) {
      const uint2 x = xe[k];
      const uint32_t w = xw[k], col = x.y >> 2;
      seg[atomicAdd(&cur[x.x & rmask], 1u)] = ((unsigned long long)col << 32) | w;
      if ((x.y & 3u) == kElPair) seg[atomicAdd(&cur[col & rmask], 1u)] = ((unsigned long long)x.x << 32) | w;
    }
  }
  __syncthreads();
  F1_STAMP(2);
  const uint64_t row = (b << low) + threadIdx.x;
  const bool live = threadIdx.x <= rmask && row < n_rows;
  unsigned long long* sg = seg + rs;
  // rows of <= kR entries are sorted in registers (one LDS read each: lanes' rows sit a few
  // entries apart, so LDS passes over them conflict on the banks); rows of kR + 1 .. kMidRow entries
  // (a few per bucket of a graph with hubs) by a whole wave each, bitonic across the lanes (round 6: a
  // lane-serial sort held its wave, and the block, for ~10 us — C3's slowest tenth of buckets); longer
  // ones by their lane in LDS
  constexpr int kR = 16;
  const bool inreg = my <= (uint32_t)kR;
  const bool midrow = live && !inreg && my <= G2N_F1W_MID;
  const bool longrow = live && my > G2N_F1W_MID;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (midrow) mlist[atomicAdd(&mcount, 1u)] = (uint16_t)threadIdx.x;
  unsigned long long r[kR];
#pragma unroll
  for (int i = 0; i < kR; i++) r[i] = (live && inreg && i < (int)my) ? sg[i] : ~0ull;  // padding sorts last
  {  // one network per wave: the longest in-register row of the wave picks it (no divergent sorts)
    uint32_t wm = (live && inreg) ? my : 0u;
#if G2N_DPP_SCAN && G2N_SYM_DPP
    wm = wave_dpp_reduce(wm, 0u, dpp_max);
#else
    for (int o = 32; o > 0; o >>= 1) wm = max(wm, (uint32_t)__shfl_xor(wm, o, 64));
#endif
    if (wm > 8) sumw_sort_net<16>(r);
    else if (wm > 4) sumw_sort_net<8>(r);
    else if (wm > 1) sumw_sort_net<4>(r);
  }
  if (longrow) sumw_sort_row(sg, my);
  __syncthreads();  // mlist
  const uint32_t n_mid = mcount;  // block-uniform
  // a mid row's lanes: entry `lane` of the row at s0 (sorted in place by the first visit); run ends and
  // run starts by shuffles
  auto mid_runs = [&](uint32_t s0, uint32_t nr, unsigned long long& x, bool& last, uint32_t& sl) {
    const uint32_t col = (uint32_t)(x >> 32);
    const bool valid = lane < nr;
    const uint32_t pcol = (uint32_t)__shfl_up((int)col, 1, 64), ncol = (uint32_t)__shfl_down((int)col, 1, 64);
    const bool start = valid && (lane == 0 || pcol != col);
    last = valid && (lane + 1 == nr || ncol != col);
    const unsigned long long upto = (2ull << lane) - 1ull;  // lanes 0..lane
    sl = 63u - (uint32_t)__clzll((__ballot(start) & upto) | 1ull);
  };
  if (n_mid) {
    for (uint32_t i = wv; i < n_mid; i += kFinTPB / 64) {
      const uint32_t rr = mlist[i], s0 = cnt[rr], nr = (rr + 1 < kFinTPB ? cnt[rr + 1] : nx) - s0;
      unsigned long long x = lane < nr ? seg[s0 + lane] : ~0ull;
#pragma unroll
      for (uint32_t k = 2; k <= 64; k <<= 1)
#pragma unroll
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
          const unsigned long long y = __shfl_xor(x, (int)j, 64);
          x = (((lane & j) == 0) == ((lane & k) == 0)) ? (x < y ? x : y) : (x < y ? y : x);
        }
      if (lane < nr) seg[s0 + lane] = x;
      bool last;
      uint32_t sl;
      mid_runs(s0, nr, x, last, sl);
      const uint32_t kept = (uint32_t)__popcll(__ballot(last));  // (the whole wave's vote, outside the branch)
      if (lane == 0) mval[rr] = kept;
    }
    __syncthreads();
  }
  uint32_t m = 0;
  if (live) {
    if (inreg) {
#pragma unroll
      for (int i = 0; i < kR; i++)
        m += (i < (int)my && (i + 1 == kR || (r[i + 1] >> 32) != (r[i] >> 32))) ? 1u : 0u;
    } else if (midrow) {
      m = mval[threadIdx.x];
    } else {
      for (uint32_t i = 0; i < my; i++) m += (i + 1 == my || (sg[i + 1] >> 32) != (sg[i] >> 32)) ? 1u : 0u;
    }
  }
  F1_STAMP(3);
  uint32_t off;
  const uint32_t tot = block_excl_scan_n<kFinTPB>(m, &off, red);
  if (threadIdx.x == 0) btot[b] = tot;
  F1_STAMP(4);
  if (live) {
    indptr[row] = (int32_t)off;  // local: k_sumw_place adds the bucket's offset
    if (row == n_rows - 1) indptr[n_rows] = (int32_t)(off + m);
    if (midrow) mval[threadIdx.x] = off;
  }
  uint32_t* oc = tcol + 2 * (uint64_t)e0;
  T* ov = tval + 2 * (uint64_t)e0;
  bool exact = true;
  // mid and long rows straight out (before the staging below reuses seg): a long row by its lane, a mid
  // row by its wave (each run's last lane sums the run: consecutive lanes write consecutive entries)
  if (longrow) {
    WSum<T> acc;
    uint32_t j = off;
    for (uint32_t i = 0; i < my; i++) {
      acc.add((uint32_t)sg[i]);
      if (i + 1 == my || (sg[i + 1] >> 32) != (sg[i] >> 32)) {
        exact &= acc.exact();
        oc[j] = (uint32_t)(sg[i] >> 32);
        ov[j] = acc.value();
        j++;
        acc = WSum<T>{};
      }
    }
  }
  if (n_mid) {
    __syncthreads();  // mval offsets
    for (uint32_t i = wv; i < n_mid; i += kFinTPB / 64) {
      const uint32_t rr = mlist[i], s0 = cnt[rr], nr = (rr + 1 < kFinTPB ? cnt[rr + 1] : nx) - s0, o = mval[rr];
      unsigned long long x = lane < nr ? seg[s0 + lane] : ~0ull;
      bool last;
      uint32_t sl;
      mid_runs(s0, nr, x, last, sl);
      const unsigned long long km = __ballot(last);
      if (last) {
        WSum<T> acc;
        for (uint32_t q = sl; q <= lane; q++) acc.add((uint32_t)seg[s0 + q]);
        exact &= acc.exact();
        const uint32_t j = o + (uint32_t)__popcll(km & ((1ull << lane) - 1ull));
        oc[j] = (uint32_t)(x >> 32);
        ov[j] = acc.value();
      }
    }
  }
  __syncthreads();  // every segment read before the staging overwrites them
  // the in-register rows through LDS (columns, then values, in seg) and out coalesced; the positions
  // of the rows written above are skipped (a column marker in the first pass, remembered per thread
  // for the second: both passes visit the same positions with the same thread)
  {
    uint32_t* sc = (uint32_t*)seg;
    if (live) {
      uint32_t j = off;
      if (inreg) {
#pragma unroll
        for (int i = 0; i < kR; i++)
          if (i < (int)my && (i + 1 == kR || (r[i + 1] >> 32) != (r[i] >> 32))) sc[j++] = (uint32_t)(r[i] >> 32);
      } else {
        for (uint32_t q = 0; q < m; q++) sc[off + q] = kStagedSkip;
      }
    }
    __syncthreads();
    uint32_t skip = 0;  // bit k: position threadIdx.x + k kFinTPB belongs to a row written above
    for (uint32_t i = threadIdx.x, k = 0; i < tot; i += kFinTPB, k++) {
      const uint32_t c = sc[i];
      if (c == kStagedSkip) skip |= 1u << k;
      else oc[i] = c;
    }
    __syncthreads();
    T* sv = (T*)seg;
    if (live && inreg) {
      WSum<T> acc;
      uint32_t j = off;
#pragma unroll
      for (int i = 0; i < kR; i++) {
        if (i < (int)my) {
          acc.add((uint32_t)r[i]);
          if (i + 1 == kR || (r[i + 1] >> 32) != (r[i] >> 32)) {
            exact &= acc.exact();
            sv[j++] = acc.value();
            acc = WSum<T>{};
          }
        }
      }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x, k = 0; i < tot; i += kFinTPB, k++)
      if (!(skip >> k & 1u)) ov[i] = sv[i];
  }
  if (!exact) ctl->w_inexact = 1;
#ifdef G2N_F1_STAMPS
  F1_STAMP(5);
  F1_STAMP(6);
  if (threadIdx.x == 0) {
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    g2n_f1_stamps[blockIdx.x * kF1Stamps + 9] = ((unsigned long long)xcc << 32) | hw;
  }
#endif
}

// F2w: bucket b's staged entries (columns, values) to their CSR place, indptr rebased.
template <class T>
__global__ void __launch_bounds__(kFinTPB) k_sumw_place(const uint32_t* __restrict__ bstart,
                                                      const uint32_t* __restrict__ btot,
                                                      const uint32_t* __restrict__ boff, uint32_t low, uint64_t n_rows,
                                                      const uint32_t* __restrict__ tcol, const T* __restrict__ tval,
                                                      int32_t* __restrict__ indptr, int32_t* __restrict__ indices,
                                                      T* __restrict__ data) {
  const uint32_t b = blockIdx.x;
  const uint32_t e0 = bstart[b], tot = btot[b], base = boff[b];
  const uint32_t* sc = tcol + 2 * (uint64_t)e0;
  const T* sv = tval + 2 * (uint64_t)e0;
  for (uint32_t i = threadIdx.x; i < tot; i += kFinTPB) {
    indices[(uint64_t)base + i] = (int32_t)sc[i];
    data[(uint64_t)base + i] = sv[i];
  }
  const uint64_t row = ((uint64_t)b << low) + threadIdx.x;
  if (threadIdx.x < (1u << low) && row < n_rows) {
    indptr[row] += (int32_t)base;
    if (row == n_rows - 1) indptr[n_rows] += (int32_t)base;
  }
}

}  // namespace g2n
