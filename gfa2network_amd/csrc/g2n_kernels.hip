// g2n_kernels.hip — gfx950 kernels of the GFA -> CSR path.
//
// Replaces, on the GPU, the reference's per-line Python loops:
//   K1 tile_count            `for line in fh` + first-byte dispatch, counted per 32 KiB tile
//                                                                 gfa2network/parser.py:114-134
//   K2 tile_parse            split(b"\t") + _parse_link/_edge/... parser.py:133-361,
//                            tag weight (fast grammar)            parser.py:179-204, builders.py:205-209
//   K2b weights_slow         exact CPython int()/float() for the rest (pylit.h)
//   K4 insert_round / lookup_fast   node2idx dict (first-touch ids)   builders.py:190-198, 218-221
//   K5 names                 dict insertion order, node_list      builders.py:284-288
//   K6 triplets              add_mat_edge + dtype cast            builders.py:222-234, 280-281
//   K7-K9 (row-bucket sort, row_bounds, row_sum, row_emulate, row_max, row_compact)
//                            coo.tocsr / A.maximum(A.T) (scipy sparsetools coo_tocsr,
//                            csr_sort_indices, csr_sum_duplicates, csr_maximum_csr)
//                            builders.py:281-283, utils.py:55
// Integer / byte work only; every kernel is HBM- or latency-bound (no MFMA).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "g2n_kernels.h"
#include "g2n_scan.hip"
#include "pylit.h"
#include "stl_sort.h"

namespace g2n {

// ------------------------------------------------------------------ helpers --------
__device__ inline uint32_t byte_match_mask(uint32_t w, uint32_t pat) {
  // 0x80 in every byte of w equal to the byte in pat (exact, no false positives)
  uint32_t x = w ^ pat;
  return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
}

// A byte source: input byte i is p[i - o].  Global memory: {in, 0}; a block's LDS-staged
// window: {lds, window start}.  The parsing code below reads through it, so one copy of the
// field logic serves both (inlined per call site, each with its own address space).
struct Src {
  const uint8_t* p;
  uint64_t o;
  uint64_t lim;  // word8_z(i) reads memory only below lim
  // LDS-staged tiles: bit b of tm[k] = byte o + 16 k + b is '\t', for bytes below tm_lim
  const uint16_t* tm = nullptr;
  uint64_t tm_lim = 0;
  __device__ uint8_t operator[](uint64_t i) const { return p[i - o]; }
  __device__ const uint8_t* ptr(uint64_t i) const { return p + (i - o); }
  __device__ uint32_t word(uint64_t i) const { return *(const uint32_t*)(p + (i - o)); }  // i, o % 4 == 0
  // 8 bytes at i (i, o % 8 == 0), zero past lim
  __device__ uint64_t word8_z(uint64_t i) const {
    if (i + 8 <= lim) return *(const uint64_t*)(p + (i - o));
    uint64_t w = 0;
    for (uint32_t b = 0; b < 8; b++)
      if (i + b < lim) w |= (uint64_t)(*this)[i + b] << (8 * b);
    return w;
  }
};

// bit b: byte b of w equals pat's byte (pat = byte * 0x0101010101010101)
__device__ inline uint32_t match_bits8(uint64_t w, uint64_t pat) {
  const uint64_t x = w ^ pat;
  const uint64_t hi = ~(((x & 0x7F7F7F7F7F7F7F7Full) + 0x7F7F7F7F7F7F7F7Full) | x | 0x7F7F7F7F7F7F7F7Full);
  return (uint32_t)(((hi >> 7) * 0x0102040810204080ull) >> 56);  // movemask of the 8 top bits
}

constexpr uint32_t kMaskSpan = 64;  // bytes a delimiter mask covers

// Bit q: byte s + q (q < min(n, 64)) is '\t' (or '\n' too, with_nl).  The 8-byte words covering
// the span are loaded independently (no dependent scan), then the bits are assembled in registers.
__device__ inline uint64_t delim_mask(const Src& in, uint64_t s, uint64_t n, bool with_nl) {
  const uint64_t a = s & ~7ull;
  const uint32_t sh = (uint32_t)(s - a);
  const uint64_t end = s + (n < kMaskSpan ? n : kMaskSpan);
  uint64_t lo = 0, hi = 0;  // bits of bytes a .. a+63, a+64 .. a+71
#pragma unroll
  for (uint32_t j = 0; j < kMaskSpan / 8 + 1; j++) {
    const uint64_t q = a + 8 * j;
    if (q < end) {
      const uint64_t w = in.word8_z(q);
      uint64_t b = match_bits8(w, 0x0909090909090909ull);
      if (with_nl) b |= match_bits8(w, 0x0A0A0A0A0A0A0A0Aull);
      if (j < 8) lo |= b << (8 * j);
      else hi = b;
    }
  }
  uint64_t r = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
  const uint64_t len = end - s;
  if (len < 64) r &= (1ull << len) - 1;
  return r;
}

// first '\t' in [p, end), or end
__device__ inline uint64_t next_tab(const Src& in, uint64_t p, uint64_t end) {
  while (p < end && (p & 3)) {
    if (in[p] == '\t') return p;
    p++;
  }
  while (p + 4 <= end) {
    uint32_t m = byte_match_mask(in.word(p), 0x09090909u);
    if (m) return p + (uint64_t)(__builtin_ctz(m) >> 3);
    p += 4;
  }
  while (p < end) {
    if (in[p] == '\t') return p;
    p++;
  }
  return end;
}

// first '\n' in [p, end), or end
__device__ inline uint64_t next_nl(const Src& in, uint64_t p, uint64_t end) {
  while (p < end && (p & 3)) {
    if (in[p] == '\n') return p;
    p++;
  }
  while (p + 4 <= end) {
    uint32_t m = byte_match_mask(in.word(p), 0x0A0A0A0Au);
    if (m) return p + (uint64_t)(__builtin_ctz(m) >> 3);
    p += 4;
  }
  while (p < end) {
    if (in[p] == '\n') return p;
    p++;
  }
  return end;
}

// first '\t' or '\n' in [p, end), or end
__device__ inline uint64_t next_delim(const Src& in, uint64_t p, uint64_t end) {
  while (p < end && (p & 3)) {
    if (in[p] == '\t' || in[p] == '\n') return p;
    p++;
  }
  while (p + 4 <= end) {
    const uint32_t w = in.word(p);
    uint32_t m = byte_match_mask(w, 0x09090909u) | byte_match_mask(w, 0x0A0A0A0Au);
    if (m) return p + (uint64_t)(__builtin_ctz(m) >> 3);
    p += 4;
  }
  while (p < end) {
    if (in[p] == '\t' || in[p] == '\n') return p;
    p++;
  }
  return end;
}

__device__ inline uint64_t next_byte(const Src& in, uint64_t p, uint64_t end, uint8_t c) {
  while (p < end && in[p] != c) p++;
  return p;
}

template <class T>
__device__ inline T wave_reduce_sum(T v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  return v;
}
template <class T>
__device__ inline T wave_reduce_min(T v) {
  for (int o = 32; o > 0; o >>= 1) {
    T w = __shfl_down(v, o, 64);
    v = w < v ? w : v;
  }
  return v;
}

// exclusive scan of one u32 per thread over a 256-thread block; returns the block total
__device__ inline uint32_t block_excl_scan_u32(uint32_t v, uint32_t* excl, uint32_t* lds /* >= 4 */) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t x = v;
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) lds[wid] = x;
  __syncthreads();
  uint32_t wbase = 0, tot = 0;
  for (int w = 0; w < kTPB / 64; w++) {
    uint32_t s = lds[w];
    if (w < wid) wbase += s;
    tot += s;
  }
  __syncthreads();
  *excl = wbase + x - v;
  return tot;
}

// 16 bytes at pos (pos 16-aligned); bytes at or beyond len read as 0
__device__ inline uint4 load16(const uint8_t* __restrict__ in, uint64_t pos, uint64_t len) {
  if (pos + 16 <= len) return *(const uint4*)(in + pos);
  uint32_t w[4] = {0, 0, 0, 0};
  for (int b = 0; b < 16; b++)
    if (pos + b < len) w[b >> 2] |= (uint32_t)in[pos + b] << ((b & 3) * 8);
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// ================================================= K1: tiles (lines, classify) ======
// The input is cut into 32 KiB tiles, one block each.  A block stages its tile (and a halo
// past it) in LDS with coalesced 16-byte loads and scans it in the same order: thread t takes
// the 16-byte chunks 256 j + t (conflict-free LDS reads).  A line belongs to the tile holding
// its first byte; its index is the number of '\n' before it (parser.py:114 `for line in fh`),
// its record kind the first-byte dispatch of parser.py:117-134 (a record type must be followed
// by '\t', '\n' or the end of input).
constexpr uint32_t kTileChunks = (uint32_t)(kTile / 16);  // 16-byte chunks per tile
constexpr uint32_t kChunkIters = kTileChunks / kTPB;       // chunks per thread

// A tile's bytes (plus kHalo past it) in registers: thread t holds the 16-byte chunks
// t + 256 j; all loads are issued before the first LDS write.  (A persistent variant that loads
// tile i + G while parsing tile i measured slower on gfx950: the prefetch registers took K2 from
// 80 to 212 VGPRs, 2 waves/SIMD, 6.3 -> 10.7 ms on C4.)
#ifndef G2N_LEAN_LINK  // experiment builds: 0 = the edge line's five tabs by five ctz (round 5)
#define G2N_LEAN_LINK 1
#endif
#ifndef G2N_EDGE_ONLY  // experiment builds: 0 = no edge-only parse loop in k_tile_lean (round 5)
#define G2N_EDGE_ONLY 1
#endif
#ifndef G2N_MASK2  // experiment builds: 0 = the lean tile's two bitmaps by two mask16 (round 5)
#define G2N_MASK2 1
#endif
#ifndef G2N_EDGE_FLAT  // experiment builds: 0 = the edge-only loop through lean_line (branch per check)
#define G2N_EDGE_FLAT 1
#endif
#ifndef G2N_LOAD_UNIFORM  // experiment builds: 0 = per-chunk bounds on every tile load (round 5)
#define G2N_LOAD_UNIFORM 1
#endif

template <uint32_t kHalo, uint32_t kT = kTPB>
struct TileRegs {
  static constexpr uint32_t kChunks = (uint32_t)((kTile + kHalo) / 16);
  static constexpr uint32_t kPer = (kChunks + kT - 1) / kT;
  uint4 r[kPer];
  __device__ inline void load(const uint8_t* __restrict__ in, uint64_t len, uint64_t t0) {
    if (G2N_LOAD_UNIFORM && t0 + (uint64_t)kChunks * 16 <= len) {  // (block-uniform) every chunk is input
#pragma unroll
      for (uint32_t j = 0; j < kPer; j++) {
        const uint32_t c = j * kT + threadIdx.x;
        r[j] = c < kChunks ? *(const uint4*)(in + t0 + (uint64_t)c * 16) : make_uint4(0, 0, 0, 0);
      }
      return;
    }
#pragma unroll
    for (uint32_t j = 0; j < kPer; j++) {  // every load in flight before any is used
      const uint32_t c = j * kT + threadIdx.x;
      const uint64_t pos = t0 + (uint64_t)c * 16;
      r[j] = (c < kChunks && pos < len) ? load16(in, pos, len) : make_uint4(0, 0, 0, 0);
    }
  }
  __device__ inline void store(uint8_t* lds) const {
#pragma unroll
    for (uint32_t j = 0; j < kPer; j++) {
      const uint32_t c = j * kT + threadIdx.x;
      if (c < kChunks) *(uint4*)(lds + (uint64_t)c * 16) = r[j];
    }
  }
};

__device__ inline uint8_t line_kind(uint8_t c0, bool exact) {
  switch (c0) {
    case 'S': return exact ? kS : kSkip;
    case 'L': case 'E': case 'C': return exact ? kEdge : kSkip;
    case 'P': case 'O': return exact ? kPO : kSkip;
    case 'H': case 'F': return kSkip;
    default: return kUnknown;  // parser.py:125-131: warned about once
  }
}

// kind of the line starting at tile offset o (input position p)
__device__ inline uint8_t kind_at(const uint8_t* buf, uint32_t o, uint64_t p, uint64_t len) {
  const uint8_t c0 = buf[o];
  return line_kind(c0, p + 1 >= len || c0 == '\n' || buf[o + 1] == '\t' || buf[o + 1] == '\n');
}

// bit b (b < 16): byte b of the 16-byte chunk v equals pat's byte (pat = byte * 0x01010101).
// The four words' match bytes are merged into one register (bit 8 b + k = byte b of word k),
// compressed to 16 bits (bit 4 b + k) and transposed as a 4 x 4 bit matrix (two delta swaps)
// into byte order — fewer VALU than four per-word gathers.
__device__ inline uint32_t mask16(uint4 v, uint32_t pat) {
  const uint32_t t = (byte_match_mask(v.x, pat) >> 7) | (byte_match_mask(v.y, pat) >> 6) |
                     (byte_match_mask(v.z, pat) >> 5) | (byte_match_mask(v.w, pat) >> 4);
  uint32_t x = (t & 0xFu) | ((t >> 4) & 0xF0u) | ((t >> 8) & 0xF00u) | ((t >> 12) & 0xF000u);
  const uint32_t t1 = (x ^ (x >> 3)) & 0x0A0Au;
  x ^= t1 ^ (t1 << 3);
  const uint32_t t2 = (x ^ (x >> 6)) & 0x00CCu;
  x ^= t2 ^ (t2 << 6);
  return x;
}

// Both bitmaps of a 16-byte chunk at once: tab bits (byte order) in the low 16 bits, newline bits in the
// high 16 (round 6; == mask16(v, 0x09..) | mask16(v, 0x0A..) << 16).  t = byte ^ 0x08 maps tab to 1 and
// newline to 2; one exact "byte < 4" test (no carry between bytes) then bit 0 / bit 1 of t pick tab /
// newline; the four words' tab bits go to bits 8b + k and newline bits to 8b + 4 + k of one word, a
// nibble unshuffle separates them into two 16-bit halves, and the 4 x 4 bit transposes of both halves
// run in the same two delta swaps (about 56 VALU for both bitmaps against about 90 for two mask16).
__device__ inline uint32_t tabnl_word(uint32_t w) {  // bit 8b + 3: byte b is a tab; bit 8b + 7: a newline
  const uint32_t t = w ^ 0x08080808u;
  const uint32_t lt4 = ~(((t & 0x7F7F7F7Fu) + 0x7C7C7C7Cu) | t) & 0x80808080u;  // bytes t < 4
  const uint32_t a = t << 7, b = t << 6;
  return ((lt4 & a & ~b) >> 4) | (lt4 & b & ~a);
}
__device__ inline uint32_t mask16x2(uint4 v) {
  uint32_t x = (tabnl_word(v.x) >> 3) | (tabnl_word(v.y) >> 2) | (tabnl_word(v.z) >> 1) | tabnl_word(v.w);
  uint32_t d = ((x >> 4) ^ x) & 0x00F000F0u;  // nibble unshuffle: tab nibbles low, newline nibbles high
  x ^= d ^ (d << 4);
  d = ((x >> 8) ^ x) & 0x0000FF00u;
  x ^= d ^ (d << 8);
  d = (x ^ (x >> 3)) & 0x0A0A0A0Au;  // 4 x 4 transposes: bit 4 b + k -> 4 k + b, both halves
  x ^= d ^ (d << 3);
  d = (x ^ (x >> 6)) & 0x00CC00CCu;
  x ^= d ^ (d << 6);
  return x;
}

// Newlines (bit b = byte b) and line starts of chunk c (bytes v) of the staged tile.  Bytes at
// or past len hold neither; a start needs the byte before it to be '\n' (or the input's start).
__device__ inline void chunk_masks(const uint8_t* buf, uint32_t c, uint64_t t0, uint64_t len, bool tile_prev_nl,
                                   uint32_t& nl, uint32_t& st, uint4 v) {
  nl = mask16(v, 0x0A0A0A0Au);
  const bool prev = c ? buf[16 * c - 1] == '\n' : tile_prev_nl;
  st = ((nl << 1) | (prev ? 1u : 0u)) & 0xFFFFu;
  const uint64_t pos = t0 + 16ull * c;
  if (pos + 16 > len) {
    const uint32_t keep = pos >= len ? 0u : ((1u << (uint32_t)(len - pos)) - 1u);
    nl &= keep;
    st &= keep;
  }
}

struct TileCnt {
  unsigned long long nl, lines, touches, edges, segs, recs;
};
__device__ __host__ inline TileCnt operator+(const TileCnt& a, const TileCnt& b) {
  return TileCnt{a.nl + b.nl, a.lines + b.lines, a.touches + b.touches, a.edges + b.edges, a.segs + b.segs,
                 a.recs + b.recs};
}

template <class T>
__device__ inline T block_sum(T v, T* lds /* >= kTPB / 64 */) {
  v = wave_reduce_sum(v);
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = v;
  __syncthreads();
  T t = 0;
#pragma unroll
  for (int w = 0; w < kTPB / 64; w++) t += lds[w];
  __syncthreads();
  return t;
}

// exclusive scan over the block (thread order) of one u64 per thread; *tot = block total
__device__ inline unsigned long long block_excl_scan_u64(unsigned long long v, unsigned long long* tot,
                                                         unsigned long long* lds /* >= kTPB / 64 */) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  unsigned long long x = v;
  for (int o = 1; o < 64; o <<= 1) {
    unsigned long long y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) lds[wid] = x;
  __syncthreads();
  unsigned long long wbase = 0, t = 0;
#pragma unroll
  for (int q = 0; q < kTPB / 64; q++) {
    const unsigned long long y = lds[q];
    if (q < wid) wbase += y;
    t += y;
  }
  __syncthreads();
  *tot = t;
  return wbase + x - v;
}

// pass 1: per tile, the '\n', lines, touches, edges, S lines and records it holds.  Per-tile
// counts are < 2^16 (32 KiB tiles), so four of them share one block reduction.
__global__ void __launch_bounds__(kTPB) k_tile_count(const uint8_t* __restrict__ in, uint64_t len, uint32_t tps,
                                                     uint32_t tpe, TileCnt* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[kTile + 16];
  __shared__ unsigned long long red[kTPB / 64];
  const uint64_t t0 = (uint64_t)blockIdx.x * kTile;
  {
    TileRegs<16> R;
    R.load(in, len, t0);
    R.store(buf);
  }
  const bool tile_prev_nl = t0 == 0 || in[t0 - 1] == '\n';
  __syncthreads();
  uint32_t nl = 0, lines = 0, edges = 0, segs = 0, po = 0;
#pragma unroll 2
  for (uint32_t j = 0; j < kChunkIters; j++) {
    const uint32_t c = j * kTPB + threadIdx.x;
    uint32_t m, st;
    chunk_masks(buf, c, t0, len, tile_prev_nl, m, st, *(const uint4*)(buf + 16 * c));
    nl += __popc(m);
    lines += __popc(st);
    while (st) {
      const uint32_t o = 16 * c + __builtin_ctz(st);
      st &= st - 1;
      const uint8_t k = kind_at(buf, o, t0 + o, len);
      segs += k == kS;
      edges += k == kEdge;
      po += k == kPO;
    }
  }
  const unsigned long long a = block_sum((unsigned long long)nl | ((unsigned long long)lines << 16) |
                                             ((unsigned long long)segs << 32) | ((unsigned long long)edges << 48),
                                         red);
  const unsigned long long b = block_sum((unsigned long long)po, red);
  if (threadIdx.x == 0) {
    TileCnt cnt;
    cnt.nl = a & 0xFFFF;
    cnt.lines = (a >> 16) & 0xFFFF;
    cnt.segs = (a >> 32) & 0xFFFF;
    cnt.edges = a >> 48;
    cnt.touches = cnt.segs * tps + cnt.edges * tpe;
    cnt.recs = cnt.segs + cnt.edges + b;
    out[blockIdx.x] = cnt;
  }
}

// K1 without LDS (G2N_K1_REG): thread t of a tile's 512 holds the 16-byte chunks t + 512 j in
// registers (coalesced loads), the byte before / after a chunk from lane t - 1 / t + 1 (one global
// byte read per wave and chunk row at each end), each line start's first two bytes picked from the
// registers.  k_tile_count stages the tile in LDS and reads the starts' bytes back from it.
#ifndef G2N_K1_REG
#define G2N_K1_REG 1
#endif
constexpr uint32_t kK1TPB = 512;
constexpr uint32_t kK1Per = (uint32_t)(kTile / 16) / kK1TPB;
__device__ inline uint32_t chunk_byte(uint4 c, uint32_t b) {  // byte b (< 16) of a chunk
  const uint32_t q = b >> 2;
  const uint32_t w = q == 0 ? c.x : q == 1 ? c.y : q == 2 ? c.z : c.w;
  return (w >> (8 * (b & 3u))) & 0xFFu;
}
__global__ void __launch_bounds__(kK1TPB) k_tile_count_r(const uint8_t* __restrict__ in, uint64_t len, uint32_t tps,
                                                         uint32_t tpe, TileCnt* __restrict__ out) {
  __shared__ unsigned long long red[2][kK1TPB / 64];
  const uint64_t t0 = (uint64_t)blockIdx.x * kTile;
  uint4 v[kK1Per];
#pragma unroll
  for (uint32_t j = 0; j < kK1Per; j++) {
    const uint64_t pos = t0 + 16ull * (j * kK1TPB + threadIdx.x);
    v[j] = pos < len ? load16(in, pos, len) : make_uint4(0, 0, 0, 0);
  }
  const int lane = threadIdx.x & 63;
  uint32_t n_nl = 0, n_st = 0, segs = 0, edges = 0, po = 0;
#pragma unroll
  for (uint32_t j = 0; j < kK1Per; j++) {
    const uint64_t r0 = t0 + 16ull * (j * kK1TPB + threadIdx.x);
    uint32_t prev_b = (uint32_t)__shfl_up((int)(v[j].w >> 24), 1, 64);
    uint32_t next_b = (uint32_t)__shfl_down((int)(v[j].x & 0xFFu), 1, 64);
    if (lane == 0) prev_b = r0 == 0 ? (uint32_t)'\n' : (r0 - 1 < len ? in[r0 - 1] : 0u);
    if (lane == 63) next_b = r0 + 16 < len ? in[r0 + 16] : 0u;
    const uint32_t valid = r0 >= len ? 0u : (len - r0 >= 16 ? 0xFFFFu : ((1u << (uint32_t)(len - r0)) - 1u));
    const uint32_t nl = mask16(v[j], 0x0A0A0A0Au) & valid;
    uint32_t st = ((nl << 1) | (prev_b == '\n' ? 1u : 0u)) & valid;
    n_nl += __popc(nl);
    n_st += __popc(st);
    while (st) {
      const uint32_t b = (uint32_t)__builtin_ctz(st);
      st &= st - 1;
      const uint32_t c0 = chunk_byte(v[j], b), c1 = b < 15 ? chunk_byte(v[j], b + 1) : next_b;
      const uint8_t k = line_kind((uint8_t)c0, r0 + b + 1 >= len || c0 == '\n' || c1 == '\t' || c1 == '\n');
      segs += k == kS;
      edges += k == kEdge;
      po += k == kPO;
    }
  }
  unsigned long long a = (unsigned long long)n_nl | ((unsigned long long)n_st << 16) |
                         ((unsigned long long)segs << 32) | ((unsigned long long)edges << 48);
  unsigned long long bpo = po;
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    bpo += __shfl_xor(bpo, o, 64);
  }
  if (lane == 0) {
    red[0][threadIdx.x >> 6] = a;
    red[1][threadIdx.x >> 6] = bpo;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (uint32_t w = 1; w < kK1TPB / 64; w++) {
      a += red[0][w];
      bpo += red[1][w];
    }
    TileCnt cnt;
    cnt.nl = a & 0xFFFF;
    cnt.lines = (a >> 16) & 0xFFFF;
    cnt.segs = (a >> 32) & 0xFFFF;
    cnt.edges = a >> 48;
    cnt.touches = cnt.segs * tps + cnt.edges * tpe;
    cnt.recs = cnt.segs + cnt.edges + bpo;
    out[blockIdx.x] = cnt;
  }
}

// ================================================================ K2: parse =======
__device__ inline void record_error(Ctl* ctl, uint64_t line, uint32_t code) {
  atomicMin(&ctl->err_key, (unsigned long long)((line << 5) | code));
}

struct EdgeLayout {
  uint64_t uo, vo, ouo, ovo;  // offsets (ou/ov may carry kConstFlag)
  uint32_t ul, vl, oul, ovl;
  uint64_t tag_start;          // first tag field start, valid when has_tags
  bool has_tags;
  uint32_t err;                // 0 or an error code
  uint64_t err_off;            // G2N_E_UNICODE: the span whose decode fails
  uint32_t err_len;
};

__device__ inline uint64_t rstrip_pm(const Src& in, uint64_t off, uint64_t len) {
  while (len > 0) {
    uint8_t c = in[off + len - 1];
    if (c != '+' && c != '-') break;
    len--;
  }
  return len;
}

__device__ inline bool int_bytes_ok(const Src& in, uint64_t s, uint64_t e) {
  return py_int_literal(in.ptr(s), e - s, false, nullptr);
}

// Field layout of an L/E/C line [s, e) ('\n' already stripped): parser.py:206-341.
__device__ inline EdgeLayout edge_layout(const Src& in, uint64_t s, uint64_t e) {
  EdgeLayout L;
  L.err = 0;
  L.has_tags = false;
  L.tag_start = e;
  uint64_t fs[10], fe[10];
  int nf = 0;
  uint64_t p = s;
  bool more = true;
  if (e - s <= kMaskSpan) {  // short line: every tab from one register mask
    uint64_t m = delim_mask(in, s, e - s, false);
#pragma unroll
    for (int k = 0; k < 10; k++) {
      fs[k] = e;
      fe[k] = e;
      if (more) {
        fs[k] = p;
        nf = k + 1;
        if (m) {
          fe[k] = s + __builtin_ctzll(m);
          m &= m - 1;
          p = fe[k] + 1;
        } else {
          more = false;
        }
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < 10; k++) {
      fs[k] = e;
      fe[k] = e;
      if (more) {
        fs[k] = p;
        fe[k] = next_tab(in, p, e);
        nf = k + 1;
        if (fe[k] == e) more = false;
        else p = fe[k] + 1;
      }
    }
  }
  const uint8_t t = in[s];
  int tag_from = 0;
  if (t == 'L') {
    if (nf < 5) { L.err = kErrMalformedL; return L; }
    uint8_t c2 = fe[2] > fs[2] ? in[fs[2]] : 0;
    if (fe[2] - fs[2] == 1 && (c2 == '+' || c2 == '-')) {
      L.uo = fs[1]; L.ul = (uint32_t)(fe[1] - fs[1]);
      L.ouo = kConstFlag | c2; L.oul = 1;
      L.vo = fs[3]; L.vl = (uint32_t)(fe[3] - fs[3]);
      L.ovo = fs[4]; L.ovl = (uint32_t)(fe[4] - fs[4]);
      if (!utf8_valid(in.ptr(L.ovo), L.ovl)) { L.err = kErrUnicode; L.err_off = L.ovo; L.err_len = L.ovl; return L; }
      tag_from = 6;
    } else {
      if (fe[1] == fs[1] || fe[2] == fs[2]) { L.err = kErrIndexBytes; return L; }
      uint8_t lu = in[fe[1] - 1], lv = in[fe[2] - 1];
      L.ouo = kConstFlag | ((lu == '+' || lu == '-') ? lu : '+'); L.oul = 1;
      L.ovo = kConstFlag | ((lv == '+' || lv == '-') ? lv : '+'); L.ovl = 1;
      L.uo = fs[1]; L.ul = (uint32_t)rstrip_pm(in, fs[1], fe[1] - fs[1]);
      L.vo = fs[2]; L.vl = (uint32_t)rstrip_pm(in, fs[2], fe[2] - fs[2]);
      tag_from = 4;
    }
  } else {
    const bool isE = t == 'E';
    if (nf < (isE ? 6 : 5)) { L.err = isE ? kErrMalformedE : kErrMalformedC; return L; }
    bool coords = nf >= 9 && int_bytes_ok(in, fs[3], fe[3]) && int_bytes_ok(in, fs[4], fe[4]) &&
                  int_bytes_ok(in, fs[6], fe[6]) && int_bytes_ok(in, fs[7], fe[7]);
    if (coords) {
      uint64_t ul = fe[2] - fs[2], vl = fe[5] - fs[5];
      L.ouo = kConstFlag | ((ul && in[fe[2] - 1] == '-') ? '-' : '+'); L.oul = 1;
      L.ovo = kConstFlag | ((vl && in[fe[5] - 1] == '-') ? '-' : '+'); L.ovl = 1;
      L.uo = fs[2]; L.ul = (uint32_t)rstrip_pm(in, fs[2], ul);
      L.vo = fs[5]; L.vl = (uint32_t)rstrip_pm(in, fs[5], vl);
      tag_from = 9;
    } else if (isE) {
      L.uo = fs[2]; L.ul = (uint32_t)(fe[2] - fs[2]);
      L.ouo = fs[3]; L.oul = (uint32_t)(fe[3] - fs[3]);
      L.vo = fs[4]; L.vl = (uint32_t)(fe[4] - fs[4]);
      L.ovo = fs[5]; L.ovl = (uint32_t)(fe[5] - fs[5]);
      tag_from = 6;
    } else {
      L.uo = fs[1]; L.ul = (uint32_t)(fe[1] - fs[1]);
      L.ouo = fs[2]; L.oul = (uint32_t)(fe[2] - fs[2]);
      L.vo = fs[3]; L.vl = (uint32_t)(fe[3] - fs[3]);
      L.ovo = fs[4]; L.ovl = (uint32_t)(fe[4] - fs[4]);
      tag_from = 5;
    }
    if (!coords) {
      if (!utf8_valid(in.ptr(L.ouo), L.oul)) { L.err = kErrUnicode; L.err_off = L.ouo; L.err_len = L.oul; return L; }
      if (!utf8_valid(in.ptr(L.ovo), L.ovl)) { L.err = kErrUnicode; L.err_off = L.ovo; L.err_len = L.ovl; return L; }
    }
  }
  // fields[tag_from:] (tag_from <= 9, static selects keep fs[] in registers)
  uint64_t ts = e;
  bool have = nf > tag_from;
  switch (tag_from) {
    case 4: ts = fs[4]; break;
    case 5: ts = fs[5]; break;
    case 6: ts = fs[6]; break;
    default: ts = fs[9]; break;
  }
  L.has_tags = have;
  L.tag_start = ts;
  return L;
}

// bits 0..3: which bytes of w are '\t' (tab) or '\t' / '\n' (with_nl)
__device__ inline uint32_t delim_bits4(uint32_t w, bool with_nl) {
  uint32_t m = byte_match_mask(w, 0x09090909u);
  if (with_nl) m |= byte_match_mask(w, 0x0A0A0A0Au);
  return ((m >> 7) & 1u) | ((m >> 14) & 2u) | ((m >> 21) & 4u) | ((m >> 28) & 8u);
}

// Tab bits of bytes [s, s + n), n <= 48: from the tile's tab bitmap when the source has one,
// else from aligned 4-byte words (false when those would read past in.lim).
__device__ inline bool tab_bits(const Src& in, uint64_t s, uint32_t n, uint64_t* out) {
  if (in.tm && s + n <= in.tm_lim) {
    const uint32_t l = (uint32_t)(s - in.o), k = l >> 4, sh = l & 15;
    const uint64_t w = (uint64_t)in.tm[k] | ((uint64_t)in.tm[k + 1] << 16) | ((uint64_t)in.tm[k + 2] << 32) |
                       ((uint64_t)in.tm[k + 3] << 48);
    *out = (w >> sh) & ((1ull << n) - 1);
    return true;
  }
  const uint64_t a = s & ~3ull;
  const uint32_t sh = (uint32_t)(s - a);
  const uint32_t nw = (sh + n + 3) >> 2;
  if (a + 4ull * nw > in.lim) return false;
  uint64_t m = 0;
  for (uint32_t j = 0; j < nw; j++) m |= (uint64_t)delim_bits4(in.word(a + 4ull * j), false) << (4 * j);
  *out = (m >> sh) & ((1ull << n) - 1);
  return true;
}

// The common L line, "L\tu\t[+-]\tv\t[+-]\t<overlap>[\t<tags>]" of at most 48 bytes, in 32-bit
// arithmetic: its tab mask from aligned 4-byte words, then the fields.  Returns false for any
// other shape (the general edge_layout then decides, errors included); when it returns true the
// layout is exactly the one edge_layout gives (parser.py:206-227, the fields[2] in {+,-} branch).
__device__ inline bool link_fast(const Src& in, uint64_t s, uint64_t e, EdgeLayout& L) {
  const uint32_t n = (uint32_t)(e - s);
  uint64_t m;
  if (n > 48 || !tab_bits(in, s, n, &m) || __popcll(m) < 5) return false;
  uint32_t p[6];
  uint64_t r = m;
#pragma unroll
  for (int k = 0; k < 6; k++) {
    p[k] = r ? (uint32_t)__builtin_ctzll(r) : n;
    r &= r - 1;
  }
  if (p[2] - p[1] != 2 || p[4] - p[3] != 2) return false;
  const uint32_t c2 = in[s + p[1] + 1], c4 = in[s + p[3] + 1];
  if ((c2 != '+' && c2 != '-') || (c4 != '+' && c4 != '-')) return false;
  L.err = 0;
  L.uo = s + p[0] + 1;
  L.ul = p[1] - p[0] - 1;
  L.ouo = kConstFlag | c2;
  L.oul = 1;
  L.vo = s + p[2] + 1;
  L.vl = p[3] - p[2] - 1;
  L.ovo = s + p[3] + 1;
  L.ovl = 1;
  L.has_tags = p[5] < n;  // fields[6:]
  L.tag_start = L.has_tags ? s + p[5] + 1 : e;
  return true;
}

__device__ inline bool span_eq(const Src& in, uint64_t off, uint64_t len, const uint8_t* __restrict__ w,
                               uint32_t wl) {
  if (len != wl) return false;
  for (uint32_t k = 0; k < wl; k++)
    if (in[off + k] != w[k]) return false;
  return true;
}

// Weight by the fast grammar.  Returns false when a matching tag needs the exact path.
__device__ inline bool weight_fast(const Src& in, uint64_t ts, uint64_t e, bool has_tags,
                                   const uint8_t* __restrict__ wt, uint32_t wtl, double* w) {
  *w = 1.0;
  if (!has_tags) return true;
  int kind = 0;  // 0 none, 1 number, 2 other
  double num = 1.0;
  uint64_t p = ts;
  while (true) {
    uint64_t fe = next_tab(in, p, e);
    uint64_t c1 = next_byte(in, p, fe, ':');
    if (c1 < fe && c1 - p == wtl && span_eq(in, p, wtl, wt, wtl)) {
      uint64_t c2 = next_byte(in, c1 + 1, fe, ':');
      if (c2 < fe) {
        for (uint64_t q = p; q < fe; q++)
          if (in[q] >= 0x80) return false;
        uint64_t tl = c2 - c1 - 1;
        uint8_t ty = in[c1 + 1];
        if (tl == 1 && ty == 'i') {
          double v;
          if (!fast_int(in.ptr(c2 + 1), fe - c2 - 1, &v)) return false;
          kind = 1;
          num = v;
        } else if (tl == 1 && ty == 'f') {
          double v;
          if (!fast_float(in.ptr(c2 + 1), fe - c2 - 1, &v)) return false;
          kind = 1;
          num = v;
        } else {
          kind = 2;
        }
      }
    }
    if (fe >= e) break;
    p = fe + 1;
  }
  *w = kind == 1 ? num : 1.0;
  return true;
}

__device__ inline void put_touch(const TouchOut& T, uint64_t t, uint64_t no, uint32_t nl, uint64_t oo, uint32_t ol,
                                 bool bidir, uint8_t kind = 2) {
  T.noff[t] = no;
  T.nlen[t] = nl;
  T.tkind[t] = kind;  // 1: S touch (first insert round), 2: edge touch
  if (bidir) {
    T.ooff[t] = oo;
    T.olen[t] = ol;
  }
}

__device__ inline uint64_t rev_ori(const Src& in, uint64_t oo, uint32_t ol) {
  // builders.py:232-233: "-" if orientation == "+" else "+"
  bool plus = (oo & kConstFlag) ? ((oo & 0xFF) == '+') : (ol == 1 && in[oo] == '+');
  return kConstFlag | (plus ? '-' : '+');
}

// Decimal-id dictionary, fused into the parse (ParseOpts.tid).  When the GFA's S lines come
// first and name their segments "1", "2", ..., "N" in order (the layout of vg / odgi / PGGB
// graphs with compacted ids, and of the C4 generator), node ids need no table: Python's dict
// gives S touch t the id t (the S-prefix dictionary), and an edge key equals an S key iff its
// bytes are the canonical decimal of some v in [1, N] (no sign, no leading zero: str(v) is the
// only spelling), plus ":+" / ":-" when bidirected (builders.py:194-198, 211-212).  So each
// edge touch's id is arithmetic on bytes the parse already holds in LDS: v - 1 (bidirected:
// 2(v - 1) + [ori == "-"]).  Any touch that breaks the premise — an S name that is not
// str(k + 1) for its line k, an S touch after an edge touch, an edge key that is no S key (a
// new node: first-touch order matters) — sets ctl->int_fail and the host runs the hash
// dictionary instead.
//
// src_dec: the canonical decimal value of the name [o, o + l) of the source, false when the
// bytes are not one.
__device__ inline bool src_dec(const Src& in, uint64_t o, uint32_t l, uint64_t* v) {
  if (l == 0 || l > 10) return false;
  if (l <= 8) {  // SWAR: two aligned 8-byte reads, digit check and value in registers
    const uint64_t a = o & ~7ull;
    const uint32_t sh = (uint32_t)(o - a) * 8;
    uint64_t w = in.word8_z(a) >> sh;
    if (sh && (o - a) + l > 8) w |= in.word8_z(a + 8) << (64 - sh);
    const uint64_t keep = l == 8 ? ~0ull : ((1ull << (8 * l)) - 1);
    w &= keep;
    const uint64_t zeros = 0x3030303030303030ull & keep;
    if ((w & 0xF0F0F0F0F0F0F0F0ull & keep) != zeros ||
        (((w & 0x0F0F0F0F0F0F0F0Full) + 0x0606060606060606ull) & 0xF0F0F0F0F0F0F0F0ull & keep) != 0 ||
        (w & 0xFF) == '0')
      return false;
    const uint64_t d = (w - zeros) << (8 * (8 - l));  // digits, most significant first, left-padded with 0s
    auto four = [](uint32_t x) {  // 4 digit bytes (most significant lowest) -> their value; shifts, no multiplies
      x = ((x << 3) + (x << 1) + (x >> 8)) & 0x00FF00FFu;
      return ((x << 6) + (x << 5) + (x << 2) + (x >> 16)) & 0xFFFFu;
    };
    *v = (uint64_t)(four((uint32_t)d) * 10000u + four((uint32_t)(d >> 32)));
    return true;
  }
  uint64_t x = 0;
  for (uint32_t j = 0; j < l; j++) {
    const uint32_t c = in[o + j];
    if (c - '0' > 9u || (j == 0 && c == '0')) return false;
    x = x * 10 + (c - '0');
  }
  *v = x;
  return true;
}

// Decimal-id premise state of one thread: fail = a premise broke; in a tile-local parse the
// S-line evidence (value - tile-local index - 1, min / max) and the largest edge-key value, checked
// against the tile bases afterwards (k_tile_lean_check)
constexpr int32_t kNoS = (int32_t)0x80000000;  // IntState.dref: no S line seen yet
struct IntState {
  uint32_t fail = 0;
  uint32_t vmax = 0;    // tile-local: largest edge-key value (< 2^31 by the parse's bound)
  int32_t dref = kNoS;  // tile-local: value - (tile-local S index + 1), the same for every S line
  __device__ void s_name(const ParseOpts& op, uint64_t v, uint64_t tb) {  // S touch tb names v
    if (op.tile_pad) {
      const int32_t d = (int32_t)((int64_t)v - (int64_t)(tb + 1));  // node ids < 2^31, tb < 2^16
      if (v > 0x7FFFFFFFull || (dref != kNoS && d != dref)) fail = 1;
      dref = d;
    } else if (v != op.s_base + tb + 1) {
      fail = 1;
    }
  }
};

// an edge touch's node id from its bytes, or false (no S key: the premise fails)
__device__ inline bool int_edge_id(const Src& in, const ParseOpts& op, uint64_t no, uint32_t nl, uint64_t oo,
                                   uint32_t ol, uint32_t* id, IntState& is) {
  uint64_t v;
  if (!src_dec(in, no, nl, &v) || v < 1 || v > op.n_seg) return false;
  is.vmax = (uint32_t)v > is.vmax ? (uint32_t)v : is.vmax;
  *id = (uint32_t)(v - 1);
  if (op.bidir) {
    const uint32_t oc = (oo & kConstFlag) ? (uint32_t)(oo & 0xFF) : (ol ? (uint32_t)in[oo] : 0u);
    if (ol != 1 || (oc != '+' && oc != '-')) return false;
    *id = 2 * *id + (oc == '-');
  }
  return true;
}

// S line i, name = [ns, ne): parser.py:163, builders.py:190-198
__device__ inline void put_segment(const Src& in, const ParseOpts& op, const TouchOut& T, uint64_t tb, uint64_t eb,
                                   uint64_t ns, uint64_t ne, IntState& is) {
  const uint32_t nl = (uint32_t)(ne - ns);
  if (op.tile_pad) {  // tile-local lean parse: no touch descriptors (tb is tile-local)
  } else if (!op.bidir) {
    put_touch(T, tb, ns, nl, 0, 0, false, 1);
  } else {
    put_touch(T, tb, ns, nl, kConstFlag | '+', 1, true, 1);
    put_touch(T, tb + 1, ns, nl, kConstFlag | '-', 1, true, 1);
  }
  if (op.tid && !is.fail) {  // no edge line before it (eb = 0), so S touch tb is node tb: its name
                              // must be str(k + 1), k = tb / tps = the S lines before it
    uint64_t v;  // (s_base: S lines of earlier ranges)
    if (eb != 0 || !src_dec(in, ns, nl, &v)) is.fail = 1;
    else is.s_name(op, v, op.bidir ? tb >> 1 : tb);
  }
}

// L / E / C line i = [s, e) ('\n' stripped), its touches from tb, its edge eb
__device__ inline void parse_edge(const Src& in, uint64_t i, uint64_t s, uint64_t e, uint64_t tb, uint64_t eb,
                                  const ParseOpts& op, const TouchOut& T, const EdgeOut& E, Ctl* ctl,
                                  uint64_t* __restrict__ worklist, IntState& is) {
  EdgeLayout L;
  if (!link_fast(in, s, e, L)) L = edge_layout(in, s, e);
  if (L.err) {
    record_error(ctl, i, L.err);
    return;
  }
  if (op.strip) {  // builders.py:202-204
    L.ul = (uint32_t)rstrip_pm(in, L.uo, L.ul);
    L.vl = (uint32_t)rstrip_pm(in, L.vo, L.vl);
  }
  double w = 1.0;
  if (op.has_wt) {
    if (!weight_fast(in, L.tag_start, e, L.has_tags, op.wt, op.wt_len, &w)) {
      unsigned long long slot = atomicAdd(&ctl->wl_count, 1ull);
      worklist[2 * slot] = i;
      worklist[2 * slot + 1] = eb;
      w = 0.0;
    }
  }
  if (op.rows) {  // lean: ids straight into the COO coordinates (k_triplets' layout)
    if (op.has_wt) E.w[eb] = w;
    if (op.tile_pad && eb >= op.tile_pad) is.fail = 1;  // the tile's slot is full: give up
    if (is.fail) return;
    uint32_t a, b, c = 0, d = 0;
    bool ok = int_edge_id(in, op, L.uo, L.ul, L.ouo, L.oul, &a, is) && int_edge_id(in, op, L.vo, L.vl, L.ovo, L.ovl, &b, is);
    if (ok && op.ktrip == 4)
      ok = int_edge_id(in, op, L.vo, L.vl, rev_ori(in, L.ovo, L.ovl), 1, &c, is) &&
           int_edge_id(in, op, L.uo, L.ul, rev_ori(in, L.ouo, L.oul), 1, &d, is);
    if (!ok) {
      is.fail = 1;
      return;
    }
    const uint64_t o = ((op.tile_pad ? (uint64_t)blockIdx.x * op.tile_pad : 0ull) + eb) * op.ktrip;
    op.rows[o] = (int32_t)a;
    op.cols[o] = (int32_t)b;
    if (op.ktrip >= 2) {
      op.rows[o + 1] = (int32_t)b;
      op.cols[o + 1] = (int32_t)a;
    }
    if (op.ktrip == 4) {
      op.rows[o + 2] = (int32_t)c;
      op.cols[o + 2] = (int32_t)d;
      op.rows[o + 3] = (int32_t)d;
      op.cols[o + 3] = (int32_t)c;
    }
    return;
  }
  E.w[eb] = w;
  E.tb[eb] = (uint32_t)tb;
  if (!op.bidir) {
    put_touch(T, tb, L.uo, L.ul, 0, 0, false);
    put_touch(T, tb + 1, L.vo, L.vl, 0, 0, false);
  } else {
    put_touch(T, tb, L.uo, L.ul, L.ouo, L.oul, true);
    put_touch(T, tb + 1, L.vo, L.vl, L.ovo, L.ovl, true);
    if (!op.keep) {  // builders.py:231-234: v:rev(ori_to), u:rev(ori_from)
      put_touch(T, tb + 2, L.vo, L.vl, rev_ori(in, L.ovo, L.ovl), 1, true);
      put_touch(T, tb + 3, L.uo, L.ul, rev_ori(in, L.ouo, L.oul), 1, true);
    }
  }
  if (op.tid && !is.fail) {
    uint32_t a, b, c = 0, d = 0;
    bool ok = int_edge_id(in, op, L.uo, L.ul, L.ouo, L.oul, &a, is) && int_edge_id(in, op, L.vo, L.vl, L.ovo, L.ovl, &b, is);
    if (ok && op.bidir && !op.keep)
      ok = int_edge_id(in, op, L.vo, L.vl, rev_ori(in, L.ovo, L.ovl), 1, &c, is) &&
           int_edge_id(in, op, L.uo, L.ul, rev_ori(in, L.ouo, L.oul), 1, &d, is);
    if (!ok) {
      is.fail = 1;
    } else {
      op.tid[tb] = a;
      op.tid[tb + 1] = b;
      if (op.bidir && !op.keep) {
        op.tid[tb + 2] = c;
        op.tid[tb + 3] = d;
      }
    }
  }
}

// Line i of kind k starting at s.  The source holds the bytes [.., bound); when nl_at_bound
// the line's '\n' is byte bound - 1 (its end is known).  Returns false when the line's fields
// run past bound < len: the line is deferred.
__device__ inline bool parse_line(const Src& in, uint64_t len, uint64_t bound, bool nl_at_bound, uint64_t i,
                                  uint8_t k, uint64_t s, uint64_t tb, uint64_t eb, const ParseOpts& op,
                                  const TouchOut& T, const EdgeOut& E, Ctl* ctl, uint64_t* __restrict__ worklist,
                                  IntState& is) {
  const bool cut = bound < len;
  if (k == kS || k == kPO) {  // the first two (S) / three (P, O) fields
    uint64_t t1 = bound, t2 = bound;
    uint64_t tb_m;
    if (nl_at_bound && bound - 1 - s <= 48 && tab_bits(in, s, (uint32_t)(bound - 1 - s), &tb_m)) {
      // the whole line's tabs from the tile bitmap; its '\n' (byte bound - 1) ends the fields
      const uint64_t nl = bound - 1;
      t1 = tb_m ? s + __builtin_ctzll(tb_m) : nl;
      tb_m &= tb_m - 1;
      t2 = t1 == nl ? bound : (tb_m ? s + __builtin_ctzll(tb_m) : nl);
    } else {  // the first two delimiters, 4-byte words at a time (stops at the second, or after 64 bytes)
      const uint64_t lim = (bound < s + kMaskSpan ? bound : s + kMaskSpan);
      uint32_t found = 0;
      for (uint64_t a = s & ~3ull; a < lim && found < 2 && a + 4 <= in.lim; a += 4) {
        uint32_t b = delim_bits4(in.word(a), true);
        if (a < s) b &= 0xFu << (uint32_t)(s - a);
        if (a + 4 > lim) b &= (1u << (uint32_t)(lim - a)) - 1u;
        while (b && found < 2) {
          const uint64_t q = a + (uint64_t)__builtin_ctz(b);
          b &= b - 1;
          if (found++ == 0) t1 = q;
          else t2 = q;
        }
      }
      if (found < 2) t1 = t2 = bound;
    }
    if (t2 == bound) {  // not both delimiters among the first 64 bytes
      t1 = next_delim(in, s, bound);
      if (t1 == bound && cut) return false;
      t2 = t1 < bound ? next_delim(in, t1 + 1, bound) : bound;
    }
    if (t1 == bound || in[t1] == '\n') {  // one field: parser.py:163 IndexError / :231 too few fields
      record_error(ctl, i, k == kS ? kErrIndexList : (in[s] == 'P' ? kErrMalformedP : kErrMalformedO));
      return true;
    }
    if (t2 == bound && cut) return false;
    if (k == kS) {
      put_segment(in, op, T, tb, eb, t1 + 1, t2, is);
    } else if (t2 == bound || in[t2] == '\n') {
      record_error(ctl, i, in[s] == 'P' ? kErrMalformedP : kErrMalformedO);
    }
    return true;
  }
  const uint64_t e = nl_at_bound ? bound - 1 : next_nl(in, s, bound);
  if (e == bound && cut) return false;
  parse_edge(in, i, s, e, tb, eb, op, T, E, ctl, worklist, is);
  return true;
}

// Lean decimal-id parse (ParseOpts.rows, not bidirected, no weight tag, no strip) of the two
// common shapes, in tile-local 32-bit arithmetic straight from the staged tile: an S line
// "S\t<name>[\t...]" and the L / E / C line link_fast accepts, at most 48 bytes before the '\n'
// at next - 1 (the next line's start in the same tile).  Same results as parse_line's
// put_segment / link_fast + int_edge_id path for these lines; false for anything else (the
// general path then parses the line).
__device__ inline bool dec_lds(const uint8_t* buf, uint32_t x, uint32_t l, uint64_t* v) {
  if (l == 0 || l > 10) return false;
  if (l > 8) {  // 9-10 digits (src_dec's loop)
    uint64_t y = 0;
    for (uint32_t j = 0; j < l; j++) {
      const uint32_t c = buf[x + j];
      if (c - '0' > 9u || (j == 0 && c == '0')) return false;
      y = y * 10 + (c - '0');
    }
    *v = y;
    return true;
  }
  const uint32_t a = x & ~7u, sh = (x - a) * 8;
  uint64_t w = *(const uint64_t*)(buf + a) >> sh;
  if (sh && (x - a) + l > 8) w |= *(const uint64_t*)(buf + a + 8) << (64 - sh);
  const uint64_t keep = l == 8 ? ~0ull : ((1ull << (8 * l)) - 1);
  w &= keep;
  const uint64_t zeros = 0x3030303030303030ull & keep;
  if ((w & 0xF0F0F0F0F0F0F0F0ull & keep) != zeros ||
      (((w & 0x0F0F0F0F0F0F0F0Full) + 0x0606060606060606ull) & 0xF0F0F0F0F0F0F0F0ull & keep) != 0 ||
      (w & 0xFF) == '0')
    return false;
  const uint64_t d = (w - zeros) << (8 * (8 - l));
  auto four = [](uint32_t y) {
    y = ((y << 3) + (y << 1) + (y >> 8)) & 0x00FF00FFu;
    return ((y << 6) + (y << 5) + (y << 2) + (y >> 16)) & 0xFFFFu;
  };
  *v = (uint64_t)(four((uint32_t)d) * 10000u + four((uint32_t)(d >> 32)));
  return true;
}

// The first p <= 8 bytes at tile offset x of the staged tile, little-endian (aligned 8-byte LDS reads)
__device__ inline uint64_t lds_prefix8(const uint8_t* buf, uint32_t x, uint32_t p) {
  const uint32_t a = x & ~7u, sh = (x & 7u) * 8;
  uint64_t w = *(const uint64_t*)(buf + a) >> sh;
  if (sh && (x & 7u) + p > 8) w |= *(const uint64_t*)(buf + a + 8) << (64 - sh);
  return p >= 8 ? w : (w & ((1ull << (8 * p)) - 1));
}

// a segment name of the decimal-id layout at tile offset x (length l): op.dpre then the canonical
// decimal (no prefix: the decimal alone) — its value
__device__ inline bool dec_name(const uint8_t* buf, uint32_t x, uint32_t l, const ParseOpts& op, uint64_t* v) {
  const uint32_t p = op.dpre_len;
  if (p) {
    if (l <= p || lds_prefix8(buf, x, p) != op.dpre) return false;
    x += p;
    l -= p;
  }
  return dec_lds(buf, x, l, v);
}

// dec_lds's 1-8 digit case on words already loaded: w0 / w1 = the aligned 8-byte LDS words at
// (x & ~7) and (x & ~7) + 8.  false for anything else (the caller takes dec_lds for 9-10 digits).
__device__ inline bool dec_words(uint64_t w0, uint64_t w1, uint32_t x, uint32_t l, uint64_t* v) {
  if (l == 0 || l > 8) return false;
  const uint32_t sh = (x & 7u) * 8;
  uint64_t w = w0 >> sh;
  if (sh && (x & 7u) + l > 8) w |= w1 << (64 - sh);
  const uint64_t keep = l == 8 ? ~0ull : ((1ull << (8 * l)) - 1);
  w &= keep;
  const uint64_t zeros = 0x3030303030303030ull & keep;
  if ((w & 0xF0F0F0F0F0F0F0F0ull & keep) != zeros ||
      (((w & 0x0F0F0F0F0F0F0F0Full) + 0x0606060606060606ull) & 0xF0F0F0F0F0F0F0F0ull & keep) != 0 ||
      (w & 0xFF) == '0')
    return false;
  const uint64_t d = (w - zeros) << (8 * (8 - l));
  auto four = [](uint32_t y) {
    y = ((y << 3) + (y << 1) + (y >> 8)) & 0x00FF00FFu;
    return ((y << 6) + (y << 5) + (y << 2) + (y >> 16)) & 0xFFFFu;
  };
  *v = (uint64_t)(four((uint32_t)d) * 10000u + four((uint32_t)(d >> 32)));
  return true;
}

// tab bits of the 64 staged bytes from chunk q: from the tile's tab bitmap, or (tabm == nullptr)
// recomputed from the staged bytes (the LDS-lean instance keeps no bitmap)
#ifndef G2N_TAB_B64  // 1: the window from two aligned 8-byte LDS reads (C4 parse 3.47 -> 3.43 ms); 0: four u16 reads
#define G2N_TAB_B64 1
#endif
__device__ inline uint64_t tab_window(const uint8_t* buf, const uint16_t* tabm, uint32_t q) {
#if G2N_TAB_B64
  if (tabm) {  // tabm is 16-byte aligned with 8 entries of padding past its last window
    const uint32_t a = q & ~3u, sh = (q & 3u) * 16;
    const uint64_t lo = *(const uint64_t*)(tabm + a), hi = *(const uint64_t*)(tabm + a + 4);
    return sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
  }
#endif
  if (tabm)
    return (uint64_t)tabm[q] | ((uint64_t)tabm[q + 1] << 16) | ((uint64_t)tabm[q + 2] << 32) |
           ((uint64_t)tabm[q + 3] << 48);
  uint64_t w = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) w |= (uint64_t)mask16(*(const uint4*)(buf + 16 * (q + i)), 0x09090909u) << (16 * i);
  return w;
}

// "<tag>:i:<int>" at tile offset x, length l: the weight float(int(value)) the reference takes
// (parser.py:179-204, builders.py:205-209) for the canonical spellings only — an optional '-' and 1-9
// digits without a leading zero; any other spelling (CPython's int() accepts more) or tag is false
// (the full parse decides)
__device__ inline bool lean_int_tag(const uint8_t* buf, uint32_t x, uint32_t l, uint32_t tl, uint64_t wt_pack,
                                    double* w) {
  if (tl == 0 || tl > 8 || l < tl + 4) return false;
  for (uint32_t k = 0; k < tl; k++)
    if (buf[x + k] != (uint8_t)(wt_pack >> (8 * k))) return false;
  if (buf[x + tl] != ':' || buf[x + tl + 1] != 'i' || buf[x + tl + 2] != ':') return false;
  uint32_t j = x + tl + 3, e = x + l;
  const bool neg = buf[j] == '-';
  j += neg ? 1u : 0u;
  const uint32_t nd = e - j;
  if (nd == 0 || nd > 9 || (buf[j] == '0' && nd > 1)) return false;
  int64_t v = 0;
  for (; j < e; j++) {
    const uint32_t c = buf[j];
    if (c - '0' > 9u) return false;
    v = v * 10 + (c - '0');
  }
  *w = (double)(neg ? -v : v);
  return true;
}

// An L / E / C line in the link_fast shape "L\t<a>\t<o>\t<b>\t<o>[\t...]" from its tab bits m (bit k =
// byte so + k; the '\n' excluded): the two names' lengths.  The record-kind check put a tab at byte 1
// (a '\n' there leaves m without a name: false), so the five tabs are byte 1; p1 = the first after it;
// p1 + 2 (the orientation byte between must be '+' / '-'); p3 = the first after p1 + 2; p3 + 2 — two
// ctz instead of one per tab (round 6).  Name a at so + 2, length la; name b at so + 5 + la, length lb.
__device__ __forceinline__ bool lean_link(const uint8_t* buf, uint64_t m, uint32_t so, uint32_t& la, uint32_t& lb) {
  m >>= 2;  // tabs from byte 2: the first name's
  if (!m) return false;
  la = (uint32_t)__builtin_ctzll(m);  // < 46
  if (!((m >> (la + 2)) & 1)) return false;
  const uint64_t m2 = m >> (la + 3);  // from the second name
  if (!m2) return false;
  lb = (uint32_t)__builtin_ctzll(m2);
  if (!((m2 >> (lb + 2)) & 1)) return false;
  const uint32_t c2 = buf[so + 3 + la], c4 = buf[so + 6 + la + lb];
  return (c2 == '+' || c2 == '-') && (c4 == '+' || c4 == '-');
}

// 64 bits of v (128 bits: lo, hi) from bit sh in [0, 63], without a branch on sh == 0
__device__ __forceinline__ uint64_t funnel64(uint64_t lo, uint64_t hi, uint32_t sh) {
  return (lo >> sh) | ((hi << 1) << (63u - sh));
}

// 4 digit values (bytes, the first in byte 0) -> their decimal value, all full-rate: the two pairs' values
// by 4-way byte dot products (b0 * 10 + b1, b2 * 10 + b3: <= 99, no carry), packed, then one 2-way
// 16-bit dot product (pair 0 * 100 + pair 1)
typedef unsigned short g2n_u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t dig4(uint32_t x) {
  const uint32_t p = __builtin_amdgcn_udot4(x, 0x0000010Au, 0u, false) |
                     (__builtin_amdgcn_udot4(x, 0x010A0000u, 0u, false) << 16);
  return __builtin_amdgcn_udot2(__builtin_bit_cast(g2n_u16x2, p), __builtin_bit_cast(g2n_u16x2, 0x00010064u), 0u,
                                false);
}

// dec_lds's canonical decimal of 1-10 digits at tile offset x, length l, as straight-line code (round 6):
// the last min(l, 8) digits from one 16-byte window (their value by dot products); the first one or two
// of a 9-10 digit name from two byte loads, only in a wave that has such a name (C4's ids have at most 8
// digits, C5's up to 9).  *ok false for another length, a byte that is not a digit, a leading '0' or a
// 10-digit value past 2.2e9 (no segment index; the caller's n_seg bound rejects the rest).  xmax: the
// last offset the staged tile may be read at (addresses of a failed line are clamped).
__device__ __forceinline__ uint32_t dec10_flat(const uint8_t* buf, uint32_t x, uint32_t l, uint32_t xmax, bool* ok) {
  x = x < xmax ? x : xmax;
  const bool longer = l - 9u < 2u;  // 9 or 10 digits
  const uint32_t lt = l < 8u ? l : 8u, lc = lt ? lt : 1u;
  const uint32_t xt = x + (longer ? l - 8u : 0u);  // the last lt digits
  const uint32_t* wp = (const uint32_t*)(buf + (xt & ~3u));  // three dwords hold the 8 bytes from xt
  const uint32_t w0 = wp[0], w1 = wp[1], w2 = wp[2], sb = (xt & 3u) * 8u;
  const uint64_t keep = ~0ull >> (64u - 8u * lc);
  const uint64_t w = (((uint64_t)__builtin_amdgcn_alignbit(w2, w1, sb) << 32) | __builtin_amdgcn_alignbit(w1, w0, sb)) & keep;
  const uint64_t dv = w & 0x0F0F0F0F0F0F0F0Full;
  bool good = (l - 1u < 10u) & ((w & 0xF0F0F0F0F0F0F0F0ull) == (0x3030303030303030ull & keep)) &
              (((dv + 0x0606060606060606ull) & 0xF0F0F0F0F0F0F0F0ull) == 0) & (longer | ((w & 0xFFu) != '0'));
  uint32_t head = 0;
  if (__any(longer)) {  // (wave-uniform)
    const uint32_t h0 = (uint32_t)buf[x] - '0', h1 = (uint32_t)buf[x + 1] - '0';
    good = good & (!longer | ((h0 - 1u <= 8u) & ((l == 9u) | ((h1 <= 9u) & (h0 * 10u + h1 <= 21u)))));
    head = longer ? (l == 10u ? h0 * 10u + h1 : h0) & 0x7Fu : 0u;  // (<= 21 when good)
  }
  *ok = good;
  const uint64_t d = dv << (8u * (8u - lc));  // the units digit in byte 7
  // (head * 10^4 + digits 1-4 of the tail) * 10^4 + digits 5-8: two 24-bit multiply-adds
  return ((head * 10000u + (dig4((uint32_t)d) & 0x3FFFu)) & 0xFFFFFFu) * 10000u + dig4((uint32_t)(d >> 32));
}

// An edge line of an edge-only tile (k_tile_lean's edge-only loop): lean_line<false>'s edge shape and
// checks as straight-line code — one verdict, every LDS load of the line issued before any check (the
// exec-mask bookkeeping of early returns was most of the loop's scalar instructions, and each early
// return serialised the next load behind it).  next == 0: past the staged window (fails).  Returns false
// when the general path must decide (the caller fails the tile); *a / *b the name values.
__device__ __forceinline__ bool lean_edge_flat(const uint8_t* buf, const uint16_t* tabm, uint32_t o, uint32_t next,
                                               const ParseOpts& op, uint32_t xmax, uint64_t* a, uint64_t* b) {
  const uint32_t n = next - 1u - o;  // (next == 0: huge)
  const uint32_t q = o >> 4;
  const uint32_t* tp = (const uint32_t*)(tabm + (q & ~1u));  // three dwords: chunks q & ~1 .. + 5
  const uint32_t t0 = tp[0], t1 = tp[1], t2 = tp[2], tb = (q & 1u) * 16u + (o & 15u);
  const uint64_t w = ((uint64_t)__builtin_amdgcn_alignbit(t2, t1, tb) << 32) | __builtin_amdgcn_alignbit(t1, t0, tb);
  const uint32_t nc = n < 48u ? (n ? n : 1u) : 48u;
  const uint64_t m1 = (w & (~0ull >> (64u - nc))) >> 2;  // tabs from byte 2 (byte 1's is the record check's)
  const uint32_t la = m1 ? (uint32_t)__builtin_ctzll(m1) : 60u;
  const uint64_t m2 = m1 >> (la + 3u);  // (la <= 60) tabs from the second name
  const uint32_t lb = m2 ? (uint32_t)__builtin_ctzll(m2) : 0u;
  const uint32_t oa = o + 3u + la, ob = o + 6u + la + lb;  // the orientation bytes
  const uint32_t c2 = buf[oa < xmax ? oa : xmax], c4 = buf[ob < xmax ? ob : xmax];
  // a tab after each orientation byte (a zero m1 / m2 has none either), each orientation '+' or '-'
  bool ok = (n - 2u < 47u) & (((m1 >> (la + 2u)) & 1u) != 0) & (((m2 >> (lb + 2u)) & 1u) != 0) &
            (((c2 - '+') & ~2u) == 0) & (((c4 - '+') & ~2u) == 0);
  uint32_t xa = o + 2u, xb = o + 5u + la, lna = la, lnb = lb;
  if (op.dpre_len) {  // (uniform) the names' constant prefix
    const uint32_t p = op.dpre_len;
    const uint32_t pa = xa < xmax ? xa : xmax, pb = xb < xmax ? xb : xmax;
    const uint64_t wa = lds_prefix8(buf, pa, p), wb = lds_prefix8(buf, pb, p);
    ok = ok & (lna > p) & (lnb > p) & (wa == op.dpre) & (wb == op.dpre);
    xa += p;
    xb += p;
    lna -= p;
    lnb -= p;
  }
  bool oka, okb;
  *a = dec10_flat(buf, xa, lna, xmax, &oka);
  *b = dec10_flat(buf, xb, lnb, xmax, &okb);
  return ok & oka & okb;
}

// kExt: the extended instance (bidirected keys, one integer weight tag), tile-local builds only
template <bool kExt = false>
__device__ inline bool lean_line(const uint8_t* buf, const uint16_t* tabm, uint32_t so, uint32_t next, uint8_t k,
                                 uint64_t t0, uint64_t tb, uint64_t eb, const ParseOpts& op, const TouchOut& T,
                                 IntState& is) {
  const uint32_t n = next - 1 - so;
  if (n > 48 && k != kS) return false;
  const uint32_t sh = so & 15;
  const uint64_t w = tab_window(buf, tabm, so >> 4);
  uint64_t m = (w >> sh) & ((1ull << (n > 48 ? 48 : n)) - 1);
  if (k == kS) {  // the name is all it needs: any length, as long as both its tabs are in view
    if (!m) return false;  // one field (or a name past the view): the general path decides
    const uint32_t t1 = (uint32_t)__builtin_ctzll(m);
    m &= m - 1;
    if (!m && n > 48) return false;
    const uint32_t t2 = m ? (uint32_t)__builtin_ctzll(m) : n;
    // no touch descriptor: a lean build that holds its premise derives the names (k_names_dec);
    // one that breaks it re-parses in full
    if (op.tid && !is.fail) {
      uint64_t v;
      if (eb != 0 || !dec_name(buf, so + t1 + 1, t2 - t1 - 1, op, &v)) is.fail = 1;
      else is.s_name(op, v, tb);
    }
    return true;
  }
  if (k != kEdge) return false;
  if constexpr (!kExt && G2N_LEAN_LINK) {  // the plain decimal build: two tab searches (lean_link)
    uint32_t la, lb;
    if (!lean_link(buf, m, so, la, lb)) return false;
    if (op.tile_pad && eb >= op.tile_pad) is.fail = 1;  // the tile's slot is full: give up
    if (is.fail) return true;
    uint64_t a, b;
    if (!dec_name(buf, so + 2, la, op, &a) || !dec_name(buf, so + 5 + la, lb, op, &b) || a > op.n_seg ||
        b > op.n_seg) {  // not an S key: the premise breaks (int_edge_id)
      is.fail = 1;
      return true;
    }
    const uint32_t vm = (uint32_t)(a > b ? a : b);
    is.vmax = vm > is.vmax ? vm : is.vmax;
    const uint64_t o = ((op.tile_pad && !op.grouped ? (uint64_t)blockIdx.x * op.tile_pad : 0ull) + eb) * op.ktrip;
    op.rows[o] = (int32_t)(a - 1);
    op.cols[o] = (int32_t)(b - 1);
    if (op.ktrip >= 2) {
      op.rows[o + 1] = (int32_t)(b - 1);
      op.cols[o + 1] = (int32_t)(a - 1);
    }
    return true;
  }
  if (__popcll(m) < 5) return false;
  uint32_t p[6];
#pragma unroll
  for (int j = 0; j < 6; j++) {
    p[j] = m ? (uint32_t)__builtin_ctzll(m) : n;
    m &= m - 1;
  }
  if (p[2] - p[1] != 2 || p[4] - p[3] != 2) return false;
  const uint32_t c2 = buf[so + p[1] + 1], c4 = buf[so + p[3] + 1];
  if ((c2 != '+' && c2 != '-') || (c4 != '+' && c4 != '-')) return false;
  if (op.tile_pad && eb >= op.tile_pad) is.fail = 1;  // the tile's slot is full: give up
  if (is.fail) return true;
  uint64_t a, b;
  if (!dec_name(buf, so + p[0] + 1, p[1] - p[0] - 1, op, &a) || !dec_name(buf, so + p[2] + 1, p[3] - p[2] - 1, op, &b) ||
      a > op.n_seg || b > op.n_seg) {  // not an S key: the premise breaks (int_edge_id)
    is.fail = 1;
    return true;
  }
  const uint32_t vm = (uint32_t)(a > b ? a : b);
  is.vmax = vm > is.vmax ? vm : is.vmax;
  const uint64_t e = (op.tile_pad && !op.grouped ? (uint64_t)blockIdx.x * op.tile_pad : 0ull) + eb;
  const uint64_t o = e * op.ktrip;
  if constexpr (kExt) {
    if (op.has_wt) {  // builders.py:205-209: the tag's value, or 1.0 without it
      double wv = 1.0;
      if (p[5] < n) {  // a field after the overlap: exactly one, the weight tag
        if (m || !lean_int_tag(buf, so + p[5] + 1, n - p[5] - 1, op.wt_len, op.wt_pack, &wv)) {
          is.fail = 1;
          return true;
        }
      }
      if (op.wenc) {  // (grouped) the code beside each of the edge's triplets
        const uint32_t code = op.wf32 ? (uint32_t)(int32_t)(float)wv : (uint32_t)(int32_t)wv;  // |wv| < 10^9
        for (uint32_t k = 0; k < op.ktrip; k++) op.wenc[o + k] = code;
      } else {
        op.ew[e] = wv;
      }
    }
    if (op.bidir) {  // builders.py:211-234: "name:o" keys, S line k minting 2k (+) and 2k + 1 (-)
      const uint32_t ia = 2u * (uint32_t)(a - 1) + (c2 == '-'), ib = 2u * (uint32_t)(b - 1) + (c4 == '-');
      op.rows[o] = (int32_t)ia;
      op.cols[o] = (int32_t)ib;
      if (op.ktrip == 4) {  // undirected (b, a), then the reverse twin (v:rev, u:rev) both ways
        op.rows[o + 1] = (int32_t)ib;
        op.cols[o + 1] = (int32_t)ia;
        op.rows[o + 2] = (int32_t)(ib ^ 1u);
        op.cols[o + 2] = (int32_t)(ia ^ 1u);
        op.rows[o + 3] = (int32_t)(ia ^ 1u);
        op.cols[o + 3] = (int32_t)(ib ^ 1u);
      }
      return true;
    }
  }
  op.rows[o] = (int32_t)(a - 1);
  op.cols[o] = (int32_t)(b - 1);
  if (op.ktrip >= 2) {
    op.rows[o + 1] = (int32_t)(b - 1);
    op.cols[o + 1] = (int32_t)(a - 1);
  }
  return true;
}

struct DeferredLine {  // at most one per tile: the line holding the tile window's last byte
  unsigned long long line;
  unsigned long long start;
  uint32_t tb, eb;
  uint32_t kind, pad_;
};

// pass 2: line starts, kinds, touches, edges of every line starting in the tile.
//  (1) one block scan over the tile's chunks' start counts ranks every line start;
//  (2) per window of kTileLines starts: the starts go to an LDS list, threads classify
//      kLinesPer consecutive lines each and one block scan gives each line its S / edge prefix;
//  (3) lanes take consecutive lines and parse them from the staged bytes (no barriers).
// The tile bases come from K1's counts (exclusive scan).  A single pass that learns them from a
// decoupled look-back over the tiles instead (no K1) measured 12.0 ms on C4 against 2.2 + 6.3
// ms: in-order waiting across the 8 XCDs (status words polled past the non-coherent L2s) stalls
// every tile behind the slowest.
// The tile-local lean instance parses every line through the lean shapes (a line outside them
// gives that parse up: the full parse runs instead), so it carries none of the general parser's
// registers (166 -> 116 VGPRs; parse 5.64 -> 5.45 ms on C4).  0: the general parser inline.
#ifndef G2N_LEAN_ONLY
#define G2N_LEAN_ONLY 1
#endif
#ifndef G2N_LEAN_LDS  // experiment: the LDS-lean tile-local instance (4 blocks per CU)
#define G2N_LEAN_LDS 0
#endif
constexpr uint32_t kTileLines = kTileChunks;            // line starts per window (= chunks: pre[] holds both)
constexpr uint32_t kLinesPer = kTileLines / kTPB;       // lines classified per thread
static_assert(kChunkIters % 4 == 0 && kTile <= 32768, "tile layout: per-tile counts fit 16 bits");

// Diagnostics build only (-DG2N_K2_STAMPS, tools/k2_stamps.py): per tile, the wall clock at the
// block's phase boundaries (thread 0) and the hardware id of the CU it ran on.
#ifdef G2N_K2_STAMPS
constexpr int kK2Stamps = 10;
__device__ unsigned long long* g2n_k2_stamps;
#define K2_STAMP(k)                                                                               \
  do {                                                                                            \
    if (kLocal && threadIdx.x == 0) g2n_k2_stamps[blockIdx.x * kK2Stamps + (k)] = wall_clock64(); \
  } while (0)
#define K2_LEAN_STAMP(k)                                                                 \
  do {                                                                                   \
    if (threadIdx.x == 0) g2n_k2_stamps[tile * kK2Stamps + (k)] = wall_clock64();        \
  } while (0)
#else
#define K2_STAMP(k) \
  do {              \
  } while (0)
#define K2_LEAN_STAMP(k) \
  do {                   \
  } while (0)
#endif

// kLocal: the tile-local lean parse (ParseOpts.tile_pad; lean, not bidirected, no weight tag, no
// strip — fixed at compile time, so that instance carries none of the other paths' code)
template <bool kLocal>
__global__ void __launch_bounds__(kTPB) k_tile_parse(const uint8_t* __restrict__ in, uint64_t len,
                                                     const TileCnt* __restrict__ base, uint32_t tps, uint32_t tpe,
                                                     ParseOpts op, uint64_t* __restrict__ ls,
                                                     uint8_t* __restrict__ kind, TouchOut T, EdgeOut E, Ctl* ctl,
                                                     uint64_t* __restrict__ worklist,
                                                     DeferredLine* __restrict__ deferred, uint64_t n_tiles,
                                                     TileCnt* __restrict__ tcnt_out, TileLean* __restrict__ tlean) {
  // kDiet (the LDS-lean tile-local instance): half-size line windows, u16 chunk ranks aliased with
  // the u32 line prefixes, no kind array and no tab bitmap (both re-read from the staged bytes)
  constexpr bool kDiet = kLocal && G2N_LEAN_LDS;
  constexpr uint32_t kWinL = kDiet ? kTileLines / 2 : kTileLines;
  constexpr uint32_t kLinesPerW = kWinL / kTPB;
  __shared__ __attribute__((aligned(16))) uint8_t buf[kTile + kTileHalo + 16];
  __shared__ __attribute__((aligned(16))) uint16_t starts[kWinL];
  __shared__ __attribute__((aligned(16))) uint32_t pre[kDiet ? kTileChunks / 2 : kTileChunks];  // chunk ranks, then line prefixes
  uint16_t* const pre16 = (uint16_t*)pre;
  __shared__ uint8_t lkind[kDiet ? 1 : kTileLines];
  __shared__ uint32_t red[kTPB / 64];
  constexpr uint32_t kMaskChunks = (uint32_t)((kTile + kTileHalo) / 16) + 4;  // + 4: tab_bits reads 4 ahead
  __shared__ __attribute__((aligned(16))) uint16_t tabm_s[kDiet ? 1 : kMaskChunks];
  uint16_t* const tabm = kDiet ? nullptr : tabm_s;
  const uint64_t tile = blockIdx.x;
  const uint64_t t0 = tile * kTile;
  K2_STAMP(0);
  {
    TileRegs<kTileHalo> R;
    R.load(in, len, t0);
    R.store(buf);
  }
  const bool tile_prev_nl = t0 == 0 || in[t0 - 1] == '\n';
  constexpr bool local = kLocal;  // tile-local lean parse: no bases (no K1); counts come out
  if constexpr (kLocal) {
    op.bidir = op.keep = op.strip = op.has_wt = 0;
    tps = 1;
    tpe = 2;
    __builtin_assume(op.rows != nullptr && op.tile_pad != 0);
  } else {
    op.tile_pad = 0;
  }
  const TileCnt b = local ? TileCnt{} : base[tile];
  __syncthreads();
  K2_STAMP(1);
  // the tile's tab bitmap (bytes past len: 0): the tile's own chunks come with pass (1), here the halo's
  if constexpr (!kDiet)
    for (uint32_t c = kTileChunks + threadIdx.x; c < kMaskChunks; c += kTPB)
      tabm[c] = (uint16_t)(16 * c + 16 <= kTile + kTileHalo + 16 ? mask16(*(const uint4*)(buf + 16 * c), 0x09090909u) : 0u);
  const uint64_t w1 = t0 + kTile + kTileHalo < len ? t0 + kTile + kTileHalo : len;
  Src L{buf, t0, t0 + kTile + kTileHalo + 16};  // bytes past len are staged as 0
  L.tm = tabm;
  L.tm_lim = t0 + kTile + kTileHalo;
  // (1) start masks of this thread's chunks (kept), counts -> ranks
  uint32_t stm[kChunkIters / 2];
  uint32_t n_nl = 0;
#pragma unroll
  for (uint32_t j = 0; j < kChunkIters; j++) {
    const uint32_t c = j * kTPB + threadIdx.x;
    const uint4 v = *(const uint4*)(buf + 16 * c);
    if constexpr (!kDiet) tabm[c] = (uint16_t)mask16(v, 0x09090909u);
    uint32_t m, st;
    chunk_masks(buf, c, t0, len, tile_prev_nl, m, st, v);
    if (j & 1) stm[j >> 1] |= st << 16;
    else stm[j >> 1] = st;
    if constexpr (kDiet) pre16[c] = (uint16_t)__popc(st);
    else pre[c] = (uint32_t)__popc(st);
    if constexpr (kLocal) n_nl += (uint32_t)__popc(m);
  }
  __syncthreads();
  K2_STAMP(2);
  uint32_t n_starts;
  {  // kChunkIters consecutive chunk counts per thread (4-word vector accesses)
    uint32_t q[kChunkIters];
    if constexpr (kDiet) {  // 8 u16 counts per 16-byte access
#pragma unroll
      for (uint32_t k = 0; k < kChunkIters; k += 8) {
        const uint4 v = *(const uint4*)(pre16 + kChunkIters * threadIdx.x + k);
        const uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; i++) {
          q[k + 2 * i] = x[i] & 0xFFFFu;
          q[k + 2 * i + 1] = x[i] >> 16;
        }
      }
    } else {
#pragma unroll
      for (uint32_t k = 0; k < kChunkIters; k += 4) {
        const uint4 v = *(const uint4*)(pre + kChunkIters * threadIdx.x + k);
        q[k] = v.x;
        q[k + 1] = v.y;
        q[k + 2] = v.z;
        q[k + 3] = v.w;
      }
    }
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < kChunkIters; k++) sum += q[k];
    uint32_t ex;
    n_starts = block_excl_scan_u32(sum, &ex, red);
#pragma unroll
    for (uint32_t k = 0; k < kChunkIters; k++) {
      const uint32_t t = q[k];
      q[k] = ex;
      ex += t;
    }
    if constexpr (kDiet) {  // ranks < 2^15 (a chunk past the last start may wrap: never read)
#pragma unroll
      for (uint32_t k = 0; k < kChunkIters; k += 8)
        *(uint4*)(pre16 + kChunkIters * threadIdx.x + k) =
            make_uint4((q[k] & 0xFFFFu) | (q[k + 1] << 16), (q[k + 2] & 0xFFFFu) | (q[k + 3] << 16),
                       (q[k + 4] & 0xFFFFu) | (q[k + 5] << 16), (q[k + 6] & 0xFFFFu) | (q[k + 7] << 16));
    } else {
#pragma unroll
      for (uint32_t k = 0; k < kChunkIters; k += 4)
        *(uint4*)(pre + kChunkIters * threadIdx.x + k) = make_uint4(q[k], q[k + 1], q[k + 2], q[k + 3]);
    }
  }
  const uint64_t idx0 = b.nl + (tile_prev_nl ? 0 : 1);  // index of the tile's first line
  __syncthreads();
  K2_STAMP(3);
  uint32_t rank[kChunkIters];
#pragma unroll
  for (uint32_t j = 0; j < kChunkIters; j++) rank[j] = kDiet ? (uint32_t)pre16[j * kTPB + threadIdx.x] : pre[j * kTPB + threadIdx.x];
  uint64_t t_run = b.touches, e_run = b.edges, s_run = 0;
  uint32_t n_po = 0;
  unsigned long long unk = ~0ull;
  IntState is;
  const bool lean_fast = op.rows && !op.bidir && !op.has_wt && !op.strip;
  for (uint32_t w0 = 0; w0 < n_starts; w0 += kWinL) {
    const uint32_t n_win = n_starts - w0 < kWinL ? n_starts - w0 : kWinL;
    __syncthreads();  // `pre` (ranks, or the last window's prefixes) is no longer read
    // (3) the window's starts, in order
#pragma unroll
    for (uint32_t j = 0; j < kChunkIters; j++) {
      uint32_t st = (stm[j >> 1] >> ((j & 1) * 16)) & 0xFFFFu;
      uint32_t r = rank[j];
      const uint32_t c = j * kTPB + threadIdx.x;
      while (st) {
        const uint32_t o = 16 * c + __builtin_ctz(st);
        st &= st - 1;
        if (r >= w0 && r < w0 + kWinL) starts[r - w0] = (uint16_t)o;
        r++;
      }
    }
    __syncthreads();
    if (w0 == 0) K2_STAMP(4);
    // kinds of kLinesPer consecutive lines per thread; prefix counts of S and edge lines
    uint32_t cs = 0, ce = 0;
    uint8_t kk[kLinesPerW];
#pragma unroll
    for (uint32_t q = 0; q < kLinesPerW; q++) {
      const uint32_t j = kLinesPerW * threadIdx.x + q;
      uint8_t k = kSkip;
      if (j < n_win) {
        const uint32_t o = starts[j];
        k = kind_at(buf, o, t0 + o, len);
        if constexpr (!kDiet) lkind[j] = k;
      }
      kk[q] = k;
      cs += k == kS;
      ce += k == kEdge;
      if constexpr (kLocal) n_po += k == kPO;
    }
    uint32_t ex;
    const uint32_t tot = block_excl_scan_u32((cs << 16) | ce, &ex, red);
#pragma unroll
    for (uint32_t q = 0; q < kLinesPerW; q++) {
      const uint32_t j = kLinesPerW * threadIdx.x + q;
      if (j < n_win) pre[j] = ex;
      ex += ((uint32_t)(kk[q] == kS) << 16) | (uint32_t)(kk[q] == kEdge);
    }
    __syncthreads();
    if (w0 == 0) K2_STAMP(5);
    // (4) parse: lane-parallel lines
#if G2N_LEAN_ONLY
    if constexpr (kLocal) {  // the lean shapes only: any other line gives the tile-local parse up
#pragma unroll 1
      for (uint32_t j = threadIdx.x; j < n_win; j += kTPB) {
        const uint32_t o = starts[j];
        const uint8_t k = kDiet ? kind_at(buf, o, t0 + o, len) : lkind[j];
        if (k == kUnknown) {
          const uint64_t i = idx0 + w0 + j;
          unk = i < unk ? i : unk;
        }
        if (k != kS && k != kEdge && k != kPO) continue;
        uint32_t next = 0;  // 1 + the line's '\n' (or its virtual one at EOF), tile-local
        if (j + 1 < n_win) {
          next = starts[j + 1];
        } else {
          const uint32_t lim = (uint32_t)(len - t0 < kTile + kTileHalo ? len - t0 : kTile + kTileHalo);
          uint32_t x = o;
          while (x < lim && buf[x] != '\n') x++;
          if (x < lim || lim == len - t0) next = x + 1;
        }
        if (!next) {
          is.fail = 1;
          continue;
        }
        if (k == kPO) {  // parser.py:229-247, 343-361: >= 3 fields, nothing else for the matrix
          const uint32_t n = next - 1 - o, sh = o & 15;
          const uint64_t w = tab_window(buf, tabm, o >> 4);
          if (__popcll((w >> sh) & ((1ull << (n > 48 ? 48 : n)) - 1)) < 2) is.fail = 1;  // the full parse decides
          continue;
        }
        const uint32_t pr = pre[j];
        const uint64_t tb = t_run + (uint64_t)(pr >> 16) + 2 * (uint64_t)(pr & 0xFFFF);
        const uint64_t eb = e_run + (pr & 0xFFFF);
        if (!lean_line(buf, tabm, o, next, k, t0, tb, eb, op, T, is)) is.fail = 1;
      }
    } else
#endif
#pragma unroll 1
    for (uint32_t j = threadIdx.x; j < n_win; j += kTPB) {
      const uint32_t o = starts[j];
      const uint8_t k = lkind[j];
      const uint64_t i = idx0 + w0 + j;
      const uint64_t p = t0 + o;
      if (!op.rows) {  // the lean parse skips them: only error / warning / slow-weight paths read them
        ls[i] = p;
        kind[i] = k;
      }
      if (k == kUnknown) unk = i < unk ? i : unk;
      if (k == kS || k == kEdge || k == kPO) {
        const uint32_t pr = pre[j];
        const uint64_t tb = t_run + (uint64_t)(pr >> 16) * tps + (uint64_t)(pr & 0xFFFF) * tpe;
        const uint64_t eb = e_run + (pr & 0xFFFF);
        // the line ends where the next one starts; the window's last line: search the staged bytes
        const bool known = j + 1 < n_win;
        if (lean_fast && known && lean_line(buf, tabm, o, starts[j + 1], k, t0, tb, eb, op, T, is)) continue;
        const uint64_t bound = known ? t0 + starts[j + 1] : w1;
        if (!parse_line(L, len, bound, known, i, k, p, tb, eb, op, T, E, ctl, worklist, is)) {
          if (local) {  // no global positions for a deferred line: the tile-local parse gives up
            is.fail = 1;
          } else {
            const unsigned long long d = atomicAdd(&ctl->n_deferred, 1ull);
            if (d < n_tiles) deferred[d] = DeferredLine{i, p, (uint32_t)tb, (uint32_t)eb, k, 0};
          }
        }
      }
    }
    t_run += (uint64_t)(tot >> 16) * tps + (uint64_t)(tot & 0xFFFF) * tpe;
    e_run += tot & 0xFFFF;
    s_run += tot >> 16;
  }
#ifdef G2N_K2_STAMPS
  K2_STAMP(6);  // thread 0's own lines parsed
  __syncthreads();
  K2_STAMP(7);  // every line of the block parsed
#endif
  unk = wave_reduce_min(unk);
  if ((threadIdx.x & 63) == 0 && unk != ~0ull) atomicMin(&ctl->warn_line, unk);
  if constexpr (kLocal) {  // the tile's counts (K1's) and its premise evidence
    if (e_run > op.tile_pad) is.fail = 1;  // more edges than the tile's slot holds
    uint32_t vm = is.vmax;
    int32_t dmn = is.dref == kNoS ? 0x7FFFFFFF : is.dref, dmx = is.dref;  // (kNoS is the int32 minimum)
    for (int o = 32; o > 0; o >>= 1) {
      vm = max(vm, (uint32_t)__shfl_xor(vm, o, 64));
      dmn = min(dmn, (int32_t)__shfl_xor(dmn, o, 64));
      dmx = max(dmx, (int32_t)__shfl_xor(dmx, o, 64));
    }
    __shared__ uint32_t rv[kTPB / 64];
    __shared__ int32_t rmn[kTPB / 64], rmx[kTPB / 64];
    if ((threadIdx.x & 63) == 0) {
      rv[threadIdx.x >> 6] = vm;
      rmn[threadIdx.x >> 6] = dmn;
      rmx[threadIdx.x >> 6] = dmx;
    }
    const uint32_t nlpo = block_sum(n_nl | (n_po << 16), red);  // per-tile counts < 2^16 (barriers)
    if (threadIdx.x == 0) {
      for (int w = 1; w < kTPB / 64; w++) {
        vm = max(vm, rv[w]);
        dmn = min(dmn, rmn[w]);
        dmx = max(dmx, rmx[w]);
      }
      TileCnt c;
      c.nl = nlpo & 0xFFFF;
      c.lines = n_starts;
      c.segs = s_run;
      c.edges = e_run;
      c.touches = t_run;
      c.recs = s_run + e_run + (nlpo >> 16);
      tcnt_out[tile] = c;
      tlean[tile] = TileLean{dmn, dmx, vm};  // no S line: dmn > dmx (the check skips the tile)
    }
  }
  if (__ballot(is.fail) && (threadIdx.x & 63) == 0) ctl->int_fail = 1;
#ifdef G2N_K2_STAMPS
  K2_STAMP(8);
  if (kLocal && threadIdx.x == 0) {
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    g2n_k2_stamps[blockIdx.x * kK2Stamps + 9] = ((unsigned long long)xcc << 32) | hw;
  }
#endif
}

// Tile-local lean parse, afterwards: tile t's S lines must name (S lines before t) + their index
// + 1 and no edge may precede them; every edge key at most the file's S count.
__global__ void __launch_bounds__(kTPB) k_tile_lean_check(const TileCnt* __restrict__ cnt,
                                                          const TileCnt* __restrict__ tbase,
                                                          const TileLean* __restrict__ tlean, uint64_t n_tiles,
                                                          uint64_t n_seg, const TileCnt* __restrict__ tot,
                                                          uint64_t s_base, const uint32_t* __restrict__ tunk, Ctl* ctl) {
  const uint64_t t = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  if (t == 0 && tunk) {  // the one-shot unsupported-record warning (ParseOpts::tunk): the first such
    const unsigned long long w = ctl->warn_tile;  // tile's record -> its line and byte offset
    if (w != ~0ull) {
      const uint32_t u = tunk[w];
      ctl->warn_line = tbase[w].lines + (u >> 15);
      ctl->warn_off = w * kTile + (u & 0x7FFFu);
    }
  }
  if (t >= n_tiles) return;
  if (!n_seg) n_seg = tot->segs;  // a whole file: its S lines (the tile scan's total)
  const TileLean e = tlean[t];
  bool bad = e.vmax > n_seg;  // (s_base: S lines before this byte range of a sharded file)
  if (cnt[t].segs)
    bad |= tbase[t].edges != 0 || e.dmin != e.dmax || e.dmin != (long long)(s_base + tbase[t].segs);
  if (bad) ctl->int_fail = 1;
}

// The same evidence for one byte range of a sharded file whose S lines before the range are not
// known yet (g2n_build_decimal_range): each S tile's offset d = dmin - (S lines before it in the
// range) must be one value for the whole range (the caller checks d == the S lines before the range
// once the ranges' counts are exchanged); no edge may precede an S line inside the range; the
// range's largest edge key goes to the caller too (checked against the file's S count).  d is
// biased by 2^62 for the unsigned atomics.
__global__ void __launch_bounds__(kTPB) k_tile_lean_evidence(const TileCnt* __restrict__ cnt,
                                                             const TileCnt* __restrict__ tbase,
                                                             const TileLean* __restrict__ tlean, uint64_t n_tiles,
                                                             Ctl* ctl) {
  const uint64_t t = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  unsigned long long vm = 0, dmn = ~0ull, dmx = 0;
  bool bad = false;
  if (t < n_tiles) {
    const TileLean e = tlean[t];
    vm = e.vmax;
    if (cnt[t].segs) {
      bad = tbase[t].edges != 0 || e.dmin != e.dmax;
      dmn = dmx = (unsigned long long)(e.dmin - (long long)tbase[t].segs + (1ll << 62));
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    vm = max(vm, (unsigned long long)__shfl_xor(vm, o, 64));
    dmn = min(dmn, (unsigned long long)__shfl_xor(dmn, o, 64));
    dmx = max(dmx, (unsigned long long)__shfl_xor(dmx, o, 64));
  }
  const bool any_bad = __ballot(bad) != 0;
  if ((threadIdx.x & 63) == 0) {
    if (any_bad) ctl->int_fail = 1;
    if (vm) atomicMax(&ctl->ev_vmax, vm);
    if (dmn != ~0ull) {
      atomicMin(&ctl->ev_dmin, dmn);
      atomicMax(&ctl->ev_dmax, dmx);
    }
  }
}

// Tile-local lean parse, last: each tile's COO slot to its stream-order place.
// (w_p / w: the extended lean parse's per-edge weights, compacted beside; null without a weight tag)
__global__ void __launch_bounds__(kTPB) k_tile_compact(const int32_t* __restrict__ rows_p,
                                                       const int32_t* __restrict__ cols_p, uint32_t pad,
                                                       uint32_t ktrip, const TileCnt* __restrict__ cnt,
                                                       const TileCnt* __restrict__ tbase, int32_t* __restrict__ rows,
                                                       int32_t* __restrict__ cols, const double* __restrict__ w_p,
                                                       double* __restrict__ w) {
  const uint64_t t = blockIdx.x;
  const uint64_t n = cnt[t].edges * ktrip, src = t * (uint64_t)pad * ktrip, dst = tbase[t].edges * ktrip;
  for (uint64_t i = threadIdx.x; i < n; i += kTPB) {
    rows[dst + i] = rows_p[src + i];
    cols[dst + i] = cols_p[src + i];
  }
  if (w_p)
    for (uint64_t i = threadIdx.x; i < cnt[t].edges; i += kTPB) w[tbase[t].edges + i] = w_p[t * (uint64_t)pad + i];
}

// Lines whose fields run past their tile's staged window: parsed from global memory.
__global__ void __launch_bounds__(64) k_parse_deferred(const uint8_t* __restrict__ in, uint64_t len,
                                                       const uint64_t* __restrict__ ls,
                                                       const uint8_t* __restrict__ kind,
                                                       const DeferredLine* __restrict__ deferred, uint64_t n,
                                                       ParseOpts op, TouchOut T, EdgeOut E, Ctl* ctl,
                                                       uint64_t* __restrict__ worklist) {
  const uint64_t j = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  if (j >= n) return;
  const DeferredLine d = deferred[j];
  const Src G{in, 0, len};
  IntState is;
  parse_line(G, len, len, false, d.line, (uint8_t)d.kind, d.start, d.tb, d.eb, op, T, E, ctl, worklist, is);
  if (is.fail) ctl->int_fail = 1;
}

// Exact weights (CPython int()/float() semantics) for the edges the fast grammar deferred.
__global__ void __launch_bounds__(64) k_weights_slow(const uint8_t* __restrict__ in_, uint64_t len,
                                                     const uint64_t* __restrict__ ls,
                                                     const uint64_t* __restrict__ worklist, uint64_t n_work,
                                                     ParseOpts op, EdgeOut E, Ctl* ctl) {
  const uint64_t j = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  if (j >= n_work) return;
  const Src in{in_, 0, len};
  const uint64_t i = worklist[2 * j], eb = worklist[2 * j + 1];
  uint64_t s = ls[i], e = ls[i + 1];
  if (e > s && in[e - 1] == '\n') e--;
  EdgeLayout L = edge_layout(in, s, e);
  Decimal dec;
  uint8_t tmp[DEC_TMP];
  // _parse_tags over fields[tag_from:], keeping only the final value for weight_tag
  int kind = 0;  // 0 none, 1 int, 2 float, 3 other
  uint64_t best_s = 0, best_e = 0;
  double fval = 0.0;
  if (L.has_tags) {
    uint64_t p = L.tag_start;
    while (true) {
      uint64_t fe = next_tab(in, p, e);
      if (utf8_valid(in.ptr(p), fe - p)) {
        uint64_t c1 = next_byte(in, p, fe, ':');
        uint64_t c2 = c1 < fe ? next_byte(in, c1 + 1, fe, ':') : fe;
        if (c2 < fe && span_eq(in, p, c1 - p, op.wt, op.wt_len)) {
          uint64_t tl = c2 - c1 - 1;
          uint8_t ty = in[c1 + 1];
          if (tl == 1 && ty == 'i') {
            if (py_int_literal(in.ptr(c2 + 1), fe - c2 - 1, true, nullptr)) {
              kind = 1;
              best_s = c2 + 1;
              best_e = fe;
            }
          } else if (tl == 1 && ty == 'f') {
            double v;
            if (py_float_literal(in.ptr(c2 + 1), fe - c2 - 1, true, &v, &dec, tmp)) {
              kind = 2;
              fval = v;
            }
          } else {
            kind = 3;
          }
        }
      }
      if (fe >= e) break;
      p = fe + 1;
    }
  }
  double w = 1.0;
  if (kind == 1) {
    py_int_literal(in.ptr(best_s), best_e - best_s, true, &dec);
    if (!py_int_to_f64(&dec, &w, tmp)) {  // builders.py:209 float(val): OverflowError
      record_error(ctl, i, kErrIntTooLarge);
      return;
    }
  } else if (kind == 2) {
    w = fval;
  }
  E.w[eb] = w;
}

// Re-parse the failing line to recover the bytes whose .decode() raised.
__global__ void k_error_detail(const uint8_t* __restrict__ in_, uint64_t len, const uint64_t* __restrict__ ls,
                               uint64_t line, Ctl* ctl) {
  const Src in{in_, 0, len};
  uint64_t s = ls[line], e = ls[line + 1];
  if (e > s && in[e - 1] == '\n') e--;
  EdgeLayout L = edge_layout(in, s, e);
  ctl->detail_off = L.err == kErrUnicode ? L.err_off : s;
  ctl->detail_len = L.err == kErrUnicode ? L.err_len : 1;
}

// records on lines before `line` (verbose progress before an error, builders.py:257-258)
__global__ void __launch_bounds__(kTPB) k_count_records(const uint8_t* __restrict__ kind, uint64_t line, Ctl* ctl) {
  const uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  unsigned long long c = 0;
  if (i < line) {
    uint8_t k = kind[i];
    c = (k == kS || k == kEdge || k == kPO) ? 1 : 0;
  }
  c = wave_reduce_sum(c);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(&ctl->n_records_before, c);
}

// ============================================================= K4: dictionary =====

__device__ inline uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

typedef unsigned __int128 u128;

// 8 bytes at aligned address a (a % 8 == 0); bytes at or past in_len read as 0
__device__ inline uint64_t rd64(const uint8_t* __restrict__ in, uint64_t in_len, uint64_t a) {
  if (a + 8 <= in_len) return *(const uint64_t*)(in + a);
  uint64_t w = 0;
  for (int b = 0; b < 8; b++)
    if (a + b < in_len) w |= (uint64_t)in[a + b] << (8 * b);
  return w;
}

// first min(n, 16) bytes at `off`, little-endian, zero padded (aligned 8-byte loads)
__device__ inline u128 load_span16(const uint8_t* __restrict__ in, uint64_t in_len, uint64_t off, uint64_t n) {
  if (n == 0) return 0;
  const uint64_t m = n < 16 ? n : 16;
  const uint64_t a = off & ~7ull, end = off + m;
  const uint32_t sh = (uint32_t)(off & 7) * 8;
  uint64_t w0 = rd64(in, in_len, a);
  uint64_t w1 = a + 8 < end ? rd64(in, in_len, a + 8) : 0;
  uint64_t w2 = a + 16 < end ? rd64(in, in_len, a + 16) : 0;
  uint64_t lo = sh ? (w0 >> sh) | (w1 << (64 - sh)) : w0;
  uint64_t hi = sh ? (w1 >> sh) | (w2 << (64 - sh)) : w1;
  u128 k = ((u128)hi << 64) | lo;
  if (m < 16) k &= (((u128)1) << (8 * m)) - 1;
  return k;
}

// The first 16 bytes of a node key (name, or name + ":" + orientation when bidirected)
// and its length.  builders.py:211-212, 234: keys are byte strings compared exactly.
struct KeyHead {
  u128 k;
  uint32_t len;
};

__device__ inline KeyHead key_head(const uint8_t* __restrict__ in, uint64_t in_len, uint64_t no, uint32_t nl,
                                   uint64_t oo, uint32_t ol, bool bidir) {
  KeyHead kh;
  kh.k = load_span16(in, in_len, no, nl);
  kh.len = nl;
  if (bidir) {
    kh.len = nl + 1 + ol;
    if (nl < 16) {
      kh.k |= ((u128)':') << (8 * nl);
      if (nl + 1 < 16) {
        u128 o = (oo & kConstFlag) ? (u128)(oo & 0xFF) : load_span16(in, in_len, oo, ol);
        kh.k |= o << (8 * (nl + 1));
      }
    }
  }
  return kh;
}

__device__ inline uint8_t touch_byte(const uint8_t* __restrict__ in, uint64_t no, uint32_t nl, uint64_t oo,
                                     uint64_t j) {
  if (j < nl) return in[no + j];
  if (j == nl) return ':';
  return (oo & kConstFlag) ? (uint8_t)(oo & 0xFF) : in[oo + (j - nl - 1)];
}

__device__ inline uint64_t key_hash(const uint8_t* __restrict__ in, const KeyHead& kh, uint64_t no, uint32_t nl,
                                    uint64_t oo) {
  const uint64_t lo = (uint64_t)kh.k, hi = (uint64_t)(kh.k >> 64);
  uint64_t h = lo * 0x9E3779B97F4A7C15ull;
  h ^= ((hi * 0xC2B2AE3D27D4EB4Full) << 31) | ((hi * 0xC2B2AE3D27D4EB4Full) >> 33);
  h ^= (uint64_t)kh.len * 0x165667B19E3779F9ull;
  for (uint64_t j = 16; j < kh.len; j++) h = (h ^ touch_byte(in, no, nl, oo, j)) * 0x100000001b3ull;  // long keys
  return fmix64(h);
}

// bytes [16, len) of two keys of equal length (only for keys longer than the inline head)
__device__ inline bool tail_eq(const uint8_t* __restrict__ in, const TouchIn& T, uint64_t a, uint64_t b, bool bidir,
                               uint32_t len) {
  const uint64_t na = T.noff[a], nb = T.noff[b];
  const uint32_t la = T.nlen[a], lb = T.nlen[b];
  const uint64_t oa = bidir ? T.ooff[a] : 0, ob = bidir ? T.ooff[b] : 0;
  for (uint64_t j = 16; j < len; j++)
    if (touch_byte(in, na, la, oa, j) != touch_byte(in, nb, lb, ob, j)) return false;
  return true;
}

// ============================ K2 lean: the tile-local decimal-id parse ========================
// The tile-local lean parse (ParseOpts.tile_pad; S lines first named "1".."N", no bidirected, no
// weight tag, no strip) as a kernel of its own.  One 512-thread block (8 waves) per 32 KiB tile
// (+ halo):
//  (1) the tile is staged in LDS, every 16-byte load in flight before the first store; from the
//      same registers (chunks 512 j + t: no LDS re-read) the tab and newline bitmaps of every
//      chunk go to LDS, one u16 each;
//  (2) thread t takes the line starts in ITS contiguous 64 bytes (chunks 4t..4t+3: one 8-byte
//      LDS read of their newline bitmaps, one 64-bit start mask), classifies them (parser.py:
//      117-134 first-byte dispatch) with every byte load in flight at once, and counts starts, S
//      and edge lines; ONE block scan of the packed counts ranks its lines in the tile, and it
//      writes one 32-bit record per line (offset, kind, S / edge prefix) at that rank;
//  (3) lane-parallel parse: line j goes to thread j mod 512 (balanced), its end is the next
//      record's offset, the fields come from the tab bitmap (lean_line), the result goes to the
//      tile's COO slot.
// 512 threads over the same 52 KB of LDS as 256 would use: 3 blocks and 6 waves per SIMD.
// Same outputs as k_tile_parse<true> (tile counts, premise evidence, COO slot) with one block
// scan instead of three.  Anything outside the lean shapes — an unsupported record (its warning
// needs global line indices), a line running past the staged window — fails the tile-local parse
// and the full parse runs (tile_local_parse).
#ifndef G2N_LEAN_TPB  // experiment builds: 1024 (32-byte regions)
#define G2N_LEAN_TPB 512
#endif
constexpr uint32_t kLeanTPB = G2N_LEAN_TPB;                             // threads per tile
constexpr uint32_t kLeanRegion = (uint32_t)(kTile / 16) / kLeanTPB;     // chunks per thread (4)
// the lean front end's halo: a lean edge line ends at most 48 bytes + its '\n' past its start, and an S /
// P / O line whose end is out of view needs only its first 48 bytes (round 6: 64 bytes staged past the
// tile instead of K1 / k_tile_parse's 2 KiB — 0.2 % of the input re-read and masked, not 6.25 %)
#ifndef G2N_LEAN_HALO
#define G2N_LEAN_HALO 64
#endif
constexpr uint32_t kLeanHalo = G2N_LEAN_HALO;
static_assert(kLeanHalo >= 64 && kLeanHalo % 16 == 0, "an edge line's 49 bytes past its start");
constexpr uint32_t kLeanChunks = (uint32_t)((kTile + kLeanHalo) / 16);  // staged chunks
constexpr uint32_t kLeanLines = 2048;                                   // line records per window
#ifndef G2N_LEAN_PAIR  // experiment builds: the decimal parse two lines per lane per step
#define G2N_LEAN_PAIR 0
#endif
#ifndef G2N_CLASSIFY_FLAT  // experiment builds: 0 = the lean classify's starts through line_kind's branches
#define G2N_CLASSIFY_FLAT 1
#endif
#ifndef G2N_LEAN_BATCH  // experiment builds: starts classified per region with their loads batched
#define G2N_LEAN_BATCH 4
#endif
constexpr uint32_t kLeanBatch = G2N_LEAN_BATCH;                         // starts classified with loads batched
static_assert(kTile <= 32768 && (kLeanRegion == 4 || kLeanRegion == 2),
              "records hold 15-bit offsets; a region's starts fit one 64-bit mask");

__device__ inline uint32_t lean_code(uint8_t kd) {  // record kind: 0 other, 1 S, 2 edge, 3 P / O
  return kd == kS ? 1u : kd == kEdge ? 2u : kd == kPO ? 3u : 0u;
}

// lean_code(line_kind(c0, exact)) as straight-line code (round 6): one bit per record letter of
// '@'..'_' tested against each kind's letters; *unk: kUnknown (not a record letter at all)
__device__ __forceinline__ uint32_t lean_code_flat(uint32_t c0, bool exact, bool* unk) {
  constexpr uint32_t kBS = 1u << ('S' - 64), kBE = (1u << ('L' - 64)) | (1u << ('E' - 64)) | (1u << ('C' - 64)),
                     kBPO = (1u << ('P' - 64)) | (1u << ('O' - 64)), kBHF = (1u << ('H' - 64)) | (1u << ('F' - 64));
  const uint32_t idx = c0 - 64u;
  const uint32_t bit = idx < 32u ? 1u << idx : 0u;
  *unk = (bit & (kBS | kBE | kBPO | kBHF)) == 0;
  const uint32_t code = (bit & kBS ? 1u : 0u) | (bit & kBE ? 2u : 0u) | (bit & kBPO ? 3u : 0u);
  return exact ? code : 0u;
}

#ifndef G2N_DPP_SCAN  // experiment builds: 0 = the lean tile's scan / reductions by ds_bpermute shuffles (round 5)
#define G2N_DPP_SCAN 1
#endif
// Wave-wide inclusive scans / reductions by DPP (gfx9 row_shr within 16-lane rows, then row_bcast:15 /
// row_bcast:31 across rows): one VALU op per step, no LDS crossbar round trip (__shfl_up / __shfl_xor
// compile to ds_bpermute).  Lanes a step has no source for take the identity (old operand).
template <class Op>
__device__ __forceinline__ uint32_t wave_dpp_incl(uint32_t v, uint32_t id, Op op) {
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, 0x111, 0xF, 0xF, false));  // row_shr:1
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, 0x112, 0xF, 0xF, false));  // row_shr:2
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, 0x114, 0xF, 0xF, false));  // row_shr:4
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, 0x118, 0xF, 0xF, false));  // row_shr:8
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, 0x142, 0xA, 0xF, false));  // row_bcast:15
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, 0x143, 0xC, 0xF, false));  // row_bcast:31
  return v;
}
__device__ __forceinline__ uint32_t dpp_add(uint32_t a, uint32_t b) { return a + b; }
__device__ __forceinline__ uint32_t dpp_max(uint32_t a, uint32_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint32_t dpp_smin(uint32_t a, uint32_t b) { return (int32_t)a < (int32_t)b ? a : b; }
__device__ __forceinline__ uint32_t dpp_smax(uint32_t a, uint32_t b) { return (int32_t)a > (int32_t)b ? a : b; }
// the wave's reduction (every lane gets it: lane 63's inclusive value)
template <class Op>
__device__ __forceinline__ uint32_t wave_dpp_reduce(uint32_t v, uint32_t id, Op op) {
  return (uint32_t)__builtin_amdgcn_readlane((int)wave_dpp_incl(v, id, op), 63);
}

// The lean tile's block scan of (starts, S lines, edge lines), each < 2^16 per tile: two 32-bit DPP wave
// scans, the waves' totals through LDS.  Returns the exclusive prefix packed as block_excl_scan_n64's.
template <uint32_t kN>
__device__ inline unsigned long long lean_block_scan(uint32_t n_st, uint32_t n_s, uint32_t n_e, unsigned long long* tot,
                                                     unsigned long long* lds /* >= kN / 64 */) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint32_t a = n_st | (n_s << 16), ia = wave_dpp_incl(a, 0u, dpp_add), ie = wave_dpp_incl(n_e, 0u, dpp_add);
  if (lane == 63) lds[wid] = (unsigned long long)ia | ((unsigned long long)ie << 32);
  __syncthreads();
  uint32_t ba = 0, be = 0, ta = 0, te = 0;
#pragma unroll
  for (int q = 0; q < (int)(kN / 64); q++) {
    const unsigned long long y = lds[q];
    if (q < wid) {
      ba += (uint32_t)y;
      be += (uint32_t)(y >> 32);
    }
    ta += (uint32_t)y;
    te += (uint32_t)(y >> 32);
  }
  __syncthreads();
  auto pack = [](uint32_t x, uint32_t e) {
    return (unsigned long long)(x & 0xFFFFu) | ((unsigned long long)(x >> 16) << 20) | ((unsigned long long)e << 40);
  };
  *tot = pack(ta, te);
  return pack(ba + ia - a, be + ie - n_e);
}

template <uint32_t kN, class T>
__device__ inline T block_excl_scan_n64(T v, T* tot, T* lds /* >= kN / 64 */) {  // exclusive; *tot = total
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  T x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const T y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) lds[wid] = x;
  __syncthreads();
  T wbase = 0, t = 0;
#pragma unroll
  for (int q = 0; q < (int)(kN / 64); q++) {
    const T y = lds[q];
    if (q < wid) wbase += y;
    t += y;
  }
  __syncthreads();
  *tot = t;
  return wbase + x - v;
}

// ---- the S-first hash dictionary on the lean front end (modes kLeanClaim / kLeanEdges) --------
// For inputs whose S lines come first with unique names that are not the decimal ids (any names):
// after K1's tile bases, kLeanClaim claims every S name in a table of 32-byte entries (hdr = hash
// tag << 32 | node id = the S line's index, meta = key length << 40 | the name's input offset,
// the first 16 key bytes inline) and records each node's name (noff / nlen); kLeanEdges parses
// every edge line's two names from the staged tile, finds them (one random 32-byte read each) and
// writes the stream-order COO.  builders.py:190-198: with every S line before every other line and
// no repeated S name, a key's first touch is its S line, so node id = S index.  Anything else — a
// repeated name (or a 32-bit tag shared by two S names), an edge key that is no S name, an S line
// after an edge line, a line outside the lean shapes — fails the pass and the classic hash tiers
// (full parse + dictionary rounds) run instead.
// Direct-address tier (modes kLeanDirClaim / kLeanDirEdges): when every S name is one common prefix
// (possibly empty) followed by a canonical decimal v < direct_cap — decimal ids out of S order,
// minigraph's "s<n>" — the table is a plain array: S line k claims direct[v] = k (a second claim of
// v is a repeated name: the pass fails), and an edge name costs one random 4-byte read instead of a
// 32-byte probe plus a key compare.  Same premise and fallbacks as the hash modes.
enum : int { kLeanDecimal = 0, kLeanClaim = 1, kLeanEdges = 2, kLeanDirClaim = 3, kLeanDirEdges = 4 };
#ifndef G2N_HL_LINES  // edge lines per thread per step in kLeanEdges (2, four probes in flight: 105 VGPRs, slower)
#define G2N_HL_LINES 1
#endif

struct HashLeanArgs {
  const TileCnt* tbase;  // K1's tile bases (exclusive scan of tcnt)
  const TileCnt* tcnt;   // K1's tile counts
  DictEntry* table;
  uint64_t mask;         // table slots - 1
  uint64_t max_probes;
  uint64_t* noff;        // kLeanClaim: node id -> input offset of its name
  uint32_t* nlen;        //             node id -> name length
  int32_t* rows;         // kLeanEdges: stream-order COO, ktrip entries per edge line
  int32_t* cols;
  uint32_t ktrip;
  const uint32_t* tlist; // the launch's tiles (k_tile_lists; block b parses tile tlist[b]), or null: tile b
  unsigned long long* tnb;  // kLeanClaim / kLeanDirClaim, per block: name bytes claimed | the largest value << 32
  uint32_t* direct;      // kLeanDir*: name value -> node id (~0u: no S line names it)
  uint64_t direct_cap;   //            values below this
  uint64_t pre;          //            the names' common prefix, little-endian (pre_len <= 8 bytes)
  uint32_t pre_len;
  uint32_t suf_len;      //            ... and common suffix (no digit in it, <= 8 bytes)
  uint64_t suf;
  uint32_t width;        //            0: canonical decimals; w: exactly w digits, leading zeros allowed
  // the edge passes' extended instance (kExt: bidirected keys / one integer weight tag, lean_line's
  // rules): node ids 2 id + [ori == '-'] with the reverse twins, the weight of edge e at ew[e]
  int bidir, has_wt;
  uint32_t wt_len;
  uint64_t wt_pack;
  double* ew;
};

#ifndef G2N_DIRECT_STORE  // kLeanDirClaim: 1 = plain stores + a count of the filled slots, 0 = CAS per S line
#define G2N_DIRECT_STORE 1
#endif

// The lean hash / direct passes' tiles, from K1's counts: lists[0] / lists[1] = how many tiles hold
// S or P / O lines (the claim passes) / edge lines (the edge passes), their indices at lists + 2 /
// lists + 2 + n_tiles (one atomic per wave: ascending within a wave).  A pass launched over its list
// instead of every tile: ~158K of C4's 192K tiles hold no S line, and a block that only reads its
// counts and exits still costs its dispatch (a claim pass over all tiles measured 3.2 ms with the
// stores taken out).
__global__ void __launch_bounds__(kTPB) k_tile_lists(const TileCnt* __restrict__ tcnt, uint64_t n_tiles,
                                                     uint32_t* __restrict__ lists) {
  const uint64_t t = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  bool cl = false, ed = false;
  if (t < n_tiles) {
    const TileCnt c = tcnt[t];
    cl = !(c.segs == 0 && c.recs == c.segs + c.edges);
    ed = c.edges != 0;
  }
  const int lane = threadIdx.x & 63;
  const unsigned long long below = (1ull << lane) - 1;
  const unsigned long long bc = __ballot(cl), be = __ballot(ed);
  uint32_t pc = 0, pe = 0;
  if (lane == 0) {
    if (bc) pc = atomicAdd(&lists[0], (uint32_t)__popcll(bc));
    if (be) pe = atomicAdd(&lists[1], (uint32_t)__popcll(be));
  }
  pc = __shfl(pc, 0, 64);
  pe = __shfl(pe, 0, 64);
  if (cl) lists[2 + pc + __popcll(bc & below)] = (uint32_t)t;
  if (ed) lists[2 + n_tiles + pe + __popcll(be & below)] = (uint32_t)t;
}

// the claim pass's per-block (bytes | vmax << 32): *bytes = their sum, *vmax = their largest value (one block)
__global__ void __launch_bounds__(1024) k_claim_totals(const unsigned long long* __restrict__ a, uint64_t n,
                                                       unsigned long long* bytes, unsigned long long* vmax) {
  __shared__ unsigned long long red[16], redm[16];
  unsigned long long x = 0, m = 0;
  for (uint64_t i = threadIdx.x; i < n; i += 1024) {
    x += a[i] & 0xFFFFFFFFull;
    m = max(m, a[i] >> 32);
  }
  for (int o = 32; o > 0; o >>= 1) {
    x += __shfl_xor(x, o, 64);
    m = max(m, (unsigned long long)__shfl_xor(m, o, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6] = x;
    redm[threadIdx.x >> 6] = m;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 16; w++) {
      x += red[w];
      m = max(m, redm[w]);
    }
    *bytes = x;
    *vmax = m;
  }
}

// the direct array's filled slots (!= ~0u), added to *out: the claim pass's duplicate check (one
// atomic per block: atomics on one address serialise, ~7 ns each)
__global__ void __launch_bounds__(256) k_direct_filled(const uint4* __restrict__ a, uint64_t cap4,
                                                       const unsigned long long* __restrict__ vmax,
                                                       unsigned long long* out) {
  __shared__ uint32_t red[4];
  const uint64_t n4 = min(cap4, *vmax / 4 + 1);  // no claimed value past vmax (the claim pass's largest)
  uint32_t c = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * 256) {
    const uint4 v = a[i];
    c += (v.x != ~0u) + (v.y != ~0u) + (v.z != ~0u) + (v.w != ~0u);
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0 && red[0] + red[1] + red[2] + red[3])
    atomicAdd(out, (unsigned long long)(red[0] + red[1] + red[2] + red[3]));
}

#ifndef G2N_DIRECT_LINES  // kLeanDirEdges: edge lines per thread per step (2 random reads each in flight)
#define G2N_DIRECT_LINES 4
#endif




// The first min(l, 16) bytes at tile offset x of the staged tile, little-endian, zero padded
// (aligned 8-byte LDS reads; never past x + l rounded up to 8)
__device__ inline u128 lds_span16(const uint8_t* buf, uint32_t x, uint32_t l) {
  if (l == 0) return 0;
  const uint32_t m = l < 16 ? l : 16, a = x & ~7u, end = x + m, sh = (x & 7u) * 8;
  const uint64_t w0 = *(const uint64_t*)(buf + a);
  const uint64_t w1 = a + 8 < end ? *(const uint64_t*)(buf + a + 8) : 0ull;
  const uint64_t w2 = a + 16 < end ? *(const uint64_t*)(buf + a + 16) : 0ull;
  const uint64_t lo = sh ? (w0 >> sh) | (w1 << (64 - sh)) : w0;
  const uint64_t hi = sh ? (w1 >> sh) | (w2 << (64 - sh)) : w1;
  u128 k = ((u128)hi << 64) | lo;
  if (m < 16) k &= (((u128)1) << (8 * m)) - 1;
  return k;
}

__device__ inline bool tail_eq_in(const uint8_t* __restrict__ in, uint64_t a, uint64_t b, uint32_t len) {
  for (uint32_t j = 16; j < len; j++)
    if (in[a + j] != in[b + j]) return false;
  return true;
}

// fixed-width digits, leading zeros allowed (zero-padded names: one width, so value <-> name)
__device__ inline bool dec_lds_pad(const uint8_t* buf, uint32_t x, uint32_t l, uint64_t* v) {
  if (l == 0 || l > 10) return false;
  uint64_t y = 0;
  for (uint32_t j = 0; j < l; j++) {
    const uint32_t c = buf[x + j];
    if (c - '0' > 9u) return false;
    y = y * 10 + (c - '0');
  }
  *v = y;
  return true;
}

// the value of the name at tile offset x (length l) when it is H.pre, a decimal and H.suf — the
// decimal canonical (no sign, no leading zero, <= 10 digits) or, with H.width, exactly that many
// digits (hifiasm's "utg000123l") — and below H.direct_cap.  Prefix, suffix and the digit rule make
// the value one name's.
__device__ inline bool lean_direct_value(const uint8_t* buf, const HashLeanArgs& H, uint32_t x, uint32_t l,
                                         uint64_t& v) {
  const uint32_t p = H.pre_len, q = H.suf_len;
  if (l <= p + q) return false;
  if (p && (uint64_t)lds_span16(buf, x, p) != H.pre) return false;
  if (q && (uint64_t)lds_span16(buf, x + l - q, q) != H.suf) return false;
  const uint32_t nd = l - p - q;
  if (H.width) return nd == H.width && dec_lds_pad(buf, x + p, nd, &v) && v < H.direct_cap;
  return dec_lds(buf, x + p, nd, &v) && v < H.direct_cap;
}

// S line at tile offset so (its '\n' at next - 1): the name's tile offset and length (fields[1],
// parser.py:133-163), false when the name is not in the 48-byte tab view (the classic parse decides)
__device__ inline bool lean_s_name(const uint8_t* buf, const uint16_t* tabm, uint32_t so, uint32_t next,
                                   uint32_t& x, uint32_t& l) {
  const uint32_t n = next - 1 - so;
  const uint64_t w = tab_window(buf, tabm, so >> 4);
  uint64_t m = (w >> (so & 15)) & ((1ull << (n > 48 ? 48 : n)) - 1);
  if (!m) return false;
  const uint32_t t1 = (uint32_t)__builtin_ctzll(m);
  m &= m - 1;
  if (!m && n > 48) return false;
  const uint32_t t2 = m ? (uint32_t)__builtin_ctzll(m) : n;
  x = so + t1 + 1;
  l = t2 - t1 - 1;
  return true;
}

// L / E / C line in the link_fast shape (lean_line's): the two names' tile offsets and lengths.
// kExt (bidirected / weighted lean tiers): also the orientations (bit 0: the first is '-', bit 1: the
// second) and, with H.has_wt, the weight — one trailing canonical "<tag>:i:<int>" field or 1.0 without
// it (builders.py:205-209; another spelling or an extra field is false: the full parse decides)
template <bool kExt = false>
__device__ inline bool lean_edge_names(const uint8_t* buf, const uint16_t* tabm, uint32_t so, uint32_t next,
                                       uint32_t& xa, uint32_t& la, uint32_t& xb, uint32_t& lb,
                                       const HashLeanArgs* H = nullptr, uint32_t* ori = nullptr, double* wv = nullptr) {
  const uint32_t n = next - 1 - so;
  if (n > 48) return false;
  const uint64_t w = tab_window(buf, tabm, so >> 4);
  uint64_t m = (w >> (so & 15)) & ((1ull << n) - 1);
  if (__popcll(m) < 5) return false;
  uint32_t p[6];
#pragma unroll
  for (int j = 0; j < 6; j++) {
    p[j] = m ? (uint32_t)__builtin_ctzll(m) : n;
    m &= m - 1;
  }
  if (p[2] - p[1] != 2 || p[4] - p[3] != 2) return false;
  const uint32_t c2 = buf[so + p[1] + 1], c4 = buf[so + p[3] + 1];
  if ((c2 != '+' && c2 != '-') || (c4 != '+' && c4 != '-')) return false;
  xa = so + p[0] + 1;
  la = p[1] - p[0] - 1;
  xb = so + p[2] + 1;
  lb = p[3] - p[2] - 1;
  if constexpr (kExt) {
    *ori = (c2 == '-' ? 1u : 0u) | (c4 == '-' ? 2u : 0u);
    *wv = 1.0;
    if (H->has_wt && p[5] < n &&
        (m || !lean_int_tag(buf, so + p[5] + 1, n - p[5] - 1, H->wt_len, H->wt_pack, wv)))
      return false;
  }
  return true;
}

// an edge's entries from its two S indices (lean hash / direct tiers): plain, or (kExt, H.bidir)
// the "name:o" ids 2 i + o and the reverse twins of an undirected bidirected build
// (builders.py:211-234, lean_line's order); edge index e, its weight when H.has_wt
template <bool kExt>
__device__ inline void lean_edge_out(const HashLeanArgs& H, uint64_t e, uint32_t ida, uint32_t idb, uint32_t ori,
                                     double wv) {
  const uint64_t o = e * H.ktrip;
  if constexpr (kExt) {
    if (H.has_wt) H.ew[e] = wv;
    if (H.bidir) {
      const uint32_t ia = 2u * ida + (ori & 1u), ib = 2u * idb + (ori >> 1);
      H.rows[o] = (int32_t)ia;
      H.cols[o] = (int32_t)ib;
      if (H.ktrip == 4) {
        H.rows[o + 1] = (int32_t)ib;
        H.cols[o + 1] = (int32_t)ia;
        H.rows[o + 2] = (int32_t)(ib ^ 1u);
        H.cols[o + 2] = (int32_t)(ia ^ 1u);
        H.rows[o + 3] = (int32_t)(ia ^ 1u);
        H.cols[o + 3] = (int32_t)(ib ^ 1u);
      }
      return;
    }
  }
  H.rows[o] = (int32_t)ida;
  H.cols[o] = (int32_t)idb;
  if (H.ktrip >= 2) {
    H.rows[o + 1] = (int32_t)idb;
    H.cols[o + 1] = (int32_t)ida;
  }
}

// key head + hash of the name at tile offset x (input offset t0 + x), the classic tiers' key_hash
__device__ inline uint64_t lean_key(const uint8_t* __restrict__ in, const uint8_t* buf, uint64_t t0, uint32_t x,
                                    uint32_t l, KeyHead& kh) {
  kh.k = lds_span16(buf, x, l);
  kh.len = l;
  return key_hash(in, kh, t0 + x, l, 0);
}

// the node id of the name at input offset no (head kh, hash h), or ~0u when no S line names it;
// (a0, b0): the first probed entry, already loaded by the caller (so several probes are in flight)
__device__ inline uint32_t lean_find(const uint8_t* __restrict__ in, const HashLeanArgs& H, const KeyHead& kh,
                                     uint64_t h, uint64_t no, uint4 a0, uint4 b0) {
  const uint32_t tag = (uint32_t)(h >> 32);
  const uint64_t k0 = (uint64_t)kh.k, k1 = (uint64_t)(kh.k >> 64);
  uint64_t idx = h & H.mask;
  for (uint64_t probe = 0; probe < H.max_probes; probe++) {
    uint4 a = a0, b = b0;
    if (probe) {
      const DictEntry* e = H.table + idx;
      a = ((const uint4*)e)[0];
      b = ((const uint4*)e)[1];
    }
    const unsigned long long hdr = ((unsigned long long)a.y << 32) | a.x;
    if (hdr == kEmptySlot) return ~0u;
    const unsigned long long meta = ((unsigned long long)a.w << 32) | a.z;
    if ((uint32_t)(hdr >> 32) == tag && (uint32_t)(meta >> 40) == kh.len &&
        (((uint64_t)b.y << 32) | b.x) == k0 && (((uint64_t)b.w << 32) | b.z) == k1 &&
        (kh.len <= 16 || tail_eq_in(in, no, meta & ((1ull << 40) - 1), kh.len)))
      return (uint32_t)hdr;
    idx = (idx + 1) & H.mask;
  }
  return ~0u;
}

using LeanRegs = TileRegs<kLeanHalo, kLeanTPB>;
#ifndef G2N_K2_PREFETCH
#define G2N_K2_PREFETCH 0
#endif

// One tile of the lean front end.  R holds the tile's staged bytes on entry (loaded by the caller);
// after they are in LDS, R is refilled with tile next_tile's bytes (next_tile < n_tiles), which stay
// in flight through this tile's parse — the persistent decimal kernel's prefetch.
template <int kMode, bool kGrouped, bool kExt = false>
__device__ __forceinline__ void lean_tile(const uint8_t* __restrict__ in, uint64_t len, ParseOpts op, Ctl* ctl,
                                          TileCnt* __restrict__ tcnt_out, TileLean* __restrict__ tlean,
                                          uint32_t* __restrict__ gcount, uint64_t gcap, const HashLeanArgs& H,
                                          const uint64_t tile, LeanRegs& R, uint64_t next_tile, uint64_t n_tiles) {
  constexpr uint32_t kW = kLeanTPB / 64;
  __shared__ __attribute__((aligned(16))) uint8_t buf[kTile + kLeanHalo + 16];
  __shared__ __attribute__((aligned(16))) uint16_t tabm[kLeanChunks + 8];
  __shared__ __attribute__((aligned(16))) uint16_t nlm[kLeanChunks + 8];
  __shared__ uint32_t rec[kLeanLines + 1];
  __shared__ unsigned long long red64[kW];
  __shared__ uint32_t s_gbase;
  __shared__ uint32_t s_unk;  // the tile's first unsupported record (op.tunk): rank << 15 | offset
  __shared__ uint32_t s_last_end;  // the tile's last line's end (see line_next)
  const uint64_t t0 = tile * kTile;
  if (!kGrouped && op.tile_pad) {  // this tile's slot (positions relative to it, as in a group slot)
    const uint64_t b = tile * (uint64_t)op.tile_pad * op.ktrip;
    op.rows += b;
    op.cols += b;
    if (kExt && op.ew) op.ew += tile * (uint64_t)op.tile_pad;  // one weight per edge line
  }
  op.grouped = op.tile_pad ? 1u : 0u;  // lean_line: positions relative to the tile's base in its slot
  if (threadIdx.x == 0) s_unk = ~0u;  // (published by the staging barrier)
  uint64_t sbase = 0, ebase = 0;     // hash modes: S lines / edge lines before this tile (K1's bases)
  if constexpr (kMode != kLeanDecimal) {
    sbase = H.tbase[tile].segs;
    ebase = H.tbase[tile].edges;
  }
  K2_LEAN_STAMP(0);
  R.store(buf);
#pragma unroll
  for (uint32_t j = 0; j < R.kPer; j++) {
    const uint32_t c = j * kLeanTPB + threadIdx.x;
    if (c < kLeanChunks) {
#if G2N_MASK2
      const uint32_t tn = mask16x2(R.r[j]);
      tabm[c] = (uint16_t)tn;
      nlm[c] = (uint16_t)(tn >> 16);
#else
      tabm[c] = (uint16_t)mask16(R.r[j], 0x09090909u);
      nlm[c] = (uint16_t)mask16(R.r[j], 0x0A0A0A0Au);
#endif
    }
  }
  if (next_tile < n_tiles) R.load(in, len, next_tile * kTile);  // in flight through this tile's parse
  if (threadIdx.x < 8) {  // tab_window reads up to 4 bitmaps past a chunk
    tabm[kLeanChunks + threadIdx.x] = 0;
    nlm[kLeanChunks + threadIdx.x] = 0;
  }
  const bool tile_prev_nl = t0 == 0 || in[t0 - 1] == '\n';
  __syncthreads();
  K2_LEAN_STAMP(1);
  IntState is;
  uint32_t claimed_bytes = 0;  // kLeanClaim: name bytes of the S lines this thread claimed (names blob size)
  uint32_t claimed_vmax = 0;   // kLeanDirClaim: the largest value it claimed
  // (2) this thread's region: chunks c0 .. c0 + 3, its starts as one 64-bit mask
  const uint32_t c0 = kLeanRegion * threadIdx.x;
  unsigned long long st;
  uint32_t n_nl;
  {
    unsigned long long nl;
    if constexpr (kLeanRegion == 4) {
      const uint2 v = *(const uint2*)(nlm + c0);
      nl = (unsigned long long)v.x | ((unsigned long long)v.y << 32);
    } else {
      nl = *(const uint32_t*)(nlm + c0);
    }
    const unsigned long long prev = c0 ? (unsigned long long)(nlm[c0 - 1] >> 15) : (tile_prev_nl ? 1ull : 0ull);
    st = (nl << 1) | prev;
    if constexpr (kLeanRegion == 2) st &= 0xFFFFFFFFull;
    const uint64_t r0 = t0 + 16ull * c0;  // a start needs a byte: none at or past len
    if (r0 + 16 * kLeanRegion > len) st &= r0 >= len ? 0ull : ((1ull << (len - r0)) - 1);
    n_nl = (uint32_t)__popcll(nl);
  }
  const uint32_t n_st = (uint32_t)__popcll(st);
  uint32_t n_s = 0, n_e = 0, n_po = 0;
  // the first kLeanBatch starts: offsets, then every first / second byte load in flight at once,
  // then the kinds (2-bit codes kept for the record pass); any further start one by one.  An
  // unsupported record (parser.py:125-131) fails the pass unless op.tunk takes it: its index among
  // the thread's starts and its offset, ranked after the scan (the warning's line, k_tile_lean_check) —
  // a first byte >= 0x80 still fails (its warning is a UnicodeDecodeError: the full parse decides)
  uint32_t codes = 0, q_unk = ~0u, o_unk = 0;
  auto unsupported = [&](uint32_t q, uint32_t o, uint32_t b0) {
    if (!op.tunk || b0 >= 0x80u) {
      is.fail = 1;
    } else if (q_unk == ~0u) {
      q_unk = q;
      o_unk = o;
    }
  };
  {
    unsigned long long m = st;
    uint32_t off[kLeanBatch];
#pragma unroll
    for (uint32_t q = 0; q < kLeanBatch; q++) {
      off[q] = m ? 16 * c0 + (uint32_t)__builtin_ctzll(m) : 0xFFFFu;
      m &= m - 1;
    }
    uint32_t x0[kLeanBatch], x1[kLeanBatch];
#pragma unroll
    for (uint32_t q = 0; q < kLeanBatch; q++) {
      const uint32_t o = off[q] == 0xFFFFu ? 0u : off[q];
      x0[q] = buf[o];
      x1[q] = buf[o + 1];
    }
#if G2N_CLASSIFY_FLAT
    // (round 6) branch-free: unsupported() as selects — the first unknown start that op.tunk takes, or
    // the failure for one it cannot (a first byte >= 0x80 or no op.tunk)
#pragma unroll
    for (uint32_t q = 0; q < kLeanBatch; q++) {
      const bool on = off[q] != 0xFFFFu;
      const bool exact = (t0 + off[q] + 1 >= len) | (x0[q] == '\n') | (x1[q] == '\t') | (x1[q] == '\n');
      bool unk = false;
      uint32_t code = lean_code_flat(x0[q], exact, &unk);
      code = on ? code : 0u;
      unk = unk & on;
      const bool hard = unk & ((op.tunk == nullptr) | (x0[q] >= 0x80u));
      is.fail |= hard ? 1u : 0u;
      const bool take = unk & !hard & (q_unk == ~0u);
      q_unk = take ? q : q_unk;
      o_unk = take ? off[q] : o_unk;
      codes |= code << (2 * q);
      n_s += code == 1;
      n_e += code == 2;
      n_po += code == 3;
    }
#else
#pragma unroll
    for (uint32_t q = 0; q < kLeanBatch; q++) {
      if (off[q] == 0xFFFFu) continue;
      const bool exact = t0 + off[q] + 1 >= len || x0[q] == '\n' || x1[q] == '\t' || x1[q] == '\n';
      const uint8_t kd = line_kind((uint8_t)x0[q], exact);
      if (kd == kUnknown) unsupported(q, off[q], x0[q]);
      const uint32_t code = lean_code(kd);
      codes |= code << (2 * q);
      n_s += code == 1;
      n_e += code == 2;
      n_po += code == 3;
    }
#endif
#pragma unroll 1
    for (uint32_t q = kLeanBatch; m; q++) {  // more than kLeanBatch lines start in these 64 bytes
      const uint32_t o = 16 * c0 + (uint32_t)__builtin_ctzll(m);
      m &= m - 1;
      const uint8_t kd = kind_at(buf, o, t0 + o, len);
      if (kd == kUnknown) unsupported(q, o, buf[o]);
      const uint32_t code = lean_code(kd);
      n_s += code == 1;
      n_e += code == 2;
      n_po += code == 3;
    }
  }
  K2_LEAN_STAMP(2);
  unsigned long long tot;
#if G2N_DPP_SCAN
  const unsigned long long ex = lean_block_scan<kLeanTPB>(n_st, n_s, n_e, &tot, red64);
#else
  const unsigned long long ex = block_excl_scan_n64<kLeanTPB>(
      (unsigned long long)n_st | ((unsigned long long)n_s << 20) | ((unsigned long long)n_e << 40), &tot, red64);
#endif
  const uint32_t n_lines = (uint32_t)(tot & 0xFFFFFu), s_tot = (uint32_t)((tot >> 20) & 0xFFFFFu),
                 e_tot = (uint32_t)(tot >> 40);
  if (q_unk != ~0u) atomicMin(&s_unk, (((uint32_t)(ex & 0xFFFFFu) + q_unk) << 15) | o_unk);  // (read at the finish)
  K2_LEAN_STAMP(3);
  const uint32_t lim = (uint32_t)(len - t0 < kTile + kLeanHalo ? len - t0 : kTile + kLeanHalo);  // staged bytes
  if (kGrouped && threadIdx.x == 0)  // this tile's place in its group slot (published by the barrier below)
    s_gbase = n_lines && e_tot <= op.tile_pad ? atomicAdd(&gcount[tile >> op.gshift], e_tot * op.ktrip) : 0u;
  // the tile's last line's end (1 + its '\n', a virtual one at EOF; 0: past the staged window), found
  // once by the thread holding that line's start, so every line's end is a record read (line_next)
  if (n_st && (uint32_t)(ex & 0xFFFFFu) + n_st == n_lines) {  // (published by the records' barrier)
    const uint32_t o = 16 * c0 + 63u - (uint32_t)__builtin_clzll(st);
    uint32_t c = o >> 4;
    uint32_t mm = (uint32_t)nlm[c] & ~((1u << (o & 15)) - 1u);
    const uint32_t ce = (lim + 15) / 16;
    while (!mm && ++c < ce) mm = nlm[c];
    s_last_end = mm ? 16 * c + (uint32_t)__builtin_ctz(mm) + 1 : (lim == len - t0 ? lim + 1 : 0u);
  }
  // windows of kLeanLines lines (one for lines of >= 16 bytes on average): each thread writes the
  // records of its lines ranked in [w0, w0 + kLeanLines] (one past: the window's last line ends where
  // the next one starts), then the window's lines are parsed
  for (uint32_t w0 = 0; w0 < n_lines; w0 += kLeanLines) {
    if (w0) __syncthreads();  // the previous window's records are read
    {
      uint32_t r = (uint32_t)(ex & 0xFFFFFu), sp = (uint32_t)((ex >> 20) & 0xFFFFFu), ep = (uint32_t)(ex >> 40);
      unsigned long long m = st;
#pragma unroll 1
      for (uint32_t q = 0; q < n_st && r <= w0 + kLeanLines; q++, r++) {
        const uint32_t o = 16 * c0 + (uint32_t)__builtin_ctzll(m);
        m &= m - 1;
        const uint32_t code = q < kLeanBatch ? (codes >> (2 * q)) & 3u : lean_code(kind_at(buf, o, t0 + o, len));
        if (w0 == 0 && code == 1 && ep) is.fail = 1;  // an S line after an edge line: not the decimal-id layout
        if (r >= w0) rec[r - w0] = o | (code << 15) | ((code == 1 ? sp : ep) << 17);
        sp += code == 1;
        ep += code == 2;
      }
    }
    __syncthreads();
    if (w0 == 0) {
      K2_LEAN_STAMP(4);
      if (kGrouped) {
        const uint64_t b = (tile >> op.gshift) * gcap + s_gbase;
        op.rows += b;
        op.cols += b;
        if (kExt && op.wenc) op.wenc += b;
      }
    }
    // (3) lane-parallel lines
    const uint32_t n_win = n_lines - w0 < kLeanLines ? n_lines - w0 : kLeanLines;
    // line j's end: 1 + its '\n' (a virtual one at EOF), tile-local; 0 = past the staged window
    auto line_next = [&](uint32_t j, uint32_t o) -> uint32_t {  // (rec[n_win] is in bounds: a select, no branch)
      const uint32_t nx = rec[j + 1] & 0x7FFFu, last = s_last_end;
      return w0 + j + 1 < n_lines ? nx : last;
    };
    if constexpr (kMode == kLeanDirEdges) {
      // kDL lines per thread per step: their 2 kDL random reads all in flight at once (the pass is
      // bound by the random-read rate of the direct array, not by the parse)
      constexpr uint32_t kDL = G2N_DIRECT_LINES;
#pragma unroll 1
      for (uint32_t j0 = threadIdx.x; j0 < n_win; j0 += kDL * kLeanTPB) {
        uint32_t va[kDL], vb[kDL], eo[kDL], ori[kDL];  // values (< 2^28), edge index in the window's tile
        double wv[kDL];
        bool act[kDL];
#pragma unroll
        for (uint32_t q = 0; q < kDL; q++) {
          const uint32_t j = j0 + q * kLeanTPB;
          act[q] = false;
          va[q] = vb[q] = eo[q] = ori[q] = 0;
          wv[q] = 1.0;
          if (j >= n_win) continue;
          const uint32_t x = rec[j];
          if (((x >> 15) & 3u) != 2u) continue;
          const uint32_t o = x & 0x7FFFu;
          const uint32_t next = line_next(j, o);
          uint32_t xa, la, xb, lb;
          uint64_t a, b;
          if (!next || !lean_edge_names<kExt>(buf, tabm, o, next, xa, la, xb, lb, &H, &ori[q], &wv[q]) ||
              !lean_direct_value(buf, H, xa, la, a) || !lean_direct_value(buf, H, xb, lb, b)) {
            is.fail = 1;
            continue;
          }
          act[q] = true;
          va[q] = (uint32_t)a;
          vb[q] = (uint32_t)b;
          eo[q] = x >> 17;
        }
        uint32_t ida[kDL], idb[kDL];
#pragma unroll
        for (uint32_t q = 0; q < kDL; q++) {
          ida[q] = act[q] ? H.direct[va[q]] : 0u;
          idb[q] = act[q] ? H.direct[vb[q]] : 0u;
        }
#pragma unroll
        for (uint32_t q = 0; q < kDL; q++) {
          if (!act[q]) continue;
          if (ida[q] == ~0u || idb[q] == ~0u) {  // a key no S line defined: a new node (not S-first)
            is.fail = 1;
            continue;
          }
          lean_edge_out<kExt>(H, ebase + eo[q], ida[q], idb[q], ori[q], wv[q]);
        }
      }
      continue;  // next window
    }
    if constexpr (kMode == kLeanEdges) {
      // kHL lines per thread per step: their names' first probes are all in flight at once
      constexpr int kHL = G2N_HL_LINES;
#pragma unroll 1
      for (uint32_t j0 = threadIdx.x; j0 < n_win; j0 += kHL * kLeanTPB) {
        bool act[kHL];
        uint32_t xs[2 * kHL], ls[2 * kHL], ori[kHL];
        double wv[kHL];
        uint64_t ebs[kHL];
#pragma unroll
        for (int q = 0; q < kHL; q++) {
          const uint32_t j = j0 + q * kLeanTPB;
          act[q] = false;
          ebs[q] = 0;
          ori[q] = 0;
          wv[q] = 1.0;
          xs[2 * q] = xs[2 * q + 1] = 0;
          ls[2 * q] = ls[2 * q + 1] = 0;
          if (j >= n_win) continue;
          const uint32_t x = rec[j];
          if (((x >> 15) & 3u) != 2u) continue;
          const uint32_t o = x & 0x7FFFu;
          const uint32_t next = line_next(j, o);
          if (!next || !lean_edge_names<kExt>(buf, tabm, o, next, xs[2 * q], ls[2 * q], xs[2 * q + 1], ls[2 * q + 1],
                                              &H, &ori[q], &wv[q])) {
            is.fail = 1;
            continue;
          }
          act[q] = true;
          ebs[q] = ebase + (x >> 17);  // the edge index
        }
        KeyHead kh[2 * kHL];
        uint64_t h[2 * kHL];
        uint4 ea[2 * kHL], eb[2 * kHL];
#pragma unroll
        for (int k = 0; k < 2 * kHL; k++) {
          h[k] = lean_key(in, buf, t0, xs[k], ls[k], kh[k]);
          if (act[k >> 1]) {
            const DictEntry* e = H.table + (h[k] & H.mask);
            ea[k] = ((const uint4*)e)[0];
            eb[k] = ((const uint4*)e)[1];
          }
        }
#pragma unroll
        for (int q = 0; q < kHL; q++) {
          if (!act[q]) continue;
          const uint32_t ida = lean_find(in, H, kh[2 * q], h[2 * q], t0 + xs[2 * q], ea[2 * q], eb[2 * q]);
          const uint32_t idb =
              lean_find(in, H, kh[2 * q + 1], h[2 * q + 1], t0 + xs[2 * q + 1], ea[2 * q + 1], eb[2 * q + 1]);
          if (ida == ~0u || idb == ~0u) {  // a key no S line defined: a new node (not S-first)
            is.fail = 1;
            continue;
          }
          lean_edge_out<kExt>(H, ebs[q], ida, idb, ori[q], wv[q]);
        }
      }
      continue;  // next window
    }
#if G2N_LEAN_PAIR
    // decimal ids: two lines per lane per step, every stage's LDS loads for both lines issued
    // together (rec -> tab window -> name words), the checks branch-free (lean_line's rules)
    if constexpr (kMode == kLeanDecimal) {
#pragma unroll 1
      for (uint32_t j0 = threadIdx.x; j0 < n_win; j0 += 2 * kLeanTPB) {
        uint32_t o[2], nx[2], cd[2], pf[2];
#pragma unroll
        for (int q = 0; q < 2; q++) {
          const uint32_t j = j0 + (uint32_t)q * kLeanTPB;
          const uint32_t x = j < n_win ? rec[j] : 0u;
          cd[q] = (x >> 15) & 3u;
          o[q] = x & 0x7FFFu;
          pf[q] = x >> 17;
          nx[q] = cd[q] ? line_next(j, o[q]) : 0u;
        }
        uint64_t w[2];
#pragma unroll
        for (int q = 0; q < 2; q++) w[q] = tab_window(buf, tabm, o[q] >> 4);
        uint32_t xa[2], la[2], xb[2], lb[2], oa[2], ob[2];
        bool good[2];
#pragma unroll
        for (int q = 0; q < 2; q++) {
          const uint32_t n = nx[q] - 1 - o[q];
          uint64_t m = (w[q] >> (o[q] & 15)) & ((1ull << (n > 48 ? 48 : n)) - 1);
          const uint32_t pc = (uint32_t)__popcll(m);
          uint32_t p[6];
#pragma unroll
          for (int k = 0; k < 6; k++) {
            p[k] = m ? (uint32_t)__builtin_ctzll(m) : n;
            m &= m - 1;
          }
          const bool s_ok = pc >= 1 && (pc >= 2 || n <= 48);
          const bool e_ok = n <= 48 && pc >= 5 && p[2] - p[1] == 2 && p[4] - p[3] == 2;
          const bool po_ok = pc >= 2;
          good[q] = cd[q] == 0 || (nx[q] != 0 && (cd[q] == 1 ? s_ok : cd[q] == 2 ? e_ok : po_ok));
          const bool s = cd[q] == 1 && good[q], e = cd[q] == 2 && good[q];
          xa[q] = s || e ? o[q] + p[0] + 1 : 0u;
          la[q] = s || e ? p[1] - p[0] - 1 : 0u;
          xb[q] = e ? o[q] + p[2] + 1 : 0u;
          lb[q] = e ? p[3] - p[2] - 1 : 0u;
          oa[q] = e ? o[q] + p[1] + 1 : 0u;  // the orientation bytes
          ob[q] = e ? o[q] + p[3] + 1 : 0u;
        }
        uint64_t wa0[2], wa1[2], wb0[2], wb1[2];
        uint32_t c2[2], c4[2];
#pragma unroll
        for (int q = 0; q < 2; q++) {
          const uint32_t a = xa[q] & ~7u, b = xb[q] & ~7u;
          wa0[q] = *(const uint64_t*)(buf + a);
          wa1[q] = *(const uint64_t*)(buf + a + 8);
          wb0[q] = *(const uint64_t*)(buf + b);
          wb1[q] = *(const uint64_t*)(buf + b + 8);
          c2[q] = buf[oa[q]];
          c4[q] = buf[ob[q]];
        }
#pragma unroll
        for (int q = 0; q < 2; q++) {
          if (!good[q]) {
            is.fail = 1;
            continue;
          }
          if (cd[q] == 1) {  // S line: its S index pf (no edge precedes it in the tile)
            if (is.fail) continue;
            uint64_t v;
            const bool dok = la[q] <= 8 ? dec_words(wa0[q], wa1[q], xa[q], la[q], &v) : dec_lds(buf, xa[q], la[q], &v);
            if (!dok) is.fail = 1;
            else is.s_name(op, v, pf[q]);
          } else if (cd[q] == 2) {
            if ((c2[q] != '+' && c2[q] != '-') || (c4[q] != '+' && c4[q] != '-') || pf[q] >= op.tile_pad) {
              is.fail = 1;
              continue;
            }
            if (is.fail) continue;
            uint64_t a, b;
            const bool aok = la[q] <= 8 ? dec_words(wa0[q], wa1[q], xa[q], la[q], &a) : dec_lds(buf, xa[q], la[q], &a);
            const bool bok = lb[q] <= 8 ? dec_words(wb0[q], wb1[q], xb[q], lb[q], &b) : dec_lds(buf, xb[q], lb[q], &b);
            if (!aok || !bok || a > op.n_seg || b > op.n_seg) {
              is.fail = 1;
              continue;
            }
            const uint32_t vm = (uint32_t)(a > b ? a : b);
            is.vmax = vm > is.vmax ? vm : is.vmax;
            const uint64_t eo = (uint64_t)pf[q] * op.ktrip;
            op.rows[eo] = (int32_t)(a - 1);
            op.cols[eo] = (int32_t)(b - 1);
            if (op.ktrip >= 2) {
              op.rows[eo + 1] = (int32_t)(b - 1);
              op.cols[eo + 1] = (int32_t)(a - 1);
            }
          }
        }
      }
      continue;  // next window
    }
#endif
    if (G2N_EDGE_ONLY && kMode == kLeanDecimal && !kExt && e_tot == n_lines) {  // (block-uniform) edge lines only: no
#pragma unroll 1                                               // record-kind branches (round 6)
      for (uint32_t j = threadIdx.x; j < n_win; j += kLeanTPB) {
        const uint32_t x = rec[j];
        const uint32_t o = x & 0x7FFFu, eb = x >> 17;
        const uint32_t next = line_next(j, o);
#if G2N_EDGE_FLAT
        uint64_t a, b;
        if (!lean_edge_flat(buf, tabm, o, next, op, kTile + kLeanHalo - 8u, &a, &b) | (eb >= op.tile_pad) |
            (a > op.n_seg) | (b > op.n_seg)) {
          is.fail = 1;  // (the general path decides; a key past the S lines is not an S key: int_edge_id)
          continue;
        }
        const uint32_t vm = (uint32_t)(a > b ? a : b);
        is.vmax = vm > is.vmax ? vm : is.vmax;
        const uint32_t eo = (eb & 0xFFFFFu) * (op.ktrip & 0xFu);  // (24-bit: eb < tile_pad, ktrip <= 4; grouped:
                                                                  // the tile's base is in rows / cols)
        op.rows[eo] = (int32_t)(a - 1);
        op.cols[eo] = (int32_t)(b - 1);
        if (op.ktrip >= 2) {
          op.rows[eo + 1] = (int32_t)(b - 1);
          op.cols[eo + 1] = (int32_t)(a - 1);
        }
#else
        if (!next || !lean_line<false>(buf, tabm, o, next, kEdge, t0, 0ull, eb, op, TouchOut{}, is))
          is.fail = 1;
#endif
      }
      continue;  // next window
    }
#pragma unroll 1
    for (uint32_t j = threadIdx.x; j < n_win; j += kLeanTPB) {
      const uint32_t x = rec[j];
      const uint32_t code = (x >> 15) & 3u;
      if (code == 0) continue;
      const uint32_t o = x & 0x7FFFu, pref = x >> 17;
      uint32_t next = line_next(j, o);
      if (!next) {  // the line runs past the staged window (a long sequence or path): an S, P or O
        if (code == 2) {  // line needs only its first fields, which must then sit in the 48-byte tab
          is.fail = 1;    // view (lean_line / lean_s_name with a line longer than it); an edge line fails
          continue;
        }
        next = o + 50;
      }
      if (code == 3) {  // parser.py:229-247, 343-361: >= 3 fields, nothing else for the matrix
        const uint32_t n = next - 1 - o, sh = o & 15;
        const uint64_t w = tab_window(buf, tabm, o >> 4);
        if (__popcll((w >> sh) & ((1ull << (n > 48 ? 48 : n)) - 1)) < 2) is.fail = 1;  // the full parse decides
        continue;
      }
      if constexpr (kMode == kLeanDirClaim) {  // S line: direct[its value] = node id (S lines before) + pref
        if (code != 1) continue;
        uint32_t x, l;
        uint64_t v;
        if (!lean_s_name(buf, tabm, o, next, x, l) || !lean_direct_value(buf, H, x, l, v)) {
          is.fail = 1;
          continue;
        }
        const uint32_t id = (uint32_t)(sbase + pref);
#if G2N_DIRECT_STORE
        // a plain store: a repeated value leaves fewer filled slots than S lines, which one count of
        // the array after the pass finds (k_direct_filled; a verify pass re-staging the tiles measured
        // slower: 4.13 against 3.70 ms)
        H.direct[v] = id;
        claimed_vmax = (uint32_t)v > claimed_vmax ? (uint32_t)v : claimed_vmax;
#else
        if (atomicCAS(H.direct + v, ~0u, id) != ~0u) {  // a repeated S name: the classic tiers decide
          is.fail = 1;
          continue;
        }
#endif
        H.noff[id] = t0 + x;
        H.nlen[id] = l;
        claimed_bytes += l;
        continue;
      } else if constexpr (kMode == kLeanClaim) {  // S line: claim its name for node id (S lines before) + pref
        if (code != 1) continue;
        uint32_t x, l;
        if (!lean_s_name(buf, tabm, o, next, x, l)) {
          is.fail = 1;
          continue;
        }
        KeyHead kh;
        const uint64_t h = lean_key(in, buf, t0, x, l, kh);
        const uint32_t id = (uint32_t)(sbase + pref), tag = (uint32_t)(h >> 32);
        const unsigned long long mine = ((unsigned long long)tag << 32) | id;
        uint64_t idx = h & H.mask;
        bool done = false;
        for (uint64_t probe = 0; probe < H.max_probes && !done; probe++) {
          DictEntry* e = H.table + idx;
          unsigned long long cur = e->hdr;
          if (cur == kEmptySlot) {
            cur = atomicCAS(&e->hdr, kEmptySlot, mine);
            if (cur == kEmptySlot) {  // claimed: the key is published for the edge pass (a later launch)
              e->meta = ((unsigned long long)l << 40) | (t0 + x);
              e->k0 = (uint64_t)kh.k;
              e->k1 = (uint64_t)(kh.k >> 64);
              H.noff[id] = t0 + x;
              H.nlen[id] = l;
              claimed_bytes += l;
              done = true;
              break;
            }
          }
          if ((uint32_t)(cur >> 32) == tag) {  // a repeated S name (or a shared tag): the classic tiers decide
            is.fail = 1;
            done = true;
            break;
          }
          idx = (idx + 1) & H.mask;
        }
        if (!done) is.fail = 1;  // no free slot within the probe bound
        continue;
      } else {
        // S line: tb = its S index (no edge precedes it); edge line: eb = its edge index
        if (!lean_line<kExt>(buf, tabm, o, next, code == 1 ? kS : kEdge, t0, code == 1 ? pref : 0ull,
                       code == 1 ? 0ull : pref, op, TouchOut{}, is))
          is.fail = 1;
      }
    }
  }
  K2_LEAN_STAMP(5);
  if constexpr (kMode != kLeanDecimal) {  // K1 counted the tile already
    if (__ballot(is.fail) && (threadIdx.x & 63) == 0) ctl->int_fail = 1;
    if constexpr (kMode == kLeanClaim || kMode == kLeanDirClaim) {
      // the block's name bytes and largest value at H.tnb[block] (k_claim_totals adds / maxes them): one
      // atomic per wave on one address measured ~2.7 ms of a 3.3 ms claim pass (34K tiles x 8 waves,
      // serialised)
      uint32_t nb = claimed_bytes, vm = claimed_vmax;
      for (int o = 32; o > 0; o >>= 1) {
        nb += (uint32_t)__shfl_xor((int)nb, o, 64);
        vm = max(vm, (uint32_t)__shfl_xor((int)vm, o, 64));
      }
      if ((threadIdx.x & 63) == 0) red64[threadIdx.x >> 6] = nb | ((unsigned long long)vm << 32);
      __syncthreads();
      if (threadIdx.x == 0) {
        unsigned long long t = red64[0];
        for (uint32_t w = 1; w < kW; w++)
          t = ((t & 0xFFFFFFFFull) + (red64[w] & 0xFFFFFFFFull)) | (max(t >> 32, red64[w] >> 32) << 32);
        H.tnb[blockIdx.x] = t;
      }
    }
#ifdef G2N_K2_STAMPS
    K2_LEAN_STAMP(6);
    if (threadIdx.x == 0) {
      uint32_t hw, xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      g2n_k2_stamps[tile * kK2Stamps + 9] = ((unsigned long long)xcc << 32) | hw;
    }
#endif
    return;
  }
  // tile counts and premise evidence
  if (e_tot > op.tile_pad) is.fail = 1;  // more edges than the tile's slot holds
  uint32_t vm = is.vmax;
  int32_t dmn = is.dref == kNoS ? 0x7FFFFFFF : is.dref, dmx = is.dref;  // (kNoS is the int32 minimum)
#if G2N_DPP_SCAN
  // (n_nl <= 2^15 and n_po < 2^15 per tile: one packed 32-bit sum)
  const uint32_t c32 = wave_dpp_reduce(n_nl | (n_po << 16), 0u, dpp_add);
  unsigned long long cnt = (unsigned long long)(c32 & 0xFFFFu) | ((unsigned long long)(c32 >> 16) << 20);
  vm = wave_dpp_reduce(vm, 0u, dpp_max);
  if (s_tot) {  // (block-uniform) no S line: every lane holds the identities already
    dmn = (int32_t)wave_dpp_reduce((uint32_t)dmn, 0x7FFFFFFFu, dpp_smin);
    dmx = (int32_t)wave_dpp_reduce((uint32_t)dmx, 0x80000000u, dpp_smax);
  }
#else
  unsigned long long cnt = (unsigned long long)n_nl | ((unsigned long long)n_po << 20);  // per tile < 2^20 each
  for (int o = 32; o > 0; o >>= 1) {
    vm = max(vm, (uint32_t)__shfl_xor(vm, o, 64));
    dmn = min(dmn, (int32_t)__shfl_xor(dmn, o, 64));
    dmx = max(dmx, (int32_t)__shfl_xor(dmx, o, 64));
    cnt += __shfl_xor(cnt, o, 64);
  }
#endif
  __shared__ uint32_t rv[kW];
  __shared__ int32_t rmn[kW], rmx[kW];
  __shared__ unsigned long long rc[kW];
  if ((threadIdx.x & 63) == 0) {
    rv[threadIdx.x >> 6] = vm;
    rmn[threadIdx.x >> 6] = dmn;
    rmx[threadIdx.x >> 6] = dmx;
    rc[threadIdx.x >> 6] = cnt;
  }
  const unsigned long long failed = __ballot(is.fail);
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)kW; w++) {
      vm = max(vm, rv[w]);
      dmn = min(dmn, rmn[w]);
      dmx = max(dmx, rmx[w]);
      cnt += rc[w];
    }
    const uint32_t npo = (uint32_t)(cnt >> 20);
    TileCnt c;
    c.nl = cnt & 0xFFFFFu;
    c.lines = n_lines;
    c.segs = s_tot;
    c.edges = e_tot;
    c.touches = (uint64_t)s_tot + 2ull * e_tot;
    c.recs = (uint64_t)s_tot + e_tot + npo;
    tcnt_out[tile] = c;
    tlean[tile] = TileLean{dmn, dmx, vm};  // no S line: dmn > dmx (the check skips the tile)
    if (s_unk != ~0u) {
      op.tunk[tile] = s_unk;
      atomicMin(&ctl->warn_tile, (unsigned long long)tile);
    }
  }
  if (failed && (threadIdx.x & 63) == 0) ctl->int_fail = 1;
  K2_LEAN_STAMP(6);
#ifdef G2N_K2_STAMPS
  if (threadIdx.x == 0) {
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    g2n_k2_stamps[tile * kK2Stamps + 9] = ((unsigned long long)xcc << 32) | hw;
  }
#endif
}

// One block per tile (the hash modes skip the tiles they have nothing to do in before loading them).
#if G2N_LEAN_PAIR  // the LDS allows 3 blocks (6 waves per SIMD): keep the VGPRs to 80
#define G2N_LEAN_ATTR __attribute__((amdgpu_flat_work_group_size(kLeanTPB, kLeanTPB), amdgpu_waves_per_eu(6, 6)))
#else
#define G2N_LEAN_ATTR __launch_bounds__(kLeanTPB, kLeanTPB == 1024 ? 2 : 1)
#endif
template <int kMode, bool kGrouped, bool kExt = false>
__global__ void G2N_LEAN_ATTR
    k_tile_lean(const uint8_t* __restrict__ in, uint64_t len, ParseOpts op, Ctl* ctl, TileCnt* __restrict__ tcnt_out,
                TileLean* __restrict__ tlean, uint32_t* __restrict__ gcount, uint64_t gcap, HashLeanArgs H) {
  const uint64_t tile = kMode != kLeanDecimal && H.tlist ? (uint64_t)H.tlist[blockIdx.x] : (uint64_t)blockIdx.x;
  if constexpr (kMode != kLeanDecimal) {  // a pass that already failed elsewhere: the rest is wasted work
    if (*(volatile const unsigned long long*)&ctl->int_fail) return;
  }
  if constexpr (kMode == kLeanClaim || kMode == kLeanDirClaim) {  // tiles with S or P / O lines (block-uniform)
    const TileCnt c = H.tcnt[tile];
    if (c.segs == 0 && c.recs == c.segs + c.edges) return;
    if (c.segs && H.tbase[tile].edges) {  // an edge line before this tile's S lines
      if (threadIdx.x == 0) ctl->int_fail = 1;
      return;
    }
  } else if constexpr (kMode == kLeanEdges || kMode == kLeanDirEdges) {  // tiles with edge lines
    if (H.tcnt[tile].edges == 0) return;
  }
  LeanRegs R;
  R.load(in, len, tile * kTile);
#if G2N_K2_PREFETCH
  // experiment: warm the L2 / Infinity Cache with the tile the block G tiles on will stage (G = the
  // blocks resident at once, a multiple of the 8 XCDs: the same XCD's L2) — one dword per 128-byte
  // line, into a sink register kept live (and drained) to the end, so no later value shares it
  uint32_t sink = 0;
  const uint64_t pf = (tile + op.pf_dist) * kTile + 128ull * threadIdx.x;
  const bool do_pf = op.pf_dist && threadIdx.x < (kTile + kLeanHalo) / 128 && pf < len;
  if (do_pf) asm volatile("global_load_dword %0, %1, off" : "=v"(sink) : "v"(in + pf) : "memory");
#endif
  lean_tile<kMode, kGrouped, kExt>(in, len, op, ctl, tcnt_out, tlean, gcount, gcap, H, tile, R, ~0ull, 0);
#if G2N_K2_PREFETCH
  asm volatile("s_waitcnt vmcnt(0)" : : "v"(sink) : "memory");
#endif
}

// The decimal-id parse persistent: a block walks tiles blockIdx.x, + gridDim.x, ... and loads the
// next one's bytes into registers while it parses the current one (the staged loads' HBM latency
// was a quarter of a block's time with one tile per block: stamps).
#ifndef G2N_K2P_WAVES  // waves per SIMD the persistent parse is compiled for (LDS allows 6: VGPRs <= 80)
#define G2N_K2P_WAVES 6
#endif
template <bool kGrouped>
__global__ void __attribute__((amdgpu_flat_work_group_size(kLeanTPB, kLeanTPB), amdgpu_waves_per_eu(G2N_K2P_WAVES, G2N_K2P_WAVES)))
    k_tile_lean_p(const uint8_t* __restrict__ in, uint64_t len, ParseOpts op, Ctl* ctl, TileCnt* __restrict__ tcnt_out,
                  TileLean* __restrict__ tlean, uint32_t* __restrict__ gcount, uint64_t gcap, uint64_t n_tiles) {
  LeanRegs R;
  uint64_t tile = blockIdx.x;
  if (tile < n_tiles) R.load(in, len, tile * kTile);
#pragma unroll 1
  for (; tile < n_tiles; tile += gridDim.x) {
    if (tile != blockIdx.x) __syncthreads();  // the previous tile's LDS fully read
    lean_tile<kLeanDecimal, kGrouped>(in, len, op, ctl, tcnt_out, tlean, gcount, gcap, HashLeanArgs{}, tile, R,
                                      tile + gridDim.x, n_tiles);
  }
}

// Open-addressing dictionary, 32-byte entries: hdr = (hash tag << 32 | first touch),
// meta = (round << 32 | key length), then the first 16 key bytes.  A touch compares its
// key against an entry only when the entry was published in an EARLIER round (launch):
// the inline bytes are then visible, and one random access resolves the touch.  Touches
// meeting a same-tag entry claimed in the current round retry next round.  The
// representative is lowered with atomicMin to the FIRST touch of the key — the order of
// Python dict insertion (builders.py:194-198, 219-221).
//
// Probing reads the whole entry with one plain 32-byte load: everything an earlier launch
// wrote is visible to it, and a line fetched during this launch can only show an entry that
// is empty (-> atomic CAS), or claimed in this round (meta round >= this round: retried next
// round), or published earlier (immutable except for the representative, which only ever
// decreases — a stale one costs at most a redundant atomicMin).
//
// Modes.  kClaim: round 1, the S-line touches claim or find their keys; it also records
// first[t] (claimed here) for every touch.  kLookup: the general rounds
// >= 2 (representatives lowered, new keys claimed).  kFast: the single lookup round of the
// S-first fast path — after round 1 every claimed entry holds the node id its S touch ranks
// to (k_assign_first), so an edge touch reads its node id straight into tid[t].  That is the
// final id only if the key's first touch is the S touch: a touch with no key (new node) or one
// preceding the S touch (rank >= nid[t], the firsts before it) sets ctl->dict_general and the
// host redoes the dictionary with the general rounds.
enum : int { kModeClaim = 0, kModeLookup = 1, kModeFast = 2 };

template <int kMode>
__global__ void __launch_bounds__(kTPB) k_insert_round(const uint8_t* __restrict__ in, uint64_t in_len, TouchIn T,
                                                       uint64_t n_t, DictEntry* __restrict__ table, uint64_t mask,
                                                       uint64_t max_probes, uint32_t* __restrict__ slot,
                                                       uint8_t* __restrict__ tstate, uint32_t round, int bidir,
                                                       Ctl* ctl, uint8_t* __restrict__ first,
                                                       const uint32_t* __restrict__ nid,
                                                       uint32_t n_first,  // claim: S touches; fast: firsts
                                                       const uint32_t* __restrict__ inv, uint32_t* __restrict__ tid) {
  const uint64_t t = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  bool deferred = false;
  bool s_touch = false;
  if (t < n_t) {
    const uint8_t st = tstate[t];
    bool claimed = false;
    const bool active = kMode == kModeClaim ? st == 1 : st != 0;
    s_touch = kMode == kModeClaim && active;
    if (active) {
      const uint64_t no = T.noff[t];
      const uint32_t nl = T.nlen[t];
      const uint64_t oo = bidir ? T.ooff[t] : 0;
      const uint32_t ol = bidir ? T.olen[t] : 0;
      const KeyHead kh = key_head(in, in_len, no, nl, oo, ol, bidir != 0);
      const uint64_t h = key_hash(in, kh, no, nl, oo);
      const uint32_t tag = (uint32_t)(h >> 32);
      const unsigned long long mine = ((unsigned long long)tag << 32) | (uint32_t)t;
      const uint64_t k0 = (uint64_t)kh.k, k1 = (uint64_t)(kh.k >> 64);
      uint64_t idx = h & mask;
      bool done = false;
      for (uint64_t probe = 0; probe < max_probes; probe++) {
        DictEntry* e = table + idx;
        const uint4 lo = ((const uint4*)e)[0], hi = ((const uint4*)e)[1];  // one plain 32-byte load
        unsigned long long cur = ((unsigned long long)lo.y << 32) | lo.x;
        unsigned long long meta = ((unsigned long long)lo.w << 32) | lo.z;
        uint64_t e0 = ((uint64_t)hi.y << 32) | hi.x, e1 = ((uint64_t)hi.w << 32) | hi.z;
        if (cur == kEmptySlot) {
          if (kMode == kModeFast) {  // a key no S line defined: a new node
            ctl->dict_general = 1;
            done = true;
            break;
          }
          cur = atomicCAS(&e->hdr, kEmptySlot, mine);
          if (cur == kEmptySlot) {  // claimed: publish the key for later rounds
            e->k0 = k0;
            e->k1 = k1;
            e->meta = ((unsigned long long)round << 32) | kh.len;
            slot[t] = (uint32_t)idx;
            tstate[t] = 0;
            claimed = true;
            done = true;
            break;
          }
          // lost the race: the entry was claimed during this launch
          meta = __hip_atomic_load(&e->meta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if ((uint32_t)(cur >> 32) == tag) {
          if ((meta >> 32) >= round) {  // published in this launch (or not yet): next round
            deferred = true;
            break;
          }
          if ((uint32_t)meta == kh.len && e0 == k0 && e1 == k1 &&
              (kh.len <= 16 ||
               tail_eq(in, T, t, (kMode == kModeFast && inv) ? inv[(uint32_t)cur] : (uint32_t)cur, bidir != 0,
                      kh.len))) {
            if (kMode == kModeFast) {
              const uint32_t id = (uint32_t)cur;  // rank of the key's S touch among the firsts
              if (id >= (nid ? nid[t] : n_first)) ctl->dict_general = 1;  // this touch precedes it
              tid[t] = id;
            } else {
              if ((uint32_t)cur > (uint32_t)t) atomicMin(&e->hdr, mine);
              slot[t] = (uint32_t)idx;
              tstate[t] = 0;
            }
            done = true;
            break;
          }
        }
        idx = (idx + 1) & mask;
      }
      if (!done && !deferred) ctl->table_overflow = 1;  // the host retries with a larger table
    }
    if (kMode == kModeClaim) first[t] = claimed ? 1 : 0;  // S-first fast path: the claimers are the first touches
  }
  // one atomic per wave for the deferred count
  unsigned long long d = __ballot(deferred);
  if ((threadIdx.x & 63) == 0 && d) atomicAdd(&ctl->deferred, (unsigned long long)__popcll(d));
  if (kMode == kModeClaim) {  // an S touch after the first n_first touches: not an S prefix (rare store)
    const unsigned long long m = __ballot(s_touch && t >= n_first);
    if ((threadIdx.x & 63) == 0 && m) ctl->s_late = 1;
  }
}

#define G2N_INS(M)                                                                                               \
  template __global__ void k_insert_round<M>(const uint8_t*, uint64_t, TouchIn, uint64_t, DictEntry*, uint64_t,  \
                                             uint64_t, uint32_t*, uint8_t*, uint32_t, int, Ctl*, uint8_t*,       \
                                             const uint32_t*, uint32_t, const uint32_t*, uint32_t*);
G2N_INS(kModeClaim)
G2N_INS(kModeLookup)
G2N_INS(kModeFast)
#undef G2N_INS

__device__ inline uint32_t touch_key_len(const TouchIn& T, uint64_t t, int bidir) {
  return T.nlen[t] + (bidir ? 1 + T.olen[t] : 0);  // name [+ ":" + orientation]
}

// The S-first lookup round (kModeFast of k_insert_round) with kBatch touches per thread: each
// stage's loads (touch descriptors, key bytes, first probed entry) are issued for the whole
// batch before any is used, so a thread keeps kBatch dependent chains in flight instead of one.
// Touches t = block base + k * kTPB + lane: every stage stays coalesced across the wave.
template <int kBatch>
__global__ void __launch_bounds__(kTPB) k_lookup_fast(const uint8_t* __restrict__ in, uint64_t in_len, TouchIn T,
                                                      uint64_t n_t, const DictEntry* __restrict__ table,
                                                      uint64_t mask, uint64_t max_probes,
                                                      const uint8_t* __restrict__ tstate, int bidir, Ctl* ctl,
                                                      const uint32_t* __restrict__ nid, uint32_t n_first,
                                                      const uint32_t* __restrict__ inv, uint32_t* __restrict__ tid) {
  const uint64_t base = (uint64_t)blockIdx.x * (kTPB * kBatch) + threadIdx.x;
  bool act[kBatch];
  uint64_t no[kBatch], oo[kBatch];
  uint32_t nl[kBatch], ol[kBatch];
#pragma unroll
  for (int k = 0; k < kBatch; k++) {
    const uint64_t t = base + (uint64_t)k * kTPB;
    act[k] = t < n_t && tstate[t] != 0;
  }
#pragma unroll
  for (int k = 0; k < kBatch; k++) {
    const uint64_t t = base + (uint64_t)k * kTPB;
    if (act[k]) {
      no[k] = T.noff[t];
      nl[k] = T.nlen[t];
      oo[k] = bidir ? T.ooff[t] : 0;
      ol[k] = bidir ? T.olen[t] : 0;
    }
  }
  KeyHead kh[kBatch];
#pragma unroll
  for (int k = 0; k < kBatch; k++)
    if (act[k]) kh[k] = key_head(in, in_len, no[k], nl[k], oo[k], ol[k], bidir != 0);
  uint64_t h[kBatch];
  uint4 lo[kBatch], hi[kBatch];
#pragma unroll
  for (int k = 0; k < kBatch; k++) {
    if (act[k]) {
      h[k] = key_hash(in, kh[k], no[k], nl[k], oo[k]);
      const DictEntry* e = table + (h[k] & mask);
      lo[k] = ((const uint4*)e)[0];
      hi[k] = ((const uint4*)e)[1];
    }
  }
  bool general = false;
#pragma unroll
  for (int k = 0; k < kBatch; k++) {
    if (!act[k]) continue;
    const uint64_t t = base + (uint64_t)k * kTPB;
    const uint32_t tag = (uint32_t)(h[k] >> 32);
    const uint64_t k0 = (uint64_t)kh[k].k, k1 = (uint64_t)(kh[k].k >> 64);
    uint64_t idx = h[k] & mask;
    uint4 a = lo[k], b = hi[k];
    bool done = false;
    for (uint64_t probe = 0; probe < max_probes; probe++) {
      if (probe) {
        const DictEntry* e = table + idx;
        a = ((const uint4*)e)[0];
        b = ((const uint4*)e)[1];
      }
      const unsigned long long cur = ((unsigned long long)a.y << 32) | a.x;
      const unsigned long long meta = ((unsigned long long)a.w << 32) | a.z;
      const uint64_t e0 = ((uint64_t)b.y << 32) | b.x, e1 = ((uint64_t)b.w << 32) | b.z;
      if (cur == kEmptySlot) {  // a key no S line defined: a new node
        general = true;
        done = true;
        break;
      }
      if ((uint32_t)(cur >> 32) == tag) {
        if ((meta >> 32) >= 2) {  // claimed after round 1: cannot happen on this path
          general = true;
          done = true;
          break;
        }
        if ((uint32_t)meta == kh[k].len && e0 == k0 && e1 == k1 &&
            (kh[k].len <= 16 || tail_eq(in, T, t, inv ? inv[(uint32_t)cur] : (uint32_t)cur, bidir != 0,
                                        kh[k].len))) {
          const uint32_t id = (uint32_t)cur;  // rank of the key's S touch among the firsts
          if (id >= (nid ? nid[t] : n_first)) general = true;  // this touch precedes it
          tid[t] = id;
          done = true;
          break;
        }
      }
      idx = (idx + 1) & mask;
    }
    if (!done) ctl->table_overflow = 1;
  }
  if (__ballot(general) && (threadIdx.x & 63) == 0) ctl->dict_general = 1;
}

template __global__ void k_lookup_fast<2>(const uint8_t*, uint64_t, TouchIn, uint64_t, const DictEntry*, uint64_t,
                                          uint64_t, const uint8_t*, int, Ctl*, const uint32_t*, uint32_t,
                                          const uint32_t*, uint32_t*);


// S-prefix dictionary (every S touch precedes every edge touch, no S key repeated): the node id
// of an S touch is its touch index; klen[id] for the names blob.
__global__ void __launch_bounds__(kTPB) k_key_len(TouchIn T, uint64_t n, int bidir, uint32_t* __restrict__ klen) {
  const uint64_t t = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  if (t < n) klen[t] = touch_key_len(T, t, bidir);
}

// S-first fast path: each round-1 claimer's entry takes its node id (its rank among the firsts);
// inv[id] = the touch holding the key's bytes, klen[id] = its length (names blob).
__global__ void __launch_bounds__(kTPB) k_assign_first(DictEntry* __restrict__ table, TouchIn T, uint64_t n_t,
                                                       int bidir, const uint8_t* __restrict__ first,
                                                       const uint32_t* __restrict__ slot,
                                                       const uint32_t* __restrict__ nid, uint32_t* __restrict__ inv,
                                                       uint32_t* __restrict__ klen) {
  const uint64_t t = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  if (t >= n_t || !first[t]) return;
  const uint32_t id = nid[t];
  ((uint32_t*)&table[slot[t]].hdr)[0] = id;  // the low half of hdr (little endian): no read back
  inv[id] = (uint32_t)t;
  klen[id] = touch_key_len(T, t, bidir);
}

// General path, after all rounds: every occupied entry holds the FIRST touch of its key.
__global__ void __launch_bounds__(kTPB) k_mark_first(const DictEntry* __restrict__ table, uint64_t cap,
                                                     uint8_t* __restrict__ first) {
  const uint64_t s = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  if (s >= cap) return;
  const unsigned long long v = table[s].hdr;
  if (v != kEmptySlot) first[(uint32_t)v] = 1;
}

// General path: each entry's representative -> its node id (= rank of the first touch).
__global__ void __launch_bounds__(kTPB) k_assign_ids(DictEntry* __restrict__ table, uint64_t cap,
                                                     const uint32_t* __restrict__ nid, uint32_t* __restrict__ inv,
                                                     uint32_t* __restrict__ klen) {
  const uint64_t s = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  if (s >= cap) return;
  const unsigned long long v = table[s].hdr;
  if (v == kEmptySlot) return;
  const uint32_t rep = (uint32_t)v, id = nid[rep];
  table[s].hdr = (v & 0xFFFFFFFF00000000ull) | id;
  inv[id] = rep;
  klen[id] = (uint32_t)table[s].meta;
}

__global__ void k_node_count(const uint8_t* __restrict__ first, const uint32_t* __restrict__ nid, uint64_t n_t,
                             Ctl* ctl) {
  ctl->n_nodes = n_t ? (uint64_t)nid[n_t - 1] + first[n_t - 1] : 0;
}

__global__ void k_names_total(const uint32_t* __restrict__ klen, uint64_t n_nodes, int64_t* __restrict__ offs,
                              Ctl* ctl) {
  const uint64_t total = n_nodes ? (uint64_t)offs[n_nodes - 1] + klen[n_nodes - 1] : 0;
  offs[n_nodes] = (int64_t)total;
  ctl->names_len = total;
}

// names blob in id order (builders.py:284-288 node_list): node `id` <- the key bytes of inv[id]
// A name of at most 16 bytes comes from three aligned 8-byte loads (all in flight together) and goes
// out as predicated byte stores; a longer one, or one within 24 bytes of the input's end, byte by
// byte (a dependent load per byte held the kernel at ~2 ms for C4's 50M names beside the finish)
__global__ void __launch_bounds__(kTPB) k_names(const uint8_t* __restrict__ in, uint64_t in_len, TouchIn T,
                                                uint64_t n_nodes, const uint32_t* __restrict__ inv,
                                                const int64_t* __restrict__ offs, int bidir,
                                                uint8_t* __restrict__ blob) {
  const uint64_t id = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  if (id >= n_nodes) return;
  const uint64_t t = inv ? inv[id] : id;  // S-prefix dictionary: id == touch
  const uint64_t o = (uint64_t)offs[id];
  const uint64_t no = T.noff[t];
  const uint32_t nl = T.nlen[t];
  // (aligned on the address itself: the input may start anywhere in its allocation, which is aligned)
  const uint8_t* p = in + no;
  const uint64_t* w = (const uint64_t*)((uintptr_t)p & ~(uintptr_t)7);
  if (nl <= 16 && (const uint8_t*)(w + 3) <= in + in_len) {
    const uint64_t w0 = w[0], w1 = w[1], w2 = w[2];
    const uint32_t sh = (uint32_t)((uintptr_t)p & 7) * 8;
    const uint64_t lo = sh ? (w0 >> sh) | (w1 << (64 - sh)) : w0, hi = sh ? (w1 >> sh) | (w2 << (64 - sh)) : w1;
#pragma unroll
    for (uint32_t j = 0; j < 16; j++)
      if (j < nl) blob[o + j] = (uint8_t)((j < 8 ? lo >> (8 * j) : hi >> (8 * (j - 8))) & 0xFF);
  } else {
    for (uint32_t j = 0; j < nl; j++) blob[o + j] = in[no + j];
  }
  if (bidir) {
    const uint64_t oo = T.ooff[t];
    const uint32_t ol = T.olen[t];
    blob[o + nl] = ':';
    for (uint32_t j = 0; j < ol; j++) blob[o + nl + 1 + j] = (oo & kConstFlag) ? (uint8_t)(oo & 0xFF) : in[oo + j];
  }
}

// Names of a bidirected lean hash / direct build: S line k's name (noff / nlen, soff = the exclusive
// scan of nlen) as node 2k "name:+" and node 2k + 1 "name:-" (builders.py:190-198: S minting both)
__global__ void __launch_bounds__(kTPB) k_names_lean_bidir(const uint8_t* __restrict__ in,
                                                           const uint64_t* __restrict__ noff,
                                                           const uint32_t* __restrict__ nlen,
                                                           const int64_t* __restrict__ soff, uint64_t n_s,
                                                           int64_t* __restrict__ offs, uint8_t* __restrict__ blob) {
  const uint64_t k = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  if (k > n_s) return;
  const uint64_t o = 2 * (uint64_t)soff[k] + 4 * k;
  offs[2 * k] = (int64_t)o;
  if (k == n_s) return;
  const uint32_t nl = nlen[k];
  offs[2 * k + 1] = (int64_t)(o + nl + 2);
  const uint8_t* src = in + noff[k];
  for (uint32_t j = 0; j < nl; j++) {
    const uint8_t b = src[j];
    blob[o + j] = b;
    blob[o + nl + 2 + j] = b;
  }
  blob[o + nl] = ':';
  blob[o + nl + 1] = '+';
  blob[o + 2 * nl + 2] = ':';
  blob[o + 2 * nl + 3] = '-';
}

// Names of a decimal-id build (the premise held: S line k names "k+1", S lines first): node id's
// key is str(k + 1) (bidirected: id = 2k + [ori == '-'], key str(k + 1) + ":+" / ":-"), so the
// names blob and its offsets are arithmetic — no key lengths, scan or gathers from the input.
__device__ __host__ inline uint32_t dec_digits(uint64_t v) {
  uint32_t d = 1;
  for (uint64_t p = 10; v >= p && d < 20; p *= 10) d++;
  return d;
}
__device__ __host__ inline uint64_t dec_digits_upto(uint64_t v) {  // sum of dec_digits(k), k = 1..v
  uint64_t s = 0, lo = 1;
  for (uint32_t d = 1; lo <= v && d < 20; d++, lo *= 10) {
    const uint64_t hi = lo * 10 - 1, top = v < hi ? v : hi;
    s += (top - lo + 1) * d;
  }
  return s;
}
__device__ __host__ inline uint64_t dec_name_off(uint64_t id, int bidir) {  // offset of node id's key
  if (!bidir) return dec_digits_upto(id);
  const uint64_t k = id >> 1;
  return 2 * (dec_digits_upto(k) + 2 * k) + ((id & 1) ? dec_digits(k + 1) + 2 : 0);
}

// node k's key str(k + 1) (bidirected: + ":+" / ":-"), byte stores.  It runs on the side stream beside
// F1, so what counts is what it takes from F1 (0.2-0.3 ms of F1's time on C4).  Measured dead ends
// (same box, tools/gpu_r4r.sh / gpu_r4u.sh): the block's names staged in LDS and written in 16-byte
// stores (+0.12-0.15 ms per build), the blob written output-centric (a thread per 16 aligned bytes,
// the names' run found by arithmetic: +0.3 ms, VALU-heavy beside F1), the names written by the
// tile-local parse as it meets each S line (K2 +0.34 ms, F1 -0.3: no gain), the names forked beside
// the partition instead of F1 (+0.4 ms on it), non-temporal stores (+0.2-0.5 ms).
// (pl bytes of pre before every key: the prefixed decimal layout, ParseOpts::dpre)
__global__ void __launch_bounds__(kTPB) k_names_dec(uint64_t n_nodes, int bidir, int64_t* __restrict__ offs,
                                                    uint8_t* __restrict__ blob, uint64_t pre, uint32_t pl) {
  const uint64_t id = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  if (id > n_nodes) return;
  uint64_t o = dec_name_off(id, bidir) + (uint64_t)pl * id;
  offs[id] = (int64_t)o;
  if (id == n_nodes) return;
  for (uint32_t j = 0; j < pl; j++) blob[o + j] = (uint8_t)(pre >> (8 * j));
  o += pl;
  uint32_t v = (uint32_t)((bidir ? id >> 1 : id) + 1);  // node ids < 2^31
  const uint32_t d = dec_digits(v);
  for (uint32_t j = d; j-- > 0;) {
    blob[o + j] = (uint8_t)('0' + v % 10u);
    v /= 10u;
  }
  if (bidir) {
    blob[o + d] = ':';
    blob[o + d + 1] = (id & 1) ? '-' : '+';
  }
}

// ============================================================ K6: triplets ========
// numpy's np.array(list_of_python_floats, dtype) element conversion (builders.py:281)
template <class T>
struct Cast;
template <>
struct Cast<uint8_t> {  // bool: w != 0
  __device__ static uint32_t go(double w, uint8_t* o) { *o = (w != 0.0) ? 1 : 0; return 0; }
};
template <>
struct Cast<int8_t> {
  __device__ static uint32_t go(double w, int8_t* o) {
    if (w != w) return kErrCastNan;
    if (__builtin_isinf(w)) return kErrCastInf;
    double t = __builtin_trunc(w);
    if (t < -128.0 || t > 127.0) return kErrCastOverflow;
    *o = (int8_t)(int)t;
    return 0;
  }
};
template <>
struct Cast<int32_t> {
  __device__ static uint32_t go(double w, int32_t* o) {
    if (w != w) return kErrCastNan;
    if (__builtin_isinf(w)) return kErrCastInf;
    double t = __builtin_trunc(w);
    if (t < -2147483648.0 || t > 2147483647.0) return kErrCastOverflow;
    *o = (int32_t)t;
    return 0;
  }
};
template <>
struct Cast<float> {  // x86 cvtsd2ss: NaN keeps sign, payload truncated, quiet bit set
  __device__ static uint32_t go(double w, float* o) {
    if (w != w) {
      uint64_t b = f64_bits(w);
      uint32_t f = (uint32_t)(b >> 32 & 0x80000000u) | 0x7FC00000u | (uint32_t)((b >> 29) & 0x3FFFFFu);
      *o = __uint_as_float(f);
    } else {
      *o = (float)w;
    }
    return 0;
  }
};
template <>
struct Cast<double> {
  __device__ static uint32_t go(double w, double* o) { *o = w; return 0; }
};

// tid: node id per touch (S-first fast path, a streaming read) — else slot -> table entry -> id.
template <class T>
__global__ void __launch_bounds__(kTPB) k_triplets(EdgeIn E, uint64_t n_e, const uint32_t* __restrict__ slot,
                                                   const DictEntry* __restrict__ table,
                                                   const uint32_t* __restrict__ tid, int tpe, int gd,
                                                   int32_t* __restrict__ rows, int32_t* __restrict__ cols,
                                                   T* __restrict__ data, Ctl* ctl) {
  const uint64_t e = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  if (e >= n_e) return;
  const uint64_t tb = E.tb[e];
  auto id = [&](uint64_t t) -> int32_t {
    return tid ? (int32_t)tid[t] : (int32_t)(uint32_t)table[slot[t]].hdr;
  };
  T v;
  const double wv = E.w[e];
  uint32_t err = Cast<T>::go(wv, &v);
  if (std::is_same<T, float>::value && !__builtin_isinf(wv) && wv == wv && __builtin_isinf((double)v))
    atomicAdd(&ctl->n_f32_overflow, 1ull);
  const int k = tpe == 4 ? 4 : (gd ? 1 : 2);
  const uint64_t o = e * (uint64_t)k;
  if (err) {
    atomicMin(&ctl->cast_key, (unsigned long long)((o << 4) | err));
    return;
  }
  int32_t a = id(tb), b = id(tb + 1);
  rows[o] = a;
  cols[o] = b;
  data[o] = v;
  if (k >= 2) {
    rows[o + 1] = b;
    cols[o + 1] = a;
    data[o + 1] = v;
  }
  if (k == 4) {  // bidirected twin (v:rev(ori_to), u:rev(ori_from)), both directions
    int32_t c = id(tb + 2), d = id(tb + 3);
    rows[o + 2] = c;
    cols[o + 2] = d;
    data[o + 2] = v;
    rows[o + 3] = d;
    cols[o + 3] = c;
    data[o + 3] = v;
  }
}

// A value as an exact int32 (bool: 0 / 1); bad when a float value is not exactly one (fraction, |v| >= 2^31,
// -0.0, inf, nan).  k_values (g2n_kernels.hip) encodes beside the cast; k_weight_encode otherwise.
template <class T>
__device__ inline uint32_t weight_enc(T v, bool& bad) {
  if constexpr (std::is_floating_point<T>::value) {
    const double d = (double)v;
    bad = !(d == __builtin_trunc(d)) || !(d > -2147483648.0 && d < 2147483648.0) || (d == 0.0 && __builtin_signbit(d));
    return bad ? 0u : (uint32_t)(int32_t)d;
  } else if constexpr (std::is_same<T, uint8_t>::value) {
    bad = false;
    return v != 0 ? 1u : 0u;
  } else {
    bad = false;
    return (uint32_t)(int32_t)v;
  }
}

// Lean decimal-id builds: the parse wrote rows / cols; this writes the values (k_triplets'
// cast, errors and float32-overflow count) when an output needs them.  uniform: no weight tag,
// every value is dtype(1.0) (no cast can fail).  enc (weighted SUM CSR outputs): the values'
// exact-int32 codes beside them for the bucket partition (csr_partition_w), ctl->w_inexact when
// one has none.
template <class T>
__global__ void __launch_bounds__(kTPB) k_values(const double* __restrict__ w, uint64_t n_e, int ktrip, int uniform,
                                                 T* __restrict__ data, Ctl* ctl, uint32_t* __restrict__ enc) {
  const uint64_t e = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  bool bad = false;
  if (e < n_e) {
    const double wv = uniform ? 1.0 : w[e];
    T v;
    const uint32_t err = Cast<T>::go(wv, &v);
    if (std::is_same<T, float>::value && !__builtin_isinf(wv) && wv == wv && __builtin_isinf((double)v))
      atomicAdd(&ctl->n_f32_overflow, 1ull);
    const uint64_t o = e * (uint64_t)ktrip;
    if (err) {
      atomicMin(&ctl->cast_key, (unsigned long long)((o << 4) | err));
    } else {
      for (int j = 0; j < ktrip; j++) data[o + j] = v;
      if (enc) {
        const uint32_t x = weight_enc<T>(v, bad);
        for (int j = 0; j < ktrip; j++) enc[o + j] = x;
      }
    }
  }
  if (enc && __ballot(bad) && (threadIdx.x & 63) == 0) ctl->w_inexact = 1;
}

// ======================================================= K7-K9: COO -> CSR ========
// scipy's coo.tocsr() = coo_tocsr (scatter rows in stream order) + csr_sort_indices
// (std::sort by column, only when some row is unsorted) + csr_sum_duplicates (left-to-right
// run sums, in dtype).  On the GPU: a STABLE radix sort by row alone (32-bit keys; the column
// and value travel as the payload) reproduces coo_tocsr's per-row stream order; one thread per
// row then sorts its entries by column (stably: equal to std::sort whenever the result can
// not depend on it) and sums runs.  Rows whose float sums could depend on std::sort's exact
// permutation are re-run with the restated libstdc++ introsort (stl_sort.h).
// x86-64 SSE semantics of scipy's `x += y` (csr_sum_duplicates), bit for bit
template <class T>
struct Acc;
template <>
struct Acc<uint8_t> {
  __device__ static uint8_t add(uint8_t x, uint8_t y) { return (x | y) ? 1 : 0; }  // npy_bool_wrapper
  __device__ static bool is_float() { return false; }
  __device__ static double limit() { return 0.0; }
};
template <>
struct Acc<int8_t> {
  __device__ static int8_t add(int8_t x, int8_t y) { return (int8_t)(uint8_t)((uint8_t)x + (uint8_t)y); }
  __device__ static bool is_float() { return false; }
  __device__ static double limit() { return 0.0; }
};
template <>
struct Acc<int32_t> {
  __device__ static int32_t add(int32_t x, int32_t y) { return (int32_t)((uint32_t)x + (uint32_t)y); }
  __device__ static bool is_float() { return false; }
  __device__ static double limit() { return 0.0; }
};
template <>
struct Acc<float> {
  __device__ static float add(float x, float y) {
    if (x != x) return __uint_as_float(__float_as_uint(x) | 0x00400000u);
    if (y != y) return __uint_as_float(__float_as_uint(y) | 0x00400000u);
    float r = x + y;
    if (r != r) return __uint_as_float(0xFFC00000u);  // x86 default NaN (inf + -inf)
    return r;
  }
  __device__ static bool is_float() { return true; }
  __device__ static double limit() { return 16777216.0; }
};
template <>
struct Acc<double> {
  __device__ static double add(double x, double y) {
    if (x != x) return bits_f64(f64_bits(x) | 0x0008000000000000ull);
    if (y != y) return bits_f64(f64_bits(y) | 0x0008000000000000ull);
    double r = x + y;
    if (r != r) return bits_f64(0xFFF8000000000000ull);
    return r;
  }
  __device__ static bool is_float() { return true; }
  __device__ static double limit() { return 9007199254740992.0; }
};

template <class T>
__device__ inline bool exact_term(T v) {
  double d = (double)v;
  return d == __builtin_trunc(d);  // integral (false for inf/nan)
}


template <class T>
struct PV {  // sort payload: the other coordinate and the value
  uint32_t c;
  T v;
};

// Sum of k copies of one value (the unweighted build: every entry is dtype(1.0)), exactly as
// the left-to-right `x += y` of csr_sum_duplicates would produce it.
template <class T>
__device__ inline T sum_copies(T one, uint64_t k);
template <>
__device__ inline uint8_t sum_copies<uint8_t>(uint8_t one, uint64_t k) { return one; }
template <>
__device__ inline int8_t sum_copies<int8_t>(int8_t one, uint64_t k) {
  return (int8_t)(uint8_t)((uint64_t)(uint8_t)one * k);
}
template <>
__device__ inline int32_t sum_copies<int32_t>(int32_t one, uint64_t k) {
  return (int32_t)(uint32_t)((uint64_t)(uint32_t)one * k);
}
template <>
__device__ inline float sum_copies<float>(float one, uint64_t k) {  // one == 1.0f: stalls at 2^24
  return (float)(k < 16777216ull ? k : 16777216ull);
}
template <>
__device__ inline double sum_copies<double>(double one, uint64_t k) {  // one == 1.0: stalls at 2^53
  return (double)(k < 9007199254740992ull ? k : 9007199254740992ull);
}

// sort inputs: key = row (column when transposed); payload = column (row) [+ value]
template <class T, bool kUniform>
__global__ void __launch_bounds__(kTPB) k_pack(const int32_t* __restrict__ rows, const int32_t* __restrict__ cols,
                                               const T* __restrict__ data, uint64_t n, int transposed,
                                               int64_t base, uint32_t* __restrict__ key, PV<T>* __restrict__ pv,
                                               uint32_t* __restrict__ pc) {
  const uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  if (i >= n) return;
  const uint32_t r = (uint32_t)rows[i], c = (uint32_t)cols[i];
  key[i] = (uint32_t)((int64_t)(transposed ? c : r) - base);  // row within the slice
  if (kUniform) {
    pc[i] = transposed ? r : c;
  } else {
    PV<T> x;
    x.c = transposed ? r : c;
    x.v = data[i];
    pv[i] = x;
  }
}

constexpr uint32_t kRowGapCap = 64;  // empty rows one k_row_bounds thread fills

// start[r] = first sorted position of row r (start[n_rows] = n), from the row changes of the
// sorted keys: position p (0 <= p <= n) where key[p-1] != key[p] starts rows key[p-1]+1 ..
// key[p] (the empty ones in between included).  A gap wider than kRowGapCap sets ctl->row_gap
// and k_row_start (binary search per row) redoes the whole array.
__global__ void __launch_bounds__(kTPB) k_row_bounds(const uint32_t* __restrict__ key, uint64_t n, uint64_t n_rows,
                                                     uint32_t* __restrict__ start, Ctl* ctl) {
  const uint64_t p = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  if (p > n) return;
  const int64_t prev = p ? (int64_t)key[p - 1] : -1;
  const int64_t cur = p < n ? (int64_t)key[p] : (int64_t)n_rows;
  if (cur == prev) return;
  if (cur - prev > (int64_t)kRowGapCap) {
    ctl->row_gap = 1;
    return;
  }
  for (int64_t r = prev + 1; r <= cur; r++) start[r] = (uint32_t)p;
}

__device__ inline uint64_t lower_bound_u32(const uint32_t* __restrict__ a, uint64_t n, uint32_t key) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    uint64_t mid = (lo + hi) >> 1;
    if (a[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__global__ void __launch_bounds__(kTPB) k_row_start(const uint32_t* __restrict__ key, uint64_t n, uint64_t n_rows,
                                                    uint32_t* __restrict__ start, const Ctl* ctl) {
  if (!ctl->row_gap) return;  // k_row_bounds covered every row
  const uint64_t r = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  if (r > n_rows) return;
  start[r] = (uint32_t)(r == n_rows ? n : lower_bound_u32(key, n, (uint32_t)r));
}

// Row sums keep the unique entries of row r at [start[r], start[r] + ucnt[r]) of structure-of-
// arrays outputs: ocol (column) and, per entry, the run length (uniform build: every value is
// dtype(1), so the sum is a function of the count) or the summed value (weighted build).
template <class T, bool kUniform>
struct RowVal {
  using type = typename std::conditional<kUniform, uint32_t, T>::type;
};

template <class T, bool kUniform>
__device__ inline T row_value(const typename RowVal<T, kUniform>::type* ov, uint32_t j, T one) {
  if constexpr (kUniform) return sum_copies<T>(one, ov[j]);
  else return ov[j];
}

// Bitonic sorting network on the first N of M register slots (indices are compile-time after
// unrolling, so the arrays stay in VGPRs).  Keys are unique or payload-free, so stability is moot.
template <int N, int M, class K>
__device__ inline void net_sort(K (&k)[M]) {
#pragma unroll
  for (int size = 2; size <= N; size <<= 1)
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1)
#pragma unroll
      for (int i = 0; i < N; i++) {
        const int j = i ^ stride;
        if (j > i) {
          const K a = k[i], b = k[j];
          const bool asc = (i & size) == 0;
          const bool sw = asc ? (a > b) : (a < b);
          k[i] = sw ? b : a;
          k[j] = sw ? a : b;
        }
      }
}
template <int N, int M, class K, class V>
__device__ inline void net_sort_kv(K (&k)[M], V (&v)[M]) {
#pragma unroll
  for (int size = 2; size <= N; size <<= 1)
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1)
#pragma unroll
      for (int i = 0; i < N; i++) {
        const int j = i ^ stride;
        if (j > i) {
          const K a = k[i], b = k[j];
          const V x = v[i], y = v[j];
          const bool asc = (i & size) == 0;
          const bool sw = asc ? (a > b) : (a < b);
          k[i] = sw ? b : a;
          k[j] = sw ? a : b;
          v[i] = sw ? y : x;
          v[j] = sw ? x : y;
        }
      }
}

constexpr uint32_t kRegRow = 16;  // rows up to this many entries are sorted in registers

// Rows are processed one per thread, but a block's 256 rows own ONE contiguous range of the
// sorted entries (start[r0] .. start[r0 + 256]) and of every per-row output, so the block stages
// its ranges through LDS: coalesced loads and stores of the whole range, lane-strided accesses
// only in LDS.  A block whose range exceeds the LDS capacity works on global memory directly.
constexpr uint32_t kStageSumU = 4096;  // entries a k_row_sum block stages (unweighted / weighted)
constexpr uint32_t kStageSumW = 2048;
constexpr uint32_t kStageMaxU = 2048;  // entries per staged range in k_row_max / k_row_compact
constexpr uint32_t kStageMaxW = 1024;

// Staging in two phases so that every load of a block's ranges is in flight at once:
// fetch (global -> registers, unrolled) for all ranges, then put (registers -> LDS).
template <uint32_t kCap, class E>
struct Stage {
  static constexpr uint32_t kN = (kCap + kTPB - 1) / kTPB;
  E r[kN];
  __device__ inline void fetch(const E* __restrict__ g, uint64_t base, uint32_t n) {
#pragma unroll
    for (uint32_t k = 0; k < kN; k++) {
      const uint32_t i = threadIdx.x + k * kTPB;
      if (i < n) r[k] = g[base + i];
    }
  }
  __device__ inline void put(E* __restrict__ lds, uint32_t n) const {
#pragma unroll
    for (uint32_t k = 0; k < kN; k++) {
      const uint32_t i = threadIdx.x + k * kTPB;
      if (i < n) lds[i] = r[k];
    }
  }
};
template <class E>
__device__ inline void block_store(E* __restrict__ g, const E* __restrict__ lds, uint64_t base, uint32_t n) {
  for (uint32_t i = threadIdx.x; i < n; i += kTPB) g[base + i] = lds[i];
}

// One row: entries in stream order (at(q), q < len; after the stable row-bucket sort) -> sorted
// unique (column, count | sum), put(j, column, value).  Rows <= kRegRow entries: register
// sorting network on (column, stream position) keys, i.e. a stable sort.  Longer rows: stable
// bottom-up merge sort in global scratch (a, b: the row's own slices of two buffers the
// row-bucket sort left free).  flag: the row's float sums could depend on std::sort's order.
template <class T, bool kUniform, class At, class Put>
__device__ inline uint32_t row_sum_one(uint32_t len, At at, Put put, void* scr_a, void* scr_b, uint64_t s,
                                       bool& sorted, bool& flag) {
  using V = typename RowVal<T, kUniform>::type;
  uint32_t u = 0;
  sorted = true;
  flag = false;
  if (len <= kRegRow) {
    if constexpr (kUniform) {
      uint32_t k[kRegRow];
#pragma unroll
      for (uint32_t q = 0; q < kRegRow; q++) k[q] = q < len ? at(q) : 0xFFFFFFFFu;
#pragma unroll
      for (uint32_t q = 1; q < kRegRow; q++)
        if (q < len && k[q] < k[q - 1]) sorted = false;
      if (!sorted) {
        if (len <= 8) net_sort<8>(k);
        else net_sort<16>(k);
      }
      uint32_t cur = k[0], cnt = 1;
#pragma unroll
      for (uint32_t q = 1; q < kRegRow; q++) {
        if (q < len) {
          if (k[q] != cur) {
            put(u++, cur, (V)cnt);
            cur = k[q];
            cnt = 0;
          }
          cnt++;
        }
      }
      put(u++, cur, (V)cnt);
    } else {
      uint64_t k[kRegRow];
      T v[kRegRow];
#pragma unroll
      for (uint32_t q = 0; q < kRegRow; q++) {
        if (q < len) {
          const PV<T> x = at(q);
          k[q] = ((uint64_t)x.c << 32) | q;
          v[q] = x.v;
        } else {
          k[q] = ~0ull;
          v[q] = (T)0;
        }
      }
#pragma unroll
      for (uint32_t q = 1; q < kRegRow; q++)
        if (q < len && (k[q] >> 32) < (k[q - 1] >> 32)) sorted = false;
      if (!sorted) {
        if (len <= 8) net_sort_kv<8>(k, v);
        else net_sort_kv<16>(k, v);
      }
      uint32_t cur = (uint32_t)(k[0] >> 32);
      T acc = v[0];
#pragma unroll
      for (uint32_t q = 1; q < kRegRow; q++) {
        if (q < len) {
          const uint32_t c = (uint32_t)(k[q] >> 32);
          if (c != cur) {
            put(u++, cur, acc);
            cur = c;
            acc = v[q];
          } else {
            acc = Acc<T>::add(acc, v[q]);
          }
        }
      }
      put(u++, cur, acc);
    }
    return u;
  }
  // ---- long row
  if constexpr (kUniform) {
    uint32_t* a = (uint32_t*)scr_a + s;
    uint32_t* b = (uint32_t*)scr_b + s;
    uint32_t prev = 0;
    for (uint32_t q = 0; q < len; q++) {
      const uint32_t c = at(q);
      if (q && c < prev) sorted = false;
      prev = c;
      a[q] = c;
    }
    if (!sorted) {
      for (uint32_t width = 1; width < len; width <<= 1) {
        for (uint32_t lo = 0; lo < len; lo += 2 * width) {
          const uint32_t mid = lo + width < len ? lo + width : len;
          const uint32_t hi = lo + 2 * width < len ? lo + 2 * width : len;
          uint32_t x = lo, y = mid, w = lo;
          while (x < mid && y < hi) b[w++] = (a[y] < a[x]) ? a[y++] : a[x++];
          while (x < mid) b[w++] = a[x++];
          while (y < hi) b[w++] = a[y++];
        }
        uint32_t* t = a;
        a = b;
        b = t;
      }
    }
    uint32_t q = 0;
    while (q < len) {
      const uint32_t c = a[q], q0 = q;
      while (q < len && a[q] == c) q++;
      put(u++, c, (V)(q - q0));
    }
  } else {
    PV<T>* a = (PV<T>*)scr_a + s;
    PV<T>* b = (PV<T>*)scr_b + s;
    uint32_t prev = 0;
    for (uint32_t q = 0; q < len; q++) {
      const PV<T> x = at(q);
      if (q && x.c < prev) sorted = false;
      prev = x.c;
      a[q] = x;
    }
    if (!sorted) {
      for (uint32_t width = 1; width < len; width <<= 1) {
        for (uint32_t lo = 0; lo < len; lo += 2 * width) {
          const uint32_t mid = lo + width < len ? lo + width : len;
          const uint32_t hi = lo + 2 * width < len ? lo + 2 * width : len;
          uint32_t x = lo, y = mid, w = lo;
          while (x < mid && y < hi) b[w++] = (a[y].c < a[x].c) ? a[y++] : a[x++];
          while (x < mid) b[w++] = a[x++];
          while (y < hi) b[w++] = a[y++];
        }
        PV<T>* t = a;
        a = b;
        b = t;
      }
    }
    uint32_t q = 0;
    while (q < len) {  // left-to-right run sums
      const uint32_t c = a[q].c, q0 = q;
      T x = a[q].v;
      bool exact = true;
      double sabs = 0.0;
      if (Acc<T>::is_float()) {
        exact = exact_term(x);
        sabs = __builtin_fabs((double)x);
      }
      q++;
      while (q < len && a[q].c == c) {
        const T y = a[q].v;
        if (Acc<T>::is_float()) {
          exact = exact && exact_term(y);
          sabs += __builtin_fabs((double)y);
        }
        x = Acc<T>::add(x, y);
        q++;
      }
      // a group of >= 3 terms whose sum depends on their order (std::sort on > 16 elements is
      // not an insertion sort, so scipy's order is not the stable one)
      if (Acc<T>::is_float() && q - q0 >= 3 && !(exact && sabs < Acc<T>::limit())) flag = true;
      put(u++, c, x);
    }
  }
  return u;
}

// coo.tocsr() per row after the row-bucket sort: row r's unique entries at
// [start[r], start[r] + ucnt[r]) of ocol / oval.
template <class T, bool kUniform>
__global__ void __launch_bounds__(kTPB) k_row_sum(const uint32_t* __restrict__ start, uint64_t n_rows,
                                                  const PV<T>* __restrict__ pv, const uint32_t* __restrict__ pc,
                                                  uint32_t* __restrict__ ocol,
                                                  typename RowVal<T, kUniform>::type* __restrict__ oval,
                                                  void* __restrict__ scr_a, void* __restrict__ scr_b,
                                                  uint32_t* __restrict__ ucnt, uint8_t* __restrict__ rowflag,
                                                  Ctl* ctl, int which) {
  using V = typename RowVal<T, kUniform>::type;
  using In = typename std::conditional<kUniform, uint32_t, PV<T>>::type;
  constexpr uint32_t kCap = kUniform ? kStageSumU : kStageSumW;
  // the row loads are independent (unrolled) and stay direct; only the lane-strided stores of
  // the unique entries are staged
  __shared__ uint32_t s_col[kCap];
  __shared__ V s_val[kCap];
  const In* gin = kUniform ? (const In*)(const void*)pc : (const In*)(const void*)pv;
  const uint64_t r0 = (uint64_t)blockIdx.x * kTPB;
  const uint64_t r1 = r0 + kTPB < n_rows ? r0 + kTPB : n_rows;
  const uint32_t b0 = start[r0], nseg = start[r1] - b0;
  const bool staged = nseg <= kCap;  // block-uniform
  const uint64_t r = r0 + threadIdx.x;
  bool sorted = true, flag = false;
  if (r < n_rows) {
    const uint32_t s = start[r], len = start[r + 1] - s;
    uint32_t u = 0;
    if (len == 1) {
      const In x = gin[s];
      uint32_t c;
      V v;
      if constexpr (kUniform) {
        c = x;
        v = 1u;
      } else {
        c = x.c;
        v = x.v;
      }
      if (staged) {
        s_col[s - b0] = c;
        s_val[s - b0] = v;
      } else {
        ocol[s] = c;
        oval[s] = v;
      }
      u = 1;
    } else if (len > 1) {
      if (staged) {
        const uint32_t o = s - b0;
        u = row_sum_one<T, kUniform>(
            len, [&](uint32_t q) { return gin[s + q]; },
            [&](uint32_t j, uint32_t c, V v) {
              s_col[o + j] = c;
              s_val[o + j] = v;
            },
            scr_a, scr_b, s, sorted, flag);
      } else {
        u = row_sum_one<T, kUniform>(
            len, [&](uint32_t q) { return gin[s + q]; },
            [&](uint32_t j, uint32_t c, V v) {
              ocol[s + j] = c;
              oval[s + j] = v;
            },
            scr_a, scr_b, s, sorted, flag);
      }
    }
    ucnt[r] = u;
    if (flag) {
      rowflag[r] = 1;
      ctl->flagged[which] = 1;
    }
  }
  if (!sorted) ctl->unsorted[which] = 1;
  if (staged) {
    __syncthreads();
    block_store(ocol, s_col, b0, nseg);
    block_store(oval, s_val, b0, nseg);
  }
}

// Flagged rows when the matrix is unsorted: exactly scipy's per-row std::sort + run sums.
template <class T>
__global__ void __launch_bounds__(64) k_row_emulate(const uint32_t* __restrict__ start, uint64_t n_rows,
                                                    const uint8_t* __restrict__ rowflag,
                                                    const PV<T>* __restrict__ pv, uint32_t* __restrict__ ocol,
                                                    T* __restrict__ oval, KV<int32_t, T>* __restrict__ kv) {
  const uint64_t r = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  if (r >= n_rows || !rowflag[r]) return;
  const uint32_t s = start[r], len = start[r + 1] - s;
  KV<int32_t, T>* a = kv + s;
  for (uint32_t q = 0; q < len; q++) {
    a[q].k = (int32_t)pv[s + q].c;
    a[q].v = pv[s + q].v;
  }
  stl_sort(a, a + len);
  uint32_t u = 0, q = 0;
  while (q < len) {
    int32_t c = a[q].k;
    T x = a[q].v;
    q++;
    while (q < len && a[q].k == c) {
      x = Acc<T>::add(x, a[q].v);
      q++;
    }
    ocol[s + u] = (uint32_t)c;
    oval[s + u] = x;
    u++;
  }
}

// SUM CSR: row r's unique entries -> indices/data at indptr[r]
template <class T, bool kUniform>
__global__ void __launch_bounds__(kTPB) k_row_compact(const uint32_t* __restrict__ start,
                                                      const uint32_t* __restrict__ ucnt,
                                                      const uint32_t* __restrict__ uoff, uint64_t n_rows,
                                                      const uint32_t* __restrict__ ocol,
                                                      const typename RowVal<T, kUniform>::type* __restrict__ oval,
                                                      T one, int32_t* __restrict__ indptr,
                                                      int32_t* __restrict__ indices, T* __restrict__ data) {
  using V = typename RowVal<T, kUniform>::type;
  constexpr uint32_t kCap = kUniform ? kStageMaxU : kStageMaxW;
  __shared__ uint32_t s_c[kCap];
  __shared__ V s_v[kCap];
  __shared__ int32_t s_i[kCap];
  __shared__ T s_d[kCap];
  const uint64_t r0 = (uint64_t)blockIdx.x * kTPB;
  const uint64_t r1 = r0 + kTPB < n_rows ? r0 + kTPB : n_rows;
  const uint32_t b0 = start[r0], nin = start[r1] - b0;
  const uint32_t o0 = uoff[r0], nout = uoff[r1 - 1] + ucnt[r1 - 1] - o0;
  const bool staged = nin <= kCap && nout <= kCap;
  if (staged) {
    Stage<kCap, uint32_t> sc;
    Stage<kCap, V> sv;
    sc.fetch(ocol, b0, nin);
    sv.fetch(oval, b0, nin);
    sc.put(s_c, nin);
    sv.put(s_v, nin);
    __syncthreads();
  }
  const uint64_t r = r0 + threadIdx.x;
  if (r < n_rows) {
    const uint32_t s = start[r], u = ucnt[r], o = uoff[r];
    indptr[r] = (int32_t)o;
    if (r == n_rows - 1) indptr[n_rows] = (int32_t)(o + u);
    for (uint32_t j = 0; j < u; j++) {
      if (staged) {
        s_i[o - o0 + j] = (int32_t)s_c[s - b0 + j];
        s_d[o - o0 + j] = row_value<T, kUniform>(s_v, s - b0 + j, one);
      } else {
        indices[o + j] = (int32_t)ocol[s + j];
        data[o + j] = row_value<T, kUniform>(oval, s + j, one);
      }
    }
  }
  if (staged) {
    __syncthreads();
    block_store(indices, s_i, o0, nout);
    block_store(data, s_d, o0, nout);
  }
}

// M = A.maximum(A.T) row by row: merge row r of B (= SUM(A)) and of BT (= SUM(A.T)), both sorted
// by column; csr_binop_csr_canonical with std::max ((a < b) ? b : a), missing = 0, zeros dropped.
// kWrite = false: count pass (mcnt); true: write pass at moff[r].
template <class T, bool kUniform, bool kWrite>
__global__ void __launch_bounds__(kTPB) k_row_max(const uint32_t* __restrict__ sa, const uint32_t* __restrict__ ua,
                                                  const uint32_t* __restrict__ ca,
                                                  const typename RowVal<T, kUniform>::type* __restrict__ va,
                                                  const uint32_t* __restrict__ st, const uint32_t* __restrict__ ut,
                                                  const uint32_t* __restrict__ ct,
                                                  const typename RowVal<T, kUniform>::type* __restrict__ vt,
                                                  T one, uint64_t n_rows, uint32_t* __restrict__ mcnt,
                                                  const uint32_t* __restrict__ moff, int32_t* __restrict__ indptr,
                                                  int32_t* __restrict__ indices, T* __restrict__ data) {
  using V = typename RowVal<T, kUniform>::type;
  constexpr uint32_t kCap = kUniform ? kStageMaxU : kStageMaxW;
  __shared__ uint32_t s_ca[kCap], s_ct[kCap];
  __shared__ V s_va[kCap], s_vt[kCap];
  __shared__ int32_t s_i[kWrite ? kCap : 1];
  __shared__ T s_d[kWrite ? kCap : 1];
  const uint64_t r0 = (uint64_t)blockIdx.x * kTPB;
  const uint64_t r1 = r0 + kTPB < n_rows ? r0 + kTPB : n_rows;
  const uint32_t a_0 = sa[r0], na_seg = sa[r1] - a_0;
  const uint32_t t_0 = st[r0], nt_seg = st[r1] - t_0;
  const uint32_t o0 = kWrite ? moff[r0] : 0;
  const uint32_t nout = kWrite ? moff[r1 - 1] + mcnt[r1 - 1] - o0 : 0;
  const bool staged = na_seg <= kCap && nt_seg <= kCap && nout <= kCap;
  if (staged) {
    Stage<kCap, uint32_t> c1, c2;
    Stage<kCap, V> v1, v2;
    c1.fetch(ca, a_0, na_seg);
    v1.fetch(va, a_0, na_seg);
    c2.fetch(ct, t_0, nt_seg);
    v2.fetch(vt, t_0, nt_seg);
    c1.put(s_ca, na_seg);
    v1.put(s_va, na_seg);
    c2.put(s_ct, nt_seg);
    v2.put(s_vt, nt_seg);
    __syncthreads();
  }
  const uint64_t r = r0 + threadIdx.x;
  if (r < n_rows) {
    const uint32_t na = ua[r], nb = ut[r];
    const uint32_t ga = sa[r], gb = st[r];
    const uint32_t base = kWrite ? moff[r] : 0;
    if (kWrite) {
      indptr[r] = (int32_t)base;
      if (r == n_rows - 1) indptr[n_rows] = (int32_t)(base + mcnt[r]);
    }
    auto merge = [&](const uint32_t* CA, const V* VA, const uint32_t* CB, const V* VB, int32_t* OI, T* OD) {
      uint32_t i = 0, j = 0, m = 0;
      auto emit = [&](uint32_t c, T x, T y) {
        const T v = (x < y) ? y : x;
        if (v != (T)0) {
          if (kWrite) {
            OI[m] = (int32_t)c;
            OD[m] = v;
          }
          m++;
        }
      };
      uint32_t cA = na ? CA[0] : 0, cB = nb ? CB[0] : 0;
      while (i < na && j < nb) {
        if (cA == cB) {
          emit(cA, row_value<T, kUniform>(VA, i, one), row_value<T, kUniform>(VB, j, one));
          i++;
          j++;
          if (i < na) cA = CA[i];
          if (j < nb) cB = CB[j];
        } else if (cA < cB) {
          emit(cA, row_value<T, kUniform>(VA, i, one), (T)0);
          i++;
          if (i < na) cA = CA[i];
        } else {
          emit(cB, (T)0, row_value<T, kUniform>(VB, j, one));
          j++;
          if (j < nb) cB = CB[j];
        }
      }
      for (; i < na; i++) emit(CA[i], row_value<T, kUniform>(VA, i, one), (T)0);
      for (; j < nb; j++) emit(CB[j], (T)0, row_value<T, kUniform>(VB, j, one));
      return m;
    };
    uint32_t m;
    if (staged)
      m = merge(s_ca + (ga - a_0), s_va + (ga - a_0), s_ct + (gb - t_0), s_vt + (gb - t_0), s_i + (base - o0),
                s_d + (base - o0));
    else
      m = merge(ca + ga, va + ga, ct + gb, vt + gb, indices + base, data + base);
    if (!kWrite) mcnt[r] = m;
  }
  if (kWrite && staged) {
    __syncthreads();
    block_store(indices, s_i, o0, nout);
    block_store(data, s_d, o0, nout);
  }
}

// ====================================================== sharded build helpers ======
// keys of a blob as S-kind touches (g2n_dedup_keys)
__global__ void __launch_bounds__(kTPB) k_keys_to_touches(const int64_t* __restrict__ offs, uint64_t n,
                                                          uint64_t* __restrict__ noff, uint32_t* __restrict__ nlen,
                                                          uint8_t* __restrict__ tkind) {
  const uint64_t t = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  if (t >= n) return;
  noff[t] = (uint64_t)offs[t];
  nlen[t] = (uint32_t)(offs[t + 1] - offs[t]);
  tkind[t] = 1;
}

// node id of every touch, whichever dictionary path ran: the claimers and (general path) every
// touch through its table slot, the other touches of the S-first paths through tid.
// s_ident: the S-prefix path (every touch an S touch, ids = claimer indices) — a claimer's id
// is its own index, no table read.
__global__ void __launch_bounds__(kTPB) k_touch_ids(uint64_t n, const uint8_t* __restrict__ first,
                                                    const uint32_t* __restrict__ slot,
                                                    const DictEntry* __restrict__ table,
                                                    const uint32_t* __restrict__ tid, int general, int s_ident,
                                                    uint32_t* __restrict__ out) {
  const uint64_t t = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  if (t >= n) return;
  if (general) out[t] = (uint32_t)table[slot[t]].hdr;
  else if (first[t]) out[t] = s_ident ? (uint32_t)t : (uint32_t)table[slot[t]].hdr;
  else out[t] = tid[t];
}

__global__ void __launch_bounds__(kTPB) k_first_of(uint64_t n_nodes, const uint32_t* __restrict__ inv,
                                                   uint32_t* __restrict__ out) {
  const uint64_t d = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  if (d < n_nodes) out[d] = inv ? inv[d] : (uint32_t)d;
}

// owner rank of a key: FNV-1a of its bytes mod n_ranks (any fixed function of the bytes works:
// equal keys must meet on one rank)
__global__ void __launch_bounds__(kTPB) k_key_owner(const uint8_t* __restrict__ blob,
                                                    const int64_t* __restrict__ offs, uint64_t n, uint32_t n_ranks,
                                                    uint32_t* __restrict__ owner, uint32_t* __restrict__ idx) {
  const uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  if (i >= n) return;
  uint64_t h = 0xcbf29ce484222325ull;
  for (int64_t p = offs[i]; p < offs[i + 1]; p++) h = (h ^ blob[p]) * 0x100000001b3ull;
  owner[i] = (uint32_t)(fmix64(h) % n_ranks);
  idx[i] = (uint32_t)i;
}

__global__ void __launch_bounds__(kTPB) k_key_lens(const int64_t* __restrict__ offs,
                                                   const uint32_t* __restrict__ perm, uint64_t n,
                                                   int64_t* __restrict__ lens) {
  const uint64_t j = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  if (j < n) lens[j] = offs[perm[j] + 1] - offs[perm[j]];
}

__global__ void __launch_bounds__(kTPB) k_copy_keys(const uint8_t* __restrict__ blob, const int64_t* __restrict__ offs,
                                                    const uint32_t* __restrict__ perm, uint64_t n,
                                                    const int64_t* __restrict__ ooffs, uint8_t* __restrict__ oblob) {
  const uint64_t j = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  if (j >= n) return;
  const int64_t s = offs[perm[j]], l = offs[perm[j] + 1] - s, o = ooffs[j];
  for (int64_t b = 0; b < l; b++) oblob[o + b] = blob[s + b];
}

// rows / cols through a local -> global id map, in place (g2n_remap_pairs).  kVec: 4 pairs per
// thread with 16-byte accesses (both arrays 16-byte aligned, checked by the host), the last
// n % 4 pairs by the scalar branch; else one pair per thread.
template <bool kVec>
__global__ void __launch_bounds__(kTPB) k_remap_pairs(const uint32_t* __restrict__ map, uint64_t n_map,
                                                      int32_t* __restrict__ rows, int32_t* __restrict__ cols,
                                                      uint64_t n, Ctl* __restrict__ ctl) {
  const uint64_t q = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  auto one = [&](uint32_t x) -> int32_t {
    if (x >= n_map) {
      atomicAdd(&ctl->bad_id, 1ull);
      return -1;
    }
    return (int32_t)map[x];
  };
  if (!kVec) {
    if (q < n) {
      rows[q] = one((uint32_t)rows[q]);
      cols[q] = one((uint32_t)cols[q]);
    }
  } else if (4 * q + 4 <= n) {
    const int4 r = reinterpret_cast<const int4*>(rows)[q];
    const int4 c = reinterpret_cast<const int4*>(cols)[q];
    const int4 ro{one((uint32_t)r.x), one((uint32_t)r.y), one((uint32_t)r.z), one((uint32_t)r.w)};
    const int4 co{one((uint32_t)c.x), one((uint32_t)c.y), one((uint32_t)c.z), one((uint32_t)c.w)};
    reinterpret_cast<int4*>(rows)[q] = ro;
    reinterpret_cast<int4*>(cols)[q] = co;
  } else if (4 * q < n) {
    for (uint64_t i = 4 * q; i < n; i++) {
      rows[i] = one((uint32_t)rows[i]);
      cols[i] = one((uint32_t)cols[i]);
    }
  }
}

// owner rank of each triplet's (remapped) row; the sort payload is the triplet index
__global__ void __launch_bounds__(kTPB) k_route_keys(const int32_t* __restrict__ rows,
                                                     const int32_t* __restrict__ cols, uint64_t n,
                                                     const uint32_t* __restrict__ map, uint64_t n_global,
                                                     uint32_t n_ranks, int transposed, uint32_t* __restrict__ owner,
                                                     uint32_t* __restrict__ idx) {
  const uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  if (i >= n) return;
  const uint32_t x = (uint32_t)(transposed ? cols[i] : rows[i]);
  const uint64_t key = map ? map[x] : x;  // no map: the ids are global already
  owner[i] = (uint32_t)(key * n_ranks / n_global);
  idx[i] = (uint32_t)i;
}

template <class W>  // an unsigned type of the data's element size; data == nullptr: coordinates only
__global__ void __launch_bounds__(kTPB) k_route_gather(const int32_t* __restrict__ rows,
                                                       const int32_t* __restrict__ cols,
                                                       const W* __restrict__ data,
                                                       const uint32_t* __restrict__ perm, uint64_t n,
                                                       const uint32_t* __restrict__ map, int transposed,
                                                       int32_t* __restrict__ orows, int32_t* __restrict__ ocols,
                                                       W* __restrict__ odata) {
  const uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  if (i >= n) return;
  const uint32_t j = perm[i];
  const int32_t r = map ? (int32_t)map[rows[j]] : rows[j], c = map ? (int32_t)map[cols[j]] : cols[j];
  orows[i] = transposed ? c : r;
  ocols[i] = transposed ? r : c;
  if (data) odata[i] = data[j];
}

__global__ void k_scan_total(const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ off, uint64_t n,
                             unsigned long long* out) {
  *out = n ? (unsigned long long)off[n - 1] + cnt[n - 1] : 0ull;
}

// ====================================================== export --format edge-list ======
// cli.py:264-281: one "u\tv\n" line per L/E/C record in stream order, u/v the record's
// endpoint keys (bidirected: "u:ori"), which are the names of the stream-order COO's row/col
// ids.  Bytes per edge: 8 B ids + |u| + |v| + 2 written, names read from the (L2-resident
// for local graphs) blob.

// per-name record, one 8-byte gather per edge endpoint: offset << 24 | length << 1 | bad, bad =
// the key's bytes are not strict UTF-8 (the export's u.decode() raises); a length that does not
// fit 23 bits is saturated and read from offs
constexpr uint64_t kMetaLen = 0x7FFFFF;

__global__ void __launch_bounds__(kTPB) k_name_meta(const uint8_t* __restrict__ blob,
                                                    const int64_t* __restrict__ offs, uint64_t n_names,
                                                    uint64_t* __restrict__ meta) {
  const uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  if (i >= n_names) return;
  const uint64_t o = (uint64_t)offs[i], n = (uint64_t)offs[i + 1] - o;
  meta[i] = (o << 24) | ((n < kMetaLen ? n : kMetaLen) << 1) | (utf8_valid(blob + o, n) ? 0u : 1u);
}

__device__ inline uint64_t meta_len(uint64_t m, uint32_t id, const int64_t* __restrict__ offs) {
  const uint64_t l = (m >> 1) & kMetaLen;
  return l == kMetaLen ? (uint64_t)(offs[id + 1] - offs[id]) : l;
}

// per-edge line length; the first edge (stream order) with an undecodable endpoint
__global__ void __launch_bounds__(kTPB) k_edge_text_len(const int32_t* __restrict__ rows,
                                                        const int32_t* __restrict__ cols, uint64_t n,
                                                        const uint64_t* __restrict__ meta,
                                                        const int64_t* __restrict__ offs, uint64_t* __restrict__ len,
                                                        ulonglong2* __restrict__ em, unsigned long long* first_bad) {
  const uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
  if (i >= n) return;
  const int32_t r = rows[i], c = cols[i];
  uint64_t mr = meta[r], mc = meta[c];
  const uint64_t lr = meta_len(mr, r, offs), lc = meta_len(mc, c, offs);
  len[i] = lr + lc + 2u;
  // the endpoints' (offset, length) for the render pass: one coalesced 16-byte read there
  // instead of two more random gathers
  em[i] = make_ulonglong2(((mr >> 24) << 24) | (lr < 0xFFFFFFu ? lr : 0xFFFFFFu), mc >> 24);
  if ((mr | mc) & 1u) atomicMin(first_bad, (unsigned long long)i);
}

// renders the lines at their scanned positions.  A block takes kTextEdges consecutive edges,
// whose text is one contiguous range [pos[e0], pos[e1]): the lines are assembled in LDS at
// their offset from the 16-byte-aligned start of that range, then written out with aligned
// 16-byte stores (byte stores only for the two partial words at the range ends, whose other
// bytes belong to the neighbouring blocks).  A range longer than the LDS stage (long names)
// is written line by line straight to HBM.
constexpr uint32_t kTextEdges = 1024;
constexpr uint32_t kTextLds = 32 * 1024;

__device__ inline void edge_line(uint8_t* d, int64_t ur, int64_t ul, int64_t vr, int64_t vl,
                                 const uint8_t* __restrict__ blob) {
  for (int64_t k = 0; k < ul; k++) d[k] = blob[ur + k];
  d[ul] = '\t';
  d += ul + 1;
  for (int64_t k = 0; k < vl; k++) d[k] = blob[vr + k];
  d[vl] = '\n';
}

__global__ void __launch_bounds__(kTPB) k_edge_text(const int32_t* __restrict__ rows, const int32_t* __restrict__ cols,
                                                    uint64_t n, const ulonglong2* __restrict__ em,
                                                    const int64_t* __restrict__ offs, const uint8_t* __restrict__ blob, const uint64_t* __restrict__ pos,
                                                    uint8_t* __restrict__ out) {
  __shared__ uint4 stage4[kTextLds / 16];
  uint8_t* stage = (uint8_t*)stage4;
  const uint64_t e0 = (uint64_t)blockIdx.x * kTextEdges;
  const uint64_t e1 = e0 + kTextEdges < n ? e0 + kTextEdges : n;
  const uint64_t p0 = pos[e0], p1 = pos[e1];  // pos holds n + 1 entries
  const uint64_t base = p0 & ~15ull;
  const bool staged = p1 - base <= kTextLds;  // block-uniform
  for (uint64_t e = e0 + threadIdx.x; e < e1; e += kTPB) {
    const ulonglong2 m = em[e];
    const uint64_t pe = pos[e];
    uint64_t ul = m.x & 0xFFFFFFu;  // |u| (saturated: from offs); |v| = line - |u| - 2
    if (ul == 0xFFFFFFu) ul = (uint64_t)(offs[rows[e] + 1] - offs[rows[e]]);
    const uint64_t vl = pos[e + 1] - pe - 2 - ul;
    edge_line(staged ? stage + (pe - base) : out + pe, (int64_t)(m.x >> 24), (int64_t)ul, (int64_t)m.y, (int64_t)vl,
              blob);
  }
  if (!staged) return;
  __syncthreads();
  const uint64_t w0 = base >> 4, w1 = (p1 + 15) >> 4;
  for (uint64_t w = w0 + threadIdx.x; w < w1; w += kTPB) {
    const uint64_t a = w << 4;
    if (a >= p0 && a + 16 <= p1) {
      *(uint4*)(out + a) = stage4[w - w0];
    } else {
      for (uint64_t b = a < p0 ? p0 : a; b < a + 16 && b < p1; b++) out[b] = stage[b - base];
    }
  }
}

// The export of a decimal-id build (lean premise held: node k's key is str(k + 1), bidirected
// id 2k + [ori == '-'] -> str(k + 1) + ":+" / ":-"): every line's length and text are arithmetic on
// its two ids, so there is no names blob, meta, per-edge length array or gather.  k_edge_dec_sum sums
// each block's kTextEdges line lengths; after a scan of those block sums k_edge_dec_text recomputes
// them, scans them inside the block and renders the block's lines in LDS (at most 1024 x 26 bytes:
// two 10-digit keys, ":o" twice, tab and newline), then writes them with aligned 16-byte stores.
// Algorithmic bytes per edge: 8 read twice + the line written.  The digit work is VALU and sets the
// render's pace: a key's digit count is clz-based (one LDS table read, no compare chain), its digits
// come four at a time by SWAR (a 4-digit value split into 2-digit then 1-digit byte lanes by
// multiply-shift: x / 100 = (x * 5243) >> 19 for x < 10^4, x / 10 = (x * 103) >> 10 for x < 100; no
// carry crosses a lane).
__device__ inline uint32_t dec4_ascii(uint32_t y) {  // y < 10^4: its 4 digits, most significant in byte 0
  const uint32_t h = (y * 5243u) >> 19;
  uint32_t z = h | ((y - h * 100u) << 16);
  const uint32_t t = ((z * 103u) >> 10) & 0x000F000Fu;
  z = t | ((z - t * 10u) << 8);
  return z | 0x30303030u;
}
struct DecKeys {  // a thread's kDecPer edges: the two keys' values (id + 1, bidirected id / 2 + 1) and digits
  uint32_t va[4], vb[4], na[4], nb[4], l[4];  // l: line length (0: past the end)
};
__device__ inline uint32_t dec_ndig(uint32_t v, const uint32_t* p10 /* LDS: 10^0 .. 10^9 */) {  // v >= 1
  const uint32_t t = ((32u - (uint32_t)__clz(v)) * 1233u) >> 12;  // log10(2^bits), 0..9
  return t + (v >= p10[t] ? 1u : 0u);
}
__device__ inline void dec_p10(uint32_t* p10) {
  if (threadIdx.x < 10) {
    uint32_t p = 1;
    for (uint32_t k = 0; k < threadIdx.x; k++) p *= 10u;
    p10[threadIdx.x] = p;
  }
  __syncthreads();
}
// the key of value v (n digits) at d, plus ":+" / ":-" when bidirected; returns the byte after it.
// (Writing every key as 8 zero-padded bytes back to front, without per-byte predicates, measured the
// same 1.19 ms on C4: the render runs at ~4.3 TB/s of ids read + text written.)
__device__ inline uint8_t* dec_key_put(uint8_t* d, uint32_t v, uint32_t n, int bidir, uint32_t id) {
  if (n > 8) {  // the leading 1-2 digits, then the low 8
    const uint32_t hi = v / 100000000u;
    v -= hi * 100000000u;
    if (hi > 9) *d++ = (uint8_t)('0' + hi / 10u);
    *d++ = (uint8_t)('0' + hi % 10u);
    n = 8;
  }
  const uint32_t a = v / 10000u;
  const uint64_t w = (((uint64_t)dec4_ascii(v - a * 10000u) << 32) | dec4_ascii(a)) >> (8u * (8u - n));
  for (uint32_t j = 0; j < n; j++) d[j] = (uint8_t)(w >> (8u * j));
  d += n;
  if (bidir) {
    d[0] = ':';
    d[1] = (id & 1u) ? '-' : '+';
    d += 2;
  }
  return d;
}
constexpr uint32_t kDecPer = kTextEdges / kTPB;  // edges per thread (4), consecutive
static_assert(kDecPer == 4 && kTextEdges * 26u + 16u <= kTextLds, "a block's lines fit the LDS stage");

__device__ inline uint32_t dec_edges_load(const int32_t* __restrict__ rows, const int32_t* __restrict__ cols,
                                          uint64_t n, uint64_t e, int bidir, const uint32_t* p10, uint32_t* r,
                                          uint32_t* c, DecKeys& K) {
  uint32_t k = 0;
  if (e + kDecPer <= n) {  // e is a multiple of 4: one 16-byte load per array
    const int4 a = *(const int4*)(rows + e), b = *(const int4*)(cols + e);
    r[0] = a.x, r[1] = a.y, r[2] = a.z, r[3] = a.w;
    c[0] = b.x, c[1] = b.y, c[2] = b.z, c[3] = b.w;
    k = kDecPer;
  } else {
    for (uint32_t j = 0; j < kDecPer; j++) r[j] = c[j] = 0;
    for (; e + k < n; k++) r[k] = (uint32_t)rows[e + k], c[k] = (uint32_t)cols[e + k];
  }
  uint32_t s = 0;
  const uint32_t sh = bidir ? 1u : 0u, ext = bidir ? 2u : 0u;
#pragma unroll
  for (uint32_t j = 0; j < kDecPer; j++) {
    K.va[j] = (r[j] >> sh) + 1u;
    K.vb[j] = (c[j] >> sh) + 1u;
    K.na[j] = dec_ndig(K.va[j], p10);
    K.nb[j] = dec_ndig(K.vb[j], p10);
    K.l[j] = j < k ? K.na[j] + K.nb[j] + 2u + 2u * ext : 0u;
    s += K.l[j];
  }
  return s;
}

__global__ void __launch_bounds__(kTPB) k_edge_dec_sum(const int32_t* __restrict__ rows,
                                                       const int32_t* __restrict__ cols, uint64_t n, int bidir,
                                                       uint64_t* __restrict__ bsum) {
  __shared__ uint32_t red[kTPB / 64];
  __shared__ uint32_t p10[10];
  dec_p10(p10);
  uint32_t r[kDecPer], c[kDecPer];
  DecKeys K;
  const uint32_t s = dec_edges_load(rows, cols, n, (uint64_t)blockIdx.x * kTextEdges + threadIdx.x * kDecPer, bidir,
                                    p10, r, c, K);
  uint32_t tot;
  block_excl_scan_n64<kTPB>(s, &tot, red);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(kTPB) k_edge_dec_text(const int32_t* __restrict__ rows,
                                                        const int32_t* __restrict__ cols, uint64_t n, int bidir,
                                                        const uint64_t* __restrict__ bpos, uint8_t* __restrict__ out) {
  __shared__ uint4 stage4[kTextLds / 16];
  __shared__ uint32_t red[kTPB / 64];
  __shared__ uint32_t p10[10];
  uint8_t* stage = (uint8_t*)stage4;
  dec_p10(p10);
  uint32_t r[kDecPer], c[kDecPer];
  DecKeys K;
  const uint32_t s = dec_edges_load(rows, cols, n, (uint64_t)blockIdx.x * kTextEdges + threadIdx.x * kDecPer, bidir,
                                    p10, r, c, K);
  uint32_t tot;
  const uint32_t x = block_excl_scan_n64<kTPB>(s, &tot, red);
  const uint64_t p0 = bpos[blockIdx.x], p1 = p0 + tot;
  const uint64_t base = p0 & ~15ull;
  uint8_t* d = stage + (p0 - base) + x;
  for (uint32_t j = 0; j < kDecPer; j++) {
    if (!K.l[j]) break;
    d = dec_key_put(d, K.va[j], K.na[j], bidir, r[j]);
    *d++ = '\t';
    d = dec_key_put(d, K.vb[j], K.nb[j], bidir, c[j]);
    *d++ = '\n';
  }
  __syncthreads();
  const uint64_t w0 = base >> 4, w1 = (p1 + 15) >> 4;
  for (uint64_t w = w0 + threadIdx.x; w < w1; w += kTPB) {
    const uint64_t a = w << 4;
    if (a >= p0 && a + 16 <= p1) {
      *(uint4*)(out + a) = stage4[w - w0];
    } else {
      for (uint64_t b = a < p0 ? p0 : a; b < a + 16 && b < p1; b++) out[b] = stage[b - base];
    }
  }
}

// ----------------------------------------------------------- explicit instances --
#define G2N_INST_U(T, U)                                                                                        \
  template __global__ void k_pack<T, U>(const int32_t*, const int32_t*, const T*, uint64_t, int, int64_t, uint32_t*, \
                                        PV<T>*, uint32_t*);                                                      \
  template __global__ void k_row_sum<T, U>(const uint32_t*, uint64_t, const PV<T>*, const uint32_t*, uint32_t*,   \
                                           RowVal<T, U>::type*, void*, void*, uint32_t*, uint8_t*, Ctl*, int);   \
  template __global__ void k_row_compact<T, U>(const uint32_t*, const uint32_t*, const uint32_t*, uint64_t,      \
                                               const uint32_t*, const RowVal<T, U>::type*, T, int32_t*,          \
                                               int32_t*, T*);                                                    \
  template __global__ void k_row_max<T, U, false>(const uint32_t*, const uint32_t*, const uint32_t*,              \
                                                  const RowVal<T, U>::type*, const uint32_t*, const uint32_t*,   \
                                                  const uint32_t*, const RowVal<T, U>::type*, T, uint64_t,       \
                                                  uint32_t*, const uint32_t*, int32_t*, int32_t*, T*);           \
  template __global__ void k_row_max<T, U, true>(const uint32_t*, const uint32_t*, const uint32_t*,               \
                                                 const RowVal<T, U>::type*, const uint32_t*, const uint32_t*,    \
                                                 const uint32_t*, const RowVal<T, U>::type*, T, uint64_t,        \
                                                 uint32_t*, const uint32_t*, int32_t*, int32_t*, T*);
#define G2N_INST(T)                                                                                              \
  template __global__ void k_values<T>(const double*, uint64_t, int, int, T*, Ctl*, uint32_t*);                             \
  template __global__ void k_triplets<T>(EdgeIn, uint64_t, const uint32_t*, const DictEntry*,                      \
                                         const uint32_t*, int, int, int32_t*, int32_t*, T*, Ctl*);                \
  template __global__ void k_row_emulate<T>(const uint32_t*, uint64_t, const uint8_t*, const PV<T>*, uint32_t*,    \
                                            T*, KV<int32_t, T>*);                                                 \
  G2N_INST_U(T, true)                                                                                            \
  G2N_INST_U(T, false)
G2N_INST(uint8_t)
G2N_INST(int8_t)
G2N_INST(int32_t)
G2N_INST(float)
G2N_INST(double)
#undef G2N_INST
#undef G2N_INST_U

}  // namespace g2n
