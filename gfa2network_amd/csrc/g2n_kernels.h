// g2n_kernels.h — device-side data layout shared by the kernels and the pipeline driver.
//
// HBM layout of one build (all SoA, sized from counts read back between phases):
//   in[len]                      GFA bytes (read-only)
//   tiles[len / 32 KiB]          per-tile counts (lines, touches, edges, ...) and their scan
//   ls[n_lines + 1]   u64        line start offsets (ls[n_lines] = len)
//   kind[n_lines]     u8         kSkip / kUnknown / kS / kEdge / kPO
//   touches (n_t):   noff u64, nlen u32, tkind u8 [, ooff u64, olen u32 when bidirected]
//   edges   (n_e):   w f64 (weight before the dtype cast), tb u32 (first touch)
//   table[cap]        32-B DictEntry (see k_insert_round), cap = pow2 >= 1.5 x expected keys
//   first u8, nid/tid/slot u32 per touch; inv/klen u32 per node id; names blob + offsets
//   rows/cols i32, data T per triplet; row-bucket sort keys u32 + payloads; per-row SoA sums
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "stl_sort.h"

namespace g2n {

constexpr int kTPB = 256;
#ifndef G2N_TILE_BYTES  // experiment builds (tools/exp_build.sh) may override the tile shape
#define G2N_TILE_BYTES 32768
#endif
#ifndef G2N_TILE_HALO
#define G2N_TILE_HALO 2048
#endif
constexpr uint64_t kTile = G2N_TILE_BYTES;    // input bytes per front-end block (K1, K2)
constexpr uint32_t kTileHalo = G2N_TILE_HALO; // bytes staged past the tile for lines that end beyond it

enum : uint8_t { kSkip = 0, kUnknown = 1, kS = 2, kEdge = 3, kPO = 4 };

// error codes (= G2N_E_* in include/g2n.h)
enum : uint32_t {
  kErrMalformedL = 1,
  kErrMalformedE = 2,
  kErrMalformedC = 3,
  kErrMalformedP = 4,
  kErrMalformedO = 5,
  kErrIndexList = 6,
  kErrIndexBytes = 7,
  kErrUnicode = 8,
  kErrIntTooLarge = 9,
  kErrCastOverflow = 10,
  kErrCastInf = 11,
  kErrCastNan = 12,
};

// an orientation span whose offset carries this flag is the constant byte (off & 0xFF)
constexpr uint64_t kConstFlag = 1ull << 62;
constexpr unsigned long long kEmptySlot = ~0ull;

// device control block: counters and first-error words (zeroed / ~0 per build)
struct Ctl {
  unsigned long long err_key;    // min over (line << 5 | code)
  unsigned long long warn_line;  // min line whose first byte is not in SLPECOHF
  unsigned long long cast_key;   // min over (triplet << 4 | code)
  unsigned long long wl_count;   // deferred weights
  unsigned long long n_lines;
  unsigned long long n_records;
  unsigned long long n_edges;
  unsigned long long n_s;
  unsigned long long n_records_before;
  unsigned long long n_nodes;
  unsigned long long names_len;
  unsigned long long table_overflow;
  unsigned long long detail_off;
  unsigned long long detail_len;
  unsigned long long unsorted[2];
  unsigned long long flagged[2];
  unsigned long long n_unique[2];
  unsigned long long n_keep;
  unsigned long long n_f32_overflow;  // edges whose float32 cast overflowed
  unsigned long long deferred;        // touches left for the next insert round
  unsigned long long dict_general;    // the S-first dictionary fast path does not apply
  unsigned long long s_late;          // an S-line touch follows an edge touch (claim round)
  unsigned long long row_gap;         // k_row_bounds met a run of empty rows too long to fill
  unsigned long long n_deferred;      // lines parsed from global memory after k_tile_parse
  unsigned long long int_fail;        // the decimal-id dictionary (k_int_ids) does not apply
  unsigned long long bucket_overflow; // k_sym_finish met a bucket over its LDS capacity
  unsigned long long bad_id;          // k_remap_pairs met an id outside its map
  unsigned long long ev_dmin, ev_dmax;  // k_tile_lean_evidence: a range's S-name offsets (+ 2^62)
  unsigned long long ev_vmax;           //   and its largest edge key
  unsigned long long w_inexact;         // the weighted bucket SUM's exactness broke (k_weight_encode / k_sumw_finish)
  unsigned long long warn_tile;         // tile-local lean parse: the first tile holding an unsupported record
  unsigned long long warn_off;          //   and that record's byte offset (k_tile_lean_check; warn_line its line)
  unsigned long long dir_vmax;          // the lean claim passes: the largest claimed value (direct tier)
};

struct ParseOpts {
  int bidir, keep, strip, has_wt;
  uint32_t wt_len;
  const uint8_t* wt;  // device copy of the weight tag bytes
  // decimal-id dictionary fused into the parse (see src_dec): when tid is set, every touch's
  // node id is computed from its own bytes while the line is staged; n_seg = S lines (an edge
  // key must name one).  A premise failure sets ctl->int_fail (the hash dictionary then runs).
  uint32_t* tid;
  uint64_t n_seg;
  uint64_t s_base;  // sharded decimal build: S lines before this byte range (0 otherwise)
  // lean mode (decimal ids only): the parse writes the stream-order COO coordinates itself —
  // rows / cols of edge e at e * ktrip (the triplet layout of k_triplets) — and skips the edge
  // touch descriptors, E.tb and (unweighted) E.w; a premise failure re-runs a full parse
  int32_t* rows;
  int32_t* cols;
  uint32_t ktrip;
  // tile-local lean parse (no K1): tile t's COO goes to rows / cols from t * tile_pad * ktrip,
  // its counts to TileCnt and its premise evidence to TileLean; 0 = positions from K1's bases
  uint32_t tile_pad;
  // tile-local lean parse into GROUP slots (k_tile_lean<true>): the kGroupTiles tiles of a group
  // share one slot; a tile's entries go, in tile order inside, at a base it takes with one atomicAdd
  // on its group's count (the group's order of tiles is arbitrary: only for consumers that do not
  // need stream order — the unweighted bucket partition); rows / cols already point at the base
  uint32_t grouped;
  // experiment (G2N_K2_PREFETCH): the one-tile-per-block lean parse warms the cache with tile
  // blockIdx + pf_dist (0: off)
  uint32_t pf_dist;
  // the extended tile-local lean parse (k_tile_lean kExt: bidirected keys, one integer weight tag):
  // edge e's weight at ew[e] (the tile slots' layout, one double per edge line); the weight tag's
  // bytes little-endian (wt_len <= 8) for the comparison against the staged line
  double* ew;
  uint64_t wt_pack;
  // the tile-local decimal parse: tile t's first unsupported record (first byte not in SLPECOHF,
  // ASCII) as its line rank in the tile << 15 | its tile offset, the tile index atomicMin'd into
  // ctl->warn_tile (the one-shot warning without the full parse); null: such a record fails the pass
  uint32_t* tunk;
  // the tile-local decimal parse behind one constant prefix (round 6: minigraph's "s1".."sN" in S order):
  // every name is these dpre_len (<= 8, no digit) bytes, little-endian, then the canonical decimal
  uint64_t dpre;
  uint32_t dpre_len;
  // group slots: 2^gshift tiles per slot (kGroupShift, fewer for small inputs: group_shift_for)
  uint32_t gshift;
  // a grouped weighted SUM CSR (round 6): each triplet's weight as the exact-int32 code the bucket
  // partition sums (weight_enc of the dtype's value: wf32 = the value rounded through float32), written
  // beside rows / cols in the group slots instead of one double per edge line (op.ew)
  uint32_t* wenc;
  uint32_t wf32;
};
constexpr uint32_t kGroupShift = 5;  // at most 32 tiles per group slot

// per-tile evidence of the decimal-id premise in a tile-local parse: every S line's name value
// minus (its S index within the tile + 1), min and max (equal, = the S lines before the tile, when
// the premise holds); the largest edge-key value
struct TileLean {
  long long dmin, dmax;
  unsigned long long vmax;
};

struct TouchOut {
  uint64_t* noff;
  uint32_t* nlen;
  uint64_t* ooff;
  uint32_t* olen;
  uint8_t* tkind;
};
// dictionary entry (32 B): see k_insert_round
struct DictEntry {
  unsigned long long hdr;   // (hash tag << 32) | first touch, later | node id; ~0 = empty
  unsigned long long meta;  // (publication round << 32) | key length; ~0 = unpublished
  unsigned long long k0, k1;  // first 16 key bytes, zero padded
};
struct TouchIn {
  const uint64_t* noff;
  const uint32_t* nlen;
  const uint64_t* ooff;
  const uint32_t* olen;
};
struct EdgeOut {
  double* w;
  uint32_t* tb;
};
struct EdgeIn {
  const double* w;
  const uint32_t* tb;
};

// ---- kernels (g2n_kernels.hip) ----
// K1-K2 (tile front end: k_tile_count, k_tile_parse, k_parse_deferred, k_weights_slow,
// k_error_detail, k_count_records) are defined in g2n_kernels.hip (same translation unit).
template <int kMode>
__global__ void k_insert_round(const uint8_t* in, uint64_t in_len, TouchIn T, uint64_t n_t, DictEntry* table,
                               uint64_t mask, uint64_t max_probes, uint32_t* slot, uint8_t* tstate, uint32_t round,
                               int bidir, Ctl* ctl, uint8_t* first, const uint32_t* nid, uint32_t n_first,
                               const uint32_t* inv, uint32_t* tid);
__global__ void k_key_len(TouchIn T, uint64_t n, int bidir, uint32_t* klen);
template <int kBatch>
__global__ void k_lookup_fast(const uint8_t* in, uint64_t in_len, TouchIn T, uint64_t n_t, const DictEntry* table,
                              uint64_t mask, uint64_t max_probes, const uint8_t* tstate, int bidir, Ctl* ctl,
                              const uint32_t* nid, uint32_t n_first, const uint32_t* inv, uint32_t* tid);
__global__ void k_assign_first(DictEntry* table, TouchIn T, uint64_t n_t, int bidir, const uint8_t* first,
                               const uint32_t* slot, const uint32_t* nid, uint32_t* inv, uint32_t* klen);
__global__ void k_mark_first(const DictEntry* table, uint64_t cap, uint8_t* first);
__global__ void k_assign_ids(DictEntry* table, uint64_t cap, const uint32_t* nid, uint32_t* inv, uint32_t* klen);
__global__ void k_node_count(const uint8_t* first, const uint32_t* nid, uint64_t n_t, Ctl* ctl);
__global__ void k_names_total(const uint32_t* klen, uint64_t n_nodes, int64_t* offs, Ctl* ctl);
__global__ void k_names(const uint8_t* in, TouchIn T, uint64_t n_nodes, const uint32_t* inv, const int64_t* offs,
                        int bidir, uint8_t* blob);
template <class T>
__global__ void k_triplets(EdgeIn E, uint64_t n_e, const uint32_t* slot, const DictEntry* table,
                           const uint32_t* tid, int tpe, int gd, int32_t* rows, int32_t* cols, T* data, Ctl* ctl);
// K7-K9 (COO -> CSR) kernels are templates defined in g2n_kernels.hip (same translation unit).

}  // namespace g2n
