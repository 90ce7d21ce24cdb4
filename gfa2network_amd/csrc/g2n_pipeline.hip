// g2n_pipeline.hip — drives the gfx950 kernels for one GFA -> CSR build.
//
// One build = one pass over the input bytes resident in HBM:
//   lines -> classify -> parse (+ exact weights) -> dictionary -> names -> triplets
//   -> [COO out]  or  sort + group sums (+ std::sort emulation rows) -> [SUM CSR]
//   -> transposed sort + sums, merge, maximum -> [MAX-SYM CSR]
// Every step is a hand-written kernel: g2n_kernels.hip (parse, dictionary, row sums), g2n_scan.hip
// (scans), g2n_sort.hip (stable radix sort), g2n_sym.hip (bucket partition), g2n_route.hip.  Counts are read back between phases (a few
// small synchronous copies per build) to size the next phase's buffers exactly.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>

#include "g2n_internal.h"
#include "g2n_kernels.hip"
#ifndef G2N_NO_GROUP_DEFAULT  // 1: never group slots (experiments)
#define G2N_NO_GROUP_DEFAULT 0
#endif
#ifndef G2N_K2_OLD  // 1: the tile-local parse through k_tile_parse<true> (experiments)
#define G2N_K2_OLD 0
#endif
#ifndef G2N_LOOKUP_BATCH  // touches per thread in the S-first lookup round (experiment builds vary it)
#define G2N_LOOKUP_BATCH 2
#endif
#include "g2n_scan.hip"
#include "g2n_sort.hip"
#include "g2n_sym.hip"
#include "g2n_route.hip"
#include "g2n_inflate.hip"
#include "g2n_keyset.hip"

#define G2N_HIP(call)                                                                                      \
  do {                                                                                                     \
    hipError_t e_ = (call);                                                                                \
    if (e_ != hipSuccess)                                                                                  \
      throw ::g2n::Failure(G2N_E_DEVICE, std::string(#call " failed: ") + hipGetErrorString(e_));          \
  } while (0)

namespace g2n {

// ----------------------------------------------------------------- arena ----------
enum Slot {
  S_IN, S_TILE_CNT, S_TILE_BASE, S_LS, S_KIND, S_NOFF, S_NLEN, S_OOFF, S_OLEN, S_EW, S_ETB, S_WL, S_TABLE,
  S_SLOT, S_FIRST, S_NID, S_FLEN, S_BLOB, S_OFFS, S_ROWS, S_COLS, S_DATA, S_KEYS0, S_KEYS1, S_VALS0, S_VALS1,
  S_KV, S_ODATA, S_INDPTR, S_INDICES, S_TEMP, S_WT, S_TKIND, S_TSTATE, S_RSTART0, S_RSTART1, S_ROUT0,
  S_ROUT1, S_UCNT0, S_UCNT1, S_UOFF, S_MCNT, S_MOFF, S_RSCR, S_RFLAG0, S_RFLAG1, S_RVAL0, S_RVAL1, S_TID,
  S_INV, S_TUNK, S_DEFER, S_FOFF64, S_BTC, S_BTV, S_BTOT, S_EBAD, S_ELEN, S_EPOS, S_ETEXT, S_EFIRST, S_EMETA, S_EL0, S_EL1,
  S_PCNT, S_POFF, S_PGRP, S_BSTART, S_SCANST, S_RBOUND, S_ROWSP, S_COLSP, S_TLEAN, S_ZIN, S_ZMEM, S_ZBAD, S_RSK, S_RSV, S_RSCNT, S_RSOFF,
  S_GCNT, S_TCN, S_FINLB, S_INDPTR64, S_INDICES64, S_WENC, S_W1, S_W2, S_TVAL, S_PW0, S_PW1, S_BSTARTA, S_DIRECT, S_RTOT, S_SCANST2, S_EWP, S_TLIST, S_TNB, S_WENCP, S_NSLOTS
};

#ifndef G2N_MIN_GROUPS  // group slots: fewer tiles per slot until the input has about this many slots
#define G2N_MIN_GROUPS 1024
#endif
#ifndef G2N_PTILE_SMALL_DIV  // partition blocks below 2^24 elements: kPartTile / this many (C2: 8 and 4 alike, 2 slower)
#define G2N_PTILE_SMALL_DIV 4
#endif
#ifndef G2N_FORK_EARLY  // experiment builds: 1 = the deferred side work forked before the partition
#define G2N_FORK_EARLY 0
#endif
#ifndef G2N_F2_OVERLAP  // bucket finish: F1 / F2 in this many bucket ranges, F2 of one beside F1 of the next (1: off)
#define G2N_F2_OVERLAP 4
#endif
#ifndef G2N_FIN_DIRECT  // bucket finish: 1 = F1 places its entries (look-back; measured slower), 0 = F1 stages + F2
#define G2N_FIN_DIRECT 0
#endif

#ifndef G2N_K2_PERSIST  // experiment builds: 1 = the persistent parse, next tile in registers (k_tile_lean_p)
#define G2N_K2_PERSIST 0
#endif
// options.test_flags (tests only; include/g2n.h G2N_TEST_*): take a path that is normally rare, same results
constexpr uint32_t kTestNoBuckets = G2N_TEST_NO_BUCKETS;
constexpr uint32_t kTestNoLean = G2N_TEST_NO_LEAN;
constexpr uint32_t kTestDictHash = G2N_TEST_DICT_HASH;
constexpr uint32_t kTestDictGeneral = G2N_TEST_DICT_GENERAL;
constexpr uint32_t kTestNoTileLocal = G2N_TEST_NO_TILE_LOCAL;
constexpr uint32_t kTestNoGroup = G2N_TEST_NO_GROUP;
constexpr uint32_t kTestNoHashLean = G2N_TEST_NO_HASH_LEAN;
constexpr uint32_t kTestThrowAfterIds = G2N_TEST_THROW_AFTER_IDS;
constexpr uint32_t kTestIndex64 = G2N_TEST_INDEX64;
constexpr uint32_t kTestDictDirect = G2N_TEST_DICT_DIRECT;
constexpr uint32_t kTestNoDirect = G2N_TEST_NO_DIRECT;
constexpr uint32_t kTestNoExtLean = G2N_TEST_NO_EXT_LEAN;
constexpr uint32_t kTestNoDecText = G2N_TEST_NO_DEC_TEXT;
constexpr uint32_t kTestNoDecPrefix = G2N_TEST_NO_DEC_PREFIX;


struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  uint64_t call = 0;  // the entry-point call that last asked for it (g2n_context::call_id)
};
struct ScanSlot {  // a scan status slot (scan_excl): the buffer it last cleared, the epoch / ticket in use
  void* p = nullptr;
  size_t cap = 0;
  uint32_t epoch = 0;
  uint64_t ticket = 0;
};

// The tile-local lean parse's COO in GROUP slots (k_tile_lean<true>): group g's entries are
// [g * gcap, g * gcap + gcount[g]) of rows / cols, its tiles in arbitrary order — for the
// unweighted bucket partition only (csr_partition), which needs no stream order.
struct GroupedCoo {
  bool active = false;
  bool failed = false;  // the partition could not take it: the build is redone without groups
  const int32_t* rows = nullptr;
  const int32_t* cols = nullptr;
  const uint32_t* gcount = nullptr;
  uint64_t gcap = 0, n_groups = 0;
  const uint32_t* wenc = nullptr;  // a weighted build's codes beside rows / cols (ParseOpts::wenc)
};

}  // namespace g2n

struct g2n_context {
  int device = 0;
  int n_cu = 256;  // compute units: persistent launches size their grid from it
  uint32_t test_flags = 0;  // options.test_flags of the current build: forces rare paths (tests)
  uint64_t err_line_off = 0;  // byte offset of the last build's error line (edge-list prefix)
  g2n::GroupedCoo gcoo;       // the current build's COO, when it went to group slots
  g2n::GroupedCoo slots;      // the last build's COO result when it stayed in group slots (G2N_RANGE_SLOTS)
  const uint32_t* wenc = nullptr;  // the current build's values as exact-int32 codes (k_values), if written
  bool no_group = false;      // redo of a build whose group-slot COO the partition refused
  g2n::ScanSlot scan_slot[g2n::S_NSLOTS];  // scan_excl's per-slot epoch / ticket state
  bool edge_text = false;     // run_edge_list's build: decimal names are left to the text render
  bool names_dec = false;     // ... and that build's names were the decimal ids (no blob written)
  hipStream_t stream = nullptr;
  hipStream_t side = nullptr;   // work that overlaps the main stream (the decimal names blob)
  hipEvent_t side_ev[2] = {nullptr, nullptr};  // main -> side fork, side -> main join
  hipStream_t place = nullptr;  // F2 (k_sym_place) of earlier bucket ranges beside F1 of later ones
  hipEvent_t ov_ev[17] = {};    // F1 range k done (main -> place); [16]: place -> main join
  bool side_pending = false;    // the main stream has not joined the side stream's last work yet
  uint64_t lean_blocks = 0;     // k_tile_lean_p blocks resident on the device at once (its grid)
  bool range_has_s = false;     // g2n_build_decimal_range: the range's evidence (k_tile_lean_evidence)
  int64_t range_d = -1;
  uint64_t range_vmax = 0;
  uint64_t range_nseg = 0;
  std::function<void()> side_work;  // launches deferred to the assembly's latency-bound finish (F1)
  std::vector<g2n::DevBuf> bufs;
  uint64_t call_id = 0;  // entry-point calls so far (enter_call): a slot no call since asked for is stale
  bool shared = false;   // a host entry points' cached context (shared_context): its callers hold no views
  size_t hbm_total = 0;  // the device's HBM (hipMemGetInfo at creation)
  g2n::Ctl* ctl = nullptr;    // device
  g2n::Ctl* h_ctl = nullptr;  // pinned host mirror
  hipEvent_t ev[G2N_MAX_PHASES + 1];
  int n_ev = 0;
  const char* ev_name[G2N_MAX_PHASES];
  std::mutex mu;
};

namespace g2n {

// Every entry point that takes a context's lock opens a call here before its first dget: slots the
// call asks for are stamped with it, so an allocation that fails in a shared context can release the
// slots only earlier calls used (a grow-only arena keeps an earlier, larger build's buffers: 40 GB of
// input text, say — beside which convert_format's 39 GB row band did not fit).  A caller's own
// context (g2n_context_create) is never released behind its back: g2n_context_trim is its tool.
static void enter_call(g2n_context* c) { c->call_id++; }

// the slots no dget of the current call has touched, freed (their contents belong to finished calls;
// results they held were valid only until this call).  Returns the bytes released.
static uint64_t release_stale(g2n_context* c) {
  for (hipStream_t s : {c->stream, c->side, c->place})
    if (s) (void)hipStreamSynchronize(s);
  uint64_t total = 0;
  for (int s = 0; s < S_NSLOTS; s++) {
    DevBuf& b = c->bufs[s];
    if (!b.p || b.call == c->call_id) continue;
    (void)hipFree(b.p);
    total += b.cap;
    b.p = nullptr;
    b.cap = 0;
    c->scan_slot[s] = ScanSlot{};  // a later allocation at the same address must be cleared again
  }
  return total;
}

// After a host entry point's call (its results already downloaded): a shared context keeps its buffers
// for the next call only while they hold at most a quarter of the device — a 1.1G-edge build's 100+ GB
// arena would otherwise stay reserved behind every later allocation of the process.
static void shrink_shared(g2n_context* c) {
  if (!c->shared || !c->hbm_total) return;
  uint64_t held = 0;
  for (const DevBuf& b : c->bufs) held += b.p ? b.cap : 0;
  if (held <= c->hbm_total / 4) return;
  c->call_id++;  // (every slot is an earlier call's now)
  (void)release_stale(c);
  c->gcoo = GroupedCoo{};
  c->slots = GroupedCoo{};
  c->wenc = nullptr;
}

static void* dbuf(g2n_context* c, int slot, size_t bytes) {
  DevBuf& b = c->bufs[slot];
  b.call = c->call_id;
  if (bytes == 0) bytes = 16;
  if (b.cap < bytes) {
    if (b.p) G2N_HIP(hipFree(b.p));
    b.p = nullptr;
    b.cap = 0;
    size_t want = bytes + bytes / 8 + 256;
    if (hipMalloc(&b.p, want) != hipSuccess) {
      (void)hipGetLastError();
      // a host entry point's context (whose results were downloaded, whose inputs are host memory):
      // once more without the earlier calls' buffers, and without the growth margin
      b.p = nullptr;
      if (c->shared && release_stale(c)) want = bytes + 256;
      if (hipMalloc(&b.p, want) != hipSuccess) {
        (void)hipGetLastError();
        b.p = nullptr;
        throw Failure(G2N_E_NOMEM, "hipMalloc of " + std::to_string(want) + " bytes failed");
      }
    }
    b.cap = want;
  }
  return b.p;
}
template <class T>
static T* dget(g2n_context* c, int slot, uint64_t count) {
  return (T*)dbuf(c, slot, (size_t)count * sizeof(T));
}

static inline unsigned grid_for(uint64_t n, unsigned tpb = kTPB) {
  uint64_t g = (n + tpb - 1) / tpb;
  return (unsigned)(g ? g : 1);
}

static void phase(g2n_context* c, const char* name) {
  if (c->n_ev >= G2N_MAX_PHASES) return;
  c->ev_name[c->n_ev] = name;
  G2N_HIP(hipEventRecord(c->ev[c->n_ev + 1], c->stream));
  c->n_ev++;
}

static void sync_ctl(g2n_context* c) {
  G2N_HIP(hipMemcpyAsync(c->h_ctl, c->ctl, sizeof(Ctl), hipMemcpyDeviceToHost, c->stream));
  G2N_HIP(hipStreamSynchronize(c->stream));
}

// the deferred side-stream launches (run_build's decimal names), forked from the main stream here
static void fork_side(g2n_context* c) {
  if (!c->side_work) return;
  G2N_HIP(hipEventRecord(c->side_ev[0], c->stream));
  G2N_HIP(hipStreamWaitEvent(c->side, c->side_ev[0], 0));
  c->side_work();
  c->side_work = nullptr;
  G2N_HIP(hipEventRecord(c->side_ev[1], c->side));
  c->side_pending = true;
}

static void join_side(g2n_context* c) {
  fork_side(c);
  if (!c->side_pending) return;
  G2N_HIP(hipStreamWaitEvent(c->stream, c->side_ev[1], 0));
  c->side_pending = false;
}

// Every entry point starts here: a build that threw may have left a deferred side launch (its
// buffers are not this call's), an unjoined side stream, or an active group-slot COO behind on
// this context.  The deferred launch is dropped, the side stream joined (its buffers may be
// reused by this call), the group slots forgotten.
static void clear_call_state(g2n_context* c) {
  c->side_work = nullptr;
  if (c->side_pending) {
    G2N_HIP(hipStreamWaitEvent(c->stream, c->side_ev[1], 0));
    c->side_pending = false;
  }
  c->gcoo = GroupedCoo{};
  c->wenc = nullptr;
}

template <class T>
static T read_dev(g2n_context* c, const T* p) {
  T v;
  G2N_HIP(hipMemcpyAsync(&v, p, sizeof(T), hipMemcpyDeviceToHost, c->stream));
  G2N_HIP(hipStreamSynchronize(c->stream));
  return v;
}

// exclusive scan of n items (k_scan_excl, decoupled look-back); *total (device, optional) = sum.
// The slot's buffer (ticket, then status words) is cleared only when it is (re)allocated or its
// epochs run out: each launch takes the next epoch and the ticket base (one launch per slot at a
// time, in the order of stream s — a slot belongs to one stream)
template <class TIn, class TOut>
static void scan_excl(g2n_context* c, const TIn* in, TOut* out, uint64_t n, TOut* total = nullptr,
                      hipStream_t s = nullptr, int slot = S_SCANST) {
  if (n == 0 && !total) return;
  if (!s) s = c->stream;
  const uint64_t tiles = scan_tiles(n);
  auto* st = dget<unsigned long long>(c, slot, tiles + 1);  // the ticket, then the status words
  ScanSlot& ss = c->scan_slot[slot];
  const size_t cap = c->bufs[slot].cap;
  if (ss.p != (void*)st || ss.cap != cap || ss.epoch >= kStEpochs) {
    G2N_HIP(hipMemsetAsync(st, 0, cap, s));
    ss.p = st;
    ss.cap = cap;
    ss.epoch = 0;
    ss.ticket = 0;
  }
  ss.epoch++;
  hipLaunchKernelGGL((k_scan_excl<TIn, TOut>), dim3((unsigned)tiles), dim3(256), 0, s, in, out, n, st + 1, st, total,
                     ss.epoch, (unsigned long long)ss.ticket);
  ss.ticket += tiles;
}
template <class T>
static void excl_scan(g2n_context* c, const T* in, T* out, uint64_t n) {
  scan_excl<T, T>(c, in, out, n);
}


static int bits_for(uint64_t n) {  // bits to hold values 0..n-1 (>= 1)
  int b = 1;
  while (b < 63 && (1ull << b) < n) b++;
  return b;
}

static size_t dtype_size(int dt) {
  switch (dt) {
    case G2N_BOOL: case G2N_INT8: return 1;
    case G2N_INT32: case G2N_FLOAT32: return 4;
    default: return 8;
  }
}

// ------------------------------------------------- SUM (coo.tocsr) on device -------
template <class T, bool kU>
struct RowSide {  // one orientation's per-row sums: row r's unique entries at [start[r], +ucnt[r])
  using V = typename RowVal<T, kU>::type;  // run length (uniform build) or summed value
  uint32_t* start;
  uint32_t* ucnt;
  uint32_t* ocol;
  V* oval;
  bool unsorted, flagged, local_unsorted;
};

// Stable LSD radix sort of (u32 key, V) pairs on key bits [begin, bits) (g2n_sort.hip): ceil(w / 8)
// passes of equal digit width; kin / vin are left intact, the result lands in kout / vout.
template <class V>
static void sort_pairs_u32(g2n_context* c, const uint32_t* kin, uint32_t* kout, const V* vin, V* vout, uint64_t n,
                           int bits, int begin = 0) {
  if (n == 0) return;
  if (n >= 0xFFFFFFFFull) throw Failure(G2N_E_UNSUPPORTED, "radix sort of 2^32 or more items");
  const int w = bits - begin > 0 ? bits - begin : 1;
  const int passes = (w + (int)kRsMaxBits - 1) / (int)kRsMaxBits;
  const uint64_t n_blk = (n + kRsTile - 1) / kRsTile;
  auto* tk = dget<uint32_t>(c, S_RSK, passes > 1 ? n : 1);
  auto* tv = dget<V>(c, S_RSV, passes > 1 ? n : 1);
  auto* cnt = dget<uint32_t>(c, S_RSCNT, (uint64_t)kRsMaxDig * n_blk);
  auto* off = dget<uint32_t>(c, S_RSOFF, (uint64_t)kRsMaxDig * n_blk);
  const uint32_t* ki = kin;
  const V* vi = vin;
  int lo = begin;
  for (int p = 0; p < passes; p++) {
    const int db = (w - (lo - begin) + (passes - p) - 1) / (passes - p);  // equal widths, rounded up first
    const uint32_t n_dig = 1u << db;
    // the last pass writes kout; earlier ones alternate so that it does
    const bool to_out = ((passes - 1 - p) & 1) == 0;
    uint32_t* ko = to_out ? kout : tk;
    V* vo = to_out ? vout : tv;
    hipLaunchKernelGGL(k_rsort_hist, dim3((unsigned)n_blk), dim3(kRsTPB), 0, c->stream, ki, n, (uint32_t)lo, n_dig,
                       cnt, n_blk);
    scan_excl<uint32_t, uint32_t>(c, cnt, off, (uint64_t)n_dig * n_blk);
    hipLaunchKernelGGL((k_rsort_scatter<V>), dim3((unsigned)n_blk), dim3(kRsTPB), 0, c->stream, ki, vi, ko, vo, n,
                       (uint32_t)lo, (uint32_t)db, (const uint32_t*)off, n_blk);
    ki = ko;
    vi = vo;
    lo += db;
  }
}

// coo.tocsr() of one orientation (transposed: of A.T), up to the per-row sorted unique entries.
// side: which set of per-row buffers (0: A, 1: A.T); transposed: key on the column;
// base: first row of the slice; force_unsorted: -1 = this matrix decides scipy's global
// has_sorted_indices, else the caller's verdict (sharded builds: the OR over all slices).
template <class T, bool kU>
static RowSide<T, kU> row_sums(g2n_context* c, const int32_t* rows, const int32_t* cols, const T* data, uint64_t n,
                               uint64_t n_rows, int side, int transposed, int64_t base = 0,
                               int force_unsorted = -1) {
  const int w = side;
  using V = typename RowVal<T, kU>::type;
  RowSide<T, kU> S{};
  auto* key_in = dget<uint32_t>(c, S_KEYS0, n);
  auto* key_out = dget<uint32_t>(c, S_KEYS1, n);
  S.start = dget<uint32_t>(c, w ? S_RSTART1 : S_RSTART0, n_rows + 1);
  S.ucnt = dget<uint32_t>(c, w ? S_UCNT1 : S_UCNT0, n_rows);
  S.ocol = dget<uint32_t>(c, w ? S_ROUT1 : S_ROUT0, n);
  S.oval = dget<V>(c, w ? S_RVAL1 : S_RVAL0, n);
  auto* rowflag = dget<uint8_t>(c, w ? S_RFLAG1 : S_RFLAG0, n_rows);
  PV<T>* pv_out = nullptr;
  uint32_t* pc_out = nullptr;
  void *scr_a = nullptr, *scr_b = nullptr;  // long-row merge scratch: buffers the sort no longer needs
  G2N_HIP(hipMemsetAsync(rowflag, 0, n_rows ? n_rows : 1, c->stream));
  const int bits = bits_for(n_rows);
  if (n) {
    if (kU) {
      auto* pc_in = dget<uint32_t>(c, S_VALS0, n);
      pc_out = dget<uint32_t>(c, S_VALS1, n);
      if (base == 0) {  // the coordinates are the sort's input as they are (rocPRIM leaves inputs intact)
        const uint32_t* r = (const uint32_t*)rows;
        const uint32_t* q = (const uint32_t*)cols;
        sort_pairs_u32<uint32_t>(c, transposed ? q : r, key_out, transposed ? r : q, pc_out, n, bits);
      } else {
        hipLaunchKernelGGL((k_pack<T, true>), dim3(grid_for(n)), dim3(kTPB), 0, c->stream, rows, cols, data, n,
                           transposed, base, key_in, (PV<T>*)nullptr, pc_in);
        sort_pairs_u32<uint32_t>(c, key_in, key_out, pc_in, pc_out, n, bits);
      }
      scr_a = key_in;
      scr_b = pc_in;
    } else {
      auto* pv_in = dget<PV<T>>(c, S_VALS0, n);
      pv_out = dget<PV<T>>(c, S_VALS1, n);
      hipLaunchKernelGGL((k_pack<T, false>), dim3(grid_for(n)), dim3(kTPB), 0, c->stream, rows, cols, data, n,
                         transposed, base, key_in, pv_in, (uint32_t*)nullptr);
      sort_pairs_u32<PV<T>>(c, key_in, key_out, pv_in, pv_out, n, bits);
      scr_a = pv_in;
      scr_b = dget<PV<T>>(c, S_RSCR, n);
    }
  }
  G2N_HIP(hipMemsetAsync(&c->ctl->row_gap, 0, sizeof(unsigned long long), c->stream));
  hipLaunchKernelGGL(k_row_bounds, dim3(grid_for(n + 1)), dim3(kTPB), 0, c->stream, key_out, n, n_rows, S.start,
                     c->ctl);
  hipLaunchKernelGGL(k_row_start, dim3(grid_for(n_rows + 1)), dim3(kTPB), 0, c->stream, key_out, n, n_rows, S.start,
                     (const Ctl*)c->ctl);
  if (n_rows)
    hipLaunchKernelGGL((k_row_sum<T, kU>), dim3(grid_for(n_rows)), dim3(kTPB), 0, c->stream, S.start, n_rows, pv_out,
                       pc_out, S.ocol, S.oval, scr_a, scr_b, S.ucnt, rowflag, c->ctl, w);
  sync_ctl(c);
  S.local_unsorted = c->h_ctl->unsorted[w] != 0;
  S.unsorted = force_unsorted >= 0 ? force_unsorted != 0 : S.local_unsorted;
  S.flagged = c->h_ctl->flagged[w] != 0;
  if constexpr (!kU) {
    if (n && S.unsorted && S.flagged) {  // scipy std::sort-ed these rows: redo them exactly
      auto* kv = dget<KV<int32_t, T>>(c, S_KV, n);
      hipLaunchKernelGGL((k_row_emulate<T>), dim3(grid_for(n_rows, 64)), dim3(64), 0, c->stream, S.start, n_rows,
                         rowflag, pv_out, S.ocol, S.oval, kv);
    }
  }
  return S;
}

// Unweighted A.maximum(A.T) (sum = false) or coo.tocsr() (sum = true) through the bucket partition
// (g2n_sym.hip): the A entries (and, for MAX-SYM, their A.T twins) are partitioned by the high bits
// of their row (one or two hand-written passes), then one finish block per bucket writes its rows'
// CSR entries at their final place.  False when
// the row ids are too wide for two passes or a bucket overflowed its LDS capacity (nothing
// usable was written: the caller runs the general path).
// The same for a sharded build's row slice [row_base, row_base + n_rows): t_rows / t_cols / n_t =
// the slice's A.T entries (MAX-SYM; rows = A's columns), each one element of side 1.
template <class T>
static bool csr_partition(g2n_context* c, const int32_t* rows, const int32_t* cols, uint64_t n_trip, uint64_t n_rows,
                          bool sum, g2n_result* R, const int32_t* t_rows = nullptr, const int32_t* t_cols = nullptr,
                          uint64_t n_t = 0, int64_t row_base = 0) {
  if (G2N_FORK_EARLY) fork_side(c);  // experiment: the side work beside the partition passes
  const bool pair = t_rows != nullptr || row_base != 0;  // one element per entry of two streams
  const int bits = bits_for(n_rows);
  const double per_row =
      (double)(pair ? n_trip + n_t : (sum ? 1 : 2) * n_trip) / (double)(n_rows ? n_rows : 1);
  // rows per bucket 2^low <= kFinTPB (one finish thread per row): about half the finish block's
  // capacity on average (kSymCap / 2 elements)
  int low = 0;
  while ((1u << (low + 1)) <= kFinTPB) low++;
  while (low > 1 && (double)(1u << low) * per_row > (double)(kSymCap / 2)) low--;
  if (low > bits) low = bits;
  const int hb = bits - low;  // bucket id bits
  // pass 2 takes up to kWideDigitBits only past 2^20 buckets (more than 2^31 elements at most 2^11 per
  // bucket): the tuned 10-bit kernels otherwise; pass 1's groups stay <= 1024 (k_part_groups)
  const int max2 = hb > 2 * (int)kMaxDigitBits ? (int)kWideDigitBits : (int)kMaxDigitBits;
  if (hb > (int)kMaxDigitBits + max2) return false;
  // two passes: at most 8 bits in pass 1 (its sub-tiles rank 8192 COO entries: longer runs per
  // digit), the rest in pass 2 (C4, hb = 18: 8 + 10 measured 9.07 ms per build against 9.19 for 9 + 9
  // and 9.39 for 10 + 8)
  const int bits1 = hb > max2 ? std::max(hb - max2, std::min(8, (hb + 1) / 2)) : hb;
  const int bits2 = hb - bits1;
  const uint32_t n_dig1 = 1u << bits1, n_dig2 = 1u << bits2;
  const uint64_t n_el = pair ? n_trip + n_t : (sum ? 1 : 2) * n_trip;
  if (n_el >= 0xFFFFFFFFull) return false;
  const uint64_t n_buckets = 1ull << hb;                      // ids of the partition
  const uint64_t n_bk = (n_rows + (1ull << low) - 1) >> low;  // buckets holding rows
  const uint32_t shift1 = (uint32_t)(low + bits2);
  const bool grouped = c->gcoo.active && !pair;
  PartSrc src{(const uint32_t*)(grouped ? c->gcoo.rows : rows), (const uint32_t*)(grouped ? c->gcoo.cols : cols),
              grouped ? c->gcoo.n_groups * c->gcoo.gcap : n_trip, (sum || pair) ? 1u : 0u,
              (const uint32_t*)t_rows, (const uint32_t*)t_cols, pair ? n_t : 0, (uint32_t)row_base,
              nullptr, nullptr, nullptr, 0, grouped ? c->gcoo.gcount : nullptr, grouped ? c->gcoo.gcap : 0,
              (sum || pair) ? 0u : (uint32_t)low + 1u};
  // pass 1: over the COO entries, both sides (grouped: one block per group slot).  MAX-SYM: pair
  // elements go out as 4-byte words (stream A, g2n_sym.hip), the rest as 8-byte elements (stream B);
  // the count matrix holds B's digits then A's, each part scanned on its own
  const bool words = !t_rows && (sum || !pair);  // passes 1 and 4 (not the two-stream slices' pass 3)
  // elements per partition block: a quarter tile below 2^24 elements, so a small input still spreads
  // over more blocks than the 256 CUs
  const uint32_t ptile = n_el >= (1ull << 24) ? kPartTile : kPartTile / G2N_PTILE_SMALL_DIV;
  src.tile = ptile;
  const uint64_t n_blk1 = grouped ? c->gcoo.n_groups : (n_el + ptile - 1) / ptile;
  const uint64_t nm1 = (uint64_t)n_dig1 * n_blk1;  // one stream's count matrix
  auto* cnt1 = dget<uint32_t>(c, S_PCNT, (words ? 2 : 1) * nm1);
  auto* off1 = dget<uint32_t>(c, S_POFF, (words ? 2 : 1) * nm1);
  auto* el1 = dget<uint2>(c, S_EL0, n_el);
  uint32_t* wa1 = words ? dget<uint32_t>(c, S_PW0, n_trip) : nullptr;
  if (sum && !t_rows) {  // the SUM CSR: one element per entry, adjacent transposed twins as one (a word)
    src.pair_bits = (uint32_t)low + 1u;
    hipLaunchKernelGGL(k_part_hist<4>, dim3((unsigned)n_blk1), dim3(kPartTPB), 0, c->stream, src, shift1, n_dig1,
                       cnt1, n_blk1);
    scan_excl<uint32_t, uint32_t>(c, cnt1, off1, 2 * nm1);  // both streams' matrices (the scatter rebases A's)
    hipLaunchKernelGGL(k_part_scatter<4>, dim3((unsigned)n_blk1), dim3(kPartTPB), 0, c->stream, src, shift1, n_dig1,
                       (const uint32_t*)off1, n_blk1, el1, wa1);
  } else if (sum || pair) {  // one element per entry
    hipLaunchKernelGGL(k_part_hist<3>, dim3((unsigned)n_blk1), dim3(kPartTPB), 0, c->stream, src, shift1, n_dig1,
                       cnt1, n_blk1);
    scan_excl<uint32_t, uint32_t>(c, cnt1, off1, (uint64_t)n_dig1 * n_blk1);
    hipLaunchKernelGGL(k_part_scatter<3>, dim3((unsigned)n_blk1), dim3(kPartTPB), 0, c->stream, src, shift1, n_dig1,
                       (const uint32_t*)off1, n_blk1, el1);
  } else {
    hipLaunchKernelGGL(k_part_hist<1>, dim3((unsigned)n_blk1), dim3(kPartTPB), 0, c->stream, src, shift1, n_dig1,
                       cnt1, n_blk1);
    scan_excl<uint32_t, uint32_t>(c, cnt1, off1, 2 * nm1);  // both streams' matrices (the scatter rebases A's)
    hipLaunchKernelGGL(k_part_scatter<1>, dim3((unsigned)n_blk1), dim3(kPartTPB), 0, c->stream, src, shift1, n_dig1,
                       (const uint32_t*)off1, n_blk1, el1, wa1);
  }
  auto* bst = dget<uint32_t>(c, S_BSTART, n_buckets + 1);
  uint32_t* bstA = words ? dget<uint32_t>(c, S_BSTARTA, n_buckets + 1) : nullptr;
  const uint2* el = el1;
  const uint32_t* wa = wa1;
  if (bits2 == 0) {
    hipLaunchKernelGGL(k_part_bucket_starts1, dim3(grid_for(n_buckets + 1)), dim3(kTPB), 0, c->stream,
                       (const uint32_t*)off1, (const uint32_t*)cnt1, n_blk1, n_buckets, bst, (const uint32_t*)nullptr);
    if (words)
      hipLaunchKernelGGL(k_part_bucket_starts1, dim3(grid_for(n_buckets + 1)), dim3(kTPB), 0, c->stream,
                         (const uint32_t*)(off1 + nm1), (const uint32_t*)(cnt1 + nm1), n_blk1, n_buckets, bstA,
                         (const uint32_t*)(off1 + nm1));
  } else {  // pass 2 inside each pass-1 group (stream A's groups: the second half of S_PGRP)
    auto* grp = dget<uint32_t>(c, S_PGRP, 4 * ((uint64_t)n_dig1 + 1));
    uint32_t* grpA = grp + 2 * ((uint64_t)n_dig1 + 1);
    PartSrc s2{nullptr, nullptr, 0, 0, nullptr, nullptr, 0, 0, el1, grp, grp + n_dig1 + 1, n_dig1, nullptr, 0, 0};
    s2.tile = ptile;
    // (one launch for both streams' groups: stream A's at grpA = grp + 2 (n_dig1 + 1))
    hipLaunchKernelGGL(k_part_groups, dim3(words ? 2 : 1), dim3(1024), 0, c->stream, (const uint32_t*)off1,
                       (const uint32_t*)cnt1, n_blk1, n_dig1, grp, ptile);
    // >= the blocks the groups need (sum of ceil(group / ptile) <= n_el / ptile + n_dig1)
    const uint64_t n_blk2 = (n_el + ptile - 1) / ptile + n_dig1;
    const uint64_t n2 = (uint64_t)n_dig2 * n_blk2;  // one stream's pass-2 count matrix
    const uint64_t ns = words ? 2 : 1;
    auto* cnt2 = dget<uint32_t>(c, S_PCNT, ns * n2);
    auto* off2 = dget<uint32_t>(c, S_POFF, std::max<uint64_t>(ns * n2, ns * nm1));
    auto* el2 = dget<uint2>(c, S_EL1, n_el);
    // pass 7: stream A's words (its count matrix after pass 2's, both scanned by one launch; its
    // offsets less the scan's value at its start, s2a.obase)
    PartSrc s2a{nullptr, nullptr, 0, 0, nullptr, nullptr, 0, 0, nullptr, grpA, grpA + n_dig1 + 1, n_dig1,
                nullptr, 0, (uint32_t)low + 1u, nullptr, wa1, ptile};
    s2a.obase = off2 + n2;
    uint32_t* wa2 = words ? dget<uint32_t>(c, S_PW1, n_trip) : nullptr;
    const bool wide = bits2 > (int)kMaxDigitBits;
    if (wide) {
      hipLaunchKernelGGL((k_part_hist<2, kWideDigitBits>), dim3((unsigned)n_blk2), dim3(kPartTPB), 0, c->stream, s2,
                         (uint32_t)low, n_dig2, cnt2, n_blk2);
      if (words)
        hipLaunchKernelGGL((k_part_hist<7, kWideDigitBits>), dim3((unsigned)n_blk2), dim3(kPartTPB), 0, c->stream,
                           s2a, 2u * (uint32_t)low, n_dig2, cnt2 + n2, n_blk2);
    } else {
      hipLaunchKernelGGL(k_part_hist<2>, dim3((unsigned)n_blk2), dim3(kPartTPB), 0, c->stream, s2, (uint32_t)low,
                         n_dig2, cnt2, n_blk2);
      if (words)
        hipLaunchKernelGGL(k_part_hist<7>, dim3((unsigned)n_blk2), dim3(kPartTPB), 0, c->stream, s2a,
                           2u * (uint32_t)low, n_dig2, cnt2 + n2, n_blk2);
    }
    scan_excl<uint32_t, uint32_t>(c, cnt2, off2, ns * n2);
    if (wide)
      hipLaunchKernelGGL((k_part_scatter<2, kWideDigitBits>), dim3((unsigned)n_blk2), dim3(kPartTPB), 0, c->stream, s2,
                         (uint32_t)low, n_dig2, (const uint32_t*)off2, n_blk2, el2);
    else
      hipLaunchKernelGGL(k_part_scatter<2>, dim3((unsigned)n_blk2), dim3(kPartTPB), 0, c->stream, s2, (uint32_t)low,
                         n_dig2, (const uint32_t*)off2, n_blk2, el2);
    hipLaunchKernelGGL(k_part_bucket_starts, dim3(grid_for(n_buckets + 1)), dim3(kTPB), 0, c->stream,
                       (const uint32_t*)off2, s2, n_dig2, n_buckets, bst);
    el = el2;
    if (words) {
      if (wide)
        hipLaunchKernelGGL((k_part_scatter<7, kWideDigitBits>), dim3((unsigned)n_blk2), dim3(kPartTPB), 0,
                           c->stream, s2a, 2u * (uint32_t)low, n_dig2, (const uint32_t*)(off2 + n2), n_blk2,
                           (uint2*)nullptr, wa2);
      else
        hipLaunchKernelGGL(k_part_scatter<7>, dim3((unsigned)n_blk2), dim3(kPartTPB), 0, c->stream, s2a,
                           2u * (uint32_t)low, n_dig2, (const uint32_t*)(off2 + n2), n_blk2, (uint2*)nullptr, wa2);
      hipLaunchKernelGGL(k_part_bucket_starts, dim3(grid_for(n_buckets + 1)), dim3(kTPB), 0, c->stream,
                         (const uint32_t*)(off2 + n2), s2a, n_dig2, n_buckets, bstA);
      wa = wa2;
    }
  }
  phase(c, "sum");
  auto* indptr = dget<int32_t>(c, S_INDPTR, n_rows + 1);
  auto* indices = dget<int32_t>(c, S_INDICES, n_el);
  T* odata = dget<T>(c, S_ODATA, n_el);
  auto* btot = dget<uint32_t>(c, S_BTOT, n_bk);
  uint2* tmp = el == el1 ? dget<uint2>(c, S_EL1, n_el) : el1;  // the pass-1 output is dead by now
  // staged entries (F1 -> F2): up to two per stored element (kElPair) — columns (u32) in tmp's 8 bytes
  // per element, the copies (u16, written only for sums of several copies) beside them
  auto* tcol = (uint32_t*)tmp;
  auto* tcn = dget<uint16_t>(c, S_TCN, 2 * n_el);
  G2N_HIP(hipMemsetAsync(&c->ctl->bucket_overflow, 0, sizeof(unsigned long long), c->stream));
#ifdef G2N_F1_STAMPS
  unsigned long long* f1st = dget<unsigned long long>(c, S_TEMP, n_bk * kF1Stamps);
  G2N_HIP(hipMemsetAsync(f1st, 0, n_bk * kF1Stamps * 8, c->stream));
  G2N_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g2n_f1_stamps), &f1st, sizeof(f1st), 0, hipMemcpyHostToDevice,
                                 c->stream));
#endif
  fork_side(c);  // F1 leaves HBM bandwidth to spare (G2N_FORK_EARLY: forked before pass 1 instead)
#if G2N_FIN_DIRECT
  // F1 places every bucket's entries itself, its offset from a decoupled look-back over the buckets
  auto* lbst = dget<uint64_t>(c, S_FINLB, n_bk);
  G2N_HIP(hipMemsetAsync(lbst, 0, n_bk * sizeof(uint64_t), c->stream));
  if (sum)
    hipLaunchKernelGGL((k_sym_finish<T, true, true>), dim3((unsigned)n_bk), dim3(kFinTPB), 0, c->stream, el,
                       (const uint32_t*)bst, (uint32_t)low, n_rows, (T)1, btot, tcol, tcn, indptr, c->ctl, lbst,
                       indices, odata, (uint32_t)row_base, wa, (const uint32_t*)bstA, 0u);
  else
    hipLaunchKernelGGL((k_sym_finish<T, false, true>), dim3((unsigned)n_bk), dim3(kFinTPB), 0, c->stream, el,
                       (const uint32_t*)bst, (uint32_t)low, n_rows, (T)1, btot, tcol, tcn, indptr, c->ctl, lbst,
                       indices, odata, (uint32_t)row_base, wa, (const uint32_t*)bstA, 0u);
#ifdef G2N_F1_STAMPS
  if (const char* out = std::getenv("G2N_F1_STAMPS_OUT")) {  // diagnostics build only
    std::vector<unsigned long long> h(n_bk * kF1Stamps);
    G2N_HIP(hipMemcpyAsync(h.data(), f1st, h.size() * 8, hipMemcpyDeviceToHost, c->stream));
    G2N_HIP(hipStreamSynchronize(c->stream));
    if (FILE* f = std::fopen(out, "wb")) {
      std::fwrite(h.data(), 8, h.size(), f);
      std::fclose(f);
    }
  }
#endif
  sync_ctl(c);
  if (c->h_ctl->bucket_overflow) return false;
  const int32_t nnz = read_dev(c, indptr + n_rows);
#else
  // F1 / F2 overlapped by bucket ranges: F1 of range k + 1 on the main stream runs beside the scan and
  // F2 of range k on the place stream (F1 is latency-bound, F2 a copy that F1 leaves bandwidth for);
  // F2 adds the entries of the ranges before its own to the range-relative offsets
  // (large builds only: on C2's 3.9K buckets the extra launches cost more than the overlap gives,
  // 0.455 -> 0.549 ms per build)
  const uint32_t n_ov = (G2N_F2_OVERLAP > 1 && n_el <= 0x7FFFFFFFull && !(c->test_flags & kTestIndex64) &&
                         n_bk >= 32768ull)
                            ? (uint32_t)std::min(G2N_F2_OVERLAP, 16)
                            : 1u;
  // range k: buckets [rb(k), rb(k + 1)), equal ranges (ranges shrinking geometrically, so that the last F2
  // is shorter, measured slower: 70 % steps over 4 or 6 ranges, 55 % over 4, +0.06-0.18 ms per C4 build)
  auto rb = [&](uint32_t k) -> uint64_t { return n_bk * k / n_ov; };
  if (n_ov > 1) {
    auto* boff = dget<uint32_t>(c, S_MOFF, n_bk + 1);
    auto* rtot = dget<uint32_t>(c, S_RTOT, n_ov);
    (void)dget<unsigned long long>(c, S_SCANST2, scan_tiles(n_bk) + 1);  // sized once, before the ranges' scans
    for (uint32_t k = 0; k < n_ov; k++) {
      const uint64_t b0 = rb(k), b1 = rb(k + 1);
      if (sum)
        hipLaunchKernelGGL((k_sym_finish<T, true, false>), dim3((unsigned)(b1 - b0)), dim3(kFinTPB), 0, c->stream, el,
                           (const uint32_t*)bst, (uint32_t)low, n_rows, (T)1, btot, tcol, tcn, indptr, c->ctl,
                           (uint64_t*)nullptr, (int32_t*)nullptr, (T*)nullptr, (uint32_t)row_base, wa,
                           (const uint32_t*)bstA, (uint32_t)b0);
      else
        hipLaunchKernelGGL((k_sym_finish<T, false, false>), dim3((unsigned)(b1 - b0)), dim3(kFinTPB), 0, c->stream,
                           el, (const uint32_t*)bst, (uint32_t)low, n_rows, (T)1, btot, tcol, tcn, indptr, c->ctl,
                           (uint64_t*)nullptr, (int32_t*)nullptr, (T*)nullptr, (uint32_t)row_base, wa,
                           (const uint32_t*)bstA, (uint32_t)b0);
      G2N_HIP(hipEventRecord(c->ov_ev[k], c->stream));
    }
    for (uint32_t k = 0; k < n_ov; k++) {
      const uint64_t b0 = rb(k), b1 = rb(k + 1);
      G2N_HIP(hipStreamWaitEvent(c->place, c->ov_ev[k], 0));
      scan_excl<uint32_t, uint32_t>(c, (const uint32_t*)(btot + b0), boff + b0, b1 - b0, rtot + k, c->place, S_SCANST2);
      hipLaunchKernelGGL((k_sym_place<T, int32_t>), dim3((unsigned)(b1 - b0)), dim3(kFinTPB), 0, c->place,
                         (const uint32_t*)bst, (const uint32_t*)btot, (const uint32_t*)boff, (uint32_t)low, n_rows,
                         (T)1, (const uint32_t*)tcol, (const uint16_t*)tcn, indptr, indices, odata, (int64_t*)nullptr,
                         (const uint32_t*)bstA, (uint32_t)b0, (const uint32_t*)rtot, k);
    }
    G2N_HIP(hipEventRecord(c->ov_ev[16], c->place));
    G2N_HIP(hipStreamWaitEvent(c->stream, c->ov_ev[16], 0));
    int32_t nnz = 0;  // one wait for the overflow flag and the entry count
    G2N_HIP(hipMemcpyAsync(&nnz, indptr + n_rows, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    sync_ctl(c);
    if (c->h_ctl->bucket_overflow) return false;
    R->format = G2N_FMT_CSR;
    R->indptr = indptr;
    R->nnz = (int64_t)nnz;
    R->indices = indices;
    R->data = odata;
    R->sum_sorted = -1;
    R->sum_t_sorted = -1;
    phase(c, sum ? "csr" : "maxsym");
    return true;
  }
  if (sum)
    hipLaunchKernelGGL((k_sym_finish<T, true, false>), dim3((unsigned)n_bk), dim3(kFinTPB), 0, c->stream, el,
                       (const uint32_t*)bst, (uint32_t)low, n_rows, (T)1, btot, tcol, tcn, indptr, c->ctl,
                       (uint64_t*)nullptr, (int32_t*)nullptr, (T*)nullptr, (uint32_t)row_base, wa,
                       (const uint32_t*)bstA, 0u);
  else
    hipLaunchKernelGGL((k_sym_finish<T, false, false>), dim3((unsigned)n_bk), dim3(kFinTPB), 0, c->stream, el,
                       (const uint32_t*)bst, (uint32_t)low, n_rows, (T)1, btot, tcol, tcn, indptr, c->ctl,
                       (uint64_t*)nullptr, (int32_t*)nullptr, (T*)nullptr, (uint32_t)row_base, wa,
                       (const uint32_t*)bstA, 0u);
#ifdef G2N_F1_STAMPS
  if (const char* out = std::getenv("G2N_F1_STAMPS_OUT")) {  // diagnostics build only
    std::vector<unsigned long long> h(n_bk * kF1Stamps);
    G2N_HIP(hipMemcpyAsync(h.data(), f1st, h.size() * 8, hipMemcpyDeviceToHost, c->stream));
    G2N_HIP(hipStreamSynchronize(c->stream));
    if (FILE* f = std::fopen(out, "wb")) {
      std::fwrite(h.data(), 8, h.size(), f);
      std::fclose(f);
    }
  }
#endif
  auto* boff = dget<uint32_t>(c, S_MOFF, n_bk + 1);
  scan_excl<uint32_t, uint32_t>(c, btot, boff, n_bk, boff + n_bk);
  // (an overflowed bucket is found after F2: its placement is then dropped with the rest)
  if (n_el > 0x7FFFFFFFull || (c->test_flags & kTestIndex64)) {
    sync_ctl(c);
    if (c->h_ctl->bucket_overflow) return false;
  }
  // scipy's index dtype (get_index_dtype(maxval=nnz)): int64 indptr / indices once the result holds
  // more than 2^31 - 1 entries (utils.py:55 coo.tocsr, builders.py:283 maximum) — only possible when
  // the partition's upper bound passes it, so the total is read only then
  // coo.tocsr() (the SUM CSR) sizes its index dtype by the COO's entries, duplicates included
  // (scipy _coo_to_compressed: maxval = coo.nnz; sum_duplicates keeps the dtype); A.maximum(A.T) by
  // the result's entries (_binopt's arrays, then the constructor's check_contents downcast).  A
  // bucket's merged entries never outnumber its expanded input: the result holds <= n_el entries.
  const bool wide = (c->test_flags & kTestIndex64) || (sum && !pair && n_trip > 0x7FFFFFFFull) ||
                    (!sum && n_el > 0x7FFFFFFFull && (uint64_t)read_dev(c, boff + n_bk) > 0x7FFFFFFFull);
  if (wide) {
    if (pair) throw Failure(G2N_E_UNSUPPORTED, "a sharded row slice of more than 2^31-1 entries");
    auto* indptr64 = dget<int64_t>(c, S_INDPTR64, n_rows + 1);
    auto* indices64 = dget<int64_t>(c, S_INDICES64, n_el);
    hipLaunchKernelGGL((k_sym_place<T, int64_t>), dim3((unsigned)n_bk), dim3(kFinTPB), 0, c->stream,
                       (const uint32_t*)bst, (const uint32_t*)btot, (const uint32_t*)boff, (uint32_t)low, n_rows, (T)1,
                       (const uint32_t*)tcol, (const uint16_t*)tcn, indptr, indices64, odata, indptr64,
                       (const uint32_t*)bstA, 0u, (const uint32_t*)nullptr, 0u);
    R->format = G2N_FMT_CSR;
    R->index_width = 8;
    R->indptr = indptr64;
    R->nnz = read_dev(c, indptr64 + n_rows);
    R->indices = indices64;
    R->data = odata;
    R->sum_sorted = -1;
    R->sum_t_sorted = -1;
    phase(c, sum ? "csr" : "maxsym");
    return true;
  }
  hipLaunchKernelGGL((k_sym_place<T, int32_t>), dim3((unsigned)n_bk), dim3(kFinTPB), 0, c->stream,
                     (const uint32_t*)bst, (const uint32_t*)btot, (const uint32_t*)boff, (uint32_t)low, n_rows, (T)1,
                     (const uint32_t*)tcol, (const uint16_t*)tcn, indptr, indices, odata, (int64_t*)nullptr,
                     (const uint32_t*)bstA, 0u, (const uint32_t*)nullptr, 0u);
  int32_t nnz = 0;  // one wait for the overflow flag and the entry count
  G2N_HIP(hipMemcpyAsync(&nnz, indptr + n_rows, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  sync_ctl(c);
  if (c->h_ctl->bucket_overflow) return false;
#endif
  R->format = G2N_FMT_CSR;
  R->indptr = indptr;
  R->nnz = (int64_t)nnz;
  R->indices = indices;
  R->data = odata;
  R->sum_sorted = -1;  // not computed: unweighted sums cannot depend on scipy's order
  R->sum_t_sorted = -1;
  phase(c, sum ? "csr" : "maxsym");
  return true;
}

// Weighted coo.tocsr() (utils.py:55 / builders.py:281 with a weight tag) through the same bucket
// partition, when no duplicate sum can depend on scipy's summation order (k_weight_encode: integer
// dtypes and bool always; float values that are integers of |v| < 2^31, not -0.0, with every
// entry's sum of magnitudes exact in T — checked per run by k_sumw_finish).  Passes 5 / 6 carry
// each element's value (u32) beside it; F1w sums a row's column runs in any order.  False, with
// nothing usable written, when the partition declines (as csr_partition) or the premise fails:
// the caller then runs the stable row-sum path.
template <class T>
static bool csr_partition_w(g2n_context* c, const int32_t* rows, const int32_t* cols, const T* data, uint64_t n_trip,
                            uint64_t n_rows, uint64_t n_cols, g2n_result* R) {
  if (n_rows >= (1ull << 30) || n_cols >= (1ull << 30) || n_trip > 0x7FFFFFFFull) return false;
  const int bits = bits_for(n_rows);
  const double per_row = (double)n_trip / (double)(n_rows ? n_rows : 1);
  int low = 0;
  while ((1u << (low + 1)) <= kFinTPB) low++;
  while (low > 1 && (double)(1u << low) * per_row > (double)(kSymCap / 2)) low--;
  if (low > bits) low = bits;
  const int hb = bits - low;
  if (hb > 2 * (int)kMaxDigitBits) return false;
  const int bits1 = hb > (int)kMaxDigitBits ? std::max(hb - (int)kMaxDigitBits, std::min(8, (hb + 1) / 2)) : hb;
  const int bits2 = hb - bits1;
  const uint32_t n_dig1 = 1u << bits1, n_dig2 = 1u << bits2;
  const uint64_t n_el = n_trip;
  const uint64_t n_buckets = 1ull << hb;
  const uint64_t n_bk = (n_rows + (1ull << low) - 1) >> low;
  const uint32_t shift1 = (uint32_t)(low + bits2);
  const uint32_t* enc = c->wenc;  // k_values wrote the codes beside the values (and w_inexact)
  if (!enc) {
    auto* e = dget<uint32_t>(c, S_WENC, n_el);
    G2N_HIP(hipMemsetAsync(&c->ctl->w_inexact, 0, sizeof(unsigned long long), c->stream));
    hipLaunchKernelGGL((k_weight_encode<T>), dim3(grid_for(n_el)), dim3(kTPB), 0, c->stream, data, n_el, e, c->ctl);
    enc = e;
  }
  G2N_HIP(hipMemsetAsync(&c->ctl->bucket_overflow, 0, sizeof(unsigned long long), c->stream));
  PartSrc src{(const uint32_t*)rows, (const uint32_t*)cols, n_trip, 1u, nullptr, nullptr, 0, 0, nullptr, nullptr,
              nullptr, 0, nullptr, 0, (uint32_t)low + 1u, enc, nullptr};
  // pass 5: the entries with their values, adjacent transposed twins of one value as one element
  const uint32_t ptile = n_el >= (1ull << 24) ? kPartTile : kPartTile / G2N_PTILE_SMALL_DIV;  // as csr_partition
  src.tile = ptile;
  const bool grouped = c->gcoo.active;  // (with the parse's codes: run_build) one block per group slot
  if (grouped) {
    src.rows = (const uint32_t*)c->gcoo.rows;
    src.cols = (const uint32_t*)c->gcoo.cols;
    src.n_entries = c->gcoo.n_groups * c->gcoo.gcap;
    src.gcount = c->gcoo.gcount;
    src.gcap = c->gcoo.gcap;
  }
  const uint64_t n_blk1 = grouped ? c->gcoo.n_groups : (n_el + ptile - 1) / ptile;
  auto* cnt1 = dget<uint32_t>(c, S_PCNT, (uint64_t)n_dig1 * n_blk1);
  auto* off1 = dget<uint32_t>(c, S_POFF, (uint64_t)n_dig1 * n_blk1);
  auto* el1 = dget<uint2>(c, S_EL0, n_el);
  auto* w1 = dget<uint32_t>(c, S_W1, n_el);
  hipLaunchKernelGGL(k_part_hist<5>, dim3((unsigned)n_blk1), dim3(kPartTPB), 0, c->stream, src, shift1, n_dig1, cnt1,
                     n_blk1);
  scan_excl<uint32_t, uint32_t>(c, cnt1, off1, (uint64_t)n_dig1 * n_blk1);
  hipLaunchKernelGGL(k_part_scatter<5>, dim3((unsigned)n_blk1), dim3(kPartTPB), 0, c->stream, src, shift1, n_dig1,
                     (const uint32_t*)off1, n_blk1, el1, w1);
  auto* bst = dget<uint32_t>(c, S_BSTART, n_buckets + 1);
  const uint2* el = el1;
  const uint32_t* ew = w1;
  if (bits2 == 0) {
    hipLaunchKernelGGL(k_part_bucket_starts1, dim3(grid_for(n_buckets + 1)), dim3(kTPB), 0, c->stream,
                       (const uint32_t*)off1, (const uint32_t*)cnt1, n_blk1, n_buckets, bst, (const uint32_t*)nullptr);
  } else {  // pass 6 inside each pass-5 group
    auto* grp = dget<uint32_t>(c, S_PGRP, 2 * ((uint64_t)n_dig1 + 1));
    PartSrc s2{nullptr, nullptr, 0, 0, nullptr, nullptr, 0, 0, el1, grp, grp + n_dig1 + 1, n_dig1, nullptr, 0, 0,
               nullptr, w1, ptile};
    hipLaunchKernelGGL(k_part_groups, dim3(1), dim3(1024), 0, c->stream, (const uint32_t*)off1, (const uint32_t*)cnt1,
                       n_blk1, n_dig1, grp, ptile);
    const uint64_t n_blk2 = (n_el + ptile - 1) / ptile + n_dig1;
    auto* cnt2 = dget<uint32_t>(c, S_PCNT, (uint64_t)n_dig2 * n_blk2);
    auto* off2 = dget<uint32_t>(c, S_POFF, std::max<uint64_t>((uint64_t)n_dig2 * n_blk2, (uint64_t)n_dig1 * n_blk1));
    auto* el2 = dget<uint2>(c, S_EL1, n_el);
    auto* w2 = dget<uint32_t>(c, S_W2, n_el);
    hipLaunchKernelGGL(k_part_hist<6>, dim3((unsigned)n_blk2), dim3(kPartTPB), 0, c->stream, s2, (uint32_t)low,
                       n_dig2, cnt2, n_blk2);
    scan_excl<uint32_t, uint32_t>(c, cnt2, off2, (uint64_t)n_dig2 * n_blk2);
    hipLaunchKernelGGL(k_part_scatter<6>, dim3((unsigned)n_blk2), dim3(kPartTPB), 0, c->stream, s2, (uint32_t)low,
                       n_dig2, (const uint32_t*)off2, n_blk2, el2, w2);
    hipLaunchKernelGGL(k_part_bucket_starts, dim3(grid_for(n_buckets + 1)), dim3(kTPB), 0, c->stream,
                       (const uint32_t*)off2, s2, n_dig2, n_buckets, bst);
    el = el2;
    ew = w2;
  }
  phase(c, "sum");
  auto* indptr = dget<int32_t>(c, S_INDPTR, n_rows + 1);
  auto* btot = dget<uint32_t>(c, S_BTOT, n_bk);
  // staged merged entries (F1w -> F2w): at most two per element (kElPair) — columns in the dead
  // partition buffer's 8 bytes per element, values in their own array
  auto* tcol = (uint32_t*)(el == el1 ? dget<uint2>(c, S_EL1, n_el) : el1);
  T* tval = dget<T>(c, S_TVAL, 2 * n_el);
  fork_side(c);  // the deferred names beside the finish (as csr_partition), not after the CSR
#ifdef G2N_F1_STAMPS
  unsigned long long* f1st = dget<unsigned long long>(c, S_TEMP, n_bk * kF1Stamps);
  G2N_HIP(hipMemsetAsync(f1st, 0, n_bk * kF1Stamps * 8, c->stream));
  G2N_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g2n_f1_stamps), &f1st, sizeof(f1st), 0, hipMemcpyHostToDevice,
                                 c->stream));
#endif
  hipLaunchKernelGGL((k_sumw_finish<T>), dim3((unsigned)n_bk), dim3(kFinTPB), 0, c->stream, el, ew,
                     (const uint32_t*)bst, (uint32_t)low, n_rows, btot, tcol, tval, indptr, c->ctl);
#ifdef G2N_F1_STAMPS
  if (const char* out = std::getenv("G2N_F1_STAMPS_OUT")) {  // diagnostics build only
    std::vector<unsigned long long> h(n_bk * kF1Stamps);
    G2N_HIP(hipMemcpyAsync(h.data(), f1st, h.size() * 8, hipMemcpyDeviceToHost, c->stream));
    G2N_HIP(hipStreamSynchronize(c->stream));
    if (FILE* f = std::fopen(out, "wb")) {
      std::fwrite(h.data(), 8, h.size(), f);
      std::fclose(f);
    }
  }
#endif
  auto* boff = dget<uint32_t>(c, S_MOFF, n_bk + 1);
  scan_excl<uint32_t, uint32_t>(c, btot, boff, n_bk, boff + n_bk);
  // (an overflowed bucket or an inexact sum is found after F2w: its placement is then dropped)
  auto* indices = dget<int32_t>(c, S_INDICES, 2 * n_el);
  T* odata = dget<T>(c, S_ODATA, 2 * n_el);
  hipLaunchKernelGGL((k_sumw_place<T>), dim3((unsigned)n_bk), dim3(kFinTPB), 0, c->stream, (const uint32_t*)bst,
                     (const uint32_t*)btot, (const uint32_t*)boff, (uint32_t)low, n_rows, (const uint32_t*)tcol,
                     (const T*)tval, indptr, indices, odata);
  int32_t nnz = 0;  // one wait for the flags and the entry count
  G2N_HIP(hipMemcpyAsync(&nnz, indptr + n_rows, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  sync_ctl(c);
  if (c->h_ctl->bucket_overflow || c->h_ctl->w_inexact) return false;
  R->format = G2N_FMT_CSR;
  R->indptr = indptr;
  R->nnz = (int64_t)nnz;
  R->indices = indices;
  R->data = odata;
  R->sum_sorted = -1;  // not computed: these sums cannot depend on scipy's order
  R->sum_t_sorted = -1;
  phase(c, "csr");
  return true;
}

template <class T, bool kU>
static void assemble_t(g2n_context* c, const int32_t* rows, const int32_t* cols, const T* data, uint64_t n_trip,
                       uint64_t n_rows, uint64_t n_cols, bool maxsym, g2n_result* R, int force_unsorted = -1) {
  if constexpr (kU) {
    if (n_trip && n_rows && (n_rows == n_cols || !maxsym) && !(c->test_flags & kTestNoBuckets) &&
        csr_partition<T>(c, rows, cols, n_trip, n_rows, !maxsym, R))
      return;
  } else {
    if (n_trip && n_rows && !maxsym && (!c->gcoo.active || c->gcoo.wenc) && !(c->test_flags & kTestNoBuckets) &&
        csr_partition_w<T>(c, rows, cols, data, n_trip, n_rows, n_cols, R))
      return;
  }
  if (c->gcoo.active) {  // the group slots hold no stream order: redo the build without them
    c->gcoo.failed = true;
    return;
  }
  // the row-sum path (weighted / float sums, or a partition that declined) keeps int32 positions
  if (n_trip >= 0x7FFFFFFFull) throw Failure(G2N_E_UNSUPPORTED, "more than 2^31-1 weighted matrix entries");
  const T one = (T)1;
  // (force_unsorted >= 0: a row band of a larger COO, g2n_coo_to_csr_band — scipy's verdict is the whole
  // matrix's; sum_sorted still reports this band's own)
  RowSide<T, kU> A = row_sums<T, kU>(c, rows, cols, data, n_trip, n_rows, 0, 0, 0, force_unsorted);
  R->sum_sorted = A.local_unsorted ? 0 : 1;
  phase(c, "sum");
  auto* indptr = dget<int32_t>(c, S_INDPTR, n_rows + 1);
  if (n_rows == 0) G2N_HIP(hipMemsetAsync(indptr, 0, sizeof(int32_t), c->stream));
  R->format = G2N_FMT_CSR;
  R->indptr = indptr;
  if (!maxsym) {
    auto* uoff = dget<uint32_t>(c, S_UOFF, n_rows);
    excl_scan<uint32_t>(c, A.ucnt, uoff, n_rows);
    auto* indices = dget<int32_t>(c, S_INDICES, n_trip);
    T* odata = dget<T>(c, S_ODATA, n_trip);
    if (n_rows) {
      hipLaunchKernelGGL((k_row_compact<T, kU>), dim3(grid_for(n_rows)), dim3(kTPB), 0, c->stream, A.start, A.ucnt,
                         uoff, n_rows, A.ocol, A.oval, one, indptr, indices, odata);
      hipLaunchKernelGGL(k_scan_total, dim3(1), dim3(1), 0, c->stream, A.ucnt, uoff, n_rows, &c->ctl->n_keep);
    }
    R->nnz = n_rows ? (int64_t)read_dev(c, &c->ctl->n_keep) : 0;
    R->indices = indices;
    R->data = odata;
    phase(c, "csr");
    return;
  }
  // A.maximum(A.T): B = SUM(A) above, BT = SUM(A.T) with A.T's own scatter order
  RowSide<T, kU> B = row_sums<T, kU>(c, rows, cols, data, n_trip, n_cols, 1, 1);
  phase(c, "sum_t");
  auto* mcnt = dget<uint32_t>(c, S_MCNT, n_rows);
  auto* moff = dget<uint32_t>(c, S_MOFF, n_rows);
  auto* indices = dget<int32_t>(c, S_INDICES, 2 * n_trip);
  T* odata = dget<T>(c, S_ODATA, 2 * n_trip);
  if (n_rows) {
    hipLaunchKernelGGL((k_row_max<T, kU, false>), dim3(grid_for(n_rows)), dim3(kTPB), 0, c->stream, A.start, A.ucnt,
                       A.ocol, A.oval, B.start, B.ucnt, B.ocol, B.oval, one, n_rows, mcnt, (const uint32_t*)nullptr,
                       (int32_t*)nullptr, (int32_t*)nullptr, (T*)nullptr);
    excl_scan<uint32_t>(c, mcnt, moff, n_rows);
    hipLaunchKernelGGL((k_row_max<T, kU, true>), dim3(grid_for(n_rows)), dim3(kTPB), 0, c->stream, A.start, A.ucnt,
                       A.ocol, A.oval, B.start, B.ucnt, B.ocol, B.oval, one, n_rows, mcnt, moff, indptr, indices,
                       odata);
    hipLaunchKernelGGL(k_scan_total, dim3(1), dim3(1), 0, c->stream, mcnt, moff, n_rows, &c->ctl->n_keep);
  }
  R->nnz = n_rows ? (int64_t)read_dev(c, &c->ctl->n_keep) : 0;
  R->indices = indices;
  R->data = odata;
  phase(c, "maxsym");
}

// The CSR row slice [base, base + n_rows) of a sharded build from its routed triplet streams:
// A's triplets with rows in the slice and (MAX-SYM) A.T's, i.e. (col, row, value) of A's
// triplets whose column is in the slice; both in global stream order.
template <class T, bool kU>
static void assemble_pair_t(g2n_context* c, const int32_t* ar, const int32_t* ac, const T* ad, uint64_t an,
                            const int32_t* tr, const int32_t* tc, const T* td, uint64_t tn, bool maxsym, int64_t base,
                            uint64_t n_rows, int force_unsorted, g2n_result* R) {
  if constexpr (kU) {  // unweighted: the bucket partition (the slice's sums cannot depend on order)
    // one rank that routed nothing passes A's own arrays swapped as the A.T stream: the whole-matrix
    // MAX-SYM partition then reads each entry once and pairs its two sides (kElPair) like one GPU
    const bool self_t = maxsym && tn == an && tr == ac && tc == ar && base == 0;
    if (self_t && an && n_rows && !(c->test_flags & kTestNoBuckets) &&
        csr_partition<T>(c, ar, ac, an, n_rows, false, R)) {
      R->sum_sorted = R->sum_t_sorted = 1;
      return;
    }
    if (an + tn && n_rows && base >= 0 && base < 0xFFFFFFFFll && !(c->test_flags & kTestNoBuckets) &&
        csr_partition<T>(c, ar, ac, an, n_rows, !maxsym, R, maxsym ? (tr ? tr : ar) : nullptr,
                         maxsym ? tc : nullptr, maxsym ? tn : 0, base ? base : 0)) {
      R->sum_sorted = R->sum_t_sorted = 1;
      return;
    }
  }
  const T one = (T)1;
  RowSide<T, kU> A = row_sums<T, kU>(c, ar, ac, ad, an, n_rows, 0, 0, base,
                                     force_unsorted < 0 ? -1 : (force_unsorted & 1));
  R->sum_sorted = A.local_unsorted ? 0 : 1;
  phase(c, "sum");
  auto* indptr = dget<int32_t>(c, S_INDPTR, n_rows + 1);
  if (n_rows == 0) G2N_HIP(hipMemsetAsync(indptr, 0, sizeof(int32_t), c->stream));
  R->format = G2N_FMT_CSR;
  R->indptr = indptr;
  if (!maxsym) {
    auto* uoff = dget<uint32_t>(c, S_UOFF, n_rows);
    excl_scan<uint32_t>(c, A.ucnt, uoff, n_rows);
    auto* indices = dget<int32_t>(c, S_INDICES, an);
    T* odata = dget<T>(c, S_ODATA, an);
    if (n_rows) {
      hipLaunchKernelGGL((k_row_compact<T, kU>), dim3(grid_for(n_rows)), dim3(kTPB), 0, c->stream, A.start, A.ucnt,
                         uoff, n_rows, A.ocol, A.oval, one, indptr, indices, odata);
      hipLaunchKernelGGL(k_scan_total, dim3(1), dim3(1), 0, c->stream, A.ucnt, uoff, n_rows, &c->ctl->n_keep);
    }
    R->nnz = n_rows ? (int64_t)read_dev(c, &c->ctl->n_keep) : 0;
    R->indices = indices;
    R->data = odata;
    phase(c, "csr");
    return;
  }
  RowSide<T, kU> B = row_sums<T, kU>(c, tr, tc, td, tn, n_rows, 1, 0, base,
                                     force_unsorted < 0 ? -1 : ((force_unsorted >> 1) & 1));
  R->sum_t_sorted = B.local_unsorted ? 0 : 1;
  phase(c, "sum_t");
  auto* mcnt = dget<uint32_t>(c, S_MCNT, n_rows);
  auto* moff = dget<uint32_t>(c, S_MOFF, n_rows);
  auto* indices = dget<int32_t>(c, S_INDICES, an + tn);
  T* odata = dget<T>(c, S_ODATA, an + tn);
  if (n_rows) {
    hipLaunchKernelGGL((k_row_max<T, kU, false>), dim3(grid_for(n_rows)), dim3(kTPB), 0, c->stream, A.start, A.ucnt,
                       A.ocol, A.oval, B.start, B.ucnt, B.ocol, B.oval, one, n_rows, mcnt, (const uint32_t*)nullptr,
                       (int32_t*)nullptr, (int32_t*)nullptr, (T*)nullptr);
    excl_scan<uint32_t>(c, mcnt, moff, n_rows);
    hipLaunchKernelGGL((k_row_max<T, kU, true>), dim3(grid_for(n_rows)), dim3(kTPB), 0, c->stream, A.start, A.ucnt,
                       A.ocol, A.oval, B.start, B.ucnt, B.ocol, B.oval, one, n_rows, mcnt, moff, indptr, indices,
                       odata);
    hipLaunchKernelGGL(k_scan_total, dim3(1), dim3(1), 0, c->stream, mcnt, moff, n_rows, &c->ctl->n_keep);
  }
  R->nnz = n_rows ? (int64_t)read_dev(c, &c->ctl->n_keep) : 0;
  R->indices = indices;
  R->data = odata;
  phase(c, "maxsym");
}

template <class T>
static void assemble(g2n_context* c, const int32_t* rows, const int32_t* cols, const T* data, uint64_t n_trip,
                     uint64_t n_rows, uint64_t n_cols, bool maxsym, bool uniform, g2n_result* R,
                     int force_unsorted = -1) {
  if (uniform) assemble_t<T, true>(c, rows, cols, data, n_trip, n_rows, n_cols, maxsym, R, force_unsorted);
  else assemble_t<T, false>(c, rows, cols, data, n_trip, n_rows, n_cols, maxsym, R, force_unsorted);
}

template <class T>
static void run_triplets(g2n_context* c, EdgeIn E, uint64_t n_e, const uint32_t* slot,
                         const DictEntry* table, const uint32_t* tid, int tpe, int gd, int32_t* rows,
                         int32_t* cols, void* data) {
  if (n_e)
    hipLaunchKernelGGL((k_triplets<T>), dim3(grid_for(n_e)), dim3(kTPB), 0, c->stream, E, n_e, slot, table, tid, tpe,
                       gd, rows, cols, (T*)data, c->ctl);
}

static void reset_ctl(g2n_context* c) {
  std::memset(c->h_ctl, 0, sizeof(Ctl));
  c->h_ctl->err_key = ~0ull;
  c->h_ctl->warn_line = ~0ull;
  c->h_ctl->cast_key = ~0ull;
  c->h_ctl->ev_dmin = ~0ull;
  c->h_ctl->warn_tile = ~0ull;
  G2N_HIP(hipMemcpyAsync(c->ctl, c->h_ctl, sizeof(Ctl), hipMemcpyHostToDevice, c->stream));
}

static void finish_timings(g2n_context* c, g2n_result* R) {
  join_side(c);
  G2N_HIP(hipStreamSynchronize(c->stream));
  R->n_phases = c->n_ev;
  for (int k = 0; k < c->n_ev; k++) {
    float ms = 0.f;
    G2N_HIP(hipEventElapsedTime(&ms, c->ev[k], c->ev[k + 1]));
    R->phase_ms[k] = ms;
    R->phase_names[k] = c->ev_name[k];
  }
}

// The pipeline.  R's pointers are device pointers into the context's arena.
// ---- dictionary (K4): first-touch node ids of the n_t touches (the first n_st are the S-line
// touches of the claim round).  est: expected distinct keys (sizes the first table).
struct DictOut {
  DictEntry* table;
  uint32_t* slot;
  uint32_t* tid;        // node id per touch (S-first paths; claimers excluded), else null
  const uint32_t* inv;  // node id -> touch with its key bytes (null: the identity)
  uint32_t* klen;       // node id -> key length
  uint8_t* first;       // first-touch flags
  bool general;         // ids came from the general insert rounds (every touch has a slot)
  uint64_t n_nodes;
};

// decimal-id dictionary (ParseOpts.tid): done by the parse (tid final), or not applicable
enum IntIds { kIntDone, kIntFailed };

static DictOut build_dictionary(g2n_context* c, const uint8_t* in, uint64_t len, const TouchOut& T, uint64_t n_t,
                                uint64_t n_st, uint64_t est, bool bidir, IntIds int_ids) {
  TouchIn TI{T.noff, T.nlen, T.ooff, T.olen};
  // Table sized for the expected number of distinct keys; a bounded probe sequence flags
  // overflow and the insert is redone with a table sized for every touch (load <= 1/2,
  // unbounded probes).
  uint64_t full_cap = 1024;
  while (full_cap < 2 * n_t) full_cap <<= 1;
  uint64_t cap = 1024;
  while (cap < est + est / 2) cap <<= 1;
  if (cap > full_cap) cap = full_cap;
  auto* slot = dget<uint32_t>(c, S_SLOT, n_t);
  auto* first = dget<uint8_t>(c, S_FIRST, n_t);
  auto* nid = dget<uint32_t>(c, S_NID, n_t);
  auto* inv = dget<uint32_t>(c, S_INV, n_t);    // node id -> touch holding its key bytes
  auto* klen = dget<uint32_t>(c, S_FLEN, n_t);  // node id -> key length
  DictEntry* table = nullptr;
  uint32_t* tid = nullptr;  // node id per touch when the S-first fast path holds
  auto* tstate = dget<uint8_t>(c, S_TSTATE, n_t);
  const uint32_t* nid_in = nid;  // fast lookup: firsts before each touch (null: n_first for every touch)
  const uint32_t* inv_in = inv;
  uint32_t n_first = 0;
  auto insert = [&](int mode, uint32_t round, uint64_t max_probes, uint32_t* tid_out) {
    G2N_HIP(hipMemsetAsync(&c->ctl->deferred, 0, sizeof(unsigned long long), c->stream));
    phase(c, "_prep");
    const dim3 g(grid_for(n_t)), b(kTPB);
    if (mode == kModeClaim)
      hipLaunchKernelGGL(k_insert_round<kModeClaim>, g, b, 0, c->stream, in, len, TI, n_t, table, cap - 1,
                         max_probes, slot, tstate, round, (int)bidir, c->ctl, first, nid_in, n_first, inv_in, tid_out);
    else if (mode == kModeLookup)
      hipLaunchKernelGGL(k_insert_round<kModeLookup>, g, b, 0, c->stream, in, len, TI, n_t, table, cap - 1,
                         max_probes, slot, tstate, round, (int)bidir, c->ctl, first, nid_in, n_first, inv_in, tid_out);
    else {
      const dim3 gb(grid_for(n_t, kTPB * G2N_LOOKUP_BATCH));  // G2N_LOOKUP_BATCH touches per thread
      hipLaunchKernelGGL(k_lookup_fast<G2N_LOOKUP_BATCH>, gb, b, 0, c->stream, in, len, TI, n_t, table, cap - 1,
                         max_probes, tstate, (int)bidir, c->ctl, nid_in, n_first, inv_in, tid_out);
    }
    phase(c, mode == kModeClaim ? "insert_claim" : "insert_lookup");
    sync_ctl(c);
  };
  auto init_table = [&]() {
    table = dget<DictEntry>(c, S_TABLE, cap);
    G2N_HIP(hipMemsetAsync(table, 0xFF, cap * sizeof(DictEntry), c->stream));
    G2N_HIP(hipMemcpyAsync(tstate, T.tkind, n_t, hipMemcpyDeviceToDevice, c->stream));
    phase(c, "table_init");
  };
  auto rank_firsts = [&]() {  // nid[t] = first touches before t; n_nodes
    scan_excl<uint8_t, uint32_t>(c, first, nid, n_t);
    hipLaunchKernelGGL(k_node_count, dim3(1), dim3(1), 0, c->stream, first, nid, n_t, c->ctl);
  };
  if (n_t) {
    // S-first fast path (a GFA whose S lines define every key before any other line uses it):
    // round 1 claims the S keys, their ranks are the node ids, one lookup round resolves every
    // other touch to its id.  Anything else is redone by the general rounds below.
    bool fast = !(c->test_flags & kTestDictGeneral);
    if (int_ids == kIntDone) {  // decimal-id dictionary: the parse wrote every edge touch's id
      hipLaunchKernelGGL(k_key_len, dim3(grid_for(n_st)), dim3(kTPB), 0, c->stream, TI, n_st, (int)bidir, klen);
      phase(c, "ids_fast");
      c->h_ctl->n_nodes = n_st;
      G2N_HIP(hipMemcpyAsync(&c->ctl->n_nodes, &c->h_ctl->n_nodes, sizeof(unsigned long long),
                             hipMemcpyHostToDevice, c->stream));
      DictOut D{};
      D.slot = slot;
      D.tid = dget<uint32_t>(c, S_TID, n_t);
      D.klen = klen;
      D.first = first;
      D.n_nodes = n_st;
      return D;
    }
    if (fast) {
      init_table();
      n_first = (uint32_t)n_st;  // claim round: flags S touches past the first n_st
      insert(kModeClaim, 1, cap >= full_cap ? cap : 4096, nullptr);
      fast = !c->h_ctl->table_overflow;
    }
    bool sprefix = false;  // ids are touch indices: no ranking pass
    if (fast) {
      sprefix = c->h_ctl->deferred == 0 && !c->h_ctl->s_late;
      if (sprefix) {
        nid_in = nullptr;
        inv_in = nullptr;
        n_first = (uint32_t)n_st;
        hipLaunchKernelGGL(k_key_len, dim3(grid_for(n_st)), dim3(kTPB), 0, c->stream, TI, n_st, (int)bidir, klen);
        c->h_ctl->n_nodes = n_st;
        G2N_HIP(hipMemcpyAsync(&c->ctl->n_nodes, &c->h_ctl->n_nodes, sizeof(unsigned long long),
                               hipMemcpyHostToDevice, c->stream));
      } else {
        rank_firsts();
        hipLaunchKernelGGL(k_assign_first, dim3(grid_for(n_t)), dim3(kTPB), 0, c->stream, table, TI, n_t,
                           (int)bidir, first, slot, nid, inv, klen);
      }
      phase(c, "ids_fast");
      tid = dget<uint32_t>(c, S_TID, n_t);
      // the lookup round resolves the touches that claimed nothing; on an S prefix whose every touch is
      // an S touch (g2n_dedup_keys' distinct keys) there are none: no launch, no host round trip
      if (!(sprefix && n_st == n_t)) insert(kModeFast, 2, cap >= full_cap ? cap : 4096, tid);
      fast = !c->h_ctl->dict_general && !c->h_ctl->table_overflow && c->h_ctl->deferred == 0;
      if (!fast) {
        tid = nullptr;
        sprefix = false;
        nid_in = nid;
        inv_in = inv;
        G2N_HIP(hipMemsetAsync(&c->ctl->table_overflow, 0, sizeof(unsigned long long), c->stream));
      }
    }
    if (!fast) {
      while (true) {
        init_table();
        const uint64_t max_probes = cap >= full_cap ? cap : 4096;
        bool overflow = false;
        for (uint32_t round = 1;; round++) {  // round 1: S touches; then every unresolved touch
          insert(round == 1 ? kModeClaim : kModeLookup, round, max_probes, nullptr);
          if (c->h_ctl->table_overflow) { overflow = true; break; }
          if (round > 1 && c->h_ctl->deferred == 0) break;
          if (round > 100000) throw Failure(G2N_E_DEVICE, "dictionary insert did not converge");
        }
        if (!overflow) break;
        if (cap >= full_cap) throw Failure(G2N_E_DEVICE, "node table overflow");
        G2N_HIP(hipMemsetAsync(&c->ctl->table_overflow, 0, sizeof(unsigned long long), c->stream));
        cap = full_cap;
      }
      G2N_HIP(hipMemsetAsync(first, 0, n_t, c->stream));
      hipLaunchKernelGGL(k_mark_first, dim3(grid_for(cap)), dim3(kTPB), 0, c->stream, table, cap, first);
      rank_firsts();
      hipLaunchKernelGGL(k_assign_ids, dim3(grid_for(cap)), dim3(kTPB), 0, c->stream, table, cap, nid, inv, klen);
      phase(c, "ids_general");
    }
  }
  sync_ctl(c);
  if (c->h_ctl->table_overflow) throw Failure(G2N_E_DEVICE, "node table overflow");
  DictOut D{};
  D.table = table;
  D.slot = slot;
  D.tid = tid;
  D.inv = inv_in;
  D.klen = klen;
  D.first = first;
  D.general = n_t && tid == nullptr;
  D.n_nodes = n_t ? c->h_ctl->n_nodes : 0;
  return D;
}

// Does the first S line (within the first 64 KiB) name segment "1"?  Chooses whether the parse
// tries the decimal-id dictionary; a wrong guess only costs a second parse.
static bool first_segment_is_one(g2n_context* c, const uint8_t* in, uint64_t len) {
  const size_t n = (size_t)std::min<uint64_t>(len, 1 << 16);
  if (n == 0) return false;
  std::vector<uint8_t> h(n);
  G2N_HIP(hipMemcpyAsync(h.data(), in, n, hipMemcpyDeviceToHost, c->stream));
  G2N_HIP(hipStreamSynchronize(c->stream));
  for (size_t p = 0; p + 3 < n;) {
    if (h[p] == 'S' && h[p + 1] == '\t') return h[p + 2] == '1' && (h[p + 3] == '\t' || h[p + 3] == '\n');
    const void* q = std::memchr(h.data() + p, '\n', n - p);
    if (!q) break;
    p = (size_t)((const uint8_t*)q - h.data()) + 1;
  }
  return true;  // no S line seen yet (long header lines): try
}

// Is the first S line's name (within the first 64 KiB) a constant prefix then "1" — minigraph's "s1"?
// The prefix (1-8 bytes, no digit, no tab) is then tried as the decimal-id layout's (ParseOpts::dpre:
// names P + str(k + 1) in S order); a wrong guess costs one tile-local pass, never the result.
static bool first_segment_prefixed(g2n_context* c, const uint8_t* in, uint64_t len, uint64_t* pre, uint32_t* pl) {
  const size_t n = (size_t)std::min<uint64_t>(len, 1 << 16);
  if (n == 0) return false;
  std::vector<uint8_t> h(n);
  G2N_HIP(hipMemcpyAsync(h.data(), in, n, hipMemcpyDeviceToHost, c->stream));
  G2N_HIP(hipStreamSynchronize(c->stream));
  for (size_t p = 0; p + 3 < n;) {
    if (h[p] == 'S' && h[p + 1] == '\t') {
      size_t e = p + 2;
      while (e < n && h[e] != '\t' && h[e] != '\n') e++;
      if (e >= n || e - (p + 2) < 2 || e - (p + 2) > 9 || h[e - 1] != '1') return false;
      uint64_t v = 0;
      for (size_t k = p + 2; k + 1 < e; k++) {
        if (h[k] - (uint32_t)'0' <= 9u) return false;
        v |= (uint64_t)h[k] << (8 * (k - p - 2));
      }
      *pre = v;
      *pl = (uint32_t)(e - 1 - (p + 2));
      return true;
    }
    const void* q = std::memchr(h.data() + p, '\n', n - p);
    if (!q) break;
    p = (size_t)((const uint8_t*)q - h.data()) + 1;
  }
  return false;
}

// The first S line's name (in the first 64 KiB) as the direct-address tier's premise: a prefix of
// at most 8 non-digit bytes, a run of at most 10 digits, a suffix of at most 8 bytes without a digit
// ("s123", "utg000123l", "node_42").  A run that starts with '0' fixes the width (zero-padded
// names: every name then has exactly that many digits); otherwise the run must be a canonical
// decimal.  False otherwise (the hash tiers decide); every other name is checked by the passes.
struct NamePattern {
  uint64_t pre = 0, suf = 0;
  uint32_t pre_len = 0, suf_len = 0, width = 0;
};
static bool first_segment_pattern(g2n_context* c, const uint8_t* in, uint64_t len, NamePattern* np) {
  const size_t n = (size_t)std::min<uint64_t>(len, 1 << 16);
  if (n == 0) return false;
  std::vector<uint8_t> h(n);
  G2N_HIP(hipMemcpyAsync(h.data(), in, n, hipMemcpyDeviceToHost, c->stream));
  G2N_HIP(hipStreamSynchronize(c->stream));
  auto digit = [&](size_t k) { return h[k] >= '0' && h[k] <= '9'; };
  for (size_t p = 0; p + 2 < n;) {
    if (h[p] == 'S' && h[p + 1] == '\t') {
      size_t e = p + 2;
      while (e < n && h[e] != '\t' && h[e] != '\n') e++;
      if (e == n) return false;
      size_t d = p + 2;
      while (d < e && !digit(d)) d++;
      size_t f = d;
      while (f < e && digit(f)) f++;
      const size_t pl = d - (p + 2), nd = f - d, sl = e - f;
      if (pl > 8 || sl > 8 || nd == 0 || nd > 10) return false;
      for (size_t k = f; k < e; k++)
        if (digit(k)) return false;
      NamePattern r;
      for (size_t k = 0; k < pl; k++) r.pre |= (uint64_t)h[p + 2 + k] << (8 * k);
      for (size_t k = 0; k < sl; k++) r.suf |= (uint64_t)h[f + k] << (8 * k);
      r.pre_len = (uint32_t)pl;
      r.suf_len = (uint32_t)sl;
      r.width = h[d] == '0' ? (uint32_t)nd : 0u;
      *np = r;
      return true;
    }
    const void* q = std::memchr(h.data() + p, '\n', n - p);
    if (!q) break;
    p = (size_t)((const uint8_t*)q - h.data()) + 1;
  }
  return false;
}

// The lean decimal-id parse in one pass over the input, without K1: every tile parses with
// tile-local positions, writes its COO to a slot of kTileEdgeCap edges and its own counts
// (k_tile_parse with ParseOpts.tile_pad); one scan of those counts gives the tile bases, a check
// confirms the premise across tiles (each tile's S names continue the S lines before it, no edge
// precedes an S line, every edge key names an S line), and the slots are compacted into the
// stream-order COO (S_ROWS / S_COLS, sized n_edges * ktrip as run_build will ask).  False when
// anything breaks the premise or needs the full parse (errors, warnings, deferred lines, a full
// slot): the caller then runs K1 and the classic parse, as if this had not run.
constexpr uint32_t kTileEdgeCap = (uint32_t)(kTile / 12) + 6;  // a lean edge line is at least 12 bytes (2736 for 32 KiB)

// grouped: the COO goes to group slots instead (k_tile_lean<true>, GroupedCoo) and is not compacted
// — for builds whose only consumer is the unweighted bucket partition.
// s_base / n_seg_all: a byte range of a sharded file with global decimal ids (options.range_s_base / range_n_segments):
// the S lines before the range and in the whole file; 0 / 0 for a whole file.
// xo (the extended instance, k_tile_lean kExt): bidirected keys and / or one integer weight tag —
// bidir / keep / has_wt / wt_len / wt_pack read from it; the per-edge weights go to S_EW in stream
// order beside the compacted COO (never group slots).
static bool tile_local_parse(g2n_context* c, const uint8_t* in, uint64_t len, uint64_t n_tiles, uint32_t ktrip,
                             TileCnt* tcnt, TileCnt* tbase, TileCnt* tot_out, bool grouped, uint64_t s_base = 0,
                             uint64_t n_seg_all = 0, bool deferred = false, const ParseOpts* xo = nullptr,
                             bool warn_ok = false, uint64_t dpre = 0, uint32_t dpre_len = 0) {
  // an extended build takes group slots when its only reader is the bucket partition: unweighted, or
  // a weighted SUM CSR whose codes the parse writes (xo->wenc set by the caller as a flag)
  if (xo && xo->has_wt && !xo->wenc) grouped = false;
#if G2N_K2_OLD
  grouped = false;  // k_tile_parse<true> writes per-tile slots only
#endif
  // 32 tiles per group slot; a small input takes fewer, so that the partition's first pass (one block
  // per group) still has about G2N_MIN_GROUPS blocks (C2's 3.7K tiles: 115 groups of 32 left most CUs idle)
  uint32_t gshift = kGroupShift;
  while (gshift > 0 && (n_tiles >> gshift) < (uint64_t)G2N_MIN_GROUPS) gshift--;
  const uint64_t n_groups = (n_tiles + (1u << gshift) - 1) >> gshift;
  const uint64_t gcap = ((uint64_t)kTileEdgeCap << gshift) * ktrip;  // entries per group slot
  const uint64_t slots = grouped ? n_groups * gcap : n_tiles * kTileEdgeCap * ktrip;
  auto* rows_p = dget<int32_t>(c, S_ROWSP, slots);
  auto* cols_p = dget<int32_t>(c, S_COLSP, slots);
  uint32_t* gcount = nullptr;
  if (grouped) {
    gcount = dget<uint32_t>(c, S_GCNT, n_groups);
    G2N_HIP(hipMemsetAsync(gcount, 0, n_groups * sizeof(uint32_t), c->stream));
  }
  auto* tlean = dget<TileLean>(c, S_TLEAN, n_tiles);
  ParseOpts lo{};
  lo.rows = rows_p;
  lo.cols = cols_p;
  lo.ktrip = ktrip;
  lo.tile_pad = kTileEdgeCap;
  lo.tid = (uint32_t*)rows_p;  // only a flag here: the lean parse writes no per-touch ids
  lo.n_seg = 0x7FFFFFFFull;    // the file's S count is known afterwards (k_tile_lean_check)
  lo.dpre = dpre;              // names behind one constant prefix (first_segment_prefixed)
  lo.dpre_len = dpre_len;
  lo.gshift = gshift;
  lo.pf_dist = G2N_K2_PREFETCH ? (uint32_t)c->lean_blocks : 0u;
  // a whole-file build takes the unsupported-record warning itself (k_tile_lean_check); a sharded range
  // leaves it to the general protocol
  uint32_t* tunk = warn_ok ? dget<uint32_t>(c, S_TUNK, n_tiles) : nullptr;
  lo.tunk = tunk;
  double* ew_p = nullptr;
  if (xo) {
    lo.bidir = xo->bidir;
    lo.keep = xo->keep;
    lo.has_wt = xo->has_wt;
    lo.wt_len = xo->wt_len;
    lo.wt_pack = xo->wt_pack;
    if (xo->has_wt && grouped) {
      lo.wenc = dget<uint32_t>(c, S_WENCP, slots);
      lo.wf32 = xo->wf32;
    } else if (xo->has_wt) {
      lo.ew = ew_p = dget<double>(c, S_EWP, n_tiles * kTileEdgeCap);
    }
  }
#ifdef G2N_K2_STAMPS
  unsigned long long* stamps = dget<unsigned long long>(c, S_TEMP, n_tiles * kK2Stamps);
  G2N_HIP(hipMemsetAsync(stamps, 0, n_tiles * kK2Stamps * 8, c->stream));
  G2N_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g2n_k2_stamps), &stamps, sizeof(stamps), 0, hipMemcpyHostToDevice,
                                 c->stream));
#endif
#if G2N_K2_OLD  // experiment builds: the k_tile_parse<true> instance
  hipLaunchKernelGGL(k_tile_parse<true>, dim3((unsigned)n_tiles), dim3(kTPB), 0, c->stream, in, len, (const TileCnt*)nullptr,
                     1u, 2u, lo, (uint64_t*)nullptr, (uint8_t*)nullptr, TouchOut{}, EdgeOut{}, c->ctl,
                     (uint64_t*)nullptr, (DeferredLine*)nullptr, n_tiles, tcnt, tlean);
#else
#if G2N_K2_PERSIST
  // persistent: as many blocks as fit on the device at once, each prefetching its next tile
  const unsigned grid = (unsigned)std::min<uint64_t>(n_tiles, (uint64_t)c->lean_blocks);
  if (grouped)
    hipLaunchKernelGGL((k_tile_lean_p<true>), dim3(grid), dim3(kLeanTPB), 0, c->stream, in, len, lo, c->ctl, tcnt,
                       tlean, gcount, gcap, n_tiles);
  else
    hipLaunchKernelGGL((k_tile_lean_p<false>), dim3(grid), dim3(kLeanTPB), 0, c->stream, in, len, lo, c->ctl, tcnt,
                       tlean, (uint32_t*)nullptr, (uint64_t)0, n_tiles);
#else
  if (xo && grouped)
    hipLaunchKernelGGL((k_tile_lean<kLeanDecimal, true, true>), dim3((unsigned)n_tiles), dim3(kLeanTPB), 0,
                       c->stream, in, len, lo, c->ctl, tcnt, tlean, gcount, gcap, HashLeanArgs{});
  else if (xo)
    hipLaunchKernelGGL((k_tile_lean<kLeanDecimal, false, true>), dim3((unsigned)n_tiles), dim3(kLeanTPB), 0,
                       c->stream, in, len, lo, c->ctl, tcnt, tlean, (uint32_t*)nullptr, (uint64_t)0, HashLeanArgs{});
  else if (grouped)
    hipLaunchKernelGGL((k_tile_lean<kLeanDecimal, true>), dim3((unsigned)n_tiles), dim3(kLeanTPB), 0, c->stream, in,
                       len, lo, c->ctl, tcnt, tlean, gcount, gcap, HashLeanArgs{});
  else
    hipLaunchKernelGGL((k_tile_lean<kLeanDecimal, false>), dim3((unsigned)n_tiles), dim3(kLeanTPB), 0, c->stream, in,
                       len, lo, c->ctl, tcnt, tlean, (uint32_t*)nullptr, (uint64_t)0, HashLeanArgs{});
#endif
#endif
  phase(c, "parse");
#ifdef G2N_K2_STAMPS
  if (const char* out = std::getenv("G2N_K2_STAMPS_OUT")) {  // diagnostics build only
    std::vector<unsigned long long> h(n_tiles * kK2Stamps);
    G2N_HIP(hipMemcpyAsync(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost, c->stream));
    G2N_HIP(hipStreamSynchronize(c->stream));
    if (FILE* f = std::fopen(out, "wb")) {
      std::fwrite(h.data(), 8, h.size(), f);
      std::fclose(f);
    }
  }
#endif
  // the tile scan, the warning's line and the premise check run unconditionally behind the parse
  // (on a failed parse their results are dropped), so the host waits once for all of them
  {
    const uint64_t n_parts = (n_tiles + kStructChunk - 1) / kStructChunk;
    auto* part = dget<TileCnt>(c, S_TEMP, n_parts + 1);
    hipLaunchKernelGGL(k_struct_reduce<TileCnt>, dim3((unsigned)n_parts), dim3(256), 0, c->stream,
                       (const TileCnt*)tcnt, n_tiles, part);
    hipLaunchKernelGGL(k_struct_scan_parts<TileCnt>, dim3(1), dim3(256), 0, c->stream, part, n_parts, part + n_parts);
    hipLaunchKernelGGL(k_struct_scan_chunks<TileCnt>, dim3((unsigned)n_parts), dim3(256), 0, c->stream,
                       (const TileCnt*)tcnt, n_tiles, (const TileCnt*)part, tbase);
    if (deferred)  // the range's offset evidence, checked by the caller across ranges
      hipLaunchKernelGGL(k_tile_lean_evidence, dim3(grid_for(n_tiles)), dim3(kTPB), 0, c->stream,
                         (const TileCnt*)tcnt, (const TileCnt*)tbase, (const TileLean*)tlean, n_tiles, c->ctl);
    else  // (the file's S count: n_seg_all, or the total the scan just wrote)
      hipLaunchKernelGGL(k_tile_lean_check, dim3(grid_for(n_tiles)), dim3(kTPB), 0, c->stream, (const TileCnt*)tcnt,
                         (const TileCnt*)tbase, (const TileLean*)tlean, n_tiles, n_seg_all,
                         (const TileCnt*)(part + n_parts), s_base, (const uint32_t*)tunk, c->ctl);
    TileCnt tot;
    G2N_HIP(hipMemcpyAsync(&tot, part + n_parts, sizeof(TileCnt), hipMemcpyDeviceToHost, c->stream));
    sync_ctl(c);
    bool ok = !c->h_ctl->int_fail && c->h_ctl->err_key == ~0ull && tot.touches < 0xFFFFFFFFull &&
              tot.edges * ktrip < 0xFFFFFFFFull;
    if (deferred) {
      const Ctl& h = *c->h_ctl;
      ok = ok && (h.ev_dmin == ~0ull || h.ev_dmin == h.ev_dmax);
      c->range_has_s = h.ev_dmin != ~0ull;
      c->range_d = c->range_has_s ? (int64_t)(h.ev_dmin - (1ull << 62)) : -1;
      c->range_vmax = h.ev_vmax;
      c->range_nseg = tot.segs;
    }
    if (ok && grouped) {
      c->gcoo.active = true;
      c->gcoo.rows = rows_p;
      c->gcoo.cols = cols_p;
      c->gcoo.gcount = gcount;
      c->gcoo.gcap = gcap;
      c->gcoo.n_groups = n_groups;
      c->gcoo.wenc = lo.wenc;
      *tot_out = tot;
      return true;
    }
    if (ok) {
      const uint64_t n_trip = tot.edges * ktrip;
      auto* rows = dget<int32_t>(c, S_ROWS, n_trip);
      auto* cols = dget<int32_t>(c, S_COLS, n_trip);
      double* ew = ew_p ? dget<double>(c, S_EW, tot.edges) : nullptr;  // E.w: k_values reads the weights there
      hipLaunchKernelGGL(k_tile_compact, dim3((unsigned)n_tiles), dim3(kTPB), 0, c->stream, (const int32_t*)rows_p,
                         (const int32_t*)cols_p, kTileEdgeCap, ktrip, (const TileCnt*)tcnt, (const TileCnt*)tbase,
                         rows, cols, (const double*)ew_p, ew);
      phase(c, "place");
      *tot_out = tot;
      return true;
    }
  }
  reset_ctl(c);  // the classic path starts from a clean slate
  return false;
}

// the edge passes' extended fields (bidirected keys / one integer weight tag) from X
static void lean_ext_args(HashLeanArgs& H, const HashLeanArgs& X) {
  H.bidir = X.bidir;
  H.has_wt = X.has_wt;
  H.wt_len = X.wt_len;
  H.wt_pack = X.wt_pack;
  H.ew = X.ew;
}

// the lean hash / direct passes' tiles (k_tile_lists): claim = tiles with S or P / O lines, edge = with edge lines
struct TileLists {
  const uint32_t* claim = nullptr;
  uint64_t n_claim = 0;
  const uint32_t* edge = nullptr;
  uint64_t n_edge = 0;
};

// The S-first hash dictionary on the lean front end (k_tile_lean kLeanClaim / kLeanEdges, after K1):
// S names claimed with node id = S index, then every edge line's names found straight from its
// staged tile and the stream-order COO written.  False (and a clean slate) when the input is not
// S-first with unique names in the lean shapes: the classic parse + dictionary tiers run instead.
static bool hash_lean_build(g2n_context* c, const uint8_t* in, uint64_t len, const TileLists& TL, const TileCnt* tcnt,
                            const TileCnt* tbase, uint64_t n_s, uint32_t ktrip, int32_t* rows, int32_t* cols,
                            const HashLeanArgs& X, uint64_t** noff_out, uint32_t** nlen_out, uint64_t* names_len) {
#ifdef G2N_K2_STAMPS
  const uint64_t n_tiles = (len + kTile - 1) / kTile;  // (the stamps buffer)
#endif
  if (n_s == 0 || n_s >= 0x7FFFFFFFull) return false;
  uint64_t cap = 1024;
#ifndef G2N_HL_LOAD_PCT  // experiment builds: the lean table's maximum load, percent
#define G2N_HL_LOAD_PCT 67
#endif
  while (cap * G2N_HL_LOAD_PCT < n_s * 100) cap <<= 1;  // load <= 2/3: probe sequences stay short
#ifdef G2N_HL_CAP_SHIFT  // experiment builds: table footprint vs probe cost
  cap <<= G2N_HL_CAP_SHIFT;
#endif
  auto* table = dget<DictEntry>(c, S_TABLE, cap);
  G2N_HIP(hipMemsetAsync(table, 0xFF, cap * sizeof(DictEntry), c->stream));
  auto* noff = dget<uint64_t>(c, S_NOFF, n_s);
  auto* nlen = dget<uint32_t>(c, S_NLEN, n_s);
  HashLeanArgs H{tbase, tcnt, table, cap - 1, cap, noff, nlen, rows, cols, ktrip};
  lean_ext_args(H, X);
  phase(c, "table_init");
#ifdef G2N_K2_STAMPS  // every k_tile_lean launch stamps: the buffer must be this build's
  unsigned long long* stamps = dget<unsigned long long>(c, S_TEMP, n_tiles * kK2Stamps);
  G2N_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g2n_k2_stamps), &stamps, sizeof(stamps), 0, hipMemcpyHostToDevice,
                                 c->stream));
#endif
  H.tlist = TL.claim;
  H.tnb = dget<unsigned long long>(c, S_TNB, TL.n_claim);
  hipLaunchKernelGGL((k_tile_lean<kLeanClaim, false>), dim3((unsigned)TL.n_claim), dim3(kLeanTPB), 0, c->stream, in, len,
                     ParseOpts{}, c->ctl, (TileCnt*)nullptr, (TileLean*)nullptr, (uint32_t*)nullptr, (uint64_t)0, H);
  hipLaunchKernelGGL(k_claim_totals, dim3(1), dim3(1024), 0, c->stream, (const unsigned long long*)H.tnb, TL.n_claim,
                     &c->ctl->names_len, &c->ctl->dir_vmax);
  phase(c, "insert_claim");
  sync_ctl(c);
  if (c->h_ctl->int_fail) {
    reset_ctl(c);
    return false;
  }
  *names_len = c->h_ctl->names_len;  // the claimed names' bytes: the names blob needs no later sync
#ifdef G2N_K2_STAMPS
  G2N_HIP(hipMemsetAsync(stamps, 0, n_tiles * kK2Stamps * 8, c->stream));  // the claim pass stamped too
#endif
  H.tlist = TL.edge;
  if (!TL.n_edge) {
  } else if (H.bidir || H.has_wt)
    hipLaunchKernelGGL((k_tile_lean<kLeanEdges, false, true>), dim3((unsigned)TL.n_edge), dim3(kLeanTPB), 0, c->stream, in,
                       len, ParseOpts{}, c->ctl, (TileCnt*)nullptr, (TileLean*)nullptr, (uint32_t*)nullptr, (uint64_t)0, H);
  else
    hipLaunchKernelGGL((k_tile_lean<kLeanEdges, false>), dim3((unsigned)TL.n_edge), dim3(kLeanTPB), 0, c->stream, in, len,
                       ParseOpts{}, c->ctl, (TileCnt*)nullptr, (TileLean*)nullptr, (uint32_t*)nullptr, (uint64_t)0, H);
  phase(c, "insert_lookup");
#ifdef G2N_K2_STAMPS
  if (const char* out = std::getenv("G2N_HL_STAMPS_OUT")) {  // diagnostics build only: the edge pass
    std::vector<unsigned long long> h(n_tiles * kK2Stamps);
    G2N_HIP(hipMemcpyAsync(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost, c->stream));
    G2N_HIP(hipStreamSynchronize(c->stream));
    if (FILE* f = std::fopen(out, "wb")) {
      std::fwrite(h.data(), 8, h.size(), f);
      std::fclose(f);
    }
  }
#endif
  sync_ctl(c);
  if (c->h_ctl->int_fail) {
    reset_ctl(c);
    return false;
  }
  *noff_out = noff;
  *nlen_out = nlen;
  return true;
}

// The direct-address tier on the lean front end (k_tile_lean kLeanDirClaim / kLeanDirEdges, after K1):
// S names that are one prefix + a canonical decimal v < cap claim direct[v] = S index, then every edge
// line's names are found with one 4-byte read each and the stream-order COO written.  cap = 4 x the S
// lines (at least 64 Ki, at most 2^28 values: 1 GiB): ids "1".."N" out of order, or with gaps, fit.
// False (and a clean slate) when any name breaks the shape, a value repeats or passes cap, or the
// input is not S-first: the lean hash tier runs next.
static bool direct_lean_build(g2n_context* c, const uint8_t* in, uint64_t len, const TileLists& TL, const TileCnt* tcnt,
                              const TileCnt* tbase, uint64_t n_s, uint32_t ktrip, int32_t* rows, int32_t* cols,
                              const NamePattern& np, const HashLeanArgs& X, uint64_t** noff_out, uint32_t** nlen_out,
                              uint64_t* names_len) {
#ifdef G2N_K2_STAMPS
  const uint64_t n_tiles = (len + kTile - 1) / kTile;  // (the stamps buffer)
#endif
  if (n_s == 0 || n_s >= 0x7FFFFFFFull) return false;
  const uint64_t cap = std::min<uint64_t>(1ull << 28, std::max<uint64_t>(4 * n_s, 1ull << 16));
  auto* direct = dget<uint32_t>(c, S_DIRECT, cap);
  G2N_HIP(hipMemsetAsync(direct, 0xFF, cap * sizeof(uint32_t), c->stream));
  auto* noff = dget<uint64_t>(c, S_NOFF, n_s);
  auto* nlen = dget<uint32_t>(c, S_NLEN, n_s);
  HashLeanArgs H{tbase, tcnt, nullptr, 0, 0, noff, nlen, rows, cols, ktrip};
  H.direct = direct;
  H.direct_cap = cap;
  H.pre = np.pre;
  H.pre_len = np.pre_len;
  H.suf = np.suf;
  H.suf_len = np.suf_len;
  H.width = np.width;
  lean_ext_args(H, X);
  phase(c, "table_init");
#ifdef G2N_K2_STAMPS  // every k_tile_lean launch stamps: the buffer must be this build's
  unsigned long long* stamps = dget<unsigned long long>(c, S_TEMP, n_tiles * kK2Stamps);
  G2N_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g2n_k2_stamps), &stamps, sizeof(stamps), 0, hipMemcpyHostToDevice,
                                 c->stream));
#endif
  H.tlist = TL.claim;
  H.tnb = dget<unsigned long long>(c, S_TNB, TL.n_claim);
  hipLaunchKernelGGL((k_tile_lean<kLeanDirClaim, false>), dim3((unsigned)TL.n_claim), dim3(kLeanTPB), 0, c->stream, in,
                     len, ParseOpts{}, c->ctl, (TileCnt*)nullptr, (TileLean*)nullptr, (uint32_t*)nullptr, (uint64_t)0, H);
  hipLaunchKernelGGL(k_claim_totals, dim3(1), dim3(1024), 0, c->stream, (const unsigned long long*)H.tnb, TL.n_claim,
                     &c->ctl->names_len, &c->ctl->dir_vmax);
#if G2N_DIRECT_STORE  // (cap is a multiple of 4; the count stops past the largest claimed value)
  G2N_HIP(hipMemsetAsync(&c->ctl->n_keep, 0, sizeof(unsigned long long), c->stream));
  hipLaunchKernelGGL(k_direct_filled, dim3((unsigned)std::min<uint64_t>(grid_for(cap / 4, 256), 2048)), dim3(256), 0,
                     c->stream, (const uint4*)direct, cap / 4, (const unsigned long long*)&c->ctl->dir_vmax,
                     &c->ctl->n_keep);
#endif
  phase(c, "direct_claim");
  sync_ctl(c);
  if (c->h_ctl->int_fail || (G2N_DIRECT_STORE && c->h_ctl->n_keep != n_s)) {  // (a repeated value: fewer filled)
    reset_ctl(c);
    return false;
  }
  *names_len = c->h_ctl->names_len;
  H.tlist = TL.edge;
  if (!TL.n_edge) {
  } else if (H.bidir || H.has_wt)
    hipLaunchKernelGGL((k_tile_lean<kLeanDirEdges, false, true>), dim3((unsigned)TL.n_edge), dim3(kLeanTPB), 0, c->stream,
                       in, len, ParseOpts{}, c->ctl, (TileCnt*)nullptr, (TileLean*)nullptr, (uint32_t*)nullptr,
                       (uint64_t)0, H);
  else
    hipLaunchKernelGGL((k_tile_lean<kLeanDirEdges, false>), dim3((unsigned)TL.n_edge), dim3(kLeanTPB), 0, c->stream, in,
                       len, ParseOpts{}, c->ctl, (TileCnt*)nullptr, (TileLean*)nullptr, (uint32_t*)nullptr, (uint64_t)0, H);
  phase(c, "direct_lookup");
  sync_ctl(c);
  if (c->h_ctl->int_fail) {
    reset_ctl(c);
    return false;
  }
  *noff_out = noff;
  *nlen_out = nlen;
  return true;
}

static int run_build(g2n_context* c, const uint8_t* in, uint64_t len, const g2n_options* o, g2n_result* R) {
  fill_defaults(R);
  clear_call_state(c);
  c->test_flags = o->test_flags;
  R->input_bytes = len;
  c->n_ev = 0;
  G2N_HIP(hipEventRecord(c->ev[0], c->stream));
  reset_ctl(c);
  const bool bidir = o->bidirected != 0, keep = o->keep_directed_bidir != 0;
  const bool gd = keep || (!bidir && o->directed != 0);  // builders.py:143
  const bool maxsym = gd && !o->asymmetric;              // builders.py:282
  const uint32_t tps = bidir ? 2 : 1;
  const uint32_t tpe = (bidir && !keep) ? 4 : 2;
  const int dt = o->dtype;
  R->dtype = dt;
  R->index_width = 4;

  const uint64_t n_tiles = (len + kTile - 1) / kTile;
  auto* tcnt = dget<TileCnt>(c, S_TILE_CNT, n_tiles + 1);
  auto* tbase = dget<TileCnt>(c, S_TILE_BASE, n_tiles + 1);
  TileCnt tot{};
  const bool shard_dec = (o->range_flags & G2N_RANGE_DECIMAL) != 0;
  // g2n_build_decimal_range: the S lines before the range are not known yet — the one-pass parse
  // reports the range's offset evidence instead of checking it (the caller checks across ranges)
  const bool shard_deferred = shard_dec && (o->range_flags & G2N_RANGE_EVIDENCE) != 0;
  c->range_has_s = false;
  c->range_d = -1;
  c->range_vmax = 0;
  c->range_nseg = 0;
  const bool first_one =
      !shard_dec && !(c->test_flags & (kTestDictHash | kTestDictGeneral | kTestDictDirect)) &&
      first_segment_is_one(c, in, len);
  // ... or "P1": the same layout behind a constant prefix P (tile-local pass only: a failed one goes to
  // the direct / hash tiers, which take any prefix)
  uint64_t dpre = 0;
  uint32_t dpre_len = 0;
  const bool first_pre = !first_one && !shard_dec && !(c->test_flags & (kTestDictHash | kTestDictGeneral |
                                                                        kTestDictDirect | kTestNoDecPrefix)) &&
                         first_segment_prefixed(c, in, len, &dpre, &dpre_len);
  // ---- the decimal-id lean parse without K1 (tile-local positions, checked and compacted after)
  // group slots when the COO's only reader is the unweighted bucket partition (a CSR output)
  const bool coo_wanted = (o->output == G2N_OUT_PARSE && !maxsym) || o->output == G2N_OUT_COO;
  // ... or a sharded decimal range whose caller takes the COO as group slots (G2N_RANGE_SLOTS: unweighted,
  // coordinates only — its route or slice CSR needs no stream order)
  const bool slots_out = shard_dec && (o->range_flags & G2N_RANGE_SLOTS) && !(o->weight_tag && *o->weight_tag) && !bidir &&
                         (o->range_flags & G2N_RANGE_NO_VALUES);
  const bool grouped = !G2N_NO_GROUP_DEFAULT && (!coo_wanted || slots_out) && !c->no_group &&
                       !(c->test_flags & (kTestNoBuckets | kTestNoGroup));
  // bidirected keys / one integer weight tag: the extended tile-local instance (whole files only)
  const size_t wt_bytes = o->weight_tag ? std::strlen(o->weight_tag) : 0;
  ParseOpts xo{};
  xo.bidir = bidir;
  xo.keep = keep;
  xo.has_wt = wt_bytes > 0;
  xo.wt_len = (uint32_t)wt_bytes;
  for (size_t k = 0; k < wt_bytes && k < 8; k++) xo.wt_pack |= (uint64_t)(uint8_t)o->weight_tag[k] << (8 * k);
  const bool ext = bidir || wt_bytes > 0;
  // a weighted SUM CSR in dtypes whose cast of a canonical <= 9-digit integer can neither fail nor lose
  // the integer's exact-int32 code (float32: the code of the rounded value) takes group slots: the parse
  // writes the codes, so neither k_tile_compact nor k_values runs (C3); a bucket partition that declines
  // (an overfull bucket, an inexact float sum) redoes the build without groups
  if (wt_bytes && grouped && !maxsym && o->output == G2N_OUT_CSR &&
      (dt == G2N_FLOAT64 || dt == G2N_FLOAT32 || dt == G2N_INT32)) {
    xo.wenc = reinterpret_cast<uint32_t*>(uintptr_t{1});  // (a flag here: tile_local_parse allocates them)
    xo.wf32 = dt == G2N_FLOAT32 ? 1u : 0u;
  }
  const bool ext_ok = !shard_dec && wt_bytes <= 8 && !(c->test_flags & kTestNoExtLean);
  // (a sharded range with global decimal ids takes it too — with or without S lines of its own)
  const bool local_done =
      n_tiles && (first_one || first_pre ||
                  (shard_dec && (shard_deferred || (o->range_s_base >= 0 && o->range_n_segments > 0)))) &&
      (!ext || ext_ok) && !o->strip_orientation && !(c->test_flags & (kTestNoLean | kTestNoTileLocal)) &&
      tile_local_parse(c, in, len, n_tiles, tpe == 4 ? 4u : (gd ? 1u : 2u), tcnt, tbase, &tot, grouped,
                       shard_dec ? (uint64_t)o->range_s_base : 0, shard_dec ? (uint64_t)o->range_n_segments : 0,
                       shard_deferred, ext ? &xo : nullptr, !shard_dec, dpre, first_pre ? dpre_len : 0u);
  const uint32_t name_pre_len = local_done && first_pre ? dpre_len : 0u;  // node k's name: P + str(k + 1)
  if (shard_deferred && n_tiles && !local_done)  // the caller counts the ranges and builds with K1 instead
    throw Failure(G2N_E_UNSUPPORTED, "sharded decimal-id range: the one-pass parse declined");
  // ---- K1: per-tile counts -> tile bases (and the lean hash / direct passes' tile lists: names that
  // are not the decimal ids)
  TileLists TL;
  const bool lists_wanted = !first_one && !shard_dec;
  if (n_tiles && !local_done) {
    if (G2N_K1_REG)
      hipLaunchKernelGGL(k_tile_count_r, dim3((unsigned)n_tiles), dim3(kK1TPB), 0, c->stream, in, len, tps, tpe, tcnt);
    else
      hipLaunchKernelGGL(k_tile_count, dim3((unsigned)n_tiles), dim3(kTPB), 0, c->stream, in, len, tps, tpe, tcnt);
    const uint64_t n_parts = (n_tiles + kStructChunk - 1) / kStructChunk;
    auto* part = dget<TileCnt>(c, S_TEMP, n_parts + 1);  // chunk sums, then the total
    hipLaunchKernelGGL(k_struct_reduce<TileCnt>, dim3((unsigned)n_parts), dim3(256), 0, c->stream,
                       (const TileCnt*)tcnt, n_tiles, part);
    hipLaunchKernelGGL(k_struct_scan_parts<TileCnt>, dim3(1), dim3(256), 0, c->stream, part, n_parts, part + n_parts);
    hipLaunchKernelGGL(k_struct_scan_chunks<TileCnt>, dim3((unsigned)n_parts), dim3(256), 0, c->stream,
                       (const TileCnt*)tcnt, n_tiles, (const TileCnt*)part, tbase);
    if (lists_wanted) {  // (read with the total: no second wait)
      auto* lists = dget<uint32_t>(c, S_TLIST, 2 + 2 * n_tiles);
      G2N_HIP(hipMemsetAsync(lists, 0, 2 * sizeof(uint32_t), c->stream));
      hipLaunchKernelGGL(k_tile_lists, dim3(grid_for(n_tiles)), dim3(kTPB), 0, c->stream, (const TileCnt*)tcnt, n_tiles,
                         lists);
      uint32_t n2[2];
      G2N_HIP(hipMemcpyAsync(n2, lists, sizeof(n2), hipMemcpyDeviceToHost, c->stream));
      tot = read_dev(c, part + n_parts);
      TL = TileLists{lists + 2, n2[0], lists + 2 + n_tiles, n2[1]};
    } else {
      tot = read_dev(c, part + n_parts);
    }
  }
  const uint64_t n_lines = tot.lines;
  const uint64_t n_e = tot.edges, n_s = tot.segs;
  const uint64_t n_t = n_s * tps + n_e * tpe;
  R->n_lines = (int64_t)n_lines;
  R->n_edges = (int64_t)n_e;
  R->n_records = (int64_t)tot.recs;
  if (n_t >= 0xFFFFFFFFull || n_e >= 0xFFFFFFFFull)
    throw Failure(G2N_E_UNSUPPORTED, "more than 2^32-1 node touches in one build");
  if (!local_done) phase(c, "tiles");

  // ---- K2: parse every line from its tile's LDS window
  // A tile-local build (local_done) is parsed already: none of the full parse's per-line / per-touch /
  // per-edge buffers is read, so none is allocated (C5-size inputs: ~100 GB of HBM).  z(n): a buffer
  // size that is 1 for such a build.
  auto z = [&](uint64_t n) -> uint64_t { return local_done ? 1 : n; };
  auto* ls = dget<uint64_t>(c, S_LS, z(n_lines + 1));
  auto* kind = dget<uint8_t>(c, S_KIND, z(n_lines));
  ParseOpts op{};
  op.bidir = bidir;
  op.keep = keep;
  op.strip = o->strip_orientation != 0;
  const size_t wtl = o->weight_tag ? std::strlen(o->weight_tag) : 0;
  op.has_wt = wtl > 0;
  op.wt_len = (uint32_t)wtl;
  if (wtl && !local_done) {  // (the full parse's copy; a tile-local build compared the tag in place: a pageable
    auto* wt = dget<uint8_t>(c, S_WT, wtl);  // H2D copy is a host wait)
    G2N_HIP(hipMemcpyAsync(wt, o->weight_tag, wtl, hipMemcpyHostToDevice, c->stream));
    op.wt = wt;
  }
  TouchOut T{dget<uint64_t>(c, S_NOFF, z(n_t)), dget<uint32_t>(c, S_NLEN, z(n_t)),
             bidir ? dget<uint64_t>(c, S_OOFF, z(n_t)) : nullptr, bidir ? dget<uint32_t>(c, S_OLEN, z(n_t)) : nullptr,
             dget<uint8_t>(c, S_TKIND, z(n_t))};
  // (E.w is read by k_values only for weights: a tile-local build holds them there when it has a tag)
  // (a grouped weighted build wrote exact-int32 codes instead: no per-edge weights at all)
  const bool codes_done = local_done && c->gcoo.active && c->gcoo.wenc;
  EdgeOut E{dget<double>(c, S_EW, local_done && (!wt_bytes || codes_done) ? 1 : n_e), dget<uint32_t>(c, S_ETB, z(n_e))};
  const int ktrip = tpe == 4 ? 4 : (gd ? 1 : 2);
  const uint64_t n_trip = n_e * (uint64_t)ktrip;
  // the stream-order COO holds int32 node ids (< 2^31 - 1, checked below) at 64-bit positions; the
  // partition counts its elements in 32 bits (more than 2^31 - 1 entries: int64 CSR indices, F2)
  if (n_trip >= 0xFFFFFFFFull) throw Failure(G2N_E_UNSUPPORTED, "more than 2^32-1 matrix entries");
  // the group slots hold a grouped tile-local build's COO (GroupedCoo): rows / cols only for a rebuild
  const bool in_groups = local_done && c->gcoo.active;
  auto* rows = dget<int32_t>(c, S_ROWS, in_groups ? 1 : n_trip);
  auto* cols = dget<int32_t>(c, S_COLS, in_groups ? 1 : n_trip);
  // decimal-id dictionary, computed by the parse itself (lean: straight into rows / cols) when
  // the first S line names "1" (a cheap guess: a wrong one costs one extra parse)
  // options.range_flags G2N_RANGE_DECIMAL: one byte range of a sharded build whose node ids are decimal and
  // GLOBAL: range_s_base S lines precede the range, range_n_segments S lines in the whole file (the
  // caller checked across ranges that no edge line precedes an S line).  Lean parse or nothing.
  if (shard_dec && (o->output != G2N_OUT_COO || o->want_node_names || o->range_s_base < 0 || o->range_n_segments < 0))
    throw Failure(G2N_E_ARG, "sharded decimal-id build: output COO without names, s_base / n_seg >= 0");
  const bool int_ids = n_t && (shard_dec || first_one);
  const bool lean = int_ids && (shard_dec || !(c->test_flags & kTestNoLean));
  if (int_ids) {
    op.tid = dget<uint32_t>(c, S_TID, z(n_t));
    op.n_seg = shard_dec ? (uint64_t)o->range_n_segments : n_s;
    op.s_base = shard_dec ? (uint64_t)o->range_s_base : 0;
  }
  auto* wl = dget<uint64_t>(c, S_WL, z(2 * n_e));
  auto* deferred = dget<DeferredLine>(c, S_DEFER, n_tiles + 1);
  if (!local_done) G2N_HIP(hipMemcpyAsync(ls + n_lines, &len, sizeof(uint64_t), hipMemcpyHostToDevice, c->stream));
  phase(c, "_prep");
  auto parse = [&](const ParseOpts& po) {
    if (n_tiles)
      hipLaunchKernelGGL(k_tile_parse<false>, dim3((unsigned)n_tiles), dim3(kTPB), 0, c->stream, in, len, tbase, tps, tpe,
                         po, ls, kind, T, E, c->ctl, wl, deferred, n_tiles, (TileCnt*)nullptr, (TileLean*)nullptr);
    sync_ctl(c);
    const uint64_t n_def = c->h_ctl->n_deferred;
    if (n_def > n_tiles) throw Failure(G2N_E_DEVICE, "internal: more deferred lines than tiles");
    if (n_def)
      hipLaunchKernelGGL(k_parse_deferred, dim3(grid_for(n_def, 64)), dim3(64), 0, c->stream, in, len, ls, kind,
                         deferred, n_def, po, T, E, c->ctl, wl);
    phase(c, "parse");
    sync_ctl(c);
  };
  // names that are not the decimal ids: the S-first hash dictionary on the lean front end first
  uint64_t* hl_noff = nullptr;
  uint32_t* hl_nlen = nullptr;
  uint64_t hl_names_len = 0;
  // (bidirected keys and / or one integer weight tag: the edge passes' extended instance)
  const bool lean_hash_ok = n_tiles && !local_done && !int_ids && (!op.has_wt || wtl <= 8) && !op.strip &&
                            !shard_dec && !(c->test_flags & (kTestDictGeneral | kTestNoHashLean)) && n_s && TL.claim;
  HashLeanArgs X{};
  X.bidir = bidir ? 1 : 0;
  X.has_wt = op.has_wt;
  X.wt_len = (uint32_t)wtl;
  X.wt_pack = xo.wt_pack;
  X.ew = E.w;
  // decimal names out of S order (or behind one prefix): the direct-address tier first
  NamePattern np;
  const bool direct_done = lean_hash_ok && !(c->test_flags & (kTestDictHash | kTestNoDirect)) &&
                           first_segment_pattern(c, in, len, &np) &&
                           direct_lean_build(c, in, len, TL, tcnt, tbase, n_s, (uint32_t)ktrip, rows, cols, np,
                                             X, &hl_noff, &hl_nlen, &hl_names_len);
  const bool hash_done = direct_done || (lean_hash_ok && hash_lean_build(c, in, len, TL, tcnt, tbase, n_s,
                                                                          (uint32_t)ktrip, rows, cols, X, &hl_noff,
                                                                          &hl_nlen, &hl_names_len));
  bool lean_done = local_done || hash_done;  // rows / cols hold the stream-order COO already
  if (lean && !local_done) {
    ParseOpts lo = op;
    lo.rows = rows;
    lo.cols = cols;
    lo.ktrip = (uint32_t)ktrip;
    parse(lo);
    // the lean parse wrote no line starts / kinds: errors, the unsupported-record warning and
    // slow weights need a full parse (decimal ids kept unless they failed)
    lean_done = !c->h_ctl->int_fail && c->h_ctl->err_key == ~0ull && c->h_ctl->warn_line == ~0ull &&
                c->h_ctl->wl_count == 0;
    if (!lean_done && shard_dec)  // errors, warnings, slow weights or ids that are not decimal
      throw Failure(G2N_E_UNSUPPORTED, "sharded decimal-id build: this range needs the general protocol");
    if (!lean_done) {
      const bool int_ok = !c->h_ctl->int_fail;
      c->h_ctl->wl_count = c->h_ctl->n_deferred = c->h_ctl->int_fail = 0;
      G2N_HIP(hipMemcpyAsync(&c->ctl->wl_count, &c->h_ctl->wl_count, sizeof(unsigned long long),
                             hipMemcpyHostToDevice, c->stream));
      G2N_HIP(hipMemcpyAsync(&c->ctl->n_deferred, &c->h_ctl->n_deferred, sizeof(unsigned long long),
                             hipMemcpyHostToDevice, c->stream));
      G2N_HIP(hipMemcpyAsync(&c->ctl->int_fail, &c->h_ctl->int_fail, sizeof(unsigned long long),
                             hipMemcpyHostToDevice, c->stream));
      if (!int_ok) op.tid = nullptr;  // not decimal ids after all: the hash dictionary
    }
  }
  if (!lean_done) parse(op);
  const uint64_t n_work = c->h_ctl->wl_count;
  if (n_work) {
    hipLaunchKernelGGL(k_weights_slow, dim3(grid_for(n_work, 64)), dim3(64), 0, c->stream, in, len, ls, wl, n_work, op, E,
                       c->ctl);
    sync_ctl(c);
    phase(c, "weights_slow");
  }

  // ---- first error in stream order; the one-shot unsupported-record warning
  uint64_t err_key = c->h_ctl->err_key;
  uint64_t err_line = err_key == ~0ull ? ~0ull : (err_key >> 5);
  int err_code = err_key == ~0ull ? 0 : (int)(err_key & 31);
  // options.unknown_warned: an earlier shard of a sharded build already met an unsupported
  // record, so later ones are skipped silently (parser.py:125-131 warns once per parser)
  const uint64_t warn_line = o->unknown_warned ? ~0ull : c->h_ctl->warn_line;
  if (warn_line != ~0ull) R->warn_line = (int64_t)warn_line;  // first unsupported line, warned or not
  if (warn_line != ~0ull && warn_line < err_line) {
    // (a tile-local lean build has no line starts: k_tile_lean_check found the record's offset)
    uint64_t off = local_done ? c->h_ctl->warn_off : read_dev(c, ls + warn_line);
    uint8_t b = read_dev(c, in + off);
    if (b >= 0x80) {  // parser.py:127 line[:1].decode() raises
      err_line = warn_line;
      err_code = G2N_E_UNICODE;
      c->h_ctl->detail_off = off;
      c->h_ctl->detail_len = 1;
    } else {
      R->has_warning = 1;
      R->warn_byte = b;
      R->warn_line = (int64_t)warn_line;
    }
  }
  if (err_code) {
    R->status = err_code;
    R->err_line = (int64_t)err_line;
    c->err_line_off = read_dev(c, ls + err_line);
    if (err_code == G2N_E_UNICODE && err_line != warn_line) {
      hipLaunchKernelGGL(k_error_detail, dim3(1), dim3(1), 0, c->stream, in, len, ls, err_line, c->ctl);
      sync_ctl(c);
    }
    if (err_code == G2N_E_UNICODE) {
      R->err_detail = in + c->h_ctl->detail_off;  // device pointer
      R->err_detail_len = (int64_t)c->h_ctl->detail_len;
    }
    hipLaunchKernelGGL(k_count_records, dim3(grid_for(err_line)), dim3(kTPB), 0, c->stream, kind, err_line, c->ctl);
    R->n_records_before_error = (int64_t)read_dev(c, &c->ctl->n_records_before);
    finish_timings(c, R);
    return R->status;
  }
  R->n_records_before_error = R->n_records;

  // ---- dictionary: first-touch node ids (K4).  A lean build whose premise held has them all: node
  // k is S line k, its key str(k + 1) (names by arithmetic, k_names_dec)
  const bool coords_done = lean_done;  // the parse wrote rows / cols
  DictOut D{};
  if (lean_done)
    D.n_nodes = n_s * tps;
  else
    // expected distinct keys: the S keys plus a few edge-only ones — or, when S keys are under 1/32 of
    // the edge touches (an S-less range of a chunked build, an edge-list-like GFA), half the edge
    // touches: a table sized for the S keys alone overflows its probe bound and is redone at full size
    D = build_dictionary(c, in, len, T, n_t, n_s * tps,
                         n_s * tps + (n_s * tps * 32 < n_e * tpe ? (n_e * tpe) / 2 : (n_e * tpe) / 16) + 1024, bidir,
                         op.tid && !c->h_ctl->int_fail ? kIntDone : kIntFailed);
  TouchIn TI{T.noff, T.nlen, T.ooff, T.olen};
  const uint64_t n_nodes = shard_dec ? (uint64_t)o->range_n_segments : D.n_nodes;  // global ids: the file's nodes
  if (n_nodes >= 0x7FFFFFFFull) throw Failure(G2N_E_UNSUPPORTED, "more than 2^31-1 nodes");
  R->n_nodes = (int64_t)n_nodes;
  phase(c, "ids");
  const bool throw_after_ids = (c->test_flags & kTestThrowAfterIds) != 0;
  if (o->want_node_names && hash_done && bidir) {  // nodes 2k / 2k + 1: S line k's name + ":+" / ":-"
    auto* offs = dget<int64_t>(c, S_OFFS, n_nodes + 1);
    auto* soff = dget<int64_t>(c, S_TEMP, n_s + 1);
    scan_excl<uint32_t, int64_t>(c, hl_nlen, soff, n_s, soff + n_s);
    const uint64_t names_len = 2 * hl_names_len + 4 * n_s;
    auto* blob = dget<uint8_t>(c, S_BLOB, names_len);
    hipLaunchKernelGGL(k_names_lean_bidir, dim3(grid_for(n_s + 1)), dim3(kTPB), 0, c->stream, in,
                       (const uint64_t*)hl_noff, (const uint32_t*)hl_nlen, (const int64_t*)soff, n_s, offs, blob);
    R->names_bytes = names_len;
    R->names_blob = blob;
    R->names_offsets = offs;
    phase(c, "names");
  } else if (o->want_node_names && hash_done) {  // node k's name: S line k's (noff / nlen from the claims)
    auto* offs = dget<int64_t>(c, S_OFFS, n_nodes + 1);
    scan_excl<uint32_t, int64_t>(c, hl_nlen, offs, n_nodes);
    hipLaunchKernelGGL(k_names_total, dim3(1), dim3(1), 0, c->stream, (const uint32_t*)hl_nlen, n_nodes, offs, c->ctl);
    const uint64_t names_len = hl_names_len;
    auto* blob = dget<uint8_t>(c, S_BLOB, names_len);
    if (n_nodes) {  // the copy on the side stream, overlapping the assembly's finish (fork_side)
      const uint64_t* no = hl_noff;
      const uint32_t* nl = hl_nlen;
      c->side_work = [c, in, len, no, nl, n_nodes, offs, blob]() {
        hipLaunchKernelGGL(k_names, dim3(grid_for(n_nodes)), dim3(kTPB), 0, c->side, in, len,
                           TouchIn{(uint64_t*)no, (uint32_t*)nl, nullptr, nullptr}, n_nodes, (const uint32_t*)nullptr,
                           (const int64_t*)offs, 0, blob);
      };
    }
    R->names_bytes = names_len;
    R->names_blob = blob;
    R->names_offsets = offs;
    phase(c, "names");
  } else if (o->want_node_names && lean_done && c->edge_text && !name_pre_len) {
    c->names_dec = true;  // k_edge_dec_text renders them from the ids
  } else if (o->want_node_names && lean_done) {
    auto* offs = dget<int64_t>(c, S_OFFS, n_nodes + 1);
    const uint64_t names_len = dec_name_off(n_nodes, (int)bidir) + (uint64_t)name_pre_len * n_nodes;
    auto* blob = dget<uint8_t>(c, S_BLOB, names_len);
    // no input but n_nodes: on the side stream, overlapping the assembly's finish (fork_side in
    // csr_partition; joined in finish_timings)
    const int bd = (int)bidir;
    const uint32_t pl = name_pre_len;
    c->side_work = [c, n_nodes, bd, offs, blob, dpre, pl]() {
      hipLaunchKernelGGL(k_names_dec, dim3(grid_for(n_nodes + 1)), dim3(kTPB), 0, c->side, n_nodes, bd, offs, blob,
                         dpre, pl);
    };
    R->names_bytes = names_len;
    R->names_blob = blob;
    R->names_offsets = offs;
    phase(c, "names");
  } else if (o->want_node_names) {  // names blob + offsets in id order
    auto* offs = dget<int64_t>(c, S_OFFS, n_nodes + 1);
    scan_excl<uint32_t, int64_t>(c, D.klen, offs, n_nodes);
    hipLaunchKernelGGL(k_names_total, dim3(1), dim3(1), 0, c->stream, D.klen, n_nodes, offs, c->ctl);
    const uint64_t names_len = read_dev(c, &c->ctl->names_len);
    auto* blob = dget<uint8_t>(c, S_BLOB, names_len);
    if (n_nodes)
      hipLaunchKernelGGL(k_names, dim3(grid_for(n_nodes)), dim3(kTPB), 0, c->stream, in, len, TI, n_nodes, D.inv,
                         offs, (int)bidir, blob);
    R->names_bytes = names_len;
    R->names_blob = blob;
    R->names_offsets = offs;
    phase(c, "names");
  }
  if (throw_after_ids) throw Failure(G2N_E_DEVICE, "test: injected failure after the ids");

  // ---- triplets (K6): stream-order COO with the dtype cast
  // values: not for a grouped build whose every value is dtype(1) (the partition reads none)
  void* data = dbuf(c, S_DATA, (in_groups && (!o->weight_tag || codes_done)) ? 16 : n_trip * dtype_size(dt));
  const bool uni = !op.has_wt;  // no weight tag: every entry is dtype(1.0)
  const bool coo_out = (o->output == G2N_OUT_PARSE && !maxsym) || o->output == G2N_OUT_COO;
  EdgeIn EI{E.w, E.tb};
  phase(c, "_prep");
  // options.range_flags G2N_RANGE_NO_VALUES: a sharded range (decimal, or a general-protocol local build) whose
  // caller routes coordinates only (uniform values, no COO result): the values array is left unwritten
  const bool no_values = uni && (o->range_flags & G2N_RANGE_NO_VALUES) != 0;
  if (coords_done) {  // values only, and only when the output or the sums read them
    if (codes_done) c->wenc = c->gcoo.wenc;  // the partition sums the parse's codes; no value is cast
    if (n_e && (coo_out || !uni) && !no_values && !codes_done) {
      // a weighted SUM CSR: the exact-int32 codes the bucket partition sums (csr_partition_w) beside
      uint32_t* enc = nullptr;
      if (!uni && !maxsym && o->output == G2N_OUT_CSR && !(c->test_flags & kTestNoBuckets) && n_trip <= 0x7FFFFFFFull)
        c->wenc = enc = dget<uint32_t>(c, S_WENC, n_trip);
#define G2N_VALUES(T) \
  hipLaunchKernelGGL(k_values<T>, dim3(grid_for(n_e)), dim3(kTPB), 0, c->stream, E.w, n_e, ktrip, (int)uni, (T*)data, \
                     c->ctl, enc)
      switch (dt) {
        case G2N_BOOL: G2N_VALUES(uint8_t); break;
        case G2N_INT8: G2N_VALUES(int8_t); break;
        case G2N_INT32: G2N_VALUES(int32_t); break;
        case G2N_FLOAT32: G2N_VALUES(float); break;
        default: G2N_VALUES(double); break;
      }
#undef G2N_VALUES
    }
    phase(c, "values");
  } else {
    switch (dt) {
      case G2N_BOOL: run_triplets<uint8_t>(c, EI, n_e, D.slot, D.table, D.tid, (int)tpe, gd, rows, cols, data); break;
      case G2N_INT8: run_triplets<int8_t>(c, EI, n_e, D.slot, D.table, D.tid, (int)tpe, gd, rows, cols, data); break;
      case G2N_INT32: run_triplets<int32_t>(c, EI, n_e, D.slot, D.table, D.tid, (int)tpe, gd, rows, cols, data); break;
      case G2N_FLOAT32: run_triplets<float>(c, EI, n_e, D.slot, D.table, D.tid, (int)tpe, gd, rows, cols, data); break;
      default: run_triplets<double>(c, EI, n_e, D.slot, D.table, D.tid, (int)tpe, gd, rows, cols, data); break;
    }
    phase(c, "triplets");
  }
  // the cast's verdict needs a host wait only when a cast ran (a build whose values are all dtype(1)
  // and unread — C2, C4 — goes on to the assembly without one)
  const bool cast_ran = !coords_done || (n_e && (coo_out || !uni) && !no_values && !codes_done);
  if (cast_ran) sync_ctl(c);
  const uint64_t cast_key = cast_ran ? c->h_ctl->cast_key : ~0ull;
  R->n_cast_overflow = cast_ran ? (int64_t)(c->h_ctl->n_f32_overflow * (uint64_t)ktrip) : 0;
  if (cast_key != ~0ull) {  // np.array(data, dtype) raises at the first bad element
    R->status = (int)(cast_key & 15);
    R->err_index = (int64_t)(cast_key >> 4);
    R->err_value = read_dev(c, E.w + (cast_key >> 4) / ktrip);
    finish_timings(c, R);
    return R->status;
  }
  if (coo_out) {  // builders.py:281: the COO itself
    R->format = G2N_FMT_COO;
    R->nnz = (int64_t)n_trip;
    R->rows = rows;
    R->cols = cols;
    R->data = data;
    c->slots = GroupedCoo{};
    if (in_groups) {  // G2N_RANGE_SLOTS: the group slots themselves (g2n_context_group_slots)
      c->slots = c->gcoo;
      R->rows = c->gcoo.rows;
      R->cols = c->gcoo.cols;
      c->gcoo.active = false;
    }
    finish_timings(c, R);
    return G2N_OK;
  }
  switch (dt) {
    case G2N_BOOL: assemble<uint8_t>(c, rows, cols, (const uint8_t*)data, n_trip, n_nodes, n_nodes, maxsym, uni, R); break;
    case G2N_INT8: assemble<int8_t>(c, rows, cols, (const int8_t*)data, n_trip, n_nodes, n_nodes, maxsym, uni, R); break;
    case G2N_INT32: assemble<int32_t>(c, rows, cols, (const int32_t*)data, n_trip, n_nodes, n_nodes, maxsym, uni, R); break;
    case G2N_FLOAT32: assemble<float>(c, rows, cols, (const float*)data, n_trip, n_nodes, n_nodes, maxsym, uni, R); break;
    default: assemble<double>(c, rows, cols, (const double*)data, n_trip, n_nodes, n_nodes, maxsym, uni, R); break;
  }
  if (c->gcoo.failed) {  // the partition refused the group-slot COO (an overfull bucket): once more without
    c->gcoo = GroupedCoo{};
    c->no_group = true;
    int rc;
    try {
      rc = run_build(c, in, len, o, R);
    } catch (...) {
      c->no_group = false;
      throw;
    }
    c->no_group = false;
    return rc;
  }
  c->gcoo.active = false;
  finish_timings(c, R);
  return G2N_OK;
}

// export --format edge-list (cli.py:264-281).  The lines come from the same parse: the
// stream-order COO of a directed, keep-orientation build (one entry per L/E/C record, ids of
// the record's endpoint keys, builders.py:199-228 with keep_directed_bidir) and its names blob;
// the text is rendered in HBM.  Result: format G2N_FMT_TEXT, data = text, nnz = its bytes.
// An endpoint key that is not UTF-8: status G2N_E_UNICODE, err_line -1, err_index = the edge,
// err_detail = the key, and the text holds the lines before it (what the reference wrote).
static int run_edge_list(g2n_context* c, const uint8_t* in, uint64_t len, const g2n_options* o, g2n_result* R) {
  g2n_options b = *o;
  b.directed = 1;
  b.keep_directed_bidir = 1;
  b.asymmetric = 1;
  b.strip_orientation = 0;
  b.weight_tag = nullptr;
  b.dtype = G2N_BOOL;
  b.output = G2N_OUT_COO;
  b.want_node_names = 1;
  b.range_flags = G2N_RANGE_NO_VALUES;  // the text reads ids only: a decimal-id build writes no values
  struct TextFlag {  // run_build leaves decimal names to the render (names_dec), exceptions included
    g2n_context* c;
    ~TextFlag() { c->edge_text = false; }
  } guard{c};
  c->edge_text = !(o->test_flags & kTestNoDecText);  // (this call's flags: run_build copies them only later)
  c->names_dec = false;
  const int rc = run_build(c, in, len, &b, R);
  c->edge_text = false;
  if (rc == G2N_OK && c->names_dec) {
    const uint64_t n = (uint64_t)R->nnz;
    const auto* rows = (const int32_t*)R->rows;
    const auto* cols = (const int32_t*)R->cols;
    const int bd = o->bidirected ? 1 : 0;
    const uint64_t nb = (n + kTextEdges - 1) / kTextEdges;
    auto* bsum = dget<uint64_t>(c, S_ELEN, nb + 1);
    auto* bpos = dget<uint64_t>(c, S_EPOS, nb + 1);
    if (nb)
      hipLaunchKernelGGL(k_edge_dec_sum, dim3((unsigned)nb), dim3(kTPB), 0, c->stream, rows, cols, n, bd, bsum);
    G2N_HIP(hipMemsetAsync(bsum + nb, 0, sizeof(uint64_t), c->stream));
    excl_scan<uint64_t>(c, bsum, bpos, nb + 1);
    const uint64_t total = read_dev(c, bpos + nb);
    auto* text = dget<uint8_t>(c, S_ETEXT, total + 16);
    if (nb)
      hipLaunchKernelGGL(k_edge_dec_text, dim3((unsigned)nb), dim3(kTPB), 0, c->stream, rows, cols, n, bd, bpos, text);
    phase(c, "edge_text");
    R->format = G2N_FMT_TEXT;
    R->rows = R->cols = nullptr;
    R->data = text;
    R->nnz = (int64_t)total;
    R->names_blob = nullptr;
    R->names_offsets = nullptr;
    R->names_bytes = 0;
    finish_timings(c, R);
    return G2N_OK;
  }
  if (rc >= G2N_E_MALFORMED_L && rc <= G2N_E_INT_TOO_LARGE && R->err_line >= 0) {
    // the reference's loop wrote the lines of the records before the failing one
    // (cli.py:270-281): render the prefix [0, start of the failing line) from the same input
    const g2n_result first = *R;
    const uint64_t off = c->err_line_off;
    fill_defaults(R);
    if (run_edge_list(c, in, off, o, R) == G2N_OK) {  // a key before it that is not UTF-8 comes first
      R->status = first.status;
      R->err_line = first.err_line;
      R->err_index = first.err_index;
      R->err_value = first.err_value;
      R->err_detail = first.err_detail;
      R->err_detail_len = first.err_detail_len;
      R->n_records_before_error = first.n_records_before_error;
    }
    R->has_warning = first.has_warning;
    R->warn_byte = first.warn_byte;
    R->warn_line = first.warn_line;
    R->n_lines = first.n_lines;
    R->n_records = first.n_records;
    return R->status;
  }
  if (rc != G2N_OK) return rc;
  const uint64_t n = (uint64_t)R->nnz, n_names = (uint64_t)R->n_nodes;
  const auto* rows = (const int32_t*)R->rows;
  const auto* cols = (const int32_t*)R->cols;
  const int64_t* offs = R->names_offsets;
  const uint8_t* blob = R->names_blob;
  auto* meta = dget<uint64_t>(c, S_EBAD, n_names + 1);
  auto* elen = dget<uint64_t>(c, S_ELEN, n + 1);
  auto* epos = dget<uint64_t>(c, S_EPOS, n + 1);
  auto* first = dget<unsigned long long>(c, S_EFIRST, 1);
  auto* em = dget<ulonglong2>(c, S_EMETA, n + 1);
  G2N_HIP(hipMemsetAsync(first, 0xFF, sizeof(unsigned long long), c->stream));
  if (n_names)
    hipLaunchKernelGGL(k_name_meta, dim3(grid_for(n_names)), dim3(kTPB), 0, c->stream, blob, offs, n_names, meta);
  if (n)
    hipLaunchKernelGGL(k_edge_text_len, dim3(grid_for(n)), dim3(kTPB), 0, c->stream, rows, cols, n, meta, offs,
                       elen, em, first);
  G2N_HIP(hipMemsetAsync(elen + n, 0, sizeof(uint64_t), c->stream));
  excl_scan<uint64_t>(c, elen, epos, n + 1);
  const uint64_t total = read_dev(c, epos + n);
  const unsigned long long fb = read_dev(c, first);
  auto* text = dget<uint8_t>(c, S_ETEXT, total + 16);
  if (n)
    hipLaunchKernelGGL(k_edge_text, dim3((unsigned)((n + kTextEdges - 1) / kTextEdges)), dim3(kTPB), 0, c->stream,
                       rows, cols, n, em, offs, blob, epos, text);
  phase(c, "edge_text");
  R->format = G2N_FMT_TEXT;
  R->rows = R->cols = nullptr;
  R->data = text;
  R->nnz = (int64_t)total;
  R->names_blob = nullptr;  // the names are in the text
  R->names_offsets = nullptr;
  R->names_bytes = 0;
  if (fb != ~0ull) {  // f"{u.decode()}\t{v.decode()}\n": u is decoded first
    const int32_t r = read_dev(c, rows + fb), cc = read_dev(c, cols + fb);
    const int32_t who = (read_dev(c, meta + r) & 1u) ? r : cc;
    const int64_t o0 = read_dev(c, offs + who), o1 = read_dev(c, offs + who + 1);
    R->nnz = (int64_t)read_dev(c, epos + fb);
    R->status = G2N_E_UNICODE;
    R->err_line = -1;
    R->err_index = (int64_t)fb;
    R->err_detail = blob + o0;
    R->err_detail_len = o1 - o0;
  }
  finish_timings(c, R);
  return R->status;
}

static int run_pipeline(g2n_context* c, const uint8_t* in, uint64_t len, const g2n_options* o, g2n_result* R) {
  c->slots = GroupedCoo{};  // (set again only by a build whose COO result stays in group slots)
  if (o->output == G2N_OUT_EDGE_LIST) return run_edge_list(c, in, len, o, R);
  return run_build(c, in, len, o, R);
}

// --------------------------------------------------------------- contexts ----------
static g2n_context* context_create(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
    (void)hipGetLastError();
    throw Failure(G2N_E_DEVICE, "no HIP device available (the GFA->CSR path runs only on the GPU)");
  }
  if (device < 0 || device >= n) throw Failure(G2N_E_ARG, "device ordinal out of range");
  std::unique_ptr<g2n_context> c(new g2n_context());
  c->device = device;
  G2N_HIP(hipSetDevice(device));
#ifndef G2N_SIDE_PRIO  // the side stream (names beside the finish) at the lowest priority, the pipeline at the
#define G2N_SIDE_PRIO 1  // highest: C4 8.21-8.28 -> 8.05-8.11 ms in a same-box A/B (the names' interference 0.33 ms)
#endif
  int least = 0, greatest = 0;  // (no priority range: plain streams)
  if (G2N_SIDE_PRIO && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess && least != greatest) {
    G2N_HIP(hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, greatest));
    G2N_HIP(hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking, least));
  } else {
    G2N_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    G2N_HIP(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
  }
  G2N_HIP(hipStreamCreateWithFlags(&c->place, hipStreamNonBlocking));  // (F2 at the pipeline's priority or the
                                                                          // lowest measured slower: 8.11-8.38 ms)
  for (auto& e : c->side_ev) G2N_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (auto& e : c->ov_ev) G2N_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  G2N_HIP(hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, device));
  if (c->n_cu <= 0) c->n_cu = 1;
  {  // the persistent decimal parse's grid: every block resident at once (LDS-limited: 3 per CU)
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_tile_lean_p<true>, kLeanTPB, 0) != hipSuccess ||
        per_cu <= 0) {
      (void)hipGetLastError();
      per_cu = 1;
    }
    c->lean_blocks = (uint64_t)per_cu * (uint64_t)c->n_cu;
  }
  c->bufs.resize(S_NSLOTS);
  G2N_HIP(hipMalloc(&c->ctl, sizeof(Ctl)));
  G2N_HIP(hipHostMalloc(&c->h_ctl, sizeof(Ctl), hipHostMallocDefault));
  for (int k = 0; k <= G2N_MAX_PHASES; k++) G2N_HIP(hipEventCreate(&c->ev[k]));
  return c.release();
}

static void context_destroy(g2n_context* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->side) (void)hipStreamSynchronize(c->side);
  if (c->place) (void)hipStreamSynchronize(c->place);
  for (auto& b : c->bufs)
    if (b.p) (void)hipFree(b.p);
  if (c->ctl) (void)hipFree(c->ctl);
  if (c->h_ctl) (void)hipHostFree(c->h_ctl);
  for (int k = 0; k <= G2N_MAX_PHASES; k++)
    if (c->ev[k]) (void)hipEventDestroy(c->ev[k]);
  for (auto& e : c->side_ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : c->ov_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->side) (void)hipStreamDestroy(c->side);
  if (c->place) (void)hipStreamDestroy(c->place);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

// one cached context per device for the host entry points
static std::mutex g_ctx_mu;
static std::map<int, g2n_context*> g_ctx;

static g2n_context* shared_context(int device) {
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  auto it = g_ctx.find(device);
  if (it != g_ctx.end()) return it->second;
  g2n_context* c = context_create(device);
  c->shared = true;
  size_t f = 0, t = 0;
  if (hipMemGetInfo(&f, &t) == hipSuccess) c->hbm_total = t;
  (void)hipGetLastError();
  g_ctx[device] = c;
  return c;
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static const void* download(g2n_context* c, HostBuf& dst, const void* src, size_t bytes) {
  dst.alloc(bytes);
  if (bytes) G2N_HIP(hipMemcpyAsync(dst.data(), src, bytes, hipMemcpyDeviceToHost, c->stream));
  return dst.data();
}

static void download_result(g2n_context* c, const g2n_result& D, HostResult* H) {
  g2n_result& R = H->r;
  std::memcpy(&R, &D, sizeof(g2n_result));
  R.priv_ = H;
  R.err_detail = nullptr;
  R.names_blob = nullptr;
  R.names_offsets = nullptr;
  R.rows = R.cols = R.indptr = R.indices = R.data = nullptr;
  if (D.err_detail) R.err_detail = (const uint8_t*)download(c, H->detail, D.err_detail, (size_t)D.err_detail_len);
  if (D.status == G2N_OK || D.format == G2N_FMT_TEXT) {  // edge-list text: the lines before a failure too
    if (D.names_blob) {
      const int64_t* offs =
          (const int64_t*)download(c, H->offs, D.names_offsets, (size_t)(D.n_nodes + 1) * sizeof(int64_t));
      G2N_HIP(hipStreamSynchronize(c->stream));
      const size_t blen = (size_t)offs[(size_t)D.n_nodes];
      R.names_blob = (const uint8_t*)download(c, H->blob, D.names_blob, blen);
      R.names_offsets = offs;
    }
    const size_t w = dtype_size(D.dtype);
    if (D.format == G2N_FMT_TEXT) {
      R.data = download(c, H->data, D.data, (size_t)D.nnz);
    } else if (D.format == G2N_FMT_COO) {
      R.rows = download(c, H->rows, D.rows, (size_t)D.nnz * 4);
      R.cols = download(c, H->cols, D.cols, (size_t)D.nnz * 4);
    } else {
      const size_t iw = D.index_width == 8 ? 8 : 4;
      R.indptr = download(c, H->indptr, D.indptr, (size_t)(D.n_nodes + 1) * iw);
      R.indices = download(c, H->indices, D.indices, (size_t)D.nnz * iw);
    }
    if (D.format != G2N_FMT_TEXT) R.data = download(c, H->data, D.data, (size_t)D.nnz * w);
  }
  G2N_HIP(hipStreamSynchronize(c->stream));
}

int build_host_fill(size_t len, const FillFn& fill, const g2n_options* opts, g2n_result** out, double read_ms) {
  g2n_context* c = shared_context(opts->device);
  std::lock_guard<std::mutex> lk(c->mu);
  enter_call(c);
  G2N_HIP(hipSetDevice(c->device));
  double t0 = now_ms();
  auto* din = dget<uint8_t>(c, S_IN, len + 16);
  G2N_HIP(hipStreamSynchronize(c->stream));  // the slot may still be read by an earlier build
  staged_upload(c->device, din, len, fill);
  double t1 = now_ms();
  g2n_result D;
  run_pipeline(c, din, len, opts, &D);
  double t2 = now_ms();
  HostResult* H = new_host_result();
  try {
    download_result(c, D, H);
  } catch (...) {
    delete H;
    throw;
  }
  H->r.host_ms_read = read_ms;
  H->r.host_ms_h2d = t1 - t0;
  H->r.host_ms_d2h = now_ms() - t2;
  shrink_shared(c);
  *out = &H->r;
  return H->r.status;
}

int build_host_bgzf(const uint8_t* z, size_t zlen, const std::vector<ZMember>& members, size_t total_out,
                    const g2n_options* opts, g2n_result** out, double read_ms) {
  g2n_context* c = shared_context(opts->device);
  std::lock_guard<std::mutex> lk(c->mu);
  enter_call(c);
  G2N_HIP(hipSetDevice(c->device));
  const double t0 = now_ms();
  auto* dz = dget<uint8_t>(c, S_ZIN, zlen + 16);
  auto* dm = dget<ZMember>(c, S_ZMEM, members.size());
  auto* bad = dget<unsigned int>(c, S_ZBAD, 1);
  auto* din = dget<uint8_t>(c, S_IN, total_out + 16);
  G2N_HIP(hipStreamSynchronize(c->stream));  // the slots may still be read by an earlier build
  staged_upload(c->device, dz, zlen, [z](size_t off, uint8_t* dst, size_t n) { std::memcpy(dst, z + off, n); });
  G2N_HIP(hipMemcpyAsync(dm, members.data(), members.size() * sizeof(ZMember), hipMemcpyHostToDevice, c->stream));
  G2N_HIP(hipMemsetAsync(bad, 0, sizeof(unsigned int), c->stream));
  hipEvent_t e0, e1;
  G2N_HIP(hipEventCreate(&e0));
  G2N_HIP(hipEventCreate(&e1));
  G2N_HIP(hipEventRecord(e0, c->stream));
  hipLaunchKernelGGL(k_inflate_members, dim3((unsigned)((members.size() + kInflTPB - 1) / kInflTPB)), dim3(kInflTPB), 0,
                     c->stream, (const uint8_t*)dz, (const ZMember*)dm, (uint64_t)members.size(), din, bad);
  G2N_HIP(hipEventRecord(e1, c->stream));
  const unsigned int n_bad = read_dev(c, bad);
  float inflate_ms = 0.f;
  G2N_HIP(hipEventElapsedTime(&inflate_ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (n_bad) return kBgzfFallback;
  const double t1 = now_ms();
  g2n_result D;
  run_pipeline(c, din, total_out, opts, &D);
  const double t2 = now_ms();
  HostResult* H = new_host_result();
  try {
    download_result(c, D, H);
  } catch (...) {
    delete H;
    throw;
  }
  H->r.host_ms_read = read_ms;
  H->r.host_ms_h2d = t1 - t0;  // upload of the compressed bytes + GPU inflate
  H->r.host_ms_d2h = now_ms() - t2;
  if (H->r.n_phases < G2N_MAX_PHASES) {  // the inflate kernel as one more device phase
    H->r.phase_names[H->r.n_phases] = "gz_inflate";
    H->r.phase_ms[H->r.n_phases++] = inflate_ms;
  }
  shrink_shared(c);
  *out = &H->r;
  return H->r.status;
}

int build_host(const void* buf, size_t len, const g2n_options* opts, g2n_result** out, double read_ms) {
  const uint8_t* src = (const uint8_t*)buf;
  return build_host_fill(
      len, [src](size_t off, uint8_t* dst, size_t n) { std::memcpy(dst, src + off, n); }, opts, out, read_ms);
}

// --------------------------------------------------------- convert_format ------
// *not_one = 1 when some value differs from T(1) (bool: false; floats: anything but exactly 1.0,
// NaN included).  Racing plain stores of the same word: no atomics needed.
template <class T>
__global__ void k_values_not_one(const T* __restrict__ d, uint64_t n, unsigned int* not_one) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  bool bad = false;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) bad |= !(d[i] == (T)1);
  if (bad) *not_one = 1u;
}

template <class T>
static void coo_to_csr_t(g2n_context* c, const int32_t* rows, const int32_t* cols, const T* data, uint64_t nnz,
                         uint64_t n_rows, uint64_t n_cols, bool uniform, g2n_result* R, int force_unsorted) {
  // uniform (every value T(1): what parse_gfa returns without a weight tag): the copy count per
  // entry is the sum, through the unweighted bucket partition — the path with int64 results past
  // 2^31 - 1 entries (scipy's _coo_to_compressed sizes its index dtype by coo.nnz)
  assemble<T>(c, rows, cols, data, nnz, n_rows, n_cols, false, uniform, R, force_unsorted);
}

// force_unsorted: -1 = this COO is the whole matrix (scipy's has_sorted_indices verdict is its own),
// 0 / 1 = one row band of a larger COO, the whole matrix's verdict given (g2n_coo_to_csr_band)
int coo_to_csr(const void* rows, const void* cols, const void* data, int64_t nnz, int64_t n_rows, int64_t n_cols,
               int32_t index_width, int32_t dtype, int32_t device, uint32_t test_flags, g2n_result** out,
               int force_unsorted = -1) {
  if (index_width != 4) throw Failure(G2N_E_UNSUPPORTED, "only int32 COO indices are supported");
  if (dtype < G2N_BOOL || dtype > G2N_FLOAT64) throw Failure(G2N_E_ARG, "unsupported dtype");
  if (nnz < 0 || n_rows < 0 || n_cols < 0) throw Failure(G2N_E_ARG, "negative size");
  if (n_rows >= 0x7FFFFFFF || n_cols >= 0x7FFFFFFF) throw Failure(G2N_E_UNSUPPORTED, "2^31-1 or more rows / columns");
  if ((uint64_t)nnz >= 0xFFFFFFFFull) throw Failure(G2N_E_UNSUPPORTED, "2^32-1 or more entries");
  g2n_context* c = shared_context(device);
  std::lock_guard<std::mutex> lk(c->mu);
  enter_call(c);
  G2N_HIP(hipSetDevice(c->device));
  clear_call_state(c);
  c->test_flags = test_flags & (kTestNoBuckets | kTestIndex64);  // the conversion's own rare paths
  const size_t w = dtype_size(dtype);
  auto* dr = dget<int32_t>(c, S_ROWS, (uint64_t)nnz);
  auto* dc = dget<int32_t>(c, S_COLS, (uint64_t)nnz);
  void* dd = dbuf(c, S_DATA, (size_t)nnz * w);
  auto* not_one = dget<unsigned int>(c, S_ZBAD, 1);
  G2N_HIP(hipMemsetAsync(not_one, 0, sizeof(unsigned int), c->stream));
  if (nnz) {
    G2N_HIP(hipMemcpyAsync(dr, rows, (size_t)nnz * 4, hipMemcpyHostToDevice, c->stream));
    G2N_HIP(hipMemcpyAsync(dc, cols, (size_t)nnz * 4, hipMemcpyHostToDevice, c->stream));
    G2N_HIP(hipMemcpyAsync(dd, data, (size_t)nnz * w, hipMemcpyHostToDevice, c->stream));
    const unsigned g = (unsigned)std::min<uint64_t>(grid_for((uint64_t)nnz), 8192);
    switch (dtype) {
      case G2N_BOOL:
      case G2N_INT8: hipLaunchKernelGGL(k_values_not_one<uint8_t>, dim3(g), dim3(kTPB), 0, c->stream,
                                        (const uint8_t*)dd, (uint64_t)nnz, not_one); break;
      case G2N_INT32: hipLaunchKernelGGL(k_values_not_one<int32_t>, dim3(g), dim3(kTPB), 0, c->stream,
                                         (const int32_t*)dd, (uint64_t)nnz, not_one); break;
      case G2N_FLOAT32: hipLaunchKernelGGL(k_values_not_one<float>, dim3(g), dim3(kTPB), 0, c->stream,
                                           (const float*)dd, (uint64_t)nnz, not_one); break;
      default: hipLaunchKernelGGL(k_values_not_one<double>, dim3(g), dim3(kTPB), 0, c->stream, (const double*)dd,
                                  (uint64_t)nnz, not_one); break;
    }
  }
  // the unweighted partition packs (col << 2 | side) in 32 bits: columns below 2^30
  const bool uniform = nnz > 0 && n_cols < (1ll << 30) && read_dev(c, not_one) == 0u;
  if ((uint64_t)nnz > 0x7FFFFFFEull && !uniform)
    throw Failure(G2N_E_UNSUPPORTED, "2^31-1 or more entries with values other than 1 (a weighted matrix)");
  g2n_result D;
  fill_defaults(&D);
  c->n_ev = 0;
  G2N_HIP(hipEventRecord(c->ev[0], c->stream));
  reset_ctl(c);
  D.dtype = dtype;
  D.index_width = 4;
  D.n_nodes = n_rows;
  switch (dtype) {
    case G2N_BOOL: coo_to_csr_t<uint8_t>(c, dr, dc, (const uint8_t*)dd, nnz, n_rows, n_cols, uniform, &D, force_unsorted); break;
    case G2N_INT8: coo_to_csr_t<int8_t>(c, dr, dc, (const int8_t*)dd, nnz, n_rows, n_cols, uniform, &D, force_unsorted); break;
    case G2N_INT32: coo_to_csr_t<int32_t>(c, dr, dc, (const int32_t*)dd, nnz, n_rows, n_cols, uniform, &D, force_unsorted); break;
    case G2N_FLOAT32: coo_to_csr_t<float>(c, dr, dc, (const float*)dd, nnz, n_rows, n_cols, uniform, &D, force_unsorted); break;
    default: coo_to_csr_t<double>(c, dr, dc, (const double*)dd, nnz, n_rows, n_cols, uniform, &D, force_unsorted); break;
  }
  finish_timings(c, &D);
  HostResult* H = new_host_result();
  try {
    download_result(c, D, H);
  } catch (...) {
    delete H;
    throw;
  }
  shrink_shared(c);
  *out = &H->r;
  return G2N_OK;
}

// --------------------------------------------------------- sharded build steps ------
static void begin_call(g2n_context* c) {
  clear_call_state(c);
  c->n_ev = 0;
  G2N_HIP(hipEventRecord(c->ev[0], c->stream));
  reset_ctl(c);
}

uint64_t dedup_keys(g2n_context* c, const uint8_t* blob, uint64_t blob_len, const int64_t* offs, uint64_t n,
                    uint32_t* ids, uint32_t* first_of) {
  begin_call(c);
  if (n >= 0xFFFFFFFFull) throw Failure(G2N_E_UNSUPPORTED, "more than 2^32-1 keys");
  if (n == 0) return 0;
  TouchOut T{dget<uint64_t>(c, S_NOFF, n), dget<uint32_t>(c, S_NLEN, n), nullptr, nullptr,
             dget<uint8_t>(c, S_TKIND, n)};
  hipLaunchKernelGGL(k_keys_to_touches, dim3(grid_for(n)), dim3(kTPB), 0, c->stream, offs, n, T.noff, T.nlen, T.tkind);
  const DictOut D = build_dictionary(c, blob, blob_len, T, n, n, n, false, kIntFailed);
  hipLaunchKernelGGL(k_touch_ids, dim3(grid_for(n)), dim3(kTPB), 0, c->stream, n, D.first, D.slot, D.table, D.tid,
                     (int)D.general, (int)(!D.general && D.inv == nullptr), ids);
  if (D.n_nodes)
    hipLaunchKernelGGL(k_first_of, dim3(grid_for(D.n_nodes)), dim3(kTPB), 0, c->stream, D.n_nodes, D.inv, first_of);
  G2N_HIP(hipStreamSynchronize(c->stream));
  return D.n_nodes;
}

void partition_keys(g2n_context* c, const uint8_t* blob, const int64_t* offs, uint64_t n, uint32_t n_ranks,
                    uint8_t* oblob, int64_t* ooffs, uint32_t* oindex, uint32_t* starts) {
  begin_call(c);
  if (n_ranks == 0 || n_ranks > 4096) throw Failure(G2N_E_ARG, "n_ranks out of range");
  if (n >= 0xFFFFFFFFull) throw Failure(G2N_E_UNSUPPORTED, "more than 2^32-1 keys");
  auto* owner = dget<uint32_t>(c, S_KEYS0, n);
  auto* owner_s = dget<uint32_t>(c, S_KEYS1, n);
  auto* idx = dget<uint32_t>(c, S_VALS0, n);
  auto* lens = dget<int64_t>(c, S_FOFF64, n + 1);
  if (n) {
    hipLaunchKernelGGL(k_key_owner, dim3(grid_for(n)), dim3(kTPB), 0, c->stream, blob, offs, n, n_ranks, owner, idx);
    sort_pairs_u32<uint32_t>(c, owner, owner_s, idx, oindex, n, bits_for(n_ranks));
    hipLaunchKernelGGL(k_key_lens, dim3(grid_for(n)), dim3(kTPB), 0, c->stream, offs, oindex, n, lens);
  }
  G2N_HIP(hipMemsetAsync(lens + n, 0, sizeof(int64_t), c->stream));
  excl_scan<int64_t>(c, lens, ooffs, n + 1);  // ooffs[n] = total bytes
  if (n)
    hipLaunchKernelGGL(k_copy_keys, dim3(grid_for(n)), dim3(kTPB), 0, c->stream, blob, offs, oindex, n, ooffs, oblob);
  G2N_HIP(hipMemsetAsync(&c->ctl->row_gap, 0, sizeof(unsigned long long), c->stream));
  hipLaunchKernelGGL(k_row_bounds, dim3(grid_for(n + 1)), dim3(kTPB), 0, c->stream, owner_s, n, (uint64_t)n_ranks,
                     starts, c->ctl);
  hipLaunchKernelGGL(k_row_start, dim3(grid_for((uint64_t)n_ranks + 1)), dim3(kTPB), 0, c->stream, owner_s, n,
                     (uint64_t)n_ranks, starts, (const Ctl*)c->ctl);
  G2N_HIP(hipStreamSynchronize(c->stream));
}

}  // namespace g2n

// The chunked build's growing key set (g2n_keyset.hip): its own device buffers (the context's arena
// is reused by the builds between calls), per-call scratch from the context.
struct g2n_keyset {
  g2n_context* ctx = nullptr;
  int device = 0;  // (free needs no context: it may be gone by then)
  g2n::KsEntry* table = nullptr;
  uint64_t cap = 0;  // entries, a power of two
  uint8_t* blob = nullptr;
  uint64_t blob_len = 0, blob_cap = 0;
  int64_t* offs = nullptr;  // n + 1
  uint64_t n = 0, offs_cap = 0;
};

namespace g2n {

template <class T>
static void ks_grow(g2n_context* c, T** p, uint64_t* cap, uint64_t used, uint64_t want) {  // keep the first used
  if (want <= *cap) return;
  uint64_t nc = *cap ? *cap : 1024;
  while (nc < want) nc *= 2;
  T* q = nullptr;
  if (hipMalloc(&q, nc * sizeof(T)) != hipSuccess) {
    (void)hipGetLastError();
    throw Failure(G2N_E_NOMEM, "keyset: hipMalloc failed");
  }
  if (used) G2N_HIP(hipMemcpyAsync(q, *p, used * sizeof(T), hipMemcpyDeviceToDevice, c->stream));
  G2N_HIP(hipStreamSynchronize(c->stream));
  if (*p) G2N_HIP(hipFree(*p));
  *p = q;
  *cap = nc;
}

static void keyset_rehash(g2n_keyset* ks, uint64_t want_keys) {
  g2n_context* c = ks->ctx;
  uint64_t cap = ks->cap ? ks->cap : 1024;
  while (cap < 2 * want_keys) cap *= 2;
  if (cap == ks->cap) return;
  if (ks->table) G2N_HIP(hipFree(ks->table));
  ks->table = nullptr;
  if (hipMalloc(&ks->table, cap * sizeof(KsEntry)) != hipSuccess) {
    (void)hipGetLastError();
    ks->cap = 0;
    throw Failure(G2N_E_NOMEM, "keyset: hipMalloc of the table failed");
  }
  ks->cap = cap;
  G2N_HIP(hipMemsetAsync(ks->table, 0xFF, cap * sizeof(KsEntry), c->stream));
  if (ks->n)  // every key again, from the set's own blob
    hipLaunchKernelGGL(k_ks_insert, dim3(grid_for(ks->n, 256)), dim3(256), 0, c->stream, ks->blob,
                       (const int64_t*)ks->offs, ks->n, (const uint32_t*)nullptr, (const uint32_t*)nullptr,
                       (const int64_t*)nullptr, (uint64_t)0, (uint64_t)0, ks->table, cap - 1, ks->blob, ks->offs,
                       (uint32_t*)nullptr, 1);
}

uint64_t keyset_add(g2n_keyset* ks, const uint8_t* blob, const int64_t* offs, uint64_t n, uint32_t* ids) {
  g2n_context* c = ks->ctx;
  begin_call(c);
  if (ks->n + n >= 0xFFFFFFFFull) throw Failure(G2N_E_UNSUPPORTED, "more than 2^32-1 keys");
  if (!ks->offs) {
    ks_grow(c, &ks->offs, &ks->offs_cap, 0, 1024);
    G2N_HIP(hipMemsetAsync(ks->offs, 0, sizeof(int64_t), c->stream));
  }
  if (n == 0) return ks->n;
  keyset_rehash(ks, ks->n + n);  // load <= 1/2 even if every key is new
  auto* fresh = dget<uint32_t>(c, S_KEYS0, n);
  auto* pos = dget<uint32_t>(c, S_KEYS1, n + 1);
  auto* lens = dget<int64_t>(c, S_FOFF64, n + 1);
  auto* bpos = dget<int64_t>(c, S_RSCR, n + 1);
  hipLaunchKernelGGL(k_ks_lookup, dim3(grid_for(n, 256)), dim3(256), 0, c->stream, blob, offs, n,
                     (const KsEntry*)ks->table, ks->cap - 1, (const uint8_t*)ks->blob, ids, fresh);
  hipLaunchKernelGGL(k_ks_new_lens, dim3(grid_for(n, 256)), dim3(256), 0, c->stream, offs, (const uint32_t*)fresh, n,
                     lens);
  scan_excl<uint32_t, uint32_t>(c, fresh, pos, n, pos + n);
  G2N_HIP(hipMemsetAsync(lens + n, 0, sizeof(int64_t), c->stream));
  scan_excl<int64_t, int64_t>(c, lens, bpos, n + 1);
  uint32_t n_new = 0;
  int64_t new_bytes = 0;
  G2N_HIP(hipMemcpyAsync(&n_new, pos + n, sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
  G2N_HIP(hipMemcpyAsync(&new_bytes, bpos + n, sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
  G2N_HIP(hipStreamSynchronize(c->stream));
  // an entry packs the key length in 24 bits and its blob offset in 40 (KsEntry.loc): refuse what
  // would not fit rather than store a truncated length
  if (ks->blob_len + (uint64_t)new_bytes > kKsOffMask)
    throw Failure(G2N_E_UNSUPPORTED, "key set blob past 2^40 bytes");
  if ((uint64_t)new_bytes > kKsMaxKeyLen) {
    auto* mx = dget<unsigned long long>(c, S_TEMP, 1);
    G2N_HIP(hipMemsetAsync(mx, 0, sizeof(unsigned long long), c->stream));
    hipLaunchKernelGGL(k_ks_max_len, dim3(std::min<uint64_t>(grid_for(n, 256), 1024)), dim3(256), 0, c->stream,
                       (const int64_t*)lens, n, mx);
    unsigned long long longest = 0;
    G2N_HIP(hipMemcpyAsync(&longest, mx, sizeof(longest), hipMemcpyDeviceToHost, c->stream));
    G2N_HIP(hipStreamSynchronize(c->stream));
    if (longest > kKsMaxKeyLen) throw Failure(G2N_E_UNSUPPORTED, "a key of 2^24 bytes or more");
  }
  if (n_new) {
    ks_grow(c, &ks->blob, &ks->blob_cap, ks->blob_len, ks->blob_len + (uint64_t)new_bytes + 16);
    ks_grow(c, &ks->offs, &ks->offs_cap, ks->n + 1, ks->n + n_new + 1);
    hipLaunchKernelGGL(k_ks_insert, dim3(grid_for(n, 256)), dim3(256), 0, c->stream, blob, offs, n,
                       (const uint32_t*)fresh, (const uint32_t*)pos, (const int64_t*)bpos, ks->n, ks->blob_len,
                       ks->table, ks->cap - 1, ks->blob, ks->offs, ids, 0);
    ks->n += n_new;
    ks->blob_len += (uint64_t)new_bytes;
  }
  G2N_HIP(hipStreamSynchronize(c->stream));
  return ks->n;
}

uint64_t gather_keys(g2n_context* c, const uint8_t* blob, const int64_t* offs, const uint32_t* index, uint64_t n,
                     uint8_t* oblob, uint64_t oblob_cap, int64_t* ooffs) {
  begin_call(c);
  if (n >= 0xFFFFFFFFull) throw Failure(G2N_E_UNSUPPORTED, "more than 2^32-1 keys");
  auto* lens = dget<int64_t>(c, S_FOFF64, n + 1);
  if (n) hipLaunchKernelGGL(k_key_lens, dim3(grid_for(n)), dim3(kTPB), 0, c->stream, offs, index, n, lens);
  G2N_HIP(hipMemsetAsync(lens + n, 0, sizeof(int64_t), c->stream));
  excl_scan<int64_t>(c, lens, ooffs, n + 1);
  int64_t total = 0;
  G2N_HIP(hipMemcpyAsync(&total, ooffs + n, sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
  G2N_HIP(hipStreamSynchronize(c->stream));
  if ((uint64_t)total > oblob_cap) throw Failure(G2N_E_ARG, "output blob smaller than the gathered keys");
  if (n && total)
    hipLaunchKernelGGL(k_copy_keys, dim3(grid_for(n)), dim3(kTPB), 0, c->stream, blob, offs, index, n, ooffs, oblob);
  G2N_HIP(hipStreamSynchronize(c->stream));
  return (uint64_t)total;
}

void order_keys(g2n_context* c, const uint32_t* first_of, const int64_t* src_idx, uint64_t nd, const uint64_t* h_ends,
                uint32_t n_src, uint64_t* out) {
  begin_call(c);
  if (n_src == 0 || n_src > 4096) throw Failure(G2N_E_ARG, "n_src out of range");
  if (!nd) return;
  auto* ends = dget<uint64_t>(c, S_TEMP, n_src);
  G2N_HIP(hipMemcpyAsync(ends, h_ends, n_src * sizeof(uint64_t), hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(k_order_keys, dim3(grid_for(nd)), dim3(kTPB), 0, c->stream, first_of, src_idx, nd,
                     (const uint64_t*)ends, n_src, out);
  G2N_HIP(hipStreamSynchronize(c->stream));
}

void rank_keys(g2n_context* c, const uint64_t* keys, uint64_t n, const uint64_t* all, const uint64_t* h_all_off,
               uint32_t n_ranks, uint32_t self, int64_t* out) {
  begin_call(c);
  if (n_ranks == 0 || n_ranks > 4096 || self >= n_ranks) throw Failure(G2N_E_ARG, "ranks out of range");
  if (!n) return;
  auto* off = dget<uint64_t>(c, S_TEMP, n_ranks + 1);
  G2N_HIP(hipMemcpyAsync(off, h_all_off, (n_ranks + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(k_rank_keys, dim3(grid_for(n)), dim3(kTPB), 0, c->stream, keys, n, all, (const uint64_t*)off,
                     n_ranks, self, out);
  G2N_HIP(hipStreamSynchronize(c->stream));
}

void remap_pairs(g2n_context* c, const uint32_t* map, uint64_t n_map, int32_t* rows, int32_t* cols, uint64_t n) {
  begin_call(c);
  if (n) {
    if (((uintptr_t)rows | (uintptr_t)cols) & 15)
      hipLaunchKernelGGL(k_remap_pairs<false>, dim3(grid_for(n)), dim3(kTPB), 0, c->stream, map, n_map, rows, cols, n,
                         c->ctl);
    else
      hipLaunchKernelGGL(k_remap_pairs<true>, dim3(grid_for((n + 3) / 4)), dim3(kTPB), 0, c->stream, map, n_map, rows,
                         cols, n, c->ctl);
  }
  sync_ctl(c);
  if (c->h_ctl->bad_id) throw Failure(G2N_E_ARG, "an id outside the map");
}

// grp (optional): rows / cols are a tile-local parse's group slots (G2N_RANGE_SLOTS) holding nnz entries
// in all; no map, no values (their order inside an owner is then slot order, which an unweighted slice
// CSR does not read)
void route_triplets(g2n_context* c, const int32_t* rows, const int32_t* cols, const void* data, uint64_t nnz,
                    int dtype, const uint32_t* map, uint64_t n_global, uint32_t n_ranks, int transposed,
                    int32_t* orows, int32_t* ocols, void* odata, uint32_t* starts, const GroupedCoo* grp = nullptr) {
  begin_call(c);
  if (n_ranks == 0 || n_ranks > 4096) throw Failure(G2N_E_ARG, "n_ranks out of range");
  if (nnz >= 0x7FFFFFFFull) throw Failure(G2N_E_UNSUPPORTED, "more than 2^31-1 triplets");
  if (grp && (map || data || n_ranks > kRouteMaxRanks))
    throw Failure(G2N_E_ARG, "group slots route coordinates only, without a map, to at most 256 ranks");
  if (n_ranks <= kRouteMaxRanks) {  // stable owner partition (g2n_route.hip)
    std::vector<uint64_t> hb(n_ranks + 1);
    for (uint32_t k = 0; k <= n_ranks; k++) hb[k] = ((uint64_t)k * n_global + n_ranks - 1) / n_ranks;
    auto* bounds = dget<uint64_t>(c, S_RBOUND, n_ranks + 1);
    G2N_HIP(hipMemcpyAsync(bounds, hb.data(), hb.size() * sizeof(uint64_t), hipMemcpyHostToDevice, c->stream));
    RouteSrc s{rows, cols, map, nnz, n_ranks, transposed, bounds};
    uint64_t n_blk = nnz ? (nnz + kRouteTile - 1) / kRouteTile : 0;
    if (grp && nnz) {  // every group's tiles (those past its count exit at once)
      s.gcount = grp->gcount;
      s.gcap = grp->gcap;
      s.tpg = (uint32_t)((grp->gcap + kRouteTile - 1) / kRouteTile);
      n_blk = grp->n_groups * s.tpg;
    }
    const uint32_t bits = n_ranks > 1 ? (uint32_t)bits_for(n_ranks) : 0u;
    if (n_blk) {
      auto* cnt = dget<uint32_t>(c, S_PCNT, (uint64_t)n_ranks * n_blk);
      auto* off = dget<uint32_t>(c, S_POFF, (uint64_t)n_ranks * n_blk);
      hipLaunchKernelGGL(k_route_count, dim3((unsigned)n_blk), dim3(kRouteTPB), 0, c->stream, s, bits, n_blk, cnt);
      scan_excl<uint32_t, uint32_t>(c, cnt, off, (uint64_t)n_ranks * n_blk);
      const size_t w = data ? dtype_size(dtype) : 0;
      const dim3 g((unsigned)n_blk), b(kRouteTPB);
      if (w == 8)
        hipLaunchKernelGGL(k_route_scatter<uint64_t>, g, b, 0, c->stream, s, bits, n_blk, (const uint32_t*)off,
                           (const uint64_t*)data, orows, ocols, (uint64_t*)odata);
      else if (w == 4)
        hipLaunchKernelGGL(k_route_scatter<uint32_t>, g, b, 0, c->stream, s, bits, n_blk, (const uint32_t*)off,
                           (const uint32_t*)data, orows, ocols, (uint32_t*)odata);
      else
        hipLaunchKernelGGL(k_route_scatter<uint8_t>, g, b, 0, c->stream, s, bits, n_blk, (const uint32_t*)off,
                           (const uint8_t*)data, orows, ocols, (uint8_t*)odata);
      hipLaunchKernelGGL(k_route_starts, dim3(grid_for(n_ranks + 1)), dim3(kTPB), 0, c->stream,
                         (const uint32_t*)off, n_blk, n_ranks, nnz, starts);
    } else {
      G2N_HIP(hipMemsetAsync(starts, 0, (n_ranks + 1) * sizeof(uint32_t), c->stream));
    }
    G2N_HIP(hipStreamSynchronize(c->stream));
    return;
  }
  auto* owner = dget<uint32_t>(c, S_KEYS0, nnz);
  auto* owner_s = dget<uint32_t>(c, S_KEYS1, nnz);
  auto* idx = dget<uint32_t>(c, S_VALS0, nnz);
  auto* perm = dget<uint32_t>(c, S_VALS1, nnz);
  if (nnz) {
    hipLaunchKernelGGL(k_route_keys, dim3(grid_for(nnz)), dim3(kTPB), 0, c->stream, rows, cols, nnz, map, n_global,
                       n_ranks, transposed, owner, idx);
    sort_pairs_u32<uint32_t>(c, owner, owner_s, idx, perm, nnz, bits_for(n_ranks));
    const size_t w = data ? dtype_size(dtype) : 0;
    const dim3 g(grid_for(nnz)), b(kTPB);
    if (w == 8)
      hipLaunchKernelGGL(k_route_gather<uint64_t>, g, b, 0, c->stream, rows, cols, (const uint64_t*)data, perm, nnz,
                         map, transposed, orows, ocols, (uint64_t*)odata);
    else if (w == 4)
      hipLaunchKernelGGL(k_route_gather<uint32_t>, g, b, 0, c->stream, rows, cols, (const uint32_t*)data, perm, nnz,
                         map, transposed, orows, ocols, (uint32_t*)odata);
    else
      hipLaunchKernelGGL(k_route_gather<uint8_t>, g, b, 0, c->stream, rows, cols, (const uint8_t*)data, perm, nnz,
                         map, transposed, orows, ocols, (uint8_t*)odata);
  }
  // rank starts from the sorted owners (the row-start kernels, n_ranks "rows")
  G2N_HIP(hipMemsetAsync(&c->ctl->row_gap, 0, sizeof(unsigned long long), c->stream));
  hipLaunchKernelGGL(k_row_bounds, dim3(grid_for(nnz + 1)), dim3(kTPB), 0, c->stream, owner_s, nnz, (uint64_t)n_ranks,
                     starts, c->ctl);
  hipLaunchKernelGGL(k_row_start, dim3(grid_for((uint64_t)n_ranks + 1)), dim3(kTPB), 0, c->stream, owner_s, nnz,
                     (uint64_t)n_ranks, starts, (const Ctl*)c->ctl);
  G2N_HIP(hipStreamSynchronize(c->stream));
}

// The CSR of a one-rank sharded decimal build straight from its range build's group slots (G2N_RANGE_SLOTS:
// with one rank every row is this rank's, so nothing routes and no stream-order COO is ever written) —
// the one-GPU partition (csr_partition over GroupedCoo).  n_entries: the entries the slots hold in all.
// G2N_E_UNSUPPORTED when the partition declines (an overfull bucket): the caller builds a stream COO.
void csr_from_group_slots(g2n_context* c, const GroupedCoo& g, uint64_t n_entries, int maxsym, uint64_t n_rows,
                          int dtype, g2n_result* R) {
  fill_defaults(R);
  begin_call(c);
  if (dtype < G2N_BOOL || dtype > G2N_FLOAT64) throw Failure(G2N_E_ARG, "unsupported dtype");
  if ((maxsym ? 2 : 1) * n_entries >= 0xFFFFFFFFull) throw Failure(G2N_E_UNSUPPORTED, "more than 2^32-1 elements");
  if (!n_entries || !n_rows || (c->test_flags & kTestNoBuckets))
    throw Failure(G2N_E_UNSUPPORTED, "group slots: no entries (the stream-order route)");
  R->dtype = dtype;
  R->index_width = 4;
  R->n_nodes = (int64_t)n_rows;
  c->gcoo = g;
  c->gcoo.active = true;
  bool ok = false;
  auto go = [&](auto tag) {
    using T = decltype(tag);
    ok = csr_partition<T>(c, g.rows, g.cols, n_entries, n_rows, !maxsym, R);
  };
  try {
    switch (dtype) {
      case G2N_BOOL: go(uint8_t{}); break;
      case G2N_INT8: go(int8_t{}); break;
      case G2N_INT32: go(int32_t{}); break;
      case G2N_FLOAT32: go(float{}); break;
      default: go(double{}); break;
    }
  } catch (...) {
    c->gcoo = GroupedCoo{};
    throw;
  }
  c->gcoo = GroupedCoo{};
  if (!ok) throw Failure(G2N_E_UNSUPPORTED, "group slots: the bucket partition declined (the stream-order route)");
  R->sum_sorted = R->sum_t_sorted = 1;
  finish_timings(c, R);
}

void csr_from_coo_pair(g2n_context* c, const int32_t* ar, const int32_t* ac, const void* ad, uint64_t an,
                       const int32_t* tr, const int32_t* tc, const void* td, uint64_t tn, int maxsym, int64_t base,
                       uint64_t n_rows, uint64_t n_cols, int dtype, int uniform, int force_unsorted, g2n_result* R) {
  fill_defaults(R);
  begin_call(c);
  if (dtype < G2N_BOOL || dtype > G2N_FLOAT64) throw Failure(G2N_E_ARG, "unsupported dtype");
  if (an + tn >= 0x7FFFFFFFull) throw Failure(G2N_E_UNSUPPORTED, "more than 2^31-1 entries");
  R->dtype = dtype;
  R->index_width = 4;
  R->n_nodes = (int64_t)n_rows;
  auto go = [&](auto tag) {
    using T = decltype(tag);
    if (uniform)
      assemble_pair_t<T, true>(c, ar, ac, (const T*)ad, an, tr, tc, (const T*)td, tn, maxsym != 0, base, n_rows,
                               force_unsorted, R);
    else
      assemble_pair_t<T, false>(c, ar, ac, (const T*)ad, an, tr, tc, (const T*)td, tn, maxsym != 0, base, n_rows,
                                force_unsorted, R);
  };
  switch (dtype) {
    case G2N_BOOL: go(uint8_t{}); break;
    case G2N_INT8: go(int8_t{}); break;
    case G2N_INT32: go(int32_t{}); break;
    case G2N_FLOAT32: go(float{}); break;
    default: go(double{}); break;
  }
  (void)n_cols;
  finish_timings(c, R);
}

}  // namespace g2n

// ------------------------------------------------------------------ C ABI --------
extern "C" {

g2n_context* g2n_context_create(int device) {
  try {
    return g2n::context_create(device);
  } catch (const g2n::Failure& f) {
    g2n::set_last_error(f.what());
  } catch (const std::exception& e) {
    g2n::set_last_error(e.what());
  }
  return nullptr;
}

void g2n_context_destroy(g2n_context* ctx) { g2n::context_destroy(ctx); }

void* g2n_context_stream(g2n_context* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int g2n_context_trim(g2n_context* ctx, const void* const* keep, uint64_t n_keep, uint64_t* freed) {
  if (!ctx || (n_keep && !keep)) {
    g2n::set_last_error("g2n_context_trim: null argument");
    return G2N_E_ARG;
  }
  try {
    std::lock_guard<std::mutex> lk(ctx->mu);
    G2N_HIP(hipSetDevice(ctx->device));
    G2N_HIP(hipStreamSynchronize(ctx->stream));
    uint64_t total = 0;
    for (int s = 0; s < g2n::S_NSLOTS; s++) {
      g2n::DevBuf& b = ctx->bufs[s];
      if (!b.p) continue;
      bool held = false;  // a buffer holding any kept pointer stays (a result the caller still reads)
      for (uint64_t k = 0; k < n_keep && !held; k++) {
        const uintptr_t p = (uintptr_t)keep[k], a = (uintptr_t)b.p;
        held = p && p >= a && p < a + b.cap;
      }
      if (held) continue;
      G2N_HIP(hipFree(b.p));
      total += b.cap;
      b.p = nullptr;
      b.cap = 0;
      ctx->scan_slot[s] = g2n::ScanSlot{};  // a later allocation at the same address must be cleared again
    }
    ctx->wenc = nullptr;
    ctx->gcoo = g2n::GroupedCoo{};
    ctx->slots = g2n::GroupedCoo{};
    if (freed) *freed = total;
    return G2N_OK;
  } catch (const g2n::Failure& f) {
    g2n::set_last_error(f.what());
    return f.status;
  }
}

int g2n_release_shared(int32_t device, uint64_t* freed) {
  g2n_context* c = nullptr;
  {
    std::lock_guard<std::mutex> lk(g2n::g_ctx_mu);
    auto it = g2n::g_ctx.find(device);
    if (it != g2n::g_ctx.end()) c = it->second;
  }
  if (freed) *freed = 0;
  if (!c) return G2N_OK;  // no host entry point has used this device yet: nothing cached
  return g2n_context_trim(c, nullptr, 0, freed);
}

int g2n_build_device(g2n_context* ctx, const void* d_input, size_t len, const g2n_options* opts, g2n_result* out) {
  if (!ctx || !opts || !out || (len && !d_input)) {
    g2n::set_last_error("g2n_build_device: null argument");
    return G2N_E_ARG;
  }
  try {
    std::lock_guard<std::mutex> lk(ctx->mu);
    g2n::enter_call(ctx);
    G2N_HIP(hipSetDevice(ctx->device));
    return g2n::run_pipeline(ctx, (const uint8_t*)d_input, len, opts, out);
  } catch (const g2n::Failure& f) {
    g2n::set_last_error(f.what());
    out->status = f.status;
    return f.status;
  } catch (const std::exception& e) {
    g2n::set_last_error(e.what());
    out->status = G2N_E_DEVICE;
    return G2N_E_DEVICE;
  }
}

int g2n_build_decimal_range(g2n_context* ctx, const void* d_input, size_t len, const g2n_options* opts,
                            int64_t* ev6, g2n_result* out) {
  if (!ctx || !opts || !out || !ev6 || (len && !d_input)) {
    g2n::set_last_error("g2n_build_decimal_range: null argument");
    return G2N_E_ARG;
  }
  if (opts->output != G2N_OUT_COO || opts->want_node_names || opts->bidirected || opts->strip_orientation ||
      (opts->weight_tag && *opts->weight_tag)) {
    g2n::set_last_error("g2n_build_decimal_range: COO output, no names, not bidirected, no weights, no strip");
    return G2N_E_ARG;
  }
  g2n_options o = *opts;
  o.range_s_base = 0;
  o.range_n_segments = 0;
  // sharded decimal ids, offset evidence instead of the check
  o.range_flags = G2N_RANGE_DECIMAL | G2N_RANGE_EVIDENCE | (opts->range_flags & (G2N_RANGE_NO_VALUES | G2N_RANGE_SLOTS));
  const int rc = g2n_build_device(ctx, d_input, len, &o, out);
  if (rc == G2N_OK) {
    ev6[0] = out->n_lines;
    ev6[1] = (int64_t)ctx->range_nseg;
    ev6[2] = out->n_edges;
    ev6[3] = out->n_records;
    ev6[4] = ctx->range_d;
    ev6[5] = (int64_t)ctx->range_vmax;
  }
  return rc;
}

int g2n_coo_to_csr_band(const void* rows, const void* cols, const void* data, int64_t nnz, int64_t n_rows,
                        int64_t n_cols, int32_t dtype, int32_t device, int32_t force_unsorted, g2n_result** out) {
  if (!out || force_unsorted < -1 || force_unsorted > 1) return G2N_E_ARG;
  *out = nullptr;
  try {
    return g2n::coo_to_csr(rows, cols, data, nnz, n_rows, n_cols, 4, dtype, device, 0, out, force_unsorted);
  } catch (const g2n::Failure& f) {
    g2n::set_last_error(f.what());
    return f.status;
  } catch (const std::exception& e) {
    g2n::set_last_error(e.what());
    return G2N_E_DEVICE;
  }
}

int g2n_coo_to_csr(const void* rows, const void* cols, const void* data, int64_t nnz, int64_t n_rows,
                   int64_t n_cols, int32_t index_width, int32_t dtype, int32_t device, uint32_t test_flags,
                   g2n_result** out) {
  if (!out) return G2N_E_ARG;
  *out = nullptr;
  try {
    return g2n::coo_to_csr(rows, cols, data, nnz, n_rows, n_cols, index_width, dtype, device, test_flags, out);
  } catch (const g2n::Failure& f) {
    g2n::set_last_error(f.what());
    return f.status;
  } catch (const std::exception& e) {
    g2n::set_last_error(e.what());
    return G2N_E_DEVICE;
  }
}

#define G2N_CTX_CALL(ctx, body)                          \
  do {                                                   \
    if (!(ctx)) {                                        \
      g2n::set_last_error("null context");               \
      return G2N_E_ARG;                                  \
    }                                                    \
    try {                                                \
      std::lock_guard<std::mutex> lk((ctx)->mu);         \
      g2n::enter_call(ctx);                              \
      G2N_HIP(hipSetDevice((ctx)->device));              \
      body;                                              \
    } catch (const g2n::Failure& f) {                    \
      g2n::set_last_error(f.what());                     \
      return f.status;                                   \
    } catch (const std::exception& e) {                  \
      g2n::set_last_error(e.what());                     \
      return G2N_E_DEVICE;                               \
    }                                                    \
  } while (0)

int g2n_dedup_keys(g2n_context* ctx, const uint8_t* d_blob, uint64_t blob_len, const int64_t* d_offsets, uint64_t n,
                   uint32_t* d_ids, uint32_t* d_first, uint64_t* n_distinct) {
  if (!n_distinct || (n && (!d_offsets || !d_ids || !d_first))) return G2N_E_ARG;
  G2N_CTX_CALL(ctx, *n_distinct = g2n::dedup_keys(ctx, d_blob, blob_len, d_offsets, n, d_ids, d_first));
  return G2N_OK;
}

int g2n_partition_keys(g2n_context* ctx, const uint8_t* d_blob, uint64_t blob_len, const int64_t* d_offsets,
                       uint64_t n, uint32_t n_ranks, uint8_t* d_out_blob, int64_t* d_out_offsets,
                       uint32_t* d_out_index, uint32_t* d_starts) {
  if (!d_starts || !d_out_offsets || !d_offsets || (n && (!d_out_index || (blob_len && (!d_blob || !d_out_blob)))))
    return G2N_E_ARG;
  G2N_CTX_CALL(ctx, g2n::partition_keys(ctx, d_blob, d_offsets, n, n_ranks, d_out_blob, d_out_offsets, d_out_index,
                                        d_starts));
  return G2N_OK;
}

int g2n_gather_keys(g2n_context* ctx, const uint8_t* d_blob, const int64_t* d_offsets, const uint32_t* d_index,
                    uint64_t n, uint8_t* d_out_blob, uint64_t out_cap, int64_t* d_out_offsets, uint64_t* out_len) {
  if (!out_len || !d_out_offsets || (n && (!d_offsets || !d_index || (out_cap && !d_out_blob)))) return G2N_E_ARG;
  G2N_CTX_CALL(ctx, *out_len = g2n::gather_keys(ctx, d_blob, d_offsets, d_index, n, d_out_blob, out_cap,
                                                d_out_offsets));
  return G2N_OK;
}

int g2n_keyset_create(g2n_context* ctx, g2n_keyset** out) {
  if (!ctx || !out) return G2N_E_ARG;
  *out = new g2n_keyset();
  (*out)->ctx = ctx;
  (*out)->device = ctx->device;
  return G2N_OK;
}

int g2n_keyset_add(g2n_keyset* ks, const uint8_t* d_blob, uint64_t blob_len, const int64_t* d_offsets, uint64_t n,
                   uint32_t* d_ids, uint64_t* n_total) {
  if (!ks || !n_total || (n && (!d_offsets || !d_ids || (blob_len && !d_blob)))) return G2N_E_ARG;
  g2n_context* ctx = ks->ctx;
  G2N_CTX_CALL(ctx, *n_total = g2n::keyset_add(ks, d_blob, d_offsets, n, d_ids));
  return G2N_OK;
}

int g2n_keyset_view(g2n_keyset* ks, const uint8_t** d_blob, const int64_t** d_offsets, uint64_t* n,
                    uint64_t* blob_len) {
  if (!ks || !d_blob || !d_offsets || !n || !blob_len) return G2N_E_ARG;
  if (!ks->offs) {
    g2n_context* ctx = ks->ctx;
    G2N_CTX_CALL(ctx, (void)g2n::keyset_add(ks, nullptr, nullptr, 0, nullptr));
  }
  *d_blob = ks->blob;
  *d_offsets = ks->offs;
  *n = ks->n;
  *blob_len = ks->blob_len;
  return G2N_OK;
}

void g2n_keyset_free(g2n_keyset* ks) {
  if (!ks) return;
  (void)hipSetDevice(ks->device);
  if (ks->table) (void)hipFree(ks->table);
  if (ks->blob) (void)hipFree(ks->blob);
  if (ks->offs) (void)hipFree(ks->offs);
  delete ks;
}

int g2n_order_keys(g2n_context* ctx, const uint32_t* d_first_of, const int64_t* d_src_idx, uint64_t nd,
                   const uint64_t* src_ends, uint32_t n_src, uint64_t* d_out) {
  if (!src_ends || (nd && (!d_first_of || !d_src_idx || !d_out))) return G2N_E_ARG;
  G2N_CTX_CALL(ctx, g2n::order_keys(ctx, d_first_of, d_src_idx, nd, src_ends, n_src, d_out));
  return G2N_OK;
}

int g2n_rank_keys(g2n_context* ctx, const uint64_t* d_keys, uint64_t n, const uint64_t* d_all,
                  const uint64_t* all_offsets, uint32_t n_ranks, uint32_t self_rank, int64_t* d_out) {
  if (!all_offsets || (n && (!d_keys || !d_out))) return G2N_E_ARG;
  G2N_CTX_CALL(ctx, g2n::rank_keys(ctx, d_keys, n, d_all, all_offsets, n_ranks, self_rank, d_out));
  return G2N_OK;
}

int g2n_remap_pairs(g2n_context* ctx, const uint32_t* d_map, uint64_t n_map, int32_t* d_rows, int32_t* d_cols,
                    uint64_t n) {
  if (n && (!d_map || !d_rows || !d_cols)) return G2N_E_ARG;
  G2N_CTX_CALL(ctx, g2n::remap_pairs(ctx, d_map, n_map, d_rows, d_cols, n));
  return G2N_OK;
}

int g2n_route_triplets(g2n_context* ctx, const int32_t* d_rows, const int32_t* d_cols, const void* d_data,
                       uint64_t nnz, int32_t dtype, const uint32_t* d_map, uint64_t n_global, uint32_t n_ranks,
                       int32_t transposed, int32_t* d_out_rows, int32_t* d_out_cols, void* d_out_data,
                       uint32_t* d_starts) {
  if (!d_starts || (nnz && (!d_rows || !d_cols || !d_data != !d_out_data || !d_out_rows || !d_out_cols)))
    return G2N_E_ARG;
  if (dtype < G2N_BOOL || dtype > G2N_FLOAT64) return G2N_E_ARG;
  G2N_CTX_CALL(ctx, g2n::route_triplets(ctx, d_rows, d_cols, d_data, nnz, dtype, d_map, n_global, n_ranks, transposed,
                                        d_out_rows, d_out_cols, d_out_data, d_starts));
  return G2N_OK;
}

int g2n_context_group_slots(g2n_context* ctx, const uint32_t** d_gcount, uint64_t* n_groups, uint64_t* gcap) {
  if (!ctx || !d_gcount || !n_groups || !gcap) return G2N_E_ARG;
  std::lock_guard<std::mutex> lk(ctx->mu);
  *d_gcount = ctx->slots.gcount;
  *n_groups = ctx->slots.gcount ? ctx->slots.n_groups : 0;
  *gcap = ctx->slots.gcount ? ctx->slots.gcap : 0;
  return G2N_OK;
}

int g2n_route_group_slots(g2n_context* ctx, const int32_t* d_rows, const int32_t* d_cols, const uint32_t* d_gcount,
                          uint64_t n_groups, uint64_t gcap, uint64_t nnz, uint64_t n_global, uint32_t n_ranks,
                          int32_t transposed, int32_t* d_out_rows, int32_t* d_out_cols, uint32_t* d_starts) {
  if (!d_starts || (nnz && (!d_rows || !d_cols || !d_gcount || !n_groups || !gcap || !d_out_rows || !d_out_cols)))
    return G2N_E_ARG;
  g2n::GroupedCoo g;
  g.rows = d_rows;
  g.cols = d_cols;
  g.gcount = d_gcount;
  g.n_groups = n_groups;
  g.gcap = gcap;
  G2N_CTX_CALL(ctx, g2n::route_triplets(ctx, d_rows, d_cols, nullptr, nnz, G2N_FLOAT64, nullptr, n_global, n_ranks,
                                        transposed, d_out_rows, d_out_cols, nullptr, d_starts, &g));
  return G2N_OK;
}

int g2n_csr_from_group_slots(g2n_context* ctx, const int32_t* d_rows, const int32_t* d_cols, const uint32_t* d_gcount,
                             uint64_t n_groups, uint64_t gcap, uint64_t nnz, int32_t maxsym, uint64_t n_rows,
                             int32_t dtype, g2n_result* out) {
  if (!out || !d_rows || !d_cols || !d_gcount || !n_groups || !gcap) return G2N_E_ARG;
  g2n::GroupedCoo g;
  g.rows = d_rows;
  g.cols = d_cols;
  g.gcount = d_gcount;
  g.n_groups = n_groups;
  g.gcap = gcap;
  G2N_CTX_CALL(ctx, g2n::csr_from_group_slots(ctx, g, nnz, maxsym, n_rows, dtype, out));
  return G2N_OK;
}

int g2n_csr_from_coo_pair(g2n_context* ctx, const int32_t* a_rows, const int32_t* a_cols, const void* a_data,
                          uint64_t a_nnz, const int32_t* t_rows, const int32_t* t_cols, const void* t_data,
                          uint64_t t_nnz, int32_t maxsym, int64_t row_base, uint64_t n_rows, uint64_t n_cols,
                          int32_t dtype, int32_t uniform, int32_t force_unsorted, g2n_result* out) {
  if (!out) return G2N_E_ARG;
  G2N_CTX_CALL(ctx, g2n::csr_from_coo_pair(ctx, a_rows, a_cols, a_data, a_nnz, t_rows, t_cols, t_data,
                                           maxsym ? t_nnz : 0, maxsym, row_base, n_rows, n_cols, dtype, uniform,
                                           force_unsorted, out));
  return G2N_OK;
}

int g2n_count_device(g2n_context* ctx, const void* d_input, size_t len, int64_t* out4) {
  if (!out4 || (len && !d_input)) return G2N_E_ARG;
  G2N_CTX_CALL(ctx, {
    const uint64_t n_tiles = (len + g2n::kTile - 1) / g2n::kTile;
    g2n::TileCnt tot{};
    if (n_tiles) {
      auto* tcnt = g2n::dget<g2n::TileCnt>(ctx, g2n::S_TILE_CNT, n_tiles + 1);
      const uint64_t n_parts = (n_tiles + g2n::kStructChunk - 1) / g2n::kStructChunk;
      auto* part = g2n::dget<g2n::TileCnt>(ctx, g2n::S_TEMP, n_parts + 1);
      hipLaunchKernelGGL(g2n::k_tile_count_r, dim3((unsigned)n_tiles), dim3(g2n::kK1TPB), 0, ctx->stream,
                         (const uint8_t*)d_input, (uint64_t)len, 1u, 2u, tcnt);
      hipLaunchKernelGGL(g2n::k_struct_reduce<g2n::TileCnt>, dim3((unsigned)n_parts), dim3(256), 0, ctx->stream,
                         (const g2n::TileCnt*)tcnt, n_tiles, part);
      hipLaunchKernelGGL(g2n::k_struct_scan_parts<g2n::TileCnt>, dim3(1), dim3(256), 0, ctx->stream, part, n_parts,
                         part + n_parts);
      tot = g2n::read_dev(ctx, part + n_parts);
    }
    out4[0] = (int64_t)tot.lines;
    out4[1] = (int64_t)tot.segs;
    out4[2] = (int64_t)tot.edges;
    out4[3] = (int64_t)tot.recs;
  });
  return G2N_OK;
}

int g2n_device_memory(int32_t device, uint64_t* free_bytes, uint64_t* total_bytes) {
  if (!free_bytes || !total_bytes) return G2N_E_ARG;
  *free_bytes = *total_bytes = 0;
  int cur = 0;
  if (hipGetDevice(&cur) != hipSuccess || hipSetDevice(device) != hipSuccess) {
    (void)hipGetLastError();
    g2n::set_last_error("g2n_device_memory: no such HIP device");
    return G2N_E_DEVICE;
  }
  size_t f = 0, t = 0;
  const hipError_t e = hipMemGetInfo(&f, &t);
  (void)hipSetDevice(cur);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    g2n::set_last_error(std::string("hipMemGetInfo failed: ") + hipGetErrorString(e));
    return G2N_E_DEVICE;
  }
  *free_bytes = f;
  *total_bytes = t;
  return G2N_OK;
}

int g2n_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

}  // extern "C"
