// g2n_internal.h — host-side plumbing shared by g2n_pipeline.hip, g2n_host.cpp and g2n_ingest.cpp.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <functional>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/g2n.h"

namespace g2n {

// Internal failure carrying a G2N_E_* status and a message for g2n_last_error().
struct Failure : std::runtime_error {
  int status;
  Failure(int s, const std::string& m) : std::runtime_error(m), status(s) {}
};

void set_last_error(const std::string& msg);

// Host threads for ingest / download (G2N_HOST_THREADS, default min(16, cores)).
int host_threads();

// Runs body(i) for i in [0, n) on up to T threads; the first exception is rethrown.
void parallel_for(size_t n, int T, const std::function<void(size_t)>& body);

// Large host buffer without value-initialisation: big allocations are 2 MiB aligned, advised
// for transparent huge pages and faulted in by host_threads() threads before a DMA lands in
// them (a fresh pageable destination otherwise caps D2H at the page-fault rate).
struct HostBuf {
  uint8_t* p = nullptr;
  size_t n = 0;
  HostBuf() = default;
  HostBuf(const HostBuf&) = delete;
  HostBuf& operator=(const HostBuf&) = delete;
  HostBuf(HostBuf&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
  HostBuf& operator=(HostBuf&& o) noexcept {
    if (this != &o) {
      reset();
      p = o.p;
      n = o.n;
      o.p = nullptr;
      o.n = 0;
    }
    return *this;
  }
  void reset();
  ~HostBuf();
  uint8_t* alloc(size_t bytes);  // discards old contents; returns p (never null)
  uint8_t* data() const { return p; }
};

// Host-side result storage: g2n_result plus the buffers its pointers refer to.
struct HostResult {
  g2n_result r;
  HostBuf detail, blob, rows, cols, indptr, indices, data, offs;
};

// Frees big host buffers on a detached thread (unmapping GBs of touched pages costs ~0.1 s/GB).
void free_later(std::vector<HostBuf>&& bufs);

HostResult* new_host_result();
void fill_defaults(g2n_result* r);

// Writes input bytes [off, off + len) to dst (a pinned staging slot).  Called concurrently
// from several threads with disjoint ranges; throws Failure on error.
using FillFn = std::function<void(size_t off, uint8_t* dst, size_t len)>;

// Copies len input bytes produced by `fill` into device memory d (on `device`) through the
// per-device pinned staging ring: host threads fill 16 MiB slots and issue async H2D copies on
// their own streams, so reading / copying overlaps the DMA.  Returns after every copy landed.
void staged_upload(int device, uint8_t* d, size_t len, const FillFn& fill);

// Runs the GPU pipeline on len input bytes delivered by `fill` (staged into HBM) and
// downloads the outputs.  read_ms = host time spent before the call (read / inflate).
int build_host_fill(size_t len, const FillFn& fill, const g2n_options* opts, g2n_result** out, double read_ms);
int build_host(const void* buf, size_t len, const g2n_options* opts, g2n_result** out, double read_ms);

// Parallel multi-member gunzip.  Members are found by their header bytes and inflated
// speculatively on host_threads() threads; the chain of members from byte 0 (zero padding
// between members skipped, gzip.py _read_eof) is then walked in order.  Returns false when
// the input is not a clean chain of valid members (bad magic, trailing garbage, corrupt or
// truncated data): the caller then runs the serial gunzip, which raises the exact error.
struct Inflated {
  std::vector<HostBuf> parts;
  std::vector<size_t> start;  // output offset of each part (+ total at the end)
  size_t total = 0;
  int members = 0;
};
// Runs f; a Failure / bad_alloc / std::exception becomes its status + g2n_last_error().
int guarded(const std::function<int()>& f);
bool gunzip_parallel(const uint8_t* in, size_t n, Inflated& out);
// One gzip member spanning the whole file (zero padding after it allowed), inflated chunk-parallel
// (g2n_pinflate.cpp); chunk_bytes 0 = sized for the host threads.  false = declined (not one
// clean member, or anything the decoder refuses): the caller runs the member-chain readers.
bool gunzip_chunked(const uint8_t* in, size_t n, size_t chunk_bytes, Inflated& out);
// One member of a BGZF chain: its deflate data z[in_off, in_off + in_len), its output
// [out_off, out_off + out_len) (ISIZE) and the trailer's CRC-32.
struct ZMember {
  unsigned long long in_off, out_off;
  uint32_t in_len, out_len, crc, pad_;
};
// A clean BGZF chain (every member's size from its 'BC' subfield, members back to back, no
// other header fields, ISIZE <= 64 KiB): true with the members and the total output size.
bool bgzf_members(const uint8_t* in, size_t n, std::vector<ZMember>& out, size_t* total_out);
// g2n_build_from_path's ".gz" path for a BGZF chain: the compressed bytes to the GPU, the members
// inflated there (g2n_inflate.hip), then the build.  kBgzfFallback: a member did not inflate
// cleanly — the caller reads the file with the host readers instead.
constexpr int kBgzfFallback = -1;
constexpr uint32_t kTestHostInflate = G2N_TEST_HOST_INFLATE;  // BGZF read by the host readers
int build_host_bgzf(const uint8_t* z, size_t zlen, const std::vector<ZMember>& members, size_t total_out,
                    const g2n_options* opts, g2n_result** out, double read_ms);
// gzip.open's reader restated (serial, exact errors): false with *sub = 1 BadGzipFile,
// 2 EOFError, 3 zlib.error, 4 BadGzipFile (CRC / length) and *msg = the exception's message;
// `out` then holds the bytes the reference's reader returned before raising (not cut to lines).
bool gunzip_exact(const uint8_t* in, size_t n, Inflated& out, int* sub, std::string* msg);

// convert CLI writers (g2n_writers.cpp)
int write_npz(const std::string& path, int n, const char* const* names, const uint8_t* const* heads,
              const uint64_t* head_lens, const void* const* datas, const uint64_t* data_lens, int level);
int write_node_map(const std::string& path, const uint8_t* blob, const int64_t* offs, uint64_t n);
int64_t first_bad_utf8(const uint8_t* blob, const int64_t* offs, uint64_t n);

}  // namespace g2n
