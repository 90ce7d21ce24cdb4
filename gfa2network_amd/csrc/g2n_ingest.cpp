// g2n_ingest.cpp — host ingest for the end-to-end entry points: raw GFA bytes into HBM, results
// back to host memory.
//
//   * staged_upload: a per-device ring of pinned 16 MiB slots; host threads fill slots (pread
//     from the page cache, or copies out of inflated members) and issue async H2D copies on
//     their own streams, so the reads overlap the DMA (north_star: "raw GFA bytes are staged
//     into HBM in pinned async chunks").  Measured on the MI355X host
//     (tools/microbench/xfer.hip, profiles/r01/xfer.jsonl): 4 threads reach 50 GB/s from
//     memory, 38 GB/s from the page cache; a single pageable hipMemcpy gets 21 GB/s.
//   * HostBuf: result buffers faulted in by parallel threads before the D2H copy lands
//     (an untouched pageable destination caps D2H at 13 GB/s, a touched one reaches 47 GB/s).
//   * gunzip: gzip.open's reader (CPython 3.10 Lib/gzip.py _GzipReader, which
//     gfa2network/parser.py:108-109 uses) restated with zlib raw inflate — the exact errors —
//     and a parallel fast path for multi-member files (BGZF, pigz -i / concatenated members,
//     the C4 64 MiB members): every member start is found from its header bytes and inflated
//     speculatively on its own thread, then the member chain is walked in file order.
#include <errno.h>
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <exception>
#include <map>
#include <mutex>
#include <thread>

#include "g2n_internal.h"

namespace g2n {

int host_threads() {
  static int t = [] {
    const char* v = std::getenv("G2N_HOST_THREADS");
    int n = v ? std::atoi(v) : 0;
    if (n <= 0) {
      n = (int)std::thread::hardware_concurrency();
      n = std::max(1, std::min(16, n));
    }
    return n;
  }();
  return t;
}

// Runs body(i) for i in [0, n) on up to T threads; the first exception is rethrown.
void parallel_for(size_t n, int T, const std::function<void(size_t)>& body) {
  if (n == 0) return;
  T = (int)std::min<size_t>((size_t)std::max(T, 1), n);
  if (T == 1) {
    for (size_t i = 0; i < n; i++) body(i);
    return;
  }
  std::atomic<size_t> next{0};
  std::exception_ptr err;
  std::mutex mu;
  std::vector<std::thread> th;
  for (int t = 0; t < T; t++)
    th.emplace_back([&] {
      try {
        for (size_t i; (i = next.fetch_add(1)) < n;) body(i);
      } catch (...) {
        std::lock_guard<std::mutex> lk(mu);
        if (!err) err = std::current_exception();
        next = n;
      }
    });
  for (auto& x : th) x.join();
  if (err) std::rethrow_exception(err);
}

// ------------------------------------------------------------------ HostBuf ------------
static constexpr size_t kHuge = (size_t)2 << 20;

HostBuf::~HostBuf() { free(p); }

void HostBuf::reset() {
  free(p);
  p = nullptr;
  n = 0;
}

uint8_t* HostBuf::alloc(size_t bytes) {
  free(p);
  p = nullptr;
  n = bytes;
  const size_t want = bytes ? bytes : 1;
  if (want < ((size_t)64 << 20)) {
    p = (uint8_t*)malloc(want);
    if (!p) throw Failure(G2N_E_NOMEM, "host allocation of " + std::to_string(want) + " bytes failed");
    return p;
  }
  const size_t al = (want + kHuge - 1) & ~(kHuge - 1);
  void* q = nullptr;
  if (posix_memalign(&q, kHuge, al) != 0 || !q)
    throw Failure(G2N_E_NOMEM, "host allocation of " + std::to_string(al) + " bytes failed");
  (void)madvise(q, al, MADV_HUGEPAGE);
  p = (uint8_t*)q;
  // fault the pages in on all host threads (one write per 4 KiB page)
  const size_t pieces = al / kHuge;
  uint8_t* base = p;
  parallel_for(pieces, host_threads(), [base](size_t i) {
    volatile uint8_t* b = base + i * kHuge;
    for (size_t o = 0; o < kHuge; o += 4096) b[o] = 0;
  });
  return p;
}

void free_later(std::vector<HostBuf>&& bufs) {
  if (bufs.empty()) return;
  auto* owned = new std::vector<HostBuf>(std::move(bufs));
  try {
    std::thread([owned] { delete owned; }).detach();
  } catch (...) {
    delete owned;
  }
}

// ------------------------------------------------------------- staged upload ------------
namespace {
constexpr size_t kSlot = (size_t)16 << 20;

struct Stager {
  int device = 0;
  int T = 0;
  std::mutex mu;
  std::vector<uint8_t*> slots;  // 2 per thread
  std::vector<hipStream_t> streams;
  std::vector<hipEvent_t> events;  // 2 per thread
};

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw Failure(G2N_E_DEVICE, std::string(what) + " failed: " + hipGetErrorString(e));
}

Stager* stager_for(int device) {
  static std::mutex g_mu;
  static std::map<int, Stager*> g;
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g.find(device);
  if (it != g.end()) return it->second;
  auto* s = new Stager();
  s->device = device;
  s->T = std::max(1, std::min(8, host_threads()));
  hip_check(hipSetDevice(device), "hipSetDevice");
  s->slots.resize(2 * s->T);
  s->events.resize(2 * s->T);
  s->streams.resize(s->T);
  for (auto& p : s->slots) hip_check(hipHostMalloc((void**)&p, kSlot, hipHostMallocDefault), "hipHostMalloc");
  for (auto& e : s->events) hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
  for (auto& st : s->streams) hip_check(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate");
  g[device] = s;
  return s;
}
}  // namespace

void staged_upload(int device, uint8_t* d, size_t len, const FillFn& fill) {
  if (len == 0) return;
  Stager* s = stager_for(device);
  std::lock_guard<std::mutex> lk(s->mu);
  const size_t nchunks = (len + kSlot - 1) / kSlot;
  const int T = (int)std::min<size_t>((size_t)s->T, nchunks);
  std::atomic<size_t> next{0};
  std::exception_ptr err;
  std::mutex emu;
  std::vector<std::thread> th;
  for (int t = 0; t < T; t++)
    th.emplace_back([&, t] {
      try {
        hip_check(hipSetDevice(device), "hipSetDevice");
        hipStream_t st = s->streams[t];
        bool used[2] = {false, false};
        int k = 0;
        try {
          for (size_t i; (i = next.fetch_add(1)) < nchunks;) {
            const size_t off = i * kSlot, n = std::min(kSlot, len - off);
            uint8_t* slot = s->slots[2 * t + k];
            hipEvent_t ev = s->events[2 * t + k];
            if (used[k]) hip_check(hipEventSynchronize(ev), "hipEventSynchronize");
            fill(off, slot, n);
            hip_check(hipMemcpyAsync(d + off, slot, n, hipMemcpyHostToDevice, st), "hipMemcpyAsync H2D");
            hip_check(hipEventRecord(ev, st), "hipEventRecord");
            used[k] = true;
            k ^= 1;
          }
        } catch (...) {
          (void)hipStreamSynchronize(st);  // never leave a DMA reading a slot we may reuse
          throw;
        }
        hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
      } catch (...) {
        std::lock_guard<std::mutex> g(emu);
        if (!err) err = std::current_exception();
        next = nchunks;
      }
    });
  for (auto& x : th) x.join();
  if (err) std::rethrow_exception(err);
}

// ------------------------------------------------------------------ gunzip --------------
// Growable inflate output (realloc of large blocks remaps, it does not copy).
namespace {
struct Grow {
  uint8_t* p = nullptr;
  size_t n = 0, cap = 0;
  ~Grow() { free(p); }
  void reserve(size_t want) {
    if (want <= cap) return;
    size_t c = std::max(want, cap + cap / 2);
    auto* q = (uint8_t*)realloc(p, c);
    if (!q) throw Failure(G2N_E_NOMEM, "host allocation failed while inflating");
    p = q;
    cap = c;
  }
};

// gzip member header per zlib's gzip wrapper rules (the fast path only; the exact reader
// below re-checks everything the way gzip.py does).  Candidate = 1f 8b 08, reserved flag bits 0.
inline bool candidate_at(const uint8_t* in, size_t n, size_t p) {
  return p + 18 <= n && in[p] == 0x1F && in[p + 1] == 0x8B && in[p + 2] == 8 && (in[p + 3] & 0xE0) == 0;
}

// Inflates the gzip member at in[start..n) with zlib's gzip wrapper (CRC + ISIZE checked).
// Returns the end offset, or 0 on any failure / when `dead` became set (speculation lost).
size_t inflate_member(const uint8_t* in, size_t n, size_t start, Grow& out, const std::atomic<bool>* dead) {
  z_stream zs;
  memset(&zs, 0, sizeof(zs));
  if (inflateInit2(&zs, 16 + MAX_WBITS) != Z_OK) return 0;
  size_t fed = start;
  out.n = 0;
  out.reserve(std::min<size_t>((size_t)256 << 20, std::max<size_t>((size_t)1 << 20, 4 * std::min<size_t>(n - start, (size_t)64 << 20))));
  size_t end = 0;
  size_t since_check = 0;
  for (;;) {
    if (zs.avail_in == 0) {
      if (fed >= n) break;  // truncated
      const size_t take = std::min<size_t>(n - fed, (size_t)1 << 30);
      zs.next_in = const_cast<Bytef*>(in + fed);
      zs.avail_in = (uInt)take;
      fed += take;
    }
    if (out.cap - out.n < ((size_t)1 << 20)) out.reserve(out.cap + ((size_t)8 << 20));
    const size_t room = std::min<size_t>(out.cap - out.n, (size_t)1 << 30);
    zs.next_out = out.p + out.n;
    zs.avail_out = (uInt)room;
    const int rc = inflate(&zs, Z_NO_FLUSH);
    const size_t produced = room - zs.avail_out;
    out.n += produced;
    if (rc == Z_STREAM_END) {
      end = (size_t)(zs.next_in - in);
      break;
    }
    if (rc != Z_OK && rc != Z_BUF_ERROR) break;
    if (rc == Z_BUF_ERROR && zs.avail_in == 0 && fed >= n) break;
    since_check += produced;
    if (since_check >= ((size_t)8 << 20)) {
      since_check = 0;
      if (dead && dead->load(std::memory_order_relaxed)) break;
    }
  }
  inflateEnd(&zs);
  return end;
}
}  // namespace

bool gunzip_parallel(const uint8_t* in, size_t n, Inflated& out) {
  out = Inflated();
  if (n == 0) {
    out.start.push_back(0);
    return true;  // gzip.open on an empty file reads b""
  }
  if (!candidate_at(in, n, 0)) return false;
  const int T = host_threads();
  // 1. member candidates, in file order
  const size_t span = (size_t)16 << 20;
  const size_t nspan = (n + span - 1) / span;
  std::vector<std::vector<size_t>> found(nspan);
  parallel_for(nspan, T, [&](size_t s) {
    const size_t lo = s * span, hi = std::min(n, lo + span);
    for (size_t p = lo; p < hi;) {
      const void* q = memchr(in + p, 0x1F, hi - p);
      if (!q) break;
      p = (size_t)((const uint8_t*)q - in);
      if (candidate_at(in, n, p)) found[s].push_back(p);
      p++;
    }
  });
  std::vector<size_t> cand;
  for (auto& f : found) cand.insert(cand.end(), f.begin(), f.end());
  found.clear();
  const size_t nc = cand.size();
  if (nc > ((size_t)1 << 22)) return false;  // pathological; let the serial reader handle it
  // few member candidates in a large file: most likely one big member, which the member-level
  // speculation below would inflate on one thread — split its deflate stream instead
  if (n >= ((size_t)64 << 20) && nc <= 64) {
    // the chunk-parallel decode holds ~15x the compressed size of buffers at once: when they
    // cannot be had it declines, and the member-chain / exact readers below inflate the file
    bool ok = false;
    try {
      ok = gunzip_chunked(in, n, 0, out);
    } catch (const Failure& f) {
      if (f.status != G2N_E_NOMEM) throw;
      out = Inflated{};
    } catch (const std::bad_alloc&) {
      out = Inflated{};
    }
    if (ok) return true;
  }

  // 2. speculative inflate of every candidate; the chain walker marks candidates that fall
  //    inside a resolved member as dead, which stops (or skips) their speculation
  std::vector<Grow> res(nc);
  std::vector<size_t> ends(nc, 0);
  std::unique_ptr<std::atomic<bool>[]> dead(new std::atomic<bool>[nc]);
  std::unique_ptr<std::atomic<int>[]> state(new std::atomic<int>[nc]);  // 0 pending, 1 done
  for (size_t i = 0; i < nc; i++) {
    dead[i] = false;
    state[i] = 0;
  }
  std::mutex mu;
  std::condition_variable cv;
  std::atomic<size_t> next{0};
  std::atomic<bool> stop{false};
  std::vector<std::thread> th;
  std::exception_ptr err;
  for (int t = 0; t < std::max(1, T); t++)
    th.emplace_back([&] {
      try {
        for (size_t i; !stop.load() && (i = next.fetch_add(1)) < nc;) {
          size_t e = 0;
          if (!dead[i].load()) e = inflate_member(in, n, cand[i], res[i], &dead[i]);
          {
            std::lock_guard<std::mutex> lk(mu);
            ends[i] = e;
            state[i] = 1;
          }
          cv.notify_all();
        }
      } catch (...) {
        std::lock_guard<std::mutex> lk(mu);
        if (!err) err = std::current_exception();
        stop = true;
        cv.notify_all();
      }
    });

  // 3. walk the member chain from byte 0
  bool ok = true;
  size_t pos = 0, ci = 0;
  std::vector<size_t> chain;
  while (ok) {
    while (ci < nc && cand[ci] < pos) dead[ci++] = true;
    if (ci >= nc || cand[ci] != pos) {
      ok = false;
      break;
    }
    {
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return state[ci].load() == 1 || stop.load(); });
      if (state[ci].load() != 1 || ends[ci] == 0) {
        ok = false;
        break;
      }
    }
    chain.push_back(ci);
    pos = ends[ci];
    ci++;
    while (pos < n && in[pos] == 0) pos++;  // zero padding (gzip.py _read_eof)
    if (pos >= n) break;
  }
  stop = true;
  for (size_t i = 0; i < nc; i++) dead[i] = true;
  for (auto& x : th) x.join();
  if (err) std::rethrow_exception(err);
  if (!ok) return false;

  out.members = (int)chain.size();
  size_t total = 0;
  for (size_t k : chain) {
    out.start.push_back(total);
    total += res[k].n;
    HostBuf b;
    b.p = res[k].p;  // adopt the realloc'd block (HostBuf frees with free())
    b.n = res[k].n;
    res[k].p = nullptr;
    out.parts.push_back(std::move(b));
  }
  out.start.push_back(total);
  out.total = total;
  return true;
}

// ------------------------------------------------------------- BGZF chains ---------------
bool bgzf_members(const uint8_t* in, size_t n, std::vector<ZMember>& out, size_t* total_out) {
  out.clear();
  size_t pos = 0, total = 0;
  auto u16 = [&](size_t p) { return (uint32_t)in[p] | ((uint32_t)in[p + 1] << 8); };
  auto u32 = [&](size_t p) { return u16(p) | (u16(p + 2) << 16); };
  while (pos < n) {
    if (n - pos < 26 || in[pos] != 0x1F || in[pos + 1] != 0x8B || in[pos + 2] != 8 || in[pos + 3] != 4)
      return false;  // FEXTRA only: bgzip's header
    const size_t xlen = u16(pos + 10);
    if (n - pos < 12 + xlen + 8) return false;
    size_t bsize = 0;
    for (size_t q = pos + 12; q + 4 <= pos + 12 + xlen;) {  // extra subfields: SI1 SI2 SLEN data
      const size_t slen = u16(q + 2);
      if (in[q] == 66 && in[q + 1] == 67 && slen == 2 && q + 6 <= pos + 12 + xlen) bsize = u16(q + 4) + 1;
      q += 4 + slen;
    }
    if (!bsize || bsize < 12 + xlen + 8 || bsize > n - pos) return false;
    ZMember m{};
    m.in_off = pos + 12 + xlen;
    m.in_len = (uint32_t)(bsize - 12 - xlen - 8);
    m.crc = u32(pos + bsize - 8);
    m.out_len = u32(pos + bsize - 4);
    if (m.out_len > 65536) return false;
    m.out_off = total;
    total += m.out_len;
    out.push_back(m);
    pos += bsize;
  }
  *total_out = total;
  return !out.empty() && total > 0;
}

// ------------------------------------------------- gzip.open's reader, restated ---------
// CPython 3.10 Lib/gzip.py _GzipReader: _read_gzip_header (:430-462), read (:464-510),
// _read_eof (:518-537); raw deflate as zlib.decompressobj(-MAX_WBITS).  Errors carry the
// exception gzip.py raises: sub 1 BadGzipFile, 2 EOFError, 3 zlib.error, 4 BadGzipFile (CRC /
// length).  Used when the parallel path declines (and so for every malformed file).
static std::string py_bytes_repr(const uint8_t* b, size_t n) {
  const bool sq = memchr(b, '\'', n) != nullptr, dq = memchr(b, '"', n) != nullptr;
  const char quote = (sq && !dq) ? '"' : '\'';
  std::string s = "b";
  s += quote;
  for (size_t i = 0; i < n; i++) {
    const uint8_t c = b[i];
    char tmp[8];
    if (c == (uint8_t)quote || c == '\\') {
      s += '\\';
      s += (char)c;
    } else if (c == '\t') {
      s += "\\t";
    } else if (c == '\n') {
      s += "\\n";
    } else if (c == '\r') {
      s += "\\r";
    } else if (c < 0x20 || c >= 0x7F) {
      snprintf(tmp, sizeof(tmp), "\\x%02x", c);
      s += tmp;
    } else {
      s += (char)c;
    }
  }
  s += quote;
  return s;
}

// Bytes gzip.py's reader has returned for one member's deflate data starting at `dstart` when
// zlib.error is raised: _GzipReader.read(8192) (io.BufferedReader's refill size) feeds
// decompress(self._fp.read(8192), 8192) — one inflate(Z_SYNC_FLUSH) with <= 8192 bytes of input
// and 8192 of output room, the unconsumed tail prepended for the next call — and the output of
// the call that fails is discarded with it (zlibmodule.c).
static size_t delivered_before_zlib_error(const uint8_t* in, size_t n, size_t dstart) {
  z_stream zs;
  memset(&zs, 0, sizeof(zs));
  if (inflateInit2(&zs, -MAX_WBITS) != Z_OK) return 0;
  uint8_t buf[8192];
  size_t p = dstart, delivered = 0;
  while (p < n) {
    const size_t take = std::min<size_t>(n - p, sizeof(buf));
    zs.next_in = const_cast<Bytef*>(in + p);
    zs.avail_in = (uInt)take;
    zs.next_out = buf;
    zs.avail_out = sizeof(buf);
    const int rc = inflate(&zs, Z_SYNC_FLUSH);
    if (rc != Z_OK && rc != Z_BUF_ERROR && rc != Z_STREAM_END) break;
    delivered += sizeof(buf) - zs.avail_out;
    p += take - zs.avail_in;
    if (rc == Z_STREAM_END || (rc == Z_BUF_ERROR && zs.avail_in == take)) break;  // no progress
  }
  inflateEnd(&zs);
  return delivered;
}

bool gunzip_exact(const uint8_t* in, size_t n, Inflated& out, int* sub, std::string* msg) {
  static const char* kEOF = "Compressed file ended before the end-of-stream marker was reached";
  out = Inflated();
  size_t pos = 0, total = 0;
  Grow g;  // the current member's output
  auto keep = [&](size_t len) {  // the member's first len bytes become a part of the output
    out.start.push_back(total);
    total += len;
    HostBuf b;
    b.p = g.p;
    b.n = len;
    g.p = nullptr;
    g.n = g.cap = 0;
    out.parts.push_back(std::move(b));
  };
  auto fail = [&](int s, const std::string& m, size_t member_bytes) {
    // the prefix the reference's line loop saw before the exception: finished members plus
    // what this member had delivered (out.total; the caller cuts it to whole lines)
    if (member_bytes) keep(member_bytes);
    out.start.push_back(total);
    out.total = total;
    *sub = s;
    *msg = m;
    return false;
  };
  for (;;) {
    if (pos >= n) break;  // magic == b"": no further member
    const size_t ml = std::min<size_t>(2, n - pos);
    if (ml < 2 || in[pos] != 0x1F || in[pos + 1] != 0x8B)
      return fail(1, "Not a gzipped file (" + py_bytes_repr(in + pos, ml) + ")", 0);
    pos += 2;
    if (n - pos < 8) return fail(2, kEOF, 0);
    const uint8_t method = in[pos], flag = in[pos + 1];
    pos += 8;
    if (method != 8) return fail(1, "Unknown compression method", 0);
    if (flag & 4) {  // FEXTRA
      if (n - pos < 2) return fail(2, kEOF, 0);
      const size_t xlen = (size_t)in[pos] | ((size_t)in[pos + 1] << 8);
      pos += 2;
      if (n - pos < xlen) return fail(2, kEOF, 0);
      pos += xlen;
    }
    for (int f : {8, 16}) {  // FNAME, FCOMMENT: NUL-terminated, EOF ends them silently
      if (flag & f)
        while (pos < n && in[pos++] != 0) {
        }
    }
    if (flag & 2) {  // FHCRC
      if (n - pos < 2) return fail(2, kEOF, 0);
      pos += 2;
    }
    z_stream zs;
    memset(&zs, 0, sizeof(zs));
    if (inflateInit2(&zs, -MAX_WBITS) != Z_OK) return fail(3, "Error -2 while preparing to decompress data", 0);
    const size_t dstart = pos;
    size_t fed = pos;
    uLong crc = crc32(0L, Z_NULL, 0);
    bool ended = false;
    g.n = 0;
    g.reserve((size_t)1 << 22);
    for (;;) {
      if (zs.avail_in == 0) {
        if (fed >= n) break;
        const size_t take = std::min<size_t>(n - fed, (size_t)1 << 30);
        zs.next_in = const_cast<Bytef*>(in + fed);
        zs.avail_in = (uInt)take;
        fed += take;
      }
      if (g.cap - g.n < ((size_t)1 << 20)) g.reserve(g.cap + ((size_t)8 << 20));
      const size_t room = std::min<size_t>(g.cap - g.n, (size_t)1 << 30);
      zs.next_out = g.p + g.n;
      zs.avail_out = (uInt)room;
      const int rc = inflate(&zs, Z_NO_FLUSH);
      const size_t produced = room - zs.avail_out;
      crc = crc32(crc, g.p + g.n, (uInt)produced);
      g.n += produced;
      if (rc == Z_STREAM_END) {
        ended = true;
        break;
      }
      if (rc == Z_OK || rc == Z_BUF_ERROR) continue;
      std::string m = zs.msg ? zs.msg : (rc == Z_DATA_ERROR ? "invalid input data" : "inconsistent stream state");
      inflateEnd(&zs);
      const size_t d = std::min(g.n, delivered_before_zlib_error(in, n, dstart));
      return fail(3, "Error " + std::to_string(rc) + " while decompressing data: " + m, d);
    }
    const size_t used_end = (size_t)(zs.next_in - in);
    inflateEnd(&zs);
    if (!ended) return fail(2, kEOF, g.n);  // every byte inflatable from the input was returned
    pos = used_end;
    if (n - pos < 8) return fail(2, kEOF, g.n);  // the member's data went out before _read_eof
    const uint32_t crc_st = (uint32_t)in[pos] | ((uint32_t)in[pos + 1] << 8) | ((uint32_t)in[pos + 2] << 16) |
                            ((uint32_t)in[pos + 3] << 24);
    const uint32_t isz = (uint32_t)in[pos + 4] | ((uint32_t)in[pos + 5] << 8) | ((uint32_t)in[pos + 6] << 16) |
                         ((uint32_t)in[pos + 7] << 24);
    pos += 8;
    if (crc_st != (uint32_t)crc) {
      char b[64];
      snprintf(b, sizeof(b), "CRC check failed 0x%x != 0x%x", crc_st, (uint32_t)crc);
      return fail(4, b, g.n);
    }
    if (isz != (uint32_t)(g.n & 0xFFFFFFFFu)) return fail(4, "Incorrect length of data produced", g.n);
    keep(g.n);
    out.members++;
    while (pos < n && in[pos] == 0) pos++;
  }
  out.start.push_back(total);
  out.total = total;
  return true;
}

}  // namespace g2n
