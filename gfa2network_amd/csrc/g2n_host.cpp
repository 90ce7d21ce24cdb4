// g2n_host.cpp — host side of the C-ABI: option defaults, errors, input ingest.
//
// Ingest follows GFAParser's source selection (gfa2network/parser.py:100-112): "-" reads
// stdin, a name ending in ".gz" is gunzipped (every concatenated member, like gzip.open),
// anything else is read raw — chosen by name, never by magic bytes.
#include <errno.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <functional>
#include <new>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "g2n_internal.h"

namespace g2n {

static thread_local std::string t_last_error;

void set_last_error(const std::string& msg) { t_last_error = msg; }

void fill_defaults(g2n_result* r) {
  std::memset(r, 0, sizeof(g2n_result));
  r->abi_version = G2N_ABI_VERSION;
  r->err_line = -1;
  r->err_index = -1;
  r->warn_line = -1;
  r->index_width = 4;
}

HostResult* new_host_result() {
  HostResult* h = new HostResult();
  fill_defaults(&h->r);
  h->r.priv_ = h;
  return h;
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static int io_failure(int err, const std::string& what, g2n_result** out) {
  HostResult* h = new_host_result();
  h->r.status = G2N_E_IO;
  h->r.err_index = err;
  set_last_error(what + ": " + std::strerror(err));
  *out = &h->r;
  return G2N_E_IO;
}

static int read_fd(int fd, HostBuf& buf, size_t* len) {
  struct stat st;
  size_t cap = (size_t)1 << 24;
  if (fstat(fd, &st) == 0) {
    if (S_ISDIR(st.st_mode)) return EISDIR;
    if (S_ISREG(st.st_mode) && st.st_size > 0) cap = (size_t)st.st_size + 1;
  }
  HostBuf cur;
  cur.alloc(cap);
  size_t n = 0;
  while (true) {
    if (n == cap) {  // grow (pipes, files that grew since fstat)
      HostBuf bigger;
      bigger.alloc(cap * 2);
      std::memcpy(bigger.p, cur.p, n);
      cur = std::move(bigger);
      cap *= 2;
    }
    ssize_t r = ::read(fd, cur.p + n, cap - n);
    if (r < 0) {
      if (errno == EINTR) continue;
      return errno;
    }
    if (r == 0) break;
    n += (size_t)r;
  }
  buf = std::move(cur);
  *len = n;
  return 0;
}

// Input bytes for the staged upload, read straight from the inflated members.
// bytes of z up to and including its last '\n' (0 if none)
static size_t whole_lines(const Inflated& z) {
  for (size_t k = z.parts.size(); k-- > 0;) {
    const auto* p = (const uint8_t*)memrchr(z.parts[k].p, '\n', z.parts[k].n);
    if (p) return z.start[k] + (size_t)(p - z.parts[k].p) + 1;
  }
  return 0;
}

static FillFn fill_from(const Inflated& z) {
  return [&z](size_t off, uint8_t* dst, size_t len) {
    size_t k = (size_t)(std::upper_bound(z.start.begin(), z.start.end(), off) - z.start.begin()) - 1;
    while (len) {
      const size_t in_part = off - z.start[k];
      const size_t take = std::min(len, z.parts[k].n - in_part);
      std::memcpy(dst, z.parts[k].p + in_part, take);
      dst += take;
      off += take;
      len -= take;
      k++;
    }
  };
}

int guarded(const std::function<int()>& f) {
  try {
    return f();
  } catch (const Failure& e) {
    set_last_error(e.what());
    return e.status;
  } catch (const std::bad_alloc&) {
    set_last_error("host allocation failed");
    return G2N_E_NOMEM;
  } catch (const std::exception& e) {
    set_last_error(e.what());
    return G2N_E_DEVICE;
  }
}

}  // namespace g2n

extern "C" {

const char* g2n_version(void) { return "gfa2network-amd " G2N_VERSION_STRING " (gfx950)"; }
uint32_t g2n_abi_version(void) { return G2N_ABI_VERSION; }
const char* g2n_last_error(void) { return g2n::t_last_error.c_str(); }

const char* g2n_status_name(int s) {
  switch (s) {
    case G2N_OK: return "G2N_OK";
    case G2N_E_MALFORMED_L: return "G2N_E_MALFORMED_L";
    case G2N_E_MALFORMED_E: return "G2N_E_MALFORMED_E";
    case G2N_E_MALFORMED_C: return "G2N_E_MALFORMED_C";
    case G2N_E_MALFORMED_P: return "G2N_E_MALFORMED_P";
    case G2N_E_MALFORMED_O: return "G2N_E_MALFORMED_O";
    case G2N_E_INDEX_LIST: return "G2N_E_INDEX_LIST";
    case G2N_E_INDEX_BYTES: return "G2N_E_INDEX_BYTES";
    case G2N_E_UNICODE: return "G2N_E_UNICODE";
    case G2N_E_INT_TOO_LARGE: return "G2N_E_INT_TOO_LARGE";
    case G2N_E_CAST_OVERFLOW: return "G2N_E_CAST_OVERFLOW";
    case G2N_E_CAST_INF: return "G2N_E_CAST_INF";
    case G2N_E_CAST_NAN: return "G2N_E_CAST_NAN";
    case G2N_E_ARG: return "G2N_E_ARG";
    case G2N_E_IO: return "G2N_E_IO";
    case G2N_E_GZIP: return "G2N_E_GZIP";
    case G2N_E_DEVICE: return "G2N_E_DEVICE";
    case G2N_E_NOMEM: return "G2N_E_NOMEM";
    case G2N_E_UNSUPPORTED: return "G2N_E_UNSUPPORTED";
    default: return "G2N_E_UNKNOWN";
  }
}

void g2n_options_init(g2n_options* o) {
  if (!o) return;
  std::memset(o, 0, sizeof(*o));
  o->abi_version = G2N_ABI_VERSION;
  o->directed = 1;
  o->dtype = G2N_FLOAT64;
  o->output = G2N_OUT_PARSE;
  o->want_node_names = 1;
}

static int check_opts(const g2n_options* o) {
  if (!o || o->abi_version != G2N_ABI_VERSION) {
    g2n::set_last_error("g2n_options: abi_version mismatch (call g2n_options_init)");
    return G2N_E_ARG;
  }
  if (o->dtype < G2N_BOOL || o->dtype > G2N_FLOAT64) {
    g2n::set_last_error("g2n_options: unsupported dtype");
    return G2N_E_ARG;
  }
  if (o->output < G2N_OUT_PARSE || o->output > G2N_OUT_EDGE_LIST) {
    g2n::set_last_error("g2n_options: unknown output");
    return G2N_E_ARG;
  }
  return G2N_OK;
}

int g2n_build_from_buffer(const void* buf, size_t len, const g2n_options* opts, g2n_result** out) {
  if (!out) return G2N_E_ARG;
  *out = nullptr;
  int rc = check_opts(opts);
  if (rc) return rc;
  if (len && !buf) return G2N_E_ARG;
  return g2n::guarded([&] { return g2n::build_host(buf, len, opts, out, 0.0); });
}

int g2n_build_from_path(const char* path, const g2n_options* opts, g2n_result** out) {
  if (!out || !path) return G2N_E_ARG;
  *out = nullptr;
  int rc = check_opts(opts);
  if (rc) return rc;
  return g2n::guarded([&]() -> int {
    const double t0 = g2n::now_ms();
    std::string p(path);
    const bool gz = p != "-" && p.size() >= 3 && p.compare(p.size() - 3, 3, ".gz") == 0;
    int fd = 0;
    if (p != "-") {
      fd = ::open(path, O_RDONLY | O_CLOEXEC);
      if (fd < 0) return g2n::io_failure(errno, p, out);
    }
    struct FdCloser {
      int fd;
      ~FdCloser() {
        if (fd > 0) ::close(fd);
      }
    } closer{fd};
    struct stat st;
    const bool regular = fd > 0 && fstat(fd, &st) == 0 && S_ISREG(st.st_mode);
    if (fd > 0 && fstat(fd, &st) == 0 && S_ISDIR(st.st_mode)) return g2n::io_failure(EISDIR, p, out);
    if (regular && !gz) {
      // plain file: pread straight into the pinned staging slots (page cache -> HBM)
      const size_t len = (size_t)st.st_size;
      const int rfd = fd;
      g2n::FillFn fill = [rfd, &p](size_t off, uint8_t* dst, size_t n) {
        size_t got = 0;
        while (got < n) {
          ssize_t r = ::pread(rfd, dst + got, n - got, (off_t)(off + got));
          if (r < 0 && errno == EINTR) continue;
          if (r <= 0) throw g2n::Failure(G2N_E_IO, p + ": " + std::strerror(r < 0 ? errno : EIO));
          got += (size_t)r;
        }
      };
      return g2n::build_host_fill(len, fill, opts, out, 0.0);
    }
    g2n::HostBuf raw;
    size_t rlen = 0;
    int err = g2n::read_fd(fd, raw, &rlen);
    if (err) return g2n::io_failure(err, p == "-" ? "<stdin>" : p, out);
    if (!gz) {
      const double t1 = g2n::now_ms();
      return g2n::build_host(raw.p, rlen, opts, out, t1 - t0);
    }
    std::vector<g2n::ZMember> zm;
    size_t zout = 0;
    if (!(opts->test_flags & g2n::kTestHostInflate) && g2n::bgzf_members(raw.p, rlen, zm, &zout)) {
      // BGZF: the members inflate on the GPU (the host readers only when one does not cleanly)
      const int rcz = g2n::build_host_bgzf(raw.p, rlen, zm, zout, opts, out, g2n::now_ms() - t0);
      if (rcz != g2n::kBgzfFallback) return rcz;
    }
    g2n::Inflated z;
    if (!g2n::gunzip_parallel(raw.p, rlen, z)) {
      int sub = 0;
      std::string msg;
      if (!g2n::gunzip_exact(raw.p, rlen, z, &sub, &msg)) {
        // parser.py:114 iterates the lines gzip returned before it raised: those whole lines are
        // parsed first, so their parse error wins, and their warning precedes the gzip error
        // (a cast error comes after the loop: the gzip error is first)
        const size_t cut = g2n::whole_lines(z);
        g2n_result* pr = nullptr;
        if (cut) {
          const int rc2 = g2n::build_host_fill(cut, g2n::fill_from(z), opts, &pr, g2n::now_ms() - t0);
          if ((rc2 >= G2N_E_MALFORMED_L && rc2 <= G2N_E_INT_TOO_LARGE) || rc2 >= G2N_E_ARG) {
            g2n::free_later(std::move(z.parts));
            *out = pr;
            return rc2;
          }
        }
        g2n::free_later(std::move(z.parts));
        if (!pr) pr = &g2n::new_host_result()->r;
        pr->status = G2N_E_GZIP;
        pr->err_index = sub;
        pr->err_line = -1;
        pr->err_value = 0.0;
        g2n::set_last_error(msg);
        *out = pr;
        return G2N_E_GZIP;
      }
    }
    {
      std::vector<g2n::HostBuf> done;
      done.push_back(std::move(raw));
      g2n::free_later(std::move(done));
    }
    const double t1 = g2n::now_ms();
    const int rc2 = g2n::build_host_fill(z.total, g2n::fill_from(z), opts, out, t1 - t0);
    g2n::free_later(std::move(z.parts));
    return rc2;
  });
}

int g2n_upload_file_range(const char* path, uint64_t offset, uint64_t len, void* d_dst, int32_t device) {
  if (!path || (len && !d_dst)) return G2N_E_ARG;
  return g2n::guarded([&]() -> int {
    const std::string p(path);
    const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) {
      g2n::set_last_error(p + ": " + std::strerror(errno));
      return G2N_E_IO;
    }
    struct FdCloser {
      int fd;
      ~FdCloser() { ::close(fd); }
    } closer{fd};
    g2n::FillFn fill = [fd, offset, &p](size_t off, uint8_t* dst, size_t n) {
      size_t got = 0;
      while (got < n) {
        ssize_t r = ::pread(fd, dst + got, n - got, (off_t)(offset + off + got));
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) throw g2n::Failure(G2N_E_IO, p + ": " + std::strerror(r < 0 ? errno : EIO));
        got += (size_t)r;
      }
    };
    g2n::staged_upload(device, (uint8_t*)d_dst, (size_t)len, fill);
    return G2N_OK;
  });
}

int g2n_gunzip(const void* buf, size_t len, int32_t parallel, void** out, size_t* out_len, int32_t* members,
               int32_t* sub) {
  if (!out || !out_len || (len && !buf)) return G2N_E_ARG;
  *out = nullptr;
  *out_len = 0;
  return g2n::guarded([&]() -> int {
    g2n::Inflated z;
    const uint8_t* in = (const uint8_t*)buf;
    if (!(parallel && g2n::gunzip_parallel(in, len, z))) {
      int s = 0;
      std::string msg;
      if (!g2n::gunzip_exact(in, len, z, &s, &msg)) {
        if (sub) *sub = s;
        // the bytes gzip.py's reader returned before raising
        auto* o = (uint8_t*)std::malloc(z.total ? z.total : 1);
        if (!o) return G2N_E_NOMEM;
        for (size_t k = 0; k < z.parts.size(); k++) std::memcpy(o + z.start[k], z.parts[k].p, z.parts[k].n);
        *out = o;
        *out_len = z.total;
        g2n::set_last_error(msg);
        return G2N_E_GZIP;
      }
    }
    auto* o = (uint8_t*)std::malloc(z.total ? z.total : 1);
    if (!o) return G2N_E_NOMEM;
    for (size_t k = 0; k < z.parts.size(); k++) std::memcpy(o + z.start[k], z.parts[k].p, z.parts[k].n);
    *out = o;
    *out_len = z.total;
    if (members) *members = z.members;
    if (sub) *sub = 0;
    return G2N_OK;
  });
}

int g2n_gunzip_chunked(const void* buf, size_t len, size_t chunk_bytes, void** out, size_t* out_len,
                       int32_t* chunks) {
  if (!out || !out_len || !buf) return G2N_E_ARG;
  *out = nullptr;
  *out_len = 0;
  return g2n::guarded([&]() -> int {
    g2n::Inflated z;
    if (!g2n::gunzip_chunked((const uint8_t*)buf, len, chunk_bytes, z)) return G2N_E_UNSUPPORTED;
    auto* o = (uint8_t*)std::malloc(z.total ? z.total : 1);
    if (!o) return G2N_E_NOMEM;
    for (size_t k = 0; k < z.parts.size(); k++) std::memcpy(o + z.start[k], z.parts[k].p, z.parts[k].n);
    *out = o;
    *out_len = z.total;
    if (chunks) *chunks = (int32_t)z.parts.size();
    return G2N_OK;
  });
}

void g2n_free(void* p) { std::free(p); }

int g2n_join_names(const uint8_t* blob, const int64_t* offsets, uint64_t n_names, uint8_t sep, uint8_t* out) {
  if (n_names == 0) return G2N_OK;
  if (!blob || !offsets || !out) return G2N_E_ARG;
  return g2n::guarded([&]() -> int {
    const uint64_t chunk = 1 << 16;
    g2n::parallel_for((n_names + chunk - 1) / chunk, g2n::host_threads(), [&](size_t c) {
      const uint64_t lo = c * chunk, hi = std::min<uint64_t>(n_names, lo + chunk);
      for (uint64_t i = lo; i < hi; i++) {
        uint8_t* d = out + offsets[i] - offsets[0] + i;
        const size_t len = (size_t)(offsets[i + 1] - offsets[i]);
        std::memcpy(d, blob + offsets[i], len);
        if (i + 1 < n_names) d[len] = sep;
      }
    });
    return G2N_OK;
  });
}

int g2n_gather_names(const uint8_t* blob, const int64_t* offsets, const int64_t* order, uint64_t n_names,
                     const int64_t* out_offsets, uint8_t* out) {
  if (n_names == 0) return G2N_OK;
  if (!blob || !offsets || !order || !out_offsets || !out) return G2N_E_ARG;
  return g2n::guarded([&]() -> int {
    const uint64_t chunk = 1 << 16;
    g2n::parallel_for((n_names + chunk - 1) / chunk, g2n::host_threads(), [&](size_t c) {
      const uint64_t lo = c * chunk, hi = std::min<uint64_t>(n_names, lo + chunk);
      for (uint64_t i = lo; i < hi; i++) {
        const int64_t k = order[i];
        std::memcpy(out + out_offsets[i] - out_offsets[0], blob + offsets[k], (size_t)(offsets[k + 1] - offsets[k]));
      }
    });
    return G2N_OK;
  });
}

int g2n_write_npz(const char* path, int32_t n_members, const char* const* names, const uint8_t* const* heads,
                  const uint64_t* head_lens, const void* const* datas, const uint64_t* data_lens, int32_t level) {
  if (!path || n_members < 0 || (n_members && (!names || !heads || !head_lens || !datas || !data_lens)))
    return G2N_E_ARG;
  return g2n::guarded(
      [&] { return g2n::write_npz(path, n_members, names, heads, head_lens, datas, data_lens, level); });
}

int g2n_write_node_map(const char* path, const uint8_t* blob, const int64_t* offsets, uint64_t n_names,
                       int32_t check_utf8, int64_t* bad_index) {
  if (!path || (n_names && (!blob || !offsets))) return G2N_E_ARG;
  if (bad_index) *bad_index = -1;
  return g2n::guarded([&]() -> int {
    uint64_t n = n_names;
    if (check_utf8) {
      const int64_t bad = g2n::first_bad_utf8(blob, offsets, n_names);
      if (bad >= 0) {
        n = (uint64_t)bad;
        if (bad_index) *bad_index = bad;
      }
    }
    return g2n::write_node_map(path, blob, offsets, n);
  });
}

int64_t g2n_first_bad_utf8(const uint8_t* blob, const int64_t* offsets, uint64_t n_names) {
  if (!n_names || !blob || !offsets) return -1;
  try {
    return g2n::first_bad_utf8(blob, offsets, n_names);
  } catch (...) {
    return -1;
  }
}

void g2n_result_free(g2n_result* r) {
  if (!r) return;
  delete static_cast<g2n::HostResult*>(r->priv_);
}

}  // extern "C"
