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

static int read_fd(int fd, std::vector<uint8_t>& buf) {
  struct stat st;
  if (fstat(fd, &st) == 0) {
    if (S_ISDIR(st.st_mode)) return EISDIR;
    if (S_ISREG(st.st_mode) && st.st_size > 0) buf.reserve((size_t)st.st_size);
  }
  const size_t chunk = 1 << 24;
  size_t n = 0;
  while (true) {
    if (buf.size() < n + chunk) buf.resize(n + chunk);
    ssize_t r = ::read(fd, buf.data() + n, chunk);
    if (r < 0) {
      if (errno == EINTR) continue;
      return errno;
    }
    if (r == 0) break;
    n += (size_t)r;
  }
  buf.resize(n);
  return 0;
}

// gzip.open semantics: members back to back, zero padding between/after members skipped
// (Lib/gzip.py _GzipReader._read_eof); any other trailing bytes must start a new member.
// Sub-codes (err_index): 1 bad magic (BadGzipFile), 2 truncated (EOFError),
// 3 corrupt deflate data (zlib.error), 4 CRC / length mismatch (BadGzipFile).
static int gunzip(const std::vector<uint8_t>& in, std::vector<uint8_t>& out, int* sub, std::string* msg) {
  size_t pos = 0;
  out.clear();
  out.reserve(in.size() * 3 + 1024);
  std::vector<uint8_t> chunk((size_t)1 << 22);
  while (true) {
    while (pos < in.size() && in[pos] == 0) pos++;
    if (pos >= in.size()) return 0;
    if (in.size() - pos < 2 || in[pos] != 0x1F || in[pos + 1] != 0x8B) {
      *sub = 1;
      *msg = "Not a gzipped file";
      return -1;
    }
    z_stream zs;
    std::memset(&zs, 0, sizeof(zs));
    if (inflateInit2(&zs, 16 + MAX_WBITS) != Z_OK) {
      *sub = 3;
      *msg = "inflateInit2 failed";
      return -1;
    }
    size_t fed = pos;  // bytes of `in` handed to zlib so far
    int rc;
    while (true) {
      if (zs.avail_in == 0 && fed < in.size()) {
        size_t take = std::min<size_t>(in.size() - fed, (size_t)1 << 30);
        zs.next_in = const_cast<Bytef*>(in.data() + fed);
        zs.avail_in = (uInt)take;
        fed += take;
      }
      zs.next_out = chunk.data();
      zs.avail_out = (uInt)chunk.size();
      rc = inflate(&zs, Z_NO_FLUSH);
      size_t produced = chunk.size() - zs.avail_out;
      out.insert(out.end(), chunk.data(), chunk.data() + produced);
      if (rc == Z_STREAM_END) break;
      if (rc == Z_OK) continue;
      if (rc == Z_BUF_ERROR && zs.avail_in == 0 && fed >= in.size()) {
        inflateEnd(&zs);
        *sub = 2;
        *msg = "Compressed file ended before the end-of-stream marker was reached";
        return -1;
      }
      if (rc == Z_BUF_ERROR) continue;
      std::string m = zs.msg ? zs.msg : "invalid data";
      inflateEnd(&zs);
      if (m.find("incorrect data check") != std::string::npos || m.find("incorrect length check") != std::string::npos) {
        *sub = 4;
        *msg = "CRC check failed";
      } else {
        *sub = 3;
        *msg = "Error -3 while decompressing data: " + m;
      }
      return -1;
    }
    pos = (size_t)(zs.next_in - in.data());
    inflateEnd(&zs);
  }
}

}  // namespace g2n

extern "C" {

const char* g2n_version(void) { return "gfa2network-amd 0.1.0 (gfx950)"; }
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
  if (o->output != G2N_OUT_PARSE && o->output != G2N_OUT_CSR && o->output != G2N_OUT_COO) {
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
  try {
    return g2n::build_host(buf, len, opts, out, 0.0);
  } catch (const g2n::Failure& f) {
    g2n::set_last_error(f.what());
    return f.status;
  } catch (const std::exception& e) {
    g2n::set_last_error(e.what());
    return G2N_E_DEVICE;
  }
}

int g2n_build_from_path(const char* path, const g2n_options* opts, g2n_result** out) {
  if (!out || !path) return G2N_E_ARG;
  *out = nullptr;
  int rc = check_opts(opts);
  if (rc) return rc;
  double t0 = g2n::now_ms();
  std::vector<uint8_t> raw;
  std::string p(path);
  if (p == "-") {
    int err = g2n::read_fd(0, raw);
    if (err) return g2n::io_failure(err, "<stdin>", out);
  } else {
    int fd = ::open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) return g2n::io_failure(errno, p, out);
    int err = g2n::read_fd(fd, raw);
    ::close(fd);
    if (err) return g2n::io_failure(err, p, out);
    if (p.size() >= 3 && p.compare(p.size() - 3, 3, ".gz") == 0) {
      std::vector<uint8_t> inflated;
      int sub = 0;
      std::string msg;
      if (g2n::gunzip(raw, inflated, &sub, &msg) != 0) {
        g2n::HostResult* h = g2n::new_host_result();
        h->r.status = G2N_E_GZIP;
        h->r.err_index = sub;
        g2n::set_last_error(msg);
        *out = &h->r;
        return G2N_E_GZIP;
      }
      raw.swap(inflated);
    }
  }
  double t1 = g2n::now_ms();
  try {
    return g2n::build_host(raw.data(), raw.size(), opts, out, t1 - t0);
  } catch (const g2n::Failure& f) {
    g2n::set_last_error(f.what());
    return f.status;
  } catch (const std::exception& e) {
    g2n::set_last_error(e.what());
    return G2N_E_DEVICE;
  }
}

void g2n_result_free(g2n_result* r) {
  if (!r) return;
  delete static_cast<g2n::HostResult*>(r->priv_);
}

}  // extern "C"
