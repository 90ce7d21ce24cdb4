// g2n_writers.cpp — the convert CLI's output files, written natively on host threads
// (SURVEY.md §8(f) 1): the matrix .npz (scipy.sparse.save_npz -> numpy savez_compressed,
// gfa2network/utils.py:85-86) and the <matrix>.nodes.tsv sidecar (utils.py:108-114).
//
//   * npz: a zip64 archive of deflated .npy members, as numpy writes it (force_zip64, method 8).
//     Each member's bytes (the .npy header the caller built with numpy's own format code, then
//     the array bytes) are cut into 8 MiB pieces deflated concurrently; every piece but the last
//     ends in a sync flush, so the pieces concatenate into one deflate stream (the pigz layout);
//     piece CRCs are combined with crc32_combine.
//   * nodes.tsv: "i\tname\n" per node id, formatted per 1M-name range on its own thread and
//     written with pwrite at offsets from a prefix sum of the line lengths.
#include <errno.h>
#include <fcntl.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <ctime>
#include <cstring>
#include <string>
#include <vector>

#include "g2n_internal.h"

namespace g2n {
namespace {

constexpr size_t kPiece = (size_t)8 << 20;

struct Piece {
  int entry;
  size_t off, len;  // within the member's bytes (header ++ data)
  std::vector<uint8_t> out;
  uLong crc = 0;
};

void put16(std::vector<uint8_t>& b, uint32_t v) {
  b.push_back((uint8_t)v);
  b.push_back((uint8_t)(v >> 8));
}
void put32(std::vector<uint8_t>& b, uint32_t v) {
  for (int k = 0; k < 4; k++) b.push_back((uint8_t)(v >> (8 * k)));
}
void put64(std::vector<uint8_t>& b, uint64_t v) {
  for (int k = 0; k < 8; k++) b.push_back((uint8_t)(v >> (8 * k)));
}

void write_all(int fd, const uint8_t* p, size_t n, const std::string& path) {
  while (n) {
    ssize_t w = ::write(fd, p, std::min<size_t>(n, (size_t)1 << 30));
    if (w < 0 && errno == EINTR) continue;
    if (w <= 0) throw Failure(G2N_E_IO, path + ": " + std::strerror(w < 0 ? errno : EIO));
    p += w;
    n -= (size_t)w;
  }
}

void pwrite_all(int fd, const uint8_t* p, size_t n, uint64_t off, const std::string& path) {
  while (n) {
    ssize_t w = ::pwrite(fd, p, std::min<size_t>(n, (size_t)1 << 30), (off_t)off);
    if (w < 0 && errno == EINTR) continue;
    if (w <= 0) throw Failure(G2N_E_IO, path + ": " + std::strerror(w < 0 ? errno : EIO));
    p += w;
    n -= (size_t)w;
    off += (uint64_t)w;
  }
}

// DOS date/time of "now" (zipfile stamps members with the local time of the write)
void dos_now(uint16_t* d, uint16_t* t) {
  time_t now = time(nullptr);
  struct tm tmv;
  localtime_r(&now, &tmv);
  *d = (uint16_t)(((tmv.tm_year - 80) << 9) | ((tmv.tm_mon + 1) << 5) | tmv.tm_mday);
  *t = (uint16_t)((tmv.tm_hour << 11) | (tmv.tm_min << 5) | (tmv.tm_sec / 2));
}

// Python's strict UTF-8 decoder accepts exactly the well-formed sequences (no overlongs, no
// surrogates, nothing above U+10FFFF).
bool utf8_ok(const uint8_t* s, size_t n) {
  size_t i = 0;
  while (i < n) {
    const uint8_t c = s[i];
    if (c < 0x80) {
      i++;
      continue;
    }
    size_t k;
    uint32_t lo = 0x80, hi = 0xBF;
    if (c >= 0xC2 && c <= 0xDF) k = 1;
    else if (c == 0xE0) { k = 2; lo = 0xA0; }
    else if (c == 0xED) { k = 2; hi = 0x9F; }
    else if (c >= 0xE1 && c <= 0xEF) k = 2;
    else if (c == 0xF0) { k = 3; lo = 0x90; }
    else if (c == 0xF4) { k = 3; hi = 0x8F; }
    else if (c >= 0xF1 && c <= 0xF3) k = 3;
    else return false;
    if (i + k >= n) return false;  // truncated sequence
    if (s[i + 1] < lo || s[i + 1] > hi) return false;
    for (size_t j = 2; j <= k; j++)
      if (s[i + j] < 0x80 || s[i + j] > 0xBF) return false;
    i += k + 1;
  }
  return true;
}

uint32_t digits(uint64_t v) {
  uint32_t d = 1;
  while (v >= 10) {
    v /= 10;
    d++;
  }
  return d;
}

}  // namespace

int write_npz(const std::string& path, int n, const char* const* names, const uint8_t* const* heads,
              const uint64_t* head_lens, const void* const* datas, const uint64_t* data_lens, int level) {
  std::vector<Piece> pieces;
  std::vector<size_t> first(n + 1);
  for (int e = 0; e < n; e++) {
    first[e] = pieces.size();
    const size_t total = head_lens[e] + data_lens[e];
    size_t off = 0;
    do {
      Piece p;
      p.entry = e;
      p.off = off;
      p.len = std::min(kPiece, total - off);
      pieces.push_back(std::move(p));
      off += kPiece;
    } while (off < total);
  }
  first[n] = pieces.size();
  parallel_for(pieces.size(), host_threads(), [&](size_t i) {
    Piece& p = pieces[i];
    const bool last = i + 1 == first[p.entry + 1];
    // the piece's bytes: a slice of header ++ data (only the first piece can touch the header)
    std::vector<uint8_t> joined;
    const uint8_t* src;
    const size_t hl = head_lens[p.entry];
    if (p.off < hl) {
      joined.resize(p.len);
      const size_t from_head = std::min(p.len, hl - p.off);
      std::memcpy(joined.data(), heads[p.entry] + p.off, from_head);
      if (p.len > from_head) std::memcpy(joined.data() + from_head, datas[p.entry], p.len - from_head);
      src = joined.data();
    } else {
      src = (const uint8_t*)datas[p.entry] + (p.off - hl);
    }
    p.crc = crc32(0L, src, (uInt)p.len);
    z_stream zs;
    std::memset(&zs, 0, sizeof(zs));
    if (deflateInit2(&zs, level, Z_DEFLATED, -MAX_WBITS, 8, Z_DEFAULT_STRATEGY) != Z_OK)
      throw Failure(G2N_E_NOMEM, "deflateInit2 failed");
    p.out.resize(deflateBound(&zs, (uLong)p.len) + 16);
    zs.next_in = const_cast<Bytef*>(src);
    zs.avail_in = (uInt)p.len;
    zs.next_out = p.out.data();
    zs.avail_out = (uInt)p.out.size();
    const int rc = deflate(&zs, last ? Z_FINISH : Z_SYNC_FLUSH);
    const bool ok = last ? rc == Z_STREAM_END : (rc == Z_OK && zs.avail_in == 0);
    p.out.resize(p.out.size() - zs.avail_out);
    deflateEnd(&zs);
    if (!ok) throw Failure(G2N_E_NOMEM, "deflate failed");
  });

  const int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0666);
  if (fd < 0) throw Failure(G2N_E_IO, path + ": " + std::strerror(errno));
  struct Closer {
    int fd;
    ~Closer() { ::close(fd); }
  } closer{fd};
  uint16_t ddate, dtime;
  dos_now(&ddate, &dtime);
  std::vector<uint8_t> cd;
  uint64_t pos = 0;
  for (int e = 0; e < n; e++) {
    uLong crc = 0;
    uint64_t csize = 0;
    for (size_t i = first[e]; i < first[e + 1]; i++) {
      crc = i == first[e] ? pieces[i].crc : crc32_combine(crc, pieces[i].crc, (z_off_t)pieces[i].len);
      csize += pieces[i].out.size();
    }
    const uint64_t usize = head_lens[e] + data_lens[e];
    const size_t nl = std::strlen(names[e]);
    std::vector<uint8_t> h;
    put32(h, 0x04034b50);
    put16(h, 45);  // version needed: zip64
    put16(h, 0);
    put16(h, 8);  // deflate
    put16(h, dtime);
    put16(h, ddate);
    put32(h, (uint32_t)crc);
    put32(h, 0xFFFFFFFFu);
    put32(h, 0xFFFFFFFFu);
    put16(h, (uint32_t)nl);
    put16(h, 20);
    h.insert(h.end(), names[e], names[e] + nl);
    put16(h, 1);  // zip64 extra: sizes
    put16(h, 16);
    put64(h, usize);
    put64(h, csize);
    write_all(fd, h.data(), h.size(), path);
    const uint64_t local = pos;
    pos += h.size();
    for (size_t i = first[e]; i < first[e + 1]; i++) {
      write_all(fd, pieces[i].out.data(), pieces[i].out.size(), path);
      pos += pieces[i].out.size();
      std::vector<uint8_t>().swap(pieces[i].out);
    }
    put32(cd, 0x02014b50);
    put16(cd, (3 << 8) | 45);  // made by: unix, 4.5
    put16(cd, 45);
    put16(cd, 0);
    put16(cd, 8);
    put16(cd, dtime);
    put16(cd, ddate);
    put32(cd, (uint32_t)crc);
    put32(cd, 0xFFFFFFFFu);
    put32(cd, 0xFFFFFFFFu);
    put16(cd, (uint32_t)nl);
    put16(cd, 28);
    put16(cd, 0);  // comment
    put16(cd, 0);  // disk
    put16(cd, 0);  // internal attributes
    put32(cd, 0600u << 16);
    put32(cd, 0xFFFFFFFFu);
    cd.insert(cd.end(), names[e], names[e] + nl);
    put16(cd, 1);  // zip64 extra: sizes and the local header offset
    put16(cd, 24);
    put64(cd, usize);
    put64(cd, csize);
    put64(cd, local);
  }
  const uint64_t cd_off = pos, cd_len = cd.size();
  std::vector<uint8_t> tail;
  put32(tail, 0x06064b50);  // zip64 end of central directory
  put64(tail, 44);
  put16(tail, 45);
  put16(tail, 45);
  put32(tail, 0);
  put32(tail, 0);
  put64(tail, (uint64_t)n);
  put64(tail, (uint64_t)n);
  put64(tail, cd_len);
  put64(tail, cd_off);
  put32(tail, 0x07064b50);  // locator
  put32(tail, 0);
  put64(tail, cd_off + cd_len);
  put32(tail, 1);
  put32(tail, 0x06054b50);  // end of central directory
  put16(tail, 0);
  put16(tail, 0);
  put16(tail, (uint32_t)std::min(n, 0xFFFF));
  put16(tail, (uint32_t)std::min(n, 0xFFFF));
  put32(tail, (uint32_t)std::min<uint64_t>(cd_len, 0xFFFFFFFFu));
  put32(tail, 0xFFFFFFFFu);
  put16(tail, 0);
  write_all(fd, cd.data(), cd.size(), path);
  write_all(fd, tail.data(), tail.size(), path);
  return G2N_OK;
}

int64_t first_bad_utf8(const uint8_t* blob, const int64_t* offs, uint64_t n) {
  const uint64_t chunk = 1 << 16;
  const size_t nch = (size_t)((n + chunk - 1) / chunk);
  std::vector<int64_t> per(nch, -1);
  parallel_for(nch, host_threads(), [&](size_t c) {
    const uint64_t lo = c * chunk, hi = std::min<uint64_t>(n, lo + chunk);
    for (uint64_t i = lo; i < hi; i++)
      if (!utf8_ok(blob + offs[i], (size_t)(offs[i + 1] - offs[i]))) {
        per[c] = (int64_t)i;
        return;
      }
  });
  for (int64_t v : per)
    if (v >= 0) return v;
  return -1;
}

int write_node_map(const std::string& path, const uint8_t* blob, const int64_t* offs, uint64_t n) {
  const uint64_t chunk = 1 << 20;
  const size_t nch = (size_t)((n + chunk - 1) / chunk);
  std::vector<uint64_t> start(nch + 1, 0);
  parallel_for(nch, host_threads(), [&](size_t c) {
    const uint64_t lo = c * chunk, hi = std::min<uint64_t>(n, lo + chunk);
    uint64_t b = (uint64_t)(offs[hi] - offs[lo]) + 2 * (hi - lo);
    for (uint64_t i = lo; i < hi; i++) b += digits(i);
    start[c + 1] = b;
  });
  for (size_t c = 0; c < nch; c++) start[c + 1] += start[c];
  const int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0666);
  if (fd < 0) throw Failure(G2N_E_IO, path + ": " + std::strerror(errno));
  struct Closer {
    int fd;
    ~Closer() { ::close(fd); }
  } closer{fd};
  if (nch && ::ftruncate(fd, (off_t)start[nch]) != 0) throw Failure(G2N_E_IO, path + ": " + std::strerror(errno));
  parallel_for(nch, host_threads(), [&](size_t c) {
    const uint64_t lo = c * chunk, hi = std::min<uint64_t>(n, lo + chunk);
    std::vector<uint8_t> buf(start[c + 1] - start[c]);
    uint8_t* d = buf.data();
    char num[24];
    for (uint64_t i = lo; i < hi; i++) {
      uint32_t k = 0;
      uint64_t v = i;
      do {
        num[k++] = (char)('0' + v % 10);
        v /= 10;
      } while (v);
      while (k) *d++ = (uint8_t)num[--k];
      *d++ = '\t';
      const size_t len = (size_t)(offs[i + 1] - offs[i]);
      std::memcpy(d, blob + offs[i], len);
      d += len;
      *d++ = '\n';
    }
    pwrite_all(fd, buf.data(), buf.size(), start[c], path);
  });
  return G2N_OK;
}

}  // namespace g2n
