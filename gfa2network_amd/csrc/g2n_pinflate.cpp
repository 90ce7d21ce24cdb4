// g2n_pinflate.cpp — chunk-parallel inflate of ONE large gzip member ("a
// speculative-parallel inflate for single-member gzip, which otherwise stays serial",
// gfa2network/parser.py:108-109 reads it with gzip.open on one thread).
//
// A single deflate stream has no index: a block's start is only known once everything before
// it has been decoded, and its back-references reach 32 KiB into output not yet produced.  So:
//   1. sync   the compressed stream is cut into chunks; every chunk (but the first) searches its
//             range, bit by bit, for a dynamic-Huffman block header whose tables are valid,
//             whose block decodes to its end-of-block code and which is followed by another
//             valid header — a candidate block start.
//   2. decode every chunk decodes from its start to the next chunk's start on its own thread.
//             The 32 KiB window before a chunk is unknown, so a chunk decodes "dirty" first: a
//             16-bit shadow window holds either a byte or the index of the unknown window byte
//             it copies, every byte copied from the unknown window is written as a placeholder
//             and recorded (position, window index), and once the last 32 KiB of output hold no
//             placeholder the chunk switches to the plain byte decoder.  A chunk must reach the
//             next chunk's start exactly at a block boundary — chunk 0 decodes from the real
//             start, so by induction every chunk start is a true block boundary and every
//             decoded byte is the stream's.
//   3. patch  in file order each chunk's placeholders take their bytes from the 32 KiB that
//             precede it (already final); CRC-32 per chunk in parallel, combined, and the ISIZE
//             checked against the member trailer.
// Anything unexpected (a chunk that overshoots the next start, a reference before the stream's
// first byte, an invalid code, more data after the member, header flags) returns false and the
// caller falls back to the exact gzip.py reader, so errors and their prefix semantics are always
// the reference's.  The decoder is stricter than zlib where they differ (incomplete codes are
// refused), never laxer.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <immintrin.h>
#include <zlib.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <memory>
#include <vector>

#include "g2n_internal.h"

namespace g2n {
namespace {

constexpr unsigned kLitBits = 11, kDistBits = 9;  // primary table widths; longer codes walk the canonical code
constexpr size_t kWin = 32768;

struct Huff {
  uint16_t count[16];
  uint16_t sym[288];
  uint32_t fast[1u << kLitBits];  // sym | len << 16; 0 = code longer than the table (or none)
  unsigned bits;
  bool empty;
};

inline unsigned rev_bits(unsigned c, unsigned len) {
  unsigned r = 0;
  for (unsigned i = 0; i < len; i++) r |= ((c >> i) & 1u) << (len - 1 - i);
  return r;
}

// Canonical Huffman code from code lengths (RFC 1951 3.2.2).  Over-subscribed codes are refused;
// incomplete ones too (zlib accepts a single length-1 code: that stream takes the exact reader),
// except an all-zero distance code when allow_empty (zlib accepts it; using it is an error).
bool build_huff(Huff& h, const uint8_t* len, unsigned n, unsigned bits, bool allow_empty) {
  memset(h.count, 0, sizeof(h.count));
  for (unsigned s = 0; s < n; s++) h.count[len[s]]++;
  h.bits = bits;
  h.empty = h.count[0] == n;
  memset(h.fast, 0, sizeof(uint32_t) << bits);
  if (h.empty) return allow_empty;
  int left = 1;
  for (unsigned l = 1; l < 16; l++) {
    left <<= 1;
    left -= h.count[l];
    if (left < 0) return false;
  }
  if (left > 0) return false;
  uint16_t offs[16];
  offs[1] = 0;
  for (unsigned l = 1; l < 15; l++) offs[l + 1] = offs[l] + h.count[l];
  for (unsigned s = 0; s < n; s++)
    if (len[s]) h.sym[offs[len[s]]++] = (uint16_t)s;
  unsigned code = 0, k = 0;
  for (unsigned l = 1; l < 16; l++) {
    for (unsigned c = 0; c < h.count[l]; c++, k++, code++) {
      if (l > bits) continue;
      const uint32_t e = h.sym[k] | (l << 16);
      for (unsigned r = rev_bits(code, l); r < (1u << bits); r += 1u << l) h.fast[r] = e;
    }
    code <<= 1;
  }
  return true;
}

// Bit reader over in[0, n): 64-bit buffer, LSB first; reading past the end yields zeros and
// raises `over`, which every decode loop checks.
struct BitIn {
  const uint8_t* in;
  size_t n, ip;  // next byte to load
  uint64_t bb = 0;
  unsigned bc = 0;
  bool over = false;
  BitIn(const uint8_t* in_, size_t n_, uint64_t bitpos) : in(in_), n(n_), ip(bitpos >> 3) {
    refill();
    const unsigned sk = (unsigned)(bitpos & 7);
    bb >>= sk;
    bc -= sk;
  }
  uint64_t pos() const { return (uint64_t)ip * 8 - bc; }
  void refill() {
    if (ip + 8 <= n) {
      uint64_t w;
      memcpy(&w, in + ip, 8);
      bb |= w << bc;
      ip += (63 - bc) >> 3;
      bc |= 56;
    } else {
      while (bc <= 56) {
        uint64_t b = 0;
        if (ip < n) b = in[ip];
        else if (ip > n + 16) over = true;
        bb |= b << bc;
        ip++;
        bc += 8;
      }
    }
  }
  void drop(unsigned k) {
    bb >>= k;
    bc -= k;
  }
  uint32_t take(unsigned k) {
    const uint32_t v = (uint32_t)(bb & ((1ull << k) - 1));
    drop(k);
    return v;
  }
  // next symbol of h (>= 15 bits buffered); -1 = no such code
  int decode(const Huff& h) {
    const uint32_t e = h.fast[bb & ((1u << h.bits) - 1)];
    if (e) {
      drop(e >> 16);
      return (int)(e & 0xFFFF);
    }
    int code = 0, first = 0, index = 0;
    for (unsigned l = 1; l < 16; l++) {
      code |= (int)((bb >> (l - 1)) & 1);
      const int c = h.count[l];
      if (code - c < first) {
        drop(l);
        return h.sym[index + (code - first)];
      }
      index += c;
      first += c;
      first <<= 1;
      code <<= 1;
    }
    return -1;
  }
};

const uint16_t kLenBase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                               35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
const uint8_t kLenExt[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
const uint16_t kDistBase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193,
                                257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
const uint8_t kDistExt[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
const uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

struct Fixed {
  Huff lit, dist;
  Fixed() {
    uint8_t l[288];
    for (int s = 0; s < 288; s++) l[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
    build_huff(lit, l, 288, kLitBits, false);
    uint8_t d[32];
    memset(d, 5, sizeof(d));
    build_huff(dist, d, 32, kDistBits, false);
  }
};
const Fixed& fixed_tables() {
  static const Fixed f;
  return f;
}

// Block header after BFINAL/BTYPE: the dynamic code tables.  false = invalid.
bool read_dynamic(BitIn& br, Huff& lit, Huff& dist) {
  br.refill();
  const unsigned hlit = br.take(5) + 257, hdist = br.take(5) + 1, hclen = br.take(4) + 4;
  if (hlit > 286 || hdist > 30) return false;
  uint8_t cl[19] = {0};
  for (unsigned i = 0; i < hclen; i++) {
    if (i == 12) br.refill();
    cl[kClOrder[i]] = (uint8_t)br.take(3);
  }
  Huff clh;
  if (!build_huff(clh, cl, 19, 7, false)) return false;
  uint8_t lens[286 + 30];
  const unsigned tot = hlit + hdist;
  for (unsigned i = 0; i < tot;) {
    br.refill();
    const int s = br.decode(clh);
    if (s < 0) return false;
    if (s < 16) {
      lens[i++] = (uint8_t)s;
      continue;
    }
    unsigned rep;
    uint8_t v = 0;
    if (s == 16) {
      if (i == 0) return false;
      v = lens[i - 1];
      rep = 3 + br.take(2);
    } else if (s == 17) {
      rep = 3 + br.take(3);
    } else {
      rep = 11 + br.take(7);
    }
    if (i + rep > tot) return false;
    memset(lens + i, v, rep);
    i += rep;
  }
  if (br.over || lens[256] == 0) return false;
  return build_huff(lit, lens, hlit, kLitBits, false) && build_huff(dist, lens + hlit, hdist, kDistBits, true);
}

// A large output reserved up front: 2 MiB-aligned, advised for transparent huge pages (one
// fault per 2 MiB instead of per 4 KiB when 16 threads fill fresh memory side by side);
// free()-compatible, so HostBuf can adopt it.  Growth past the reservation reallocs.
void* reserve_huge(size_t bytes) {
  const size_t h = (size_t)2 << 20, al = (bytes + h - 1) & ~(h - 1);
  void* q = nullptr;
  if (posix_memalign(&q, h, al) != 0 || !q) throw Failure(G2N_E_NOMEM, "host allocation failed while inflating");
  (void)madvise(q, al, MADV_HUGEPAGE);
  return q;
}

struct Out {
  uint8_t* p = nullptr;
  size_t n = 0, cap = 0;
  ~Out() { free(p); }
  void reserve(size_t want) {
    free(p);
    p = (uint8_t*)reserve_huge(want);
    cap = want;
  }
  void room(size_t want) {
    if (cap - n >= want) return;
    size_t c = std::max(n + want, cap + cap / 2 + ((size_t)1 << 20));
    auto* q = (uint8_t*)realloc(p, c);
    if (!q) throw Failure(G2N_E_NOMEM, "host allocation failed while inflating");
    p = q;
    cap = c;
  }
};

// 16-bit shadow of a chunk's output while its window is unknown: entry 32768 + p is output
// byte p (< 256) or 256 + k for byte k of the 32 KiB before the chunk; entries 0..32767 are
// that unknown window itself.
struct Shadow {
  uint16_t* p = nullptr;
  size_t cap = 0;
  ~Shadow() { free(p); }
  void reserve(size_t want) {
    free(p);
    p = (uint16_t*)reserve_huge(want * sizeof(uint16_t));
    cap = want;
  }
  void room(size_t want) {
    if (cap >= want) return;
    size_t c = std::max(want, cap + cap / 2 + ((size_t)1 << 20));
    auto* q = (uint16_t*)realloc(p, c * sizeof(uint16_t));
    if (!q) throw Failure(G2N_E_NOMEM, "host allocation failed while inflating");
    p = q;
    cap = c;
  }
};

struct alignas(128) Chunk {  // chunks decode side by side: no shared cache lines
  uint64_t sync = 0;         // bit offset of the first block this chunk decodes (chunk 0: stream start)
  bool present = false;      // a start was found in this chunk's range
  bool ok = false;           // decoded to the start of chunk `next`, or to the stream's end
  size_t next = 0;           // the chunk whose start this one reached (ok && !final_seen)
  bool final_seen = false;   // the stream's BFINAL block ended in this chunk
  uint64_t end_bits = 0;
  Out out;
  Shadow sh;
  size_t dirty_len = 0;      // out[0, dirty_len) waits for the window (shadow holds the truth)
  std::unique_ptr<uint8_t[]> win;  // the 32 KiB before the chunk, once known
};

// Decoder over one chunk: dirty (16-bit shadow) until the last 32 KiB of output reference no
// unknown window byte, then plain bytes.
struct Dec {
  Chunk& c;
  bool dirty;
  uint64_t last_dirty_end = 0;  // 1 + position of the latest unknown-window byte
  size_t trial_cap = ~(size_t)0;  // output bound of a trial decode (a false block start may babble)
  Dec(Chunk& c_, bool unknown_window) : c(c_), dirty(unknown_window) {
    if (dirty) {
      c.sh.room(std::max<size_t>(kWin + ((size_t)1 << 20), kWin + c.out.cap));
      for (size_t k = 0; k < kWin; k++) c.sh.p[k] = (uint16_t)(256 + k);
    }
  }

  // One Huffman block.  true = end-of-block reached.  The bit reader and the output cursor live
  // in locals for the loop (byte stores could alias them otherwise, and chunks decoding side by
  // side would share their cache lines).
  bool codes(BitIn& br_io, const Huff& lit, const Huff& dist) {
    BitIn br = br_io;
    Out& out = c.out;
    uint8_t* op = out.p;
    size_t n = out.n, cap = out.cap;
    bool ok = false;
    if (dirty) {
      uint16_t* sh = c.sh.p + kWin;
      size_t shcap = c.sh.cap - kWin;
      uint64_t ldirty = last_dirty_end;
      for (;;) {
        if (n >= ldirty + kWin) {  // window free of unknown bytes: plain decoding
          dirty = false;
          c.dirty_len = n;
          for (size_t p = n - kWin; p < n; p++) op[p] = (uint8_t)sh[p];  // the plain decoder's history
          break;
        }
        if (cap - n < 300 || shcap - n < 300) {
          if (n > trial_cap) goto done;
          out.n = n;
          out.room(300);
          op = out.p;
          cap = out.cap;
          c.sh.room(kWin + n + 300);
          sh = c.sh.p + kWin;
          shcap = c.sh.cap - kWin;
        }
        br.refill();
        if (br.over) goto done;
        const int s = br.decode(lit);
        if (s < 0) goto done;
        if (s < 256) {
          sh[n++] = (uint16_t)s;  // out[0, dirty_len) is written once, from the shadow, when resolved
          continue;
        }
        if (s == 256) {
          ok = true;
          last_dirty_end = ldirty;
          goto done;
        }
        const unsigned ls = (unsigned)s - 257;
        if (ls >= 29 || dist.empty) goto done;
        const unsigned len = kLenBase[ls] + br.take(kLenExt[ls]);
        const int d = br.decode(dist);
        if (d < 0 || d >= 30) goto done;
        const size_t dd = kDistBase[d] + br.take(kDistExt[d]);
        unsigned unk = 0;
        const uint16_t* src = sh + n - dd;  // >= sh - 32768: inside the unknown-window prefix
        for (unsigned k = 0; k < len; k++) {
          const uint16_t v = src[k];
          sh[n + k] = v;
          unk |= v;
        }
        n += len;
        if (unk >= 256) ldirty = n;
      }
      last_dirty_end = ldirty;
    }
    for (;;) {
      if (cap - n < 300) {
        if (n > trial_cap) break;
        out.n = n;
        out.room(300);
        op = out.p;
        cap = out.cap;
      }
      br.refill();
      if (br.over) break;
      const int s = br.decode(lit);
      if (s < 0) break;
      if (s < 256) {
        op[n++] = (uint8_t)s;
        continue;
      }
      if (s == 256) {
        ok = true;
        break;
      }
      const unsigned ls = (unsigned)s - 257;
      if (ls >= 29 || dist.empty) break;
      const unsigned len = kLenBase[ls] + br.take(kLenExt[ls]);
      const int d = br.decode(dist);
      if (d < 0 || d >= 30) break;
      const size_t dd = kDistBase[d] + br.take(kDistExt[d]);
      if (dd > n) break;  // only the stream's first chunk can get here with a short history
      uint8_t* o = op + n;
      const uint8_t* src = o - dd;
      if (dd >= 8) {
        for (unsigned k = 0; k < len; k += 8) {  // may overshoot by <= 7 bytes (room 300)
          uint64_t w;
          memcpy(&w, src + k, 8);
          memcpy(o + k, &w, 8);
        }
      } else if (dd == 1) {
        memset(o, src[0], len);
      } else {
        for (unsigned k = 0; k < len; k++) o[k] = src[k];
      }
      n += len;
    }
  done:
    out.n = n;
    br_io = br;
    return ok;
  }

  // Stored block after its 3 header bits.
  bool stored(BitIn& br) {
    Out& out = c.out;
    const uint64_t byte = (br.pos() + 7) >> 3;
    if (byte + 4 > br.n) return false;
    const uint8_t* q = br.in + byte;
    const unsigned len = q[0] | (q[1] << 8), nlen = q[2] | (q[3] << 8);
    if ((len ^ 0xFFFF) != nlen || byte + 4 + len > br.n) return false;
    out.room(len + 16);
    memcpy(out.p + out.n, q + 4, len);
    if (dirty) {
      c.sh.room(kWin + out.n + len + 16);
      for (unsigned k = 0; k < len; k++) c.sh.p[kWin + out.n + k] = q[4 + k];
    }
    out.n += len;
    br = BitIn(br.in, br.n, (byte + 4 + len) * 8);
    return true;
  }

  // One block at br.  false = invalid; *final = BFINAL.
  bool block(BitIn& br, bool* final) {
    br.refill();
    *final = br.take(1);
    const unsigned type = br.take(2);
    if (type == 0) return stored(br);
    if (type == 1) return codes(br, fixed_tables().lit, fixed_tables().dist);
    if (type == 2) {
      Huff lit, dist;
      return read_dynamic(br, lit, dist) && codes(br, lit, dist);
    }
    return false;
  }
  void finish() {
    if (dirty) c.dirty_len = c.out.n;
  }
};

// Is there a plausible (non-final, dynamic) block start at bit p?  Its tables must be valid,
// the block must decode to its end-of-block code (unknown window) and a valid block header
// must follow.
bool plausible_start(const uint8_t* in, size_t n, uint64_t p) {
  BitIn br(in, n, p);
  if ((br.bb & 7) != 4) return false;  // BFINAL 0, BTYPE 2
  if (((br.bb >> 3) & 31) > 29 || ((br.bb >> 8) & 31) > 29) return false;
  br.drop(3);
  Huff lit, dist;
  if (!read_dynamic(br, lit, dist)) return false;
  Chunk scratch;
  Dec dec(scratch, true);
  dec.trial_cap = (size_t)8 << 20;  // a real block holds <= 16K symbols (zlib): <= 4.2 MB of output
  if (!dec.codes(br, lit, dist) || br.over || scratch.out.n == 0) return false;
  br.refill();
  const unsigned type = (unsigned)((br.bb >> 1) & 3);
  if (type == 3) return false;
  if (type == 2) {
    br.drop(3);
    Huff l2, d2;
    if (!read_dynamic(br, l2, d2)) return false;
  }
  return true;
}

// CRC-32 (gzip's reflected 0x04C11DB7) by carry-less multiplication: four 128-bit lanes folded
// over 64-byte blocks, folded to one lane, to 64 bits, then a Barrett reduction (Intel's
// "Fast CRC Computation for Generic Polynomials Using PCLMULQDQ"; the constants are
// x^k mod P for the fold distances and the Barrett pair).  crc is zlib's running value.
__attribute__((target("pclmul,sse4.1"))) inline __m128i fold(__m128i x, __m128i kk, __m128i y) {
  return _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x, kk, 0x00), _mm_clmulepi64_si128(x, kk, 0x11)), y);
}

__attribute__((target("pclmul,sse4.1"))) uint32_t crc32_fold(uint32_t crc, const uint8_t* p, size_t n) {
  if (n < 64) return (uint32_t)crc32(crc, p, (uInt)n);
  alignas(16) static const uint64_t k12[2] = {0x0154442bd4ull, 0x01c6e41596ull};
  alignas(16) static const uint64_t k34[2] = {0x01751997d0ull, 0x00ccaa009eull};
  alignas(16) static const uint64_t k50[2] = {0x0163cd6124ull, 0};
  alignas(16) static const uint64_t pmu[2] = {0x01db710641ull, 0x01f7011641ull};
  const size_t body = n & ~(size_t)15;
  const uint8_t* q = p;
  size_t left = body;
  __m128i a0 = _mm_loadu_si128((const __m128i*)q), a1 = _mm_loadu_si128((const __m128i*)(q + 16));
  __m128i a2 = _mm_loadu_si128((const __m128i*)(q + 32)), a3 = _mm_loadu_si128((const __m128i*)(q + 48));
  a0 = _mm_xor_si128(a0, _mm_cvtsi32_si128((int)~crc));
  __m128i k = _mm_load_si128((const __m128i*)k12);
  q += 64;
  left -= 64;
  while (left >= 64) {
    a0 = fold(a0, k, _mm_loadu_si128((const __m128i*)q));
    a1 = fold(a1, k, _mm_loadu_si128((const __m128i*)(q + 16)));
    a2 = fold(a2, k, _mm_loadu_si128((const __m128i*)(q + 32)));
    a3 = fold(a3, k, _mm_loadu_si128((const __m128i*)(q + 48)));
    q += 64;
    left -= 64;
  }
  k = _mm_load_si128((const __m128i*)k34);
  a0 = fold(a0, k, a1);
  a0 = fold(a0, k, a2);
  a0 = fold(a0, k, a3);
  while (left >= 16) {
    a0 = fold(a0, k, _mm_loadu_si128((const __m128i*)q));
    q += 16;
    left -= 16;
  }
  const __m128i lo32 = _mm_setr_epi32(~0, 0, ~0, 0);
  __m128i x = _mm_xor_si128(_mm_srli_si128(a0, 8), _mm_clmulepi64_si128(a0, k, 0x10));  // 128 -> 64 bits
  const __m128i k5 = _mm_loadl_epi64((const __m128i*)k50);
  x = _mm_xor_si128(_mm_clmulepi64_si128(_mm_and_si128(x, lo32), k5, 0x00), _mm_srli_si128(x, 4));
  const __m128i pm = _mm_load_si128((const __m128i*)pmu);  // Barrett reduction to 32 bits
  __m128i t = _mm_clmulepi64_si128(_mm_and_si128(x, lo32), pm, 0x10);
  t = _mm_clmulepi64_si128(_mm_and_si128(t, lo32), pm, 0x00);
  crc = ~(uint32_t)_mm_extract_epi32(_mm_xor_si128(x, t), 1);
  return n > body ? (uint32_t)crc32(crc, p + body, (uInt)(n - body)) : crc;
}

uint32_t crc32_any(uint32_t crc, const uint8_t* p, size_t n) {
  static const bool clmul = __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1");
  if (clmul) return crc32_fold(crc, p, n);
  for (size_t o = 0; o < n;) {
    const size_t step = std::min<size_t>(n - o, (size_t)1 << 30);
    crc = (uint32_t)crc32(crc, p + o, (uInt)step);
    o += step;
  }
  return crc;
}

size_t gzip_header_end(const uint8_t* in, size_t n) {
  if (n < 18 || in[0] != 0x1F || in[1] != 0x8B || in[2] != 8) return 0;
  const uint8_t flg = in[3];
  if (flg & 0xE0) return 0;
  size_t p = 10;
  if (flg & 4) {
    if (p + 2 > n) return 0;
    p += 2 + (in[p] | (in[p + 1] << 8));
  }
  for (int z : {8, 16})
    if (flg & z) {
      while (p < n && in[p]) p++;
      p++;
    }
  if (flg & 2) p += 2;
  return p < n ? p : 0;
}

}  // namespace

bool gunzip_chunked(const uint8_t* in, size_t n, size_t chunk_bytes, Inflated& out) {
  // G2N_PINFLATE_TRACE=1: phase times to stderr (diagnostics only; changes nothing)
  static const bool trace = getenv("G2N_PINFLATE_TRACE") != nullptr;
  const auto t0 = std::chrono::steady_clock::now();
  auto mark = [&](const char* what) {
    if (trace)
      fprintf(stderr, "[pinflate] %s %.1f ms\n", what,
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  };
  const size_t ds = gzip_header_end(in, n);
  if (!ds) return false;
  const int T = host_threads();
  if (!chunk_bytes) chunk_bytes = std::max<size_t>((size_t)4 << 20, (n - ds) / (4 * (size_t)std::max(T, 1)) + 1);
  const size_t nch = std::max<size_t>(1, (n - ds + chunk_bytes - 1) / chunk_bytes);
  std::vector<Chunk> ch(nch);

  // 1. chunk starts: the first plausible block start in each chunk's byte range
  ch[0].sync = (uint64_t)ds * 8;
  ch[0].present = true;
  parallel_for(nch - 1, T, [&](size_t j) {
    const size_t c = j + 1;
    const uint64_t lo = (uint64_t)(ds + c * chunk_bytes) * 8;
    const uint64_t hi = (uint64_t)std::min(n, ds + (c + 1) * chunk_bytes) * 8;
    for (uint64_t p = lo; p < hi; p++)
      if (plausible_start(in, n, p)) {
        ch[c].sync = p;
        ch[c].present = true;
        return;
      }
  });

  mark("sync");
  // 2. every present chunk decodes until it stands on a later chunk's start at a block boundary
  //    (a start that turns out false is stepped over), or to the stream's BFINAL block
  parallel_for(nch, T, [&](size_t k) {
    Chunk& c = ch[k];
    if (!c.present) return;
    const size_t guess = 5 * std::min(chunk_bytes, n) + ((size_t)1 << 20);  // GFA text deflates ~3.3:1
    c.out.reserve(guess);
    if (k) c.sh.reserve(kWin + guess);
    Dec dec(c, k != 0);
    BitIn br(in, n, c.sync);
    size_t j = k + 1;
    for (;;) {
      const uint64_t at = br.pos();
      while (j < nch && (!ch[j].present || ch[j].sync < at)) j++;
      if (j < nch && ch[j].sync == at) {
        c.next = j;
        break;
      }
      bool final = false;
      if (!dec.block(br, &final) || br.over) return;  // a false start (or a stream to refuse)
      if (final) {
        c.final_seen = true;
        break;
      }
    }
    dec.finish();
    c.end_bits = br.pos();
    c.ok = true;
  });
  mark("decode");
  std::vector<size_t> chain;
  for (size_t k = 0;;) {
    if (!ch[k].ok) return false;
    chain.push_back(k);
    if (ch[k].final_seen) break;
    k = ch[k].next;
  }
  const Chunk& tail = ch[chain.back()];
  const size_t trailer = (size_t)((tail.end_bits + 7) >> 3);
  if (trailer + 8 > n) return false;
  for (size_t p = trailer + 8; p < n; p++)
    if (in[p]) return false;  // another member (or garbage): the member-chain readers handle it

  // 3. windows in file order (each from the final bytes of the chunks before), then every
  //    chunk's unknown-window bytes in parallel, and the CRC
  size_t have = 0;
  std::unique_ptr<uint8_t[]> win(new uint8_t[kWin]());
  auto final_byte = [](const Chunk& x, const uint8_t* w, size_t p) -> int {
    if (p >= x.dirty_len) return x.out.p[p];
    const uint16_t v = x.sh.p[kWin + p];
    return v < 256 ? v : w[v - 256];
  };
  for (size_t k : chain) {
    Chunk& x = ch[k];
    x.win.reset(new uint8_t[kWin]);
    memcpy(x.win.get(), win.get(), kWin);
    if (x.dirty_len && have < kWin) {  // a reference before the stream's first byte?
      for (size_t p = 0; p < x.dirty_len; p++)
        if (x.sh.p[kWin + p] >= 256 && (size_t)(x.sh.p[kWin + p] - 256) < kWin - have) return false;
    }
    const size_t len = x.out.n;
    uint8_t nw[kWin];
    const size_t keep = len >= kWin ? 0 : kWin - len;
    memcpy(nw, win.get() + kWin - keep, keep);
    for (size_t q = keep; q < kWin; q++) nw[q] = (uint8_t)final_byte(x, x.win.get(), len - (kWin - q));
    memcpy(win.get(), nw, kWin);
    have = std::min(kWin, have + len);
  }
  mark("windows");
  std::vector<uLong> crc(chain.size());
  parallel_for(chain.size(), T, [&](size_t i) {
    Chunk& x = ch[chain[i]];
    const uint8_t* w = x.win.get();
    const uint16_t* sh = x.sh.p ? x.sh.p + kWin : nullptr;
    uint32_t c = 0;
    for (size_t o = 0; o < x.out.n;) {  // 64 KiB pieces: resolved, then CRC'd while in cache
      const size_t e = std::min(x.out.n, o + ((size_t)1 << 16));
      for (size_t p = o; p < std::min(e, x.dirty_len); p++) {
        const uint16_t v = sh[p];
        x.out.p[p] = v < 256 ? (uint8_t)v : w[v - 256];
      }
      c = crc32_any(c, x.out.p + o, e - o);
      o = e;
    }
    free(x.sh.p);
    x.sh.p = nullptr;
    crc[i] = c;
  });
  uLong total_crc = crc32(0L, Z_NULL, 0);
  size_t total = 0;
  for (size_t i = 0; i < chain.size(); i++) {
    total_crc = crc32_combine(total_crc, crc[i], (z_off_t)ch[chain[i]].out.n);  // z_off_t: 64-bit on LP64
    total += ch[chain[i]].out.n;
  }
  mark("resolve+crc");
  if (trace) fprintf(stderr, "[pinflate] %zu chunks, %zu on the chain, %zu B out\n", nch, chain.size(), total);
  const uint8_t* t = in + trailer;
  const uint32_t want_crc = t[0] | (t[1] << 8) | (t[2] << 16) | ((uint32_t)t[3] << 24);
  const uint32_t want_len = t[4] | (t[5] << 8) | (t[6] << 16) | ((uint32_t)t[7] << 24);
  if ((uint32_t)total_crc != want_crc || (uint32_t)total != want_len) return false;

  out = Inflated();
  out.members = 1;
  size_t at = 0;
  for (size_t k : chain) {
    Chunk& x = ch[k];
    out.start.push_back(at);
    at += x.out.n;
    HostBuf b;
    b.p = x.out.p;  // adopt the realloc'd block (HostBuf frees with free())
    b.n = x.out.n;
    x.out.p = nullptr;
    out.parts.push_back(std::move(b));
  }
  out.start.push_back(at);
  out.total = at;
  return true;
}

}  // namespace g2n
