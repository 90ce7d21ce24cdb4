// g2n_inflate.hip — BGZF members inflated on the GPU (gzip.open of a bgzip file, parser.py:108-109).
//
// A BGZF file (htslib's bgzip) is a chain of gzip members of at most 64 KiB of output, each
// carrying its own total size in a 'BC' header subfield, so the host locates every member from
// the headers alone (bgzf_members, g2n_ingest.cpp) and the members inflate independently: one
// lane per member, RFC 1951 decoded canonically (stored / fixed / dynamic blocks; the Huffman
// count + symbol tables of each lane in LDS), the output written at the member's offset and its
// CRC-32 and length checked against the trailer.  Anything unexpected — an invalid or incomplete
// code, a distance past the output, a length or CRC mismatch — marks the member bad, and the
// host then reads the file with its exact gzip.py restatement instead (same bytes, or the same
// exception), so this path never decides an error itself.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "g2n_internal.h"

namespace g2n {

constexpr uint32_t kInflTPB = 64;  // one wave per block: 64 members, ~1 KB of LDS tables each

struct InflTables {
  uint8_t lens[320];           // code lengths of one dynamic block (literal/length + distance)
  uint16_t lcount[16], lsym[288];
  uint16_t dcount[16], dsym[32];
  uint16_t offs[16];
};
// k_inflate_members' LDS (kInflTPB tables + the 1 KB CRC table, ~68.6 KB) is sized for gfx950's
// 160 KB per CU; a 64 KB-LDS target would fail at launch, not here
static_assert(kInflTPB * sizeof(InflTables) + 256 * sizeof(uint32_t) <= 160 * 1024,
              "k_inflate_members: LDS tables exceed gfx950's 160 KB");

__constant__ uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                      31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t kDistBase[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,   65,    97,    129,
                                       193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

struct BitIn {
  const uint8_t* p;
  uint32_t n, pos;
  uint64_t buf;
  uint32_t cnt;
  __device__ void refill() {
    while (cnt <= 56 && pos < n) {
      buf |= (uint64_t)p[pos++] << cnt;
      cnt += 8;
    }
  }
  __device__ bool bits(uint32_t k, uint32_t* v) {  // k <= 32
    if (cnt < k) {
      refill();
      if (cnt < k) return false;
    }
    *v = (uint32_t)(buf & ((1ull << k) - 1));
    buf >>= k;
    cnt -= k;
    return true;
  }
};

// canonical Huffman table from n code lengths; false unless the code is complete (zlib accepts
// some incomplete codes; those members go to the host reader)
__device__ inline bool infl_build(const uint8_t* len, uint32_t n, uint16_t* count, uint16_t* sym, uint16_t* offs) {
  for (int l = 0; l < 16; l++) count[l] = 0;
  for (uint32_t s = 0; s < n; s++) count[len[s]]++;
  if (count[0] == n) return false;
  int left = 1;
  for (int l = 1; l < 16; l++) {
    left <<= 1;
    left -= count[l];
    if (left < 0) return false;
  }
  if (left != 0) return false;
  offs[1] = 0;
  for (int l = 1; l < 15; l++) offs[l + 1] = offs[l] + count[l];
  for (uint32_t s = 0; s < n; s++)
    if (len[s]) sym[offs[len[s]]++] = (uint16_t)s;
  return true;
}

// one symbol; -1 when the bits run out or the code is not in the table
__device__ inline int infl_decode(BitIn& b, const uint16_t* count, const uint16_t* sym) {
  if (b.cnt < 15) b.refill();
  uint32_t peek = (uint32_t)b.buf;
  int code = 0, first = 0, index = 0;
  for (uint32_t l = 1; l <= 15 && l <= b.cnt; l++) {
    code |= (int)(peek & 1u);
    peek >>= 1;
    const int c = count[l];
    if (code - c < first) {
      b.buf >>= l;
      b.cnt -= l;
      return sym[index + (code - first)];
    }
    index += c;
    first += c;
    first <<= 1;
    code <<= 1;
  }
  return -1;
}

__global__ void __launch_bounds__(kInflTPB) k_inflate_members(const uint8_t* __restrict__ z,
                                                              const ZMember* __restrict__ mem, uint64_t n_members,
                                                              uint8_t* __restrict__ out,
                                                              unsigned int* __restrict__ n_bad) {
  __shared__ InflTables tabs[kInflTPB];
  __shared__ uint32_t crc_tab[256];
  // 64 x 1056 B + 1 KB = 68.6 KB: needs gfx950's 160 KB of LDS per workgroup (the Makefile's
  // ARCH is gfx950; older CDNA parts have 64 KB and would fail this launch)
  static_assert(sizeof(tabs) + sizeof(crc_tab) <= 160 * 1024, "k_inflate_members LDS exceeds gfx950's 160 KB");
  for (uint32_t k = threadIdx.x; k < 256; k += kInflTPB) {
    uint32_t c = k;
    for (int j = 0; j < 8; j++) c = (c & 1u) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    crc_tab[k] = c;
  }
  __syncthreads();
  const uint64_t mi = (uint64_t)blockIdx.x * kInflTPB + threadIdx.x;
  if (mi >= n_members) return;
  InflTables& T = tabs[threadIdx.x];
  const ZMember m = mem[mi];
  BitIn b{z + m.in_off, m.in_len, 0, 0ull, 0};
  uint8_t* dst = out + m.out_off;
  const uint32_t cap = m.out_len;
  uint32_t pos = 0, crc = 0xFFFFFFFFu;
  bool ok = true, last = false;
  auto put = [&](uint8_t v) {
    dst[pos++] = v;
    crc = crc_tab[(crc ^ v) & 0xFFu] ^ (crc >> 8);
  };
  while (ok && !last) {
    uint32_t hdr;
    if (!b.bits(3, &hdr)) {
      ok = false;
      break;
    }
    last = hdr & 1u;
    const uint32_t type = hdr >> 1;
    if (type == 0) {  // stored: to the byte boundary, LEN, NLEN, LEN bytes
      const uint32_t drop = b.cnt & 7u;
      b.buf >>= drop;
      b.cnt -= drop;
      uint32_t ln, nln;
      if (!b.bits(16, &ln) || !b.bits(16, &nln) || (ln ^ 0xFFFFu) != nln || pos + ln > cap) {
        ok = false;
        break;
      }
      for (uint32_t k = 0; k < ln && ok; k++) {
        uint32_t v;
        ok = b.bits(8, &v);
        if (ok) put((uint8_t)v);
      }
      continue;
    }
    if (type == 1) {  // fixed codes
      for (int s = 0; s < 288; s++) T.lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
      for (int s = 0; s < 30; s++) T.lens[288 + s] = 5;
      // the fixed literal/length code is complete; the fixed distance code (30 of 32) is not, as
      // RFC 1951 defines it: build it by hand
      ok = infl_build(T.lens, 288, T.lcount, T.lsym, T.offs);
      for (int l = 0; l < 16; l++) T.dcount[l] = 0;
      T.dcount[5] = 30;
      for (int s = 0; s < 30; s++) T.dsym[s] = (uint16_t)s;
    } else if (type == 2) {  // dynamic codes
      uint32_t nlen, ndist, ncode;
      if (!b.bits(5, &nlen) || !b.bits(5, &ndist) || !b.bits(4, &ncode)) {
        ok = false;
        break;
      }
      nlen += 257;
      ndist += 1;
      ncode += 4;
      if (nlen > 286 || ndist > 30) {
        ok = false;
        break;
      }
      for (int k = 0; k < 19; k++) T.lens[k] = 0;
      for (uint32_t k = 0; k < ncode && ok; k++) {
        uint32_t v;
        ok = b.bits(3, &v);
        T.lens[kClOrder[k]] = (uint8_t)v;
      }
      ok = ok && infl_build(T.lens, 19, T.lcount, T.lsym, T.offs);  // the code-length code
      uint32_t idx = 0;
      while (ok && idx < nlen + ndist) {
        const int s = infl_decode(b, T.lcount, T.lsym);
        if (s < 0) {
          ok = false;
        } else if (s < 16) {
          T.lens[idx++] = (uint8_t)s;
        } else {
          uint32_t rep, v = 0;
          if (s == 16) {
            if (idx == 0 || !b.bits(2, &rep)) {
              ok = false;
              break;
            }
            v = T.lens[idx - 1];
            rep += 3;
          } else if (s == 17) {
            ok = b.bits(3, &rep);
            rep += 3;
          } else {
            ok = b.bits(7, &rep);
            rep += 11;
          }
          if (!ok || idx + rep > nlen + ndist) {
            ok = false;
            break;
          }
          while (rep--) T.lens[idx++] = (uint8_t)v;
        }
      }
      ok = ok && T.lens[256] != 0;  // an end-of-block code must exist
      ok = ok && infl_build(T.lens, nlen, T.lcount, T.lsym, T.offs) &&
           infl_build(T.lens + nlen, ndist, T.dcount, T.dsym, T.offs);
    } else {
      ok = false;
    }
    while (ok) {  // the block's symbols
      const int s = infl_decode(b, T.lcount, T.lsym);
      if (s < 0 || s > 285) {
        ok = false;
      } else if (s < 256) {
        if (pos >= cap) ok = false;
        else put((uint8_t)s);
      } else if (s == 256) {
        break;
      } else {
        uint32_t e, ln = kLenBase[s - 257], d;
        if (!b.bits(kLenExtra[s - 257], &e)) {
          ok = false;
          break;
        }
        ln += e;
        const int ds = infl_decode(b, T.dcount, T.dsym);
        if (ds < 0 || ds > 29 || !b.bits(kDistExtra[ds], &e)) {
          ok = false;
          break;
        }
        d = kDistBase[ds] + e;
        if (d > pos || pos + ln > cap) {
          ok = false;
          break;
        }
        for (uint32_t k = 0; k < ln; k++) put(dst[pos - d]);
      }
    }
  }
  // the deflate data must end exactly where the member's trailer starts (gzip.py reads the
  // trailer right after the final block), its output be ISIZE bytes with the trailer's CRC
  ok = ok && b.pos - b.cnt / 8 == b.n && pos == cap && (crc ^ 0xFFFFFFFFu) == m.crc;
  if (!ok) atomicAdd(n_bad, 1u);
}

}  // namespace g2n
