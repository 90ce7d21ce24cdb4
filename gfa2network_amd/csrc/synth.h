// synth.h — deterministic synthetic pangenome-like GFA, host+device.
//
// The same counter-based generator runs on the CPU (files for the reference / oracle
// timings) and on the GPU (bench.py builds its HBM-resident workload in place), and both
// produce identical bytes for the same spec:
//   line 0:            H\tVN:Z:1.0
//   S lines i=1..N_S:  S\t{name(i)}\t{seq}  |seq| ~ Geometric(1/8) over ACGT;
//                      name(i) = "i", or (names = 1) "s" + 8 hex digits of a u32 bijection of i,
//                      or (names = 2) the decimal of a permutation of 1..N_S (affine mod N_S),
//                      or (names = 3) "s" + the decimal of i (minigraph's layout: prefixed, in S order)
//   L lines j:         L\t{name(src)}\t{o1}\t{name(dst)}\t{o2}\t0M[\tRC:i:{k}]
//                      src ~ U[1,N_S], dst = min(src + Geometric(5/16), N_S) (far = 1: dst ~ U[1,N_S]),
//                      o = '+' with probability 922/1024, k ~ U[1,99]
// Integer-only draws (splitmix64 of (seed, stream, index, chunk)) keep host == device.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define G2N_HD __host__ __device__
#else
#define G2N_HD
#endif

namespace g2n {

struct SynthSpec {
  uint64_t n_s, n_l, seed;
  int32_t rc;
  int32_t names;  // 0: decimal "i"; 1: hashed "s%08x" of synth_name_mix(i) (n_s < 2^32); 2: permuted decimal;
                  // 3: prefixed "s" + "i" in S order
  int32_t far;    // 1: dst ~ U[1, N_S] instead of src + Geometric(5/16)
  uint64_t pmul;  // names = 2: multiplier coprime to n_s (synth_perm_mul)
};

G2N_HD inline uint64_t synth_gcd(uint64_t a, uint64_t b) {
  while (b) {
    const uint64_t t = a % b;
    a = b;
    b = t;
  }
  return a;
}

// names = 2: segment i is named perm(i) = ((i - 1) * pmul + n_s / 2) mod n_s + 1, a bijection of 1..n_s
// (pmul coprime to n_s): decimal names "1".."N" in a shuffled order, perm(1) != 1 for n_s > 1
inline uint64_t synth_perm_mul(uint64_t n) {
  if (n < 2) return 1;
  uint64_t a = 2654435761ull % n;
  if (a < 2) a = 2;
  while (synth_gcd(a, n) != 1) a++;
  return a;
}

G2N_HD inline uint64_t synth_perm(const struct SynthSpec& s, uint64_t i) {
  return (uint64_t)(((unsigned __int128)(i - 1) * s.pmul + (s.n_s >> 1)) % s.n_s) + 1;
}

G2N_HD inline uint64_t smix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

G2N_HD inline uint64_t synth_rnd(uint64_t seed, uint64_t stream, uint64_t i, uint64_t k) {
  return smix64(smix64(seed ^ (stream << 56) ^ (k * 0x632BE59BD9B4E019ull)) ^ i);
}

G2N_HD inline uint32_t synth_digits(uint64_t x) {
  uint32_t d = 1;
  while (x >= 10) { x /= 10; d++; }
  return d;
}

// Geometric(1/8) on {1, 2, ...}: 3-bit trials, success on 0
G2N_HD inline uint32_t synth_seq_len(const SynthSpec& s, uint64_t i) {
  uint32_t n = 1;
  for (uint64_t k = 0; k < 64; k++) {
    uint64_t h = synth_rnd(s.seed, 1, i, k);
    for (int b = 0; b < 21; b++) {
      if (((h >> (3 * b)) & 7) == 0) return n;
      n++;
    }
  }
  return n;
}

struct SynthLink {
  uint64_t src, dst, k;
  char o1, o2;
};

G2N_HD inline SynthLink synth_link(const SynthSpec& s, uint64_t j) {
  SynthLink L;
  L.src = synth_rnd(s.seed, 3, j, 0) % s.n_s + 1;
  uint64_t g = 1;
  for (uint64_t k = 0; k < 64; k++) {  // Geometric(5/16): 4-bit trials, success below 5
    uint64_t h = synth_rnd(s.seed, 4, j, k);
    bool done = false;
    for (int b = 0; b < 16; b++) {
      if (((h >> (4 * b)) & 15) < 5) { done = true; break; }
      g++;
    }
    if (done) break;
  }
  L.dst = L.src + g > s.n_s ? s.n_s : L.src + g;
  if (s.far) L.dst = synth_rnd(s.seed, 7, j, 0) % s.n_s + 1;
  uint64_t h = synth_rnd(s.seed, 5, j, 0);
  L.o1 = (h & 1023) < 922 ? '+' : '-';
  L.o2 = ((h >> 10) & 1023) < 922 ? '+' : '-';
  L.k = synth_rnd(s.seed, 6, j, 0) % 99 + 1;
  return L;
}

G2N_HD inline uint32_t synth_name_len(const SynthSpec& s, uint64_t i);

G2N_HD inline uint64_t synth_n_lines(const SynthSpec& s) { return 1 + s.n_s + s.n_l; }

G2N_HD inline uint32_t synth_line_len(const SynthSpec& s, uint64_t line) {
  if (line == 0) return 11;  // "H\tVN:Z:1.0\n"
  if (line <= s.n_s) return 2 + synth_name_len(s, line) + 1 + synth_seq_len(s, line) + 1;
  SynthLink L = synth_link(s, line - 1 - s.n_s);
  uint32_t n = 2 + synth_name_len(s, L.src) + 3 + synth_name_len(s, L.dst) + 3 + 2 + 1;  // ...\t0M\n
  if (s.rc) n += 6 + synth_digits(L.k);
  return n;
}

G2N_HD inline char* synth_put_u64(char* o, uint64_t x) {
  uint32_t d = synth_digits(x);
  for (uint32_t k = d; k > 0; k--) {
    o[k - 1] = (char)('0' + x % 10);
    x /= 10;
  }
  return o + d;
}

// a bijection of u32 (xor-shift / odd-multiply steps are each invertible mod 2^32)
G2N_HD inline uint32_t synth_name_mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

G2N_HD inline uint32_t synth_name_len(const SynthSpec& s, uint64_t i) {
  return s.names == 1 ? 9u : (s.names == 3 ? 1u : 0u) + synth_digits(s.names == 2 ? synth_perm(s, i) : i);
}

G2N_HD inline char* synth_put_name(const SynthSpec& s, char* o, uint64_t i) {
  if (!s.names) return synth_put_u64(o, i);
  if (s.names == 2) return synth_put_u64(o, synth_perm(s, i));
  if (s.names == 3) {
    *o++ = 's';
    return synth_put_u64(o, i);
  }
  const uint32_t h = synth_name_mix((uint32_t)i);
  *o++ = 's';
  for (int k = 7; k >= 0; k--) {
    const uint32_t d = (h >> (4 * k)) & 15u;
    *o++ = (char)(d < 10 ? '0' + d : 'a' + d - 10);
  }
  return o;
}

G2N_HD inline void synth_write_line(const SynthSpec& s, uint64_t line, char* o) {
  if (line == 0) {
    const char h[11] = {'H', '\t', 'V', 'N', ':', 'Z', ':', '1', '.', '0', '\n'};
    for (int k = 0; k < 11; k++) o[k] = h[k];
    return;
  }
  if (line <= s.n_s) {
    *o++ = 'S';
    *o++ = '\t';
    o = synth_put_name(s, o, line);
    *o++ = '\t';
    uint32_t n = synth_seq_len(s, line);
    const char acgt[4] = {'A', 'C', 'G', 'T'};
    for (uint32_t p = 0; p < n; p += 32) {
      uint64_t h = synth_rnd(s.seed, 2, line, p / 32);
      for (uint32_t q = p; q < n && q < p + 32; q++) *o++ = acgt[(h >> (2 * (q - p))) & 3];
    }
    *o = '\n';
    return;
  }
  SynthLink L = synth_link(s, line - 1 - s.n_s);
  *o++ = 'L';
  *o++ = '\t';
  o = synth_put_name(s, o, L.src);
  *o++ = '\t';
  *o++ = L.o1;
  *o++ = '\t';
  o = synth_put_name(s, o, L.dst);
  *o++ = '\t';
  *o++ = L.o2;
  *o++ = '\t';
  *o++ = '0';
  *o++ = 'M';
  if (s.rc) {
    *o++ = '\t';
    *o++ = 'R';
    *o++ = 'C';
    *o++ = ':';
    *o++ = 'i';
    *o++ = ':';
    o = synth_put_u64(o, L.k);
  }
  *o = '\n';
}

}  // namespace g2n
