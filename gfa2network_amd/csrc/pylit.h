// pylit.h — CPython literal semantics the reference relies on, as host+device code.
//
// The reference turns GFA bytes into numbers with CPython builtins:
//   * tag values:  int(value) / float(value) on a decoded str   gfa2network/parser.py:187-198
//   * E/C coords:  int(fields[k]) on bytes (a validity test)      gfa2network/parser.py:255-263, 303-311
//   * weights:     float(val) of the tag's int                    gfa2network/builders.py:209
//   * .decode():   strict UTF-8 (orientation fields, tag fields)  parser.py:183, 212, 291, 337
// Restated here from CPython 3.10's published behaviour (Objects/longobject.c
// PyLong_FromString, Objects/unicodeobject.c _PyUnicode_TransformDecimalAndSpaceToASCII,
// Objects/floatobject.c float_from_string_inner, Python/pystrtod.c _Py_parse_inf_or_nan,
// Python/dtoa.c grammar; correctly rounded decimal->binary64) so the GPU path can run
// them for every edge.  Correct rounding of arbitrary decimal strings uses a big-decimal
// shift-and-round conversion (the "simple decimal conversion" of the Go strconv package's
// decimal.go, rewritten here): exact for any digit count, used only on the slow path.
//
// Everything is G2N_HD so tests/test_host_headers.py (tests/native/hostcheck.cpp) compiles it with g++ and fuzzes
// it against CPython's own int()/float() on the CPU; the GPU kernels include the same code.
#pragma once
#include <stdint.h>

#include "unicode_tables.h"

#if defined(__HIPCC__)
#define G2N_HD __host__ __device__
#else
#define G2N_HD
#endif

namespace g2n {

// ------------------------------------------------------------------ UTF-8 --------
// CPython's strict decoder: no overlongs, no surrogates, nothing above U+10FFFF.
G2N_HD inline bool utf8_valid(const uint8_t* p, uint64_t n) {
  uint64_t i = 0;
  while (i < n) {
    uint8_t c = p[i];
    if (c < 0x80) { i++; continue; }
    int len;
    uint8_t lo = 0x80, hi = 0xBF;
    if (c >= 0xC2 && c <= 0xDF) len = 2;
    else if (c == 0xE0) { len = 3; lo = 0xA0; }
    else if (c >= 0xE1 && c <= 0xEC) len = 3;
    else if (c == 0xED) { len = 3; hi = 0x9F; }
    else if (c >= 0xEE && c <= 0xEF) len = 3;
    else if (c == 0xF0) { len = 4; lo = 0x90; }
    else if (c >= 0xF1 && c <= 0xF3) len = 4;
    else if (c == 0xF4) { len = 4; hi = 0x8F; }
    else return false;
    if (i + (uint64_t)len > n) return false;
    uint8_t c1 = p[i + 1];
    if (c1 < lo || c1 > hi) return false;
    for (int k = 2; k < len; k++) {
      uint8_t ck = p[i + k];
      if (ck < 0x80 || ck > 0xBF) return false;
    }
    i += (uint64_t)len;
  }
  return true;
}

// Next code point of VALID UTF-8.
G2N_HD inline uint32_t utf8_next(const uint8_t* p, uint64_t* i) {
  uint8_t c = p[*i];
  if (c < 0x80) { *i += 1; return c; }
  if (c < 0xE0) { uint32_t cp = ((uint32_t)(c & 0x1F) << 6) | (p[*i + 1] & 0x3F); *i += 2; return cp; }
  if (c < 0xF0) {
    uint32_t cp = ((uint32_t)(c & 0x0F) << 12) | ((uint32_t)(p[*i + 1] & 0x3F) << 6) | (p[*i + 2] & 0x3F);
    *i += 3;
    return cp;
  }
  uint32_t cp = ((uint32_t)(c & 0x07) << 18) | ((uint32_t)(p[*i + 1] & 0x3F) << 12) |
                ((uint32_t)(p[*i + 2] & 0x3F) << 6) | (p[*i + 3] & 0x3F);
  *i += 4;
  return cp;
}

// _PyUnicode_TransformDecimalAndSpaceToASCII for one code point: the ASCII char it becomes
// (code points < 127 unchanged), or -1 when it makes the literal invalid.
G2N_HD inline int py_transform_cp(uint32_t cp) {
  if (cp < 127) return (int)cp;
  for (int k = 0; k < G2N_UNI_NSPACE; k++)
    if (g2n_uni_space[k] == cp) return ' ';
  for (int k = 0; k < G2N_UNI_NDIGIT_RUNS; k++)
    if (cp >= g2n_uni_digit_first[k] && cp <= g2n_uni_digit_last[k])
      return '0' + (int)g2n_uni_digit_value[k] + (int)(cp - g2n_uni_digit_first[k]);
  return -1;
}

G2N_HD inline bool py_isspace(int c) {  // Py_ISSPACE (ASCII)
  return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f';
}
G2N_HD inline bool py_isdigit(int c) { return c >= '0' && c <= '9'; }

// Iterates the chars a literal is parsed from: bytes as-is (int(bytes)) or the
// transform of a decoded str (int(str) / float(str)).
struct CharIter {
  const uint8_t* p;
  uint64_t n, i;
  bool transform;
  G2N_HD bool done() const { return i >= n; }
  G2N_HD int next() {
    if (!transform) return p[i++];  // bytes: >= 0x80 is not a digit/space/sign -> invalid
    uint32_t cp = utf8_next(p, &i);
    return py_transform_cp(cp);
  }
};

// ------------------------------------------------------- big decimal -> binary64 --
// value = 0.d[0]d[1]...d[nd-1] * 10^dp ; digits beyond DEC_MAX are dropped with trunc set.
constexpr int DEC_MAX = 800;
constexpr int DEC_TMP = 820;

struct Decimal {
  uint8_t d[DEC_MAX];
  int32_t nd;
  int32_t dp;
  bool neg;
  bool trunc;
  bool sig;  // a significant (non-leading-zero) digit has been seen
};

G2N_HD inline void dec_init(Decimal* a) {
  a->nd = 0;
  a->dp = 0;
  a->neg = false;
  a->trunc = false;
  a->sig = false;
}

// A mantissa digit before the decimal point.
G2N_HD inline void dec_int_digit(Decimal* a, int c) {
  if (!a->sig && c == 0) return;
  a->sig = true;
  if (a->nd < DEC_MAX) a->d[a->nd++] = (uint8_t)c;
  else if (c != 0) a->trunc = true;
  if (a->dp < 1000000000) a->dp++;
}

// A mantissa digit after the decimal point.
G2N_HD inline void dec_frac_digit(Decimal* a, int c) {
  if (!a->sig && c == 0) {
    if (a->dp > -1000000000) a->dp--;
    return;
  }
  a->sig = true;
  if (a->nd < DEC_MAX) a->d[a->nd++] = (uint8_t)c;
  else if (c != 0) a->trunc = true;
}

G2N_HD inline void dec_trim(Decimal* a) {
  while (a->nd > 0 && a->d[a->nd - 1] == 0) a->nd--;
  if (a->nd == 0) a->dp = 0;
}

// divide by 2^k, k <= 60
G2N_HD inline void dec_rshift(Decimal* a, uint32_t k) {
  int r = 0, w = 0;
  uint64_t n = 0;
  for (; (n >> k) == 0; r++) {
    if (r >= a->nd) {
      if (n == 0) {
        a->nd = 0;
        return;
      }
      while ((n >> k) == 0) {
        n = n * 10;
        r++;
      }
      break;
    }
    n = n * 10 + a->d[r];
  }
  a->dp -= r - 1;
  const uint64_t mask = (((uint64_t)1) << k) - 1;
  for (; r < a->nd; r++) {
    uint64_t c = a->d[r];
    uint64_t dig = n >> k;
    n &= mask;
    a->d[w++] = (uint8_t)dig;
    n = n * 10 + c;
  }
  while (n > 0) {
    uint64_t dig = n >> k;
    n &= mask;
    if (w < DEC_MAX) a->d[w++] = (uint8_t)dig;
    else if (dig > 0) a->trunc = true;
    n = n * 10;
  }
  a->nd = w;
  dec_trim(a);
}

// multiply by 2^k, k <= 60 (tmp: DEC_TMP bytes of scratch)
G2N_HD inline void dec_lshift(Decimal* a, uint32_t k, uint8_t* tmp) {
  int w = DEC_TMP;
  uint64_t n = 0;
  for (int r = a->nd - 1; r >= 0; r--) {
    n += ((uint64_t)a->d[r]) << k;
    uint64_t q = n / 10;
    tmp[--w] = (uint8_t)(n - 10 * q);
    n = q;
  }
  while (n > 0) {
    uint64_t q = n / 10;
    tmp[--w] = (uint8_t)(n - 10 * q);
    n = q;
  }
  int len = DEC_TMP - w;
  int delta = len - a->nd;
  int keep = len < DEC_MAX ? len : DEC_MAX;
  for (int i = 0; i < keep; i++) a->d[i] = tmp[w + i];
  for (int i = keep; i < len; i++)
    if (tmp[w + i]) a->trunc = true;
  a->nd = keep;
  a->dp += delta;
  dec_trim(a);
}

G2N_HD inline void dec_shift(Decimal* a, int k, uint8_t* tmp) {
  if (a->nd == 0) return;
  if (k > 0) {
    while (k > 60) { dec_lshift(a, 60, tmp); k -= 60; }
    dec_lshift(a, (uint32_t)k, tmp);
  } else if (k < 0) {
    while (k < -60) { dec_rshift(a, 60); k += 60; }
    dec_rshift(a, (uint32_t)(-k));
  }
}

G2N_HD inline bool dec_round_up(const Decimal* a, int nd) {
  if (nd < 0 || nd >= a->nd) return false;
  if (a->d[nd] == 5 && nd + 1 == a->nd) {  // exactly halfway: to even (or up if truncated)
    if (a->trunc) return true;
    return nd > 0 && (a->d[nd - 1] % 2) == 1;
  }
  return a->d[nd] >= 5;
}

G2N_HD inline uint64_t dec_rounded_integer(const Decimal* a) {
  if (a->dp > 20) return ~(uint64_t)0;
  int i;
  uint64_t n = 0;
  for (i = 0; i < a->dp && i < a->nd; i++) n = n * 10 + a->d[i];
  for (; i < a->dp; i++) n *= 10;
  if (dec_round_up(a, a->dp)) n++;
  return n;
}

// Correctly rounded (to nearest, ties to even) binary64 bits of the decimal; *overflow
// set (and +-inf returned) when the rounded value exceeds DBL_MAX.
constexpr int kPowTab[9] = {1, 3, 6, 9, 13, 16, 19, 23, 26};
constexpr double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                               1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

G2N_HD inline uint64_t dec_to_f64_bits(Decimal* d, bool* overflow, uint8_t* tmp) {
  const int mantbits = 52, expbits = 11, bias = -1023;
  int exp = 0;
  uint64_t mant = 0;
  uint64_t bits;
  *overflow = false;
  if (d->nd == 0) {
    exp = bias;
    goto out;
  }
  if (d->dp > 310) goto ovf;
  if (d->dp < -330) {
    exp = bias;
    goto out;
  }
  while (d->dp > 0) {
    int n = d->dp >= 9 ? 27 : kPowTab[d->dp];
    dec_shift(d, -n, tmp);
    exp += n;
  }
  while (d->dp < 0 || (d->dp == 0 && d->d[0] < 5)) {
    int n = -d->dp >= 9 ? 27 : kPowTab[-d->dp];
    dec_shift(d, n, tmp);
    exp -= n;
  }
  exp--;  // [0.5, 1) -> [1, 2)
  if (exp < bias + 1) {
    int n = bias + 1 - exp;
    dec_shift(d, -n, tmp);
    exp += n;
  }
  if (exp - bias >= (1 << expbits) - 1) goto ovf;
  dec_shift(d, 1 + mantbits, tmp);
  mant = dec_rounded_integer(d);
  if (mant == (((uint64_t)2) << mantbits)) {
    mant >>= 1;
    exp++;
    if (exp - bias >= (1 << expbits) - 1) goto ovf;
  }
  if ((mant & (((uint64_t)1) << mantbits)) == 0) exp = bias;  // denormal
  goto out;
ovf:
  mant = 0;
  exp = (1 << expbits) - 1 + bias;
  *overflow = true;
out:
  bits = mant & ((((uint64_t)1) << mantbits) - 1);
  bits |= ((uint64_t)((exp - bias) & ((1 << expbits) - 1))) << mantbits;
  if (d->neg) bits |= ((uint64_t)1) << 63;
  return bits;
}

G2N_HD inline double bits_f64(uint64_t b) {
  union { uint64_t u; double d; } x;
  x.u = b;
  return x.d;
}
G2N_HD inline uint64_t f64_bits(double v) {
  union { uint64_t u; double d; } x;
  x.d = v;
  return x.u;
}

// ------------------------------------------------------------- int() --------------
// PyLong_FromString(base 10) acceptance: ws* [+-]? D(_?D)* ws*, at most 4300 digits
// (sys.int_info.default_max_str_digits); ws = Py_ISSPACE.  `transform` selects int(str)
// (non-ASCII space/digits mapped first) vs int(bytes) (ASCII only).  When dec != nullptr
// the digits are accumulated into it as an integer.
G2N_HD inline bool py_int_literal(const uint8_t* p, uint64_t n, bool transform, Decimal* dec) {
  enum { LEAD, SIGN, DIG, UND, TRAIL };
  int st = LEAD;
  uint64_t ndig = 0;
  bool neg = false;
  if (dec) dec_init(dec);
  CharIter it{p, n, 0, transform};
  while (!it.done()) {
    int c = it.next();
    if (c < 0 || c == 0) return false;
    switch (st) {
      case LEAD:
        if (py_isspace(c)) break;
        if (c == '+' || c == '-') { neg = c == '-'; st = SIGN; break; }
        if (py_isdigit(c)) { st = DIG; ndig++; if (dec) dec_int_digit(dec, c - '0'); break; }
        return false;
      case SIGN:
        if (py_isdigit(c)) { st = DIG; ndig++; if (dec) dec_int_digit(dec, c - '0'); break; }
        return false;
      case DIG:
        if (py_isdigit(c)) { ndig++; if (dec) dec_int_digit(dec, c - '0'); break; }
        if (c == '_') { st = UND; break; }
        if (py_isspace(c)) { st = TRAIL; break; }
        return false;
      case UND:
        if (py_isdigit(c)) { st = DIG; ndig++; if (dec) dec_int_digit(dec, c - '0'); break; }
        return false;
      default:  // TRAIL
        if (py_isspace(c)) break;
        return false;
    }
  }
  if (!(st == DIG || st == TRAIL)) return false;
  if (ndig > 4300) return false;
  if (dec) {
    dec_trim(dec);
    dec->neg = neg && dec->nd > 0;  // ints have no negative zero
  }
  return true;
}

// float(int): OverflowError when the correctly rounded value exceeds DBL_MAX.
G2N_HD inline bool py_int_to_f64(Decimal* dec, double* out, uint8_t* tmp) {
  bool ovf;
  uint64_t b = dec_to_f64_bits(dec, &ovf, tmp);
  if (ovf) return false;
  *out = bits_f64(b);
  return true;
}

// ------------------------------------------------------------ float() ------------
G2N_HD inline int ascii_lower(int c) { return (c >= 'A' && c <= 'Z') ? c - 'A' + 'a' : c; }

// float(str): underscores only between digits (_Py_string_to_number_with_underscores),
// ws stripped, then [+-]?(D+[.D*]|.D+)([eE][+-]?D+)? or [+-]?(inf|infinity|nan), any case.
G2N_HD inline bool py_float_literal(const uint8_t* p, uint64_t n, bool transform, double* out, Decimal* dec,
                                    uint8_t* tmp) {
  enum { LEAD, SIGN, INT, DOT0, FRAC, E, ESIGN, EDIG, WORD, TRAIL };
  int st = LEAD;
  bool neg = false, eneg = false, word_ok = false;
  int64_t ev = 0;
  char word[9];
  int wl = 0;
  int prev = 0;
  bool pend_us = false;
  dec_init(dec);
  CharIter it{p, n, 0, transform};
  while (!it.done()) {
    int c = it.next();
    if (c < 0 || c == 0) return false;
    if (c == '_') {
      if (!py_isdigit(prev)) return false;
      pend_us = true;
      prev = c;
      continue;
    }
    if (pend_us && !py_isdigit(c)) return false;
    pend_us = false;
    prev = c;
    switch (st) {
      case LEAD:
        if (py_isspace(c)) break;
        if (c == '+' || c == '-') { neg = c == '-'; st = SIGN; break; }
        /* fallthrough */
      case SIGN:
        if (py_isdigit(c)) { st = INT; dec_int_digit(dec, c - '0'); break; }
        if (c == '.') { st = DOT0; break; }
        if ((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z')) { st = WORD; word[wl++] = (char)ascii_lower(c); break; }
        return false;
      case INT:
        if (py_isdigit(c)) { dec_int_digit(dec, c - '0'); break; }
        if (c == '.') { st = FRAC; break; }
        if (c == 'e' || c == 'E') { st = E; break; }
        if (py_isspace(c)) { st = TRAIL; break; }
        return false;
      case DOT0:
        if (py_isdigit(c)) { st = FRAC; dec_frac_digit(dec, c - '0'); break; }
        return false;
      case FRAC:
        if (py_isdigit(c)) { dec_frac_digit(dec, c - '0'); break; }
        if (c == 'e' || c == 'E') { st = E; break; }
        if (py_isspace(c)) { st = TRAIL; break; }
        return false;
      case E:
        if (c == '+' || c == '-') { eneg = c == '-'; st = ESIGN; break; }
        /* fallthrough */
      case ESIGN:
        if (py_isdigit(c)) { st = EDIG; ev = c - '0'; break; }
        return false;
      case EDIG:
        if (py_isdigit(c)) { if (ev < 100000000) ev = ev * 10 + (c - '0'); break; }
        if (py_isspace(c)) { st = TRAIL; break; }
        return false;
      case WORD:
        if ((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z')) {
          if (wl >= 8) return false;
          word[wl++] = (char)ascii_lower(c);
          break;
        }
        if (py_isspace(c)) { st = TRAIL; word_ok = true; break; }
        return false;
      default:  // TRAIL
        if (py_isspace(c)) break;
        return false;
    }
  }
  if (pend_us) return false;
  if (st == WORD) word_ok = true;
  if (word_ok) {
    word[wl] = 0;
    bool is_inf = (wl == 3 && word[0] == 'i' && word[1] == 'n' && word[2] == 'f') ||
                  (wl == 8 && word[0] == 'i' && word[1] == 'n' && word[2] == 'f' && word[3] == 'i' &&
                   word[4] == 'n' && word[5] == 'i' && word[6] == 't' && word[7] == 'y');
    bool is_nan = wl == 3 && word[0] == 'n' && word[1] == 'a' && word[2] == 'n';
    if (is_inf) { *out = bits_f64(neg ? 0xFFF0000000000000ull : 0x7FF0000000000000ull); return true; }
    if (is_nan) { *out = bits_f64(neg ? 0xFFF8000000000000ull : 0x7FF8000000000000ull); return true; }
    return false;
  }
  if (!(st == INT || st == FRAC || st == EDIG || st == TRAIL)) return false;
  dec_trim(dec);
  if (dec->nd > 0) {
    int64_t e = eneg ? -ev : ev;
    int64_t ndp = (int64_t)dec->dp + e;
    if (ndp > 100000) ndp = 100000;
    if (ndp < -100000) ndp = -100000;
    dec->dp = (int32_t)ndp;
  }
  dec->neg = neg;
  bool ovf;
  *out = bits_f64(dec_to_f64_bits(dec, &ovf, tmp));  // float() returns +-inf on overflow
  return true;
}

// ------------------------------------------------------------ fast paths ----------
// Fast grammars the parse kernel resolves inline; anything else is deferred to the exact
// slow path above (same result, just slower).
// int:   [+-]?[0-9]{1,15}                      (exact in binary64)
G2N_HD inline bool fast_int(const uint8_t* p, uint64_t n, double* out) {
  uint64_t i = 0;
  bool neg = false;
  if (n == 0) return false;
  if (p[0] == '+' || p[0] == '-') { neg = p[0] == '-'; i = 1; }
  uint64_t nd = n - i;
  if (nd == 0 || nd > 15) return false;
  int64_t v = 0;
  for (; i < n; i++) {
    uint8_t c = p[i];
    if (c < '0' || c > '9') return false;
    v = v * 10 + (c - '0');
  }
  *out = (double)(neg ? -v : v);  // -0 -> +0.0 (ints have no negative zero)
  return true;
}

// float: [+-]?D*[.D*]([eE][+-]?D{1,3})? with 1..15 mantissa digits and a decimal exponent
// of magnitude <= 22 (Clinger's exact case: one correctly rounded multiply or divide).
G2N_HD inline bool fast_float(const uint8_t* p, uint64_t n, double* out) {
  uint64_t i = 0;
  bool neg = false;
  if (n == 0) return false;
  if (p[0] == '+' || p[0] == '-') { neg = p[0] == '-'; i = 1; }
  uint64_t m = 0;
  int nd = 0, fd = 0;
  bool dot = false;
  for (; i < n; i++) {
    uint8_t c = p[i];
    if (c >= '0' && c <= '9') {
      if (++nd > 15) return false;
      m = m * 10 + (c - '0');
      if (dot) fd++;
    } else if (c == '.' && !dot) {
      dot = true;
    } else {
      break;
    }
  }
  if (nd == 0) return false;
  int e = 0;
  if (i < n) {
    if (p[i] != 'e' && p[i] != 'E') return false;
    i++;
    bool en = false;
    if (i < n && (p[i] == '+' || p[i] == '-')) { en = p[i] == '-'; i++; }
    int ed = 0;
    for (; i < n; i++) {
      uint8_t c = p[i];
      if (c < '0' || c > '9') return false;
      if (++ed > 3) return false;
      e = e * 10 + (c - '0');
    }
    if (ed == 0) return false;
    if (en) e = -e;
  }
  int E = e - fd;
  double v;
  if (m == 0) {
    v = 0.0;
  } else if (E >= 0 && E <= 22) {
    v = (double)m * kPow10[E];
  } else if (E < 0 && E >= -22) {
    v = (double)m / kPow10[-E];
  } else {
    return false;
  }
  *out = neg ? -v : v;
  return true;
}

}  // namespace g2n
