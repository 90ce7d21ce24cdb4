// Host build of the product's host+device headers (pylit.h, stl_sort.h) so the CPU test
// suite can fuzz them against CPython's int()/float() and libstdc++'s std::sort.
#include <algorithm>
#include <cstdint>
#include <vector>

#include "../../gfa2network_amd/csrc/pylit.h"
#include "../../gfa2network_amd/csrc/stl_sort.h"

extern "C" {

int hc_py_float(const uint8_t* p, int64_t n, double* out) {
  if (!g2n::utf8_valid(p, (uint64_t)n)) return 0;
  static thread_local g2n::Decimal dec;
  uint8_t tmp[g2n::DEC_TMP];
  return g2n::py_float_literal(p, (uint64_t)n, true, out, &dec, tmp) ? 1 : 0;
}

// 0 invalid, 1 ok (*out = float(int(s))), 2 valid int whose float() overflows
int hc_py_int(const uint8_t* p, int64_t n, int transform, double* out) {
  if (transform && !g2n::utf8_valid(p, (uint64_t)n)) return 0;
  static thread_local g2n::Decimal dec;
  uint8_t tmp[g2n::DEC_TMP];
  if (!g2n::py_int_literal(p, (uint64_t)n, transform != 0, &dec)) return 0;
  return g2n::py_int_to_f64(&dec, out, tmp) ? 1 : 2;
}

int hc_fast_int(const uint8_t* p, int64_t n, double* out) { return g2n::fast_int(p, (uint64_t)n, out) ? 1 : 0; }
int hc_fast_float(const uint8_t* p, int64_t n, double* out) { return g2n::fast_float(p, (uint64_t)n, out) ? 1 : 0; }
int hc_utf8_valid(const uint8_t* p, int64_t n) { return g2n::utf8_valid(p, (uint64_t)n) ? 1 : 0; }

// Sort (key, original position) pairs by key with std::sort and with the restatement;
// write both resulting position permutations.
void hc_sort_both(const int32_t* keys, int64_t n, int32_t* out_std, int32_t* out_emul) {
  std::vector<std::pair<int32_t, int32_t>> a((size_t)n);
  std::vector<g2n::KV<int32_t, int32_t>> b((size_t)n);
  for (int64_t i = 0; i < n; i++) {
    a[i] = {keys[i], (int32_t)i};
    b[i] = {keys[i], (int32_t)i};
  }
  std::sort(a.begin(), a.end(), [](const std::pair<int32_t, int32_t>& x, const std::pair<int32_t, int32_t>& y) {
    return x.first < y.first;
  });
  if (n) g2n::stl_sort(b.data(), b.data() + n);
  for (int64_t i = 0; i < n; i++) {
    out_std[i] = a[i].second;
    out_emul[i] = b[i].v;
  }
}
}
