// Host-side code of libg2n (gzip ingest, the convert CLI's writers) under AddressSanitizer and
// UndefinedBehaviorSanitizer: built with g++ from gfa2network_amd/csrc/g2n_ingest.cpp and
// g2n_writers.cpp plus this driver by tests/test_sanitizers.py (CPU only; the GPU paths of those
// files are linked but never called).  Exercises the parallel and serial gzip readers on clean
// member chains, truncations, corruptions and trailing garbage (checking the prefix contract of
// gunzip_exact), the .npz / .nodes.tsv writers and the UTF-8 scan.  Prints "OK" and exits 0.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include <zlib.h>

#include <functional>
#include <random>
#include <string>
#include <vector>

#include "../../gfa2network_amd/csrc/g2n_internal.h"

namespace g2n {
static thread_local std::string t_err;
void set_last_error(const std::string& msg) { t_err = msg; }  // g2n_host.cpp's, not linked here
int guarded(const std::function<int()>& f) {  // g2n_host.cpp's, not linked here
  try {
    return f();
  } catch (const Failure& e) {
    set_last_error(e.what());
    return e.status;
  }
}
}  // namespace g2n

static int failures = 0;
#define CHECK(c)                                                     \
  do {                                                               \
    if (!(c)) {                                                      \
      fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);   \
      failures++;                                                    \
    }                                                                \
  } while (0)

static std::vector<uint8_t> member(const std::vector<uint8_t>& d, int level) {
  z_stream zs;
  memset(&zs, 0, sizeof(zs));
  deflateInit2(&zs, level, Z_DEFLATED, -MAX_WBITS, 8, Z_DEFAULT_STRATEGY);
  std::vector<uint8_t> out = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, 0, 0xff};
  std::vector<uint8_t> buf(deflateBound(&zs, d.size()) + 16);
  zs.next_in = const_cast<Bytef*>(d.data());
  zs.avail_in = (uInt)d.size();
  zs.next_out = buf.data();
  zs.avail_out = (uInt)buf.size();
  deflate(&zs, Z_FINISH);
  out.insert(out.end(), buf.data(), buf.data() + zs.total_out);
  deflateEnd(&zs);
  const uint32_t crc = (uint32_t)crc32(0, d.data(), (uInt)d.size()), n = (uint32_t)d.size();
  for (int k = 0; k < 4; k++) out.push_back((uint8_t)(crc >> (8 * k)));
  for (int k = 0; k < 4; k++) out.push_back((uint8_t)(n >> (8 * k)));
  return out;
}

static std::vector<uint8_t> flat(const g2n::Inflated& z) {
  std::vector<uint8_t> v(z.total);
  for (size_t k = 0; k < z.parts.size(); k++)
    if (z.parts[k].n) memcpy(v.data() + z.start[k], z.parts[k].p, z.parts[k].n);
  return v;
}

static void gzip_checks() {
  std::mt19937_64 rng(7);
  std::string t;
  for (int i = 1; i <= 60000; i++) t += "S\t" + std::to_string(i) + "\tACGT\n";
  for (int i = 0; i < 120000; i++)
    t += "L\t" + std::to_string(1 + rng() % 60000) + "\t+\t" + std::to_string(1 + rng() % 60000) + "\t-\t0M\n";
  const std::vector<uint8_t> text(t.begin(), t.end());
  std::vector<uint8_t> blob;
  std::vector<size_t> cuts = {0};
  while (cuts.back() < text.size()) cuts.push_back(std::min(text.size(), cuts.back() + 1 + rng() % 400000));
  for (size_t k = 0; k + 1 < cuts.size(); k++) {
    auto m = member(std::vector<uint8_t>(text.begin() + cuts[k], text.begin() + cuts[k + 1]), (int)(rng() % 10));
    blob.insert(blob.end(), m.begin(), m.end());
    for (uint64_t p = rng() % 3; p; p--) blob.push_back(0);  // padding
  }
  {  // clean chains, both readers
    g2n::Inflated a, b;
    int sub = 0;
    std::string msg;
    CHECK(g2n::gunzip_parallel(blob.data(), blob.size(), a));
    CHECK(flat(a) == text);
    CHECK(g2n::gunzip_exact(blob.data(), blob.size(), b, &sub, &msg));
    CHECK(flat(b) == text);
  }
  {  // one member over the whole text: the chunk-parallel inflate, clean and damaged
    auto one = member(text, 6);
    g2n::Inflated a;
    CHECK(g2n::gunzip_chunked(one.data(), one.size(), 1 << 14, a));
    CHECK(flat(a) == text && a.parts.size() > 1);
    for (int trial = 0; trial < 40; trial++) {
      std::vector<uint8_t> bad = one;
      const size_t at = 10 + rng() % (bad.size() - 10);
      if (trial % 2) bad.resize(at);
      else bad[at] ^= (uint8_t)(1u << (rng() % 8));
      g2n::Inflated c, d;
      int sub = 0;
      std::string msg;
      const bool ok_ch = g2n::gunzip_chunked(bad.data(), bad.size(), 1 << 13, c);
      const bool ok = g2n::gunzip_exact(bad.data(), bad.size(), d, &sub, &msg);
      if (ok_ch) CHECK(ok && flat(c) == flat(d));
    }
  }
  for (int trial = 0; trial < 60; trial++) {  // damaged: no crash; the prefix is a prefix
    std::vector<uint8_t> bad = blob;
    const size_t at = rng() % bad.size();
    switch (trial % 4) {
      case 0: bad.resize(at); break;
      case 1:
        for (size_t k = at; k < std::min(bad.size(), at + 1 + rng() % 64); k++) bad[k] = (uint8_t)rng();
        break;
      case 2: bad[at] ^= (uint8_t)(1u << (rng() % 8)); break;
      default: bad.insert(bad.end(), {'x', 'y', 0x1f}); break;
    }
    g2n::Inflated a, b;
    int sub = 0;
    std::string msg;
    const bool ok_par = g2n::gunzip_parallel(bad.data(), bad.size(), a);
    const bool ok = g2n::gunzip_exact(bad.data(), bad.size(), b, &sub, &msg);
    if (ok_par) CHECK(ok && flat(a) == flat(b));
    const auto got = flat(b);
    CHECK(got.size() <= text.size() || trial % 4 == 1 || trial % 4 == 2);
    if (!ok) {
      CHECK(sub >= 1 && sub <= 4 && !msg.empty());
      if (trial % 4 == 0) CHECK(memcmp(got.data(), text.data(), got.size()) == 0);  // truncation
    }
  }
}

static void writer_checks() {
  char dir[] = "/tmp/g2nsanXXXXXX";
  CHECK(mkdtemp(dir) != nullptr);
  const std::string npz = std::string(dir) + "/m.npz", tsv = std::string(dir) + "/m.nodes.tsv";
  std::vector<int32_t> a(300000);
  std::vector<double> d(a.size());
  for (size_t i = 0; i < a.size(); i++) {
    a[i] = (int32_t)(i * 7);
    d[i] = (double)i * 0.5;
  }
  const char* names[] = {"indices.npy", "data.npy", "empty.npy"};
  const std::string h0 = "\x93NUMPY\x01\x00v\x00{'descr': '<i4', 'fortran_order': False, 'shape': (300000,), }";
  const std::string h1 = "\x93NUMPY\x01\x00v\x00{'descr': '<f8', 'fortran_order': False, 'shape': (300000,), }";
  const std::string h2 = "\x93NUMPY\x01\x00v\x00{'descr': '<f8', 'fortran_order': False, 'shape': (0,), }";
  const uint8_t* heads[] = {(const uint8_t*)h0.data(), (const uint8_t*)h1.data(), (const uint8_t*)h2.data()};
  const uint64_t hl[] = {h0.size(), h1.size(), h2.size()};
  const void* datas[] = {a.data(), d.data(), nullptr};
  const uint64_t dl[] = {a.size() * 4, d.size() * 8, 0};
  for (int level : {0, 1, 6}) CHECK(g2n::write_npz(npz, 3, names, heads, hl, datas, dl, level) == 0);
  std::string blob;
  std::vector<int64_t> offs = {0};
  for (int i = 0; i < 200000; i++) {
    blob += "node_" + std::to_string(i) + (i % 1000 == 0 ? "\xc3\xa9" : "");
    offs.push_back((int64_t)blob.size());
  }
  CHECK(g2n::first_bad_utf8((const uint8_t*)blob.data(), offs.data(), offs.size() - 1) == -1);
  CHECK(g2n::write_node_map(tsv, (const uint8_t*)blob.data(), offs.data(), offs.size() - 1) == 0);
  blob[offs[12345] + 2] = (char)0xff;
  CHECK(g2n::first_bad_utf8((const uint8_t*)blob.data(), offs.data(), offs.size() - 1) == 12345);
  CHECK(g2n::first_bad_utf8((const uint8_t*)blob.data(), offs.data(), 0) == -1);
  unlink(npz.c_str());
  unlink(tsv.c_str());
  rmdir(dir);
}

// g2n_split_render (split_on_alignment's record mapping) on random GFA2 / GFA1 records:
// coordinates in and out of range, missing segments, duplicate S, fallbacks, ragged lines.
static void split_checks() {
  std::mt19937_64 rng(11);
  for (int trial = 0; trial < 200; trial++) {
    std::string t;
    const int ns = 1 + (int)(rng() % 6);
    auto seg = [&] { return std::string(1, (char)('a' + rng() % (ns + 2))); };
    for (int i = 0; i < 40; i++) {
      switch (rng() % 6) {
        case 0: t += "S\t" + seg() + "\t" + std::to_string((int)(rng() % 12) - 2) + "\t*\n"; break;
        case 1: t += "S\t" + seg() + (rng() % 2 ? "\t*" : "") + "\n"; break;
        case 2:
          t += "E\te\t" + seg() + "+\t" + std::to_string(rng() % 9) + "\t" + std::to_string(rng() % 12) + "\t" + seg() +
               "-\t" + std::to_string((int)(rng() % 9) - 1) + "\t" + std::to_string(rng() % 12) + "\t*" +
               (rng() % 2 ? "\tRC:i:3" : "") + "\n";
          break;
        case 3: t += "C\t" + seg() + "\t+\t" + seg() + "\t-\t" + std::to_string(rng() % 5) + "\t*\n"; break;
        case 4: t += "L\t" + seg() + "\t+\t" + seg() + "\t-\t0M\n"; break;
        default: t += "L\t" + seg() + "+\t" + seg() + "\t*\r\n"; break;
      }
    }
    if (rng() % 3 == 0) t.resize(rng() % (t.size() + 1));  // ragged last line
    for (int bidir = 0; bidir < 2; bidir++) {
      g2n_split_out* o = nullptr;
      const int rc = g2n_split_render(t.data(), t.size(), bidir, &o);
      if (rc != G2N_OK) {
        CHECK(o == nullptr);  // a short record the GPU parse would have rejected first
        continue;
      }
      const uint8_t *text, *names, *ws;
      const int64_t *no, *wo, *per;
      const int32_t* wk;
      uint64_t tl, nn, nw, nsg;
      int32_t many;
      g2n_split_get(o, &text, &tl, &names, &no, &nn, &ws, &wo, &wk, &nw, &many);
      g2n_split_segments(o, &per, &nsg);
      int64_t sum = 0;
      for (uint64_t k = 0; k < nsg; k++) sum += per[k];
      CHECK((uint64_t)sum == nn && no[0] == 0);
      CHECK(tl == 0 || text[tl - 1] == '\n');
      g2n_split_free(o);
    }
  }
}

int main() {
  split_checks();
  gzip_checks();
  writer_checks();
  if (failures) return 1;
  printf("OK\n");
  return 0;
}
