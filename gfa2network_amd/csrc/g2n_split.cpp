// g2n_split.cpp — parse_gfa(..., split_on_alignment=True) (gfa2network/builders.py:110-128 →
// _parse_gfa_split, builders.py:302-568), matrix outputs.
//
// The reference parses every record first, cuts each segment at the alignment coordinates its
// GFA2 E / GFA1 C records name, and then feeds a NEW record stream through the matrix loop:
// the interval segments ("<id>:<a>-<b>") with a "+/+" link between consecutive intervals,
// every E/C record re-targeted to the interval its coordinates name, every L record to the
// interval spanning its segment.  This file computes that mapping (host work proportional to
// the records; the dictionary is the segment set, not the touches) and RENDERS the new stream
// as GFA text that the GPU build parses with the reference's main-path semantics
// (g2n_build_from_buffer): "S\t<interval>" for the interval segments and
// "E\t*\t<u>\t<ori>\t<v>\t<ori>[\t<original tag fields>]" for every link / edge (an interval
// name holds ':' so the E line always takes parser.py:289-295's orientation-only form, whose
// tags are fields[6:] — the same tag dict the reference's record carried).
//
// Bidirected builds mint the plain interval keys for the Segment records (builders.py:474-476,
// not "<id>:+"/"<id>:-" as the main path's S lines do); those keys are never touched by an edge
// ("<interval>:<ori>" keys are), so the caller renders the edges alone and inserts each
// segment's interval nodes ahead of the oriented keys its chain links mint (a monotonic id map).
//
// The input must already have parsed cleanly (the caller runs the GPU build on it first: every
// parser error, warning and gzip failure is the reference's); this pass only needs the fields.
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "g2n_internal.h"

namespace g2n {
namespace {

using SV = std::string_view;

// int() of a bytes field (CPython 3.10 _PyLong_FromBytes, base 10): ASCII whitespace around,
// one sign, digits with single '_' between digits, <= 4300 digits (sys.int_info's default
// str-digits limit).  0 = int (in *v), 1 = ValueError, 2 = an int beyond int64 (unsupported).
int py_int_bytes(SV s, int64_t* v) {
  auto sp = [](unsigned char c) { return c == ' ' || (c >= 9 && c <= 13); };
  size_t i = 0, n = s.size();
  while (i < n && sp((unsigned char)s[i])) i++;
  while (n > i && sp((unsigned char)s[n - 1])) n--;
  bool neg = false;
  if (i < n && (s[i] == '+' || s[i] == '-')) neg = s[i++] == '-';
  if (i >= n) return 1;
  unsigned __int128 acc = 0;
  size_t digits = 0;
  bool prev_digit = false, big = false;
  for (; i < n; i++) {
    const unsigned char c = (unsigned char)s[i];
    if (c == '_') {
      if (!prev_digit || i + 1 >= n || s[i + 1] < '0' || s[i + 1] > '9') return 1;
      prev_digit = false;
      continue;
    }
    if (c < '0' || c > '9') return 1;
    prev_digit = true;
    digits++;
    if (!big) {
      acc = acc * 10 + (c - '0');
      if (acc > ((unsigned __int128)1 << 63)) big = true;
    }
  }
  if (digits > 4300) return 1;
  if (big || (!neg && acc > (unsigned __int128)INT64_MAX)) return 2;
  *v = neg ? (int64_t)(0 - (uint64_t)acc) : (int64_t)acc;
  return 0;
}

struct Fields {
  std::vector<SV> f;
  void split(SV line) {
    f.clear();
    size_t a = 0;
    for (;;) {
      const size_t t = line.find('\t', a);
      if (t == SV::npos) {
        f.push_back(line.substr(a));
        return;
      }
      f.push_back(line.substr(a, t - a));
      a = t + 1;
    }
  }
  // the bytes of fields[k:] joined by tabs (the original tag fields), empty view if none
  SV tail(SV line, size_t k) const {
    if (k >= f.size()) return SV();
    return SV(f[k].data(), (size_t)(line.data() + line.size() - f[k].data()));
  }
};

SV rstrip_pm(SV s) {
  while (!s.empty() && (s.back() == '+' || s.back() == '-')) s.remove_suffix(1);
  return s;
}

struct Edge {  // E / C record (parser.py:42-71) or L record (parser.py:21-30)
  SV u, v, ou, ov;
  bool coords = false;
  int64_t us = 0, ue = 0, vs = 0, ve = 0;
  bool has_tags = false;
  SV tags;
};

struct Seg {
  SV id;
  bool has_len = false;
  int64_t len = 0;
  std::vector<int64_t> bps;     // breakpoints; then the interval bounds (sorted, distinct, + the single-point rule)
  size_t first_interval = 0;    // index into the interval names
  size_t n_intervals = 0;
  size_t full = 0;              // interval index of full_segment
};

std::string interval_name(SV id, int64_t a, int64_t b) {
  std::string s(id);
  s += ':';
  s += std::to_string(a);
  s += '-';
  s += std::to_string(b);
  return s;
}

}  // namespace
}  // namespace g2n

struct g2n_split_out {
  std::string text;
  std::string names;
  std::vector<int64_t> name_offs;
  std::string warn_segs;           // missing segment names, concatenated
  std::vector<int64_t> warn_offs;
  std::vector<int32_t> warn_kind;  // 0 edge (builders.py:389-393), 1 link (builders.py:415-419)
  int32_t many_nodes = 0;          // builders.py:379-380
  std::vector<int64_t> seg_intervals;  // intervals per segment, in the segments dict's order
};

extern "C" {

int g2n_split_render(const void* buf, size_t len, int32_t bidirected, g2n_split_out** out) {
  using namespace g2n;
  if (!out || (len && !buf)) return G2N_E_ARG;
  *out = nullptr;
  return guarded([&]() -> int {
    auto* o = new g2n_split_out();
    std::unique_ptr<g2n_split_out> hold(o);
    const char* b = (const char*)buf;
    std::unordered_map<SV, size_t> seg_of;                  // segments dict (insertion order)
    std::vector<Seg> segs;
    std::unordered_map<SV, std::vector<int64_t>> bp_other;  // breakpoints of names without an S yet
    std::vector<Edge> edges, links;
    Fields F;
    auto add_bp = [&](SV name, int64_t x) {
      auto it = seg_of.find(name);
      if (it != seg_of.end()) segs[it->second].bps.push_back(x);
      else bp_other[name].push_back(x);
    };
    for (size_t p = 0; p < len;) {
      const char* nl = (const char*)memchr(b + p, '\n', len - p);
      const size_t e = nl ? (size_t)(nl - b) : len;
      const SV line(b + p, e - p);
      p = e + 1;
      if (line.empty()) continue;
      const char k = line[0];
      if (k != 'S' && k != 'L' && k != 'E' && k != 'C') continue;  // P / O: checked by the GPU parse
      F.split(line);
      const auto& f = F.f;
      if (f[0].size() != 1) continue;  // rec_type must be exactly b"S" etc. (parser.py:134-173)
      if (k == 'S') {  // parser.py:135-163: length = int(fields[2]) when it parses
        if (f.size() < 2) return G2N_E_ARG;  // IndexError: the GPU parse raised it first
        bool has_len = false;
        int64_t L = 0;
        if (f.size() > 2) {
          const int r = py_int_bytes(f[2], &L);
          if (r == 2) throw Failure(G2N_E_UNSUPPORTED, "split_on_alignment: a segment length beyond int64");
          has_len = r == 0;
        }
        auto it = seg_of.find(f[1]);
        size_t si;
        if (it == seg_of.end()) {
          si = segs.size();
          seg_of.emplace(f[1], si);
          segs.emplace_back();
          segs[si].id = f[1];
          auto ob = bp_other.find(f[1]);
          if (ob != bp_other.end()) {
            segs[si].bps = std::move(ob->second);
            bp_other.erase(ob);
          }
        } else {
          si = it->second;
        }
        Seg& s = segs[si];
        s.has_len = has_len;  // segments[rec.id] = rec: the last record's length
        s.len = L;
        if (has_len) {
          s.bps.push_back(0);
          s.bps.push_back(L);
        }
        continue;
      }
      Edge r;
      if (k == 'L') {  // parser.py:206-227
        if (f.size() < 5) return G2N_E_ARG;
        if (f[2] == "+" || f[2] == "-") {
          r.u = f[1], r.ou = f[2], r.v = f[3], r.ov = f[4];
          r.has_tags = f.size() > 6;
          r.tags = F.tail(line, 6);
        } else {
          static const char plus = '+';
          if (f[1].empty() || f[2].empty()) return G2N_E_ARG;
          r.ou = (f[1].back() == '+' || f[1].back() == '-') ? SV(&f[1].back(), 1) : SV(&plus, 1);
          r.ov = (f[2].back() == '+' || f[2].back() == '-') ? SV(&f[2].back(), 1) : SV(&plus, 1);
          r.u = rstrip_pm(f[1]), r.v = rstrip_pm(f[2]);
          r.has_tags = f.size() > 4;
          r.tags = F.tail(line, 4);
        }
        links.push_back(r);
        continue;
      }
      const size_t min_fields = k == 'E' ? 6 : 5;
      if (f.size() < min_fields) return G2N_E_ARG;
      bool gfa2 = false;
      if (f.size() >= 9) {
        int rc[4];
        int64_t c[4];
        const size_t idx[4] = {3, 4, 6, 7};
        gfa2 = true;
        for (int q = 0; q < 4; q++) {
          rc[q] = py_int_bytes(f[idx[q]], &c[q]);
          if (rc[q] == 1) gfa2 = false;
        }
        if (gfa2) {
          for (int q = 0; q < 4; q++)
            if (rc[q] == 2) throw Failure(G2N_E_UNSUPPORTED, "split_on_alignment: a coordinate beyond int64");
          static const char plus = '+', minus = '-';
          r.ou = SV(!f[2].empty() && f[2].back() == '-' ? &minus : &plus, 1);
          r.ov = SV(!f[5].empty() && f[5].back() == '-' ? &minus : &plus, 1);
          r.u = rstrip_pm(f[2]), r.v = rstrip_pm(f[5]);
          r.coords = true;
          r.us = c[0], r.ue = c[1], r.vs = c[2], r.ve = c[3];
          r.has_tags = f.size() > 9;
          r.tags = F.tail(line, 9);
        }
      }
      if (!gfa2) {
        const size_t o0 = k == 'E' ? 2 : 1;  // E: fields[2..5]; C: fields[1..4]
        r.u = f[o0], r.ou = f[o0 + 1], r.v = f[o0 + 2], r.ov = f[o0 + 3];
        r.has_tags = f.size() > o0 + 4;
        r.tags = F.tail(line, o0 + 4);
      } else {  // builders.py:337-344: the four coordinates are breakpoints
        add_bp(r.u, r.us);
        add_bp(r.u, r.ue);
        add_bp(r.v, r.vs);
        add_bp(r.v, r.ve);
      }
      edges.push_back(r);
    }

    // builders.py:352-377: intervals per segment, in the segments dict's order
    std::string& T = o->text;
    auto put_seg_line = [&](SV nid) {
      if (bidirected) return;
      T += "S\t";
      T.append(nid.data(), nid.size());
      T += '\n';
    };
    auto put_edge_line = [&](SV u, SV ou, SV v, SV ov, bool has_tags, SV tags) {
      T += "E\t*\t";
      T.append(u.data(), u.size());
      T += '\t';
      T.append(ou.data(), ou.size());
      T += '\t';
      T.append(v.data(), v.size());
      T += '\t';
      T.append(ov.data(), ov.size());
      if (has_tags) {
        T += '\t';
        T.append(tags.data(), tags.size());
      }
      T += '\n';
    };
    std::vector<int64_t> name_off = {0};
    std::string& names = o->names;
    auto name = [&](size_t i) { return SV(names.data() + name_off[i], (size_t)(name_off[i + 1] - name_off[i])); };
    size_t n_mapping = 0;
    for (Seg& s : segs) {
      std::sort(s.bps.begin(), s.bps.end());
      s.bps.erase(std::unique(s.bps.begin(), s.bps.end()), s.bps.end());
      std::vector<int64_t>& bp = s.bps;  // sorted(breakpoints.get(seg_id, {0}))
      if (bp.empty()) bp.push_back(0);
      if (bp.size() == 1) bp.push_back(s.has_len ? s.len : bp[0]);
      s.first_interval = name_off.size() - 1;
      s.n_intervals = bp.size() - 1;
      o->seg_intervals.push_back((int64_t)s.n_intervals);
      bool found_full = false;
      for (size_t q = 0; q + 1 < bp.size(); q++) {
        names += interval_name(s.id, bp[q], bp[q + 1]);
        name_off.push_back((int64_t)names.size());
        if (!found_full && s.has_len && bp[q] == 0 && bp[q + 1] == s.len) {
          found_full = true;
          s.full = s.first_interval + q;
        }
      }
      if (!found_full) s.full = s.first_interval;
      // len(mapping): the interval keys, (seg, None, None), and (seg, 0, length) when new
      n_mapping += s.n_intervals + 1;
      if (s.has_len) {
        bool is_key = false;
        for (size_t q = 0; q + 1 < bp.size(); q++) is_key |= bp[q] == 0 && bp[q + 1] == s.len;
        if (!is_key) n_mapping++;
      }
      for (size_t q = 0; q < s.n_intervals; q++) put_seg_line(name(s.first_interval + q));
      for (size_t q = 0; q + 1 < s.n_intervals; q++) {
        static const char plus = '+';
        put_edge_line(name(s.first_interval + q), SV(&plus, 1), name(s.first_interval + q + 1), SV(&plus, 1),
                      false, SV());
      }
    }
    o->many_nodes = n_mapping > 10 * segs.size();

    // builders.py:382-408: E / C records to the interval their coordinates name
    auto lookup = [&](SV seg, bool coords, int64_t a, int64_t c, size_t* out_name) -> bool {
      auto it = seg_of.find(seg);
      if (it == seg_of.end()) return false;
      const Seg& s = segs[it->second];
      if (!coords || (s.has_len && a == 0 && c == s.len)) {
        *out_name = s.full;
        return true;
      }
      const std::vector<int64_t>& bp = s.bps;  // consecutive bounds (a, c)?
      auto q = std::lower_bound(bp.begin(), bp.end() - 1, a) - bp.begin();
      if (bp.size() == 2 && bp[1] < bp[0]) q = 0;  // the single-point rule may leave [x, len] unsorted
      if ((size_t)q + 1 < bp.size() && bp[q] == a && bp[q + 1] == c) {
        *out_name = s.first_interval + q;
        return true;
      }
      return false;
    };
    auto warn = [&](int kind, SV seg) {
      o->warn_kind.push_back(kind);
      o->warn_segs.append(seg.data(), seg.size());
      o->warn_offs.push_back((int64_t)o->warn_segs.size());
    };
    o->warn_offs.push_back(0);
    for (const Edge& r : edges) {
      size_t iu, iv;
      const bool hu = lookup(r.u, r.coords, r.us, r.ue, &iu);
      const bool hv = hu && lookup(r.v, r.coords, r.vs, r.ve, &iv);
      if (!hu || !hv) {
        warn(0, hu ? r.v : r.u);
        continue;
      }
      put_edge_line(name(iu), r.ou, name(iv), r.ov, r.has_tags, r.tags);
    }
    // builders.py:410-430: L records to the interval spanning the segment
    for (const Edge& r : links) {
      auto a = seg_of.find(r.u);
      auto c = seg_of.find(r.v);
      if (a == seg_of.end() || c == seg_of.end()) {
        warn(1, a == seg_of.end() ? r.u : r.v);
        continue;
      }
      put_edge_line(name(segs[a->second].full), r.ou, name(segs[c->second].full), r.ov, r.has_tags, r.tags);
    }
    o->name_offs = std::move(name_off);
    *out = hold.release();
    return G2N_OK;
  });
}

void g2n_split_get(const g2n_split_out* o, const uint8_t** text, uint64_t* text_len, const uint8_t** names,
                   const int64_t** name_offs, uint64_t* n_names, const uint8_t** warn_segs,
                   const int64_t** warn_offs, const int32_t** warn_kind, uint64_t* n_warn, int32_t* many_nodes) {
  *text = (const uint8_t*)o->text.data();
  *text_len = o->text.size();
  *names = (const uint8_t*)o->names.data();
  *name_offs = o->name_offs.data();
  *n_names = o->name_offs.size() - 1;
  *warn_segs = (const uint8_t*)o->warn_segs.data();
  *warn_offs = o->warn_offs.data();
  *warn_kind = o->warn_kind.data();
  *n_warn = o->warn_kind.size();
  *many_nodes = o->many_nodes;
}

void g2n_split_segments(const g2n_split_out* o, const int64_t** intervals, uint64_t* n_segments) {
  *intervals = o->seg_intervals.data();
  *n_segments = o->seg_intervals.size();
}

void g2n_split_free(g2n_split_out* o) { delete o; }

}  // extern "C"
