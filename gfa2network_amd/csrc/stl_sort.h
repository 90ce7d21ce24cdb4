// stl_sort.h — restatement of libstdc++'s std::sort (introsort) for a range of
// (key, value) pairs compared by key only, usable in device code.
//
// Why: scipy's csr_sort_indices (scipy/sparse/sparsetools/csr.h, reached from
// convert_format / A.maximum via coo.tocsr -> csr.sum_duplicates) sorts each row's
// (col, val) pairs with std::sort and a first-only comparator.  std::sort is not
// stable, so for float dtypes the order in which csr_sum_duplicates then adds
// duplicates depends on libstdc++'s exact permutation.  Rows that need it are
// re-sorted on the GPU with this restatement so sums match scipy bit for bit.
//
// Third-party algorithm restated (not copied): GNU libstdc++ (GCC 11) bits/stl_algo.h
// __sort / __introsort_loop (_S_threshold = 16, depth limit 2*floor(log2 n)),
// __unguarded_partition_pivot / __move_median_to_first / __unguarded_partition,
// __final_insertion_sort / __insertion_sort / __unguarded_linear_insert, and
// bits/stl_heap.h __make_heap / __adjust_heap / __push_heap / __pop_heap /
// __sort_heap (the __partial_sort fallback).  Checked against the real std::sort in
// tests/test_host_headers.py (tests/native/hostcheck.cpp).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define G2N_HD __host__ __device__
#else
#define G2N_HD
#endif

namespace g2n {

template <class K, class V>
struct KV {
  K k;
  V v;
};

template <class K, class V>
G2N_HD inline void kv_swap(KV<K, V>* a, KV<K, V>* b) {
  KV<K, V> t = *a;
  *a = *b;
  *b = t;
}

template <class K, class V>
G2N_HD inline void stl_move_median_to_first(KV<K, V>* result, KV<K, V>* a, KV<K, V>* b, KV<K, V>* c) {
  if (a->k < b->k) {
    if (b->k < c->k) kv_swap(result, b);
    else if (a->k < c->k) kv_swap(result, c);
    else kv_swap(result, a);
  } else if (a->k < c->k) {
    kv_swap(result, a);
  } else if (b->k < c->k) {
    kv_swap(result, c);
  } else {
    kv_swap(result, b);
  }
}

template <class K, class V>
G2N_HD inline KV<K, V>* stl_unguarded_partition(KV<K, V>* first, KV<K, V>* last, KV<K, V>* pivot) {
  while (true) {
    while (first->k < pivot->k) ++first;
    --last;
    while (pivot->k < last->k) --last;
    if (!(first < last)) return first;
    kv_swap(first, last);
    ++first;
  }
}

template <class K, class V>
G2N_HD inline void stl_push_heap(KV<K, V>* first, int64_t hole, int64_t top, KV<K, V> value) {
  int64_t parent = (hole - 1) / 2;
  while (hole > top && first[parent].k < value.k) {
    first[hole] = first[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  first[hole] = value;
}

template <class K, class V>
G2N_HD inline void stl_adjust_heap(KV<K, V>* first, int64_t hole, int64_t len, KV<K, V> value) {
  const int64_t top = hole;
  int64_t child = hole;
  while (child < (len - 1) / 2) {
    child = 2 * (child + 1);
    if (first[child].k < first[child - 1].k) child--;
    first[hole] = first[child];
    hole = child;
  }
  if ((len & 1) == 0 && child == (len - 2) / 2) {
    child = 2 * (child + 1);
    first[hole] = first[child - 1];
    hole = child - 1;
  }
  stl_push_heap(first, hole, top, value);
}

template <class K, class V>
G2N_HD inline void stl_make_heap(KV<K, V>* first, KV<K, V>* last) {
  int64_t len = last - first;
  if (len < 2) return;
  int64_t parent = (len - 2) / 2;
  while (true) {
    KV<K, V> value = first[parent];
    stl_adjust_heap(first, parent, len, value);
    if (parent == 0) return;
    parent--;
  }
}

template <class K, class V>
G2N_HD inline void stl_pop_heap(KV<K, V>* first, KV<K, V>* last, KV<K, V>* result) {
  KV<K, V> value = *result;
  *result = *first;
  stl_adjust_heap(first, (int64_t)0, (int64_t)(last - first), value);
}

template <class K, class V>
G2N_HD inline void stl_partial_sort_all(KV<K, V>* first, KV<K, V>* last) {
  // __partial_sort(first, last, last): __heap_select (= make_heap, no tail) + __sort_heap
  stl_make_heap(first, last);
  while (last - first > 1) {
    --last;
    stl_pop_heap(first, last, last);
  }
}

template <class K, class V>
G2N_HD inline void stl_unguarded_linear_insert(KV<K, V>* last) {
  KV<K, V> val = *last;
  KV<K, V>* next = last - 1;
  while (val.k < next->k) {
    *last = *next;
    last = next;
    --next;
  }
  *last = val;
}

template <class K, class V>
G2N_HD inline void stl_insertion_sort(KV<K, V>* first, KV<K, V>* last) {
  if (first == last) return;
  for (KV<K, V>* i = first + 1; i != last; ++i) {
    if (i->k < first->k) {
      KV<K, V> val = *i;
      for (KV<K, V>* p = i; p != first; --p) *p = *(p - 1);  // move_backward
      *first = val;
    } else {
      stl_unguarded_linear_insert(i);
    }
  }
}

G2N_HD inline int stl_lg(int64_t n) {
  int r = -1;
  while (n) { n >>= 1; r++; }
  return r;
}

// __introsort_loop, written with an explicit stack in place of the recursion on the
// right part (depth-first, right part first: same visiting order as the recursion).
template <class K, class V>
G2N_HD inline void stl_introsort_loop(KV<K, V>* first, KV<K, V>* last, int depth_limit) {
  struct Frame { KV<K, V>* first; KV<K, V>* last; int depth; };
  Frame stack[128];
  int sp = 0;
  stack[sp++] = Frame{first, last, depth_limit};
  while (sp > 0) {
    Frame fr = stack[--sp];
    KV<K, V>* f = fr.first;
    KV<K, V>* l = fr.last;
    int depth = fr.depth;
    // The recursive original:  while (l - f > 16) { if (!depth) {partial_sort; return;}
    //   --depth; cut = partition; introsort_loop(cut, l, depth); l = cut; }
    // The recursive call on [cut, l) completes before the loop continues on [f, cut);
    // we push the continuation [f, cut) first and the call [cut, l) on top.
    if (l - f <= 16) continue;
    if (depth == 0) {
      stl_partial_sort_all(f, l);
      continue;
    }
    --depth;
    KV<K, V>* mid = f + (l - f) / 2;
    stl_move_median_to_first(f, f + 1, mid, l - 1);
    KV<K, V>* cut = stl_unguarded_partition(f + 1, l, f);
    stack[sp++] = Frame{f, cut, depth};
    stack[sp++] = Frame{cut, l, depth};
  }
}

template <class K, class V>
G2N_HD inline void stl_sort(KV<K, V>* first, KV<K, V>* last) {
  if (first == last) return;
  stl_introsort_loop(first, last, stl_lg(last - first) * 2);
  // __final_insertion_sort
  if (last - first > 16) {
    stl_insertion_sort(first, first + 16);
    for (KV<K, V>* i = first + 16; i != last; ++i) stl_unguarded_linear_insert(i);
  } else {
    stl_insertion_sort(first, last);
  }
}

}  // namespace g2n
