/*
 * g2n_synth.h — benchmark-input support exported by libg2n.so (not part of the
 * reference's interface).  Generates the deterministic synthetic GFA of SURVEY.md §8(d)
 * (gfa2network_amd/csrc/synth.h) on the host (files for CPU baselines) or straight into
 * HBM (bench.py's device-resident workload).  Host and device bytes are identical.
 */
#ifndef G2N_SYNTH_H
#define G2N_SYNTH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct g2n_synth_spec {
  uint64_t n_segments; /* S lines, named 1..n_segments (names = 0) */
  uint64_t n_links;    /* L lines */
  uint64_t seed;
  int32_t rc_tag;      /* append RC:i:k to every L line */
  int32_t names;       /* 0: segment i is "i"; 1: "s" + 8 hex digits of a bijection of i
                          (unique, not decimal: the hash-dictionary / general sharded paths);
                          2: the decimal of a permutation of 1..n_segments (decimal names out of
                          order: the direct-address dictionary tier); 3: "s" + the decimal of i
                          (minigraph's s1..sN: prefixed names in S order) */
  int32_t far_links;   /* 1: an L line's second segment is uniform over all segments (no id
                          locality: every edge's two rows fall in different CSR buckets) */
} g2n_synth_spec;

/* host: malloc'd buffer of the whole file (free with g2n_synth_free_host) */
int g2n_synth_host(const g2n_synth_spec *spec, int n_threads, uint8_t **out, size_t *len);
void g2n_synth_free_host(uint8_t *buf);

/* device: hipMalloc'd buffer on `device` (free with g2n_synth_free_device) */
int g2n_synth_device(int device, const g2n_synth_spec *spec, void **d_out, size_t *len);
void g2n_synth_free_device(void *d_buf);

/* copy device bytes back (for checks) */
int g2n_synth_download(void *host_dst, const void *d_src, size_t len);

#ifdef __cplusplus
}
#endif
#endif /* G2N_SYNTH_H */
