/*
 * g2n.h — C-ABI of the MI355X-native GFA -> CSR ingest path (libg2n.so).
 *
 * Drop-in boundary for the hot path of sclipman/gfa2network (reference @ 2025-07-04).
 * The reference is pure Python and has no FFI of its own; these entry
 * points are what its Python call surface binds through ctypes (INTEGRATION.md shows the
 * stub a maintainer adds).  Plain pointers and sizes only: no torch / numpy types.
 *
 *   g2n_build_from_path    replaces GFAParser(path) iteration + the build_matrix=True
 *                          branch of parse_gfa      gfa2network/parser.py:95-176,
 *                                                    gfa2network/builders.py:129-299
 *   g2n_build_from_buffer  same, for an in-memory / already-read file object
 *                          (GFAParser(BinaryIO) parser.py:90-92, stdin parser.py:104-105)
 *   g2n_build_device       same, input already resident in HBM (the measured hot path)
 *   g2n_coo_to_csr         replaces convert_format(A, "csr") = A.asformat("csr")
 *                          for a COO matrix   gfa2network/utils.py:40-63 (scipy coo.tocsr)
 *
 * Output selection (g2n_options.output):
 *   G2N_OUT_PARSE  exactly what parse_gfa(..., build_matrix=True) returns: the MAX-SYM
 *                  CSR when graph_directed and not asymmetric (builders.py:282-283),
 *                  otherwise the stream-order, unsummed COO (builders.py:281).
 *   G2N_OUT_CSR    what convert_format(parse_gfa(...), "csr") returns (cli.py:239).
 *   G2N_OUT_EDGE_LIST  the bytes `gfa2network export --format edge-list [--bidirected]`
 *                  writes (cli.py:264-281): "u\tv\n" per L/E/C record in stream order
 *                  (bidirected: "u:ori\tv:ori\n").  Only `bidirected` is read from the
 *                  options.  Result format G2N_FMT_TEXT: data = the text, nnz = its length.
 *                  An endpoint key that is not UTF-8 (the export's u.decode() raises):
 *                  status G2N_E_UNICODE with err_line = -1, err_index = the edge record,
 *                  err_detail = the key, and the text holds the lines written before it.
 *                  Parse errors (err_line >= 0) carry no text: the caller renders the
 *                  input's prefix [0, start of err_line) to reproduce the partial output.
 *
 * Errors: a non-zero status is one of G2N_E_*; each maps 1:1 to the exception the
 * reference raises for the same input (type + message; the Python shim re-raises it).
 * Everything runs on the GPU: there is no CPU fallback.  Without a usable HIP device the
 * build entry points return G2N_E_DEVICE.
 */
#ifndef G2N_H
#define G2N_H

#include <stddef.h>
#include <stdint.h>

#define G2N_VERSION_STRING "0.3.0" /* == gfa2network_amd.__version__ (tests check) */

#ifdef __cplusplus
extern "C" {
#endif

#define G2N_ABI_VERSION 2u /* 2: named range / test fields replace options.reserved[] */

/* ---- status codes ------------------------------------------------------------------ */
enum {
  G2N_OK = 0,
  G2N_E_MALFORMED_L = 1,   /* ValueError("Malformed L record")   parser.py:208-209 */
  G2N_E_MALFORMED_E = 2,   /* ValueError("Malformed E record")   parser.py:251-252 */
  G2N_E_MALFORMED_C = 3,   /* ValueError("Malformed C record")   parser.py:299-300 */
  G2N_E_MALFORMED_P = 4,   /* ValueError("Malformed P record")   parser.py:231-232 */
  G2N_E_MALFORMED_O = 5,   /* ValueError("Malformed O record")   parser.py:345-346 */
  G2N_E_INDEX_LIST = 6,    /* IndexError("list index out of range"): S without a name, parser.py:163 */
  G2N_E_INDEX_BYTES = 7,   /* IndexError("index out of range"): u_field[-1] on b"", parser.py:220-221 */
  G2N_E_UNICODE = 8,       /* UnicodeDecodeError: err_detail bytes .decode() (parser.py:127,212,214,291,293,337,339) */
  G2N_E_INT_TOO_LARGE = 9, /* OverflowError("int too large to convert to float"), builders.py:209 */
  G2N_E_CAST_OVERFLOW = 10,/* OverflowError("Python integer X out of bounds for <dtype>"), builders.py:281 */
  G2N_E_CAST_INF = 11,     /* OverflowError("cannot convert float infinity to integer"), builders.py:281 */
  G2N_E_CAST_NAN = 12,     /* ValueError("cannot convert float NaN to integer"), builders.py:281 */
  G2N_E_ARG = 13,          /* invalid options / arguments */
  G2N_E_IO = 14,           /* OSError opening/reading the input; errno in err_index */
  G2N_E_GZIP = 15,         /* corrupt gzip stream (gzip.open path, parser.py:108-109) */
  G2N_E_DEVICE = 16,       /* no usable HIP device / HIP runtime failure */
  G2N_E_NOMEM = 17,        /* host or device allocation failure */
  G2N_E_UNSUPPORTED = 18   /* input exceeds a documented implementation limit */
};

/* ---- matrix dtypes (cli.py:92-97 --dtype choices) ------------------------------------ */
enum { G2N_BOOL = 0, G2N_INT8 = 1, G2N_INT32 = 2, G2N_FLOAT32 = 3, G2N_FLOAT64 = 4 };

enum { G2N_OUT_PARSE = 0, G2N_OUT_CSR = 1, G2N_OUT_COO = 2, G2N_OUT_EDGE_LIST = 3 };
enum { G2N_FMT_COO = 0, G2N_FMT_CSR = 1, G2N_FMT_TEXT = 2 };

/* Mirrors parse_gfa's keyword arguments that affect the matrix (builders.py:30-50). */
typedef struct g2n_options {
  uint32_t abi_version;        /* = G2N_ABI_VERSION */
  int32_t directed;            /* default 1 */
  int32_t bidirected;          /* default 0 */
  int32_t keep_directed_bidir; /* default 0 */
  int32_t asymmetric;          /* default 0 */
  int32_t strip_orientation;   /* default 0 */
  int32_t dtype;               /* G2N_* dtype, default G2N_FLOAT64 */
  int32_t output;              /* G2N_OUT_PARSE (default) | G2N_OUT_CSR | G2N_OUT_COO (the
                                  stream-order COO in every mode: one shard of a sharded build) */
  const char *weight_tag;      /* UTF-8, NUL-terminated; NULL or "" = no weights */
  int32_t want_node_names;     /* 1 (default): produce the names blob in id order */
  int32_t device;              /* HIP device ordinal, default 0 */
  /* ---- set by the sharded / chunked protocol (gfa2network_amd/shard.py); 0 in a plain build ---- */
  int32_t unknown_warned;      /* 1: unsupported records are skipped silently (an earlier byte range
                                  of the same file already raised the one-shot warning) */
  int32_t range_flags;         /* G2N_RANGE_* bits, below */
  int64_t range_s_base;        /* G2N_RANGE_DECIMAL: S lines in the file before this byte range */
  int64_t range_n_segments;    /* G2N_RANGE_DECIMAL: S lines in the whole file */
  /* ---- tests only ---- */
  uint32_t test_flags;         /* G2N_TEST_* bits: take a normally rare path (same results) */
  int32_t reserved_[3];        /* must be 0 (g2n_options_init) */
} g2n_options;

/* g2n_options.range_flags */
enum {
  G2N_RANGE_DECIMAL = 1,        /* one byte range of a sharded decimal-id build: this range's node ids
                                   are global decimals (range_s_base / range_n_segments); output
                                   G2N_OUT_COO, no names; G2N_E_UNSUPPORTED when the range needs the
                                   general protocol (ids that are not decimal, errors, warnings, slow
                                   weights) */
  G2N_RANGE_EVIDENCE = 2,       /* with DECIMAL: report the range's evidence instead of checking the
                                   premise (set by g2n_build_decimal_range) */
  G2N_RANGE_NO_VALUES = 4,      /* no weight tag and the caller reads coordinates only: the result's
                                   values are left unwritten */
  G2N_RANGE_SLOTS = 8           /* with DECIMAL and NO_VALUES (unweighted, not bidirected): the COO stays
                                   in the tile-local parse's group slots (no stream-order compaction);
                                   result rows / cols are the slot arrays, nnz the entries they hold,
                                   the layout from g2n_context_group_slots — what
                                   g2n_route_group_slots and g2n_csr_from_group_slots read */
};

/* g2n_options.test_flags (tests only; every real build leaves 0): the same results through a path
 * that is normally rare on the given input. */
enum {
  G2N_TEST_NO_BUCKETS = 2,      /* MAX-SYM / SUM CSR through the general row sums */
  G2N_TEST_NO_LEAN = 4,         /* decimal ids without the lean parse */
  G2N_TEST_DICT_HASH = 8,       /* hash dictionary (no decimal ids, no direct-address tier) */
  G2N_TEST_DICT_GENERAL = 16,   /* general dictionary rounds */
  G2N_TEST_NO_TILE_LOCAL = 32,  /* decimal ids parsed after K1 (not the tile-local pass) */
  G2N_TEST_HOST_INFLATE = 64,   /* a BGZF .gz read by the host readers (not inflated on the GPU) */
  G2N_TEST_NO_GROUP = 128,      /* tile-local parse into per-tile slots + compaction */
  G2N_TEST_NO_HASH_LEAN = 256,  /* the classic hash tiers, never the lean S-first one */
  G2N_TEST_THROW_AFTER_IDS = 512, /* the build fails (G2N_E_DEVICE) once its ids are set up */
  G2N_TEST_INDEX64 = 1024,      /* CSR results in int64 indptr / indices (the > 2^31 - 1 entries path) */
  G2N_TEST_DICT_DIRECT = 2048,  /* decimal ids in S order through the direct-address tier */
  G2N_TEST_NO_DIRECT = 4096,    /* never the direct-address tier (the lean hash tier instead) */
  G2N_TEST_NO_EXT_LEAN = 8192,  /* bidirected / weighted decimal builds: K1 + the lean parse, not the
                                   extended tile-local parse */
  G2N_TEST_NO_DEC_TEXT = 16384, /* edge-list export of a decimal-id build through the names blob, not
                                   the arithmetic render */
  G2N_TEST_NO_DEC_PREFIX = 32768 /* names "P1".."PN" in S order through the direct-address tier, not
                                   the tile-local decimal parse behind the prefix */
};

#define G2N_MAX_PHASES 40

/* Result of one build.  All pointers are owned by the result (host memory for the
 * host entry points, device memory for g2n_build_device) and stay valid until
 * g2n_result_free (or, for g2n_build_device, until the next build on the context). */
typedef struct g2n_result {
  uint32_t abi_version;
  int32_t status;              /* G2N_OK or G2N_E_* */
  int64_t err_line;            /* 0-based input line of the failing record (parse errors) */
  int64_t err_index;           /* cast errors: element index in the triplet stream; IO: errno */
  double err_value;            /* cast errors: the offending float64 value */
  const uint8_t *err_detail;   /* G2N_E_UNICODE: the bytes whose .decode() raises */
  int64_t err_detail_len;
  int32_t has_warning;         /* RuntimeWarning("Skipping unsupported record: <c>") */
  int32_t warn_byte;           /* <c> (first byte of the first unsupported line) */
  int64_t warn_line;           /* first unsupported-record line (-1: none), warned or not */
  int64_t n_lines;             /* lines seen (Python binary line iteration) */
  int64_t n_records;           /* records the parser yielded (S/L/E/C/P/O) */
  int64_t n_records_before_error;
  int64_t n_edges;             /* L + E + C records */
  int64_t n_nodes;             /* matrix is n_nodes x n_nodes */
  const uint8_t *names_blob;   /* node keys in id order (builders.py:284-288), concatenated */
  const int64_t *names_offsets;/* n_nodes + 1 offsets into names_blob */
  int32_t format;              /* G2N_FMT_COO | G2N_FMT_CSR */
  int32_t dtype;
  int32_t index_width;         /* 4 (int32) or 8 (int64) for rows/cols/indptr/indices */
  int32_t sum_sorted;          /* scipy has_sorted_indices of the scattered COO (diagnostic; -1: not
                                  computed — the CSR came from the bucket partition) */
  int64_t nnz;                 /* COO: triplet count; CSR: stored entries */
  const void *rows;            /* COO */
  const void *cols;            /* COO */
  const void *indptr;          /* CSR: n_nodes + 1 */
  const void *indices;         /* CSR */
  const void *data;            /* nnz elements of dtype */
  uint64_t names_bytes;        /* names blob length (0 when want_node_names is 0) */
  int64_t n_cast_overflow;     /* float32 casts that overflowed to +-inf: numpy warns
                                  RuntimeWarning("overflow encountered in cast") once each */
  uint64_t input_bytes;        /* uncompressed GFA bytes parsed */
  int32_t n_phases;            /* device phase timings (hipEvent, pipeline stream) */
  int32_t sum_t_sorted;        /* MAX-SYM: has_sorted_indices of A.T's scattered COO (diagnostic) */
  double phase_ms[G2N_MAX_PHASES];
  const char *phase_names[G2N_MAX_PHASES];
  double host_ms_read;         /* host ingest (read / inflate) */
  double host_ms_h2d;          /* host -> device copy of the input */
  double host_ms_d2h;          /* device -> host copy of the outputs */
  void *priv_;
} g2n_result;

/* ---- library ------------------------------------------------------------------------- */
const char *g2n_version(void);
uint32_t g2n_abi_version(void);
void g2n_options_init(g2n_options *opts);      /* reference defaults (builders.py:30-50) */
int g2n_device_count(void);                    /* HIP devices visible (0 without a GPU) */
/* hipMemGetInfo of `device`: free / total HBM bytes (G2N_E_DEVICE without such a device).  What
 * parse_gfa sizes its one-GPU chunked build by (gfa2network_amd/api.py), without torch. */
int g2n_device_memory(int32_t device, uint64_t *free_bytes, uint64_t *total_bytes);
/* The host entry points (g2n_build_from_path / _buffer, g2n_coo_to_csr) keep one cached context per
 * device whose grow-only buffers outlive the call (results are host copies).  This frees them all
 * (*freed: the bytes released): what parse_gfa does before sizing a build against free HBM when an
 * earlier, larger build's buffers would otherwise count as used. */
int g2n_release_shared(int32_t device, uint64_t *freed);
const char *g2n_last_error(void);              /* thread-local message of the last failure */
const char *g2n_status_name(int status);

/* ---- host entry points (results in host memory) ---------------------------------------- */
/* path: "-" = stdin; a name ending in ".gz" is gunzipped (multi-member); anything else is
 * read raw — the same rule as parser.py:100-112 (by name, not by magic bytes). */
int g2n_build_from_path(const char *path, const g2n_options *opts, g2n_result **out);
int g2n_build_from_buffer(const void *buf, size_t len, const g2n_options *opts, g2n_result **out);
void g2n_result_free(g2n_result *res);

/* gzip.open(...).read() of an in-memory .gz file (parser.py:108-109): the reader that
 * g2n_build_from_path uses for ".gz" names.  parallel = 1: members are inflated concurrently
 * on host threads (G2N_HOST_THREADS) when the file is a clean member chain, else serially;
 * parallel = 0: always the serial reader.  On success *out (free with g2n_free) holds *out_len
 * bytes and *members the member count.  On failure returns G2N_E_GZIP, *sub = the exception
 * gzip.py raises (1 BadGzipFile, 2 EOFError, 3 zlib.error, 4 BadGzipFile CRC/length),
 * g2n_last_error() its message, and *out / *out_len the bytes gzip.py's reader returned before
 * raising (io.BufferedReader refills of 8192: what a line loop over gzip.open sees; g2n_free it). */
int g2n_gunzip(const void *buf, size_t len, int32_t parallel, void **out, size_t *out_len, int32_t *members,
               int32_t *sub);
/* The chunk-parallel single-member inflate alone (what g2n_gunzip's parallel path tries first
 * for a file of >= 64 MiB with few member candidates): one gzip member to the end of the file
 * (zero padding allowed), its deflate stream cut into chunks of chunk_bytes compressed bytes
 * (0 = sized for the host threads) that are inflated concurrently.  G2N_OK with *out / *out_len
 * (g2n_free) and *chunks = the chunks that decoded from a block start of their own; G2N_E_UNSUPPORTED
 * when it declines (not one clean member, or a stream its decoder refuses: the exact reader decides).
 * Replaces gzip.open's serial read of one member (parser.py:108-109). */
int g2n_gunzip_chunked(const void *buf, size_t len, size_t chunk_bytes, void **out, size_t *out_len,
                       int32_t *chunks);
void g2n_free(void *p);

/* parse_gfa(..., split_on_alignment=True) (builders.py:110-128 -> _parse_gfa_split,
 * builders.py:302-568), host side: the segments cut at the E / C alignment coordinates, the
 * records re-targeted to the intervals, and that record stream rendered as GFA text ("S" lines
 * for the interval segments unless bidirected, "E\t*\tu\tori\tv\tori[\ttags]" for every link
 * and edge) for g2n_build_from_buffer to build with the reference's main-path semantics.  The
 * input must have parsed cleanly first (errors are the plain parse's).  names = the interval
 * segments in mint order (bidirected: placed before the GPU build's nodes); warn_* = the
 * "skipping edge / link" warnings in order (kind 0 edge, 1 link; the segment bytes);
 * many_nodes = the ">10x more nodes" warning; g2n_split_segments = intervals per segment.  G2N_E_UNSUPPORTED for a length or coordinate
 * beyond int64.  Free with g2n_split_free. */
typedef struct g2n_split_out g2n_split_out;
int g2n_split_render(const void *buf, size_t len, int32_t bidirected, g2n_split_out **out);
void g2n_split_get(const g2n_split_out *o, const uint8_t **text, uint64_t *text_len, const uint8_t **names,
                   const int64_t **name_offs, uint64_t *n_names, const uint8_t **warn_segs,
                   const int64_t **warn_offs, const int32_t **warn_kind, uint64_t *n_warn, int32_t *many_nodes);
/* intervals per segment (the segments dict's order): the bidirected id map's block sizes */
void g2n_split_segments(const g2n_split_out *o, const int64_t **intervals, uint64_t *n_segments);
void g2n_split_free(g2n_split_out *o);

/* The node list's bytes joined by `sep` (builders.py:284-288 node_list, built in one pass by
 * the Python shim): out (n_names ? blob_len + n_names - 1 : 0 bytes) = name 0, sep, name 1, ...
 * with name i = blob[offsets[i] .. offsets[i+1]).  Host memory, parallel over host threads. */
int g2n_join_names(const uint8_t *blob, const int64_t *offsets, uint64_t n_names, uint8_t sep, uint8_t *out);

/* Names in a new order: out name i = name order[i] of (blob, offsets), written at out_offsets[i] -
 * out_offsets[0] (the caller scans the reordered lengths).  The sharded build's node list: each
 * owner rank's distinct keys arrive in owner order and are put in global id order
 * (builders.py:284-288 node_list = keys in node2idx insertion order).  Host threads. */
int g2n_gather_names(const uint8_t *blob, const int64_t *offsets, const int64_t *order, uint64_t n_names,
                     const int64_t *out_offsets, uint8_t *out);

/* ---- convert CLI writers (host threads) -------------------------------------------------
 * scipy.sparse.save_npz(path, A) as `convert --matrix x.npz` calls it (utils.py:85-86): a
 * zip64 archive of deflated members (numpy savez_compressed's layout).  Member i is named
 * names[i] and holds heads[i] (its .npy header, head_lens[i] bytes, built by numpy's format
 * code) followed by datas[i] (data_lens[i] bytes).  level: zlib level (-1 = zlib's default, as
 * numpy).  Returns G2N_E_IO (errno text in g2n_last_error) when the file cannot be written. */
int g2n_write_npz(const char *path, int32_t n_members, const char *const *names, const uint8_t *const *heads,
                  const uint64_t *head_lens, const void *const *datas, const uint64_t *data_lens, int32_t level);

/* save_node_map (utils.py:108-114): "i\tname\n" for the names blob/offsets in id order.
 * check_utf8 = 1 (raw_bytes_id names, decoded while writing): only the names before the first
 * one that is not valid UTF-8 are written and *bad_index is its id (-1: all valid). */
int g2n_write_node_map(const char *path, const uint8_t *blob, const int64_t *offsets, uint64_t n_names,
                       int32_t check_utf8, int64_t *bad_index);

/* Index of the first name that is not valid UTF-8 (Python's strict decoder), or -1. */
int64_t g2n_first_bad_utf8(const uint8_t *blob, const int64_t *offsets, uint64_t n_names);

/* convert_format(A, "csr") for a COO matrix (utils.py:40-63 -> scipy coo.tocsr):
 * sums duplicates in dtype with scipy's summation order, keeps explicit zeros.
 * rows/cols have index_width (4) bytes per element, data has dtype elements; n_rows x n_cols
 * (each < 2^31 - 1).  indptr / indices come back in scipy's index dtype: int64 (index_width 8)
 * once nnz passes 2^31 - 1 (_coo_to_compressed: maxval = coo.nnz, duplicates included).  Up to
 * 2^32 - 2 entries when every value is dtype(1) (a parse without a weight tag); other values
 * past 2^31 - 2 entries return G2N_E_UNSUPPORTED.  test_flags: G2N_TEST_INDEX64 /
 * G2N_TEST_NO_BUCKETS (tests only; 0 otherwise). */
int g2n_coo_to_csr(const void *rows, const void *cols, const void *data, int64_t nnz, int64_t n_rows,
                   int64_t n_cols, int32_t index_width, int32_t dtype, int32_t device, uint32_t test_flags,
                   g2n_result **out);

/* One row band of a COO too large for g2n_coo_to_csr's weighted limit (rows band-local, 0..n_rows-1,
 * in the whole COO's stream order): the band's CSR.  force_unsorted = -1: the band's own sortedness
 * decides (as for a whole matrix); 0 / 1: scipy's has_sorted_indices verdict of the WHOLE matrix
 * (coo.tocsr -> sum_duplicates sorts every row when any is unsorted, utils.py:55), which decides
 * the order float duplicates are summed in.  result.sum_sorted: this band's own verdict (-1: the
 * band's sums cannot depend on order).  The caller (gfa2network_amd/_native.py coo_to_csr) cuts the
 * bands, asks each for its verdict, re-runs the sorted ones with 1 when another is unsorted, and
 * concatenates them with int64 indptr / indices as scipy returns past 2^31 - 1 entries. */
int g2n_coo_to_csr_band(const void *rows, const void *cols, const void *data, int64_t nnz, int64_t n_rows,
                        int64_t n_cols, int32_t dtype, int32_t device, int32_t force_unsorted, g2n_result **out);

/* ---- device-resident entry points (the measured hot path) ------------------------------ */
typedef struct g2n_context g2n_context;
g2n_context *g2n_context_create(int device);   /* NULL on failure (see g2n_last_error) */
void g2n_context_destroy(g2n_context *ctx);
void *g2n_context_stream(g2n_context *ctx);    /* the hipStream_t the pipeline runs on */
/* d_input: len bytes already in this device's HBM.  The result's pointers are DEVICE
 * pointers owned by ctx, valid until the next build on ctx.  The call returns after the
 * stream has drained (counts must be read back); phase timings are hipEvent-based. */
int g2n_build_device(g2n_context *ctx, const void *d_input, size_t len, const g2n_options *opts,
                     g2n_result *out);
/* Release ctx's grow-only arena buffers except those holding one of the n_keep device pointers
 * (results the caller still reads, e.g. a build's rows / cols): the working set of one sharded rank
 * between protocol stages (its dictionary, touch descriptors, partition buffers), which would
 * otherwise stay allocated until ctx's next build needs them.  *freed (optional) = bytes released.
 * No reference counterpart (the reference has no device memory); a later call re-allocates. */
int g2n_context_trim(g2n_context *ctx, const void *const *keep, uint64_t n_keep, uint64_t *freed);

/* ---- sharded build: device-side steps of one file split over ranks --------
 * Each rank builds its byte range with output = G2N_OUT_COO (local ids = first-touch order
 * inside the range, local names blob).  The protocol (gfa2network_amd/shard.py) routes names
 * to owner ranks, where g2n_dedup_keys keeps the first occurrence of each key in arrival
 * order (arrivals are concatenated in rank order, so that is the global first-touch order);
 * global ids go back to the ranks, g2n_route_triplets remaps and partitions the COO by the
 * owner of each row (and, for MAX-SYM, of each column: the A.T stream), and
 * g2n_csr_from_coo_pair builds the rank's CSR row slice.  All pointers are DEVICE pointers
 * on ctx's device; calls return after the stream drained. */

/* keys i in [0, n): bytes d_blob[d_offsets[i] .. d_offsets[i+1]).  d_ids[i] = index of key i's
 * distinct key, numbered in order of first occurrence; d_first[k] = first occurrence of
 * distinct key k (k < *n_distinct; d_first sized n).  Exact byte comparison. */
int g2n_dedup_keys(g2n_context *ctx, const uint8_t *d_blob, uint64_t blob_len, const int64_t *d_offsets,
                   uint64_t n, uint32_t *d_ids, uint32_t *d_first, uint64_t *n_distinct);

/* A growing device set of byte keys with dense ids in insertion order (the chunked build's
 * file-wide names, gfa2network_amd/shard.py _chunked_general; replaces re-running
 * g2n_dedup_keys over every key so far for each chunk).  g2n_keyset_add looks up keys i < n
 * (d_blob / d_offsets as for g2n_dedup_keys; DISTINCT within one call): d_ids[i] = the key's id,
 * a key not in the set yet taking the next id in call order (builders.py:194-198 first-touch
 * minting); *n_total = keys in the set after the call.  g2n_keyset_view: the set's keys in id
 * order (device pointers owned by the set, valid until its next add or free).  The set works on
 * ctx's device and stream; ctx must outlive every add / view (g2n_keyset_free does not use it). */
typedef struct g2n_keyset g2n_keyset;
int g2n_keyset_create(g2n_context *ctx, g2n_keyset **out);
int g2n_keyset_add(g2n_keyset *ks, const uint8_t *d_blob, uint64_t blob_len, const int64_t *d_offsets, uint64_t n,
                   uint32_t *d_ids, uint64_t *n_total);
int g2n_keyset_view(g2n_keyset *ks, const uint8_t **d_blob, const int64_t **d_offsets, uint64_t *n,
                    uint64_t *blob_len);
void g2n_keyset_free(g2n_keyset *ks);

/* Key i of the names blob goes to rank (FNV-1a of its bytes) mod n_ranks: the keys, grouped
 * by rank (order kept within a rank), to d_out_blob / d_out_offsets (n + 1); d_out_index[j] =
 * the input index of output key j; d_starts[r] = first output key of rank r. */
int g2n_partition_keys(g2n_context *ctx, const uint8_t *d_blob, uint64_t blob_len, const int64_t *d_offsets,
                       uint64_t n, uint32_t n_ranks, uint8_t *d_out_blob, int64_t *d_out_offsets,
                       uint32_t *d_out_index, uint32_t *d_starts);

/* Keys d_index[j] (j < n) of a names blob, in that order, to d_out_blob (out_cap bytes) and
 * d_out_offsets (n + 1); *out_len = bytes written.  G2N_E_ARG if they exceed out_cap (nothing
 * written to d_out_blob then).  The owner's distinct keys for the names gather. */
int g2n_gather_keys(g2n_context *ctx, const uint8_t *d_blob, const int64_t *d_offsets, const uint32_t *d_index,
                    uint64_t n, uint8_t *d_out_blob, uint64_t out_cap, int64_t *d_out_offsets, uint64_t *out_len);

/* d_rows[i] = d_map[d_rows[i]], d_cols[i] = d_map[d_cols[i]] in place (i < n): a range's COO
 * from local to global ids.  G2N_E_ARG if an id is >= n_map (those entries become -1). */
int g2n_remap_pairs(g2n_context *ctx, const uint32_t *d_map, uint64_t n_map, int32_t *d_rows, int32_t *d_cols,
                    uint64_t n);

/* Triplet i = (d_map[d_rows[i]],d_map[d_cols[i]], d_data[i]) (transposed: row and column
 * swapped) goes to rank floor(row * n_ranks / n_global); the output holds them grouped by
 * rank, stream order kept within a rank; d_starts[r] = first output of rank r
 * (d_starts[n_ranks] = nnz).  Outputs sized nnz (data: nnz elements of dtype).  d_map may be
 * NULL: the identity map (the rows / cols already hold global ids, the decimal-id shard path).
 * d_data and d_out_data both NULL: the coordinates only (uniform values need no routing). */
int g2n_route_triplets(g2n_context *ctx, const int32_t *d_rows, const int32_t *d_cols, const void *d_data,
                       uint64_t nnz, int32_t dtype, const uint32_t *d_map, uint64_t n_global, uint32_t n_ranks,
                       int32_t transposed, int32_t *d_out_rows, int32_t *d_out_cols, void *d_out_data,
                       uint32_t *d_starts);

/* CSR of rows [row_base, row_base + n_rows) from the stream-order triplets of A whose rows
 * fall there (global row ids) and, for MAX-SYM, those of A.T (rows = A's columns):
 * maxsym = 0: coo.tocsr() of A's slice; 1: A.maximum(A.T)'s slice.  uniform: every value is
 * dtype(1) (no weight tag).  force_unsorted: -1 = this slice decides scipy's
 * has_sorted_indices; else the caller's global verdicts (the OR over all slices), bit 0 for
 * A, bit 1 for A.T (only weighted float rows of > 16 entries depend on them).  The result's
 * sum_sorted / sum_t_sorted report this slice's own verdicts.  Result pointers are device pointers
 * owned by ctx (format CSR, n_nodes = n_rows). */
int g2n_csr_from_coo_pair(g2n_context *ctx, const int32_t *a_rows, const int32_t *a_cols, const void *a_data,
                          uint64_t a_nnz, const int32_t *t_rows, const int32_t *t_cols, const void *t_data,
                          uint64_t t_nnz, int32_t maxsym, int64_t row_base, uint64_t n_rows, uint64_t n_cols,
                          int32_t dtype, int32_t uniform, int32_t force_unsorted, g2n_result *out);

/* Group slots (round 6): a sharded decimal range built with G2N_RANGE_SLOTS keeps its COO where the
 * tile-local parse wrote it — group g's entries at [g * gcap, g * gcap + gcount[g]) of rows / cols —
 * instead of compacting it into stream order.  g2n_context_group_slots reports the last build's layout
 * on ctx (n_groups 0: the last build left none); valid until ctx's next build.
 * g2n_route_group_slots: g2n_route_triplets of those slots (coordinates only, no map, n_ranks <= 256;
 *   nnz = the entries they hold; within an owner the order is slot order, which an unweighted slice
 *   CSR does not read).
 * g2n_csr_from_group_slots: a ONE-rank group's whole CSR (row_base 0, n_rows rows) from the slots —
 *   the SUM CSR (maxsym 0) or A.maximum(A.T) (maxsym 1) of unit values, the single-GPU bucket
 *   partition; G2N_E_UNSUPPORTED when it declines (no entries, an overfull bucket): the caller then
 *   builds the range's stream-order COO and calls g2n_csr_from_coo_pair. */
int g2n_context_group_slots(g2n_context *ctx, const uint32_t **d_gcount, uint64_t *n_groups, uint64_t *gcap);
int g2n_route_group_slots(g2n_context *ctx, const int32_t *d_rows, const int32_t *d_cols, const uint32_t *d_gcount,
                          uint64_t n_groups, uint64_t gcap, uint64_t nnz, uint64_t n_global, uint32_t n_ranks,
                          int32_t transposed, int32_t *d_out_rows, int32_t *d_out_cols, uint32_t *d_starts);
int g2n_csr_from_group_slots(g2n_context *ctx, const int32_t *d_rows, const int32_t *d_cols, const uint32_t *d_gcount,
                             uint64_t n_groups, uint64_t gcap, uint64_t nnz, int32_t maxsym, uint64_t n_rows,
                             int32_t dtype, g2n_result *out);

/* The general protocol's global node ids (shard.py step 4; builders.py:194-198 first-touch order
 * across byte ranges), on an owner rank's distinct keys (g2n_dedup_keys):
 * g2n_order_keys: out[j] = (source rank << 32) | the key's local id there, for the key's first arrival
 *   f = d_first_of[j], the source being the one whose arrival range holds f (src_ends: the sources'
 *   inclusive arrival-count prefix sums, host memory, n_src <= 4096); d_src_idx[f] = the local id the
 *   source sent with arrival f.  The keys ascend with j.
 * g2n_rank_keys: out[j] = j + the number of keys smaller than d_keys[j] in every other owner's sorted
 *   run of d_all (runs at all_offsets[o] .. all_offsets[o + 1], host memory): the key's global id. */
int g2n_order_keys(g2n_context *ctx, const uint32_t *d_first_of, const int64_t *d_src_idx, uint64_t nd,
                   const uint64_t *src_ends, uint32_t n_src, uint64_t *d_out);
int g2n_rank_keys(g2n_context *ctx, const uint64_t *d_keys, uint64_t n, const uint64_t *d_all,
                  const uint64_t *all_offsets, uint32_t n_ranks, uint32_t self_rank, int64_t *d_out);

/* One rank's byte range of a file split over ranks: bytes [offset, offset + len) of path, read
 * with pread into pinned staging slots and copied to d_dst (len bytes of `device`'s HBM). */
int g2n_upload_file_range(const char *path, uint64_t offset, uint64_t len, void *d_dst, int32_t device);

/* The record counts of a device-resident range, before any build (what the ranks of a sharded
 * build exchange first): out4 = {lines, S lines, edge records (L/E/C), records (S/L/E/C/P/O)}. */
int g2n_count_device(g2n_context *ctx, const void *d_input, size_t len, int64_t *out4);

/* One byte range of a sharded decimal-id build (S lines named "1".."N" in order), built BEFORE the
 * ranges' record counts are exchanged: one pass of the tile-local lean parse writes the range's
 * stream-order COO over GLOBAL ids (name value - 1; builders.py:190-198 first-touch order when the
 * premise holds) and reports the evidence the caller checks across ranges (shard.py):
 *   ev6 = {lines, S lines, edge records, records,
 *          d: the range's first S line names d + 1 and every later one continues it (-1: no S line;
 *             the premise needs d == the S lines of the ranges before),
 *          the largest edge key value (the premise needs it <= the file's S lines)}.
 * Options: output G2N_OUT_COO, no names, not bidirected, no weight tag, no strip (else G2N_E_ARG);
 * range_* are set by the call (G2N_RANGE_NO_VALUES is kept).  G2N_E_UNSUPPORTED when the one pass declines (a line past
 * its tile window, a record outside the lean shapes, S names that are not one decimal run, an S
 * line after an edge line in the range): the caller then counts the ranges (g2n_count_device) and
 * builds with G2N_RANGE_DECIMAL (g2n_build_device), whose check decides.  Replaces the count pass of
 * the sharded build for the common layout; results as g2n_build_device's (device pointers). */
int g2n_build_decimal_range(g2n_context *ctx, const void *d_input, size_t len, const g2n_options *opts,
                            int64_t *ev6, g2n_result *out);

#ifdef __cplusplus
}
#endif
#endif /* G2N_H */
