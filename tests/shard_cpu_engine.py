"""CPU engine for the sharded-build protocol (gfa2network_amd/shard.py) — TEST INFRASTRUCTURE.

Drives the product's exchange protocol on gloo without a GPU: each step the HIP engine does on
the device is done here by the oracle (per-range build) and numpy/scipy (key partition, dedup,
routing, per-slice coo.tocsr() / maximum).  Only tests import it.
"""
from __future__ import annotations

import zlib

import numpy as np
import scipy.sparse as sp
import torch

from gfa2network_amd.shard import TORCH_DTYPES, LocalShard

NP = {"bool": np.uint8, "int8": np.int8, "int32": np.int32, "float32": np.float32, "float64": np.float64}


class _CpuKeyset:
    """HipEngine.keyset's contract on the host: ids in insertion order, the keys of one add distinct."""

    def __init__(self):
        self.ids, self.keys = {}, []

    def add(self, blob, offsets):
        b, off = blob.numpy().tobytes(), offsets.numpy()
        out = []
        for i in range(len(off) - 1):
            k = b[off[i]:off[i + 1]]
            if k not in self.ids:
                self.ids[k] = len(self.keys)
                self.keys.append(k)
            out.append(self.ids[k])
        return torch.tensor(out, dtype=torch.int32), len(self.keys)

    def names(self):
        offs = np.zeros(len(self.keys) + 1, dtype=np.int64)
        np.cumsum([len(k) for k in self.keys], out=offs[1:])
        return torch.from_numpy(np.frombuffer(b"".join(self.keys), dtype=np.uint8).copy()), torch.from_numpy(offs)

    def close(self):
        pass


class CpuEngine:
    device = torch.device("cpu")

    def __init__(self, oracle_mod):
        self.oracle = oracle_mod

    def cat(self, xs):  # (HipEngine.cat's contract)
        return torch.cat(xs) if len(xs) > 1 else xs[0]

    def local_build(self, buf, opts, unknown_warned=False):
        o = self.oracle.run(bytes(buf.numpy()), **opts)
        if unknown_warned and o.status == 8:
            raise NotImplementedError("the oracle has no silent-unknown-record mode")
        sh = LocalShard(status=o.status, err_line=o.err_line, err_index=o.err_index, err_value=o.err_value,
                        err_detail=o.err_detail, warn_line=o.warn_line if o.has_warning else -1,
                        has_warning=o.has_warning, warn_byte=o.warn_byte, n_lines=o.n_lines,
                        n_records=o.n_records, n_records_before_error=o.n_records_before_error,
                        n_edges=0, n_local_nodes=o.n_nodes,
                        n_cast_overflow=o.n_cast_overflow)
        if o.status != 0:
            return sh
        bidir, keep = opts.get("bidirected", False), opts.get("keep_directed_bidir", False)
        gd = keep or (not bidir and opts.get("directed", True))
        ktrip = 4 if (bidir and not keep) else (1 if gd else 2)
        sh.n_edges = len(o.rows) // ktrip
        dt = opts.get("dtype", "float64")
        sh.rows = torch.from_numpy(o.rows.astype(np.int32))
        sh.cols = torch.from_numpy(o.cols.astype(np.int32))
        sh.data = torch.from_numpy(np.ascontiguousarray(o.data).view(NP[dt]).copy())
        sh.names_blob = torch.from_numpy(o.names_blob.copy())
        sh.names_offsets = torch.from_numpy(o.names_offsets.astype(np.int64))
        return sh

    def read_range(self, path, offset, length):
        import os

        with open(path, "rb") as fh:
            return torch.from_numpy(np.frombuffer(os.pread(fh.fileno(), length, offset), dtype=np.uint8).copy())

    def count(self, buf):
        """{lines, S lines, edge records, records} of the range: first-byte dispatch as K1 does it
        (a record type must be followed by a tab, a newline or the end of the input)."""
        b = bytes(buf.numpy())
        lines = b.split(b"\n")
        if lines and lines[-1] == b"":
            lines.pop()
        kind = [ln[:1] if (len(ln) == 1 or ln[1:2] == b"\t") else b"" for ln in lines]
        segs = sum(k == b"S" for k in kind)
        edges = sum(k in (b"L", b"E", b"C") for k in kind)
        po = sum(k in (b"P", b"O") for k in kind)
        return [len(lines), segs, edges, segs + edges + po]

    def build_decimal(self, buf, opts, s_base, n_seg, view=False, values=True):
        """The oracle's range build with its local ids mapped to GLOBAL decimal ids, or None when a
        key is not the canonical decimal of a segment (or the range has a warning / error)."""
        o = self.oracle.run(bytes(buf.numpy()), **opts)
        if o.status != 0 or o.has_warning:
            return None
        bidir = opts.get("bidirected", False)
        blob, off = o.names_blob.tobytes(), o.names_offsets
        gid = np.empty(o.n_nodes, dtype=np.int64)
        for i in range(o.n_nodes):
            k = blob[off[i]:off[i + 1]]
            name, ori = (k[:-2], k[-1:]) if bidir else (k, b"")
            if bidir and (len(k) < 3 or k[-2:-1] != b":" or ori not in (b"+", b"-")):
                return None
            if not name.isdigit() or name[:1] == b"0" or not (1 <= int(name) <= n_seg):
                return None
            gid[i] = (int(name) - 1) * (2 if bidir else 1) + (ori == b"-")
        # S lines of this range must be named s_base + 1, s_base + 2, ... in order
        s_names = [ln.split(b"\t")[1] for ln in bytes(buf.numpy()).split(b"\n")
                   if ln[:2] == b"S\t" and len(ln.split(b"\t")) > 1]
        if s_names != [str(s_base + k + 1).encode() for k in range(len(s_names))]:
            return None
        sh = self.local_build(buf, opts)
        sh.rows = torch.from_numpy(gid[sh.rows.numpy()].astype(np.int32))
        sh.cols = torch.from_numpy(gid[sh.cols.numpy()].astype(np.int32))
        sh.n_local_nodes = n_seg * (2 if bidir else 1)
        return sh

    def build_decimal_range(self, buf, opts, view=False, values=True):
        """g2n_build_decimal_range's contract on the oracle: the range's COO over global decimal ids
        and its evidence [lines, S lines, edges, records, d, largest edge key], or None when the one
        pass would decline (not one run of canonical decimal S names, an S line after an edge line,
        an edge key that is no canonical decimal, an error or warning in the range)."""
        b = bytes(buf.numpy())
        o = self.oracle.run(b, **opts)
        if o.status != 0 or o.has_warning:
            return None
        recs = [ln.split(b"\t") for ln in b.split(b"\n") if ln[:2] in (b"S\t", b"L\t", b"E\t", b"C\t")]
        canon = lambda k: k.isdigit() and k[:1] != b"0"  # noqa: E731 - str(v) is v's only spelling
        s_names, seen_edge, vmax = [], False, 0
        for f in recs:
            if f[0] == b"S":
                if seen_edge or len(f) < 2 or not canon(f[1]):
                    return None
                s_names.append(int(f[1]))
            else:
                seen_edge = True
        d = s_names[0] - 1 if s_names else -1
        if s_names != list(range(d + 1, d + 1 + len(s_names))):
            return None
        blob, off = o.names_blob.tobytes(), o.names_offsets
        gid = np.empty(o.n_nodes, dtype=np.int64)
        for i in range(o.n_nodes):
            k = blob[off[i]:off[i + 1]]
            if not canon(k) or int(k) > 2**31 - 2:
                return None
            gid[i] = int(k) - 1
        sh = self.local_build(buf, opts)
        if sh.rows.numel():
            vmax = int(max(gid[sh.rows.numpy()].max(), gid[sh.cols.numpy()].max())) + 1
        sh.rows = torch.from_numpy(gid[sh.rows.numpy()].astype(np.int32))
        sh.cols = torch.from_numpy(gid[sh.cols.numpy()].astype(np.int32))
        c = self.count(buf)
        return sh, [c[0], c[1], c[2], c[3], d, vmax]

    def partition_keys(self, blob, offsets, n_ranks):
        b, off = blob.numpy().tobytes(), offsets.numpy()
        n = len(off) - 1
        keys = [b[off[i]:off[i + 1]] for i in range(n)]
        owner = np.array([zlib.crc32(k) % n_ranks for k in keys], dtype=np.int64)
        order = np.argsort(owner, kind="stable")
        oblob = b"".join(keys[i] for i in order)
        ooff = np.zeros(n + 1, dtype=np.int64)
        ooff[1:] = np.cumsum([len(keys[i]) for i in order])
        starts = np.searchsorted(owner[order], np.arange(n_ranks + 1)).astype(np.int32)
        return (torch.from_numpy(np.frombuffer(oblob, dtype=np.uint8).copy()), torch.from_numpy(ooff),
                torch.from_numpy(order.astype(np.int32)), torch.from_numpy(starts))

    def order_keys(self, first_of, src_idx, src_counts):
        """g2n_order_keys on the host: (source rank << 32) | local id of each distinct key's first arrival."""
        f = first_of.numpy().astype(np.int64)
        ends = np.cumsum(np.asarray(src_counts, dtype=np.int64))
        src = np.searchsorted(ends, f, side="right").astype(np.int64)
        return torch.from_numpy((src << 32) | src_idx.numpy().astype(np.int64)[f])

    def rank_keys(self, keys, all_keys, rank):
        """g2n_rank_keys on the host: index + the smaller keys of every other owner."""
        k = keys.numpy()
        g = np.arange(len(k), dtype=np.int64)
        for o, other in enumerate(all_keys):
            if o != rank and other.numel():
                g += np.searchsorted(other.numpy(), k, side="left")
        return torch.from_numpy(g)

    def dedup_keys(self, blob, offsets):
        b, off = blob.numpy().tobytes(), offsets.numpy()
        seen, ids, first = {}, [], []
        for i in range(len(off) - 1):
            k = b[off[i]:off[i + 1]]
            if k not in seen:
                seen[k] = len(first)
                first.append(i)
            ids.append(seen[k])
        return (torch.tensor(ids, dtype=torch.int32), torch.tensor(first, dtype=torch.int32), len(first))

    def keyset(self):
        return _CpuKeyset()

    def gather_keys(self, blob, offsets, index, nbytes):
        b, off = blob.numpy().tobytes(), offsets.numpy()
        keys = [b[off[i]:off[i + 1]] for i in index.numpy().astype(np.int64)]
        ooff = np.zeros(len(keys) + 1, dtype=np.int64)
        ooff[1:] = np.cumsum([len(k) for k in keys])
        assert ooff[-1] == nbytes
        return torch.from_numpy(np.frombuffer(b"".join(keys), dtype=np.uint8).copy()), torch.from_numpy(ooff)

    def remap_pairs(self, rows, cols, gmap):
        m = gmap.numpy().astype(np.int64)
        return (torch.from_numpy(m[rows.numpy()].astype(np.int32)), torch.from_numpy(m[cols.numpy()].astype(np.int32)))

    def route_triplets(self, rows, cols, data, dtype, gmap, n_global, n_ranks, transposed):
        if gmap is None:  # ids are global already (decimal fast path)
            r, c = rows.numpy().astype(np.int64), cols.numpy().astype(np.int64)
        else:
            m = gmap.numpy().astype(np.int64)
            r, c = m[rows.numpy()], m[cols.numpy()]
        if transposed:
            r, c = c, r
        owner = r * n_ranks // max(n_global, 1)
        order = np.argsort(owner, kind="stable")
        starts = np.searchsorted(owner[order], np.arange(n_ranks + 1)).astype(np.int32)
        d = None if data is None else torch.from_numpy(data.numpy()[order].copy())  # None: uniform values
        return (torch.from_numpy(r[order].astype(np.int32)), torch.from_numpy(c[order].astype(np.int32)), d,
                torch.from_numpy(starts))

    def csr_pair(self, a, t, maxsym, row_base, n_rows, n_cols, dtype, uniform, force_unsorted):
        npdt = np.bool_ if dtype == "bool" else NP[dtype]

        def csr(x):
            rows = x[0].numpy().astype(np.int64) - row_base
            vals = (np.ones(len(rows), dtype=npdt) if uniform or x[2] is None
                    else x[2].numpy().view(NP[dtype]).astype(npdt))
            return sp.coo_matrix((vals, (rows, x[1].numpy().astype(np.int64))),
                                 shape=(n_rows, n_cols)).tocsr()

        M = csr(a)
        if maxsym:
            M = M.maximum(csr(t))
        data = M.data.astype(NP[dtype]) if dtype != "bool" else M.data.astype(np.uint8)
        tdt = getattr(torch, TORCH_DTYPES[dtype])
        return (torch.from_numpy(M.indptr.astype(np.int32)), torch.from_numpy(M.indices.astype(np.int32)),
                torch.from_numpy(data).to(tdt), False, False)

    # the chunked build's source / memory hooks (shard.build_chunked)
    free_bytes = 1 << 60

    def upload(self, arr):
        return torch.from_numpy(np.array(arr, dtype=np.uint8))

    def free_memory(self):
        return self.free_bytes

    def reset(self):
        pass

    def close(self):
        pass
