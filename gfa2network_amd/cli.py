"""``python -m gfa2network_amd convert ...`` — the reference's ``convert --matrix`` front-end.

Same global flags (they precede the subcommand) and ``convert`` flags as
gfa2network/cli.py:22-135, same handler order (cli.py:193-250): print the backend, parse,
``convert_format``, ``save_matrix`` (dense guard -> SystemExit), then the
``<matrix>.nodes.tsv`` sidecar.  ``export --format edge-list`` (cli.py:264-281) renders its
lines on the GPU from the same parse.  Graph outputs (``--graph``, export graphml / gexf /
json) and stats / distance / distance-matrix are outside the GPU GFA->CSR path.
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

from . import __version__
from .api import convert_format, export_edge_list, parse_gfa, parse_gfa_names, save_matrix, save_node_map_native


def _parser() -> argparse.ArgumentParser:
    parser = argparse.ArgumentParser(prog="gfa2network")
    parser.add_argument("--version", action="version", version=f"gfa2network-amd {__version__}")
    parser.add_argument("--raw-bytes-id", action="store_true", help="Use raw bytes for node identifiers (legacy)")
    parser.add_argument("--max-dense-gb", type=float, default=5.0, help="Abort dense matrix saves over N GB (default 5)")
    parser.add_argument("--max-tag-mb", type=float, default=100.0, help="Warn when stored tags exceed N MB (default 100)")
    parser.add_argument("--device", type=int, default=0, help="HIP device ordinal (GPU build option)")
    sub = parser.add_subparsers(dest="cmd", required=True)

    p = sub.add_parser("convert", help="Convert GFA to a sparse adjacency matrix")
    p.add_argument("gfa", help="Input *.gfa* file or - for stdin")
    p.add_argument("--backend", choices=["networkx", "igraph"], default="networkx", help="Graph backend to use")
    g = p.add_mutually_exclusive_group()
    g.add_argument("--directed", dest="directed", action="store_true", default=True, help="Treat graph as directed")
    g.add_argument("--undirected", dest="directed", action="store_false", help="Treat graph as undirected")
    p.add_argument("--graph", action="store_true", help="Build a NetworkX object (not supported on the GPU path)")
    p.add_argument("--matrix", metavar="PATH", help="Write adjacency matrix to PATH (.npz|.npy|.csv)")
    p.add_argument("--save-matrix", dest="matrix", metavar="PATH", help=argparse.SUPPRESS)
    p.add_argument("--matrix-format", default="csr", help="Sparse format for .npz (csr|csc|coo|dok)")
    p.add_argument("--dtype", choices=["bool", "int8", "int32", "float32", "float64"], default="float64",
                   help="Data type for adjacency matrix")
    p.add_argument("--asymmetric", action="store_true", help="Do not mirror upper triangle")
    p.add_argument("--no-node-map", action="store_true", help="Do not write <matrix>.nodes.tsv sidecar")
    p.add_argument("--weight-tag")
    p.add_argument("--store-seq", action="store_true")
    p.add_argument("--store-tags", action="store_true")
    p.add_argument("--split-on-alignment", action="store_true", help="Split segments at alignment boundaries")
    p.add_argument("--strip-orientation", action="store_true", help="Strip +/- from IDs (v0.1 behaviour)")
    p.add_argument("--bidirected", action="store_true", help="Use bidirected representation")
    p.add_argument("--keep-directed-bidir", action="store_true", help="Keep original directed bidirected behaviour")
    p.add_argument("--verbose", action="store_true")
    p.add_argument("-o", "--output", metavar="PATH", help="Write graph pickle to PATH (not supported)")
    p_exp = sub.add_parser("export", help="Stream edges in simple formats")  # cli.py:137-149
    p_exp.add_argument("gfa")
    p_exp.add_argument("--format", default="edge-list", choices=["edge-list", "graphml", "gexf", "json"])
    p_exp.add_argument("--bidirected", action="store_true")
    p_exp.add_argument("--keep-directed-bidir", action="store_true",
                       help="Keep original directed bidirected behaviour")
    p_exp.add_argument("--output", help="Output path", default="-")
    for name in ("stats", "distance", "distance-matrix"):
        sp_ = sub.add_parser(name, help="(outside the GPU GFA->CSR path)")
        sp_.add_argument("rest", nargs=argparse.REMAINDER)
    return parser


def main(argv: list[str] | None = None) -> None:
    parser = _parser()
    args = parser.parse_args(argv)
    if args.cmd == "export":
        if args.format != "edge-list":
            parser.error(f"export --format {args.format} builds a NetworkX graph, outside the GPU GFA->CSR path")
        export_edge_list(args.gfa, args.output, bidirected=args.bidirected, device=args.device)
        return
    if args.cmd != "convert":
        parser.error(f"'{args.cmd}' is outside the GPU GFA->CSR path; use the reference gfa2network for it")
    if not args.graph and not args.matrix:
        parser.error("convert requires --graph or --matrix")
    if args.graph:
        parser.error("--graph (NetworkX / igraph objects) is outside the GPU GFA->CSR path")
    print(f"Using backend: {args.backend}")
    want_nodes = not args.no_node_map
    kw = dict(
        directed=args.directed,
        weight_tag=args.weight_tag,
        store_seq=args.store_seq,
        store_tags=args.store_tags,
        strip_orientation=args.strip_orientation,
        verbose=args.verbose,
        bidirected=args.bidirected,
        keep_directed_bidir=args.keep_directed_bidir,
        backend=args.backend,
        dtype=args.dtype,
        asymmetric=args.asymmetric,
        raw_bytes_id=args.raw_bytes_id,
        max_tag_mb=args.max_tag_mb,
        split_on_alignment=args.split_on_alignment,
        device=args.device,
    )
    if want_nodes:  # names stay a blob: the sidecar is written natively (no Python list)
        A, blob, offs = parse_gfa_names(args.gfa, **kw)
    else:
        A = parse_gfa(args.gfa, build_graph=False, build_matrix=True, return_node_list=False, **kw)
    A = convert_format(A, args.matrix_format, verbose=args.verbose)
    try:
        save_matrix(A, Path(args.matrix), verbose=args.verbose, max_dense_gb=args.max_dense_gb)
    except MemoryError as exc:
        raise SystemExit(str(exc)) from exc
    if want_nodes:
        save_node_map_native(blob, offs, Path(str(args.matrix) + ".nodes.tsv"), args.raw_bytes_id)


if __name__ == "__main__":  # pragma: no cover
    main(sys.argv[1:])
