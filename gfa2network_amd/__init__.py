"""gfa2network_amd — MI355X-native GFA -> CSR ingest for the gfa2network call surface.

Drop-in for the reference's matrix path: ``parse_gfa(..., build_matrix=True)``,
``convert_format`` and the ``convert --matrix`` CLI (sclipman/gfa2network
gfa2network/__init__.py:3-14).  The work runs in hand-written gfx950 kernels behind the
C-ABI in include/g2n.h (libg2n.so, loaded with ctypes).
"""
from .api import convert_format, export_edge_list, parse_gfa, parse_gfa_sharded

__version__ = "0.3.0"

__all__ = ["parse_gfa", "parse_gfa_sharded", "convert_format", "export_edge_list", "__version__"]
