"""CPU restatement of the reference's GFA -> matrix path.

TEST INFRASTRUCTURE ONLY (the checker): tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may use it; the gfa2network_amd product never imports it.
"""
