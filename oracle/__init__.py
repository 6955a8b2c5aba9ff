"""CPU oracles -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker. The product (rna_clique_amd,
librcgpu.so) never imports, links or executes anything here.
"""
