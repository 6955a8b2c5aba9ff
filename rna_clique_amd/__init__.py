"""MI355X-native pairwise-distance engine for RNA-clique.

Replaces the reference's all-pairs BLAST+ alignment, reciprocal-best-hit gene
matches tables, gene matches graph and SampleSimilarity distance matrix with
hand-written HIP kernels (librcgpu.so, include/rcgpu.h), behind the reference's
Python API (rna_clique(), SampleSimilarity, HomologFinder).
"""
__version__ = "0.1.0"
