"""Host-only timing of the native graph.pkl writer on a synthetic C5-shaped
graph (no GPU): S samples x G genes, every sample pair's table in
combinations order matching gene i to gene i (an ideal ortholog set, as C5s
nearly is), so the edge count is C(S, 2) x G (C5: 128 x 100 000 -> 813 M;
--genes 25000 is a quarter of it). RC_OUT_TIMING=1 prints the writer's phases.

  python scripts/pickle_bench.py --samples 128 --genes 25000 --out /tmp/g.pkl
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=128)
    ap.add_argument("--genes", type=int, default=25000)
    ap.add_argument("--out", default="/tmp/rc_pickle_bench.pkl")
    ap.add_argument("--check", action="store_true", help="pickle.load it back and compare with build_graph (small sizes)")
    a = ap.parse_args()
    os.environ.setdefault("RC_OUT_TIMING", "1")
    import ctypes
    from rna_clique_amd import _native
    L = _native.lib()
    h = ctypes.c_void_p()
    _native.check(L.rc_graph_pickle_begin(ctypes.byref(h)))
    rng = np.random.default_rng(5)
    genes = np.arange(a.genes, dtype=np.int64)
    t0 = time.perf_counter()
    tabs = []
    for s1 in range(a.samples):
        for s2 in range(s1 + 1, a.samples):
            q = rng.permutation(genes) if a.check else genes
            tabs.append((s2, s1, q, q))
            _native.check(L.rc_graph_pickle_add(h, s2, s1, q.ctypes.data, q.ctypes.data, len(q)))
    t1 = time.perf_counter()
    names = [f"/data/sample_{i:03d}/top.fasta".encode() for i in range(a.samples)]
    arr = (ctypes.c_char_p * len(names))(*names)
    _native.check(L.rc_graph_pickle_write(h, a.out.encode(), len(names), arr))
    t2 = time.perf_counter()
    L.rc_graph_pickle_free(h)
    sz = os.path.getsize(a.out)
    print(f"edges {len(tabs) * a.genes}  add {t1 - t0:.2f} s  write {t2 - t1:.2f} s  "
          f"{sz / 1e9:.2f} GB  {sz / 1e9 / (t2 - t1):.2f} GB/s", flush=True)
    if a.check:
        import pickle
        import networkx as nx  # noqa: F401
        g = pickle.load(open(a.out, "rb"))
        print("nodes", g.number_of_nodes(), "edges", g.number_of_edges())
    os.remove(a.out)


if __name__ == "__main__":
    main()
