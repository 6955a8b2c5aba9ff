"""graph.pkl (and matrix.h5) from a C5-shaped edge set on one GPU: a
graph-only engine with S samples x G genes (metadata only, no bases), every
sample pair matching gene i to gene i (C5s is nearly that: 806.8 M edges of
C(128, 2) x 100 000 = 812.8 M), the records imported as an all-gather leaves
them, then the graph phase, matrix.h5 and graph.pkl, each timed
(RC_OUT_TIMING=1: the writer's phases on stderr).

  python scripts/graph_out_bench.py --samples 128 --genes 100000 --out-dir /tmp/rc_gout
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=128)
    ap.add_argument("--genes", type=int, default=100000)
    ap.add_argument("--out-dir", default="/tmp/rc_gout")
    ap.add_argument("--json", default=None)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--keep", action="store_true")
    a = ap.parse_args()
    os.environ.setdefault("RC_OUT_TIMING", "1")
    from rna_clique_amd import _native
    from rna_clique_amd.engine import Engine
    from rna_clique_amd.h5 import write_matrix
    from rna_clique_amd.similarity import SampleSimilarity
    S, G = a.samples, a.genes
    os.makedirs(a.out_dir, exist_ok=True)
    t0 = time.perf_counter()
    g = Engine(device=0)
    offs = np.arange(G + 1, dtype=np.uint64) * 1000
    gene = np.arange(G, dtype=np.int32)
    iso = np.zeros(G, dtype=np.int32)
    for s in range(S):
        g.add_sample(f"/data/sample_{s:03d}/top.fasta", None, offs, gene, iso)
    pairs = g.pair_order()
    rec = np.empty((len(pairs), G, 5), dtype=np.uint32)
    ar = np.arange(G, dtype=np.uint32)
    for p, (sa, sb) in enumerate(pairs):
        rec[p, :, 0] = sb * G + ar
        rec[p, :, 1] = sa * G + ar
        rec[p, :, 2] = p
        rec[p, :, 3] = 990
        rec[p, :, 4] = 1000
    rec = rec.reshape(-1).view(np.uint8)
    t1 = time.perf_counter()
    g.import_edges(rec)
    del rec
    t2 = time.perf_counter()
    sim = SampleSimilarity.from_engine(g)
    mpath = os.path.join(a.out_dir, "matrix.h5")
    write_matrix(sim.get_dissimilarity_df(), mpath)
    t3 = time.perf_counter()
    gpath = os.path.join(a.out_dir, "graph.pkl")
    _native.check(_native.lib().rc_write_graph(g._h, gpath.encode(), a.threads))
    t4 = time.perf_counter()
    out = {"samples": S, "genes": G, "edges": len(pairs) * G, "gen_s": round(t1 - t0, 2),
           "import_graph_s": round(t2 - t1, 3), "matrix_h5_s": round(t3 - t2, 3),
           "graph_pkl_s": round(t4 - t3, 3), "graph_pkl_gb": round(os.path.getsize(gpath) / 1e9, 3),
           "to_matrix_s": round(t3 - t1, 3), "to_every_output_s": round(t4 - t1, 3)}
    try:
        out["thp"] = open("/sys/kernel/mm/transparent_hugepage/enabled").read().strip()
    except OSError:
        pass
    print(json.dumps(out), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)
    if not a.keep:
        os.remove(gpath)
        os.remove(mpath)
    g.close()


if __name__ == "__main__":
    main()
