"""The whole C5 job (BASELINE configs[4]: 128 samples x 100 000 genes, 200 bp -
5 kb, 8 x MI355X) emulated on one GPU, end to end to the distance matrix.

An 8-GPU run is one rank per GPU: rank r aligns the pairs of its rectangle of
the pair triangle (rc_plan_pairs) holding only its samples, runs top-N /
reciprocal best hits for them, and all-gathers its graph edges; every rank
then runs the graph phase over all of them (distributed.sharded_run). Here
the 8 ranks run one after another on the one GPU of the box -- each engine
holds only its rank's samples, exports its edges and is closed -- and the
concatenated edges are imported into a graph-only engine (as every rank is
after the all-gather), which gives the C5 matrix (build_graph.py:40-68,
filtered_distance.py:30-39, rna_clique.py:171-177).

Checks (any failure: exit 1):
* every rank's owned pairs are its plan's; per rank, --oracle-pairs pairs (spread over
  its rectangle) bit-exact against the C oracle (both directed searches,
  the pair's table and unfiltered sums; oracle/parity.compare_pair_fast), the
  oracle running on the host beside the next ranks' GPU work;
* the graph engine's unfiltered sums of every pair equal the owning rank's
  own (a pair's table depends on nothing else);
* the matrix is symmetric, hollow, in [0, 1]; NJ on it gives the simulated
  128-taxon tree (Robinson-Foulds 0, the reference's verify_distances.py
  check);
* HBM: each rank's engine peak against distributed.hbm_footprint's model,
  the graph engine's device bytes against its own model.

Outputs (--outputs DIR): each rank writes the od2 gene matches tables of the
pairs it owns (find_all_pairs.write_pair_tables: pandas table-format HDF5,
find_all_pairs.py:87,90-117) and the graph engine -- every rank after the
exchange, rank 0 writing -- graph.pkl (build_graph over all pairs' edges,
filtering_step.py:157-159), timed, with their bytes; each rank's files are
deleted once measured (C5's tables are ~2 x 10^8 rows per rank).

Writes one JSON (per-rank time table, projection of 8-GPU pairs/s from the
slowest rank, checks) to --out; prints progress lines meanwhile.

    python scripts/c5_full.py [--config C5] [--shards 8] [--oracle-pairs 2] [--outputs DIR]
                              [--out gpurun_out/c5_full.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


class Heartbeat:
    """A progress line every 30 s while a step runs (GPU runs are killed after
    3 minutes without output)."""

    def __init__(self, what):
        self.what, self.stop = what, threading.Event()
        self.t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        t0 = time.time()
        while not self.stop.wait(30):
            print(f"  ... {self.what}: {time.time() - t0:.0f} s", flush=True)

    def __enter__(self):
        print(f"{self.what}", flush=True)
        self.t.start()
        return self

    def __exit__(self, *a):
        self.stop.set()
        self.t.join()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C5")
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--oracle-pairs", type=int, default=2, help="pairs per rank checked against the oracle")
    ap.add_argument("--out", default="gpurun_out/c5_full.json")
    ap.add_argument("--outputs", default=None, help="scratch directory: write (and time) every rank's od2 "
                                                     "tables and graph.pkl there")
    args = ap.parse_args()
    # torch's HIP runtime first, then librcgpu.so (bench.shard_emulation)
    import torch
    torch.cuda.init()
    import numpy as np
    from concurrent.futures import ThreadPoolExecutor
    from rna_clique_amd import distributed
    from rna_clique_amd import _native
    from rna_clique_amd.engine import Engine
    from rna_clique_amd.simulate import CONFIGS, simulate
    from oracle.align import OracleDB
    from oracle.parity import capture_pairs, compare_pair_fast as compare_pair, oracle_threads
    from treecheck import nj_splits, robinson_foulds, tree_splits

    S = args.shards
    cfg = dict(CONFIGS[args.config])
    t_all = time.perf_counter()
    # C5 has per-node random streams (a rank's samples alone); other configs
    # (quick rehearsals) are generated whole once
    whole = None
    if cfg.get("node_rng"):
        meta, tree = simulate(only=[], **cfg)
    else:
        whole, tree = simulate(**cfg)
        meta = whole
    N = len(meta)
    bases = [int(s.tx_offsets[-1]) for s in meta]
    genes = [len(np.unique(s.gene)) for s in meta]
    order, first = distributed.plan_pairs(bases, S)
    model = distributed.hbm_footprint(bases, genes, S)
    pool = ThreadPoolExecutor(max(1, oracle_threads()))
    pending = []   # (rank, a, b, samples kept for the oracle, db, futures, capture)
    ranks, parts, own_usums = [], [], {}
    failures = []
    for r in range(S):
        need = distributed.needed_samples(bases, S, r)
        with Heartbeat(f"rank {r}/{S}: generate {len(need)} samples"):
            t0 = time.perf_counter()
            samples = simulate(only=sorted(need), **cfg)[0] if whole is None else whole
            t_gen = time.perf_counter() - t0
        _native.lib().rc_dev_peak_reset()   # each rank's own engine peak (ranks run one after another)
        eng = Engine(device=0, shard_rank=r, shard_count=S)
        for i, s in enumerate(samples):
            eng.add_sample(s.name, s.seq if i in need else None, s.tx_offsets, s.gene, s.iso)
        eng.upload()
        with Heartbeat(f"rank {r}/{S}: align + finish"):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.align()
            t1 = time.perf_counter()
            eng.finish()
            t2 = time.perf_counter()
        tm = eng.timings()
        own = eng.owned_pairs()
        edges = eng.export_edges()
        parts.append(edges)
        # the graph phase over the rank's own edges: its unfiltered sums (and
        # the picked pairs' captures) -- a pair's table depends on nothing else
        t3 = time.perf_counter()
        eng.import_edges(edges)
        t_own_graph = time.perf_counter() - t3
        unum, uden = eng.pair_sums(unfiltered=True)
        for a, b in own:
            own_usums[(a, b)] = (int(unum[a, b]), int(uden[a, b]))
        picks = sorted({own[(i * len(own)) // args.oracle_pairs] for i in range(args.oracle_pairs)}) if own else []
        cap = capture_pairs(eng, picks)
        outw = None
        if args.outputs:
            # this rank's od2 tables (the pairs it owns), then deleted
            import shutil
            from rna_clique_amd.find_all_pairs import write_pair_tables
            d = os.path.join(args.outputs, f"od2_r{r}")
            with Heartbeat(f"rank {r}/{S}: od2 tables"):
                t0w = time.perf_counter()
                paths = write_pair_tables(eng, [s.name for s in samples], d, lambda x: x, "h5", 16)
                tw = time.perf_counter() - t0w
            nbytes = sum(os.path.getsize(pth) for pth in paths.values())
            outw = {"tables": len(paths), "tables_s": round(tw, 2), "tables_gb": round(nbytes / 1e9, 2)}
            shutil.rmtree(d, ignore_errors=True)
        if own != order[int(first[r]):int(first[r + 1])]:
            failures.append(f"rank {r}: owned pairs differ from the plan")
        st = eng.stats()
        row = {"rank": r, "pairs": len(own), "resident_samples": len(need),
               "resident_gbp": round(sum(bases[i] for i in need) / 1e9, 3),
               "gen_s": round(t_gen, 1), "align_s": round(t1 - t0, 3), "finish_s": round(t2 - t1, 3),
               "rank_s": round(t2 - t0, 3), "own_graph_s": round(t_own_graph, 3),
               "tiles": tm["tiles"], "index_ms": round(tm["index_ms"], 1), "dust_ms": round(tm["dust_ms"], 1),
               "seed_kernel_ms": round(tm["seed_kernel_ms"], 1), "align_kernel_ms": round(tm["align_kernel_ms"], 1),
               "rbh_ms": round(tm["rbh_ms"], 1), "ext_steps": tm["ext_steps"], "ext_wide": tm["ext_wide"],
               "ext_deferred": tm["ext_deferred"], "candidates": st["candidates"], "hsps": st["hsps"],
               "edges": int(len(edges) // Engine.edge_record_size()),
               "engine_peak_gb": round(tm["dev_peak_bytes"] / 1e9, 2), "hbm_model_gb": round(model[r] / 1e9, 2),
               "picks": picks, "outputs": dict(outw, rows=int(st["table_rows"])) if outw else None}
        ranks.append(row)
        print(json.dumps(row), flush=True)
        eng.close()
        del eng
        # the oracle for this rank's picks runs on the host beside the next
        # ranks (the C oracle releases the GIL); only the picks' samples stay
        for a, b in picks:
            db = OracleDB([samples[a], samples[b]])
            futs = {qs: pool.submit(db.align, qs[0], qs[1], 28, 108, 1e-99, False, cap["dust"])
                    for qs in ((0, 1), (1, 0))}
            pending.append((r, a, b, {a: samples[a], b: samples[b]}, db, futs, cap))
        del samples
    # graph-only engine: every rank's edges, as each rank holds them after the all-gather
    with Heartbeat(f"graph phase: {sum(x['edges'] for x in ranks)} edges of {S} ranks"):
        allrec = np.concatenate(parts)
        del parts
        _native.lib().rc_dev_peak_reset()
        g = Engine(device=0, shard_rank=0, shard_count=S)
        for s in meta:
            g.add_sample(s.name, None, s.tx_offsets, s.gene, s.iso)
        t0 = time.perf_counter()
        g.import_edges(allrec)
        t_graph = time.perf_counter() - t0
        n_edges = len(allrec) // Engine.edge_record_size()
        del allrec
        gst = g.stats()
        print(json.dumps({"graph_stats": gst}), flush=True)
        from rna_clique_amd._native import NativeError
        try:
            labels, mat = g.distance()
        except NativeError as ex:
            # a pair without ideal rows: the reference's NoIdealComponentsError
            # (filtered_distance.py:242-247); consistent only if no ideal
            # component exists at all (an ideal clique spans every pair)
            print(f"distance: {ex}", flush=True)
            labels, mat = None, None
        gtm = g.timings()
        graph_out = None
        t_matrix = None
        if args.outputs and mat is not None:
            # matrix.h5 (rank 0, as soon as the distances exist: rna_clique.py)
            from rna_clique_amd.h5 import write_matrix
            from rna_clique_amd.similarity import SampleSimilarity
            mp = os.path.join(args.outputs, "matrix.h5")
            t0w = time.perf_counter()
            write_matrix(SampleSimilarity.from_engine(g).get_dissimilarity_df(), mp)
            t_matrix = time.perf_counter() - t0w
            os.remove(mp)
        if args.outputs:
            # graph.pkl from the exchanged edges (rank 0 writes it), then deleted
            from rna_clique_amd.similarity import SampleSimilarity
            gp = os.path.join(args.outputs, "graph.pkl")
            t0w = time.perf_counter()
            SampleSimilarity.from_engine(g).write_graph(gp)
            graph_out = {"graph_pkl_s": round(time.perf_counter() - t0w, 2),
                         "graph_pkl_gb": round(os.path.getsize(gp) / 1e9, 2)}
            os.remove(gp)
            print(json.dumps({"graph_pkl": graph_out}), flush=True)
        unum, uden = g.pair_sums(unfiltered=True)
        num, den = g.pair_sums()
        g_bytes = gtm["dev_bytes"]
        g.close()
    bad_sums = [(a, b) for (a, b), v in own_usums.items() if (int(unum[a, b]), int(uden[a, b])) != v]
    if bad_sums:
        failures.append(f"unfiltered sums differ from the owning rank's for {len(bad_sums)} pairs, e.g. {bad_sums[:3]}")
    off = ~np.eye(N, dtype=bool)
    rf = None
    if mat is None:
        if gst["ideal_components"] != 0 or np.any(den[off] != 0):
            failures.append("NoIdealComponentsError although ideal components exist")
    else:
        if not (np.array_equal(mat, mat.T) and np.all(np.diag(mat) == 0) and np.all((mat >= 0) & (mat <= 1))):
            failures.append("matrix not symmetric / hollow / in [0, 1]")
        if not np.all(den[off] > 0):
            failures.append("a pair with no ideal rows")
        parent, _, leaves = tree
        truth = tree_splits(parent, leaves, {leaf: meta[i].name for i, leaf in enumerate(leaves)})
        rf = robinson_foulds(nj_splits(mat, list(labels)), truth)
        if rf != 0:
            failures.append(f"NJ tree of the matrix: Robinson-Foulds {rf} vs the simulated tree")
    # graph engine model: edge records + per-gene union-find / ideal arrays + pair sums
    n_genes = sum(genes)
    g_model = n_edges * Engine.edge_record_size() + n_genes * 17 + len(order) * 32
    with Heartbeat(f"oracle: {len(pending)} pairs"):
        checked = []
        for r, a, b, smp, db, futs, cap in pending:
            ora = {qs: f.result() for qs, f in futs.items()}
            msgs = compare_pair(cap, smp, a, b, db, ora)
            checked.append({"rank": r, "pair": [a, b], "hsps": int(sum(len(v) for v in ora.values())),
                            "ok": not msgs})
            failures += msgs[:5]
    pool.shutdown()
    slow = max(ranks, key=lambda x: x["rank_s"])
    out = {
        "config": args.config, "samples": N, "pairs": len(order), "shards": S,
        "ranks": ranks,
        "graph": {"edges": n_edges, "import_s": round(t_graph, 3), "stats": gst, "outputs": graph_out,
                  "device_gb": round(g_bytes / 1e9, 2), "model_gb": round(g_model / 1e9, 2),
                  "graph_ms": round(gtm["graph_ms"], 1), "reduce_ms": round(gtm["reduce_ms"], 1)},
        "matrix": None if mat is None else {
            "labels": labels, "min_offdiag": float(mat[off].min()), "max": float(mat.max()),
            "rf_vs_simulated_tree": rf},
        "no_ideal_components": mat is None,
        "unfiltered_pairs_with_rows": int(np.count_nonzero(uden[off]) // 2),
        "oracle_pairs": checked,
        # one GPU per rank: the job takes the slowest rank's align + finish,
        # then the exchange and the graph phase (measured here on one GPU)
        "projection_8gpu": {"slowest_rank": slow["rank"], "slowest_rank_s": slow["rank_s"],
                            "graph_phase_s": round(t_graph, 3),
                            "pairs_per_s_align_only": round(len(order) / slow["rank_s"], 1),
                            "pairs_per_s_with_graph": round(len(order) / (slow["rank_s"] + t_graph), 1),
                            "sum_rank_s": round(sum(x["rank_s"] for x in ranks), 3),
                            "balance": round(sum(x["rank_s"] for x in ranks) / (S * slow["rank_s"]), 3)},
        # the whole job's wall-clock on 8 GPUs from the parts measured here:
        # the ranks align in parallel and meet at the edge exchange (the
        # slowest rank), every rank runs the graph phase (here: from host
        # memory, 806.8 M records H2D included -- on 8 GPUs they arrive over
        # RCCL device to device), then rank 0 writes matrix.h5, its tables and
        # graph.pkl while the other ranks write their own tables
        "end_to_end_8gpu": None if t_matrix is None or graph_out is None else {
            "to_matrix_h5_s": round(slow["rank_s"] + t_graph + t_matrix, 2),
            "to_every_output_s": round(slow["rank_s"] + t_graph + max(
                t_matrix + ranks[0]["outputs"]["tables_s"] + graph_out["graph_pkl_s"],
                max(x["outputs"]["tables_s"] for x in ranks)), 2),
            "parts_s": {"slowest_rank_align_finish": slow["rank_s"], "graph_phase_from_host": round(t_graph, 3),
                        "matrix_h5": round(t_matrix, 3), "rank0_tables": ranks[0]["outputs"]["tables_s"],
                        "graph_pkl": graph_out["graph_pkl_s"],
                        "slowest_rank_tables": max(x["outputs"]["tables_s"] for x in ranks)}},
        "wall_s": round(time.perf_counter() - t_all, 1),
        "failures": failures,
    }
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in ("projection_8gpu", "end_to_end_8gpu", "wall_s", "failures")}), flush=True)
    print(json.dumps(out["graph"]), flush=True)
    return 1 if failures else 0


if __name__ == "__main__":
    sys.exit(main())
