"""GPU: the sharded path at BASELINE configuration scale.

* C4 (64 x 50 000, BASELINE configs[3]) cut into the 8 shards of an 8-GPU
  run, the shard engines run one after another on the one GPU of the box,
  each holding only its own pairs' samples and closed after exporting its
  edges; the concatenated edges imported into a graph-only engine give the
  unsharded run's distances, sums, edges and ideal nodes bit for bit, and
  every shard's tables equal the unsharded tables of the same pairs
  (find_all_pairs.py:224-228 runs the pairs independently).
* C5 (128 x 100 000, 200 bp - 5 kb, BASELINE configs[4]): the rank of 8 with
  the largest modelled HBM footprint alone on the GPU with only its ~60 of 128
  samples generated and resident, cut into alignment tiles: whole-shard
  properties, determinism, four owned pairs bit-exact vs the oracle, and the
  measured HBM use against distributed.hbm_footprint's model.
"""
import json
import os

import numpy as np
import pytest

from oracle.parity import check_pairs

pytestmark = pytest.mark.gpu


def _edge_digest(rec):
    """(count, order-independent 64-bit digests) of fixed-size records, an
    (n, record bytes) uint8 array (records are unique, so equal digests mean
    equal sets up to hash collisions)."""
    n, rs = rec.shape
    if rs % 8:
        rec = np.concatenate([rec, np.zeros((n, 8 - rs % 8), np.uint8)], axis=1)
    u = np.ascontiguousarray(rec).view(np.uint64)
    h = np.zeros(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        for c in range(u.shape[1]):
            x = (u[:, c] + np.uint64(0x9E3779B97F4A7C15) * np.uint64(c + 1)) ^ h
            x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            h = x ^ (x >> np.uint64(31))
        return n, int(h.sum(dtype=np.uint64)), int(np.bitwise_xor.reduce(h)) if n else 0


def _records(arr, rs):
    return np.ascontiguousarray(arr).view(np.uint8).reshape(-1, rs)


class _heartbeat:
    """Prints a line every 30 s while a long step runs (GPU runs are killed
    after 3 minutes without output; pytest -s shows these), for at most
    10 minutes: a step that hangs still goes silent."""

    def __init__(self, what):
        import threading
        self.what, self.stop = what, threading.Event()
        self.t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        import time
        t0 = time.time()
        while not self.stop.wait(30) and time.time() - t0 < 600:
            print(f"  ... {self.what}: {time.time() - t0:.0f} s", flush=True)

    def __enter__(self):
        print(f"  {self.what}", flush=True)
        self.t.start()
        return self

    def __exit__(self, *a):
        self.stop.set()
        self.t.join()


def _record(name, obj):
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.path.join("gpurun_out", f"{name}.json"), "w") as f:
        json.dump(obj, f, indent=1)


@pytest.mark.heartbeat(400)
def test_C4_eight_shards_match_unsharded(native):
    from rna_clique_amd import distributed
    from rna_clique_amd.engine import Engine
    from rna_clique_amd.simulate import CONFIGS, simulate
    with _heartbeat("C4: simulate"):
        samples, _ = simulate(**CONFIGS["C4"])
    N, S = len(samples), 8
    bases = [int(s.tx_offsets[-1]) for s in samples]
    ref = Engine(device=0)
    for s in samples:
        ref.add_sample(s.name, s.seq, s.tx_offsets, s.gene, s.iso)
    ref.run()
    want = {"distance": ref.distance()[1], "sums": ref.pair_sums(), "usums": ref.pair_sums(unfiltered=True),
            "edges": _edge_digest(_records(ref.edges(), 16)), "ideal": sorted(zip(*ref.ideal_nodes())), "stats": ref.stats()}
    order, first = distributed.plan_pairs(bases, S)
    # six pairs of every shard: first, last and four spread between
    check = {}
    for r in range(S):
        own = order[int(first[r]):int(first[r + 1])]
        for k in sorted({0, len(own) - 1, *(len(own) * j // 5 for j in range(1, 5))}):
            check[own[k]] = ref.pair_rows(*own[k]).tobytes()
    ref.close()
    parts, resident = [], []
    for r in range(S):
        print(f"  C4 shard {r}", flush=True)
        need = distributed.needed_samples(bases, S, r)
        resident.append(len(need))
        e = Engine(device=0, shard_rank=r, shard_count=S)
        for i, s in enumerate(samples):
            e.add_sample(s.name, s.seq if i in need else None, s.tx_offsets, s.gene, s.iso)
        e.align()
        e.finish()
        assert e.owned_pairs() == order[int(first[r]):int(first[r + 1])]
        for p in e.owned_pairs():
            if p in check:
                assert e.pair_rows(*p).tobytes() == check[p], (r, p)
        parts.append(e.export_edges())
        e.close()
    assert max(resident) < N
    # graph-only (a fresh engine given every shard's edges, as each rank is
    # after the all-gather; the same shard plan, hence the same pair numbering)
    g = Engine(device=0, shard_rank=0, shard_count=S)
    for s in samples:
        g.add_sample(s.name, None, s.tx_offsets, s.gene, s.iso)
    g.import_edges(np.concatenate(parts))
    assert np.array_equal(g.distance()[1], want["distance"])
    for got, exp in ((g.pair_sums(), want["sums"]), (g.pair_sums(unfiltered=True), want["usums"])):
        assert np.array_equal(got[0], exp[0]) and np.array_equal(got[1], exp[1])
    assert _edge_digest(_records(g.edges(), 16)) == want["edges"]
    assert sorted(zip(*g.ideal_nodes())) == want["ideal"]
    st = g.stats()
    for k in ("edges", "components", "ideal_components", "ideal_nodes", "sample_count"):
        assert st[k] == want["stats"][k], k
    _record("C4_shards", {"resident_samples": resident, "edges": st["edges"], "checked_pairs": len(check)})
    g.close()


@pytest.mark.heartbeat(300)
def test_graph_phase_at_C5_size(native):
    """The graph phase alone at C5's size (build_graph.py:40-68,
    filtered_distance.py:30-39): 128 samples x 100 000 genes (12.8 M nodes)
    and every pair's edge of every gene family -- 8.1 x 10^8 edge records,
    16 GB, as a graph-only engine holds them after the 8-rank all-gather.
    Families are 128-cliques (ideal) except: f % 10 == 0 misses its (0, 1)
    edge (not complete), f % 10 == 5 gains an edge to family f + 1 (one
    component of 256 nodes). Components, ideal components and nodes, the
    filtered and unfiltered sums of every pair and the matrix are known in
    closed form."""
    from rna_clique_amd.engine import Engine
    N, G = 128, 100_000
    rs = Engine.edge_record_size()
    dt = np.dtype([("a", np.uint32), ("b", np.uint32), ("pair", np.uint32), ("nident", np.int32),
                   ("den", np.int32)])
    assert dt.itemsize == rs
    f = np.arange(G, dtype=np.uint32)
    nid = (1000 + f % 7).astype(np.int32)
    dn = (1100 + f % 3).astype(np.int32)
    drop = f % 10 == 0
    extra = np.nonzero(f % 10 == 5)[0].astype(np.uint32)
    n_pairs = N * (N - 1) // 2
    n = n_pairs * G - int(drop.sum()) + len(extra)
    with _heartbeat(f"graph at C5 size: {n} edge records"):
        rec = np.zeros(n, dtype=dt)
        w = 0
        keep01 = f[~drop]
        for b in range(1, N):
            for a in range(b):
                p = b * (b - 1) // 2 + a   # a single shard's pair order: subject-major
                ff = keep01 if (a, b) == (0, 1) else f
                k = len(ff)
                sl = rec[w:w + k]
                sl["a"] = a * G + ff
                sl["b"] = b * G + ff
                sl["pair"] = p
                sl["nident"] = nid[ff]
                sl["den"] = dn[ff]
                w += k
        sl = rec[w:]
        sl["a"] = extra            # sample 0, family f
        sl["b"] = G + extra + 1    # sample 1, family f + 1
        sl["pair"] = 0
        sl["nident"] = 7
        sl["den"] = 9
        assert w + len(extra) == n
        g = Engine(device=0)
        for s in range(N):
            g.add_sample(f"S{s:03d}", None, np.arange(G + 1, dtype=np.uint64) * 1000,
                         np.arange(1, G + 1, dtype=np.int32), np.ones(G, dtype=np.int32))
        t0 = __import__("time").perf_counter()
        g.import_edges(rec.view(np.uint8))
        t_import = __import__("time").perf_counter() - t0
        del rec, sl
        st = g.stats()
        ideal = (f % 10 != 0) & (f % 10 != 5) & (f % 10 != 6)
        assert st["edges"] == n
        assert st["nodes"] == N * G
        assert st["components"] == G - len(extra)
        assert st["ideal_components"] == int(ideal.sum())
        assert st["ideal_nodes"] == int(ideal.sum()) * N
        assert st["sample_count"] == N
        num, den = g.pair_sums()
        unum, uden = g.pair_sums(unfiltered=True)
        want_n, want_d = int(nid[ideal].astype(np.int64).sum()), int(dn[ideal].astype(np.int64).sum())
        off = ~np.eye(N, dtype=bool)
        assert np.all(num[off] == want_n) and np.all(den[off] == want_d)
        all_n, all_d = int(nid.astype(np.int64).sum()), int(dn.astype(np.int64).sum())
        u01 = (all_n - int(nid[drop].astype(np.int64).sum()) + 7 * len(extra),
               all_d - int(dn[drop].astype(np.int64).sum()) + 9 * len(extra))
        assert (int(unum[0, 1]), int(uden[0, 1])) == u01 == (int(unum[1, 0]), int(uden[1, 0]))
        m01 = np.zeros((N, N), dtype=bool)
        m01[0, 1] = m01[1, 0] = True
        assert np.all(unum[off & ~m01] == all_n) and np.all(uden[off & ~m01] == all_d)
        labels, mat = g.distance()
        assert labels == [f"S{s:03d}" for s in range(N)]
        want = np.full((N, N), (want_d - want_n) / want_d)
        np.fill_diagonal(want, 0.0)
        assert np.array_equal(mat, want)
        tm = g.timings()
        _record("graph_C5_size", {"edges": n, "import_s": t_import, "graph_ms": tm["graph_ms"],
                                  "reduce_ms": tm["reduce_ms"], "device_gb": tm["dev_bytes"] / 1e9})
        g.close()


@pytest.mark.heartbeat(600)
def test_C5_one_rank_shard(native):
    import torch
    from bench import shard_samples
    from rna_clique_amd import distributed
    from rna_clique_amd.engine import Engine
    from rna_clique_amd.simulate import CONFIGS, simulate
    S = 8
    # the rank with the largest modelled footprint (from the metadata alone)
    meta, _ = simulate(only=[], **CONFIGS["C5"])
    bases = [int(s.tx_offsets[-1]) for s in meta]
    genes = [len(np.unique(s.gene)) for s in meta]
    del meta
    model = distributed.hbm_footprint(bases, genes, S)
    R = int(np.argmax(model))
    with _heartbeat(f"C5: generate rank {R}'s samples"):
        samples, need, (order, first) = shard_samples("C5", S, R)
    assert len(need) < len(samples) and all((samples[i].seq is None) == (i not in need) for i in range(128))
    free0, _ = torch.cuda.mem_get_info(0)
    native.rc_dev_peak_reset()   # this engine's own peak, not an earlier test's
    eng = Engine(device=0, shard_rank=R, shard_count=S)
    for i, s in enumerate(samples):
        eng.add_sample(s.name, s.seq if i in need else None, s.tx_offsets, s.gene, s.iso)
    with _heartbeat("C5: align + finish"):
        eng.align()
        eng.finish()
    tm = eng.timings()
    print(f"  C5 rank {R}: {tm['tiles']:.0f} tiles, {tm['total_ms']:.0f} ms", flush=True)
    assert tm["tiles"] > 1
    free1, _ = torch.cuda.mem_get_info(0)
    own = eng.owned_pairs()
    assert own == order[int(first[R]):int(first[R + 1])] and len(own) > 900
    edges = eng.export_edges()
    # determinism: the rank's whole pass again gives the same edges
    eng.align()
    eng.finish()
    again = eng.export_edges()
    rs = Engine.edge_record_size()
    assert _edge_digest(_records(again, rs)) == _edge_digest(_records(edges, rs))
    eng.import_edges(edges)   # the graph phase over this rank's own edges
    st = eng.stats()
    num, den = eng.pair_sums()
    unum, uden = eng.pair_sums(unfiltered=True)
    assert np.array_equal(unum, unum.T) and np.array_equal(uden, uden.T)
    for a, b in own:
        assert 0 < unum[a, b] <= uden[a, b]
        assert 0 <= num[a, b] <= unum[a, b] and 0 <= den[a, b] <= uden[a, b]
    peak = eng.timings()["dev_peak_bytes"]
    _record("C5_shard", {"rank": R, "pairs": len(own), "resident_samples": len(need),
                         "device_used_gb": (free0 - free1) / 1e9, "engine_peak_gb": peak / 1e9,
                         "hbm_model_gb": model[R] / 1e9, "timings": tm, "stats": st})
    # the model is what planning relies on: the engine's own peak within 20 %
    assert 0.8 * model[R] < peak < 1.2 * model[R]
    # four owned pairs against the oracle (both directed searches, table,
    # sums), spread over the rank's rectangle
    picks = [own[0], own[len(own) // 4], own[len(own) // 2], own[(3 * len(own)) // 4]]
    with _heartbeat(f"C5: oracle on pairs {picks}"):
        msgs = check_pairs(eng, samples, picks)
    assert not msgs, "\n".join(msgs[:10])
    eng.close()
