"""GPU: the drop-in API end to end, and the sharded (multi-GPU) path emulated
with several shard engines on one device. Checked against the CPU oracles and
against the unsharded engine, bit for bit."""
import heapq
import itertools
import os
import pickle
from collections import defaultdict

import numpy as np
import pandas as pd
import pytest

from oracle.parity import full_check

pytestmark = pytest.mark.gpu


def _load(eng, samples):
    for s in samples:
        eng.add_sample(s.name, s.seq, s.tx_offsets, s.gene, s.iso)
    return eng


@pytest.mark.parametrize("shards", [2, 3, 7])
def test_sharded_engines_match_unsharded(native, shards):
    from rna_clique_amd.engine import Engine
    from rna_clique_amd.simulate import simulate
    samples, _ = simulate(5, 120, seed=4, p_iso2=0.2, indel_rate=0.002)
    ref = _load(Engine(device=0), samples)
    ref.run()
    engines = [_load(Engine(device=0, shard_rank=r, shard_count=shards), samples)
               for r in range(shards)]
    owned = []
    for e in engines:
        e.align()
        e.finish()
        owned.append(range(*e.shard_pairs()))
    # the pair numbering is the shard plan's, the same on every shard
    pairs = engines[0].pair_order()
    assert all(e.pair_order() == pairs for e in engines)
    assert sorted(pairs) == sorted((a, b) for b in range(len(samples)) for a in range(b))
    assert sorted(itertools.chain(*owned)) == list(range(len(pairs)))
    allb = np.concatenate([e.export_edges() for e in engines])
    for e, own in zip(engines, owned):
        e.import_edges(allb)
        assert np.array_equal(e.pair_sums()[0], ref.pair_sums()[0])
        assert np.array_equal(e.pair_sums()[1], ref.pair_sums()[1])
        assert np.array_equal(e.distance()[1], ref.distance()[1])
        key = lambda x: tuple(x)  # noqa: E731
        assert sorted(map(key, e.edges().tolist())) == sorted(map(key, ref.edges().tolist()))
        assert sorted(zip(*e.ideal_nodes())) == sorted(zip(*ref.ideal_nodes()))
        for p in own:
            a, b = pairs[p]
            assert e.pair_rows(a, b).tobytes() == ref.pair_rows(a, b).tobytes()
        st, rst = e.stats(), ref.stats()
        for k in ("edges", "components", "ideal_components", "ideal_nodes", "sample_count"):
            assert st[k] == rst[k], k
        # the graph from the exchanged edges is build_graph's, orders included
        from rna_clique_amd.similarity import SampleSimilarity
        g, g_ref = SampleSimilarity.from_engine(e).graph, SampleSimilarity.from_engine(ref).graph
        assert list(g.nodes) == list(g_ref.nodes)
        assert all(list(g.adj[n]) == list(g_ref.adj[n]) for n in g_ref.nodes)


@pytest.mark.parametrize("shards", [3])
def test_dust_masks_once_per_sample(native, shards):
    """rc_dust_masks / rc_set_dust_masks: the masks a pass of their own makes
    are the run's masks bit for bit (poly-A tails: DUST masks something), and
    sharded engines that take each other's masks (every sample masked by one
    shard, distributed.dust_owners) give the unsharded run's results."""
    from rna_clique_amd import distributed
    from rna_clique_amd.engine import Engine
    from rna_clique_amd.simulate import simulate
    samples, _ = simulate(5, 120, seed=9, p_iso2=0.2, polya=(0.5, 12, 40))
    ref = _load(Engine(device=0), samples)
    ref.run()
    eng = _load(Engine(device=0), samples)
    words = eng.dust_masks([4, 0, 2])
    o = 0
    for s in (4, 0, 2):
        nb = len(samples[s].seq)
        nw = (nb + 63) // 64
        bits = np.unpackbits(words[o:o + nw].view(np.uint8), bitorder="little")
        assert np.array_equal(bits[:nb], ref.dust_mask(s)), s
        assert not bits[nb:].any()
        o += nw
    assert o == len(words) and ref.dust_mask(4).any()
    # a mask pass after a run leaves that run's results readable and unchanged
    rows01, hs10, dist = ref.pair_rows(0, 1).tobytes(), ref.hsps(1, 0).tobytes(), ref.distance()[1]
    again = ref.dust_masks([1, 3])
    assert ref.pair_rows(0, 1).tobytes() == rows01 and ref.hsps(1, 0).tobytes() == hs10
    assert np.array_equal(ref.distance()[1], dist)
    assert again.tobytes() == eng.dust_masks([1, 3]).tobytes()
    # that pass recomputed samples 1 and 3 on the run's own tile: their masks
    # read back, any other sample's is gone and says so (RC_E_STATE), until the
    # next alignment masks every sample again
    from rna_clique_amd._native import NativeError
    nb1 = len(samples[1].seq)
    assert np.array_equal(ref.dust_mask(1),
                          np.unpackbits(again[:(nb1 + 63) // 64].view(np.uint8), bitorder="little")[:nb1])
    for s in (0, 2, 4):
        with pytest.raises(NativeError, match="did not mask"):
            ref.dust_mask(s)
    ref.run()
    assert ref.dust_mask(4).any()
    # every sample masked once, by its owner shard; each shard takes them all
    bases = [len(s.seq) for s in samples]
    owner = distributed.dust_owners(bases, shards)
    engines = [_load(Engine(device=0, shard_rank=r, shard_count=shards), samples) for r in range(shards)]
    made = [e.dust_masks([s for s in range(len(samples)) if owner[s] == r]) for r, e in enumerate(engines)]
    everyone = [s for r in range(shards) for s in range(len(samples)) if owner[s] == r]
    allw = np.concatenate(made)
    for e in engines:
        e.set_dust_masks(everyone, allw)
        e.align()
        e.finish()
    allb = np.concatenate([e.export_edges() for e in engines])
    pairs = engines[0].pair_order()
    for e in engines:
        e.import_edges(allb)
        assert np.array_equal(e.distance()[1], ref.distance()[1])
        for p in range(*e.shard_pairs()):
            a, b = pairs[p]
            assert e.pair_rows(a, b).tobytes() == ref.pair_rows(a, b).tobytes()
            assert e.hsps(a, b).tobytes() == ref.hsps(a, b).tobytes()
            assert e.hsps(b, a).tobytes() == ref.hsps(b, a).tobytes()


def test_dust_masks_in_several_passes(native, monkeypatch):
    """rc_dust_masks over more bases than one alignment tile holds (a C5
    rank masks ~4 Gbp): the samples go through as many mask passes as the
    tile limit needs (forced small here), repeats included, with the same
    words as one pass."""
    from rna_clique_amd.engine import Engine
    from rna_clique_amd.simulate import simulate
    samples, _ = simulate(5, 120, seed=19, p_iso2=0.2, polya=(0.5, 12, 40))
    order = [3, 0, 4, 1, 3]
    one = _load(Engine(device=0), samples).dust_masks(order)
    per = max(len(s.seq) for s in samples)
    monkeypatch.setenv("RC_TILE_BASES", str(2 * per))
    eng = _load(Engine(device=0, shard_rank=1, shard_count=3), samples)
    need = sorted({s for p in eng.owned_pairs() for s in p})
    many = eng.dust_masks([s for s in order if s in need])
    ref = np.concatenate([one[sum((len(samples[t].seq) + 63) // 64 for t in order[:i]):][:(len(samples[s].seq) + 63) // 64]
                          for i, s in enumerate(order) if s in need])
    assert many.tobytes() == ref.tobytes() and many.any()


def _top_select(sample, top):
    """Top-gene rule restated: max coverage per gene, heapq.nlargest((cov, gene))."""
    best = defaultdict(float)
    for c, g in zip(sample.cov.tolist(), sample.gene.tolist()):
        best[g] = max(best[g], float(f"{c:.6f}"))   # the coverage as the FASTA id prints it
    keep = {k for _, k in heapq.nlargest(top, ((v, k) for k, v in best.items()))}
    return np.array([g in keep for g in sample.gene.tolist()])


def _subset(sample, mask, name):
    from rna_clique_amd.simulate import Sample
    idx = np.flatnonzero(mask)
    offs = sample.tx_offsets
    seq = np.concatenate([sample.seq[offs[i]:offs[i + 1]] for i in idx]) if len(idx) else \
        np.zeros(0, np.uint8)
    lens = np.array([offs[i + 1] - offs[i] for i in idx], dtype=np.uint64)
    return Sample(name, seq, np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64),
                  sample.gene[idx], sample.iso[idx], sample.cov[idx])


def test_rna_clique_end_to_end(native, tmp_path):
    from rna_clique_amd.rna_clique import rna_clique
    from rna_clique_amd.simulate import simulate
    samples, _ = simulate(4, 150, seed=9, p_iso2=0.2, indel_rate=0.002)
    dirs = []
    for s in samples:
        d = tmp_path / "in" / s.name
        d.mkdir(parents=True)
        s.write_fasta(d / "transcripts.fasta")
        dirs.append(d)
    od1, od2 = tmp_path / "od1", tmp_path / "od2"
    sim, pts = rna_clique(dirs, od1, od2, tmp_path / "cache", tmp_path / "graph.pkl",
                          tmp_path / "matrix.h5", top_genes=100, jobs=2)
    assert pts == {od1 / f"{s.name}_top.fasta": s.name for s in samples}
    top = [_subset(s, _top_select(s, 100), str(od1 / f"{s.name}_top.fasta")) for s in samples]
    msgs, summary = full_check(sim.engine, top)
    assert not msgs, "\n".join(msgs[:10])
    df = sim.get_dissimilarity_df()
    assert list(df.index) == sorted(t.name for t in top)
    assert np.array_equal(df.to_numpy(), summary["matrix"])
    # gene matches tables on disk (pandas table-format HDF5, key gene_matches)
    from rna_clique_amd.tables import read_table
    for a, b in itertools.combinations(range(len(samples)), 2):
        t = read_table(od2 / f"{samples[a].name}--{samples[b].name}.h5")
        rows = sim.engine.pair_rows(a, b)
        assert list(t.index) == rows["label"].tolist()
        assert (t["nident"].to_numpy() == rows["hsp"]["nident"]).all()
        assert set(t["ssample"].astype(str)) <= {top[a].name}
    # graph.pkl: the networkx graph build_graph would make
    with open(tmp_path / "graph.pkl", "rb") as f:
        g = pickle.load(f)
    assert g.number_of_edges() == summary["stats"]["edges"]
    # ... node, neighbour and edge order included (the file comes from the
    # edge records sorted on the device; sim.graph is build_graph over the
    # pairs' rows in combinations order)
    g_ref = sim.graph
    assert list(g.nodes) == list(g_ref.nodes)
    assert all(list(g.adj[n]) == list(g_ref.adj[n]) for n in g_ref.nodes)
    assert list(g.edges) == list(g_ref.edges)
    assert sim.sample_count == len(samples)
    assert (tmp_path / "matrix.h5").stat().st_size > 0
    # restricted tables sum to the same fractions
    for (ka, kb), t in sim.restricted_comparison_dfs():
        a, b = [x.name for x in top].index(ka), [x.name for x in top].index(kb)
        num, den = sim.engine.pair_sums()
        assert int(t["nident"].sum()) == num[a, b]
        assert int((t["length"] - t["gaps"]).sum()) == den[a, b]


LIBHDF5 = "/opt/conda/lib/libhdf5.so.103"


@pytest.mark.skipif(not os.path.exists(LIBHDF5), reason="no libhdf5 to read the file back")
def test_matrix_h5_from_run(native, tmp_path):
    from h5read import H5 as _H5
    from rna_clique_amd.engine import Engine
    from rna_clique_amd.h5 import write_matrix
    from rna_clique_amd.similarity import SampleSimilarity
    from rna_clique_amd.simulate import simulate
    samples, _ = simulate(3, 80, seed=12)
    eng = _load(Engine(device=0), samples)
    eng.run()
    df = SampleSimilarity.from_engine(eng).get_dissimilarity_df()
    write_matrix(df, tmp_path / "m.h5")
    h = _H5()
    f = h.open(tmp_path / "m.h5")
    assert np.array_equal(h.doubles(f, "/matrix/block0_values"), df.to_numpy())
    assert h.strings(f, "/matrix/axis1") == list(df.index)


def _shard_worker(rank, world, port, q, graph_dir=None):
    import os as _os
    import torch.distributed as dist
    _os.environ["MASTER_ADDR"] = "127.0.0.1"
    _os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rna_clique_amd import distributed
        from rna_clique_amd.engine import Engine
        from rna_clique_amd.simulate import simulate
        samples, _ = simulate(5, 100, seed=31, p_iso2=0.2, indel_rate=0.002)
        eng = _load(Engine(device=0, shard_rank=rank, shard_count=world), samples)
        distributed.sharded_run(eng)
        gfile = None
        if graph_dir is not None:
            # graph.pkl of a sharded run: the native writer over the exchanged edges
            from rna_clique_amd.similarity import SampleSimilarity
            gfile = _os.path.join(graph_dir, f"graph_{rank}.pkl")
            SampleSimilarity.from_engine(eng).write_graph(gfile)
        q.put((rank, eng.distance()[1].tobytes(), eng.stats()["edges"], gfile))
    finally:
        dist.destroy_process_group()


def test_two_processes_share_the_pairs(native, tmp_path):
    """world_size 2, one engine per process on the same GPU, gloo exchange:
    the same distances as one engine, and each rank's graph.pkl (native
    writer over the exchanged edges) is build_graph's graph: its nodes and
    edges, in its node order and neighbour order (the exchanged edges come
    per pair in pair order, in the order of each pair's rows)."""
    import socket
    import torch.multiprocessing as mp
    from rna_clique_amd.engine import Engine
    from rna_clique_amd.simulate import simulate
    samples, _ = simulate(5, 100, seed=31, p_iso2=0.2, indel_rate=0.002)
    ref = _load(Engine(device=0), samples)
    ref.run()
    want = ref.distance()[1]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_shard_worker, args=(r, 2, port, q, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    import pickle
    from rna_clique_amd.similarity import SampleSimilarity
    g_ref = SampleSimilarity.from_engine(ref).graph
    ref_edges = {frozenset(e) for e in g_ref.edges}
    for _, blob, edges, gfile in got:
        assert np.frombuffer(blob, dtype=np.float64).reshape(want.shape).tobytes() == want.tobytes()
        assert edges == ref.stats()["edges"]
        with open(gfile, "rb") as f:
            g = pickle.load(f)
        assert set(g.nodes) == set(g_ref.nodes)
        assert {frozenset(e) for e in g.edges} == ref_edges
        assert list(g.nodes) == list(g_ref.nodes)
        assert all(list(g.adj[n]) == list(g_ref.adj[n]) for n in g_ref.nodes)


# ------------------------------------------------- SampleSimilarity(graph, tables)

def _golden_inputs(fx, cols):
    import networkx as nx
    exp = fx["expected"]
    g = nx.Graph()
    g.add_nodes_from(tuple(n) for n in exp["nodes"])
    g.add_edges_from((tuple(u), tuple(v)) for u, v in exp["edges"])
    dfs = []
    for key, rows in exp["tables"].items():
        t1, t2 = key.split("|")
        df = pd.DataFrame([dict(zip(cols, r)) for r in rows], columns=cols)
        df = df.set_index("label")
        dfs.append((frozenset((t1, t2)), df))
    return g, dfs


def test_sample_similarity_from_graph_and_tables_golden(native):
    """The reference constructor SampleSimilarity(graph, comparison_dfs)
    (filtered_distance.py:162-169) on the reference's own golden graphs and
    tables: ideal nodes, sample_count and distances as the reference computed
    them (components, filter and sums on the GPU, graph-only engine)."""
    import json
    from rna_clique_amd.similarity import NoIdealComponentsError, SampleSimilarity
    d = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "post_alignment.json")))
    checked = 0
    for fx in d["fixtures"]:
        exp = fx["expected"]
        if any(k != "matrix" for k in exp["errors"]):
            continue
        g, dfs = _golden_inputs(fx, d["columns"])
        sim = SampleSimilarity(g, dfs)
        assert sim.sample_count == exp["sample_count"]
        assert sorted(map(list, sim.valid.itertuples(index=False, name=None))) == exp["valid"]
        if exp["matrix"] is None:
            with pytest.raises(NoIdealComponentsError):
                sim.get_dissimilarity_df()
        else:
            df = sim.get_dissimilarity_df()
            assert list(df.index) == exp["matrix"]["labels"]
            assert np.array_equal(df.to_numpy(), np.array(exp["matrix"]["values"]))
        # a sample_count the graph cannot meet: no ideal component at all
        with pytest.raises(NoIdealComponentsError):
            SampleSimilarity(g, dfs, sample_count=exp["sample_count"] + 1).get_dissimilarity_df()
        checked += 1
    assert checked >= 15


def test_sample_similarity_arbitrary_graph(native):
    """A graph that is not build_graph(tables): an extra edge without table
    rows, table rows whose edge is missing from the graph, an isolated node
    (which still counts toward sample_count) -- against the restated
    reference semantics (oracle/post_oracle.py)."""
    import json
    import networkx as nx
    from oracle import post_oracle
    from rna_clique_amd.similarity import SampleSimilarity
    d = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "post_alignment.json")))
    fx = next(f for f in d["fixtures"] if not f["expected"]["errors"] and f["expected"]["matrix"])
    g, dfs = _golden_inputs(fx, d["columns"])
    edges = list(g.edges)
    g.remove_edge(*edges[0])          # its table rows now only count toward the sums
    u, v = edges[1][0], edges[-1][1]
    if u[0] != v[0]:
        g.add_edge(u, v)              # an edge no table row gives
    g.add_node(("zzz_isolated", 7))   # a sample of its own
    sim = SampleSimilarity(g, dfs)
    nodes = set(g.nodes)
    gedges = {tuple(sorted(e)) for e in g.edges}
    valid = post_oracle.ideal_nodes(nodes, gedges)
    assert sim.sample_count == post_oracle.sample_count(nodes)
    assert sorted(map(tuple, sim.valid.itertuples(index=False, name=None))) == sorted(valid)
    num, den = sim.pair_sums()
    lab = sim.labels
    for k, df in dfs:
        rows = df.reset_index().to_dict("records")
        ss, qs = rows[0]["ssample"], rows[0]["qsample"]
        want = post_oracle.pair_sums(ss, qs, rows, valid)
        a, b = lab.index(ss), lab.index(qs)
        assert (int(num[a, b]), int(den[a, b])) == want


def test_sample_similarity_matrix_samples_from_tables(native):
    """The matrix's samples are the tables' samples (similarity_computer.py:
    216-226: sorted key elements of the similarities), not the graph's: a
    sample known only from graph nodes -- with an explicit sample_count, so
    the ideal filter is unchanged -- is no row of the matrix, and the matrix
    is the reference's golden one. An empty table is skipped
    (mapping_from_dfs; the reference fails on it)."""
    import json
    from rna_clique_amd.similarity import SampleSimilarity
    d = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "post_alignment.json")))
    fx = next(f for f in d["fixtures"] if not f["expected"]["errors"] and f["expected"]["matrix"])
    exp = fx["expected"]
    g, dfs = _golden_inputs(fx, d["columns"])
    g.add_node(("zzz_graph_only", 7))
    g.add_edge(("zzz_graph_only", 8), ("zzz_graph_only2", 9))
    sim = SampleSimilarity(g, dfs, sample_count=exp["sample_count"])
    assert "zzz_graph_only" in sim.labels
    df = sim.get_dissimilarity_df()
    assert list(df.index) == exp["matrix"]["labels"] == list(df.columns)
    assert np.array_equal(df.to_numpy(), np.array(exp["matrix"]["values"]))
    assert set(sim.get_similarities().key_elements()) == set(exp["matrix"]["labels"])
    empty = dfs[0][1].iloc[0:0]
    kept = list(SampleSimilarity.mapping_from_dfs([empty] + [t for _, t in dfs]))
    assert len(kept) == len(dfs)


def test_tables_and_graph_reload(native, tmp_path):
    """The resume path (CS3): rna_clique() writes od2 tables and graph.pkl,
    SampleSimilarity.from_filenames reads them back and gives the same
    matrix; find_all_pairs / filtering_step (the reference's phase-1 entry
    points) produce the same tables."""
    import glob
    from rna_clique_amd.filtering_step import filtering_step
    from rna_clique_amd.rna_clique import rna_clique
    from rna_clique_amd.similarity import SampleSimilarity
    from rna_clique_amd.simulate import simulate
    samples, _ = simulate(4, 150, seed=19, p_iso2=0.2, indel_rate=0.002, p_revcomp=0.3)
    dirs = []
    for s in samples:
        dd = tmp_path / "in" / s.name
        dd.mkdir(parents=True)
        s.write_fasta(dd / "transcripts.fasta")
        dirs.append(dd)
    sim, pts = rna_clique(dirs, tmp_path / "od1", tmp_path / "od2", None, tmp_path / "graph.pkl",
                          tmp_path / "matrix.h5", top_genes=120, jobs=2)
    want = sim.get_dissimilarity_df()
    fns = sorted(glob.glob(str(tmp_path / "od2" / "*")))
    assert len(fns) == 6
    back = SampleSimilarity.from_filenames(tmp_path / "graph.pkl", fns)
    got = back.get_dissimilarity_df()
    assert list(got.index) == list(want.index)
    assert np.array_equal(got.to_numpy(), want.to_numpy())
    assert back.sample_count == sim.sample_count
    # phase 1 through the reference's entry points
    tables, paths, graph, n, p2s = filtering_step(dirs, tmp_path / "f_od1", tmp_path / "f_od2", None,
                                                 tmp_path / "f_graph.pkl", 120)
    assert n == 6 and sorted(p2s.values()) == sorted(s.name for s in samples)
    paths = list(paths)
    got_tables = list(tables)
    assert len(got_tables) == len(paths) == 6
    assert graph.number_of_edges() == sim.graph.number_of_edges()
    again = SampleSimilarity(graph, list(SampleSimilarity.mapping_from_dfs(got_tables)))
    assert np.array_equal(again.get_dissimilarity_df().to_numpy(), want.to_numpy())


@pytest.mark.parametrize("split,share", [(1, 1), (0, 1), (1, 0)])
def test_tiles_match_one_pass(native, monkeypatch, split, share):
    """A shard whose samples do not fit one alignment pass is cut into tiles
    (a- and b-chunks, positions relative to each tile, HSPs appended): forced
    here with a small RC_TILE_BASES, the results equal one pass bit for bit.
    split 1 (default): tiles with every a below every b place the b chunk at
    a fixed position, and consecutive tiles of one b chunk reuse its 16-mer
    index and DUST masks; split 0 (RC_TILE_SPLIT=0) rebuilds both per tile.
    share 0 (RC_SHARE=0: the two directed searches one after the other) puts
    the a part into the index too, so split tiles must not reuse it."""
    monkeypatch.setenv("RC_TILE_SPLIT", str(split))
    monkeypatch.setenv("RC_SHARE", str(share))
    from rna_clique_amd.engine import Engine
    from rna_clique_amd.simulate import simulate
    samples, _ = simulate(6, 150, seed=23, p_iso2=0.2, indel_rate=0.002, p_revcomp=0.3,
                          polya=(0.2, 15, 40))
    ref = _load(Engine(device=0), samples)
    ref.run()
    per = max(int(s.tx_offsets[-1]) for s in samples)
    monkeypatch.setenv("RC_TILE_BASES", str(3 * per))
    eng = _load(Engine(device=0), samples)
    eng.run()
    tm = eng.timings()
    assert tm["tiles"] > 1 and (tm["index_reused"] > 0) == bool(split and share)
    for q in range(6):
        for s in range(6):
            if q != s:
                assert eng.hsps(q, s).tobytes() == ref.hsps(q, s).tobytes(), (q, s)
    for a, b in itertools.combinations(range(6), 2):
        assert eng.pair_rows(a, b).tobytes() == ref.pair_rows(a, b).tobytes()
    assert np.array_equal(eng.distance()[1], ref.distance()[1])
    msgs, _ = full_check(eng, samples)
    assert not msgs, "\n".join(msgs[:10])


@pytest.mark.parametrize("shards", [3, 5])
def test_shards_hold_only_their_samples(native, monkeypatch, shards):
    """Sharded engines given only the sequences of their own pairs' samples
    (the others as metadata) -- and, for 5 shards, cut into tiles too --
    equal the unsharded engine."""
    from rna_clique_amd import distributed
    from rna_clique_amd.engine import Engine
    from rna_clique_amd.simulate import simulate
    samples, _ = simulate(7, 100, seed=29, p_iso2=0.2, indel_rate=0.002, p_revcomp=0.3)
    ref = _load(Engine(device=0), samples)
    ref.run()
    bases = [int(s.tx_offsets[-1]) for s in samples]
    if shards == 5:
        monkeypatch.setenv("RC_TILE_BASES", str(2 * max(bases)))
    engines = []
    for r in range(shards):
        need = distributed.needed_samples(bases, shards, r)
        assert len(need) < len(samples) or shards < 3
        e = Engine(device=0, shard_rank=r, shard_count=shards)
        for i, s in enumerate(samples):
            e.add_sample(s.name, s.seq if i in need else None, s.tx_offsets, s.gene, s.iso)
        e.align()
        e.finish()
        engines.append(e)
    allb = np.concatenate([e.export_edges() for e in engines])
    pairs = engines[0].pair_order()
    for e in engines:
        e.import_edges(allb)
        assert np.array_equal(e.distance()[1], ref.distance()[1])
        for p in range(*e.shard_pairs()):
            a, b = pairs[p]
            assert e.pair_rows(a, b).tobytes() == ref.pair_rows(a, b).tobytes()
    # a shard missing one of its own samples refuses to run
    from rna_clique_amd._native import NativeError
    bad = Engine(device=0, shard_rank=0, shard_count=shards)
    for i, s in enumerate(samples):
        bad.add_sample(s.name, None, s.tx_offsets, s.gene, s.iso)
    with pytest.raises(NativeError):
        bad.align()


def test_device_edge_exchange_and_sharded_tables(native):
    """The device-pointer edge path (rc_export_edges / rc_import_edges with
    on_device=1, what the RCCL exchange uses): shard engines export into
    CUDA tensors, the concatenation is imported from device memory, and the
    result equals the unsharded engine. SampleSimilarity(store_dfs=True) on a
    shard holds that shard's tables; the union over shards is the full set."""
    import torch
    from rna_clique_amd.engine import Engine
    from rna_clique_amd.similarity import SampleSimilarity
    from rna_clique_amd.tables import pair_table
    from rna_clique_amd.simulate import simulate
    samples, _ = simulate(5, 120, seed=37, p_iso2=0.2, indel_rate=0.002)
    ref = _load(Engine(device=0), samples)
    ref.run()
    engines = [_load(Engine(device=0, shard_rank=r, shard_count=3), samples) for r in range(3)]
    rs = engines[0].edge_record_size()
    parts = []
    for e in engines:
        e.align()
        e.finish()
        t = torch.empty(max(e.local_edge_count() * rs, 1), dtype=torch.uint8, device="cuda")
        n = e.export_edges(t)
        assert n == e.local_edge_count()
        torch.cuda.synchronize()
        assert t[:n * rs].cpu().numpy().tobytes() == e.export_edges().tobytes()
        parts.append(t[:n * rs])
    allt = torch.cat(parts)
    torch.cuda.synchronize()
    seen = {}
    for e in engines:
        e.import_edges(allt, allt.numel() // rs)
        assert np.array_equal(e.distance()[1], ref.distance()[1])
        sim = SampleSimilarity.from_engine(e, store_dfs=True)
        assert np.array_equal(sim.get_dissimilarity_df().to_numpy(),
                              SampleSimilarity.from_engine(ref).get_dissimilarity_df().to_numpy())
        for k, df in sim.comparison_dfs.items():
            assert k not in seen
            seen[k] = df
    labels = ref.labels
    assert len(seen) == 10
    for a, b in itertools.combinations(range(5), 2):
        want = pair_table(ref, a, b, labels)
        got = seen[(labels[a], labels[b])] if (labels[a], labels[b]) in seen else \
            seen[(labels[b], labels[a])]
        pd.testing.assert_frame_equal(got, want)


def _rccl_worker(port, q):
    import os as _os
    import torch
    import torch.distributed as dist
    _os.environ["MASTER_ADDR"] = "127.0.0.1"
    _os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        from rna_clique_amd import distributed
        from rna_clique_amd.engine import Engine
        from rna_clique_amd.simulate import simulate
        samples, _ = simulate(4, 100, seed=41, polya=(0.5, 12, 40))
        eng = _load(Engine(device=0, shard_rank=0, shard_count=1), samples)
        # the DUST masks over RCCL too (one rank owns them all): device
        # buffers, all-gather, rc_set_dust_masks from the device
        distributed.exchange_dust(eng, force=True)
        distributed.sharded_run(eng)        # RCCL branch: device export, all-gather, device import
        got = (eng.distance()[1].tobytes(), eng.hsps(0, 1).tobytes(), eng.hsps(1, 0).tobytes())
        # again with the alignment working set freed before the exchange
        # (rc_trim), then a third run that allocates it anew
        distributed.sharded_run(eng, trim=True)
        again = (eng.distance()[1].tobytes(), eng.hsps(0, 1).tobytes(), eng.hsps(1, 0).tobytes())
        distributed.sharded_run(eng)
        third = (eng.distance()[1].tobytes(), eng.hsps(0, 1).tobytes(), eng.hsps(1, 0).tobytes())
        q.put(got if got == again == third else None)
    finally:
        dist.destroy_process_group()


def test_rccl_exchange_world1(native):
    """exchange_dust and exchange_edges over an RCCL process group (world 1 on
    the one GPU of the test box: the device-to-device branches end to end)."""
    import socket
    import torch.multiprocessing as mp
    from rna_clique_amd.engine import Engine
    from rna_clique_amd.simulate import simulate
    samples, _ = simulate(4, 100, seed=41, polya=(0.5, 12, 40))
    ref = _load(Engine(device=0), samples)
    ref.run()
    assert ref.dust_mask(0).any()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(port, q))
    p.start()
    got = q.get(timeout=300)
    p.join(timeout=120)
    assert p.exitcode == 0
    assert got == (ref.distance()[1].tobytes(), ref.hsps(0, 1).tobytes(), ref.hsps(1, 0).tobytes())


def test_trim_and_edge_parts(native):
    """rc_trim frees the alignment working set of a finished run (device
    bytes drop; rows, HSPs and distances stay readable and unchanged; the
    next run allocates it again and gives the same results), and
    rc_import_edge_parts takes padded blocks -- from the host or the device,
    device records range-checked on the device."""
    import torch
    from rna_clique_amd._native import NativeError
    from rna_clique_amd.engine import Engine
    from rna_clique_amd.simulate import simulate
    samples, _ = simulate(4, 120, seed=43, p_iso2=0.2, polya=(0.3, 12, 40))
    eng = _load(Engine(device=0), samples)
    eng.run()
    pairs = list(itertools.combinations(range(4), 2))
    rows = {p: eng.pair_rows(*p).tobytes() for p in pairs}
    hs = eng.hsps(3, 1).tobytes()
    dist0 = eng.distance()[1]
    edges = eng.export_edges()
    before = eng.timings()["dev_bytes"]
    eng.trim()
    after = eng.timings()["dev_bytes"]
    assert after < before - (64 << 20), (before, after)
    assert {p: eng.pair_rows(*p).tobytes() for p in pairs} == rows and eng.hsps(3, 1).tobytes() == hs
    assert np.array_equal(eng.distance()[1], dist0)
    with pytest.raises(NativeError):
        eng.dust_mask(0)   # no tile loaded after a trim
    rs = Engine.edge_record_size()
    recs = edges.reshape(-1, rs)
    n = len(recs)
    counts = [n // 3, n // 3, n - 2 * (n // 3)]
    stride = max(counts) + 7
    buf = np.full((3 * stride, rs), 0xAB, dtype=np.uint8)   # padding is garbage, never read
    o = 0
    for r, c in enumerate(counts):
        buf[r * stride:r * stride + c] = recs[o:o + c]
        o += c
    eng.import_edge_parts(buf.ravel(), counts, stride)
    assert np.array_equal(eng.distance()[1], dist0)
    dev = torch.from_numpy(buf.ravel().copy()).cuda()
    eng.import_edge_parts(dev, counts, stride)
    assert np.array_equal(eng.distance()[1], dist0)
    bad = buf.copy()
    bad[stride + 1, 0:4] = 0xFF   # node id a out of range in block 1
    with pytest.raises(NativeError, match="out of range"):
        eng.import_edge_parts(torch.from_numpy(bad.ravel()).cuda(), counts, stride)
    with pytest.raises(NativeError, match="out of range"):
        eng.import_edge_parts(bad.ravel(), counts, stride)
    eng.run()   # the working set allocated again
    assert {p: eng.pair_rows(*p).tobytes() for p in pairs} == rows and eng.hsps(3, 1).tobytes() == hs
    assert np.array_equal(eng.distance()[1], dist0)
