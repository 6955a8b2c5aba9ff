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
    # gene matches tables on disk (write_table's pickle form)
    for a, b in itertools.combinations(range(len(samples)), 2):
        t = pd.read_pickle(od2 / f"{samples[a].name}--{samples[b].name}.pkl")
        rows = sim.engine.pair_rows(a, b)
        assert list(t.index) == rows["label"].tolist()
        assert (t["nident"].to_numpy() == rows["hsp"]["nident"]).all()
        assert set(t["ssample"].astype(str)) <= {top[a].name}
    # graph.pkl: the networkx graph build_graph would make
    with open(tmp_path / "graph.pkl", "rb") as f:
        g = pickle.load(f)
    assert g.number_of_edges() == summary["stats"]["edges"]
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
    df = SampleSimilarity(eng).get_dissimilarity_df()
    write_matrix(df, tmp_path / "m.h5")
    h = _H5()
    f = h.open(tmp_path / "m.h5")
    assert np.array_equal(h.doubles(f, "/matrix/block0_values"), df.to_numpy())
    assert h.strings(f, "/matrix/axis1") == list(df.index)


def _shard_worker(rank, world, port, q):
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
        q.put((rank, eng.distance()[1].tobytes(), eng.stats()["edges"]))
    finally:
        dist.destroy_process_group()


def test_two_processes_share_the_pairs(native):
    """world_size 2, one engine per process on the same GPU, gloo exchange:
    the same distances as one engine."""
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
    procs = [ctx.Process(target=_shard_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for _, blob, edges in got:
        assert np.frombuffer(blob, dtype=np.float64).reshape(want.shape).tobytes() == want.tobytes()
        assert edges == ref.stats()["edges"]
