"""Diagnostic: does a sharded run's graph.pkl (native writer over the
exchanged edges) have build_graph's node and neighbour ORDER, not only its
node and edge sets? Two and three shard engines on one GPU vs one engine."""
import os
import pickle
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from rna_clique_amd.engine import Engine  # noqa: E402
from rna_clique_amd.similarity import SampleSimilarity  # noqa: E402
from rna_clique_amd.simulate import simulate  # noqa: E402


def load(eng, samples):
    for s in samples:
        eng.add_sample(s.name, s.seq, s.tx_offsets, s.gene, s.iso)
    return eng


samples, _ = simulate(5, 120, seed=4, p_iso2=0.2, indel_rate=0.002, p_paralog=0.05)
ref = load(Engine(device=0), samples)
ref.run()
g_ref = SampleSimilarity.from_engine(ref).graph
tmp = tempfile.mkdtemp()
for shards in (2, 3):
    engines = [load(Engine(device=0, shard_rank=r, shard_count=shards), samples) for r in range(shards)]
    for e in engines:
        e.align()
        e.finish()
    allb = np.concatenate([e.export_edges() for e in engines])
    for r, e in enumerate(engines):
        e.import_edges(allb)
        f = os.path.join(tmp, f"g{shards}_{r}.pkl")
        SampleSimilarity.from_engine(e).write_graph(f)
        with open(f, "rb") as fh:
            g = pickle.load(fh)
        same_sets = set(g.nodes) == set(g_ref.nodes) and {frozenset(x) for x in g.edges} == {
            frozenset(x) for x in g_ref.edges}
        node_order = list(g.nodes) == list(g_ref.nodes)
        adj_order = all(list(g.adj[n]) == list(g_ref.adj[n]) for n in g_ref.nodes) if node_order else False
        gm = SampleSimilarity.from_engine(e).graph
        mem = list(gm.nodes) == list(g_ref.nodes) and all(list(gm.adj[n]) == list(g_ref.adj[n]) for n in g_ref.nodes)
        print(f"shards {shards} rank {r}: sets {same_sets} node order {node_order} adjacency order {adj_order}"
              f" in-memory graph order {mem}")
        if not node_order:
            a, b = list(g.nodes), list(g_ref.nodes)
            i = next(i for i in range(min(len(a), len(b))) if a[i] != b[i])
            print("  first difference at", i, a[i:i + 3], b[i:i + 3])
