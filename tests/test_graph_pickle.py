"""graph.pkl by the native writer (graph_pickle.cpp) against build_graph +
pickle (build_graph.py:40-68, filtering_step.py:158-159): pickle.load must
give the same networkx Graph -- nodes, node order, each node's neighbour
order, edges, and the edge data dict shared by both ends."""
import pickle

import numpy as np
import pytest

from rna_clique_amd.tables import build_graph, write_graph_pickle


def _tables(rng, names, pairs, n, gene_hi):
    out = []
    for sa, qa in pairs:
        sg = rng.integers(0, gene_hi, n)
        qg = rng.integers(0, gene_hi, n)
        out.append((sa, qa, sg, qg))
    return out


def _as_rows(tabs, names):
    return [(names[sa], names[qa], np.rec.fromarrays([sg, qg], names="sgene,qgene")) for sa, qa, sg, qg in tabs]


@pytest.mark.parametrize("seed,n,gene_hi", [(0, 0, 10), (1, 1, 5), (2, 400, 50), (3, 3000, 100000),
                                            (4, 2500, 2500)])
def test_graph_pickle_equals_build_graph(native, tmp_path, seed, n, gene_hi):
    rng = np.random.default_rng(seed)
    names = ["/d/od1/s0_top.fasta", "/d/od1/s1_top.fasta", "/d/od1/sé2_top.fasta", "s3"]
    pairs = [(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)]
    tabs = _tables(rng, names, pairs, n, gene_hi)
    if n:
        tabs[0][2][:3] = 3_000_000_000     # genes past 32 bits
        tabs[1][3][:2] = -7                # and negative ones
        tabs[2][2][0] = tabs[2][3][0]      # a (sample, gene) pair seen from both sides
    path = tmp_path / "graph.pkl"
    write_graph_pickle(path, tabs, names)
    with open(path, "rb") as f:
        g = pickle.load(f)
    want = build_graph(_as_rows(tabs, names))
    assert type(g) is type(want)
    assert list(g.nodes) == list(want.nodes)
    assert [list(g.adj[u]) for u in g.nodes] == [list(want.adj[u]) for u in want.nodes]
    assert list(g.edges) == list(want.edges)
    for u, v in list(g.edges)[:50]:
        assert g.adj[u][v] is g.adj[v][u]
    assert g.graph == want.graph
