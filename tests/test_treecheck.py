"""CPU: the neighbour-joining / Robinson-Foulds helper the science-level GPU
tests use (tests/treecheck.py), on trees whose answer is known."""
import itertools

import numpy as np

from treecheck import nj_splits, robinson_foulds, tree_splits


def _tree_distances(parent, blen, leaves):
    """Path lengths between leaves of a parent-array tree (an additive metric:
    neighbour joining must return the tree exactly)."""
    def path(v):
        out = []
        while v >= 0:
            out.append(v)
            v = int(parent[v])
        return out
    n = len(leaves)
    D = np.zeros((n, n))
    for i, j in itertools.combinations(range(n), 2):
        pi, pj = path(leaves[i]), path(leaves[j])
        common = set(pi) & set(pj)
        D[i, j] = D[j, i] = sum(blen[v] for v in pi if v not in common) + \
            sum(blen[v] for v in pj if v not in common)
    return D


def test_nj_recovers_additive_trees():
    from rna_clique_amd.simulate import birth_death_tree
    for seed, taxa in [(1, 4), (2, 8), (3, 16), (4, 32)]:
        parent, blen, leaves = birth_death_tree(taxa, np.random.default_rng(seed))
        labels = [f"T{i}" for i in range(taxa)]
        D = _tree_distances(parent, blen, leaves)
        truth = tree_splits(parent, leaves, dict(zip(leaves, labels)))
        assert len(truth) == taxa - 3   # a binary unrooted tree
        assert robinson_foulds(nj_splits(D, labels), truth) == 0
        if taxa >= 8:   # a wrong labelling is detected
            swapped = labels[:]
            swapped[0], swapped[-1] = swapped[-1], swapped[0]
            assert robinson_foulds(nj_splits(D, swapped), truth) > 0
