"""Neighbour joining and Robinson-Foulds distance (test helper).

The reference's only results-level check (tests/verify_install/
verify_distances.py:39-55) builds a neighbour-joining tree from matrix.h5 with
Biopython's DistanceTreeConstructor and asserts a Robinson-Foulds distance of
0 against the simulated true tree (dendropy). Neither library is installed
here, so both are restated: NJ (Saitou & Nei 1987) on the distance matrix, and
RF as the size of the symmetric difference of the non-trivial bipartitions.
"""
from __future__ import annotations

import numpy as np


def _split(members, leaves):
    """Canonical form of the bipartition {members | rest}: the side without
    the first leaf, as a frozenset (trivial splits -> None)."""
    m = frozenset(members)
    rest = frozenset(leaves) - m
    if len(m) < 2 or len(rest) < 2:
        return None
    first = min(leaves)
    return rest if first in m else m


def nj_splits(D, labels):
    """Non-trivial bipartitions of the neighbour-joining tree of D."""
    D = np.array(D, dtype=np.float64)
    clusters = [frozenset([x]) for x in labels]
    splits = set()
    while len(clusters) > 3:
        n = len(clusters)
        r = D.sum(axis=1)
        Q = (n - 2) * D - r[:, None] - r[None, :]
        np.fill_diagonal(Q, np.inf)
        i, j = np.unravel_index(int(np.argmin(Q)), Q.shape)
        i, j = min(i, j), max(i, j)
        new = clusters[i] | clusters[j]
        s = _split(new, labels)
        if s is not None:
            splits.add(s)
        d_new = 0.5 * (D[i] + D[j] - D[i, j])
        keep = [k for k in range(n) if k not in (i, j)]
        D2 = np.zeros((len(keep) + 1, len(keep) + 1))
        D2[:-1, :-1] = D[np.ix_(keep, keep)]
        D2[-1, :-1] = D2[:-1, -1] = d_new[keep]
        D = D2
        clusters = [clusters[k] for k in keep] + [new]
    # the last three clusters meet at one node: each is a split
    for c in clusters:
        s = _split(c, labels)
        if s is not None:
            splits.add(s)
    return splits


def tree_splits(parent, leaves, leaf_label):
    """Non-trivial bipartitions of a rooted tree given as a parent array
    (simulate.birth_death_tree), restricted to `leaves`."""
    parent = np.asarray(parent)
    below = {v: set() for v in range(len(parent))}
    for leaf in leaves:
        v = leaf
        while v >= 0:
            below[v].add(leaf_label[leaf])
            v = int(parent[v])
    labels = [leaf_label[x] for x in leaves]
    out = set()
    for v, members in below.items():
        if members:
            s = _split(members, labels)
            if s is not None:
                out.add(s)
    return out


def robinson_foulds(a, b):
    return len(a ^ b)
