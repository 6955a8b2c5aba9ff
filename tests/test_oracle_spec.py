"""CPU checks of the alignment oracle's spec (oracle/align_oracle.c header).

Spec 4b (canonical roles): the greedy extension of a seed is evaluated with the
lower-numbered sample in its first role, so both directed searches of a pair
get the same geometric HSP from the same seed. On plus-strand data without
DUST both searches extend the same first seeds (the forward (x, y) and reverse
(y, x) orders agree on colinear seeds), so the reverse search must equal the
mirror image of the forward one (spec 5b) -- with indels, where the greedy
step's move ties decide gap counts. Minus-strand candidates start the two
searches at opposite ends; there the searches may differ (gapopen), and the
GPU's shared candidate set extends each search's own first seed.
"""
import numpy as np

from oracle.align import OracleDB
from rna_clique_amd.simulate import simulate


def _key(h):
    return tuple(int(h[k]) for k in h.dtype.names if k != "evalue")


def test_canonical_roles_make_plus_strand_searches_mirror_images():
    samples, _ = simulate(3, 400, seed=21, p_iso2=0.2, indel_rate=0.004)
    db = OracleDB(samples)
    n = 0
    for a, b in ((0, 1), (0, 2), (1, 2)):
        ind = db.align(b, a, symmetric=False)
        sym = db.align(b, a, symmetric=True)
        assert sorted(map(_key, ind)) == sorted(map(_key, sym))
        n += len(ind)
        assert np.any(ind["gaps"] > 0)   # indels: move ties do occur
    assert n > 1000


def test_minus_strand_searches_start_at_opposite_seeds():
    """Documents why the GPU's shared candidate set keeps a second first seed
    (cand_box2) for the reverse search: on the minus strand the two searches
    start at opposite ends of the alignment and may report other HSPs (gap
    opens, or an HSP near the e-value cut)."""
    samples, _ = simulate(2, 400, seed=22, indel_rate=0.004, p_revcomp=0.5)
    db = OracleDB(samples)
    ind = db.align(1, 0, symmetric=False)
    sym = db.align(1, 0, symmetric=True)
    assert set(map(_key, ind)) != set(map(_key, sym))
    plus_i = sorted(_key(h) for h in ind if h["strand"] == 0)
    plus_s = sorted(_key(h) for h in sym if h["strand"] == 0)
    assert plus_i == plus_s
