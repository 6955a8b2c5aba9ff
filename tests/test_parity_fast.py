"""The vectorised pair check (oracle/parity.compare_pair_fast) agrees with the
plain one (compare_pair, post_oracle pinned to the reference's fixtures) on
real oracle alignments: silent on a faithful capture, and naming the first
differing HSP, row or sum when one field is off."""
import numpy as np
import pytest

from oracle import post_oracle
from oracle.align import OracleDB
from oracle.parity import compare_pair, compare_pair_fast, hits_for_post
from rna_clique_amd import _native as nat


def _capture_from_oracle(samples, db, ora, names):
    """What capture_pairs would hold for an engine that equals the oracle:
    both searches' HSPs (engine layout, local transcripts), the table rows
    and the unfiltered sums."""
    hs = {}
    for (q, s), arr in ora.items():
        h = np.zeros(len(arr), dtype=nat.HSP_DTYPE)
        for f in nat.HSP_DTYPE.names:
            h[f] = arr[f]
        h["q_tx"] = arr["q_tx"] - db.tx_base[q]
        h["s_tx"] = arr["s_tx"] - db.tx_base[s]
        hs[(q, s)] = h
    hits = hits_for_post(samples, db, ora, names)
    table = post_oracle.run_pipeline(names, hits, post_oracle.default_parse_id)["tables"][(names[0], names[1])]
    rows = np.zeros(len(table), dtype=nat.ROW_DTYPE)
    for i, r in enumerate(table):
        for f in ("qgene", "qiso", "sgene", "siso", "label"):
            rows[i][f] = r[f]
        rows[i]["reverse"] = int(r["reverse"])
        h = rows[i]["hsp"]
        h["bits10"] = int(round(r["bitscore"] * 10))
        for f in ("nident", "length", "gaps", "mismatch", "gapopen", "qstart", "qend", "sstart", "send"):
            h[f] = r[f]
        h["strand"] = 1 if r["sstrand"] == "minus" else 0
        rows[i]["hsp"] = h
    us = (sum(r["nident"] for r in table), sum(r["length"] - r["gaps"] for r in table))
    return {"labels": names, "pairs": {(0, 1): {"hsps": hs, "rows": rows, "usums": us}},
            "symmetric": False, "dust": (20, 64, 1)}


@pytest.mark.parametrize("seed", [3, 8])
def test_fast_pair_check_equals_plain(seed):
    from rna_clique_amd.simulate import simulate
    samples, _ = simulate(2, 300, seed=seed, p_iso2=0.3, indel_rate=0.003, polya=(0.3, 10, 40))
    db = OracleDB(samples)
    ora = {(q, s): db.align(q, s, 28, 108, 1e-99, False, (20, 64, 1)) for q, s in ((0, 1), (1, 0))}
    names = [s.name for s in samples]
    cap = _capture_from_oracle(samples, db, ora, names)
    assert len(cap["pairs"][(0, 1)]["rows"]) > 100
    assert compare_pair(cap, samples, 0, 1, db, ora) == []
    assert compare_pair_fast(cap, samples, 0, 1, db, ora) == []
    # one field off in a table row, an HSP, the sums: both checks say so
    rows = cap["pairs"][(0, 1)]["rows"]
    rows[57]["hsp"]["nident"] += 1
    for check in (compare_pair, compare_pair_fast):
        assert any("first differing row" in m for m in check(cap, samples, 0, 1, db, ora))
    rows[57]["hsp"]["nident"] -= 1
    rows[12]["label"] += 1
    assert any("first differing row" in m for m in compare_pair_fast(cap, samples, 0, 1, db, ora))
    rows[12]["label"] -= 1
    cap["pairs"][(0, 1)]["hsps"][(1, 0)][3]["send"] += 1
    assert any("HSP 3" in m for m in compare_pair_fast(cap, samples, 0, 1, db, ora))
    cap["pairs"][(0, 1)]["hsps"][(1, 0)][3]["send"] -= 1
    cap["pairs"][(0, 1)]["rows"] = rows[:-1]
    assert any("rows on GPU" in m for m in compare_pair_fast(cap, samples, 0, 1, db, ora))
    cap["pairs"][(0, 1)]["rows"] = rows
    cap["pairs"][(0, 1)]["usums"] = (cap["pairs"][(0, 1)]["usums"][0] + 1, cap["pairs"][(0, 1)]["usums"][1])
    assert any("unfiltered sums" in m for m in compare_pair_fast(cap, samples, 0, 1, db, ora))
