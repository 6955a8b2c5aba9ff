"""Vectorised (numpy) restatement of the gene matches table step, for checking
large sample pairs. TEST INFRASTRUCTURE ONLY (tests/, bench.py's
cpu_baseline leg): the checker, never the product.

Same semantics as post_oracle.match_table (find_homologs.py:215-302), which
stays the plain restatement pinned by the reference's golden fixtures;
tests/test_oracle_golden.py checks this one on the same fixtures and against
post_oracle on randomised tie-heavy inputs. A row set is a dict of equal-length
numpy arrays ("columns"), in BLAST output order; "bits" is the bit score (or
the oracle's bits10, which orders the same).

  highest_bitscores   find_homologs.py:135-164: groupby(key) in sorted key
                      order, inside a group descending bitscore with ties in
                      frame order (pandas' stable nlargest); keep="all" keeps
                      every row >= the n-th largest, keep="first" the first n
  match_table         F = top rows per qgene of the forward search (query t2),
                      R = those of the reverse search with q/s swapped; the
                      inner merge on (qgene, sgene) keeps the left order: the
                      F rows with a partner, then the R rows with a partner in
                      the order the merge first reaches them; best per
                      (qgene, sgene), then best per qgene
"""
from __future__ import annotations

import numpy as np

ROW_FIELDS = ("qgene", "qiso", "sgene", "siso", "bits", "nident", "length", "gaps", "mismatch",
              "gapopen", "qstart", "qend", "sstart", "send", "strand")


def _take(rows, idx):
    return {k: v[idx] for k, v in rows.items()}


def highest_bitscores(rows, n=1, key=("qgene",), keep="all"):
    m = len(rows["bits"])
    if m == 0:
        return _take(rows, np.zeros(0, dtype=np.int64))
    pos = np.arange(m)
    order = np.lexsort((pos, -rows["bits"]) + tuple(rows[k] for k in reversed(key)))
    kk = [rows[k][order] for k in key]
    bits = rows["bits"][order]
    newg = np.ones(m, dtype=bool)
    newg[1:] = np.zeros(m - 1, dtype=bool)
    for a in kk:
        newg[1:] |= a[1:] != a[:-1]
    gid = np.cumsum(newg) - 1
    start = np.flatnonzero(newg)
    size = np.diff(np.append(start, m))
    rank = pos - start[gid]
    if keep == "all":
        big = size[gid] > n
        thr = bits[np.minimum(start + n - 1, m - 1)][gid]
        sel = ~big | (bits >= thr)
    else:
        sel = rank < n
    return _take(rows, order[sel])


def match_table(fwd, rev, top_matches=1, keep_all=True):
    """fwd: the search query = t2, subject = t1; rev: query = t1, subject =
    t2 (both with a "label" column = their output position). Returns the final
    rows (qgene in t2, sgene in t1) with "label" = the reference's index label
    and "reverse"."""
    F = highest_bitscores(fwd, top_matches, ("qgene",), "all")
    R = highest_bitscores(rev, top_matches, ("qgene",), "all")
    F["reverse"] = np.zeros(len(F["bits"]), dtype=bool)
    Rr = dict(R)
    Rr["qgene"], Rr["sgene"] = R["sgene"], R["qgene"]
    Rr["qiso"], Rr["siso"] = R["siso"], R["qiso"]
    Rr["reverse"] = np.ones(len(R["bits"]), dtype=bool)
    nf, nr = len(F["bits"]), len(Rr["bits"])
    keys = np.stack([np.concatenate([F["qgene"], Rr["qgene"]]), np.concatenate([F["sgene"], Rr["sgene"]])], 1)
    if nf + nr:
        _, inv = np.unique(keys, axis=0, return_inverse=True)
        inv = inv.reshape(-1)
        nk = int(inv.max()) + 1
    else:
        inv, nk = np.zeros(0, dtype=np.int64), 0
    fk, rk = inv[:nf], inv[nf:]
    has_r = np.zeros(nk, dtype=bool)
    has_r[rk] = True
    first_f = np.full(nk, nf, dtype=np.int64)
    np.minimum.at(first_f, fk, np.arange(nf))
    ix = np.flatnonzero(has_r[fk])
    rmatch = np.flatnonzero(first_f[rk] < nf)
    iy = rmatch[np.lexsort((rmatch, first_f[rk][rmatch]))]
    cols = set(F) & set(Rr)
    concat = {k: np.concatenate([F[k][ix], Rr[k][iy]]) for k in cols}
    concat["label"] = np.arange(len(ix) + len(iy))   # reset_index
    per_pair = highest_bitscores(concat, 1, ("qgene", "sgene"), "all")
    return highest_bitscores(per_pair, 1, ("qgene",), "all" if keep_all else "first")


def rows_from_dicts(hits, parse_id):
    """BLAST-tabular dicts (post_oracle's input) -> columns, label = position."""
    out = {k: [] for k in ROW_FIELDS}
    for h in hits:
        _, qg, qi = parse_id(h["qseqid"])
        _, sg, si = parse_id(h["sseqid"])
        out["qgene"].append(int(qg))
        out["qiso"].append(int(qi))
        out["sgene"].append(int(sg))
        out["siso"].append(int(si))
        out["bits"].append(h["bitscore"])
        for k in ROW_FIELDS[5:]:
            if k == "strand":
                out[k].append(1 if h["sstrand"] == "minus" else 0)
            else:
                out[k].append(int(h[k]))
    cols = {k: np.asarray(v, dtype=np.float64 if k == "bits" else np.int64) for k, v in out.items()}
    cols["label"] = np.arange(len(hits))
    return cols


def parsed_ids(sample, parse_id):
    """(gene, iso) arrays of a sample's transcripts, from their IDs (the
    reference parses every BLAST seqid, find_homologs.py:124-129)."""
    ids = sample.ids() if callable(sample.ids) else sample.ids
    g = np.empty(len(ids), dtype=np.int64)
    i = np.empty(len(ids), dtype=np.int64)
    for k, s in enumerate(ids):
        _, gg, ii = parse_id(s)
        g[k], i[k] = int(gg), int(ii)
    return g, i


def rows_from_hsps(arr, q_base, s_base, q_ids, s_ids):
    """Oracle HSP array of one directed search -> columns (label = output
    position). q_ids / s_ids: parsed_ids of the query and subject samples;
    q_base / s_base: the samples' first global transcript index."""
    qt = arr["q_tx"].astype(np.int64) - q_base
    st = arr["s_tx"].astype(np.int64) - s_base
    cols = {"qgene": q_ids[0][qt], "qiso": q_ids[1][qt], "sgene": s_ids[0][st], "siso": s_ids[1][st]}
    cols["bits"] = arr["bits10"].astype(np.int64)   # (bitscore = bits10 / 10: the same order)
    for k in ROW_FIELDS[5:]:
        cols[k] = arr[k].astype(np.int64)
    cols["label"] = np.arange(len(arr))
    return cols
