"""CPU oracle for the post-alignment stage (RBH table -> graph -> ideal filter
-> distance matrix). TEST INFRASTRUCTURE ONLY: imported by tests/, by
`__graft_entry__.smoke()` and by bench.py's cpu_baseline leg, as the checker.
The product (rna_clique_amd + librcgpu.so) never imports it.

Plain-Python restatement of the reference, one function per reference step:

  highest_bitscores         find_homologs.py:135-164 (pandas groupby+nlargest)
  match_table               find_homologs.py:215-302 (HomologFinder.get_match_table)
  build_graph               build_graph.py:40-68
  ideal_components          filtered_distance.py:25-39, graph.py:9-24
  sample_count              filtered_distance.py:171-182
  restricted rows / sums    filtered_distance.py:66-124, similarity_computer.py:21-42
  distance_matrix           similarity_computer.py:216-345

Pinned against tests/golden/post_alignment.json (captured from the reference
itself by tests/golden/make_golden.py).

A row is a dict with the 20 gene-matches-table columns (docs/formats.md:231-252)
plus "label" (the pandas index label the reference keeps, A7).
"""
from __future__ import annotations

import itertools
from fractions import Fraction

HSP_FIELDS = ["pident", "length", "mismatch", "gapopen", "qstart", "qend",
              "sstart", "send", "evalue", "bitscore", "gaps", "nident",
              "sstrand"]


class NoIdealComponentsError(Exception):
    """filtered_distance.py:126-127."""


def highest_bitscores(rows, n=1, key=("qgene",), keep="all"):
    """groupby(key)['bitscore'].nlargest(n, keep) -> rows (find_homologs.py:135-164).

    Groups come out in sorted key order; inside a group rows are in descending
    bitscore with ties in frame order (pandas' stable selection). keep="all"
    keeps every row >= the n-th largest value (duplicates counted).
    """
    groups = {}
    for r in rows:
        groups.setdefault(tuple(r[k] for k in key), []).append(r)
    out = []
    for gk in sorted(groups):
        g = groups[gk]
        order = sorted(range(len(g)), key=lambda i: -g[i]["bitscore"])
        if keep == "all":
            if len(g) <= n:
                take = order
            else:
                thr = g[order[n - 1]]["bitscore"]
                take = [i for i in order if g[i]["bitscore"] >= thr]
        else:  # "first"
            take = order[:n]
        out.extend(g[i] for i in take)
    return out


def parse_hits(hits, parse_id):
    """find_homologs.py:124-129: HSP rows -> rows with (q|s)(gene|iso), labelled
    by their position in the BLAST output."""
    out = []
    for label, h in enumerate(hits):
        r = {k: h[k] for k in HSP_FIELDS}
        _, qg, qi = parse_id(h["qseqid"])
        _, sg, si = parse_id(h["sseqid"])
        r.update(qgene=int(qg), qiso=int(qi), sgene=int(sg), siso=int(si),
                 label=label)
        out.append(r)
    return out


def match_table(fwd_hits, rev_hits, top_matches=1, keep_all=True):
    """HomologFinder.get_match_table (find_homologs.py:215-302).

    fwd_hits: parsed rows of the search query=t2, subject=t1 (`reverse`=False).
    rev_hits: parsed rows of the search query=t1, subject=t2 (`reverse`=True).
    Returns the final rows (qgene in t2, sgene in t1) in reference order, with
    the reference's index labels.
    """
    F = highest_bitscores(fwd_hits, top_matches, ("qgene",), "all")
    R = highest_bitscores(rev_hits, top_matches, ("qgene",), "all")
    F = [dict(r, reverse=False) for r in F]
    Rr = []
    for r in R:  # rename q<->s for seqid/gene/iso only (find_homologs.py:248-255)
        x = dict(r, reverse=True)
        x["qgene"], x["sgene"] = r["sgene"], r["qgene"]
        x["qiso"], x["siso"] = r["siso"], r["qiso"]
        Rr.append(x)
    # inner merge on (qgene, sgene), left order preserved (find_homologs.py:268-278)
    by_pair = {}
    for r in Rr:
        by_pair.setdefault((r["qgene"], r["sgene"]), []).append(r)
    ix, iy, seen_x, seen_y = [], [], set(), set()
    for f in F:
        for r in by_pair.get((f["qgene"], f["sgene"]), []):
            if f["label"] not in seen_x:
                seen_x.add(f["label"])
                ix.append(f)
            if r["label"] not in seen_y:
                seen_y.add(r["label"])
                iy.append(r)
    concat = [dict(r, label=i) for i, r in enumerate(ix + iy)]  # reset_index
    per_pair = highest_bitscores(concat, 1, ("qgene", "sgene"), "all")
    return highest_bitscores(per_pair, 1, ("qgene",),
                             "all" if keep_all else "first")


def build_graph(tables):
    """build_graph.py:40-68. tables: iterable of (ssample, qsample, rows).
    Returns (nodes, edges) with nodes (sample, gene) and undirected edges as
    sorted tuples (networkx Graph collapses duplicates)."""
    nodes, edges = set(), set()
    for ss, qs, rows in tables:
        for r in rows:
            u, v = (ss, r["sgene"]), (qs, r["qgene"])
            nodes.add(u)
            nodes.add(v)
            edges.add(tuple(sorted((u, v))))
    return nodes, edges


def components(nodes, edges):
    parent = {v: v for v in nodes}

    def find(x):
        while parent[x] != x:
            parent[x] = parent[parent[x]]
            x = parent[x]
        return x

    for u, v in edges:
        ru, rv = find(u), find(v)
        if ru != rv:
            parent[max(ru, rv)] = min(ru, rv)
    comps = {}
    for v in nodes:
        comps.setdefault(find(v), set()).add(v)
    return list(comps.values()), find


def sample_count(nodes):
    """filtered_distance.py:171-182: distinct samples among graph nodes."""
    return len({s for s, _ in nodes})


def ideal_nodes(nodes, edges, samples=None):
    """Nodes of ideal components: |V| == samples and 2|E| == |V|(|V|-1)
    (filtered_distance.py:25-39)."""
    if samples is None:
        samples = sample_count(nodes)
    comps, find = components(nodes, edges)
    ecount = {}
    for u, v in edges:
        r = find(u)
        ecount[r] = ecount.get(r, 0) + 1
    valid = set()
    for c in comps:
        r = find(next(iter(c)))
        if len(c) == samples and 2 * ecount.get(r, 0) == len(c) * (len(c) - 1):
            valid |= c
    return valid


def pair_sums(ssample, qsample, rows, valid):
    """restrict_multi + similarities_from_dfs sums (filtered_distance.py:66-124,
    similarity_computer.py:37-41): (sum nident, sum(length - gaps))."""
    num = den = 0
    for r in rows:
        if (ssample, r["sgene"]) in valid and (qsample, r["qgene"]) in valid:
            num += r["nident"]
            den += r["length"] - r["gaps"]
    return num, den


def distance_matrix(samples, sums):
    """similarity_computer.py:216-345: labels in sorted() order, diagonal 0,
    d = float(1 - Fraction(num, den)). sums: {(a, b): (num, den)} for a != b."""
    labels = sorted(samples)
    idx = {s: i for i, s in enumerate(labels)}
    n = len(labels)
    mat = [[0.0] * n for _ in range(n)]
    for (a, b), (num, den) in sums.items():
        if den == 0:
            raise NoIdealComponentsError()
        d = float(1 - Fraction(num, den))
        mat[idx[a]][idx[b]] = mat[idx[b]][idx[a]] = d
    return labels, mat


def run_pipeline(samples, hits_by_search, parse_id, top_matches=1,
                 keep_all=True):
    """Whole post-alignment path for samples in input order.

    hits_by_search[(query_sample, subject_sample)] -> list of HSP dicts
    (qseqid, sseqid + HSP_FIELDS). Mirrors find_all_pairs (combinations in
    input order, t1 = ssample, t2 = qsample) -> build_graph -> SampleSimilarity.
    """
    tables = {}
    for t1, t2 in itertools.combinations(samples, 2):
        fwd = parse_hits(hits_by_search.get((t2, t1), []), parse_id)
        rev = parse_hits(hits_by_search.get((t1, t2), []), parse_id)
        rows = match_table(fwd, rev, top_matches, keep_all)
        for r in rows:
            r["ssample"], r["qsample"] = t1, t2
        tables[(t1, t2)] = rows
    nodes, edges = build_graph((a, b, r) for (a, b), r in tables.items())
    sc = sample_count(nodes)
    valid = ideal_nodes(nodes, edges, sc)
    sums = {k: pair_sums(k[0], k[1], rows, valid) for k, rows in tables.items()}
    return {"tables": tables, "nodes": nodes, "edges": edges,
            "sample_count": sc, "valid": valid, "sums": sums}


_DEFAULT_RE = None


def default_parse_id(s):
    """transcripts.py:8 default regex: cov float, gene int, isoform int."""
    import re
    global _DEFAULT_RE
    if _DEFAULT_RE is None:
        _DEFAULT_RE = re.compile(r"^.*cov_([0-9]+(?:\.[0-9]+))_g([0-9]+)_i([0-9]+)")
    m = _DEFAULT_RE.search(s)
    if m is None:
        raise ValueError(f"Could not parse transcript ID {s}.")
    return float(m.group(1)), int(m.group(2)), int(m.group(3))
