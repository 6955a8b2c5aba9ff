"""Parity checks between the native engine and the CPU oracles.

TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench.py).
The engine is the thing checked; the oracles (align_oracle.c for the
alignment restatement, post_oracle.py pinned to the reference for the rest)
are the checkers.
"""
from __future__ import annotations

import itertools

import numpy as np

from . import post_oracle
from .align import OracleDB

INT_FIELDS = ["qstart", "qend", "sstart", "send", "length", "nident",
              "mismatch", "gaps", "gapopen", "score_half", "bits10", "strand"]
ROW_COMPARE = ["label", "qgene", "qiso", "sgene", "siso", "reverse", "bitscore",
               "nident", "length", "gaps", "mismatch", "gapopen", "qstart",
               "qend", "sstart", "send", "sstrand"]


def oracle_all_hsps(db: OracleDB, n_samples, word_size=28, xdrop_half=108,
                    evalue=1e-99, symmetric=False, dust=None, threads=None):
    """Every directed search (q, s), q != s, with the C oracle -- run on a
    thread pool (ctypes releases the GIL; the oracle keeps no global state)."""
    from concurrent.futures import ThreadPoolExecutor
    perms = list(itertools.permutations(range(n_samples), 2))
    run = lambda qs: db.align(qs[0], qs[1], word_size, xdrop_half, evalue, symmetric, dust)  # noqa: E731
    with ThreadPoolExecutor(threads or oracle_threads()) as ex:
        return dict(zip(perms, ex.map(run, perms)))


def oracle_threads():
    """Worker threads for the oracle in tests: the cores this process may
    use, at most 16 (the GPU box's CPU share for test runs)."""
    return max(1, min(16, usable_cores()["cores"]))


def usable_cores():
    """The CPUs this process may run on: its affinity mask, and the cgroup
    CPU quota when one is set (cgroup v2 cpu.max). {"cores": min of both,
    "affinity": n, "quota": q or None}."""
    import math
    import os
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q != "max":
            quota = max(1, math.ceil(int(q) / int(p)))
    except (OSError, ValueError):
        pass
    return {"cores": max(1, min(aff, quota or aff)), "affinity": aff, "quota": quota}


def diff_hsps(eng, ora, db: OracleDB, q, s):
    """Engine HSPs of search (q, s) (transcript indices local to the samples)
    vs oracle HSPs (global transcript indices), every integer field, in order
    (column-wise over the arrays). Returns a list of messages."""
    msgs = []
    qb, sb = db.tx_base[q], db.tx_base[s]
    if len(eng) != len(ora):
        msgs.append(f"search {q}->{s}: {len(eng)} HSPs on GPU vs {len(ora)} in oracle")
    m = min(len(eng), len(ora))
    if not m:
        return msgs
    a, b = eng[:m], ora[:m]
    ea = np.stack([a["q_tx"].astype(np.int64) + qb, a["s_tx"].astype(np.int64) + sb] +
                  [a[f].astype(np.int64) for f in INT_FIELDS], 1)
    eb = np.stack([b["q_tx"].astype(np.int64), b["s_tx"].astype(np.int64)] +
                  [b[f].astype(np.int64) for f in INT_FIELDS], 1)
    bad = np.flatnonzero((ea != eb).any(1))
    if len(bad):
        i = int(bad[0])
        msgs.append(f"search {q}->{s} HSP {i}: GPU {ea[i].tolist()} vs oracle {eb[i].tolist()}")
    return msgs


def _ids(s):
    return s.ids() if callable(s.ids) else s.ids


def hits_for_post(samples, db: OracleDB, hsps_by_search, names=None):
    """Oracle HSP arrays -> BLAST-tabular dicts keyed by sample labels
    (`names`, default each sample's .name)."""
    names = names or [s.name for s in samples]
    ids = [_ids(s) for s in samples]
    out = {}
    for (q, s), arr in hsps_by_search.items():
        rows = []
        for h in arr:
            qt = int(h["q_tx"]) - db.tx_base[q]
            st = int(h["s_tx"]) - db.tx_base[s]
            rows.append({
                "qseqid": ids[q][qt], "sseqid": ids[s][st],
                "pident": 0.0, "length": int(h["length"]),
                "mismatch": int(h["mismatch"]), "gapopen": int(h["gapopen"]),
                "qstart": int(h["qstart"]), "qend": int(h["qend"]),
                "sstart": int(h["sstart"]), "send": int(h["send"]),
                "evalue": float(h["evalue"]), "bitscore": int(h["bits10"]) / 10.0,
                "gaps": int(h["gaps"]), "nident": int(h["nident"]),
                "sstrand": "minus" if int(h["strand"]) else "plus"})
        out[(names[q], names[s])] = rows
    return out


def engine_rows_as_dicts(rows):
    out = []
    for r in rows:
        h = r["hsp"]
        out.append({
            "label": int(r["label"]), "qgene": int(r["qgene"]), "qiso": int(r["qiso"]),
            "sgene": int(r["sgene"]), "siso": int(r["siso"]),
            "reverse": bool(r["reverse"]), "bitscore": int(h["bits10"]) / 10.0,
            "nident": int(h["nident"]), "length": int(h["length"]),
            "gaps": int(h["gaps"]), "mismatch": int(h["mismatch"]),
            "gapopen": int(h["gapopen"]), "qstart": int(h["qstart"]),
            "qend": int(h["qend"]), "sstart": int(h["sstart"]), "send": int(h["send"]),
            "sstrand": "minus" if int(h["strand"]) else "plus"})
    return out


def diff_rows(eng_rows, ora_rows, tag=""):
    a = [[r[k] for k in ROW_COMPARE] for r in engine_rows_as_dicts(eng_rows)]
    b = [[r[k] for k in ROW_COMPARE] for r in ora_rows]
    if a == b:
        return []
    msgs = [f"{tag}: {len(a)} rows on GPU vs {len(b)} in oracle"]
    for x, y in zip(a, b):
        if x != y:
            msgs.append(f"{tag}: first differing row GPU {x} vs oracle {y}")
            break
    return msgs


def full_check(engine, samples, word_size=28, xdrop_half=108, evalue=1e-99,
               top_matches=1, keep_all=True, check_hsps=True):
    """Engine (already run) vs oracles on the same samples, in the engine's
    alignment mode (independent directed searches or spec 5b; DUST or not).
    Returns messages (empty = bit-exact parity) and a small summary dict."""
    db = OracleDB(samples)
    N = len(samples)
    ora = oracle_all_hsps(db, N, word_size, xdrop_half, evalue,
                          getattr(engine, "symmetric", False), getattr(engine, "dust", None))
    msgs = []
    if check_hsps:
        for (q, s), arr in ora.items():
            msgs += diff_hsps(engine.hsps(q, s), arr, db, q, s)
    names = list(getattr(engine, "labels", None) or [s.name for s in samples])
    hits = hits_for_post(samples, db, ora, names)
    res = post_oracle.run_pipeline(names, hits, post_oracle.default_parse_id,
                                   top_matches, keep_all)
    for a in range(N):
        for b in range(a + 1, N):
            msgs += diff_rows(engine.pair_rows(a, b), res["tables"][(names[a], names[b])],
                              f"pair {a},{b}")
    e_edges = engine.edges()
    eng_edges = sorted(tuple(sorted(((names[e["sample_a"]], int(e["gene_a"])),
                                     (names[e["sample_b"]], int(e["gene_b"])))))
                       for e in e_edges)
    ora_edges = sorted(res["edges"])
    if eng_edges != ora_edges:
        msgs.append(f"edges: {len(eng_edges)} on GPU vs {len(ora_edges)} in oracle")
    s_, g_ = engine.ideal_nodes()
    eng_valid = sorted((names[a], int(b)) for a, b in zip(s_, g_))
    if eng_valid != sorted(res["valid"]):
        msgs.append(f"ideal nodes: {len(eng_valid)} on GPU vs {len(res['valid'])} in oracle")
    st = engine.stats()
    if st["sample_count"] != res["sample_count"]:
        msgs.append(f"sample_count {st['sample_count']} vs {res['sample_count']}")
    num, den = engine.pair_sums()
    for (ta, tb), (n_, d_) in res["sums"].items():
        a, b = names.index(ta), names.index(tb)
        if (int(num[a, b]), int(den[a, b])) != (n_, d_):
            msgs.append(f"sums {ta},{tb}: GPU {(int(num[a, b]), int(den[a, b]))} vs {(n_, d_)}")
    ok_matrix = None
    try:
        labels_o, mat_o = post_oracle.distance_matrix(names, res["sums"])
        labels_e, mat_e = engine.distance()
        if labels_e != labels_o or not np.array_equal(mat_e, np.array(mat_o)):
            msgs.append("distance matrix differs")
        ok_matrix = mat_e
    except post_oracle.NoIdealComponentsError:
        try:
            engine.distance()
            msgs.append("engine produced a matrix where the reference raises NoIdealComponentsError")
        except Exception:
            pass
    summary = {"hsps": int(sum(len(v) for v in ora.values())),
               "edges": len(ora_edges), "ideal_nodes": len(res["valid"]),
               "stats": st, "matrix": ok_matrix}
    return msgs, summary


def capture_pairs(engine, pairs):
    """The engine's side of check_pairs, copied to the host (so that the
    engine can be closed before the oracle finishes): per pair (a, b) both
    directed searches' HSPs, the gene matches table rows and the unfiltered
    sums. The engine must have its graph phase done (pair_sums)."""
    num, den = engine.pair_sums(unfiltered=True)
    out = {}
    for a, b in pairs:
        out[(a, b)] = {"hsps": {(0, 1): engine.hsps(a, b), (1, 0): engine.hsps(b, a)},
                       "rows": engine.pair_rows(a, b), "usums": (int(num[a, b]), int(den[a, b]))}
    return {"labels": list(engine.labels), "pairs": out,
            "symmetric": getattr(engine, "symmetric", False), "dust": getattr(engine, "dust", None)}


FAST_ROW_COMPARE = [("label", "label"), ("qgene", "qgene"), ("qiso", "qiso"), ("sgene", "sgene"),
                    ("siso", "siso"), ("reverse", "reverse"), ("bits10", "bits"), ("nident", "nident"),
                    ("length", "length"), ("gaps", "gaps"), ("mismatch", "mismatch"), ("gapopen", "gapopen"),
                    ("qstart", "qstart"), ("qend", "qend"), ("sstart", "sstart"), ("send", "send"),
                    ("strand", "strand")]


def diff_rows_fast(eng_rows, table, tag=""):
    """diff_rows over arrays: engine rows vs post_fast.match_table's columns
    (the same fields as ROW_COMPARE; bit scores as bits10)."""
    n, m = len(eng_rows), len(table["label"])
    msgs = [] if n == m else [f"{tag}: {n} rows on GPU vs {m} in oracle"]
    k = min(n, m)
    if not k:
        return msgs
    h = eng_rows["hsp"]
    ga = np.stack([(h[f] if f in h.dtype.names else eng_rows[f])[:k].astype(np.int64) for f, _ in FAST_ROW_COMPARE], 1)
    gb = np.stack([table[t][:k].astype(np.int64) for _, t in FAST_ROW_COMPARE], 1)
    bad = np.flatnonzero((ga != gb).any(1))
    if len(bad):
        i = int(bad[0])
        msgs.append(f"{tag}: first differing row GPU {ga[i].tolist()} vs oracle {gb[i].tolist()} "
                    f"({[f for f, _ in FAST_ROW_COMPARE]})")
    return msgs


def compare_pair_fast(cap, samples, a, b, db, ora, top_matches=1, keep_all=True):
    """compare_pair with the vectorised table restatement (oracle/post_fast.py,
    checked against post_oracle and the reference's fixtures on the CPU): the
    check of a full-size pair takes well under a second of Python instead of
    ~10 s."""
    from . import post_fast
    got = cap["pairs"][(a, b)]
    msgs = []
    for (q, s), arr in ora.items():
        msgs += [f"pair {a},{b}: {m}" for m in diff_hsps(got["hsps"][(q, s)], arr, db, q, s)]
    ids = [post_fast.parsed_ids(samples[a], post_oracle.default_parse_id),
           post_fast.parsed_ids(samples[b], post_oracle.default_parse_id)]
    # the forward search of the table is query = t2 (local 1), subject = t1
    fwd = post_fast.rows_from_hsps(ora[(1, 0)], db.tx_base[1], db.tx_base[0], ids[1], ids[0])
    rev = post_fast.rows_from_hsps(ora[(0, 1)], db.tx_base[0], db.tx_base[1], ids[0], ids[1])
    table = post_fast.match_table(fwd, rev, top_matches, keep_all)
    msgs += diff_rows_fast(got["rows"], table, f"pair {a},{b}")
    want = (int(table["nident"].sum()), int((table["length"] - table["gaps"]).sum()))
    if got["usums"] != want:
        msgs.append(f"pair {a},{b}: unfiltered sums {got['usums']} vs {want}")
    return msgs


def compare_pair(cap, samples, a, b, db, ora, top_matches=1, keep_all=True):
    """A captured pair (capture_pairs) against the oracle's two directed
    searches of it: db = OracleDB([samples[a], samples[b]]), ora = {(0, 1):
    db.align(0, 1, ...), (1, 0): db.align(1, 0, ...)}. HSPs bit for bit, then
    the pair's table through the pinned post-alignment oracle and its
    unfiltered sums. Returns messages (empty = parity)."""
    got = cap["pairs"][(a, b)]
    names = cap["labels"]
    msgs = []
    for (q, s), arr in ora.items():
        msgs += [f"pair {a},{b}: {m}" for m in diff_hsps(got["hsps"][(q, s)], arr, db, q, s)]
    pn = [names[a], names[b]]
    hits = hits_for_post([samples[a], samples[b]], db, ora, pn)
    out = post_oracle.run_pipeline(pn, hits, post_oracle.default_parse_id, top_matches, keep_all)
    table = out["tables"][(pn[0], pn[1])]
    msgs += diff_rows(got["rows"], table, f"pair {a},{b}")
    want = (sum(r["nident"] for r in table), sum(r["length"] - r["gaps"] for r in table))
    if got["usums"] != want:
        msgs.append(f"pair {a},{b}: unfiltered sums {got['usums']} vs {want}")
    return msgs


def check_pairs(engine, samples, pairs, word_size=28, xdrop_half=108, evalue=1e-99,
                top_matches=1, keep_all=True, threads=None):
    """Bit-exact check of selected sample pairs of a (large) engine run: for
    each pair (a, b), both directed searches with the oracle on the two samples
    alone (a pair's HSPs and gene matches table depend on nothing else), then
    the pair's table through the pinned post-alignment oracle, and the pair's
    unfiltered sums. Returns messages (empty = parity)."""
    from concurrent.futures import ThreadPoolExecutor
    cap = capture_pairs(engine, pairs)
    sym, dust = cap["symmetric"], cap["dust"]
    dbs = {(a, b): OracleDB([samples[a], samples[b]]) for a, b in pairs}
    jobs = [(a, b, q, s) for a, b in pairs for q, s in ((0, 1), (1, 0))]
    run = lambda j: dbs[j[:2]].align(j[2], j[3], word_size, xdrop_half, evalue, sym, dust)  # noqa: E731
    with ThreadPoolExecutor(threads or oracle_threads()) as ex:
        res = dict(zip(jobs, ex.map(run, jobs)))
    msgs = []
    for a, b in pairs:
        ora = {(0, 1): res[(a, b, 0, 1)], (1, 0): res[(a, b, 1, 0)]}
        msgs += compare_pair_fast(cap, samples, a, b, dbs[(a, b)], ora, top_matches, keep_all)
    return msgs
