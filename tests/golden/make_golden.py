"""Capture golden vectors for the post-alignment stage from the reference.

TEST INFRASTRUCTURE ONLY -- run in the build container, where /root/reference
exists:

    python tests/golden/make_golden.py

It builds synthetic BLAST-style HSP tables (outfmt 6 columns + gaps nident
sstrand, as `find_homologs.py:124,209` request), feeds them through the
reference's own code (stub-imported by ref_harness.py):

  HomologFinder.get_match_table      find_homologs.py:215-302
  (ssample/qsample labelling)        find_all_pairs.py:82-86
  build_graph                        build_graph.py:40-68
  SampleSimilarity(...).valid        filtered_distance.py:184-196
  SampleSimilarity.restricted        filtered_distance.py:199-210
  get_dissimilarity_df               similarity_computer.py:367-375

and writes inputs + outputs to tests/golden/post_alignment.json. The fixture is
data (inputs and expected outputs); no reference source is copied.
"""
from __future__ import annotations

import itertools
import json
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ref_harness  # noqa: E402

HSP_COLUMNS = ["qseqid", "sseqid", "pident", "length", "mismatch", "gapopen",
               "qstart", "qend", "sstart", "send", "evalue", "bitscore",
               "gaps", "nident", "sstrand"]
TABLE_COLUMNS = ["pident", "length", "mismatch", "gapopen", "qstart", "qend",
                 "sstart", "send", "evalue", "bitscore", "gaps", "nident",
                 "sstrand", "qgene", "qiso", "sgene", "siso", "reverse",
                 "ssample", "qsample"]


def _tx_name(gene, iso, cov):
    return f"NODE_{gene * 10 + iso}_length_1000_cov_{cov:.6f}_g{gene}_i{iso}"


def make_case(seed, n_samples, n_families, p_present=0.92, p_iso2=0.2,
              p_paralog=0.15, p_asym=0.2, p_minus=0.1, p_drop=0.03):
    """Synthetic HSP tables for every ordered sample pair.

    Families play the role of orthologous gene groups; paralog hits, isoforms,
    F/R bitscore asymmetry and dropped hits create ties, non-ideal components
    and missing pairs.
    """
    rng = np.random.default_rng(seed)
    samples = [f"out/od1/T{i}_top.fasta" for i in range(n_samples)]
    txs = {}       # sample -> list of (gene, iso, family, cov)
    fam_gene = {}  # (sample, family) -> gene
    for si, s in enumerate(samples):
        genes = rng.choice(np.arange(1, 10 * n_families + 1), size=n_families,
                           replace=False)
        lst = []
        for f in range(n_families):
            if rng.random() > p_present:
                continue
            g = int(genes[f])
            fam_gene[(s, f)] = g
            niso = 2 if rng.random() < p_iso2 else 1
            for iso in range(1, niso + 1):
                lst.append((g, iso, f, float(rng.uniform(1, 1000))))
        txs[s] = lst
    # a symmetric "true" bitscore per (family, unordered sample pair)
    base = {}
    for f in range(n_families):
        for a, b in itertools.combinations(samples, 2):
            base[(f, a, b)] = base[(f, b, a)] = float(rng.integers(300, 340) * 3)
    hits = {}
    for q, s in itertools.permutations(samples, 2):
        rows = []
        for (g, iso, f, cov) in txs[q]:
            qrows = []
            if (s, f) in fam_gene:
                sg = fam_gene[(s, f)]
                for (g2, iso2, f2, cov2) in txs[s]:
                    if g2 != sg:
                        continue
                    if rng.random() < p_drop:
                        continue
                    bits = base[(f, q, s)]
                    if rng.random() < p_asym:
                        bits += float(rng.choice([-3.0, -1.0, 1.0, 2.0]))
                    if iso2 > 1 or iso > 1:
                        bits -= float(rng.choice([0.0, 0.0, 1.0]))
                    qrows.append((g2, iso2, cov2, bits))
            if txs[s] and rng.random() < p_paralog:
                g2, iso2, f2, cov2 = txs[s][int(rng.integers(len(txs[s])))]
                top = max([r[3] for r in qrows], default=900.0)
                bits = top if rng.random() < 0.35 else top - float(rng.integers(1, 200))
                qrows.append((g2, iso2, cov2, bits))
            qrows.sort(key=lambda r: -r[3])
            for (g2, iso2, cov2, bits) in qrows:
                length = int(rng.integers(400, 1600))
                gaps = int(rng.choice([0, 0, 0, 1, 2, 5]))
                mism = int(rng.integers(0, 30))
                nident = length - gaps - mism
                minus = rng.random() < p_minus
                qs = int(rng.integers(1, 50))
                ss = int(rng.integers(1, 50))
                rows.append({
                    "qseqid": _tx_name(g, iso, cov),
                    "sseqid": _tx_name(g2, iso2, cov2),
                    "pident": round(100.0 * nident / length, 3),
                    "length": length, "mismatch": mism,
                    "gapopen": min(gaps, int(rng.integers(0, 3))),
                    "qstart": qs, "qend": qs + length - 1,
                    "sstart": ss + length - 1 if minus else ss,
                    "send": ss if minus else ss + length - 1,
                    "evalue": 0.0, "bitscore": bits, "gaps": gaps,
                    "nident": nident, "sstrand": "minus" if minus else "plus",
                })
        hits[(q, s)] = rows
    return samples, hits


def run_reference(samples, hits, top_matches, keep_all):
    import pandas as pd
    ref = ref_harness.reference_modules()
    ref_harness.FAKE_BLAST_DB.clear()
    for (q, s), rows in hits.items():
        ref_harness.FAKE_BLAST_DB[(q, s)] = pd.DataFrame(rows, columns=HSP_COLUMNS)
    parser = ref.transcripts.TranscriptID.parser_from_re(ref.transcripts.default_gene_re)
    out = {"tables": {}, "errors": {}}
    tables = []
    q1_ok = True
    for t1, t2 in itertools.combinations(samples, 2):
        hf = ref.find_homologs.HomologFinder(parser, top_matches, 1e-99, keep_all)
        try:
            table = hf.get_match_table(t1, t2)
        except Exception as e:  # reference failure is recorded, not hidden
            out["errors"][f"{t1}|{t2}"] = f"{type(e).__name__}: {e}"
            continue
        # find_all_pairs.py:82-86
        table["ssample"] = str(t1)
        table["qsample"] = str(t2)
        rows = []
        for label, r in zip(table.index.tolist(), table.to_dict("records")):
            rows.append([int(label)] + [
                (bool(r[c]) if c == "reverse" else
                 (float(r[c]) if c in ("pident", "evalue", "bitscore") else
                  (str(r[c]) if c in ("sstrand", "ssample", "qsample") else int(r[c]))))
                for c in TABLE_COLUMNS])
        out["tables"][f"{t1}|{t2}"] = rows
        if len(table) and 0 not in table.index:
            q1_ok = False  # mapping_from_dfs would raise KeyError: 0 (Q1)
        tables.append((t1, t2, table))
    out["mapping_from_dfs_ok"] = q1_ok
    if out["errors"]:
        return out
    graph = ref.build_graph.build_graph(t for (_, _, t) in tables)
    edges = sorted(sorted([list(u), list(v)]) for u, v in graph.edges)
    out["edges"] = edges
    out["nodes"] = sorted(list(n) for n in graph.nodes)
    # Pair keys taken from the pair itself (Q1: mapping_from_dfs uses a label
    # lookup that fails when row 0 was filtered out).
    sim = ref.filtered_distance.SampleSimilarity(
        graph, [(frozenset((t2, t1)), t) for (t1, t2, t) in tables])
    out["sample_count"] = int(sim.sample_count)
    out["valid"] = sorted([str(s), int(g)] for s, g in
                          sim.valid.itertuples(index=False))
    sums = {}
    for t1, t2, t in tables:
        r = sim.restricted(t)
        sums[f"{t1}|{t2}"] = [int(r["nident"].sum()),
                              int(r["length"].sum() - r["gaps"].sum())]
    out["sums"] = sums
    try:
        df = sim.get_dissimilarity_df()
        out["matrix"] = {"labels": [str(x) for x in df.index],
                         "values": df.values.tolist()}
    except ref.filtered_distance.NoIdealComponentsError:
        out["matrix"] = None
        out["errors"]["matrix"] = "NoIdealComponentsError"
    return out


def no_ideal_case():
    """3 samples whose only component has 4 vertices: no ideal components,
    so the reference raises NoIdealComponentsError (filtered_distance.py:242-247)."""
    A, B, C = [f"out/od1/T{i}_top.fasta" for i in range(3)]

    def row(qg, sg, bits):
        return {"qseqid": _tx_name(qg, 1, 5.0), "sseqid": _tx_name(sg, 1, 5.0),
                "pident": 99.0, "length": 500, "mismatch": 5, "gapopen": 0,
                "qstart": 1, "qend": 500, "sstart": 1, "send": 500,
                "evalue": 0.0, "bitscore": bits, "gaps": 0, "nident": 495,
                "sstrand": "plus"}
    hits = {(B, A): [row(2, 1, 900.0)], (A, B): [row(1, 2, 900.0)],
            (C, B): [row(3, 2, 900.0)], (B, C): [row(2, 3, 900.0)],
            (C, A): [row(4, 1, 900.0)], (A, C): [row(1, 4, 900.0)]}
    return [A, B, C], hits


CASES = [
    # (seed, samples, families)
    (11, 3, 12),
    (12, 4, 25),
    (13, 4, 40),
    (14, 5, 30),
    (15, 3, 8),
    (16, 6, 20),
]
PARAMS = [(1, True), (1, False), (2, True)]


def _compact(hits):
    return {f"{q}|{s}": [[r[c] for c in HSP_COLUMNS] for r in rows]
            for (q, s), rows in hits.items()}


def main():
    fixtures = []
    for seed, ns, nf in CASES:
        samples, hits = make_case(seed, ns, nf)
        for top_matches, keep_all in PARAMS:
            res = run_reference(samples, hits, top_matches, keep_all)
            fixtures.append({
                "seed": seed, "top_matches": top_matches, "keep_all": keep_all,
                "samples": samples,
                "hits": _compact(hits),
                "expected": res,
            })
    # A case with one empty directed search and one with no ideal components.
    samples, hits = make_case(21, 3, 6, p_present=1.0)
    q, s = samples[2], samples[0]
    hits[(q, s)] = []
    fixtures.append({"seed": 21, "top_matches": 1, "keep_all": True,
                     "samples": samples,
                     "hits": _compact(hits),
                     "expected": run_reference(samples, hits, 1, True)})
    samples, hits = no_ideal_case()
    fixtures.append({"seed": 22, "top_matches": 1, "keep_all": True,
                     "samples": samples,
                     "hits": _compact(hits),
                     "expected": run_reference(samples, hits, 1, True)})
    path = os.path.join(HERE, "post_alignment.json")
    with open(path, "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py",
                   "reference": "actapia/rna_clique (stub-imported post-alignment modules)",
                   "columns": ["label"] + TABLE_COLUMNS,
                   "hsp_columns": HSP_COLUMNS,
                   "fixtures": fixtures}, f, separators=(",", ":"))
    print(f"wrote {path}: {len(fixtures)} fixtures, "
          f"{os.path.getsize(path) / 1e3:.0f} kB")
    for fx in fixtures:
        e = fx["expected"]
        print(fx["seed"], fx["top_matches"], fx["keep_all"], "tables",
              sum(len(v) for v in e["tables"].values()), "errors", e["errors"],
              "q1ok", e.get("mapping_from_dfs_ok"),
              "valid", len(e.get("valid", [])))


if __name__ == "__main__":
    main()
