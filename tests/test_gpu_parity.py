"""GPU parity: the HIP path against the CPU oracles, bit for bit.

Alignment: oracle/align_oracle.c (restated megablast; parity vs BLAST itself is
unpinned), in the engine's mode: by default both directed
searches of a pair run independently with DUST on the query (blastn's
defaults); spec 5b (symmetric) and DUST off are options, tested too.
Post-alignment: oracle/post_oracle.py, itself pinned to the reference by
tests/golden/post_alignment.json -- and the engine is also run directly on
those golden HSP tables (external-alignment mode).
"""
import json
import os

import numpy as np
import pytest

from oracle.parity import full_check

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "post_alignment.json")


def _engine(**kw):
    from rna_clique_amd.engine import Engine
    return Engine(device=0, **kw)


def _run_sim(samples, **kw):
    eng = _engine(**kw)
    for s in samples:
        eng.add_sample(s.name, s.seq, s.tx_offsets, s.gene, s.iso)
    eng.run()
    return eng


@pytest.mark.parametrize("seed,taxa,genes,iso,indel", [
    (1, 3, 80, 0.0, 0.0),
    (2, 4, 150, 0.2, 0.002),
    (3, 5, 120, 0.1, 0.004),
])
def test_simulated_parity(native, seed, taxa, genes, iso, indel):
    from rna_clique_amd.simulate import simulate
    samples, _ = simulate(taxa, genes, seed=seed, p_iso2=iso, indel_rate=indel)
    eng = _run_sim(samples)
    msgs, summary = full_check(eng, samples)
    assert not msgs, "\n".join(msgs[:10])
    assert summary["hsps"] > 0 and summary["ideal_nodes"] > 0


@pytest.mark.parametrize("symmetric,dust,share", [(True, False, 1), (False, False, 1), (False, (20, 64, 1), 1),
                                                 (False, (12, 48, 3), 1), (False, False, 0),
                                                 (False, (20, 64, 1), 0)])
def test_alignment_modes(native, monkeypatch, symmetric, dust, share):
    """Both alignment modes (independent directed searches / spec 5b) and
    DUST on, off, or with other parameters, on isoforms, indels, minus-strand
    transcripts and poly-A tails. Independent searches run from one shared
    candidate set by default (share 1) or one search after the other
    (RC_SHARE=0); both must equal the oracle's two independent searches."""
    monkeypatch.setenv("RC_SHARE", str(share))
    from rna_clique_amd.simulate import simulate
    samples, _ = simulate(4, 120, seed=12, p_iso2=0.2, indel_rate=0.003, p_revcomp=0.5,
                          polya=(0.3, 10, 40))
    eng = _run_sim(samples, symmetric=symmetric, dust=dust)
    msgs, summary = full_check(eng, samples)
    assert not msgs, "\n".join(msgs[:10])
    assert summary["hsps"] > 0 and summary["ideal_nodes"] > 0
    if share and dust == (20, 64, 1):
        # this corpus has reverse-search runs no forward word finds (poly-A
        # context): the reverse pass's seeds merged into forward candidates
        assert eng.timings()["reverse_seeds"] > 0


@pytest.mark.parametrize("dust", [None, (30, 64, 1), (4, 32, 1), (11, 20, 2), (49, 64, 1)])
def test_dust_mask_parity(native, dust):
    """The GPU DUST masks (rc_dust_mask) equal the oracle's, base for base, on
    transcripts with poly-A tails, dinucleotide and triplet repeats, ambiguous
    bases inside low-complexity runs, and plain random sequence; at the
    default level and at levels that track 0, 2 and 5-9 earlier occurrences
    per triplet (the kernel's u32 and u64 state words)."""
    from oracle.align import OracleDB
    from rna_clique_amd.simulate import simulate
    samples, _ = simulate(3, 150, seed=13, polya=(0.5, 5, 120))
    rng = np.random.default_rng(3)
    motifs = [b"AC", b"CAG", b"T", b"GATA", b"ACGTTGCA", b"AAAAAAAAAAAAAAAAAAAAAAANAAAAAAAA"]
    for s in samples:
        seq = s.seq.copy()
        offs = s.tx_offsets.astype(np.int64)
        for t in rng.choice(s.n_tx, size=s.n_tx // 3, replace=False):
            a, b = int(offs[t]), int(offs[t + 1])
            m = motifs[int(rng.integers(len(motifs)))]
            ln = int(rng.integers(8, 150))
            rep = np.frombuffer((m * (ln // len(m) + 1))[:ln], dtype=np.uint8)
            if b - a > ln + 10:
                p = int(rng.integers(a, b - ln))
                seq[p:p + ln] = rep
        s.seq = seq
    eng = _run_sim(samples, dust=dust)
    db = OracleDB(samples)
    masked = 0
    for i in range(len(samples)):
        got = eng.dust_mask(i)
        want = db.dust_mask(i, *eng.dust)
        assert got.shape == want.shape
        bad = np.flatnonzero(got != want)
        assert bad.size == 0, f"sample {i}: {bad.size} bases differ, first at {bad[:5]}"
        masked += int(want.sum())
    assert masked > 1000
    if dust is not None:
        return
    msgs, _ = full_check(eng, samples)
    assert not msgs, "\n".join(msgs[:10])


def test_dust_long_repeats_across_chunks(native):
    """Low-complexity stretches of 1-4 kb inside 3-7 kb transcripts: runs
    that cross the DUST kernel's 1024-base lane chunks, and lanes whose event
    lists fill and are flushed in the middle of a scan (the events of one
    owner lane then continue in a later round). Masks base for base against
    the oracle at the default level and at a level that tracks more
    occurrences per triplet."""
    from oracle.align import OracleDB
    from rna_clique_amd.simulate import simulate
    samples, _ = simulate(2, 30, seed=29, len_uniform=(3000, 7000))
    rng = np.random.default_rng(29)
    motifs = [b"A", b"AC", b"CAG", b"GATA", b"ACGTTGCA", b"TTAGGG", b"AAAAAAAAAGAAAAAA"]
    for s in samples:
        seq = s.seq.copy()
        offs = s.tx_offsets.astype(np.int64)
        for t in range(s.n_tx):
            a, b = int(offs[t]), int(offs[t + 1])
            m = motifs[int(rng.integers(len(motifs)))]
            ln = int(rng.integers(1000, 4000))
            if b - a > ln + 100:
                p = int(rng.integers(a, b - ln))
                seq[p:p + ln] = np.frombuffer((m * (ln // len(m) + 1))[:ln], dtype=np.uint8)
        s.seq = seq
    for dust in (None, (11, 64, 1)):
        eng = _run_sim(samples, dust=dust)
        db = OracleDB(samples)
        masked = 0
        for i in range(len(samples)):
            got = eng.dust_mask(i)
            want = db.dust_mask(i, *eng.dust)
            bad = np.flatnonzero(got != want)
            assert bad.size == 0, f"dust {dust}, sample {i}: {bad.size} bases differ, first at {bad[:5]}"
            masked += int(want.sum())
        assert masked > 30000
        eng.close()


def test_isoform_rich_genes_and_repeats(native):
    """Genes with 30 isoforms in every sample plus shared poly-A tails: one
    (query gene, subject sample) pass holds thousands of seeds, more than the
    seed kernel's LDS, so the global-memory passes (and their retry with a
    larger scratch) run. Parity with DUST on and off."""
    from rna_clique_amd.simulate import simulate
    samples, _ = simulate(3, 60, seed=14, len_loc=1200, len_n=400, len_p=0.5, rich_genes=3,
                          rich_iso=30, p_iso2=0.1, polya=(0.6, 20, 60))
    for dust in (None, False):
        eng = _run_sim(samples, dust=dust)
        msgs, summary = full_check(eng, samples)
        assert not msgs, "\n".join(msgs[:10])
        assert eng.timings()["big_passes"] > 0
        eng.close()


def test_gene_with_201_isoforms(native):
    """A gene with 201 transcripts in both samples (more than the seed
    kernel's LDS isoform tables, ISO_LDS = 128, and than round 2's limit of
    127): the seed kernel reads that gene's isoform tables from HBM, its
    (gene, sample) passes run from global memory, and every HSP, table row,
    edge and distance is bit-exact vs the oracle. The reference keeps every
    isoform of a top gene (select_top_genes.py:121-127) and groups by qgene
    with no bound (find_homologs.py:130)."""
    import numpy as np
    from rna_clique_amd.simulate import simulate
    samples, _ = simulate(2, 30, seed=31, len_loc=1200, len_n=400, len_p=0.5, rich_genes=1, rich_iso=201)
    assert all(np.bincount(s.gene).max() == 201 for s in samples)
    eng = _run_sim(samples)
    msgs, summary = full_check(eng, samples)
    assert not msgs, "\n".join(msgs[:10])
    assert summary["hsps"] > 100000 and eng.timings()["big_passes"] > 0
    eng.close()


def test_simulated_parity_variants(native):
    """Minus-strand transcripts, recent paralogs (reciprocal-best-hit ties,
    non-ideal components), isoforms and indels together."""
    from rna_clique_amd.simulate import simulate
    samples, _ = simulate(5, 200, seed=15, p_iso2=0.15, indel_rate=0.002, p_revcomp=0.5,
                          p_paralog=0.08, polya=(0.2, 15, 40))
    eng = _run_sim(samples)
    msgs, summary = full_check(eng, samples)
    assert not msgs, "\n".join(msgs[:10])
    st = eng.stats()
    assert st["components"] > st["ideal_components"] > 0


@pytest.mark.parametrize("share", ["1", "0"])
def test_hsp_overflow_retry(native, monkeypatch, share):
    """A first HSP overflow buffer far too small (RC_OVF_CAP0): the engine
    redoes only extend_kernel with a larger one (the row kernels' results and
    the defer lists stand) -- same HSPs as the oracle, same statistics as a
    run without the retry."""
    from rna_clique_amd.simulate import simulate
    samples, _ = simulate(4, 150, seed=23, p_iso2=0.2, indel_rate=0.004, p_revcomp=0.5, p_paralog=0.1)
    monkeypatch.setenv("RC_SHARE", share)
    ref = _run_sim(samples)
    want = ref.stats()
    ref.close()
    monkeypatch.setenv("RC_OVF_CAP0", "8")
    eng = _run_sim(samples)
    assert eng.timings()["ext_retries"] >= 1
    assert eng.stats() == want
    msgs, summary = full_check(eng, samples)
    assert not msgs, "\n".join(msgs[:10])
    assert summary["hsps"] > 0


def test_simulated_parity_large_index(native):
    """More than 2^20 indexed positions: the onesweep-sorted index (smaller
    ones take rocPRIM's merge-sort path, sorted on all 64 bits)."""
    from rna_clique_amd.simulate import simulate
    samples, _ = simulate(3, 500, seed=41, p_iso2=0.1)
    assert sum(s.seq.size for s in samples) > 2 * (1 << 20)
    eng = _run_sim(samples)
    msgs, summary = full_check(eng, samples)
    assert not msgs, "\n".join(msgs[:10])
    assert summary["hsps"] > 0


@pytest.mark.parametrize("amb_rate", [0.002, 0.02])
def test_simulated_parity_ambiguous(native, amb_rate):
    """Non-ACGT bytes (N, IUPAC codes, either case) and lowercase bases: the
    ambiguity-mask kernels (seed and extension) against the oracle, where a
    non-ACGT base never matches and no index window contains one."""
    from rna_clique_amd.simulate import simulate
    samples, _ = simulate(4, 100, seed=31, p_iso2=0.2, indel_rate=0.002)
    rng = np.random.default_rng(5)
    junk = np.frombuffer(b"NnRYKMSWryx-", dtype=np.uint8)
    for s in samples:
        seq = s.seq.copy()
        low = rng.random(seq.size) < 0.05
        seq[low] |= 0x20
        pos = np.flatnonzero(rng.random(seq.size) < amb_rate)
        seq[pos] = junk[rng.integers(0, junk.size, pos.size)]
        s.seq = seq
    eng = _run_sim(samples)
    msgs, summary = full_check(eng, samples)
    assert not msgs, "\n".join(msgs[:10])
    assert summary["hsps"] > 0


@pytest.mark.parametrize("lens,indel", [((200, 9000), 0.002), (None, 0.03)])
def test_simulated_parity_long_and_gappy(native, lens, indel):
    """Long transcripts (past the LDS staging limit, global-memory path) and
    indel-rich pairs (wide live bands)."""
    from rna_clique_amd.simulate import simulate
    kw = {"len_uniform": lens} if lens else {}
    samples, _ = simulate(4, 60, seed=21, p_iso2=0.2, indel_rate=indel, **kw)
    eng = _run_sim(samples)
    msgs, summary = full_check(eng, samples)
    assert not msgs, "\n".join(msgs[:10])
    assert summary["hsps"] > 0
    # transcripts past the row kernels' slot run on its windowed form: none
    # is left to the one-wave kernel for its length
    tm = eng.timings()
    assert tm["defer_length"] == 0 and tm["defer_gaveup"] == 0


@pytest.mark.parametrize("words,share,amb", [(4, 1, False), (9, 1, False), (5, 0, False), (6, 1, True)])
def test_windowed_staging_exact(native, monkeypatch, words, share, amb):
    """The row kernels' windowed staging (windows of `words` u64 words, 80 to
    240 bases past the read margin: a refill every few steps) gives every HSP,
    table and distance of the whole-transcript staging: indels (wide live
    bands, the 64-lane pass resuming 32-lane extensions), minus strands,
    isoforms, poly-A tails, ambiguous bases; shared and one-by-one searches."""
    monkeypatch.setenv("RC_WIN_WORDS", str(words))
    monkeypatch.setenv("RC_SHARE", str(share))
    from rna_clique_amd.simulate import simulate
    samples, _ = simulate(4, 100, seed=23, p_iso2=0.2, indel_rate=0.004, p_revcomp=0.5, polya=(0.3, 10, 40),
                          len_loc=600, len_n=2000, len_p=0.5)
    if amb:
        rng = np.random.default_rng(7)
        for sm in samples:
            seq = sm.seq.copy()
            pos = np.flatnonzero(rng.random(seq.size) < 0.003)
            seq[pos] = ord("N")
            sm.seq = seq
    eng = _run_sim(samples)
    msgs, summary = full_check(eng, samples)
    assert not msgs, "\n".join(msgs[:10])
    tm = eng.timings()
    assert summary["hsps"] > 0 and tm["defer_length"] == 0 and (tm["ext_wide"] > 0 or not share)


@pytest.mark.parametrize("later,rows,cap,words", [("1", "64", None, None), ("1", "32", None, None),
                                                   ("1", "64", "7", None), ("0", None, None, None),
                                                   ("1", "64", None, "6")])
def test_later_seed_rounds_exact(native, monkeypatch, later, rows, cap, words):
    """Searches with a seed outside their first HSP's box (indels): the
    later-seed rounds (each round extends every such search's next seed on
    the row kernels; a finishing kernel purges and cuts) give every HSP, table
    and distance of the oracle -- with later seeds on 64-lane rows (default)
    or 32-lane rows first, with a state capacity of 7 searches (the rest run
    whole on extend_kernel), with the rounds off, and with windowed staging."""
    monkeypatch.setenv("RC_LATER", later)
    if rows:
        monkeypatch.setenv("RC_LATER_ROWS", rows)
    if cap:
        monkeypatch.setenv("RC_LATER_CAP", cap)
    if words:
        monkeypatch.setenv("RC_WIN_WORDS", words)
    from rna_clique_amd.simulate import simulate
    samples, _ = simulate(4, 100, seed=29, p_iso2=0.2, indel_rate=0.012, p_revcomp=0.5, polya=(0.3, 10, 40),
                          len_loc=600, len_n=2000, len_p=0.5)
    eng = _run_sim(samples)
    msgs, summary = full_check(eng, samples)
    assert not msgs, "\n".join(msgs[:10])
    tm = eng.timings()
    assert summary["hsps"] > 0 and tm["defer_outside"] > 0
    if later == "1":
        assert tm["later_seeds"] > 0
        assert (tm["later_whole"] > 0) == (cap is not None)
    else:
        assert tm["later_seeds"] == 0


@pytest.mark.parametrize("top_matches,keep_all,two_pass", [(1, True, False), (1, False, False), (2, True, False),
                                                            (2, True, True), (1, False, True)])
def test_simulated_parity_options(native, monkeypatch, top_matches, keep_all, two_pass):
    """two_pass: the RBH step's fallback (a second pass over the groups, used
    when an item has more rows or edges than its slots) forced by RC_RBH_TWO_PASS."""
    if two_pass:
        monkeypatch.setenv("RC_RBH_TWO_PASS", "1")
    from rna_clique_amd.simulate import simulate
    samples, _ = simulate(4, 100, seed=11, p_iso2=0.3, indel_rate=0.003)
    eng = _run_sim(samples, top_matches=top_matches, keep_all=keep_all)
    msgs, _ = full_check(eng, samples, top_matches=top_matches, keep_all=keep_all,
                         check_hsps=False)
    assert not msgs, "\n".join(msgs[:10])


def _golden_engine(fx, hc):
    """Engine in external-alignment mode fed with a golden fixture's HSPs."""
    from oracle.post_oracle import default_parse_id
    from rna_clique_amd import _native as nat
    samples = fx["samples"]
    tx = {s: {} for s in samples}       # sample -> id -> (index)
    for key, rows in fx["hits"].items():
        q, s = key.split("|")
        for r in rows:
            h = dict(zip(hc, r))
            tx[q].setdefault(h["qseqid"], len(tx[q]))
            tx[s].setdefault(h["sseqid"], len(tx[s]))
    eng = _engine(top_matches=fx["top_matches"], keep_all=fx["keep_all"])
    for s in samples:
        ids = sorted(tx[s], key=tx[s].get)
        if not ids:
            ids = ["NODE_cov_1.0_g999999_i1"]
            tx[s][ids[0]] = 0
        seq = np.frombuffer(b"ACGT" * 50 * len(ids), dtype=np.uint8)
        offs = np.arange(len(ids) + 1, dtype=np.uint64) * 200
        parsed = [default_parse_id(i) for i in ids]
        eng.add_sample(s, seq, offs, [p[1] for p in parsed], [p[2] for p in parsed])
    for key, rows in fx["hits"].items():
        q, s = key.split("|")
        arr = np.zeros(len(rows), dtype=nat.HSP_DTYPE)
        for i, r in enumerate(rows):
            h = dict(zip(hc, r))
            arr[i]["q_tx"] = tx[q][h["qseqid"]]
            arr[i]["s_tx"] = tx[s][h["sseqid"]]
            for f in ("qstart", "qend", "sstart", "send", "length", "nident",
                      "mismatch", "gaps", "gapopen"):
                arr[i][f] = h[f]
            arr[i]["bits10"] = int(round(h["bitscore"] * 10))
            arr[i]["strand"] = 1 if h["sstrand"] == "minus" else 0
        eng.add_hsps(samples.index(q), samples.index(s), arr)
    eng.run()
    return eng


def test_golden_reference_tables(native):
    """The engine's RBH/graph/filter/distance kernels reproduce the reference's
    own outputs on the golden HSP tables (labels and row order included)."""
    from oracle.parity import engine_rows_as_dicts
    from rna_clique_amd._native import NativeError, RC_E_NO_IDEAL
    d = json.load(open(GOLDEN))
    cols, hc = d["columns"], d["hsp_columns"]
    checked = 0
    for fx in d["fixtures"]:
        exp = fx["expected"]
        if any(k != "matrix" for k in exp["errors"]):
            continue   # the reference itself crashed (recorded quirk)
        eng = _golden_engine(fx, hc)
        samples = fx["samples"]
        for key, rows in exp["tables"].items():
            t1, t2 = key.split("|")
            got = engine_rows_as_dicts(eng.pair_rows(samples.index(t1), samples.index(t2)))
            want = [dict(zip(cols, r)) for r in rows]
            keys = ["label", "qgene", "qiso", "sgene", "siso", "reverse", "bitscore",
                    "nident", "length", "gaps", "qstart", "qend", "sstart", "send", "sstrand"]
            assert [[g[k] for k in keys] for g in got] == [[w[k] for k in keys] for w in want], \
                f"seed {fx['seed']} pair {key}"
        edges = sorted(sorted([[samples[e["sample_a"]], int(e["gene_a"])],
                               [samples[e["sample_b"]], int(e["gene_b"])]])
                       for e in eng.edges())
        assert edges == exp["edges"], f"seed {fx['seed']} edges"
        s_, g_ = eng.ideal_nodes()
        assert sorted([samples[a], int(b)] for a, b in zip(s_, g_)) == exp["valid"]
        assert eng.stats()["sample_count"] == exp["sample_count"]
        num, den = eng.pair_sums()
        for key, (n_, d_) in exp["sums"].items():
            t1, t2 = key.split("|")
            a, b = samples.index(t1), samples.index(t2)
            assert (int(num[a, b]), int(den[a, b])) == (n_, d_)
        if exp["matrix"] is None:
            with pytest.raises(NativeError) as ei:
                eng.distance()
            assert ei.value.code == RC_E_NO_IDEAL
        else:
            labels, mat = eng.distance()
            assert labels == exp["matrix"]["labels"]
            assert np.array_equal(mat, np.array(exp["matrix"]["values"]))
        # UnfilteredSimilarity (unfiltered_distance.py:9-16) from the GPU sums,
        # against the reduction restated over the reference's golden tables
        from rna_clique_amd.similarity import UnfilteredSimilarity
        from test_oracle_golden import unfiltered_expected
        usim = UnfilteredSimilarity(eng)
        want = unfiltered_expected(exp)
        if want is None:
            with pytest.raises(ZeroDivisionError):
                usim.get_dissimilarity_df()
        else:
            udf = usim.get_dissimilarity_df()
            assert [str(x) for x in udf.index] == want["labels"]
            assert np.array_equal(udf.values, np.array(want["values"]))
        eng.close()
        checked += 1
    assert checked >= 15


def test_homolog_finder_single_pair(native, tmp_path):
    """find_homologs' HomologFinder.get_match_table on two top-genes FASTA
    files equals the pair's table from a full run (same engine path), and
    the CLI's Fraction equals the unfiltered sums of that pair."""
    from fractions import Fraction
    from rna_clique_amd.find_homologs import HomologFinder, match_table_similarity
    from rna_clique_amd.simulate import simulate
    from rna_clique_amd.similarity import UnfilteredSimilarity
    from rna_clique_amd.tables import pair_table
    from rna_clique_amd.transcripts import TranscriptID, default_gene_re
    samples, _ = simulate(2, 90, seed=31, p_iso2=0.2, indel_rate=0.002)
    paths = []
    for s in samples:
        p = tmp_path / f"{s.name}_top.fasta"
        s.write_fasta(p)
        paths.append(p)
    hf = HomologFinder(TranscriptID.parser_from_re(default_gene_re), 1, 1e-99, True)
    table = hf.get_match_table(paths[0], paths[1])
    assert list(table.columns[-5:]) == ["qgene", "qiso", "sgene", "siso", "reverse"]
    assert len(table) > 0
    eng = _run_sim(samples)
    full = pair_table(eng, 0, 1)
    cols = list(table.columns)
    assert table.index.tolist() == full.index.tolist()
    assert table[cols].astype(str).values.tolist() == full[cols].astype(str).values.tolist()
    num, den = eng.pair_sums(unfiltered=True)
    assert match_table_similarity(table) == Fraction(int(num[0, 1]), int(den[0, 1]))
    sims = UnfilteredSimilarity(eng).get_similarities()
    assert sims[(samples[0].name, samples[1].name)] == Fraction(int(num[0, 1]), int(den[0, 1]))
    dedup = HomologFinder.without_duplicates(table)
    assert list(dedup.columns) == ["qgene", "sgene"] and len(dedup) <= len(table)
    eng.close()
    # the find_homologs command: matches, then the Fraction (or a float with -f)
    import contextlib
    import io
    from rna_clique_amd.find_homologs import main
    for extra, want in (([], str(Fraction(int(num[0, 1]), int(den[0, 1])))),
                        (["-q", "-f"], str(float(Fraction(int(num[0, 1]), int(den[0, 1])))))):
        out, err = io.StringIO(), io.StringIO()
        with contextlib.redirect_stdout(out), contextlib.redirect_stderr(err):
            main([*extra, str(paths[0]), str(paths[1])])
        lines = out.getvalue().splitlines()
        assert lines[-1] == want
        assert len(lines) == (1 if extra else len(dedup) + 1)
        assert err.getvalue().strip() == f"Found {len(dedup)} matches."


def test_repeat_runs_identical(native):
    """Two runs of the same engine give identical results (deterministic)."""
    from rna_clique_amd.simulate import simulate
    samples, _ = simulate(4, 120, seed=5, p_iso2=0.2, indel_rate=0.002)
    eng = _run_sim(samples)
    h1 = [eng.hsps(q, s) for q in range(4) for s in range(4) if q != s]
    _, m1 = eng.distance()
    eng.run()
    h2 = [eng.hsps(q, s) for q in range(4) for s in range(4) if q != s]
    _, m2 = eng.distance()
    assert all(np.array_equal(a, b) for a, b in zip(h1, h2))
    assert np.array_equal(m1, m2)



def _with_degenerate(s, rng, gene0, only=False):
    """Sample s plus transcripts the index and DUST must get right at their
    edges: 1, 15, 16 and 17 bases (no 16-mer, exactly one, two), all-N, a
    300-base poly-A run, a dinucleotide repeat and a 16-mer flanked by N.
    only=True keeps just those."""
    from rna_clique_amd.simulate import Sample
    extra = [b"A", b"ACGTACGTACGTACG", b"ACGTTGCAACGTTGCA", b"ACGTTGCAACGTTGCAT", b"N" * 300,
             b"A" * 300, b"AC" * 150,
             b"N" * 20 + bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), 16)) + b"N" * 20]
    seqs = [] if only else [s.seq.tobytes()]
    lens = [] if only else list(np.diff(s.tx_offsets.astype(np.int64)))
    for x in extra:
        seqs.append(x)
        lens.append(len(x))
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    k = len(extra)
    keep = 0 if only else s.n_tx
    return Sample(s.name, np.frombuffer(b"".join(seqs), dtype=np.uint8).copy(), offs,
                  np.concatenate([s.gene[:keep], np.arange(gene0, gene0 + k)]).astype(np.int32),
                  np.concatenate([s.iso[:keep], np.ones(k)]).astype(np.int32),
                  np.concatenate([s.cov[:keep], 1.0 + np.arange(k) / 7.0]))


@pytest.mark.parametrize("dust", [None, False])
def test_degenerate_transcripts(native, dust):
    """Transcripts shorter than a 16-mer, exactly one or two 16-mers long,
    all-N, wholly low-complexity (DUST masks every base), plus one sample made
    of nothing else: the index fill's per-transcript slots, the sort's
    segments and DUST's ends are where these break. Parity with the oracle
    on every output; and a run whose index is empty (no transcript holds a
    16-mer) ends with no HSPs and the reference's no-ideal-components error."""
    from rna_clique_amd._native import NativeError, RC_E_NO_IDEAL
    from rna_clique_amd.simulate import simulate
    samples, _ = simulate(3, 80, seed=52, p_iso2=0.2, polya=(0.3, 10, 40))
    rng = np.random.default_rng(52)
    samples = [_with_degenerate(s, rng, 100000) for s in samples]
    samples.append(_with_degenerate(samples[0], rng, 200000, only=True))
    samples[-1].name = "only_degenerate"
    eng = _run_sim(samples, dust=dust)
    msgs, summary = full_check(eng, samples)
    assert not msgs, "\n".join(msgs[:10])
    assert summary["hsps"] > 0 and summary["ideal_nodes"] > 0
    eng.close()
    tiny = []
    for i, s in enumerate(simulate(2, 10, seed=53)[0]):
        t = _with_degenerate(s, rng, 300000, only=True)
        keep = [j for j in range(t.n_tx) if t.tx_offsets[j + 1] - t.tx_offsets[j] < 16]
        seq = b"".join(t.seq[t.tx_offsets[j]:t.tx_offsets[j + 1]].tobytes() for j in keep)
        lens = [int(t.tx_offsets[j + 1] - t.tx_offsets[j]) for j in keep]
        t.seq = np.frombuffer(seq, dtype=np.uint8).copy()
        t.tx_offsets = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        t.gene, t.iso, t.cov = t.gene[keep], t.iso[keep], t.cov[keep]
        tiny.append(t)
    eng = _run_sim(tiny, dust=dust)
    assert all(len(eng.hsps(q, s)) == 0 for q in range(2) for s in range(2) if q != s)
    assert len(eng.edges()) == 0
    with pytest.raises(NativeError) as ei:
        eng.distance()
    assert ei.value.code == RC_E_NO_IDEAL
    eng.close()


def test_more_than_256_samples(native):
    """300 samples (round 3 refused more than 256: 8-bit sample fields, a
    256-bit subject mask, one seed pass over all subjects). The reference
    enumerates any N (find_all_pairs.py:224). Pairs on both sides of 256 --
    sample indices in the seed passes' second 256-sample block -- bit-exact
    against the oracle (both directed searches, tables, unfiltered sums);
    the matrix hollow and symmetric, every pair with ideal rows."""
    import itertools
    from oracle.parity import check_pairs
    from rna_clique_amd.simulate import simulate
    # (rate 0.003: the 300-taxon tree's deepest pair is 16 branch-length units
    # apart, ~5 % divergence -- every gene a 300-clique, as at C3)
    samples, _ = simulate(300, 12, seed=61, mutation_rate=0.003)
    eng = _run_sim(samples)
    st = eng.stats()
    assert st["sample_count"] == 300 and st["ideal_components"] > 0
    picks = [(0, 1), (0, 299), (255, 256), (256, 257), (100, 280), (298, 299), (17, 255), (254, 299)]
    msgs = check_pairs(eng, samples, picks)
    assert not msgs, "\n".join(msgs[:10])
    labels, mat = eng.distance()
    assert np.array_equal(mat, mat.T) and np.all(np.diag(mat) == 0)
    # every pair has a table (ideal rows on both sides)
    num, den = eng.pair_sums()
    assert all(den[a, b] > 0 for a, b in itertools.combinations(range(300), 2))
    eng.close()


def test_reverse_pass_beyond_256_subjects(native):
    """The reverse pass (shared searches with DUST: reverse-search runs no
    forward word finds, from poly-A context) over more than 256 subject
    samples: queries past sample 256 take a second 256-sample pass (round 5
    and earlier stopped after the first). Samples 0-255 and 256-299 are two
    unrelated corpora (no run of 28 matching bases between them), the second
    with poly-A tails, so the reverse-only seeds of the whole run are exactly
    those of the two corpora run alone; every pair among samples 256-299 and
    pairs across the blocks bit-exact against the oracle."""
    import dataclasses
    import itertools
    from oracle.parity import check_pairs
    from rna_clique_amd.simulate import simulate
    low, _ = simulate(256, 8, seed=62, mutation_rate=0.003, p_revcomp=0.3)
    high, _ = simulate(44, 8, seed=63, mutation_rate=0.003, polya=(0.6, 10, 60), p_revcomp=0.3)
    high = [dataclasses.replace(s, name="H" + s.name) for s in high]
    samples = low + high
    counts = []
    for part in (low, high, samples):
        eng = _run_sim(part)
        counts.append(eng.timings()["reverse_seeds"])
        if part is not samples:
            eng.close()
    assert counts[1] > 0 and counts[2] == counts[0] + counts[1], counts
    picks = list(itertools.combinations(range(256, 300), 2))
    picks += [(a, b) for a in range(0, 256, 17) for b in (256, 271, 299)]
    msgs = check_pairs(eng, samples, picks)
    assert not msgs, "\n".join(msgs[:10])
    eng.close()


def test_gene_with_4200_isoforms(native):
    """A gene with 4200 transcripts (more than round 3's 4095: the 12-bit
    isoform field of the seed key; the field now takes what the longest
    transcript leaves, 65535 here) against a one-isoform ortholog, bit-exact
    vs the oracle. The reference keeps every isoform (select_top_genes.py:
    121-127)."""
    from rna_clique_amd.simulate import Sample, simulate
    samples, _ = simulate(2, 20, seed=62, len_loc=900, len_n=200, len_p=0.5)
    s = samples[0]
    rng = np.random.default_rng(5)
    g0 = int(s.gene[0])
    base = s.seq[int(s.tx_offsets[0]):int(s.tx_offsets[1])]
    seqs, genes, isos, covs = [], [], [], []
    for i in range(4200):
        v = base.copy()
        pos = rng.choice(v.size, size=max(1, v.size // 60), replace=False)
        v[pos] = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, pos.size)]
        seqs.append(v)
        genes.append(g0)
        isos.append(i + 1)
        covs.append(float(s.cov[0]) * 0.999 ** i)
    for t in range(1, s.n_tx):
        seqs.append(s.seq[int(s.tx_offsets[t]):int(s.tx_offsets[t + 1])])
        genes.append(int(s.gene[t]))
        isos.append(int(s.iso[t]))
        covs.append(float(s.cov[t]))
    offs = np.zeros(len(seqs) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([x.size for x in seqs])
    samples[0] = Sample(s.name, np.concatenate(seqs), offs, np.array(genes, np.int32), np.array(isos, np.int32),
                        np.array(covs))
    eng = _run_sim(samples)
    msgs, summary = full_check(eng, samples)
    assert not msgs, "\n".join(msgs[:10])
    assert summary["hsps"] > 4200
    eng.close()
