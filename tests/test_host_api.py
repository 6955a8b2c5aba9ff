"""Host side of the drop-in: transcript ids, FASTA, top-gene selection,
tables, SampleSimilarity, matrix.h5, shard planning. No GPU needed."""
import ctypes
import heapq
import itertools
import os
import re
from collections import defaultdict
from fractions import Fraction

import numpy as np
import pandas as pd
import pytest

from rna_clique_amd import _native as nat
from rna_clique_amd.transcripts import (TranscriptID, TranscriptIDParseError,
                                        default_gene_re, default_parser)

# ---------------------------------------------------------------- transcript ids


def test_default_parser_rnaspades_ids():
    t = default_parser("NODE_1_length_2000_cov_12.500000_g7_i3")
    assert t == (12.5, 7, 3) and isinstance(t.gene, int) and isinstance(t.coverage, float)
    assert t.isoform == 3


def test_default_parser_requires_decimal_coverage():
    # transcripts.py:8 -- the coverage group needs a decimal point
    with pytest.raises(TranscriptIDParseError):
        default_parser("NODE_cov_12_g7_i3")
    with pytest.raises(TranscriptIDParseError):
        default_parser("something else")


def test_named_and_positional_groups():
    p = TranscriptID.parser_from_re(re.compile(r"g(?P<gene>\d+)_c([\d.]+)_i(\d+)"))
    assert p("g12_c3.5_i2") == (3.5, 12, 2)
    p2 = TranscriptID.parser_from_re(r"(?P<isoform>\d+)\|(?P<gene>\d+)\|(?P<coverage>[\d.]+)")
    assert p2("4|9|1.25") == (1.25, 9, 4)
    short = TranscriptID.parser_from_re(r"c([\d.]+)_g(\d+)")
    with pytest.raises(TranscriptIDParseError):
        short("c1.0_g2")


# ---------------------------------------------------------------- FASTA


def _bio_like_parse(text):
    """Bio.SeqIO "fasta" semantics restated (SimpleFastaParser)."""
    recs, title, lines = [], None, []
    for line in text.splitlines(keepends=True):
        if line.startswith(">"):
            if title is not None:
                recs.append((title, "".join(lines).replace(" ", "").replace("\r", "")))
            title, lines = line[1:].rstrip(), []
        elif title is not None:
            lines.append(line.rstrip())
    if title is not None:
        recs.append((title, "".join(lines).replace(" ", "").replace("\r", "")))
    return recs


ODD_FASTA = ("junk before\n\n>NODE_cov_1.5_g1_i1 desc words\r\nACGT ACGT\r\nac\n\n"
             ">NODE_cov_2.0_g2_i1\n>empty_next\nNNNN\t\nAC GT  \n>last_no_newline\nTTTT")


def test_fasta_reader_matches_biopython_semantics(tmp_path, native):
    from rna_clique_amd.fasta import FastaFile
    p = tmp_path / "t.fasta"
    p.write_bytes(ODD_FASTA.encode())
    want = _bio_like_parse(ODD_FASTA)
    with FastaFile(p) as f:
        assert f.titles == [t for t, _ in want]
        assert f.ids == [t.split(None, 1)[0] for t, _ in want]
        seq, offs = f.select()
        got = [seq[offs[i]:offs[i + 1]].tobytes().decode() for i in range(len(f))]
        assert got == [s for _, s in want]
        keep = np.array([1, 0, 1, 1], dtype=np.uint8)
        seq2, offs2 = f.select(keep)
        assert [seq2[offs2[i]:offs2[i + 1]].tobytes().decode() for i in range(3)] == \
            [want[0][1], want[2][1], want[3][1]]


def test_fasta_write_layout(tmp_path, native):
    from rna_clique_amd.fasta import FastaFile
    rng = np.random.default_rng(1)
    seqs = ["".join(rng.choice(list("ACGT"), n)) for n in (0, 59, 60, 61, 250)]
    src = tmp_path / "in.fasta"
    src.write_text("".join(f">r{i} x y\n{s[:33]}\n{s[33:]}\n" for i, s in enumerate(seqs)))
    out = tmp_path / "out.fasta"
    with FastaFile(src) as f:
        f.write(out, np.array([1, 1, 0, 1, 1], dtype=np.uint8))
    expect = ""
    for i in (0, 1, 3, 4):   # Bio.SeqIO.write: '>' + description, 60 columns
        expect += f">r{i} x y\n" + "".join(seqs[i][k:k + 60] + "\n" for k in range(0, len(seqs[i]), 60))
    assert out.read_text() == expect


# ---------------------------------------------------------------- top genes


def _ids_with_ties():
    rows = [(5.0, 1, 1), (7.0, 1, 2), (7.0, 2, 1), (3.0, 3, 1), (7.0, 4, 1), (1.0, 5, 1),
            (0.5, 5, 2), (7.0, 6, 1)]
    return [f"NODE_x_cov_{c:.6f}_g{g}_i{i}" for c, g, i in rows]


def test_top_gene_rule_matches_reference():
    from rna_clique_amd.select_top_genes import top_gene_ids
    ids = _ids_with_ties()
    best = defaultdict(float)
    for i in ids:
        c, g, _ = default_parser(i)
        best[g] = max(best[g], c)
    for n in range(0, 8):
        want = [k for _, k in heapq.nlargest(n, ((v, k) for k, v in best.items()))]
        got, _, _ = top_gene_ids(ids, n)
        assert got == want
    got, _, _ = top_gene_ids(ids, 3)
    assert got == [6, 4, 2]   # coverage 7.0 ties broken by the larger gene id


def test_select_top_sample(tmp_path, native):
    from rna_clique_amd.select_top_genes import TopGeneSelector, select_top_sample
    d = tmp_path / "S1.v2"
    d.mkdir()
    ids = _ids_with_ties()
    rng = np.random.default_rng(2)
    seqs = ["".join(rng.choice(list("ACGT"), 70 + 5 * k)) for k in range(len(ids))]
    (d / "transcripts.fasta").write_text("".join(f">{i}\n{s}\n" for i, s in zip(ids, seqs)))
    out = tmp_path / "od1"
    out.mkdir()
    s = select_top_sample(out, "transcripts.fasta", d, 3)
    assert s.path == out / "S1_top.fasta" and s.name == "S1"   # Q4: stem drops ".v2"
    keep = [k for k, i in enumerate(ids) if default_parser(i).gene in (2, 4, 6)]
    assert s.ids == [ids[k] for k in keep]
    assert list(s.gene) == [default_parser(ids[k]).gene for k in keep]
    got = [s.seq[s.tx_offsets[i]:s.tx_offsets[i + 1]].tobytes().decode() for i in range(s.n_tx)]
    assert got == [seqs[k] for k in keep]
    sel = TopGeneSelector.from_path(d / "transcripts.fasta", 3)
    assert list(sel.get_top_genes()) == [6, 4, 2]
    assert [r.id for r in sel.get_top_gene_seqs()] == s.ids
    assert s.path.read_text().startswith(">" + ids[keep[0]] + "\n")


# ---------------------------------------------------------------- tables


def _rows(n, rng):
    r = np.zeros(n, dtype=nat.ROW_DTYPE)
    r["qgene"] = rng.integers(0, 100, n)
    r["sgene"] = rng.integers(0, 100, n)
    r["reverse"] = rng.integers(0, 2, n)
    r["label"] = np.arange(n) * 3
    h = r["hsp"]
    h["length"] = rng.integers(100, 2000, n)
    h["nident"] = h["length"] - rng.integers(0, 50, n)
    h["bits10"] = rng.integers(1000, 30000, n)
    h["strand"] = rng.integers(0, 2, n)
    h["evalue"] = 10.0 ** -rng.uniform(99, 200, n)
    r["hsp"] = h
    return r


def test_rows_to_table_schema():
    from rna_clique_amd.tables import TABLE_COLUMNS, rows_to_table
    rng = np.random.default_rng(3)
    rows = _rows(50, rng)
    t = rows_to_table(rows, "od1/A_top.fasta", "od1/B_top.fasta")
    assert list(t.columns) == TABLE_COLUMNS
    assert list(t.index) == list(rows["label"])
    assert (t["bitscore"].to_numpy() == rows["hsp"]["bits10"] / 10.0).all()
    assert set(t["sstrand"]) <= {"plus", "minus"}
    assert t["reverse"].dtype == bool
    ev = rows["hsp"]["evalue"]
    assert (t["evalue"].to_numpy()[ev < 1e-180] == 0.0).all()
    m = ev >= 1e-180
    assert np.allclose(t["evalue"].to_numpy()[m], ev[m], rtol=5e-3)
    assert str(t["ssample"].dtype) == "category"


# ---------------------------------------------------------------- SampleSimilarity


class FakeEngine:
    """Duck-typed finished engine: what SampleSimilarity reads."""

    def __init__(self, labels, num, den, valid=()):
        self.labels = list(labels)
        self._num, self._den = np.asarray(num, np.int64), np.asarray(den, np.int64)
        self._valid = list(valid)

    def stats(self):
        return {"sample_count": len(self.labels)}

    def pair_sums(self):
        return self._num, self._den

    def ideal_nodes(self):
        return (np.array([s for s, _ in self._valid], np.int32),
                np.array([g for _, g in self._valid], np.int32))

    def distance(self, order):
        n_, d_ = self._num[np.ix_(order, order)], self._den[np.ix_(order, order)]
        if (d_[~np.eye(len(order), dtype=bool)] == 0).any():
            raise nat.NativeError(nat.RC_E_NO_IDEAL, "no ideal")
        out = np.zeros_like(n_, dtype=np.float64)
        off = ~np.eye(len(order), dtype=bool)
        out[off] = (d_[off] - n_[off]) / d_[off]
        return [self.labels[i] for i in order], out


def test_sample_similarity_numbers():
    from rna_clique_amd.similarity import SampleSimilarity
    labels = ["od1/c_top.fasta", "od1/a_top.fasta", "od1/b_top.fasta"]
    num = np.array([[0, 7, 5], [7, 0, 11], [5, 11, 0]])
    den = np.array([[0, 9, 13], [9, 0, 17], [13, 17, 0]])
    sim = SampleSimilarity.from_engine(FakeEngine(labels, num, den, [(0, 4), (1, 4)]))
    assert sim.samples == sorted(labels)
    s = sim.get_similarities()
    assert s[[labels[0], labels[1]]] == Fraction(7, 9) == s[[labels[1], labels[0]]]
    assert s[[labels[2], labels[2]]] == 1
    d = sim.get_dissimilarity_df()
    assert list(d.index) == sorted(labels) and list(d.columns) == sorted(labels)
    for a, b in itertools.permutations(range(3), 2):
        want = float(1 - Fraction(int(num[a, b]), int(den[a, b])))
        assert d.loc[labels[a], labels[b]] == want
    sm = sim.get_similarity_df()
    assert sm.loc[labels[0], labels[2]] == float(Fraction(5, 13))
    assert list(sim.valid.itertuples(index=False, name=None)) == [(labels[0], 4), (labels[1], 4)]


def test_sample_similarity_no_ideal():
    from rna_clique_amd.similarity import NoIdealComponentsError, SampleSimilarity
    sim = SampleSimilarity.from_engine(FakeEngine(["a", "b"], [[0, 0], [0, 0]], [[0, 0], [0, 0]]))
    with pytest.raises(NoIdealComponentsError):
        sim.get_dissimilarity_df()


# ---------------------------------------------------------------- matrix.h5

from h5read import LIBHDF5, H5 as _H5  # noqa: E402


@pytest.mark.skipif(not os.path.exists(LIBHDF5), reason="no libhdf5 to read the file back")
def test_matrix_h5_reads_back_with_libhdf5(tmp_path):
    from rna_clique_amd.h5 import write_matrix
    labels = [f"out/od1/S{i}_top.fasta" for i in (3, 1, 22)]
    rng = np.random.default_rng(5)
    m = rng.random((3, 3))
    df = pd.DataFrame(m, index=labels, columns=labels)
    p = tmp_path / "matrix.h5"
    write_matrix(df, p)
    h = _H5()
    f = h.open(p)
    assert np.array_equal(h.doubles(f, "/matrix/block0_values"), m)
    assert h.strings(f, "/matrix/axis0") == labels
    assert h.strings(f, "/matrix/axis1") == labels
    assert h.strings(f, "/matrix/block0_items") == labels
    assert h.attr(f, "/matrix", "pandas_type").rstrip(b"\0") == b"frame"
    assert h.attr(f, "/matrix", "encoding").rstrip(b"\0") == b"UTF-8"
    assert h.attr(f, "/matrix", "ndim") == (2).to_bytes(8, "little")
    assert h.attr(f, "/matrix", "nblocks") == (1).to_bytes(8, "little")
    assert h.attr(f, "/matrix/block0_values", "transposed") == b"\x01"
    assert h.attr(f, "/matrix/axis0", "kind").rstrip(b"\0") == b"string"
    assert h.n_links(f, "/") == 1 and h.n_links(f, "/matrix") == 4
    h.L.H5Fclose(f)


# ---------------------------------------------------------------- shard planning


@pytest.mark.parametrize("n,shards", [(4, 1), (4, 2), (5, 8), (32, 8), (13, 3), (2, 4), (64, 8), (32, 5),
                                      (300, 1), (300, 8), (1000, 8)])
def test_plan_shards_partitions_pairs(native, n, shards):
    from rna_clique_amd.distributed import plan_pairs, plan_shards
    rng = np.random.default_rng(n * 7 + shards)
    bases = rng.integers(1_000, 1_000_000, n)
    pairs, first = plan_pairs(bases, shards)
    assert np.array_equal(first, plan_shards(bases, shards))
    n_pairs = n * (n - 1) // 2
    assert first[0] == 0 and first[-1] == n_pairs
    assert (np.diff(first) >= 0).all()
    # every pair exactly once, a < b
    assert sorted(pairs, key=lambda p: (p[1], p[0])) == [(a, b) for b in range(n) for a in range(b)]
    if shards == 1:   # one shard: plain subject-major order
        assert pairs == [(a, b) for b in range(n) for a in range(b)]
    for r in range(shards):
        own = pairs[first[r]:first[r + 1]]
        if not own:
            continue
        # one rectangle: the shard's subjects (its index) and queries are
        # contiguous sample ranges, and it holds every pair inside them
        bs, as_ = sorted({b for _, b in own}), sorted({a for a, _ in own})
        assert bs == list(range(bs[0], bs[-1] + 1))
        assert as_ == list(range(as_[0], as_[-1] + 1))
        want = {(a, b) for b in bs for a in as_ if a < b}
        assert set(own) == want
        # subject-major inside the shard
        assert own == sorted(own, key=lambda p: (p[1], p[0]))
    if n_pairs >= 4 * shards:
        # the modelled load of the largest shard is within 2x of the even split
        cost = lambda own: (sum(bases[a] + bases[b] for a, b in own)  # noqa: E731
                            + 5 * sum(bases[a] for a in {a for a, _ in own})
                            + 11 * sum(bases[b] for b in {b for _, b in own}))
        loads = [cost(pairs[first[r]:first[r + 1]]) for r in range(shards)]
        assert max(loads) <= 2 * sum(bases[a] + bases[b] for a, b in pairs) / shards + 16 * max(bases) * n


def test_downcast_int_matches_pandas():
    """tables.downcast_int (shrink_df's fast path) gives pandas' double
    to_numeric downcast (find_homologs.py:58-80) dtype and values."""
    import numpy as np
    import pandas as pd
    from rna_clique_amd.tables import downcast_int
    rng = np.random.default_rng(0)
    cases = [np.array([0]), np.array([-1]), np.array([127, 128]), np.array([255]), np.array([256]),
             np.array([-129, 5]), np.array([65535]), np.array([65536, 0]), np.array([-32769]),
             np.array([2 ** 31]), np.array([-(2 ** 31) - 1]), np.array([2 ** 63 - 1])]
    for dt in (np.int32, np.int64, np.uint32):
        for hi in (2, 200, 70000, 5_000_000_000):
            a = rng.integers(0, hi, 50)
            if dt != np.uint32 and hi < 2 ** 31:
                cases.append((a - hi // 3).astype(dt))
            if hi < np.iinfo(dt).max:
                cases.append(a.astype(dt))
    for a in cases:
        want = pd.to_numeric(pd.to_numeric(pd.Series(a), downcast="integer"), downcast="unsigned")
        got = downcast_int(a)
        assert got.dtype == want.dtype, (a, got.dtype, want.dtype)
        assert (got == want.to_numpy()).all()


def test_pytables_branch_is_serialised(tmp_path, monkeypatch):
    """When PyTables is importable, write_table goes through df.to_hdf, which
    is not thread-safe (PyTables releases the GIL around HDF5): callers on
    several threads must never be inside it twice at once. (The engine's own
    od2 tables are written natively, rc_write_outputs; write_table is the
    reference's entry point for any DataFrame.)"""
    import sys
    import threading
    import time
    import types
    from concurrent.futures import ThreadPoolExecutor
    import numpy as np
    import pandas as pd
    from rna_clique_amd import _native
    from rna_clique_amd.tables import rows_to_table, write_table
    monkeypatch.setitem(sys.modules, "tables", types.ModuleType("tables"))
    state = {"in": 0, "max": 0, "calls": 0}
    guard = threading.Lock()

    def fake_to_hdf(self, path, key=None, format=None, **kw):
        with guard:
            state["in"] += 1
            state["calls"] += 1
            state["max"] = max(state["max"], state["in"])
        time.sleep(0.02)
        assert key == "gene_matches" and format == "table" and len(self) == 3
        with guard:
            state["in"] -= 1
    monkeypatch.setattr(pd.DataFrame, "to_hdf", fake_to_hdf)
    r = np.zeros(3, dtype=_native.ROW_DTYPE)
    r["qgene"], r["sgene"], r["label"] = [1, 2, 3], [4, 5, 6], [0, 1, 2]
    r["hsp"]["length"], r["hsp"]["nident"], r["hsp"]["bits10"] = 100, 99, 1800
    df = rows_to_table(r, "od1/A_top.fasta", "od1/B_top.fasta")
    with ThreadPoolExecutor(6) as ex:
        list(ex.map(lambda i: write_table(df, tmp_path / f"t{i}.h5"), range(6)))
    assert state["calls"] == 6
    assert state["max"] == 1
