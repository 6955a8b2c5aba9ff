"""The native od2 table writer (csrc/od2_tables.cpp, rc_table_write_rows) writes
the same bytes as the Python writer, h5.write_frame_table(rows_to_table(rows))
-- whose files real PyTables + pandas read back (tests/test_h5_pytables.py) --
for tables of every column-dtype combination shrink_df can produce, both
strands, e-values across BLAST's print rule, empty tables and non-ASCII sample
labels (gene_matches_tables.py:42-56, find_homologs.py:58-80). CPU only."""
import ctypes

import numpy as np
import pytest


def _rows(n, rng, *, big_gene=False, neg=False, minus=0.3, long_len=False, huge=False):
    from rna_clique_amd import _native as nat
    r = np.zeros(n, dtype=nat.ROW_DTYPE)
    r["qgene"] = rng.integers(1, 70000 if big_gene else 250, n)
    r["sgene"] = rng.integers(1, 200, n)
    r["qiso"] = rng.integers(1, 3, n)
    r["siso"] = 1
    r["q_tx"] = rng.integers(0, 1000, n)
    r["s_tx"] = rng.integers(0, 1000, n)
    r["label"] = rng.permutation(3 * n)[:n] if n else []
    r["reverse"] = rng.integers(0, 2, n)
    h = r["hsp"]
    L = rng.integers(30, 70000 if long_len else 250, n)
    h["length"] = L
    h["nident"] = L - rng.integers(0, 7, n)
    h["mismatch"] = rng.integers(0, 5, n)
    h["gapopen"] = rng.integers(0, 3, n)
    h["gaps"] = rng.integers(0, 4, n)
    h["qstart"] = rng.integers(1, 60, n)
    h["qend"] = h["qstart"] + L
    h["sstart"] = rng.integers(-5 if neg else 1, 60, n)
    h["send"] = h["sstart"] + L
    h["bits10"] = rng.integers(500, 2_000_000 if huge else 4000, n)
    h["score_half"] = rng.integers(100, 4000, n)
    ev = 10.0 ** rng.uniform(-300, -3, n)
    ev[rng.random(n) < 0.2] = 0.0
    h["evalue"] = ev
    h["strand"] = (rng.random(n) < minus).astype(np.int32)
    return r


CASES = [
    dict(n=500),
    dict(n=500, big_gene=True),
    dict(n=500, neg=True),
    dict(n=500, minus=0.0),
    dict(n=500, minus=1.0),
    dict(n=300, long_len=True, big_gene=True, neg=True),
    dict(n=200, huge=True),
    dict(n=1),
    dict(n=0),
]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_native_table_equals_python_writer(native, tmp_path, case):
    from rna_clique_amd import _native as nat
    from rna_clique_amd.h5 import write_frame_table
    from rna_clique_amd.tables import rows_to_table
    rng = np.random.default_rng(100 + case)
    rows = _rows(rng=rng, **CASES[case])
    ss, qs = ("out/od1/T0_top.fasta", "out/od1/Sample-β_top.fasta") if case % 2 else ("od1/A_top.fasta", "od1/B")
    py = tmp_path / "py.h5"
    write_frame_table(py, rows_to_table(rows, ss, qs), key="gene_matches")
    nv = tmp_path / "native.h5"
    rows = np.ascontiguousarray(rows)
    nat.check(nat.lib().rc_table_write_rows(rows.ctypes.data_as(ctypes.c_void_p), len(rows), ss.encode(),
                                            qs.encode(), str(nv).encode()))
    a, b = py.read_bytes(), nv.read_bytes()
    if a != b:
        i = next(k for k in range(min(len(a), len(b))) if a[k] != b[k]) if a[:len(b)] != b[:len(a)] else None
        raise AssertionError(f"files differ: sizes {len(a)} vs {len(b)}, first difference at byte {i}")


def test_native_table_reads_back(native, tmp_path):
    """The native file read back through the HDF5 C library (h5.read_frame_table)
    is the frame rows_to_table builds."""
    import pandas as pd
    from rna_clique_amd import _native as nat
    from rna_clique_amd.tables import read_table, rows_to_table
    try:
        from rna_clique_amd.h5 import _Lib
        _Lib()
    except ImportError:
        pytest.skip("no HDF5 C library")
    rows = np.ascontiguousarray(_rows(800, np.random.default_rng(7), neg=True))
    p = tmp_path / "x--y.h5"
    nat.check(nat.lib().rc_table_write_rows(rows.ctypes.data_as(ctypes.c_void_p), len(rows), b"x", b"y",
                                            str(p).encode()))
    got = read_table(p)
    want = rows_to_table(rows, "x", "y")
    pd.testing.assert_frame_equal(got, want, check_categorical=False)
