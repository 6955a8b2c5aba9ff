"""The HDF5 writers (rna_clique_amd/h5.py) read back by real PyTables + pandas.

matrix.h5 (fixed format, rna_clique.py:176-177) and the od2 gene matches
tables (format="table", key "gene_matches", gene_matches_tables.py:42-56) are
written without PyTables by this package; here `pandas.read_hdf` -- running
in /opt/conda's Python 3.9, which has PyTables (tests/pytables_ref.py) --
must return exactly the frame that was written. Skipped where that
interpreter is missing.
"""
import json
import os
import subprocess

import numpy as np
import pandas as pd
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
PY39 = "/opt/conda/bin/python3.9"


def _ref(*args):
    env = {"PATH": "/opt/conda/bin:/usr/bin", "HOME": "/tmp"}
    return subprocess.run([PY39, os.path.join(HERE, "pytables_ref.py"), *map(str, args)], env=env,
                          capture_output=True, text=True, timeout=120)


def _have_pytables():
    if not os.path.exists(PY39):
        return False
    r = subprocess.run([PY39, "-c", "import tables, pandas"], env={"PATH": "/opt/conda/bin:/usr/bin", "HOME": "/tmp"},
                       capture_output=True, timeout=60)
    # tables itself fails on numpy >= 1.24 without the shims: the checker applies them
    return r.returncode == 0 or b"typeDict" in r.stderr


pytestmark = pytest.mark.skipif(not _have_pytables(), reason="no PyTables interpreter in /opt/conda")


def read_back(path, key, tmp_path):
    out = tmp_path / "read.json"
    r = _ref("read", path, key, out)
    assert r.returncode == 0, r.stderr[-2000:]
    with open(out) as f:
        return json.load(f)


@pytest.mark.parametrize("n", [1, 2, 5, 33])
def test_matrix_h5_reads_back(tmp_path, n):
    from rna_clique_amd.h5 import write_matrix
    rng = np.random.default_rng(n)
    labels = [f"/data/run_{i}/od1/sample_{i:03d}_top.fasta" for i in range(n)]
    m = rng.random((n, n))
    m = (m + m.T) / 2
    np.fill_diagonal(m, 0.0)
    df = pd.DataFrame(m, index=labels, columns=labels)
    path = tmp_path / "matrix.h5"
    write_matrix(df, path)
    got = read_back(path, "matrix", tmp_path)
    assert got["columns"] == labels and got["index"] == labels
    vals = np.array([got["data"][c]["values"] for c in labels]).T
    assert got["data"][labels[0]]["dtype"] == "float64"
    assert np.array_equal(vals, m)


def _gene_table(n, seed, s1="/x/od1/s1_top.fasta", s2="/x/od1/s2_top.fasta"):
    from rna_clique_amd._native import ROW_DTYPE
    from rna_clique_amd.tables import rows_to_table
    rng = np.random.default_rng(seed)
    r = np.zeros(n, dtype=ROW_DTYPE)
    r["qgene"] = rng.integers(0, 70000, n)
    r["qiso"] = rng.integers(1, 3, n)
    r["sgene"] = rng.integers(0, 300, n)
    r["siso"] = 1
    r["reverse"] = rng.integers(0, 2, n)
    r["label"] = rng.permutation(n)
    h = r["hsp"]
    h["nident"] = rng.integers(30, 5000, n)
    h["length"] = h["nident"] + rng.integers(0, 40, n)
    h["mismatch"] = rng.integers(0, 30, n)
    h["gapopen"] = rng.integers(0, 3, n)
    h["gaps"] = h["gapopen"] * 2
    h["qstart"] = rng.integers(1, 300, n)
    h["qend"] = h["qstart"] + h["length"]
    h["sstart"] = rng.integers(1, 70000, n)
    h["send"] = h["sstart"] + h["length"]
    h["evalue"] = 10.0 ** -rng.integers(100, 200, n)
    h["bits10"] = rng.integers(500, 90000, n)
    h["strand"] = rng.integers(0, 2, n)
    return rows_to_table(r, s1, s2)


def _assert_same(df, got):
    assert got["columns"] == list(df.columns)
    assert got["index"] == df.index.tolist()
    for c in df.columns:
        s, g = df[c], got["data"][c]
        if isinstance(s.dtype, pd.CategoricalDtype):
            assert g["dtype"] == "category"
            assert g["categories"] == [str(x) for x in s.cat.categories]
            assert g["values"] == [str(x) for x in s.astype(object)]
        elif s.dtype == object:
            assert g["dtype"] == "object" and g["values"] == [str(x) for x in s]
        else:
            assert g["dtype"] == str(s.dtype), (c, g["dtype"], s.dtype)
            assert g["values"] == s.to_numpy().tolist(), c


@pytest.mark.parametrize("n,seed", [(0, 1), (1, 2), (7, 3), (2500, 4)])
def test_gene_matches_table_reads_back(tmp_path, n, seed):
    """od2 tables as write_table writes them without PyTables: pandas.read_hdf
    returns the same frame -- columns, dtypes (downcast integers, float64,
    bool, strings, categoricals with their categories), index labels."""
    from rna_clique_amd.tables import write_table
    df = _gene_table(n, seed)
    path = tmp_path / "s1--s2.h5"
    write_table(df, path)
    _assert_same(df, read_back(path, "gene_matches", tmp_path))


def _frame_json(df):
    d = {"index": df.index.tolist(), "index_dtype": str(df.index.dtype), "columns": list(df.columns), "data": {}}
    for c in df.columns:
        s = df[c]
        if isinstance(s.dtype, pd.CategoricalDtype):
            d["data"][c] = {"dtype": "category", "categories": [str(x) for x in s.cat.categories],
                            "values": [str(x) for x in s.astype(object)]}
        elif s.dtype == object:
            d["data"][c] = {"dtype": "object", "values": [str(x) for x in s]}
        else:
            d["data"][c] = {"dtype": str(s.dtype), "values": s.to_numpy().tolist()}
    return d


@pytest.mark.parametrize("n,seed", [(0, 5), (9, 6), (3000, 7)])
def test_read_table_without_pytables(tmp_path, n, seed):
    """read_table's .h5 path without PyTables (the HDF5 C library) returns the
    frame exactly, on this package's files and on files PyTables + pandas
    wrote (chunked, with the index's search structure)."""
    from rna_clique_amd.h5 import read_frame_table
    from rna_clique_amd.tables import write_table
    df = _gene_table(n, seed)
    ours = tmp_path / "ours.h5"
    write_table(df, ours)
    pd.testing.assert_frame_equal(read_frame_table(ours), df)
    src = tmp_path / "in.json"
    with open(src, "w") as f:
        json.dump(_frame_json(df), f)
    theirs = tmp_path / "theirs.h5"
    r = _ref("write", src, theirs, "gene_matches", "table")
    assert r.returncode == 0, r.stderr[-2000:]
    if n == 0:
        # pandas writes no object for an empty frame in table format (reading
        # it back is a KeyError there); this package writes an empty table
        with pytest.raises(KeyError):
            read_frame_table(theirs)
        return
    pd.testing.assert_frame_equal(read_frame_table(theirs), df)
