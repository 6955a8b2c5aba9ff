"""Gene matches tables and graph in the reference's in-memory and on-disk forms.

The engine keeps every table on the GPU; these helpers materialise them only
when a caller asks (store_dfs, od2 files, graph.pkl):

* `pair_table` -> the DataFrame HomologFinder.get_match_table returns plus the
  ssample/qsample columns find_homologs_and_save adds (find_all_pairs.py:57-88;
  schema docs/formats.md:231-252), with the index labels the reference keeps.
* `build_graph` -> the networkx Graph build_graph.py:40-68 makes from those
  tables, with the same node and edge insertion order.
* `write_table` / `read_table` -> gene_matches_tables.py:42-56 (.pkl via
  pandas; .h5 in pandas' table format, with or without PyTables).
"""
from __future__ import annotations

import numbers
import threading
from pathlib import Path

import numpy as np
import pandas as pd

TABLE_COLUMNS = ["pident", "length", "mismatch", "gapopen", "qstart", "qend", "sstart",
                 "send", "evalue", "bitscore", "gaps", "nident", "sstrand", "qgene",
                 "qiso", "sgene", "siso", "reverse", "ssample", "qsample"]


def blast_evalue(e):
    """E-value as BLAST's tabular output prints it, read back as a float:
    "0.0" below 1e-180, else three significant digits (the form shown in
    docs/formats.md:262, e.g. 8.75e-152)."""
    e = np.asarray(e, dtype=np.float64)
    # a table holds few distinct e-values: print and parse those only
    u, inv = np.unique(e, return_inverse=True)
    out = np.char.mod("%.2e", u).astype(np.float64)[inv].reshape(e.shape)
    out[e < 1.0e-180] = 0.0
    return out


def blast_pident(nident, length):
    """pident = 100 * nident / length printed with 3 decimals."""
    p = 100.0 * np.asarray(nident, dtype=np.float64) / np.maximum(np.asarray(length), 1)
    u, inv = np.unique(p, return_inverse=True)   # distinct ratios only
    return np.char.mod("%.3f", u).astype(np.float64)[inv].reshape(p.shape)


_UNSIGNED = (np.uint8, np.uint16, np.uint32, np.uint64)
_SIGNED = (np.int8, np.int16, np.int32, np.int64)


def downcast_int(a: np.ndarray) -> np.ndarray:
    """pd.to_numeric(pd.to_numeric(a, downcast="integer"), downcast="unsigned")
    for a non-empty integer array, from its min and max: the smallest signed
    type holding the values, then the smallest unsigned one if none is
    negative -- i.e. the smallest unsigned type when all are >= 0."""
    mn, mx = int(a.min()), int(a.max())
    for t in (_UNSIGNED if mn >= 0 else _SIGNED):
        i = np.iinfo(t)
        if i.min <= mn and mx <= i.max:
            return a.astype(t, copy=False)
    return a


def shrink_df(df: pd.DataFrame) -> pd.DataFrame:
    """Downcast integer columns (find_homologs.py:58-80)."""
    df = df.copy()
    for col in df.columns:
        if issubclass(df[col].dtype.type, numbers.Integral):
            if len(df):
                df[col] = downcast_int(df[col].to_numpy())
            else:
                df[col] = pd.to_numeric(pd.to_numeric(df[col], downcast="integer"), downcast="unsigned")
    return df


def rows_to_table(rows: np.ndarray, ssample: str, qsample: str) -> pd.DataFrame:
    """Engine rows (ROW_DTYPE) of one sample pair -> reference table."""
    h = rows["hsp"]
    df = pd.DataFrame({
        "pident": blast_pident(h["nident"], h["length"]),
        "length": h["length"], "mismatch": h["mismatch"], "gapopen": h["gapopen"],
        "qstart": h["qstart"], "qend": h["qend"], "sstart": h["sstart"], "send": h["send"],
        "evalue": blast_evalue(h["evalue"]),
        "bitscore": h["bits10"].astype(np.float64) / 10.0,
        "gaps": h["gaps"], "nident": h["nident"],
        "sstrand": np.where(h["strand"] != 0, "minus", "plus"),
        "qgene": rows["qgene"], "qiso": rows["qiso"],
        "sgene": rows["sgene"], "siso": rows["siso"],
        "reverse": rows["reverse"].astype(bool),
    }, index=pd.Index(rows["label"].astype(np.int64)))
    df = shrink_df(df)
    one = np.zeros(len(df), dtype=np.int8)
    df["ssample"] = pd.Categorical.from_codes(one, categories=[ssample])
    df["qsample"] = pd.Categorical.from_codes(one, categories=[qsample])
    return df[TABLE_COLUMNS]


def pair_table(engine, a: int, b: int, labels=None) -> pd.DataFrame:
    """Gene matches table of samples a < b (a = t1 = ssample, b = t2 = qsample)."""
    labels = labels or engine.labels
    return rows_to_table(engine.pair_rows(a, b), labels[a], labels[b])


# PyTables and a default (non-thread-safe) HDF5 build must not be entered from
# two threads at once, and PyTables releases the GIL around HDF5 calls: every
# to_hdf / read_hdf of this module holds this lock (write_pair_tables writes
# tables from a thread pool)
_HDF5_LOCK = threading.Lock()


def write_table(df: pd.DataFrame, path: Path):
    """gene_matches_tables.py:42-56: .pkl via pandas; .h5 in pandas' table
    format under key "gene_matches" -- through PyTables when it is importable
    (serialised by _HDF5_LOCK), else written directly (h5.write_frame_table;
    read back by PyTables in tests/test_h5_pytables.py)."""
    path = Path(path)
    if path.suffix == ".pkl":
        df.to_pickle(path)
    elif path.suffix == ".h5":
        try:
            import tables  # noqa: F401
        except ImportError:
            from .h5 import write_frame_table
            write_frame_table(path, df, key="gene_matches")
        else:
            with _HDF5_LOCK:
                df.to_hdf(path, key="gene_matches", format="table")
    else:
        raise ValueError(f"Could not determine file type for extension {path.suffix}.")


def read_table(path: Path) -> pd.DataFrame:
    """gene_matches_tables.py read_table: a table write_table wrote (.pkl is
    this package's own pickle output; .h5 through PyTables when importable,
    else through the HDF5 C library, h5.read_frame_table)."""
    path = Path(path)
    if path.suffix == ".pkl":
        return pd.read_pickle(path)
    if path.suffix == ".h5":
        try:
            import tables  # noqa: F401
        except ImportError:
            from .h5 import read_frame_table
            return read_frame_table(path, key="gene_matches")
        with _HDF5_LOCK:
            return pd.read_hdf(path, key="gene_matches")
    raise ValueError(f"Could not determine file type for extension {path.suffix}.")


def build_graph(tables):
    """build_graph.py:40-68 over (ssample, qsample, rows) triples or DataFrames:
    per table, the s-nodes, then the q-nodes, then the edges, in row order."""
    import networkx as nx
    g = nx.Graph()
    for t in tables:
        if isinstance(t, pd.DataFrame):
            ss = t["ssample"].astype(object).to_numpy()
            qs = t["qsample"].astype(object).to_numpy()
            sg = t["sgene"].to_numpy()
            qg = t["qgene"].to_numpy()
            sn = list(zip(ss, sg.tolist()))
            qn = list(zip(qs, qg.tolist()))
        else:
            ssample, qsample, rows = t
            sn = [(ssample, x) for x in rows["sgene"].tolist()]
            qn = [(qsample, x) for x in rows["qgene"].tolist()]
        g.add_nodes_from(sn)
        g.add_nodes_from(qn)
        g.add_edges_from(zip(sn, qn))
    return g


def write_engine_outputs(engine, pairs, table_paths=None, graph_path=None, threads=8):
    """The od2 table files (`table_paths[i]` for `pairs[i]` = (a, b), a < b)
    and/or graph.pkl of an engine run, natively (rc_write_outputs): each
    pair's rows leave the GPU once; table files are written by `threads` host
    threads in pandas' table format -- the bytes h5.write_frame_table writes
    for pair_table(engine, a, b), tests/test_od2_native.py -- and the graph
    pickle (build_graph over `pairs` in order, then pickle.dump) beside them,
    all outside the interpreter (the GIL is released for the whole call)."""
    import ctypes
    from . import _native
    n = len(pairs)
    a = np.ascontiguousarray([p[0] for p in pairs], dtype=np.int32)
    b = np.ascontiguousarray([p[1] for p in pairs], dtype=np.int32)
    tp = None
    if table_paths is not None:
        enc = [str(x).encode() for x in table_paths]
        if len(enc) != n:
            raise ValueError("one table path per pair")
        tp = (ctypes.c_char_p * max(n, 1))(*enc)
    _native.check(_native.lib().rc_write_outputs(
        engine._h, n, a.ctypes.data_as(ctypes.c_void_p), b.ctypes.data_as(ctypes.c_void_p),
        ctypes.cast(tp, ctypes.c_void_p) if tp is not None else None,
        str(graph_path).encode() if graph_path is not None else None, int(threads)))


def write_graph_pickle(path, tables, names):
    """graph.pkl of the graph build_graph would make from `tables` -- an
    iterable of (ssample index, qsample index, sgene array, qgene array), in
    build_graph's table order, sample indices into `names` -- written by the
    native pickle writer (graph_pickle.cpp) without building it in Python.
    pickle.load gives the networkx Graph build_graph returns (node,
    neighbour and edge order included)."""
    import ctypes
    from . import _native
    L = _native.lib()
    h = ctypes.c_void_p()
    _native.check(L.rc_graph_pickle_begin(ctypes.byref(h)))
    try:
        for sa, qa, sg, qg in tables:
            sg = np.ascontiguousarray(sg, dtype=np.int64)
            qg = np.ascontiguousarray(qg, dtype=np.int64)
            _native.check(L.rc_graph_pickle_add(h, int(sa), int(qa), sg.ctypes.data, qg.ctypes.data, len(sg)))
        enc = [str(n).encode() for n in names]
        arr = (ctypes.c_char_p * max(len(enc), 1))(*enc)
        _native.check(L.rc_graph_pickle_write(h, str(path).encode(), len(enc), arr))
    finally:
        L.rc_graph_pickle_free(h)
