"""SampleSimilarity over the GPU engine.

Same interface as the reference's SampleSimilarity / ComparisonSimilarityComputer
(filtered_distance.py:129-317, similarity_computer.py:44-375), but every number
comes from librcgpu.so: the gene matches graph, its connected components and
ideal-clique filter, the restricted sums and the distances are computed on the
GPU. Two ways in:

* `SampleSimilarity(graph, comparison_dfs, sample_count=None)` -- the
  reference's constructor (and `from_filenames(graph_fn, table_fns)`, the
  resume path of the filtered_distance CLI): the graph's edges and the tables'
  rows go to a graph-only engine (rc_import_edges), which runs components, the
  ideal filter, the restricted sums and the distances;
* `SampleSimilarity.from_engine(engine)` -- a finished alignment run, whose
  tables and graph stay on the GPU and are only materialised on request.

Semantics kept from the reference:
* sample_count = distinct samples among graph nodes (filtered_distance.py:171-182);
* similarity = Fraction(sum nident, sum length - sum gaps) over the restricted
  table (similarity_computer.py:21-42); an empty restricted table raises
  NoIdealComponentsError (filtered_distance.py:234-247);
* distance = float(1 - similarity), correctly rounded, rows and columns in
  sorted() order of the sample labels (similarity_computer.py:216-345).
"""
from __future__ import annotations

import itertools
from fractions import Fraction
from functools import cached_property

import numpy as np
import pandas as pd

from . import _native as nat
from .tables import build_graph, pair_table


class NoIdealComponentsError(Exception):
    pass


class PairDict(dict):
    """Mapping keyed by unordered sample pairs; `d[[a, b]] == d[[b, a]]`
    (the MultisetKeyDict lookups the reference uses)."""

    @staticmethod
    def key(k):
        if isinstance(k, (frozenset, set)):
            k = tuple(k) * (2 if len(k) == 1 else 1)
        a, b = k
        return (a, b) if a <= b else (b, a)

    def __getitem__(self, k):
        return super().__getitem__(self.key(k))

    def __setitem__(self, k, v):
        super().__setitem__(self.key(k), v)

    def __contains__(self, k):
        return super().__contains__(self.key(k))

    def key_elements(self):
        return set(itertools.chain.from_iterable(self.keys()))

    def multiset_iter(self):
        return iter(self.items())


class SampleSimilarity:
    """Similarities of samples from the gene matches graph and tables."""

    sample_gene_columns = [[a + b for b in ["sample", "gene"]] for a in ["s", "q"]]
    categorical_columns = ["qsample", "ssample", "sstrand"]

    def __init__(self, graph, comparison_dfs, sample_count=None, *, device=0):
        """filtered_distance.py:162-169: `graph` a networkx graph of (sample,
        gene) nodes, `comparison_dfs` the gene matches tables as an iterable
        of (pair of samples, table) or a mapping."""
        items = comparison_dfs.items() if hasattr(comparison_dfs, "items") else comparison_dfs
        self._stored = PairDict()
        for k, df in items:
            self._stored[tuple(k) if len(k) == 2 else tuple(k) * 2] = df
        self._graph = graph
        self.engine = _graph_engine(graph, list(self._stored.items()), sample_count, device)
        self.labels = list(self.engine.labels)
        self._sample_count = self.engine.stats()["sample_count"]
        # the similarities are those of the given tables' pairs, and the
        # matrix's samples the tables' samples (similarity_computer.py:216-226:
        # samples = key elements of the similarities); a sample known only
        # from graph nodes is no row of the matrix
        idx = {lab: i for i, lab in enumerate(self.labels)}
        self._sim_pairs = sorted({tuple(sorted((idx[str(a)], idx[str(b)])))
                                  for a, b in self._stored.keys() if str(a) != str(b)})
        self._samples = None

    @classmethod
    def from_engine(cls, engine, store_dfs: bool = False):
        """The similarities of a finished engine run (rna_clique(), find_all_pairs)."""
        self = cls.__new__(cls)
        self.engine = engine
        self.labels = list(engine.labels)
        self._sample_count = engine.stats()["sample_count"]
        self._graph = None
        self._stored = PairDict(self._table_iter()) if store_dfs else None
        self._sim_pairs = None   # every pair of the run
        self._samples = None
        return self

    @classmethod
    def mapping_from_dfs(cls, dfs):
        """(pair, table) from each table's own qsample/ssample columns
        (similarity_computer.py:90-115; the first row rather than label 0,
        see SURVEY.md Q1). An empty table names no samples: the reference
        fails on it (KeyError from df["qsample"][0], Q1/Q3); here it is
        skipped, so its pair is not among the similarities (and its samples
        are in the matrix only if another table names them) --
        tests/test_gpu_api.py::test_sample_similarity_matrix_samples_from_tables."""
        for df in dfs:
            if len(df):
                yield frozenset((str(df["qsample"].iloc[0]), str(df["ssample"].iloc[0]))), df

    @classmethod
    def _read_table(cls, table_path, remove_seqids=True, convert_to_categorical=True):
        """similarity_computer.py:117-164 (the reference's categorical step
        tests `table.index` and is a no-op, Q2; this one converts)."""
        from .tables import read_table
        table = read_table(table_path)
        if remove_seqids:
            table = table.drop(columns=[c for c in ("qseqid", "sseqid") if c in table.columns])
        if convert_to_categorical:
            cols = [c for c in cls.categorical_columns if c in table.columns]
            table[cols] = table[cols].astype("category")
        return table

    @classmethod
    def from_filenames(cls, graph_fn, comparison_fns, store_dfs=True, remove_seqids=True,
                       convert_to_categorical=True, **kwargs):
        """filtered_distance.py:250-317: the pickled graph and the gene
        matches tables written by a previous run (rna_clique(), the
        find_all_pairs / filtering_step entry points)."""
        import pickle
        with open(graph_fn, "rb") as f:
            graph = pickle.load(f)
        dfs = [cls._read_table(p, remove_seqids, convert_to_categorical) for p in comparison_fns]
        return cls(graph, list(cls.mapping_from_dfs(dfs)), **kwargs)

    # ------------------------------------------------------------ tables
    def _pairs(self):
        return itertools.combinations(range(len(self.labels)), 2)

    def _table_pairs(self):
        """The pairs whose tables this engine holds: all of them, or on a
        sharded run (world > 1) this rank's pairs only -- each rank then
        holds (and rna_clique(store_dfs=True) / write_pair_tables write) a
        disjoint part of the table set, the union over ranks being the whole."""
        if getattr(self.engine, "shard_count", 1) > 1:
            return sorted(tuple(sorted(p)) for p in self.engine.owned_pairs())
        return self._pairs()

    def _table_iter(self):
        for a, b in self._table_pairs():
            yield (self.labels[a], self.labels[b]), pair_table(self.engine, a, b, self.labels)

    @property
    def comparison_dfs(self):
        """Pair -> gene matches table (a PairDict when stored, else a fresh
        generator of (pair, table) from the engine)."""
        return self._stored if self._stored is not None else self._table_iter()

    @property
    def graph(self):
        """The gene matches graph (networkx): the one given, or the one
        build_graph.py:40-68 makes from an engine run's tables. A sharded
        engine holds only its own pairs' tables, but every shard has all
        graph edges after the exchange, per pair in pair order and in the
        order of each pair's rows: build_graph over those per-pair edge
        tables gives the same graph, node and neighbour order included."""
        if self._graph is not None:
            return self._graph
        if getattr(self.engine, "shard_count", 1) > 1:
            self._graph = build_graph(
                (self.labels[sa], self.labels[qa], {"sgene": sg, "qgene": qg})
                for sa, qa, sg, qg in self._edge_tables())
            return self._graph

        def rows():
            for a, b in self._pairs():
                yield self.labels[a], self.labels[b], self.engine.pair_rows(a, b)
        self._graph = build_graph(rows())
        return self._graph

    def _edge_tables(self):
        """A sharded engine's exchanged edges as per-pair tables (ssample,
        qsample, sgene array, qgene array) in pair order, each in its rows'
        order (the record order inside a pair is kept)."""
        import numpy as np
        e = self.engine.edges()
        o = np.lexsort((e["sample_b"], e["sample_a"]))   # stable: record order inside a pair
        e = e[o]
        key = e["sample_a"].astype(np.int64) * (1 << 32) + e["sample_b"].astype(np.int64)
        cut = np.flatnonzero(np.diff(key)) + 1
        for r in (np.split(np.arange(len(e)), cut) if len(e) else []):
            yield int(e["sample_a"][r[0]]), int(e["sample_b"][r[0]]), e["gene_a"][r], e["gene_b"][r]

    def write_graph(self, path):
        """graph.pkl (filtering_step.py:158-159): the pickle of `graph`. For an
        engine run whose graph was never built in Python, the native writer
        streams the pairs' rows (tables.write_graph_pickle: the same Graph on
        pickle.load, without per-edge Python inserts)."""
        if self._graph is None and self.engine is not None:
            # the engine's edge records, sorted on the device into every
            # pair's table in combinations order (rc_write_graph)
            from . import _native
            try:
                _native.check(_native.lib().rc_write_graph(self.engine._h, str(path).encode(), 16))
                return
            except _native.NativeError as ex:
                if ex.code != _native.RC_E_STATE:
                    raise
        if self._graph is None and getattr(self.engine, "shard_count", 1) == 1:
            from .tables import write_engine_outputs
            write_engine_outputs(self.engine, list(self._pairs()), None, path)
            return
        if self._graph is None:
            # a sharded run holds every edge but only its own pairs' rows: the
            # exchanged edges as per-pair tables through the same writer
            from .tables import write_graph_pickle
            write_graph_pickle(path, self._edge_tables(), self.labels)
            return
        from .filtering_step import dump_graph
        dump_graph(self.graph, path)

    @property
    def sample_count(self):
        return self._sample_count

    @cached_property
    def valid(self) -> pd.DataFrame:
        """(sample, gene) of every ideal-component node."""
        s, g = self.engine.ideal_nodes()
        return pd.DataFrame({"sample": [self.labels[i] for i in s.tolist()],
                             "gene": g.astype(np.int64)}, columns=["sample", "gene"])

    def restricted(self, comp_df: pd.DataFrame) -> pd.DataFrame:
        """Rows whose (ssample, sgene) and (qsample, qgene) are both valid
        (filtered_distance.py:197-210)."""
        v = set(zip(self.valid["sample"], self.valid["gene"].tolist()))
        keep = np.ones(len(comp_df), dtype=bool)
        for scol, gcol in self.sample_gene_columns:
            keep &= np.fromiter(((s, int(x)) in v for s, x in
                                 zip(comp_df[scol].astype(object), comp_df[gcol])),
                                dtype=bool, count=len(comp_df))
        return comp_df.loc[keep]

    def restricted_comparison_dfs(self):
        src = self._stored.items() if self._stored is not None else self._table_iter()
        for k, df in src:
            yield k, self.restricted(df)

    # ------------------------------------------------------------ numbers
    def pair_sums(self):
        """(num, den) int64 N x N: restricted sums of nident and length - gaps."""
        return self.engine.pair_sums()

    def _sim_pair_iter(self):
        return self._sim_pairs if getattr(self, "_sim_pairs", None) is not None else self._pairs()

    @cached_property
    def similarities(self) -> PairDict:
        num, den = self.pair_sums()
        res = PairDict()
        for a, b in self._sim_pair_iter():
            if den[a, b] == 0:
                raise NoIdealComponentsError()
            res[(self.labels[a], self.labels[b])] = Fraction(int(num[a, b]), int(den[a, b]))
        self._samples = sorted(res.key_elements())
        for s in self._samples:
            res[(s, s)] = 1
        return res

    @classmethod
    def similarity_to_dissimilarity(cls, sim):
        return 1 - sim

    def get_similarities(self) -> PairDict:
        return self.similarities

    def get_dissimilarities(self) -> PairDict:
        return PairDict({k: self.similarity_to_dissimilarity(v)
                         for k, v in self.similarities.items()})

    @property
    def samples(self):
        if self._samples is None:
            if getattr(self, "_sim_pairs", None) is not None:
                self._samples = sorted({self.labels[i] for p in self._sim_pairs for i in p})
            else:
                self._samples = sorted(set(self.labels)) if len(self.labels) > 1 else []
        return self._samples

    def _order(self):
        idx = {l: i for i, l in enumerate(self.labels)}
        return [idx[s] for s in self.samples]

    def get_similarity_matrix(self) -> np.ndarray:
        self.similarities   # raises NoIdealComponentsError like the reference
        num, den = self.pair_sums()
        o = self._order()
        if not o:
            return np.zeros((0, 0))
        n_, d_ = num[np.ix_(o, o)].astype(np.float64), den[np.ix_(o, o)].astype(np.float64)
        out = np.ones((len(o), len(o)))
        off = ~np.eye(len(o), dtype=bool)
        out[off] = n_[off] / d_[off]
        return out

    def get_dissimilarity_matrix(self) -> np.ndarray:
        self.similarities
        if not self.samples:
            return np.zeros((0, 0))
        try:
            _, mat = self.engine.distance(self._order())
        except nat.NativeError as e:
            if e.code == nat.RC_E_NO_IDEAL:
                raise NoIdealComponentsError() from e
            raise
        return mat

    def _matrix_to_df(self, mat):
        return pd.DataFrame(mat).set_axis(self.samples, axis=1).set_axis(self.samples, axis=0)

    def get_similarity_df(self) -> pd.DataFrame:
        return self._matrix_to_df(self.get_similarity_matrix())

    def get_dissimilarity_df(self) -> pd.DataFrame:
        return self._matrix_to_df(self.get_dissimilarity_matrix())


def _table_sums(df: pd.DataFrame):
    """(sum nident, sum length - sum gaps) of one gene matches table, as exact
    ints (similarities_from_dfs, similarity_computer.py:21-42)."""
    return int(df["nident"].sum()), int(df["length"].sum() - df["gaps"].sum())


class UnfilteredSimilarity:
    """Similarities from whole gene matches tables, without the ideal-clique
    filter (unfiltered_distance.py:9-16 over ComparisonSimilarityComputer,
    similarity_computer.py:44-375).

    Built on a finished engine (the sums come from the GPU's per-pair
    reduction over every table row, rc_pair_sums_unfiltered) or on tables
    (`from_dfs` / `from_filenames`: the sums of the given DataFrames). As in
    the reference, a pair whose table is empty makes `similarities` raise
    ZeroDivisionError (Fraction(x, 0))."""

    def __init__(self, engine=None, comparison_dfs=None, sample_count=None):
        if (engine is None) == (comparison_dfs is None):
            raise ValueError("give an engine or comparison_dfs")
        self.engine = engine
        self._comparison_dfs = comparison_dfs
        self._sample_count = sample_count
        self._samples = None

    @classmethod
    def from_dfs(cls, comparison_dfs, sample_count=None):
        """comparison_dfs: iterable of (pair of sample names, table), or a
        mapping with such items (the reference's comparison_dfs forms)."""
        items = comparison_dfs.items() if hasattr(comparison_dfs, "items") else comparison_dfs
        return cls(comparison_dfs=[(tuple(k), df) for k, df in items], sample_count=sample_count)

    @classmethod
    def mapping_from_dfs(cls, dfs):
        """(pair, table) from each table's own qsample/ssample columns
        (similarity_computer.py:90-115; the first row rather than label 0,
        see SURVEY.md Q1)."""
        for df in dfs:
            yield (str(df["qsample"].iloc[0]), str(df["ssample"].iloc[0])), df

    @classmethod
    def from_filenames(cls, paths):
        """Tables written by tables.write_table (this package's own files)."""
        from .tables import read_table
        return cls.from_dfs(list(cls.mapping_from_dfs(read_table(p) for p in paths)))

    # ------------------------------------------------------------ numbers
    def _pair_sums(self):
        """{(a, b): (num, den)} over unordered sample pairs."""
        out = PairDict()
        if self.engine is not None:
            labels = list(self.engine.labels)
            num, den = self.engine.pair_sums(unfiltered=True)
            for a, b in itertools.combinations(range(len(labels)), 2):
                out[(labels[a], labels[b])] = (int(num[a, b]), int(den[a, b]))
        else:
            for (a, b), df in self._comparison_dfs:
                n, d = _table_sums(df)
                if (a, b) in out:
                    n0, d0 = out[(a, b)]
                    n, d = n0 + n, d0 + d
                out[(a, b)] = (n, d)
        return out

    @property
    def sample_count(self):
        if self._sample_count is None:
            self._sample_count = len(self._pair_sums().key_elements())
        return self._sample_count

    @cached_property
    def similarities(self) -> PairDict:
        res = PairDict()
        for k, (n, d) in self._pair_sums().items():
            res[k] = Fraction(n, d)   # ZeroDivisionError on an empty table, as the reference
        self._samples = sorted(res.key_elements())
        for s in self._samples:
            res[(s, s)] = 1
        return res

    similarity_to_dissimilarity = SampleSimilarity.similarity_to_dissimilarity

    def get_similarities(self) -> PairDict:
        return self.similarities

    def get_dissimilarities(self) -> PairDict:
        return PairDict({k: self.similarity_to_dissimilarity(v) for k, v in self.similarities.items()})

    @property
    def samples(self):
        if self._samples is None:
            self.similarities
        return self._samples

    def _pair_dict_to_matrix(self, d) -> np.ndarray:
        s = self.samples
        out = np.zeros((len(s), len(s)))
        for i, a in enumerate(s):
            for j, b in enumerate(s):
                out[i, j] = float(d[(a, b)])   # float(Fraction): correctly rounded
        return out

    def get_similarity_matrix(self) -> np.ndarray:
        return self._pair_dict_to_matrix(self.similarities)

    def get_dissimilarity_matrix(self) -> np.ndarray:
        return self._pair_dict_to_matrix(self.get_dissimilarities())

    def _matrix_to_df(self, mat):
        return pd.DataFrame(mat).set_axis(self.samples, axis=1).set_axis(self.samples, axis=0)

    def get_similarity_df(self) -> pd.DataFrame:
        return self._matrix_to_df(self.get_similarity_matrix())

    def get_dissimilarity_df(self) -> pd.DataFrame:
        return self._matrix_to_df(self.get_dissimilarity_matrix())


def _graph_engine(graph, items, sample_count, device):
    """A graph-only engine for SampleSimilarity(graph, comparison_dfs): every
    sample with one zero-length transcript per gene (the graph's and the
    tables' genes), then one record per graph edge carrying the sums of its
    table rows, sums-only records for table rows whose edge is not in the
    graph, and node records for isolated graph nodes (rc_import_edges)."""
    from .engine import Engine
    genes = {}
    nodes_by_sample = {}
    for s, g in graph.nodes:
        genes.setdefault(str(s), set()).add(int(g))
    tables = []
    for (ka, kb), df in items:
        if not len(df):
            continue
        ss, qs = str(df["ssample"].iloc[0]), str(df["qsample"].iloc[0])
        sg = df["sgene"].to_numpy(dtype=np.int64)
        qg = df["qgene"].to_numpy(dtype=np.int64)
        genes.setdefault(ss, set()).update(np.unique(sg).tolist())
        genes.setdefault(qs, set()).update(np.unique(qg).tolist())
        tables.append((ss, qs, sg, qg, df["nident"].to_numpy(dtype=np.int64),
                       (df["length"].to_numpy(dtype=np.int64) - df["gaps"].to_numpy(dtype=np.int64))))
    for (ka, kb), _ in items:   # samples of empty tables still exist
        genes.setdefault(str(ka), set())
        genes.setdefault(str(kb), set())
    labels = sorted(genes)
    eng = Engine(device=device)
    base, garr = {}, {}
    off = 0
    for lab in labels:
        g = np.array(sorted(genes[lab]), dtype=np.int64)
        garr[lab], base[lab] = g, off
        off += len(g)
        eng.add_sample(lab, np.zeros(0, np.uint8), np.zeros(len(g) + 1, np.uint64), g.astype(np.int32),
                       np.ones(len(g), np.int32))
    pidx = {pr: i for i, pr in enumerate(eng.pair_order())}
    sid = {lab: i for i, lab in enumerate(labels)}

    def node(lab, g):
        return base[lab] + np.searchsorted(garr[lab], g)

    def pair_of(sa, sb):
        a, b = sid[sa], sid[sb]
        return pidx[(min(a, b), max(a, b))]

    # graph edges, keyed by their unordered node pair
    edge_keys = {}
    for (su, gu), (sv, gv) in graph.edges:
        su, sv = str(su), str(sv)
        u, v = int(node(su, int(gu))), int(node(sv, int(gv)))
        edge_keys[(min(u, v), max(u, v))] = pair_of(su, sv) if su != sv else 0
    recs = []
    for ss, qs, sg, qg, ni, dn in tables:
        a, b = node(ss, sg), node(qs, qg)
        lo, hi = np.minimum(a, b), np.maximum(a, b)
        key = lo.astype(np.uint64) << np.uint64(32) | hi.astype(np.uint64)
        uk, inv = np.unique(key, return_inverse=True)
        sn = np.bincount(inv, weights=ni).astype(np.int64)
        sd = np.bincount(inv, weights=dn).astype(np.int64)
        p = pair_of(ss, qs)
        for k, n_, d_ in zip(uk.tolist(), sn.tolist(), sd.tolist()):
            u, v = k >> 32, k & 0xFFFFFFFF
            in_graph = edge_keys.pop((u, v), None) is not None
            recs.append((u, v, p if in_graph else p | nat.RC_EDGE_SUM_ONLY, n_, d_))
    for (u, v), p in edge_keys.items():   # graph edges without table rows
        recs.append((u, v, p, 0, 0))
    for n in graph.nodes:
        if graph.degree(n) == 0:
            u = int(node(str(n[0]), int(n[1])))
            recs.append((u, u, nat.RC_NODE_ONLY, 0, 0))
    arr = np.array(recs, dtype=nat.EDGE_RECORD_DTYPE) if recs else np.zeros(0, nat.EDGE_RECORD_DTYPE)
    if sample_count is not None:
        eng.set_sample_count(int(sample_count))
    eng.import_edges(arr.view(np.uint8))
    return eng
