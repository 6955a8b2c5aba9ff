"""SampleSimilarity over the GPU engine.

Same interface as the reference's SampleSimilarity / ComparisonSimilarityComputer
(filtered_distance.py:129-247, similarity_computer.py:44-375), but every number
comes from librcgpu.so: the gene matches graph, its connected components and
ideal-clique filter, the restricted sums and the distances are computed on the
GPU. Tables and the networkx graph are only materialised on request.

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
    """Similarities of the samples of one finished engine run."""

    sample_gene_columns = [[a + b for b in ["sample", "gene"]] for a in ["s", "q"]]
    categorical_columns = ["qsample", "ssample", "sstrand"]

    def __init__(self, engine, store_dfs: bool = False, sample_count=None):
        self.engine = engine
        self.labels = list(engine.labels)
        st = engine.stats()
        if sample_count is not None and sample_count != st["sample_count"]:
            raise ValueError("a sample_count other than the graph's is not supported")
        self._sample_count = st["sample_count"]
        self._stored = PairDict(self._table_iter()) if store_dfs else None
        self._samples = None

    # ------------------------------------------------------------ tables
    def _pairs(self):
        return itertools.combinations(range(len(self.labels)), 2)

    def _table_iter(self):
        for a, b in self._pairs():
            yield (self.labels[a], self.labels[b]), pair_table(self.engine, a, b, self.labels)

    @property
    def comparison_dfs(self):
        """Pair -> gene matches table (a PairDict when store_dfs, else a fresh
        generator of (pair, table))."""
        return self._stored if self._stored is not None else self._table_iter()

    @cached_property
    def graph(self):
        """The gene matches graph (networkx), as build_graph.py:40-68 makes it.
        A sharded engine holds only its own pairs' tables, but every shard has
        all graph edges after the exchange: the graph is built from those
        (same nodes and edges; insertion order by pair, then edge)."""
        if getattr(self.engine, "shard_count", 1) > 1:
            import networkx as nx
            e = self.engine.edges()
            g = nx.Graph()
            for r in e.tolist():
                d = dict(zip(e.dtype.names, r))
                g.add_edge((self.labels[d["sample_a"]], int(d["gene_a"])),
                           (self.labels[d["sample_b"]], int(d["gene_b"])))
            return g

        def rows():
            for a, b in self._pairs():
                yield self.labels[a], self.labels[b], self.engine.pair_rows(a, b)
        return build_graph(rows())

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

    @cached_property
    def similarities(self) -> PairDict:
        num, den = self.pair_sums()
        res = PairDict()
        for a, b in self._pairs():
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
