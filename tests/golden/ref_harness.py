"""Stub-import harness for the reference's post-alignment modules.

TEST INFRASTRUCTURE ONLY. This file runs in the build container (where
/root/reference exists) to capture golden vectors; it is never imported by the
product, by `-m gpu` tests, by `smoke()` or by `bench.py`.

The reference's post-alignment path (find_homologs.HomologFinder.get_match_table,
build_graph.build_graph, filtered_distance.SampleSimilarity,
similarity_computer.*) imports a few things that are absent here:
  * rna_clique.config      -- PEP 695 syntax (config.py:631) does not parse on 3.10;
                              only build_parser()/main() use it, so a placeholder
                              module is enough.
  * simple_blast           -- replaced by a fake TabularBlastnSearch whose `.hits`
                              returns a prepared HSP DataFrame keyed by
                              (query, subject) (find_homologs.py:124 passes
                              (path2, path1) = (query, subject)).
  * multiset_key_dict      -- a small MultisetKeyDict / FrozenMultiset.
  * more_itertools.consume
The stubs replace plumbing and containers only, never arithmetic.
"""
from __future__ import annotations

import collections
import os
import sys
import types

REF_SRC = "/root/reference/src"


class _MultisetKeyDict:
    """Minimal stand-in for multiset_key_dict.MultisetKeyDict.

    Keys are unordered multisets of hashable, sortable elements; they are kept
    canonically as sorted tuples.
    """

    def __init__(self, src=None):
        self._dict = {}
        if src is None:
            return
        items = src.items() if hasattr(src, "items") else src
        for k, v in items:
            self._dict[self._canon(k)] = v

    def __class_getitem__(cls, item):
        return cls

    @staticmethod
    def _canon(k):
        if isinstance(k, _FrozenMultiset):
            return k.key
        return tuple(sorted(k))

    def __getitem__(self, k):
        return self._dict[self._canon(k)]

    def __setitem__(self, k, v):
        self._dict[self._canon(k)] = v

    def __or__(self, other):
        res = _MultisetKeyDict()
        res._dict = dict(self._dict)
        res._dict.update(other._dict)
        return res

    def __len__(self):
        return len(self._dict)

    def items(self):
        return ((_FrozenMultiset(k), v) for k, v in self._dict.items())

    def multiset_iter(self):
        return self.items()

    def __iter__(self):
        return self.multiset_iter()

    def key_elements(self):
        s = set()
        for k in self._dict:
            s.update(k)
        return s


class _FrozenMultiset:
    def __init__(self, elems=()):
        self.key = tuple(sorted(elems))

    def __class_getitem__(cls, item):
        return cls

    def __iter__(self):
        return iter(self.key)

    def __hash__(self):
        return hash(self.key)

    def __eq__(self, other):
        return isinstance(other, _FrozenMultiset) and self.key == other.key


# (query, subject) -> DataFrame of HSP rows, filled by the caller.
FAKE_BLAST_DB: dict = {}


class _FakeTabularBlastnSearch:
    def __init__(self, query, subject, evalue=None, additional_columns=None,
                 db_cache=None, **kw):
        self.query = str(query)
        self.subject = str(subject)
        self._hits = None

    @property
    def hits(self):
        # simple_blast's `hits` is one cached DataFrame per search:
        # find_homologs.py:125-129 mutates it and then reads it again.
        if self._hits is None:
            self._hits = FAKE_BLAST_DB[(self.query, self.subject)].copy()
        return self._hits


class _FakeBlastDBCache:
    def __init__(self, loc):
        self._cache = {}

    def makedb(self, path):
        self._cache[str(path)] = str(path)


def install_stubs():
    """Insert stub modules and put the reference source on sys.path."""
    if "rna_clique.find_homologs" in sys.modules:
        return
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    cfg = types.ModuleType("rna_clique.config")

    class _Placeholder:
        def __init__(self, *a, **k):
            raise RuntimeError("config stub: CLI not available in harness")

    cfg.RNACliqueConfigArgumentManager = _Placeholder
    cfg.RNACliqueConfig = _Placeholder
    sb = types.ModuleType("simple_blast")
    sbb = types.ModuleType("simple_blast.blasting")
    sbb.TabularBlastnSearch = _FakeTabularBlastnSearch
    sb.blasting = sbb
    sb.BlastDBCache = _FakeBlastDBCache
    mkd = types.ModuleType("multiset_key_dict")
    mkd.MultisetKeyDict = _MultisetKeyDict
    mkd.FrozenMultiset = _FrozenMultiset
    mit = types.ModuleType("more_itertools")
    mit.consume = lambda it, n=None: collections.deque(it, maxlen=0)
    sys.modules.update({
        "simple_blast": sb,
        "simple_blast.blasting": sbb,
        "multiset_key_dict": mkd,
        "more_itertools": mit,
    })
    if REF_SRC not in sys.path:
        sys.path.insert(0, REF_SRC)
    import rna_clique  # noqa: F401  (package __init__ is empty)
    sys.modules["rna_clique.config"] = cfg
    rna_clique.config = cfg


def reference_modules():
    install_stubs()
    from rna_clique import find_homologs, build_graph, filtered_distance
    from rna_clique import similarity_computer, transcripts
    return types.SimpleNamespace(
        find_homologs=find_homologs,
        build_graph=build_graph,
        filtered_distance=filtered_distance,
        similarity_computer=similarity_computer,
        transcripts=transcripts,
    )
