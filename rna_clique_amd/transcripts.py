"""Transcript FASTA ids -> (coverage, gene, isoform).

Same contract as the reference's transcripts module (transcripts.py:8-126):

* `default_gene_re` is the rnaSPAdes pattern; the coverage group requires a
  decimal point.
* A parser made by `TranscriptID.parser_from_re(expr)` takes each field from
  the group of the same name when the pattern has one; the fields without a
  named group take the pattern's unnamed groups in order (coverage, gene,
  isoform). No match, or too few groups, raises TranscriptIDParseError.
* TranscriptID converts its fields on construction (float, int, int).

Id parsing stays on the host (user-supplied regex); everything downstream of
it runs on the GPU.
"""
from __future__ import annotations

import re
from typing import Callable, NamedTuple

default_gene_re = re.compile(r"^.*cov_([0-9]+(?:\.[0-9]+))_g([0-9]+)_i([0-9]+)")


class TranscriptIDParseError(Exception):
    pass


class _TranscriptIDBase(NamedTuple):
    coverage: float
    gene: int
    isoform: int


class TranscriptID(_TranscriptIDBase):
    """(coverage, gene, isoform) of one transcript, converted on construction."""

    def __new__(cls, coverage, gene, isoform):
        return super().__new__(cls, float(coverage), int(gene), int(isoform))

    @classmethod
    def parser_from_re(cls, expr: re.Pattern | str) -> Callable[[str], "TranscriptID"]:
        return RegexIDParser(expr, cls)


class RegexIDParser:
    """Callable id parser for one compiled pattern (picklable, unlike a
    closure, so it can travel to worker processes)."""

    FIELDS = ("coverage", "gene", "isoform")

    def __init__(self, expr, cls=TranscriptID):
        self.expr = re.compile(expr) if isinstance(expr, str) else expr
        self.cls = cls
        named = self.expr.groupindex
        self._named = [f for f in self.FIELDS if f in named]
        rest = [f for f in self.FIELDS if f not in named]
        taken = set(named.values())
        unnamed = [i for i in range(1, self.expr.groups + 2) if i not in taken]
        # a field whose group index exceeds the pattern's groups fails at parse
        # time, as in the reference (transcripts.py:111-122)
        self._positional = list(zip(rest, unnamed))
        self._short = len(unnamed) < len(rest)

    def __call__(self, id_: str) -> TranscriptID:
        m = self.expr.search(id_)
        if m is None or self._short:
            raise TranscriptIDParseError(f"Could not parse transcript ID {id_}.")
        d = {f: m.group(f) for f in self._named}
        for f, i in self._positional:
            if i > self.expr.groups:
                raise TranscriptIDParseError(f"Could not parse transcript ID {id_}.")
            d[f] = m.group(i)
        return self.cls(**d)

    def __repr__(self):
        return f"RegexIDParser({self.expr.pattern!r})"


default_parser = TranscriptID.parser_from_re(default_gene_re)


def fasta_id(title: str) -> str:
    """Bio.SeqIO's record id: the title's first whitespace-separated token."""
    parts = title.split(None, 1)
    return parts[0] if parts else ""
