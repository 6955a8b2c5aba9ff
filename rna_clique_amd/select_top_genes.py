"""Top-n genes by k-mer coverage (the caller side of the hot path).

Mirrors TopGeneSelector (select_top_genes.py:37-136) and select_top_and_save
(select_top_genes_all.py:12-46) with the same selection rule: a gene's coverage
is the maximum over its isoforms, and the top n are
`heapq.nlargest(n, (coverage, gene))`, so coverage ties go to the larger gene
id. The FASTA passes run in the native reader (csrc/fasta.cpp); only id
parsing is Python.
"""
from __future__ import annotations

import dataclasses
import heapq
import os
import re
from collections import defaultdict
from pathlib import Path
from typing import Callable, Iterable, Iterator

import numpy as np

from .fasta import FastaFile, Record
from .transcripts import TranscriptID, default_parser


def _is_default(parse_transcript_id):
    """The parser is the default rnaSPAdes regex parser (transcripts.py)."""
    from .transcripts import RegexIDParser, default_gene_re
    return (isinstance(parse_transcript_id, RegexIDParser) and parse_transcript_id.cls is TranscriptID
            and parse_transcript_id.expr.pattern == default_gene_re.pattern
            and parse_transcript_id.expr.flags == default_gene_re.flags)


def _fast_default_ids(ids, parse_transcript_id):
    """(coverage float64, gene int64, isoform int64) arrays for the default
    rnaSPAdes pattern in one regex pass over all ids, or None when the parser
    is anything else or some id does not match (the per-id path then raises
    TranscriptIDParseError exactly as the reference does)."""
    from .transcripts import default_gene_re
    if not _is_default(parse_transcript_id):
        return None
    ids = list(ids)
    if any("\n" in i for i in ids):
        return None
    # `^` per line, `.*` never crosses a newline: line i's match is exactly
    # expr.search(ids[i]) (greedy, so the last cov_/_g/_i group of the id)
    rx = re.compile(default_gene_re.pattern, default_gene_re.flags | re.MULTILINE)
    found = rx.findall("\n".join(ids))
    if len(found) != len(ids):
        return None
    if not found:
        return np.zeros(0), np.zeros(0, np.int64), np.zeros(0, np.int64)
    cov_s, gene_s, iso_s = zip(*found)
    cov = np.array([float(c) for c in cov_s], dtype=np.float64)
    return cov, np.array(gene_s, dtype=np.int64), np.array(iso_s, dtype=np.int64)


def _top_from_arrays(cov, genes, isos, top):
    """top_gene_ids on parsed arrays: per gene the max coverage, then
    nlargest(top, (cov, gene)) -- descending by coverage, ties to the larger
    gene id."""
    if top <= 0 or len(genes) == 0:
        return [], genes, isos
    o = np.lexsort((-cov, genes))
    g_sorted = genes[o]
    first = np.ones(len(o), dtype=bool)
    first[1:] = g_sorted[1:] != g_sorted[:-1]
    ug, ucov = g_sorted[first], cov[o][first]
    sel = np.lexsort((-ug, -ucov))[:top]
    return ug[sel].tolist(), genes, isos


def top_gene_ids(ids: Iterable[str], top: int, parse_transcript_id=default_parser):
    """(top gene ids in nlargest order, per-record (gene, isoform) arrays)."""
    ids = list(ids)
    fast = _fast_default_ids(ids, parse_transcript_id)
    if fast is not None:
        return _top_from_arrays(*fast, top)
    best = defaultdict(float)
    genes, isos = [], []
    for id_ in ids:
        cov, gene, iso = parse_transcript_id(id_)
        gene = int(gene)
        genes.append(gene)
        isos.append(int(iso))
        best[gene] = max(best[gene], float(cov))
    top_ids = [k for _, k in heapq.nlargest(top, ((v, k) for k, v in best.items()))]
    return top_ids, np.asarray(genes, dtype=np.int64), np.asarray(isos, dtype=np.int64)


class TopGeneSelector:
    """Select the transcripts of the top n genes by k-mer coverage.

    `transcripts` is a nullary callable returning an iterator of records with
    an `id` attribute (Record, or anything SeqRecord-like)."""

    def __init__(self, transcripts: Callable[[], Iterator[Record]], top: int,
                 parse_transcript_id: Callable[[str], TranscriptID] = default_parser):
        self.transcripts = transcripts
        self.top = top
        self.parse_transcript_id = parse_transcript_id

    def get_top_genes(self) -> Iterator[int]:
        top_ids, _, _ = top_gene_ids((t.id for t in self.transcripts()), self.top,
                                     self.parse_transcript_id)
        yield from top_ids

    def get_top_gene_seqs(self) -> Iterator[Record]:
        keep = set(self.get_top_genes())
        for t in self.transcripts():
            _, gene, _ = self.parse_transcript_id(t.id)
            if int(gene) in keep:
                yield t

    @classmethod
    def from_path(cls, path, *args, **kwargs):
        def it():
            with FastaFile(path) as f:
                yield from f.records()
        return cls(it, *args, **kwargs)

    @classmethod
    def from_sequences(cls, seqs, *args, **kwargs):
        return cls(lambda: seqs, *args, **kwargs)


@dataclasses.dataclass
class TopSample:
    """One sample's top-genes transcripts as the engine takes them."""
    path: Path               # od1/{stem}_top.fasta: the sample's label (A9)
    name: str                # directory stem
    seq: np.ndarray          # uint8 ASCII, concatenated
    tx_offsets: np.ndarray   # uint64, n_tx + 1
    gene: np.ndarray         # int32
    iso: np.ndarray          # int32
    ids_src: object          # the ids (list), or a callable making them on first use

    @property
    def ids(self) -> list:
        if callable(self.ids_src):
            self.ids_src = self.ids_src()
        return self.ids_src

    @property
    def n_tx(self):
        return len(self.gene)


def _int32(a, what):
    if len(a) and (a.min() < -2**31 or a.max() >= 2**31):
        raise ValueError(f"{what} id outside int32 (the reference downcasts to int32, "
                         "find_homologs.py:58-80)")
    return a.astype(np.int32)


def select_top_sample(out_dir, transcripts: str, x, top: int,
                      parse_transcript_id=default_parser, write=True) -> TopSample:
    """select_top_and_save plus the arrays for the engine, in one FASTA pass.

    Writes `out_dir/{x.stem}_top.fasta` (Bio.SeqIO layout, 60 columns) unless
    write=False."""
    x = Path(x)
    out = Path(out_dir) / (x.stem + "_top.fasta")
    with FastaFile(x / transcripts) as f:
        parsed = f.parse_rnaspades() if _is_default(parse_transcript_id) else None
        if parsed is not None:
            top_ids, genes, isos = _top_from_arrays(*parsed, top)
        else:
            top_ids, genes, isos = top_gene_ids(f.ids, top, parse_transcript_id)
        keep = np.isin(genes, np.asarray(top_ids, dtype=np.int64)).astype(np.uint8)
        if write:
            f.write(out, keep)
        seq, offs = f.select(keep)
        sel = keep.astype(bool)
    # the kept ids are only decoded when someone asks (titles stay in f)
    return TopSample(out, x.stem, seq, offs, _int32(genes[sel], "gene"),
                     _int32(isos[sel], "isoform"),
                     lambda: [i for i, k in zip(f.ids, sel) if k])


def select_top_and_save(out_dir, transcripts: str, x, *args):
    """Reference signature (select_top_genes_all.py:12-46): returns
    (path of the written top-genes FASTA, sample name)."""
    s = select_top_sample(out_dir, transcripts, x, *args)
    return s.path, s.name


def load_top_fasta(path, parse_transcript_id=default_parser, name=None) -> TopSample:
    """Read an existing top-genes FASTA (e.g. od1/X_top.fasta) whole."""
    path = Path(path)
    with FastaFile(path) as f:
        genes, isos = [], []
        for id_ in f.ids:
            _, g, i = parse_transcript_id(id_)
            genes.append(int(g))
            isos.append(int(i))
        seq, offs = f.select(None)
        ids = list(f.ids)
    stem = path.stem[:-4] if path.stem.endswith("_top") else path.stem
    return TopSample(path, name or stem, seq, offs,
                     _int32(np.asarray(genes, dtype=np.int64), "gene"),
                     _int32(np.asarray(isos, dtype=np.int64), "isoform"), ids)
