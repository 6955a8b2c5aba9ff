"""filtering_step: phase 1 of RNA-clique (filtering_step.py:61-164).

Top-gene selection per sample (od1/{stem}_top.fasta), the gene matches table
of every pair (od2, find_all_pairs), and the gene matches graph pickled to
`output_graph` (build_graph). Same arguments and return value as the
reference: (tables read back from disk, table paths, graph, number of
tables, {top-genes FASTA path: sample name}).
"""
from __future__ import annotations

import itertools
import multiprocessing
import os
import pickle
from pathlib import Path
from typing import Callable, Iterable

from .find_all_pairs import find_all_pairs
from .rna_clique import select_all
from .tables import build_graph
from .transcripts import TranscriptID, default_gene_re


def dump_graph(graph, path):
    """graph.pkl as filtering_step.py:158-159 writes it (written atomically)."""
    tmp = str(path) + ".tmp"
    with open(tmp, "wb") as f:
        pickle.dump(graph, f, pickle.HIGHEST_PROTOCOL)
    os.replace(tmp, path)


def filtering_step(dirs: Iterable[Path], out_dir_1: Path, out_dir_2: Path, cache_dir: Path,
                   output_graph: Path, top_genes: int, transcripts: str = "transcripts.fasta",
                   top_matches: int = 1,
                   id_parser: Callable = TranscriptID.parser_from_re(default_gene_re),
                   evalue: float = 1e-99, keep_all: bool = True,
                   jobs: int = multiprocessing.cpu_count() - 1, *, device: int = 0, process_group=None):
    from .similarity import SampleSimilarity
    samples = select_all(dirs, out_dir_1, transcripts, top_genes, id_parser, max(1, jobs))
    path_to_sample = {s.path: s.name for s in samples}
    eng = []
    tables, table_paths, num_tables = find_all_pairs(
        path_to_sample, out_dir_2, cache_dir, path_to_sample.__getitem__,
        hf_args=[id_parser, top_matches, evalue, keep_all], jobs=jobs, device=device,
        process_group=process_group, engine_out=eng)
    # a sharded run holds only its own pairs' tables, but every edge
    graph = build_graph(tables) if eng[0].shard_count == 1 else SampleSimilarity.from_engine(eng[0]).graph
    dump_graph(graph, output_graph)
    paths1, paths2 = itertools.tee(table_paths)
    return map(SampleSimilarity._read_table, paths1), paths2, graph, num_tables, path_to_sample
