"""find_all_pairs: the gene matches table of every pair of samples.

Mirrors the reference's entry point (find_all_pairs.py:161-233): the same
arguments and return value -- (tables, table paths, C(N, 2)) -- and the same
table files `{output_dir}/{sample1}--{sample2}.{ext}` for the pairs of
`itertools.combinations(inputs, 2)` (make_output_path, :90-117; ssample =
the first path, qsample = the second, find_homologs_and_save :57-88).

Underneath, instead of a BLAST database per sample and 2 x C(N, 2) blastn
subprocesses on a process pool, all pairs run at once in one engine on the
GPU (librcgpu.so); with an initialised torch.distributed group the pairs are
sharded across ranks (distributed.py) and each rank writes the tables of the
pairs it owns. `cache_dir` (the BLAST database cache) is accepted and unused.
Tables are written as HDF5 in pandas' "table" format under key
"gene_matches" (`write_table`; without PyTables, h5.write_frame_table),
on a thread pool of `jobs` workers.
"""
from __future__ import annotations

import itertools
import multiprocessing
import threading
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path
from typing import Callable, Iterable, Optional

from .select_top_genes import load_top_fasta
from .tables import pair_table, rows_to_table, write_table
from .transcripts import TranscriptID, default_gene_re


def table_extension() -> str:
    """h5, as the reference writes them (pandas table format; written without
    PyTables when it is absent, h5.write_frame_table)."""
    return "h5"


def make_output_path(dir_: Path, t1: Path, t2: Path, path_to_sample: Optional[Callable] = None,
                     extension: str = "h5") -> Path:
    """find_all_pairs.py:90-117."""
    ts = [t1, t2]
    if path_to_sample:
        ts = [path_to_sample(t) for t in ts]
    return Path(dir_) / "{}--{}.{}".format(*ts, extension)


def find_all_pairs(inputs: Iterable[Path], output_dir: Path, cache_dir: Optional[Path],
                   path_to_sample: Callable[[Path], str], hf_args: Iterable = (),
                   jobs: int = multiprocessing.cpu_count() - 1, *, device: int = 0,
                   process_group=None, engine_out: Optional[list] = None):
    """Gene matches tables for all pairs of input samples (top-genes FASTA
    paths). hf_args = [id_parser, top_matches, evalue, keep_all] as
    HomologFinder takes them. Returns (tables, table paths, number of tables);
    the tables are written before this returns. engine_out, if given,
    receives the engine (its graph, sums and distances stay on the GPU)."""
    from .rna_clique import run_engine
    inputs = list(inputs)
    hf = list(hf_args)
    id_parser = hf[0] if len(hf) > 0 else TranscriptID.parser_from_re(default_gene_re)
    top_matches = hf[1] if len(hf) > 1 else 1
    evalue = hf[2] if len(hf) > 2 else 1e-99
    keep_all = hf[3] if len(hf) > 3 else True
    samples = [load_top_fasta(p, id_parser) for p in inputs]
    eng = run_engine(samples, top_matches, evalue, keep_all, device, process_group)
    if engine_out is not None:
        engine_out.append(eng)
    ext = table_extension()
    out_paths = write_pair_tables(eng, inputs, output_dir, path_to_sample, ext, jobs)

    def tables():
        for a, b in itertools.combinations(range(len(inputs)), 2):
            if (a, b) in out_paths:
                yield pair_table(eng, a, b)
    # the table files in combinations order; a sharded run (rank of a
    # torch.distributed group) returns the pairs it owns and wrote only, and
    # counts those (unsharded: all C(N, 2), the reference's count)
    paths = (out_paths[ab] for ab in itertools.combinations(range(len(inputs)), 2) if ab in out_paths)
    return tables(), paths, len(out_paths)


def write_pair_tables(eng, inputs, output_dir, path_to_sample, ext, jobs: int = 8, graph_path=None) -> dict:
    """Write the tables of the pairs this engine owns; {(a, b): path}. .h5
    tables (and graph.pkl when `graph_path` is given: build_graph over every
    pair, a single-shard engine) are written natively in one pass
    (tables.write_engine_outputs); .pkl tables through pandas."""
    output_dir = Path(output_dir)
    output_dir.mkdir(parents=True, exist_ok=True)
    own = set(eng.owned_pairs())
    out = {}
    for a, b in itertools.combinations(range(len(inputs)), 2):
        if (a, b) in own:
            out[(a, b)] = make_output_path(output_dir, inputs[a], inputs[b], path_to_sample, ext)
    if ext == "h5":
        from .tables import write_engine_outputs
        write_engine_outputs(eng, list(out), [out[p] for p in out], graph_path, max(1, jobs))
        return out
    if graph_path is not None:
        raise ValueError("graph_path is written with .h5 tables only")
    labels = eng.labels
    lock = threading.Lock()

    def one(ab):
        with lock:   # the engine's device -> host copies, one pair at a time
            rows = eng.pair_rows(*ab)
        write_table(rows_to_table(rows, labels[ab[0]], labels[ab[1]]), out[ab])
    # table building and writing are numpy / file work: threads overlap them
    with ThreadPoolExecutor(max_workers=max(1, min(jobs, len(out)))) as ex:
        list(ex.map(one, list(out)))
    return out
