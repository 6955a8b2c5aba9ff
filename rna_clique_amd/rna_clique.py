"""rna_clique(): the reference's top-level API over the GPU engine.

Same parameters and return value as the reference (rna_clique.py:28-178):
top-genes selection per input directory -> all-pairs alignment, gene matches
tables, gene matches graph and ideal-clique filter -> SampleSimilarity, with
the distance matrix written to `output_matrix` under key "matrix".

What changes underneath:
* steps 2-6 run in librcgpu.so (hand-written HIP for gfx950) for the whole
  pair set at once instead of C(N,2) pairs of blastn subprocesses plus pandas
  and networkx;
* `cache_dir` (BLAST DB cache) is accepted and unused: the seed index lives in
  HBM and is rebuilt per run;
* gene matches tables are written to `out_dir_2` as `{s1}--{s2}.h5`
  (write_table, gene_matches_tables.py:42-56: pandas table format, key
  "gene_matches", written without PyTables when it is absent;
  `table_format="pkl"` writes pickles, "none" skips them);
* `output_graph` is the networkx pickle of build_graph (filtering_step.py:
  158-159), written by a native pickle writer from the engine's rows (the
  same Graph on pickle.load, without building it in Python);
* `jobs` bounds the host threads of the top-genes step.
"""
from __future__ import annotations

import multiprocessing
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path
from typing import Callable, Iterable, Optional

from .engine import Engine
from .h5 import write_matrix
from .select_top_genes import select_top_sample
from .similarity import NoIdealComponentsError, SampleSimilarity  # noqa: F401
from .transcripts import TranscriptID, TranscriptIDParseError, default_gene_re  # noqa: F401


def select_iter(dirs, out_dir_1, transcripts, top_genes, id_parser, jobs=1):
    """select_top_and_save over every input directory (filtering_step.py:
    129-143) on `jobs` threads, yielded in input order as each completes."""
    dirs = [Path(d) for d in dirs]
    Path(out_dir_1).mkdir(parents=True, exist_ok=True)
    work = lambda d: select_top_sample(out_dir_1, transcripts, d, top_genes, id_parser)  # noqa: E731
    if jobs <= 1 or len(dirs) <= 1:
        yield from (work(d) for d in dirs)
        return
    with ThreadPoolExecutor(max_workers=min(jobs, len(dirs))) as ex:
        yield from ex.map(work, dirs)


def select_all(dirs, out_dir_1, transcripts, top_genes, id_parser, jobs=1):
    """select_iter as a list."""
    return list(select_iter(dirs, out_dir_1, transcripts, top_genes, id_parser, jobs))


def run_engine(samples, top_matches=1, evalue=1e-99, keep_all=True, device=0,
               process_group=None, loaded=None, **engine_kwargs) -> Engine:
    """Load the samples (labels = top-genes FASTA paths) and run the whole
    path. With an initialised torch.distributed group of size > 1 the sample
    pairs are sharded across ranks (see distributed.py). `samples` may be an
    iterator (one GPU: each sample goes to the device as it arrives, beside
    the selection of the next ones); `loaded(list)` is called with all of them
    before the run."""
    from . import distributed
    world, rank = distributed.world(process_group)
    eng = Engine(top_matches=top_matches, keep_all=keep_all, evalue=evalue,
                 device=device, shard_rank=rank, shard_count=world, **engine_kwargs)
    if world > 1:
        # a shard holds the sequences of its own pairs' samples only
        samples = list(samples)
        need = distributed.needed_samples([int(s.tx_offsets[-1]) for s in samples], world, rank)
    got = []
    for i, s in enumerate(samples):
        eng.add_sample(str(s.path), s.seq if world == 1 or i in need else None, s.tx_offsets, s.gene, s.iso)
        got.append(s)
    if loaded is not None:
        loaded(got)
    if world == 1:
        eng.run()
    else:
        distributed.sharded_run(eng, process_group)
    return eng


def rna_clique(
        dirs: Iterable[Path],
        out_dir_1: Path,
        out_dir_2: Optional[Path],
        cache_dir: Optional[Path],
        output_graph: Optional[Path],
        output_matrix: Optional[Path],
        top_genes: int,
        transcripts: str = "transcripts.fasta",
        top_matches: int = 1,
        id_parser: Callable[[str], TranscriptID] = TranscriptID.parser_from_re(default_gene_re),
        evalue: float = 1e-99,
        keep_all: bool = True,
        store_dfs: bool = False,
        jobs: int = multiprocessing.cpu_count() - 1,
        *,
        device: int = 0,
        table_format: Optional[str] = None,
        process_group=None,
) -> tuple[SampleSimilarity, dict[Path, str]]:
    """Full RNA-clique analysis of the transcriptomes in `dirs` (see the
    module docstring for what differs from the reference underneath).

    Returns (SampleSimilarity, {top-genes FASTA path: sample name})."""
    import time
    t0 = time.perf_counter()
    # the selection of later samples runs beside the upload of earlier ones
    got, t1 = [], [0.0]

    def loaded(ss):
        got.extend(ss)
        t1[0] = time.perf_counter()
    eng = run_engine(select_iter(dirs, out_dir_1, transcripts, top_genes, id_parser, max(1, jobs)),
                     top_matches, evalue, keep_all, device, process_group, loaded=loaded)
    samples, t1 = got, t1[0]
    pts = {s.path: s.name for s in samples}
    t2 = time.perf_counter()
    sim = SampleSimilarity.from_engine(eng, store_dfs=store_dfs)
    from . import distributed
    writer = distributed.world(process_group)[1] == 0
    # matrix.h5 as soon as the distances exist: it does not wait for the
    # tables or graph.pkl (the reference writes graph.pkl first,
    # filtering_step.py:157-159 then rna_clique.py:175-177; the outputs are
    # independent)
    if writer and output_matrix is not None:
        write_matrix(sim.get_dissimilarity_df(), output_matrix)
    t3 = time.perf_counter()
    graph_done = False
    if out_dir_2 is not None and table_format != "none":
        # every rank writes the tables of the pairs it owns (all of them on one
        # GPU); on one GPU, graph.pkl is written in the same native pass
        from .find_all_pairs import table_extension, write_pair_tables
        ext = table_format or table_extension()
        gpath = output_graph if (writer and output_graph is not None and ext == "h5"
                                 and eng.shard_count == 1) else None
        write_pair_tables(eng, [s.path for s in samples], out_dir_2, pts.__getitem__, ext, max(1, jobs),
                          graph_path=gpath)
        graph_done = gpath is not None
    t4 = time.perf_counter()
    if writer and output_graph is not None and not graph_done:
        sim.write_graph(output_graph)
    last_timings.clear()
    last_timings.update(select_s=t1 - t0, engine_s=t2 - t1, matrix_s=t3 - t2, tables_s=t4 - t3,
                        graph_s=time.perf_counter() - t4, to_matrix_s=t3 - t0)
    return sim, pts


# wall-clock phases of the last rna_clique() call in this process (seconds):
# top-gene selection with the inputs' upload beside it, engine (GPU path),
# matrix.h5, od2 tables (+ graph.pkl on one GPU), graph.pkl (sharded runs);
# to_matrix_s: from the call to matrix.h5 on disk
last_timings: dict = {}
