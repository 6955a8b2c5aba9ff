"""Single sample pair: the gene matches table of two top-genes FASTA files.

Mirrors the reference's HomologFinder (find_homologs.py:166-325): the same
constructor arguments and `get_match_table(transcripts1, transcripts2)`, which
returns the table of the pair with qgene/qiso from transcripts2 and
sgene/siso from transcripts1 (find_homologs.py:215-302; schema
docs/formats.md:231-252, without the ssample/qsample columns that
find_all_pairs adds). Underneath, the two directed BLAST searches and the
pandas merges are one engine run on the GPU over the two samples.

`match_table_similarity` is the number find_homologs' CLI prints
(find_homologs.py:355-362): Fraction(sum nident, sum length - sum gaps) over
the whole table.
"""
from __future__ import annotations

from fractions import Fraction
from pathlib import Path
from typing import Callable, Optional

import pandas as pd

from .engine import Engine
from .select_top_genes import load_top_fasta
from .tables import rows_to_table
from .transcripts import TranscriptID


class HomologFinder:
    """Gene matches tables for pairs of transcriptomes (find_homologs.py:166)."""

    merge_columns = ["qgene", "sgene"]

    def __init__(self, parse_transcript_id: Callable[[str], TranscriptID], top_n: int,
                 evalue: float, keep_all: bool, debug: bool = False, *, device: int = 0,
                 **engine_kwargs):
        assert top_n is not None
        self.parse_transcript_id = parse_transcript_id
        self.top_n = top_n
        self.evalue = evalue
        self.keep_all = keep_all
        self.debug = debug
        self.device = device
        self.engine_kwargs = engine_kwargs

    def get_match_table(self, transcripts1: Path, transcripts2: Path) -> pd.DataFrame:
        t1 = load_top_fasta(transcripts1, self.parse_transcript_id)
        t2 = load_top_fasta(transcripts2, self.parse_transcript_id)
        with Engine(top_matches=self.top_n, keep_all=self.keep_all, evalue=self.evalue,
                    device=self.device, **self.engine_kwargs) as eng:
            eng.add_sample(str(t1.path), t1.seq, t1.tx_offsets, t1.gene, t1.iso)
            eng.add_sample(str(t2.path), t2.seq, t2.tx_offsets, t2.gene, t2.iso)
            eng.run()
            rows = eng.pair_rows(0, 1)
        table = rows_to_table(rows, str(t1.path), str(t2.path))
        return table.drop(columns=["ssample", "qsample"])

    @classmethod
    def without_duplicates(cls, df: pd.DataFrame, columns: Optional[list] = None) -> pd.DataFrame:
        """The given columns (default merge_columns) without duplicate rows
        (find_homologs.py:308-323)."""
        if columns is None:
            columns = cls.merge_columns
        return df[columns].drop_duplicates()


def match_table_similarity(table: pd.DataFrame) -> Fraction:
    """Fraction(sum nident, sum length - sum gaps) over a whole table
    (find_homologs.py:355-362)."""
    return Fraction(int(table["nident"].sum()), int(table["length"].sum() - table["gaps"].sum()))


def main(argv=None):
    """The find_homologs command (find_homologs.py:327-363): one sample pair's
    gene matches, then the pair's distance as a Fraction (or a float with -f):
    prints the deduplicated (qgene, sgene) matches unless -q, "Found N
    matches." on stderr. `python -m rna_clique_amd.find_homologs T1 T2`."""
    import argparse
    import sys
    from .transcripts import TranscriptIDParseError, default_gene_re
    ap = argparse.ArgumentParser(description="Compute a genetic distance for one pair of samples.")
    ap.add_argument("--transcript-id-regex", default=default_gene_re.pattern,
                    help="regex with the gene and isoform groups of a transcript ID")
    ap.add_argument("--evalue", type=float, default=1e-99)
    ap.add_argument("--top-matches", type=int, default=1)
    ap.add_argument("--keep-all", type=lambda v: str(v).lower() in ("1", "true", "yes"), default=True)
    ap.add_argument("transcripts1", type=Path, help="path to the (top n) transcripts for the first sample")
    ap.add_argument("transcripts2", type=Path, help="path to the (top n) transcripts for the second sample")
    ap.add_argument("-q", "--quiet", action="store_true", help="hide the matches found")
    ap.add_argument("-f", "--report-float", action="store_true", help="report float instead of fraction")
    args = ap.parse_args(argv)
    finder = HomologFinder(TranscriptID.parser_from_re(args.transcript_id_regex), args.top_matches,
                           args.evalue, args.keep_all)
    try:
        best = finder.get_match_table(args.transcripts1, args.transcripts2)
    except TranscriptIDParseError:
        print(f"Could not parse a transcript ID with the regex {args.transcript_id_regex!r}.", file=sys.stderr)
        raise
    dedup = finder.without_duplicates(best)
    if not args.quiet:
        for match in dedup.itertuples(index=False):
            print(*match)
    print(f"Found {len(dedup)} matches.", file=sys.stderr)
    dist = match_table_similarity(best)
    print(float(dist) if args.report_float else dist)


if __name__ == "__main__":
    main()
