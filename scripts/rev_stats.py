"""Reverse-pass statistics (shared searches with DUST) on the GPU test corpora:
near-mask index entries and reverse-only seeds per dataset, plus a parity
check of each run against the oracle. Usage: python scripts/rev_stats.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oracle.parity import full_check  # noqa: E402
from rna_clique_amd.engine import Engine  # noqa: E402
from rna_clique_amd.simulate import simulate  # noqa: E402

CASES = {
    "modes": dict(taxa=4, genes=120, seed=12, p_iso2=0.2, indel_rate=0.003, p_revcomp=0.5, polya=(0.3, 10, 40)),
    "polya_rich": dict(taxa=3, genes=150, seed=13, polya=(0.5, 5, 120)),
    "repeats": dict(taxa=3, genes=60, seed=14, len_loc=1200, len_n=400, len_p=0.5, rich_genes=3, rich_iso=30,
                    p_iso2=0.1, polya=(0.6, 20, 60)),
}

for name, kw in CASES.items():
    samples, _ = simulate(**kw)
    with Engine(device=0) as eng:
        for s in samples:
            eng.add_sample(s.name, s.seq, s.tx_offsets, s.gene, s.iso)
        eng.run()
        tm = eng.timings()
        msgs, summary = full_check(eng, samples)
    print(f"{name}: near_index {tm['near_index']:.0f} reverse_seeds {tm['reverse_seeds']:.0f} "
          f"hsps {summary['hsps']} parity {'ok' if not msgs else 'FAIL ' + msgs[0]}", flush=True)
