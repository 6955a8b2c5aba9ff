"""Synthetic transcriptomes for tests and benchmarks.

The reference's own test data come from its `distance_sequence_simulator`
submodule, which is empty in this checkout (.gitmodules:1-3). This generator
follows the configuration the reference's install test feeds it
(tests/verify_install/minimal_config.yaml:1-39):

* a birth-death tree (birth 1.0, death 0.5) grown until `taxa` lineages exist;
* transcript lengths `loc + Binomial(n, p)` (1950 + B(1000, 0.1) there);
* HKY85 substitutions along every branch at `mutation_rate` substitutions per
  site per unit branch length (equal base frequencies, kappa = 2);
* coverage Uniform(0, 10000), printed with decimals so that the default
  transcript-ID regex (transcripts.py:8) parses it, distinct per gene;
* ids "NODE_cov_{cov}_g{gene}_i{iso}".

Extras for correctness runs (all off by default):
* p_iso2: a fraction of genes gets a second isoform with a skipped internal
  segment (alternative splicing); rich_genes x rich_iso: genes with many
  isoforms (different skipped segments, every taxon);
* indel_rate: short insertions/deletions;
* p_revcomp: per taxon, genes whose transcripts are reported on the other
  strand (assemblers orient transcripts arbitrarily: minus-strand hits);
* p_paralog: genes duplicated in one random taxon (a recent copy with 0-0.5 %
  divergence: reciprocal-best-hit ties and non-ideal components);
* polya = (fraction, lo, hi): poly-A tails of lo..hi bases on a fraction of
  transcripts (low-complexity sequence shared by unrelated transcripts).
Gene ids are permuted per taxon so nothing can rely on ortholog ids matching.
"""
from __future__ import annotations

import dataclasses
import math

import numpy as np

_BASES = np.frombuffer(b"ACGT", dtype=np.uint8)


@dataclasses.dataclass
class Sample:
    """One taxon's transcriptome, kept as flat arrays (FASTA-free)."""
    name: str
    seq: np.ndarray          # uint8 ASCII, all transcripts concatenated
    tx_offsets: np.ndarray   # uint64, n_tx + 1
    gene: np.ndarray         # int32 gene id per transcript
    iso: np.ndarray          # int32 isoform id per transcript
    cov: np.ndarray          # float64 coverage per transcript

    @property
    def n_tx(self):
        return len(self.gene)

    def ids(self):
        return [f"NODE_cov_{c:.6f}_g{g}_i{i}" for c, g, i in
                zip(self.cov, self.gene, self.iso)]

    def transcript(self, t):
        return self.seq[self.tx_offsets[t]:self.tx_offsets[t + 1]].tobytes().decode()

    def write_fasta(self, path, width=80):
        """FASTA with `width`-column sequence lines (bytes-level, no per-base
        Python work)."""
        seq = self.seq.tobytes()
        offs = self.tx_offsets
        parts = []
        for t, name in enumerate(self.ids()):
            a, b = int(offs[t]), int(offs[t + 1])
            parts.append(b">" + name.encode() + b"\n")
            parts.append(b"\n".join(seq[k:min(k + width, b)] for k in range(a, b, width)))
            parts.append(b"\n")
        with open(path, "wb") as f:
            f.write(b"".join(parts))


def birth_death_tree(taxa, rng, birth=1.0, death=0.5):
    """Grow a birth-death tree until `taxa` lineages are alive.

    Returns (parent, branch_length, leaves) with node 0 the root.
    """
    while True:
        parent, blen, start = [-1], [0.0], [0.0]
        alive = [0]
        t = 0.0
        while 0 < len(alive) < taxa:
            rate = len(alive) * (birth + death)
            t += rng.exponential(1.0 / rate)
            k = int(rng.integers(len(alive)))
            node = alive.pop(k)
            blen[node] = t - start[node]
            if rng.random() < birth / (birth + death):
                for _ in range(2):
                    parent.append(node)
                    blen.append(0.0)
                    start.append(t)
                    alive.append(len(parent) - 1)
        if len(alive) == taxa:
            t += rng.exponential(1.0 / (len(alive) * (birth + death)))
            for a in alive:
                blen[a] = t - start[a]
            return np.array(parent), np.array(blen), sorted(alive)


def _hky85_mutate(seq, expected_subs, rng, kappa=2.0):
    """Substitutions on uint8 codes 0..3 (A C G T) for one branch."""
    # with equal base frequencies HKY85's total rate splits into transitions
    # (A<->G, C<->T) with weight kappa and two transversions with weight 1
    n = seq.size
    p_change = 1.0 - math.exp(-expected_subs)
    k = rng.binomial(n, p_change)
    if k == 0:
        return seq
    pos = rng.choice(n, size=k, replace=False)
    r = rng.random(k) * (kappa + 2.0)
    old = seq[pos]
    transition = old ^ 2                  # A(0)<->G(2), C(1)<->T(3)
    tv1 = old ^ 1
    tv2 = old ^ 3
    new = np.where(r < kappa, transition, np.where(r < kappa + 1.0, tv1, tv2))
    out = seq.copy()
    out[pos] = new.astype(np.uint8)
    return out


def _hky85_mutate_sparse(seq, expected_subs, rng, kappa=2.0, inplace=False):
    """_hky85_mutate for long sequences: site draws with replacement, repeats
    dropped (k^2 / 2n of k sites, ~0.2 % at C5), so no O(n) choice; inplace
    reuses `seq` (its last use)."""
    n = seq.size
    k = rng.binomial(n, 1.0 - math.exp(-expected_subs))
    if k == 0:
        # a copy unless this is the parent's last use: a sibling mutated in
        # place later must not rewrite this one
        return seq if inplace else seq.copy()
    pos = np.unique(rng.integers(0, n, size=k))
    r = rng.random(pos.size) * (kappa + 2.0)
    old = seq[pos]
    new = np.where(r < kappa, old ^ 2, np.where(r < kappa + 1.0, old ^ 1, old ^ 3))
    out = seq if inplace else seq.copy()
    out[pos] = new.astype(np.uint8)
    return out


_ASCII_TABLE = bytes(_BASES.tolist()) + bytes(252)


def _ascii(codes):
    """uint8 codes 0..3 -> ASCII bases (bytes.translate: ~10x a fancy index)."""
    return np.frombuffer(codes.tobytes().translate(_ASCII_TABLE), dtype=np.uint8)


def _indels(gene_seqs, rate, rng):
    """Short insertions/deletions (1-6 bp) at `rate` per base."""
    out = []
    for s in gene_seqs:
        k = rng.binomial(s.size, rate)
        if k == 0:
            out.append(s)
            continue
        s = s.tolist()
        for _ in range(k):
            p = int(rng.integers(len(s)))
            ln = int(rng.integers(1, 7))
            if rng.random() < 0.5:
                del s[p:p + ln]
            else:
                s[p:p] = rng.integers(0, 4, size=ln).tolist()
        out.append(np.array(s, dtype=np.uint8))
    return out


def _revcomp(codes):
    return (3 - codes[::-1]).astype(np.uint8)


def simulate(taxa, genes, seed=487, len_loc=1950, len_n=1000, len_p=0.1,
             len_uniform=None, mutation_rate=0.01, p_iso2=0.0, indel_rate=0.0,
             permute_genes=True, prefix="T", p_revcomp=0.0, p_paralog=0.0,
             rich_genes=0, rich_iso=1, polya=None, node_rng=False, only=None):
    """Simulate `taxa` transcriptomes with `genes` orthologous genes each.

    len_uniform=(lo, hi) draws lengths uniformly instead of loc + Binomial.
    node_rng: every tree node's substitutions and every leaf's own draws come
    from their own seeded stream (default_rng([seed, 2, node]) and
    default_rng([seed, 3, leaf index])), so any subset of the leaves can be
    generated alone with the same bases -- the C5 mode (33 Gbp; a shard needs
    only its own samples).
    only: with node_rng, the leaf indices whose sequences are generated; the
    other samples come back with seq None and their metadata (transcript
    offsets, gene and isoform ids, coverage), as a shard that does not align
    them adds them (rc_add_sample with seq NULL).
    Returns (samples, tree) where tree = (parent, branch_length, leaves).
    """
    plain = (p_iso2 == 0 and indel_rate == 0 and p_revcomp == 0 and p_paralog == 0
             and not rich_genes and polya is None)
    if only is not None and not (node_rng and plain):
        raise ValueError("only= needs node_rng=True and no per-gene extras")
    rng = np.random.default_rng(seed)
    parent, blen, leaves = birth_death_tree(taxa, rng)
    if len_uniform is not None:
        lengths = rng.integers(len_uniform[0], len_uniform[1] + 1, size=genes)
    else:
        lengths = len_loc + rng.binomial(len_n, len_p, size=genes)
    total = int(lengths.sum())
    offs = np.zeros(genes + 1, dtype=np.int64)
    offs[1:] = np.cumsum(lengths)
    children = {}
    for v, p in enumerate(parent):
        if p >= 0:
            children.setdefault(int(p), []).append(v)
    wanted = set(range(len(leaves))) if only is None else {int(i) for i in only}
    # nodes on the way to a wanted leaf (node_rng: the other subtrees are skipped)
    live = set()
    for li in wanted:
        v = int(leaves[li])
        while v >= 0 and v not in live:
            live.add(v)
            v = int(parent[v])
    if node_rng:
        root = np.random.default_rng([seed, 1]).integers(0, 4, size=total, dtype=np.uint8)
    else:
        root = rng.integers(0, 4, size=total, dtype=np.uint8)
    # depth-first, keeping only the sequences still needed
    seqs = {0: root}
    leaf_seq = {}
    stack = [0]
    while stack:
        v = stack.pop()
        s = seqs.pop(v)
        kids = children.get(v, [])
        if not kids:
            leaf_seq[v] = s
            continue
        live_kids = [c for c in kids if c in live]
        for c in kids:
            if node_rng:
                if c in live:
                    seqs[c] = _hky85_mutate_sparse(s, mutation_rate * blen[c], np.random.default_rng([seed, 2, c]),
                                                   inplace=c == live_kids[-1])
                    stack.append(c)
            else:
                seqs[c] = _hky85_mutate(s, mutation_rate * blen[c], rng)
                stack.append(c)
        del s
    iso2 = rng.random(genes) < p_iso2
    rich = set(rng.choice(genes, size=min(rich_genes, genes), replace=False).tolist()) if rich_genes else set()
    # skipped segments of the isoform-rich genes, shared by every taxon
    rich_cuts = {g: [(int(a), int(a) + int(w)) for a, w in zip(
        rng.integers(50, max(51, lengths[g] - 200), size=rich_iso - 1),
        rng.integers(30, 120, size=rich_iso - 1))] for g in sorted(rich)}
    # (draws only for enabled extras: the default data stay those of earlier rounds)
    paralog_taxon = np.full(genes, -1)
    paralog_div = np.zeros(genes)
    if p_paralog > 0:
        paralog_taxon = np.where(rng.random(genes) < p_paralog, rng.integers(0, taxa, size=genes), -1)
        paralog_div = rng.choice([0.0, 0.002, 0.005], size=genes)
    cov = rng.uniform(0, 10000, size=genes)
    samples = []
    for li, leaf in enumerate(leaves):
        lrng = np.random.default_rng([seed, 3, li]) if node_rng else rng
        if plain:
            # one isoform per gene in gene order: the transcripts are the leaf
            # sequence itself (the same data the per-gene loop below builds)
            gid = (lrng.permutation(genes) if permute_genes else np.arange(genes)) + 1
            tcov = cov * lrng.uniform(0.9, 1.1, size=genes)
            s = leaf_seq.pop(leaf, None)
            samples.append(Sample(
                name=f"{prefix}{li}", seq=None if s is None else _ascii(s),
                tx_offsets=offs.astype(np.uint64), gene=gid.astype(np.int32),
                iso=np.ones(genes, dtype=np.int32), cov=tcov.astype(np.float64)))
            del s
            continue
        rng = lrng
        s = leaf_seq[leaf]
        gseqs = [s[offs[g]:offs[g + 1]] for g in range(genes)]
        if indel_rate > 0:
            gseqs = _indels(gseqs, indel_rate, rng)
        n_par = int((paralog_taxon == li).sum())
        gid = (rng.permutation(genes + n_par) if permute_genes else np.arange(genes + n_par)) + 1
        flip = rng.random(genes + n_par) < p_revcomp if p_revcomp > 0 else np.zeros(genes + n_par, bool)
        parts, gene_l, iso_l, cov_l = [], [], [], []
        # per-taxon coverage jitter keeps top-n selection meaningful but distinct
        tcov = cov * rng.uniform(0.9, 1.1, size=genes)
        extra = genes
        for g in range(genes):
            copies = [(g, gseqs[g], tcov[g])]
            if paralog_taxon[g] == li:
                dup = _hky85_mutate(gseqs[g], paralog_div[g], rng) if paralog_div[g] > 0 else gseqs[g]
                copies.append((extra, dup, tcov[g] * 0.77))
                extra += 1
            for k, gs, cv in copies:
                isos = [gs]
                if g in rich:
                    isos += [np.concatenate([gs[:a], gs[b:]]) for a, b in rich_cuts[g] if b < gs.size]
                elif iso2[g] and gs.size > 400:
                    a = int(rng.integers(100, gs.size // 2))
                    b = a + int(rng.integers(60, 160))
                    isos.append(np.concatenate([gs[:a], gs[b:]]))
                for i, t in enumerate(isos):
                    if polya is not None and rng.random() < polya[0]:
                        t = np.concatenate([t, np.zeros(int(rng.integers(polya[1], polya[2] + 1)), np.uint8)])
                    parts.append(_revcomp(t) if flip[k] else t)
                    gene_l.append(gid[k]); iso_l.append(i + 1); cov_l.append(cv * (0.5 ** i))
        lens = np.array([p.size for p in parts], dtype=np.uint64)
        txo = np.zeros(len(parts) + 1, dtype=np.uint64)
        txo[1:] = np.cumsum(lens)
        codes = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
        samples.append(Sample(
            name=f"{prefix}{li}",
            seq=_BASES[codes],
            tx_offsets=txo,
            gene=np.array(gene_l, dtype=np.int32),
            iso=np.array(iso_l, dtype=np.int32),
            cov=np.array(cov_l, dtype=np.float64)))
    return samples, (parent, blen, leaves)


# BASELINE.json configs.
CONFIGS = {
    "C1": dict(taxa=4, genes=1000, seed=487),
    "C2": dict(taxa=8, genes=10000, seed=488),
    "C3": dict(taxa=32, genes=50000, seed=489, len_loc=950, len_n=100, len_p=0.5),
    "C4": dict(taxa=64, genes=50000, seed=490, len_loc=950, len_n=100, len_p=0.5),
    # C5 uses per-node random streams: one shard's samples can be generated alone
    "C5": dict(taxa=128, genes=100000, seed=491, len_uniform=(200, 5000), node_rng=True),
    # C5's tree is deep (its deepest pair 22.3 branch-length units apart, C4's
    # 8.1): at minimal_config's rate 0.01 that pair differs at ~19 % of sites
    # and no gene keeps a reciprocal best hit in all 8128 pairs, so no ideal
    # 128-clique exists and the reference raises NoIdealComponentsError. C5s:
    # the same samples' shape and tree at rate 0.0036 (deepest pair ~8 %, C4's)
    "C5s": dict(taxa=128, genes=100000, seed=491, len_uniform=(200, 5000), node_rng=True, mutation_rate=0.0036),
    # C3 with the features of real transcriptomes (correctness variant of the
    # GPU tests; a bench workload too): 10 % two-isoform genes, indels, half the
    # genes on the minus strand, 2 % recent paralogs, poly-A tails on 20 %
    "C3v": dict(taxa=32, genes=50000, seed=489, len_loc=950, len_n=100, len_p=0.5, p_iso2=0.1,
                indel_rate=0.002, p_revcomp=0.5, p_paralog=0.02, polya=(0.2, 15, 40)),
}
