"""ctypes front end of the C alignment oracle (oracle/align_oracle.c).

TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py cpu_baseline). Builds the
oracle with `make -C oracle` on first use when the library is missing.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liborc.so")


class OrcHsp(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in ("q_tx", "s_tx")] + \
               [(n, ctypes.c_int32) for n in (
                   "qstart", "qend", "sstart", "send", "length", "nident",
                   "mismatch", "gaps", "gapopen", "score_half", "bits10",
                   "strand")] + [("evalue", ctypes.c_double)]


class OrcParams(ctypes.Structure):
    _fields_ = [("word_size", ctypes.c_int32), ("xdrop_half", ctypes.c_int32),
                ("evalue", ctypes.c_double), ("symmetric", ctypes.c_int32),
                ("dust_level", ctypes.c_int32), ("dust_window", ctypes.c_int32),
                ("dust_linker", ctypes.c_int32)]


# base codes of the oracle: A C G T (either case) -> 0..3, anything else 4
CODE_LUT = np.full(256, 4, dtype=np.uint8)
for _i, _c in enumerate(b"ACGT"):
    CODE_LUT[_c] = CODE_LUT[_c | 0x20] = _i


HSP_DTYPE = np.dtype([(n, np.uint32) for n in ("q_tx", "s_tx")] +
                     [(n, np.int32) for n in (
                         "qstart", "qend", "sstart", "send", "length", "nident",
                         "mismatch", "gaps", "gapopen", "score_half", "bits10",
                         "strand")] + [("evalue", np.float64)])
assert HSP_DTYPE.itemsize == ctypes.sizeof(OrcHsp)

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-C", HERE], check=True,
                           stdout=subprocess.DEVNULL)
        L = ctypes.CDLL(LIB)
        P = ctypes.POINTER
        L.orc_align.argtypes = [
            ctypes.c_char_p, ctypes.c_uint64, P(ctypes.c_uint64), P(ctypes.c_int32),
            ctypes.c_uint32, P(ctypes.c_uint32), P(ctypes.c_uint32), ctypes.c_uint32,
            P(ctypes.c_int32), ctypes.c_int32, ctypes.c_int32, P(OrcParams),
            P(P(OrcHsp)), P(ctypes.c_uint64)]
        L.orc_align.restype = ctypes.c_int
        L.orc_align_codes.argtypes = [ctypes.c_void_p] + L.orc_align.argtypes[2:]
        L.orc_align_codes.restype = ctypes.c_int
        L.orc_free.argtypes = [ctypes.c_void_p]
        L.orc_dust.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                               ctypes.c_int32, ctypes.c_void_p]
        L.orc_bits10.argtypes = [ctypes.c_int32]
        L.orc_bits10.restype = ctypes.c_int32
        L.orc_threshold.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                    ctypes.c_double]
        L.orc_threshold.restype = ctypes.c_int32
        L.orc_evalue.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                 ctypes.c_int32]
        L.orc_evalue.restype = ctypes.c_double
        _lib = L
    return _lib


class OracleDB:
    """All samples concatenated, with the global transcript and gene numbering
    the engine also uses: transcripts sample-major in input order; genes
    per sample in ascending gene id, sample-major; a gene's transcripts in
    input order."""

    def __init__(self, samples):
        self.samples = samples
        seqs, starts, tx_sample, genes_all = [], [0], [], []
        self.tx_base = []
        base = 0
        for si, s in enumerate(samples):
            self.tx_base.append(len(tx_sample))
            seqs.append(np.asarray(s.seq, dtype=np.uint8))
            offs = np.asarray(s.tx_offsets, dtype=np.uint64)
            starts.extend((offs[1:] + base).tolist())
            base += int(offs[-1])
            tx_sample.extend([si] * s.n_tx)
        self.codes = CODE_LUT[np.concatenate(seqs)] if seqs else np.zeros(1, np.uint8)
        self.tx_start = np.array(starts, dtype=np.uint64)
        self.tx_sample = np.array(tx_sample, dtype=np.int32)
        gene_tx_off, gene_tx, gene_sample, gene_id = [0], [], [], []
        self.tx_gene = np.zeros(len(tx_sample), dtype=np.int64)
        for si, s in enumerate(samples):
            # genes in ascending id, each gene's transcripts in input order (a
            # stable sort by gene id)
            g = np.asarray(s.gene)
            order = np.argsort(g, kind="stable")
            gids, first, counts = np.unique(g[order], return_index=True, return_counts=True)
            members = order + self.tx_base[si]
            self.tx_gene[members] = len(gene_sample) + np.repeat(np.arange(len(gids)), counts)
            gene_tx.extend(members.tolist())
            gene_tx_off.extend((len(gene_tx) - len(members) + first + counts).tolist())
            gene_sample.extend([si] * len(gids))
            gene_id.extend(gids.tolist())
        self.gene_tx_off = np.array(gene_tx_off, dtype=np.uint32)
        self.gene_tx = np.array(gene_tx, dtype=np.uint32)
        self.gene_sample = np.array(gene_sample, dtype=np.int32)
        self.gene_id = np.array(gene_id, dtype=np.int64)

    def align(self, qsample, tsample, word_size=28, xdrop_half=108, evalue=1e-99,
              symmetric=False, dust=None):
        """One directed search (query sample qsample, subject tsample).
        symmetric: spec 5b (the pair extended once, the higher-numbered
        sample's search reported as mirror images); default: the search run
        on its own, as BLAST runs each direction. dust: (level, window,
        linker) of symmetric DUST on the query, or None."""
        L = lib()
        P = ctypes.POINTER
        out = P(OrcHsp)()
        n = ctypes.c_uint64()
        dl, dw, dk = dust if dust else (0, 64, 1)
        prm = OrcParams(word_size, xdrop_half, evalue, 1 if symmetric else 0, dl, dw, dk)
        rc = L.orc_align_codes(
            self.codes.ctypes.data_as(ctypes.c_void_p),
            self.tx_start.ctypes.data_as(P(ctypes.c_uint64)),
            self.tx_sample.ctypes.data_as(P(ctypes.c_int32)),
            len(self.tx_sample),
            self.gene_tx_off.ctypes.data_as(P(ctypes.c_uint32)),
            self.gene_tx.ctypes.data_as(P(ctypes.c_uint32)),
            len(self.gene_sample),
            self.gene_sample.ctypes.data_as(P(ctypes.c_int32)),
            qsample, tsample, ctypes.byref(prm), ctypes.byref(out), ctypes.byref(n))
        if rc != 0:
            raise RuntimeError(f"orc_align failed: {rc}")
        buf = np.ctypeslib.as_array(out, shape=(n.value,)) if n.value else None
        res = np.zeros(n.value, dtype=HSP_DTYPE)
        if n.value:
            res[:] = np.frombuffer(
                ctypes.string_at(out, n.value * HSP_DTYPE.itemsize), dtype=HSP_DTYPE)
        L.orc_free(out)
        del buf
        return res

    def dust_mask(self, sample, level=20, window=64, linker=1):
        """The oracle's DUST mask (spec 1b) of one sample's transcripts,
        concatenated (uint8 per base)."""
        L = lib()
        out = []
        for t in range(self.tx_base[sample], self.tx_base[sample] + self.samples[sample].n_tx):
            a, b = int(self.tx_start[t]), int(self.tx_start[t + 1])
            c = np.ascontiguousarray(self.codes[a:b])
            m = np.zeros(max(1, b - a), dtype=np.uint8)
            L.orc_dust(c.ctypes.data_as(ctypes.c_void_p), b - a, level, window, linker,
                       m.ctypes.data_as(ctypes.c_void_p))
            out.append(m[:b - a])
        return np.concatenate(out) if out else np.zeros(0, np.uint8)

    def hsp_rows(self, hsps):
        """Oracle HSPs -> BLAST-tabular-like dicts (for oracle.post_oracle)."""
        rows = []
        for h in hsps:
            q, s = int(h["q_tx"]), int(h["s_tx"])
            rows.append({
                "qgene_id": int(self.gene_id[self.tx_gene[q]]),
                "sgene_id": int(self.gene_id[self.tx_gene[s]]),
                "q_tx": q, "s_tx": s,
                **{k: int(h[k]) for k in ("qstart", "qend", "sstart", "send",
                                         "length", "nident", "mismatch", "gaps",
                                         "gapopen", "score_half", "bits10",
                                         "strand")},
                "evalue": float(h["evalue"])})
        return rows
