"""FASTA files through the native reader (rc_fasta_*, csrc/fasta.cpp).

One mmap'd pass splits records; titles come back to Python for id parsing;
selected sequences are copied straight into the flat arrays the engine takes.
There is no Python fallback: the reader is part of librcgpu.so.
"""
from __future__ import annotations

import ctypes
import os
import re
from typing import NamedTuple

import numpy as np

from . import _native as nat
from .transcripts import fasta_id

# whitespace str.split() splits on, other than the newline separator
_WS = re.compile(r"[ \t\r\x0b\x0c\x1c-\x1f\x85\xa0\u1680\u2000-\u200a\u2028\u2029\u202f\u205f\u3000]")


class Record(NamedTuple):
    """The parts of a Bio.SeqRecord the pipeline uses."""
    id: str
    description: str
    seq: str


class FastaFile:
    """A parsed FASTA file. `titles[i]` is record i's header line (without
    '>'), `ids[i]` its first token, `lengths[i]` its sequence length."""

    def __init__(self, path):
        self.path = os.fspath(path)
        h = ctypes.c_void_p()
        nat.check(nat.lib().rc_fasta_open(self.path.encode(), ctypes.byref(h)))
        self._h = h
        n, nb, tb = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        nat.check(nat.lib().rc_fasta_info(h, ctypes.byref(n), ctypes.byref(nb), ctypes.byref(tb)))
        self.n_records, self.n_bases = n.value, nb.value
        buf = np.zeros(max(tb.value, 1), dtype=np.uint8)
        offs = np.zeros(n.value + 1, dtype=np.uint64)
        self.lengths = np.zeros(n.value, dtype=np.uint64)
        nat.check(nat.lib().rc_fasta_titles(h, buf.ctypes.data_as(ctypes.c_void_p),
                                            offs.ctypes.data_as(ctypes.c_void_p),
                                            self.lengths.ctypes.data_as(ctypes.c_void_p)))
        self._tbuf, self._toffs = buf[:tb.value], offs
        self._titles = self._ids = None

    @property
    def titles(self):
        """Header lines (decoded on first use: one decode of the titles joined
        by newlines -- a title never holds one, and an ASCII newline ends any
        broken UTF-8 sequence exactly where a per-title decode would)."""
        if self._titles is None:
            if self.n_records:
                joined = np.insert(self._tbuf, self._toffs[1:-1].astype(np.int64), ord("\n"))
                self._titles = joined.tobytes().decode("utf-8", errors="replace").split("\n")
            else:
                self._titles = []
        return self._titles

    @property
    def ids(self):
        """Record ids: each title's first whitespace-separated token."""
        if self._ids is None:
            t = self.titles
            if _WS.search("\n".join(t)) is None:
                self._ids = list(t)   # no whitespace: the id is the whole title
            else:
                self._ids = [fasta_id(x) for x in t]
        return self._ids

    def parse_rnaspades(self):
        """(coverage float64, gene int64, isoform int64) per record under the
        default rnaSPAdes id pattern, parsed natively; None when some record is
        undecided there (the caller parses with the regex instead)."""
        n = self.n_records
        cov = np.zeros(n, dtype=np.float64)
        gene = np.zeros(n, dtype=np.int64)
        iso = np.zeros(n, dtype=np.int64)
        bad = ctypes.c_uint64()
        nat.check(nat.lib().rc_fasta_parse_rnaspades(
            self._h, cov.ctypes.data_as(ctypes.c_void_p), gene.ctypes.data_as(ctypes.c_void_p),
            iso.ctypes.data_as(ctypes.c_void_p), ctypes.byref(bad)))
        return None if bad.value else (cov, gene, iso)

    def close(self):
        if getattr(self, "_h", None):
            nat.lib().rc_fasta_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __len__(self):
        return self.n_records

    def _mask(self, keep):
        if keep is None:
            return None, self.n_records, int(self.lengths.sum())
        keep = np.ascontiguousarray(keep, dtype=np.uint8)
        if len(keep) != self.n_records:
            raise ValueError("keep mask must have one entry per record")
        return keep, int(keep.sum()), int(self.lengths[keep.astype(bool)].sum())

    def select(self, keep=None):
        """(seq uint8 ASCII, tx_offsets uint64[n+1]) of the kept records."""
        keep, n, nb = self._mask(keep)
        seq = np.zeros(max(nb, 1), dtype=np.uint8)
        offs = np.zeros(n + 1, dtype=np.uint64)
        nat.check(nat.lib().rc_fasta_select(
            self._h, None if keep is None else keep.ctypes.data_as(ctypes.c_void_p),
            seq.ctypes.data_as(ctypes.c_void_p), offs.ctypes.data_as(ctypes.c_void_p)))
        return seq[:nb], offs

    def write(self, path, keep=None, width=60):
        """Write the kept records as Bio.SeqIO.write(records, path, "fasta")."""
        keep, _, _ = self._mask(keep)
        nat.check(nat.lib().rc_fasta_write(
            self._h, None if keep is None else keep.ctypes.data_as(ctypes.c_void_p),
            os.fspath(path).encode(), int(width)))

    def records(self, keep=None):
        """Iterate Record(id, description, seq) of the kept records."""
        seq, offs = self.select(keep)
        idx = range(self.n_records) if keep is None else np.flatnonzero(np.asarray(keep))
        for k, i in enumerate(idx):
            yield Record(self.ids[i], self.titles[i],
                         seq[offs[k]:offs[k + 1]].tobytes().decode("ascii", errors="replace"))
