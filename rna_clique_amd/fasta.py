"""FASTA files through the native reader (rc_fasta_*, csrc/fasta.cpp).

One mmap'd pass splits records; titles come back to Python for id parsing;
selected sequences are copied straight into the flat arrays the engine takes.
There is no Python fallback: the reader is part of librcgpu.so.
"""
from __future__ import annotations

import ctypes
import os
from typing import NamedTuple

import numpy as np

from . import _native as nat
from .transcripts import fasta_id


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
        raw = buf[:tb.value].tobytes()
        o = offs.tolist()
        self.titles = [raw[o[i]:o[i + 1]].decode("utf-8", errors="replace")
                       for i in range(n.value)]
        self.ids = [fasta_id(t) for t in self.titles]

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
