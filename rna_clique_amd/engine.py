"""Python handle over one native engine (one GPU).

Thin wrapper: inputs are copied into the engine, all compute runs in
librcgpu.so (hand-written HIP for gfx950), results come back as numpy arrays.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as nat


class Engine:
    """One engine = one device. Samples are numbered in the order they are
    added (the reference's `inputs` order)."""

    def __init__(self, top_matches=1, keep_all=True, evalue=1e-99, word_size=28,
                 xdrop_half=108, device=0, shard_rank=0, shard_count=1, symmetric=False,
                 dust=None):
        """dust: None = the default (rc_default_opts), False = off, or
        (level, window, linker)."""
        L = nat.lib()
        o = nat.RcOpts()
        L.rc_default_opts(ctypes.byref(o))
        o.top_matches = int(top_matches)
        o.keep_all = 1 if keep_all else 0
        o.evalue = float(evalue)
        o.word_size = int(word_size)
        o.xdrop_half = int(xdrop_half)
        o.device = int(device)
        o.shard_rank = int(shard_rank)
        o.shard_count = int(shard_count)
        o.symmetric = 1 if symmetric else 0
        if dust is False:
            o.dust_level = 0
        elif dust is not None:
            o.dust_level, o.dust_window, o.dust_linker = (int(v) for v in dust)
        self.symmetric = bool(symmetric)
        self.dust = (o.dust_level, o.dust_window, o.dust_linker) if o.dust_level else None
        h = ctypes.c_void_p()
        nat.check(L.rc_create(ctypes.byref(o), ctypes.byref(h)))
        self._h = h
        self.labels = []
        self.n_tx = []
        self.bases = []      # each sample's sequence length (resident or not)
        self.resident = []
        self.shard_count = int(shard_count)

    def close(self):
        if getattr(self, "_h", None):
            nat.lib().rc_destroy(self._h)
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

    # ------------------------------------------------------------- inputs
    def add_sample(self, label, seq, tx_offsets, gene, iso):
        """seq None: a sample this engine does not align (a sharded run holds
        only the samples of its own pairs) -- its transcripts and genes still
        count for the graph and the e-value statistics."""
        seq = None if seq is None else np.ascontiguousarray(seq, dtype=np.uint8)
        offs = np.ascontiguousarray(tx_offsets, dtype=np.uint64)
        gene = np.ascontiguousarray(gene, dtype=np.int32)
        iso = np.ascontiguousarray(iso, dtype=np.int32)
        n_tx = len(gene)
        if len(offs) != n_tx + 1 or len(iso) != n_tx:
            raise ValueError("tx_offsets must have n_tx + 1 entries, iso n_tx")
        sid = ctypes.c_int32()
        P = ctypes.POINTER
        nat.check(nat.lib().rc_add_sample(
            self._h, str(label).encode(), None if seq is None else seq.ctypes.data_as(ctypes.c_char_p),
            offs.ctypes.data_as(P(ctypes.c_uint64)), gene.ctypes.data_as(P(ctypes.c_int32)),
            iso.ctypes.data_as(P(ctypes.c_int32)), n_tx, ctypes.byref(sid)))
        self.labels.append(str(label))
        self.n_tx.append(n_tx)
        self.bases.append(int(offs[-1]) if n_tx else 0)
        self.resident.append(seq is not None)
        return sid.value

    def add_hsps(self, q, s, hsps):
        arr = np.ascontiguousarray(hsps, dtype=nat.HSP_DTYPE)
        nat.check(nat.lib().rc_add_hsps(self._h, int(q), int(s),
                                        arr.ctypes.data_as(ctypes.c_void_p), len(arr)))

    # ------------------------------------------------------------- phases
    def upload(self):
        nat.check(nat.lib().rc_upload(self._h))

    def run(self):
        nat.check(nat.lib().rc_run(self._h))

    def align(self):
        nat.check(nat.lib().rc_align(self._h))

    def finish(self):
        nat.check(nat.lib().rc_finish(self._h))

    def pair_order(self):
        """The engine's pair numbering [(a, b), ...], a < b: shard by shard,
        subject-major inside a shard (rc_pair_order; one shard: (0,1), (0,2),
        (1,2), (0,3), ...)."""
        n = len(self.labels)
        m = n * (n - 1) // 2
        pa, pb = np.zeros(max(m, 1), dtype=np.int32), np.zeros(max(m, 1), dtype=np.int32)
        nat.check(nat.lib().rc_pair_order(self._h, pa.ctypes.data_as(ctypes.c_void_p),
                                          pb.ctypes.data_as(ctypes.c_void_p)))
        return list(zip(pa[:m].tolist(), pb[:m].tolist()))

    def owned_pairs(self):
        """(a, b) pairs whose tables this shard holds."""
        first, last = self.shard_pairs()
        return self.pair_order()[first:last]

    def shard_pairs(self):
        """[first, last) of this shard's sample pairs in pair_order()."""
        a, b = ctypes.c_int64(), ctypes.c_int64()
        nat.check(nat.lib().rc_shard_pairs(self._h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def local_edge_count(self):
        n = ctypes.c_uint64()
        nat.check(nat.lib().rc_export_edges(self._h, None, 0, ctypes.byref(n), 0))
        return n.value

    @staticmethod
    def edge_record_size():
        return int(nat.lib().rc_edge_record_size())

    def export_edges(self, out=None):
        """This shard's graph edges as opaque records: into `out` (a uint8
        tensor: CUDA, written device-to-device, or CPU) or a new host uint8
        array."""
        L = nat.lib()
        n = ctypes.c_uint64()
        nat.check(L.rc_export_edges(self._h, None, 0, ctypes.byref(n), 0))
        rs = self.edge_record_size()
        if out is not None:
            if out.numel() < n.value * rs:
                raise ValueError("edge buffer too small")
            if n.value:
                nat.check(L.rc_export_edges(self._h, ctypes.c_void_p(out.data_ptr()), n.value,
                                            ctypes.byref(n), 1 if out.is_cuda else 0))
            return n.value
        buf = np.zeros(n.value * rs, dtype=np.uint8)
        if n.value:
            nat.check(L.rc_export_edges(self._h, buf.ctypes.data_as(ctypes.c_void_p), n.value,
                                        ctypes.byref(n), 0))
        return buf

    def set_sample_count(self, sample_count):
        """The ideal-component test's sample count (0: from the graph)."""
        nat.check(nat.lib().rc_set_sample_count(self._h, int(sample_count)))

    def import_edges(self, buf, n=None):
        """All shards' edges (host uint8 array, or CUDA tensor + record count)
        -> graph, ideal filter, pair sums."""
        L = nat.lib()
        rs = self.edge_record_size()
        if isinstance(buf, np.ndarray):
            buf = np.ascontiguousarray(buf, dtype=np.uint8)
            if len(buf) % rs:
                raise ValueError("edge buffer size is not a multiple of the record size")
            nat.check(L.rc_import_edges(self._h, buf.ctypes.data_as(ctypes.c_void_p), len(buf) // rs, 0))
        else:
            n = buf.numel() // rs if n is None else int(n)
            nat.check(L.rc_import_edges(self._h, ctypes.c_void_p(buf.data_ptr()), n, 1))

    def import_edge_parts(self, buf, counts, stride):
        """import_edges from blocks: block r starts at record r * stride of
        `buf` (a CUDA uint8 tensor or host uint8 array) and holds counts[r]
        records -- e.g. an all-gather's padded receive buffer as it is."""
        L = nat.lib()
        c = np.ascontiguousarray(counts, dtype=np.uint64)
        if not isinstance(buf, np.ndarray) and not buf.is_cuda:
            buf = buf.numpy()
        if isinstance(buf, np.ndarray):
            buf = np.ascontiguousarray(buf, dtype=np.uint8)
            ptr, dev = buf.ctypes.data_as(ctypes.c_void_p), 0
        else:
            ptr, dev = ctypes.c_void_p(buf.data_ptr()), 1
        nat.check(L.rc_import_edge_parts(self._h, ptr, c.ctypes.data_as(ctypes.c_void_p), len(c), int(stride), dev))

    def trim(self):
        """Free the alignment working set of a finished run (rc_trim): rows,
        HSPs and edges stay; the next align() allocates it again."""
        nat.check(nat.lib().rc_trim(self._h))

    # ------------------------------------------------------------- results
    def _sized(self, fn, dtype, *args):
        n = ctypes.c_uint64()
        nat.check(fn(self._h, *args, None, 0, ctypes.byref(n)))
        out = np.zeros(n.value, dtype=dtype)
        if n.value:
            nat.check(fn(self._h, *args, out.ctypes.data_as(ctypes.c_void_p), n.value,
                         ctypes.byref(n)))
        return out

    def hsps(self, q, s):
        return self._sized(nat.lib().rc_hsps, nat.HSP_DTYPE, int(q), int(s))

    def pair_rows(self, s1, s2):
        return self._sized(nat.lib().rc_pair_rows, nat.ROW_DTYPE, int(s1), int(s2))

    def edges(self):
        return self._sized(nat.lib().rc_edges, nat.EDGE_DTYPE)

    def ideal_nodes(self):
        L = nat.lib()
        n = ctypes.c_uint64()
        nat.check(L.rc_ideal_nodes(self._h, None, None, 0, ctypes.byref(n)))
        s = np.zeros(n.value, dtype=np.int32)
        g = np.zeros(n.value, dtype=np.int32)
        nat.check(L.rc_ideal_nodes(self._h, s.ctypes.data_as(ctypes.c_void_p),
                                   g.ctypes.data_as(ctypes.c_void_p), n.value, ctypes.byref(n)))
        return s, g

    def stats(self):
        st = nat.RcStats()
        nat.check(nat.lib().rc_graph_stats(self._h, ctypes.byref(st)))
        return {k: getattr(st, k) for k, _ in nat.RcStats._fields_ if k != "pad"}

    def pair_sums(self, unfiltered=False):
        """(num, den) int64 N x N: sums of nident and of length - gaps over the
        rows of each pair's gene matches table inside ideal components, or
        over all of them (unfiltered=True)."""
        n = len(self.labels)
        num = np.zeros((n, n), dtype=np.int64)
        den = np.zeros((n, n), dtype=np.int64)
        fn = nat.lib().rc_pair_sums_unfiltered if unfiltered else nat.lib().rc_pair_sums
        nat.check(fn(self._h, num.ctypes.data_as(ctypes.c_void_p), den.ctypes.data_as(ctypes.c_void_p)))
        return num, den

    def distance(self, order=None):
        """Distances with rows/columns in `order` (default: every sample in
        sorted label order, similarity_computer.py:220; a subset of the
        samples gives their matrix only). Raises NativeError(RC_E_NO_IDEAL)
        when a pair has no ideal rows."""
        n = len(self.labels)
        if order is None:
            order = sorted(range(n), key=lambda i: self.labels[i])
        order = np.ascontiguousarray(order, dtype=np.int32)
        m = len(order)
        out = np.zeros((m, m), dtype=np.float64)
        nat.check(nat.lib().rc_distance_subset(self._h, order.ctypes.data_as(ctypes.c_void_p), m,
                                               out.ctypes.data_as(ctypes.c_void_p)))
        return [self.labels[i] for i in order], out

    def dust_mask(self, s):
        """DUST mask of sample s (uint8 per base, 1 = masked query base)."""
        return self._sized(nat.lib().rc_dust_mask, np.uint8, int(s))

    def dust_masks(self, samples, out=None):
        """The DUST masks of resident samples, computed in a pass of their own
        (before align): uint64 words, ceil(bases / 64) per sample in the given
        order (rc_dust_masks). Into `out` (a CUDA uint64/int64 tensor, device
        to device) or a new host array."""
        L = nat.lib()
        ss = np.ascontiguousarray(list(samples), dtype=np.int32)
        sp = ss.ctypes.data_as(ctypes.c_void_p)
        n = ctypes.c_uint64()
        nat.check(L.rc_dust_masks(self._h, sp, len(ss), None, 0, ctypes.byref(n), 0))
        if out is not None:
            if out.numel() < n.value:
                raise ValueError("mask buffer too small")
            nat.check(L.rc_dust_masks(self._h, sp, len(ss), ctypes.c_void_p(out.data_ptr()), n.value,
                                      ctypes.byref(n), 1))
            return n.value
        buf = np.zeros(n.value, dtype=np.uint64)
        nat.check(L.rc_dust_masks(self._h, sp, len(ss), buf.ctypes.data_as(ctypes.c_void_p), n.value,
                                  ctypes.byref(n), 0))
        return buf

    def set_dust_masks(self, samples, bits):
        """Masks for these samples (layout of dust_masks; a host uint64 array
        or a CUDA tensor): align copies them instead of running DUST on them."""
        L = nat.lib()
        ss = np.ascontiguousarray(list(samples), dtype=np.int32)
        sp = ss.ctypes.data_as(ctypes.c_void_p)
        if isinstance(bits, np.ndarray):
            b = np.ascontiguousarray(bits, dtype=np.uint64)
            nat.check(L.rc_set_dust_masks(self._h, sp, len(ss), b.ctypes.data_as(ctypes.c_void_p), len(b), 0))
        else:
            nat.check(L.rc_set_dust_masks(self._h, sp, len(ss), ctypes.c_void_p(bits.data_ptr()), bits.numel(), 1))

    def timings(self):
        t = nat.RcTiming()
        nat.check(nat.lib().rc_timings(self._h, ctypes.byref(t)))
        return {k: getattr(t, k) for k, _ in nat.RcTiming._fields_}
