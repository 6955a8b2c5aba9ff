"""ctypes bindings of librcgpu.so (include/rcgpu.h).

There is no fallback: if the shared library is missing or fails to load, every
entry point raises. Build it with `python -c "import __graft_entry__ as g;
g.build()"` (or rna_clique_amd.build.build_native()).
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# RC_LIB: an alternative build of the same library (e.g. the cycle-instrumented one)
LIB_PATH = os.environ.get("RC_LIB") or os.path.join(HERE, "librcgpu.so")

RC_OK = 0
RC_E_ARG = -1
RC_E_STATE = -2
RC_E_HIP = -3
RC_E_NOMEM = -4
RC_E_NO_IDEAL = -5
RC_E_CAPACITY = -6
RC_E_LIMIT = -7


class RcOpts(ctypes.Structure):
    _fields_ = [("top_matches", ctypes.c_int32), ("keep_all", ctypes.c_int32),
                ("evalue", ctypes.c_double), ("word_size", ctypes.c_int32),
                ("xdrop_half", ctypes.c_int32), ("device", ctypes.c_int32),
                ("shard_rank", ctypes.c_int32), ("shard_count", ctypes.c_int32),
                ("symmetric", ctypes.c_int32), ("dust_level", ctypes.c_int32),
                ("dust_window", ctypes.c_int32), ("dust_linker", ctypes.c_int32)]


HSP_FIELDS = ["q_tx", "s_tx", "qstart", "qend", "sstart", "send", "length",
              "nident", "mismatch", "gaps", "gapopen", "score_half", "bits10",
              "strand"]
HSP_DTYPE = np.dtype([("q_tx", np.uint32), ("s_tx", np.uint32)] +
                     [(n, np.int32) for n in HSP_FIELDS[2:]] +
                     [("evalue", np.float64)])


class RcHsp(ctypes.Structure):
    _fields_ = [("q_tx", ctypes.c_uint32), ("s_tx", ctypes.c_uint32)] + \
               [(n, ctypes.c_int32) for n in HSP_FIELDS[2:]] + \
               [("evalue", ctypes.c_double)]


ROW_DTYPE = np.dtype([("qgene", np.int32), ("qiso", np.int32), ("sgene", np.int32),
                      ("siso", np.int32), ("q_tx", np.uint32), ("s_tx", np.uint32),
                      ("reverse", np.int32), ("label", np.int32), ("hsp", HSP_DTYPE)])


class RcRow(ctypes.Structure):
    _fields_ = [("qgene", ctypes.c_int32), ("qiso", ctypes.c_int32),
                ("sgene", ctypes.c_int32), ("siso", ctypes.c_int32),
                ("q_tx", ctypes.c_uint32), ("s_tx", ctypes.c_uint32),
                ("reverse", ctypes.c_int32), ("label", ctypes.c_int32),
                ("hsp", RcHsp)]


class RcStats(ctypes.Structure):
    _fields_ = [("nodes", ctypes.c_int64), ("edges", ctypes.c_int64),
                ("components", ctypes.c_int64), ("ideal_components", ctypes.c_int64),
                ("ideal_nodes", ctypes.c_int64), ("sample_count", ctypes.c_int32),
                ("pad", ctypes.c_int32), ("hsps", ctypes.c_int64),
                ("table_rows", ctypes.c_int64), ("seeds", ctypes.c_int64),
                ("candidates", ctypes.c_int64)]


EDGE_DTYPE = np.dtype([("sample_a", np.int32), ("gene_a", np.int32),
                       ("sample_b", np.int32), ("gene_b", np.int32)])

# rc_edge_record (rc_import_edges' host records, graph-only mode)
EDGE_RECORD_DTYPE = np.dtype([("a", np.uint32), ("b", np.uint32), ("pair", np.uint32),
                              ("nident", np.int32), ("den", np.int32)])
RC_EDGE_SUM_ONLY = 0x80000000
RC_NODE_ONLY = 0x7FFFFFFF


class RcTiming(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in (
        "pack_ms", "index_ms", "align_ms", "topn_ms", "rbh_ms", "graph_ms",
        "reduce_ms", "total_ms", "seed_kernel_ms", "align_kernel_ms", "ext_steps",
        "ext_calls", "ext_fullband", "ext_deferred", "big_passes", "tiles", "dust_ms",
        "band_bound", "maxhsp_bound", "ext_second", "near_index", "reverse_seeds", "ext_slides", "ext_wide", "dev_bytes",
        "dev_peak_bytes", "defer_length", "defer_gaveup", "defer_outside", "index_reused",
        "ext_retries", "load_ms", "align_wall_ms", "host_wait_ms", "later_seeds", "later_whole")]


assert HSP_DTYPE.itemsize == ctypes.sizeof(RcHsp)
assert ROW_DTYPE.itemsize == ctypes.sizeof(RcRow)

# Every entry point of include/rcgpu.h with its ctypes signature.
P = ctypes.POINTER
VP = ctypes.c_void_p
SIGNATURES = {
    "rc_default_opts": (None, [P(RcOpts)]),
    "rc_create": (ctypes.c_int, [P(RcOpts), P(VP)]),
    "rc_destroy": (ctypes.c_int, [VP]),
    "rc_last_error": (ctypes.c_char_p, []),
    "rc_dev_peak_reset": (None, []),
    "rc_add_sample": (ctypes.c_int, [VP, ctypes.c_char_p, ctypes.c_char_p,
                                     P(ctypes.c_uint64), P(ctypes.c_int32),
                                     P(ctypes.c_int32), ctypes.c_uint32,
                                     P(ctypes.c_int32)]),
    "rc_add_hsps": (ctypes.c_int, [VP, ctypes.c_int32, ctypes.c_int32, VP, ctypes.c_uint64]),
    "rc_upload": (ctypes.c_int, [VP]),
    "rc_run": (ctypes.c_int, [VP]),
    "rc_align": (ctypes.c_int, [VP]),
    "rc_finish": (ctypes.c_int, [VP]),
    "rc_edge_record_size": (ctypes.c_uint64, []),
    "rc_export_edges": (ctypes.c_int, [VP, VP, ctypes.c_uint64, P(ctypes.c_uint64), ctypes.c_int]),
    "rc_import_edges": (ctypes.c_int, [VP, VP, ctypes.c_uint64, ctypes.c_int]),
    "rc_import_edge_parts": (ctypes.c_int, [VP, VP, VP, ctypes.c_int32, ctypes.c_uint64, ctypes.c_int]),
    "rc_trim": (ctypes.c_int, [VP]),
    "rc_set_sample_count": (ctypes.c_int, [VP, ctypes.c_int32]),
    "rc_shard_pairs": (ctypes.c_int, [VP, P(ctypes.c_int64), P(ctypes.c_int64)]),
    "rc_plan_shards": (ctypes.c_int, [VP, ctypes.c_int32, ctypes.c_int32, VP]),
    "rc_plan_pairs": (ctypes.c_int, [VP, ctypes.c_int32, ctypes.c_int32, VP, VP, VP]),
    "rc_pair_order": (ctypes.c_int, [VP, VP, VP]),
    "rc_hsps": (ctypes.c_int, [VP, ctypes.c_int32, ctypes.c_int32, VP, ctypes.c_uint64,
                               P(ctypes.c_uint64)]),
    "rc_pair_rows": (ctypes.c_int, [VP, ctypes.c_int32, ctypes.c_int32, VP, ctypes.c_uint64,
                                    P(ctypes.c_uint64)]),
    "rc_graph_stats": (ctypes.c_int, [VP, P(RcStats)]),
    "rc_edges": (ctypes.c_int, [VP, VP, ctypes.c_uint64, P(ctypes.c_uint64)]),
    "rc_ideal_nodes": (ctypes.c_int, [VP, VP, VP, ctypes.c_uint64, P(ctypes.c_uint64)]),
    "rc_pair_sums": (ctypes.c_int, [VP, VP, VP]),
    "rc_pair_sums_unfiltered": (ctypes.c_int, [VP, VP, VP]),
    "rc_distance": (ctypes.c_int, [VP, VP, VP]),
    "rc_distance_subset": (ctypes.c_int, [VP, VP, ctypes.c_int32, VP]),
    "rc_timings": (ctypes.c_int, [VP, P(RcTiming)]),
    "rc_dust_mask": (ctypes.c_int, [VP, ctypes.c_int32, VP, ctypes.c_uint64, P(ctypes.c_uint64)]),
    "rc_dust_masks": (ctypes.c_int, [VP, VP, ctypes.c_int32, VP, ctypes.c_uint64, P(ctypes.c_uint64), ctypes.c_int]),
    "rc_set_dust_masks": (ctypes.c_int, [VP, VP, ctypes.c_int32, VP, ctypes.c_uint64, ctypes.c_int]),
    "rc_fasta_open": (ctypes.c_int, [ctypes.c_char_p, P(VP)]),
    "rc_fasta_close": (ctypes.c_int, [VP]),
    "rc_fasta_info": (ctypes.c_int, [VP, P(ctypes.c_uint64), P(ctypes.c_uint64), P(ctypes.c_uint64)]),
    "rc_fasta_titles": (ctypes.c_int, [VP, VP, VP, VP]),
    "rc_fasta_parse_rnaspades": (ctypes.c_int, [VP, VP, VP, VP, VP]),
    "rc_fasta_select": (ctypes.c_int, [VP, VP, VP, VP]),
    "rc_fasta_write": (ctypes.c_int, [VP, VP, ctypes.c_char_p, ctypes.c_int32]),
    "rc_write_outputs": (ctypes.c_int, [VP, ctypes.c_int32, VP, VP, VP, ctypes.c_char_p, ctypes.c_int32]),
    "rc_write_graph": (ctypes.c_int, [VP, ctypes.c_char_p, ctypes.c_int32]),
    "rc_table_write_rows": (ctypes.c_int, [VP, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]),
    "rc_graph_pickle_begin": (ctypes.c_int, [P(VP)]),
    "rc_graph_pickle_add": (ctypes.c_int, [VP, ctypes.c_int32, ctypes.c_int32, VP, VP, ctypes.c_uint64]),
    "rc_graph_pickle_write": (ctypes.c_int, [VP, ctypes.c_char_p, ctypes.c_int32, VP]),
    "rc_graph_pickle_free": (None, [VP]),
}

_lib = None


class NativeError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"rcgpu error {code}: {msg}")
        self.code = code


def lib():
    """Load librcgpu.so (raises if it is missing: there is no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build the HIP engine first "
                "(python -c 'import __graft_entry__ as g; g.build()')")
        if "torch" in sys.modules:
            # torch bundles its own HIP runtime: when the caller uses torch on
            # the GPU too (torch.distributed, CUDA tensors handed to the
            # engine), bring torch's up first -- its lazy init after this
            # library's runtime was seen to find no device
            try:
                import torch
                if torch.cuda.is_available():
                    torch.cuda.init()
            except Exception:
                pass
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(code):
    if code != RC_OK:
        msg = lib().rc_last_error().decode(errors="replace")
        raise NativeError(code, msg)
