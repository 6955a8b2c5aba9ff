"""The C-ABI library loads and exports every entry point include/rcgpu.h
declares (no compute calls: this runs without a GPU)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "rcgpu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rc_[a-z_]+)\s*\(", src)))


def test_header_declares_expected_api():
    names = _declared()
    for n in ("rc_create", "rc_add_sample", "rc_run", "rc_pair_rows", "rc_graph_stats",
              "rc_edges", "rc_pair_sums", "rc_distance", "rc_last_error", "rc_destroy"):
        assert n in names


def test_library_exports_every_declared_symbol(native):
    lib = ctypes.CDLL(os.path.join(ROOT, "rna_clique_amd", "librcgpu.so"))
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_python_bindings_cover_header(native):
    from rna_clique_amd import _native
    assert sorted(_native.SIGNATURES) == _declared()


def test_defaults_follow_reference_config(native):
    from rna_clique_amd import _native
    o = _native.RcOpts()
    native.rc_default_opts(ctypes.byref(o))
    # config.py:77-81: top_matches 1, evalue 1e-99, keep_all True; megablast word 28
    assert (o.top_matches, o.keep_all, o.evalue, o.word_size) == (1, 1, 1e-99, 28)
