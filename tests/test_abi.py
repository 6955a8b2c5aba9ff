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


def _header_struct_fields(name):
    """(field, C type) of `typedef struct name {...}` in rcgpu.h, in order."""
    src = open(os.path.join(ROOT, "include", "rcgpu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    body = re.search(r"typedef struct %s \{(.*?)\}" % name, src, flags=re.S).group(1)
    out = []
    for decl in body.split(";"):
        decl = decl.strip()
        if not decl:
            continue
        ctype, names = decl.split(None, 1)
        out += [(n.strip(), ctype) for n in names.split(",")]
    return out


def test_integration_snippet_matches_header():
    """INTEGRATION.md's reference-side ctypes binding declares rc_opts with the
    header's fields in the header's order and types (a short struct there
    would let rc_default_opts write past it), as _native.RcOpts does."""
    from rna_clique_amd import _native
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    m = re.search(r"class rc_opts\(ctypes\.Structure\):.*?_fields_ = (\[.*?\])\n", doc, flags=re.S)
    assert m, "no rc_opts binding in INTEGRATION.md"
    snippet = eval(m.group(1), {"ctypes": ctypes})   # the doc's own literal list of (name, ctypes type)
    cmap = {"int32_t": ctypes.c_int32, "double": ctypes.c_double}
    header = [(n, cmap[t]) for n, t in _header_struct_fields("rc_opts")]
    assert len(header) == 12
    assert snippet == header
    assert list(_native.RcOpts._fields_) == header

    class Snip(ctypes.Structure):
        _fields_ = snippet
    assert ctypes.sizeof(Snip) == ctypes.sizeof(_native.RcOpts)
