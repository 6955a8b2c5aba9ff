"""A small HDF5 writer for the distance matrix (matrix.h5) without PyTables.

The reference saves the matrix with `DataFrame.to_hdf(path, key="matrix")`
(rna_clique.py:176-177, 205-206), i.e. pandas' *fixed* format written through
PyTables (docs/formats.md:346-352). PyTables is not importable in this image
(SURVEY.md §8c), so this module writes the same object tree directly:

    /                   CLASS, PYTABLES_FORMAT_VERSION, TITLE, VERSION
    /matrix             pandas_type="frame", pandas_version, encoding, errors,
                        ndim=2, axis0_variety, axis1_variety, nblocks=1,
                        block0_items_variety   (+ PyTables group attrs)
    /matrix/axis0       column labels, fixed-length byte strings, kind="string"
    /matrix/axis1       row labels, likewise
    /matrix/block0_items  column labels again
    /matrix/block0_values float64 N x N (the matrix), transposed=1

File format: superblock v0, version-1 object headers, symbol-table groups
(v1 B-tree + local heap + one symbol-table node), contiguous datasets. That is
the classic layout every HDF5 reader since 1.6 understands. Only what the
matrix needs is implemented: groups of at most 8 children, scalar/1-D/2-D
datasets of float64, int64 and fixed-length strings, scalar attributes.
"""
from __future__ import annotations

import os
import struct

import numpy as np

UNDEF = 0xFFFFFFFFFFFFFFFF
LEAF_K = 4          # group leaf node K (symbol-table node holds 2K entries)
INTERNAL_K = 16     # group internal node K (B-tree node holds 2K children)
HEAP_FREE_NULL = 1  # "no free block" in a local heap


def _pad8(b: bytes) -> bytes:
    return b + b"\0" * (-len(b) % 8)


# ---------------------------------------------------------------- datatypes
def _dt_float64():
    # class 1 (float), version 1; little endian, mantissa normalisation 2
    # (implied msb), sign bit 63; offset 0, precision 64, exponent 52/11,
    # mantissa 0/52, bias 1023
    return struct.pack("<B3BI", 0x11, 0x20, 63, 0, 8) + struct.pack("<HHBBBBI", 0, 64, 52, 11, 0, 52, 1023)


def _dt_int(size, signed=True):
    return struct.pack("<B3BI", 0x10, 0x08 if signed else 0, 0, 0, size) + struct.pack("<HH", 0, 8 * size)


def _dt_string(size, utf8=True, nullterm=True):
    bits = (0 if nullterm else 1) | ((1 if utf8 else 0) << 4)
    return struct.pack("<B3BI", 0x13, bits, 0, 0, size)


def _dataspace(shape):
    return struct.pack("<BBBB4x", 1, len(shape), 0, 0) + b"".join(struct.pack("<Q", d) for d in shape)


def _value(v):
    """Python/numpy value -> (datatype bytes, shape, raw data bytes)."""
    if isinstance(v, (str, bytes)):
        raw = v.encode("utf-8") if isinstance(v, str) else v
        raw = raw if raw else b"\0"
        return _dt_string(len(raw), utf8=isinstance(v, str)), (), raw
    if isinstance(v, (bool, np.bool_)):
        return _dt_int(1), (), struct.pack("<b", int(v))
    if isinstance(v, (int, np.integer)):
        return _dt_int(8), (), struct.pack("<q", int(v))
    if isinstance(v, (float, np.floating)):
        return _dt_float64(), (), struct.pack("<d", float(v))
    a = np.asarray(v)
    if a.dtype.kind == "f":
        a = np.ascontiguousarray(a, dtype="<f8")
        return _dt_float64(), a.shape, a.tobytes()
    if a.dtype.kind in "iu":
        a = np.ascontiguousarray(a, dtype="<i8")
        return _dt_int(8), a.shape, a.tobytes()
    if a.dtype.kind == "S":
        a = np.ascontiguousarray(a)
        return _dt_string(a.dtype.itemsize, utf8=False), a.shape, a.tobytes()
    raise TypeError(f"unsupported HDF5 value {type(v)} {getattr(a, 'dtype', None)}")


# ---------------------------------------------------------------- messages
def _msg(mtype, body, flags=0):
    body = _pad8(body)
    return struct.pack("<HHB3x", mtype, len(body), flags) + body


def _attr_msg(name, value):
    dt, shape, raw = _value(value)
    ds = _dataspace(shape)
    nm = name.encode() + b"\0"
    body = struct.pack("<BBHHH", 1, 0, len(nm), len(dt), len(ds)) + _pad8(nm) + _pad8(dt) + _pad8(ds) + raw
    return _msg(0x000C, body)


def _object_header(messages):
    data = b"".join(messages)
    return struct.pack("<BBHII4x", 1, 0, len(messages), 1, len(data)) + data


class _File:
    def __init__(self):
        self.buf = bytearray(96)   # superblock v0 placeholder

    def alloc(self, data: bytes) -> int:
        addr = len(self.buf)
        self.buf += _pad8(bytes(data))
        return addr


class Dataset:
    def __init__(self, data, attrs=None):
        self.data = data
        self.attrs = dict(attrs or {})

    def write(self, f: _File) -> int:
        dt, shape, raw = _value(self.data)
        if not shape:
            raise ValueError("datasets must be arrays")
        addr = f.alloc(raw) if raw else UNDEF
        layout = struct.pack("<BBQQ", 3, 1, addr, len(raw))
        fill = struct.pack("<BBBB", 2, 2, 2, 0)   # v2: late alloc, fill never, undefined
        msgs = [_msg(0x0001, _dataspace(shape)), _msg(0x0003, dt, flags=1),
                _msg(0x0005, fill, flags=1), _msg(0x0008, layout)]
        msgs += [_attr_msg(k, v) for k, v in self.attrs.items()]
        return f.alloc(_object_header(msgs))


class Group:
    def __init__(self, attrs=None, children=None):
        self.attrs = dict(attrs or {})
        self.children = dict(children or {})

    def write(self, f: _File):
        """Returns (object header address, B-tree address, heap address)."""
        names = sorted(self.children, key=lambda s: s.encode())
        if len(names) > 2 * LEAF_K:
            raise ValueError("group has more children than one symbol-table node holds")
        child_addr = {n: self.children[n].write(f) for n in names}
        child_addr = {n: (a[0] if isinstance(a, tuple) else a) for n, a in child_addr.items()}
        # local heap: "" at offset 0, then the names
        heap = bytearray(8)
        name_off = {}
        for n in names:
            name_off[n] = len(heap)
            heap += _pad8(n.encode() + b"\0")
        heap_data = f.alloc(bytes(heap))
        heap_addr = f.alloc(b"HEAP" + struct.pack("<B3xQQQ", 0, len(heap), HEAP_FREE_NULL, heap_data))
        # symbol-table node with 2K entry slots
        ents = b"".join(struct.pack("<QQII16x", name_off[n], child_addr[n], 0, 0) for n in names)
        ents += b"\0" * (40 * (2 * LEAF_K - len(names)))
        snod = f.alloc(b"SNOD" + struct.pack("<BBH", 1, 0, len(names)) + ents)
        # v1 B-tree (group node, level 0) with 2K child slots and 2K+1 keys
        nkeys, nchild = 2 * INTERNAL_K + 1, 2 * INTERNAL_K
        body = struct.pack("<BBHQQ", 0, 0, 1 if names else 0, UNDEF, UNDEF)
        if names:
            body += struct.pack("<QQQ", 0, snod, name_off[names[-1]])
            body += b"\0" * (8 * (nkeys + nchild) - 24)
        else:
            body += b"\0" * (8 * (nkeys + nchild))
        btree = f.alloc(b"TREE" + body)
        msgs = [_msg(0x0011, struct.pack("<QQ", btree, heap_addr))]
        msgs += [_attr_msg(k, v) for k, v in self.attrs.items()]
        return f.alloc(_object_header(msgs)), btree, heap_addr


def write_tree(path, root: Group):
    f = _File()
    ohdr, btree, heap = root.write(f)
    eof = len(f.buf)
    sb = b"\x89HDF\r\n\x1a\n" + struct.pack("<8B", 0, 0, 0, 0, 0, 8, 8, 0)
    sb += struct.pack("<HHI", LEAF_K, INTERNAL_K, 0)
    sb += struct.pack("<QQQQ", 0, UNDEF, eof, UNDEF)
    sb += struct.pack("<QQII", 0, ohdr, 1, 0) + struct.pack("<QQ", btree, heap)
    assert len(sb) == 96
    f.buf[:96] = sb
    tmp = os.fspath(path) + ".tmp"
    with open(tmp, "wb") as fh:
        fh.write(f.buf)
    os.replace(tmp, path)


# ---------------------------------------------------------------- pandas layout
_PT_GROUP = {"CLASS": "GROUP", "TITLE": "", "VERSION": "1.0"}
_PT_ARRAY = {"CLASS": "ARRAY", "FLAVOR": "numpy", "TITLE": "", "VERSION": "2.4"}


def _labels(values, encoding="UTF-8"):
    enc = [str(v).encode(encoding) for v in values]
    size = max([1] + [len(e) for e in enc])
    return np.array(enc, dtype=f"S{size}")


def write_frame_fixed(path, values, index, columns, key="matrix"):
    """Write a float64 DataFrame the way `df.to_hdf(path, key=key)` (fixed
    format) lays it out."""
    values = np.ascontiguousarray(values, dtype=np.float64)
    if values.shape != (len(index), len(columns)):
        raise ValueError("values shape does not match the labels")
    cols = _labels(columns)
    rows = _labels(index)
    frame = Group(
        attrs={**_PT_GROUP, "pandas_type": "frame", "pandas_version": "0.15.2",
               "encoding": "UTF-8", "errors": "strict", "ndim": 2,
               "axis0_variety": "regular", "axis1_variety": "regular", "nblocks": 1,
               "block0_items_variety": "regular"},
        children={
            "axis0": Dataset(cols, {**_PT_ARRAY, "kind": "string"}),
            "axis1": Dataset(rows, {**_PT_ARRAY, "kind": "string"}),
            "block0_items": Dataset(cols, {**_PT_ARRAY, "kind": "string"}),
            # pandas stores block.values.T (= the frame's values) with transposed=True
            "block0_values": Dataset(values, {**_PT_ARRAY, "transposed": True}),
        })
    root = Group(attrs={**_PT_GROUP, "PYTABLES_FORMAT_VERSION": "2.1"},
                 children={key: frame})
    write_tree(path, root)


def write_matrix(df, path, key="matrix"):
    """matrix.h5 writer: pandas.to_hdf when PyTables is importable, else the
    equivalent layout written by this module."""
    try:
        import tables  # noqa: F401
    except ImportError:
        write_frame_fixed(path, df.to_numpy(dtype=np.float64), list(df.index), list(df.columns), key)
        return
    df.to_hdf(path, key=key)
